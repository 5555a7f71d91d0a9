// k_dist.hip -- squared input distances ||v_k - z_c||^2 as a stand-alone pass, and the Kalman
// whitening that consumes them (gfx950).
//
// The fused whitening of k_lgssm.hip (whiten_kfu_mfma) keeps the pseudo-input fragments of its 64
// columns in registers, which caps the input dimension at D = 64.  GPAR's output p has D = p - 1
// (GPAR_scaled_examples.jl:132-175; BASELINE config 5 runs P = 256 outputs, so D up to 255), and
// the reference computes Kfu = pairwise(k_o, V, Z) for any D (dtc.jl:104,
// gpar_scaled_inference.jl:89,156).  For D > 64 the distance contraction runs here as its own
// fp64-MFMA GEMM with the D dimension streamed through LDS in 16-wide K-steps:
//
//   d2[k][c] = |v_k - g|^2 + |z_c - g|^2 - 2 (v_k - g).(z_c - g)
//
// with g the centre of the 256-pseudo-input group of column c (zcenter, the same centring the
// fused kernel uses: Distances.jl's Gram form with the cancellation of the shared offset removed,
// SURVEY §8a a1).  Matern-1/2 needs direct differences (its kernel is not smooth in d^2 at 0), so
// it gets a VALU tile kernel instead.  The distances are theta-independent; whiten_kfu_d2 then
// evaluates Kfu = s_o kappa(sqrt(d2) / l_o) on the fly, runs the chunk-local Kalman filter and
// overwrites d2 with beta_loc in place (one read + one write of N x Mp doubles).
#include "device_common.hpp"

namespace gpar {

typedef double d4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------- distance GEMM
// 128 x 128 (steps x columns) tile per 256-thread workgroup, 2 x 2 waves of 4 x 4
// v_mfma_f64_16x16x4_f64 tiles, K-step 16 double-buffered through LDS (k-major rows padded to
// kDLds: the 16 lanes of a fragment read 16 consecutive doubles, conflict-free).  The norms of
// the centred rows are accumulated by the staging threads themselves.
constexpr int kDT = 128, kDBK = 16, kDLds = 136;

__global__ __launch_bounds__(256, 2) void dist2_mfma_kernel(
    const double* __restrict__ v, int64_t ldv, int64_t n, const double* __restrict__ z,
    int64_t ldz, int64_t m, int64_t mp, int d, const double* __restrict__ zc, int64_t zld,
    double* __restrict__ out, int64_t ldo) {
  __shared__ __attribute__((aligned(16))) double smem[2 * 2 * kDBK * kDLds];
  __shared__ double vn_s[kDT], zn_s[kDT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t r0 = (int64_t)blockIdx.x * kDT, c0 = (int64_t)blockIdx.y * kDT;
  const double* cg = zc + (c0 >> 8) * zld;   // 128-column tiles never straddle a 256-group
  const int srow = tid >> 1, sk = (tid & 1) * 8;
  const int64_t arow = r0 + srow, brow = c0 + srow;
  const bool av = arow < n, bv = brow < m;
  const int64_t arc = av ? arow : n - 1, brc = bv ? brow : (m > 0 ? m - 1 : 0);
  double ra[8], rb[8];
  double an = 0.0, bn = 0.0;
  auto load = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int kk = k0 + sk + q;
      const int kc = kk < d ? kk : d - 1;
      const double g = cg[kc];
      const double a = v[arc * ldv + kc] - g;
      const double b = z[brc * ldz + kc] - g;
      ra[q] = (av && kk < d) ? a : 0.0;
      rb[q] = (bv && kk < d) ? b : 0.0;
      an = fma(ra[q], ra[q], an);
      bn = fma(rb[q], rb[q], bn);
    }
  };
  auto store = [&](int buf) {
    double* la = smem + (buf * 2 + 0) * kDBK * kDLds;
    double* lb = smem + (buf * 2 + 1) * kDBK * kDLds;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      la[(sk + q) * kDLds + srow] = ra[q];
      lb[(sk + q) * kDLds + srow] = rb[q];
    }
  };
  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = d4{0.0, 0.0, 0.0, 0.0};
  const int nsteps = (d + kDBK - 1) / kDBK;
  load(0);
  store(0);
  __syncthreads();
  const int frow = lane >> 4, fcol = lane & 15;
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    const bool more = s + 1 < nsteps;
    if (more) load((s + 1) * kDBK);
    const double* la = smem + (buf * 2 + 0) * kDBK * kDLds;
    const double* lb = smem + (buf * 2 + 1) * kDBK * kDLds;
#pragma unroll
    for (int ks = 0; ks < kDBK / 4; ++ks) {
      double fa[4], fb[4];
      const int kr = ks * 4 + frow;
#pragma unroll
      for (int a = 0; a < 4; ++a) fa[a] = la[kr * kDLds + wr * 64 + a * 16 + fcol];
#pragma unroll
      for (int c = 0; c < 4; ++c) fb[c] = lb[kr * kDLds + wc * 64 + c * 16 + fcol];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[a][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[a], fb[c], acc[a][c], 0, 0, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }
  // row norms: the two staging threads of a row hold complementary halves of every K-step
  an += __shfl_xor(an, 1, 64);
  bn += __shfl_xor(bn, 1, 64);
  if ((tid & 1) == 0) {
    vn_s[srow] = an;
    zn_s[srow] = bn;
  }
  __syncthreads();
  // C layout: lane holds rows frow + 4 r, column fcol of each 16 x 16 tile
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = wr * 64 + a * 16 + frow + 4 * r;
      const int64_t row = r0 + rl;
      if (row >= n) continue;
      const double vn = vn_s[rl];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cl = wc * 64 + c * 16 + fcol;
        const int64_t col = c0 + cl;
        if (col < mp) out[row * ldo + col] = col < m ? vn + zn_s[cl] - 2.0 * acc[a][c][r] : 0.0;
      }
    }
}

// ---------------------------------------------------------------------------- direct distances
// Matern-1/2: d2 = sum_i (v_k,i - z_c,i)^2 by direct differences (as the oracle and the fused
// whiten_kfu do).  One column per thread, 64 steps per workgroup tile, the tile's V rows staged
// through LDS 16 dimensions at a time (read back as broadcasts); the column's 16 z values of the
// current slice sit in registers.
constexpr int kDRows = 64, kDDim = 16;

__global__ __launch_bounds__(256) void dist2_direct_kernel(
    const double* __restrict__ v, int64_t ldv, int64_t n, const double* __restrict__ z,
    int64_t ldz, int64_t m, int64_t mp, int d, double* __restrict__ out, int64_t ldo) {
  __shared__ double vs[kDRows][kDDim + 1];
  const int tid = threadIdx.x;
  const int64_t c = (int64_t)blockIdx.y * 256 + tid;
  const int64_t k0 = (int64_t)blockIdx.x * kDRows;
  const bool cv = c < m;
  const int64_t cc = cv ? c : 0;
  double acc[kDRows];
#pragma unroll
  for (int r = 0; r < kDRows; ++r) acc[r] = 0.0;
  for (int i0 = 0; i0 < d; i0 += kDDim) {
    __syncthreads();
    for (int e = tid; e < kDRows * kDDim; e += 256) {
      const int r = e / kDDim, i = e % kDDim;
      const int64_t k = k0 + r;
      vs[r][i] = (k < n && i0 + i < d) ? v[k * ldv + i0 + i] : 0.0;
    }
    double zr[kDDim];
#pragma unroll
    for (int i = 0; i < kDDim; ++i) zr[i] = (i0 + i < d) ? z[cc * ldz + i0 + i] : 0.0;
    __syncthreads();
    const int ni = (d - i0 < kDDim) ? d - i0 : kDDim;
    if (ni == kDDim) {
#pragma unroll
      for (int r = 0; r < kDRows; ++r)
#pragma unroll
        for (int i = 0; i < kDDim; ++i) {
          const double a = vs[r][i] - zr[i];
          acc[r] = fma(a, a, acc[r]);
        }
    } else {
#pragma unroll
      for (int r = 0; r < kDRows; ++r)
        for (int i = 0; i < ni; ++i) {
          const double a = vs[r][i] - zr[i];
          acc[r] = fma(a, a, acc[r]);
        }
    }
  }
  if (c < mp) {
#pragma unroll
    for (int r = 0; r < kDRows; ++r) {
      const int64_t k = k0 + r;
      if (k < n) out[k * ldo + c] = cv ? acc[r] : 0.0;
    }
  }
}

// ---------------------------------------------------------------------------- whitening from d2
// beta_loc[k][c] = chunk-local whitened Kfu column c, Kfu[k][c] = s_o kappa(sqrt(d2[k][c]) / l_o),
// reading d2 from `src` (ld lds) and writing beta (ld ldb; in place when src == beta: every
// thread reads only rows ahead of the ones it has written, of its own column).  grid (nch,
// ceil(mp / 256)), one column per thread; per 16-step sub-tile the gains records and fix-up rows
// are staged in LDS (uniform, read back as broadcasts) and the next sub-tile's 16 d2 values are
// prefetched into registers, so the loads of sub-tile s + 1 are in flight under the kernel
// evaluations and the filter recursion of sub-tile s.  Outputs as whiten_kfu (send, hsum).
constexpr int kWT = 16;

template <int TK, int OK>
__global__ __launch_bounds__(256) void whiten_kfu_d2(
    const double* __restrict__ rec, const double* src, int64_t lds, int64_t m, int64_t mp,
    int64_t n, int L, double inv_lo, double s_o, double* beta, int64_t ldb,
    double* __restrict__ send, int64_t mc, const double* __restrict__ g,
    double* __restrict__ hsum) {
  constexpr int SD = Sde<TK>::d;
  constexpr int RS = Rec<SD>::size;
  __shared__ __attribute__((aligned(16))) double rl[kWT * RS];
  __shared__ __attribute__((aligned(16))) double gl[kWT * kGStride];
  const int tid = threadIdx.x;
  const int64_t j = blockIdx.x;
  const int64_t c = (int64_t)blockIdx.y * 256 + tid;
  const bool colv = c < m, cola = c < mp;
  const int64_t cc = cola ? c : 0;
  const int64_t k0 = j * L;
  const int64_t k1 = (k0 + L < n) ? k0 + L : n;
  double mst[SD], hs[SD];
#pragma unroll
  for (int i = 0; i < SD; ++i) mst[i] = hs[i] = 0.0;
  double px[kWT], pr, pg;
  auto prefetch = [&](int64_t kt_) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < kWT; ++r) {
      const int64_t k = (kt_ + r < n) ? kt_ + r : n - 1;
      px[r] = src[k * lds + cc];
    }
    const int64_t ir = kt_ * RS + tid;
    pr = rec[ir < n * RS ? ir : n * RS - 1];
    const int64_t ig = kt_ * kGStride + tid;
    pg = g[ig < n * kGStride ? ig : n * kGStride - 1];
  };
  if (k0 < k1) prefetch(k0);
  for (int64_t kt = k0; kt < k1; kt += kWT) {
    const int nt = (kt + kWT <= k1) ? kWT : (int)(k1 - kt);
    __syncthreads();
    if (tid < kWT * RS) rl[tid] = tid < nt * RS ? pr : 0.0;
    if (tid < kWT * kGStride) gl[tid] = tid < nt * kGStride ? pg : 0.0;
    double x[kWT];
#pragma unroll
    for (int r = 0; r < kWT; ++r) x[r] = px[r];
    __syncthreads();
    if (kt + kWT < k1) prefetch(kt + kWT);
#pragma unroll
    for (int r = 0; r < kWT; ++r) {
      double d2 = x[r];
      if constexpr (OK == KEQ) d2 = d2 > 0.0 ? d2 : 0.0;   // the Matern forms clamp in sqrt_pos
      x[r] = colv ? skappa_sq<OK>(d2, inv_lo, s_o) : 0.0;
    }
    auto step = [&](int kk) __attribute__((always_inline)) {
      const double* rr = rl + kk * RS;
      double mm[SD];
#pragma unroll
      for (int i = 0; i < SD; ++i) {
        double a2 = 0.0;
#pragma unroll
        for (int q = 0; q < SD; ++q) a2 = fma(rr[i * SD + q], mst[q], a2);
        mm[i] = a2;
      }
      const double ev = x[kk] - mm[0];
      const double al = ev * rr[SD * SD + SD];
#pragma unroll
      for (int i = 0; i < SD; ++i) mst[i] = fma(rr[SD * SD + i], ev, mm[i]);
#pragma unroll
      for (int i = 0; i < SD; ++i) hs[i] = fma(al, gl[kk * kGStride + i], hs[i]);
      if (cola) beta[(kt + kk) * ldb + c] = al;
    };
    if (nt == kWT) {
#pragma unroll
      for (int kk = 0; kk < kWT; ++kk) step(kk);
    } else {
#pragma unroll
      for (int kk = 0; kk < kWT; ++kk)
        if (kk < nt) step(kk);
    }
  }
  if (cola) {
#pragma unroll
    for (int i = 0; i < SD; ++i) {
      send[(j * mc + c) * kSStride + i] = mst[i];
      if (hsum) hsum[(j * mc + c) * kSStride + i] = hs[i];
    }
  }
}

// ---------------------------------------------------------------------------- wide centres
// zc[g * zld + i] = mean over the group's (<= 256) pseudo-inputs of z[c][i], any d (one thread per
// dimension, the group's columns summed in order).
__global__ __launch_bounds__(256) void zcenter_wide_kernel(const double* __restrict__ z,
                                                           int64_t ldz, int d, int64_t m,
                                                           int64_t zld, double* __restrict__ zc) {
  const int64_t g = blockIdx.x;
  const int64_t c0 = g * 256, c1 = (c0 + 256 < m) ? c0 + 256 : m;
  for (int i = threadIdx.x; i < zld; i += 256) {
    double s = 0.0;
    if (i < d)
      for (int64_t c = c0; c < c1; ++c) s += z[c * ldz + i];
    zc[g * zld + i] = (i < d && c1 > c0) ? s / (double)(c1 - c0) : 0.0;
  }
}

}  // namespace gpar

// ============================================================================ launch wrappers
#include "launch.hpp"

namespace gpar {

int64_t zc_stride(int d) {
  if (d <= 64) return mfma_dp_bucket(d);
  return (d + 3) / 4 * 4;
}

void launch_zcenter_wide(hipStream_t st, const double* z, int64_t ldz, int d, int64_t m,
                         int64_t mp, double* zc) {
  zcenter_wide_kernel<<<(unsigned)((mp + 255) / 256), 256, 0, st>>>(z, ldz, d, m, zc_stride(d), zc);
}

void launch_dist2(hipStream_t st, int out_kind, const double* v, int64_t ldv, int64_t n,
                  const double* z, int64_t ldz, int64_t m, int64_t mp, int d, const double* zc,
                  double* out, int64_t ldo) {
  if (n <= 0) return;
  if (out_kind == KM12) {
    dim3 grid((unsigned)((n + kDRows - 1) / kDRows), (unsigned)((mp + 255) / 256));
    dist2_direct_kernel<<<grid, 256, 0, st>>>(v, ldv, n, z, ldz, m, mp, d, out, ldo);
  } else {
    dim3 grid((unsigned)((n + kDT - 1) / kDT), (unsigned)((mp + kDT - 1) / kDT));
    dist2_mfma_kernel<<<grid, 256, 0, st>>>(v, ldv, n, z, ldz, m, mp, d, zc, zc_stride(d), out, ldo);
  }
}

template <int TK, int OK>
static void launch_wd2_k(hipStream_t st, dim3 grid, const double* rec, const double* src,
                         int64_t lds, int64_t m, int64_t mp, int64_t n, int L, double inv_lo,
                         double s_o, double* beta, int64_t ldb, double* send, int64_t mc,
                         const double* g, double* hsum) {
  whiten_kfu_d2<TK, OK><<<grid, 256, 0, st>>>(rec, src, lds, m, mp, n, L, inv_lo, s_o, beta, ldb,
                                              send, mc, g, hsum);
}

template <int TK>
static void launch_wd2_t(hipStream_t st, int ok, dim3 grid, const double* rec, const double* src,
                         int64_t lds, int64_t m, int64_t mp, int64_t n, int L, double inv_lo,
                         double s_o, double* beta, int64_t ldb, double* send, int64_t mc,
                         const double* g, double* hsum) {
  switch (ok) {
    case KM12: launch_wd2_k<TK, KM12>(st, grid, rec, src, lds, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case KM32: launch_wd2_k<TK, KM32>(st, grid, rec, src, lds, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case KEQ: launch_wd2_k<TK, KEQ>(st, grid, rec, src, lds, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    default: launch_wd2_k<TK, KM52>(st, grid, rec, src, lds, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
  }
}

void launch_whiten_kfu_d2(hipStream_t st, int time_kind, int out_kind, const double* rec,
                          const double* src, int64_t lds, int64_t m, int64_t mp, int64_t n, int L,
                          int64_t nch, double inv_lo, double s_o, double* beta, int64_t ldb,
                          double* send, int64_t mc, const double* g, double* hsum) {
  dim3 grid((unsigned)nch, (unsigned)((mp + 255) / 256));
  switch (time_kind) {
    case KM12: launch_wd2_t<KM12>(st, out_kind, grid, rec, src, lds, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case KM32: launch_wd2_t<KM32>(st, out_kind, grid, rec, src, lds, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    default: launch_wd2_t<KM52>(st, out_kind, grid, rec, src, lds, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
  }
}

}  // namespace gpar
