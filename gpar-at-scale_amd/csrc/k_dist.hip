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
// it gets a VALU tile kernel instead.  whiten_kfu_d2x2 then evaluates Kfu = s_o kappa(sqrt(d2) /
// l_o) on the fly, runs the chunk-local Kalman filter and writes beta_loc (one read + one write of
// N x Mp doubles): in place over d2 for D > 64, or from the fit's distance cache -- the distances
// are theta-independent, so gpar_host.cpp (attach_dist_cache) computes them once per fit for the
// outputs it caches and every objective evaluation reads them.
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
    double* __restrict__ out, int64_t ldo, int rout) {
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
        if (col < mp) {
          const double d2 = col < m ? vn + zn_s[cl] - 2.0 * acc[a][c][r] : 0.0;
          out[row * ldo + col] = rout ? sqrt_pos(d2) : d2;
        }
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
    int64_t ldz, int64_t m, int64_t mp, int d, double* __restrict__ out, int64_t ldo, int rout) {
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
      if (k < n) {
        const double d2 = cv ? acc[r] : 0.0;
        out[k * ldo + c] = rout ? sqrt_pos(d2) : d2;
      }
    }
  }
}

// ---------------------------------------------------------------------------- whitening from d2
// beta_loc[k][c] = chunk-local whitened Kfu column c, Kfu[k][c] = s_o kappa(sqrt(d2[k][c]) / l_o),
// reading d2 from `src` (ld lds) and writing beta (ld ldb; in place when src == beta: each thread
// reads only rows ahead of the ones it has written, of its own columns).  Laid out for issue
// efficiency: each thread runs TWO adjacent columns (16-byte d2 loads and beta stores; every gains
// record read from LDS serves both recursions, which also interleave), and the whole chunk's
// records and fix-up rows (L <= 256 steps, 40 KB) are staged in LDS once, so the chunk runs with
// no workgroup barrier after the first.  grid (nch, ceil(mp / 512)); the next kW2T rows' d2 pairs
// are prefetched into registers under the current rows' kernel evaluations and recursions; the
// exp constants come in as a kernel argument (SGPR operands, see ExpNegConsts).  Outputs as
// whiten_kfu (send, hsum).  Measured at N = 1e6, M = 512: 1.74 ms = 4.7 TB/s of d2 read + beta
// write (8.2 GB); the single-column form with per-16-row staging took 2.13 ms; occupancy 3
// (4-row tiles) and inline exp constants measured the same.  Requires L <= kW2MaxL, even lds /
// ldb, 16-byte aligned src / beta (mp is a multiple of 128).
constexpr int kW2MaxL = 256;

constexpr int kW2T = 8;     // rows of d2 prefetched per thread
constexpr int kW2Occ = 2;   // workgroups per CU

// RIN: src holds the distances r = sqrt_pos(d2) (the fit's cache, Matern kernels) instead of d2.
// CR: rec holds compact records {K, rs} (gains_phase3<D, true>); each step's transition A_k is
// recomputed here from t (tau = (t_k - t_{k-1}) / l_t, as the gains pass computes it) while the
// chunk's records are staged, which cuts the gains pass's HBM writes by more than half.
template <int TK, int OK, bool RIN, bool CR>
__global__ __launch_bounds__(256, kW2Occ) void whiten_kfu_d2x2(
    const double* __restrict__ rec, const double* src, int64_t lds, int64_t m, int64_t mp,
    int64_t n, int L, double inv_lo, double s_o, double* beta, int64_t ldb,
    double* __restrict__ send, int64_t mc, const double* __restrict__ g,
    double* __restrict__ hsum, ExpNegConsts ek, const double* __restrict__ tt, double l_t) {
  constexpr int SD = Sde<TK>::d;
  constexpr int RS = Rec<SD>::size;
  // the chunk's step rows {A_k, K_k, rs_k, g_k}, 16 doubles each, read one double per lane and
  // broadcast by DPP (fmac_row, device_common.hpp)
  constexpr int RK = SD * SD, RR = SD * SD + SD, RG = SD * SD + SD + 1;
  static_assert(RG + SD <= 16, "step row");
  __shared__ __attribute__((aligned(16))) double rg[kW2MaxL * 16];
  const int tid = threadIdx.x;
  const int64_t j = blockIdx.x;
  const int64_t c = ((int64_t)blockIdx.y * 256 + tid) * 2;   // first of the thread's two columns
  const bool cola = c < mp;                                  // mp even: both or neither
  const bool v0 = c < m, v1 = c + 1 < m;
  const int64_t cc = cola ? c : 0;
  const int64_t k0 = j * L;
  const int64_t k1 = (k0 + L < n) ? k0 + L : n;
  const int nk = (int)(k1 - k0);
  // the chunk's records and fix-up rows, once
  if constexpr (CR) {
    constexpr int CS = CRec<SD>::size;
    for (int e = tid; e < nk; e += 256) {
      const int64_t k = k0 + e;
      double A[SD][SD];
      sde_transition<SD>((k == 0) ? 1.0 : (tt[k] - tt[k - 1]) / l_t, A);
#pragma unroll
      for (int i = 0; i < SD; ++i)
#pragma unroll
        for (int q = 0; q < SD; ++q) rg[e * 16 + i * SD + q] = A[i][q];
#pragma unroll
      for (int i = 0; i <= SD; ++i) rg[e * 16 + RK + i] = rec[k * CS + i];
    }
  } else {
    for (int e = tid; e < nk * RS; e += 256)
      if (e % RS < RG) rg[e / RS * 16 + e % RS] = rec[k0 * RS + e];
  }
  for (int e = tid; e < nk * kGStride; e += 256)
    if (e % kGStride < SD) rg[e / kGStride * 16 + RG + e % kGStride] = g[k0 * kGStride + e];
  double ma[SD], mb[SD], ha[SD], hb[SD];
#pragma unroll
  for (int i = 0; i < SD; ++i) ma[i] = mb[i] = ha[i] = hb[i] = 0.0;
  const double* sp = src + k0 * lds + cc;
  double* bp = beta + k0 * ldb + cc;
  double2 px[kW2T];
  auto prefetch = [&](int r0) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < kW2T; ++r) {
      const int rr = (r0 + r < nk) ? r0 + r : nk - 1;
      {
        typedef double v2d __attribute__((ext_vector_type(2)));
        const v2d t = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(sp + (int64_t)rr * lds));
        px[r].x = t.x;
        px[r].y = t.y;
      }
    }
  };
  if (nk > 0) prefetch(0);
  __syncthreads();
  for (int r0 = 0; r0 < nk; r0 += kW2T) {
    double2 x[kW2T];
#pragma unroll
    for (int r = 0; r < kW2T; ++r) x[r] = px[r];
    if (r0 + kW2T < nk) prefetch(r0 + kW2T);
#pragma unroll
    for (int r = 0; r < kW2T; ++r) {
      double a = x[r].x, b = x[r].y;
      if constexpr (OK == KEQ) {
        a = a > 0.0 ? a : 0.0;
        b = b > 0.0 ? b : 0.0;
      }
      // evaluated for every column and selected after: a guarded evaluation compiles to one
      // exec-masked branch per element, and the 16 independent exp chains of the 8-row block could
      // then not interleave (padding columns read finite cache entries or the clamped rows; their
      // values are dropped by the select)
      double ka, kb;
      if constexpr (RIN) {
        ka = skappa_r_k<OK>(a, inv_lo, s_o, ek);
        kb = skappa_r_k<OK>(b, inv_lo, s_o, ek);
      } else {
        ka = skappa_sq_k<OK>(a, inv_lo, s_o, ek);
        kb = skappa_sq_k<OK>(b, inv_lo, s_o, ek);
      }
      x[r].x = v0 ? ka : 0.0;
      x[r].y = v1 ? kb : 0.0;
    }
    auto step = [&](int r) __attribute__((always_inline)) {
      const double row = rg[(r0 + r) * 16 + (tid & 15)];
      double pa[SD], pb[SD];
      static_for<SD>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        double sa = 0.0, sb = 0.0;
        static_for<SD>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          sa = fmac_row<i * SD + q>(sa, row, ma[q]);
          sb = fmac_row<i * SD + q>(sb, row, mb[q]);
        });
        pa[i] = sa;
        pb[i] = sb;
      });
      const double ea = x[r].x - pa[0], eb = x[r].y - pb[0];
      const double rs = bcast_row<RR>(row);
      const double aa = ea * rs, ab = eb * rs;
      static_for<SD>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        ma[i] = fmac_row<RK + i>(pa[i], row, ea);
        mb[i] = fmac_row<RK + i>(pb[i], row, eb);
        ha[i] = fmac_row<RG + i>(ha[i], row, aa);
        hb[i] = fmac_row<RG + i>(hb[i], row, ab);
      });
      if (cola) {
        double2 o;
        o.x = aa;
        o.y = ab;
        typedef double v2d __attribute__((ext_vector_type(2)));
        v2d t;
        t.x = o.x;
        t.y = o.y;
        __builtin_nontemporal_store(t, reinterpret_cast<v2d*>(bp + (int64_t)(r0 + r) * ldb));
      }
    };
    if (r0 + kW2T <= nk) {
#pragma unroll
      for (int r = 0; r < kW2T; ++r) step(r);
    } else {   // the chunk's last rows (n not a multiple of 8): unrolled, uniform predicate
      const int nr = nk - r0;
#pragma unroll
      for (int r = 0; r < kW2T; ++r)
        if (r < nr) step(r);
    }
  }
  if (cola) {
#pragma unroll
    for (int i = 0; i < SD; ++i) {
      send[(j * mc + c) * kSStride + i] = ma[i];
      send[(j * mc + c + 1) * kSStride + i] = mb[i];
      if (hsum) {
        hsum[(j * mc + c) * kSStride + i] = ha[i];
        hsum[(j * mc + c + 1) * kSStride + i] = hb[i];
      }
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
#include <stdexcept>

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
                  double* out, int64_t ldo, bool take_sqrt) {
  if (n <= 0) return;
  const int rout = take_sqrt ? 1 : 0;
  if (out_kind == KM12) {
    dim3 grid((unsigned)((n + kDRows - 1) / kDRows), (unsigned)((mp + 255) / 256));
    dist2_direct_kernel<<<grid, 256, 0, st>>>(v, ldv, n, z, ldz, m, mp, d, out, ldo, rout);
  } else {
    dim3 grid((unsigned)((n + kDT - 1) / kDT), (unsigned)((mp + kDT - 1) / kDT));
    dist2_mfma_kernel<<<grid, 256, 0, st>>>(v, ldv, n, z, ldz, m, mp, d, zc, zc_stride(d), out, ldo,
                                            rout);
  }
}

template <int TK, int OK, bool RIN>
static void launch_wd2_k(hipStream_t st, dim3 grid, const double* rec, const double* src,
                         int64_t lds, int64_t m, int64_t mp, int64_t n, int L, double inv_lo,
                         double s_o, double* beta, int64_t ldb, double* send, int64_t mc,
                         const double* g, double* hsum, const double* tt, double l_t) {
  if (L > kW2MaxL || (lds & 1) || (ldb & 1))
    throw std::runtime_error("whiten_kfu_d2x2: chunk length > 256 or odd leading dimension");
  if (tt)
    whiten_kfu_d2x2<TK, OK, RIN, true><<<grid, 256, 0, st>>>(rec, src, lds, m, mp, n, L, inv_lo,
                                                             s_o, beta, ldb, send, mc, g, hsum,
                                                             exp_neg_consts(), tt, l_t);
  else
    whiten_kfu_d2x2<TK, OK, RIN, false><<<grid, 256, 0, st>>>(rec, src, lds, m, mp, n, L, inv_lo,
                                                              s_o, beta, ldb, send, mc, g, hsum,
                                                              exp_neg_consts(), nullptr, 0.0);
}

template <int TK>
static void launch_wd2_t(hipStream_t st, int ok, bool rin, dim3 grid, const double* rec,
                         const double* src, int64_t lds, int64_t m, int64_t mp, int64_t n, int L,
                         double inv_lo, double s_o, double* beta, int64_t ldb, double* send,
                         int64_t mc, const double* g, double* hsum, const double* tt, double l_t) {
#define WD2_ARGS st, grid, rec, src, lds, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum, tt, l_t
  if (rin) {
    switch (ok) {
      case KM12: launch_wd2_k<TK, KM12, true>(WD2_ARGS); break;
      case KM32: launch_wd2_k<TK, KM32, true>(WD2_ARGS); break;
      case KEQ: throw std::runtime_error("whiten_kfu_d2x2: EQ takes squared distances");
      default: launch_wd2_k<TK, KM52, true>(WD2_ARGS); break;
    }
  } else {
    switch (ok) {
      case KM12: launch_wd2_k<TK, KM12, false>(WD2_ARGS); break;
      case KM32: launch_wd2_k<TK, KM32, false>(WD2_ARGS); break;
      case KEQ: launch_wd2_k<TK, KEQ, false>(WD2_ARGS); break;
      default: launch_wd2_k<TK, KM52, false>(WD2_ARGS); break;
    }
  }
#undef WD2_ARGS
}


void launch_whiten_kfu_d2(hipStream_t st, int time_kind, int out_kind, const double* rec,
                          const double* src, int64_t lds, int64_t m, int64_t mp, int64_t n, int L,
                          int64_t nch, double inv_lo, double s_o, double* beta, int64_t ldb,
                          double* send, int64_t mc, const double* g, double* hsum, bool src_is_r,
                          const double* t_compact, double l_t) {
  dim3 grid((unsigned)nch, (unsigned)((mp + 511) / 512));
#define WD2T_ARGS st, out_kind, src_is_r, grid, rec, src, lds, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum, t_compact, l_t
  switch (time_kind) {
    case KM12: launch_wd2_t<KM12>(WD2T_ARGS); break;
    case KM32: launch_wd2_t<KM32>(WD2T_ARGS); break;
    default: launch_wd2_t<KM52>(WD2T_ARGS); break;
  }
#undef WD2T_ARGS
}

}  // namespace gpar
