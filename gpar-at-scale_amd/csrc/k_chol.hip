// k_chol.hip -- blocked fp64 Cholesky, triangular inverse and the M x M products of the DTC
// dense tail on gfx950, batched over outputs.
//
// The reference factors cov(u) and Lambda with LAPACK on the CPU (dtc.jl:119-120,
// gpar_scaled_inference.jl:159,188).  Here an Mp x Mp SPD matrix (Mp a multiple of 64; the
// rows/columns past m are identity padding) is factored right-looking in 64 x 64 blocks:
//   potrf_diag   factor the diagonal block in LDS and invert it (T_kk = L_kk^-1)
//   potrf_panel  L_ik = A_ik T_kk^T                     (one workgroup per block row)
//   potrf_update A_ij -= L_ik L_jk^T, k < j <= i         (one workgroup per trailing tile)
// and the full inverse T = L^-1 follows block diagonal by block diagonal:
//   tinv_step    T_{j+d, j} = -T_{j+d, j+d} sum_{k=j}^{j+d-1} L_{j+d,k} T_{k,j}
// Every block product is a 64 x 64 x 64 v_mfma_f64_16x16x4_f64 tile from LDS: wave w owns rows
// 16w..16w+15, four 16 x 16 accumulators (C/D: col = lane & 15, row = (lane >> 4) + 4 r).
// Matrices are row-major, lower triangle meaningful, one Mp x Mp slab per problem.
#include "device_common.hpp"

namespace gpar {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kNB = 64;
constexpr int kSA = 66;   // LDS stride of a row-indexed (A) operand: conflict-free fragments
constexpr int kSB = 80;   // LDS stride of a k-indexed (B) operand

struct CholJob2 {
  double* A;        // Mp x Mp (ld) in: SPD lower; out: L
  double* T;        // Mp x Mp full inverse L^-1 (may be null unless tinv runs)
  double* Td;       // [nb][64 x 64] inverses of the diagonal blocks
  int* status;      // set to 1 on a non-positive pivot
};

// C(64x64) += A(64xK) B(Kx64) from LDS; wave w accumulates rows 16w.. into acc[ct].
__device__ __forceinline__ void mma64(const double* As, const double* Bs, d4 (&acc)[4], int lane,
                                      int wave, int kmax) {
  const int r = 16 * wave + (lane & 15);
  const int kq = lane >> 4;
  for (int k = 0; k < kmax; k += 4) {
    const double a = As[r * kSA + k + kq];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const double b = Bs[(k + kq) * kSB + ct * 16 + (lane & 15)];
      acc[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[ct], 0, 0, 0);
    }
  }
}

__device__ __forceinline__ void zero4(d4 (&acc)[4]) {
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) acc[ct] = d4{0.0, 0.0, 0.0, 0.0};
}

// load a 64 x 64 block (row-major, ld) into LDS as A operand (rows) or as B operand; trans:
// the block is stored transposed (S[k][c] = G[c][k]).
__device__ __forceinline__ void load_a(double* S, const double* G, int64_t ld, int tid) {
  for (int e = tid; e < kNB * kNB; e += 256) S[(e >> 6) * kSA + (e & 63)] = G[(int64_t)(e >> 6) * ld + (e & 63)];
}
__device__ __forceinline__ void load_b(double* S, const double* G, int64_t ld, int tid, bool trans) {
  if (!trans) {
    for (int e = tid; e < kNB * kNB; e += 256) S[(e >> 6) * kSB + (e & 63)] = G[(int64_t)(e >> 6) * ld + (e & 63)];
  } else {
    for (int e = tid; e < kNB * kNB; e += 256) S[(e & 63) * kSB + (e >> 6)] = G[(int64_t)(e >> 6) * ld + (e & 63)];
  }
}
// The same block loads split in two: global -> 16 registers per thread (issued before a block
// product, so the next k-step's loads are in flight under its MFMAs), then registers -> LDS.
struct BlkRegs {
  double v[16];
};
__device__ __forceinline__ void fetch_blk(BlkRegs& r, const double* G, int64_t ld, int tid) {
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = tid + 256 * u;
    r.v[u] = G[(int64_t)(e >> 6) * ld + (e & 63)];
  }
}
__device__ __forceinline__ void put_a(double* S, const BlkRegs& r, int tid) {
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = tid + 256 * u;
    S[(e >> 6) * kSA + (e & 63)] = r.v[u];
  }
}
__device__ __forceinline__ void put_b(double* S, const BlkRegs& r, int tid, bool trans) {
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = tid + 256 * u;
    if (!trans)
      S[(e >> 6) * kSB + (e & 63)] = r.v[u];
    else
      S[(e & 63) * kSB + (e >> 6)] = r.v[u];
  }
}
// store acc (optionally scaled) into a row-major global block: G = alpha * acc (+ G if add)
__device__ __forceinline__ void store_c(double* G, int64_t ld, const d4 (&acc)[4], int lane, int wave,
                                        double alpha, bool add) {
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * wave + (lane >> 4) + 4 * r, col = ct * 16 + (lane & 15);
      double* p = G + (int64_t)row * ld + col;
      *p = add ? fma(alpha, acc[ct][r], *p) : alpha * acc[ct][r];
    }
}

// ---------------------------------------------------------------- diagonal block
// The 64 x 64 diagonal block is factored by 256 threads: thread (row i = t & 63, class
// c = t >> 6) keeps the entries j = c + 4u (u < 16) of row i in registers.  Unscaled
// elimination: after step k, S_ij (j > k) holds A_ij - sum_{p<=k} A_ip A_jp / piv_p, and the
// entry that has just become final (column k + 1) is published to LDS, so every step is one
// barrier + 16 independent broadcast reads of column k.  Then the inverse T_kk = L_kk^-1,
// right-looking with the partial sums of row r in registers: row k of T is published, then
// every row r > k adds L_rk T_k. (one barrier per row).
constexpr int kSD = kNB + 1;

// 1 / p for p > 0: v_rcp_f64 seed + two Newton steps (~1 ulp)
__device__ __forceinline__ double rcp_pos(double p) {
  double r = __builtin_amdgcn_rcp(p);
  double e = fma(-p, r, 1.0);
  r = fma(r, e, r);
  e = fma(-p, r, 1.0);
  return fma(r, e, r);
}

// x of lane l, in every lane (two v_readlane_b32)
__device__ __forceinline__ double bcast_lane(double x, int l) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)v, l);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
  return __hiloint2double(hi, lo);
}

__global__ __launch_bounds__(256) void potrf_diag(const CholJob2* __restrict__ jobs, int64_t ld,
                                                  int kb, int want_t) {
  const CholJob2 jb = jobs[blockIdx.x];
  const int tid = threadIdx.x;
  __shared__ double S[kNB * kSD];
  __shared__ double dinv[kNB], dkk[kNB];
  double* Ablk = jb.A + (int64_t)kb * kNB * ld + (int64_t)kb * kNB;
  const int i = tid & 63;
  bool bad = false;
  // The elimination in one wave, lane i holding row i in registers: at step k every lane
  // publishes its column-k entry to LDS (one contiguous ds_write) and reads the pivot and the
  // column back as broadcasts -- a wave's LDS operations complete in order, so no barrier -- and
  // updates its row.  The same operations in the same order as the r05 form (four waves, row i's
  // 64 entries split over them, column k + 1 published through LDS behind a workgroup barrier
  // per step: 63 barriers, 71 us per 64 x 64 block, r06l probe; v_readlane broadcasts, 50 us),
  // so L is unchanged bit for bit.  Entries above the diagonal take the updates too (never read).
  __shared__ double colk[kNB];
  if (tid < 64) {
    double a[kNB];
#pragma unroll
    for (int c = 0; c < kNB; ++c) a[c] = c <= i ? Ablk[(int64_t)i * ld + c] : 0.0;
#pragma unroll
    for (int k = 0; k < kNB - 1; ++k) {
      colk[i] = a[k];
      double piv = colk[k];
      if (!(piv > 0.0)) { bad = true; piv = 1.0; }
      const double c = (i > k) ? a[k] * rcp_pos(piv) : 0.0;
#pragma unroll
      for (int j = k + 1; j < kNB; ++j) a[j] = fma(-c, colk[j], a[j]);
    }
#pragma unroll
    for (int c = 0; c < kNB; ++c) S[i * kSD + c] = a[c];
  }
  __syncthreads();
  if (!(S[(kNB - 1) * kSD + kNB - 1] > 0.0)) bad = true;
  // scale: L_kk = sqrt(piv_k), L_ik = A_ik / L_kk
  if (tid < kNB) {
    const double pv = S[tid * kSD + tid];
    const double dk = sqrt(pv > 0.0 ? pv : 1.0);
    dkk[tid] = dk;
    dinv[tid] = 1.0 / dk;
  }
  __syncthreads();
  for (int e = tid; e < kNB * kNB; e += 256) {
    const int r = e >> 6, c = e & 63;
    double v = 0.0;
    if (c < r) v = S[r * kSD + c] * dinv[c];
    else if (c == r) v = dkk[r];
    Ablk[(int64_t)r * ld + c] = v;
    if (c <= r) S[r * kSD + c] = v;
  }
  __syncthreads();
  // T = L^-1 by forward substitution in one wave, lane c holding column c in registers:
  // T_rc = -(sum_{k<r} L_rk T_kc) / L_rr, the L_rk broadcast from LDS.  The dot product is split
  // into four partial sums over k = c + q (mod 4), combined as (p0 + p1) + (p2 + p3) -- the r05
  // form's four lanes per column and their two shuffles, so T is unchanged bit for bit -- but
  // kept by k mod 4 (static registers; T_kc = 0 for k < c adds nothing) and relabelled per lane
  // at the end of each row.  (r05: one row per step behind a wave barrier, each step's k loop a
  // chain of dependent LDS reads: ~45 us of the 64 x 64 block.)
  if (tid < kNB) {
    const int c = tid, cr = c & 3;
    double tc[kNB];
#pragma unroll
    for (int r = 0; r < kNB; ++r) {
      double b4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k = 0; k < r; ++k) b4[k & 3] = fma(S[r * kSD + k], tc[k], b4[k & 3]);
      // p_q = b4[(q + c) & 3]
      const double p0 = cr == 0 ? b4[0] : cr == 1 ? b4[1] : cr == 2 ? b4[2] : b4[3];
      const double p1 = cr == 0 ? b4[1] : cr == 1 ? b4[2] : cr == 2 ? b4[3] : b4[0];
      const double p2 = cr == 0 ? b4[2] : cr == 1 ? b4[3] : cr == 2 ? b4[0] : b4[1];
      const double p3 = cr == 0 ? b4[3] : cr == 1 ? b4[0] : cr == 2 ? b4[1] : b4[2];
      const double acc = (p0 + p1) + (p2 + p3);
      tc[r] = r > c ? -acc * dinv[r] : (r == c ? dinv[r] : 0.0);
    }
    double* Td = jb.Td + (int64_t)kb * kNB * kNB;
    double* Tb = want_t ? jb.T + (int64_t)kb * kNB * ld + (int64_t)kb * kNB : nullptr;
#pragma unroll
    for (int r = 0; r < kNB; ++r) {
      Td[r * kNB + c] = tc[r];
      if (Tb) Tb[(int64_t)r * ld + c] = tc[r];
    }
  }
  if (bad && tid == 0) *jb.status = 1;
}

// ---------------------------------------------------------------- panel: L_ik = A_ik T_kk^T
__global__ __launch_bounds__(256) void potrf_panel(const CholJob2* __restrict__ jobs, int64_t ld,
                                                   int kb) {
  const CholJob2 jb = jobs[blockIdx.y];
  const int i = kb + 1 + blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ double As[kNB * kSA];
  __shared__ double Bs[kNB * kSB];
  double* Aik = jb.A + (int64_t)i * kNB * ld + (int64_t)kb * kNB;
  load_a(As, Aik, ld, tid);
  load_b(Bs, jb.Td + (int64_t)kb * kNB * kNB, kNB, tid, /*trans=*/true);
  __syncthreads();
  d4 acc[4];
  zero4(acc);
  mma64(As, Bs, acc, lane, wave, kNB);
  __syncthreads();
  store_c(Aik, ld, acc, lane, wave, 1.0, false);
}

// ---------------------------------------------------------------- trailing: A_ij -= L_ik L_jk^T
__global__ __launch_bounds__(256) void potrf_update(const CholJob2* __restrict__ jobs, int64_t ld,
                                                    int kb) {
  const CholJob2 jb = jobs[blockIdx.y];
  int t = blockIdx.x, a = 0;
  while ((a + 1) * (a + 2) / 2 <= t) ++a;
  const int i = kb + 1 + a, j = kb + 1 + (t - a * (a + 1) / 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ double As[kNB * kSA];
  __shared__ double Bs[kNB * kSB];
  load_a(As, jb.A + (int64_t)i * kNB * ld + (int64_t)kb * kNB, ld, tid);
  load_b(Bs, jb.A + (int64_t)j * kNB * ld + (int64_t)kb * kNB, ld, tid, /*trans=*/true);
  __syncthreads();
  d4 acc[4];
  zero4(acc);
  mma64(As, Bs, acc, lane, wave, kNB);
  store_c(jb.A + (int64_t)i * kNB * ld + (int64_t)j * kNB, ld, acc, lane, wave, -1.0, true);
}

// ---------------------------------------------------------------- inverse, block diagonal d
__global__ __launch_bounds__(256) void tinv_step(const CholJob2* __restrict__ jobs, int64_t ld, int d) {
  const CholJob2 jb = jobs[blockIdx.y];
  const int j = blockIdx.x, i = j + d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ double As[kNB * kSA];
  __shared__ double Bs[kNB * kSB];
  d4 acc[4];
  zero4(acc);
  // L_ik and T_kj of step k + 1 are fetched into registers under step k's block product
  BlkRegs ra, rb;
  fetch_blk(ra, jb.A + (int64_t)i * kNB * ld + (int64_t)j * kNB, ld, tid);   // L_ij
  fetch_blk(rb, jb.T + (int64_t)j * kNB * ld + (int64_t)j * kNB, ld, tid);   // T_jj
  for (int k = j; k < i; ++k) {
    __syncthreads();
    put_a(As, ra, tid);
    put_b(Bs, rb, tid, false);
    __syncthreads();
    if (k + 1 < i) {
      fetch_blk(ra, jb.A + (int64_t)i * kNB * ld + (int64_t)(k + 1) * kNB, ld, tid);
      fetch_blk(rb, jb.T + (int64_t)(k + 1) * kNB * ld + (int64_t)j * kNB, ld, tid);
    }
    mma64(As, Bs, acc, lane, wave, kNB);
  }
  __syncthreads();
  // S -> Bs, T_ii -> As, T_ij = -T_ii S
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      Bs[(16 * wave + (lane >> 4) + 4 * r) * kSB + ct * 16 + (lane & 15)] = acc[ct][r];
  load_a(As, jb.Td + (int64_t)i * kNB * kNB, kNB, tid);
  __syncthreads();
  zero4(acc);
  mma64(As, Bs, acc, lane, wave, kNB);
  store_c(jb.T + (int64_t)i * kNB * ld + (int64_t)j * kNB, ld, acc, lane, wave, -1.0, false);
}

// ---------------------------------------------------------------- Lambda = T G T^T + I
// mode 0: X = T G (all tiles; T lower: k <= i).  mode 1: Lam = X T^T + I (tiles i >= j; k <= j).
struct TgtJob {
  const double* T;
  const double* G;
  double* X;
  double* Lam;
};
__global__ __launch_bounds__(256) void tgt_kernel(const TgtJob* __restrict__ jobs, int64_t ld, int nb,
                                                  int mode) {
  const TgtJob jb = jobs[blockIdx.y];
  int i, j;
  if (mode == 0) {
    i = blockIdx.x / nb;
    j = blockIdx.x % nb;
  } else {
    int t = blockIdx.x, a = 0;
    while ((a + 1) * (a + 2) / 2 <= t) ++a;
    i = a;
    j = t - a * (a + 1) / 2;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ double As[kNB * kSA];
  __shared__ double Bs[kNB * kSB];
  d4 acc[4];
  zero4(acc);
  const int kend = (mode == 0) ? i : j;
  // the operands of step k: mode 0 T_ik, G_kj; mode 1 X_ik, T_jk (transposed into LDS); step
  // k + 1's are fetched into registers under step k's block product
  auto src_a = [&](int k) {
    return (mode == 0 ? jb.T : jb.X) + (int64_t)i * kNB * ld + (int64_t)k * kNB;
  };
  auto src_b = [&](int k) {
    return mode == 0 ? jb.G + (int64_t)k * kNB * ld + (int64_t)j * kNB
                     : jb.T + (int64_t)j * kNB * ld + (int64_t)k * kNB;
  };
  BlkRegs ra, rb;
  fetch_blk(ra, src_a(0), ld, tid);
  fetch_blk(rb, src_b(0), ld, tid);
  for (int k = 0; k <= kend; ++k) {
    __syncthreads();
    put_a(As, ra, tid);
    put_b(Bs, rb, tid, mode != 0);
    __syncthreads();
    if (k + 1 <= kend) {
      fetch_blk(ra, src_a(k + 1), ld, tid);
      fetch_blk(rb, src_b(k + 1), ld, tid);
    }
    mma64(As, Bs, acc, lane, wave, kNB);
  }
  if (mode == 0) {
    store_c(jb.X + (int64_t)i * kNB * ld + (int64_t)j * kNB, ld, acc, lane, wave, 1.0, false);
  } else {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * wave + (lane >> 4) + 4 * r, col = ct * 16 + (lane & 15);
        const double v = acc[ct][r] + ((i == j && row == col) ? 1.0 : 0.0);
        jb.Lam[(int64_t)(i * kNB + row) * ld + j * kNB + col] = v;
      }
  }
}

// ---------------------------------------------------------------- DTC finish
// dtc = -1/2 [N log 2pi + sum log S + 2 sum log diag L_lam + |alpha|^2 - |L_lam^-1 T_u r|^2]
// (dtc.jl:122-125; A alpha = L_u^-1 beta^T alpha = T_u r).  b = T_u r by rows (one wave per
// row, coalesced), then the blocked forward solve with the diagonal-block inverses of L_lam.
// q(u) mode (me != null): m_e = L_lam^-T L_lam^-1 b via the same blocks, backward.
struct Finish2Job {
  const double* Tu;      // L_u^-1 (full lower)
  const double* Llam;    // chol(Lambda)
  const double* Tdl;     // [nb][64 x 64] inverses of L_lam's diagonal blocks
  const double* r;       // beta^T alpha (mp)
  const double* logs;    // per-chunk sum log S
  int64_t nch;
  const double* a2part;  // per-block partial sums of alpha^2
  int64_t npart;
  int64_t n;
  const int* status;     // 2 flags
  double* out;           // dtc
  double* me;            // q(u): m_e (mp) when non-null
};

__global__ __launch_bounds__(256) void finish2_kernel(const Finish2Job* __restrict__ jobs, int64_t ld,
                                                      int nb) {
  const Finish2Job jb = jobs[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mp = nb * kNB;
  __shared__ double b[2048], w[2048], red[4][4];
  // b = T_u r: groups of 16 rows per wave, lanes along k, 16 independent loads in flight per lane
  // (one row at a time, each row's loads then its reduction, was a chain of HBM latencies)
  for (int g = wave; g < mp / 16; g += 4) {
    double s16[16];
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) s16[rr] = 0.0;
    const int kcn = (16 * g + 15) / kNB + 1;
    for (int kc = 0; kc < kcn; ++kc) {
      const int k = kc * kNB + lane;
      const double rk = jb.r[k];
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int row = 16 * g + rr;
        const double tv = jb.Tu[(int64_t)row * ld + k];
        s16[rr] = fma(k <= row ? tv : 0.0, rk, s16[rr]);
      }
    }
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      const double v = wave_sum(s16[rr]);
      if (lane == 0) b[16 * g + rr] = v;
    }
  }
  __syncthreads();
  __shared__ double part[kNB];
  __shared__ double Tds[kNB * kSD];
  __shared__ double partq[4][64];
  // Forward solve L_lam w = b block by block: part = b_I - sum_{J<I} L_IJ w_J, then w_I = Td_I part.
  // Each wave takes 16 of the block's rows with its lanes along k (coalesced 512-byte row segments,
  // 16 independent loads in flight per lane) and reduces them across the lanes; Td_I's product
  // splits k over the four waves.  (r05: four threads per row walked k with stride 4, each step a
  // dependent global load: 0.31 ms per round of 8 outputs at the eeg shard, r06i trace.)
  for (int I = 0; I < nb; ++I) {
    const int row = tid & 63, q = tid >> 6;
    const double* Td = jb.Tdl + (int64_t)I * kNB * kNB;
    for (int e = tid; e < kNB * kNB; e += 256) Tds[(e >> 6) * kSD + (e & 63)] = Td[e];
    double s16[16];
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) s16[rr] = 0.0;
    const double* L0 = jb.Llam + (int64_t)(I * kNB + 16 * wave) * ld;
    for (int kc = 0; kc < I; ++kc) {
      const int k = kc * kNB + lane;
      const double wk = w[k];
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) s16[rr] = fma(L0[(int64_t)rr * ld + k], wk, s16[rr]);
    }
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      const double v = wave_sum(s16[rr]);
      if (lane == 0) part[16 * wave + rr] = b[I * kNB + 16 * wave + rr] - v;
    }
    __syncthreads();
    double acc = 0.0;
    for (int k = q; k <= row; k += 4) acc = fma(Tds[row * kSD + k], part[k], acc);
    partq[q][row] = acc;
    __syncthreads();
    if (q == 0) w[I * kNB + row] = (partq[0][row] + partq[1][row]) + (partq[2][row] + partq[3][row]);
    __syncthreads();
  }
  if (jb.me) {
    // backward: x_I = Td_I^T (w_I - sum_{J>I} L_JI^T x_J) (lanes along the block's columns:
    // coalesced rows of L), x stored in b
    __shared__ double part2[4][kNB];
    for (int I = nb - 1; I >= 0; --I) {
      const int row = tid & 63, q = tid >> 6;
      double s = 0.0;
      for (int k = (I + 1) * kNB + q; k < mp; k += 4)
        s = fma(jb.Llam[(int64_t)k * ld + I * kNB + row], b[k], s);
      part2[q][row] = s;
      const double* Td = jb.Tdl + (int64_t)I * kNB * kNB;
      for (int e = tid; e < kNB * kNB; e += 256) Tds[(e >> 6) * kSD + (e & 63)] = Td[e];
      __syncthreads();
      if (q == 0) part[row] = w[I * kNB + row] - (part2[0][row] + part2[1][row] + part2[2][row] + part2[3][row]);
      __syncthreads();
      if (q == 0) {
        double acc = 0.0;
        for (int k = row; k < kNB; ++k) acc = fma(Tds[k * kSD + row], part[k], acc);
        b[I * kNB + row] = acc;
      }
      __syncthreads();
    }
    for (int i = tid; i < mp; i += 256) jb.me[i] = b[i];
    return;
  }
  double ldl = 0.0, vv = 0.0, ls = 0.0, a2 = 0.0;
  for (int i = tid; i < mp; i += 256) {
    ldl += log(jb.Llam[(int64_t)i * ld + i]);
    vv = fma(w[i], w[i], vv);
  }
  for (int64_t j = tid; j < jb.nch; j += 256) ls += jb.logs[j];
  for (int64_t j = tid; j < jb.npart; j += 256) a2 += jb.a2part[j];
  ldl = wave_sum(ldl);
  vv = wave_sum(vv);
  ls = wave_sum(ls);
  a2 = wave_sum(a2);
  if (lane == 0) {
    red[wave][0] = ldl;
    red[wave][1] = vv;
    red[wave][2] = ls;
    red[wave][3] = a2;
  }
  __syncthreads();
  if (tid == 0) {
    double s[4] = {0, 0, 0, 0};
    for (int q = 0; q < 4; ++q)
      for (int c = 0; c < 4; ++c) s[c] += red[q][c];
    const double tmp = s[2] + 2.0 * s[0] + s[3] - s[1];
    double dtc = -((double)jb.n * kLog2Pi + tmp) / 2.0;
    if (jb.status[0] || jb.status[1]) dtc = __builtin_nan("");
    *jb.out = dtc;
  }
}

// y_j = sum_{i >= j} T_ij x_i (T lower, row-major ld): one thread per column, coalesced rows.
__global__ __launch_bounds__(256) void gemv_tn_lower(const double* __restrict__ T, int64_t ld, int mp,
                                                     const double* __restrict__ x, double* __restrict__ y) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= mp) return;
  double s = 0.0;
  for (int i = j; i < mp; ++i) s = fma(T[(int64_t)i * ld + j], x[i], s);
  y[j] = s;
}

}  // namespace gpar

// ============================================================================ launch wrappers
#include "launch.hpp"

namespace gpar {

// Factor every problem's Mp x Mp matrix in place (and its full inverse when want_t).
void launch_chol_blocked(hipStream_t st, const CholJob2Host* jobs_dev, int njobs, int64_t ld,
                         int nb, bool want_t) {
  const auto* jobs = reinterpret_cast<const CholJob2*>(jobs_dev);
  for (int kb = 0; kb < nb; ++kb) {
    potrf_diag<<<njobs, 256, 0, st>>>(jobs, ld, kb, want_t ? 1 : 0);
    const int rows = nb - kb - 1;
    if (rows > 0) {
      potrf_panel<<<dim3(rows, njobs), 256, 0, st>>>(jobs, ld, kb);
      potrf_update<<<dim3(rows * (rows + 1) / 2, njobs), 256, 0, st>>>(jobs, ld, kb);
    }
  }
  if (want_t)
    for (int d = 1; d < nb; ++d) tinv_step<<<dim3(nb - d, njobs), 256, 0, st>>>(jobs, ld, d);
}

void launch_tgt(hipStream_t st, const TgtJobHost* jobs_dev, int njobs, int64_t ld, int nb) {
  const auto* jobs = reinterpret_cast<const TgtJob*>(jobs_dev);
  tgt_kernel<<<dim3(nb * nb, njobs), 256, 0, st>>>(jobs, ld, nb, 0);
  tgt_kernel<<<dim3(nb * (nb + 1) / 2, njobs), 256, 0, st>>>(jobs, ld, nb, 1);
}

void launch_tg(hipStream_t st, const TgtJobHost* jobs_dev, int njobs, int64_t ld, int nb) {
  tgt_kernel<<<dim3(nb * nb, njobs), 256, 0, st>>>(reinterpret_cast<const TgtJob*>(jobs_dev), ld, nb, 0);
}

void launch_gemv_tn_lower(hipStream_t st, const double* T, int64_t ld, int mp, const double* x,
                          double* y) {
  gemv_tn_lower<<<(mp + 255) / 256, 256, 0, st>>>(T, ld, mp, x, y);
}

void launch_finish2(hipStream_t st, const Finish2JobHost* jobs_dev, int njobs, int64_t ld, int nb) {
  finish2_kernel<<<njobs, 256, 0, st>>>(reinterpret_cast<const Finish2Job*>(jobs_dev), ld, nb);
}

}  // namespace gpar
