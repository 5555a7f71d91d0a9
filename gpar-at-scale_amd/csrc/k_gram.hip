// k_gram.hip -- the dominant contraction of the DTC objective on fp64 MFMA.
//
// G = beta^T beta (M x M) and r = beta^T alpha over N time steps, where
// beta[k, c] = beta_loc[k, c] + g_k . cin[chunk(k)][c] applies the chunk fix-up of the
// time-chunked Kalman whitening on the fly (k_lgssm.hip), so the corrected beta is never
// written to HBM.  In the reference this is the M x M x N trsm + gemm of dtc.jl:119-120
// (A = L_u^{-1} beta^T; Lambda = A A^T + I), which the build reassociates as
// Lambda = L_u^{-1} (beta^T beta) L_u^{-T} + I.
//
// Tiling: one 256-thread workgroup = one 128 x 128 lower-triangle tile of G over one
// split of the time axis (split-K).  4 waves as 2 x 2, each 64 x 64 = 4 x 4 MFMA tiles of
// v_mfma_f64_16x16x4_f64 (C/D: col = lane & 15, row = (lane >> 4) + 4 * reg).
// K-step = 16 time rows staged global -> VGPR (fix-up) -> LDS, double buffered.
// Blocks of one split run on one XCD group (blockIdx % 8) so the split's rows are
// shared through that XCD's L2 by its tiles.
#include "device_common.hpp"

namespace gpar {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kGT = 128;          // tile edge
constexpr int kBK = 16;           // time rows per K-step
constexpr int kLdsStride = 144;   // padded LDS row (doubles): rows r and r+1 hit opposite bank halves
#ifndef GRAM_VARIANT
#define GRAM_VARIANT 0   // ablation builds only (scratch/gram_bench): 1 no fix-up, 2 no beta loads, 3 no MFMA, 4 no staging
#endif

template <int D>
__global__ __launch_bounds__(256, 2) void gram_kernel(
    const double* __restrict__ beta, int64_t ldb, int64_t n, const double* __restrict__ g,
    const double* __restrict__ cin, int64_t mc, int L, const double* __restrict__ alpha,
    int ntb, int ntiles, int nsplit, int64_t rows_per_split, double* __restrict__ part,
    double* __restrict__ rpart) {
  // one LDS array: [2 buf][2 operand][kBK rows x kLdsStride] | g/alpha ring [2][kBK][4 + 1] | r reduce [128]
  constexpr int kTileD = kBK * kLdsStride;
  constexpr int kGRing = kBK * 5;
  __shared__ __attribute__((aligned(16))) double smem[4 * kTileD + 2 * kGRing + 128];
  double* rred = smem + 4 * kTileD + 2 * kGRing;

  // XCD-aware decode: blocks b and b+8 share an XCD; give each XCD group whole splits.
  const int b = blockIdx.x;
  const int xg = b & 7;
  const int q = b >> 3;
  const int split = (q / ntiles) * 8 + xg;
  const int tile = q % ntiles;
  if (split >= nsplit) return;
  int ti = 0;
  while ((ti + 1) * (ti + 2) / 2 <= tile) ++ti;
  const int tj = tile - ti * (ti + 1) / 2;
  const bool diag = (ti == tj);
  const int64_t i0 = (int64_t)ti * kGT, j0 = (int64_t)tj * kGT;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int sc = tid & 127;   // staging column
  const int rg = tid >> 7;    // staging row group (wave-uniform)
  const int rgu = __builtin_amdgcn_readfirstlane(rg);

  const int64_t kb = (int64_t)split * rows_per_split;
  int64_t ke = kb + rows_per_split;
  if (ke > n) ke = n;

  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = d4{0.0, 0.0, 0.0, 0.0};

  double racc = 0.0;
  double gpre = 0.0;
  struct Regs {
    double bI[8], bJ[8], cI[D], cJ[D];
  };
  Regs RA, RB;

  // Pipeline (one barrier per K-step, beta loads two K-steps ahead):
  //   load(s+2)          raw beta / carry loads into the free register set
  //   gload(s+2)         the K-step's g_k rows + alpha_k (80 doubles, one per thread)
  //   MFMAs(s)           from lds[s & 1], interleaved with
  //   store_rows(s+1)    fix-up beta += g_k . c_chunk (g from the LDS ring) -> lds[(s+1) & 1]
  //   gstore(s+2)        ring slot (s+2) & 1 == s & 1, last read by store_rows(s) a barrier ago
  // A global load consumed soon after issue stalls the wave (hipcc waits vmcnt), so every
  // beta load has one full MFMA phase plus one barrier to land.  Rows past the split are
  // clamped + masked (branch-free).
  auto load = [&](Regs& R, int64_t k0) {
    const int64_t ch = k0 / L;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      R.cI[i] = cin[(ch * mc + i0 + sc) * kSStride + i];
      R.cJ[i] = cin[(ch * mc + j0 + sc) * kSStride + i];
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int64_t k = k0 + rgu + 2 * r;
      const int64_t kc = (k < n) ? k : n - 1;
#if GRAM_VARIANT == 2
      R.bI[r] = (double)kc;
      R.bJ[r] = (double)kc;
#else
      R.bI[r] = beta[kc * ldb + i0 + sc];
      R.bJ[r] = beta[kc * ldb + j0 + sc];
#endif
    }
  };
  auto gload = [&](int64_t k0) {
    if (tid < kBK * 5) {
      const int row = tid / 5, col = tid % 5;
      const int64_t k = k0 + row;
      const int64_t kc = (k < n) ? k : n - 1;
      gpre = (col < 4) ? g[kc * kGStride + col] : alpha[kc];
    }
  };
  auto gstore = [&](int slot) {
    if (tid < kBK * 5) smem[4 * kTileD + slot * kGRing + tid] = gpre;
  };
  auto store_rows = [&](const Regs& R, int64_t k0, int buf, int r0, int nr) {
    const double* gr = smem + 4 * kTileD + buf * kGRing;
    double* ldsI = smem + (buf * 2 + 0) * kTileD;
    double* ldsJ = smem + (buf * 2 + 1) * kTileD;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (r < r0 || r >= r0 + nr) continue;
      const int row = rgu + 2 * r;
      const int64_t k = k0 + row;
      const double msk = (k < ke) ? 1.0 : 0.0;
      double vi = R.bI[r], vj = R.bJ[r];
#if GRAM_VARIANT != 1
#pragma unroll
      for (int i = 0; i < D; ++i) {
        const double gi = gr[row * 5 + i];
        vi = fma(gi, R.cI[i], vi);
        vj = fma(gi, R.cJ[i], vj);
      }
#endif
      vi *= msk;
      racc = fma(gr[row * 5 + 4], vi, racc);
      ldsI[row * kLdsStride + sc] = vi;
      ldsJ[row * kLdsStride + sc] = vj * msk;
    }
  };

  const int nsteps = (int)((ke - kb + kBK - 1) / kBK);
  const int frow = lane >> 4, fcol = lane & 15;
  if (nsteps > 0) {
    gload(kb);
    load(RA, kb);
    gstore(0);
    if (nsteps > 1) {
      gload(kb + kBK);
      load(RB, kb + kBK);
    }
    __syncthreads();
    store_rows(RA, kb, 0, 0, 8);
    if (nsteps > 1) gstore(1);
  }
  __syncthreads();
  // one K-step: Rcur holds step s+1 (staged during the MFMAs), Rnxt receives step s+2
  auto kstep = [&](int s, const Regs& Rcur, Regs& Rnxt) {
    const int buf = s & 1;
    const bool more = (s + 1) < nsteps;
    const bool more2 = (s + 2) < nsteps;
#if GRAM_VARIANT != 4
    if (more2) load(Rnxt, kb + (int64_t)(s + 2) * kBK);
#endif
    if (more2) gload(kb + (int64_t)(s + 2) * kBK);
    const double* la = smem + (buf * 2 + 0) * kTileD;
    const double* lb = smem + (buf * 2 + 1) * kTileD;
    const int64_t kn = kb + (int64_t)(s + 1) * kBK;
#pragma unroll
    for (int ks = 0; ks < kBK / 4; ++ks) {
      double fa[4], fb[4];
      const int row = ks * 4 + frow;
#pragma unroll
      for (int a = 0; a < 4; ++a) fa[a] = la[row * kLdsStride + wr * 64 + a * 16 + fcol];
#pragma unroll
      for (int c = 0; c < 4; ++c) fb[c] = lb[row * kLdsStride + wc * 64 + c * 16 + fcol];
#if GRAM_VARIANT == 3
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[a][c][0] += fa[a] * fb[c];
#else
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[a][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[a], fb[c], acc[a][c], 0, 0, 0);
#endif
#if GRAM_VARIANT != 4
      if (more) store_rows(Rcur, kn, buf ^ 1, 2 * ks, 2);
#endif
    }
    if (more2) gstore(buf);
    __syncthreads();
  };
  for (int s = 0; s < nsteps; s += 2) {
    kstep(s, RB, RA);
    if (s + 1 < nsteps) kstep(s + 1, RA, RB);
  }

  double* pt = part + ((int64_t)split * ntiles + tile) * (kGT * kGT);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 64 + a * 16 + frow + 4 * r;
        const int col = wc * 64 + c * 16 + fcol;
        pt[row * kGT + col] = acc[a][c][r];
      }
  if (diag) {
    if (rg == 1) rred[sc] = racc;
    __syncthreads();
    if (rg == 0) rpart[((int64_t)split * ntb + ti) * kGT + sc] = racc + rred[sc];
  }
}

// Sum split partials in split order (deterministic) into the full symmetric G (ldg) and r.
__global__ __launch_bounds__(256) void gram_reduce(const double* __restrict__ part,
                                                   const double* __restrict__ rpart, int ntb,
                                                   int ntiles, int nsplit, double* __restrict__ G,
                                                   int64_t ldg, double* __restrict__ r) {
  const int tile = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;   // element within the tile
  int ti = 0;
  while ((ti + 1) * (ti + 2) / 2 <= tile) ++ti;
  const int tj = tile - ti * (ti + 1) / 2;
  if (e < kGT * kGT && !(ti == tj && e / kGT < e % kGT)) {
    double s = 0.0;
    for (int sp = 0; sp < nsplit; ++sp) s += part[((int64_t)sp * ntiles + tile) * (kGT * kGT) + e];
    const int64_t row = (int64_t)ti * kGT + e / kGT, col = (int64_t)tj * kGT + e % kGT;
    G[row * ldg + col] = s;
    G[col * ldg + row] = s;
  }
  if (ti == tj && blockIdx.x == 0 && threadIdx.x < kGT) {
    double s = 0.0;
    for (int sp = 0; sp < nsplit; ++sp) s += rpart[((int64_t)sp * ntb + ti) * kGT + threadIdx.x];
    r[(int64_t)ti * kGT + threadIdx.x] = s;
  }
}

// Materialise the corrected beta (only for the (dtc, A) parity entry point).
template <int D>
__global__ __launch_bounds__(256) void beta_fix_kernel(double* __restrict__ beta, int64_t ldb,
                                                       int64_t n, const double* __restrict__ g,
                                                       const double* __restrict__ cin, int64_t mc,
                                                       int L) {
  const int64_t e = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (e >= n * ldb) return;
  const int64_t k = e / ldb, c = e % ldb;
  const int64_t ch = k / L;
  double v = beta[e];
#pragma unroll
  for (int i = 0; i < D; ++i) v = fma(g[k * kGStride + i], cin[(ch * mc + c) * kSStride + i], v);
  beta[e] = v;
}

}  // namespace gpar

// ============================================================================ launch wrappers
#include "launch.hpp"

namespace gpar {

GramPlan gram_plan(int64_t n, int64_t mp) {
  GramPlan p;
  p.ntb = (int)(mp / kGT);
  p.ntiles = p.ntb * (p.ntb + 1) / 2;
  int ns = 512 / p.ntiles;
  ns = (ns / 8) * 8;
  if (ns < 8) ns = 8;
  int64_t maxs = (n + 255) / 256;          // keep >= 256 rows per split
  if (maxs < 8) maxs = 8;
  if (ns > maxs) ns = (int)((maxs / 8) * 8);
  if (ns < 8) ns = 8;
  p.nsplit = ns;
  int64_t rps = (n + ns - 1) / ns;
  rps = ((rps + kBK - 1) / kBK) * kBK;
  p.rows_per_split = rps;
  return p;
}

void launch_gram(hipStream_t st, int sdim, const GramPlan& plan, const double* beta,
                 int64_t ldb, int64_t n, const double* g, const double* cin, int64_t mc, int L,
                 const double* alpha, double* part, double* rpart, double* G, int64_t ldg,
                 double* r) {
  const int nblk = plan.ntiles * plan.nsplit;

  switch (sdim) {
    case 1: gram_kernel<1><<<nblk, 256, 0, st>>>(beta, ldb, n, g, cin, mc, L, alpha, plan.ntb, plan.ntiles, plan.nsplit, plan.rows_per_split, part, rpart); break;
    case 2: gram_kernel<2><<<nblk, 256, 0, st>>>(beta, ldb, n, g, cin, mc, L, alpha, plan.ntb, plan.ntiles, plan.nsplit, plan.rows_per_split, part, rpart); break;
    default: gram_kernel<3><<<nblk, 256, 0, st>>>(beta, ldb, n, g, cin, mc, L, alpha, plan.ntb, plan.ntiles, plan.nsplit, plan.rows_per_split, part, rpart); break;
  }
  dim3 rgrid((kGT * kGT + 255) / 256, plan.ntiles);
  gram_reduce<<<rgrid, 256, 0, st>>>(part, rpart, plan.ntb, plan.ntiles, plan.nsplit, G, ldg, r);
}

void launch_beta_fix(hipStream_t st, int sdim, double* beta, int64_t ldb, int64_t n,
                     const double* g, const double* cin, int64_t mc, int L) {
  const unsigned nb = (unsigned)((n * ldb + 255) / 256);
  switch (sdim) {
    case 1: beta_fix_kernel<1><<<nb, 256, 0, st>>>(beta, ldb, n, g, cin, mc, L); break;
    case 2: beta_fix_kernel<2><<<nb, 256, 0, st>>>(beta, ldb, n, g, cin, mc, L); break;
    default: beta_fix_kernel<3><<<nb, 256, 0, st>>>(beta, ldb, n, g, cin, mc, L); break;
  }
}

}  // namespace gpar
