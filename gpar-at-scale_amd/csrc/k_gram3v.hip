// k_gram3v.hip -- the v3 Gram's diagonal-block and chunk-correction kernels (layout and the OFF
// kernel: k_gram.hip, "v3: fat waves").  Their accumulators (DG: 18 tiles = 144 VGPRs; correction:
// 16 tiles = 128) fit the architectural VGPRs, and this file is compiled with VGPR-form MFMAs
// (-mllvm -amdgpu-mfma-vgpr-form, Makefile): with the default heuristic the compiler puts the
// MFMAs in AGPR form but carries some tiles across the K-loop in VGPRs, copying every
// accumulator twice per K-step.
#include "gram_common.hpp"

namespace gpar {

// DG(q): the lower triangle of diagonal 128-block q (panels 2q, 2q + 1), tiles split 18 + 18 over
// the two waves (gram_common.hpp); wave h stages panel 2q + h (slot h) and, for the r = beta^T
// alpha partials, reads that panel against the alpha rows staged with it.
__global__ __launch_bounds__(128) void gram3_dg_kernel(
    const double* __restrict__ beta, int64_t ldb, int64_t n, const double* __restrict__ alpha,
    int npan, int ndg, int sdg, int64_t rows, int64_t slot0, double* __restrict__ part,
    double* __restrict__ rpart, int bt_lo, int bt_cnt, int sw, int64_t rows_w,
    const GramGroupPtrs* __restrict__ grp) {
  if (grp) {
    const GramGroupPtrs& q = grp[blockIdx.y];
    beta = q.beta; alpha = q.alpha; part = q.part; rpart = q.rpart;
  }
  __shared__ __attribute__((aligned(16))) double smem[4 * kPanelD + 2 * 2 * kBK];
  double* ringa = smem + 4 * kPanelD;

  // work items [bt_lo, bt_lo + bt_cnt) of the ndg x sdg (group, split) items
  const int per = (bt_cnt + 7) >> 3;
  const int lb = ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);   // XCD-major deal
  if (lb >= bt_cnt) return;
  const int bt = bt_lo + lb;
  const int gid = bt % ndg, split = bt / ndg;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pA = 2 * gid + wave;

  // the first sw splits take rows_w rows each (the share that runs on the whitening CUs can be
  // sized apart from the rest), the others `rows`; both multiples of kBK
  const int64_t kb = split < sw ? (int64_t)split * rows_w
                                : (int64_t)sw * rows_w + (int64_t)(split - sw) * rows;
  int64_t ke = kb + (split < sw ? rows_w : rows);
  if (ke > n) ke = n;
  const int nsteps = (int)(ke > kb ? (ke - kb + kBK - 1) / kBK : 0);

  double racc4[4] = {0.0, 0.0, 0.0, 0.0};
  const int lq = lane >> 4, lc = lane & 15;
  const int hl = lane >> 5, cl2 = (lane & 31) * 2;
  const uint32_t boffA =
      (uint32_t)(((int64_t)hl * ldb + (int64_t)pA * kPW + (cl2 ^ (hl << 4))) * 8);
  const char* bbase = reinterpret_cast<const char*>(beta);
  const double* zrow = beta + n * ldb;   // a zero padding row (alpha rows past n read it)
  auto issue = [&](int s) __attribute__((always_inline)) {
    const int64_t k0 = kb + (int64_t)s * kBK;
    double* img = smem + ((s & 1) * 2 + wave) * kPanelD;
#pragma unroll
    for (int i = 0; i < kBK / 2; ++i) {
      const char* rowp = bbase + (k0 + 2 * i) * ldb * 8;
      __builtin_amdgcn_global_load_lds(rowp + boffA, img + 2 * i * kPW, 16, 0, 0);
    }
    if (lane < 32) {
      const int64_t kr = k0 + (lane >> 1);
      const unsigned* as = kr < n ? reinterpret_cast<const unsigned*>(alpha + kr) + (lane & 1)
                                  : reinterpret_cast<const unsigned*>(zrow);
      __builtin_amdgcn_global_load_lds(as, ringa + ((s & 1) * 2 + wave) * kBK, 4, 0, 0);
    }
  };
  const int frow = lane >> 4, fcol = lane & 15;
  const int par = frow & 1;
  auto foff = [&](int sl, int t) __attribute__((always_inline)) {
    return sl * kPanelD + frow * kPW + ((t ^ par) << 4) + fcol;
  };
  const int roff = wave * kPanelD + lq * kPW + lc;
  auto r_update = [&](int s, const double* base) __attribute__((always_inline)) {
    const double* ar = ringa + ((s & 1) * 2 + wave) * kBK;
    const double* im = base + roff;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const double av = ar[lq + 4 * i];
      const int rsw = (i * 4 + lq) & 1;
#pragma unroll
      for (int c = 0; c < 4; ++c) racc4[c] = fma(av, im[4 * i * kPW + ((c ^ rsw) << 4)], racc4[c]);
    }
  };

  if (nsteps > 0) issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  double* ptile = part + (((slot0 + bt) * 2 + wave) * kF3T) * 256;
  auto dg_body = [&](auto htag) __attribute__((always_inline)) {
    constexpr int H = decltype(htag)::value;
    constexpr int NA = d2_na<H>(), NB = d2_nb<H>();
    d4 acc[kD2T];
#pragma unroll
    for (int t = 0; t < kD2T; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
    int offa[NA], offb[NB];
#pragma unroll
    for (int ia = 0; ia < NA; ++ia) {
      const int r = d2_row<H>(ia);
      offa[ia] = foff(r >> 2, r & 3);
    }
#pragma unroll
    for (int c = 0; c < NB; ++c) offb[c] = foff(c >> 2, c & 3);
    for (int s = 0; s < nsteps; ++s) {
      if (s + 1 < nsteps) issue(s + 1);
      const double* base = smem + (s & 1) * 2 * kPanelD;
      double fa[2][NA], fb[2][NB];
#pragma unroll
      for (int ia = 0; ia < NA; ++ia) fa[0][ia] = base[offa[ia]];
#pragma unroll
      for (int c = 0; c < NB; ++c) fb[0][c] = base[offb[c]];
#pragma unroll
      for (int ks = 0; ks < kBK / 4; ++ks) {
        const int cur = ks & 1;
        if (ks + 1 < kBK / 4) {
#pragma unroll
          for (int ia = 0; ia < NA; ++ia) fa[cur ^ 1][ia] = base[offa[ia] + (ks + 1) * 4 * kPW];
#pragma unroll
          for (int c = 0; c < NB; ++c) fb[cur ^ 1][c] = base[offb[c] + (ks + 1) * 4 * kPW];
        }
#pragma unroll
        for (int ia = 0; ia < NA; ++ia)
#pragma unroll
          for (int c = 0; c <= d2_row<H>(ia); ++c)
            acc[d2_tile<H>(ia, c)] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                fa[cur][ia], fb[cur][c], acc[d2_tile<H>(ia, c)], 0, 0, 0);
      }
      r_update(s, base);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
#pragma unroll
    for (int t = 0; t < kD2T; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) ptile[t * 256 + (frow + 4 * r) * 16 + fcol] = acc[t][r];
  };
  if (wave == 0)
    dg_body(std::integral_constant<int, 0>{});
  else
    dg_body(std::integral_constant<int, 1>{});
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    double v = racc4[c];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lq == 0) rpart[(int64_t)split * npan * kPW + (int64_t)pA * kPW + c * 16 + lc] = v;
  }
}

// Chunk correction G += sum_j (E_j C_j^T + C_j E_j^T), r += sum_j C_j q_j (k_gram.hip header) over
// chunks [j0, j1) of correction split cs.  One 4-wave workgroup per (group, split); each wave
// owns a 64 x 64 block = 4 x 4 tiles:
//   * OFF(a, b): wave w -> rows of panel 2a + (w >> 1), columns 2b * 64 + (w & 1) * 64 ..;
//     its tiles land in the OFF partial slot of wave w >> 1, tile i * 8 + (w & 1) * 4 + c;
//   * DG(q): waves 0..2 -> the diagonal block's quadrants (0,0), (1,0), (1,1) (tiles above the
//     diagonal are computed and dropped); every wave also sums r for 32 of the block's columns.
// Operands straight from global memory: E_j / C_j are stored [column][4] per chunk, exactly the
// 16 x 4 (A) and 4 x 16 (B) MFMA fragments; chunk j + 1's are loaded under chunk j's MFMAs.
template <int D>
__global__ __launch_bounds__(256) void gram3_corr_kernel(
    const double* __restrict__ ecor, const double* __restrict__ cin, const double* __restrict__ qv,
    int64_t mc, int64_t nch, int npan, int noff, int ndg, int soff, int sdg, int ncs,
    double* __restrict__ part, double* __restrict__ rpart, const GramGroupPtrs* __restrict__ grp) {
  if (grp) {
    const GramGroupPtrs& q = grp[blockIdx.y];
    ecor = q.ecor; cin = q.cin; qv = q.qv; part = q.part; rpart = q.rpart;
  }
  const int ng = noff + ndg;
  const int g = (int)blockIdx.x % ng, cs = (int)blockIdx.x / ng;
  const int64_t j0 = (int64_t)cs * nch / ncs, j1 = (int64_t)(cs + 1) * nch / ncs;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int lq = lane >> 4, lc = lane & 15;
  const bool cv = lq < D;
  const int64_t cstride = mc * kSStride;

  const bool is_dg = g >= noff;
  int64_t row0, col0;   // first G row / column of this wave's 64 x 64 block
  int qr = 0, qc = 0;   // DG quadrant
  int a = 1, bo = 0;
  if (!is_dg) {
    while (a * (a + 1) / 2 <= g) ++a;
    bo = g - a * (a - 1) / 2;
    row0 = (int64_t)(2 * a + (wave >> 1)) * kPW;
    col0 = (int64_t)(2 * bo) * kPW + (wave & 1) * 64;
  } else {
    qr = wave == 0 ? 0 : 1;
    qc = wave == 2 ? 1 : 0;
    row0 = (int64_t)2 * (g - noff) * kPW + qr * 64;
    col0 = (int64_t)2 * (g - noff) * kPW + qc * 64;
  }
  const bool active = !is_dg || wave < 3;

  d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[i][c] = d4{0.0, 0.0, 0.0, 0.0};
  double racc[2] = {0.0, 0.0};
  const int64_t rcol0 = is_dg ? (int64_t)2 * (g - noff) * kPW + wave * 32 : 0;

  const int64_t oa = (row0 + lc) * kSStride + lq;
  const int64_t ob = (col0 + lc) * kSStride + lq;
  const int64_t orr = (rcol0 + lc) * kSStride + lq;
  double ea[4], ca[4], eb[4], cb[4], cr[2], qq = 0.0;
  auto ld = [&](int64_t jj) __attribute__((always_inline)) {
    const double* ej = ecor + jj * cstride;
    const double* cj = cin + jj * cstride;
    if (active) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        ea[t] = ej[oa + t * 16 * kSStride];
        ca[t] = cv ? cj[oa + t * 16 * kSStride] : 0.0;
        eb[t] = ej[ob + t * 16 * kSStride];
        cb[t] = cv ? cj[ob + t * 16 * kSStride] : 0.0;
      }
    }
    if (is_dg) {
#pragma unroll
      for (int h = 0; h < 2; ++h) cr[h] = cv ? cj[orr + h * 16 * kSStride] : 0.0;
      qq = cv ? qv[jj * 4 + lq] : 0.0;
    }
  };
  if (j0 < j1) ld(j0);
  for (int64_t jj = j0; jj < j1; ++jj) {
    double xa[4], ya[4], xb[4], yb[4], xr[2];
    const double xq = qq;
#pragma unroll
    for (int t = 0; t < 4; ++t) { xa[t] = ea[t]; ya[t] = ca[t]; xb[t] = eb[t]; yb[t] = cb[t]; }
    xr[0] = cr[0]; xr[1] = cr[1];
    if (jj + 1 < j1) ld(jj + 1);
    if (active) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[i][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[i], yb[c], acc[i][c], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[i][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya[i], xb[c], acc[i][c], 0, 0, 0);
    }
    if (is_dg) {
      racc[0] = fma(xr[0], xq, racc[0]);
      racc[1] = fma(xr[1], xq, racc[1]);
    }
  }

  const int frow = lane >> 4, fcol = lane & 15;
  if (!is_dg) {
    const int64_t slot = (int64_t)g + (int64_t)(soff + cs) * noff;
    double* ptile = part + ((slot * 2 + (wave >> 1)) * kF3T + (wave & 1) * 4) * 256;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ptile[(i * 8 + c) * 256 + (frow + 4 * r) * 16 + fcol] = acc[i][c][r];
    return;
  }
  const int64_t slot = (int64_t)noff * (soff + ncs) + (g - noff) + (int64_t)(sdg + cs) * ndg;
  if (active) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = qr * 4 + i;   // local tile row in the diagonal block
      const int h = d2_half_of(rr), tb = d2_base_of(rr);
      double* prow = part + ((slot * 2 + h) * kF3T + tb) * 256;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cc = qc * 4 + c;
        if (cc > rr) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) prow[cc * 256 + (frow + 4 * r) * 16 + fcol] = acc[i][c][r];
      }
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    double v = racc[h];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lq == 0) rpart[(int64_t)(sdg + cs) * npan * kPW + rcol0 + h * 16 + lc] = v;
  }
}

// Slim chunk correction, for running CONCURRENTLY with gram3_off_kernel on a second stream: a
// wave owns 2 x 4 tiles (64 accumulator VGPRs) and stays within the <= 124 registers per lane that
// the OFF wave (132 VGPRs + 256 AGPRs) leaves free on its SIMD, and it uses no LDS.  Grid:
// (noff + ndg) groups x 2 workgroups x ncs chunk splits, 4 waves each; the 8 waves of a group
// cover its 8 x 8 tiles as 2 x 4 blocks (row pair wg >> 1, column half wg & 1).  DG groups skip
// the two blocks above the diagonal and every wave sums r's chunk term for 16 of the block's
// columns.  Partial slots as gram3_corr_kernel.
template <int D>
__global__ __launch_bounds__(256) void gram3_corr_slim_kernel(
    const double* __restrict__ ecor, const double* __restrict__ cin, const double* __restrict__ qv,
    int64_t mc, int64_t nch, int npan, int noff, int ndg, int soff, int sdg, int ncs,
    double* __restrict__ part, double* __restrict__ rpart, const GramGroupPtrs* __restrict__ grp) {
  if (grp) {
    const GramGroupPtrs& q = grp[blockIdx.y];
    ecor = q.ecor; cin = q.cin; qv = q.qv; part = q.part; rpart = q.rpart;
  }
  const int ng = noff + ndg;
  const int g = (int)blockIdx.x % ng;
  const int hw = ((int)blockIdx.x / ng) & 1, cs = (int)blockIdx.x / (2 * ng);
  const int64_t j0 = (int64_t)cs * nch / ncs, j1 = (int64_t)(cs + 1) * nch / ncs;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wg = hw * 4 + wave;           // 0..7 within the group
  const int rb = wg >> 1, cb = wg & 1;    // row tiles 2 rb, 2 rb + 1; column tiles 4 cb .. 4 cb + 3
  const int lq = lane >> 4, lc = lane & 15;
  const bool cv = lq < D;
  const int64_t cstride = mc * kSStride;

  const bool is_dg = g >= noff;
  int64_t base_r, base_c;   // G row / column of local tile 0
  if (!is_dg) {
    int a = 1;
    while (a * (a + 1) / 2 <= g) ++a;
    const int bo = g - a * (a - 1) / 2;
    base_r = (int64_t)(2 * a) * kPW;
    base_c = (int64_t)(2 * bo) * kPW;
  } else {
    base_r = base_c = (int64_t)2 * (g - noff) * kPW;
  }
  const bool active = !is_dg || !(cb == 1 && rb < 2);

  d4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[i][c] = d4{0.0, 0.0, 0.0, 0.0};
  double racc = 0.0;
  // K-lane packing: chunk j contributes 2 d rank-1 terms, sum_q E[:, q] C[:, q]^T and
  // sum_q C[:, q] E[:, q]^T; two chunks' 4 d terms fill d MFMAs of K = 4 exactly (slot
  // s = 4 m + lane's k: chunk j + s / 2d, term u = s % 2d: u < d -> (E_u, C_u), else (C_u-d, E_u-d))
  // instead of 4 MFMAs with the state lanes q >= d zero.
  const int64_t ra = (base_r + rb * 32 + lc) * kSStride;   // row operand, column offset
  const int64_t rbo = (base_c + cb * 64 + lc) * kSStride;  // column operand
  const int64_t orr = (base_c + wg * 16 + lc) * kSStride + lq;
  for (int64_t jj = j0; jj < j1; jj += 2) {
    if (active) {
#pragma unroll
      for (int m = 0; m < D; ++m) {
        const int sl = 4 * m + lq;
        const int64_t ch = jj + sl / (2 * D);
        const int u = sl % (2 * D);
        const bool ok = ch < j1;
        const int q = u < D ? u : u - D;
        const double* srcA = (u < D ? ecor : cin) + (ok ? ch : jj) * cstride + q;
        const double* srcB = (u < D ? cin : ecor) + (ok ? ch : jj) * cstride + q;
        double fa[2], fb[4];
#pragma unroll
        for (int t = 0; t < 2; ++t) fa[t] = ok ? srcA[ra + t * 16 * kSStride] : 0.0;
#pragma unroll
        for (int t = 0; t < 4; ++t) fb[t] = ok ? srcB[rbo + t * 16 * kSStride] : 0.0;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            acc[i][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[i], fb[c], acc[i][c], 0, 0, 0);
      }
    }
    if (is_dg) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (jj + k < j1) {
          const double cr = cv ? cin[(jj + k) * cstride + orr] : 0.0;
          const double qq = cv ? qv[(jj + k) * 4 + lq] : 0.0;
          racc = fma(cr, qq, racc);
        }
      }
    }
  }

  const int frow = lane >> 4, fcol = lane & 15;
  if (!is_dg) {
    const int64_t slot = (int64_t)g + (int64_t)(soff + cs) * noff;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rr = rb * 2 + i;   // local row tile 0..7: OFF wave rr >> 2, tile row rr & 3
      double* prow = part + ((slot * 2 + (rr >> 2)) * kF3T + (rr & 3) * 8 + cb * 4) * 256;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) prow[c * 256 + (frow + 4 * r) * 16 + fcol] = acc[i][c][r];
    }
    return;
  }
  const int64_t slot = (int64_t)noff * (soff + ncs) + (g - noff) + (int64_t)(sdg + cs) * ndg;
  if (active) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rr = rb * 2 + i;
      const int h = d2_half_of(rr), tb = d2_base_of(rr);
      double* prow = part + ((slot * 2 + h) * kF3T + tb) * 256;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cc = cb * 4 + c;
        if (cc > rr) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) prow[cc * 256 + (frow + 4 * r) * 16 + fcol] = acc[i][c][r];
      }
    }
  }
  double v = racc;
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  if (lq == 0) rpart[(int64_t)(sdg + cs) * npan * kPW + base_c + wg * 16 + lc] = v;
}

void launch_gram3_corr_slim(hipStream_t st, int sdim, const double* ecor, const double* cin,
                            const double* qv, int64_t mc, int64_t nch, int npan, int noff, int ndg,
                            int soff, int sdg, int ncs, double* part, double* rpart,
                            const GramGroupPtrs* grp, int ngrp) {
  const dim3 nwg((unsigned)((noff + ndg) * 2 * ncs), (unsigned)ngrp);
#define GRAM3C_ARGS ecor, cin, qv, mc, nch, npan, noff, ndg, soff, sdg, ncs, part, rpart, grp
  switch (sdim) {
    case 1: gram3_corr_slim_kernel<1><<<nwg, 256, 0, st>>>(GRAM3C_ARGS); break;
    case 2: gram3_corr_slim_kernel<2><<<nwg, 256, 0, st>>>(GRAM3C_ARGS); break;
    default: gram3_corr_slim_kernel<3><<<nwg, 256, 0, st>>>(GRAM3C_ARGS); break;
  }
#undef GRAM3C_ARGS
}

void launch_gram3_dg(hipStream_t st, int nwg, const double* beta, int64_t ldb, int64_t n,
                     const double* alpha, int npan, int ndg, int sdg, int64_t rows,
                     int64_t slot0, double* part, double* rpart, int bt_lo, int bt_cnt, int sw,
                     int64_t rows_w, const GramGroupPtrs* grp, int ngrp) {
  if (bt_cnt < 0) bt_cnt = ndg * sdg - bt_lo;
  if (bt_cnt <= 0) return;
  if (nwg <= 0) nwg = ((bt_cnt + 7) / 8) * 8;
  gram3_dg_kernel<<<dim3((unsigned)nwg, (unsigned)ngrp), 128, 0, st>>>(
      beta, ldb, n, alpha, npan, ndg, sdg, rows, slot0, part, rpart, bt_lo, bt_cnt, sw, rows_w, grp);
}

void launch_gram3_corr(hipStream_t st, int sdim, const double* ecor, const double* cin,
                       const double* qv, int64_t mc, int64_t nch, int npan, int noff, int ndg,
                       int soff, int sdg, int ncs, double* part, double* rpart,
                       const GramGroupPtrs* grp, int ngrp) {
  const dim3 nwg((unsigned)((noff + ndg) * ncs), (unsigned)ngrp);
#define GRAM3C_ARGS ecor, cin, qv, mc, nch, npan, noff, ndg, soff, sdg, ncs, part, rpart, grp
  switch (sdim) {
    case 1: gram3_corr_kernel<1><<<nwg, 256, 0, st>>>(GRAM3C_ARGS); break;
    case 2: gram3_corr_kernel<2><<<nwg, 256, 0, st>>>(GRAM3C_ARGS); break;
    default: gram3_corr_kernel<3><<<nwg, 256, 0, st>>>(GRAM3C_ARGS); break;
  }
#undef GRAM3C_ARGS
}

}  // namespace gpar
