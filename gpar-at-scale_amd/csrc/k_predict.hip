// k_predict.hip -- scaled-GPAR prediction (gpar_scaled_inference.jl:63-135) on gfx950.
//
// The reference draws e ~ q(u), forms f_x = Cf*u U_u^{-1} e and RTS-smooths y* - f_x 100 times.
// The build uses the same model through linear algebra on the merged (train + test) grid:
//   S x = x - R Sigma^{-1} x,   Sigma^{-1} = W^T W  (whitening + adjoint, k_lgssm.hip)
//   f*_e = S y* + (I - S) Cf*u U_u^{-1} e = S y* + Q U_u^{-1} e,   Q = R Sigma^{-1} Cf*u
// so with V = L_D^{-1} L_u^{-1} (q(u) = N(m_e, D^{-1}), D = L_D L_D^T):
//   mean_i = (S y*)_i + Q_i w,  w = U_u^{-1} m_e
//   f*_{i,s} = mean_i + Z_i xi_s,  Z = Q V^T,  xi_s ~ N(0, I)      (MC, reference-faithful)
//   var_i = |Z_i|^2                                                 (ANALYTIC, S -> infinity)
#include "device_common.hpp"

namespace gpar {

typedef double d4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------- merge train + test
// Stable sortperm of vcat(train, test) (gpar_scaled_inference.jl:75-87) for ascending inputs:
// train k -> k + #{test < t_k};  test i -> i + #{train <= t*_i}.
__device__ __forceinline__ int64_t lower_bound(const double* a, int64_t n, double x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int64_t upper_bound(const double* a, int64_t n, double x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Scatter one side (train or test) into the merged arrays.  A workgroup takes 256 consecutive
// rows: each thread finds its row's merged position, then the group copies the rows' d inputs
// cooperatively (consecutive threads -> consecutive elements: the reads are coalesced and the
// writes nearly so, both sides being sorted), instead of one thread striding over its own row's
// d values (measured 0.8 ms per side at 1e6 rows).
__global__ __launch_bounds__(256) void merge_side(const double* __restrict__ ts, int64_t ns,
                                                  const double* __restrict__ other, int64_t no,
                                                  int is_test, const double* __restrict__ ys,
                                                  double rval, const double* __restrict__ vs,
                                                  int64_t ldvs, int d,
                                                  double* __restrict__ tm, double* __restrict__ ym,
                                                  double* __restrict__ rm, double* __restrict__ vm,
                                                  int64_t ldvm, int64_t* __restrict__ pos_out) {
  __shared__ int64_t lpos[256];
  const int64_t r0 = blockIdx.x * (int64_t)256;
  const int64_t k = r0 + threadIdx.x;
  if (k < ns) {
    const double tk = ts[k];
    const int64_t pos = k + (is_test ? upper_bound(other, no, tk) : lower_bound(other, no, tk));
    tm[pos] = tk;
    ym[pos] = ys ? ys[k] : 0.0;
    rm[pos] = rval;
    if (pos_out) pos_out[k] = pos;
    lpos[threadIdx.x] = pos;
  }
  if (d <= 0) return;
  __syncthreads();
  const int rows = (int)((ns - r0) < 256 ? (ns - r0) : 256);
  const int total = rows * d;   // <= 256 x 256
  for (int e = threadIdx.x; e < total; e += 256) {
    const int r = e / d, i = e - r * d;
    vm[lpos[r] * ldvm + i] = vs[(r0 + r) * ldvs + i];
  }
}

// ---------------------------------------------------------------------------- per test row
// X: merged grid rows of local adjoint outputs (columns 0..m-1 = Cf*u columns, column mp = y*),
// h: adjoint fix-up vectors, chat: backward carries [nch][mc][4].  One wave per test point:
//   Q[i][c] = R_k u_{k,c}, mean_i = y*_k - R_k u_{k,y} + Q_i . w.
template <int D>
__global__ __launch_bounds__(256) void predict_rows(const double* __restrict__ X, int64_t ldx,
                                                    const double* __restrict__ h,
                                                    const double* __restrict__ chat, int64_t mc,
                                                    int64_t mp, int64_t m, int L,
                                                    const int64_t* __restrict__ pos,
                                                    int64_t nstar, const double* __restrict__ rm,
                                                    const double* __restrict__ ym,
                                                    const double* __restrict__ w,
                                                    double* __restrict__ Q, int64_t ldq,
                                                    double* __restrict__ mean) {
  const int64_t i = blockIdx.x * (int64_t)4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= nstar) return;
  const int64_t k = pos[i];
  const int64_t j = k >> __builtin_ctz(L);  // L is a power of two (kChunk)
  const double R = rm[k];
  double hk[D];
#pragma unroll
  for (int q = 0; q < D; ++q) hk[q] = h[k * kGStride + q];
  double dot = 0.0;
  for (int64_t c = lane; c < mp; c += 64) {
    const double* ch = chat + (j * mc + c) * kSStride;
    double u = X[k * ldx + c];
#pragma unroll
    for (int q = 0; q < D; ++q) u = fma(hk[q], ch[q], u);
    const double qv = (c < m) ? R * u : 0.0;
    Q[i * ldq + c] = qv;
    if (c < m) dot = fma(qv, w[c], dot);
  }
  dot = wave_sum(dot);
  if (lane == 0) {
    const double* ch = chat + (j * mc + mp) * kSStride;
    double u = X[k * ldx + mp];
#pragma unroll
    for (int q = 0; q < D; ++q) u = fma(hk[q], ch[q], u);
    mean[i] = ym[k] - R * u + dot;
  }
}

// ---------------------------------------------------------------------------- GEMM  C = A B^T
// A: rows x K (row-major, lda), B: cols x K (row-major, ldb); 128 x 128 tile per 256-thread
// block (2 x 2 waves of 4 x 4 v_mfma_f64_16x16x4_f64), K-step 16 through LDS (k-major,
// padded rows: conflict-free fragment reads, see k_gram.hip).
// Epilogues: mode 0: C written (ldc) + rowsq[colblock][row] = sum_c C^2 over the tile (rowsq
//            null: C only);
//            mode 1: MC statistics over the tile's first `valid_cols` columns:
//                    out0[row] = base[row] + mean_c C, out1[row] = Bessel std_c C;
//            mode 2: rowsq[colblock][row][2] = (sum_c C, sum_c C^2) over the tile's columns
//                    < cols, combined by mc_stats_finish (MC with more than 128 samples).
// tri: B is lower triangular (B[j][k] = 0 for k > j, exactly), so column tile c0 only needs
//      k < c0 + 128 (V = L_D^{-1} L_u^{-1}: 37.5% of the MFMAs at M = 512).
constexpr int kPT = 128, kPBK = 16, kPLds = 144;

__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(
    const double* __restrict__ A, int64_t lda, const double* __restrict__ B, int64_t ldb,
    int64_t rows, int64_t cols, int64_t K, int mode, double* __restrict__ C, int64_t ldc,
    double* __restrict__ rowsq, int64_t valid_cols, const double* __restrict__ base,
    double* __restrict__ out0, double* __restrict__ out1, int tri) {
  __shared__ __attribute__((aligned(16))) double smem[2 * 2 * kPBK * kPLds + 2 * 128 * 2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t r0 = (int64_t)blockIdx.x * kPT, c0 = (int64_t)blockIdx.y * kPT;
  if (tri && c0 + kPT < K) K = c0 + kPT;   // the rest of B's rows in this tile are zero
  // staging: thread t loads row (t >> 1) of the A / B tile, k offset (t & 1) * 8, 8 doubles
  const int srow = tid >> 1, sk = (tid & 1) * 8;
  const int64_t arow = r0 + srow, brow = c0 + srow;
  const bool av = arow < rows, bv = brow < cols;
  double ra[8], rb[8];
  // branch-free loads: indices clamped, out-of-range elements masked after the load
  const int64_t arc = av ? arow : rows - 1, brc = bv ? brow : cols - 1;
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int64_t kk = k0 + sk + q;
      const int64_t kc = kk < K ? kk : K - 1;
      ra[q] = A[arc * lda + kc] * ((av && kk < K) ? 1.0 : 0.0);
      rb[q] = B[brc * ldb + kc] * ((bv && kk < K) ? 1.0 : 0.0);
    }
  };
  auto store = [&](int buf) {
    double* la = smem + (buf * 2 + 0) * kPBK * kPLds;
    double* lb = smem + (buf * 2 + 1) * kPBK * kPLds;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      la[(sk + q) * kPLds + srow] = ra[q];
      lb[(sk + q) * kPLds + srow] = rb[q];
    }
  };
  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = d4{0.0, 0.0, 0.0, 0.0};
  const int nsteps = (int)((K + kPBK - 1) / kPBK);
  load(0);
  store(0);
  __syncthreads();
  const int frow = lane >> 4, fcol = lane & 15;
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    const bool more = s + 1 < nsteps;
    if (more) load((int64_t)(s + 1) * kPBK);
    const double* la = smem + (buf * 2 + 0) * kPBK * kPLds;
    const double* lb = smem + (buf * 2 + 1) * kPBK * kPLds;
#pragma unroll
    for (int ks = 0; ks < kPBK / 4; ++ks) {
      double fa[4], fb[4];
      const int kr = ks * 4 + frow;
#pragma unroll
      for (int a = 0; a < 4; ++a) fa[a] = la[kr * kPLds + wr * 64 + a * 16 + fcol];
#pragma unroll
      for (int c = 0; c < 4; ++c) fb[c] = lb[kr * kPLds + wc * 64 + c * 16 + fcol];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[a][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[a], fb[c], acc[a][c], 0, 0, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }
  // epilogue: per-lane partial row reductions over this wave's 64 columns
  double* red = smem + 2 * 2 * kPBK * kPLds;   // [2 (wc)][128 rows] x 2 quantities
  double s1[4][4], s2[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double p = 0.0, p2 = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int64_t col = c0 + wc * 64 + c * 16 + fcol;
        const double v = acc[a][c][r];
        const bool ok = (mode == 1) ? (col - c0 < valid_cols) : (col < cols);
        if (ok) { p += v; p2 = fma(v, v, p2); }
        if (mode == 0) {
          const int64_t row = r0 + wr * 64 + a * 16 + frow + 4 * r;
          if (C && row < rows && col < cols) C[row * ldc + col] = v;
        }
      }
      s1[a][r] = p;
      s2[a][r] = p2;
    }
  // reduce across the 16 lanes sharing a row (fcol)
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        s1[a][r] += __shfl_xor(s1[a][r], off, 64);
        s2[a][r] += __shfl_xor(s2[a][r], off, 64);
      }
    }
  if (fcol == 0) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wr * 64 + a * 16 + frow + 4 * r;
        red[(wc * 128 + rl) * 2 + 0] = s1[a][r];
        red[(wc * 128 + rl) * 2 + 1] = s2[a][r];
      }
  }
  __syncthreads();
  if (tid < 128) {
    const int64_t row = r0 + tid;
    if (row < rows) {
      const double t1 = red[(0 * 128 + tid) * 2 + 0] + red[(1 * 128 + tid) * 2 + 0];
      const double t2 = red[(0 * 128 + tid) * 2 + 1] + red[(1 * 128 + tid) * 2 + 1];
      if (mode == 0) {
        if (rowsq) rowsq[(int64_t)blockIdx.y * rows + row] = t2;
      } else if (mode == 2) {
        // MC over more than one 128-column tile: partial sum / sum of squares of this tile
        rowsq[((int64_t)blockIdx.y * rows + row) * 2 + 0] = t1;
        rowsq[((int64_t)blockIdx.y * rows + row) * 2 + 1] = t2;
      } else {
        // MC: f_s = base + F_s; Bessel-corrected std over the valid_cols samples
        const double S = (double)valid_cols;
        const double mu = t1 / S;
        const double var = (t2 - S * mu * mu) / (S - 1.0);
        out0[row] = base[row] + mu;
        out1[row] = sqrt(var > 0.0 ? var : 0.0);
      }
    }
  }
}

// ---------------------------------------------------------------------------- rows + variance, fused
// predict_var<D, NG>: predict_rows and the ANALYTIC variance var_i = |Q_i V^T|^2 in one pass; Q is
// never stored (predict_rows wrote N* x Mp doubles that gemm_nt then read once per 128-column
// tile, 10.3 GB per launch at N* = 1e6 by the counters).  A workgroup takes 64 test rows, wave w
// the 16 rows 16 w .. 16 w + 15 against all T = 4 NG column tiles of Z (16 wide; NG = Mp / 64;
// the accumulators fill the AGPRs).  Each lane computes its own A fragments on the fly: row fcol
// of its wave, Q[i][c] = R_k (X[k][c] + h_k . chat[j][c]) at the 4 columns of every k-step it
// feeds to the MFMA (loaded two k-steps ahead), and its share of the mean's dot with w.
// V's k-slab of each step (16 k of every column still needed) goes global -> LDS by DMA
// (global_load_lds_dwordx4, 8 columns x 128 B per wave-instruction), column-major with the
// 16-byte k-pairs of column c XOR-swizzled by (c >> 1) & 7 on the source side, so the MFMA
// fragment reads (16 columns x one k) hit 16 distinct bank pairs.  V is lower triangular, so tile
// t needs only k-steps s <= t; the k-loop runs in NG phases of 4 steps, phase G with the tiles
// 4 G .. T - 1: every wave has the same work at every step (one barrier per step), no MFMA sits
// under a branch (a branch around MFMAs made the register allocator copy the accumulators at
// every join), and the tiles of group G already past their diagonal multiply V's exact zeros in
// phase G's later steps (56 % of the dense MFMAs at M = 512; gemm_nt's 128-column skip: 62.5 %).
// V must be zero outside its m x m block (the caller clears the Mp x Mp buffer).
constexpr int kVRows = 64;
template <int V_> struct IntC { static constexpr int value = V_; };
// 16 bytes global -> LDS by DMA (wave-uniform LDS base + lane * 16).  A plain __device__ function:
// the builtin inside the kernel template's lambdas made the host pass drop the launch stubs.
__device__ __forceinline__ void dma16(const double* src, double* lds) {
  __builtin_amdgcn_global_load_lds(src, lds, 16, 0, 0);
}

// The same by inline asm, for the prefetching path of predict_var: an LDS-DMA the compiler sees
// makes it wait for every outstanding load (vmcnt(0)) before any later LDS read it cannot prove
// disjoint, the prefetches included; these are invisible to it, and the kernel waits for them
// itself.  lds: the wave-uniform LDS byte address of lane 0's 16 bytes.
__device__ __forceinline__ void dma16a(const double* src, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory", "m0");
}

template <int D, int NG>
__global__ __launch_bounds__(256, 1) void predict_var(
    const double* __restrict__ X, int64_t ldx, const double* __restrict__ h,
    const double* __restrict__ chat, int64_t mc, int64_t mp, int m, int L,
    const int64_t* __restrict__ pos, int64_t nstar, const double* __restrict__ rm,
    const double* __restrict__ ym, const double* __restrict__ w, const double* __restrict__ V,
    int64_t ldv, double* __restrict__ mean, double* __restrict__ stdv) {
  constexpr int T = 4 * NG, NC = 64 * NG, NS = 4 * NG;   // tiles, columns, k-steps
  __shared__ __attribute__((aligned(16))) double lb[2][NC * 16];
  __shared__ double lw[NC];   // w, zero past m
  // two-step-ahead operand rings (slot s % 3): X's 16 columns of k-step s for the 64 rows (row r's
  // 16-byte pieces at slot p ^ (r & 7)), and the chunk carries chat of the <= 2 chunks the rows
  // lie in (chunk slot, 16 columns, kSStride)
  __shared__ __attribute__((aligned(16))) double lx[3][kVRows * 16];
  __shared__ __attribute__((aligned(16))) double lc[3][2 * 16 * kSStride];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int frow = lane >> 4, fcol = lane & 15;
  // ---- this lane's Q row (the MFMA A operand's row fcol)
  const int64_t i = (int64_t)blockIdx.x * kVRows + wave * 16 + fcol;
  const bool rv = i < nstar;
  const int64_t k = pos[rv ? i : nstar - 1];
  const int64_t j = k >> __builtin_ctz(L);   // L is a power of two (kChunk)
  const double R = rm[k];
  double hk[D];
#pragma unroll
  for (int q = 0; q < D; ++q) hk[q] = h[k * kGStride + q];
  const double* xr = X + k * ldx;
  const double* cr = chat + j * mc * kSStride;
  // raw inputs of the A fragments of the next k-step: X's and chat's columns at this lane's row
  double xa[1][4], ca[1][4][D];
  auto loadA = [&](int s, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = s * 16 + ks * 4 + frow;   // < Mp: inside X's and chat's rows
      xa[st][ks] = xr[c];
#pragma unroll
      for (int q = 0; q < D; ++q) ca[st][ks][q] = cr[c * kSStride + q];
    }
  };
  double dot = 0.0;
  double fa[4];
  auto makeA = [&](int s, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = s * 16 + ks * 4 + frow;
      double u = xa[st][ks];
#pragma unroll
      for (int q = 0; q < D; ++q) u = fma(hk[q], ca[st][ks][q], u);
      const bool ok = rv && c < m;
      fa[ks] = ok ? R * u : 0.0;
      dot = fma(fa[ks], lw[c], dot);
    }
  };
  // ---- V's k-slab of step s into lb[buf]: wave-instruction q moves columns 8 q .. 8 q + 7 (lane
  //      -> column 8 q + lane / 8, physical pair lane % 8 = logical pair ^ ((column >> 1) & 7));
  //      columns of groups already finished (< 64 (s / 4)) are not moved again
  //      (instruction q = wave + 4 r: column 8 q + lane / 8, whose (c >> 1) & 7 depends on the
  //      lane and the wave's parity only, so the source is one lane base + r * 32 rows of V)
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int dc = lane >> 3, dp = lane & 7;
  const int kp = dp ^ ((4 * (wv & 1) + (dc >> 1)) & 7);
  const double* vsrc = V + (int64_t)(8 * wv + dc) * ldv + 2 * kp;
  auto dmaB = [&](int s, int buf) __attribute__((always_inline)) {
    const int q0 = 8 * (s >> 2);   // first instruction still needed (8 per 64-column group)
#pragma unroll
    for (int r = 0; r < NC / 32; ++r) {
      const int q = wv + 4 * r;
      if (q < q0) continue;   // wave-uniform
      dma16(vsrc + (int64_t)r * 32 * ldv + s * 16, &lb[0][0] + buf * (NC * 16) + q * 128);
    }
  };
  // ---- workgroups whose 64 rows lie in <= 2 chunks take the prefetching path: every operand of
  //      step s is in LDS, moved by DMA during step s - 2, and read by inline asm (a compiler-visible
  //      LDS read behind an outstanding LDS-DMA makes the compiler wait for every load, the
  //      prefetch included); the loop then has no compiler-tracked loads and the only waits are the
  //      per-step vmcnt + s_barrier below
  const int sh = __builtin_ctz(L);
  const int64_t i0 = (int64_t)blockIdx.x * kVRows;
  const int64_t i1 = (i0 + kVRows < nstar ? i0 + kVRows : nstar) - 1;
  const int64_t jlo = pos[i0] >> sh, jhi = pos[i1] >> sh;
  const bool pf = jhi - jlo <= 1;   // workgroup-uniform
  const double* xsrc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int rl = wave * 16 + (lane >> 3) + 8 * q;
    const int64_t ir = i0 + rl;
    const int64_t kr = pos[ir < nstar ? ir : nstar - 1];
    xsrc[q] = X + kr * ldx + 2 * ((lane & 7) ^ (rl & 7));
  }
  // wave 0 moves the carries: lane -> chunk slot lane / 32, 16-byte piece lane % 32
  const double* csrc = chat + ((jlo + ((lane >> 5) ? (jhi - jlo) : 0)) * mc) * kSStride + 2 * (lane & 31);
  const uint32_t lbb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)(&lb[0][0]);
  const uint32_t lxb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)(&lx[0][0]);
  const uint32_t lcb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)(&lc[0][0]);
  auto dmaXC = [&](int s) __attribute__((always_inline)) {
    const uint32_t dx = lxb + 8u * (uint32_t)((s % 3) * (kVRows * 16) + (wv * 16) * 16);
#pragma unroll
    for (int q = 0; q < 2; ++q) dma16a(xsrc[q] + s * 16, dx + 8u * (uint32_t)(q * 128));
    if (wv == 0) dma16a(csrc + s * 16 * kSStride, lcb + 8u * (uint32_t)((s % 3) * (2 * 16 * kSStride)));
  };
  auto dmaBa = [&](int s, int buf) __attribute__((always_inline)) {   // dmaB by dma16a
    const int q0 = 8 * (s >> 2);
#pragma unroll
    for (int r = 0; r < NC / 32; ++r) {
      const int q = wv + 4 * r;
      if (q < q0) continue;   // wave-uniform
      dma16a(vsrc + (int64_t)r * 32 * ldv + s * 16, lbb + 8u * (uint32_t)(buf * (NC * 16) + q * 128));
    }
  };
  // this lane's LDS byte offsets in slot 0: its 4 X operands (row 16 wave + fcol), its chunk
  // slot's carries of columns frow + 4 ks, and w
  const int xrl = wave * 16 + fcol;
  const uint32_t lwb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)(&lw[0]);
  uint32_t xo[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int cl = ks * 4 + frow;
    xo[ks] = lxb + 8u * (uint32_t)(xrl * 16 + ((((cl >> 1) ^ (xrl & 7)) << 1) + (cl & 1)));
  }
  const int cslot = (int)(j - jlo) & 1;
  const uint32_t co = lcb + 8u * (uint32_t)(cslot * 16 * kSStride + frow * kSStride);
  double wa[4];
  // operands of step s into xa / ca / wa (columns s 16 + 4 ks + frow); q = 0..2 of the carries are
  // read whatever D (kSStride = 4 keeps them in bounds)
  auto readA = [&](int s) __attribute__((always_inline)) {
    const uint32_t sx = (uint32_t)(s % 3) * (uint32_t)(kVRows * 16 * 8);
    const uint32_t sc = co + (uint32_t)(s % 3) * (uint32_t)(2 * 16 * kSStride * 8);
    const uint32_t sw = lwb + 8u * (uint32_t)(s * 16 + frow);
    double c3[4][3];
    asm volatile(
        "ds_read_b64 %0, %20\n\t"
        "ds_read_b64 %1, %21\n\t"
        "ds_read_b64 %2, %22\n\t"
        "ds_read_b64 %3, %23\n\t"
        "ds_read_b64 %4, %24\n\t"
        "ds_read_b64 %5, %24 offset:8\n\t"
        "ds_read_b64 %6, %24 offset:16\n\t"
        "ds_read_b64 %7, %24 offset:128\n\t"
        "ds_read_b64 %8, %24 offset:136\n\t"
        "ds_read_b64 %9, %24 offset:144\n\t"
        "ds_read_b64 %10, %24 offset:256\n\t"
        "ds_read_b64 %11, %24 offset:264\n\t"
        "ds_read_b64 %12, %24 offset:272\n\t"
        "ds_read_b64 %13, %24 offset:384\n\t"
        "ds_read_b64 %14, %24 offset:392\n\t"
        "ds_read_b64 %15, %24 offset:400\n\t"
        "ds_read_b64 %16, %25\n\t"
        "ds_read_b64 %17, %25 offset:32\n\t"
        "ds_read_b64 %18, %25 offset:64\n\t"
        "ds_read_b64 %19, %25 offset:96\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=v"(xa[0][0]), "=v"(xa[0][1]), "=v"(xa[0][2]), "=v"(xa[0][3]),
          "=v"(c3[0][0]), "=v"(c3[0][1]), "=v"(c3[0][2]), "=v"(c3[1][0]), "=v"(c3[1][1]),
          "=v"(c3[1][2]), "=v"(c3[2][0]), "=v"(c3[2][1]), "=v"(c3[2][2]), "=v"(c3[3][0]),
          "=v"(c3[3][1]), "=v"(c3[3][2]), "=v"(wa[0]), "=v"(wa[1]), "=v"(wa[2]), "=v"(wa[3])
        : "v"(xo[0] + sx), "v"(xo[1] + sx), "v"(xo[2] + sx), "v"(xo[3] + sx), "v"(sc), "v"(sw));
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int q = 0; q < D; ++q) ca[0][ks][q] = c3[ks][q];
  };
  d4 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
  for (int c = tid; c < NC; c += 256) lw[c] = c < m ? w[c] : 0.0;
  if (pf) {
    dmaBa(0, 0);
    dmaXC(0);
    if (NS > 1) dmaXC(1);
  } else {
    loadA(0, 0);
    dmaB(0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // one k-step s with tiles T0 .. T - 1: fa from the inputs loaded during step s - 1; then the
  // loads of step s + 1 (A inputs; slab s + 1 -> lb[(s + 1) & 1] by DMA) under this step's
  // MFMAs; wait for them, barrier
  auto step = [&](auto t0c, auto pfc, int s) __attribute__((always_inline)) {
    constexpr int T0 = decltype(t0c)::value;
    constexpr bool PF = decltype(pfc)::value;
    bool x2 = false;
    if constexpr (PF) {
      // step s's operands from the rings (landed before the previous step's barrier), then the
      // V slab of s + 1 and the operands of s + 2
      readA(s);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int c = s * 16 + ks * 4 + frow;
        double u = xa[0][ks];
#pragma unroll
        for (int q = 0; q < D; ++q) u = fma(hk[q], ca[0][ks][q], u);
        const bool ok = rv && c < m;
        fa[ks] = ok ? R * u : 0.0;
        dot = fma(fa[ks], wa[ks], dot);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < NS) dmaBa(s + 1, (s + 1) & 1);
      x2 = s + 2 < NS;
      if (x2) dmaXC(s + 2);
    } else
    {
      makeA(s, 0);
      if (s + 1 < NS) {
        loadA(s + 1, 0);
        dmaB(s + 1, (s + 1) & 1);
      }
    }
    const double* B = &lb[0][0] + (s & 1) * (NC * 16);
    // tile t's 4 fragments are read one tile ahead, each tile's reads in a scheduling region of
    // their own: with two tiles' reads in one region the compiler paired them into
    // ds_read2st64_b64, which banks by (a/4) mod 32 and 16-lane groups — 16 LDS cycles per pair
    // with this layout's 2-way conflicts, against 4 for the two ds_read_b64 the layout is
    // conflict-free for (PMC r04ag: 47 % of the LDS cycles were conflicts)
    auto readB = [&](int t, double* bf) __attribute__((always_inline)) {
      const int c = t * 16 + fcol;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int kk = ks * 4 + frow;
        bf[ks] = B[c * 16 + (((kk >> 1) ^ ((c >> 1) & 7)) << 1) + (kk & 1)];
      }
    };
    double bn[4];
    readB(T0, bn);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = T0; t < T; ++t) {
      double bc[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) bc[ks] = bn[ks];
      if (t + 1 < T) readB(t + 1, bn);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[ks], bc[ks], acc[t], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (PF) {
      // all but step s + 2's DMAs (issued last: X 2 per wave, the carries 1 more on wave 0) have
      // landed; a bare s_barrier (__syncthreads would first wait for every load, the prefetch
      // included); this step's LDS reads were consumed before it
      if (x2) {
        if (wv == 0)
          asm volatile("s_waitcnt vmcnt(3)\n\ts_barrier" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      }
    } else
    {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  };
  // phase G: k-steps 4 G .. 4 G + 3 with tiles 4 G .. T - 1.  Phase 0's first step is peeled (a
  // loop whose accumulators enter as the zero constant copied them every step)
  auto phase = [&](auto gc, auto pfc) __attribute__((always_inline)) {
    constexpr int G = decltype(gc)::value;
    int s = 4 * G;
    if constexpr (G == 0) step(IntC<0>{}, pfc, s++);
#pragma unroll 1
    for (; s < 4 * G + 4; ++s) step(IntC<4 * G>{}, pfc, s);
  };
  static_assert(NG >= 1 && NG <= 8, "NG in 1..8");
  auto phases = [&](auto pfc) __attribute__((always_inline)) {
    phase(IntC<0>{}, pfc);
    if constexpr (NG > 1) phase(IntC<1>{}, pfc);
    if constexpr (NG > 2) phase(IntC<2>{}, pfc);
    if constexpr (NG > 3) phase(IntC<3>{}, pfc);
    if constexpr (NG > 4) phase(IntC<4>{}, pfc);
    if constexpr (NG > 5) phase(IntC<5>{}, pfc);
    if constexpr (NG > 6) phase(IntC<6>{}, pfc);
    if constexpr (NG > 7) phase(IntC<7>{}, pfc);
  };
  if (pf)
    phases(std::true_type{});
  else
    phases(std::false_type{});
  // ---- epilogue: row sums of squares (rows frow + 4 r of the wave's 16) over the tiles and the
  //      16 lanes of a row; the mean's dot over the 4 lanes (frow) sharing a row
  double s2[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double v = 0.0;
#pragma unroll
    for (int t = 0; t < T; ++t) v = fma(acc[t][r], acc[t][r], v);
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) v += __shfl_xor(v, off, 64);
    s2[r] = v;
  }
  dot += __shfl_xor(dot, 16, 64);
  dot += __shfl_xor(dot, 32, 64);
  if (fcol == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t ir = (int64_t)blockIdx.x * kVRows + wave * 16 + frow + 4 * r;
      if (ir < nstar) stdv[ir] = sqrt(s2[r]);
    }
  }
  if (frow == 0 && rv) {
    double u = xr[mp];
#pragma unroll
    for (int q = 0; q < D; ++q) u = fma(hk[q], cr[mp * kSStride + q], u);
    mean[i] = ym[k] - R * u + dot;
  }
}

// var_i = sum over column blocks of rowsq; std = sqrt(var)
__global__ void rowsq_finish(const double* __restrict__ rowsq, int64_t rows, int nblk,
                             double* __restrict__ std_out) {
  const int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (i >= rows) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += rowsq[(int64_t)b * rows + i];
  std_out[i] = sqrt(s);
}

// MC statistics from mode-2 partials: out0 = base + mean, out1 = Bessel std over S samples
__global__ void mc_stats_finish(const double* __restrict__ part, int64_t rows, int nblk, double S,
                                const double* __restrict__ base, double* __restrict__ out0,
                                double* __restrict__ out1) {
  const int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (i >= rows) return;
  double t1 = 0.0, t2 = 0.0;
  for (int b = 0; b < nblk; ++b) {
    t1 += part[((int64_t)b * rows + i) * 2 + 0];
    t2 += part[((int64_t)b * rows + i) * 2 + 1];
  }
  const double mu = t1 / S;
  const double var = (t2 - S * mu * mu) / (S - 1.0);
  out0[i] = base[i] + mu;
  out1[i] = sqrt(var > 0.0 ? var : 0.0);
}

// MC factor W = Lc^T X (m x m, row-major, ld), Lc = chol(inv(D)) lower (Distributions'
// MvNormal(m_e, Symmetric(inv(D))) draws m_e + Lc xi, gpar_scaled_inference.jl:103,185) and
// X = L_u^{-1} lower: W[j][k] = sum_{l >= max(j,k)} Lc[l][j] X[l][k].  Row i of Z = Q W^T is then
// the draw's loading (I - S) K*_i U_u^{-1} Lc.  Zero outside m x m.
__global__ __launch_bounds__(256) void mc_factor_kernel(const double* __restrict__ Lc,
                                                        const double* __restrict__ X, int64_t ld,
                                                        int m, double* __restrict__ W) {
  const int j = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int k = blockIdx.x * 16 + (threadIdx.x & 15);
  if (j >= ld || k >= ld) return;
  double s = 0.0;
  if (j < m && k < m)
    for (int l = j > k ? j : k; l < m; ++l) s = fma(Lc[(int64_t)l * ld + j], X[(int64_t)l * ld + k], s);
  W[(int64_t)j * ld + k] = s;
}

// dst = src on the leading m x m block, identity on the padding (ld x ld)
__global__ void pad_identity_copy(const double* __restrict__ src, int64_t ld, int m,
                                  double* __restrict__ dst) {
  const int i = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int j = blockIdx.x * 16 + (threadIdx.x & 15);
  if (i >= ld || j >= ld) return;
  dst[(int64_t)i * ld + j] = (i < m && j < m) ? src[(int64_t)i * ld + j] : (i == j ? 1.0 : 0.0);
}

// ---------------------------------------------------------------------------- normal draws
// xi[s * ld + m] ~ N(0, 1) for s < S, m < M (zero beyond): counter_normal(seed, s, m)
// (device_common.hpp), independent of the launch geometry and of the padding ld (gpar_mc_normals
// exports the same draws unpadded).
__global__ void normal_kernel(double* __restrict__ xi, int64_t ld, int64_t S, int64_t M,
                              int64_t Sp, uint64_t seed) {
  const int64_t e = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (e >= Sp * ld) return;
  const int64_t s = e / ld, m = e % ld;
  xi[e] = (s < S && m < M) ? counter_normal(seed, (uint64_t)s, (uint64_t)m) : 0.0;
}

// ---------------------------------------------------------------------------- chain scatter / gather
// dst[b * ldd + pos[k]] = src[b * lds + k]   (train observations of every chain onto the merged grid)
__global__ void scatter_chains(const double* __restrict__ src, int64_t lds, int64_t ns,
                               const int64_t* __restrict__ pos, double* __restrict__ dst,
                               int64_t ldd) {
  const int64_t k = blockIdx.x * (int64_t)256 + threadIdx.x;
  const int b = blockIdx.y;
  if (k >= ns) return;
  dst[(int64_t)b * ldd + pos[k]] = src[(int64_t)b * lds + k];
}

// dst[b * ldd + i] = src[b * lds + pos[i]]   (test-point marginals back in input order)
__global__ void gather_chains(const double* __restrict__ src, int64_t lds, int64_t ns,
                              const int64_t* __restrict__ pos, double* __restrict__ dst,
                              int64_t ldd) {
  const int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= ns) return;
  dst[(int64_t)b * ldd + i] = src[(int64_t)b * lds + pos[i]];
}

}  // namespace gpar

// ============================================================================ launch wrappers
#include "launch.hpp"

namespace gpar {

void launch_merge_side(hipStream_t st, const double* ts, int64_t ns, const double* other,
                       int64_t no, int is_test, const double* ys, double rval, const double* vs,
                       int64_t ldvs, int d, double* tm, double* ym, double* rm, double* vm,
                       int64_t ldvm, int64_t* pos_out) {
  if (ns <= 0) return;
  merge_side<<<(unsigned)((ns + 255) / 256), 256, 0, st>>>(ts, ns, other, no, is_test, ys, rval, vs,
                                                           ldvs, d, tm, ym, rm, vm, ldvm, pos_out);
}

void launch_predict_rows(hipStream_t st, int sdim, const double* X, int64_t ldx, const double* h,
                         const double* chat, int64_t mc, int64_t mp, int64_t m, int L,
                         const int64_t* pos, int64_t nstar, const double* rm, const double* ym,
                         const double* w, double* Q, int64_t ldq, double* mean) {
  const unsigned nb = (unsigned)((nstar + 3) / 4);
  switch (sdim) {
    case 1: predict_rows<1><<<nb, 256, 0, st>>>(X, ldx, h, chat, mc, mp, m, L, pos, nstar, rm, ym, w, Q, ldq, mean); break;
    case 2: predict_rows<2><<<nb, 256, 0, st>>>(X, ldx, h, chat, mc, mp, m, L, pos, nstar, rm, ym, w, Q, ldq, mean); break;
    default: predict_rows<3><<<nb, 256, 0, st>>>(X, ldx, h, chat, mc, mp, m, L, pos, nstar, rm, ym, w, Q, ldq, mean); break;
  }
}

int predict_var_tiles(int64_t mp) {   // NG (64-column groups) of predict_var; 0: unsupported
  return (mp >= 64 && mp <= 512 && mp % 64 == 0) ? (int)(mp / 64) : 0;
}

void launch_predict_var(hipStream_t st, int sdim, const double* X, int64_t ldx, const double* h,
                        const double* chat, int64_t mc, int64_t mp, int64_t m, int L,
                        const int64_t* pos, int64_t nstar, const double* rm, const double* ym,
                        const double* w, const double* V, int64_t ldv, double* mean, double* stdv) {
  if (nstar <= 0) return;
  const unsigned nb = (unsigned)((nstar + kVRows - 1) / kVRows);
#define GPAR_PV(DD, NN)                                                                          \
  predict_var<DD, NN><<<nb, 256, 0, st>>>(X, ldx, h, chat, mc, mp, (int)m, L, pos, nstar, rm, ym, \
                                          w, V, ldv, mean, stdv)
#define GPAR_PV_NG(DD)                  \
  switch (predict_var_tiles(mp)) {     \
    case 2: GPAR_PV(DD, 2); break;      \
    case 4: GPAR_PV(DD, 4); break;      \
    case 6: GPAR_PV(DD, 6); break;      \
    default: GPAR_PV(DD, 8); break;     \
  }
  switch (sdim) {
    case 1: GPAR_PV_NG(1); break;
    case 2: GPAR_PV_NG(2); break;
    default: GPAR_PV_NG(3); break;
  }
#undef GPAR_PV_NG
#undef GPAR_PV
}

void launch_gemm_nt(hipStream_t st, const double* A, int64_t lda, const double* B, int64_t ldb,
                    int64_t rows, int64_t cols, int64_t K, int mode, double* C, int64_t ldc,
                    double* rowsq, int64_t valid_cols, const double* base, double* out0,
                    double* out1, int tri) {
  dim3 grid((unsigned)((rows + kPT - 1) / kPT), (unsigned)((cols + kPT - 1) / kPT));
  gemm_nt_kernel<<<grid, 256, 0, st>>>(A, lda, B, ldb, rows, cols, K, mode, C, ldc, rowsq,
                                       valid_cols, base, out0, out1, tri);
}

void launch_rowsq_finish(hipStream_t st, const double* rowsq, int64_t rows, int nblk,
                         double* std_out) {
  rowsq_finish<<<(unsigned)((rows + 255) / 256), 256, 0, st>>>(rowsq, rows, nblk, std_out);
}

void launch_mc_stats_finish(hipStream_t st, const double* part, int64_t rows, int nblk, int64_t S,
                           const double* base, double* out0, double* out1) {
  mc_stats_finish<<<(unsigned)((rows + 255) / 256), 256, 0, st>>>(part, rows, nblk, (double)S, base,
                                                                  out0, out1);
}

void launch_mc_factor(hipStream_t st, const double* Lc, const double* X, int64_t ld, int m,
                      double* W) {
  dim3 grid((unsigned)((ld + 15) / 16), (unsigned)((ld + 15) / 16));
  mc_factor_kernel<<<grid, 256, 0, st>>>(Lc, X, ld, m, W);
}

void launch_pad_identity_copy(hipStream_t st, const double* src, int64_t ld, int m, double* dst) {
  dim3 grid((unsigned)((ld + 15) / 16), (unsigned)((ld + 15) / 16));
  pad_identity_copy<<<grid, 256, 0, st>>>(src, ld, m, dst);
}

void launch_normal(hipStream_t st, double* xi, int64_t ld, int64_t S, int64_t M, int64_t Sp,
                   uint64_t seed) {
  normal_kernel<<<(unsigned)((Sp * ld + 255) / 256), 256, 0, st>>>(xi, ld, S, M, Sp, seed);
}

void launch_scatter_chains(hipStream_t st, const double* src, int64_t lds, int64_t ns,
                           const int64_t* pos, double* dst, int64_t ldd, int nchains) {
  dim3 grid((unsigned)((ns + 255) / 256), (unsigned)nchains);
  scatter_chains<<<grid, 256, 0, st>>>(src, lds, ns, pos, dst, ldd);
}

void launch_gather_chains(hipStream_t st, const double* src, int64_t lds, int64_t ns,
                          const int64_t* pos, double* dst, int64_t ldd, int nchains) {
  dim3 grid((unsigned)((ns + 255) / 256), (unsigned)nchains);
  gather_chains<<<grid, 256, 0, st>>>(src, lds, ns, pos, dst, ldd);
}

}  // namespace gpar
