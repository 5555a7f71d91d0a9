// k_dense.hip -- the M x M dense fp64 tail of the DTC objective / q(u) on gfx950.
//
// Replaces the reference's LAPACK calls on the pseudo-point side:
//   cholesky(Symmetric(cov(u)))            dtc.jl:119, gpar_scaled_inference.jl:159
//   U' \ beta',  A * A' + I, cholesky       dtc.jl:119-120 (reassociated: see k_gram.hip)
//   logdet(Lambda), Lambda.U' \ (A alpha)   dtc.jl:122-125
//   B_ef * B_ef' + I, chol_D \ (B b_y), inv gpar_scaled_inference.jl:187-192
// Matrices are row-major, lower triangle meaningful, leading dimension ld.  Batched over
// outputs: one job per output (blockIdx selects the job).
#include "device_common.hpp"

namespace gpar {

typedef double d4 __attribute__((ext_vector_type(4)));

struct KuuJob {
  const double* z;
  int64_t ldz;
  int d;
  int kind;
  double inv_l, s, diag_add;
  double* K;
  int64_t ldk;
  int m;
  int mpad;   // rows/columns m..mpad-1 are identity padding (blocked factorisation size)
};

struct CholJob {
  double* A;
  int64_t ld;
  int m;
  double diag_add;     // added to the diagonal before factoring (Lambda = ... + I)
  int* status;         // set to 1 on a non-positive pivot (PosDefException)
};

struct TrsmJob {
  const double* L;     // lower triangular (ld ldl)
  int64_t ldl;
  const double* B;     // right-hand sides, B[i * ldb + j] (or B[j * ldb + i] if transB)
  int64_t ldb;
  double* X;           // X = L^{-1} B, X[i * ldx + j]
  int64_t ldx;
  int m;
  int64_t ncols;
  int transB;
  int transX;          // X stored transposed: X[j * ldx + i]
};

// ---------------------------------------------------------------------------- Kuu
// One 16 x 16 tile of K per workgroup.  The tile's 16 + 16 pseudo-inputs are staged in LDS 64
// dimensions at a time (coalesced row reads), then each thread forms its d2 in the same order as a
// plain loop over the dimensions: the per-element global reads of two strided rows took 0.94 ms
// for the north batch's 63 x 512^2 entries, at the head of every Nelder-Mead round (r05y trace).
__global__ __launch_bounds__(256) void kuu_kernel(const KuuJob* __restrict__ jobs) {
  const KuuJob jb = jobs[blockIdx.z];
  __shared__ double zi[16][65], zj[16][65];
  const int tid = threadIdx.x, ti = tid >> 4, tj = tid & 15;
  const int i0 = blockIdx.y * 16, j0 = blockIdx.x * 16;
  if (i0 >= jb.mpad || j0 >= jb.mpad) return;   // workgroup-uniform
  const int i = i0 + ti, j = j0 + tj;
  double d2 = 0.0;
  if (i0 < jb.m && j0 < jb.m) {   // workgroup-uniform: a tile with a real row and column
    for (int q0 = 0; q0 < jb.d; q0 += 64) {
      const int nq = (jb.d - q0 < 64) ? jb.d - q0 : 64;
      __syncthreads();
      for (int e = tid; e < 16 * 64; e += 256) {
        const int r = e >> 6, q = e & 63;
        const bool qv = q < nq;
        zi[r][q] = (qv && i0 + r < jb.m) ? jb.z[(int64_t)(i0 + r) * jb.ldz + q0 + q] : 0.0;
        zj[r][q] = (qv && j0 + r < jb.m) ? jb.z[(int64_t)(j0 + r) * jb.ldz + q0 + q] : 0.0;
      }
      __syncthreads();
      for (int q = 0; q < nq; ++q) {
        const double a = zi[ti][q] - zj[tj][q];
        d2 = fma(a, a, d2);
      }
    }
  }
  if (i >= jb.mpad || j >= jb.mpad) return;
  if (i >= jb.m || j >= jb.m) {
    jb.K[(int64_t)i * jb.ldk + j] = (i == j) ? 1.0 : 0.0;
    return;
  }
  double v;
  if (jb.kind == KEQ)
    v = jb.s * exp(-0.5 * d2 * jb.inv_l * jb.inv_l);
  else
    v = jb.s * kappa_rt(jb.kind, sqrt(d2) * jb.inv_l);
  if (i == j) v += jb.diag_add;
  jb.K[(int64_t)i * jb.ldk + j] = v;
}

// ---------------------------------------------------------------------------- Cholesky
// Right-looking blocked Cholesky (NB = 16), one 256-thread workgroup per matrix; the
// trailing update A22 -= L21 L21^T runs on v_mfma_f64_16x16x4_f64.
__global__ __launch_bounds__(256) void chol_kernel(const CholJob* __restrict__ jobs) {
  const CholJob jb = jobs[blockIdx.x];
  double* A = jb.A;
  const int64_t ld = jb.ld;
  const int m = jb.m;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  __shared__ double Ld[16][17];
  __shared__ int bad;
  if (tid == 0) bad = 0;
  if (jb.diag_add != 0.0)
    for (int i = tid; i < m; i += 256) A[i * ld + i] += jb.diag_add;
  __syncthreads();
  for (int kb = 0; kb < m; kb += 16) {
    const int nb = (m - kb < 16) ? m - kb : 16;
    {
      const int i = tid >> 4, q = tid & 15;
      if (i < nb && q <= i) Ld[i][q] = A[(int64_t)(kb + i) * ld + kb + q];
    }
    __syncthreads();
    for (int jj = 0; jj < nb; ++jj) {
      if (tid == 0) {
        double dv = Ld[jj][jj];
        if (!(dv > 0.0)) { bad = 1; dv = 1.0; }
        Ld[jj][jj] = sqrt(dv);
      }
      __syncthreads();
      if (tid > jj && tid < nb) Ld[tid][jj] /= Ld[jj][jj];
      __syncthreads();
      const int i = tid >> 4, q = tid & 15;
      if (q > jj && q <= i && i < nb) Ld[i][q] -= Ld[i][jj] * Ld[q][jj];
      __syncthreads();
    }
    {
      const int i = tid >> 4, q = tid & 15;
      if (i < nb && q <= i) A[(int64_t)(kb + i) * ld + kb + q] = Ld[i][q];
    }
    // panel: rows below solve x L_D^T = a
    for (int i = kb + nb + tid; i < m; i += 256) {
      double x[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) x[q] = (q < nb) ? A[(int64_t)i * ld + kb + q] : 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (q < nb) {
          double s = x[q];
#pragma unroll
          for (int p = 0; p < q; ++p) s -= x[p] * Ld[q][p];
          x[q] = s / Ld[q][q];
        }
      }
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (q < nb) A[(int64_t)i * ld + kb + q] = x[q];
    }
    __syncthreads();
    // trailing update on MFMA: tiles of 16 x 16 with row block >= col block
    const int r0 = kb + nb;
    if (r0 < m) {
      const int T = (m - r0 + 15) / 16;
      const int ntile = T * (T + 1) / 2;
      for (int tt = wave; tt < ntile; tt += 4) {
        int a = 0;
        while ((a + 1) * (a + 2) / 2 <= tt) ++a;
        const int c = tt - a * (a + 1) / 2;
        const int rb = r0 + a * 16, cb = r0 + c * 16;
        d4 acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb + (lane >> 4) + 4 * r, col = cb + (lane & 15);
          acc[r] = (row < m && col < m) ? A[(int64_t)row * ld + col] : 0.0;
        }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int kk = ks * 4 + (lane >> 4);
          const int ra = rb + (lane & 15), rbb = cb + (lane & 15);
          const double fa = (kk < nb && ra < m) ? -A[(int64_t)ra * ld + kb + kk] : 0.0;
          const double fb = (kk < nb && rbb < m) ? A[(int64_t)rbb * ld + kb + kk] : 0.0;
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(fa, fb, acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb + (lane >> 4) + 4 * r, col = cb + (lane & 15);
          if (row < m && col < m && col <= row) A[(int64_t)row * ld + col] = acc[r];
        }
      }
    }
    __syncthreads();
  }
  if (tid == 0 && bad) *jb.status = 1;
}

// ---------------------------------------------------------------------------- TRSM
// X = L^{-1} B (or L^{-1} B^T): one 16-column right-hand-side tile per workgroup of 4 waves.
// Row blocks of 16 are solved in order.  Block ib's update  B_ib - sum_{kb < ib} L_{ib,kb} X_kb
// is split over the 4 waves by kb mod 4 (v_mfma_f64_16x16x4, operands from L2), the 4 partial
// tiles are summed through LDS, and 16 lanes run the 16-row substitution against the diagonal
// block staged in LDS.  (The earlier form had one wave walk every kb of a tile: a 4x longer
// dependent chain, with 4x fewer workgroups.)
__global__ __launch_bounds__(256) void trsm_kernel(const TrsmJob* __restrict__ jobs) {
  const TrsmJob jb = jobs[blockIdx.y];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * 16;
  if (c0 >= jb.ncols) return;
  const int m = jb.m;
  __shared__ double part[4][16][17];
  __shared__ double Ld[16][17];
  const int nblk = (m + 15) / 16;
  const int fr = lane & 15, fq = lane >> 4;
  const int64_t colf = c0 + fr;                    // this lane's fragment column
  const bool colv = colf < jb.ncols;
  for (int ib = 0; ib < nblk; ++ib) {
    const int r0 = ib * 16;
    {
      const int i = tid >> 4, j = tid & 15;
      Ld[i][j] = (r0 + i < m && r0 + j < m && j <= i) ? jb.L[(int64_t)(r0 + i) * jb.ldl + r0 + j] : 0.0;
    }
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    if (wave == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + fq + 4 * r;
        double v = 0.0;
        if (row < m && colv)
          v = jb.transB ? jb.B[colf * jb.ldb + row] : jb.B[(int64_t)row * jb.ldb + colf];
        acc[r] = v;
      }
    }
    const int ra = r0 + fr;
    const bool rav = ra < m;
#pragma unroll 2
    for (int kb = wave; kb < ib; kb += 4) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int kk = kb * 16 + ks * 4 + fq;
        const double fa = rav ? -jb.L[(int64_t)ra * jb.ldl + kk] : 0.0;
        const double fb = colv ? (jb.transX ? jb.X[colf * jb.ldx + kk] : jb.X[(int64_t)kk * jb.ldx + colf])
                               : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(fa, fb, acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) part[wave][fq + 4 * r][fr] = acc[r];
    __syncthreads();
    if (wave == 0 && lane < 16) {
      const int64_t col = c0 + lane;
      double x[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (r0 + i < m) {
          double s = ((part[0][i][lane] + part[1][i][lane]) + part[2][i][lane]) + part[3][i][lane];
#pragma unroll
          for (int q = 0; q < i; ++q) s = fma(-Ld[i][q], x[q], s);
          x[i] = s / Ld[i][i];
        } else {
          x[i] = 0.0;
        }
      }
      if (col < jb.ncols) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (r0 + i < m) {
            if (jb.transX) jb.X[col * jb.ldx + r0 + i] = x[i];
            else jb.X[(int64_t)(r0 + i) * jb.ldx + col] = x[i];
          }
      }
    }
    __syncthreads();
  }
}

constexpr int kMaxMTrsv = 2048;

// ---------------------------------------------------------------------------- single-wave vector solves
// x = L^{-1} b (forward) into LDS array x (length m); one wave.
__device__ void wave_forward(const double* __restrict__ L, int64_t ld, int m,
                             const double* b, double* x, int lane) {
  for (int i = 0; i < m; ++i) {
    double s = 0.0;
    for (int p = lane; p < i; p += 64) s = fma(L[(int64_t)i * ld + p], x[p], s);
    s = wave_sum(s);
    if (lane == 0) x[i] = (b[i] - s) / L[(int64_t)i * ld + i];
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
  }
}

// x = L^{-T} b (backward); one wave.
__device__ void wave_backward_t(const double* __restrict__ L, int64_t ld, int m,
                                const double* b, double* x, int lane) {
  for (int i = m - 1; i >= 0; --i) {
    double s = 0.0;
    for (int p = i + 1 + lane; p < m; p += 64) s = fma(L[(int64_t)p * ld + i], x[p], s);
    s = wave_sum(s);
    if (lane == 0) x[i] = (b[i] - s) / L[(int64_t)i * ld + i];
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
  }
}

// x = L^{-1} b (trans = 0) or x = L^{-T} b (trans = 1); one wave, batched over blockIdx.
struct TrsvJob {
  const double* L;
  int64_t ld;
  int m;
  const double* b;
  double* x;
  int trans;
};

__global__ __launch_bounds__(64) void trsv_kernel(const TrsvJob* __restrict__ jobs) {
  const TrsvJob jb = jobs[blockIdx.x];
  __shared__ double xs[kMaxMTrsv], bs[kMaxMTrsv];
  for (int i = threadIdx.x; i < jb.m; i += 64) bs[i] = jb.b[i];
  __syncthreads();
  if (jb.trans)
    wave_backward_t(jb.L, jb.ld, jb.m, bs, xs, threadIdx.x);
  else
    wave_forward(jb.L, jb.ld, jb.m, bs, xs, threadIdx.x);
  __syncthreads();
  for (int i = threadIdx.x; i < jb.m; i += 64) jb.x[i] = xs[i];
}

struct FinishJob {
  const double* Lu;      // chol(Kuu [+ sigma^2 I])
  const double* Llam;    // chol(Lambda)
  int64_t ld;
  int m;
  const double* r;       // beta^T alpha
  const double* logs;    // per-chunk sum log S
  int64_t nch;
  const double* a2part;  // per-block partial sums of alpha^2
  int64_t npart;
  int64_t n;
  const int* status;     // Cholesky failure flags (2)
  double* out;           // dtc
  double* me;            // q(u): m_e (length m) when non-null
};

constexpr int kMaxM = 2048;

// DTC objective: -0.5 [N log 2pi + sum log S + logdet Lambda + |alpha|^2 - |L_lam^{-1} L_u^{-1} r|^2]
// (dtc.jl:122-125 with A alpha = L_u^{-1} beta^T alpha).  q(u) mode (me != null):
// m_e = D^{-1} L_u^{-1} r (gpar_scaled_inference.jl:189).
__global__ __launch_bounds__(64) void finish_kernel(const FinishJob* __restrict__ jobs) {
  const FinishJob jb = jobs[blockIdx.x];
  const int lane = threadIdx.x;
  __shared__ double w[kMaxM], v[kMaxM];
  const int m = jb.m;
  wave_forward(jb.Lu, jb.ld, m, jb.r, w, lane);
  wave_forward(jb.Llam, jb.ld, m, w, v, lane);
  if (jb.me) {
    wave_backward_t(jb.Llam, jb.ld, m, v, w, lane);
    for (int i = lane; i < m; i += 64) jb.me[i] = w[i];
    return;
  }
  double ld = 0.0, vv = 0.0, ls = 0.0, a2 = 0.0;
  for (int i = lane; i < m; i += 64) {
    ld += log(jb.Llam[(int64_t)i * jb.ld + i]);
    vv = fma(v[i], v[i], vv);
  }
  for (int64_t j = lane; j < jb.nch; j += 64) ls += jb.logs[j];
  for (int64_t j = lane; j < jb.npart; j += 64) a2 += jb.a2part[j];
  ld = wave_sum(ld);
  vv = wave_sum(vv);
  ls = wave_sum(ls);
  a2 = wave_sum(a2);
  if (lane == 0) {
    const double tmp = ls + 2.0 * ld + a2 - vv;
    double dtc = -((double)jb.n * kLog2Pi + tmp) / 2.0;
    if (jb.status[0] || jb.status[1]) dtc = __builtin_nan("");
    *jb.out = dtc;
  }
}

// C = X^T X (m x m, X row-major m x m, ld), symmetric -- inv(D) = L_D^{-T} L_D^{-1}.
__global__ __launch_bounds__(256) void gram_small_kernel(const double* __restrict__ X, int64_t ldx,
                                                         int m, double* __restrict__ C,
                                                         int64_t ldc) {
  const int i = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int j = blockIdx.x * 16 + (threadIdx.x & 15);
  if (i >= m || j >= m) return;
  double s = 0.0;
  for (int k = 0; k < m; ++k) s = fma(X[(int64_t)k * ldx + i], X[(int64_t)k * ldx + j], s);
  C[(int64_t)i * ldc + j] = s;
}

// Symmetrise: C = (C + C^T) / 2 is not needed for gram_small; transpose copy helper:
// out[j * ldo + i] = in[i * ldi + j] for i >= j else 0 (upper factor U = L^T, column-major
// output == row-major L).  Used to return U_u.
__global__ void lower_to_upper_colmajor(const double* __restrict__ L, int64_t ldl, int m,
                                        double* __restrict__ U) {
  const int i = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int j = blockIdx.x * 16 + (threadIdx.x & 15);
  if (i >= m || j >= m) return;
  // U (upper, column-major): U[r + c*m] with r <= c equals L[c][r]
  U[(int64_t)i + (int64_t)j * m] = (i <= j) ? L[(int64_t)j * ldl + i] : 0.0;
}

__global__ void eye_kernel(double* __restrict__ A, int64_t ld, int m) {
  const int i = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int j = blockIdx.x * 16 + (threadIdx.x & 15);
  if (i >= m || j >= m) return;
  A[(int64_t)i * ld + j] = (i == j) ? 1.0 : 0.0;
}

}  // namespace gpar

// ============================================================================ launch wrappers
#include "launch.hpp"

namespace gpar {

void launch_kuu(hipStream_t st, const KuuJobHost* jobs_dev, int njobs, int mmax) {
  dim3 grid((mmax + 15) / 16, (mmax + 15) / 16, njobs);
  kuu_kernel<<<grid, 256, 0, st>>>(reinterpret_cast<const KuuJob*>(jobs_dev));
}

void launch_chol(hipStream_t st, const CholJobHost* jobs_dev, int njobs) {
  chol_kernel<<<njobs, 256, 0, st>>>(reinterpret_cast<const CholJob*>(jobs_dev));
}

void launch_trsm(hipStream_t st, const TrsmJobHost* jobs_dev, int njobs, int64_t ncols_max) {
  dim3 grid((unsigned)((ncols_max + 15) / 16), njobs);
  trsm_kernel<<<grid, 256, 0, st>>>(reinterpret_cast<const TrsmJob*>(jobs_dev));
}

void launch_finish(hipStream_t st, const FinishJobHost* jobs_dev, int njobs) {
  finish_kernel<<<njobs, 64, 0, st>>>(reinterpret_cast<const FinishJob*>(jobs_dev));
}

void launch_gram_small(hipStream_t st, const double* X, int64_t ldx, int m, double* C,
                       int64_t ldc) {
  dim3 grid((m + 15) / 16, (m + 15) / 16);
  gram_small_kernel<<<grid, 256, 0, st>>>(X, ldx, m, C, ldc);
}

void launch_lower_to_upper_colmajor(hipStream_t st, const double* L, int64_t ldl, int m,
                                    double* U) {
  dim3 grid((m + 15) / 16, (m + 15) / 16);
  lower_to_upper_colmajor<<<grid, 256, 0, st>>>(L, ldl, m, U);
}

void launch_eye(hipStream_t st, double* A, int64_t ld, int m) {
  dim3 grid((m + 15) / 16, (m + 15) / 16);
  eye_kernel<<<grid, 256, 0, st>>>(A, ld, m);
}

void launch_trsv(hipStream_t st, const TrsvJobHost* jobs_dev, int njobs) {
  trsv_kernel<<<njobs, 64, 0, st>>>(reinterpret_cast<const TrsvJob*>(jobs_dev));
}

}  // namespace gpar
