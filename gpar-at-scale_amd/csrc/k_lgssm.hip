// k_lgssm.hip -- state-space (Kalman) sweeps of the time GP on gfx950.
//
// Replaces the sequential TemporalGPs `decorrelate`/`logpdf` calls of the reference
// (dtc.jl:106-117, gpar_scaled_inference.jl:170-183, temporal_gp_inference.jl:78) with a
// time-chunked formulation whose every sequential dependency is short:
//
//  gains (data-independent, per chain = per output or temporal chain):
//    phase 1  per chunk: fold the chunk's covariance elements (A, C, J) of the parallel
//             Kalman filter (Sarkka & Garcia-Fernandez 2021, covariance part only);
//    phase 2  per chain: exclusive scan of the chunk aggregates -> filtered covariance at
//             every chunk start;
//    phase 3  per chunk: ordinary Riccati recursion from that covariance, emitting the
//             per-step record {A_k, K_k, 1/sqrt(S_k)}, the fix-up vectors
//             g_k = -rs_k (A_k Phi_{k-1})[0,:], the chunk transition Phi_j and sum log S_k.
//  columns (data): the filter is affine in the data with data-independent coefficients,
//    m_k = (I - K_k h) A_k m_{k-1} + K_k x_k, so each chunk is filtered from a zero state
//    (whiten_*), the true chunk-start states follow from a short carry recursion over chunks
//    (carry_kernel), and alpha_k(true) = alpha_k(local) + g_k . c_chunk (applied by the
//    consumer: vec_fix_kernel here, the Gram loader in k_gram.hip).
#include "device_common.hpp"
#include "nm_dev.hpp"

#include <atomic>
#include <cstdlib>

namespace gpar {

struct ChainParams {
  double inv_l;   // 1 / time lengthscale
  double l;       // time lengthscale
  double s;       // time-kernel variance (time_var^2)
  double r;       // observation noise variance (sigma^2), used when no noise vector
};

template <int D>
struct Elem {
  double A[D][D];
  double C[D][D];
  double J[D][D];
};

template <int D>
__device__ __forceinline__ void elem_identity(Elem<D>& e) {
  mat_eye(e.A);
  mat_zero(e.C);
  mat_zero(e.J);
}

// e = e1 (earlier) (x) e2 (later)
template <int D>
__device__ __forceinline__ void elem_combine(const Elem<D>& e1, const Elem<D>& e2, Elem<D>& out) {
  double Mi[D][D], M[D][D], T[D][D], X[D][D], V[D][D], U[D][D];
  mat_mul(e1.C, e2.J, Mi);
#pragma unroll
  for (int i = 0; i < D; ++i) Mi[i][i] += 1.0;
  mat_inv(Mi, M);
  mat_mul(e2.A, M, T);                 // T = A2 M
  Elem<D> r;
  mat_mul(T, e1.A, r.A);               // A = A2 M A1
  mat_mul(T, e1.C, X);                 // X = A2 M C1
  mat_mul_bt(X, e2.A, r.C);            // C = A2 M C1 A2^T + C2
  mat_mul(M, e1.A, V);                 // V = M A1
  mat_mul(e2.J, e1.A, U);              // U = J2 A1
  mat_mul_at(V, U, r.J);               // J = A1^T M^T J2 A1 + J1
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      r.C[i][j] += e2.C[i][j];
      r.J[i][j] += e1.J[i][j];
    }
  // keep the covariance parts exactly symmetric
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < i; ++j) {
      const double c = 0.5 * (r.C[i][j] + r.C[j][i]);
      r.C[i][j] = c; r.C[j][i] = c;
      const double q = 0.5 * (r.J[i][j] + r.J[j][i]);
      r.J[i][j] = q; r.J[j][i] = q;
    }
  out = r;
}

// Observation noise of step k: the shared per-step vector when given (prediction grids: 1e10 at
// test points, gpar_scaled_inference.jl:100-107), where a negative entry means "this chain's
// own sigma^2" (train points of chains with different sigma, temporal_gp_inference.jl:93-97).
__device__ __forceinline__ double step_noise(const double* __restrict__ noise, int64_t k,
                                            const ChainParams& cp) {
  if (!noise) return cp.r;
  const double v = noise[k];
  return v < 0.0 ? cp.r : v;
}

// Transition + process noise of a step of scaled length tau (stationary start: tau_0 = 1).
template <int D>
__device__ __forceinline__ void step_model_tau(double tau, const ChainParams& cp,
                                               double (&A)[D][D], double (&Q)[D][D]) {
  sde_transition<D>(tau, A);
  double Pinf[D][D], X[D][D];
  sde_pinf<D>(cp.s, Pinf);
  mat_mul(A, Pinf, X);
  mat_mul_bt(X, A, Q);
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) Q[i][j] = Pinf[i][j] - Q[i][j];
}

// Transition + process noise for step k of chain p.
template <int D>
__device__ __forceinline__ void step_model(const double* __restrict__ t, int64_t k,
                                           const ChainParams& cp, double (&A)[D][D],
                                           double (&Q)[D][D]) {
  step_model_tau<D>((k == 0) ? 1.0 : (t[k] - t[k - 1]) / cp.l, cp, A, Q);
}

// Per-thread sequential sweeps over a chunk (gains phases 1 and 3) read their step inputs
// (t_k, the noise entry, the data value) kStepPF steps ahead through a register pipeline: a load
// consumed in the same step is waited on at once, and on gfx9 vmcnt also counts every store the
// thread issued before it, so each step would stall for a full memory round trip.  The loop
// stays rolled (an unrolled block of steps doubles the VGPRs of these 3x3 recursions).
constexpr int kStepPF = 2;
struct StepPipe {
  double t[kStepPF], r[kStepPF], y[kStepPF];
  const double *tp, *np, *yp;
  int64_t k1;
  __device__ __forceinline__ void load(int slot, int64_t k) {
    const int64_t kk = k < k1 ? k : k1 - 1;
    t[slot] = tp[kk];
    r[slot] = np ? np[kk] : 0.0;
    y[slot] = yp ? yp[kk] : 0.0;
  }
  __device__ __forceinline__ void init(const double* t_, const double* n_, const double* y_,
                                       int64_t k0, int64_t k1_) {
    tp = t_; np = n_; yp = y_; k1 = k1_;
#pragma unroll
    for (int s = 0; s < kStepPF; ++s) load(s, k0 + s);
  }
  // values of step k (slot 0), then shift and fetch step k + kStepPF
  __device__ __forceinline__ void next(int64_t k, double& tk, double& rk, double& yk) {
    tk = t[0]; rk = r[0]; yk = y[0];
#pragma unroll
    for (int s = 0; s + 1 < kStepPF; ++s) { t[s] = t[s + 1]; r[s] = r[s + 1]; y[s] = y[s + 1]; }
    load(kStepPF - 1, k + kStepPF);
  }
};

// Covariance element of a step (Sarkka & Garcia-Fernandez, Lemma 7 without the data parts):
// the chain's first step from the stationary start, and every later step.  (One function with a
// `first` branch let clang merge the two branches' element stores through a pointer select, which
// put two of the element's entries in scratch memory: 24 bytes per lane and 0.35 GB of scratch
// traffic per ssm phase-1 dispatch, PMC r06.)
template <int D>
__device__ __forceinline__ void step_elem_first(double tau, const ChainParams& cp, double R,
                                                Elem<D>& e) {
  double A[D][D], Q[D][D];
  step_model_tau<D>(tau, cp, A, Q);
  double P0[D][D], X[D][D], Pm[D][D];
  sde_pinf<D>(cp.s, P0);
  mat_mul(A, P0, X);
  mat_mul_bt(X, A, Pm);
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) Pm[i][j] += Q[i][j];
  const double S = Pm[0][0] + R;
  mat_zero(e.A);
  mat_zero(e.J);
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) e.C[i][j] = Pm[i][j] - (Pm[i][0] / S) * Pm[0][j];
}
template <int D>
__device__ __forceinline__ void step_elem_next(double tau, const ChainParams& cp, double R,
                                               Elem<D>& e) {
  double A[D][D], Q[D][D];
  step_model_tau<D>(tau, cp, A, Q);
  const double S = Q[0][0] + R;
  const double iS = 1.0 / S;
#pragma unroll
  for (int i = 0; i < D; ++i) {
    const double kk = Q[i][0] * iS;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      e.A[i][j] = A[i][j] - kk * A[0][j];
      e.C[i][j] = Q[i][j] - kk * Q[0][j];
      e.J[i][j] = A[0][i] * A[0][j] * iS;
    }
  }
}

template <int D>
__device__ __forceinline__ void elem_store(double* __restrict__ p, const Elem<D>& e) {
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      p[i * D + j] = e.A[i][j];
      p[D * D + i * D + j] = e.C[i][j];
      p[2 * D * D + i * D + j] = e.J[i][j];
    }
}

template <int D>
__device__ __forceinline__ void elem_load(const double* __restrict__ p, Elem<D>& e) {
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      e.A[i][j] = p[i * D + j];
      e.C[i][j] = p[D * D + i * D + j];
      e.J[i][j] = p[2 * D * D + i * D + j];
    }
}

// ---------------------------------------------------------------------------- phase 1
// The chunk's aggregate element.  SUB lanes per chunk (SUB = 4 where the chains are too few to
// fill the chip with one lane per chunk: a rank's 8-output eeg shard has 49 waves, the ssm
// config's 16 chains one wave per SIMD, and each lane's 256 dependent steps then run at the
// latency of its fp64 chain): lane q folds steps [q L / SUB, (q + 1) L / SUB) of the chunk and the
// SUB partial elements are combined in time order through lane shuffles, (e0 e1)(e2 e3).
template <int D>
__device__ __forceinline__ void elem_shfl_down(const Elem<D>& e, int off, Elem<D>& o) {
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      o.A[i][j] = __shfl_down(e.A[i][j], off, 64);
      o.C[i][j] = __shfl_down(e.C[i][j], off, 64);
      o.J[i][j] = __shfl_down(e.J[i][j], off, 64);
    }
}

// Per-chunk values read by a one-workgroup-per-chain scan (gains_phase2: the aggregates;
// chain_carry_lml: MOM's per-chunk outputs) are stored in "run slot" order: chunk j of chain p at
// p 256 run + (j % run) 256 + j / run, run = ceil(nch / 256).  The scan's thread t walks chunks
// t run .. t run + run - 1, so its u-th chunk sits at u 256 + t and each of its loads is
// contiguous across the wave (in chunk order each load touched 64 lines: 35 us per scan at 16
// chains x 3907 chunks, 20 us in slot order).
__host__ __device__ __forceinline__ int64_t run_len(int64_t nch) { return (nch + 255) / 256; }
__device__ __forceinline__ int64_t run_slot(int p, int64_t j, int64_t nch) {
  const int64_t r = run_len(nch);
  return (int64_t)p * 256 * r + (j % r) * 256 + j / r;
}

constexpr int kP1B = 2;   // gains_phase1: steps per input block

template <int D, int SUB>
__global__ __launch_bounds__(256) void gains_phase1(const double* __restrict__ t, int64_t n,
                                                    int L, int64_t nch,
                                                    const ChainParams* __restrict__ cps,
                                                    const double* __restrict__ noise,
                                                    double* __restrict__ agg) {
  static_assert(SUB == 1 || SUB == 4, "sub-lanes per chunk");
  const int64_t gl = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t j = gl / SUB;
  const int q = (int)(gl % SUB);
  const int p = blockIdx.y;
  if (SUB == 1 && j >= nch) return;
  const bool live = j < nch;   // SUB > 1: every lane stays for the shuffles
  const ChainParams cp = cps[p];
  const int64_t jc = live ? j : 0;
  const int64_t c0 = jc * L;
  const int64_t c1 = (c0 + L < n) ? c0 + L : n;
  const int64_t Ls = L / SUB;
  const int64_t k0 = live ? (c0 + q * Ls < c1 ? c0 + q * Ls : c1) : c1;
  const int64_t k1 = (SUB == 1) ? c1 : (k0 + Ls < c1 ? k0 + Ls : c1);
  Elem<D> acc, e;
  elem_identity(acc);   // identity (x) e == e exactly: one code path for every step
  double tprev = k0 > 0 ? t[k0 - 1] : 0.0;
  // the step inputs in two static register blocks of kP1B steps, one block fetched while the other
  // is consumed (a rotating prefetch queue -- StepPipe -- moves pending loads between registers,
  // and each move waits for its load)
  constexpr int PB = kP1B;
  double tb[2][PB], rb[2][PB];
  auto fetch = [&](int buf, int64_t kb) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < PB; ++u) {
      const int64_t kk = kb + u < k1 ? kb + u : k1 - 1;
      tb[buf][u] = t[kk];
      rb[buf][u] = noise ? noise[kk] : 0.0;
    }
  };
  auto noise_of = [&](double rk) __attribute__((always_inline)) {
    return noise ? (rk < 0.0 ? cp.r : rk) : cp.r;
  };
  auto step = [&](int64_t k, double tk, double rk) __attribute__((always_inline)) {
    const double tau = (tk - tprev) / cp.l;
    tprev = tk;
    step_elem_next<D>(tau, cp, noise_of(rk), e);
    elem_combine<D>(acc, e, acc);
  };
  // the chain's first step (stationary start, tau = 1), peeled off the loop
  int64_t ks = k0;
  if (k0 == 0 && k1 > 0) {
    tprev = t[0];
    step_elem_first<D>(1.0, cp, noise_of(noise ? noise[0] : 0.0), e);
    elem_combine<D>(acc, e, acc);
    ks = 1;
  }
  if (ks < k1) fetch(0, ks);
  for (int64_t kb = ks; kb < k1; kb += 2 * PB) {
    fetch(1, kb + PB);
#pragma unroll
    for (int u = 0; u < PB; ++u)
      if (kb + u < k1) step(kb + u, tb[0][u], rb[0][u]);
    fetch(0, kb + 2 * PB);
#pragma unroll
    for (int u = 0; u < PB; ++u)
      if (kb + PB + u < k1) step(kb + PB + u, tb[1][u], rb[1][u]);
  }
  if constexpr (SUB > 1) {
#pragma unroll
    for (int off = 1; off < SUB; off <<= 1) {
      Elem<D> o;
      elem_shfl_down(acc, off, o);
      if ((q & (2 * off - 1)) == 0) elem_combine<D>(acc, o, acc);
    }
    if (q != 0 || !live) return;
  }
  elem_store<D>(agg + run_slot(p, j, nch) * (3 * D * D), acc);
}

// ---------------------------------------------------------------------------- phase 2
// One workgroup per chain: exclusive scan over chunk aggregates; writes the filtered
// covariance at the end of chunk j-1 into pstart[j] (j >= 1).
template <int D>
constexpr int kP2B = D == 3 ? 4 : 8;   // aggregates per batch of loads (3 D^2 doubles each)
template <int D>
__global__ __launch_bounds__(256) void gains_phase2(int64_t nch, const double* __restrict__ agg,
                                                    double* __restrict__ pstart) {
  constexpr int E = 3 * D * D;
  __shared__ double buf[2][256 * E];
  const int p = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t per = run_len(nch);
  const int64_t j0 = tid * per;
  const int64_t j1 = (j0 + per < nch) ? j0 + per : nch;
  // the aggregates in run-slot order: chunk j0 + u at u 256 + tid
  const double* a = agg + (int64_t)p * 256 * per * E + (int64_t)tid * E;
  auto at = [&](int64_t j) __attribute__((always_inline)) { return a + (j - j0) * 256 * E; };
  // a thread's run is read kP2B aggregates at a time, every load issued before the first combine
  // (one memory latency per batch instead of one per aggregate: 33 -> ~10 us at 3907 chunks)
  constexpr int KB = kP2B<D>;
  Elem<D> loc;
  elem_identity(loc);
  for (int64_t jb = j0; jb < j1; jb += KB) {
    Elem<D> eb[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u)
      if (jb + u < j1) elem_load<D>(at(jb + u), eb[u]);
#pragma unroll
    for (int u = 0; u < KB; ++u)
      if (jb + u < j1) elem_combine<D>(loc, eb[u], loc);
  }
  elem_store<D>(&buf[0][tid * E], loc);
  __syncthreads();
  int cur = 0;
  for (int off = 1; off < 256; off <<= 1) {
    Elem<D> mine;
    elem_load<D>(&buf[cur][tid * E], mine);
    if (tid >= off) {
      Elem<D> prev;
      elem_load<D>(&buf[cur][(tid - off) * E], prev);
      elem_combine<D>(prev, mine, mine);
    }
    elem_store<D>(&buf[cur ^ 1][tid * E], mine);
    __syncthreads();
    cur ^= 1;
  }
  Elem<D> pre;
  if (tid == 0) {
    elem_identity(pre);
  } else {
    elem_load<D>(&buf[cur][(tid - 1) * E], pre);
  }
  double* ps = pstart + (int64_t)p * nch * (D * D);
  for (int64_t jb = j0; jb < j1; jb += KB) {
    Elem<D> eb[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u)
      if (jb + u < j1) elem_load<D>(at(jb + u), eb[u]);
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int64_t j = jb + u;
      if (j < j1) {
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) ps[j * D * D + i * D + q] = pre.C[i][q];
        elem_combine<D>(pre, eb[u], pre);
      }
    }
  }
}

// ---------------------------------------------------------------------------- phase 3
// Riccati recursion inside each chunk from the scanned start covariance.
//   rec[k]   = {A_k (row-major), K_k, rs_k = 1/sqrt(S_k)}
//   g[k]     = -rs_k * (A_k Phi_{j,k-1})[0, :]
//   phi[j]   = prod_{k in chunk} (I - K_k e1^T) A_k   (D x D)
//   logs[j]  = sum_{k in chunk} log S_k
// With `smooth` output (prediction): pf[k] = filtered covariance (D x D), used by the RTS pass.
// With `ys` (the DTC objective): the chain's own data vector ys[p] is filtered from a zero state
// in the same pass, with the record still in registers (what whiten_vec would do in a second pass
// over rec): alpha_loc[p * n + k] and the chunk end state asend[(p * nch + j) * 4 + i].
//
// Memory ordering (r05).  On gfx9 one counter (vmcnt) tracks loads and stores in issue order, so a
// wait for a load also waits for every store issued before it.  Each step stores its record and
// fix-up row, and each step needs its inputs (t_k, the noise entry, y_k).  The inputs are loaded
// kGainsPF steps ahead into static register slots (the step loop unrolled by kGainsPF, so a slot's
// pending load is never copied: a register rotation of a pending load forces an immediate wait),
// and every store is issued unconditionally -- lanes past the chain's end write to a sink -- so the
// number of memory operations between a slot's load and its use is fixed and the compiler's wait
// covers only the load, never the stores behind it.  (r04: a StepPipe rotation plus branch-skipped
// stores made every step wait for all outstanding memory: ~2 us per step, the 62-chain launch
// 5.3 ms writing at 1.95 TB/s.)
__device__ double g_gains_sink[64 * 16];   // 16 doubles per lane: the widest masked store (pf)

constexpr int kGainsPF = 4;

// MOM (the temporal-only chains' logpdf, chains_logpdf): no record, fix-up row or alpha is written;
// each chunk leaves the moments of its chunk-local alpha against the fix-up rows instead,
//   mom[j] = {s0 = sum alpha_loc^2, s1 = sum alpha_loc g_k (D), s2 = sum g_k g_k^T (packed upper)},
// from which sum_k alpha_k^2 = sum_j s0 + 2 c_j . s1 + c_j^T s2 c_j once the carry has given the
// chunks' incoming states c_j (alpha_k = alpha_loc,k + g_k . c_j, as vec_fix applies it).
constexpr int kMomStride = 12;   // >= 1 + D + D (D + 1) / 2 for D <= 3
// MOM's per-chunk outputs (phi, logS, the end state, the moments) go to run_slot order (above)

template <int D, bool COMPACT, bool HAS_Y, bool HAS_NOISE, bool HAS_PF, bool MASKED, bool MOM>
__global__ __launch_bounds__(256, 2) void gains_phase3(int64_t blk0, const double* __restrict__ t,
                                                    int64_t n,
                                                    int L, int64_t nch,
                                                    const ChainParams* __restrict__ cps,
                                                    const double* __restrict__ noise,
                                                    const double* __restrict__ pstart,
                                                    double* __restrict__ rec,
                                                    double* __restrict__ g,
                                                    double* __restrict__ phi,
                                                    double* __restrict__ logs,
                                                    double* __restrict__ pf,
                                                    const double* const* __restrict__ ys,
                                                    double* __restrict__ alpha_loc,
                                                    double* __restrict__ asend,
                                                    double* __restrict__ mom) {
  static_assert(!MOM || (HAS_Y && !COMPACT && !HAS_PF), "moments: the data filter only");
  // COMPACT: the record written is {K_k, rs_k} (CRec), its A_k recomputed by the consumer from the
  // step's time difference (whiten_kfu_d2x2's staging); RP stays the full record's pitch
  constexpr int RS = COMPACT ? CRec<D>::size : Rec<D>::size;
  // Output staging: thread = chunk, so a plain per-thread store of step s's record writes 64
  // lines 32 KB apart per instruction.  Each wave parks its 64 records (and the g rows) in LDS
  // and writes them back 16 bytes per lane, RS/2 lanes per record; the alpha values are parked
  // kGainsPF steps at a time and written back per chunk.
  constexpr int RP = Rec<D>::size + 1;
  constexpr int PF = kGainsPF;
  constexpr int AS = PF;        // alpha steps per flush: one per unrolled block
  __shared__ double rbuf[4][64 * RP];
  __shared__ double abuf[4][64 * (AS + 1)];
  // MASKED = false: a block of 256 whole chunks (every chunk but the last is L steps long), so no
  // lane is ever masked; the last block of each chain (MASKED) handles the partial last chunk and
  // the lanes past nch
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t j = (blk0 + blockIdx.x) * (int64_t)blockDim.x + threadIdx.x;
  const int64_t jw = j - lane;  // the wave's first chunk
  const int p = blockIdx.y;
  const bool jv = !MASKED || j < nch;
  const ChainParams cp = cps[p];
  const int64_t k0 = (jv ? j : nch - 1) * L;
  const int64_t k1 = !MASKED ? k0 + L : ((k0 + L < n) ? k0 + L : n);
  double P[D][D];
  if (j == 0 || !jv) {
    sde_pinf<D>(cp.s, P);
  } else {
    const double* ps = pstart + ((int64_t)p * nch + j) * (D * D);
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) P[i][q] = ps[i * D + q];
  }
  double Phi[D][D];
  mat_eye(Phi);
  double lsum = 0.0;
  const double* yp = HAS_Y ? ys[p] : nullptr;
  double* ap = HAS_Y ? alpha_loc + (int64_t)p * n : nullptr;
  double ma[D];
#pragma unroll
  for (int i = 0; i < D; ++i) ma[i] = 0.0;
  double ms[kMomStride];
#pragma unroll
  for (int e = 0; e < kMomStride; ++e) ms[e] = 0.0;
  double* rp = rec + (int64_t)p * n * RS;
  double* gp = g + (int64_t)p * n * kGStride;
  double* pfp = HAS_PF ? pf + (int64_t)p * n * (D * D) : nullptr;
  double* sink = g_gains_sink + 16 * lane;
  double* rb = rbuf[wave];
  double* ab = abuf[wave];
  double tprev = k0 > 0 ? t[k0 - 1] : 0.0;
  // step inputs, slot u = step sb + u of the current block (loads clamped in bounds)
  double tq[PF], rq[PF], yq[PF];
  auto load = [&](int u, int64_t k) __attribute__((always_inline)) {
    const int64_t kk = (!MASKED && k + PF <= k0 + L) ? k : (k < k1 ? k : k1 - 1);
    tq[u] = t[kk];
    if constexpr (HAS_NOISE) rq[u] = noise[kk];
    if constexpr (HAS_Y) yq[u] = yp[kk];
  };
#pragma unroll
  for (int u = 0; u < PF; ++u) load(u, k0 + u);
  // every lane runs all L steps (the wave writes cooperatively); past k1 nothing is committed
  for (int sb = 0; sb < L; sb += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int sidx = sb + u;
      const int64_t k = k0 + sidx;
      const bool live = !MASKED || (jv && k < k1);
      const double tk = tq[u];
      const double rk = HAS_NOISE ? rq[u] : 0.0;
      const double yk = HAS_Y ? yq[u] : 0.0;
      load(u, k + PF);
      double A[D][D], Q[D][D], X[D][D], Pm[D][D];
      step_model_tau<D>((k == 0) ? 1.0 : (tk - tprev) / cp.l, cp, A, Q);
      tprev = tk;
      mat_mul(A, P, X);
      mat_mul_bt(X, A, Pm);
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int q = 0; q < D; ++q) Pm[i][q] += Q[i][q];
      const double R = HAS_NOISE ? (rk < 0.0 ? cp.r : rk) : cp.r;
      const double S = Pm[0][0] + R;
      const double rs = 1.0 / sqrt(S);
      double Kg[D];
#pragma unroll
      for (int i = 0; i < D; ++i) Kg[i] = Pm[i][0] / S;
      double AP[D][D];
      mat_mul(A, Phi, AP);
      // the record {A, K, rs, pad} (COMPACT: {K, rs, pad}) and g_k = -rs (A Phi)[0, :]
      constexpr int KO = COMPACT ? 0 : D * D;   // K's offset in the record
      double recv[RS];
      if constexpr (!COMPACT) {
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) recv[i * D + q] = A[i][q];
      }
#pragma unroll
      for (int i = 0; i < D; ++i) recv[KO + i] = Kg[i];
      recv[KO + D] = rs;
#pragma unroll
      for (int e = KO + D + 1; e < RS; ++e) recv[e] = 0.0;
      double gk[kGStride];
#pragma unroll
      for (int q = 0; q < kGStride; ++q) gk[q] = q < D ? -rs * AP[0][q] : 0.0;
      if constexpr (MOM) {
        // nothing stored: the moments are accumulated with alpha below
      } else if constexpr (MASKED) {   // the chain's last block: each lane stores its own record directly
        double* dr = live ? rp + k * RS : sink;
#pragma unroll
        for (int e = 0; e < RS; e += 2)
          *reinterpret_cast<double2*>(dr + e) = double2{recv[e], recv[e + 1]};
        double* dg = live ? gp + k * kGStride : sink;
#pragma unroll
        for (int e = 0; e < kGStride; e += 2)
          *reinterpret_cast<double2*>(dg + e) = double2{gk[e], gk[e + 1]};
      } else {   // parked in LDS, written back coalesced below
#pragma unroll
        for (int e = 0; e < RS; ++e) rb[lane * RP + e] = recv[e];
      }
      if (live) {
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) P[i][q] = Pm[i][q] - Kg[i] * Pm[0][q];
        // Phi <- (I - K e1^T) A Phi
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) Phi[i][q] = AP[i][q] - Kg[i] * AP[0][q];
        lsum += log(S);
      }
      if constexpr (HAS_Y) {   // alpha filter from zero (same arithmetic as whiten_kfu's column recursion)
        double mm[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
          double a2 = 0.0;
#pragma unroll
          for (int q = 0; q < D; ++q) a2 = fma(A[i][q], ma[q], a2);
          mm[i] = a2;
        }
        const double ev = yk - mm[0];
        if constexpr (MOM) {
          if (live) {
            const double al = ev * rs;
            ms[0] = fma(al, al, ms[0]);
            int e = 1 + D;
#pragma unroll
            for (int i = 0; i < D; ++i) {
              ms[1 + i] = fma(al, gk[i], ms[1 + i]);
#pragma unroll
              for (int q = i; q < D; ++q) {
                ms[e] = fma(gk[i], gk[q], ms[e]);
                ++e;
              }
            }
          }
        } else if constexpr (MASKED)
          *(live ? ap + k : sink) = ev * rs;
        else
          ab[lane * (AS + 1) + u] = ev * rs;
        if (live) {
#pragma unroll
          for (int i = 0; i < D; ++i) ma[i] = fma(Kg[i], ev, mm[i]);
        }
      }
      if constexpr (HAS_PF) {
        double* dst = live ? pfp + k * D * D : sink;
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) dst[i * D + q] = P[i][q];
      }
      if constexpr (!MASKED && !MOM) {
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's parked values landed
        __builtin_amdgcn_wave_barrier();
        // write back: lane -> (record rr = e / (RS/2), 16-byte piece e % (RS/2))
  #pragma unroll
        for (int it = 0; it < RS / 2; ++it) {
          const int e = it * 64 + lane;
          const int rr = e / (RS / 2), pc = e % (RS / 2);
          const int64_t jr = jw + rr;
          const int64_t kr = jr * L + sidx;
          double2 v;
          v.x = rb[rr * RP + 2 * pc];
          v.y = rb[rr * RP + 2 * pc + 1];
          double* dst = rp + kr * RS + 2 * pc;
          *reinterpret_cast<double2*>(dst) = v;
        }
        // g rows: two 16-byte pieces per step, straight from registers through a lane exchange
        __builtin_amdgcn_wave_barrier();
  #pragma unroll
        for (int q = 0; q < kGStride; ++q) rb[lane * RP + q] = gk[q];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
  #pragma unroll
        for (int it = 0; it < 2; ++it) {
          const int e = it * 64 + lane;
          const int rr = e >> 1, pc = e & 1;
          const int64_t jr = jw + rr;
          const int64_t kr = jr * L + sidx;
          double2 v;
          v.x = rb[rr * RP + 2 * pc];
          v.y = rb[rr * RP + 2 * pc + 1];
          double* dst = gp + kr * kGStride + 2 * pc;
          *reinterpret_cast<double2*>(dst) = v;
        }
        __builtin_amdgcn_wave_barrier();   // rb is rewritten by the next step
      }
      // keep the unrolled steps apart: interleaving them only lengthens live ranges (spills)
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (HAS_Y && !MASKED && !MOM) {   // the block's AS alpha values of the wave's 64 chunks
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int it = 0; it < AS; ++it) {
        const int e = it * 64 + lane;
        const int rr = e / AS, pc = e % AS;
        const int64_t jr = jw + rr;
        const int64_t kr = jr * L + sb + pc;
        ap[kr] = ab[rr * (AS + 1) + pc];
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (!jv) return;
  const int64_t jo = MOM ? run_slot(p, j, nch) : (int64_t)p * nch + j;
  double* ph = phi + jo * (D * D);
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) ph[i * D + q] = Phi[i][q];
  logs[jo] = lsum;
  if constexpr (HAS_Y) {
    double* sp = asend + jo * kSStride;
#pragma unroll
    for (int i = 0; i < kSStride; ++i) sp[i] = i < D ? ma[i] : 0.0;
  }
  if constexpr (MOM) {
    double* mp_ = mom + jo * kMomStride;
#pragma unroll
    for (int e = 0; e < kMomStride; ++e) mp_[e] = ms[e];
  }
}

// ---------------------------------------------------------------------------- phase 3, fast path
// The same recursion and outputs as gains_phase3 for the chains' whole blocks (256 chunks of
// exactly L = 256 steps) and, in the same launch, each chain's masked last block, with the step
// loop's memory operations counted so that its waits are exact:
//   * the step inputs (t, and y or the noise vector) reach LDS by LDS-DMA (global_load_lds_dwordx4:
//     two steps of the lane's chunk per instruction) into a per-wave ring of kG3Ring pair slots,
//     one unrolled block (kG3Blk steps) ahead;
//   * the record / fix-up row / alpha stores, g3_stores_per_block(...) per block, are counted;
//   * at the top of block b, after issuing block b + 1's DMAs, `s_waitcnt vmcnt(S + 2 NA)` leaves
//     block b - 1's S stores and block b + 1's 2 NA DMAs in flight and retires block b's DMAs:
//     no step ever waits for a store.
// (hipcc does not count the asm DMAs, and the loop's only other memory operations are its plain
// stores, which it never waits for, so it inserts no vmcnt of its own; the ring is read only by
// the wave that filled it, after its own covering vmcnt -- MI355X_MICROARCH.md item 7.  The
// stores are plain C++ stores, not asm, so that hipcc's hazard recognizer sees their operands:
// a first version with asm stores, whose address registers hipcc rewrote in the next cycle,
// produced wrong records.)
constexpr int kG3L = 256;      // == kChunk
constexpr int kG3Blk = 4;      // steps per unrolled block (two DMA pairs)
constexpr int kG3Ring = 4;     // pair slots per array (two blocks)

template <int D, bool COMPACT, bool HAS_PF, bool MOM = false, bool MASKED = false>
__host__ __device__ constexpr int g3_stores_per_block(bool has_y) {
  constexpr int RS = COMPACT ? CRec<D>::size : Rec<D>::size;
  constexpr int PFS = HAS_PF ? (D * D + 1) / 2 : 0;   // the filtered covariance, 16 B pieces
  // the block's alpha: two 16-byte pairs per lane (masked block: four 8-byte halves)
  return MOM ? 0 : kG3Blk * (RS / 2 + 2 + PFS) + (has_y ? (MASKED ? 4 : 2) : 0);
}

typedef double g3d2 __attribute__((ext_vector_type(2)));

// plain stores (hipcc emits them, and its hazard recognizer sees them; it counts no VMEM load in
// the loop, so it never waits for them): one global_store_dwordx4 / _dwordx2 each
__device__ __forceinline__ void g3_store16(double* dst, g3d2 v) {
  *reinterpret_cast<g3d2*>(dst) = v;
}
__device__ __forceinline__ void g3_store8(double* dst, double v) { *dst = v; }
__device__ __forceinline__ void g3_dma16(const double* src, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory", "m0");
}

// MASKED: the chain's last block of 256 chunks -- lanes past nch run chunk nch - 1's inputs and
// store to the sink, the partial last chunk's steps past n are not committed, and its inputs are
// read in whole 16-byte pairs (the arrays are 16-byte aligned, so a pair holding a valid element
// never leaves its page) up to the last one holding a valid step.
// (the masked block -- one per chain -- is allowed the whole register file: its selects would
// otherwise spill, and one such block per chain never fills a CU anyway)
// the kernel's LDS, shared by its two bodies (whole blocks and the masked last block)
template <int D, bool HAS_Y, bool HAS_NOISE, bool MOM>
struct G3Lds {
  static constexpr int RP = Rec<D>::size + 1;
  static constexpr int NA = 1 + (HAS_Y ? 1 : 0) + (HAS_NOISE ? 1 : 0);   // input arrays staged
  double rbuf[4][MOM ? 1 : 64 * RP];
  double abuf[4][MOM ? 1 : 64 * kG3Blk];
  alignas(16) double ring[4][NA][kG3Ring][64 * 2];
};

template <int D, bool COMPACT, bool HAS_Y, bool HAS_NOISE, bool HAS_PF, bool MOM, bool MASKED>
__device__ __forceinline__ void g3_body(
    G3Lds<D, HAS_Y, HAS_NOISE, MOM>& sh, const double* __restrict__ t, int64_t n, int64_t nch,
    const ChainParams* __restrict__ cps,
    const double* __restrict__ noise, const double* __restrict__ pstart, double* __restrict__ rec,
    double* __restrict__ g, double* __restrict__ phi, double* __restrict__ logs,
    double* __restrict__ pf, const double* const* __restrict__ ys, double* __restrict__ alpha_loc,
    double* __restrict__ asend, double* __restrict__ mom) {
  static_assert(!MOM || (HAS_Y && !COMPACT && !HAS_PF), "moments: the data filter only");
  constexpr int L = kG3L;
  constexpr int RS = COMPACT ? CRec<D>::size : Rec<D>::size;
  constexpr int RP = Rec<D>::size + 1;
  constexpr int NA = 1 + (HAS_Y ? 1 : 0) + (HAS_NOISE ? 1 : 0);   // input arrays staged
  constexpr int S = g3_stores_per_block<D, COMPACT, HAS_PF, MOM, MASKED>(HAS_Y);
  constexpr int VM = S + 2 * NA;   // ops allowed in flight at a block's wait
  static_assert(VM <= 63, "vmcnt holds at most 63 outstanding operations");
  auto& rbuf = sh.rbuf;
  auto& abuf = sh.abuf;
  auto& ring = sh.ring;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t jw = j - lane;
  const bool jv = !MASKED || j < nch;
  const int64_t jc = jv ? j : nch - 1;   // the chunk whose inputs this lane reads
  const int p = blockIdx.y;
  const ChainParams cp = cps[p];
  const int64_t k0 = jc * L;
  const int64_t k1 = MASKED ? (k0 + L < n ? k0 + L : n) : k0 + L;
  const int qmax = (int)((k1 - 1 - k0) >> 1);   // the last pair holding a valid step
  double P[D][D];
  if (jc == 0) {
    sde_pinf<D>(cp.s, P);
  } else {
    const double* ps = pstart + ((int64_t)p * nch + jc) * (D * D);
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) P[i][q] = ps[i * D + q];
  }
  double tprev = k0 > 0 ? t[k0 - 1] : 0.0;
  const double* yp = HAS_Y ? ys[p] : nullptr;
  double* ap = HAS_Y ? alpha_loc + (int64_t)p * n : nullptr;
  double* rp = rec + (int64_t)p * n * RS;
  double* gp = g + (int64_t)p * n * kGStride;
  double* pfp = HAS_PF ? pf + (int64_t)p * n * (D * D) : nullptr;
  double* rb = rbuf[wave];
  double* ab = abuf[wave];
  double* sink = g_gains_sink + 16 * lane;   // masked stores (MASKED only)
  // every ordinary load is retired here, where hipcc can see it: none may stay pending into the
  // loop, whose asm operations hipcc does not count
  __builtin_amdgcn_s_waitcnt(0);
  const double* src[NA];
  src[0] = t + k0;
  if constexpr (HAS_Y) src[1] = yp + k0;
  if constexpr (HAS_NOISE) src[NA - 1] = noise + k0;
  const uint32_t ring0 =
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)(&ring[wave][0][0][0]);
  // pair q of every array into ring slot q % kG3Ring (a pair past the chunk's last valid one
  // re-reads that one: in bounds, never consumed)
  auto issue_pair = [&](int q) __attribute__((always_inline)) {
    const int qq = MASKED ? (q < qmax ? q : qmax) : (q < L / 2 ? q : 0);
#pragma unroll
    for (int a = 0; a < NA; ++a)
      g3_dma16(src[a] + 2 * qq, ring0 + (uint32_t)(((a * kG3Ring) + (q % kG3Ring)) * 1024));
  };
  issue_pair(0);
  issue_pair(1);
  double Phi[D][D];
  mat_eye(Phi);
  double lsum = 0.0;
  double ma[D];
#pragma unroll
  for (int i = 0; i < D; ++i) ma[i] = 0.0;
  double ms[MOM ? kMomStride : 1];
#pragma unroll
  for (int e = 0; e < (MOM ? kMomStride : 1); ++e) ms[e] = 0.0;
  for (int sb = 0; sb < L; sb += kG3Blk) {
    const int q0 = sb / 2;
    issue_pair(q0 + 2);
    issue_pair(q0 + 3);
    // block b's pairs were issued before block b - 1's S stores and block b + 1's 2 NA DMAs
    // (block 0: before block 1's DMAs only)
    if (sb == 0)
      asm volatile("s_waitcnt vmcnt(%0)" : : "n"(2 * NA) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" : : "n"(VM) : "memory");
    // the block's inputs: two pairs per array, one 16-byte LDS read per pair
    double tin[kG3Blk], rin[kG3Blk], yin[kG3Blk];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int slot = (q0 + h) % kG3Ring;
      const g3d2 tv = *reinterpret_cast<const g3d2*>(&ring[wave][0][slot][2 * lane]);
      tin[2 * h] = tv.x;
      tin[2 * h + 1] = tv.y;
      if constexpr (HAS_Y) {
        const g3d2 yv = *reinterpret_cast<const g3d2*>(&ring[wave][1][slot][2 * lane]);
        yin[2 * h] = yv.x;
        yin[2 * h + 1] = yv.y;
      }
      if constexpr (HAS_NOISE) {
        const g3d2 rv = *reinterpret_cast<const g3d2*>(&ring[wave][NA - 1][slot][2 * lane]);
        rin[2 * h] = rv.x;
        rin[2 * h + 1] = rv.y;
      }
    }
#pragma unroll
    for (int u = 0; u < kG3Blk; ++u) {
      const int sidx = sb + u;
      const int64_t k = k0 + sidx;
      const bool live = !MASKED || (jv && k < k1);
      const double tk = tin[u];
      double A[D][D], Q[D][D], X[D][D], Pm[D][D];
      step_model_tau<D>((k == 0) ? 1.0 : (tk - tprev) / cp.l, cp, A, Q);
      tprev = tk;
      mat_mul(A, P, X);
      mat_mul_bt(X, A, Pm);
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int q = 0; q < D; ++q) Pm[i][q] += Q[i][q];
      const double R = HAS_NOISE ? (rin[u] < 0.0 ? cp.r : rin[u]) : cp.r;
      const double Sv = Pm[0][0] + R;
      const double rs = 1.0 / sqrt(Sv);
      double Kg[D];
#pragma unroll
      for (int i = 0; i < D; ++i) Kg[i] = Pm[i][0] / Sv;
      double AP[D][D];
      mat_mul(A, Phi, AP);
      // park the record {A, K, rs, pad} (COMPACT: {K, rs, pad})
      constexpr int KO = COMPACT ? 0 : D * D;
      if constexpr (!MOM) {
        if constexpr (!COMPACT) {
#pragma unroll
          for (int i = 0; i < D; ++i)
#pragma unroll
            for (int q = 0; q < D; ++q) rb[lane * RP + i * D + q] = A[i][q];
        }
#pragma unroll
        for (int i = 0; i < D; ++i) rb[lane * RP + KO + i] = Kg[i];
        rb[lane * RP + KO + D] = rs;
#pragma unroll
        for (int e = KO + D + 1; e < RS; ++e) rb[lane * RP + e] = 0.0;
      }
      double gk[kGStride];
#pragma unroll
      for (int q = 0; q < kGStride; ++q) gk[q] = q < D ? -rs * AP[0][q] : 0.0;
      if (live) {
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) P[i][q] = Pm[i][q] - Kg[i] * Pm[0][q];
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) Phi[i][q] = AP[i][q] - Kg[i] * AP[0][q];
        lsum += log(Sv);
      }
      if constexpr (HAS_Y) {   // alpha filter from zero (whiten_kfu's column recursion)
        double mm[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
          double a2 = 0.0;
#pragma unroll
          for (int q = 0; q < D; ++q) a2 = fma(A[i][q], ma[q], a2);
          mm[i] = a2;
        }
        const double ev = yin[u] - mm[0];
        if constexpr (MOM) {
          // every term selected on live: a step past the chunk's end re-runs stale inputs (its
          // tau may be negative, S_k then negative and rs NaN), so no product of it may reach ms
          const double al = live ? ev * rs : 0.0;
          ms[0] = fma(al, al, ms[0]);
          int e = 1 + D;
#pragma unroll
          for (int i = 0; i < D; ++i) {
            ms[1 + i] = live ? fma(al, gk[i], ms[1 + i]) : ms[1 + i];
#pragma unroll
            for (int q = i; q < D; ++q) {
              ms[e] = live ? fma(gk[i], gk[q], ms[e]) : ms[e];
              ++e;
            }
          }
        } else {
          ab[lane * kG3Blk + u] = ev * rs;
        }
        if (live) {
#pragma unroll
          for (int i = 0; i < D; ++i) ma[i] = fma(Kg[i], ev, mm[i]);
        }
      }
      if constexpr (HAS_PF) {   // the filtered covariance, straight from registers (16-byte pieces)
        double pv[2 * ((D * D + 1) / 2)];
#pragma unroll
        for (int e = 0; e < D * D; ++e) pv[e] = P[e / D][e % D];
        if constexpr ((D * D) % 2) pv[D * D] = 0.0;
        double* dst = live ? pfp + k * (D * D) : sink;
#pragma unroll
        for (int e = 0; e + 1 < D * D; e += 2) g3_store16(dst + e, g3d2{pv[e], pv[e + 1]});
        if constexpr ((D * D) % 2) {
          // odd count: the last double as an 8-byte store, padded to one 16-byte piece's count
          g3_store8(dst + D * D - 1, pv[D * D - 1]);
        }
      }
      if constexpr (!MOM) {
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's parked values landed
        __builtin_amdgcn_wave_barrier();
        // write back: lane -> (record rr = e / (RS/2), 16-byte piece e % (RS/2))
#pragma unroll
        for (int it = 0; it < RS / 2; ++it) {
          const int e = it * 64 + lane;
          const int rr = e / (RS / 2), pc = e % (RS / 2);
          const int64_t kr = (jw + rr) * L + sidx;
          double* dst = (!MASKED || (jw + rr < nch && kr < n)) ? rp + kr * RS + 2 * pc : sink;
          g3_store16(dst, g3d2{rb[rr * RP + 2 * pc], rb[rr * RP + 2 * pc + 1]});
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < kGStride; ++q) rb[lane * RP + q] = gk[q];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const int e = it * 64 + lane;
          const int rr = e >> 1, pc = e & 1;
          const int64_t kr = (jw + rr) * L + sidx;
          double* dst = (!MASKED || (jw + rr < nch && kr < n)) ? gp + kr * kGStride + 2 * pc : sink;
          g3_store16(dst, g3d2{rb[rr * RP + 2 * pc], rb[rr * RP + 2 * pc + 1]});
        }
        __builtin_amdgcn_wave_barrier();   // rb is rewritten by the next step
      }
    }
    if constexpr (HAS_Y && !MOM) {   // the block's alpha values: 64 chunks x 4 steps, 16 bytes per lane
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int e = it * 64 + lane;
        const int rr = e >> 1, pc = e & 1;
        const int64_t kr = (jw + rr) * L + sb + 2 * pc;
        if constexpr (MASKED) {   // two 8-byte halves, each committed only inside the chunk
          const int64_t kend = ((jw + rr) * L + L < n) ? (jw + rr) * L + L : n;
          const bool cv = jw + rr < nch;
          g3_store8((cv && kr < kend) ? ap + kr : sink, ab[rr * kG3Blk + 2 * pc]);
          g3_store8((cv && kr + 1 < kend) ? ap + kr + 1 : sink + 1, ab[rr * kG3Blk + 2 * pc + 1]);
        } else {
          g3_store16(ap + kr, g3d2{ab[rr * kG3Blk + 2 * pc], ab[rr * kG3Blk + 2 * pc + 1]});
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" : : : "memory");   // the ring's last DMAs land before exit
  if (!jv) return;
  const int64_t jo = MOM ? run_slot(p, j, nch) : (int64_t)p * nch + j;
  double* ph = phi + jo * (D * D);
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) ph[i * D + q] = Phi[i][q];
  logs[jo] = lsum;
  if constexpr (HAS_Y) {
    double* sp = asend + jo * kSStride;
#pragma unroll
    for (int i = 0; i < kSStride; ++i) sp[i] = i < D ? ma[i] : 0.0;
  }
  if constexpr (MOM) {
    double* mp_ = mom + jo * kMomStride;
#pragma unroll
    for (int e = 0; e < kMomStride; ++e) mp_[e] = ms[e];
  }
}

// one launch per chain group: blocks 0 .. gridDim.x - 2 are whole (256 chunks of L steps), the
// last block of each chain runs the masked body, concurrently with the others (a separate
// launch of it used to serialise one more 256-step recursion behind the whole blocks)
// (the full-record data-filter variants of the 3-state model need the whole register file for
// the masked body: under a 2-blocks bound they spill)
template <int D, bool COMPACT, bool HAS_Y, bool HAS_NOISE, bool HAS_PF>
constexpr int g3_min_blocks() {
  return (D == 3 && !COMPACT && HAS_Y && !HAS_NOISE && !HAS_PF) ? 1 : 2;
}

template <int D, bool COMPACT, bool HAS_Y, bool HAS_NOISE, bool HAS_PF, bool MOM>
__global__ __launch_bounds__(256, (g3_min_blocks<D, COMPACT, HAS_Y, HAS_NOISE, HAS_PF>())) void
gains_phase3_fast(
    const double* __restrict__ t, int64_t n, int64_t nch, const ChainParams* __restrict__ cps,
    const double* __restrict__ noise, const double* __restrict__ pstart, double* __restrict__ rec,
    double* __restrict__ g, double* __restrict__ phi, double* __restrict__ logs,
    double* __restrict__ pf, const double* const* __restrict__ ys, double* __restrict__ alpha_loc,
    double* __restrict__ asend, double* __restrict__ mom) {
  __shared__ G3Lds<D, HAS_Y, HAS_NOISE, MOM> sh;
  if (blockIdx.x + 1 == gridDim.x)
    g3_body<D, COMPACT, HAS_Y, HAS_NOISE, HAS_PF, MOM, true>(sh, t, n, nch, cps, noise, pstart, rec,
                                                             g, phi, logs, pf, ys, alpha_loc,
                                                             asend, mom);
  else
    g3_body<D, COMPACT, HAS_Y, HAS_NOISE, HAS_PF, MOM, false>(sh, t, n, nch, cps, noise, pstart,
                                                              rec, g, phi, logs, pf, ys, alpha_loc,
                                                              asend, mom);
}

// ---------------------------------------------------------------------------- whitening of Kfu columns
// beta_loc[k, c] = chunk-local whitened Kfu[k, c] with Kfu computed on the fly:
// Kfu[k, c] = s_o kappa(||v_k - z_c|| / l_o)   (Stheno pairwise, dtc.jl:104).
// grid: (nch, ceil(mp / 256)); block 256, one column per thread.
// send[(j * mc + c) * 4 + i] = local end state of chunk j;
// hsum[(j * mc + c) * 4 + i] = sum_{k in chunk j} beta_loc[k, c] g_k[i]  (H_j, the chunk's
// moment against the fix-up rows: the Gram applies the carry fix-up through it, k_gram.hip;
// null: not wanted).
constexpr int kVTile = 32;

template <int TK, int OK, int DP>
__global__ __launch_bounds__(256) void whiten_kfu(
    const double* __restrict__ rec, const double* __restrict__ v, int64_t ldv, int d,
    const double* __restrict__ z, int64_t ldz, int64_t m, int64_t mp, int64_t n, int L,
    double inv_lo, double s_o, double* __restrict__ beta, int64_t ldb, double* __restrict__ send,
    int64_t mc, const double* __restrict__ g, double* __restrict__ hsum) {
  constexpr int D = Sde<TK>::d;
  constexpr int RS = Rec<D>::size;
  __shared__ __attribute__((aligned(16))) double vs[kVTile][DP];
  __shared__ double gs[kVTile * kGStride];
  const int64_t j = blockIdx.x;
  const int64_t c = (int64_t)blockIdx.y * 256 + threadIdx.x;
  const bool valid = c < m;
  const bool active = c < mp;
  double zr[DP];
#pragma unroll
  for (int i = 0; i < DP; ++i) zr[i] = (valid && i < d) ? z[c * ldz + i] : 0.0;
  double mst[D], hs[D];
#pragma unroll
  for (int i = 0; i < D; ++i) mst[i] = hs[i] = 0.0;
  const int64_t k0 = j * L;
  const int64_t k1 = (k0 + L < n) ? k0 + L : n;
  for (int64_t kt = k0; kt < k1; kt += kVTile) {
    const int nt = (kt + kVTile <= k1) ? kVTile : (int)(k1 - kt);
    __syncthreads();
    for (int e = threadIdx.x; e < kVTile * DP; e += 256) {
      const int kk = e / DP, i = e % DP;
      vs[kk][i] = (kk < nt && i < d) ? v[(kt + kk) * ldv + i] : 0.0;
    }
    if (threadIdx.x < kVTile * kGStride)
      gs[threadIdx.x] = (threadIdx.x < nt * kGStride) ? g[kt * kGStride + threadIdx.x] : 0.0;
    __syncthreads();
    for (int kk = 0; kk < nt; ++kk) {
      const int64_t k = kt + kk;
      double d2a = 0.0, d2b = 0.0;
#pragma unroll
      for (int i = 0; i < DP; i += 2) {
        const double a0 = vs[kk][i] - zr[i];
        d2a = fma(a0, a0, d2a);
        if (i + 1 < DP) {
          const double a1 = vs[kk][i + 1] - zr[i + 1];
          d2b = fma(a1, a1, d2b);
        }
      }
      const double x = valid ? skappa_sq<OK>(d2a + d2b, inv_lo, s_o) : 0.0;
      const double* r = rec + k * RS;
      double mm[D];
#pragma unroll
      for (int i = 0; i < D; ++i) {
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < D; ++q) acc = fma(r[i * D + q], mst[q], acc);
        mm[i] = acc;
      }
      const double ev = x - mm[0];
      const double al = ev * r[D * D + D];
#pragma unroll
      for (int i = 0; i < D; ++i) mst[i] = fma(r[D * D + i], ev, mm[i]);
#pragma unroll
      for (int i = 0; i < D; ++i) hs[i] = fma(al, gs[kk * kGStride + i], hs[i]);
      if (active) beta[k * ldb + c] = al;
    }
  }
  if (active) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      send[(j * mc + c) * kSStride + i] = mst[i];
      if (hsum) hsum[(j * mc + c) * kSStride + i] = hs[i];
    }
  }
}

// ---------------------------------------------------------------------------- whitening of Kfu columns, MFMA form
// Same output as whiten_kfu, with Kfu built by v_mfma_f64_16x16x4_f64 in the Gram form
// |v - z|^2 = |v - c|^2 + |z - c|^2 - 2 (v - c).(z - c)  (Distances.jl's pairwise form as used by
// Stheno), centred to limit
// cancellation (c = mean of the block's 256 pseudo-inputs).  Per 16-step sub-tile and wave (64 columns): DP/4 x 4 MFMAs give the 16 x 64
// cross products in the C layout (lane: column ct*16 + (l&15), steps (l>>4) + 4r), the kernel
// values are evaluated there (16 per lane, independent -> ILP), transposed through LDS, and the
// lane of column c then runs the 16 filter steps.  Used for the smooth kernels (Matern-3/2,
// Matern-5/2, EQ: a d^2 error of eps |v - c| |z - c| is harmless); Matern-1/2 keeps the direct
// form (its kappa is not smooth in d^2 at 0).
constexpr int kMT = 16;   // steps per sub-tile

template <int TK, int OK, int DP>
__global__ __launch_bounds__(256, 2) void whiten_kfu_mfma(
    const double* __restrict__ rec, const double* __restrict__ v, int64_t ldv, int d,
    const double* __restrict__ z, int64_t ldz, const double* __restrict__ zc, int64_t m,
    int64_t mp, int64_t n, int L, double inv_lo, double s_o, double* __restrict__ beta,
    int64_t ldb, double* __restrict__ send, int64_t mc, const double* __restrict__ g,
    double* __restrict__ hsum) {
  typedef double d4 __attribute__((ext_vector_type(4)));
  constexpr int SD = Sde<TK>::d;
  constexpr int RS = Rec<SD>::size;
  constexpr int VS = DP + 2;      // V tile row stride: conflict-free A-fragment reads
  constexpr int NKS = DP / 4;
  __shared__ __attribute__((aligned(16))) double vs[kMT * VS];
  __shared__ __attribute__((aligned(16))) double xt[4][kMT][65];
  // the sub-tile's step rows {A_k (SD x SD), K_k (SD), rs_k, g_k (SD)}, 16 doubles each (fmac_row)
  constexpr int RK = SD * SD, RR = SD * SD + SD, RG = SD * SD + SD + 1;
  static_assert(RG + SD <= 16, "step row");
  __shared__ __attribute__((aligned(16))) double rg[kMT * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t j = blockIdx.x;
  const int64_t cw0 = (int64_t)blockIdx.y * 256 + wave * 64;   // wave's first column
  const int64_t col = cw0 + lane;                               // recursion column of this lane
  const int fr = lane & 15, fq = lane >> 4;
  // centre of this block's 256 pseudo-inputs (subtracted from V while staging, from Z here)
  const double* cg = zc + (int64_t)blockIdx.y * DP;
  // B fragments (z - c) and |z - c|^2 of the C-layout columns ct*16 + fr
  double bf[4][NKS];
  double zn[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const int64_t zcol = cw0 + ct * 16 + fr;
    const bool zv = zcol < m;
    const int64_t zcc = zv ? zcol : 0;
    double part = 0.0;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int dim = 4 * ks + fq;
      const double zz = (zv && dim < d) ? z[zcc * ldz + dim] - cg[dim] : 0.0;
      bf[ct][ks] = zz;
      part = fma(zz, zz, part);
    }
    part += __shfl_xor(part, 16, 64);
    part += __shfl_xor(part, 32, 64);
    zn[ct] = part;   // full |z - c|^2 of column ct*16 + fr (dims padded with zeros)
  }
  const int nks = (d + 3) / 4;
  double mst[SD], hs[SD];
#pragma unroll
  for (int i = 0; i < SD; ++i) mst[i] = hs[i] = 0.0;
  const int64_t k0 = j * L;
  const int64_t k1 = (k0 + L < n) ? k0 + L : n;
  const bool colv = col < m, cola = col < mp;
  // next sub-tile's V rows and gains records are prefetched into registers (one MFMA /
  // kernel-evaluation phase ahead) and written to LDS between the two barriers.  The loads are
  // unconditional (clamped in-bounds addresses) and the masks are applied at commit, so no wait
  // is forced at the load: vmcnt also counts this wave's beta stores, and a wait right after
  // the prefetch would stall on the previous sub-tile's 16 stores.
  constexpr int VPT = (kMT * DP + 255) / 256;   // V elements per thread
  double pv[VPT], pcg[VPT], pr, pg;
  int pkk[VPT], pii[VPT];
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    const int e = tid + q * 256;
    pkk[q] = e < kMT * DP ? e / DP : kMT;   // row kMT: never committed
    pii[q] = e % DP;
    pcg[q] = pii[q] < d ? cg[pii[q]] : 0.0;
  }
  const int dl = d - 1;
  auto prefetch = [&](int64_t kt_) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      int64_t kr = kt_ + (pkk[q] < kMT ? pkk[q] : 0);
      kr = kr < n ? kr : n - 1;
      pv[q] = v[kr * ldv + (pii[q] < d ? pii[q] : dl)];
    }
    int64_t ir = kt_ * RS + tid;
    pr = rec[ir < n * RS ? ir : n * RS - 1];
    int64_t ig = kt_ * kGStride + tid;
    pg = g[ig < n * kGStride ? ig : n * kGStride - 1];
  };
  auto commit = [&](int nt_) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      const int e = tid + q * 256;
      if (e < kMT * DP)
        vs[pkk[q] * VS + pii[q]] = (pkk[q] < nt_ && pii[q] < d) ? pv[q] - pcg[q] : 0.0;
    }
    if (tid < kMT * RS && tid % RS < RG) rg[tid / RS * 16 + tid % RS] = tid < nt_ * RS ? pr : 0.0;
    if (tid < kMT * kGStride && tid % kGStride < SD)
      rg[tid / kGStride * 16 + RG + tid % kGStride] = tid < nt_ * kGStride ? pg : 0.0;
  };
  // beta of a sub-tile is left in the wave's xt rows by the recursion and flushed to HBM at the
  // start of the next iteration, after commit's wait: the stores then drain behind a whole
  // sub-tile of compute before the next wait on this wave's vmcnt.
  int ntp = 0;
  int64_t ktp = k0;
  // Lane l stores rows 2i + l/32, column pair 2(l%32), +1 of the wave's 64 columns: 8 x 16 B
  // stores per sub-tile instead of 16 x 8 B (store issue, not bandwidth, bounds this tail).
  const int fh = lane >> 5, fc2 = (lane & 31) * 2;
  auto flush = [&]() __attribute__((always_inline)) {
    if (cw0 < mp && ntp == kMT) {   // all LDS reads first, then the 8 stores (no per-row branch)
      double2 v2[kMT / 2];
#pragma unroll
      for (int i = 0; i < kMT / 2; ++i) {
        v2[i].x = xt[wave][2 * i + fh][fc2];
        v2[i].y = xt[wave][2 * i + fh][fc2 + 1];
      }
#pragma unroll
      for (int i = 0; i < kMT / 2; ++i)
        *reinterpret_cast<double2*>(beta + (ktp + 2 * i + fh) * ldb + cw0 + fc2) = v2[i];
    } else if (cw0 < mp) {   // mp is a multiple of 128: whole waves are in or out
#pragma unroll
      for (int i = 0; i < kMT / 2; ++i) {
        const int kk = 2 * i + fh;
        if (kk < ntp) {
          double2 v2;
          v2.x = xt[wave][kk][fc2];
          v2.y = xt[wave][kk][fc2 + 1];
          *reinterpret_cast<double2*>(beta + (ktp + kk) * ldb + cw0 + fc2) = v2;
        }
      }
    }
  };
  if (k0 < k1) prefetch(k0);
  for (int64_t kt = k0; kt < k1; kt += kMT) {
    const int nt = (kt + kMT <= k1) ? kMT : (int)(k1 - kt);
    __syncthreads();
    commit(nt);
    __syncthreads();
    flush();
    if (kt + kMT < k1) prefetch(kt + kMT);
    // cross products (v - c).(z - c) and the step norms |v - c|^2
    d4 acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = d4{0.0, 0.0, 0.0, 0.0};
    // DP <= 32: all A fragments are read before the first MFMA (dims >= d are staged as zeros,
    // so the norm runs over every ks and keeps the reads unconditional: one LDS latency per
    // sub-tile instead of one per ks); the MFMAs skip ks >= nks.  DP >= 48 keeps the per-ks
    // form: its VGPRs are already at the limit.
    double vnp = 0.0;
    if constexpr (DP <= 32) {
      double af[NKS];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) af[ks] = vs[fr * VS + 4 * ks + fq];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) vnp = fma(af[ks], af[ks], vnp);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        if (ks < nks) {
#pragma unroll
          for (int ct = 0; ct < 4; ++ct)
            acc[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[ks], bf[ct][ks], acc[ct], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        if (ks < nks) {
          const double a = vs[fr * VS + 4 * ks + fq];
          vnp = fma(a, a, vnp);
#pragma unroll
          for (int ct = 0; ct < 4; ++ct)
            acc[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bf[ct][ks], acc[ct], 0, 0, 0);
        }
      }
    }
    vnp += __shfl_xor(vnp, 16, 64);
    vnp += __shfl_xor(vnp, 32, 64);   // lanes fr, fr+16, fr+32, fr+48 hold |v_fr - c|^2
    // kernel values in the C layout: step fq + 4 r, column ct*16 + fr
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double vn = __shfl(vnp, fq + 4 * r, 64);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        double d2 = vn + zn[ct] - 2.0 * acc[ct][r];
        if constexpr (OK == KEQ) d2 = d2 > 0.0 ? d2 : 0.0;   // the Matern forms clamp in sqrt_pos
        xt[wave][fq + 4 * r][ct * 16 + fr] = skappa_sq<OK>(d2, inv_lo, s_o);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
    auto step = [&](int kk, double x, double row) __attribute__((always_inline)) {
      double mm[SD];
      static_for<SD>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        double a2 = 0.0;
        static_for<SD>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          a2 = fmac_row<i * SD + q>(a2, row, mst[q]);
        });
        mm[i] = a2;
      });
      const double ev = x - mm[0];
      const double al = ev * bcast_row<RR>(row);
      static_for<SD>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        mst[i] = fmac_row<RK + i>(mm[i], row, ev);
        hs[i] = fmac_row<RG + i>(hs[i], row, al);
      });
      xt[wave][kk][lane] = al;
    };
    auto xval = [&](int kk) __attribute__((always_inline)) { return colv ? xt[wave][kk][lane] : 0.0; };
    auto rval = [&](int kk) __attribute__((always_inline)) { return rg[kk * 16 + (lane & 15)]; };
    if (nt == kMT) {   // unrolled, each step's x and row read kPW steps ahead of their use
      constexpr int kPW = DP <= 32 ? 8 : 4;
      double xs[kMT], rows[kMT];
#pragma unroll
      for (int kk = 0; kk < kPW; ++kk) {
        xs[kk] = xval(kk);
        rows[kk] = rval(kk);
      }
#pragma unroll
      for (int kk = 0; kk < kMT; ++kk) {
        if (kk + kPW < kMT) {
          xs[kk + kPW] = xval(kk + kPW);
          rows[kk + kPW] = rval(kk + kPW);
        }
        step(kk, xs[kk], rows[kk]);
      }
    } else {
      for (int kk = 0; kk < nt; ++kk) step(kk, xval(kk), rval(kk));
    }
    ntp = nt;
    ktp = kt;
  }
  flush();
  if (cola) {
#pragma unroll
    for (int i = 0; i < SD; ++i) {
      send[(j * mc + col) * kSStride + i] = mst[i];
      if (hsum) hsum[(j * mc + col) * kSStride + i] = hs[i];
    }
  }
}

// Centres of the pseudo-input column groups (256 columns each): zc[g][i] = mean_c z[c][i].
// Block of 256 threads = dp dims x (256 / dp) column lanes, 8 independent loads in flight per
// thread, partial sums combined through LDS in a fixed order.
__global__ __launch_bounds__(256) void zcenter_kernel(const double* __restrict__ z, int64_t ldz,
                                                      int d, int64_t m, int dp,
                                                      double* __restrict__ zc) {
  __shared__ double red[256];
  const int64_t g = blockIdx.x;
  const int i = threadIdx.x % dp, q = threadIdx.x / dp, nq = 256 / dp;
  const int64_t c0 = g * 256, c1 = (c0 + 256 < m) ? c0 + 256 : m;
  double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (i < d && q < nq) {   // dp = 48: threads 240..255 idle
    for (int64_t c = c0 + q; c < c1; c += 8 * nq) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t cc = c + (int64_t)u * nq;
        if (cc < c1) s[u] += z[cc * ldz + i];
      }
    }
  }
  red[threadIdx.x] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (threadIdx.x < dp) {
    double t = 0.0;
    for (int u = 0; u < nq; ++u) t += red[u * dp + threadIdx.x];
    const int64_t cnt = c1 - c0;
    zc[g * dp + threadIdx.x] = (cnt > 0 && threadIdx.x < d) ? t / (double)cnt : 0.0;
  }
}

// ---------------------------------------------------------------------------- whitening of a vector per chain
// One 64-lane wave per (chunk, chain).  The chunk's filter from a zero state is the affine
// recurrence m_k = Abar_k m_{k-1} + K_k x_k (Abar_k = (I - K_k e1^T) A_k), so it is scanned
// in parallel: lane l filters steps 4l..4l+3 from zero (alpha', local end state e_l, transfer
// T_l, and gamma_k = -rs_k (A_k T_{k-1})[0, :]), a Hillis-Steele scan over the 64 lanes composes
// (T, e) into each segment's incoming state s_l, and alpha_k = alpha'_k + gamma_k . s_l.
// x_c[k] = y[c * ldy + k]; alpha_loc[c * lda + k * astride]; chunk end state (from zero at the
// chunk start; the carry across chunks is vec_fix's) -> send[c * sendstride + (j * mc + col) * 4].
constexpr int kVecL = 256;   // == host chunk length (64 lanes x 4 steps)
constexpr int kVecSeg = kVecL / 64;

__device__ __forceinline__ double shfl_up_d(double v, int off, int lane) {
  return __shfl(v, lane >= off ? lane - off : lane, 64);
}

template <int D>
__global__ __launch_bounds__(64) void whiten_vec(const double* __restrict__ rec, int64_t recstride,
                                                 const double* __restrict__ y, int64_t ldy,
                                                 int64_t n, int L, int64_t nch,
                                                 double* __restrict__ alpha, int64_t lda,
                                                 double* __restrict__ send, int64_t sendstride,
                                                 int64_t mc, int64_t col, int64_t astride) {
  constexpr int RS = Rec<D>::size;
  const int64_t j = blockIdx.x;
  const int c = blockIdx.y;
  const int lane = threadIdx.x;
  const double* rp = rec + (int64_t)c * recstride;
  const double* yp = y + (int64_t)c * ldy;
  const int64_t k0 = j * L + (int64_t)lane * kVecSeg;
  const int64_t kend = (j * L + L < n) ? j * L + L : n;
  // ---- local pass over this lane's segment
  double m[D], T[D][D], gam[kVecSeg][D], al[kVecSeg];
#pragma unroll
  for (int i = 0; i < D; ++i) m[i] = 0.0;
  mat_eye(T);
#pragma unroll
  for (int u = 0; u < kVecSeg; ++u) {
    const int64_t k = k0 + u;
    const bool live = k < kend;
    const double* r = rp + (live ? k : 0) * RS;
    double A[D][D], K[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
#pragma unroll
      for (int q = 0; q < D; ++q) A[i][q] = live ? r[i * D + q] : (i == q ? 1.0 : 0.0);
      K[i] = live ? r[D * D + i] : 0.0;
    }
    const double rs = live ? r[D * D + D] : 0.0;
    const double x = live ? yp[k] : 0.0;
    double mm[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < D; ++q) acc = fma(A[i][q], m[q], acc);
      mm[i] = acc;
    }
    const double ev = x - mm[0];
    al[u] = ev * rs;
#pragma unroll
    for (int i = 0; i < D; ++i) m[i] = fma(K[i], ev, mm[i]);
    // gamma = -rs (A T)[0, :];  T <- (I - K e1^T) A T
    double AT[D][D];
    mat_mul(A, T, AT);
#pragma unroll
    for (int q = 0; q < D; ++q) gam[u][q] = -rs * AT[0][q];
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) T[i][q] = fma(-K[i], AT[0][q], AT[i][q]);
  }
  // ---- inclusive scan of the segment maps s -> T s + e over the lanes
  double e[D];
#pragma unroll
  for (int i = 0; i < D; ++i) e[i] = m[i];
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    double Tp[D][D], ep[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      ep[i] = shfl_up_d(e[i], off, lane);
#pragma unroll
      for (int q = 0; q < D; ++q) Tp[i][q] = shfl_up_d(T[i][q], off, lane);
    }
    if (lane >= off) {
      double Tn[D][D], en[D];
#pragma unroll
      for (int i = 0; i < D; ++i) {
        double acc = e[i];
#pragma unroll
        for (int q = 0; q < D; ++q) acc = fma(T[i][q], ep[q], acc);
        en[i] = acc;
      }
      mat_mul(T, Tp, Tn);
#pragma unroll
      for (int i = 0; i < D; ++i) {
        e[i] = en[i];
#pragma unroll
        for (int q = 0; q < D; ++q) T[i][q] = Tn[i][q];
      }
    }
  }
  // incoming state of segment l = inclusive result of lane l - 1
  double sin_[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    const double v = shfl_up_d(e[i], 1, lane);
    sin_[i] = lane > 0 ? v : 0.0;
  }
  double* ap = alpha + (int64_t)c * lda;
#pragma unroll
  for (int u = 0; u < kVecSeg; ++u) {
    const int64_t k = k0 + u;
    double a = al[u];
#pragma unroll
    for (int q = 0; q < D; ++q) a = fma(gam[u][q], sin_[q], a);
    if (k < kend) ap[k * astride] = a;
  }
  if (lane == 63) {
    double* sp = send + (int64_t)c * sendstride;
#pragma unroll
    for (int i = 0; i < D; ++i) sp[(j * mc + col) * kSStride + i] = e[i];
  }
}

// ---------------------------------------------------------------------------- carry over chunks
// cin[j][c] = true filter state at the start of chunk j: cin[0] = 0,
// cin[j+1] = Phi_j cin[j] + send[j].  Two-level: groups of GS chunks.
//   a) per (group, column): group end state from zero            -> gend
//   b) per group: Psi_g = prod Phi_j over the group               -> psi
//   c) per column: sequential over groups                          -> gin
//   d) per (group, column): re-propagate inside the group          -> cin
// Chains (blockIdx.z) are independent; per-chain strides: phistride, sstride (send/cin),
// gstride_ (gend/gin), psistride.
// REV: the adjoint's backward carry (chunks visited last to first, Phi transposed):
// out[J-1] = 0, out[j] = Phi_{j+1}^T out[j+1] + b_{j+1}.
template <int D, bool REV>
__device__ __forceinline__ void carry_step(const double* __restrict__ ph, int64_t r,
                                           const double* __restrict__ sv, double (&st)[D]) {
  double nx[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    double acc = sv[i];
#pragma unroll
    for (int q = 0; q < D; ++q)
      acc = fma(REV ? ph[r * D * D + q * D + i] : ph[r * D * D + i * D + q], st[q], acc);
    nx[i] = acc;
  }
#pragma unroll
  for (int i = 0; i < D; ++i) st[i] = nx[i];
}

// The group's chunk transitions, staged once per block into LDS (uniform across the block's
// columns): read from memory inside the sequential loop they were scalar loads, each waited on.
constexpr int kMaxCarryGS = 128;   // carry_group_size caps the group length here
template <int D, bool REV>
__device__ __forceinline__ void stage_phi(const double* __restrict__ ph, int64_t nch, int64_t j0,
                                          int64_t j1, double* __restrict__ lph) {
  const int cnt = (int)(j1 - j0) * D * D;
  for (int e = threadIdx.x; e < cnt; e += blockDim.x) {
    const int64_t jj = j0 + e / (D * D);
    const int64_t r = REV ? nch - 1 - jj : jj;
    lph[e] = ph[r * D * D + e % (D * D)];
  }
  __syncthreads();
}

template <int D, bool REV>
__global__ __launch_bounds__(256) void carry_group_local(const double* __restrict__ phi, int64_t phistride,
                                                         const double* __restrict__ send, int64_t sstride,
                                                         int64_t nch, int64_t mc, int64_t ncols, int GS,
                                                         double* __restrict__ gend, int64_t gstride_,
                                                         double* __restrict__ psi, int64_t psistride) {
  __shared__ double lph[kMaxCarryGS * D * D];
  const int64_t gidx = blockIdx.y;
  const int b = blockIdx.z;
  const double* ph = phi + (int64_t)b * phistride;
  const double* sp = send + (int64_t)b * sstride;
  const int64_t j0 = gidx * GS;
  const int64_t j1 = (j0 + GS < nch) ? j0 + GS : nch;
  stage_phi<D, REV>(ph, nch, j0, j1, lph);
  if (blockIdx.x == gridDim.x - 1) {   // the extra column block: the group's Psi = prod Phi_j
    if (threadIdx.x == 0) {
      double P[D][D], X[D][D], F[D][D];
      mat_eye(P);
      for (int64_t j = j0; j < j1; ++j) {
        const double* f = lph + (j - j0) * D * D;
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) F[i][q] = REV ? f[q * D + i] : f[i * D + q];
        mat_mul(F, P, X);
        mat_copy(X, P);
      }
      double* pp = psi + (int64_t)b * psistride + gidx * D * D;
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int q = 0; q < D; ++q) pp[i * D + q] = P[i][q];
    }
    return;
  }
  const int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (c >= ncols) return;
  double st[D];
#pragma unroll
  for (int i = 0; i < D; ++i) st[i] = 0.0;
#pragma unroll 16
  for (int64_t j = j0; j < j1; ++j) {
    const int64_t r = REV ? nch - 1 - j : j;
    carry_step<D, REV>(lph + (j - j0) * D * D, 0, sp + (r * mc + c) * kSStride, st);
  }
  double* ge = gend + (int64_t)b * gstride_ + (gidx * mc + c) * kSStride;
#pragma unroll
  for (int i = 0; i < D; ++i) ge[i] = st[i];
}

template <int D, bool REV>
__global__ __launch_bounds__(256) void carry_group_phi(const double* __restrict__ phi, int64_t phistride,
                                                       int64_t nch, int GS, int64_t ngroups,
                                                       double* __restrict__ psi, int64_t psistride) {
  const int64_t gidx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (gidx >= ngroups) return;
  const double* ph = phi + (int64_t)b * phistride;
  const int64_t j0 = gidx * GS;
  const int64_t j1 = (j0 + GS < nch) ? j0 + GS : nch;
  double P[D][D], X[D][D], F[D][D];
  mat_eye(P);
  for (int64_t j = j0; j < j1; ++j) {
    const int64_t r = REV ? nch - 1 - j : j;
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q)
        F[i][q] = REV ? ph[r * D * D + q * D + i] : ph[r * D * D + i * D + q];
    mat_mul(F, P, X);
    mat_copy(X, P);
  }
  double* ps = psi + (int64_t)b * psistride + gidx * D * D;
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) ps[i * D + q] = P[i][q];
}

template <int D>
__global__ __launch_bounds__(256) void carry_group_scan(const double* __restrict__ psi, int64_t psistride,
                                                        const double* __restrict__ gend,
                                                        double* __restrict__ gin, int64_t gstride_,
                                                        int64_t ngroups, int64_t mc, int64_t ncols) {
  const int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (c >= ncols) return;
  const double* ps = psi + (int64_t)b * psistride;
  const double* ge = gend + (int64_t)b * gstride_;
  double* gi = gin + (int64_t)b * gstride_;
  double st[D];
#pragma unroll
  for (int i = 0; i < D; ++i) st[i] = 0.0;
#pragma unroll 8
  for (int64_t g = 0; g < ngroups; ++g) {
    const int64_t o = (g * mc + c) * kSStride;
#pragma unroll
    for (int i = 0; i < D; ++i) gi[o + i] = st[i];
    double nx[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double acc = ge[o + i];
#pragma unroll
      for (int q = 0; q < D; ++q) acc = fma(ps[g * D * D + i * D + q], st[q], acc);
      nx[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < D; ++i) st[i] = nx[i];
  }
}

template <int D, bool REV>
__global__ __launch_bounds__(256) void carry_group_apply(const double* __restrict__ phi, int64_t phistride,
                                                         const double* __restrict__ send,
                                                         double* __restrict__ cin, int64_t sstride,
                                                         const double* __restrict__ gin, int64_t gstride_,
                                                         int64_t nch, int64_t mc, int64_t ncols, int GS) {
  __shared__ double lph[kMaxCarryGS * D * D];
  const int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t gidx = blockIdx.y;
  const int b = blockIdx.z;
  const double* ph = phi + (int64_t)b * phistride;
  const double* sp = send + (int64_t)b * sstride;
  double* cp = cin + (int64_t)b * sstride;
  const int64_t j0 = gidx * GS;
  const int64_t j1 = (j0 + GS < nch) ? j0 + GS : nch;
  stage_phi<D, REV>(ph, nch, j0, j1, lph);
  if (c >= ncols) return;
  const double* gi = gin + (int64_t)b * gstride_ + (gidx * mc + c) * kSStride;
  double st[D];
#pragma unroll
  for (int i = 0; i < D; ++i) st[i] = gi[i];
#pragma unroll 16
  for (int64_t j = j0; j < j1; ++j) {
    const int64_t r = REV ? nch - 1 - j : j;
    const int64_t o = (r * mc + c) * kSStride;
#pragma unroll
    for (int i = 0; i < D; ++i) cp[o + i] = st[i];
    carry_step<D, REV>(lph + (j - j0) * D * D, 0, sp + o, st);
  }
}

// ---------------------------------------------------------------------------- adjoint (Sigma^{-1} = W^T W)
// The whitening alpha = W x is lower triangular; its adjoint u = W^T w runs backwards with the
// same gains records:  u_k = rs_k w_k + K_k . lambda_k,  lambda_{k-1} = A_k^T (lambda_k - u_k e1),
// lambda_{N-1} = 0.  Chunked like the forward pass: from lambda = 0 at each chunk end, then
// u_k(true) = u_k(local) + h_k . chat_j with h_k = Gamma_{j,k}^T K_k,
// Gamma_{j,k1-1} = I, Gamma_{j,k-1} = Abar_k^T Gamma_{j,k}, and the backward carry chat over
// chunks with Phi_j^T (carry kernels, REV = true).
template <int D>
__global__ __launch_bounds__(256) void gains_adjoint(const double* __restrict__ rec, int64_t n,
                                                     int L, int64_t nch, double* __restrict__ h) {
  constexpr int RS = Rec<D>::size;
  const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int p = blockIdx.y;
  if (j >= nch) return;
  const double* rp = rec + (int64_t)p * n * RS;
  double* hp = h + (int64_t)p * n * kGStride;
  const int64_t k0 = j * L;
  const int64_t k1 = (k0 + L < n) ? k0 + L : n;
  double Gm[D][D];
  mat_eye(Gm);
  for (int64_t k = k1 - 1; k >= k0; --k) {
    const double* r = rp + k * RS;
    double A[D][D], K[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      K[i] = r[D * D + i];
#pragma unroll
      for (int q = 0; q < D; ++q) A[i][q] = r[i * D + q];
    }
    // h_k = Gamma^T K
#pragma unroll
    for (int q = 0; q < D; ++q) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < D; ++i) acc = fma(Gm[i][q], K[i], acc);
      hp[k * kGStride + q] = acc;
    }
    // Gamma <- Abar^T Gamma,  Abar = A - K A[0,:]
    double Ab[D][D], X[D][D];
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) Ab[i][q] = A[i][q] - K[i] * A[0][q];
    mat_mul_at(Ab, Gm, X);
    mat_copy(X, Gm);
  }
}

// Backward local pass over a column-major-in-rows matrix X (row k, column c at X[k*ldx + c]):
// reads w = X[k][c] + g_k . cin[j][c] (forward fix-up applied on the fly), writes u_loc in place,
// and the chunk's backward end state (lambda before its first step) to bend[(j*mc + c)*4].
// grid: (nch, ceil(ncols / 64)); block 64 (one column per lane).
template <int D>
__global__ __launch_bounds__(64) void adjoint_local(double* __restrict__ X, int64_t ldx,
                                                    int64_t ncols, const double* __restrict__ rec,
                                                    const double* __restrict__ g,
                                                    const double* __restrict__ cin, int64_t mc,
                                                    int64_t n, int L, double* __restrict__ bend,
                                                    int64_t xstride, int64_t sstride) {
  constexpr int RS = Rec<D>::size;
  const int64_t j = blockIdx.x;
  {
    const int b = blockIdx.z;   // chain: gains (rec, g) are per chain, X / cin / bend strided
    X += (int64_t)b * xstride;
    rec += (int64_t)b * n * RS;
    g += (int64_t)b * n * kGStride;
    cin += (int64_t)b * sstride;
    bend += (int64_t)b * sstride;
  }
  const int64_t c = (int64_t)blockIdx.y * 64 + threadIdx.x;
  const bool act = c < ncols;
  const int64_t cc = act ? c : 0;
  const int64_t k0 = j * L;
  const int64_t k1 = (k0 + L < n) ? k0 + L : n;
  double cf[D];
#pragma unroll
  for (int i = 0; i < D; ++i) cf[i] = cin[(j * mc + cc) * kSStride + i];
  double lam[D];
#pragma unroll
  for (int i = 0; i < D; ++i) lam[i] = 0.0;
#pragma unroll 4
  for (int64_t k = k1 - 1; k >= k0; --k) {
    const double* r = rec + k * RS;
    const double* gk = g + k * kGStride;
    double w = X[k * ldx + cc];
#pragma unroll
    for (int i = 0; i < D; ++i) w = fma(gk[i], cf[i], w);
    double u = w * r[D * D + D];
#pragma unroll
    for (int i = 0; i < D; ++i) u = fma(r[D * D + i], lam[i], u);
    lam[0] -= u;
    double nl[D];
#pragma unroll
    for (int q = 0; q < D; ++q) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < D; ++i) acc = fma(r[i * D + q], lam[i], acc);
      nl[q] = acc;
    }
#pragma unroll
    for (int i = 0; i < D; ++i) lam[i] = nl[i];
    if (act) X[k * ldx + c] = u;
  }
  if (act) {
#pragma unroll
    for (int i = 0; i < D; ++i) bend[(j * mc + c) * kSStride + i] = lam[i];
  }
}

// One column (the temporal chains' smoothing, gpar_lgssm_smooth): one lane per (chunk, chain)
// instead of a 64-lane workgroup per chunk with one lane active (r05: 125 k workgroups, 3.6 ms for
// the ssm config's 16 chains x 2e6 steps).  The same arithmetic per step as adjoint_local.
template <int D>
__global__ __launch_bounds__(256) void adjoint_local_col(double* __restrict__ X,
                                                         const double* __restrict__ rec,
                                                         const double* __restrict__ g,
                                                         const double* __restrict__ cin, int64_t n,
                                                         int L, int64_t nch,
                                                         double* __restrict__ bend,
                                                         int64_t xstride, int64_t sstride) {
  constexpr int RS = Rec<D>::size;
  const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (j >= nch) return;
  X += (int64_t)b * xstride;
  rec += (int64_t)b * n * RS;
  g += (int64_t)b * n * kGStride;
  cin += (int64_t)b * sstride;
  bend += (int64_t)b * sstride;
  const int64_t k0 = j * L;
  const int64_t k1 = (k0 + L < n) ? k0 + L : n;
  double cf[D], lam[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    cf[i] = cin[j * kSStride + i];
    lam[i] = 0.0;
  }
#pragma unroll 4
  for (int64_t k = k1 - 1; k >= k0; --k) {
    const double* r = rec + k * RS;
    const double* gk = g + k * kGStride;
    double w = X[k];
#pragma unroll
    for (int i = 0; i < D; ++i) w = fma(gk[i], cf[i], w);
    double u = w * r[D * D + D];
#pragma unroll
    for (int i = 0; i < D; ++i) u = fma(r[D * D + i], lam[i], u);
    lam[0] -= u;
    double nl[D];
#pragma unroll
    for (int q = 0; q < D; ++q) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < D; ++i) acc = fma(r[i * D + q], lam[i], acc);
      nl[q] = acc;
    }
#pragma unroll
    for (int i = 0; i < D; ++i) lam[i] = nl[i];
    X[k] = u;
  }
#pragma unroll
  for (int i = 0; i < D; ++i) bend[j * kSStride + i] = lam[i];
}

// Wide form for the prediction's many columns: a 256-column workgroup per chunk stages the
// chunk's gains records and fix-up rows in LDS once (read back as broadcasts; from memory they
// were scalar loads waited on step by step), and with `wmask` writes u only at the rows the
// caller reads (test points: wmask[k] >= 1e10, gpar_scaled_inference.jl:100-107).  A wave whose
// 64 columns are all past ncols leaves after the staging (the prediction's ncols = Mp + 1 left a
// third of the workgroups carrying one column through the whole chunk).  X goes through a buffer
// descriptor over the chunk's rows: each thread keeps kAdjPF rows in flight ahead of the
// recursion, and the store of u at a train row gets an out-of-range offset and is dropped by the
// hardware.  With plain loads / a predicated store the branches made the compiler wait for every
// load at every step (vmcnt(0)): one row in flight per thread, 77 % of wave time waiting.
constexpr int kAdjPF = 8;

template <int D, int CW>
__global__ __launch_bounds__(CW) void adjoint_local_wide(double* __restrict__ X, int64_t ldx,
                                                         int64_t ncols, const double* __restrict__ rec,
                                                         const double* __restrict__ g,
                                                         const double* __restrict__ cin, int64_t mc,
                                                         int64_t n, int L, double* __restrict__ bend,
                                                         const double* __restrict__ wmask) {
  constexpr int RS = Rec<D>::size;
  constexpr int RU = D * D + D + 1;   // record entries used
  // a step's record entries, then its fix-up row, in a 16-double row: lane i of every 16-lane DPP
  // row reads element i (one ds_read_b64, 2 LDS cycles) and the FMAs take the element they need by
  // row_newbcast (fmac_row).  The broadcast ds_read_b128 form cost 32 LDS cycles per wave-step
  // against ≈ 70 DP cycles, with 9 waves of a workgroup on one CU's LDS (r04ai: 63 % of the LDS
  // array's cycles with ds_read2_b64; r05q: the DPP row).
  constexpr int RP = 16;
  static_assert(RU + D <= RP, "step row");
  __shared__ __attribute__((aligned(16))) double lrec[256 * RP];
  __shared__ unsigned char lw[256];
  const int64_t j = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t c = (int64_t)blockIdx.y * CW + tid;
  const bool act = c < ncols;
  const int64_t cc = act ? c : 0;
  const int64_t k0 = j * L;
  const int64_t k1 = (k0 + L < n) ? k0 + L : n;
  const int nk = (int)(k1 - k0);
  for (int e = tid; e < nk * RU; e += CW) lrec[(e / RU) * RP + e % RU] = rec[(k0 + e / RU) * RS + e % RU];
  for (int e = tid; e < nk * D; e += CW) lrec[(e / D) * RP + RU + e % D] = g[(k0 + e / D) * kGStride + e % D];
  if (tid < nk) lw[tid] = wmask ? (wmask[k0 + tid] >= 1e10) : 1;
  __syncthreads();
  if ((int64_t)blockIdx.y * CW + (tid & ~63) >= ncols) return;   // the whole wave is idle
  double cf[D];
#pragma unroll
  for (int i = 0; i < D; ++i) cf[i] = cin[(j * mc + cc) * kSStride + i];
  double lam[D];
#pragma unroll
  for (int i = 0; i < D; ++i) lam[i] = 0.0;
  // the chunk's rows of X: [k0, k1) x ldx doubles (< 4 GiB for any L x ldx the library uses)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      X + k0 * ldx, (short)0, __builtin_amdgcn_readfirstlane((int)((int64_t)nk * ldx * 8)),
      0x00020000);
  const uint32_t col = (uint32_t)cc * 8u, rowb = (uint32_t)ldx * 8u;
  auto ld = [&](int s) {   // X[k0 + s][cc], s clamped to row 0 (a spare reload at the end)
    const uint32_t off = (uint32_t)(s > 0 ? s : 0) * rowb + col;
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, off, 0, 0));
  };
  const int rl = tid & 15;
  auto stepfn = [&](int s, double w) {
    const double row = lrec[s * RP + rl];
    static_for<D>([&](auto ic) {   // w += g_k . c_j
      constexpr int i = decltype(ic)::value;
      w = fmac_row<RU + i>(w, row, cf[i]);
    });
    double u = w * bcast_row<D * D + D>(row);
    static_for<D>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      u = fmac_row<D * D + i>(u, row, lam[i]);
    });
    lam[0] -= u;
    double nl[D];
    static_for<D>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      double acc = 0.0;
      static_for<D>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        acc = fmac_row<i * D + q>(acc, row, lam[i]);
      });
      nl[q] = acc;
    });
#pragma unroll
    for (int i = 0; i < D; ++i) lam[i] = nl[i];
    // u only where the caller reads it; elsewhere an out-of-range offset (dropped)
    const uint32_t off = (act && lw[s]) ? (uint32_t)s * rowb + col : ~0u;
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, u), xr, off, 0, 0);
  };
  // a short last chunk's top nk % kAdjPF rows one by one, then whole groups with the ring
  const int rem = nk % kAdjPF;
  for (int s = nk - 1; s >= nk - rem; --s) stepfn(s, ld(s));
  const int top0 = nk - rem - 1;
  double xb[kAdjPF];   // xb[p]: row top - p of the current group
#pragma unroll
  for (int p = 0; p < kAdjPF; ++p) xb[p] = ld(top0 - p);
  for (int top = top0; top >= 0; top -= kAdjPF) {
#pragma unroll
    for (int p = 0; p < kAdjPF; ++p) {
      const int s = top - p;
      const double w = xb[p];
      xb[p] = ld(s - kAdjPF);
      stepfn(s, w);
    }
  }
  if (act) {
#pragma unroll
    for (int i = 0; i < D; ++i) bend[(j * mc + c) * kSStride + i] = lam[i];
  }
}

// ---------------------------------------------------------------------------- smoothed mean of f
// f_k = y_k - R_k (Sigma^{-1} y)_k   (S y = y - R Sigma^{-1} y), with
// (Sigma^{-1} y)_k = u_loc_k + h_k . chat_{chunk(k)};  u_loc: adjoint output (contiguous per chain).
template <int D>
__global__ __launch_bounds__(256) void smooth_mean(const double* __restrict__ u,
                                                   const double* __restrict__ h,
                                                   const double* __restrict__ chat, int64_t sstride,
                                                   const double* __restrict__ y, int64_t ldy,
                                                   const double* __restrict__ noise,
                                                   const ChainParams* __restrict__ cps, int64_t n,
                                                   int L, double* __restrict__ mean, int64_t ldm) {
  const int64_t k = blockIdx.x * (int64_t)256 + threadIdx.x;
  const int b = blockIdx.y;
  if (k >= n) return;
  const int64_t j = k >> __builtin_ctz(L);  // L is a power of two (kChunk)
  const double* hk = h + ((int64_t)b * n + k) * kGStride;
  const double* ch = chat + (int64_t)b * sstride + j * kSStride;
  double uu = u[(int64_t)b * n + k];
#pragma unroll
  for (int i = 0; i < D; ++i) uu = fma(hk[i], ch[i], uu);
  const double R = step_noise(noise, k, cps[b]);
  mean[(int64_t)b * ldm + k] = y[(int64_t)b * ldy + k] - R * uu;
}

// ---------------------------------------------------------------------------- smoothed covariance
// RTS: P^s_k = G_k P^s_{k+1} G_k^T + C_k,  G_k = P_k A_{k+1}^T (P^-_{k+1})^{-1},
// C_k = P_k - G_k P^-_{k+1} G_k^T  (G_{N-1} = 0, C_{N-1} = P_{N-1}).  Chunked: local from 0 at
// each chunk end, P^s_k = local + Gamma_k Phat_j Gamma_k^T with Gamma_k = G_k ... G_{k1-1};
// the per-chunk aggregate (local P^s at the chunk start, Gamma_{k0}) feeds a backward carry.
// Only var_k = P^s_k[0,0] (the latent f, H = e1) is emitted.
template <int D>
__global__ __launch_bounds__(256) void cov_local(const double* __restrict__ t,
                                                 const double* __restrict__ rec,
                                                 const double* __restrict__ pf,
                                                 const ChainParams* __restrict__ cps, int64_t n,
                                                 int L, int64_t nch, double* __restrict__ vloc,
                                                 double* __restrict__ gam,
                                                 double* __restrict__ agg) {
  constexpr int RS = Rec<D>::size;
  const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (j >= nch) return;
  const ChainParams cp = cps[b];
  const double* rp = rec + (int64_t)b * n * RS;
  const double* pp = pf + (int64_t)b * n * D * D;
  const int64_t k0 = j * L;
  const int64_t k1 = (k0 + L < n) ? k0 + L : n;
  double Ps[D][D], Gm[D][D];
  mat_zero(Ps);
  mat_eye(Gm);
  for (int64_t k = k1 - 1; k >= k0; --k) {
    double P[D][D];
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) P[i][q] = pp[k * D * D + i * D + q];
    double G[D][D], C[D][D];
    if (k == n - 1) {
      mat_zero(G);
      mat_copy(P, C);
    } else {
      double A1[D][D], Q1[D][D], X[D][D], Pm[D][D], Pmi[D][D];
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int q = 0; q < D; ++q) A1[i][q] = rp[(k + 1) * RS + i * D + q];
      // Q_{k+1} = s Pinf - A Pinf A^T (same construction as step_model)
      double Pinf[D][D];
      sde_pinf<D>(cp.s, Pinf);
      mat_mul(A1, Pinf, X);
      mat_mul_bt(X, A1, Q1);
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int q = 0; q < D; ++q) Q1[i][q] = Pinf[i][q] - Q1[i][q];
      mat_mul(A1, P, X);
      mat_mul_bt(X, A1, Pm);
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int q = 0; q < D; ++q) Pm[i][q] += Q1[i][q];
      mat_inv(Pm, Pmi);
      mat_mul_bt(P, A1, X);        // P A^T
      mat_mul(X, Pmi, G);          // G = P A^T Pm^{-1}
      double GP[D][D], GPG[D][D];
      mat_mul(G, Pm, GP);
      mat_mul_bt(GP, G, GPG);
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int q = 0; q < D; ++q) C[i][q] = P[i][q] - GPG[i][q];
    }
    double T[D][D], U[D][D];
    mat_mul(G, Ps, T);
    mat_mul_bt(T, G, U);
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) Ps[i][q] = U[i][q] + C[i][q];
    mat_mul(G, Gm, T);
    mat_copy(T, Gm);
    vloc[(int64_t)b * n + k] = Ps[0][0];
#pragma unroll
    for (int q = 0; q < D; ++q) gam[((int64_t)b * n + k) * kGStride + q] = Gm[0][q];
  }
  double* ag = agg + ((int64_t)b * nch + j) * (2 * D * D);
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) {
      ag[i * D + q] = Ps[i][q];
      ag[D * D + i * D + q] = Gm[i][q];
    }
}

// The temporal chains' backward smoothing pass in one kernel, one lane per (chunk, chain): per
// step the three chunk-local backward recursions that gains_adjoint (h_k), adjoint_local_col
// (u_k, the chunk's adjoint end state) and cov_local (the local smoothed variance and Gamma row)
// ran as three launches, each re-reading the step's gains record (r06: 1.12 + 1.03 + 1.74 ms at
// the ssm config's 16 chains x 2e6 steps, latency-bound at two waves per SIMD).  The same
// arithmetic in the same order per recursion, so the results are bit-identical to the three
// kernels; interleaved, the three independent dependency chains hide each other's latency and the
// record, fix-up row and filtered covariance are read once.
template <int D>
__global__ __launch_bounds__(256) void smooth_back(const double* __restrict__ rec,
                                                   const double* __restrict__ g,
                                                   const double* __restrict__ pf,
                                                   const ChainParams* __restrict__ cps,
                                                   const double* __restrict__ cin,
                                                   double* __restrict__ X, double* __restrict__ h,
                                                   double* __restrict__ vloc,
                                                   double* __restrict__ gam,
                                                   double* __restrict__ agg,
                                                   double* __restrict__ bend, int64_t n, int L,
                                                   int64_t nch, int64_t xstride, int64_t sstride) {
  constexpr int RS = Rec<D>::size;
  const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (j >= nch) return;
  const ChainParams cp = cps[b];
  rec += (int64_t)b * n * RS;
  g += (int64_t)b * n * kGStride;
  pf += (int64_t)b * n * D * D;
  X += (int64_t)b * xstride;
  h += (int64_t)b * n * kGStride;
  vloc += (int64_t)b * n;
  gam += (int64_t)b * n * kGStride;
  cin += (int64_t)b * sstride;
  bend += (int64_t)b * sstride;
  const int64_t k0 = j * L;
  const int64_t k1 = (k0 + L < n) ? k0 + L : n;
  double cf[D], lam[D], Ga[D][D], Ps[D][D], Gm[D][D], A1[D][D], Pinf[D][D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    cf[i] = cin[j * kSStride + i];
    lam[i] = 0.0;
  }
  mat_eye(Ga);
  mat_zero(Ps);
  mat_eye(Gm);
  sde_pinf<D>(cp.s, Pinf);
  if (k1 < n) {   // A_{k1}: the transition into the next chunk's first step
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) A1[i][q] = rec[k1 * RS + i * D + q];
  } else {
    mat_zero(A1);
  }
  // a step's inputs (its record, fix-up row, adjoint input and filtered covariance), fetched one
  // step ahead into the other of two static register sets while the current step computes (in
  // step order each step waited out its loads, at about two waves per SIMD)
  struct In {
    double A[D][D], K[D], rs, gk[D], x, P[D][D];
  };
  auto fetch = [&](In& in, int64_t k) __attribute__((always_inline)) {
    const double* r = rec + k * RS;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      in.K[i] = r[D * D + i];
#pragma unroll
      for (int q = 0; q < D; ++q) in.A[i][q] = r[i * D + q];
    }
    in.rs = r[D * D + D];
#pragma unroll
    for (int i = 0; i < D; ++i) in.gk[i] = g[k * kGStride + i];
    in.x = X[k];
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) in.P[i][q] = pf[k * D * D + i * D + q];
  };
  auto step = [&](const In& in, int64_t k) __attribute__((always_inline)) {
    const double(&A)[D][D] = in.A;
    const double(&K)[D] = in.K;
    const double rs = in.rs;
    // ---- gains_adjoint: h_k = Gamma^T K, Gamma <- Abar^T Gamma
#pragma unroll
    for (int q = 0; q < D; ++q) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < D; ++i) acc = fma(Ga[i][q], K[i], acc);
      h[k * kGStride + q] = acc;
    }
    {
      double Ab[D][D], T[D][D];
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int q = 0; q < D; ++q) Ab[i][q] = A[i][q] - K[i] * A[0][q];
      mat_mul_at(Ab, Ga, T);
      mat_copy(T, Ga);
    }
    // ---- adjoint_local_col: u_k and lambda
    {
      double w = in.x;
#pragma unroll
      for (int i = 0; i < D; ++i) w = fma(in.gk[i], cf[i], w);
      double u = w * rs;
#pragma unroll
      for (int i = 0; i < D; ++i) u = fma(K[i], lam[i], u);
      lam[0] -= u;
      double nl[D];
#pragma unroll
      for (int q = 0; q < D; ++q) {
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < D; ++i) acc = fma(A[i][q], lam[i], acc);
        nl[q] = acc;
      }
#pragma unroll
      for (int i = 0; i < D; ++i) lam[i] = nl[i];
      X[k] = u;
    }
    // ---- cov_local: the local smoothed covariance and Gamma's first row
    {
      const double(&P)[D][D] = in.P;
      double G[D][D], C[D][D];
      if (k == n - 1) {
        mat_zero(G);
        mat_copy(P, C);
      } else {
        double Q1[D][D], T[D][D], Pm[D][D], Pmi[D][D];
        mat_mul(A1, Pinf, T);
        mat_mul_bt(T, A1, Q1);
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) Q1[i][q] = Pinf[i][q] - Q1[i][q];
        mat_mul(A1, P, T);
        mat_mul_bt(T, A1, Pm);
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) Pm[i][q] += Q1[i][q];
        mat_inv(Pm, Pmi);
        mat_mul_bt(P, A1, T);
        mat_mul(T, Pmi, G);
        double GP[D][D], GPG[D][D];
        mat_mul(G, Pm, GP);
        mat_mul_bt(GP, G, GPG);
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) C[i][q] = P[i][q] - GPG[i][q];
      }
      double T[D][D], U[D][D];
      mat_mul(G, Ps, T);
      mat_mul_bt(T, G, U);
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int q = 0; q < D; ++q) Ps[i][q] = U[i][q] + C[i][q];
      mat_mul(G, Gm, T);
      mat_copy(T, Gm);
      vloc[k] = Ps[0][0];
#pragma unroll
      for (int q = 0; q < D; ++q) gam[k * kGStride + q] = Gm[0][q];
    }
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) A1[i][q] = A[i][q];
  };
  In b0, b1;
  if (k1 - 1 >= k0) fetch(b0, k1 - 1);
  for (int64_t k = k1 - 1; k >= k0; k -= 2) {
    if (k - 1 >= k0) fetch(b1, k - 1);
    step(b0, k);
    if (k - 1 < k0) break;
    if (k - 2 >= k0) fetch(b0, k - 2);
    step(b1, k - 1);
  }
#pragma unroll
  for (int i = 0; i < D; ++i) bend[j * kSStride + i] = lam[i];
  double* ag = agg + ((int64_t)b * nch + j) * (2 * D * D);
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) {
      ag[i * D + q] = Ps[i][q];
      ag[D * D + i * D + q] = Gm[i][q];
    }
}

// Backward carry over chunks: Phat_{J-1} = 0, Phat_{j-1} = f_j(Phat_j) = S_j + Gamma_j Phat_j
// Gamma_j^T with S_j = the chunk's local smoothed covariance at its start and Gamma_j its
// transfer (agg).  The maps compose, (S_a, Gamma_a) o (S_b, Gamma_b) = (S_a + Gamma_a S_b
// Gamma_a^T, Gamma_a Gamma_b), so the carry is a two-level scan like the means' (carry_group_*):
//   a) cov_group_local, per (group of GS chunks, chain): the group's composite map   -> gagg
//   b) cov_group_scan, per chain: the groups right to left from Phat = 0              -> gin
//   c) cov_group_apply, per (group, chain): Phat at each of the group's chunks        -> phat
// (Round 5 ran the recursion serially, one thread per chain over all 7813 chunks of the ssm
// config's merged grid: 3.7 ms of 16 threads on a 256-CU chip.)  The last group reproduces the
// serial order; elsewhere the association differs (rounding only).
template <int D>
__device__ __forceinline__ void cov_map_apply(const double* __restrict__ ag, double (&Ph)[D][D]) {
  double Gm[D][D], T[D][D], U[D][D];
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) Gm[i][q] = ag[D * D + i * D + q];
  mat_mul(Gm, Ph, T);
  mat_mul_bt(T, Gm, U);
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) Ph[i][q] = ag[i * D + q] + U[i][q];
}

template <int D>
__global__ __launch_bounds__(256) void cov_group_local(const double* __restrict__ agg, int64_t nch,
                                                       int GS, int64_t ng, int nchains,
                                                       double* __restrict__ gagg) {
  const int64_t gi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (gi >= ng) return;
  const int64_t j0 = gi * GS, j1 = (j0 + GS < nch) ? j0 + GS : nch;
  double S[D][D], Gm[D][D];
  mat_zero(S);
  mat_eye(Gm);
  for (int64_t j = j1 - 1; j >= j0; --j) {   // F <- f_j o F
    const double* ag = agg + ((int64_t)b * nch + j) * (2 * D * D);
    double Gj[D][D], T[D][D], U[D][D];
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) Gj[i][q] = ag[D * D + i * D + q];
    mat_mul(Gj, S, T);
    mat_mul_bt(T, Gj, U);
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) S[i][q] = ag[i * D + q] + U[i][q];
    mat_mul(Gj, Gm, T);
    mat_copy(T, Gm);
  }
  double* o = gagg + ((int64_t)b * ng + gi) * (2 * D * D);
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) {
      o[i * D + q] = S[i][q];
      o[D * D + i * D + q] = Gm[i][q];
    }
}

template <int D>
__global__ __launch_bounds__(64) void cov_group_scan(const double* __restrict__ gagg, int64_t ng,
                                                     int nchains, double* __restrict__ gin) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nchains) return;
  double Ph[D][D];
  mat_zero(Ph);
  for (int64_t g = ng - 1; g >= 0; --g) {
    double* o = gin + ((int64_t)b * ng + g) * (D * D);
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) o[i * D + q] = Ph[i][q];
    cov_map_apply<D>(gagg + ((int64_t)b * ng + g) * (2 * D * D), Ph);
  }
}

template <int D>
__global__ __launch_bounds__(256) void cov_group_apply(const double* __restrict__ agg,
                                                       const double* __restrict__ gin, int64_t nch,
                                                       int GS, int64_t ng, int nchains,
                                                       double* __restrict__ phat) {
  const int64_t gi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (gi >= ng) return;
  const int64_t j0 = gi * GS, j1 = (j0 + GS < nch) ? j0 + GS : nch;
  double Ph[D][D];
  const double* gp = gin + ((int64_t)b * ng + gi) * (D * D);
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) Ph[i][q] = gp[i * D + q];
  for (int64_t j = j1 - 1; j >= j0; --j) {
    double* o = phat + ((int64_t)b * nch + j) * (D * D);
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) o[i * D + q] = Ph[i][q];
    cov_map_apply<D>(agg + ((int64_t)b * nch + j) * (2 * D * D), Ph);
  }
}

template <int D>
__global__ __launch_bounds__(256) void cov_out(const double* __restrict__ vloc,
                                               const double* __restrict__ gam,
                                               const double* __restrict__ phat, int64_t n, int L,
                                               int64_t nch, double* __restrict__ var, int64_t ldv) {
  const int64_t k = blockIdx.x * (int64_t)256 + threadIdx.x;
  const int b = blockIdx.y;
  if (k >= n) return;
  const int64_t j = k >> __builtin_ctz(L);  // L is a power of two (kChunk)
  const double* gk = gam + ((int64_t)b * n + k) * kGStride;
  const double* P = phat + ((int64_t)b * nch + j) * (D * D);
  double v = vloc[(int64_t)b * n + k];
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) v = fma(gk[i] * P[i * D + q], gk[q], v);
  var[(int64_t)b * ldv + k] = v;
}

// ---------------------------------------------------------------------------- fix-up of a vector
// alpha[k] += g_k . cin[chunk(k)][col]; per-block partial sums of alpha^2 into part[b][blk].
// One 256-thread block per chunk (L == 256).  With `hsum` (single chain, the DTC objective) the
// block also prepares the Gram's chunk correction (k_gram.hip):
//   W_j = sum_k g_k g_k^T,  q_j = sum_k g_k alpha_k  (alpha fixed)       -> qout[j * 4 + i]
//   E_j[c] = H_j[c] + W_j C_j[c] / 2   for the ncols beta columns, in place of H_j (hsum).
template <int D>
__global__ __launch_bounds__(256) void vec_fix(double* __restrict__ alpha, int64_t lda,
                                               const double* __restrict__ g, int64_t gstride,
                                               const double* __restrict__ cin, int64_t sstride,
                                               int64_t mc, int64_t col, int64_t n, int L,
                                               double* __restrict__ part, double* __restrict__ hsum,
                                               int64_t ncols, double* __restrict__ qout) {
  constexpr int NW = D * (D + 1) / 2;   // packed upper triangle of W
  constexpr int NV = 1 + NW + D;        // alpha^2 | W | q
  __shared__ double red[4][NV];
  __shared__ double wq[NW + D];
  const int b = blockIdx.y;
  const int64_t j = blockIdx.x;
  const int64_t k = j * L + threadIdx.x;
  double vals[NV];
#pragma unroll
  for (int e = 0; e < NV; ++e) vals[e] = 0.0;
  if (k < n) {
    const double* gp = g + (int64_t)b * gstride + k * kGStride;
    const double* cp = cin + (int64_t)b * sstride + (j * mc + col) * kSStride;
    double a = alpha[(int64_t)b * lda + k];
    double gk[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      gk[i] = gp[i];
      a = fma(gk[i], cp[i], a);
    }
    alpha[(int64_t)b * lda + k] = a;
    vals[0] = a * a;
    int e = 1;
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = i; q < D; ++q) vals[e++] = gk[i] * gk[q];
#pragma unroll
    for (int i = 0; i < D; ++i) vals[1 + NW + i] = gk[i] * a;
  }
  const int nv = hsum ? NV : 1;
  for (int e = 0; e < nv; ++e) {
    const double v = wave_sum(vals[e]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][e] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    part[(int64_t)b * gridDim.x + blockIdx.x] = ((red[0][0] + red[1][0]) + red[2][0]) + red[3][0];
  if (!hsum) return;
  if (threadIdx.x < NW + D) {
    const int e = 1 + threadIdx.x;
    wq[threadIdx.x] = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
  }
  __syncthreads();
  if (threadIdx.x < 4) qout[j * 4 + threadIdx.x] = threadIdx.x < D ? wq[NW + threadIdx.x] : 0.0;
  double W[D][D];
  {
    int e = 0;
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = i; q < D; ++q) {
        W[i][q] = wq[e];
        W[q][i] = wq[e];
        ++e;
      }
  }
  for (int64_t c = threadIdx.x; c < ncols; c += 256) {
    const double* cp = cin + (j * mc + c) * kSStride;
    double* hp = hsum + (j * mc + c) * kSStride;
    double cv[D], ev[D];
#pragma unroll
    for (int i = 0; i < D; ++i) cv[i] = cp[i];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < D; ++q) acc = fma(W[i][q], cv[q], acc);
      ev[i] = fma(0.5, acc, hp[i]);
    }
#pragma unroll
    for (int i = 0; i < kSStride; ++i) hp[i] = i < D ? ev[i] : 0.0;
  }
}

// ---------------------------------------------------------------------------- chain log-likelihood
// lml[b] = -0.5 (n log 2pi + sum logS + sum alpha^2), partials summed in a fixed order.
__global__ void chain_lml(const double* __restrict__ logs, int64_t nch,
                          const double* __restrict__ a2part, int64_t npart, int64_t n,
                          double* __restrict__ lml) {
  const int b = blockIdx.x;
  __shared__ double red[2][256];
  double s1 = 0.0, s2 = 0.0;
  for (int64_t j = threadIdx.x; j < nch; j += 256) s1 += logs[(int64_t)b * nch + j];
  for (int64_t j = threadIdx.x; j < npart; j += 256) s2 += a2part[(int64_t)b * npart + j];
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      red[0][threadIdx.x] += red[0][threadIdx.x + off];
      red[1][threadIdx.x] += red[1][threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) lml[b] = -0.5 * ((double)n * kLog2Pi + red[0][0] + red[1][0]);
}

// The chains fit on the device (nm_dev.hpp): chain b's machine takes -v, and its next point's
// parameters go where the next round's gains read them.  Called by the whole workgroup; the
// record is staged in LDS (one coalesced copy each way) so the machine's dependent accesses are
// LDS reads, not HBM round trips.
__device__ void nm_chain_step(NmDev<3>* __restrict__ nm, ChainParams* __restrict__ cps,
                              int* __restrict__ active, int b, double v) {
  constexpr int kW = (int)(sizeof(NmDev<3>) / sizeof(int));
  static_assert(sizeof(NmDev<3>) % sizeof(int) == 0, "NmDev<3> in whole words");
  __shared__ NmDev<3> ls;
  int* lw = reinterpret_cast<int*>(&ls);
  const int* gw = reinterpret_cast<const int*>(nm + b);
  for (int w = threadIdx.x; w < kW; w += blockDim.x) lw[w] = gw[w];
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    if (ls.st != NmDev<3>::Done) {
      double f = -v;
      if (!isfinite(f)) f = INFINITY;
      nm_tell(ls, f);
      if (ls.st != NmDev<3>::Done) {
        // unpack() (host.hpp: exp(p) + 1e-3) and chains_logpdf's parameters
        const double l = exp(ls.pending[0]) + 1e-3, pv = exp(ls.pending[1]) + 1e-3,
                     ns = exp(ls.pending[2]) + 1e-3;
        cps[b] = ChainParams{1.0 / l, l, pv * pv, ns * ns};
        run = 1;
      }
    }
    active[b] = run;
  }
  __syncthreads();
  int* ow = reinterpret_cast<int*>(nm + b);
  for (int w = threadIdx.x; w < kW; w += blockDim.x) ow[w] = lw[w];
}

// A chain's logpdf from the phase-3 moments (MOM) in one workgroup per chain, its chunk carry
// included: lml = -0.5 (n log 2pi + sum_j [logS_j + s0_j + 2 c_j . s1_j + c_j^T s2_j c_j]), c_j
// the state entering chunk j (c_0 = 0, c_{j+1} = Phi_j c_j + send_j).  Thread t owns a run of
// consecutive chunks: it composes its run's affine map, a workgroup scan of the 256 maps gives
// each run's incoming state, and the run is walked once more for the chunk terms, its loads
// issued KB chunks at a time.  (r06: the three-launch group carry and a separate reduction took
// 40 us per round at 3907 chunks, this 35 us; staging segments of 1024 chunks through LDS with
// coalesced loads measured 63 us -- four segments' scans and barriers.)  nm (optional): the
// device Nelder-Mead step after the value (nm_chain_step).
template <int D>
__global__ __launch_bounds__(256) void chain_carry_lml(
    const double* __restrict__ phi, int64_t phistride, const double* __restrict__ send,
    int64_t sstride, const double* __restrict__ logs, const double* __restrict__ mom, int64_t nch,
    int64_t n, double* __restrict__ lml, NmDev<3>* __restrict__ nm, ChainParams* __restrict__ cps,
    int* __restrict__ active) {
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const double* ph = phi + (int64_t)b * phistride;
  const double* sp = send + (int64_t)b * sstride;
  const int64_t run = run_len(nch);
  const int64_t j0 = (int64_t)t * run < nch ? (int64_t)t * run : nch;
  const int64_t j1 = j0 + run < nch ? j0 + run : nch;
  // chunk j = j0 + u of this thread's run sits at slot u 256 + t (mom_slot)
  auto slot = [&](int64_t j) __attribute__((always_inline)) { return (j - j0) * 256 + t; };
  const double* lgb = logs + (int64_t)b * 256 * run;
  const double* mob = mom + (int64_t)b * 256 * run * kMomStride;
  constexpr int KB = D == 3 ? 4 : 8;
  // the run's map x -> A x + c
  double A[D][D], c[D];
  mat_eye(A);
#pragma unroll
  for (int i = 0; i < D; ++i) c[i] = 0.0;
  for (int64_t jb = j0; jb < j1; jb += KB) {
    double Fb[KB][D * D], Sb[KB][D];
#pragma unroll
    for (int u = 0; u < KB; ++u)
      if (jb + u < j1) {
#pragma unroll
        for (int e = 0; e < D * D; ++e) Fb[u][e] = ph[slot(jb + u) * D * D + e];
#pragma unroll
        for (int i = 0; i < D; ++i) Sb[u][i] = sp[slot(jb + u) * kSStride + i];
      }
#pragma unroll
    for (int u = 0; u < KB; ++u)
      if (jb + u < j1) {
        double F[D][D], X[D][D], y[D];
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
          for (int q = 0; q < D; ++q) F[i][q] = Fb[u][i * D + q];
        mat_mul(F, A, X);
        mat_copy(X, A);
#pragma unroll
        for (int i = 0; i < D; ++i) {
          double acc = Sb[u][i];
#pragma unroll
          for (int q = 0; q < D; ++q) acc = fma(F[i][q], c[q], acc);
          y[i] = acc;
        }
#pragma unroll
        for (int i = 0; i < D; ++i) c[i] = y[i];
      }
  }
  // inclusive scan of the runs' maps (Hillis-Steele, composition: later after earlier)
  constexpr int E = D * D + D;
  __shared__ double sm[2][256 * E];
  int cur = 0;
#pragma unroll
  for (int i = 0; i < D; ++i) {
#pragma unroll
    for (int q = 0; q < D; ++q) sm[0][t * E + i * D + q] = A[i][q];
    sm[0][t * E + D * D + i] = c[i];
  }
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const double* src = sm[cur];
    double* dst = sm[cur ^ 1];
    if (t >= off) {
      // (A_t, c_t) o (A_{t-off}, c_{t-off}) = (A_t A_{t-off}, A_t c_{t-off} + c_t)
      const double* e = src + (t - off) * E;
      const double* f = src + t * E;
#pragma unroll
      for (int i = 0; i < D; ++i) {
#pragma unroll
        for (int q = 0; q < D; ++q) {
          double acc = 0.0;
#pragma unroll
          for (int k = 0; k < D; ++k) acc = fma(f[i * D + k], e[k * D + q], acc);
          dst[t * E + i * D + q] = acc;
        }
        double acc = f[D * D + i];
#pragma unroll
        for (int k = 0; k < D; ++k) acc = fma(f[i * D + k], e[D * D + k], acc);
        dst[t * E + D * D + i] = acc;
      }
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) dst[t * E + e] = src[t * E + e];
    }
    __syncthreads();
    cur ^= 1;
  }
  // the run's incoming state: the inclusive prefix of the runs before it, applied to 0
  double x[D];
#pragma unroll
  for (int i = 0; i < D; ++i) x[i] = t > 0 ? sm[cur][(t - 1) * E + D * D + i] : 0.0;
  double s = 0.0;
  constexpr int NM = 1 + D + D * (D + 1) / 2;   // moments used per chunk
  for (int64_t jb = j0; jb < j1; jb += KB) {
    double Fb[KB][D * D], Sb[KB][D], Mb[KB][NM], Lb[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u)
      if (jb + u < j1) {
        const int64_t so = slot(jb + u);
#pragma unroll
        for (int e = 0; e < D * D; ++e) Fb[u][e] = ph[so * D * D + e];
#pragma unroll
        for (int i = 0; i < D; ++i) Sb[u][i] = sp[so * kSStride + i];
        const double* m = mob + so * kMomStride;
#pragma unroll
        for (int e = 0; e < NM; ++e) Mb[u][e] = m[e];
        Lb[u] = lgb[so];
      }
#pragma unroll
    for (int u = 0; u < KB; ++u)
      if (jb + u < j1) {
        const double* m = Mb[u];
        double v = Lb[u] + m[0];
        int e = 1 + D;
#pragma unroll
        for (int i = 0; i < D; ++i) {
          v = fma(2.0 * x[i], m[1 + i], v);
#pragma unroll
          for (int q = i; q < D; ++q) {
            v = fma((q == i ? 1.0 : 2.0) * x[i] * x[q], m[e], v);
            ++e;
          }
        }
        s += v;
        carry_step<D, false>(Fb[u], 0, Sb[u], x);
      }
  }
  __syncthreads();   // sm is reused for the reduction
  double* red = sm[0];
  red[t] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) red[t] += red[t + off];
    __syncthreads();
  }
  const double v = -0.5 * ((double)n * kLog2Pi + red[0]);
  if (t == 0) lml[b] = v;
  if (nm) nm_chain_step(nm, cps, active, b, v);
}

}  // namespace gpar

// ============================================================================ launch wrappers
#include "launch.hpp"
static_assert(gpar::kMomStride == gpar::kGainsMomStride, "moment stride");

namespace gpar {

// phase-3 launches by path since the library was loaded (gpar_debug_counter "gains_fast" /
// "gains_general"): lets a test assert which kernel a case actually ran
std::atomic<int64_t> g_gains_fast_launches{0}, g_gains_general_launches{0};

#define GPAR_DISPATCH_D(D, ...)                                   \
  switch (D) {                                                    \
    case 1: { constexpr int DD = 1; __VA_ARGS__; } break;         \
    case 2: { constexpr int DD = 2; __VA_ARGS__; } break;         \
    default: { constexpr int DD = 3; __VA_ARGS__; } break;        \
  }

// every combination of the optional inputs / outputs is its own instantiation of gains_phase3
// (no dead registers or branches for the ones a caller does not pass)
template <int D, bool C, bool Y, bool NZ, bool PFX, bool MOM>
static void launch_phase3_blocks(dim3 grid, hipStream_t st, const double* t, int64_t n, int L,
                                 int64_t nch, const ChainParams* cps, const double* noise,
                                 const double* pstart, double* rec, double* g, double* phi,
                                 double* logs, double* pf, const double* const* ys,
                                 double* alpha_loc, double* asend, double* mom, bool fast_ok) {
  // the whole blocks (every chunk L steps, no lane masked) by the fast path when its counted
  // waits fit the vmcnt field, then each chain's last (masked) block
  const dim3 gfull(grid.x - 1, grid.y), glast(1, grid.y);
  const int64_t last = grid.x - 1;
  constexpr int NA = 1 + (Y ? 1 : 0) + (NZ ? 1 : 0);
  if constexpr (g3_stores_per_block<D, C, PFX, MOM, true>(Y) + 2 * NA <= 63) {
    if (L == kG3L && fast_ok) {
      gains_phase3_fast<D, C, Y, NZ, PFX, MOM><<<grid, 256, 0, st>>>(
          t, n, nch, cps, noise, pstart, rec, g, phi, logs, pf, ys, alpha_loc, asend, mom);
      g_gains_fast_launches.fetch_add(1, std::memory_order_relaxed);
      return;
    }
  }
  if (gfull.x)
    gains_phase3<D, C, Y, NZ, PFX, false, MOM><<<gfull, 256, 0, st>>>(0, t, n, L, nch, cps, noise,
                                                                      pstart, rec, g, phi, logs, pf,
                                                                      ys, alpha_loc, asend, mom);
  gains_phase3<D, C, Y, NZ, PFX, true, MOM><<<glast, 256, 0, st>>>(last, t, n, L, nch, cps, noise,
                                                                   pstart, rec, g, phi, logs, pf, ys,
                                                                   alpha_loc, asend, mom);
  g_gains_general_launches.fetch_add(1, std::memory_order_relaxed);
}

template <int D, bool C, bool Y, bool NZ>
static void launch_phase3_pf(dim3 grid, hipStream_t st, const double* t, int64_t n, int L,
                             int64_t nch, const ChainParams* cps, const double* noise,
                             const double* pstart, double* rec, double* g, double* phi,
                             double* logs, double* pf, const double* const* ys,
                             double* alpha_loc, double* asend, bool fast_ok) {
  if (pf)
    launch_phase3_blocks<D, C, Y, NZ, true, false>(grid, st, t, n, L, nch, cps, noise, pstart, rec,
                                                   g, phi, logs, pf, ys, alpha_loc, asend, nullptr,
                                                   fast_ok);
  else
    launch_phase3_blocks<D, C, Y, NZ, false, false>(grid, st, t, n, L, nch, cps, noise, pstart, rec,
                                                    g, phi, logs, pf, ys, alpha_loc, asend, nullptr,
                                                    fast_ok);
}

template <int D>
static void launch_phase3(dim3 grid, hipStream_t st, const double* t, int64_t n, int L,
                          int64_t nch, const ChainParams* cps, const double* noise,
                          const double* pstart, double* rec, double* g, double* phi, double* logs,
                          double* pf, const double* const* ys, double* alpha_loc, double* asend,
                          bool compact, bool fast_ok, double* mom) {
  if (mom) {   // the chains' logpdf: the data filter's moments only (no noise vector, no pf)
    launch_phase3_blocks<D, false, true, false, false, true>(grid, st, t, n, L, nch, cps, nullptr,
                                                             pstart, nullptr, nullptr, phi, logs,
                                                             nullptr, ys, nullptr, asend, mom,
                                                             fast_ok);
    return;
  }
#define GPAR_P3(C, Y, NZ) \
  launch_phase3_pf<D, C, Y, NZ>(grid, st, t, n, L, nch, cps, noise, pstart, rec, g, phi, logs, pf, \
                                ys, alpha_loc, asend, fast_ok)
  const bool y = ys != nullptr, nz = noise != nullptr;
  if (compact) {
    if (y) { if (nz) GPAR_P3(true, true, true); else GPAR_P3(true, true, false); }
    else { if (nz) GPAR_P3(true, false, true); else GPAR_P3(true, false, false); }
  } else {
    if (y) { if (nz) GPAR_P3(false, true, true); else GPAR_P3(false, true, false); }
    else { if (nz) GPAR_P3(false, false, true); else GPAR_P3(false, false, false); }
  }
#undef GPAR_P3
}

void launch_gains(hipStream_t st, int sdim, const double* t, int64_t n, int L, int64_t nch,
                  int nchains, const ChainParamsHost* cps_dev, const double* noise,
                  double* agg, double* pstart, double* rec, double* g, double* phi,
                  double* logs, double* pf, const double* const* ys, double* alpha_loc,
                  double* asend, bool compact, bool ys_aligned16, double* moments) {
  const ChainParams* cps = reinterpret_cast<const ChainParams*>(cps_dev);
  dim3 grid((unsigned)((nch + 255) / 256), (unsigned)nchains);
  GPAR_DISPATCH_D(sdim, {
    // four lanes per chunk below ~four waves per SIMD of chunks (gains_phase1)
    if ((int64_t)nchains * nch < 4 * 1024 * 64) {
      dim3 g4((unsigned)((4 * nch + 255) / 256), (unsigned)nchains);
      gains_phase1<DD, 4><<<g4, 256, 0, st>>>(t, n, L, nch, cps, noise, agg);
    } else {
      gains_phase1<DD, 1><<<grid, 256, 0, st>>>(t, n, L, nch, cps, noise, agg);
    }
    gains_phase2<DD><<<nchains, 256, 0, st>>>(nch, agg, pstart);
    // the fast phase 3 stages its inputs by 16-byte LDS-DMA: every input array 16-byte aligned
    // (GPAR_GAINS_FAST=0: the general kernel everywhere, for the fast path's bit-identity test)
    const char* fe = std::getenv("GPAR_GAINS_FAST");
    const bool a16 = ((uintptr_t)t % 16 == 0) && ((uintptr_t)noise % 16 == 0) &&
                     (!ys || ys_aligned16) && !(fe && fe[0] == '0');
    launch_phase3<DD>(grid, st, t, n, L, nch, cps, noise, pstart, rec, g, phi, logs, pf, ys,
                      alpha_loc, asend, compact, a16, moments);
  });
}

template <int TK, int OK>
static void launch_whiten_kfu_k(hipStream_t st, int dp, dim3 grid, const double* rec,
                                const double* v, int64_t ldv, int d, const double* z,
                                int64_t ldz, int64_t m, int64_t mp, int64_t n, int L,
                                double inv_lo, double s_o, double* beta, int64_t ldb,
                                double* send, int64_t mc, const double* g, double* hsum) {
  switch (dp) {
    case 4: whiten_kfu<TK, OK, 4><<<grid, 256, 0, st>>>(rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case 8: whiten_kfu<TK, OK, 8><<<grid, 256, 0, st>>>(rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case 16: whiten_kfu<TK, OK, 16><<<grid, 256, 0, st>>>(rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case 32: whiten_kfu<TK, OK, 32><<<grid, 256, 0, st>>>(rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    default: whiten_kfu<TK, OK, 64><<<grid, 256, 0, st>>>(rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
  }
}

template <int TK>
static void launch_whiten_kfu_t(hipStream_t st, int ok, int dp, dim3 grid, const double* rec,
                                const double* v, int64_t ldv, int d, const double* z,
                                int64_t ldz, int64_t m, int64_t mp, int64_t n, int L,
                                double inv_lo, double s_o, double* beta, int64_t ldb,
                                double* send, int64_t mc, const double* g, double* hsum) {
  switch (ok) {
    case KM12: launch_whiten_kfu_k<TK, KM12>(st, dp, grid, rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case KM32: launch_whiten_kfu_k<TK, KM32>(st, dp, grid, rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case KM52: launch_whiten_kfu_k<TK, KM52>(st, dp, grid, rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    default: launch_whiten_kfu_k<TK, KEQ>(st, dp, grid, rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
  }
}

int dp_bucket(int d) {
  if (d <= 4) return 4;
  if (d <= 8) return 8;
  if (d <= 16) return 16;
  if (d <= 32) return 32;
  if (d <= 64) return 64;
  return -1;
}

template <int TK, int OK>
static void launch_whiten_mfma_k(hipStream_t st, int dp, dim3 grid, const double* rec,
                                 const double* v, int64_t ldv, int d, const double* z,
                                 int64_t ldz, const double* zc, int64_t m, int64_t mp, int64_t n,
                                 int L, double inv_lo, double s_o, double* beta, int64_t ldb,
                                 double* send, int64_t mc, const double* g, double* hsum) {
  switch (dp) {
    case 16: whiten_kfu_mfma<TK, OK, 16><<<grid, 256, 0, st>>>(rec, v, ldv, d, z, ldz, zc, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case 32: whiten_kfu_mfma<TK, OK, 32><<<grid, 256, 0, st>>>(rec, v, ldv, d, z, ldz, zc, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case 48: whiten_kfu_mfma<TK, OK, 48><<<grid, 256, 0, st>>>(rec, v, ldv, d, z, ldz, zc, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    default: whiten_kfu_mfma<TK, OK, 64><<<grid, 256, 0, st>>>(rec, v, ldv, d, z, ldz, zc, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
  }
}

template <int TK>
static void launch_whiten_mfma_t(hipStream_t st, int dp, dim3 grid, const double* rec,
                                 const double* v, int64_t ldv, int d, const double* z,
                                 int64_t ldz, const double* zc, int64_t m, int64_t mp, int64_t n,
                                 int L, int ok, double inv_lo, double s_o, double* beta,
                                 int64_t ldb, double* send, int64_t mc, const double* g,
                                 double* hsum) {
  switch (ok) {
    case KM32: launch_whiten_mfma_k<TK, KM32>(st, dp, grid, rec, v, ldv, d, z, ldz, zc, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case KEQ: launch_whiten_mfma_k<TK, KEQ>(st, dp, grid, rec, v, ldv, d, z, ldz, zc, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    default: launch_whiten_mfma_k<TK, KM52>(st, dp, grid, rec, v, ldv, d, z, ldz, zc, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
  }
}

int mfma_dp_bucket(int d) {
  if (d <= 16) return 16;
  if (d <= 32) return 32;
  if (d <= 48) return 48;
  if (d <= 64) return 64;
  return -1;
}

void launch_zcenter(hipStream_t st, const double* z, int64_t ldz, int d, int64_t m, int64_t mp,
                    double* zc) {
  zcenter_kernel<<<(unsigned)((mp + 255) / 256), 256, 0, st>>>(z, ldz, d, m, mfma_dp_bucket(d), zc);
}

void launch_whiten_kfu_mfma(hipStream_t st, int time_kind, int out_kind, const double* rec,
                            const double* v, int64_t ldv, int d, const double* z, int64_t ldz,
                            const double* zc, int64_t m, int64_t mp, int64_t n, int L, int64_t nch,
                            double inv_lo, double s_o, double* beta, int64_t ldb, double* send,
                            int64_t mc, const double* g, double* hsum) {
  const int dp = mfma_dp_bucket(d);
  dim3 grid((unsigned)nch, (unsigned)((mp + 255) / 256));
  switch (time_kind) {
    case KM12: launch_whiten_mfma_t<KM12>(st, dp, grid, rec, v, ldv, d, z, ldz, zc, m, mp, n, L, out_kind, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case KM32: launch_whiten_mfma_t<KM32>(st, dp, grid, rec, v, ldv, d, z, ldz, zc, m, mp, n, L, out_kind, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    default: launch_whiten_mfma_t<KM52>(st, dp, grid, rec, v, ldv, d, z, ldz, zc, m, mp, n, L, out_kind, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
  }
}

void launch_whiten_kfu(hipStream_t st, int time_kind, int out_kind, const double* rec,
                       const double* v, int64_t ldv, int d, const double* z, int64_t ldz,
                       int64_t m, int64_t mp, int64_t n, int L, int64_t nch, double inv_lo,
                       double s_o, double* beta, int64_t ldb, double* send, int64_t mc,
                       const double* g, double* hsum) {
  dim3 grid((unsigned)nch, (unsigned)((mp + 255) / 256));
  const int dp = dp_bucket(d);
  switch (time_kind) {
    case KM12: launch_whiten_kfu_t<KM12>(st, out_kind, dp, grid, rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    case KM32: launch_whiten_kfu_t<KM32>(st, out_kind, dp, grid, rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
    default: launch_whiten_kfu_t<KM52>(st, out_kind, dp, grid, rec, v, ldv, d, z, ldz, m, mp, n, L, inv_lo, s_o, beta, ldb, send, mc, g, hsum); break;
  }
}

void launch_whiten_vec(hipStream_t st, int sdim, const double* rec, int64_t recstride,
                       const double* y, int64_t ldy, int64_t n, int L, int64_t nch, int nchains,
                       double* alpha, int64_t lda, double* send, int64_t sendstride, int64_t mc,
                       int64_t col, int64_t astride) {
  dim3 grid((unsigned)nch, (unsigned)nchains);
  GPAR_DISPATCH_D(sdim, whiten_vec<DD><<<grid, 64, 0, st>>>(rec, recstride, y, ldy, n, L, nch, alpha, lda, send, sendstride, mc, col, astride));
}

int carry_group_size(int64_t nch) {
  int gs = 1;
  while ((int64_t)gs * gs < nch && gs < kMaxCarryGS) ++gs;
  return gs;
}

void launch_carry(hipStream_t st, int sdim, const double* phi, int64_t phistride,
                  const double* send, double* cin, int64_t sstride, int64_t nch, int64_t mc,
                  int64_t ncols, int nchains, double* gend, double* gin, double* psi, bool rev) {
  const int GS = carry_group_size(nch);
  const int64_t ng = (nch + GS - 1) / GS;
  const int64_t gstride_ = ng * mc * kSStride;
  const int64_t psistride = ng * sdim * sdim;
  dim3 g3((unsigned)((ncols + 255) / 256), (unsigned)ng, (unsigned)nchains);
  dim3 g3p((unsigned)((ncols + 255) / 256 + 1), (unsigned)ng, (unsigned)nchains);   // + Psi block
  dim3 gc((unsigned)((ncols + 255) / 256), (unsigned)nchains);
#define GPAR_CARRY_LAUNCH(RV)                                                                       \
  GPAR_DISPATCH_D(sdim, {                                                                          \
    carry_group_local<DD, RV><<<g3p, 256, 0, st>>>(phi, phistride, send, sstride, nch, mc, ncols, GS, gend, gstride_, psi, psistride); \
    carry_group_scan<DD><<<gc, 256, 0, st>>>(psi, psistride, gend, gin, gstride_, ng, mc, ncols);   \
    carry_group_apply<DD, RV><<<g3, 256, 0, st>>>(phi, phistride, send, cin, sstride, gin, gstride_, nch, mc, ncols, GS); \
  })
  if (rev) {
    GPAR_CARRY_LAUNCH(true);
  } else {
    GPAR_CARRY_LAUNCH(false);
  }
#undef GPAR_CARRY_LAUNCH
}

void launch_chain_carry_lml(hipStream_t st, int sdim, const double* phi, int64_t phistride,
                            const double* send, int64_t sstride, const double* logs,
                            const double* mom, int64_t nch, int64_t n, int nchains, double* lml,
                            NmDev<3>* nm, ChainParamsHost* cps, int* active) {
  GPAR_DISPATCH_D(sdim, chain_carry_lml<DD><<<nchains, 256, 0, st>>>(
                            phi, phistride, send, sstride, logs, mom, nch, n, lml, nm,
                            reinterpret_cast<ChainParams*>(cps), active));
}

void launch_gains_adjoint(hipStream_t st, int sdim, const double* rec, int64_t n, int L,
                          int64_t nch, int nchains, double* h) {
  dim3 grid((unsigned)((nch + 255) / 256), (unsigned)nchains);
  GPAR_DISPATCH_D(sdim, gains_adjoint<DD><<<grid, 256, 0, st>>>(rec, n, L, nch, h));
}

void launch_adjoint_local(hipStream_t st, int sdim, double* X, int64_t ldx, int64_t ncols,
                          const double* rec, const double* g, const double* cin, int64_t mc,
                          int64_t n, int L, int64_t nch, double* bend, int nchains,
                          int64_t xstride, int64_t sstride) {
  if (ncols == 1 && ldx == 1 && mc == 1) {   // one column per chain: a lane per chunk
    dim3 gc((unsigned)((nch + 255) / 256), (unsigned)nchains);
    GPAR_DISPATCH_D(sdim, adjoint_local_col<DD><<<gc, 256, 0, st>>>(X, rec, g, cin, n, L, nch, bend, xstride, sstride));
    return;
  }
  dim3 grid((unsigned)nch, (unsigned)((ncols + 63) / 64), (unsigned)nchains);
  GPAR_DISPATCH_D(sdim, adjoint_local<DD><<<grid, 64, 0, st>>>(X, ldx, ncols, rec, g, cin, mc, n, L, bend, xstride, sstride));
}

void launch_adjoint_local_wide(hipStream_t st, int sdim, double* X, int64_t ldx, int64_t ncols,
                               const double* rec, const double* g, const double* cin, int64_t mc,
                               int64_t n, int L, int64_t nch, double* bend, const double* wmask) {
  // a prediction's Mp + 1 <= 576 columns in one workgroup per chunk: the whole row of X is read
  // by one workgroup at a time (256-column workgroups otherwise)
  if (ncols <= 576 && ncols > 256) {
    dim3 grid((unsigned)nch, 1u);
    GPAR_DISPATCH_D(sdim, (adjoint_local_wide<DD, 576><<<grid, 576, 0, st>>>(X, ldx, ncols, rec, g, cin, mc, n, L, bend, wmask)));
    return;
  }
  dim3 grid((unsigned)nch, (unsigned)((ncols + 255) / 256));
  GPAR_DISPATCH_D(sdim, (adjoint_local_wide<DD, 256><<<grid, 256, 0, st>>>(X, ldx, ncols, rec, g, cin, mc, n, L, bend, wmask)));
}

void launch_smooth_mean(hipStream_t st, int sdim, const double* u, const double* h,
                        const double* chat, int64_t sstride, const double* y, int64_t ldy,
                        const double* noise, const ChainParamsHost* cps, int64_t n, int L,
                        int nchains, double* mean, int64_t ldm) {
  dim3 grid((unsigned)((n + 255) / 256), (unsigned)nchains);
  GPAR_DISPATCH_D(sdim, smooth_mean<DD><<<grid, 256, 0, st>>>(u, h, chat, sstride, y, ldy, noise, reinterpret_cast<const ChainParams*>(cps), n, L, mean, ldm));
}

int64_t cov_carry_scratch_doubles(int sdim, int64_t nch, int nchains) {
  const int64_t ng = (nch + carry_group_size(nch) - 1) / carry_group_size(nch);
  return (int64_t)nchains * ng * 3 * sdim * sdim;
}

void launch_smooth_back(hipStream_t st, int sdim, const double* rec, const double* g,
                        const double* pf, const ChainParamsHost* cps, const double* cin, double* X,
                        double* h, double* vloc, double* gam, double* agg, double* bend, int64_t n,
                        int L, int64_t nch, int nchains, int64_t xstride, int64_t sstride) {
  dim3 grid((unsigned)((nch + 255) / 256), (unsigned)nchains);
  const ChainParams* c = reinterpret_cast<const ChainParams*>(cps);
  GPAR_DISPATCH_D(sdim, smooth_back<DD><<<grid, 256, 0, st>>>(rec, g, pf, c, cin, X, h, vloc, gam, agg, bend, n, L, nch, xstride, sstride));
}

void launch_cov_smooth(hipStream_t st, int sdim, const double* t, const double* rec,
                       const double* pf, const ChainParamsHost* cps, int64_t n, int L,
                       int64_t nch, int nchains, double* vloc, double* gam, double* agg,
                       double* phat, double* var, int64_t ldv, double* scratch, bool local_done) {
  dim3 grid((unsigned)((nch + 255) / 256), (unsigned)nchains);
  dim3 gout((unsigned)((n + 255) / 256), (unsigned)nchains);
  const ChainParams* c = reinterpret_cast<const ChainParams*>(cps);
  const int GS = carry_group_size(nch);
  const int64_t ng = (nch + GS - 1) / GS;
  dim3 gg((unsigned)((ng + 255) / 256), (unsigned)nchains);
  GPAR_DISPATCH_D(sdim, {
    double* gagg = scratch;
    double* gin = scratch + (int64_t)nchains * ng * 2 * DD * DD;
    if (!local_done) cov_local<DD><<<grid, 256, 0, st>>>(t, rec, pf, c, n, L, nch, vloc, gam, agg);
    cov_group_local<DD><<<gg, 256, 0, st>>>(agg, nch, GS, ng, nchains, gagg);
    cov_group_scan<DD><<<(nchains + 63) / 64, 64, 0, st>>>(gagg, ng, nchains, gin);
    cov_group_apply<DD><<<gg, 256, 0, st>>>(agg, gin, nch, GS, ng, nchains, phat);
    cov_out<DD><<<gout, 256, 0, st>>>(vloc, gam, phat, n, L, nch, var, ldv);
  });
}

int64_t vec_fix_blocks(int64_t n) { return (n + 255) / 256; }

void launch_vec_fix(hipStream_t st, int sdim, double* alpha, int64_t lda, const double* g,
                    int64_t gstride, const double* cin, int64_t sstride, int64_t mc,
                    int64_t col, int64_t n, int L, int nchains, double* part, double* hsum,
                    int64_t ncols, double* qout) {
  dim3 grid((unsigned)vec_fix_blocks(n), (unsigned)nchains);
  GPAR_DISPATCH_D(sdim, vec_fix<DD><<<grid, 256, 0, st>>>(alpha, lda, g, gstride, cin, sstride, mc, col, n, L, part, hsum, ncols, qout));
}

void launch_chain_lml(hipStream_t st, const double* logs, int64_t nch, const double* a2part,
                      int64_t npart, int64_t n, int nchains, double* lml) {
  chain_lml<<<nchains, 256, 0, st>>>(logs, nch, a2part, npart, n, lml);
}

}  // namespace gpar
