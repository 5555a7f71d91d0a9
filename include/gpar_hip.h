/*
 * gpar_hip.h -- C-ABI of the MI355X-native GPAR-at-scale hot path.
 *
 * The reference (TudorParas/GPAR-at-scale) is a Julia package whose hot path is a set
 * of plain Julia functions.  Each entry point below replaces one of them; the Julia
 * `ccall` binding a maintainer would add is julia/GPARatScaleHIP.jl (INTEGRATION.md explains
 * how to wire it in), the Python ctypes mirror is gpar-at-scale_amd/python/gparatscale/.
 *
 * Conventions
 *   - return value: gpar_status (0 = OK); gpar_last_error(ctx) describes the failure.
 *     GPAR_ERR_NOT_PD mirrors Julia's PosDefException thrown by `cholesky`
 *     (dtc.jl:119-120, gpar_scaled_inference.jl:159,188); GPAR_ERR_ARG mirrors the
 *     DomainError of util.jl:112-117 and malformed inputs.
 *   - fp64 only.  Sizes are int64_t.  Calls are synchronous on return.
 *   - Pointers are borrowed: read-only inputs, never retained past return.  Inputs live
 *     in host memory (mem = GPAR_MEM_HOST) or are already resident in device HBM
 *     (mem = GPAR_MEM_DEVICE, e.g. torch tensors' data_ptr()).  Outputs follow the same
 *     `mem` as the inputs of the call unless stated otherwise.
 *   - Inputs V (one point = one column of the reference's ColVecs, util.jl:16-31): point k,
 *     dimension i lives at v[k*ldv + i]; ldv >= d lets V be a view into an N x P
 *     row-major output matrix (GPAR's previous outputs).
 *   - theta in natural units, as returned by unpack_gpar (util.jl:45-55):
 *     (time_l, time_var, out_l, out_var, noise_sigma); kernel variances are the squares
 *     (dtc.jl:31,37).  log_theta = the reference's i_log_* initial values.
 *   - One gpar_ctx per GPU, one host thread per ctx (not thread-safe).
 */
#ifndef GPAR_HIP_H
#define GPAR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPAR_ABI_VERSION 1

typedef enum gpar_status {
  GPAR_OK = 0,
  GPAR_ERR_ARG = 1,         /* invalid argument (DomainError / malformed input)        */
  GPAR_ERR_NOT_PD = 2,      /* Cholesky of a non positive-definite matrix              */
  GPAR_ERR_HIP = 3,         /* HIP runtime failure                                     */
  GPAR_ERR_OOM = 4,         /* device allocation failed                                */
  GPAR_ERR_UNSUPPORTED = 5, /* configuration outside what the kernels implement        */
  GPAR_ERR_STATE = 6        /* context misuse (NULL ctx, ...)                          */
} gpar_status;

typedef enum gpar_kernel {
  GPAR_MATERN12 = 0, /* Stheno Matern12() */
  GPAR_MATERN32 = 1, /* Stheno Matern32() */
  GPAR_MATERN52 = 2, /* Stheno Matern52() (the reference's default everywhere) */
  GPAR_EQ = 3        /* Stheno EQ(): output kernel only (no finite state-space form) */
} gpar_kernel;

typedef enum gpar_mem { GPAR_MEM_HOST = 0, GPAR_MEM_DEVICE = 1 } gpar_mem;

typedef enum gpar_predict_mode {
  GPAR_PREDICT_ANALYTIC = 0, /* exact S -> infinity limit of the reference's MC estimator */
  GPAR_PREDICT_MC = 1,       /* reference-faithful Monte Carlo (gpar_scaled_inference.jl:110-130) */
  GPAR_PREDICT_PATH = 2      /* Monte Carlo over posterior paths (src/gp/tmp.jl:119-167): per sample
                                a q(u) draw and a posterior_rand path of the time GP (simulation
                                smoother, gpar_lgssm_posterior_rand) */
} gpar_predict_mode;

typedef struct gpar_ctx gpar_ctx;

/* One scaled-GPAR output: the arguments of compute_gpar_dtc_objective / get_optim_scaled_gpar_params
 * (dtc.jl:11-25, 83-91) with the FiniteGPs f = GP(k_o)(V, sigma^2), u = GP(k_o)(Z, sigma^2) unfolded. */
typedef struct gpar_problem {
  int64_t n;            /* training points N                                           */
  int64_t m;            /* pseudo-points M                                             */
  int64_t d;            /* input dimension D = number of previous outputs (>= 1)       */
  const double* t;      /* [n] time locations, ascending (dtc.jl:102 does not sort)    */
  const double* v;      /* inputs,        point k dim i at v[k*ldv + i]                */
  int64_t ldv;          /* >= d                                                        */
  const double* z;      /* pseudo-inputs, point j dim i at z[j*ldz + i]                */
  int64_t ldz;          /* >= d                                                        */
  const double* y;      /* [n] targets                                                 */
  int32_t out_kernel;   /* gpar_kernel of f_x (dtc.jl:16)                              */
  int32_t time_kernel;  /* GPAR_MATERN12/32/52 of f_t (dtc.jl:17)                      */
  int32_t kuu_noise;    /* 1: Kuu + sigma^2 I as FiniteGP cov(u) (dtc.jl:35,119)       */
  int32_t mem;          /* gpar_mem of t, v, z, y                                      */
  int32_t qu_kuu_noise; /* q(u)/prediction: 0 = Cuu without noise as the reference
                           (gpar_scaled_inference.jl:157); 1 = Cuu + sigma^2 I like the
                           objective (opt-in: robust when pseudo-inputs nearly coincide)     */
} gpar_problem;

typedef struct gpar_fit_options {
  int32_t max_evals;      /* >0: objective evaluations per output incl. the final centroid
                             evaluation (the build's reproducible budget); 0 = unlimited   */
  int32_t max_iterations; /* Optim.Options iterations (default 1000)                      */
  double g_tol;           /* Optim NelderMead convergence tolerance (default 1e-8; <0 off)  */
  double time_limit;      /* seconds of wall clock (dtc.jl:21 optimization_time_limit);
                             <=0 = none                                                    */
} gpar_fit_options;

/* ---------------------------------------------------------------- context */
int32_t gpar_abi_version(void);
int32_t gpar_ctx_create(int32_t device, gpar_ctx** out);
int32_t gpar_ctx_destroy(gpar_ctx* ctx);
const char* gpar_last_error(const gpar_ctx* ctx);
/* bytes of device workspace currently held by the context */
int64_t gpar_ctx_workspace_bytes(const gpar_ctx* ctx);
/* release cached device workspace */
int32_t gpar_ctx_trim(gpar_ctx* ctx);
/* Kernel timing with HIP events on the context's stream (bench / roofline support).
 * name: "gram" (the fp64 MFMA Gram contraction), "whiten" (Kfu assembly + Kalman whitening),
 * "gains" (parallel Riccati scan), "dense" (M x M Cholesky / solves).  total_ms accumulates
 * over launches since the last reset. */
int32_t gpar_ctx_set_profiling(gpar_ctx* ctx, int32_t on);
int32_t gpar_ctx_kernel_stats(gpar_ctx* ctx, const char* name, int64_t* launches, double* total_ms);
int32_t gpar_ctx_reset_stats(gpar_ctx* ctx);
/* Algorithmic work of the timed launches of a family since the last reset (for rooflines):
 * "gram": flops, N M (M + 1) per launch; "whiten": HBM bytes, 8 N (D + M + 20) per launch (V read,
 * gains records + fix-up rows, beta written), with M in place of D when the distances come from the
 * fit's cache or a distance pass; "dist2": flops, 2 N Mp D per distance pass (the fit's cache fill,
 * or the per-evaluation pass of an uncached output wider than 64). */
int32_t gpar_ctx_kernel_work(gpar_ctx* ctx, const char* name, double* work);
/* Process-wide diagnostic counters (tests; no device work): "gains_fast" / "gains_general" = the
 * gains' phase-3 launches that took the LDS-DMA fast kernel / the general kernels since the library
 * was loaded.  -1 for an unknown name. */
int64_t gpar_debug_counter(const char* name);
/* Concurrency of batched calls (gpar_dtc_objective / gpar_fit with nprob > 1): lanes = 2
 * alternates the outputs' whitening + Gram between two HIP streams with separate workspaces so
 * one output's whitening overlaps another's Gram (~1 % faster at N = 1e6, M = 512, two beta
 * buffers); 1 (the default) serialises them on the context stream. */
int32_t gpar_ctx_set_lanes(gpar_ctx* ctx, int32_t lanes);
/* CU split of the batched fit (one lane): with cus_per_xcd = w > 0, each output's Kfu assembly +
 * whitening runs on w CUs of every XCD while the previous output's Gram runs on the other 32 - w
 * (CU-masked HIP streams; a w/32 share of the Gram's diagonal-block work also goes to the
 * whitening side).  w = 0: whole-chip kernels, one after the other.  w must be a multiple of 4
 * below 32 (equal SE widths).  An explicit w applies to every batched
 * fit; -1 restores the default: w = 8 for batched fits with N * Mp^2 >= 1e11 (smaller Grams run
 * whole-chip), 0 on devices without 256 CUs; the environment variable GPAR_SPLIT_CUS sets an
 * explicit width at context creation.  Results agree with the whole-chip schedule up to the
 * Gram's split plan (last bits; deterministic for a given w). */
int32_t gpar_ctx_set_cu_split(gpar_ctx* ctx, int32_t cus_per_xcd);
/* Round-overlapping batched fit (on by default; the environment variable GPAR_OVERLAP=0 turns it
 * off at context creation): on the CU-split schedule with 4..16 outputs per call (one rank's
 * shard of the north job; a call with more outputs has long rounds and keeps the round-by-round
 * schedule, which measured faster there), gpar_fit /
 * gpar_fit_predict deal the outputs into two groups whose Nelder-Mead rounds take turns, so one
 * group's dense tail, host step and next-round gains overlap the other group's whitenings and
 * Grams instead of draining the chip after every round.  Each output evaluates the same points
 * with the same arithmetic: results are bit-identical either way. */
int32_t gpar_ctx_set_fit_overlap(gpar_ctx* ctx, int32_t on);
/* ANALYTIC prediction with m <= 512 (on by default; GPAR_PREDICT_FUSED=0 turns it off at context
 * creation): the test rows' Q_i = R Sigma^{-1} Cf*u rows, the mean and the variance |Q_i V^T|^2
 * in one fused kernel (predict_var), Q never stored; off: predict_rows writes Q and gemm_nt reads
 * it.  Same quantities, summed in a different order (last bits). */
int32_t gpar_ctx_set_predict_fused(gpar_ctx* ctx, int32_t on);
/* Schedule knobs: each selects an order or a placement of the same launches, never different
 * arithmetic, so results are bit-identical with any setting (tests/test_gpu_schedule.py):
 *   "overlap"       1: round-overlapping batched fit, as gpar_ctx_set_fit_overlap (default 1)
 *   "overlap_group" outputs per group of the round overlap: 0 (default) = groups of 8 in calls of
 *                   4..16 outputs (larger calls: round by round); g > 0 = groups of g in any call
 *                   of >= 4 outputs
 *   "qu_batch"      1: gpar_fit_predict runs q(u) batched over the outputs (default 1)
 *   "dense_early"   1: the G-independent half of the dense tail ahead of a split round's Grams, on
 *                   the Gram stream (default); 0: after the Grams
 *   "post_gram"     1: a split job's short chain (carry, vec_fix) on the Gram CUs behind the previous
 *                   Gram's correction instead of on the whitening CUs after its whitening; 0: never;
 *                   -1 (default): in the round-overlapping fit only
 *   "compact_rec"   1: the CU-split fit's gains write compact records {K_k, rs_k} and the cached
 *                   whitening recomputes each step's transition A_k from t (the same bits; an
 *                   output whose distances are not cached then whitens through the distance pass
 *                   instead of the fused kernel: last bits); 0: full records {A_k, K_k, rs_k};
 *                   -1 (default): in the round-overlapping fit when every output is cached
 *   "predict_lanes" 1 or 2: streams gpar_fit_predict's predictions alternate over (default 2)
 *   "serialize"     1: every launch of every schedule on the context's one stream, in issue order,
 *                   with the same plans, CU shares of work items and workspaces: the order-free
 *                   reference the concurrent schedule equals bit for bit (default 0)
 *   "predict_fused" as gpar_ctx_set_predict_fused (changes the summation order: last bits)
 *   "dg_rows_w"     percent more rows per diagonal-block time split on the whitening CUs of a
 *                   split Gram, fewer on the Gram CUs; -100 (default) = auto: 40 in the
 *                   round-by-round fit, 20 in the round overlap (changes G's summation grouping:
 *                   last bits, like predict_fused)
 *   "gram_group"    outputs per grouped Gram of an unsplit batched fit: the group's outputs whiten
 *                   over two streams into buffers of their own and one set of Gram launches covers
 *                   them all (grid y = output), each with 1/g of the time splits; -1 (default) =
 *                   auto: groups of 8 when one output's N Mp^2 <= 5e10 (the dtc / eeg configs),
 *                   0 = per-output Grams; a plan like dg_rows_w (G's summation grouping: last bits)
 *   "fit_chunks"    outputs per consecutive sub-batch of a gpar_fit whose outputs' distances the
 *                   cache cannot hold all at once: each sub-batch computes its distances once
 *                   and every evaluation reads them, instead of the outputs left uncached
 *                   recomputing theirs every evaluation.  -1 (default) = auto: fits too large
 *                   to pipeline (beta > 8 GB: the N = 1e7, M = 1024 stress config): the outputs
 *                   with D < 17 (fused whitening, never cached) as one sub-batch, the others in
 *                   sub-batches of as many outputs as the free memory (or an explicit
 *                   gpar_ctx_set_dist_cache budget) holds; 0 = one batch; k >= 1 = sub-batches
 *                   of k consecutive outputs.  Not for gpar_fit_predict / gpar_fit_posterior.  Each
 *                   output's fit is independent of its batch, so a sub-batched fit equals the
 *                   one-batch fit with every output cached bit for bit
 *   "device_nm"     the chains fit of gpar_sde_predictions steps its Nelder-Mead machines on
 *                   the device after each evaluation round (1, default: rounds queue back to
 *                   back, the host reads the running count one batch of 8 rounds behind) or on
 *                   the host after each round's values come back (0).  A fit with a wall-clock
 *                   time limit always runs on the host.  The same steps; the device's exp() in
 *                   the chain parameters may move a value in its last bit
 * The environment variable GPAR_<KNOB> (upper case) sets a knob at context creation.
 * GPAR_ERR_ARG for an unknown knob or value.  Every non-default value is a supported schedule
 * mode; the A/B-only knobs of round 4 (split_head, dg_share, tail_cus, predict_d2, dense_early 2)
 * were measured slower at both the north job and the 8-output shard and deleted. */
int32_t gpar_ctx_set_schedule(gpar_ctx* ctx, const char* knob, int32_t value);
int32_t gpar_ctx_get_schedule(const gpar_ctx* ctx, const char* knob, int32_t* value);
/* The CU split in effect (0 when off or unsupported). */
int32_t gpar_ctx_get_cu_split(const gpar_ctx* ctx, int32_t* cus_per_xcd);
/* Distance cache of gpar_fit / gpar_fit_predict: the input distances |v_k - z_c| (squared for EQ)
 * are theta-independent, so they are computed once per fit call (N x Mp doubles per output, widest
 * outputs first) and every objective evaluation's whitening reads them instead of rebuilding them
 * inside the fused kernel.  Which outputs: D >= 17; every output (D >= 1) in a batched fit over
 * N >= 2^16 points that runs the pipelined CU-split schedule (gpar_ctx_set_cu_split), where the
 * whitening has a quarter of the chip.  bytes = -1 (the default): the budget is the free device
 * memory less 1 % of the part and less the workspace the call still has to allocate (the fit's,
 * and gpar_fit_predict's predictions'); 0: off; > 0: that budget.  A cache allocation that fails
 * stops the cache there, and a later workspace allocation that finds no memory evicts cache slots
 * and retries, so the cache never turns into an out-of-memory failure.  The cached distances are
 * the same Gram-form values the fused kernel builds, in another summation order: results agree
 * with an uncached fit to the last bits (fitted theta rtol 1e-9), and gpar_fit_predict, which
 * reuses the fit's Gram at the fitted theta for q(u), can then differ from gpar_predict in the
 * last bits.  Device memory taken by the cache is not visible to other allocators in the process
 * (torch's caching allocator) while the fit runs. */
int32_t gpar_ctx_set_dist_cache(gpar_ctx* ctx, int64_t bytes);
/* keep = 0 (the default): the cache is released when the fit call returns.  keep = 1: the buffers
 * stay in the context's workspace and the next fit reuses them (no re-allocation), evictable by
 * any later allocation that runs out of memory; gpar_ctx_trim or keep = 0 releases them. */
int32_t gpar_ctx_set_dist_cache_keep(gpar_ctx* ctx, int32_t keep);
/* outputs_cached: outputs the last fit call cached; evictions: cache slots evicted by
 * out-of-memory retries since the context was created; bytes_held: cache bytes held now.
 * Any pointer may be NULL. */
int32_t gpar_ctx_dist_cache_stats(const gpar_ctx* ctx, int32_t* outputs_cached, int32_t* evictions,
                                  int64_t* bytes_held);
/* Producer ordering for GPAR_MEM_DEVICE inputs: with enable = 1, every later call on ctx first
 * makes its streams wait (device side, hipStreamWaitEvent) for all work queued so far on
 * `stream` (a hipStream_t; 0 = the null stream), e.g. the copies that produced its device inputs
 * on the caller's stream.  enable = 0 turns it off (the default). */
int32_t gpar_ctx_set_input_stream(gpar_ctx* ctx, void* stream, int32_t enable);

/* ---------------------------------------------------------------- DTC objective
 * Replaces compute_gpar_dtc_objective (src/gp/dtc.jl:83-128), batched over `nprob`
 * independent outputs.  theta: nprob x 5 (natural units, row per output), host memory.
 * dtc_out: [nprob] log marginal likelihood (DTC), host memory. */
int32_t gpar_dtc_objective(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                           const double* theta, double* dtc_out);

/* Same, for one output, also returning the reference's second tuple element
 * A = chol(cov(u)).U' \ beta'  (M x N, column-major: A[i + j*m]), host memory.
 * Materialises A: intended for parity checks at modest N*M. */
int32_t gpar_dtc_objective_A(gpar_ctx* ctx, const gpar_problem* prob, const double* theta,
                             double* dtc_out, double* A_out);

/* The distances Kfu = pairwise(k_o, V, Z) is built from (dtc.jl:104; Stheno evaluates k_o on
 * Distances.jl's pairwise distances), as the fit's distance cache holds them: dist_out[k*m + c] =
 * |v_k - z_c| for the Matern output kernels (Gram form |v|^2 + |z|^2 - 2 v.z about per-256-column
 * centres, clamped at 0, for Matern-3/2 / 5/2; direct differences for Matern-1/2) and the squared
 * distance for EQ.  n x m, in prob->mem.  For parity checks of the cache. */
int32_t gpar_pairwise_distances(gpar_ctx* ctx, const gpar_problem* prob, double* dist_out);

/* ---------------------------------------------------------------- fit
 * Replaces get_optim_scaled_gpar_params (src/gp/dtc.jl:11-77): Nelder-Mead over the 5
 * log-hyperparameters maximising the DTC objective, batched over nprob outputs (one GPU
 * evaluation round serves every output's pending simplex point).
 * log_theta0: nprob x 5 initial log-params (host).  theta_out: nprob x 5 natural units
 * (host).  nlml_out: [nprob] final -dtc (host, may be NULL).  evals_out: [nprob] (may be NULL). */
int32_t gpar_fit(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                 const double* log_theta0, const gpar_fit_options* opts,
                 double* theta_out, double* nlml_out, int32_t* evals_out);

/* ---------------------------------------------------------------- q(u)
 * Replaces compute_q_u (src/gp/gpar_scaled_inference.jl:141-196) at theta (natural units).
 * Cuu carries NO noise here (:157); prob->kuu_noise is ignored.  Outputs (host):
 * m_e [m], cov [m x m] = inv(D) (Symmetric), U_u [m x m] upper Cholesky factor of Cuu;
 * matrices column-major. */
int32_t gpar_q_u(gpar_ctx* ctx, const gpar_problem* prob, const double* theta,
                 double* m_e, double* cov, double* U_u);

/* ---------------------------------------------------------------- prediction
 * Replaces the prediction half of get_gpar_scaled_predictions
 * (src/gp/gpar_scaled_inference.jl:63-135) at a fitted theta: q(u), merge train+test,
 * Cf*u, LGSSM with R = sigma^2 (train) / 1e10 (test), RTS smoothing.
 * t_star [n_star], v_star point k dim i at v_star[k*ldvs + i]; in prob->mem.
 * mean/std [n_star] in prob->mem.  ANALYTIC: mean and std of the latent f (the MC
 * estimator's S -> infinity limit); MC: `samples` (2..65536; the reference takes 100) draws with
 * the given seed (gpar_mc_normals), mean and Bessel-corrected std over samples as the reference
 * does; PATH: tmp.jl's variant, each sample's smoothed mean replaced by a posterior path draw
 * (q(u) draws gpar_mc_normals, path draws gpar_path_normals), so the std also carries the time
 * GP's posterior variance. */
int32_t gpar_predict(gpar_ctx* ctx, const gpar_problem* prob, const double* theta,
                     int64_t n_star, const double* t_star, const double* v_star, int64_t ldvs,
                     int32_t mode, int32_t samples, uint64_t seed, double* mean, double* std);

/* The standard-normal draws MC mode uses for (samples, m, seed): xi_out[s*m + j] is the j-th
 * coordinate of draw s (host, samples x m).  The m_e sample of draw s is m_e + chol(inv(D)).L
 * xi_s, as Distributions' rand(MvNormal(m_e, Symmetric(inv(D)))) maps a standard-normal vector
 * (gpar_scaled_inference.jl:103,185), so a host-side restatement fed these draws reproduces the
 * device's MC estimate.  gpar_fit_predict draws output i with seed + i. */
int32_t gpar_mc_normals(gpar_ctx* ctx, int32_t samples, int64_t m, uint64_t seed, double* xi_out);

/* The posterior-path draws of GPAR_PREDICT_PATH / gpar_lgssm_posterior_rand for (samples, n, d,
 * seed), host samples x n x d: with d = D + 1 (D = 1, 2, 3, the state dimension of Matern-1/2, 3/2,
 * 5/2), xi_out[(s*n + k)*d + i] for i < D is the state noise of step k of sample s's prior path and
 * i = D its observation noise (the simulation smoother, gpar_lgssm_posterior_rand).  Independent of
 * the q(u) draws of the same seed (gpar_mc_normals). */
int32_t gpar_path_normals(gpar_ctx* ctx, int32_t samples, int64_t n, int32_t d, uint64_t seed,
                          double* xi_out);

/* ---------------------------------------------------------------- fit + predict
 * Replaces get_gpar_scaled_predictions (src/gp/gpar_scaled_inference.jl:20-136) -- the fit of
 * get_optim_scaled_gpar_params, then q(u) and the prediction at the fitted theta -- for `nprob`
 * outputs at once: the batched fit of gpar_fit, then per output exactly gpar_predict at its
 * fitted theta (theta_out row i).  With probs[i].qu_kuu_noise = 1, q(u)'s Gram at the fitted
 * theta is the one the fit already computed there (same kernels, same inputs: bit-identical), so
 * it is reused instead of recomputed; with the reference's noise-free Cuu q(u) recomputes it from
 * the fixed-up beta (less rounding for the ill-conditioned Cuu: the fit's correction-form Gram
 * measured 1.5e-7 relative off the oracle there).  Test inputs: t_star [n_star]
 * shared, output i's at v_star[i] (point k dim j at v_star[i][k*ldvs[i] + j]); mean_out[i],
 * std_out[i] [n_star]; all in probs[i].mem (one memory space for all outputs).  MC mode draws
 * output i with seed + i. */
int32_t gpar_fit_predict(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                         const double* log_theta0, const gpar_fit_options* opts, int64_t n_star,
                         const double* t_star, const double* const* v_star, const int64_t* ldvs,
                         int32_t mode, int32_t samples, uint64_t seed, double* theta_out,
                         double* nlml_out, int32_t* evals_out, double* const* mean_out,
                         double* const* std_out);

/* Same, with chained inference inputs (examples/GPAR_scaled_examples.jl:172 passes y2's predicted
 * means as y3's inference inputs; examples/eeg.jl:249,274 likewise): the fit is batched as above,
 * the predictions then run in output order i = 0..nprob-1, and after output i's prediction its
 * mean is also written to column chain_col[i] of `chain` (point k at chain[k*ld_chain + col];
 * chain_col[i] < 0: not written).  A later output's v_star may point into `chain` (e.g. v_star[i] =
 * chain, ldvs[i] = ld_chain, its first d columns holding earlier outputs' predicted means) and
 * then reads them.  chain in probs[0].mem; device writes are stream-ordered before the next
 * prediction reads them.  Order outputs so that every producer precedes its consumers. */
int32_t gpar_fit_predict_chain(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                               const double* log_theta0, const gpar_fit_options* opts,
                               int64_t n_star, const double* t_star, const double* const* v_star,
                               const int64_t* ldvs, int32_t mode, int32_t samples, uint64_t seed,
                               double* chain, int64_t ld_chain, const int32_t* chain_col,
                               double* theta_out, double* nlml_out, int32_t* evals_out,
                               double* const* mean_out, double* const* std_out);

/* ---------------------------------------------------------------- posterior objects
 * get_gpar_scaled_predictions (src/gp/gpar_scaled_inference.jl:20-136) split at the point where it
 * first reads the inference inputs: gpar_fit_posterior runs the batched fit of gpar_fit and q(u)
 * at every output's fitted theta (:63-73, compute_q_u :141-196; with the fit's Gram where
 * gpar_fit_predict reuses it) and keeps q(u) on the device; gpar_posterior_predict then runs output i's
 * prediction for inference inputs that may arrive later -- the chained sweep of
 * examples/GPAR_scaled_examples.jl:172 and examples/eeg.jl:249,274, where output p's inputs are
 * the predicted means of outputs < p, possibly owned by other ranks.  gpar_posterior_predict
 * equals the prediction half of gpar_fit_predict bit for bit.  Device problems' t, v, z, y are
 * borrowed until gpar_posterior_destroy (host problems are copied to the device); the posterior
 * holds ~3 Mp^2 doubles of device memory per output and belongs to ctx's device.  t_star, v_star,
 * mean, std of a predict call are in the problems' memory space. */
typedef struct gpar_posterior gpar_posterior;
int32_t gpar_fit_posterior(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                           const double* log_theta0, const gpar_fit_options* opts,
                           double* theta_out, double* nlml_out, int32_t* evals_out,
                           gpar_posterior** out);
int32_t gpar_posterior_predict(gpar_ctx* ctx, const gpar_posterior* post, int32_t i,
                               int64_t n_star, const double* t_star, const double* v_star,
                               int64_t ldvs, int32_t mode, int32_t samples, uint64_t seed,
                               double* mean, double* std);
/* Queue the part of output i's prediction that does not read the inference inputs -- the merged
 * train + test grid's gains and adjoint fix-up rows for the (device, ascending) test times t_star
 * -- on the context's side stream, and return.  The next gpar_posterior_predict for the same
 * posterior, output, t_star pointer and n_star uses it (bit-identical results) instead of
 * computing it in line; a chained sweep prepares output p + 1 before predicting output p, so the
 * two overlap.  Two slots per context: a third prepare reuses the oldest (its predict falls back to
 * the in-line path).  Device-memory posteriors only.  The kernels queued here read t_star
 * asynchronously: t_star must stay allocated and unmodified until the matching
 * gpar_posterior_predict has run (or the context is synchronised).  Slots are matched on the
 * posterior's identity, not its address: a slot left by a destroyed posterior is never used. */
int32_t gpar_posterior_prepare(gpar_ctx* ctx, const gpar_posterior* post, int32_t i,
                               int64_t n_star, const double* t_star);
int32_t gpar_posterior_destroy(gpar_posterior* post);

/* ---------------------------------------------------------------- temporal-only (LGSSM) chains
 * `nchains` independent chains sharing the time grid t [n] (ascending); chain c's
 * observations at y[c*ldy + k].  theta: nchains x 3 natural (l, process_var, noise_sigma)
 * (unpack_gp, util.jl:36-43), host.
 *
 * logpdf(create_lgssm(t, l, pv, sigma, k), y)  (temporal_gp_inference.jl:69-82):
 * lml_out [nchains] host. */
int32_t gpar_lgssm_logpdf(gpar_ctx* ctx, int32_t nchains, int64_t n, const double* t,
                          const double* y, int64_t ldy, int32_t kernel, const double* theta,
                          int32_t mem, double* lml_out);

/* smooth(create_lgssm(...; noise_vector), y) marginals of f (temporal_gp_inference.jl:109,
 * gpar_scaled_inference.jl:117): noise [n] per-step observation variance shared by all
 * chains (NULL = noise_sigma^2 everywhere).  mean/var [nchains*ldy layout like y], in mem. */
int32_t gpar_lgssm_smooth(gpar_ctx* ctx, int32_t nchains, int64_t n, const double* t,
                          const double* y, int64_t ldy, const double* noise, int32_t kernel,
                          const double* theta, int32_t mem, double* mean, double* var);

/* posterior_rand(rng, create_lgssm(t, l, pv, sigma, k; noise_vector), y, samples) (TemporalGPs,
 * called at src/gp/tmp.jl:161-167): `samples` joint draws of the latent f over the grid t from
 * its posterior given y, by the simulation smoother of Durbin & Koopman (2002): a prior path x~
 * with its observations y~, then f = x~[0] + E[f | y - y~] (oracle/gpar_oracle.py
 * lgssm_posterior_rand restates it; exact posterior draws, like forward-filter backward-sample,
 * whose backward coefficients are numerically unstable on clustered grids), draws
 * gpar_path_normals(samples, n, D + 1, seed).  theta: 3 natural (l, process_var, noise_sigma); noise:
 * per-step observation variance or NULL (sigma^2).  f_out[s*n + k] (samples x n), in mem. */
int32_t gpar_lgssm_posterior_rand(gpar_ctx* ctx, int64_t n, const double* t, const double* y,
                                  const double* noise, int32_t kernel, const double* theta,
                                  int32_t samples, uint64_t seed, int32_t mem, double* f_out);

/* get_sde_predictions (temporal_gp_inference.jl:45-114): NM fit of (l, pv, sigma) per chain
 * on -logpdf, then smoothing over the merged train+test grid; marginals of f at t_star.
 * log_theta0 nchains x 3 (host); theta_out nchains x 3 (host); mean/var: chain c at
 * [c*n_star + k], in mem. */
int32_t gpar_sde_predictions(gpar_ctx* ctx, int32_t nchains, int64_t n, const double* t,
                             const double* y, int64_t ldy, int64_t n_star, const double* t_star,
                             int32_t kernel, const double* log_theta0,
                             const gpar_fit_options* opts, int32_t mem, double* theta_out,
                             double* mean, double* var);

/* ---------------------------------------------------------------- exact GP / GPAR (config 1)
 * logpdf(f(x, sigma^2), y) with the GPAR kernel s_t k_t(x[0]/l_t) + s_o k_o(x[1:]/l_o)
 * (optimized.jl:132-154); x point k dim i at x[k*ldx + i], dx = 1 + #previous outputs
 * (dx == 1: plain GP on time, optimized.jl:28-36, theta = (l, pv, sigma, -, -) uses
 * entries 0, 1 and 4).  theta: 5 natural (host).  lml_out host. */
int32_t gpar_exact_logpdf(gpar_ctx* ctx, int64_t n, int64_t dx, const double* x, int64_t ldx,
                          const double* y, int32_t time_kernel, int32_t out_kernel,
                          const double* theta, int32_t mem, double* lml_out);

/* Posterior marginals of f at x_star (optimized.jl:94,236 + marginals): mean/var [n_star]. */
int32_t gpar_exact_posterior(gpar_ctx* ctx, int64_t n, int64_t dx, const double* x, int64_t ldx,
                             const double* y, int64_t n_star, const double* x_star,
                             int64_t ldxs, int32_t time_kernel, int32_t out_kernel,
                             const double* theta, int32_t mem, double* mean, double* var);

/* ---------------------------------------------------------------- Nelder-Mead (host only)
 * The optimiser gpar_fit / gpar_sde_predictions run (Optim.jl NelderMead restated:
 * AffineSimplexer(0.025, 0.5), adaptive parameters, g_tol, iterations, time_limit, and the final
 * centroid evaluation of Optim's after_while!), exposed as an ask/tell state machine so a
 * host-language driver (the reference's Julia, a test) can step it with its own objective.
 * No GPU involved. */
typedef struct gpar_nm gpar_nm;
int32_t gpar_nm_create(int32_t n, const double* x0, const gpar_fit_options* opts, gpar_nm** out);
int32_t gpar_nm_destroy(gpar_nm* nm);
/* 1 while the optimiser wants more evaluations; x receives the next point (n doubles) */
int32_t gpar_nm_ask(gpar_nm* nm, double* x);
int32_t gpar_nm_tell(gpar_nm* nm, double f);
/* minimiser (n doubles), its value and the number of evaluations / iterations so far */
int32_t gpar_nm_result(const gpar_nm* nm, double* x_min, double* f_min, int32_t* evals,
                       int32_t* iterations);

#ifdef __cplusplus
}
#endif
#endif /* GPAR_HIP_H */
