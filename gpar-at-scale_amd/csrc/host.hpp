// host.hpp -- internals shared by the host units of the C-ABI (include/gpar_hip.h): the context,
// workspace and upload helpers, problem / stage / dense-tail structs, and the functions one unit
// calls in another.  Host orchestration only: every number is computed by the gfx950 kernels
// (k_*.hip); there is no CPU fallback.
#pragma once
#include "gpar_hip.h"

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <memory>
#include <optional>
#include <vector>

#include "launch.hpp"
#include "nelder_mead.hpp"
#include "nm_dev.hpp"

namespace gpar {
struct PredPrep;
constexpr int kDgRowsAuto = -100;   // gpar_ctx::dg_rows_w "auto"
}

struct gpar_ctx {
  int device = 0;
  hipStream_t stream = nullptr;   // the stream every launch goes to (see OnStream)
  hipStream_t main = nullptr;     // the context's stream
  hipStream_t side = nullptr;     // second stream: alternate outputs of a batch run here
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_pw = nullptr, ev_pc[2] = {nullptr, nullptr};   // the fit's pipelined Gram stage
  // Schedule knobs (gpar_ctx_set_schedule; GPAR_<KNOB> in the environment at creation).  Every
  // one selects an order or a placement of the same launches, never different arithmetic:
  // results are bit-identical with any setting (tests/test_gpu_schedule.py).
  // gpar_ctx_set_cu_split(w): the pipelined fit's whitening runs on w CUs of every XCD and the
  // Gram (its co-running correction too) on the other 32 - w, concurrently (CU-masked streams)
  int split_w = 0, split_mask_w = 0;
  bool split_forced = false;      // set explicitly: no problem-size gate (split_active)
  // s_d: the round-overlapping fit's dense tails, on the whitening CUs (fit_overlapped)
  hipStream_t s_w = nullptr, s_g = nullptr, s_g2 = nullptr, s_d = nullptr;
  hipEvent_t ev_gd[2] = {nullptr, nullptr}, ev_sp = nullptr;
  hipEvent_t ev_dn = nullptr;                    // split round start: the dense prefix follows the context stream
  hipEvent_t ev_gr = nullptr;                    // split round: the other outputs' gains done
  hipEvent_t ev_wd = nullptr;                    // split job: its whitening is done (post_gram)
  // gpar_posterior_prepare's two slots (PredPrep, host.hpp): ready on the side stream / free again
  // (their prediction done on the context stream)
  hipEvent_t ev_prep_ready[2] = {nullptr, nullptr}, ev_prep_free[2] = {nullptr, nullptr};
  std::vector<gpar::PredPrep> prep;   // the two slots (sized on first use)
  int prep_next = 0;
  // gpar_ctx_set_input_stream: every call first waits (device side) for the work queued so far on
  // the caller's stream, e.g. the copies that produce its device inputs
  bool has_input_stream = false;
  hipStream_t input_stream = nullptr;
  hipEvent_t ev_input = nullptr;
  int lanes = 1;                  // gpar_ctx_set_lanes: streams a batch's outputs alternate over
  int64_t dist_cache_bytes = -1;  // gpar_ctx_set_dist_cache: -1 auto, 0 off, else a byte budget
  bool dist_cache_keep = false;   // gpar_ctx_set_dist_cache_keep: hold the cache past the fit call
  // per distance-cache slot ("distcache<i>"): still resident.  An allocation that runs out of
  // memory evicts the whole cache (ws) and clears these, so the fit's later launches fall back to
  // the fused kernel instead of failing (the cache is recomputable, never required)
  std::vector<char> cache_valid;
  int32_t cache_outputs = 0;      // outputs the last fit call cached
  int32_t cache_evictions = 0;    // OOM evictions since the context was created
  // Pinned upload arenas of the round-overlapping fit (fit_overlapped): with `staging` set, h2d
  // copies through it, so an upload queued behind running work never blocks the host (a
  // pageable-memory copy may wait for its stream).  One arena per output group, reset when that
  // group's previous round has been consumed.
  struct Staging {
    char* host = nullptr;
    size_t cap = 0, used = 0;
  };
  std::vector<Staging> stage;   // one per output group (deque-like: grown before use, never moved after)
  Staging* staging = nullptr;
  bool overlap = true;            // "overlap": round-overlapping batched fit (gpar_ctx_set_fit_overlap)
  int predict_lanes = 2;          // "predict_lanes": gpar_fit_predict's predictions over 1 or 2 streams
  bool predict_fused = true;      // "predict_fused": predict_var (off: predict_rows + gemm_nt; last bits differ)
  bool qu_batch = true;           // "qu_batch": gpar_fit_predict's q(u) batched over the outputs
  // "dense_early": the G-independent dense tail ahead of a split round's Grams on the Gram stream
  // (1), or after the Grams (0)
  int dense_early = 1;
  int post_gram = -1;             // "post_gram": a split job's short chain on the Gram CUs (s_g2): 1, 0, -1 = round overlap only
  int compact_rec = -1;           // "compact_rec": compact gains records: 1, 0, -1 = round overlap only
  // "gram_group": outputs per grouped Gram launch set in an unsplit batched fit of small problems
  // (run_gram_stage): 0 = off, >= 2 that many, 1 = off, -1 = auto (kGramGroupAuto below)
  int gram_group = -1;
  // set by eval_dtc when the round's dense prefix runs on s_d: the round's first Gram waits for it
  // (beside a Gram the latency-bound 64 x 64 launches slowed it 4.4 -> 5.3 ms at the eeg shard)
  hipEvent_t gram_after = nullptr;
  // "fit_chunks": outputs per consecutive sub-batch of a gpar_fit whose distances the cache
  // cannot all hold at once (fit_impl): -1 = auto (unpipelined fits of outputs with D >= 17, the
  // stress config), 0 = off (one batch), k >= 1 = sub-batches of k outputs
  int fit_chunks = -1;
  // "device_nm": the chains fit (gpar_sde_predictions) steps its Nelder-Mead machines on the
  // device between rounds (1), or on the host after each round's values come back (0; also any
  // fit with a wall-clock time limit)
  int device_nm = 1;
  // "dg_rows_w": percent more rows per DG split on the whitening CUs (fewer on the Gram CUs);
  // kDgRowsAuto: +40 in the round-by-round fit, where the whitening side (3.19 ms whitening since
  // the DPP step rows, r05r) has time to spare and the Gram CUs' side sets the span (north, same
  // box, 3 pairs: 5.074 ms per Gram / 17.584 s per job at +10 with the r05p whitening, 5.012 ms /
  // 17.384 s at +40; +60: 5.25 ms), +20 in the round overlap, whose whitening side also runs the
  // other group's tails and gains (the 8-output shard 3/8, r05r: 2.278 s at 0, 2.244 at +20,
  // 2.304 at +40; with the r04 whitening 0 was best, r04ad)
  int dg_rows_w = gpar::kDgRowsAuto;
  // "serialize": side, s_w, s_g, s_g2 and s_d all alias `main`, so every launch runs in issue order
  // on one stream (the created streams stay in own_*): the order-free reference the concurrent
  // schedule must equal bit for bit.  Plans, CU shares of work items and workspaces are unchanged.
  bool serialize = false;
  // own_s: s_w, s_g, s_g2 and s_d (the round overlap's dense tails and gains, on the whitening CUs)
  hipStream_t own_side = nullptr, own_s[4] = {nullptr, nullptr, nullptr, nullptr};
  std::string ws_suffix;          // appended to workspace names (a prediction lane's own buffers)
  std::vector<hipEvent_t> ev_grp;   // fit_overlapped: a group's values are in (one per group)
  std::vector<hipEvent_t> ev_gn;    // fit_overlapped: a group's gains are done
  // "overlap_group": outputs per group of the round overlap; 0 (auto) = groups of
  // kOverlapGroupAuto in calls of 4..kOverlapMaxOutputs outputs, g > 0 = groups of g in any call
  // of >= 4 outputs
  int overlap_group = 0;
  std::string err;
  struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
  };
  std::unordered_map<std::string, Buf> bufs;
  // event-based kernel timing (gpar_ctx_set_profiling)
  bool profiling = false;
  struct Pending {
    hipEvent_t e0, e1;
    double work;   // algorithmic work of the timed launches (flops or HBM bytes, per family)
  };
  struct Stat {
    std::vector<Pending> pending;
    int64_t launches = 0;
    double ms = 0.0;
    double work = 0.0;
  };
  std::unordered_map<std::string, Stat> stats;
  // profiling marks of a round-by-round fit round (eval_dtc): its first Gram's start and its last
  // Gram's end on the Gram stream ("round_head" / "round_tail" stats)
  hipEvent_t mark_first = nullptr, mark_last = nullptr;
  hipEvent_t mark_h[3] = {nullptr, nullptr, nullptr};   // the round head's first job: gains, W, P
  // event sequences: stats[names[i]] += time from ev[i - 1] to ev[i] (flush_stats)
  struct MarkSeq {
    std::vector<std::string> names;
    std::vector<hipEvent_t> ev;
  };
  std::vector<MarkSeq> mark_seqs;
};

// MC predictions: most draws a call takes (xi is samples x Mp doubles of workspace)
static constexpr int kMaxSamples = 65536;

namespace gpar {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHECK(x)                                                                    \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      throw ::gpar::Error(e_ == hipErrorOutOfMemory ? GPAR_ERR_OOM : GPAR_ERR_HIP,     \
                          std::string(#x) + ": " + hipGetErrorString(e_));             \
  } while (0)

#define ARGCHECK(c, msg)                                     \
  do {                                                       \
    if (!(c)) throw ::gpar::Error(GPAR_ERR_ARG, (msg));      \
  } while (0)

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(GPAR_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// RAII timing scope: records HIP events around the enclosed launches on the ctx stream.
// work: the algorithmic work of the enclosed launches (gpar_ctx_kernel_work).
struct Timed {
  gpar_ctx* c;
  const char* name;
  hipEvent_t e1 = nullptr;
  Timed(gpar_ctx* c_, const char* n, double work = 0.0) : c(c_), name(n) {
    if (!c->profiling) return;
    hipEvent_t e0;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, c->stream);
    c->stats[name].pending.push_back({e0, e1, work});
  }
  ~Timed() {
    if (e1) (void)hipEventRecord(e1, c->stream);
  }
};
void flush_stats(gpar_ctx* c);

inline bool is_cache_buf(const std::string& name) { return name.rfind("distcache", 0) == 0; }
void sync_all(gpar_ctx* c);
int64_t release_dist_cache(gpar_ctx* c, int64_t bytes = INT64_MAX);
void* ws_bytes(gpar_ctx* c, const std::string& name, size_t bytes);

template <class T>
inline T* ws(gpar_ctx* c, const std::string& name, size_t count) {
  return reinterpret_cast<T*>(ws_bytes(c, name, count * sizeof(T)));
}

template <class T>
inline void h2d(gpar_ctx* c, T* dst, const T* src, size_t count) {
  if (!count) return;
  const size_t bytes = count * sizeof(T);
  if (c->staging) {   // through the pinned arena: never waits for the stream
    gpar_ctx::Staging& s = *c->staging;
    const size_t off = (s.used + 255) & ~(size_t)255;
    if (off + bytes > s.cap) throw Error(GPAR_ERR_STATE, "upload staging arena exhausted");
    std::memcpy(s.host + off, src, bytes);
    s.used = off + bytes;
    HIPCHECK(hipMemcpyAsync(dst, s.host + off, bytes, hipMemcpyHostToDevice, c->stream));
    return;
  }
  HIPCHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
}
template <class T>
inline void d2h(gpar_ctx* c, T* dst, const T* src, size_t count) {
  if (count) HIPCHECK(hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyDeviceToHost, c->stream));
}
inline void sync(gpar_ctx* c) { HIPCHECK(hipStreamSynchronize(c->stream)); }
void h2d_rows(gpar_ctx* c, double* dst, const double* src, int64_t ld, int64_t width,
                     int64_t rows);

// Route the launches of a scope to another stream (all helpers launch on c->stream).
struct OnStream {
  gpar_ctx* c;
  hipStream_t saved;
  OnStream(gpar_ctx* c_, hipStream_t s) : c(c_), saved(c_->stream) { c->stream = s; }
  ~OnStream() { c->stream = saved; }
};

constexpr int kChunk = 256;   // time-chunk length of the Kalman sweeps (power of two, multiple of 16)
static_assert(kChunk == 256, "vec_fix runs one 256-thread block per chunk");
constexpr int kSStride = 4;   // chunk state vectors padded to 4 doubles (device_common.hpp)
constexpr int64_t kFusedMaxD = 64;   // widest input the fused Kfu + whitening kernels take
constexpr int64_t kPipeMaxBetaBytes = (int64_t)8 << 30;   // second beta buffer of the pipelined fit
// default gpar_ctx_set_cu_split width: 8 of every XCD's 32 CUs whiten beside the Gram (north job
// 20.66 -> 19.69 s per job in same-box pairs; 4 starves the whitening: 28.4 s)
constexpr int kDefaultCuSplit = 8;
// the default split applies to batched fits whose Gram is big enough to amortise it: N Mp^2 >= 1e11
// (north, N = 1e6, M = 512: 2.6e11; the N = 1e5 configs measured slower split: dtc 389 vs 297 ms
// per job, eeg 3.09 vs 3.07 s)
constexpr double kSplitMinWork = 1e11;
inline bool split_active(const gpar_ctx* c, int64_t n, int64_t mp) {
  return c->split_w > 0 && c->lanes == 1 &&
         (c->split_forced || (double)n * (double)mp * (double)mp >= kSplitMinWork);
}

inline int sde_dim(int kind) {
  if (kind == GPAR_MATERN12) return 1;
  if (kind == GPAR_MATERN32) return 2;
  if (kind == GPAR_MATERN52) return 3;
  throw Error(GPAR_ERR_UNSUPPORTED, "time kernel has no finite state-space form (EQ)");
}

inline int64_t round_up(int64_t x, int64_t q) { return ((x + q - 1) / q) * q; }
void run_carry(gpar_ctx* c, int sdim, const double* phi, int64_t phistride,
                      const double* send, double* cin, int64_t sstride, int64_t nch, int64_t mc,
                      int64_t ncols, int nchains, const std::string& tag, bool rev = false);

// --------------------------------------------------------------------------- problems on device
struct DevProblem {
  int64_t n, m, d, mp, mc, nch;
  const double *t, *v, *z, *y;
  const double* t_user;  // caller's pointer (grouping key)
  const double* zc;      // centres of the pseudo-input column groups (MFMA whitening), per problem
  int64_t ldv, ldz;
  int ok, tk, sdim, kuu_noise, qu_noise;
  // distances (n x mp, ld mp), theta-independent: computed once per fit when the distance cache
  // holds this output (fit_impl), else null.  Squared for EQ, r = |v_k - z_c| for the Matern
  // kernels (d2_is_r), so their square root is taken once per fit, not per evaluation
  const double* d2 = nullptr;
  bool d2_is_r = false;
  int cache_slot = -1;   // its gpar_ctx::cache_valid entry (an OOM eviction clears it)
};

// The cached distances of p if they are still resident, else null (fused kernel).
inline const double* cached_d2(const gpar_ctx* c, const DevProblem& p) {
  if (!p.d2 || p.cache_slot < 0 || p.cache_slot >= (int)c->cache_valid.size()) return nullptr;
  return c->cache_valid[p.cache_slot] ? p.d2 : nullptr;
}
bool shares_grid(const std::vector<DevProblem>& P);
bool fit_pipelined(const gpar_ctx* c, const std::vector<DevProblem>& P, bool fix_beta = false);
void check_sorted_host(const double* t, int64_t n);
void check_problem(const gpar_problem& p);
void check_batch(const gpar_problem* probs, int nprob);
DevProblem prepare_problem(gpar_ctx* c, const gpar_problem& p, int idx);
// prepare_problem for every problem of a batch; host inputs several problems share (t, the v base)
// are uploaded once (upload_shared_block)
std::vector<DevProblem> prepare_batch(gpar_ctx* c, const gpar_problem* probs, int nprob);
std::pair<const double*, int64_t> upload_shared_block(gpar_ctx* c, const std::string& name,
                                                      const double* src, int64_t ld, int64_t width,
                                                      int64_t rows);

struct Theta {
  double l_t, sv_t, l_o, sv_o, sigma;
};

// --------------------------------------------------------------------------- gains
struct GainsOut {
  double *rec, *g, *phi, *logs, *pf;
  int64_t recstride, gstride, phistride;
  // compact records {K, rs} (CRec): the whitening recomputes A_k from t (whiten_kfu_any)
  bool compact = false;
  const double* t = nullptr;
};
// The gains of `nchains` chains sharing t: uploads and workspace (plan_gains), launched over any
// chain ranges on any streams (GainsPlan::launch) -- the split fit launches them group by group on
// the whitening stream ahead of the whitenings that read them.
struct GainsPlan {
  gpar_ctx* c = nullptr;
  int sdim = 0, nchains = 0;
  const double* t = nullptr;
  int64_t n = 0, nch = 0;
  int64_t nchs = 0;   // per-chunk output slots per chain (nch; moments: 256 ceil(nch / 256))
  const double* noise = nullptr;
  ChainParamsHost* dcps = nullptr;
  double *agg = nullptr, *pst = nullptr;
  GainsOut o{};
  const double** dys = nullptr;
  bool ys_aligned16 = false;   // every ys[i] 16-byte aligned (the fast gains path's LDS-DMA)
  double *alpha_loc = nullptr, *asend = nullptr;
  double* moments = nullptr;   // chains_logpdf: per-chunk data moments instead of records
  void launch(hipStream_t st, int first, int count) const;
};
GainsPlan plan_gains(gpar_ctx* c, int sdim, const double* t, int64_t n,
                     const std::vector<ChainParamsHost>& cps, const double* noise, bool want_pf,
                     const std::string& tag, const std::vector<const double*>* ys = nullptr,
                     double* alpha_loc = nullptr, double* asend = nullptr, bool compact = false,
                     double* moments = nullptr);
GainsOut run_gains(gpar_ctx* c, int sdim, const double* t, int64_t n,
                          const std::vector<ChainParamsHost>& cps, const double* noise,
                          bool want_pf, const std::string& tag,
                          const std::vector<const double*>* ys = nullptr,
                          double* alpha_loc = nullptr, double* asend = nullptr,
                          bool compact = false);
// gi: the output's gains (compact records: the whitening goes through whiten_kfu_d2x2, the
// distances of an uncached output through a separate pass)
// d2_in_beta: the caller already wrote the distances into beta (a separately timed pass)
void whiten_kfu_any(gpar_ctx* c, const DevProblem& p, const GainsOut& gi, const double* v,
                           int64_t ldv, int64_t n, int64_t nch, const Theta& th, double* beta,
                           int64_t ldb, double* send, double* hsum, bool d2_in_beta = false);

// --------------------------------------------------------------------------- Gram stage
struct GramOut {
  double *G, *r, *a2part, *logs;  // per problem
  int64_t ldg, npart;
};

// Workspace of one Gram-stage buffer (two when outputs are pipelined or laned): beta (n + 16 rows,
// the Gram's LDS-DMA reads whole 16-row K-steps), alpha (outputs whose gains are not shared), the
// chunk states and the Gram's chunk-correction inputs.
struct StageBufs {
  int idx;   // 0 / 1: workspace names, carry tags
  double *beta, *alpha, *send, *cin, *hsum, *qv;
};
StageBufs stage_bufs(gpar_ctx* c, int l, int64_t n, int64_t mpmax);

// One output-evaluation in the Gram stage: the problem at hyperparameters th with its gains;
// alpha = L_Sigma^-1 y (asend: its chunk end states from the batched gains pass, which filtered
// alpha_loc already; null: alpha is whitened in stage_post into alpha); where G / r / the
// alpha^2 partials go.  group / last: the round-overlapping fit's bookkeeping.
struct StageJob {
  const DevProblem* p = nullptr;
  const Theta* th = nullptr;
  GainsOut gi{};
  double* alpha = nullptr;
  const double* asend = nullptr;
  double *G = nullptr, *r = nullptr, *a2part = nullptr;
  int64_t ldg = 0;
  int group = -1;
  bool last = false;
};
void stage_whiten(gpar_ctx* c, const StageJob& j, const StageBufs& b);
void stage_post(gpar_ctx* c, const StageJob& j, const StageBufs& b, bool fix_beta);
void stage_gram(gpar_ctx* c, const StageJob& j, const StageBufs& b, bool fix_beta,
                       bool one_per_cu, const std::string& part_sfx, hipStream_t side, int cus,
                       hipStream_t st_w = nullptr, hipEvent_t ev_w = nullptr, int w_frac32 = 0,
                       int dg_rows_w = 0);
void reserve_gram_parts(gpar_ctx* c, const std::vector<DevProblem>& P, int nlanes);

// The CU-split pipeline: whitening + short chain of job k on w CUs of every XCD (s_w),
// concurrently with job k-1's Gram on the other 32 - w (s_g, its co-running correction on s_g2).
// Jobs are numbered across push() calls, so a caller can keep feeding it (the round-overlapping
// fit does, across Nelder-Mead rounds): beta buffer k & 1; W(k) waits for G(k-2) (same buffers),
// G(k) for P(k), and a w/32 share of G(k)'s DG items runs on s_w after P(k+1) -- both sides then
// end together -- once G(k-1)'s reduction is done (the partial slots are reused).
struct SplitPipe {
  gpar_ctx* c;
  StageBufs buf[2];
  int gcus;
  int64_t k = 0;              // jobs whitened so far
  bool has_pending = false;   // job k - 1 whitened, its Gram not yet issued
  StageJob pending;
  std::function<void(const StageJob&, int64_t)> on_gram;   // right after job k's Gram is issued

  SplitPipe(gpar_ctx* c_, int64_t n, int64_t mpmax)
      : c(c_), gcus(8 * (32 - c_->split_w)) {
    buf[0] = stage_bufs(c, 0, n, mpmax);
    buf[1] = stage_bufs(c, 1, n, mpmax);
  }
  void start() {   // the split streams follow everything queued on the context stream so far
    HIPCHECK(hipEventRecord(c->ev_sp, c->stream));
    for (hipStream_t st : {c->s_w, c->s_g, c->s_g2}) HIPCHECK(hipStreamWaitEvent(st, c->ev_sp, 0));
  }
  // the short chains on the Gram CUs' second stream (gpar_ctx::post_gram; the round overlap's
  // whitening CUs also run the other group's dense tails and gains)
  bool post_gram = false;
  int dg_rows_w = 0;   // percent more rows per DG split on the whitening CUs (stage_gram)
  void push(const StageJob& j) {
    {
      OnStream on_(c, c->s_w);
      if (k >= 2) HIPCHECK(hipStreamWaitEvent(c->s_w, c->ev_gd[k & 1], 0));
      if (k == 0 && c->mark_h[0]) HIPCHECK(hipEventRecord(c->mark_h[0], c->s_w));
      stage_whiten(c, j, buf[k & 1]);
      if (k == 0 && c->mark_h[1]) HIPCHECK(hipEventRecord(c->mark_h[1], c->s_w));
      if (post_gram) {
        HIPCHECK(hipEventRecord(c->ev_wd, c->s_w));
      } else {
        stage_post(c, j, buf[k & 1], false);
        if (k == 0 && c->mark_h[2]) HIPCHECK(hipEventRecord(c->mark_h[2], c->s_w));
        HIPCHECK(hipEventRecord(c->ev_pc[k & 1], c->s_w));
      }
    }
    if (has_pending) issue_gram();
    if (post_gram) {
      // the short chain on the Gram CUs' second stream, behind the previous Gram's co-running
      // correction (issued just above), so the whitening side goes on with that Gram's DG share
      OnStream on_(c, c->s_g2);
      HIPCHECK(hipStreamWaitEvent(c->s_g2, c->ev_wd, 0));
      stage_post(c, j, buf[k & 1], false);
      if (k == 0 && c->mark_h[2]) HIPCHECK(hipEventRecord(c->mark_h[2], c->s_g2));
      HIPCHECK(hipEventRecord(c->ev_pc[k & 1], c->s_g2));
    }
    pending = j;
    has_pending = true;
    ++k;
  }
  void issue_gram() {
    const int64_t i = k - 1;
    {
      OnStream on_(c, c->s_g);
      HIPCHECK(hipStreamWaitEvent(c->s_g, c->ev_pc[i & 1], 0));
      if (i == 0 && c->mark_first) HIPCHECK(hipEventRecord(c->mark_first, c->s_g));
      if (i >= 1) HIPCHECK(hipStreamWaitEvent(c->s_w, c->ev_gd[(i - 1) & 1], 0));
      // the DG share reads alpha after vec_fix and the zeroed beta tail: P(i) on the whitening
      // stream orders it; on the Gram CUs' stream (post_gram) the share waits for it
      if (post_gram) HIPCHECK(hipStreamWaitEvent(c->s_w, c->ev_pc[i & 1], 0));
      stage_gram(c, pending, buf[i & 1], false, false, "", c->s_g2, gcus, c->s_w, c->ev_pw,
                 c->split_w, dg_rows_w);
      HIPCHECK(hipEventRecord(c->ev_gd[i & 1], c->s_g));
    }
    has_pending = false;
    if (on_gram) on_gram(pending, i);
  }
  void flush() {
    if (has_pending) issue_gram();
  }
  // stream st waits for every job issued so far (the last Gram follows every P, DG share and
  // correction)
  void join(hipStream_t st) {
    HIPCHECK(hipEventRecord(c->ev_sp, c->s_g));
    HIPCHECK(hipStreamWaitEvent(st, c->ev_sp, 0));
  }
};
GramOut run_gram_stage(gpar_ctx* c, const std::vector<DevProblem>& P,
                              const std::vector<Theta>& th, bool fix_beta = false);

// --------------------------------------------------------------------------- dense tail
struct DenseOut {
  double *Lu, *Llam;   // chol(Kuu [+ s2 I]) and chol(Lambda), row-major lower, ld x ld per problem
  double *Tu;          // L_u^-1 (full lower)
  double *Tl;          // L_lam^-1 (full lower; q(u) mode only, else null)
  double *Tdl;         // inverses of L_lam's 64 x 64 diagonal blocks
  int* status;         // 2 flags per problem
  int64_t ld;
  int nb;
};
DenseOut run_dense_pre(gpar_ctx* c, const std::vector<DevProblem>& P,
                              const std::vector<Theta>& th, int64_t ld, bool qu_mode);
void run_dense_post(gpar_ctx* c, const std::vector<DevProblem>& P, const GramOut& go,
                           const DenseOut& o);
DenseOut run_dense(gpar_ctx* c, const std::vector<DevProblem>& P,
                          const std::vector<Theta>& th, const GramOut& go, bool qu_mode);
Finish2JobHost finish_job(const DenseOut& dn, const GramOut& go, const DevProblem& p, int i,
                                 int64_t nch, double* out, double* me);
std::vector<Theta> thetas_from(const double* theta, int np);
// async (the unsplit round overlap, fit_overlapped_unsplit): the values and Cholesky status
// flags go to pinned host memory by async copies, `done` is recorded after them and eval_dtc
// returns without waiting (out / status_out untouched)
bool grouped_gram_eligible(gpar_ctx* c, const std::vector<DevProblem>& P);
struct EvalAsync {
  double* hout = nullptr;   // pinned, one value per problem
  int* hstat = nullptr;     // pinned, two flags per problem
  hipEvent_t done = nullptr;
};
void eval_dtc(gpar_ctx* c, const std::vector<DevProblem>& P, const std::vector<Theta>& th,
                     double* out, std::vector<int>& status_out, GramOut* gram_out = nullptr,
                     const EvalAsync* async = nullptr);


struct QuOut {
  double *me, *cov, *Ucol;
  const double *Tu, *Tl;   // L_u^-1, L_D^-1 (full lower, ld)
  int64_t ld;
  int nb;
};

// compute_q_u (gpar_scaled_inference.jl:141-196): Cuu without noise, D = L_u^-1 G L_u^-T + I,
// m_e = D^-1 L_u^-1 r, cov = inv(D) = L_D^-T L_D^-1, U_u = chol(Cuu).U.
// The Gram (beta^T beta, beta^T alpha; ld = mp) of one output at one theta, kept by the fit
// (fit_impl) for its best evaluation so that q(u) at the fitted theta need not recompute it.
struct GramCache {
  const double* G = nullptr;
  const double* r = nullptr;
};

// the fit's kept Grams (fit_impl, for gpar_fit_predict): output i's at its returned minimiser
struct FitKeep {
  std::vector<GramCache> gram;
  std::vector<char> valid;
};
QuOut run_q_u(gpar_ctx* c, const DevProblem& p, const Theta& th,
                     const GramCache* gc = nullptr);

// q(u) and the substitutions every prediction mode needs, for all outputs of a gpar_fit_predict
// call at once (a batched prediction used to run them per output: the blocked Cholesky, the
// finish, three trsm and a trsv, each a latency-bound launch of one small job, ~4 ms per output
// and a host sync each).  Per output i: Lu, LD (chol(Cuu), chol(D)), me = m_e, w = U_u^{-1} m_e
// = L_u^{-T} m_e, X1 = L_u^{-1}, Vm = L_D^{-1} L_u^{-1} (zero outside m x m), and for the MC / path
// modes cov = inv(D) = X^T X, X = L_D^{-1} (the same substitutions as run_q_u + predict_impl).
struct QuPre {
  const double *Lu, *LD, *me, *w, *X1, *Vm, *cov;
  int64_t ld;
  int nb;
};
// The part of one output's prediction that does not read the inference inputs, queued ahead on
// the side stream (gpar_posterior_prepare): the merged grid's gains and the adjoint's fix-up
// vectors h for given test times.  A slot is consumed by the matching gpar_posterior_predict.
// A slot is matched by the posterior's unique id (never by its address, which a later
// gpar_fit_posterior may reuse after gpar_posterior_destroy), the output index and the test times.
struct PredPrep {
  uint64_t post_id = 0;
  int out = -1;
  const double* ts = nullptr;
  int64_t n_star = 0;
  GainsOut g{};
  double* h = nullptr;
  bool valid = false;
};
std::vector<QuPre> run_q_u_batch(gpar_ctx* c, const std::vector<DevProblem>& P,
                                        const std::vector<Theta>& T, const FitKeep& keep,
                                        bool want_cov);
void chains_logpdf(gpar_ctx* c, const std::vector<const double*>& ys, int64_t n, const double* t,
                   int sdim, const double* theta, double* lml);


// --------------------------------------------------------------------------- posterior paths
// The path draws of a seed are decorrelated from its q(u) draws (gpar_path_normals exports them).
constexpr uint64_t kPathSeedXor = 0x5851F42D4C957F2Dull;
inline uint64_t path_seed(uint64_t seed) { return seed ^ kPathSeedXor; }
void path_samples(gpar_ctx* c, int sdim, const GainsOut& g, const ChainParamsHost& cp,
                         const double* t, const double* noise, int64_t n, const double* ym,
                         const double* fx, int64_t ldfx, int S, uint64_t seed, double* F);
void predict_impl(gpar_ctx* c, const DevProblem& P, const Theta& th, int mem,
                         int64_t n_star, const double* t_star_in, const double* v_star_in,
                         int64_t ldvs, int mode, int samples, uint64_t seed, double* mean_out,
                         double* std_out, const GramCache* gc = nullptr, bool defer = false,
                         const QuPre* pre = nullptr, const PredPrep* prep = nullptr);
void chains_smooth(gpar_ctx* c, int nchains, int64_t n, const double* t, const double* y,
                          int64_t ldy, const double* noise, int sdim,
                          const std::vector<ChainParamsHost>& cps, double* mean, double* var,
                          int64_t ldo);
std::vector<ChainParamsHost> chain_params(const double* theta, int nchains);

inline double unpack(double p) { return std::exp(p) + 1e-3; }
void enter(gpar_ctx* c);
int fail(gpar_ctx* c, int code, const char* what);
int64_t fit_ws_estimate(const gpar_ctx* c, const std::vector<DevProblem>& P);
int64_t predict_ws_estimate(int64_t n, int64_t n_star, int64_t mp, int64_t d, int mode,
                                   int samples, bool fused);
std::vector<DevProblem> attach_dist_cache(gpar_ctx* c, const std::vector<DevProblem>& P,
                                                 int64_t later_bytes);
void fit_impl(gpar_ctx* ctx, const std::vector<DevProblem>& P0, const double* log_theta0,
                     const gpar_fit_options& o, double* theta_out, double* nlml_out,
                     int32_t* evals_out, FitKeep* keep, int64_t later_bytes = 0);

}  // namespace gpar


#define API_BEGIN(ctx)                                          \
  if (!(ctx)) return GPAR_ERR_STATE;                            \
  try {                                                         \
    enter(ctx);

#define API_END(ctx)                                            \
  }                                                             \
  catch (const gpar::Error& e) {                                \
    return fail((ctx), e.code, e.what());                       \
  }                                                             \
  catch (const std::exception& e) {                             \
    return fail((ctx), GPAR_ERR_HIP, e.what());                 \
  }                                                             \
  return GPAR_OK;
