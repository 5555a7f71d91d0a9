// gpar_host.cpp -- C-ABI (include/gpar_hip.h) of the MI355X GPAR hot path.
//
// Host orchestration only: argument checking, device workspace, kernel sequencing, the
// batched Nelder-Mead driver.  Every number is computed by the gfx950 kernels in
// k_lgssm.hip / k_gram.hip / k_dense.hip / k_predict.hip; there is no CPU fallback.
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
#include <optional>
#include <vector>

#include "launch.hpp"
#include "nelder_mead.hpp"

struct gpar_ctx {
  int device = 0;
  hipStream_t stream = nullptr;   // the stream every launch goes to (see OnStream)
  hipStream_t main = nullptr;     // the context's stream
  hipStream_t side = nullptr;     // second stream: alternate outputs of a batch run here
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_pw = nullptr, ev_pc[2] = {nullptr, nullptr};   // the fit's pipelined Gram stage
  bool pipeline = true;           // GPAR_PIPELINE=0 turns the pipelined Gram stage off (A/B)
  // gpar_ctx_set_cu_split(w): the pipelined fit's whitening runs on w CUs of every XCD and the
  // Gram (its co-running correction too) on the other 32 - w, concurrently (CU-masked streams)
  int split_w = 0, split_mask_w = 0;
  bool split_forced = false;      // set explicitly: no problem-size gate (split_active)
  bool split_dgw = true;          // a w/32 share of the DG items on the whitening CUs
  // s_d: the round-overlapping fit's dense tails, on the whitening CUs (fit_overlapped)
  hipStream_t s_w = nullptr, s_g = nullptr, s_g2 = nullptr, s_d = nullptr;
  hipEvent_t ev_gd[2] = {nullptr, nullptr}, ev_sp = nullptr;
  hipEvent_t ev_g0 = nullptr, ev_gr = nullptr;   // split round start: gains uploaded / the rest's gains done
  hipEvent_t ev_dn = nullptr;                    // split round start: the dense prefix follows the context stream
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
  Staging stage[2];
  Staging* staging = nullptr;
  bool overlap = true;            // gpar_ctx_set_fit_overlap (GPAR_OVERLAP=0 at creation): A/B
  // gpar_fit_predict's predictions alternate over two streams (GPAR_PREDICT_LANES=1: one)
  int predict_lanes = 2;
  bool predict_fused = true;      // GPAR_PREDICT_FUSED=0: predict_rows + gemm_nt (A/B)
  bool qu_batch = true;           // GPAR_QU_BATCH=0: gpar_fit_predict's q(u) per output (A/B)
  bool dense_early = true;        // GPAR_DENSE_EARLY=0: the whole dense tail after the round's Grams (A/B)
  int overlap_max = 16;           // GPAR_OVERLAP_MAX: largest call that takes the round overlap (kOverlapMaxOutputs; A/B)
  int overlap_b = 0;              // GPAR_OVERLAP_B: size of the overlap's second group (0: halves; A/B)
  bool split_head = true;         // GPAR_SPLIT_HEAD=0: the split round's first job on the whitening CUs, gains in one launch (A/B)
  std::string ws_suffix;          // appended to workspace names (a prediction lane's own buffers)
  hipEvent_t ev_grp[2] = {nullptr, nullptr};   // fit_overlapped: a group's values are in
  hipEvent_t ev_gn[2] = {nullptr, nullptr};    // fit_overlapped: a group's gains are done
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

static void check_launch(const char* what) {
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

static void flush_stats(gpar_ctx* c) {
  (void)hipStreamSynchronize(c->stream);
  for (auto& kv : c->stats) {
    for (auto& pr : kv.second.pending) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, pr.e0, pr.e1) == hipSuccess) {
        kv.second.ms += ms;
        kv.second.launches += 1;
        kv.second.work += pr.work;
      }
      (void)hipEventDestroy(pr.e0);
      (void)hipEventDestroy(pr.e1);
    }
    kv.second.pending.clear();
  }
}

static bool is_cache_buf(const std::string& name) { return name.rfind("distcache", 0) == 0; }

static void sync_all(gpar_ctx* c) {
  for (hipStream_t st : {c->main, c->side, c->s_w, c->s_g, c->s_g2, c->s_d})
    if (st) HIPCHECK(hipStreamSynchronize(st));
}

// Free distance-cache buffers, the highest slots first, until at least `bytes` are released
// (INT64_MAX: all of them), once all queued work is done (nothing in flight can still read
// them), and mark those slots gone: whiten_kfu_any checks the slot before every launch.
// Returns the bytes freed.
static int64_t release_dist_cache(gpar_ctx* c, int64_t bytes = INT64_MAX) {
  int64_t freed = 0;
  bool synced = false;
  for (int s = (int)c->cache_valid.size() - 1; s >= 0 && freed < bytes; --s) {
    auto it = c->bufs.find("distcache" + std::to_string(s));
    if (it == c->bufs.end()) continue;
    if (!synced) sync_all(c);
    synced = true;
    if (it->second.p) HIPCHECK(hipFree(it->second.p));
    freed += (int64_t)it->second.bytes;
    c->bufs.erase(it);
    c->cache_valid[s] = 0;
  }
  return freed;
}

// Grow-only named workspace.  Out of memory: the distance cache is the one optional holder, so
// its slots are evicted (the last ones first, as many as the request needs) and the allocation
// retried (not for the cache's own buffers, which must not evict their siblings).
static void* ws_bytes(gpar_ctx* c, const std::string& name, size_t bytes) {
  if (bytes == 0) bytes = 16;
  const bool evict = !is_cache_buf(name);   // eviction erases cache entries (b below)
  auto& b = c->bufs[c->ws_suffix.empty() || !evict ? name : name + c->ws_suffix];
  if (b.bytes < bytes) {
    if (b.p) HIPCHECK(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    hipError_t e = hipMalloc(&b.p, bytes);
    while (e == hipErrorOutOfMemory && evict) {
      (void)hipGetLastError();
      b.p = nullptr;
      if (release_dist_cache(c, (int64_t)bytes) == 0) break;
      ++c->cache_evictions;
      e = hipMalloc(&b.p, bytes);
    }
    if (e != hipSuccess) {
      (void)hipGetLastError();
      b.p = nullptr;
      throw Error(e == hipErrorOutOfMemory ? GPAR_ERR_OOM : GPAR_ERR_HIP,
                  "hipMalloc(" + name + ", " + std::to_string(bytes) + " B): " + hipGetErrorString(e));
    }
    b.bytes = bytes;
  }
  return b.p;
}

template <class T>
static T* ws(gpar_ctx* c, const std::string& name, size_t count) {
  return reinterpret_cast<T*>(ws_bytes(c, name, count * sizeof(T)));
}

template <class T>
static void h2d(gpar_ctx* c, T* dst, const T* src, size_t count) {
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
static void d2h(gpar_ctx* c, T* dst, const T* src, size_t count) {
  if (count) HIPCHECK(hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyDeviceToHost, c->stream));
}
static void sync(gpar_ctx* c) { HIPCHECK(hipStreamSynchronize(c->stream)); }
// rows x width doubles from a host matrix with leading dimension ld into a packed device matrix:
// one linear copy when the rows are already packed (a pitched copy from pageable memory goes row
// by row: 10^6 rows of a few doubles took seconds)
static void h2d_rows(gpar_ctx* c, double* dst, const double* src, int64_t ld, int64_t width,
                     int64_t rows) {
  if (ld == width)
    h2d(c, dst, src, (size_t)rows * width);
  else
    HIPCHECK(hipMemcpy2DAsync(dst, width * sizeof(double), src, ld * sizeof(double),
                              width * sizeof(double), rows, hipMemcpyHostToDevice, c->stream));
}

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
static bool split_active(const gpar_ctx* c, int64_t n, int64_t mp) {
  return c->split_w > 0 && c->lanes == 1 &&
         (c->split_forced || (double)n * (double)mp * (double)mp >= kSplitMinWork);
}

static int sde_dim(int kind) {
  if (kind == GPAR_MATERN12) return 1;
  if (kind == GPAR_MATERN32) return 2;
  if (kind == GPAR_MATERN52) return 3;
  throw Error(GPAR_ERR_UNSUPPORTED, "time kernel has no finite state-space form (EQ)");
}

static int64_t round_up(int64_t x, int64_t q) { return ((x + q - 1) / q) * q; }

// Two-level carry over chunks (k_lgssm.hip launch_carry) with context workspace.
static void run_carry(gpar_ctx* c, int sdim, const double* phi, int64_t phistride,
                      const double* send, double* cin, int64_t sstride, int64_t nch, int64_t mc,
                      int64_t ncols, int nchains, const std::string& tag, bool rev = false) {
  const int gs = carry_group_size(nch);
  const int64_t ng = (nch + gs - 1) / gs;
  double* gend = ws<double>(c, tag + "_gend", (size_t)nchains * ng * mc * 4);
  double* gin = ws<double>(c, tag + "_gin", (size_t)nchains * ng * mc * 4);
  double* psi = ws<double>(c, tag + "_psi", (size_t)nchains * ng * sdim * sdim);
  launch_carry(c->stream, sdim, phi, phistride, send, cin, sstride, nch, mc, ncols, nchains, gend,
               gin, psi, rev);
}

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
static const double* cached_d2(const gpar_ctx* c, const DevProblem& p) {
  if (!p.d2 || p.cache_slot < 0 || p.cache_slot >= (int)c->cache_valid.size()) return nullptr;
  return c->cache_valid[p.cache_slot] ? p.d2 : nullptr;
}

// Every problem of the batch shares the time grid (same caller pointer, n and SDE order): one
// batched gains launch serves them all.
static bool shares_grid(const std::vector<DevProblem>& P) {
  for (auto& p : P)
    if (p.t_user != P[0].t_user || p.n != P[0].n || p.sdim != P[0].sdim) return false;
  return true;
}

// The one-lane pipelined Gram stage (run_gram_stage): several outputs on one grid, two beta
// buffers (only when a second beta fits comfortably: the north job's 4.1 GB, not the N = 1e7,
// M = 1024 stress config's 82 GB).  The CU split and the all-D distance cache apply only on top of it.
static bool fit_pipelined(const gpar_ctx* c, const std::vector<DevProblem>& P, bool fix_beta = false) {
  int64_t mpmax = 0;
  for (auto& p : P) mpmax = std::max(mpmax, p.mp);
  const int64_t beta_bytes = (P[0].n + 16) * mpmax * (int64_t)sizeof(double);
  return P.size() > 1 && !fix_beta && c->lanes == 1 && shares_grid(P) && c->pipeline &&
         beta_bytes <= kPipeMaxBetaBytes;
}

static void check_sorted_host(const double* t, int64_t n) {
  for (int64_t k = 1; k < n; ++k)
    ARGCHECK(t[k] >= t[k - 1], "time locations must be ascending (dtc.jl:102 does not sort)");
}

// Host-side argument checks of one problem (no device work).
static void check_problem(const gpar_problem& p) {
  ARGCHECK(p.n >= 1 && p.m >= 1, "n and m must be >= 1");
  ARGCHECK(p.d >= 1, "d must be >= 1 (use the LGSSM entry points for time-only outputs)");
  ARGCHECK(p.ldv >= p.d && p.ldz >= p.d, "ldv/ldz must be >= d");
  ARGCHECK(p.t && p.v && p.z && p.y, "null input pointer");
  ARGCHECK(p.out_kernel >= 0 && p.out_kernel <= 3, "bad out_kernel");
  ARGCHECK(p.time_kernel >= 0 && p.time_kernel <= 3, "bad time_kernel");
  ARGCHECK(p.mem == GPAR_MEM_HOST || p.mem == GPAR_MEM_DEVICE, "bad mem");
  if (p.m > 2048) throw Error(GPAR_ERR_UNSUPPORTED, "m > 2048 not supported");
  (void)sde_dim(p.time_kernel);
  if (p.mem == GPAR_MEM_HOST) check_sorted_host(p.t, p.n);
}

// Every problem of a batched call is validated before the first launch: a failure part-way
// through the launch loop would leave kernels reading caller memory the caller then frees.
static void check_batch(const gpar_problem* probs, int nprob) {
  ARGCHECK(probs && nprob >= 1, "null argument");
  for (int i = 0; i < nprob; ++i) {
    check_problem(probs[i]);
    ARGCHECK(probs[i].n == probs[0].n, "all problems of one call must share n");
    ARGCHECK(probs[i].mem == probs[0].mem, "all problems of one call must share one memory space");
  }
}

static DevProblem prepare_problem(gpar_ctx* c, const gpar_problem& p, int idx) {
  check_problem(p);
  DevProblem d{};
  d.n = p.n;
  d.m = p.m;
  d.d = p.d;
  d.mp = round_up(p.m, kGramTile);
  d.mc = d.mp + 1;
  d.nch = (p.n + kChunk - 1) / kChunk;
  d.ok = p.out_kernel;
  d.tk = p.time_kernel;
  d.sdim = sde_dim(p.time_kernel);
  d.kuu_noise = p.kuu_noise;
  d.qu_noise = p.qu_kuu_noise;
  d.t_user = p.t;
  // Z is theta-independent: its group centres are computed once per prepared problem
  double* zc = ws<double>(c, "prob" + std::to_string(idx) + "_zc",
                          (size_t)((d.mp + 255) / 256) * zc_stride((int)d.d));
  d.zc = zc;
  auto centres = [&]() {
    if (d.ok == GPAR_MATERN12) return;
    if (d.d <= kFusedMaxD) launch_zcenter(c->stream, d.z, d.ldz, (int)d.d, d.m, d.mp, zc);
    else launch_zcenter_wide(c->stream, d.z, d.ldz, (int)d.d, d.m, d.mp, zc);
  };
  if (p.mem == GPAR_MEM_DEVICE) {
    d.t = p.t; d.v = p.v; d.z = p.z; d.y = p.y;
    d.ldv = p.ldv; d.ldz = p.ldz;
    centres();
    return d;
  }
  const std::string k = "prob" + std::to_string(idx);
  double* t = ws<double>(c, k + "_t", p.n);
  double* v = ws<double>(c, k + "_v", (size_t)p.n * p.d);
  double* z = ws<double>(c, k + "_z", (size_t)p.m * p.d);
  double* y = ws<double>(c, k + "_y", p.n);
  h2d(c, t, p.t, p.n);
  h2d(c, y, p.y, p.n);
  h2d_rows(c, v, p.v, p.ldv, p.d, p.n);
  h2d_rows(c, z, p.z, p.ldz, p.d, p.m);
  d.t = t; d.v = v; d.z = z; d.y = y;
  d.ldv = p.d; d.ldz = p.d;
  centres();
  return d;
}

struct Theta {
  double l_t, sv_t, l_o, sv_o, sigma;
};

// --------------------------------------------------------------------------- gains
struct GainsOut {
  double *rec, *g, *phi, *logs, *pf;
  int64_t recstride, gstride, phistride;
};

// Data-independent per-step filter quantities for `nchains` chains sharing t (n steps).
// With ys (one device data vector per chain): the chains' alpha_loc / chunk end states are
// filtered inside the gains pass (alpha_loc: nchains x n, asend: nchains x nch x 4).
static GainsOut run_gains(gpar_ctx* c, int sdim, const double* t, int64_t n,
                          const std::vector<ChainParamsHost>& cps, const double* noise,
                          bool want_pf, const std::string& tag,
                          const std::vector<const double*>* ys = nullptr,
                          double* alpha_loc = nullptr, double* asend = nullptr,
                          hipStream_t st_rest = nullptr) {
  const int nchains = (int)cps.size();
  const int64_t nch = (n + kChunk - 1) / kChunk;
  const int rs = rec_size(sdim);
  const int d2 = sdim * sdim;
  ChainParamsHost* dcps = ws<ChainParamsHost>(c, tag + "_cps", nchains);
  h2d(c, dcps, cps.data(), nchains);
  double* agg = ws<double>(c, tag + "_agg", (size_t)nchains * nch * 3 * d2);
  double* pst = ws<double>(c, tag + "_pstart", (size_t)nchains * nch * d2);
  GainsOut o;
  o.recstride = n * rs;
  o.gstride = n * 4;
  o.phistride = nch * d2;
  o.rec = ws<double>(c, tag + "_rec", (size_t)nchains * n * rs);
  o.g = ws<double>(c, tag + "_g", (size_t)nchains * n * 4);
  o.phi = ws<double>(c, tag + "_phi", (size_t)nchains * nch * d2);
  o.logs = ws<double>(c, tag + "_logs", (size_t)nchains * nch);
  o.pf = want_pf ? ws<double>(c, tag + "_pf", (size_t)nchains * n * d2) : nullptr;
  const double** dys = nullptr;
  if (ys) {
    dys = ws<const double*>(c, tag + "_ys", nchains);
    h2d(c, dys, ys->data(), nchains);
  }
  // st_rest: chain 0 on c->stream, chains 1.. on st_rest (after the uploads above), which then
  // records c->ev_gr; the chains' arrays are strided per chain, so a range is a pointer offset
  const int n0 = (st_rest && nchains > 1) ? 1 : nchains;
  if (n0 < nchains) HIPCHECK(hipEventRecord(c->ev_g0, c->stream));
  {
    Timed tm_(c, "gains");
    launch_gains(c->stream, sdim, t, n, kChunk, nch, n0, dcps, noise, agg, pst, o.rec, o.g,
                 o.phi, o.logs, o.pf, dys, alpha_loc, asend);
  }
  if (n0 < nchains) {
    HIPCHECK(hipStreamWaitEvent(st_rest, c->ev_g0, 0));
    launch_gains(st_rest, sdim, t, n, kChunk, nch, nchains - n0, dcps + n0, noise,
                 agg + (size_t)n0 * nch * 3 * d2, pst + (size_t)n0 * nch * d2,
                 o.rec + (size_t)n0 * o.recstride, o.g + (size_t)n0 * o.gstride,
                 o.phi + (size_t)n0 * o.phistride, o.logs + (size_t)n0 * nch,
                 o.pf ? o.pf + (size_t)n0 * n * d2 : nullptr, dys ? dys + n0 : nullptr,
                 alpha_loc ? alpha_loc + (size_t)n0 * n : nullptr,
                 asend ? asend + (size_t)n0 * nch * kSStride : nullptr);
    HIPCHECK(hipEventRecord(c->ev_gr, st_rest));
  }
  check_launch("gains");
  return o;
}


// Kfu assembly + chunk-local whitening: fp64-MFMA Gram-form kernel for the smooth output
// kernels, direct-difference kernel for Matern-1/2 (kappa not smooth in d^2 at 0).
// Inputs wider than kFusedMaxD (the fused kernels keep a column's pseudo-input in registers):
// the squared distances are a separate MFMA (or direct-difference) pass into beta itself, which
// the whitening then reads and overwrites in place (k_dist.hip).
static void whiten_kfu_any(gpar_ctx* c, const DevProblem& p, const double* rec, const double* v,
                           int64_t ldv, int64_t n, int64_t nch, const Theta& th, double* beta,
                           int64_t ldb, double* send, const double* g, double* hsum) {
  const double s_o = th.sv_o * th.sv_o;
  const double* d2 = cached_d2(c, p);
  if (d2 && v == p.v) {   // the fit's training inputs, distances cached (fit_impl)
    launch_whiten_kfu_d2(c->stream, p.tk, p.ok, rec, d2, p.mp, p.m, p.mp, n, kChunk, nch,
                         1.0 / th.l_o, s_o, beta, ldb, send, p.mc, g, hsum, p.d2_is_r);
  } else if (p.d > kFusedMaxD) {
    launch_dist2(c->stream, p.ok, v, ldv, n, p.z, p.ldz, p.m, p.mp, (int)p.d, p.zc, beta, ldb);
    launch_whiten_kfu_d2(c->stream, p.tk, p.ok, rec, beta, ldb, p.m, p.mp, n, kChunk, nch,
                         1.0 / th.l_o, s_o, beta, ldb, send, p.mc, g, hsum);
  } else if (p.ok == GPAR_MATERN12) {
    launch_whiten_kfu(c->stream, p.tk, p.ok, rec, v, ldv, (int)p.d, p.z, p.ldz, p.m, p.mp, n,
                      kChunk, nch, 1.0 / th.l_o, s_o, beta, ldb, send, p.mc, g, hsum);
  } else {
    launch_whiten_kfu_mfma(c->stream, p.tk, p.ok, rec, v, ldv, (int)p.d, p.z, p.ldz, p.zc, p.m, p.mp,
                           n, kChunk, nch, 1.0 / th.l_o, s_o, beta, ldb, send, p.mc, g, hsum);
  }
}

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

static StageBufs stage_bufs(gpar_ctx* c, int l, int64_t n, int64_t mpmax) {
  const int64_t nch = (n + kChunk - 1) / kChunk;
  const std::string sfx = l ? "_1" : "";
  StageBufs b;
  b.idx = l;
  b.beta = ws<double>(c, "beta" + sfx, (size_t)(n + 16) * mpmax);
  b.alpha = ws<double>(c, "alpha" + sfx, (size_t)n);
  b.send = ws<double>(c, "send" + sfx, (size_t)nch * (mpmax + 1) * 4);
  b.cin = ws<double>(c, "cin" + sfx, (size_t)nch * (mpmax + 1) * 4);
  b.hsum = ws<double>(c, "hsum" + sfx, (size_t)nch * (mpmax + 1) * 4);
  b.qv = ws<double>(c, "qv" + sfx, (size_t)nch * 4);
  return b;
}

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

// Kfu assembly + chunk-local whitening of j's output into b.beta, on c->stream.
static void stage_whiten(gpar_ctx* c, const StageJob& j, const StageBufs& b) {
  const DevProblem& p = *j.p;
  // algorithmic HBM bytes: the inputs (V, or the cached distances), the gains records and
  // fix-up rows (16 + 4 doubles per step), beta written (m columns)
  const double in_cols = cached_d2(c, p) ? (double)p.m : (double)p.d;
  Timed tm_(c, "whiten", 8.0 * (double)p.n * (in_cols + (double)p.m + 20.0));
  whiten_kfu_any(c, p, j.gi.rec, p.v, p.ldv, p.n, p.nch, *j.th, b.beta, p.mp, b.send, j.gi.g,
                 b.hsum);
  check_launch("whiten_kfu");
}

// The short chain between a whitening and its Gram, on c->stream: alpha's chunk end states, the
// chunk carry, vec_fix (alpha fix-up, the Gram's correction E_j = H_j + W_j C_j / 2 and q_j), the
// beta tail (and the beta fix-up pass when fix_beta).
static void stage_post(gpar_ctx* c, const StageJob& j, const StageBufs& b, bool fix_beta) {
  const DevProblem& p = *j.p;
  const int64_t n = p.n, nch = p.nch;
  if (j.asend) {   // alpha's chunk end states -> column mp of the carry input
    HIPCHECK(hipMemcpy2DAsync(b.send + (size_t)p.mp * kSStride, (size_t)p.mc * kSStride * sizeof(double),
                              j.asend, kSStride * sizeof(double), kSStride * sizeof(double), nch,
                              hipMemcpyDeviceToDevice, c->stream));
  } else {
    launch_whiten_vec(c->stream, p.sdim, j.gi.rec, 0, p.y, 0, n, kChunk, nch, 1, j.alpha, 0, b.send,
                      0, p.mc, p.mp);
  }
  check_launch("whiten_vec");
  run_carry(c, p.sdim, j.gi.phi, 0, b.send, b.cin, 0, nch, p.mc, p.mc, 1,
            b.idx ? "fitc_1" : "fitc");
  check_launch("carry");
  launch_vec_fix(c->stream, p.sdim, j.alpha, 0, j.gi.g, 0, b.cin, 0, p.mc, p.mp, n, kChunk, 1,
                 j.a2part, fix_beta ? nullptr : b.hsum, p.mp, b.qv);
  check_launch("vec_fix");
  if (fix_beta) {
    launch_beta_fix(c->stream, p.sdim, b.beta, p.mp, n, j.gi.g, b.cin, p.mc, kChunk);
    check_launch("beta_fix");
  }
  HIPCHECK(hipMemsetAsync(b.beta + (size_t)n * p.mp, 0, (size_t)16 * p.mp * sizeof(double), c->stream));
}

// G = beta^T beta, r = beta^T alpha of j on c->stream, which may use `cus` CUs; side: the stream of
// the co-running chunk correction; st_w: the first w_frac32 / 32 of the DG kernel's work items run
// there (ev_w joins them).  one_per_cu: the two-lane plan (one Gram workgroup per CU).
static void stage_gram(gpar_ctx* c, const StageJob& j, const StageBufs& b, bool fix_beta,
                       bool one_per_cu, const std::string& part_sfx, hipStream_t side, int cus,
                       hipStream_t st_w = nullptr, hipEvent_t ev_w = nullptr, int w_frac32 = 0) {
  const DevProblem& p = *j.p;
  const GramPlan plan = gram_plan(p.n, p.mp, one_per_cu, cus, st_w ? 256 : cus);
  const int w_items = st_w ? plan.ndg * plan.sdg * w_frac32 / 32 : 0;
  double* part = ws<double>(c, "gram_part" + part_sfx, (size_t)plan.part_doubles);
  double* rpart = ws<double>(c, "gram_rpart" + part_sfx, (size_t)plan.rpart_doubles);
  {
    Timed tm_(c, "gram", (double)p.n * (double)p.m * (double)(p.m + 1));   // flops of beta^T beta
    launch_gram(c->stream, p.sdim, plan, b.beta, p.mp, p.n, fix_beta ? nullptr : b.hsum, b.cin,
                b.qv, p.mc, kChunk, j.alpha, part, rpart, j.G, j.ldg, j.r, side, c->ev_fork,
                c->ev_join, st_w, ev_w, w_items);
  }
  check_launch("gram");
}

// The Gram partials, sized once for the largest plan any problem of the batch can take: growing
// them mid-batch would free a buffer another stream's kernels may still be using.
static void reserve_gram_parts(gpar_ctx* c, const std::vector<DevProblem>& P, int nlanes) {
  int64_t pd = 0, rd = 0;
  for (const auto& p : P)
    for (int cus : {256, 8 * (32 - c->split_w)})
      for (int dgc : {cus, 256}) {
        if (cus <= 0) continue;
        const GramPlan pl = gram_plan(p.n, p.mp, nlanes > 1, cus, dgc);
        pd = std::max(pd, pl.part_doubles);
        rd = std::max(rd, pl.rpart_doubles);
      }
  for (int l = 0; l < nlanes; ++l) {
    const std::string sfx = l ? "_1" : "";
    (void)ws<double>(c, "gram_part" + sfx, (size_t)pd);
    (void)ws<double>(c, "gram_rpart" + sfx, (size_t)rd);
  }
}

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
  bool head = false;           // job 0 runs whole-chip on the caller's stream (split_head)
  void push(const StageJob& j) {
    if (k == 0 && head) {
      // nothing runs on the Gram CUs before the first Gram: the first whitening and its short
      // chain take the whole chip (the caller's unmasked stream, which the split streams follow
      // since start()); the whitening side continues after them
      stage_whiten(c, j, buf[0]);
      stage_post(c, j, buf[0], false);
      HIPCHECK(hipEventRecord(c->ev_pc[0], c->stream));
      HIPCHECK(hipStreamWaitEvent(c->s_w, c->ev_pc[0], 0));
    } else {
      OnStream on_(c, c->s_w);
      if (k >= 2) HIPCHECK(hipStreamWaitEvent(c->s_w, c->ev_gd[k & 1], 0));
      stage_whiten(c, j, buf[k & 1]);
      stage_post(c, j, buf[k & 1], false);
      HIPCHECK(hipEventRecord(c->ev_pc[k & 1], c->s_w));
    }
    if (has_pending) issue_gram();
    pending = j;
    has_pending = true;
    ++k;
  }
  void issue_gram() {
    const int64_t i = k - 1;
    {
      OnStream on_(c, c->s_g);
      HIPCHECK(hipStreamWaitEvent(c->s_g, c->ev_pc[i & 1], 0));
      if (c->split_dgw) {
        if (i >= 1) HIPCHECK(hipStreamWaitEvent(c->s_w, c->ev_gd[(i - 1) & 1], 0));
        stage_gram(c, pending, buf[i & 1], false, false, "", c->s_g2, gcus, c->s_w, c->ev_pw,
                   c->split_w);
      } else {
        stage_gram(c, pending, buf[i & 1], false, false, "", c->s_g2, gcus);
      }
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

// For every problem: G = beta^T beta, r = beta^T alpha, sum alpha^2 partials, sum log S
// partials, at hyperparameters th.
// fix_beta = false (the objective): the Gram streams the chunk-local beta and adds the chunk
//   correction sum_j E_j C_j^T + C_j E_j^T (k_gram.hip) -- no extra pass over beta.
// fix_beta = true (q(u), the (dtc, A) entry point): beta is fixed up in place first and the
//   Gram is a plain beta^T beta.  One extra pass over beta, but G carries the rounding of the
//   true beta only: q(u) factors the noise-free Cuu (cond >= 1e7), which amplifies the ~10x
//   larger rounding of the correction form (emulated: 7e-15 vs 7e-16 of max |G|).
static GramOut run_gram_stage(gpar_ctx* c, const std::vector<DevProblem>& P,
                              const std::vector<Theta>& th, bool fix_beta = false) {
  const int np = (int)P.size();
  int64_t mpmax = 0, n = P[0].n;
  for (auto& p : P) mpmax = std::max(mpmax, p.mp);
  const int64_t nch = (n + kChunk - 1) / kChunk;
  const int64_t npart = vec_fix_blocks(n);
  GramOut o;
  o.ldg = mpmax;
  o.npart = npart;
  o.G = ws<double>(c, "G", (size_t)np * mpmax * mpmax);
  o.r = ws<double>(c, "r", (size_t)np * mpmax);
  o.a2part = ws<double>(c, "a2part", (size_t)np * npart);
  o.logs = ws<double>(c, "logs_all", (size_t)np * nch);
  // problems narrower than the batch's widest: their G / r padding must read as zero in the
  // dense tail (the Gram writes only the mp x mp corner)
  for (int i = 0; i < np; ++i)
    if (P[i].mp != mpmax) {
      HIPCHECK(hipMemsetAsync(o.G + (size_t)i * mpmax * mpmax, 0, (size_t)mpmax * mpmax * sizeof(double), c->stream));
      HIPCHECK(hipMemsetAsync(o.r + (size_t)i * mpmax, 0, (size_t)mpmax * sizeof(double), c->stream));
    }

  // group problems sharing (t, n, time kernel) into one batched gains launch
  const bool shared = shares_grid(P);
  const bool pipe = fit_pipelined(c, P, fix_beta);
  const bool split_pipe = pipe && split_active(c, n, mpmax);
  const bool split_head = split_pipe && c->split_head && shared && np > 1;
  const double* logs_src = nullptr;
  std::vector<GainsOut> gains(np);
  // shared gains: every output's alpha_loc (y filtered from zero per chunk) comes out of the
  // gains pass itself; only its chunk end states are copied into the carry's alpha column
  double* alpha_all = nullptr;
  double* asend_all = nullptr;
  if (shared) {
    std::vector<ChainParamsHost> cps(np);
    std::vector<const double*> ys(np);
    for (int i = 0; i < np; ++i) {
      cps[i] = {1.0 / th[i].l_t, th[i].l_t, th[i].sv_t * th[i].sv_t, th[i].sigma * th[i].sigma};
      ys[i] = P[i].y;
    }
    alpha_all = ws<double>(c, "alpha_all", (size_t)np * n);
    asend_all = ws<double>(c, "asend_all", (size_t)np * nch * kSStride);
    // split pipeline: the first output's gains alone on the context stream, so its whitening can
    // start, the others' on s_g2 (Gram CUs, idle until the first Gram's correction)
    GainsOut g = run_gains(c, P[0].sdim, P[0].t, n, cps, nullptr, false, "fit", &ys, alpha_all,
                           asend_all, split_head ? c->s_g2 : nullptr);
    for (int i = 0; i < np; ++i) {
      gains[i] = g;
      gains[i].rec = g.rec + (size_t)i * g.recstride;
      gains[i].g = g.g + (size_t)i * g.gstride;
      gains[i].phi = g.phi + (size_t)i * g.phistride;
      gains[i].logs = g.logs + (size_t)i * nch;
    }
    if (!split_head)   // else after the pipeline (the other outputs' gains run on s_g2)
      HIPCHECK(hipMemcpyAsync(o.logs, g.logs, (size_t)np * nch * sizeof(double),
                              hipMemcpyDeviceToDevice, c->stream));
    logs_src = g.logs;
  }

  // Outputs alternate between the context stream and a side stream, each with its own
  // beta / alpha / carry workspace, so one output's (VALU-bound) whitening overlaps another's
  // (MFMA-bound) Gram.  Gains are shared: the side stream waits for them (fork event).
  const int nlanes = (np > 1 && !fix_beta && c->lanes > 1) ? 2 : 1;
  // One lane, pipelined (the batched fit): the big kernels stay in order on the context stream,
  // whitening(i + 1) issued ahead of Gram(i), and output i's short chain between them (alpha's end
  // states, the chunk carry, vec_fix, the beta tail) runs on the side stream beside a whitening
  // instead of on the critical path.  Two beta / carry buffers (fit_pipelined).
  reserve_gram_parts(c, P, nlanes);
  // the stage job of output i, its gains (per output unless shared) run on c->stream
  std::vector<StageJob> jobs(np);
  std::vector<double*> alpha_own(np, nullptr);
  auto job = [&](int i, const StageBufs& b) -> const StageJob& {
    StageJob& j = jobs[i];
    j.p = &P[i];
    j.th = &th[i];
    if (shared) {
      j.gi = gains[i];
      j.alpha = alpha_all + (size_t)i * n;
      j.asend = asend_all + (size_t)i * nch * kSStride;
    } else {
      std::vector<ChainParamsHost> cps(1);
      cps[0] = {1.0 / th[i].l_t, th[i].l_t, th[i].sv_t * th[i].sv_t, th[i].sigma * th[i].sigma};
      j.gi = run_gains(c, P[i].sdim, P[i].t, n, cps, nullptr, false, b.idx ? "fit1_1" : "fit1");
      HIPCHECK(hipMemcpyAsync(o.logs + (size_t)i * nch, j.gi.logs, nch * sizeof(double),
                              hipMemcpyDeviceToDevice, c->stream));
      j.alpha = b.alpha;
      j.asend = nullptr;
    }
    j.G = o.G + (size_t)i * mpmax * mpmax;
    j.r = o.r + (size_t)i * mpmax;
    j.a2part = o.a2part + (size_t)i * npart;
    j.ldg = mpmax;
    return j;
  };
  if (split_pipe) {
    SplitPipe sp(c, n, mpmax);
    sp.head = split_head;
    sp.start();
    // the whitening side needs every output's gains from job 1 on
    if (split_head) HIPCHECK(hipStreamWaitEvent(c->s_w, c->ev_gr, 0));
    for (int i = 0; i < np; ++i) sp.push(job(i, sp.buf[i & 1]));
    sp.flush();
    sp.join(c->stream);   // a prediction lane's q(u) runs this on the side stream
    if (split_head) {     // s_g2's gains precede the last Gram's correction, which join covers
      HIPCHECK(hipStreamWaitEvent(c->stream, c->ev_gr, 0));
      HIPCHECK(hipMemcpyAsync(o.logs, logs_src, (size_t)np * nch * sizeof(double),
                              hipMemcpyDeviceToDevice, c->stream));
    }
    return o;
  }
  StageBufs bufs[2];
  const int nbuf = (nlanes > 1 || pipe) ? 2 : 1;
  for (int l = 0; l < nbuf; ++l) bufs[l] = stage_bufs(c, l, n, mpmax);
  if (nlanes > 1) {
    HIPCHECK(hipEventRecord(c->ev_fork, c->stream));
    HIPCHECK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
  }
  if (pipe) {
    // main: W0 W1 G0 W2 G1 W3 G2 ...; side: P0 after W0, P(i+1) after G(i), so P(i+1) runs beside
    // W(i+2) and G(i+1) waits for it.  (P(i+1) right after W(i+1) would start with G(i) and queue
    // G(i)'s co-running correction behind it on the side stream: 4.17 -> 4.93 ms per Gram.)
    auto issue_post = [&](int i) {
      HIPCHECK(hipEventRecord(c->ev_pw, c->main));
      HIPCHECK(hipStreamWaitEvent(c->side, c->ev_pw, 0));
      {
        OnStream on_(c, c->side);
        stage_post(c, jobs[i], bufs[i % nbuf], false);
      }
      HIPCHECK(hipEventRecord(c->ev_pc[i & 1], c->side));
    };
    stage_whiten(c, job(0, bufs[0]), bufs[0]);
    issue_post(0);
    for (int i = 0; i < np; ++i) {
      if (i + 1 < np) stage_whiten(c, job(i + 1, bufs[(i + 1) % nbuf]), bufs[(i + 1) % nbuf]);
      HIPCHECK(hipStreamWaitEvent(c->main, c->ev_pc[i & 1], 0));
      stage_gram(c, jobs[i], bufs[i % nbuf], false, false, "", c->side, 256);
      if (i + 1 < np) issue_post(i + 1);
    }
    // every side-stream item has been waited for: P(np-1) by G(np-1), the corrections by their Gram
    return o;
  }
  // one lane: the caller's stream (a prediction lane's q(u) may run on the side stream; its
  // Gram's co-running correction then goes to main)
  const hipStream_t base = c->stream;
  const hipStream_t helper = base == c->side ? c->main : c->side;
  for (int i = 0; i < np; ++i) {
    const int lane = i % nlanes;
    const StageBufs& b = bufs[i % nbuf];
    OnStream on_(c, lane ? c->side : base);
    const StageJob& j = job(i, b);
    stage_whiten(c, j, b);
    stage_post(c, j, b, fix_beta);
    stage_gram(c, j, b, fix_beta, nlanes > 1, (nlanes > 1 && lane) ? "_1" : "",
               nlanes == 1 ? helper : nullptr, 256);
  }
  if (nlanes > 1) {   // join: the dense tail on the context stream needs every G
    HIPCHECK(hipEventRecord(c->ev_join, c->side));
    HIPCHECK(hipStreamWaitEvent(c->main, c->ev_join, 0));
  }
  return o;
}

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

// L_u = chol(Kuu [+ s2 I]), T_u = L_u^-1, Lambda = T_u G T_u^T + I, L_lam = chol(Lambda) for
// every problem: blocked 64 x 64 MFMA kernels (k_chol.hip), matrices padded with identity to
// ld = Mp (padding contributes log 1 = 0 and zero right-hand sides).  run_dense_pre is the part
// that does not read G (Kuu, its Cholesky factor and inverse), run_dense_post the rest.
static DenseOut run_dense_pre(gpar_ctx* c, const std::vector<DevProblem>& P,
                              const std::vector<Theta>& th, int64_t ld, bool qu_mode) {
  const int np = (int)P.size();
  const int nb = (int)(ld / kDenseNB);
  DenseOut o;
  o.ld = ld;
  o.nb = nb;
  const size_t sq = (size_t)ld * ld;
  o.Lu = ws<double>(c, "Kuu", (size_t)np * sq);
  o.Llam = ws<double>(c, "Lam", (size_t)np * sq);
  o.Tu = ws<double>(c, "Tu", (size_t)np * sq);
  double* Tdu = ws<double>(c, "Tdu", (size_t)np * nb * kDenseNB * kDenseNB);
  o.Tdl = ws<double>(c, "Tdl", (size_t)np * nb * kDenseNB * kDenseNB);
  o.Tl = nullptr;
  o.status = ws<int>(c, "status", (size_t)np * 2);
  HIPCHECK(hipMemsetAsync(o.status, 0, np * 2 * sizeof(int), c->stream));
  std::vector<KuuJobHost> kj(np);
  std::vector<CholJob2Host> cu(np);
  for (int i = 0; i < np; ++i) {
    const DevProblem& p = P[i];
    const double s2 = th[i].sigma * th[i].sigma;
    kj[i] = {p.z, p.ldz, (int)p.d, p.ok, 1.0 / th[i].l_o, th[i].sv_o * th[i].sv_o,
             (qu_mode ? p.qu_noise : p.kuu_noise) ? s2 : 0.0, o.Lu + i * sq, ld, (int)p.m, (int)ld};
    cu[i] = {o.Lu + i * sq, o.Tu + i * sq, Tdu + (size_t)i * nb * kDenseNB * kDenseNB, o.status + 2 * i};
  }
  auto* dkj = ws<KuuJobHost>(c, "kuujobs", np);
  auto* dcu = ws<CholJob2Host>(c, "chol2u", np);
  h2d(c, dkj, kj.data(), np);
  h2d(c, dcu, cu.data(), np);
  Timed tm_(c, "dense");
  launch_kuu(c->stream, dkj, np, (int)ld);
  check_launch("kuu");
  launch_chol_blocked(c->stream, dcu, np, ld, nb, /*want_t=*/true);
  check_launch("chol(Kuu)");
  return o;
}

static void run_dense_post(gpar_ctx* c, const std::vector<DevProblem>& P, const GramOut& go,
                           const DenseOut& o) {
  const int np = (int)P.size();
  const int64_t ld = o.ld;
  const int nb = o.nb;
  const size_t sq = (size_t)ld * ld;
  double* X = ws<double>(c, "TG", (size_t)np * sq);
  std::vector<CholJob2Host> cl(np);
  std::vector<TgtJobHost> tj(np);
  for (int i = 0; i < np; ++i) {
    cl[i] = {o.Llam + i * sq, o.Tl ? o.Tl + i * sq : nullptr,
             o.Tdl + (size_t)i * nb * kDenseNB * kDenseNB, o.status + 2 * i + 1};
    tj[i] = {o.Tu + i * sq, go.G + i * sq, X + i * sq, o.Llam + i * sq};
  }
  auto* dcl = ws<CholJob2Host>(c, "chol2l", np);
  auto* dtj = ws<TgtJobHost>(c, "tgtjobs", np);
  h2d(c, dcl, cl.data(), np);
  h2d(c, dtj, tj.data(), np);
  Timed tm_(c, "dense");
  launch_tgt(c->stream, dtj, np, ld, nb);
  check_launch("Lambda = T G T^T + I");
  launch_chol_blocked(c->stream, dcl, np, ld, nb, /*want_t=*/false);
  check_launch("chol(Lambda)");
}

static DenseOut run_dense(gpar_ctx* c, const std::vector<DevProblem>& P,
                          const std::vector<Theta>& th, const GramOut& go, bool qu_mode) {
  DenseOut o = run_dense_pre(c, P, th, go.ldg, qu_mode);
  run_dense_post(c, P, go, o);
  return o;
}

static Finish2JobHost finish_job(const DenseOut& dn, const GramOut& go, const DevProblem& p, int i,
                                 int64_t nch, double* out, double* me) {
  const size_t sq = (size_t)dn.ld * dn.ld;
  return Finish2JobHost{dn.Tu + i * sq, dn.Llam + i * sq,
                        dn.Tdl + (size_t)i * dn.nb * kDenseNB * kDenseNB, go.r + (size_t)i * go.ldg,
                        go.logs + (size_t)i * nch, nch, go.a2part + (size_t)i * go.npart, go.npart,
                        p.n, dn.status + 2 * i, out, me};
}

static std::vector<Theta> thetas_from(const double* theta, int np) {
  std::vector<Theta> th(np);
  for (int i = 0; i < np; ++i) {
    const double* q = theta + 5 * i;
    th[i] = {q[0], q[1], q[2], q[3], q[4]};
    for (int j = 0; j < 5; ++j)
      ARGCHECK(std::isfinite(q[j]) && q[j] > 0.0, "theta entries must be positive and finite");
  }
  return th;
}

// DTC objective for all problems; status_out[i] = 1 if a Cholesky failed for problem i.
static void eval_dtc(gpar_ctx* c, const std::vector<DevProblem>& P, const std::vector<Theta>& th,
                     double* out, std::vector<int>& status_out, GramOut* gram_out = nullptr) {
  const int np = (int)P.size();
  // On the CU-split pipeline the G-independent half of the dense tail (Kuu, its factor and
  // inverse) goes first on the Gram stream: it runs beside the gains and the first whitening,
  // while the Gram CUs would otherwise wait, instead of after the round's last Gram.
  int64_t mpmax = 0;
  for (const auto& p : P) mpmax = std::max(mpmax, p.mp);
  const bool early = c->dense_early && fit_pipelined(c, P) && split_active(c, P[0].n, mpmax);
  DenseOut dn{};
  if (early) {
    // the Gram stream first follows everything queued on the context stream (host inputs' uploads,
    // the pseudo-input centres, the distance cache), then factors Kuu beside the round's gains
    HIPCHECK(hipEventRecord(c->ev_dn, c->stream));
    HIPCHECK(hipStreamWaitEvent(c->s_g, c->ev_dn, 0));
    OnStream on_(c, c->s_g);
    dn = run_dense_pre(c, P, th, mpmax, false);
  }
  GramOut go = run_gram_stage(c, P, th);
  if (gram_out) *gram_out = go;
  if (!early) dn = run_dense_pre(c, P, th, go.ldg, false);
  run_dense_post(c, P, go, dn);
  const int64_t nch = P[0].nch;
  std::vector<Finish2JobHost> fj(np);
  double* dout = ws<double>(c, "dtc_out", np);
  for (int i = 0; i < np; ++i) fj[i] = finish_job(dn, go, P[i], i, nch, dout + i, nullptr);
  auto* dfj = ws<Finish2JobHost>(c, "finishjobs", np);
  h2d(c, dfj, fj.data(), np);
  launch_finish2(c->stream, dfj, np, dn.ld, dn.nb);
  check_launch("finish");
  std::vector<int> st(2 * np);
  d2h(c, out, dout, np);
  d2h(c, st.data(), dn.status, 2 * np);
  sync(c);
  status_out.assign(np, 0);
  for (int i = 0; i < np; ++i) status_out[i] = st[2 * i] || st[2 * i + 1];
}


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

static QuOut run_q_u(gpar_ctx* c, const DevProblem& p, const Theta& th,
                     const GramCache* gc = nullptr) {
  std::vector<DevProblem> P{p};
  std::vector<Theta> T{th};
  // The extra beta fix-up pass is for the noise-free Cuu only; with qu_kuu_noise the factor is
  // the objective's regularised Kuu + s2 I and the objective's correction-form Gram is enough --
  // the very Gram the fit computed at this theta, when the caller hands it over (gc).
  GramOut go;
  if (gc && gc->G && p.qu_noise) {
    go.ldg = p.mp;
    go.npart = 1;
    go.G = const_cast<double*>(gc->G);
    go.r = const_cast<double*>(gc->r);
    go.a2part = ws<double>(c, "qu_zero_a2", 1);          // dtc terms: unused in q(u) mode
    go.logs = ws<double>(c, "qu_zero_logs", (size_t)p.nch);
    HIPCHECK(hipMemsetAsync(go.a2part, 0, sizeof(double), c->stream));
    HIPCHECK(hipMemsetAsync(go.logs, 0, (size_t)p.nch * sizeof(double), c->stream));
  } else {
    go = run_gram_stage(c, P, T, /*fix_beta=*/!p.qu_noise);
  }
  DenseOut dn = run_dense(c, P, T, go, /*qu_mode=*/true);
  QuOut q;
  q.ld = dn.ld;
  q.me = ws<double>(c, "qu_me", dn.ld);
  Finish2JobHost fj = finish_job(dn, go, p, 0, p.nch, ws<double>(c, "dtc_out", 1), q.me);
  auto* dfj = ws<Finish2JobHost>(c, "finishjobs", 1);
  h2d(c, dfj, &fj, 1);
  launch_finish2(c->stream, dfj, 1, dn.ld, dn.nb);
  check_launch("finish(q_u)");
  // X = L_D^{-1} I by substitution; cov = X^T X.  q(u) factors the noise-free Cuu
  // (gpar_scaled_inference.jl:157; cond up to ~1e10), where products of explicit inverses lose
  // accuracy that triangular substitution keeps -- the objective's T_u = chol(Kuu + s2 I)^-1
  // is regularised by the noise and stays on the blocked-inverse path.
  double* I = ws<double>(c, "qu_eye", (size_t)dn.ld * dn.ld);
  double* X = ws<double>(c, "qu_X", (size_t)dn.ld * dn.ld);
  q.cov = ws<double>(c, "qu_cov", (size_t)dn.ld * dn.ld);
  q.Tu = dn.Tu;
  q.Tl = nullptr;
  q.nb = dn.nb;
  launch_eye(c->stream, I, dn.ld, (int)p.m);
  TrsmJobHost tj{dn.Llam, dn.ld, I, dn.ld, X, dn.ld, (int)p.m, p.m, 0, 0};
  auto* dtj = ws<TrsmJobHost>(c, "trsmjobsQ", 1);
  h2d(c, dtj, &tj, 1);
  launch_trsm(c->stream, dtj, 1, p.m);
  launch_gram_small(c->stream, X, dn.ld, (int)p.m, q.cov, dn.ld);
  q.Ucol = ws<double>(c, "qu_U", (size_t)p.m * p.m);
  launch_lower_to_upper_colmajor(c->stream, dn.Lu, dn.ld, (int)p.m, q.Ucol);
  check_launch("q_u tail");
  int st[2];
  d2h(c, st, dn.status, 2);
  sync(c);
  if (st[0]) throw Error(GPAR_ERR_NOT_PD, "PosDefException: cholesky(Symmetric(Cuu)) failed (gpar_scaled_inference.jl:159)");
  if (st[1]) throw Error(GPAR_ERR_NOT_PD, "PosDefException: cholesky(Symmetric(D)) failed (gpar_scaled_inference.jl:188)");
  return q;
}

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

static std::vector<QuPre> run_q_u_batch(gpar_ctx* c, const std::vector<DevProblem>& P,
                                        const std::vector<Theta>& T, const FitKeep& keep,
                                        bool want_cov) {
  const int np = (int)P.size();
  int64_t mpmax = 0, mmax = 0;
  for (const auto& p : P) { mpmax = std::max(mpmax, p.mp); mmax = std::max(mmax, p.m); }
  const bool qn = P[0].qu_noise;
  bool kept = qn;
  for (int i = 0; i < np; ++i)
    kept = kept && i < (int)keep.valid.size() && keep.valid[i] && keep.gram[i].G;
  GramOut go;
  const size_t sq = (size_t)mpmax * mpmax;
  if (kept) {   // the fit's Grams at the fitted theta, packed at the batch's ld
    go.ldg = mpmax;
    go.npart = 1;
    go.G = ws<double>(c, "qub_G", (size_t)np * sq);
    go.r = ws<double>(c, "qub_r", (size_t)np * mpmax);
    go.a2part = ws<double>(c, "qub_zero_a2", (size_t)np);   // dtc terms: unused in q(u) mode
    go.logs = ws<double>(c, "qub_zero_logs", (size_t)np * P[0].nch);
    HIPCHECK(hipMemsetAsync(go.a2part, 0, (size_t)np * sizeof(double), c->stream));
    HIPCHECK(hipMemsetAsync(go.logs, 0, (size_t)np * P[0].nch * sizeof(double), c->stream));
    HIPCHECK(hipMemsetAsync(go.G, 0, (size_t)np * sq * sizeof(double), c->stream));
    HIPCHECK(hipMemsetAsync(go.r, 0, (size_t)np * mpmax * sizeof(double), c->stream));
    for (int i = 0; i < np; ++i) {
      const GramCache& g = keep.gram[i];
      HIPCHECK(hipMemcpy2DAsync(go.G + i * sq, mpmax * sizeof(double), g.G, P[i].mp * sizeof(double),
                                P[i].mp * sizeof(double), P[i].mp, hipMemcpyDeviceToDevice, c->stream));
      HIPCHECK(hipMemcpyAsync(go.r + (size_t)i * mpmax, g.r, P[i].mp * sizeof(double),
                              hipMemcpyDeviceToDevice, c->stream));
    }
  } else {
    go = run_gram_stage(c, P, T, /*fix_beta=*/!qn);
  }
  DenseOut dn = run_dense(c, P, T, go, /*qu_mode=*/true);
  const int64_t ld = dn.ld;
  double* me = ws<double>(c, "qub_me", (size_t)np * ld);
  double* dout = ws<double>(c, "qub_out", (size_t)np);
  std::vector<Finish2JobHost> fj(np);
  for (int i = 0; i < np; ++i) fj[i] = finish_job(dn, go, P[i], i, P[0].nch, dout + i, me + i * ld);
  auto* dfj = ws<Finish2JobHost>(c, "qub_finish", np);
  h2d(c, dfj, fj.data(), np);
  launch_finish2(c->stream, dfj, np, ld, dn.nb);
  check_launch("finish(q_u batch)");
  std::vector<int> st(2 * np);
  d2h(c, st.data(), dn.status, 2 * np);
  sync(c);
  for (int i = 0; i < np; ++i) {
    if (st[2 * i]) throw Error(GPAR_ERR_NOT_PD, "PosDefException: cholesky(Symmetric(Cuu)) failed (gpar_scaled_inference.jl:159), output " + std::to_string(i));
    if (st[2 * i + 1]) throw Error(GPAR_ERR_NOT_PD, "PosDefException: cholesky(Symmetric(D)) failed (gpar_scaled_inference.jl:188), output " + std::to_string(i));
  }
  // w, X1, Vm (and X, cov) by substitution, one launch each for all outputs
  double* I = ws<double>(c, "qub_eye", (size_t)ld * ld);
  double* w = ws<double>(c, "qub_w", (size_t)np * ld);
  double* X1 = ws<double>(c, "qub_X1", (size_t)np * ld * ld);
  double* Vm = ws<double>(c, "qub_V", (size_t)np * ld * ld);
  HIPCHECK(hipMemsetAsync(Vm, 0, (size_t)np * ld * ld * sizeof(double), c->stream));
  launch_eye(c->stream, I, ld, (int)mmax);
  std::vector<TrsvJobHost> tv(np);
  std::vector<TrsmJobHost> t1(np), t2(np), t3(np);
  double* Xc = want_cov ? ws<double>(c, "qub_Xc", (size_t)np * ld * ld) : nullptr;
  double* cov = want_cov ? ws<double>(c, "qub_cov", (size_t)np * ld * ld) : nullptr;
  for (int i = 0; i < np; ++i) {
    const double* Lu = dn.Lu + i * (size_t)ld * ld;
    const double* LD = dn.Llam + i * (size_t)ld * ld;
    const int m = (int)P[i].m;
    tv[i] = {Lu, ld, m, me + i * ld, w + i * ld, 1};
    t1[i] = {Lu, ld, I, ld, X1 + i * (size_t)ld * ld, ld, m, P[i].m, 0, 0};
    t2[i] = {LD, ld, X1 + i * (size_t)ld * ld, ld, Vm + i * (size_t)ld * ld, ld, m, P[i].m, 0, 0};
    if (want_cov) t3[i] = {LD, ld, I, ld, Xc + i * (size_t)ld * ld, ld, m, P[i].m, 0, 0};
  }
  auto* dtv = ws<TrsvJobHost>(c, "qub_trsv", np);
  auto* dt1 = ws<TrsmJobHost>(c, "qub_trsm1", np);
  auto* dt2 = ws<TrsmJobHost>(c, "qub_trsm2", np);
  h2d(c, dtv, tv.data(), np);
  h2d(c, dt1, t1.data(), np);
  h2d(c, dt2, t2.data(), np);
  launch_trsv(c->stream, dtv, np);
  launch_trsm(c->stream, dt1, np, mmax);
  launch_trsm(c->stream, dt2, np, mmax);
  if (want_cov) {
    auto* dt3 = ws<TrsmJobHost>(c, "qub_trsm3", np);
    h2d(c, dt3, t3.data(), np);
    launch_trsm(c->stream, dt3, np, mmax);
    for (int i = 0; i < np; ++i)
      launch_gram_small(c->stream, Xc + i * (size_t)ld * ld, ld, (int)P[i].m, cov + i * (size_t)ld * ld, ld);
  }
  check_launch("q_u batch substitutions");
  std::vector<QuPre> out(np);
  for (int i = 0; i < np; ++i)
    out[i] = {dn.Lu + i * (size_t)ld * ld, dn.Llam + i * (size_t)ld * ld, me + i * ld, w + i * ld,
              X1 + i * (size_t)ld * ld, Vm + i * (size_t)ld * ld,
              want_cov ? cov + i * (size_t)ld * ld : nullptr, ld, dn.nb};
  return out;
}

// logpdf of independent LGSSM chains sharing t (device pointers).
static void chains_logpdf(gpar_ctx* c, int nchains, int64_t n, const double* t, const double* y,
                          int64_t ldy, int kernel, int sdim, const double* theta, double* lml) {
  std::vector<ChainParamsHost> cps(nchains);
  for (int i = 0; i < nchains; ++i) {
    const double l = theta[3 * i], pv = theta[3 * i + 1], ns = theta[3 * i + 2];
    ARGCHECK(l > 0 && pv > 0 && ns > 0, "theta entries must be positive");
    cps[i] = {1.0 / l, l, pv * pv, ns * ns};
  }
  const int64_t nch = (n + kChunk - 1) / kChunk;
  GainsOut g = run_gains(c, sdim, t, n, cps, nullptr, false, "chain");
  double* alpha = ws<double>(c, "chain_alpha", (size_t)nchains * n);
  double* send = ws<double>(c, "chain_send", (size_t)nchains * nch * 4);
  double* cin = ws<double>(c, "chain_cin", (size_t)nchains * nch * 4);
  const int64_t npart = vec_fix_blocks(n);
  double* a2 = ws<double>(c, "chain_a2", (size_t)nchains * npart);
  double* dl = ws<double>(c, "chain_lml", nchains);
  launch_whiten_vec(c->stream, sdim, g.rec, g.recstride, y, ldy, n, kChunk, nch, nchains, alpha, n,
                    send, nch * 4, 1, 0);
  run_carry(c, sdim, g.phi, g.phistride, send, cin, nch * 4, nch, 1, 1, nchains, "chainc");
  launch_vec_fix(c->stream, sdim, alpha, n, g.g, g.gstride, cin, nch * 4, 1, 0, n, kChunk, nchains, a2);
  launch_chain_lml(c->stream, g.logs, nch, a2, npart, n, nchains, dl);
  check_launch("chains_logpdf");
  d2h(c, lml, dl, nchains);
  sync(c);
}


// --------------------------------------------------------------------------- posterior paths
// The path draws of a seed are decorrelated from its q(u) draws (gpar_path_normals exports them).
constexpr uint64_t kPathSeedXor = 0x5851F42D4C957F2Dull;
static uint64_t path_seed(uint64_t seed) { return seed ^ kPathSeedXor; }

// S joint posterior samples of the latent f along one LGSSM chain (TemporalGPs posterior_rand,
// tmp.jl:161-167) with the simulation smoother (k_path.hip): gains g of the chain over the n steps
// of the grid t (params cp, observation noise `noise` per step or cp.r), data v_{k,s} = ym[k] - fx[k * ldfx + s]
// (fx null: ym[k] for every sample).  Samples -> F[k * S + s].
static void path_samples(gpar_ctx* c, int sdim, const GainsOut& g, const ChainParamsHost& cp,
                         const double* t, const double* noise, int64_t n, const double* ym,
                         const double* fx, int64_t ldfx, int S, uint64_t seed, double* F) {
  const int64_t nch = (n + kChunk - 1) / kChunk;
  const size_t cs = (size_t)nch * S * kSStride;
  double* lq = ws<double>(c, "path_lq", (size_t)n * sdim * sdim);
  double* phia = ws<double>(c, "path_phia", (size_t)nch * sdim * sdim);
  double* z = ws<double>(c, "path_z", (size_t)S * n);
  double* X = ws<double>(c, "path_X", (size_t)n * S);
  double* h = ws<double>(c, "path_h", (size_t)n * 4);   // the adjoint fix-up rows (kGStride)
  double* sp_ = ws<double>(c, "path_sp", cs);
  double* cp_ = ws<double>(c, "path_cp", cs);
  double* send = ws<double>(c, "path_send", cs);
  double* cin = ws<double>(c, "path_cin", cs);
  double* bend = ws<double>(c, "path_bend", cs);
  double* chat = ws<double>(c, "path_chat", cs);
  const uint64_t ps = path_seed(seed);
  Timed tm_(c, "path");
  // prior paths: local pass, carry with the chunk transfers prod A_k, final pass (x~[0] -> F,
  // the data columns v - y~ -> z)
  launch_dk_consts(c->stream, sdim, t, n, cp.inv_l, cp.s, lq);
  launch_dk_phi(c->stream, sdim, g.rec, n, kChunk, nch, phia);
  launch_dk_prior(c->stream, sdim, g.rec, lq, noise, cp.r, n, kChunk, nch, S, ps, ym, fx, ldfx,
                  nullptr, sp_, nullptr, nullptr);
  run_carry(c, sdim, phia, 0, sp_, cp_, 0, nch, S, S, 1, "pathp");
  launch_dk_prior(c->stream, sdim, g.rec, lq, noise, cp.r, n, kChunk, nch, S, ps, ym, fx, ldfx,
                  cp_, nullptr, F, z);
  // smoother mean of the S columns (shared gains): whitening into X (column s), carry, adjoint,
  // reverse carry -- the prediction's machinery -- then F += v - R Sigma^{-1} v
  launch_whiten_vec(c->stream, sdim, g.rec, 0, z, n, n, kChunk, nch, S, X, 1, send, kSStride, S, 0,
                    /*astride=*/S);
  run_carry(c, sdim, g.phi, 0, send, cin, 0, nch, S, S, 1, "pathf");
  launch_gains_adjoint(c->stream, sdim, g.rec, n, kChunk, nch, 1, h);
  launch_adjoint_local_wide(c->stream, sdim, X, S, S, g.rec, g.g, cin, S, n, kChunk, nch, bend,
                            nullptr);
  run_carry(c, sdim, g.phi, 0, bend, chat, 0, nch, S, S, 1, "pathb", /*rev=*/true);
  launch_dk_finish(c->stream, sdim, X, S, h, chat, z, noise, cp.r, n, kChunk, nch, S, F);
  check_launch("path samples");
}

// --------------------------------------------------------------------------- prediction
// Prediction half of get_gpar_scaled_predictions (gpar_scaled_inference.jl:63-135); see the
// header of k_predict.hip for the algebra.
// defer (device memory only): the outputs are queued on c->stream but not waited for -- the caller
// synchronises (gpar_fit_predict's prediction lanes).
static void predict_impl(gpar_ctx* c, const DevProblem& P, const Theta& th, int mem,
                         int64_t n_star, const double* t_star_in, const double* v_star_in,
                         int64_t ldvs, int mode, int samples, uint64_t seed, double* mean_out,
                         double* std_out, const GramCache* gc = nullptr, bool defer = false,
                         const QuPre* pre = nullptr) {
  const int64_t n = P.n, m = P.m, d = P.d, mp = P.mp, mc = P.mc;
  // ---- test inputs on device, ascending (host inputs are stably sorted here, outputs
  //      un-permuted at the end; device inputs must already be ascending)
  std::vector<int64_t> perm;
  const double* ts = t_star_in;
  const double* vs = v_star_in;
  int64_t ldv_s = ldvs;
  if (mem == GPAR_MEM_HOST) {
    double* dts = ws<double>(c, "pr_ts", n_star);
    double* dvs = ws<double>(c, "pr_vs", (size_t)n_star * d);
    if (std::is_sorted(t_star_in, t_star_in + n_star)) {   // already ascending: no permutation
      h2d(c, dts, t_star_in, n_star);
      h2d_rows(c, dvs, v_star_in, ldvs, d, n_star);
    } else {
      perm.resize(n_star);
      for (int64_t i = 0; i < n_star; ++i) perm[i] = i;
      std::stable_sort(perm.begin(), perm.end(),
                       [&](int64_t a, int64_t b) { return t_star_in[a] < t_star_in[b]; });
      std::vector<double> tsh(n_star), vsh((size_t)n_star * d);
      for (int64_t i = 0; i < n_star; ++i) {
        tsh[i] = t_star_in[perm[i]];
        for (int64_t q = 0; q < d; ++q) vsh[i * d + q] = v_star_in[perm[i] * ldvs + q];
      }
      h2d(c, dts, tsh.data(), n_star);
      h2d(c, dvs, vsh.data(), (size_t)n_star * d);
    }
    sync(c);
    ts = dts;
    vs = dvs;
    ldv_s = d;
  }
  // ---- q(u): m_e, L_u = chol(Cuu), L_D = chol(D); w = L_u^{-T} m_e, X1 = L_u^{-1} and
  //      V = L_D^{-1} L_u^{-1} by substitution (noise-free Cuu: see run_q_u) -- or all of it
  //      precomputed for a batch of outputs (run_q_u_batch)
  QuOut q{};
  const double *Lu, *LD, *w, *X1, *Vm;
  int64_t ld;
  if (pre) {
    ld = pre->ld;
    Lu = pre->Lu;
    LD = pre->LD;
    w = pre->w;
    X1 = pre->X1;
    Vm = pre->Vm;
    q.ld = ld;
    q.nb = pre->nb;
    q.me = const_cast<double*>(pre->me);
    q.cov = const_cast<double*>(pre->cov);
  } else {
    q = run_q_u(c, P, th, gc);
    Lu = ws<double>(c, "Kuu", 1);
    LD = ws<double>(c, "Lam", 1);
    ld = q.ld;
    double* wv = ws<double>(c, "pr_w", ld);
    TrsvJobHost tv{Lu, ld, (int)m, q.me, wv, 1};
    auto* dtv = ws<TrsvJobHost>(c, "pr_trsv", 1);
    h2d(c, dtv, &tv, 1);
    launch_trsv(c->stream, dtv, 1);
    double* I = ws<double>(c, "qu_eye", (size_t)ld * ld);
    double* X1v = ws<double>(c, "pr_X1", (size_t)ld * ld);
    double* Vmv = ws<double>(c, "pr_V", (size_t)ld * ld);
    launch_eye(c->stream, I, ld, (int)m);
    // V = 0 outside its m x m block (predict_var reads the whole ld x ld buffer)
    HIPCHECK(hipMemsetAsync(Vmv, 0, (size_t)ld * ld * sizeof(double), c->stream));
    TrsmJobHost tj[2] = {{Lu, ld, I, ld, X1v, ld, (int)m, m, 0, 0}, {LD, ld, X1v, ld, Vmv, ld, (int)m, m, 0, 0}};
    auto* dtj = ws<TrsmJobHost>(c, "pr_trsm", 2);
    h2d(c, dtj, tj, 2);
    launch_trsm(c->stream, dtj, 1, m);
    launch_trsm(c->stream, dtj + 1, 1, m);
    w = wv;
    X1 = X1v;
    Vm = Vmv;
  }
  check_launch("predict: q(u) tail");
  // ---- merged grid
  const int64_t nt = n + n_star;
  const int64_t nch = (nt + kChunk - 1) / kChunk;
  double* tm = ws<double>(c, "pr_tm", nt);
  double* ym = ws<double>(c, "pr_ym", nt);
  double* rm = ws<double>(c, "pr_rm", nt);
  double* vm = ws<double>(c, "pr_vm", (size_t)nt * d);
  int64_t* pos = ws<int64_t>(c, "pr_pos", n_star);
  const double s2 = th.sigma * th.sigma;
  launch_merge_side(c->stream, P.t, n, ts, n_star, 0, P.y, s2, P.v, P.ldv, (int)d, tm, ym, rm, vm, d, nullptr);
  launch_merge_side(c->stream, ts, n_star, P.t, n, 1, nullptr, 1e10, vs, ldv_s, (int)d, tm, ym, rm, vm, d, pos);
  check_launch("predict: merge");
  // q(u) draws as Distributions samples q_u = MvNormal(m_e, Symmetric(inv(D)))
  // (gpar_scaled_inference.jl:103,185): m_e + Lc xi with Lc = chol(inv(D)) lower, so a given xi
  // (gpar_mc_normals) gives the reference's sample; W = Lc^T L_u^{-1} carries it through U_u^{-1}.
  int* stc = nullptr;
  auto mc_factor = [&]() {
    double* Lc = ws<double>(c, "pr_Lc", (size_t)ld * ld);
    double* Tdc = ws<double>(c, "pr_Tdc", (size_t)q.nb * kDenseNB * kDenseNB);
    stc = ws<int>(c, "pr_stc", 1);
    HIPCHECK(hipMemsetAsync(stc, 0, sizeof(int), c->stream));
    launch_pad_identity_copy(c->stream, q.cov, ld, (int)m, Lc);
    CholJob2Host cj{Lc, nullptr, Tdc, stc};
    auto* dcj = ws<CholJob2Host>(c, "pr_cholc", 1);
    h2d(c, dcj, &cj, 1);
    launch_chol_blocked(c->stream, dcj, 1, ld, q.nb, /*want_t=*/false);
    double* W = ws<double>(c, "pr_W", (size_t)ld * ld);
    launch_mc_factor(c->stream, Lc, X1, ld, (int)m, W);
    check_launch("predict: MC factor");
    return W;
  };
  auto check_mc_factor = [&]() {
    int st = 0;
    d2h(c, &st, stc, 1);
    sync(c);
    if (st) throw Error(GPAR_ERR_NOT_PD, "PosDefException: cholesky(Symmetric(inv(D))) failed (MvNormal, gpar_scaled_inference.jl:185)");
  };
  // ---- gains on the merged grid (noise sigma^2 train / 1e10 test)
  std::vector<ChainParamsHost> cps{{1.0 / th.l_t, th.l_t, th.sv_t * th.sv_t, s2}};
  const bool path = mode == GPAR_PREDICT_PATH;
  GainsOut g = run_gains(c, P.sdim, tm, nt, cps, rm, false, "pred");
  double* dmean = ws<double>(c, "pr_mean", n_star);
  double* dstd = ws<double>(c, "pr_std", n_star);
  if (path) {
    // tmp.jl:119-167: per sample, fx_s = Cf*u U_u^{-1} e_s (e_s ~ q(u)) on the merged grid, then a
    // posterior path of the time GP given y* - fx_s (simulation smoother, path_samples), f*_s = fx_s + f_t,s
    double* W = mc_factor();
    double* xi = ws<double>(c, "pr_xi", (size_t)samples * mp);
    launch_normal(c->stream, xi, mp, samples, m, samples, seed);
    double* Bm = ws<double>(c, "pr_Bm", (size_t)samples * mp);
    launch_path_bmat(c->stream, W, ld, w, xi, mp, samples, (int)m, mp, Bm, mp);
    double* Ks = ws<double>(c, "pr_Ks", (size_t)nt * mp);   // Cf*u (gpar_scaled_inference.jl:89)
    launch_dist2(c->stream, P.ok, vm, d, nt, P.z, P.ldz, m, mp, (int)d, P.zc, Ks, mp,
                 /*take_sqrt=*/P.ok != GPAR_EQ);
    launch_kfu_from_dist(c->stream, P.ok, Ks, nt, m, mp, 1.0 / th.l_o, th.sv_o * th.sv_o);
    double* FX = ws<double>(c, "pr_FX", (size_t)nt * samples);
    double* fxsq = ws<double>(c, "pr_fxsq", (size_t)nt);
    launch_gemm_nt(c->stream, Ks, mp, Bm, mp, nt, samples, m, 0, FX, samples, fxsq, 0, nullptr,
                   nullptr, nullptr, 0);
    check_launch("predict: path fx");
    double* F = ws<double>(c, "pr_F", (size_t)nt * samples);
    path_samples(c, P.sdim, g, cps[0], tm, rm, nt, ym, FX, samples, samples, seed, F);
    launch_path_stats(c->stream, FX, samples, F, samples, pos, n_star, dmean, dstd);
    check_launch("predict: path stats");
    check_mc_factor();
  } else {
    // ---- whiten Cf*u columns (on the fly) and y* into X, forward carry
    const int64_t ldx = mp + 64;
    double* X = ws<double>(c, "pr_X", (size_t)nt * ldx);
    double* send = ws<double>(c, "pr_send", (size_t)nch * mc * 4);
    double* cin = ws<double>(c, "pr_cin", (size_t)nch * mc * 4);
    double* bend = ws<double>(c, "pr_bend", (size_t)nch * mc * 4);
    double* chat = ws<double>(c, "pr_chat", (size_t)nch * mc * 4);
    double* h = ws<double>(c, "pr_h", (size_t)nt * 4);
    {   // algorithmic HBM bytes: merged inputs V* (d) read, gains records + fix-up rows (20), the
        // m whitened Cf*u columns written, per merged row
      Timed tm_(c, "pred_whiten", 8.0 * (double)nt * ((double)d + (double)m + 20.0));
      whiten_kfu_any(c, P, g.rec, vm, d, nt, nch, th, X, ldx, send, g.g, nullptr);
      launch_whiten_vec(c->stream, P.sdim, g.rec, 0, ym, 0, nt, kChunk, nch, 1, X + mp, 0, send, 0,
                        mc, mp, ldx);
    }
    check_launch("predict: whiten");
    run_carry(c, P.sdim, g.phi, 0, send, cin, 0, nch, mc, mc, 1, "predf");
    // ---- adjoint: Sigma^{-1} x = W^T (W x)
    launch_gains_adjoint(c->stream, P.sdim, g.rec, nt, kChunk, nch, 1, h);
    // u is read back only at the test rows (predict_rows), where rm = 1e10
    {   // bytes: the mc whitened columns read per merged row, records + fix-up rows + R (21), u
        // written at the test rows
      Timed tm_(c, "pred_adjoint", 8.0 * ((double)nt * ((double)mc + 21.0) + (double)n_star * (double)mc));
      launch_adjoint_local_wide(c->stream, P.sdim, X, ldx, mc, g.rec, g.g, cin, mc, nt, kChunk, nch,
                                bend, rm);
    }
    check_launch("predict: adjoint");
    run_carry(c, P.sdim, g.phi, 0, bend, chat, 0, nch, mc, mc, 1, "predb", /*rev=*/true);
    // ---- ANALYTIC with m <= 512: rows, mean and |Q_i V^T| in one pass, Q never stored
    if (mode == GPAR_PREDICT_ANALYTIC && c->predict_fused && ld == mp && predict_var_tiles(mp) > 0) {
      {   // flops of |Q_i V^T|^2 with V lower triangular, as pred_gemm
        Timed tm_(c, "pred_var", (double)n_star * (double)m * (double)(m + 1));
        launch_predict_var(c->stream, P.sdim, X, ldx, h, chat, mc, mp, m, kChunk, pos, n_star, rm,
                           ym, w, Vm, ld, dmean, dstd);
      }
      check_launch("predict: rows + variance");
      goto outputs;
    }
    // ---- per test row: Q = R Sigma^{-1} Cf*u, mean
    double* Q = ws<double>(c, "pr_Q", (size_t)n_star * mp);
    {   // bytes: u rows at the test points read, Q rows written (mp each)
      Timed tm_(c, "pred_rows", 16.0 * (double)n_star * (double)mp);
      launch_predict_rows(c->stream, P.sdim, X, ldx, h, chat, mc, mp, m, kChunk, pos, n_star, rm, ym,
                          w, Q, mp, dmean);
    }
    check_launch("predict: rows");
    // ---- Z = Q V^T;  ANALYTIC: std = |Z_i|;  MC: f_s = mean + Z xi_s, mean/std over samples
    const int ncb = (int)((m + 127) / 128);
    if (mode == GPAR_PREDICT_ANALYTIC) {
      double* rowsq = ws<double>(c, "pr_rowsq", (size_t)ncb * n_star);
      {   // flops of |Q_i V^T|^2 with V lower triangular: 2 n* sum_c (c + 1) = n* m (m + 1)
        Timed tm_(c, "pred_gemm", (double)n_star * (double)m * (double)(m + 1));
        launch_gemm_nt(c->stream, Q, mp, Vm, ld, n_star, m, m, 0, nullptr, 0, rowsq, 0, nullptr,
                       nullptr, nullptr, /*tri=*/1);
      }
      launch_rowsq_finish(c->stream, rowsq, n_star, ncb, dstd);
    } else {
      // MC: f_s = mean + (I - S) K* U_u^{-1} Lc xi_s
      double* W = mc_factor();
      double* Z = ws<double>(c, "pr_Z", (size_t)n_star * mp);
      double* rowsq = ws<double>(c, "pr_rowsq", (size_t)ncb * n_star);
      double* xi = ws<double>(c, "pr_xi", (size_t)samples * mp);
      double* mmc = ws<double>(c, "pr_mmc", n_star);
      launch_gemm_nt(c->stream, Q, mp, W, ld, n_star, m, m, 0, Z, mp, rowsq, 0, nullptr, nullptr,
                     nullptr, /*tri=*/0);
      launch_normal(c->stream, xi, mp, samples, m, samples, seed);
      if (samples <= 128) {   // one column tile: statistics in the GEMM epilogue
        launch_gemm_nt(c->stream, Z, mp, xi, mp, n_star, samples, m, 1, nullptr, 0, nullptr, samples,
                       dmean, mmc, dstd);
      } else {
        const int nsb = (int)((samples + 127) / 128);
        double* part = ws<double>(c, "pr_mcpart", (size_t)nsb * n_star * 2);
        launch_gemm_nt(c->stream, Z, mp, xi, mp, n_star, samples, m, 2, nullptr, 0, part, 0, nullptr,
                       nullptr, nullptr);
        launch_mc_stats_finish(c->stream, part, n_star, nsb, samples, dmean, mmc, dstd);
      }
      dmean = mmc;
      check_mc_factor();
    }
    check_launch("predict: gemm");
  }
outputs:
  // ---- outputs
  if (mem == GPAR_MEM_DEVICE) {
    HIPCHECK(hipMemcpyAsync(mean_out, dmean, n_star * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    HIPCHECK(hipMemcpyAsync(std_out, dstd, n_star * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    if (!defer) sync(c);
  } else if (perm.empty()) {   // t* was ascending: straight into the caller's buffers
    d2h(c, mean_out, dmean, n_star);
    d2h(c, std_out, dstd, n_star);
    sync(c);
  } else {
    std::vector<double> hm(n_star), hs(n_star);
    d2h(c, hm.data(), dmean, n_star);
    d2h(c, hs.data(), dstd, n_star);
    sync(c);
    for (int64_t i = 0; i < n_star; ++i) {
      mean_out[perm[i]] = hm[i];
      std_out[perm[i]] = hs[i];
    }
  }
}


// --------------------------------------------------------------------------- temporal chains: smoothing
// Smoothed marginals of f for chains sharing the grid t (device pointers): mean = y - R Sigma^-1 y,
// var = RTS P^s[0,0].  noise: per-step observation variance (negative = chain sigma^2) or null.
static void chains_smooth(gpar_ctx* c, int nchains, int64_t n, const double* t, const double* y,
                          int64_t ldy, const double* noise, int sdim,
                          const std::vector<ChainParamsHost>& cps, double* mean, double* var,
                          int64_t ldo) {
  const int64_t nch = (n + kChunk - 1) / kChunk;
  GainsOut g = run_gains(c, sdim, t, n, cps, noise, /*want_pf=*/true, "sm");
  double* u = ws<double>(c, "sm_u", (size_t)nchains * n);
  double* send = ws<double>(c, "sm_send", (size_t)nchains * nch * 4);
  double* cin = ws<double>(c, "sm_cin", (size_t)nchains * nch * 4);
  double* bend = ws<double>(c, "sm_bend", (size_t)nchains * nch * 4);
  double* chat = ws<double>(c, "sm_chat", (size_t)nchains * nch * 4);
  double* h = ws<double>(c, "sm_h", (size_t)nchains * n * 4);
  const int64_t ss = nch * 4;
  launch_whiten_vec(c->stream, sdim, g.rec, g.recstride, y, ldy, n, kChunk, nch, nchains, u, n,
                    send, ss, 1, 0);
  run_carry(c, sdim, g.phi, g.phistride, send, cin, ss, nch, 1, 1, nchains, "smf");
  launch_gains_adjoint(c->stream, sdim, g.rec, n, kChunk, nch, nchains, h);
  launch_adjoint_local(c->stream, sdim, u, 1, 1, g.rec, g.g, cin, 1, n, kChunk, nch, bend, nchains,
                       n, ss);
  run_carry(c, sdim, g.phi, g.phistride, bend, chat, ss, nch, 1, 1, nchains, "smb", true);
  auto* dcps = ws<ChainParamsHost>(c, "sm_cps2", nchains);
  h2d(c, dcps, cps.data(), nchains);
  launch_smooth_mean(c->stream, sdim, u, h, chat, ss, y, ldy, noise, dcps, n, kChunk, nchains, mean,
                     ldo);
  double* vloc = ws<double>(c, "sm_vloc", (size_t)nchains * n);
  double* gam = ws<double>(c, "sm_gam", (size_t)nchains * n * 4);
  double* agg = ws<double>(c, "sm_agg", (size_t)nchains * nch * 2 * sdim * sdim);
  double* phat = ws<double>(c, "sm_phat", (size_t)nchains * nch * sdim * sdim);
  launch_cov_smooth(c->stream, sdim, t, g.rec, g.pf, dcps, n, kChunk, nch, nchains, vloc, gam, agg,
                    phat, var, ldo);
  check_launch("chains_smooth");
}

static std::vector<ChainParamsHost> chain_params(const double* theta, int nchains) {
  std::vector<ChainParamsHost> cps(nchains);
  for (int i = 0; i < nchains; ++i) {
    const double l = theta[3 * i], pv = theta[3 * i + 1], ns = theta[3 * i + 2];
    ARGCHECK(l > 0 && pv > 0 && ns > 0 && std::isfinite(l + pv + ns), "theta entries must be positive");
    cps[i] = {1.0 / l, l, pv * pv, ns * ns};
  }
  return cps;
}

static double unpack(double p) { return std::exp(p) + 1e-3; }

}  // namespace gpar

using namespace gpar;

// Entry: order the context's streams after the caller's input stream (if one was set).
static void enter(gpar_ctx* c) {
  c->err.clear();
  HIPCHECK(hipSetDevice(c->device));
  c->stream = c->main;
  if (c->has_input_stream) {
    HIPCHECK(hipEventRecord(c->ev_input, c->input_stream));
    HIPCHECK(hipStreamWaitEvent(c->main, c->ev_input, 0));
    HIPCHECK(hipStreamWaitEvent(c->side, c->ev_input, 0));
  }
}

// Failure exit: nothing queued by the failed call may still be reading caller memory when the
// error returns (callers free their inputs on an error), so both streams are drained first.
static int fail(gpar_ctx* c, int code, const char* what) {
  c->err = what;
  c->stream = c->main;
  (void)hipStreamSynchronize(c->main);
  (void)hipStreamSynchronize(c->side);
  for (hipStream_t st : {c->s_w, c->s_g, c->s_g2, c->s_d})
    if (st) (void)hipStreamSynchronize(st);
  (void)hipGetLastError();
  return code;
}

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

// CU split of the pipelined fit (gpar_ctx_set_cu_split): CU-masked streams for the whitening
// (mask bits [0, 8w): bit i is a CU of XCD i % 8, the bits of one XCD walk its four SEs in turn,
// tools/ubench/cumask_probe.cpp) and for the Gram (the other bits).  w a multiple of 4 keeps every
// SE of both sides equally wide: workgroups are dealt to the SEs evenly, so an SE with fewer CUs
// than its neighbours sets the pace (w = 6 measured slower than w = 4).
static int set_cu_split(gpar_ctx* c, int w, bool forced) {
  if (w < 0 || w >= 32 || w % 4) return GPAR_ERR_ARG;
  if (w > 0 && w != c->split_mask_w) {
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, c->device) != hipSuccess) return GPAR_ERR_HIP;
    if (pr.multiProcessorCount != 256) return GPAR_ERR_UNSUPPORTED;   // the MI355X layout only
    // a stream's CU mask is fixed at its creation: a new width gets new streams
    for (hipStream_t* st : {&c->s_w, &c->s_g, &c->s_g2, &c->s_d})
      if (*st) {
        (void)hipStreamSynchronize(*st);
        (void)hipStreamDestroy(*st);
        *st = nullptr;
      }
    c->split_mask_w = 0;
    c->split_w = 0;
    uint32_t mw[8] = {0}, mg[8] = {0};
    for (int i = 0; i < 256; ++i) (i < 8 * w ? mw : mg)[i / 32] |= 1u << (i % 32);
    if (hipExtStreamCreateWithCUMask(&c->s_w, 8, mw) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&c->s_g, 8, mg) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&c->s_g2, 8, mg) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&c->s_d, 8, mw) != hipSuccess)
      return GPAR_ERR_HIP;
    if (!c->ev_sp &&
        (hipEventCreateWithFlags(&c->ev_gd[0], hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&c->ev_gd[1], hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&c->ev_sp, hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&c->ev_g0, hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&c->ev_gr, hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&c->ev_dn, hipEventDisableTiming) != hipSuccess))
      return GPAR_ERR_HIP;
    c->split_mask_w = w;
  }
  c->split_w = w;
  c->split_forced = forced;
  return GPAR_OK;
}

extern "C" {

int32_t gpar_abi_version(void) { return GPAR_ABI_VERSION; }

int32_t gpar_ctx_create(int32_t device, gpar_ctx** out) {
  if (!out) return GPAR_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return GPAR_ERR_HIP;
  if (device < 0 || device >= n) return GPAR_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return GPAR_ERR_HIP;
  auto* c = new gpar_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->main, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_input, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_pw, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_pc[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_pc[1], hipEventDisableTiming) != hipSuccess) {
    delete c;
    return GPAR_ERR_HIP;
  }
  c->stream = c->main;
  if (const char* e = std::getenv("GPAR_PIPELINE")) c->pipeline = std::atoi(e) != 0;
  if (const char* e = std::getenv("GPAR_OVERLAP")) c->overlap = std::atoi(e) != 0;
  if (const char* e = std::getenv("GPAR_PREDICT_FUSED")) c->predict_fused = std::atoi(e) != 0;
  if (const char* e = std::getenv("GPAR_QU_BATCH")) c->qu_batch = std::atoi(e) != 0;
  if (const char* e = std::getenv("GPAR_DENSE_EARLY")) c->dense_early = std::atoi(e) != 0;
  if (const char* e = std::getenv("GPAR_OVERLAP_MAX")) c->overlap_max = std::atoi(e);
  if (const char* e = std::getenv("GPAR_OVERLAP_B")) c->overlap_b = std::atoi(e);
  if (const char* e = std::getenv("GPAR_SPLIT_HEAD")) c->split_head = std::atoi(e) != 0;
  if (const char* e = std::getenv("GPAR_PREDICT_LANES")) c->predict_lanes = std::atoi(e) > 1 ? 2 : 1;
  // A/B knobs: GPAR_SPLIT_CUS overrides the default CU split, GPAR_SPLIT_DGW=0 keeps the DG
  // kernel off the whitening CUs
  if (const char* e = std::getenv("GPAR_SPLIT_DGW")) c->split_dgw = std::atoi(e) != 0;
  const char* e_split = std::getenv("GPAR_SPLIT_CUS");
  if (e_split)
    (void)set_cu_split(c, std::atoi(e_split), true);
  else
    (void)set_cu_split(c, kDefaultCuSplit, false);   // stays 0 where unsupported
  *out = c;
  return GPAR_OK;
}

int32_t gpar_ctx_destroy(gpar_ctx* ctx) {
  if (!ctx) return GPAR_ERR_STATE;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->main);
  (void)hipStreamSynchronize(ctx->side);
  for (auto& kv : ctx->bufs)
    if (kv.second.p) (void)hipFree(kv.second.p);
  (void)hipEventDestroy(ctx->ev_fork);
  (void)hipEventDestroy(ctx->ev_join);
  (void)hipEventDestroy(ctx->ev_input);
  (void)hipEventDestroy(ctx->ev_pw);
  (void)hipEventDestroy(ctx->ev_pc[0]);
  (void)hipEventDestroy(ctx->ev_pc[1]);
  {
    for (hipStream_t st : {ctx->s_w, ctx->s_g, ctx->s_g2, ctx->s_d})
      if (st) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
      }
    for (hipEvent_t ev : {ctx->ev_gd[0], ctx->ev_gd[1], ctx->ev_sp, ctx->ev_grp[0], ctx->ev_grp[1],
                          ctx->ev_gn[0], ctx->ev_gn[1], ctx->ev_g0, ctx->ev_gr, ctx->ev_dn})
      if (ev) (void)hipEventDestroy(ev);
    for (auto& s : ctx->stage)
      if (s.host) (void)hipHostFree(s.host);
  }
  (void)hipStreamDestroy(ctx->side);
  (void)hipStreamDestroy(ctx->main);
  delete ctx;
  return GPAR_OK;
}

const char* gpar_last_error(const gpar_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int64_t gpar_ctx_workspace_bytes(const gpar_ctx* ctx) {
  if (!ctx) return 0;
  int64_t s = 0;
  for (auto& kv : ctx->bufs) s += (int64_t)kv.second.bytes;
  return s;
}

int32_t gpar_ctx_trim(gpar_ctx* ctx) {
  API_BEGIN(ctx)
  HIPCHECK(hipStreamSynchronize(ctx->stream));
  sync_all(ctx);
  for (auto& kv : ctx->bufs)
    if (kv.second.p) HIPCHECK(hipFree(kv.second.p));
  ctx->bufs.clear();
  std::fill(ctx->cache_valid.begin(), ctx->cache_valid.end(), 0);
  API_END(ctx)
}

int32_t gpar_ctx_set_profiling(gpar_ctx* ctx, int32_t on) {
  API_BEGIN(ctx)
  ctx->profiling = on != 0;
  API_END(ctx)
}

int32_t gpar_ctx_kernel_stats(gpar_ctx* ctx, const char* name, int64_t* launches, double* total_ms) {
  API_BEGIN(ctx)
  ARGCHECK(name && launches && total_ms, "null argument");
  flush_stats(ctx);
  auto it = ctx->stats.find(name);
  *launches = it == ctx->stats.end() ? 0 : it->second.launches;
  *total_ms = it == ctx->stats.end() ? 0.0 : it->second.ms;
  API_END(ctx)
}

int32_t gpar_ctx_kernel_work(gpar_ctx* ctx, const char* name, double* work) {
  API_BEGIN(ctx)
  ARGCHECK(name && work, "null argument");
  flush_stats(ctx);
  auto it = ctx->stats.find(name);
  *work = it == ctx->stats.end() ? 0.0 : it->second.work;
  API_END(ctx)
}

int32_t gpar_ctx_set_input_stream(gpar_ctx* ctx, void* stream, int32_t enable) {
  if (!ctx) return GPAR_ERR_STATE;
  ctx->has_input_stream = enable != 0;
  ctx->input_stream = reinterpret_cast<hipStream_t>(stream);
  return GPAR_OK;
}

int32_t gpar_ctx_set_lanes(gpar_ctx* ctx, int32_t lanes) {
  if (!ctx) return GPAR_ERR_STATE;
  if (lanes != 1 && lanes != 2) {
    ctx->err = "gpar_ctx_set_lanes: lanes must be 1 or 2";
    return GPAR_ERR_ARG;
  }
  ctx->lanes = lanes;
  return GPAR_OK;
}

int32_t gpar_ctx_set_cu_split(gpar_ctx* ctx, int32_t cus_per_xcd) {
  if (!ctx) return GPAR_ERR_STATE;
  (void)hipSetDevice(ctx->device);
  // -1: back to the default (kDefaultCuSplit, gated by problem size); else that width, always
  const int rc = cus_per_xcd == -1 ? set_cu_split(ctx, kDefaultCuSplit, false)
                                   : set_cu_split(ctx, cus_per_xcd, true);
  if (rc != GPAR_OK)
    ctx->err = "gpar_ctx_set_cu_split: cus_per_xcd must be -1 (default), 0 or a multiple of 4 "
               "below 32 (256-CU devices)";
  return rc;
}

int32_t gpar_ctx_set_predict_fused(gpar_ctx* ctx, int32_t on) {
  if (!ctx) return GPAR_ERR_STATE;
  ctx->predict_fused = on != 0;
  return GPAR_OK;
}

int32_t gpar_ctx_set_fit_overlap(gpar_ctx* ctx, int32_t on) {
  if (!ctx) return GPAR_ERR_STATE;
  ctx->overlap = on != 0;
  return GPAR_OK;
}

int32_t gpar_ctx_get_cu_split(const gpar_ctx* ctx, int32_t* cus_per_xcd) {
  if (!ctx) return GPAR_ERR_STATE;
  if (!cus_per_xcd) return GPAR_ERR_ARG;
  *cus_per_xcd = ctx->split_w;
  return GPAR_OK;
}

int32_t gpar_ctx_set_dist_cache(gpar_ctx* ctx, int64_t bytes) {
  API_BEGIN(ctx)
  ARGCHECK(bytes >= -1, "bytes must be -1 (auto), 0 (off) or a budget");
  ctx->dist_cache_bytes = bytes;
  API_END(ctx)
}

int32_t gpar_ctx_set_dist_cache_keep(gpar_ctx* ctx, int32_t keep) {
  API_BEGIN(ctx)
  ctx->dist_cache_keep = keep != 0;
  if (!keep) release_dist_cache(ctx);
  API_END(ctx)
}

int32_t gpar_ctx_dist_cache_stats(const gpar_ctx* ctx, int32_t* outputs_cached, int32_t* evictions,
                                  int64_t* bytes_held) {
  if (!ctx) return GPAR_ERR_STATE;
  int64_t held = 0;
  for (auto& kv : ctx->bufs)
    if (is_cache_buf(kv.first)) held += (int64_t)kv.second.bytes;
  if (outputs_cached) *outputs_cached = ctx->cache_outputs;
  if (evictions) *evictions = ctx->cache_evictions;
  if (bytes_held) *bytes_held = held;
  return GPAR_OK;
}

int32_t gpar_pairwise_distances(gpar_ctx* ctx, const gpar_problem* prob, double* dist_out) {
  API_BEGIN(ctx)
  ARGCHECK(prob && dist_out, "null argument");
  DevProblem p = prepare_problem(ctx, *prob, 0);
  // the fit's distance-cache kernel, as gpar_fit fills a cache slot (attach_dist_cache)
  double* d = ws<double>(ctx, "pw_dist", (size_t)p.n * p.mp);
  launch_dist2(ctx->stream, p.ok, p.v, p.ldv, p.n, p.z, p.ldz, p.m, p.mp, (int)p.d, p.zc, d, p.mp,
               /*take_sqrt=*/p.ok != GPAR_EQ);
  check_launch("dist2 (pairwise)");
  HIPCHECK(hipMemcpy2DAsync(dist_out, p.m * sizeof(double), d, p.mp * sizeof(double),
                            p.m * sizeof(double), p.n,
                            prob->mem == GPAR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                            ctx->stream));
  sync(ctx);
  API_END(ctx)
}

int32_t gpar_ctx_reset_stats(gpar_ctx* ctx) {
  API_BEGIN(ctx)
  flush_stats(ctx);
  ctx->stats.clear();
  API_END(ctx)
}

int32_t gpar_dtc_objective(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                           const double* theta, double* dtc_out) {
  API_BEGIN(ctx)
  ARGCHECK(probs && nprob >= 1 && theta && dtc_out, "null argument");
  check_batch(probs, nprob);
  std::vector<DevProblem> P;
  for (int i = 0; i < nprob; ++i) P.push_back(prepare_problem(ctx, probs[i], i));
  std::vector<Theta> th = thetas_from(theta, nprob);
  std::vector<int> st;
  eval_dtc(ctx, P, th, dtc_out, st);
  for (int i = 0; i < nprob; ++i)
    if (st[i])
      throw Error(GPAR_ERR_NOT_PD, "PosDefException: Cholesky failed for output " + std::to_string(i));
  API_END(ctx)
}

// Batched Nelder-Mead over the outputs: one objective round serves every pending point.
// keep (optional): per output, the Gram of its lowest-value evaluation (ld = mp) in context
// workspace, and whether that evaluation is the returned minimiser (bitwise).

// Distance cache: the squared distances |v_k - z_c|^2 do not depend on theta, so for the
// outputs it holds they are computed once per fit (dist2, k_dist.hip) and every evaluation's
// whitening reads them (whiten_kfu_d2, memory-bound) instead of rebuilding the distance
// contraction on MFMA inside the fused kernel, whose cost grows with D.  Measured at N = 1e6,
// M = 512: fused 1.62 / 2.13 / 2.6 / 3.2 ms at D = 16 / 32 / 48 / 63, cached 1.75 ms at any D;
// so outputs with D >= kDistCacheMinD are cached, widest first, while the budget lasts
// (gpar_ctx_set_dist_cache; default: the free HBM less a reserve).  n x mp doubles each.
constexpr int64_t kDistCacheMinD = 17;
// With the CU split the whitening runs on a quarter of the chip, where the fused kernel is
// compute-bound (D <= 16: 5.05 ms per launch on 64 CUs against 3.62 ms for the cached one), so a
// batched fit over long series caches every output the budget holds (the narrowest fit last; at
// the north config all 63: 258 GB, 10 GB of the 309 GB left free after the predictions).  Short
// series (N < 2^16) keep the D >= 17 rule: there the fused kernel is latency-bound either way, and
// the small-D fits then stay on the arithmetic a single-output q(u) recomputes (gpar_fit_predict's
// reused Gram stays bit-identical to gpar_predict's).
constexpr int64_t kDistCacheMinDSplit = 1;
constexpr int64_t kDistCacheSplitMinN = (int64_t)1 << 16;

// Device bytes a batched fit's evaluations allocate besides the cache (run_gram_stage, run_dense,
// the kept Grams): the cache's auto budget leaves room for them.
static int64_t fit_ws_estimate(const gpar_ctx* c, const std::vector<DevProblem>& P) {
  const int64_t np = (int64_t)P.size(), n = P[0].n, nch = (n + kChunk - 1) / kChunk;
  int64_t mpmax = 0, rs = 4;
  for (auto& p : P) {
    mpmax = std::max(mpmax, p.mp);
    rs = std::max<int64_t>(rs, rec_size(p.sdim));
  }
  const int64_t nbuf = (fit_pipelined(c, P) || c->lanes > 1) ? 2 : 1;
  const GramPlan pl = gram_plan(n, mpmax, false, 256, 256);
  const int64_t doubles = nbuf * ((n + 16) * mpmax + n + 3 * nch * (mpmax + 1) * 4)   // beta, carries
                          + np * n * (rs + 5)                 // gains records, fix-up rows, alpha
                          + 7 * np * mpmax * mpmax            // G, dense tail, kept Grams
                          + 2 * (pl.part_doubles + pl.rpart_doubles);
  return doubles * (int64_t)sizeof(double);
}

// The same for the prediction of a gpar_fit_predict call (predict_impl, merged grid of n + n_star).
static int64_t predict_ws_estimate(int64_t n, int64_t n_star, int64_t mp, int64_t d, int mode,
                                   int samples, bool fused) {
  const int64_t nt = n + n_star, nch = (nt + kChunk - 1) / kChunk;
  int64_t doubles = nt * (mp + 64)                 // whitened Cf*u + y*
                    + n_star * ((fused ? 0 : mp) + 8 + d)   // Q rows (not with predict_var), mean / std, sorted test inputs
                    + nt * (20 + 8 + d)            // gains records, grid, merged inputs
                    + 4 * nch * (mp + 1) * 4       // carries
                    + 8 * mp * mp;                 // q(u) dense
  if (mode == GPAR_PREDICT_MC) doubles += n_star * mp + (int64_t)samples * mp + 2 * n_star * ((samples + 127) / 128);
  if (mode == GPAR_PREDICT_PATH)   // Cf*u, fx, the data columns, their whitening and the samples
    doubles += nt * mp + (int64_t)samples * (4 * nt + 2 * mp) + 6 * nch * samples * kSStride;
  return doubles * (int64_t)sizeof(double);
}

// later_bytes: what the call allocates after the cache (fit_ws_estimate + predict_ws_estimate).
static std::vector<DevProblem> attach_dist_cache(gpar_ctx* c, const std::vector<DevProblem>& P,
                                                 int64_t later_bytes) {
  std::vector<DevProblem> Q = P;
  c->cache_outputs = 0;
  if (c->dist_cache_bytes == 0) return Q;
  // explicit budget: total cache bytes.  auto: new allocations take at most the free HBM less a
  // reserve -- 1 % of the part plus the workspace the call still has to allocate (what the
  // context already holds under other names is reused) -- and cache buffers the context already
  // holds (gpar_ctx_set_dist_cache_keep) are reused at no cost.  Either way an allocation that
  // fails stops the cache there, and a later workspace allocation that finds no memory evicts
  // cache slots (ws_bytes), so the cache never turns into an out-of-memory failure.
  int64_t budget = c->dist_cache_bytes;
  int64_t fresh = INT64_MAX;
  if (budget < 0) {
    size_t fr = 0, tot = 0;
    HIPCHECK(hipMemGetInfo(&fr, &tot));
    int64_t held_other = 0;
    for (auto& kv : c->bufs)
      if (!is_cache_buf(kv.first)) held_other += (int64_t)kv.second.bytes;
    const int64_t need = std::max<int64_t>(0, later_bytes - held_other);
    const int64_t reserve = std::max<int64_t>((int64_t)1 << 30, (int64_t)(tot / 100)) + need;
    fresh = std::max<int64_t>(0, (int64_t)fr - reserve);
    budget = INT64_MAX;
  }
  std::vector<int> order(P.size());
  for (size_t i = 0; i < P.size(); ++i) order[i] = (int)i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return P[a].d > P[b].d; });
  int64_t mpmax = 0;
  for (auto& p : P) mpmax = std::max(mpmax, p.mp);
  // every output (D >= 1) only where the whitening runs on the CU split's quarter of the chip,
  // i.e. the pipelined split schedule actually runs (fit_pipelined && split_active)
  const int64_t min_d = (fit_pipelined(c, P) && split_active(c, P[0].n, mpmax) &&
                         P[0].n >= kDistCacheSplitMinN) ? kDistCacheMinDSplit : kDistCacheMinD;
  int slot = 0;
  for (int i : order) {
    const DevProblem& p = P[i];
    if (p.d < min_d) continue;
    const int64_t bytes = p.n * p.mp * (int64_t)sizeof(double);
    const std::string name = "distcache" + std::to_string(slot);
    const auto it = c->bufs.find(name);
    const int64_t held = it != c->bufs.end() ? (int64_t)it->second.bytes : 0;
    const int64_t need = held >= bytes ? 0 : bytes - held;   // ws() frees the smaller one first
    if (bytes > budget || need > fresh) continue;
    double* d2 = nullptr;
    try {
      d2 = reinterpret_cast<double*>(ws_bytes(c, name, (size_t)bytes));
    } catch (const Error& e) {
      if (e.code != GPAR_ERR_OOM) throw;
      c->bufs.erase(name);   // another tenant took the memory: cache what fits so far
      break;
    }
    budget -= bytes;
    fresh -= need;
    if ((int)c->cache_valid.size() <= slot) c->cache_valid.resize(slot + 1, 0);
    c->cache_valid[slot] = 1;
    launch_dist2(c->stream, p.ok, p.v, p.ldv, p.n, p.z, p.ldz, p.m, p.mp, (int)p.d, p.zc, d2, p.mp,
                 /*take_sqrt=*/p.ok != GPAR_EQ);
    check_launch("dist2 (cache)");
    Q[i].d2 = d2;
    Q[i].d2_is_r = p.ok != GPAR_EQ;
    Q[i].cache_slot = slot;
    ++slot;
  }
  c->cache_outputs = slot;
  return Q;
}

// ---------------------------------------------------------------- round-overlapping batched fit
// fit_impl's batched Nelder-Mead evaluates one simplex point per output per round.  Round by
// round (eval_dtc), every round drains the chip: its first whitening runs alone, its last Gram
// runs alone, then the next round's gains, the dense tail and a host sync.  On the CU-split
// schedule with >= 4 outputs, fit_overlapped deals the outputs into two groups that take turns:
// while the host waits for group A's values (A's dense tail runs on the whitening CUs, which have
// slack beside the Gram) and steps A's simplices, group B's whitenings and Grams keep both sides of the
// split busy, and A's next round (gains on the whitening CUs, then its jobs) is queued behind
// them -- one drain per fit instead of one per round.  Every output evaluates exactly the points
// its own simplex asks for, in the same order, with the same kernels and per-problem arithmetic
// (batched gains and dense-tail launches compute each problem independently), so the fit equals
// the round-by-round one bit for bit.  Uploads go through pinned arenas (gpar_ctx::staging): a
// pageable copy queued behind running work could block the host and stall the pipeline.
struct OverlapGroup {
  int id = 0;
  std::vector<int> members;        // output indices dealt to this group
  std::vector<int> act;            // this round's active members
  std::vector<Theta> th;           // their hyperparameters this round
  std::vector<DevProblem> sub;     // their problems (stable while their jobs are queued)
  GramOut go{};                    // one G / r / alpha^2 / log S slot per member
  double *alpha_all = nullptr, *asend_all = nullptr, *dout = nullptr;
  double* hout = nullptr;          // pinned: -dtc values of the round
  int* hstat = nullptr;            // pinned: Cholesky status flags (2 per output)
  size_t res_bytes = 0;            // the arena's result prefix
  bool in_flight = false;
};

// Round overlap pays where the drain after each Nelder-Mead round is a large part of the round:
// one 8-way shard of the north job (8 outputs per call) 2.70 -> 2.45 s per step; with all 63
// north outputs in one call the round is long and the concurrent gains / dense tails on the
// whitening CUs slow every Gram instead (5.13 -> 5.46 ms; 18.45 vs 18.75 s per job,
// profiles/bench_r03d_*.json).
constexpr int kOverlapMaxOutputs = 16;

using AcceptFn = std::function<void(int, double, const double*, const double*, int64_t)>;

static void fit_overlapped(gpar_ctx* c, const std::vector<DevProblem>& P,
                           std::vector<NelderMead>& nm, const AcceptFn& accept) {
  const int np = (int)P.size();
  const int64_t n = P[0].n, nch = P[0].nch, npart = vec_fix_blocks(n);
  int64_t mpmax = 0;
  for (auto& p : P) mpmax = std::max(mpmax, p.mp);
  const size_t sq = (size_t)mpmax * mpmax;
  for (hipEvent_t* ev : {&c->ev_grp[0], &c->ev_grp[1], &c->ev_gn[0], &c->ev_gn[1]})
    if (!*ev) HIPCHECK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
  OverlapGroup grp[2];
  // outputs dealt alternately; with c->overlap_b > 0 (A/B) group B is every k-th output instead
  // (about overlap_b of them), group A the rest
  if (c->overlap_b > 0 && c->overlap_b < np) {
    const int k = std::max(2, np / c->overlap_b);
    for (int i = 0; i < np; ++i) grp[(i % k == k - 1) ? 1 : 0].members.push_back(i);
  } else {
    for (int i = 0; i < np; ++i) grp[i & 1].members.push_back(i);
  }
  for (int g = 0; g < 2; ++g) {
    OverlapGroup& G = grp[g];
    G.id = g;
    const size_t cap = G.members.size();
    const std::string sfx = g ? "B" : "A";
    G.go.ldg = mpmax;
    G.go.npart = npart;
    G.go.G = ws<double>(c, "ovG" + sfx, cap * sq);
    G.go.r = ws<double>(c, "ovr" + sfx, cap * mpmax);
    G.go.a2part = ws<double>(c, "ova2" + sfx, cap * npart);
    G.go.logs = ws<double>(c, "ovlogs" + sfx, cap * nch);
    G.alpha_all = ws<double>(c, "ovalpha" + sfx, cap * n);
    G.asend_all = ws<double>(c, "ovasend" + sfx, cap * nch * kSStride);
    G.dout = ws<double>(c, "ovout" + sfx, cap);
    gpar_ctx::Staging& s = c->stage[g];
    const size_t vbytes = (cap * sizeof(double) + 255) & ~(size_t)255;
    G.res_bytes = vbytes + ((2 * cap * sizeof(int) + 255) & ~(size_t)255);
    const size_t need = G.res_bytes + ((size_t)1 << 20) + cap * 4096;
    if (s.cap < need) {
      if (s.host) HIPCHECK(hipHostFree(s.host));
      s.host = nullptr;
      s.cap = 0;
      HIPCHECK(hipHostMalloc((void**)&s.host, need, hipHostMallocDefault));
      s.cap = need;
    }
    G.hout = reinterpret_cast<double*>(s.host);
    G.hstat = reinterpret_cast<int*>(s.host + vbytes);
  }
  reserve_gram_parts(c, P, 1);
  struct StagingScope {   // h2d through group g's pinned arena inside the scope
    gpar_ctx* c;
    StagingScope(gpar_ctx* c_, int g) : c(c_) { c->staging = &c->stage[g]; }
    ~StagingScope() { c->staging = nullptr; }
  };

  SplitPipe sp(c, n, mpmax);
  // a group's dense tail + finish on the context stream as soon as its round's last Gram is
  // issued; its values land in pinned memory, ev_grp[g] marks them
  // (on the whitening CUs: beside the Gram on the whole chip it slowed every Gram by ~5 %)
  auto issue_dense = [&](OverlapGroup& G, int64_t job) {
    OnStream on_(c, c->s_d);
    StagingScope st_(c, G.id);
    HIPCHECK(hipStreamWaitEvent(c->s_d, c->ev_gd[job & 1], 0));
    const int na = (int)G.act.size();
    DenseOut dn = run_dense(c, G.sub, G.th, G.go, false);
    std::vector<Finish2JobHost> fj(na);
    for (int a = 0; a < na; ++a) fj[a] = finish_job(dn, G.go, G.sub[a], a, nch, G.dout + a, nullptr);
    auto* dfj = ws<Finish2JobHost>(c, "finishjobs", np);
    h2d(c, dfj, fj.data(), na);
    launch_finish2(c->s_d, dfj, na, dn.ld, dn.nb);
    check_launch("finish");
    HIPCHECK(hipMemcpyAsync(G.hout, G.dout, na * sizeof(double), hipMemcpyDeviceToHost, c->s_d));
    HIPCHECK(hipMemcpyAsync(G.hstat, dn.status, 2 * na * sizeof(int), hipMemcpyDeviceToHost, c->s_d));
    HIPCHECK(hipEventRecord(c->ev_grp[G.id], c->s_d));
  };
  sp.on_gram = [&](const StageJob& j, int64_t job) {
    if (j.last) issue_dense(grp[j.group], job);
  };
  // ask every active member for its next point; queue the group's gains and its jobs
  auto begin_round = [&](OverlapGroup& G) {
    G.act.clear();
    for (int i : G.members)
      if (!nm[i].done()) G.act.push_back(i);
    if (G.act.empty()) return;
    const int na = (int)G.act.size();
    G.th.clear();
    G.sub.clear();
    std::vector<ChainParamsHost> cps(na);
    std::vector<const double*> ys(na);
    for (int a = 0; a < na; ++a) {
      const int i = G.act[a];
      const auto& x = nm[i].ask();
      G.th.push_back({unpack(x[0]), unpack(x[1]), unpack(x[2]), unpack(x[3]), unpack(x[4])});
      G.sub.push_back(P[i]);
      const Theta& t = G.th.back();
      cps[a] = {1.0 / t.l_t, t.l_t, t.sv_t * t.sv_t, t.sigma * t.sigma};
      ys[a] = P[i].y;
    }
    c->stage[G.id].used = G.res_bytes;   // the previous round's uploads have been consumed
    // the gains run on the whitening CUs beside the other group's whitenings (s_d), not in the
    // whitening stream's order: queued there they delayed the next whitening, and with it the
    // DG share that ends the previous Gram
    GainsOut gn;
    {
      OnStream on_(c, c->s_d);
      StagingScope st_(c, G.id);
      gn = run_gains(c, P[0].sdim, P[0].t, n, cps, nullptr, false, G.id ? "fitB" : "fitA", &ys,
                     G.alpha_all, G.asend_all);
      HIPCHECK(hipMemcpyAsync(G.go.logs, gn.logs, (size_t)na * nch * sizeof(double),
                              hipMemcpyDeviceToDevice, c->s_d));
      HIPCHECK(hipEventRecord(c->ev_gn[G.id], c->s_d));
      HIPCHECK(hipStreamWaitEvent(c->s_w, c->ev_gn[G.id], 0));
    }
    {   // narrower outputs: their G / r slot padding must read as zero in the dense tail
      OnStream on_(c, c->s_g);
      for (int a = 0; a < na; ++a)
        if (G.sub[a].mp != mpmax) {
          HIPCHECK(hipMemsetAsync(G.go.G + a * sq, 0, sq * sizeof(double), c->s_g));
          HIPCHECK(hipMemsetAsync(G.go.r + (size_t)a * mpmax, 0, mpmax * sizeof(double), c->s_g));
        }
    }
    for (int a = 0; a < na; ++a) {
      StageJob j;
      j.p = &G.sub[a];
      j.th = &G.th[a];
      j.gi = gn;
      j.gi.rec = gn.rec + (size_t)a * gn.recstride;
      j.gi.g = gn.g + (size_t)a * gn.gstride;
      j.gi.phi = gn.phi + (size_t)a * gn.phistride;
      j.gi.logs = gn.logs + (size_t)a * nch;
      j.alpha = G.alpha_all + (size_t)a * n;
      j.asend = G.asend_all + (size_t)a * nch * kSStride;
      j.G = G.go.G + a * sq;
      j.r = G.go.r + (size_t)a * mpmax;
      j.a2part = G.go.a2part + (size_t)a * npart;
      j.ldg = mpmax;
      j.group = G.id;
      j.last = a == na - 1;
      sp.push(j);
    }
    G.in_flight = true;
  };
  // wait for a group's values and hand them to its simplices (Gram copies of kept points go to
  // the Gram stream, ahead of the group's next Grams)
  auto finish_round = [&](OverlapGroup& G) {
    if (sp.has_pending && sp.pending.group == G.id) sp.flush();   // its last Gram, then its tail
    HIPCHECK(hipEventSynchronize(c->ev_grp[G.id]));
    OnStream on_(c, c->s_g);
    for (size_t a = 0; a < G.act.size(); ++a) {
      double f = -G.hout[a];
      if (G.hstat[2 * a] || G.hstat[2 * a + 1] || !std::isfinite(f)) f = INFINITY;
      accept(G.act[a], f, G.go.G + a * sq, G.go.r + a * mpmax, mpmax);
    }
    G.in_flight = false;
  };
  sp.start();
  HIPCHECK(hipStreamWaitEvent(c->s_d, c->ev_sp, 0));   // the inputs / distance cache on main
  begin_round(grp[0]);
  begin_round(grp[1]);
  for (int g = 0; grp[0].in_flight || grp[1].in_flight; g ^= 1) {
    if (!grp[g].in_flight) continue;
    finish_round(grp[g]);
    begin_round(grp[g]);
  }
  sp.flush();
  sp.join(c->main);
}

static void fit_impl(gpar_ctx* ctx, const std::vector<DevProblem>& P0, const double* log_theta0,
                     const gpar_fit_options& o, double* theta_out, double* nlml_out,
                     int32_t* evals_out, FitKeep* keep, int64_t later_bytes = 0) {
  // the cache lives for this fit call only, unless the caller keeps it (gpar_ctx_set_dist_cache_keep)
  struct CacheRelease {
    gpar_ctx* c;
    ~CacheRelease() {
      if (c->dist_cache_keep) return;
      try {
        release_dist_cache(c);
      } catch (...) {
      }
    }
  } release_{ctx};
  const std::vector<DevProblem> P =
      attach_dist_cache(ctx, P0, fit_ws_estimate(ctx, P0) + later_bytes);
  const int nprob = (int)P.size();
  std::vector<NelderMead> nm;
  nm.reserve(nprob);
  for (int i = 0; i < nprob; ++i)
    nm.emplace_back(std::vector<double>(log_theta0 + 5 * i, log_theta0 + 5 * i + 5), o.max_evals,
                    o.max_iterations, o.g_tol, o.time_limit);
  std::vector<double> best_f(nprob, INFINITY);
  std::vector<std::vector<double>> best_x(nprob);
  std::vector<double*> kG(nprob, nullptr), kr(nprob, nullptr);
  if (keep) {
    for (int i = 0; i < nprob; ++i) {
      const size_t mp = (size_t)P[i].mp;
      kG[i] = ws<double>(ctx, "fitkeep_G" + std::to_string(i), mp * mp);
      kr[i] = ws<double>(ctx, "fitkeep_r" + std::to_string(i), mp);
    }
  }
  // one evaluated point of output i: keep its Gram if it is the best so far (on c->stream, before
  // the slot is reused), then tell the simplex
  const AcceptFn accept = [&](int i, double f, const double* Gs, const double* rs, int64_t ldg) {
    if (keep && f < best_f[i]) {
      best_f[i] = f;
      best_x[i] = nm[i].ask();
      const size_t mp = (size_t)P[i].mp;
      HIPCHECK(hipMemcpy2DAsync(kG[i], mp * sizeof(double), Gs, ldg * sizeof(double),
                                mp * sizeof(double), mp, hipMemcpyDeviceToDevice, ctx->stream));
      HIPCHECK(hipMemcpyAsync(kr[i], rs, mp * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    }
    nm[i].tell(f);
  };
  int64_t mpmax = 0;
  for (auto& p : P) mpmax = std::max(mpmax, p.mp);
  if (ctx->overlap && nprob >= 4 && nprob <= ctx->overlap_max && fit_pipelined(ctx, P) &&
      split_active(ctx, P[0].n, mpmax))
    fit_overlapped(ctx, P, nm, accept);
  std::vector<double> vals;
  while (true) {
    std::vector<int> act;
    for (int i = 0; i < nprob; ++i)
      if (!nm[i].done()) act.push_back(i);
    if (act.empty()) break;
    std::vector<DevProblem> sub;
    std::vector<Theta> th;
    for (int i : act) {
      sub.push_back(P[i]);
      const auto& x = nm[i].ask();
      th.push_back({unpack(x[0]), unpack(x[1]), unpack(x[2]), unpack(x[3]), unpack(x[4])});
    }
    vals.assign(act.size(), 0.0);
    std::vector<int> st;
    GramOut go{};
    eval_dtc(ctx, sub, th, vals.data(), st, keep ? &go : nullptr);
    for (size_t a = 0; a < act.size(); ++a) {
      double f = -vals[a];
      if (st[a] || !std::isfinite(f)) f = INFINITY;  // PosDefException -> reject the point
      accept(act[a], f, keep ? go.G + a * go.ldg * go.ldg : nullptr,
             keep ? go.r + a * go.ldg : nullptr, go.ldg);
    }
  }
  for (int i = 0; i < nprob; ++i) {
    const auto& x = nm[i].x_min();
    for (int j = 0; j < 5; ++j) theta_out[5 * i + j] = unpack(x[j]);
    if (nlml_out) nlml_out[i] = nm[i].f_min();
    if (evals_out) evals_out[i] = nm[i].evals();
  }
  if (keep) {
    keep->gram.assign(nprob, GramCache{});
    keep->valid.assign(nprob, 0);
    for (int i = 0; i < nprob; ++i) {
      keep->valid[i] = !best_x[i].empty() && best_x[i] == nm[i].x_min();
      if (keep->valid[i]) keep->gram[i] = GramCache{kG[i], kr[i]};
    }
  }
}

int32_t gpar_fit(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                 const double* log_theta0, const gpar_fit_options* opts, double* theta_out,
                 double* nlml_out, int32_t* evals_out) {
  API_BEGIN(ctx)
  ARGCHECK(probs && nprob >= 1 && log_theta0 && theta_out, "null argument");
  check_batch(probs, nprob);
  gpar_fit_options o{0, 1000, 1e-8, 0.0};
  if (opts) o = *opts;
  std::vector<DevProblem> P;
  for (int i = 0; i < nprob; ++i) P.push_back(prepare_problem(ctx, probs[i], i));
  fit_impl(ctx, P, log_theta0, o, theta_out, nlml_out, evals_out, nullptr);
  API_END(ctx)
}

// get_gpar_scaled_predictions for a batch: batched fit, then each output's prediction at its
// fitted theta (in output order).  chain (optional): after output i's prediction its mean is also
// written to column chain_col[i] of chain (point k at chain[k * ld_chain + col]), so later outputs'
// v_star may point into chain and read earlier outputs' predicted means as inference inputs.
static void fit_predict_impl(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                             const double* log_theta0, const gpar_fit_options* opts, int64_t n_star,
                             const double* t_star, const double* const* v_star, const int64_t* ldvs,
                             int32_t mode, int32_t samples, uint64_t seed, double* chain,
                             int64_t ld_chain, const int32_t* chain_col, double* theta_out,
                             double* nlml_out, int32_t* evals_out, double* const* mean_out,
                             double* const* std_out) {
  ARGCHECK(probs && nprob >= 1 && log_theta0 && theta_out && t_star && v_star && ldvs &&
               mean_out && std_out, "null argument");
  ARGCHECK(n_star >= 1, "n_star must be >= 1");
  ARGCHECK(mode == GPAR_PREDICT_ANALYTIC || mode == GPAR_PREDICT_MC || mode == GPAR_PREDICT_PATH,
           "bad mode");
  if (mode != GPAR_PREDICT_ANALYTIC)
    ARGCHECK(samples >= 2 && samples <= kMaxSamples, "MC / path modes take 2..65536 samples");
  for (int i = 0; i < nprob; ++i) {
    ARGCHECK(v_star[i] && mean_out[i] && std_out[i], "null per-output pointer");
    ARGCHECK(ldvs[i] >= probs[i].d, "ldvs must be >= d");
    if (chain) ARGCHECK(chain_col[i] < ld_chain, "chain_col must be < ld_chain");
  }
  check_batch(probs, nprob);
  gpar_fit_options o{0, 1000, 1e-8, 0.0};
  if (opts) o = *opts;
  std::vector<DevProblem> P;
  for (int i = 0; i < nprob; ++i) P.push_back(prepare_problem(ctx, probs[i], i));
  FitKeep keep;
  const int mem = probs[0].mem;
  // Prediction lanes: with device-memory outputs and no chain between the predictions, outputs
  // alternate over the context's two streams, each lane with its own workspace (name suffix), so
  // one output's memory-bound passes (merge, adjoint, rows) run beside the other's DP / MFMA work
  // (whitening, variance GEMM).  A lane's host syncs (q(u)'s Cholesky status) wait for that lane
  // only.
  const bool lanes = mem == GPAR_MEM_DEVICE && !chain && nprob > 1 && ctx->predict_lanes > 1;
  // the predictions' workspace (named buffers, reused across the outputs: the largest counts)
  int64_t pred_bytes = 0;
  for (const auto& p : P)
    pred_bytes = std::max(pred_bytes, predict_ws_estimate(p.n, n_star, p.mp, p.d, mode, samples,
                                                          mode == GPAR_PREDICT_ANALYTIC &&
                                                              ctx->predict_fused &&
                                                              predict_var_tiles(p.mp) > 0));
  fit_impl(ctx, P, log_theta0, o, theta_out, nlml_out, evals_out, &keep, (lanes ? 2 : 1) * pred_bytes);
  struct LaneScope {   // a lane's stream and workspace names; restored on any exit
    gpar_ctx* c;
    hipStream_t saved;
    LaneScope(gpar_ctx* c_, int lane) : c(c_), saved(c_->stream) {
      c->stream = lane ? c->side : c->main;
      c->ws_suffix = lane ? "~1" : "";
    }
    ~LaneScope() {
      c->stream = saved;
      c->ws_suffix.clear();
    }
  };
  // wall time of the predictions (both lanes): from here on the context stream to the join
  std::optional<Timed> tm_pred;
  tm_pred.emplace(ctx, "predictions");
  // q(u) and its substitutions for every output at once (one sync), when the outputs share the
  // q(u) convention
  bool same_qu = true;
  for (const auto& p : P) same_qu = same_qu && p.qu_noise == P[0].qu_noise;
  std::vector<QuPre> pre;
  if (ctx->qu_batch && nprob > 1 && same_qu) {
    std::vector<Theta> T;
    for (int i = 0; i < nprob; ++i) {
      const double* q = theta_out + 5 * i;
      T.push_back(Theta{q[0], q[1], q[2], q[3], q[4]});
    }
    pre = run_q_u_batch(ctx, P, T, keep, mode != GPAR_PREDICT_ANALYTIC);
  }
  if (lanes) {   // the side lane follows the fit (kept Grams, inputs) on the context stream
    HIPCHECK(hipEventRecord(ctx->ev_fork, ctx->main));
    HIPCHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
  }
  for (int i = 0; i < nprob; ++i) {
    const double* q = theta_out + 5 * i;
    const Theta th{q[0], q[1], q[2], q[3], q[4]};
    LaneScope lane_(ctx, lanes ? (i & 1) : 0);
    predict_impl(ctx, P[i], th, mem, n_star, t_star, v_star[i], ldvs[i], mode, samples,
                 seed + (uint64_t)i, mean_out[i], std_out[i],
                 keep.valid[i] ? &keep.gram[i] : nullptr, /*defer=*/lanes,
                 pre.empty() ? nullptr : &pre[i]);
    if (chain && chain_col[i] >= 0) {
      double* dst = chain + chain_col[i];
      if (mem == GPAR_MEM_DEVICE) {   // stream-ordered before the next output's merge reads it
        HIPCHECK(hipMemcpy2DAsync(dst, ld_chain * sizeof(double), mean_out[i], sizeof(double),
                                  sizeof(double), n_star, hipMemcpyDeviceToDevice, ctx->stream));
      } else {
        for (int64_t k = 0; k < n_star; ++k) dst[k * ld_chain] = mean_out[i][k];
      }
    }
  }
  if (lanes) {
    HIPCHECK(hipEventRecord(ctx->ev_join, ctx->side));
    HIPCHECK(hipStreamWaitEvent(ctx->main, ctx->ev_join, 0));
  }
  tm_pred.reset();
  if (lanes || (chain && mem == GPAR_MEM_DEVICE)) sync(ctx);
}

int32_t gpar_fit_predict(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                         const double* log_theta0, const gpar_fit_options* opts, int64_t n_star,
                         const double* t_star, const double* const* v_star, const int64_t* ldvs,
                         int32_t mode, int32_t samples, uint64_t seed, double* theta_out,
                         double* nlml_out, int32_t* evals_out, double* const* mean_out,
                         double* const* std_out) {
  API_BEGIN(ctx)
  fit_predict_impl(ctx, probs, nprob, log_theta0, opts, n_star, t_star, v_star, ldvs, mode, samples,
                   seed, nullptr, 0, nullptr, theta_out, nlml_out, evals_out, mean_out, std_out);
  API_END(ctx)
}

int32_t gpar_fit_predict_chain(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                               const double* log_theta0, const gpar_fit_options* opts,
                               int64_t n_star, const double* t_star, const double* const* v_star,
                               const int64_t* ldvs, int32_t mode, int32_t samples, uint64_t seed,
                               double* chain, int64_t ld_chain, const int32_t* chain_col,
                               double* theta_out, double* nlml_out, int32_t* evals_out,
                               double* const* mean_out, double* const* std_out) {
  API_BEGIN(ctx)
  ARGCHECK(chain && chain_col && ld_chain >= 1, "null chain argument");
  fit_predict_impl(ctx, probs, nprob, log_theta0, opts, n_star, t_star, v_star, ldvs, mode, samples,
                   seed, chain, ld_chain, chain_col, theta_out, nlml_out, evals_out, mean_out,
                   std_out);
  API_END(ctx)
}

int32_t gpar_dtc_objective_A(gpar_ctx* ctx, const gpar_problem* prob, const double* theta,
                             double* dtc_out, double* A_out) {
  API_BEGIN(ctx)
  ARGCHECK(prob && theta && dtc_out && A_out, "null argument");
  std::vector<DevProblem> P{prepare_problem(ctx, *prob, 0)};
  std::vector<Theta> th = thetas_from(theta, 1);
  GramOut go = run_gram_stage(ctx, P, th, /*fix_beta=*/true);
  DenseOut dn = run_dense(ctx, P, th, go, false);
  const DevProblem& p = P[0];
  const int64_t nch = p.nch;
  Finish2JobHost fj = finish_job(dn, go, p, 0, nch, ws<double>(ctx, "dtc_out", 1), nullptr);
  auto* dfj = ws<Finish2JobHost>(ctx, "finishjobs", 1);
  h2d(ctx, dfj, &fj, 1);
  launch_finish2(ctx->stream, dfj, 1, dn.ld, dn.nb);
  check_launch("finish");
  // A = L_u^{-1} beta^T (M x N), written column-major: A[i + j*m] -> transX with ldx = m
  double* A = ws<double>(ctx, "A_out", (size_t)p.m * p.n);
  TrsmJobHost tj{dn.Lu, dn.ld, ws<double>(ctx, "beta", 1), p.mp, A, p.m, (int)p.m, p.n, 1, 1};
  auto* dtj = ws<TrsmJobHost>(ctx, "trsmjobsA", 1);
  h2d(ctx, dtj, &tj, 1);
  launch_trsm(ctx->stream, dtj, 1, p.n);
  check_launch("trsm(A)");
  int st[2];
  d2h(ctx, st, dn.status, 2);
  d2h(ctx, dtc_out, fj.out, 1);
  if (prob->mem == GPAR_MEM_DEVICE)
    HIPCHECK(hipMemcpyAsync(A_out, A, (size_t)p.m * p.n * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
  else
    d2h(ctx, A_out, A, (size_t)p.m * p.n);
  sync(ctx);
  if (st[0] || st[1]) throw Error(GPAR_ERR_NOT_PD, "PosDefException: Cholesky failed");
  API_END(ctx)
}

int32_t gpar_q_u(gpar_ctx* ctx, const gpar_problem* prob, const double* theta, double* m_e,
                 double* cov, double* U_u) {
  API_BEGIN(ctx)
  ARGCHECK(prob && theta && m_e && cov && U_u, "null argument");
  std::vector<DevProblem> P{prepare_problem(ctx, *prob, 0)};
  std::vector<Theta> th = thetas_from(theta, 1);
  QuOut q = run_q_u(ctx, P[0], th[0]);
  const int64_t m = P[0].m;
  if (prob->mem == GPAR_MEM_DEVICE) {
    HIPCHECK(hipMemcpyAsync(m_e, q.me, m * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHECK(hipMemcpy2DAsync(cov, m * sizeof(double), q.cov, q.ld * sizeof(double), m * sizeof(double), m, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHECK(hipMemcpyAsync(U_u, q.Ucol, m * m * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
  } else {
    d2h(ctx, m_e, q.me, m);
    HIPCHECK(hipMemcpy2DAsync(cov, m * sizeof(double), q.cov, q.ld * sizeof(double), m * sizeof(double), m, hipMemcpyDeviceToHost, ctx->stream));
    d2h(ctx, U_u, q.Ucol, (size_t)m * m);
  }
  sync(ctx);
  API_END(ctx)
}

int32_t gpar_lgssm_logpdf(gpar_ctx* ctx, int32_t nchains, int64_t n, const double* t,
                          const double* y, int64_t ldy, int32_t kernel, const double* theta,
                          int32_t mem, double* lml_out) {
  API_BEGIN(ctx)
  ARGCHECK(nchains >= 1 && n >= 1 && t && y && theta && lml_out, "bad argument");
  ARGCHECK(ldy >= n, "ldy must be >= n");
  const int sdim = sde_dim(kernel);
  const double* dt = t;
  const double* dy = y;
  if (mem == GPAR_MEM_HOST) {
    check_sorted_host(t, n);
    double* tt = ws<double>(ctx, "lg_t", n);
    double* yy = ws<double>(ctx, "lg_y", (size_t)nchains * n);
    h2d(ctx, tt, t, n);
    HIPCHECK(hipMemcpy2DAsync(yy, n * sizeof(double), y, ldy * sizeof(double), n * sizeof(double), nchains, hipMemcpyHostToDevice, ctx->stream));
    dt = tt;
    dy = yy;
    ldy = n;
  }
  std::vector<double> lml(nchains);
  chains_logpdf(ctx, nchains, n, dt, dy, ldy, kernel, sdim, theta, lml.data());
  for (int i = 0; i < nchains; ++i) lml_out[i] = lml[i];
  API_END(ctx)
}

int32_t gpar_predict(gpar_ctx* ctx, const gpar_problem* prob, const double* theta,
                     int64_t n_star, const double* t_star, const double* v_star, int64_t ldvs,
                     int32_t mode, int32_t samples, uint64_t seed, double* mean, double* std) {
  API_BEGIN(ctx)
  ARGCHECK(prob && theta && t_star && v_star && mean && std, "null argument");
  ARGCHECK(n_star >= 1, "n_star must be >= 1");
  ARGCHECK(ldvs >= prob->d, "ldvs must be >= d");
  ARGCHECK(mode == GPAR_PREDICT_ANALYTIC || mode == GPAR_PREDICT_MC || mode == GPAR_PREDICT_PATH,
           "bad mode");
  if (mode != GPAR_PREDICT_ANALYTIC)
    ARGCHECK(samples >= 2 && samples <= kMaxSamples, "MC / path modes take 2..65536 samples");
  DevProblem P = prepare_problem(ctx, *prob, 0);
  std::vector<Theta> th = thetas_from(theta, 1);
  predict_impl(ctx, P, th[0], prob->mem, n_star, t_star, v_star, ldvs, mode, samples, seed, mean, std);
  API_END(ctx)
}

int32_t gpar_mc_normals(gpar_ctx* ctx, int32_t samples, int64_t m, uint64_t seed, double* xi_out) {
  API_BEGIN(ctx)
  ARGCHECK(xi_out, "null argument");
  ARGCHECK(samples >= 1 && samples <= kMaxSamples, "samples must be in 1..65536");
  ARGCHECK(m >= 1 && m <= (int64_t)1 << 20, "m out of range");
  double* xi = ws<double>(ctx, "mc_xi_export", (size_t)samples * m);
  launch_normal(ctx->stream, xi, m, samples, m, samples, seed);
  check_launch("normal draws");
  d2h(ctx, xi_out, xi, (size_t)samples * m);
  sync(ctx);
  API_END(ctx)
}

int32_t gpar_path_normals(gpar_ctx* ctx, int32_t samples, int64_t n, int32_t d, uint64_t seed,
                          double* xi_out) {
  API_BEGIN(ctx)
  ARGCHECK(xi_out, "null argument");
  ARGCHECK(samples >= 1 && samples <= kMaxSamples, "samples must be in 1..65536");
  ARGCHECK(d >= 1 && d <= 4 && n >= 1 && n * d <= ((int64_t)1 << 32) - 1, "n, d out of range");
  double* xi = ws<double>(ctx, "path_xi_export", (size_t)samples * n * d);
  launch_normal(ctx->stream, xi, n * d, samples, n * d, samples, path_seed(seed));
  check_launch("path normal draws");
  d2h(ctx, xi_out, xi, (size_t)samples * n * d);
  sync(ctx);
  API_END(ctx)
}

int32_t gpar_lgssm_posterior_rand(gpar_ctx* ctx, int64_t n, const double* t, const double* y,
                                  const double* noise, int32_t kernel, const double* theta,
                                  int32_t samples, uint64_t seed, int32_t mem, double* f_out) {
  API_BEGIN(ctx)
  ARGCHECK(n >= 1 && t && y && theta && f_out, "bad argument");
  ARGCHECK(samples >= 1 && samples <= kMaxSamples, "samples must be in 1..65536");
  ARGCHECK(mem == GPAR_MEM_HOST || mem == GPAR_MEM_DEVICE, "bad mem");
  ARGCHECK(n <= ((int64_t)1 << 32) / 3, "n out of range");
  const int sdim = sde_dim(kernel);
  std::vector<ChainParamsHost> cps = chain_params(theta, 1);
  const double *dt = t, *dy = y, *dn = noise;
  if (mem == GPAR_MEM_HOST) {
    check_sorted_host(t, n);
    double* tt = ws<double>(ctx, "lpr_t", n);
    double* yy = ws<double>(ctx, "lpr_y", n);
    h2d(ctx, tt, t, n);
    h2d(ctx, yy, y, n);
    if (noise) {
      double* nn = ws<double>(ctx, "lpr_noise", n);
      h2d(ctx, nn, noise, n);
      dn = nn;
    }
    dt = tt;
    dy = yy;
  }
  GainsOut g = run_gains(ctx, sdim, dt, n, cps, dn, false, "lpr");
  double* F = ws<double>(ctx, "lpr_F", (size_t)n * samples);
  path_samples(ctx, sdim, g, cps[0], dt, dn, n, dy, nullptr, 0, samples, seed, F);
  double* out = mem == GPAR_MEM_DEVICE ? f_out : ws<double>(ctx, "lpr_out", (size_t)n * samples);
  launch_path_transpose(ctx->stream, F, n, samples, out);
  check_launch("posterior_rand");
  if (mem == GPAR_MEM_HOST) d2h(ctx, f_out, out, (size_t)n * samples);
  sync(ctx);
  API_END(ctx)
}

int32_t gpar_lgssm_smooth(gpar_ctx* ctx, int32_t nchains, int64_t n, const double* t,
                          const double* y, int64_t ldy, const double* noise, int32_t kernel,
                          const double* theta, int32_t mem, double* mean, double* var) {
  API_BEGIN(ctx)
  ARGCHECK(nchains >= 1 && n >= 1 && t && y && theta && mean && var, "bad argument");
  ARGCHECK(ldy >= n, "ldy must be >= n");
  const int sdim = sde_dim(kernel);
  std::vector<ChainParamsHost> cps = chain_params(theta, nchains);
  const double *dt = t, *dy = y, *dn = noise;
  double *dm = mean, *dv = var;
  if (mem == GPAR_MEM_HOST) {
    check_sorted_host(t, n);
    double* tt = ws<double>(ctx, "ls_t", n);
    double* yy = ws<double>(ctx, "ls_y", (size_t)nchains * n);
    h2d(ctx, tt, t, n);
    HIPCHECK(hipMemcpy2DAsync(yy, n * sizeof(double), y, ldy * sizeof(double), n * sizeof(double), nchains, hipMemcpyHostToDevice, ctx->stream));
    if (noise) {
      double* nn = ws<double>(ctx, "ls_noise", n);
      h2d(ctx, nn, noise, n);
      dn = nn;
    }
    dt = tt;
    dy = yy;
    dm = ws<double>(ctx, "ls_mean", (size_t)nchains * n);
    dv = ws<double>(ctx, "ls_var", (size_t)nchains * n);
  }
  chains_smooth(ctx, nchains, n, dt, dy, mem == GPAR_MEM_HOST ? n : ldy, dn, sdim, cps, dm, dv,
                mem == GPAR_MEM_HOST ? n : ldy);
  if (mem == GPAR_MEM_HOST) {
    HIPCHECK(hipMemcpy2DAsync(mean, ldy * sizeof(double), dm, n * sizeof(double), n * sizeof(double), nchains, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHECK(hipMemcpy2DAsync(var, ldy * sizeof(double), dv, n * sizeof(double), n * sizeof(double), nchains, hipMemcpyDeviceToHost, ctx->stream));
  }
  sync(ctx);
  API_END(ctx)
}

int32_t gpar_sde_predictions(gpar_ctx* ctx, int32_t nchains, int64_t n, const double* t,
                             const double* y, int64_t ldy, int64_t n_star, const double* t_star,
                             int32_t kernel, const double* log_theta0,
                             const gpar_fit_options* opts, int32_t mem, double* theta_out,
                             double* mean, double* var) {
  API_BEGIN(ctx)
  ARGCHECK(nchains >= 1 && n >= 1 && n_star >= 1 && t && y && t_star && log_theta0 && theta_out &&
               mean && var, "bad argument");
  ARGCHECK(ldy >= n, "ldy must be >= n");
  const int sdim = sde_dim(kernel);
  gpar_fit_options o{0, 1000, 1e-8, 0.0};
  if (opts) o = *opts;
  // ---- inputs on device; test times ascending (host: stable-sorted here, un-permuted after)
  const double *dt = t, *dy = y, *dts = t_star;
  int64_t ldyd = ldy;
  std::vector<int64_t> perm;
  if (mem == GPAR_MEM_HOST) {
    check_sorted_host(t, n);
    double* tt = ws<double>(ctx, "sp_t", n);
    double* yy = ws<double>(ctx, "sp_y", (size_t)nchains * n);
    h2d(ctx, tt, t, n);
    HIPCHECK(hipMemcpy2DAsync(yy, n * sizeof(double), y, ldy * sizeof(double), n * sizeof(double), nchains, hipMemcpyHostToDevice, ctx->stream));
    perm.resize(n_star);
    for (int64_t i = 0; i < n_star; ++i) perm[i] = i;
    std::stable_sort(perm.begin(), perm.end(), [&](int64_t a, int64_t b) { return t_star[a] < t_star[b]; });
    std::vector<double> tsh(n_star);
    for (int64_t i = 0; i < n_star; ++i) tsh[i] = t_star[perm[i]];
    double* ts = ws<double>(ctx, "sp_ts", n_star);
    h2d(ctx, ts, tsh.data(), n_star);
    sync(ctx);
    dt = tt; dy = yy; dts = ts; ldyd = n;
  }
  // ---- NM fit of (l, process_var, noise_sigma) per chain on -logpdf (temporal_gp_inference.jl:69-82)
  std::vector<NelderMead> nm;
  nm.reserve(nchains);
  for (int i = 0; i < nchains; ++i)
    nm.emplace_back(std::vector<double>(log_theta0 + 3 * i, log_theta0 + 3 * i + 3), o.max_evals,
                    o.max_iterations, o.g_tol, o.time_limit);
  double* ysub = ws<double>(ctx, "sp_ysub", (size_t)nchains * n);
  while (true) {
    std::vector<int> act;
    for (int i = 0; i < nchains; ++i)
      if (!nm[i].done()) act.push_back(i);
    if (act.empty()) break;
    std::vector<double> th(3 * act.size());
    for (size_t a = 0; a < act.size(); ++a) {
      const auto& x = nm[act[a]].ask();
      for (int q = 0; q < 3; ++q) th[3 * a + q] = unpack(x[q]);
      HIPCHECK(hipMemcpyAsync(ysub + a * n, dy + (size_t)act[a] * ldyd, n * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    }
    std::vector<double> lml(act.size());
    chains_logpdf(ctx, (int)act.size(), n, dt, ysub, n, kernel, sdim, th.data(), lml.data());
    for (size_t a = 0; a < act.size(); ++a) {
      double f = -lml[a];
      if (!std::isfinite(f)) f = INFINITY;
      nm[act[a]].tell(f);
    }
  }
  std::vector<double> theta(3 * nchains);
  for (int i = 0; i < nchains; ++i)
    for (int q = 0; q < 3; ++q) theta[3 * i + q] = theta_out[3 * i + q] = unpack(nm[i].x_min()[q]);
  // ---- merged grid: y* = y (train) / 0 (test), R = sigma_c^2 (train, -1 flag) / 1e10 (test)
  const int64_t nt = n + n_star;
  double* tm = ws<double>(ctx, "sp_tm", nt);
  double* ym = ws<double>(ctx, "sp_ym", (size_t)nchains * nt);
  double* rm = ws<double>(ctx, "sp_rm", nt);
  double* dummy = ws<double>(ctx, "sp_dummy", nt);
  int64_t* ptr = ws<int64_t>(ctx, "sp_ptr", n);
  int64_t* pts = ws<int64_t>(ctx, "sp_pts", n_star);
  launch_merge_side(ctx->stream, dt, n, dts, n_star, 0, nullptr, -1.0, dt, 1, 0, tm, dummy, rm, dummy, 1, ptr);
  launch_merge_side(ctx->stream, dts, n_star, dt, n, 1, nullptr, 1e10, dts, 1, 0, tm, dummy, rm, dummy, 1, pts);
  HIPCHECK(hipMemsetAsync(ym, 0, (size_t)nchains * nt * sizeof(double), ctx->stream));
  launch_scatter_chains(ctx->stream, dy, ldyd, n, ptr, ym, nt, nchains);
  double* mm = ws<double>(ctx, "sp_mean", (size_t)nchains * nt);
  double* vv = ws<double>(ctx, "sp_var", (size_t)nchains * nt);
  chains_smooth(ctx, nchains, nt, tm, ym, nt, rm, sdim, chain_params(theta.data(), nchains), mm, vv, nt);
  double* om = ws<double>(ctx, "sp_om", (size_t)nchains * n_star);
  double* ov = ws<double>(ctx, "sp_ov", (size_t)nchains * n_star);
  launch_gather_chains(ctx->stream, mm, nt, n_star, pts, om, n_star, nchains);
  launch_gather_chains(ctx->stream, vv, nt, n_star, pts, ov, n_star, nchains);
  check_launch("sde_predictions");
  if (mem == GPAR_MEM_DEVICE) {
    HIPCHECK(hipMemcpyAsync(mean, om, (size_t)nchains * n_star * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHECK(hipMemcpyAsync(var, ov, (size_t)nchains * n_star * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    sync(ctx);
  } else {
    std::vector<double> hm((size_t)nchains * n_star), hv((size_t)nchains * n_star);
    d2h(ctx, hm.data(), om, hm.size());
    d2h(ctx, hv.data(), ov, hv.size());
    sync(ctx);
    for (int b = 0; b < nchains; ++b)
      for (int64_t i = 0; i < n_star; ++i) {
        mean[(size_t)b * n_star + perm[i]] = hm[(size_t)b * n_star + i];
        var[(size_t)b * n_star + perm[i]] = hv[(size_t)b * n_star + i];
      }
  }
  API_END(ctx)
}

// ---------------------------------------------------------------- exact GP / GPAR (a10)
namespace gpar {
struct ExactIn {
  const double* x;   // device, point-major, ld dx
  const double* y;   // device
  double inv_lt, s_t, inv_lo, s_o, s2;
};

// theta: (l_t, time_var, l_o, out_var, sigma); dx == 1 uses entries 0, 1, 4 (optimized.jl:28-36).
static ExactIn exact_prepare(gpar_ctx* c, int64_t n, int64_t dx, const double* x, int64_t ldx,
                             const double* y, int32_t tk, int32_t ok, const double* theta,
                             int32_t mem, const char* tag) {
  ARGCHECK(n >= 1 && n <= 2048, "exact GP supports 1 <= n <= 2048");
  ARGCHECK(dx >= 1 && ldx >= dx && x && y && theta, "bad argument");
  ARGCHECK(tk >= GPAR_MATERN12 && tk <= GPAR_EQ && ok >= GPAR_MATERN12 && ok <= GPAR_EQ,
           "unknown kernel");
  ARGCHECK(mem == GPAR_MEM_HOST || mem == GPAR_MEM_DEVICE, "bad mem");
  const int used[3] = {0, 1, 4};
  for (int q : used) ARGCHECK(std::isfinite(theta[q]) && theta[q] > 0.0, "theta entries must be positive");
  if (dx > 1)
    for (int q = 2; q < 4; ++q) ARGCHECK(std::isfinite(theta[q]) && theta[q] > 0.0, "theta entries must be positive");
  ExactIn e;
  e.inv_lt = 1.0 / theta[0];
  e.s_t = theta[1] * theta[1];
  e.inv_lo = dx > 1 ? 1.0 / theta[2] : 0.0;
  e.s_o = dx > 1 ? theta[3] * theta[3] : 0.0;
  e.s2 = theta[4] * theta[4];
  if (mem == GPAR_MEM_HOST) {
    double* xx = ws<double>(c, std::string(tag) + "_x", (size_t)n * dx);
    double* yy = ws<double>(c, std::string(tag) + "_y", (size_t)n);
    HIPCHECK(hipMemcpy2DAsync(xx, dx * sizeof(double), x, ldx * sizeof(double), dx * sizeof(double),
                              n, hipMemcpyHostToDevice, c->stream));
    h2d(c, yy, y, n);
    e.x = xx;
    e.y = yy;
  } else {
    ARGCHECK(ldx == dx, "device inputs must be dense (ldx == dx)");
    e.x = x;
    e.y = y;
  }
  return e;
}

// L = chol(K(x, x) + s2 I) (row-major n x n in ws "ex_L"), w = L^{-1} y.
static void exact_factor(gpar_ctx* c, const ExactIn& e, int64_t n, int64_t dx, int32_t tk,
                         int32_t ok, double** L_out, double** w_out, int** status_out) {
  double* L = ws<double>(c, "ex_L", (size_t)n * n);
  double* w = ws<double>(c, "ex_w", (size_t)n);
  int* status = ws<int>(c, "ex_status", 1);
  HIPCHECK(hipMemsetAsync(status, 0, sizeof(int), c->stream));
  Timed tm_(c, "exact");
  launch_exact_cov(c->stream, e.x, dx, n, e.x, dx, n, (int)dx, tk, ok, e.inv_lt, e.s_t, e.inv_lo,
                   e.s_o, e.s2, L, n);
  check_launch("exact_cov");
  CholJobHost cj{L, n, (int)n, 0.0, status};
  auto* dcj = ws<CholJobHost>(c, "ex_chol", 1);
  h2d(c, dcj, &cj, 1);
  launch_chol(c->stream, dcj, 1);
  check_launch("exact chol");
  TrsvJobHost tj{L, n, (int)n, e.y, w, 0};
  auto* dtj = ws<TrsvJobHost>(c, "ex_trsv", 1);
  h2d(c, dtj, &tj, 1);
  launch_trsv(c->stream, dtj, 1);
  check_launch("exact trsv");
  *L_out = L;
  *w_out = w;
  *status_out = status;
}

static void exact_check_pd(gpar_ctx* c, const int* status) {
  int st = 0;
  d2h(c, &st, status, 1);
  sync(c);
  if (st) throw Error(GPAR_ERR_NOT_PD, "cholesky: K + sigma^2 I is not positive definite");
}
}  // namespace gpar

int32_t gpar_exact_logpdf(gpar_ctx* ctx, int64_t n, int64_t dx, const double* x, int64_t ldx,
                          const double* y, int32_t time_kernel, int32_t out_kernel,
                          const double* theta, int32_t mem, double* lml_out) {
  API_BEGIN(ctx)
  ARGCHECK(lml_out, "null output");
  ExactIn e = exact_prepare(ctx, n, dx, x, ldx, y, time_kernel, out_kernel, theta, mem, "exl");
  double *L, *w;
  int* status;
  exact_factor(ctx, e, n, dx, time_kernel, out_kernel, &L, &w, &status);
  double* dout = ws<double>(ctx, "ex_out", 1);
  launch_exact_logpdf_finish(ctx->stream, L, n, (int)n, w, status, dout);
  check_launch("exact finish");
  exact_check_pd(ctx, status);
  d2h(ctx, lml_out, dout, 1);
  sync(ctx);
  API_END(ctx)
}

int32_t gpar_exact_posterior(gpar_ctx* ctx, int64_t n, int64_t dx, const double* x, int64_t ldx,
                             const double* y, int64_t n_star, const double* x_star,
                             int64_t ldxs, int32_t time_kernel, int32_t out_kernel,
                             const double* theta, int32_t mem, double* mean, double* var) {
  API_BEGIN(ctx)
  ARGCHECK(n_star >= 1 && x_star && ldxs >= dx && mean && var, "bad argument");
  ExactIn e = exact_prepare(ctx, n, dx, x, ldx, y, time_kernel, out_kernel, theta, mem, "exp");
  const double* xs = x_star;
  if (mem == GPAR_MEM_HOST) {
    double* xx = ws<double>(ctx, "exp_xs", (size_t)n_star * dx);
    HIPCHECK(hipMemcpy2DAsync(xx, dx * sizeof(double), x_star, ldxs * sizeof(double),
                              dx * sizeof(double), n_star, hipMemcpyHostToDevice, ctx->stream));
    xs = xx;
  } else {
    ARGCHECK(ldxs == dx, "device inputs must be dense (ldxs == dx)");
  }
  double *L, *w;
  int* status;
  exact_factor(ctx, e, n, dx, time_kernel, out_kernel, &L, &w, &status);
  double* Ks = ws<double>(ctx, "ex_Ks", (size_t)n * n_star);
  double* W = ws<double>(ctx, "ex_W", (size_t)n * n_star);
  launch_exact_cov(ctx->stream, e.x, dx, n, xs, dx, n_star, (int)dx, time_kernel, out_kernel,
                   e.inv_lt, e.s_t, e.inv_lo, e.s_o, 0.0, Ks, n_star);
  check_launch("exact cross cov");
  TrsmJobHost tj{L, n, Ks, n_star, W, n_star, (int)n, n_star, 0, 0};
  auto* dtj = ws<TrsmJobHost>(ctx, "ex_trsm", 1);
  h2d(ctx, dtj, &tj, 1);
  launch_trsm(ctx->stream, dtj, 1, n_star);
  check_launch("exact trsm");
  double* dm = mean;
  double* dv = var;
  if (mem == GPAR_MEM_HOST) {
    dm = ws<double>(ctx, "exp_mean", n_star);
    dv = ws<double>(ctx, "exp_var", n_star);
  }
  launch_exact_post(ctx->stream, W, n_star, (int)n, n_star, w, e.s_t + e.s_o, dm, dv);
  check_launch("exact posterior");
  exact_check_pd(ctx, status);
  if (mem == GPAR_MEM_HOST) {
    d2h(ctx, mean, dm, n_star);
    d2h(ctx, var, dv, n_star);
  }
  sync(ctx);
  API_END(ctx)
}

// ---------------------------------------------------------------- host-only Nelder-Mead
struct gpar_nm {
  gpar::NelderMead nm;
};

int32_t gpar_nm_create(int32_t n, const double* x0, const gpar_fit_options* opts, gpar_nm** out) {
  if (!out || !x0 || n < 1) return GPAR_ERR_ARG;
  gpar_fit_options o{0, 1000, 1e-8, 0.0};
  if (opts) o = *opts;
  *out = new gpar_nm{gpar::NelderMead(std::vector<double>(x0, x0 + n), o.max_evals,
                                      o.max_iterations, o.g_tol, o.time_limit)};
  return GPAR_OK;
}

int32_t gpar_nm_destroy(gpar_nm* nm) {
  delete nm;
  return GPAR_OK;
}

int32_t gpar_nm_ask(gpar_nm* nm, double* x) {
  if (!nm || !x) return -1;
  if (nm->nm.done()) return 0;
  const auto& p = nm->nm.ask();
  std::copy(p.begin(), p.end(), x);
  return 1;
}

int32_t gpar_nm_tell(gpar_nm* nm, double f) {
  if (!nm || nm->nm.done()) return GPAR_ERR_STATE;
  nm->nm.tell(f);
  return GPAR_OK;
}

int32_t gpar_nm_result(const gpar_nm* nm, double* x_min, double* f_min, int32_t* evals,
                       int32_t* iterations) {
  if (!nm) return GPAR_ERR_STATE;
  const auto& x = nm->nm.x_min();
  if (x_min) std::copy(x.begin(), x.end(), x_min);
  if (f_min) *f_min = nm->nm.f_min();
  if (evals) *evals = nm->nm.evals();
  if (iterations) *iterations = nm->nm.iterations();
  return GPAR_OK;
}

}  // extern "C"
