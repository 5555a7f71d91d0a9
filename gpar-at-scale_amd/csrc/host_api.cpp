// host_api.cpp -- context lifetime, options, telemetry and gpar_dtc_objective.
#include "host.hpp"

#include <cctype>

namespace gpar {

// Entry: order the context's streams after the caller's input stream (if one was set).
void enter(gpar_ctx* c) {
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
int fail(gpar_ctx* c, int code, const char* what) {
  c->err = what;
  c->stream = c->main;
  (void)hipStreamSynchronize(c->main);
  (void)hipStreamSynchronize(c->own_side);
  for (hipStream_t st : c->own_s)
    if (st) (void)hipStreamSynchronize(st);
  (void)hipGetLastError();
  return code;
}

// The stream handles launches use: the created streams, or all `main` when serialized.
static void route_streams(gpar_ctx* c) {
  c->side = c->serialize ? c->main : c->own_side;
  hipStream_t* act[4] = {&c->s_w, &c->s_g, &c->s_g2, &c->s_d};
  for (int i = 0; i < 4; ++i) *act[i] = (c->serialize && c->own_s[i]) ? c->main : c->own_s[i];
}

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
    for (hipStream_t& st : c->own_s)
      if (st) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
        st = nullptr;
      }
    route_streams(c);
    c->split_mask_w = 0;
    c->split_w = 0;
    // own_s: s_w (whitening), s_g (Gram), s_g2 (its co-running correction), s_d (dense tails)
    uint32_t mw[8] = {0}, mg[8] = {0};
    for (int i = 0; i < 256; ++i) (i < 8 * w ? mw : mg)[i / 32] |= 1u << (i % 32);
    const uint32_t* masks[4] = {mw, mg, mg, mw};
    for (int i = 0; i < 4; ++i)
      if (hipExtStreamCreateWithCUMask(&c->own_s[i], 8, masks[i]) != hipSuccess) return GPAR_ERR_HIP;
    route_streams(c);
    if (!c->ev_sp &&
        (hipEventCreateWithFlags(&c->ev_gd[0], hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&c->ev_gd[1], hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&c->ev_sp, hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&c->ev_dn, hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&c->ev_gr, hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&c->ev_wd, hipEventDisableTiming) != hipSuccess))
      return GPAR_ERR_HIP;
    c->split_mask_w = w;
  }
  c->split_w = w;
  c->split_forced = forced;
  return GPAR_OK;
}

// Every knob's non-default values are supported modes (round 5 deleted the A/B-only ones: the
// split round head's variants, the dense prefix on a stream of its own, the DG share, the round
// overlap's tail placement and the prediction's distance-pass whitening, each measured slower).
static constexpr const char* kScheduleKnobs[] = {"overlap", "overlap_group", "predict_fused",
                                                  "qu_batch", "dense_early", "predict_lanes",
                                                  "serialize", "post_gram", "compact_rec",
                                                  "dg_rows_w", "gram_group", "fit_chunks",
                                                  "device_nm"};

// gpar_ctx_set_schedule / gpar_ctx_get_schedule (GPAR_ERR_ARG: unknown knob or value).
static int set_schedule(gpar_ctx* c, const std::string& k, int v) {
  if (k == "overlap") c->overlap = v != 0;
  else if (k == "overlap_group") {
    if (v < 0) return GPAR_ERR_ARG;
    c->overlap_group = v;
  }
  else if (k == "predict_fused") c->predict_fused = v != 0;
  else if (k == "qu_batch") c->qu_batch = v != 0;
  else if (k == "dense_early") {
    if (v < 0 || v > 1) return GPAR_ERR_ARG;
    c->dense_early = (int)v;
  }
  else if (k == "dg_rows_w") {
    if ((v < -50 || v > 100) && v != kDgRowsAuto) return GPAR_ERR_ARG;
    c->dg_rows_w = v;
  } else if (k == "compact_rec") {
    if (v < -1 || v > 1) return GPAR_ERR_ARG;
    c->compact_rec = v;
  }
  else if (k == "gram_group") {
    if (v < -1 || v > 64) return GPAR_ERR_ARG;
    c->gram_group = v;
  }
  else if (k == "fit_chunks") {
    if (v < -1 || v > 4096) return GPAR_ERR_ARG;
    c->fit_chunks = v;
  }
  else if (k == "device_nm") {
    if (v < 0 || v > 1) return GPAR_ERR_ARG;
    c->device_nm = v;
  }
  else if (k == "post_gram") {
    if (v < -1 || v > 1) return GPAR_ERR_ARG;
    c->post_gram = v;
  }
  else if (k == "predict_lanes") {
    if (v != 1 && v != 2) return GPAR_ERR_ARG;
    c->predict_lanes = v;
  } else if (k == "serialize") {
    // the streams about to be re-routed must not hold queued work
    (void)hipStreamSynchronize(c->main);
    (void)hipStreamSynchronize(c->own_side);
    for (hipStream_t st : c->own_s)
      if (st) (void)hipStreamSynchronize(st);
    c->serialize = v != 0;
    route_streams(c);
  } else {
    return GPAR_ERR_ARG;
  }
  return GPAR_OK;
}

static int get_schedule(const gpar_ctx* c, const std::string& k, int32_t* v) {
  if (k == "overlap") *v = c->overlap;
  else if (k == "overlap_group") *v = c->overlap_group;
  else if (k == "predict_fused") *v = c->predict_fused;
  else if (k == "qu_batch") *v = c->qu_batch;
  else if (k == "dense_early") *v = c->dense_early;
  else if (k == "post_gram") *v = c->post_gram;
  else if (k == "compact_rec") *v = c->compact_rec;
  else if (k == "dg_rows_w") *v = c->dg_rows_w;
  else if (k == "gram_group") *v = c->gram_group;
  else if (k == "fit_chunks") *v = c->fit_chunks;
  else if (k == "device_nm") *v = c->device_nm;
  else if (k == "predict_lanes") *v = c->predict_lanes;
  else if (k == "serialize") *v = c->serialize;
  else return GPAR_ERR_ARG;
  return GPAR_OK;
}
}  // namespace gpar
using namespace gpar;
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
      hipStreamCreateWithFlags(&c->own_side, hipStreamNonBlocking) != hipSuccess ||
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
  route_streams(c);
  // schedule knobs from the environment (GPAR_OVERLAP=0, GPAR_SERIALIZE=1, ...)
  for (const char* k : kScheduleKnobs) {
    std::string env = "GPAR_";
    for (const char* q = k; *q; ++q) env += (char)std::toupper((unsigned char)*q);
    if (const char* e = std::getenv(env.c_str())) (void)set_schedule(c, k, std::atoi(e));
  }
  // GPAR_SPLIT_CUS overrides the default CU split
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
  (void)hipStreamSynchronize(ctx->own_side);
  for (auto& kv : ctx->bufs)
    if (kv.second.p) (void)hipFree(kv.second.p);
  (void)hipEventDestroy(ctx->ev_fork);
  (void)hipEventDestroy(ctx->ev_join);
  (void)hipEventDestroy(ctx->ev_input);
  (void)hipEventDestroy(ctx->ev_pw);
  (void)hipEventDestroy(ctx->ev_pc[0]);
  (void)hipEventDestroy(ctx->ev_pc[1]);
  {
    for (hipStream_t st : ctx->own_s)
      if (st) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
      }
    for (hipEvent_t ev : {ctx->ev_gd[0], ctx->ev_gd[1], ctx->ev_sp, ctx->ev_dn,
                          ctx->ev_gr, ctx->ev_wd, ctx->ev_prep_ready[0],
                          ctx->ev_prep_ready[1], ctx->ev_prep_free[0], ctx->ev_prep_free[1]})
      if (ev) (void)hipEventDestroy(ev);
    for (const auto* evs : {&ctx->ev_grp, &ctx->ev_gn})
      for (hipEvent_t ev : *evs)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& s : ctx->stage)
      if (s.host) (void)hipHostFree(s.host);
  }
  (void)hipStreamDestroy(ctx->own_side);
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

int64_t gpar_debug_counter(const char* name) {
  if (!name) return -1;
  if (std::strcmp(name, "gains_fast") == 0) return g_gains_fast_launches.load();
  if (std::strcmp(name, "gains_general") == 0) return g_gains_general_launches.load();
  return -1;
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

int32_t gpar_ctx_set_schedule(gpar_ctx* ctx, const char* knob, int32_t value) {
  if (!ctx) return GPAR_ERR_STATE;
  const int rc = knob ? set_schedule(ctx, knob, value) : GPAR_ERR_ARG;
  if (rc != GPAR_OK)
    ctx->err = std::string("gpar_ctx_set_schedule: unknown knob or bad value: ") + (knob ? knob : "(null)");
  return rc;
}

int32_t gpar_ctx_get_schedule(const gpar_ctx* ctx, const char* knob, int32_t* value) {
  if (!ctx) return GPAR_ERR_STATE;
  if (!knob || !value) return GPAR_ERR_ARG;
  return get_schedule(ctx, knob, value);
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
  P = prepare_batch(ctx, probs, nprob);
  std::vector<Theta> th = thetas_from(theta, nprob);
  std::vector<int> st;
  eval_dtc(ctx, P, th, dtc_out, st);
  for (int i = 0; i < nprob; ++i)
    if (st[i])
      throw Error(GPAR_ERR_NOT_PD, "PosDefException: Cholesky failed for output " + std::to_string(i));
  API_END(ctx)
}
}  // extern "C"
