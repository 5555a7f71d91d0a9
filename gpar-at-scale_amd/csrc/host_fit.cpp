// host_fit.cpp -- the batched Nelder-Mead fit: distance cache, round-overlapping schedule,
// gpar_fit, and the host-only ask/tell optimiser.
#include "host.hpp"

namespace gpar {

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
int64_t fit_ws_estimate(const gpar_ctx* c, const std::vector<DevProblem>& P) {
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
int64_t predict_ws_estimate(int64_t n, int64_t n_star, int64_t mp, int64_t d, int mode,
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
std::vector<DevProblem> attach_dist_cache(gpar_ctx* c, const std::vector<DevProblem>& P,
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
    {
      Timed td_(c, "dist2", 2.0 * (double)p.n * (double)p.mp * (double)p.d);
      launch_dist2(c->stream, p.ok, p.v, p.ldv, p.n, p.z, p.ldz, p.m, p.mp, (int)p.d, p.zc, d2,
                   p.mp, /*take_sqrt=*/p.ok != GPAR_EQ);
    }
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
// one 8-way shard of the north job (8 outputs per call, two groups of 4) 2.70 -> 2.45 s per step.
// With all 63 north outputs in two groups of 32 the round is long and each group's burst of gains
// and dense tails on the whitening CUs slowed every Gram instead (5.13 -> 5.46 ms; 18.45 vs
// 18.75 s per job, profiles/bench_r03d_*.json); groups of gpar_ctx::overlap_group outputs spread
// that work over the round.  Auto (overlap_group 0): groups of kOverlapGroupAuto in calls of up to
// kOverlapMaxOutputs outputs; larger calls keep the round-by-round schedule.
constexpr int kOverlapMaxOutputs = 16;
constexpr int kOverlapGroupAuto = 8;

using AcceptFn = std::function<void(int, double, const double*, const double*, int64_t)>;

static void fit_overlapped(gpar_ctx* c, const std::vector<DevProblem>& P,
                           std::vector<NelderMead>& nm, const AcceptFn& accept) {
  const int np = (int)P.size();
  const int64_t n = P[0].n, nch = P[0].nch, npart = vec_fix_blocks(n);
  int64_t mpmax = 0;
  for (auto& p : P) mpmax = std::max(mpmax, p.mp);
  const size_t sq = (size_t)mpmax * mpmax;
  // K groups of about overlap_group outputs (at least two), dealt round-robin
  const int gs = c->overlap_group > 0 ? c->overlap_group : kOverlapGroupAuto;
  const int K = std::max(2, (np + gs - 1) / gs);
  for (auto* evs : {&c->ev_grp, &c->ev_gn})
    while ((int)evs->size() < K) {
      hipEvent_t ev;
      HIPCHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      evs->push_back(ev);
    }
  if ((int)c->stage.size() < K) c->stage.resize(K);   // no arena is in use between calls
  std::vector<OverlapGroup> grp(K);
  for (int i = 0; i < np; ++i) grp[i % K].members.push_back(i);
  for (int g = 0; g < K; ++g) {
    OverlapGroup& G = grp[g];
    G.id = g;
    const size_t cap = G.members.size();
    const std::string sfx = "g" + std::to_string(g);
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

  // compact gains records (compact_rec -1 = auto) when every output already whitens through
  // whiten_kfu_d2x2 (cached distances, or inputs wider than the fused kernels take): an uncached
  // narrow output would otherwise switch from the fused whitening to the distance pass (last bits)
  bool all_d2 = true;
  for (const auto& p : P) all_d2 = all_d2 && (cached_d2(c, p) || p.d > kFusedMaxD);
  const bool compact = c->compact_rec == 1 || (c->compact_rec == -1 && all_d2);
  SplitPipe sp(c, n, mpmax);
  // the short chains on the Gram CUs: the whitening CUs also run the other group's dense tails and
  // gains here (one 8-output shard of the north job: 2.356 -> 2.329 s per step, r04p; the
  // round-by-round 63-output fit is slower with it, 17.75 -> 18.69 s)
  sp.post_gram = c->post_gram != 0;
  sp.dg_rows_w = c->dg_rows_w == kDgRowsAuto ? 20 : c->dg_rows_w;
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
    // compact records (auto): the gains beside the other group's whitenings write 72 instead of
    // 168 bytes per step, the 8-output shard 2.329 -> 2.296 s per step (r04w)
    // the gains run on the whitening CUs beside the other group's whitenings (s_d), not in the
    // whitening stream's order: queued there they delayed the next whitening, and with it the
    // DG share that ends the previous Gram
    GainsOut gn;
    {
      OnStream on_(c, c->s_d);
      StagingScope st_(c, G.id);
      gn = run_gains(c, P[0].sdim, P[0].t, n, cps, nullptr, false, "fitg" + std::to_string(G.id),
                     &ys, G.alpha_all, G.asend_all, compact);
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
  for (auto& G : grp) begin_round(G);
  auto any_in_flight = [&]() {
    for (const auto& G : grp)
      if (G.in_flight) return true;
    return false;
  };
  for (int g = 0; any_in_flight(); g = (g + 1) % K) {
    if (!grp[g].in_flight) continue;
    finish_round(grp[g]);
    begin_round(grp[g]);
  }
  sp.flush();
  sp.join(c->main);
}

// ---------------------------------------------------------------- unsplit round overlap
// The same idea for the batched fits that do not take the CU split (N Mp^2 < 1e11: the dtc and eeg
// configs, one rank's eeg shard), whose rounds run eval_dtc's unsplit schedule with the grouped
// Gram.  There a round is one grouped Gram (3.8 ms for a rank's 8 eeg outputs) and a boundary of
// about as long of latency-bound work -- the dense tail's 64 x 64 launches, the host's simplex
// step, the next round's gains, whitenings and chunk carries (profiles/trace_eeg_shard0of8_r06m_gaps.txt).
// The outputs are dealt round-robin into K groups (2, or groups of overlap_group outputs); each
// group's rounds run on streams of their own (group 0: the context's main / side / dense streams,
// the others three each) with workspaces of their own (ws_suffix; the distance cache is shared and
// only read) and pinned upload arenas, and eval_dtc returns as soon as a round is queued (its values
// land in pinned memory behind an event).  The host takes the groups in turn: wait for a group's
// values, step its simplices, queue its next round -- which then runs beside the other groups'
// rounds, one group's boundary under another's Gram.  Every output evaluates the points its own
// simplex asks for with the same kernels; only its group's grouped-Gram plan (sized for the
// group's outputs) differs from the one-group round, so the fit matches the round-by-round one
// within rounding, and bit for bit its serialized twin (every group on the main stream).
// Measured (r06ov1/2, one box): a rank's eeg shard (8 outputs, M = 512) 407 / 410 -> 393 / 397 ms
// per step with two groups of 4 -- the groups' Grams slow 1.75 -> 2.7 ms beside the other group's
// whitenings (the fp64 pipe they share), which eats most of the boundary they hide; four groups of
// 2: 576 ms, three: 554 ms (every group pays the boundary's launch chains); the 1-GPU eeg job (two
// groups of 32) 2398 -> 2350 / 2414 ms (noise); dtc (M = 256, its Gram a third of its round)
// 167 -> 172 ms.  So: two groups, calls of 4..16 outputs with Mp >= 512 (or any overlap_group).
constexpr int kOverlapUnsplitMax = 16;
constexpr int64_t kOverlapUnsplitMinMp = 512;

static void fit_overlapped_unsplit(gpar_ctx* c, const std::vector<DevProblem>& P,
                                   std::vector<NelderMead>& nm, const AcceptFn& accept) {
  const int np = (int)P.size();
  const int K = c->overlap_group > 0 ? std::max(2, (np + c->overlap_group - 1) / c->overlap_group) : 2;
  struct UGroup {
    int id = 0;
    std::vector<int> members, act;
    std::vector<Theta> th;
    std::vector<DevProblem> sub;
    GramOut go{};
    hipStream_t st[3] = {nullptr, nullptr, nullptr};   // main, side, dense
    double* hout = nullptr;
    int* hstat = nullptr;
    hipEvent_t done = nullptr;
    size_t res_bytes = 0;
    bool in_flight = false;
  };
  std::vector<UGroup> grp(K);
  for (int i = 0; i < np; ++i) grp[i % K].members.push_back(i);
  // streams and events made here are released on every exit, after their work
  struct Owned {
    std::vector<hipStream_t> st;
    std::vector<hipEvent_t> ev;
    ~Owned() {
      for (hipStream_t s : st) {
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
      }
      for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }
  } own;
  auto make_stream = [&]() {
    if (c->serialize) return c->main;   // the order-free twin: every group on the main stream
    hipStream_t s;
    HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    own.st.push_back(s);
    return s;
  };
  if ((int)c->stage.size() < K) c->stage.resize(K);   // no arena is in use between calls
  HIPCHECK(hipEventRecord(c->ev_fork, c->main));   // the inputs and the distance cache, on main
  for (int g = 0; g < K; ++g) {
    UGroup& G = grp[g];
    G.id = g;
    if (g == 0) {
      G.st[0] = c->main;
      G.st[1] = c->side;
      G.st[2] = c->s_d;
    } else {
      for (hipStream_t& s : G.st) {
        s = make_stream();
        HIPCHECK(hipStreamWaitEvent(s, c->ev_fork, 0));
      }
    }
    HIPCHECK(hipEventCreateWithFlags(&G.done, hipEventDisableTiming));
    own.ev.push_back(G.done);
    const size_t cap = G.members.size();
    gpar_ctx::Staging& a = c->stage[g];
    const size_t vbytes = (cap * sizeof(double) + 255) & ~(size_t)255;
    G.res_bytes = vbytes + ((2 * cap * sizeof(int) + 255) & ~(size_t)255);
    const size_t need = G.res_bytes + ((size_t)1 << 20) + cap * 4096;
    if (a.cap < need) {
      if (a.host) HIPCHECK(hipHostFree(a.host));
      a.host = nullptr;
      a.cap = 0;
      HIPCHECK(hipHostMalloc((void**)&a.host, need, hipHostMallocDefault));
      a.cap = need;
    }
    G.hout = reinterpret_cast<double*>(a.host);
    G.hstat = reinterpret_cast<int*>(a.host + vbytes);
  }
  // a group's streams, workspaces and upload arena, for the scope of its launches
  struct GroupScope {
    gpar_ctx* c;
    hipStream_t saved[4];
    std::string sfx;
    GroupScope(gpar_ctx* c_, const UGroup& G) : c(c_) {
      saved[0] = c->stream;
      saved[1] = c->main;
      saved[2] = c->side;
      saved[3] = c->s_d;
      c->stream = c->main = G.st[0];
      c->side = G.st[1];
      c->s_d = G.st[2];
      sfx = c->ws_suffix;
      if (G.id > 0) c->ws_suffix = sfx + "~ov" + std::to_string(G.id);
      c->staging = &c->stage[G.id];
    }
    ~GroupScope() {
      c->stream = saved[0];
      c->main = saved[1];
      c->side = saved[2];
      c->s_d = saved[3];
      c->ws_suffix = sfx;
      c->staging = nullptr;
    }
  };
  auto issue = [&](UGroup& G) {
    G.act.clear();
    for (int i : G.members)
      if (!nm[i].done()) G.act.push_back(i);
    if (G.act.empty()) return;
    G.th.clear();
    G.sub.clear();
    for (int i : G.act) {
      const auto& x = nm[i].ask();
      G.th.push_back({unpack(x[0]), unpack(x[1]), unpack(x[2]), unpack(x[3]), unpack(x[4])});
      G.sub.push_back(P[i]);
    }
    c->stage[G.id].used = G.res_bytes;   // the previous round's uploads have been consumed
    GroupScope gs_(c, G);
    const EvalAsync as{G.hout, G.hstat, G.done};
    std::vector<int> unused;
    eval_dtc(c, G.sub, G.th, nullptr, unused, &G.go, &as);
    G.in_flight = true;
  };
  auto finish = [&](UGroup& G) {
    HIPCHECK(hipEventSynchronize(G.done));
    OnStream on_(c, G.st[0]);   // a kept point's Gram copy, ahead of the group's next round
    const size_t sq = (size_t)G.go.ldg * G.go.ldg;
    for (size_t a = 0; a < G.act.size(); ++a) {
      double f = -G.hout[a];
      if (G.hstat[2 * a] || G.hstat[2 * a + 1] || !std::isfinite(f)) f = INFINITY;
      accept(G.act[a], f, G.go.G + a * sq, G.go.r + a * G.go.ldg, G.go.ldg);
    }
    G.in_flight = false;
  };
  for (auto& G : grp) issue(G);
  auto any_in_flight = [&]() {
    for (const auto& G : grp)
      if (G.in_flight) return true;
    return false;
  };
  for (int g = 0; any_in_flight(); g = (g + 1) % K) {
    if (!grp[g].in_flight) continue;
    finish(grp[g]);
    issue(grp[g]);
  }
  // the context's stream follows every group's work (kept Grams, the streams released above)
  for (int g = 1; g < K; ++g)
    for (hipStream_t s : grp[g].st)
      if (s != c->main) {
        HIPCHECK(hipEventRecord(c->ev_join, s));
        HIPCHECK(hipStreamWaitEvent(c->main, c->ev_join, 0));
      }
}

// Cache-resident sub-batches.  The batched fit evaluates every output once per Nelder-Mead round,
// so an output's cached distances are only reused if the cache holds the whole batch; where it
// cannot (BASELINE config 5: N = 1e7, M = 1024, 82 GB of distances per output, 32 outputs per
// rank), the uncached outputs recompute their distances every evaluation (a pass of 2 N Mp D
// flops: at D = 255 more than half the Gram's; 27 % of the r06a stress step).  Each output's fit
// is independent of the batch it runs in, so the fit runs instead in consecutive sub-batches whose
// distances all fit, each computing them once.  Returns the sub-batches (output indices), or none
// for one batch.  Auto (fit_chunks -1): where the fit is not pipelined (beta above
// kPipeMaxBetaBytes: the per-round batching then buys only the batched gains and dense-tail
// launches) and the free memory holds fewer of the cacheable outputs' (D >= kDistCacheMinD)
// distances than the batch has: the narrower outputs (fused whitening, no cache) as one sub-batch,
// then the cacheable ones k at a time.  fit_chunks = k >= 1: k consecutive outputs at a time.
static std::vector<std::vector<int>> cache_chunks(gpar_ctx* c, const std::vector<DevProblem>& P,
                                                  int64_t later_bytes) {
  const int np = (int)P.size();
  std::vector<std::vector<int>> out;
  if (np < 2 || c->dist_cache_bytes == 0 || c->fit_chunks == 0) return out;
  if (c->fit_chunks > 0) {
    if (c->fit_chunks >= np) return out;
    for (int i0 = 0; i0 < np; i0 += c->fit_chunks) {
      out.emplace_back();
      for (int i = i0; i < std::min(np, i0 + c->fit_chunks); ++i) out.back().push_back(i);
    }
    return out;
  }
  if (fit_pipelined(c, P)) return out;
  std::vector<int> narrow, wide;
  for (int i = 0; i < np; ++i) (P[i].d >= kDistCacheMinD ? wide : narrow).push_back(i);
  if (wide.size() < 2) return out;
  int k = 0;
  if (c->dist_cache_bytes > 0) {   // an explicit budget: the cacheable outputs it holds
    int64_t b = 0;
    for (int i : wide) {
      const int64_t bytes = P[i].n * P[i].mp * (int64_t)sizeof(double);
      if (b + bytes > c->dist_cache_bytes) break;
      b += bytes;
      ++k;
    }
  } else {
    size_t fr = 0, tot = 0;
    HIPCHECK(hipMemGetInfo(&fr, &tot));
    int64_t held = 0;   // the context's buffers are reused by the sub-batches
    for (auto& kv : c->bufs) held += (int64_t)kv.second.bytes;
    const int64_t reserve = std::max<int64_t>((int64_t)1 << 30, (int64_t)(tot / 100));
    const int64_t avail = (int64_t)fr + held - reserve;
    for (int kk = (int)wide.size(); kk >= 1; --kk) {
      std::vector<DevProblem> sub;
      int64_t need = later_bytes;
      for (int a = 0; a < kk; ++a) {
        sub.push_back(P[wide[a]]);
        need += P[wide[a]].n * P[wide[a]].mp * (int64_t)sizeof(double);
      }
      need += fit_ws_estimate(c, sub);
      if (need <= avail) {
        k = kk;
        break;
      }
    }
  }
  if (k < 1 || k >= (int)wide.size()) return out;
  if (!narrow.empty()) out.push_back(narrow);
  for (size_t a = 0; a < wide.size(); a += (size_t)k)
    out.emplace_back(wide.begin() + a, wide.begin() + std::min(wide.size(), a + (size_t)k));
  return out;
}

void fit_impl(gpar_ctx* ctx, const std::vector<DevProblem>& P0, const double* log_theta0,
                     const gpar_fit_options& o, double* theta_out, double* nlml_out,
                     int32_t* evals_out, FitKeep* keep, int64_t later_bytes) {
  if (!keep) {   // (the kept Grams are named by batch index: one batch when they are wanted)
    const std::vector<std::vector<int>> chunks = cache_chunks(ctx, P0, later_bytes);
    if (!chunks.empty()) {
      // each sub-batch is one batch, and the cache buffers pass from one sub-batch to the next
      // (re-allocating tens of GB per sub-batch costs seconds: fresh VRAM is cleared); released at
      // the end unless the caller keeps them
      struct Restore {
        gpar_ctx* c;
        int chunks;
        bool keep;
        ~Restore() {
          c->fit_chunks = chunks;
          c->dist_cache_keep = keep;
          if (keep) return;
          try {
            release_dist_cache(c);
          } catch (...) {
          }
        }
      } restore_{ctx, ctx->fit_chunks, ctx->dist_cache_keep};
      ctx->fit_chunks = 0;
      ctx->dist_cache_keep = true;
      for (const auto& idx : chunks) {
        const size_t k = idx.size();
        std::vector<DevProblem> sub;
        std::vector<double> x0(5 * k), th(5 * k), nl(k);
        std::vector<int32_t> ev(k);
        for (size_t a = 0; a < k; ++a) {
          sub.push_back(P0[idx[a]]);
          std::copy(log_theta0 + 5 * idx[a], log_theta0 + 5 * idx[a] + 5, x0.begin() + 5 * a);
        }
        fit_impl(ctx, sub, x0.data(), o, th.data(), nl.data(), ev.data(), nullptr, later_bytes);
        for (size_t a = 0; a < k; ++a) {
          std::copy(th.begin() + 5 * a, th.begin() + 5 * a + 5, theta_out + 5 * idx[a]);
          if (nlml_out) nlml_out[idx[a]] = nl[a];
          if (evals_out) evals_out[idx[a]] = ev[a];
        }
      }
      return;
    }
  }
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
  // the whole fit after its distance cache, on the context stream (every schedule ends joined to it
  // or synchronised): the bench's fit time against its Gram spans
  std::optional<Timed> tm_fit;
  tm_fit.emplace(ctx, "fit_call");
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
  if (ctx->overlap && nprob >= 4 && (nprob <= kOverlapMaxOutputs || ctx->overlap_group > 0) &&
      fit_pipelined(ctx, P) &&
      split_active(ctx, P[0].n, mpmax))
    fit_overlapped(ctx, P, nm, accept);
  else if (ctx->overlap && nprob >= 4 &&
           ((nprob <= kOverlapUnsplitMax && mpmax >= kOverlapUnsplitMinMp) ||
            ctx->overlap_group > 0) &&
           fit_pipelined(ctx, P) && !split_active(ctx, P[0].n, mpmax) &&
           grouped_gram_eligible(ctx, P))
    fit_overlapped_unsplit(ctx, P, nm, accept);
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
  tm_fit.reset();
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
}  // namespace gpar
using namespace gpar;
extern "C" {

int32_t gpar_fit(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                 const double* log_theta0, const gpar_fit_options* opts, double* theta_out,
                 double* nlml_out, int32_t* evals_out) {
  API_BEGIN(ctx)
  ARGCHECK(probs && nprob >= 1 && log_theta0 && theta_out, "null argument");
  check_batch(probs, nprob);
  gpar_fit_options o{0, 1000, 1e-8, 0.0};
  if (opts) o = *opts;
  std::vector<DevProblem> P;
  P = prepare_batch(ctx, probs, nprob);
  fit_impl(ctx, P, log_theta0, o, theta_out, nlml_out, evals_out, nullptr);
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
