// host_objective.cpp -- the DTC objective: Kfu + whitening, the Gram stage (pipelined /
// CU-split), the blocked dense tail; gpar_dtc_objective_A.
#include "host.hpp"

namespace gpar {


// Kfu assembly + chunk-local whitening: fp64-MFMA Gram-form kernel for the smooth output
// kernels, direct-difference kernel for Matern-1/2 (kappa not smooth in d^2 at 0).
// Inputs wider than kFusedMaxD (the fused kernels keep a column's pseudo-input in registers):
// the squared distances are a separate MFMA (or direct-difference) pass into beta itself, which
// the whitening then reads and overwrites in place (k_dist.hip).
void whiten_kfu_any(gpar_ctx* c, const DevProblem& p, const GainsOut& gi, const double* v,
                           int64_t ldv, int64_t n, int64_t nch, const Theta& th, double* beta,
                           int64_t ldb, double* send, double* hsum, bool d2_in_beta) {
  const double s_o = th.sv_o * th.sv_o;
  const double* rec = gi.rec;
  const double* g = gi.g;
  // compact records: A_k recomputed from t inside whiten_kfu_d2x2 (the only whitening that can)
  const double* tc = gi.compact ? gi.t : nullptr;
  const double* d2 = cached_d2(c, p);
  if (d2 && v == p.v) {   // the fit's training inputs, distances cached (fit_impl)
    launch_whiten_kfu_d2(c->stream, p.tk, p.ok, rec, d2, p.mp, p.m, p.mp, n, kChunk, nch,
                         1.0 / th.l_o, s_o, beta, ldb, send, p.mc, g, hsum, p.d2_is_r, tc, th.l_t);
  } else if (p.d > kFusedMaxD || gi.compact) {
    if (!d2_in_beta)   // else the caller's (timed) distance pass already wrote them
      launch_dist2(c->stream, p.ok, v, ldv, n, p.z, p.ldz, p.m, p.mp, (int)p.d, p.zc, beta, ldb);
    launch_whiten_kfu_d2(c->stream, p.tk, p.ok, rec, beta, ldb, p.m, p.mp, n, kChunk, nch,
                         1.0 / th.l_o, s_o, beta, ldb, send, p.mc, g, hsum, false, tc, th.l_t);
  } else if (p.ok == GPAR_MATERN12) {
    launch_whiten_kfu(c->stream, p.tk, p.ok, rec, v, ldv, (int)p.d, p.z, p.ldz, p.m, p.mp, n,
                      kChunk, nch, 1.0 / th.l_o, s_o, beta, ldb, send, p.mc, g, hsum);
  } else {
    launch_whiten_kfu_mfma(c->stream, p.tk, p.ok, rec, v, ldv, (int)p.d, p.z, p.ldz, p.zc, p.m, p.mp,
                           n, kChunk, nch, 1.0 / th.l_o, s_o, beta, ldb, send, p.mc, g, hsum);
  }
}

StageBufs stage_bufs(gpar_ctx* c, int l, int64_t n, int64_t mpmax) {
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

// The grouped Gram's per-output stage buffers: slot `slot` of a group, carry tags of stream lane
// `lane` (its carry workspaces are reused output after output on that lane).
static StageBufs stage_bufs_grp(gpar_ctx* c, int lane, int slot, int64_t n, int64_t mpmax,
                                double* send = nullptr, double* cin = nullptr) {
  const int64_t nch = (n + kChunk - 1) / kChunk;
  const std::string sfx = "_g" + std::to_string(slot);
  StageBufs b;
  b.idx = lane;
  b.beta = ws<double>(c, "beta" + sfx, (size_t)(n + 16) * mpmax);
  b.alpha = ws<double>(c, "alpha" + sfx, (size_t)n);
  // the carry's input / output: the group's shared arrays when its carries run batched
  b.send = send ? send : ws<double>(c, "send" + sfx, (size_t)nch * (mpmax + 1) * 4);
  b.cin = cin ? cin : ws<double>(c, "cin" + sfx, (size_t)nch * (mpmax + 1) * 4);
  b.hsum = ws<double>(c, "hsum" + sfx, (size_t)nch * (mpmax + 1) * 4);
  b.qv = ws<double>(c, "qv" + sfx, (size_t)nch * 4);
  return b;
}

// Outputs per grouped Gram launch set (0: per-output Grams).  Small problems only: one output's
// Gram (N Mp^2 <= kGramGroupMaxWork) has too few (group, split) items to fill the chip without
// splitting time so finely that its partial sums and chunk correction cost as much as the GEMM
// (N = 1e5, M = 256: 0.22 ms per launch against 0.084 ms of MFMA work, r05i); grouped, the same
// items come from several outputs with 1/g of the time splits each.  Groups of 8 (r06, eeg at
// N = 1e5, M = 512, 64 outputs, one box: g = 4 2413, 6 3366, 8 2411, 12 2883, 16 2533 ms per job;
// sizes that leave noff * soff off a multiple of 8 lose the XCD deal's balance).
constexpr double kGramGroupMaxWork = 5e10;
constexpr int kGramGroupAuto = 8;
constexpr int64_t kGramGroupMaxBytes = (int64_t)24 << 30;   // the group's beta buffers
constexpr int64_t kGrpMinRows = 4096;   // rows per OFF workgroup below which the share stays 1/cnt
static int gram_group_size(gpar_ctx* c, const std::vector<DevProblem>& P, int64_t n,
                           int64_t mpmax, bool fix_beta, int nlanes, bool split_pipe) {
  const int np = (int)P.size();
  if (fix_beta || nlanes > 1 || split_pipe || np < 2) return 0;
  // the grouped launch takes one chunk-correction template (sdim) and carry stride (mc) for the
  // whole group: outputs with another time kernel keep the per-output Grams
  for (const auto& p : P)
    if (p.mp != mpmax || p.n != n || p.sdim != P[0].sdim || p.mc != P[0].mc) return 0;
  int g = c->gram_group;
  if (g == 0 || g == 1) return 0;
  if (g < 0) {
    if ((double)n * (double)mpmax * (double)mpmax > kGramGroupMaxWork) return 0;
    g = kGramGroupAuto;
  }
  g = std::min(g, np);
  const int64_t beta_bytes = (n + 16) * mpmax * (int64_t)sizeof(double);
  while (g > 1 && (int64_t)g * beta_bytes > kGramGroupMaxBytes) --g;
  return g >= 2 ? g : 0;
}

// an unsplit batched round of these problems would run the grouped Gram
bool grouped_gram_eligible(gpar_ctx* c, const std::vector<DevProblem>& P) {
  int64_t mpmax = 0;
  for (const auto& p : P) mpmax = std::max(mpmax, p.mp);
  return gram_group_size(c, P, P[0].n, mpmax, false, 1, false) >= 2;
}

// Kfu assembly + chunk-local whitening of j's output into b.beta, on c->stream.
void stage_whiten(gpar_ctx* c, const StageJob& j, const StageBufs& b) {
  const DevProblem& p = *j.p;
  // uncached inputs wider than the fused kernels take (or compact records): the distances go
  // into beta first, a pass of its own ("dist2": 2 N Mp D flops of MFMA cross products)
  const bool cached = cached_d2(c, p) != nullptr;
  const bool pass = !cached && (p.d > kFusedMaxD || j.gi.compact);
  if (pass) {
    Timed td_(c, "dist2", 2.0 * (double)p.n * (double)p.mp * (double)p.d);
    launch_dist2(c->stream, p.ok, p.v, p.ldv, p.n, p.z, p.ldz, p.m, p.mp, (int)p.d, p.zc, b.beta,
                 p.mp);
    check_launch("dist2");
  }
  // algorithmic HBM bytes: the inputs (V, or the distances), the gains records and fix-up rows
  // (16 + 4 doubles per step), beta written (m columns)
  const double in_cols = (cached || pass) ? (double)p.m : (double)p.d;
  Timed tm_(c, "whiten", 8.0 * (double)p.n * (in_cols + (double)p.m + 20.0));
  whiten_kfu_any(c, p, j.gi, p.v, p.ldv, p.n, p.nch, *j.th, b.beta, p.mp, b.send, b.hsum, pass);
  check_launch("whiten_kfu");
}

// The short chain between a whitening and its Gram, on c->stream: alpha's chunk end states, the
// chunk carry, vec_fix (alpha fix-up, the Gram's correction E_j = H_j + W_j C_j / 2 and q_j), the
// beta tail (and the beta fix-up pass when fix_beta).  In three parts so that the grouped Gram can
// run the carries of a whole group in one batched launch set (stage_post_head / _tail).
static void stage_post_head(gpar_ctx* c, const StageJob& j, const StageBufs& b) {
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
}

static void stage_post_tail(gpar_ctx* c, const StageJob& j, const StageBufs& b, bool fix_beta) {
  const DevProblem& p = *j.p;
  const int64_t n = p.n;
  launch_vec_fix(c->stream, p.sdim, j.alpha, 0, j.gi.g, 0, b.cin, 0, p.mc, p.mp, n, kChunk, 1,
                 j.a2part, fix_beta ? nullptr : b.hsum, p.mp, b.qv);
  check_launch("vec_fix");
  if (fix_beta) {
    launch_beta_fix(c->stream, p.sdim, b.beta, p.mp, n, j.gi.g, b.cin, p.mc, kChunk);
    check_launch("beta_fix");
  }
  HIPCHECK(hipMemsetAsync(b.beta + (size_t)n * p.mp, 0, (size_t)16 * p.mp * sizeof(double), c->stream));
}

void stage_post(gpar_ctx* c, const StageJob& j, const StageBufs& b, bool fix_beta) {
  const DevProblem& p = *j.p;
  stage_post_head(c, j, b);
  run_carry(c, p.sdim, j.gi.phi, 0, b.send, b.cin, 0, p.nch, p.mc, p.mc, 1,
            b.idx ? "fitc_1" : "fitc");
  check_launch("carry");
  stage_post_tail(c, j, b, fix_beta);
}

// G = beta^T beta, r = beta^T alpha of j on c->stream, which may use `cus` CUs; side: the stream of
// the co-running chunk correction; st_w: the first w_frac32 / 32 of the DG kernel's work items run
// there (ev_w joins them).  one_per_cu: the two-lane plan (one Gram workgroup per CU).
void stage_gram(gpar_ctx* c, const StageJob& j, const StageBufs& b, bool fix_beta,
                       bool one_per_cu, const std::string& part_sfx, hipStream_t side, int cus,
                       hipStream_t st_w, hipEvent_t ev_w, int w_frac32, int dg_rows_w) {
  const DevProblem& p = *j.p;
  if (c->gram_after) {   // the round's dense prefix (eval_dtc) first
    HIPCHECK(hipStreamWaitEvent(c->stream, c->gram_after, 0));
    c->gram_after = nullptr;
  }
  GramPlan plan = gram_plan(p.n, p.mp, one_per_cu, cus, st_w ? 256 : cus);
  const int w_items = st_w ? plan.ndg * plan.sdg * w_frac32 / 32 : 0;
  // dg_rows_w: the DG time splits that run on the whitening CUs take that many percent more rows
  // (the rest fewer), moving diagonal-block work between the two sides in finer steps than whole
  // rounds of items
  if (st_w && w_items > 0 && dg_rows_w != 0 && plan.v3 && plan.sdg * c->split_w % 32 == 0) {
    const int sw = plan.sdg * c->split_w / 32;
    auto up = [](int64_t r) { return (r + kBKRows - 1) / kBKRows * kBKRows; };
    const int64_t rw = up(plan.rows_dg * (100 + dg_rows_w) / 100);
    const int64_t rest = p.n - (int64_t)sw * rw;
    if (rw > 0 && rest > 0 && plan.sdg > sw) {
      plan.dg_sw = sw;
      plan.dg_rows_w = rw;
      plan.rows_dg = up((rest + plan.sdg - sw - 1) / (plan.sdg - sw));
    }
  }
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
void reserve_gram_parts(gpar_ctx* c, const std::vector<DevProblem>& P, int nlanes) {
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

// For every problem: G = beta^T beta, r = beta^T alpha, sum alpha^2 partials, sum log S
// partials, at hyperparameters th.
// fix_beta = false (the objective): the Gram streams the chunk-local beta and adds the chunk
//   correction sum_j E_j C_j^T + C_j E_j^T (k_gram.hip) -- no extra pass over beta.
// fix_beta = true (q(u), the (dtc, A) entry point): beta is fixed up in place first and the
//   Gram is a plain beta^T beta.  One extra pass over beta, but G carries the rounding of the
//   true beta only: q(u) factors the noise-free Cuu (cond >= 1e7), which amplifies the ~10x
//   larger rounding of the correction form (emulated: 7e-15 vs 7e-16 of max |G|).
GramOut run_gram_stage(gpar_ctx* c, const std::vector<DevProblem>& P,
                              const std::vector<Theta>& th, bool fix_beta) {
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
  // a split round's head: the first output's gains on the whitening CUs and the others' beside
  // them on the Gram CUs (r04j; the variants tried in r04 -- every gains first, whole-chip or not;
  // the first job on the Gram CUs; the late gains beside the Grams -- measured slower)
  const bool split_head = split_pipe && shared && np > 1;
  const double* logs_src = nullptr;
  std::vector<GainsOut> gains(np);
  GainsPlan gplan;
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
    // split pipeline (split_head): the first output's gains on the whitening CUs, ahead of its
    // whitening there, and the others' at the same time on the Gram CUs, ahead of the first Gram;
    // the second whitening waits for them (below).  Tried: the first whitening whole-chip, beside
    // the others' gains (head 8.6 ms per round, r04f) or ahead of them (they then delayed the
    // second whitening and every Gram after it, r04i); the others' gains in groups on the
    // whitening stream (they delayed the Grams' DG share: 5.10 -> 5.24 ms per Gram, r04h).
    // compact records (split pipeline only: its every whitening is whiten_kfu_d2x2) when asked:
    // in the round-by-round fit they made the round head's first whitening slower beside the
    // other outputs' (now faster) gains, 5.6 -> 8.6 ms per round, 17.77 -> 17.91 s per job (r04x)
    gplan = plan_gains(c, P[0].sdim, P[0].t, n, cps, nullptr, false, "fit", &ys, alpha_all,
                       asend_all, /*compact=*/split_pipe && c->compact_rec == 1);
    if (!split_head) gplan.launch(c->stream, 0, np);
    const GainsOut& g = gplan.o;
    for (int i = 0; i < np; ++i) {
      gains[i] = g;
      gains[i].rec = g.rec + (size_t)i * g.recstride;
      gains[i].g = g.g + (size_t)i * g.gstride;
      gains[i].phi = g.phi + (size_t)i * g.phistride;
      gains[i].logs = g.logs + (size_t)i * nch;
    }
    if (!split_head)   // else after the pipeline (later groups' gains run on the whitening stream)
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
    sp.post_gram = c->post_gram == 1;
    sp.dg_rows_w = c->dg_rows_w == kDgRowsAuto ? 40 : c->dg_rows_w;
    sp.start();
    if (split_head) {
      gplan.launch(c->s_w, 0, 1);
      gplan.launch(c->s_g2, 1, np - 1);
      HIPCHECK(hipEventRecord(c->ev_gr, c->s_g2));
    }
    for (int i = 0; i < np; ++i) {
      if (i == 1 && split_head) HIPCHECK(hipStreamWaitEvent(c->s_w, c->ev_gr, 0));
      sp.push(job(i, sp.buf[i & 1]));
    }
    sp.flush();
    if (c->mark_last) HIPCHECK(hipEventRecord(c->mark_last, c->s_g));
    sp.join(c->stream);   // a prediction lane's q(u) runs this on the side stream
    if (split_head)       // every gains launch precedes the second whitening, which join covers
      HIPCHECK(hipMemcpyAsync(o.logs, logs_src, (size_t)np * nch * sizeof(double),
                              hipMemcpyDeviceToDevice, c->stream));
    return o;
  }
  const int gsz = gram_group_size(c, P, n, mpmax, fix_beta, nlanes, split_pipe);
  if (gsz >= 2) {
    // Grouped Gram: per group of gsz outputs, their whitenings and short chains alternate over the
    // context and side streams into buffers of their own, then one set of Gram launches covers the
    // whole group (grid y = output, GramGroupPtrs table), its plan sized for 1/gsz of the chip per
    // output.  A different split plan than the per-output Gram's: G moves within rounding.
    const hipStream_t base = c->stream;
    const int ngroups = (np + gsz - 1) / gsz;
    auto* tab = ws<GramGroupPtrs>(c, "gram_grp_tab", (size_t)ngroups * gsz);
    // The per-output CU share: 256 / cnt, doubled while the OFF workgroups keep >= kGrpMinRows
    // rows each (twice the split workgroups: the eeg shard's group of 8 at N = 1e5, M = 512 went
    // 4.46 -> 3.81 ms per Gram, OFF 10000 -> 4762 rows; dtc's 1563-row OFF slices lose 13 % when
    // halved again: per-workgroup prologue and more partials to reduce)
    auto plan_of = [&](int cnt) {
      const int cus = std::max(256 / cnt, 8);
      const GramPlan p2 = gram_plan(n, mpmax, false, 2 * cus, 2 * cus);
      if (p2.noff > 0 && p2.rows_off >= kGrpMinRows) return p2;
      return gram_plan(n, mpmax, false, cus, cus);
    };
    // the partials, sized once for every group's plan (no buffer may move under a running launch)
    int64_t pd = 0, rd = 0;
    for (int cnt : {gsz, np % gsz})
      if (cnt > 0) {
        const GramPlan pl = plan_of(cnt);
        pd = std::max(pd, pl.part_doubles);
        rd = std::max(rd, pl.rpart_doubles);
      }
    double* part = ws<double>(c, "gram_part_grp", (size_t)gsz * pd);
    double* rpart = ws<double>(c, "gram_rpart_grp", (size_t)gsz * rd);
    // shared gains (one grid; the outputs' transfers phi strided in one array): the group's chunk
    // carries run as one batched launch set after its whitenings (r06: three small latency-bound
    // launches per output were 0.8 ms of a rank's eeg round boundary, r06d trace)
    const bool batch_post = shared;
    const int64_t sstr = nch * (mpmax + 1) * 4;
    double* send_grp = batch_post ? ws<double>(c, "send_grp", (size_t)gsz * sstr) : nullptr;
    double* cin_grp = batch_post ? ws<double>(c, "cin_grp", (size_t)gsz * sstr) : nullptr;
    for (int g0 = 0, gi = 0; g0 < np; g0 += gsz, ++gi) {
      const int cnt = std::min(gsz, np - g0);
      const GramPlan plan = plan_of(cnt);
      // the side lane starts after everything queued so far (the gains, the previous group's Gram,
      // which still reads the buffers this group overwrites)
      HIPCHECK(hipEventRecord(c->ev_fork, base));
      HIPCHECK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
      std::vector<StageBufs> gb(cnt);
      std::vector<GramGroupPtrs> th_tab(cnt);
      double work = 0.0;
      for (int k = 0; k < cnt; ++k) {
        const int i = g0 + k, lane = k & 1;
        gb[k] = batch_post ? stage_bufs_grp(c, lane, k, n, mpmax, send_grp + (size_t)k * sstr,
                                            cin_grp + (size_t)k * sstr)
                           : stage_bufs_grp(c, lane, k, n, mpmax);
        OnStream on_(c, lane ? c->side : base);
        const StageJob& j = job(i, gb[k]);
        stage_whiten(c, j, gb[k]);
        if (!batch_post) stage_post(c, j, gb[k], false);
        th_tab[k] = {gb[k].beta, j.alpha, gb[k].hsum, gb[k].cin, gb[k].qv,
                     part + (size_t)k * pd, rpart + (size_t)k * rd,
                     j.G, j.r};
        work += (double)P[i].n * (double)P[i].m * (double)(P[i].m + 1);
      }
      HIPCHECK(hipEventRecord(c->ev_join, c->side));
      HIPCHECK(hipStreamWaitEvent(base, c->ev_join, 0));
      if (batch_post) {   // on the context stream, after both lanes' whitenings
        for (int k = 0; k < cnt; ++k) stage_post_head(c, jobs[g0 + k], gb[k]);
        run_carry(c, P[g0].sdim, gains[g0].phi, gplan.o.phistride, send_grp, cin_grp, sstr, nch,
                  P[g0].mc, P[g0].mc, cnt, "fitc_grp");
        check_launch("carry (grouped)");
        for (int k = 0; k < cnt; ++k) stage_post_tail(c, jobs[g0 + k], gb[k], false);
      }
      GramGroupPtrs* dtab = tab + (size_t)gi * gsz;
      h2d(c, dtab, th_tab.data(), (size_t)cnt);
      if (c->gram_after) {   // the round's dense prefix (eval_dtc) first
        HIPCHECK(hipStreamWaitEvent(base, c->gram_after, 0));
        c->gram_after = nullptr;
      }
      {
        Timed tm_(c, "gram", work);   // flops of every beta^T beta of the group
        launch_gram_grouped(base, P[g0].sdim, plan, dtab, cnt, mpmax, n, P[g0].mc, kChunk, mpmax,
                            c->side, c->ev_fork, c->ev_join);
      }
      check_launch("gram (grouped)");
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

// L_u = chol(Kuu [+ s2 I]), T_u = L_u^-1, Lambda = T_u G T_u^T + I, L_lam = chol(Lambda) for
// every problem: blocked 64 x 64 MFMA kernels (k_chol.hip), matrices padded with identity to
// ld = Mp (padding contributes log 1 = 0 and zero right-hand sides).  run_dense_pre is the part
// that does not read G (Kuu, its Cholesky factor and inverse), run_dense_post the rest.
DenseOut run_dense_pre(gpar_ctx* c, const std::vector<DevProblem>& P,
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

void run_dense_post(gpar_ctx* c, const std::vector<DevProblem>& P, const GramOut& go,
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

DenseOut run_dense(gpar_ctx* c, const std::vector<DevProblem>& P,
                          const std::vector<Theta>& th, const GramOut& go, bool qu_mode) {
  DenseOut o = run_dense_pre(c, P, th, go.ldg, qu_mode);
  run_dense_post(c, P, go, o);
  return o;
}

Finish2JobHost finish_job(const DenseOut& dn, const GramOut& go, const DevProblem& p, int i,
                                 int64_t nch, double* out, double* me) {
  const size_t sq = (size_t)dn.ld * dn.ld;
  return Finish2JobHost{dn.Tu + i * sq, dn.Llam + i * sq,
                        dn.Tdl + (size_t)i * dn.nb * kDenseNB * kDenseNB, go.r + (size_t)i * go.ldg,
                        go.logs + (size_t)i * nch, nch, go.a2part + (size_t)i * go.npart, go.npart,
                        p.n, dn.status + 2 * i, out, me};
}

std::vector<Theta> thetas_from(const double* theta, int np) {
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
void eval_dtc(gpar_ctx* c, const std::vector<DevProblem>& P, const std::vector<Theta>& th,
                     double* out, std::vector<int>& status_out, GramOut* gram_out,
                     const EvalAsync* async) {
  const int np = (int)P.size();
  // one Nelder-Mead round of a batched fit, entry to values (the bench's round overhead: this
  // span less the round's Gram spans is what does not overlap a Gram)
  Timed tm_round(c, "fit_round");
  // with profiling: marks along the round (flush_stats turns consecutive marks into stats):
  // entry -> the first output's gains ("head_gains") -> its whitening ("head_w0") -> its short
  // chain ("head_p0") -> the first Gram's start ("head_gram_wait") -> the last Gram's end
  // ("round_grams") -> the values on the host ("round_tail")
  gpar_ctx::MarkSeq seq;
  int64_t mpm = 0;
  for (const auto& p : P) mpm = std::max(mpm, p.mp);
  if (c->profiling && fit_pipelined(c, P) && split_active(c, P[0].n, mpm)) {   // SplitPipe marks
    seq.names = {"", "head_gains", "head_w0", "head_p0", "head_gram_wait", "round_grams",
                 "round_tail"};
    seq.ev.assign(seq.names.size(), nullptr);
    for (hipEvent_t& e : seq.ev) HIPCHECK(hipEventCreate(&e));
    c->mark_h[0] = seq.ev[1];
    c->mark_h[1] = seq.ev[2];
    c->mark_h[2] = seq.ev[3];
    c->mark_first = seq.ev[4];
    c->mark_last = seq.ev[5];
    HIPCHECK(hipEventRecord(seq.ev[0], c->stream));
  }
  struct Marks {   // hands the sequence to the stats (flush_stats destroys its events), on any exit
    gpar_ctx* c;
    gpar_ctx::MarkSeq& seq;
    ~Marks() {
      if (seq.ev.empty()) return;
      c->mark_seqs.push_back(std::move(seq));
      c->mark_first = c->mark_last = nullptr;
      for (hipEvent_t& e : c->mark_h) e = nullptr;
    }
  } marks_{c, seq};
  // On the CU-split pipeline the G-independent half of the dense tail (Kuu, its factor and
  // inverse) goes first on the Gram stream: it runs beside the gains and the first whitening,
  // while the Gram CUs would otherwise wait, instead of after the round's last Gram.  (On the
  // dense stream over the whitening CUs instead, r04e, it slowed every Gram 5.11 -> 5.16 ms: the
  // Gram's diagonal-block share runs there.)
  int64_t mpmax = 0;
  for (const auto& p : P) mpmax = std::max(mpmax, p.mp);
  const bool early = c->dense_early && fit_pipelined(c, P) && split_active(c, P[0].n, mpmax);
  // Unsplit batched rounds (the dtc / eeg configs, a rank's eeg shard): the same G-independent
  // half on the dense stream (s_d), beside the round's gains, whitenings and Grams instead of
  // after the last Gram -- a chain of latency-bound 64 x 64 launches (eeg shard 0/8, r06d trace:
  // 2.2 ms of a 5.3 ms round boundary was the dense tail)
  const bool early_side = !early && c->dense_early && P.size() > 1 && c->s_d != nullptr;
  DenseOut dn{};
  if (early_side) {
    HIPCHECK(hipEventRecord(c->ev_dn, c->stream));
    HIPCHECK(hipStreamWaitEvent(c->s_d, c->ev_dn, 0));
    OnStream on_(c, c->s_d);
    dn = run_dense_pre(c, P, th, mpmax, false);
    HIPCHECK(hipEventRecord(c->ev_dn, c->s_d));
    c->gram_after = c->ev_dn;
  }
  if (early) {
    // the Gram stream first follows everything queued on the context stream (host inputs' uploads,
    // the pseudo-input centres, the distance cache), then factors Kuu beside the round's gains
    // (on a Gram-CU stream of its own, r04ae, the first Gram no longer queued behind it but shared
    // the Gram CUs with it: 17.67 -> 17.70 s per job)
    HIPCHECK(hipEventRecord(c->ev_dn, c->stream));
    HIPCHECK(hipStreamWaitEvent(c->s_g, c->ev_dn, 0));
    OnStream on_(c, c->s_g);
    dn = run_dense_pre(c, P, th, mpmax, false);
  }
  GramOut go = run_gram_stage(c, P, th);
  if (gram_out) *gram_out = go;
  if (early_side) {
    c->gram_after = nullptr;   // (consumed by the first Gram; cleared if there was none)
    HIPCHECK(hipStreamWaitEvent(c->stream, c->ev_dn, 0));
  }
  else if (!early) dn = run_dense_pre(c, P, th, go.ldg, false);
  run_dense_post(c, P, go, dn);
  const int64_t nch = P[0].nch;
  std::vector<Finish2JobHost> fj(np);
  double* dout = ws<double>(c, "dtc_out", np);
  for (int i = 0; i < np; ++i) fj[i] = finish_job(dn, go, P[i], i, nch, dout + i, nullptr);
  auto* dfj = ws<Finish2JobHost>(c, "finishjobs", np);
  h2d(c, dfj, fj.data(), np);
  launch_finish2(c->stream, dfj, np, dn.ld, dn.nb);
  check_launch("finish");
  if (async) {
    HIPCHECK(hipMemcpyAsync(async->hout, dout, np * sizeof(double), hipMemcpyDeviceToHost,
                            c->stream));
    HIPCHECK(hipMemcpyAsync(async->hstat, dn.status, 2 * np * sizeof(int), hipMemcpyDeviceToHost,
                            c->stream));
    if (!seq.ev.empty()) HIPCHECK(hipEventRecord(seq.ev.back(), c->stream));
    HIPCHECK(hipEventRecord(async->done, c->stream));
    return;
  }
  std::vector<int> st(2 * np);
  d2h(c, out, dout, np);
  d2h(c, st.data(), dn.status, 2 * np);
  if (!seq.ev.empty()) HIPCHECK(hipEventRecord(seq.ev.back(), c->stream));
  sync(c);
  status_out.assign(np, 0);
  for (int i = 0; i < np; ++i) status_out[i] = st[2 * i] || st[2 * i + 1];
}
}  // namespace gpar
using namespace gpar;
extern "C" {

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
}  // extern "C"
