// host_lgssm.cpp -- temporal-only LGSSM chains (logpdf, RTS smoothing, get_sde_predictions,
// posterior paths' entry) and the exact GP / GPAR (config 1).
#include "host.hpp"

namespace gpar {

// logpdf of independent LGSSM chains sharing t (device pointers; ys: each chain's data vector).
// Timed "chains_logpdf": algorithmic bytes 8 n (t, once) + 8 n per chain (y); the per-chunk
// outputs (about 0.7 bytes per step and chain) are not counted.
// One pass: the gains recursion filters each chain's y from zero per chunk and keeps, per chunk,
// sum log S_k and the moments of the chunk-local alpha against the fix-up rows (no per-step
// record, fix-up row or alpha reaches HBM: t and y are read, 32 + 96 bytes per chunk written);
// the carry gives each chunk's incoming state and sum alpha_k^2 follows from the moments (r05;
// before, the gains wrote 160 bytes per step and chain and whiten_vec / vec_fix read them back).
// The plan uploads the chain parameters and sets up the workspace; each launch is one round into
// dl (device, one value per chain).
struct ChainsLml {
  GainsPlan gp;
  double *send = nullptr, *mom = nullptr, *dl = nullptr;
  int sdim = 0, nchains = 0;
  int64_t n = 0, nch = 0;
};

static ChainsLml plan_chains_lml(gpar_ctx* c, const std::vector<const double*>& ys, int64_t n,
                                 const double* t, int sdim,
                                 const std::vector<ChainParamsHost>& cps) {
  ChainsLml q;
  q.sdim = sdim;
  q.nchains = (int)ys.size();
  q.n = n;
  q.nch = (n + kChunk - 1) / kChunk;
  const int64_t nchs = 256 * ((q.nch + 255) / 256);   // GainsPlan::nchs of a moments plan
  q.send = ws<double>(c, "chain_send", (size_t)q.nchains * nchs * kSStride);
  q.mom = ws<double>(c, "chain_mom", (size_t)q.nchains * nchs * kGainsMomStride);
  q.dl = ws<double>(c, "chain_lml", q.nchains);
  q.gp = plan_gains(c, sdim, t, n, cps, nullptr, false, "chain", &ys, nullptr, q.send, false,
                    q.mom);
  return q;
}

static double chains_lml_bytes(const ChainsLml& q) { return 8.0 * (double)q.n * (1.0 + q.nchains); }

// one round's launches; timed: one "chains_logpdf" span around them (the device-stepped fit times
// whole batches of rounds instead: two event records per round were a third of its 15 us boundary)
static void launch_chains_lml(gpar_ctx* c, const ChainsLml& q, NmDev<3>* nm = nullptr,
                              int* active = nullptr, bool timed = true) {
  std::optional<Timed> tm_;
  if (timed) tm_.emplace(c, "chains_logpdf", chains_lml_bytes(q));
  q.gp.launch(c->stream, 0, q.nchains);
  const GainsOut& g = q.gp.o;
  launch_chain_carry_lml(c->stream, q.sdim, g.phi, g.phistride, q.send, q.gp.nchs * kSStride, g.logs,
                         q.mom, q.nch, q.n, q.nchains, q.dl, nm, q.gp.dcps, active);
  check_launch("chains_logpdf");
}

void chains_logpdf(gpar_ctx* c, const std::vector<const double*>& ys, int64_t n, const double* t,
                   int sdim, const double* theta, double* lml) {
  const int nchains = (int)ys.size();
  std::vector<ChainParamsHost> cps(nchains);
  for (int i = 0; i < nchains; ++i) {
    const double l = theta[3 * i], pv = theta[3 * i + 1], ns = theta[3 * i + 2];
    ARGCHECK(l > 0 && pv > 0 && ns > 0, "theta entries must be positive");
    cps[i] = {1.0 / l, l, pv * pv, ns * ns};
  }
  const ChainsLml q = plan_chains_lml(c, ys, n, t, sdim, cps);
  launch_chains_lml(c, q);
  d2h(c, lml, q.dl, nchains);
  sync(c);
}

// The chains' Nelder-Mead fit with the machines on the device (nm_dev.hpp): every round's logpdf
// launches queue on the stream in batches of kNmBatch rounds, the last of them (chain_carry_lml)
// stepping each chain's machine; the host reads one batch behind which machines still run (the last batch
// of a fit that ends on g_tol or its iteration cap is evaluated and discarded).  The rounds
// evaluate every chain (the host loop packs the running ones): a finished machine ignores its
// values.  log_theta0 / theta: nchains x 3 (packed, then unpacked, as the host loop).
constexpr int kNmBatch = 8;

static void fit_chains_device(gpar_ctx* c, int nchains, int64_t n, const double* t,
                              const double* y, int64_t ldy, int sdim, const double* log_theta0,
                              const gpar_fit_options& o, double* theta) {
  std::vector<NmDev<3>> hs(nchains);
  bool any = false;
  for (int i = 0; i < nchains; ++i) {
    nm_init(hs[i], log_theta0 + 3 * i, o.max_evals, o.max_iterations, o.g_tol);
    any = any || hs[i].st != NmDev<3>::Done;
  }
  if (any) {
    // round 0's parameters as the host loop sets them
    std::vector<ChainParamsHost> cps(nchains);
    std::vector<const double*> ys(nchains);
    for (int i = 0; i < nchains; ++i) {
      const double l = unpack(hs[i].pending[0]), pv = unpack(hs[i].pending[1]),
                   ns = unpack(hs[i].pending[2]);
      cps[i] = {1.0 / l, l, pv * pv, ns * ns};
      ys[i] = y + (size_t)i * ldy;
    }
    const ChainsLml q = plan_chains_lml(c, ys, n, t, sdim, cps);
    auto* dnm = ws<NmDev<3>>(c, "nm_dev", nchains);
    h2d(c, dnm, hs.data(), nchains);
    int* dact = ws<int>(c, "nm_active", nchains);
    int* hact = nullptr;
    HIPCHECK(hipHostMalloc((void**)&hact, 2 * (size_t)nchains * sizeof(int), hipHostMallocDefault));
    std::unique_ptr<int, void (*)(int*)> hact_(hact, [](int* p) { (void)hipHostFree(p); });
    hipEvent_t ev[2];
    HIPCHECK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
    struct Evs {
      hipEvent_t* e;
      ~Evs() { (void)hipEventDestroy(e[0]); (void)hipEventDestroy(e[1]); }
    } evs_{ev};
    const int64_t cap = o.max_evals > 0 ? (int64_t)o.max_evals : INT64_MAX;
    int64_t r = 0;
    for (int k = 0; r < cap; ++k) {
      const int64_t nb = std::min<int64_t>(kNmBatch, cap - r);
      {
        Timed tm_(c, "chains_logpdf", chains_lml_bytes(q) * (double)nb);
        for (int64_t b = 0; b < nb; ++b) launch_chains_lml(c, q, dnm, dact, /*timed=*/false);
      }
      r += nb;
      HIPCHECK(hipMemcpyAsync(hact + (k & 1) * nchains, dact, nchains * sizeof(int),
                              hipMemcpyDeviceToHost, c->stream));
      HIPCHECK(hipEventRecord(ev[k & 1], c->stream));
      if (k >= 1) {
        HIPCHECK(hipEventSynchronize(ev[(k - 1) & 1]));
        const int* a = hact + ((k - 1) & 1) * nchains;
        if (std::none_of(a, a + nchains, [](int x) { return x != 0; })) break;
      }
    }
    d2h(c, hs.data(), dnm, nchains);
    sync(c);
  }
  for (int i = 0; i < nchains; ++i)
    for (int q = 0; q < 3; ++q) theta[3 * i + q] = unpack(hs[i].x_min[q]);
}

// The same fit with the machines on the host (NelderMead), one round trip per round: the running
// chains' values come back, each machine steps, the next round's parameters go up.
static void fit_chains_host(gpar_ctx* c, int nchains, int64_t n, const double* t, const double* y,
                            int64_t ldy, int sdim, const double* log_theta0,
                            const gpar_fit_options& o, double* theta) {
  std::vector<NelderMead> nm;
  nm.reserve(nchains);
  for (int i = 0; i < nchains; ++i)
    nm.emplace_back(std::vector<double>(log_theta0 + 3 * i, log_theta0 + 3 * i + 3), o.max_evals,
                    o.max_iterations, o.g_tol, o.time_limit);
  while (true) {
    std::vector<int> act;
    for (int i = 0; i < nchains; ++i)
      if (!nm[i].done()) act.push_back(i);
    if (act.empty()) break;
    // the active chains' own data columns (no copy into a packed block)
    std::vector<double> th(3 * act.size());
    std::vector<const double*> ys(act.size());
    for (size_t a = 0; a < act.size(); ++a) {
      const auto& x = nm[act[a]].ask();
      for (int q = 0; q < 3; ++q) th[3 * a + q] = unpack(x[q]);
      ys[a] = y + (size_t)act[a] * ldy;
    }
    std::vector<double> lml(act.size());
    chains_logpdf(c, ys, n, t, sdim, th.data(), lml.data());
    for (size_t a = 0; a < act.size(); ++a) {
      double f = -lml[a];
      if (!std::isfinite(f)) f = INFINITY;
      nm[act[a]].tell(f);
    }
  }
  for (int i = 0; i < nchains; ++i)
    for (int q = 0; q < 3; ++q) theta[3 * i + q] = unpack(nm[i].x_min()[q]);
}

// --------------------------------------------------------------------------- temporal chains: smoothing
// Smoothed marginals of f for chains sharing the grid t (device pointers): mean = y - R Sigma^-1 y,
// var = RTS P^s[0,0].  noise: per-step observation variance (negative = chain sigma^2) or null.
void chains_smooth(gpar_ctx* c, int nchains, int64_t n, const double* t, const double* y,
                          int64_t ldy, const double* noise, int sdim,
                          const std::vector<ChainParamsHost>& cps, double* mean, double* var,
                          int64_t ldo) {
  const int64_t nch = (n + kChunk - 1) / kChunk;
  // Timed "chains_smooth": algorithmic bytes 8 n (t) + 8 n (noise, when given) + 24 n per chain
  // (y in, mean and variance out)
  Timed tm_(c, "chains_smooth", 8.0 * (double)n * ((noise ? 2.0 : 1.0) + 3.0 * nchains));
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
  auto* dcps = ws<ChainParamsHost>(c, "sm_cps2", nchains);
  h2d(c, dcps, cps.data(), nchains);
  double* vloc = ws<double>(c, "sm_vloc", (size_t)nchains * n);
  double* gam = ws<double>(c, "sm_gam", (size_t)nchains * n * 4);
  double* agg = ws<double>(c, "sm_agg", (size_t)nchains * nch * 2 * sdim * sdim);
  double* phat = ws<double>(c, "sm_phat", (size_t)nchains * nch * sdim * sdim);
  // the backward pass in one launch (r06; gains_adjoint + adjoint_local + cov_local before)
  launch_smooth_back(c->stream, sdim, g.rec, g.g, g.pf, dcps, cin, u, h, vloc, gam, agg, bend, n,
                     kChunk, nch, nchains, n, ss);
  run_carry(c, sdim, g.phi, g.phistride, bend, chat, ss, nch, 1, 1, nchains, "smb", true);
  launch_smooth_mean(c->stream, sdim, u, h, chat, ss, y, ldy, noise, dcps, n, kChunk, nchains, mean,
                     ldo);
  double* cscr = ws<double>(c, "sm_covscan", (size_t)cov_carry_scratch_doubles(sdim, nch, nchains));
  launch_cov_smooth(c->stream, sdim, t, g.rec, g.pf, dcps, n, kChunk, nch, nchains, vloc, gam, agg,
                    phat, var, ldo, cscr, /*local_done=*/true);
  check_launch("chains_smooth");
}

std::vector<ChainParamsHost> chain_params(const double* theta, int nchains) {
  std::vector<ChainParamsHost> cps(nchains);
  for (int i = 0; i < nchains; ++i) {
    const double l = theta[3 * i], pv = theta[3 * i + 1], ns = theta[3 * i + 2];
    ARGCHECK(l > 0 && pv > 0 && ns > 0 && std::isfinite(l + pv + ns), "theta entries must be positive");
    cps[i] = {1.0 / l, l, pv * pv, ns * ns};
  }
  return cps;
}
}  // namespace gpar
using namespace gpar;
extern "C" {

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
  std::vector<const double*> ys(nchains);
  for (int i = 0; i < nchains; ++i) ys[i] = dy + (size_t)i * ldy;
  chains_logpdf(ctx, ys, n, dt, sdim, theta, lml.data());
  for (int i = 0; i < nchains; ++i) lml_out[i] = lml[i];
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
  std::vector<double> theta(3 * nchains);
  if (ctx->device_nm && !(o.time_limit > 0))
    fit_chains_device(ctx, nchains, n, dt, dy, ldyd, sdim, log_theta0, o, theta.data());
  else
    fit_chains_host(ctx, nchains, n, dt, dy, ldyd, sdim, log_theta0, o, theta.data());
  for (int i = 0; i < 3 * nchains; ++i) theta_out[i] = theta[i];
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
}  // extern "C"
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
using namespace gpar;
extern "C" {

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
}  // extern "C"
