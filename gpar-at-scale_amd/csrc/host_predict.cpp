// host_predict.cpp -- q(u), the prediction modes (analytic, MC, posterior paths), the batched
// fit + predict driver, and their C-ABI entries.
#include "host.hpp"

#include <atomic>

namespace gpar {

QuOut run_q_u(gpar_ctx* c, const DevProblem& p, const Theta& th,
                     const GramCache* gc) {
  std::vector<DevProblem> P{p};
  std::vector<Theta> T{th};
  // G = beta^T beta and r = beta^T alpha do not depend on Cuu's jitter (only L_u does,
  // gpar_scaled_inference.jl:157-187), but their rounding matters for the noise-free Cuu: it takes
  // the extra beta fix-up pass (a plain beta^T beta of the true beta carries ~10x less rounding
  // than the objective's correction form, and cond(Cuu) up to ~1e10 amplifies it -- reusing the
  // fit's correction-form Gram there measured 1.5e-7 relative off the oracle's std, r04a).  With
  // qu_kuu_noise the factor is the objective's regularised Kuu + s2 I and the correction-form Gram
  // the fit computed at this theta is reused when the caller hands it over (gc).
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

std::vector<QuPre> run_q_u_batch(gpar_ctx* c, const std::vector<DevProblem>& P,
                                        const std::vector<Theta>& T, const FitKeep& keep,
                                        bool want_cov) {
  const int np = (int)P.size();
  int64_t mpmax = 0, mmax = 0;
  for (const auto& p : P) { mpmax = std::max(mpmax, p.mp); mmax = std::max(mmax, p.m); }
  const bool qn = P[0].qu_noise;
  bool kept = qn;   // the fit's Grams serve the regularised convention only (run_q_u)
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

// S joint posterior samples of the latent f along one LGSSM chain (TemporalGPs posterior_rand,
// tmp.jl:161-167) with the simulation smoother (k_path.hip): gains g of the chain over the n steps
// of the grid t (params cp, observation noise `noise` per step or cp.r), data v_{k,s} = ym[k] - fx[k * ldfx + s]
// (fx null: ym[k] for every sample).  Samples -> F[k * S + s].
void path_samples(gpar_ctx* c, int sdim, const GainsOut& g, const ChainParamsHost& cp,
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
void predict_impl(gpar_ctx* c, const DevProblem& P, const Theta& th, int mem,
                         int64_t n_star, const double* t_star_in, const double* v_star_in,
                         int64_t ldvs, int mode, int samples, uint64_t seed, double* mean_out,
                         double* std_out, const GramCache* gc, bool defer,
                         const QuPre* pre, const PredPrep* prep) {
  const int64_t n = P.n, m = P.m, d = P.d, mp = P.mp, mc = P.mc;
  if (mode == GPAR_PREDICT_PATH)   // path draw (s, k, i): counter index k (sdim + 1) + i, 32 bits
    ARGCHECK((n + n_star) * (P.sdim + 1) <= ((int64_t)1 << 32),
             "path mode: (n + n_star) * (state dimension + 1) must be <= 2^32");
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
  GainsOut g;
  if (prep) {   // computed ahead on the side stream (gpar_posterior_prepare)
    HIPCHECK(hipStreamWaitEvent(c->stream, c->ev_prep_ready[prep - c->prep.data()], 0));
    g = prep->g;
  } else {
    g = run_gains(c, P.sdim, tm, nt, cps, rm, false, "pred");
  }
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
    // FX only: no row sums (mode 0 writes them per 128-column block when asked)
    launch_gemm_nt(c->stream, Ks, mp, Bm, mp, nt, samples, m, 0, FX, samples, nullptr, 0, nullptr,
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
    double* h = prep ? prep->h : ws<double>(c, "pr_h", (size_t)nt * 4);
    {   // algorithmic HBM bytes: merged inputs V* (d) read, gains records + fix-up rows (20), the
        // m whitened Cf*u columns written, per merged row
      Timed tm_(c, "pred_whiten", 8.0 * (double)nt * ((double)d + (double)m + 20.0));
      whiten_kfu_any(c, P, g, vm, d, nt, nch, th, X, ldx, send, nullptr);
      launch_whiten_vec(c->stream, P.sdim, g.rec, 0, ym, 0, nt, kChunk, nch, 1, X + mp, 0, send, 0,
                        mc, mp, ldx);
    }
    check_launch("predict: whiten");
    run_carry(c, P.sdim, g.phi, 0, send, cin, 0, nch, mc, mc, 1, "predf");
    // ---- adjoint: Sigma^{-1} x = W^T (W x)
    if (!prep) launch_gains_adjoint(c->stream, P.sdim, g.rec, nt, kChunk, nch, 1, h);
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
  // the prepared slot may be refilled once this prediction has read it
  if (prep) HIPCHECK(hipEventRecord(c->ev_prep_free[prep - c->prep.data()], c->stream));
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
  P = prepare_batch(ctx, probs, nprob);
  FitKeep keep;
  const int mem = probs[0].mem;
  // Prediction lanes: with device-memory outputs and no chain between the predictions, outputs
  // alternate over the context's two streams, each lane with its own workspace (name suffix), so
  // one output's memory-bound passes (merge, adjoint, rows) run beside the other's DP / MFMA work
  // (whitening, variance GEMM).  A lane's host syncs (q(u)'s Cholesky status) wait for that lane
  // only.
  // Host-memory batches without a chain: the test inputs go up once after the fit (t* sorted once;
  // every distinct v* base -- GPAR's outputs read column prefixes of one N* x P matrix -- in one
  // linear copy), the predictions run on device buffers (with lanes), and the means / stds come
  // down at the end.  (With a chain, later outputs read host columns the earlier predictions
  // write: those predictions keep the per-output host path.)
  const bool stage = mem == GPAR_MEM_HOST && !chain;
  const bool lanes = (mem == GPAR_MEM_DEVICE || stage) && !chain && nprob > 1 &&
                     ctx->predict_lanes > 1;
  // the predictions' workspace (named buffers, reused across the outputs: the largest counts)
  int64_t pred_bytes = 0;
  for (const auto& p : P)
    pred_bytes = std::max(pred_bytes, predict_ws_estimate(p.n, n_star, p.mp, p.d, mode, samples,
                                                          mode == GPAR_PREDICT_ANALYTIC &&
                                                              ctx->predict_fused &&
                                                              predict_var_tiles(p.mp) > 0));
  int64_t stage_bytes = 0;
  if (stage) {
    stage_bytes = 8 * n_star * (1 + 2 * (int64_t)nprob);
    for (int i = 0; i < nprob; ++i) stage_bytes += 8 * n_star * ldvs[i];   // upper bound
  }
  fit_impl(ctx, P, log_theta0, o, theta_out, nlml_out, evals_out, &keep,
           (lanes ? 2 : 1) * pred_bytes + stage_bytes);
  std::vector<int64_t> perm;
  std::vector<const double*> vs_dev(nprob, nullptr);
  std::vector<int64_t> lds_dev(nprob, 0);
  const double* ts_dev = t_star;
  double* res = nullptr;   // staged outputs: [nprob][mean, std][n_star]
  if (stage) {
    if (!std::is_sorted(t_star, t_star + n_star)) {
      perm.resize(n_star);
      for (int64_t k = 0; k < n_star; ++k) perm[k] = k;
      std::stable_sort(perm.begin(), perm.end(),
                       [&](int64_t a, int64_t b) { return t_star[a] < t_star[b]; });
    }
    std::vector<double> tmp;
    double* tsd = ws<double>(ctx, "fph_ts", n_star);
    if (perm.empty()) {
      h2d(ctx, tsd, t_star, n_star);
    } else {
      tmp.resize(n_star);
      for (int64_t k = 0; k < n_star; ++k) tmp[k] = t_star[perm[k]];
      h2d(ctx, tsd, tmp.data(), n_star);
      sync(ctx);
    }
    ts_dev = tsd;
    std::vector<int> grp(nprob, -1);
    int ng = 0;
    for (int i = 0; i < nprob; ++i) {
      for (int j = 0; j < i && grp[i] < 0; ++j)
        if (v_star[j] == v_star[i] && ldvs[j] == ldvs[i]) grp[i] = grp[j];
      if (grp[i] < 0) grp[i] = ng++;
    }
    for (int g = 0; g < ng; ++g) {
      int64_t wmax = 0;
      int first = -1;
      for (int i = 0; i < nprob; ++i)
        if (grp[i] == g) {
          wmax = std::max(wmax, probs[i].d);
          if (first < 0) first = i;
        }
      std::pair<const double*, int64_t> b;
      if (perm.empty()) {
        b = upload_shared_block(ctx, "fph_vs" + std::to_string(g), v_star[first], ldvs[first], wmax,
                                n_star);
      } else {   // the rows in t*'s ascending order, gathered on the host
        tmp.assign((size_t)n_star * wmax, 0.0);
        for (int64_t k = 0; k < n_star; ++k)
          for (int64_t q = 0; q < wmax; ++q) tmp[k * wmax + q] = v_star[first][perm[k] * ldvs[first] + q];
        b = upload_shared_block(ctx, "fph_vs" + std::to_string(g), tmp.data(), wmax, wmax, n_star);
        sync(ctx);
      }
      for (int i = 0; i < nprob; ++i)
        if (grp[i] == g) {
          vs_dev[i] = b.first;
          lds_dev[i] = b.second;
        }
    }
    res = ws<double>(ctx, "fph_res", (size_t)nprob * 2 * n_star);
  }
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
    if (stage)
      predict_impl(ctx, P[i], th, GPAR_MEM_DEVICE, n_star, ts_dev, vs_dev[i], lds_dev[i], mode,
                   samples, seed + (uint64_t)i, res + (size_t)(2 * i) * n_star,
                   res + (size_t)(2 * i + 1) * n_star, keep.valid[i] ? &keep.gram[i] : nullptr,
                   /*defer=*/true, pre.empty() ? nullptr : &pre[i]);
    else
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
  if (lanes || stage || (chain && mem == GPAR_MEM_DEVICE)) sync(ctx);
  if (stage) {   // the staged means / stds into the caller's host buffers, in t*'s input order
    std::vector<double> h(perm.empty() ? 0 : (size_t)2 * n_star);
    for (int i = 0; i < nprob; ++i) {
      const double* src = res + (size_t)(2 * i) * n_star;
      if (perm.empty()) {
        d2h(ctx, mean_out[i], src, n_star);
        d2h(ctx, std_out[i], src + n_star, n_star);
      } else {
        d2h(ctx, h.data(), src, (size_t)2 * n_star);
        sync(ctx);
        for (int64_t k = 0; k < n_star; ++k) {
          mean_out[i][perm[k]] = h[k];
          std_out[i][perm[k]] = h[n_star + k];
        }
      }
    }
    sync(ctx);
  }
}
}  // namespace gpar
using namespace gpar;
extern "C" {

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
  const int sdim = sde_dim(kernel);
  // draw (s, k, i) is counter_normal(seed, s, k (sdim + 1) + i): the index must fit 32 bits
  ARGCHECK(n * (sdim + 1) <= ((int64_t)1 << 32), "n * (state dimension + 1) must be <= 2^32");
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
}  // extern "C"

// ---------------------------------------------------------------- posterior objects
// gpar_fit_posterior keeps, per output, everything get_gpar_scaled_predictions computes before it
// reads the inference inputs (gpar_scaled_inference.jl:20-73: the fit and q(u), :141-196), so a
// caller whose inference inputs arrive later -- the chained sweep of GPAR_scaled_examples.jl:172,
// eeg.jl:249,274, one owner per output across ranks -- runs only the V*-dependent prediction per
// output (gpar_posterior_predict).
struct gpar_posterior {
  // unique over the process's lifetime: gpar_posterior_prepare's slots match on it, so a slot left
  // by a destroyed posterior can never be taken for a new one at the same address
  uint64_t id = 0;
  int device = 0;
  int mem = GPAR_MEM_DEVICE;   // memory space of the problems (and of every predict call's I/O)
  struct Out {
    gpar::DevProblem p;        // t, v, z, y: borrowed (device problems) or owned (host problems)
    gpar::Theta th;
    gpar::QuPre q;             // me, w, X1, Vm, cov in owned device memory
  };
  std::vector<Out> outs;
  std::vector<void*> owned;    // hipMalloc'd blocks, freed by gpar_posterior_destroy
  ~gpar_posterior() {
    (void)hipSetDevice(device);
    for (void* b : owned) (void)hipFree(b);
  }
};

namespace gpar {

static double* post_alloc(gpar_posterior* post, size_t doubles) {
  void* b = nullptr;
  const hipError_t e = hipMalloc(&b, std::max<size_t>(doubles, 1) * sizeof(double));
  if (e != hipSuccess) {
    (void)hipGetLastError();
    throw Error(e == hipErrorOutOfMemory ? GPAR_ERR_OOM : GPAR_ERR_HIP,
                std::string("gpar_fit_posterior: hipMalloc: ") + hipGetErrorString(e));
  }
  post->owned.push_back(b);
  return reinterpret_cast<double*>(b);
}

// device copy of `doubles` doubles on the context stream into posterior-owned memory
static const double* post_keep(gpar_ctx* c, gpar_posterior* post, const double* src, size_t doubles) {
  double* dst = post_alloc(post, doubles);
  HIPCHECK(hipMemcpyAsync(dst, src, doubles * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
  return dst;
}

}  // namespace gpar

using namespace gpar;
extern "C" {

int32_t gpar_fit_posterior(gpar_ctx* ctx, const gpar_problem* probs, int32_t nprob,
                           const double* log_theta0, const gpar_fit_options* opts,
                           double* theta_out, double* nlml_out, int32_t* evals_out,
                           gpar_posterior** out) {
  if (out) *out = nullptr;
  std::unique_ptr<gpar_posterior> post;
  API_BEGIN(ctx)
  ARGCHECK(probs && nprob >= 1 && log_theta0 && theta_out && out, "null argument");
  check_batch(probs, nprob);
  gpar_fit_options o{0, 1000, 1e-8, 0.0};
  if (opts) o = *opts;
  std::vector<DevProblem> P;
  P = prepare_batch(ctx, probs, nprob);
  FitKeep keep;
  fit_impl(ctx, P, log_theta0, o, theta_out, nlml_out, evals_out, &keep);
  post.reset(new gpar_posterior());
  static std::atomic<uint64_t> next_id{1};
  post->id = next_id.fetch_add(1);
  post->device = ctx->device;
  post->mem = probs[0].mem;
  post->outs.resize(nprob);
  for (int i = 0; i < nprob; ++i) {
    const double* q = theta_out + 5 * i;
    post->outs[i].th = Theta{q[0], q[1], q[2], q[3], q[4]};
  }
  // q(u) batched per convention (run_q_u_batch takes one), each batch copied out of the workspace
  // before the next overwrites it
  for (int qn : {0, 1}) {
    std::vector<int> idx;
    for (int i = 0; i < nprob; ++i)
      if (P[i].qu_noise == qn) idx.push_back(i);
    if (idx.empty()) continue;
    std::vector<DevProblem> Pq;
    std::vector<Theta> Tq;
    FitKeep kq;
    for (int i : idx) {
      Pq.push_back(P[i]);
      Tq.push_back(post->outs[i].th);
      kq.gram.push_back(keep.gram[i]);
      kq.valid.push_back(keep.valid[i]);
    }
    std::vector<QuPre> pre = run_q_u_batch(ctx, Pq, Tq, kq, /*want_cov=*/true);
    for (size_t a = 0; a < idx.size(); ++a) {
      const QuPre& s = pre[a];
      const size_t sq = (size_t)s.ld * s.ld;
      QuPre& d = post->outs[idx[a]].q;
      d = s;
      d.Lu = d.LD = nullptr;   // prediction reads w, X1, Vm (and me, cov: MC / path) only
      d.me = post_keep(ctx, post.get(), s.me, s.ld);
      d.w = post_keep(ctx, post.get(), s.w, s.ld);
      d.X1 = post_keep(ctx, post.get(), s.X1, sq);
      d.Vm = post_keep(ctx, post.get(), s.Vm, sq);
      d.cov = post_keep(ctx, post.get(), s.cov, sq);
    }
    sync(ctx);
  }
  // the problems: device inputs stay the caller's (borrowed until gpar_posterior_destroy); host
  // inputs were uploaded into workspace that later calls reuse, so they are copied (a time grid or
  // input base several outputs share, once)
  std::unordered_map<const double*, const double*> shared;
  auto keep_once = [&](const double* src, size_t doubles) {
    auto it = shared.find(src);
    if (it != shared.end()) return it->second;
    const double* dst = post_keep(ctx, post.get(), src, doubles);
    shared[src] = dst;
    return dst;
  };
  for (int i = 0; i < nprob; ++i) {
    DevProblem d = P[i];
    d.d2 = nullptr;   // the fit's distance cache is not the posterior's
    d.cache_slot = -1;
    d.zc = post_keep(ctx, post.get(), P[i].zc, (size_t)((d.mp + 255) / 256) * zc_stride((int)d.d));
    if (probs[0].mem == GPAR_MEM_HOST) {
      d.t = keep_once(P[i].t, d.n);
      d.y = post_keep(ctx, post.get(), P[i].y, d.n);
      d.v = keep_once(P[i].v, (size_t)d.n * d.ldv);
      d.z = post_keep(ctx, post.get(), P[i].z, (size_t)d.m * d.ldz);
    }
    post->outs[i].p = d;
  }
  sync(ctx);
  *out = post.release();
  API_END(ctx)
}

int32_t gpar_posterior_prepare(gpar_ctx* ctx, const gpar_posterior* post, int32_t i,
                               int64_t n_star, const double* t_star) {
  API_BEGIN(ctx)
  ARGCHECK(post && t_star, "null argument");
  ARGCHECK(post->device == ctx->device, "the posterior belongs to another device's context");
  ARGCHECK(post->mem == GPAR_MEM_DEVICE, "gpar_posterior_prepare: device-memory posteriors only");
  ARGCHECK(i >= 0 && i < (int32_t)post->outs.size(), "output index out of range");
  ARGCHECK(n_star >= 1, "n_star must be >= 1");
  const gpar_posterior::Out& o = post->outs[i];
  const DevProblem& P = o.p;
  if (ctx->prep.empty()) ctx->prep.resize(2);
  for (int k = 0; k < 2; ++k)
    for (hipEvent_t* ev : {&ctx->ev_prep_ready[k], &ctx->ev_prep_free[k]})
      if (!*ev) HIPCHECK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
  const int slot = ctx->prep_next;
  ctx->prep_next ^= 1;
  PredPrep& s = ctx->prep[slot];
  s.valid = false;
  // the side stream follows the context stream (inputs, earlier calls) and the slot's last reader
  HIPCHECK(hipEventRecord(ctx->ev_fork, ctx->main));
  HIPCHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
  HIPCHECK(hipStreamWaitEvent(ctx->side, ctx->ev_prep_free[slot], 0));
  const std::string tag = "prep" + std::to_string(slot);
  const int64_t nt = P.n + n_star;
  const int64_t nch = (nt + kChunk - 1) / kChunk;
  {
    OnStream on_(ctx, ctx->side);
    // the merged grid's times and noise (predict_impl merges the inputs again, identically)
    double* tm = ws<double>(ctx, tag + "_tm", nt);
    double* ym = ws<double>(ctx, tag + "_ym", nt);
    double* rm = ws<double>(ctx, tag + "_rm", nt);
    const double s2 = o.th.sigma * o.th.sigma;
    launch_merge_side(ctx->stream, P.t, P.n, t_star, n_star, 0, P.y, s2, nullptr, 0, 0, tm, ym, rm,
                      nullptr, 0, nullptr);
    launch_merge_side(ctx->stream, t_star, n_star, P.t, P.n, 1, nullptr, 1e10, nullptr, 0, 0, tm, ym,
                      rm, nullptr, 0, nullptr);
    check_launch("prepare: merge");
    std::vector<ChainParamsHost> cps{{1.0 / o.th.l_t, o.th.l_t, o.th.sv_t * o.th.sv_t, s2}};
    s.g = run_gains(ctx, P.sdim, tm, nt, cps, rm, false, tag);
    s.h = ws<double>(ctx, tag + "_h", (size_t)nt * 4);
    launch_gains_adjoint(ctx->stream, P.sdim, s.g.rec, nt, kChunk, nch, 1, s.h);
    check_launch("prepare: gains");
    HIPCHECK(hipEventRecord(ctx->ev_prep_ready[slot], ctx->side));
  }
  s.post_id = post->id;
  s.out = i;
  s.ts = t_star;
  s.n_star = n_star;
  s.valid = true;
  API_END(ctx)
}

int32_t gpar_posterior_predict(gpar_ctx* ctx, const gpar_posterior* post, int32_t i,
                               int64_t n_star, const double* t_star, const double* v_star,
                               int64_t ldvs, int32_t mode, int32_t samples, uint64_t seed,
                               double* mean, double* std) {
  API_BEGIN(ctx)
  ARGCHECK(post && t_star && v_star && mean && std, "null argument");
  ARGCHECK(post->device == ctx->device, "the posterior belongs to another device's context");
  ARGCHECK(i >= 0 && i < (int32_t)post->outs.size(), "output index out of range");
  const gpar_posterior::Out& o = post->outs[i];
  ARGCHECK(n_star >= 1, "n_star must be >= 1");
  ARGCHECK(ldvs >= o.p.d, "ldvs must be >= d");
  ARGCHECK(mode == GPAR_PREDICT_ANALYTIC || mode == GPAR_PREDICT_MC || mode == GPAR_PREDICT_PATH,
           "bad mode");
  if (mode != GPAR_PREDICT_ANALYTIC)
    ARGCHECK(samples >= 2 && samples <= kMaxSamples, "MC / path modes take 2..65536 samples");
  // a slot gpar_posterior_prepare filled for this output and these test times
  const PredPrep* prep = nullptr;
  for (PredPrep& s : ctx->prep)
    if (s.valid && s.post_id == post->id && s.out == i && s.ts == t_star && s.n_star == n_star) {
      s.valid = false;
      prep = &s;
    }
  predict_impl(ctx, o.p, o.th, post->mem, n_star, t_star, v_star, ldvs, mode, samples, seed, mean,
               std, nullptr, false, &o.q, prep);
  API_END(ctx)
}

int32_t gpar_posterior_destroy(gpar_posterior* post) {
  delete post;
  return GPAR_OK;
}

}  // extern "C"
