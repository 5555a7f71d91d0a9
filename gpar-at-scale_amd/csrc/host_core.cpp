// host_core.cpp -- workspace, uploads, problems on the device, the gains pass (see host.hpp).
#include "host.hpp"

namespace gpar {

void flush_stats(gpar_ctx* c) {
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
  for (auto& q : c->mark_seqs) {
    for (size_t i = 1; i < q.ev.size(); ++i) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, q.ev[i - 1], q.ev[i]) == hipSuccess) {
        auto& st = c->stats[q.names[i]];
        st.ms += ms;
        st.launches += 1;
      }
    }
    for (hipEvent_t e : q.ev) (void)hipEventDestroy(e);
  }
  c->mark_seqs.clear();
  (void)hipGetLastError();   // an event pair that was never recorded must not fail a later launch check
}

void sync_all(gpar_ctx* c) {
  for (hipStream_t st : {c->main, c->side, c->s_w, c->s_g, c->s_g2, c->s_d})
    if (st) HIPCHECK(hipStreamSynchronize(st));
}

// Free distance-cache buffers, the highest slots first, until at least `bytes` are released
// (INT64_MAX: all of them), once all queued work is done (nothing in flight can still read
// them), and mark those slots gone: whiten_kfu_any checks the slot before every launch.
// Returns the bytes freed.
int64_t release_dist_cache(gpar_ctx* c, int64_t bytes) {
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
void* ws_bytes(gpar_ctx* c, const std::string& name, size_t bytes) {
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
// rows x width doubles from a host matrix with leading dimension ld into a packed device matrix:
// one linear copy when the rows are already packed (a pitched copy from pageable memory goes row
// by row: 10^6 rows of a few doubles took seconds)
void h2d_rows(gpar_ctx* c, double* dst, const double* src, int64_t ld, int64_t width,
                     int64_t rows) {
  if (ld == width)
    h2d(c, dst, src, (size_t)rows * width);
  else
    HIPCHECK(hipMemcpy2DAsync(dst, width * sizeof(double), src, ld * sizeof(double),
                              width * sizeof(double), rows, hipMemcpyHostToDevice, c->stream));
}

// Two-level carry over chunks (k_lgssm.hip launch_carry) with context workspace.
void run_carry(gpar_ctx* c, int sdim, const double* phi, int64_t phistride,
                      const double* send, double* cin, int64_t sstride, int64_t nch, int64_t mc,
                      int64_t ncols, int nchains, const std::string& tag, bool rev) {
  const int gs = carry_group_size(nch);
  const int64_t ng = (nch + gs - 1) / gs;
  double* gend = ws<double>(c, tag + "_gend", (size_t)nchains * ng * mc * 4);
  double* gin = ws<double>(c, tag + "_gin", (size_t)nchains * ng * mc * 4);
  double* psi = ws<double>(c, tag + "_psi", (size_t)nchains * ng * sdim * sdim);
  launch_carry(c->stream, sdim, phi, phistride, send, cin, sstride, nch, mc, ncols, nchains, gend,
               gin, psi, rev);
}

// Every problem of the batch shares the time grid (same caller pointer, n and SDE order): one
// batched gains launch serves them all.
bool shares_grid(const std::vector<DevProblem>& P) {
  for (auto& p : P)
    if (p.t_user != P[0].t_user || p.n != P[0].n || p.sdim != P[0].sdim) return false;
  return true;
}

// The one-lane pipelined Gram stage (run_gram_stage): several outputs on one grid, two beta
// buffers (only when a second beta fits comfortably: the north job's 4.1 GB, not the N = 1e7,
// M = 1024 stress config's 82 GB).  The CU split and the all-D distance cache apply only on top of it.
bool fit_pipelined(const gpar_ctx* c, const std::vector<DevProblem>& P, bool fix_beta) {
  int64_t mpmax = 0;
  for (auto& p : P) mpmax = std::max(mpmax, p.mp);
  const int64_t beta_bytes = (P[0].n + 16) * mpmax * (int64_t)sizeof(double);
  return P.size() > 1 && !fix_beta && c->lanes == 1 && shares_grid(P) &&
         beta_bytes <= kPipeMaxBetaBytes;
}

void check_sorted_host(const double* t, int64_t n) {
  for (int64_t k = 1; k < n; ++k)
    ARGCHECK(t[k] >= t[k - 1], "time locations must be ascending (dtc.jl:102 does not sort)");
}

// Host-side argument checks of one problem (no device work).
void check_problem(const gpar_problem& p) {
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
void check_batch(const gpar_problem* probs, int nprob) {
  ARGCHECK(probs && nprob >= 1, "null argument");
  for (int i = 0; i < nprob; ++i) {
    check_problem(probs[i]);
    ARGCHECK(probs[i].n == probs[0].n, "all problems of one call must share n");
    ARGCHECK(probs[i].mem == probs[0].mem, "all problems of one call must share one memory space");
  }
}

DevProblem prepare_problem(gpar_ctx* c, const gpar_problem& p, int idx) {
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

// Rows x width doubles of a host matrix (leading dimension ld) that several problems read as
// column prefixes: uploaded once.  The whole ld-wide block goes up in one linear copy when it is
// at most twice as wide as what they read (GPAR's outputs read the first p - 1 columns of one
// N x P matrix of earlier outputs: ld = P, widest read P - 1), else the widest prefix (pitched).
// Returns the device buffer and its leading dimension.
std::pair<const double*, int64_t> upload_shared_block(gpar_ctx* c, const std::string& name,
                                                      const double* src, int64_t ld, int64_t width,
                                                      int64_t rows) {
  const int64_t w = ld <= 2 * width ? ld : width;
  double* dst = ws<double>(c, name, (size_t)rows * w);
  h2d_rows(c, dst, src, ld, w, rows);
  return {dst, w};
}

std::vector<DevProblem> prepare_batch(gpar_ctx* c, const gpar_problem* probs, int nprob) {
  std::vector<DevProblem> P;
  if (probs[0].mem != GPAR_MEM_HOST || nprob < 2) {
    for (int i = 0; i < nprob; ++i) P.push_back(prepare_problem(c, probs[i], i));
    return P;
  }
  // host inputs several problems share -- the time grid, the matrix of earlier outputs -- go up
  // once; each problem then runs as a device problem over views of them
  std::vector<gpar_problem> q(probs, probs + nprob);
  std::vector<int> tgrp(nprob, -1), vgrp(nprob, -1);
  int nt = 0, nv = 0;
  for (int i = 0; i < nprob; ++i) {
    for (int j = 0; j < i && tgrp[i] < 0; ++j)
      if (probs[j].t == probs[i].t) tgrp[i] = tgrp[j];
    if (tgrp[i] < 0) tgrp[i] = nt++;
    for (int j = 0; j < i && vgrp[i] < 0; ++j)
      if (probs[j].v == probs[i].v && probs[j].ldv == probs[i].ldv) vgrp[i] = vgrp[j];
    if (vgrp[i] < 0) vgrp[i] = nv++;
  }
  std::vector<const double*> tdev(nt, nullptr);
  std::vector<std::pair<const double*, int64_t>> vdev(nv, {nullptr, 0});
  for (int g = 0; g < nv; ++g) {
    int64_t wmax = 0, first = -1;
    for (int i = 0; i < nprob; ++i)
      if (vgrp[i] == g) {
        wmax = std::max(wmax, probs[i].d);
        if (first < 0) first = i;
      }
    const gpar_problem& r = probs[first];
    vdev[g] = upload_shared_block(c, "pb_v" + std::to_string(g), r.v, r.ldv, wmax, r.n);
  }
  for (int i = 0; i < nprob; ++i) {
    const int g = tgrp[i];
    if (!tdev[g]) {
      double* t = ws<double>(c, "pb_t" + std::to_string(g), probs[i].n);
      h2d(c, t, probs[i].t, probs[i].n);
      tdev[g] = t;
    }
    const std::string k = "prob" + std::to_string(i);
    double* z = ws<double>(c, k + "_z", (size_t)probs[i].m * probs[i].d);
    double* y = ws<double>(c, k + "_y", probs[i].n);
    h2d(c, y, probs[i].y, probs[i].n);
    h2d_rows(c, z, probs[i].z, probs[i].ldz, probs[i].d, probs[i].m);
    q[i].t = tdev[g];
    q[i].v = vdev[vgrp[i]].first;
    q[i].ldv = vdev[vgrp[i]].second;
    q[i].z = z;
    q[i].ldz = probs[i].d;
    q[i].y = y;
    q[i].mem = GPAR_MEM_DEVICE;
    P.push_back(prepare_problem(c, q[i], i));
    P.back().t_user = probs[i].t;
  }
  return P;
}

// Data-independent per-step filter quantities for `nchains` chains sharing t (n steps).
// With ys (one device data vector per chain): the chains' alpha_loc / chunk end states are
// filtered inside the gains pass (alpha_loc: nchains x n, asend: nchains x nch x 4).
GainsPlan plan_gains(gpar_ctx* c, int sdim, const double* t, int64_t n,
                     const std::vector<ChainParamsHost>& cps, const double* noise, bool want_pf,
                     const std::string& tag, const std::vector<const double*>* ys,
                     double* alpha_loc, double* asend, bool compact, double* moments) {
  GainsPlan gp;
  gp.c = c;
  gp.sdim = sdim;
  gp.t = t;
  gp.n = n;
  gp.nchains = (int)cps.size();
  gp.nch = (n + kChunk - 1) / kChunk;
  gp.noise = noise;
  const int nchains = gp.nchains;
  const int64_t nch = gp.nch;
  const int rs = compact ? crec_size(sdim) : rec_size(sdim);
  const int d2 = sdim * sdim;
  gp.dcps = ws<ChainParamsHost>(c, tag + "_cps", nchains);
  h2d(c, gp.dcps, cps.data(), nchains);
  // the chunk aggregates in gains_phase2's run-slot order: 256 ceil(nch / 256) slots per chain
  gp.agg = ws<double>(c, tag + "_agg", (size_t)nchains * 256 * ((nch + 255) / 256) * 3 * d2);
  gp.pst = ws<double>(c, tag + "_pstart", (size_t)nchains * nch * d2);
  GainsOut& o = gp.o;
  o.recstride = n * rs;
  o.gstride = n * 4;
  // moments: the per-chunk outputs in chain_carry_lml's slot order (k_lgssm.hip mom_slot), 256
  // ceil(nch / 256) slots per chain
  gp.nchs = moments ? 256 * ((nch + 255) / 256) : nch;
  const int64_t nchs = gp.nchs;
  o.phistride = nchs * d2;
  // moments (the chains' logpdf): no per-step record or fix-up row is written
  o.rec = moments ? nullptr : ws<double>(c, tag + "_rec", (size_t)nchains * n * rs);
  o.g = moments ? nullptr : ws<double>(c, tag + "_g", (size_t)nchains * n * 4);
  o.phi = ws<double>(c, tag + "_phi", (size_t)nchains * nchs * d2);
  o.logs = ws<double>(c, tag + "_logs", (size_t)nchains * nchs);
  o.pf = want_pf ? ws<double>(c, tag + "_pf", (size_t)nchains * n * d2) : nullptr;
  o.compact = compact;
  o.t = t;
  if (ys) {
    gp.dys = ws<const double*>(c, tag + "_ys", nchains);
    h2d(c, gp.dys, ys->data(), nchains);
    gp.ys_aligned16 = true;
    for (const double* y : *ys) gp.ys_aligned16 = gp.ys_aligned16 && (uintptr_t)y % 16 == 0;
  }
  gp.alpha_loc = alpha_loc;
  gp.asend = asend;
  gp.moments = moments;
  return gp;
}

// chains [first, first + count) on stream st; the chains' arrays are strided per chain, so a
// range is a pointer offset
void GainsPlan::launch(hipStream_t st, int first, int count) const {
  if (count <= 0) return;
  const int d2 = sdim * sdim;
  OnStream on_(c, st);
  Timed tm_(c, "gains");
  launch_gains(st, sdim, t, n, kChunk, nch, count, dcps + first, noise,
               agg + (size_t)first * 256 * ((nch + 255) / 256) * 3 * d2,
               pst + (size_t)first * nch * d2,
               o.rec ? o.rec + (size_t)first * o.recstride : nullptr,
               o.g ? o.g + (size_t)first * o.gstride : nullptr,
               o.phi + (size_t)first * o.phistride, o.logs + (size_t)first * nchs,
               o.pf ? o.pf + (size_t)first * n * d2 : nullptr, dys ? dys + first : nullptr,
               alpha_loc ? alpha_loc + (size_t)first * n : nullptr,
               asend ? asend + (size_t)first * nchs * kSStride : nullptr, o.compact, ys_aligned16,
               moments ? moments + (size_t)first * nchs * kGainsMomStride : nullptr);
  check_launch("gains");
}

GainsOut run_gains(gpar_ctx* c, int sdim, const double* t, int64_t n,
                          const std::vector<ChainParamsHost>& cps, const double* noise,
                          bool want_pf, const std::string& tag,
                          const std::vector<const double*>* ys,
                          double* alpha_loc, double* asend, bool compact) {
  GainsPlan gp = plan_gains(c, sdim, t, n, cps, noise, want_pf, tag, ys, alpha_loc, asend, compact);
  gp.launch(c->stream, 0, gp.nchains);
  return gp.o;
}
}  // namespace gpar
