// launch.hpp -- host-callable launch wrappers of the gfx950 kernels (one per .hip file).
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdint>

namespace gpar {

// Mirrors of the device job structs (identical layout).
struct ChainParamsHost {
  double inv_l, l, s, r;
};
struct KuuJobHost {
  const double* z;
  int64_t ldz;
  int d;
  int kind;
  double inv_l, s, diag_add;
  double* K;
  int64_t ldk;
  int m;
  int mpad;
};
struct CholJobHost {
  double* A;
  int64_t ld;
  int m;
  double diag_add;
  int* status;
};
struct TrsmJobHost {
  const double* L;
  int64_t ldl;
  const double* B;
  int64_t ldb;
  double* X;
  int64_t ldx;
  int m;
  int64_t ncols;
  int transB;
  int transX;
};
struct FinishJobHost {
  const double* Lu;
  const double* Llam;
  int64_t ld;
  int m;
  const double* r;
  const double* logs;
  int64_t nch;
  const double* a2part;
  int64_t npart;
  int64_t n;
  const int* status;
  double* out;
  double* me;
};

struct TrsvJobHost {
  const double* L;
  int64_t ld;
  int m;
  const double* b;
  double* x;
  int trans;
};

struct GramPlan {
  int npan = 0, nsplit = 0;   // 64-column panels, time splits of r (the DG kernel's)
  int64_t part_doubles = 0, rpart_doubles = 0;
  // v2 decomposition (k_gram.hip): OFF / DG workgroup counts, their time splits and rows
  int v2 = 0, noff = 0, ndg = 0, soff = 0, sdg = 0;
  int64_t rows_off = 0, rows_dg = 0;
  // one workgroup per CU (gram_plan(..., one_per_cu)): launched with padding LDS so a second Gram
  // workgroup cannot join, leaving each CU room for the other stream lane's whitening
  int one_per_cu = 0;
  int v3 = 0;   // fat-wave kernels (gram3_*: 2-wave workgroups, 32-tile OFF waves)
  int ncs = 0;  // v3 chunk-correction splits
  int ncs_slim = 0;  // ... of the slim correction that runs beside the OFF kernel
  // v3 DG time splits sized apart: the first dg_sw take dg_rows_w rows each (0: all rows_dg)
  int dg_sw = 0;
  int64_t dg_rows_w = 0;
};

// Grouped Gram (one set of launches for several outputs of one size, grid y = output): each
// kernel takes its per-output pointers from row blockIdx.y of this device table
struct GramGroupPtrs {
  const double* beta;
  const double* alpha;
  const double* ecor;
  const double* cin;
  const double* qv;
  double* part;
  double* rpart;
  double* G;
  double* r;
};

constexpr int kGramTile = 128;
constexpr int kBKRows = 16;   // the Gram kernels' time rows per K-step (gram_common.hpp kBK)
constexpr int kRecStride3 = 16;

inline int rec_size(int sdim) { return sdim == 3 ? 16 : (sdim == 2 ? 8 : 4); }

// k_lgssm.hip
// phase-3 launches of launch_gains by path (k_lgssm.hip; gpar_debug_counter)
extern std::atomic<int64_t> g_gains_fast_launches, g_gains_general_launches;
void launch_gains(hipStream_t st, int sdim, const double* t, int64_t n, int L, int64_t nch,
                  int nchains, const ChainParamsHost* cps_dev, const double* noise,
                  double* agg, double* pstart, double* rec, double* g, double* phi,
                  double* logs, double* pf, const double* const* ys = nullptr,
                  double* alpha_loc = nullptr, double* asend = nullptr, bool compact = false,
                  bool ys_aligned16 = false, double* moments = nullptr);
// the chains' logpdf from the gains' moments (moments != null in launch_gains; kMomStride doubles
// per chunk) and the carried chunk states cin [nchains][nch][4]
constexpr int kGainsMomStride = 12;
// a chain's logpdf from the phase-3 moments, its chunk carry included (one workgroup per chain);
// nm (optional): the chains fit on the device (nm_dev.hpp) -- each chain's Nelder-Mead machine
// takes the value and writes the next round's parameters into cps; active[chain] = 1 while its
// machine runs
template <int N>
struct NmDev;
void launch_chain_carry_lml(hipStream_t st, int sdim, const double* phi, int64_t phistride,
                            const double* send, int64_t sstride, const double* logs,
                            const double* mom, int64_t nch, int64_t n, int nchains, double* lml,
                            NmDev<3>* nm = nullptr, ChainParamsHost* cps = nullptr,
                            int* active = nullptr);
// compact gains records {K, rs, pad} (gains_phase3<D, true>): doubles per step
inline int crec_size(int sdim) { return sdim == 1 ? 2 : 4; }
int dp_bucket(int d);
void launch_whiten_kfu(hipStream_t st, int time_kind, int out_kind, const double* rec,
                       const double* v, int64_t ldv, int d, const double* z, int64_t ldz,
                       int64_t m, int64_t mp, int64_t n, int L, int64_t nch, double inv_lo,
                       double s_o, double* beta, int64_t ldb, double* send, int64_t mc,
                       const double* g, double* hsum);
// MFMA Gram-form Kfu (smooth out kernels: Matern-3/2, Matern-5/2, EQ); zc: (mp/256) x 64
// pseudo-input centres from launch_zcenter (theta-independent: once per problem)
int mfma_dp_bucket(int d);
void launch_zcenter(hipStream_t st, const double* z, int64_t ldz, int d, int64_t m, int64_t mp,
                    double* zc);
void launch_whiten_kfu_mfma(hipStream_t st, int time_kind, int out_kind, const double* rec,
                            const double* v, int64_t ldv, int d, const double* z, int64_t ldz,
                            const double* zc, int64_t m, int64_t mp, int64_t n, int L, int64_t nch,
                            double inv_lo, double s_o, double* beta, int64_t ldb, double* send,
                            int64_t mc, const double* g, double* hsum);
// k_dist.hip: D > 64 (and any D when the distances are precomputed).  zc_stride(d): doubles per
// 256-column group in the centres array (launch_zcenter for d <= 64, launch_zcenter_wide above).
int64_t zc_stride(int d);
void launch_zcenter_wide(hipStream_t st, const double* z, int64_t ldz, int d, int64_t m,
                         int64_t mp, double* zc);
// d2[k][c] (k < n, c < mp; 0 for c >= m) into out (ld ldo): MFMA Gram form, centred per 256-column
// group (smooth kernels), or direct differences (out_kind = Matern-1/2); take_sqrt: r = sqrt_pos(d2)
// instead (the Matern kernels' distance cache)
void launch_dist2(hipStream_t st, int out_kind, const double* v, int64_t ldv, int64_t n,
                  const double* z, int64_t ldz, int64_t m, int64_t mp, int d, const double* zc,
                  double* out, int64_t ldo, bool take_sqrt = false);
// whiten_kfu from precomputed squared distances (src may equal beta: in place), or from the
// distances themselves (src_is_r: the fit's cache for the Matern kernels)
void launch_whiten_kfu_d2(hipStream_t st, int time_kind, int out_kind, const double* rec,
                          const double* src, int64_t lds, int64_t m, int64_t mp, int64_t n, int L,
                          int64_t nch, double inv_lo, double s_o, double* beta, int64_t ldb,
                          double* send, int64_t mc, const double* g, double* hsum,
                          bool src_is_r = false, const double* t_compact = nullptr,
                          double l_t = 0.0);
void launch_whiten_vec(hipStream_t st, int sdim, const double* rec, int64_t recstride,
                       const double* y, int64_t ldy, int64_t n, int L, int64_t nch, int nchains,
                       double* alpha, int64_t lda, double* send, int64_t sendstride, int64_t mc,
                       int64_t col, int64_t astride = 1);
int carry_group_size(int64_t nch);
// gend/gin: nchains * ngroups * mc * 4 doubles; psi: nchains * ngroups * sdim^2 doubles
void launch_carry(hipStream_t st, int sdim, const double* phi, int64_t phistride,
                  const double* send, double* cin, int64_t sstride, int64_t nch, int64_t mc,
                  int64_t ncols, int nchains, double* gend, double* gin, double* psi,
                  bool rev = false);
// adjoint (backward) pass helpers
void launch_gains_adjoint(hipStream_t st, int sdim, const double* rec, int64_t n, int L,
                          int64_t nch, int nchains, double* h);
void launch_adjoint_local(hipStream_t st, int sdim, double* X, int64_t ldx, int64_t ncols,
                          const double* rec, const double* g, const double* cin, int64_t mc,
                          int64_t n, int L, int64_t nch, double* bend, int nchains = 1,
                          int64_t xstride = 0, int64_t sstride = 0);
// Single chain, many columns (prediction): LDS-staged gains; wmask (optional): write u only at
// rows with wmask[k] >= 1e10 (the merged grid's test points).
void launch_adjoint_local_wide(hipStream_t st, int sdim, double* X, int64_t ldx, int64_t ncols,
                               const double* rec, const double* g, const double* cin, int64_t mc,
                               int64_t n, int L, int64_t nch, double* bend, const double* wmask);
// temporal chains: smoothed mean f = y - R Sigma^{-1} y, smoothed variance of f (RTS)
void launch_smooth_mean(hipStream_t st, int sdim, const double* u, const double* h,
                        const double* chat, int64_t sstride, const double* y, int64_t ldy,
                        const double* noise, const ChainParamsHost* cps, int64_t n, int L,
                        int nchains, double* mean, int64_t ldm);
// vloc/var: nchains * n; gam: nchains * n * 4; agg: nchains * nch * 2 sdim^2; phat: nchains * nch * sdim^2
// scratch: cov_carry_scratch_doubles(sdim, nch, nchains) doubles (the carry's group maps)
int64_t cov_carry_scratch_doubles(int sdim, int64_t nch, int nchains);
void launch_cov_smooth(hipStream_t st, int sdim, const double* t, const double* rec,
                       const double* pf, const ChainParamsHost* cps, int64_t n, int L,
                       int64_t nch, int nchains, double* vloc, double* gam, double* agg,
                       double* phat, double* var, int64_t ldv, double* scratch,
                       bool local_done = false);
// the chains' backward pass (h, u in place of X, bend; vloc, gam, agg) in one launch: what
// launch_gains_adjoint + launch_adjoint_local (one column) + cov_local compute, bit for bit
void launch_smooth_back(hipStream_t st, int sdim, const double* rec, const double* g,
                        const double* pf, const ChainParamsHost* cps, const double* cin, double* X,
                        double* h, double* vloc, double* gam, double* agg, double* bend, int64_t n,
                        int L, int64_t nch, int nchains, int64_t xstride, int64_t sstride);
int64_t vec_fix_blocks(int64_t n);
void launch_vec_fix(hipStream_t st, int sdim, double* alpha, int64_t lda, const double* g,
                    int64_t gstride, const double* cin, int64_t sstride, int64_t mc,
                    int64_t col, int64_t n, int L, int nchains, double* part,
                    double* hsum = nullptr, int64_t ncols = 0, double* qout = nullptr);
void launch_chain_lml(hipStream_t st, const double* logs, int64_t nch, const double* a2part,
                      int64_t npart, int64_t n, int nchains, double* lml);

// k_gram.hip
// cus: the CUs the Gram's stream may use (v3 plan; 256 = the whole chip)
// dg_cus: the CUs the v3 DG kernel's items are planned for (0: cus)
GramPlan gram_plan(int64_t n, int64_t mp, bool one_per_cu = false, int cus = 256, int dg_cus = 0);
// ecor: E_j (nch x mc x 4, vec_fix), cin: C_j (carry), qv: q_j (nch x 4, vec_fix)
void launch_gram(hipStream_t st, int sdim, const GramPlan& plan, const double* beta,
                 int64_t ldb, int64_t n, const double* ecor, const double* cin, const double* qv,
                 int64_t mc, int L, const double* alpha, double* part, double* rpart, double* G,
                 int64_t ldg, double* r, hipStream_t side = nullptr,
                 hipEvent_t ev_a = nullptr, hipEvent_t ev_b = nullptr,
                 hipStream_t st_w = nullptr, hipEvent_t ev_w = nullptr, int w_items = 0);
void launch_gram_grouped(hipStream_t st, int sdim, const GramPlan& plan, const GramGroupPtrs* grp,
                         int ngrp, int64_t ldb, int64_t n, int64_t mc, int L, int64_t ldg,
                         hipStream_t side, hipEvent_t ev_a, hipEvent_t ev_b);
void launch_beta_fix(hipStream_t st, int sdim, double* beta, int64_t ldb, int64_t n,
                     const double* g, const double* cin, int64_t mc, int L);

// k_dense.hip
void launch_kuu(hipStream_t st, const KuuJobHost* jobs_dev, int njobs, int mmax);
void launch_chol(hipStream_t st, const CholJobHost* jobs_dev, int njobs);
void launch_trsm(hipStream_t st, const TrsmJobHost* jobs_dev, int njobs, int64_t ncols_max);
void launch_finish(hipStream_t st, const FinishJobHost* jobs_dev, int njobs);
void launch_gram_small(hipStream_t st, const double* X, int64_t ldx, int m, double* C,
                       int64_t ldc);
void launch_lower_to_upper_colmajor(hipStream_t st, const double* L, int64_t ldl, int m,
                                    double* U);
void launch_eye(hipStream_t st, double* A, int64_t ld, int m);
void launch_trsv(hipStream_t st, const TrsvJobHost* jobs_dev, int njobs);

// k_predict.hip
void launch_merge_side(hipStream_t st, const double* ts, int64_t ns, const double* other,
                       int64_t no, int is_test, const double* ys, double rval, const double* vs,
                       int64_t ldvs, int d, double* tm, double* ym, double* rm, double* vm,
                       int64_t ldvm, int64_t* pos_out);
void launch_predict_rows(hipStream_t st, int sdim, const double* X, int64_t ldx, const double* h,
                         const double* chat, int64_t mc, int64_t mp, int64_t m, int L,
                         const int64_t* pos, int64_t nstar, const double* rm, const double* ym,
                         const double* w, double* Q, int64_t ldq, double* mean);
// fused predict_rows + ANALYTIC variance (Mp in {128, 256, 384, 512}: predict_var_tiles(Mp) > 0;
// V zero outside its m x m block, ld = Mp)
int predict_var_tiles(int64_t mp);
void launch_predict_var(hipStream_t st, int sdim, const double* X, int64_t ldx, const double* h,
                        const double* chat, int64_t mc, int64_t mp, int64_t m, int L,
                        const int64_t* pos, int64_t nstar, const double* rm, const double* ym,
                        const double* w, const double* V, int64_t ldv, double* mean, double* stdv);
void launch_gemm_nt(hipStream_t st, const double* A, int64_t lda, const double* B, int64_t ldb,
                    int64_t rows, int64_t cols, int64_t K, int mode, double* C, int64_t ldc,
                    double* rowsq, int64_t valid_cols, const double* base, double* out0,
                    double* out1, int tri = 0);
void launch_rowsq_finish(hipStream_t st, const double* rowsq, int64_t rows, int nblk,
                         double* std_out);
void launch_mc_stats_finish(hipStream_t st, const double* part, int64_t rows, int nblk, int64_t S,
                           const double* base, double* out0, double* out1);
void launch_mc_factor(hipStream_t st, const double* Lc, const double* X, int64_t ld, int m,
                      double* W);
void launch_pad_identity_copy(hipStream_t st, const double* src, int64_t ld, int m, double* dst);
void launch_normal(hipStream_t st, double* xi, int64_t ld, int64_t S, int64_t M, int64_t Sp,
                   uint64_t seed);
void launch_scatter_chains(hipStream_t st, const double* src, int64_t lds, int64_t ns,
                           const int64_t* pos, double* dst, int64_t ldd, int nchains);
void launch_gather_chains(hipStream_t st, const double* src, int64_t lds, int64_t ns,
                          const int64_t* pos, double* dst, int64_t ldd, int nchains);

// k_path.hip (posterior path sampling: the simulation smoother batched over samples; layouts in
// the file header)
void launch_kfu_from_dist(hipStream_t st, int out_kind, double* K, int64_t n, int64_t m,
                          int64_t mp, double inv_l, double s);
void launch_path_bmat(hipStream_t st, const double* W, int64_t ld, const double* w, const double* xi,
                      int64_t ldxi, int S, int m, int64_t mp, double* Bm, int64_t ldb);
void launch_dk_consts(hipStream_t st, int sdim, const double* t, int64_t n, double inv_l, double s,
                      double* lq);
void launch_dk_phi(hipStream_t st, int sdim, const double* rec, int64_t n, int L, int64_t nch,
                   double* phia);
void launch_dk_prior(hipStream_t st, int sdim, const double* rec, const double* lq,
                     const double* noise, double r, int64_t n, int L, int64_t nch, int S,
                     uint64_t seed, const double* ym, const double* fx, int64_t ldfx,
                     const double* cin, double* send, double* ft, double* z);
void launch_dk_finish(hipStream_t st, int sdim, const double* X, int64_t ldx, const double* h,
                      const double* chat, const double* z, const double* noise, double r,
                      int64_t n, int L, int64_t nch, int S, double* f);
void launch_path_stats(hipStream_t st, const double* fx, int64_t ldfx, const double* F, int S,
                       const int64_t* pos, int64_t nstar, double* mean, double* std);
void launch_path_transpose(hipStream_t st, const double* F, int64_t n, int S, double* out);

// k_exact.hip
void launch_exact_cov(hipStream_t st, const double* x, int64_t ldx, int64_t n, const double* x2,
                      int64_t ldx2, int64_t n2, int dx, int tk, int ok, double inv_lt, double s_t,
                      double inv_lo, double s_o, double diag, double* K, int64_t ldk);
void launch_exact_logpdf_finish(hipStream_t st, const double* L, int64_t ld, int n, const double* w,
                                const int* status, double* out);
void launch_exact_post(hipStream_t st, const double* W, int64_t ldw, int n, int64_t n_star,
                       const double* w, double kss, double* mean, double* var);

// k_chol.hip (blocked dense tail)
struct CholJob2Host {
  double* A;
  double* T;
  double* Td;
  int* status;
};
struct TgtJobHost {
  const double* T;
  const double* G;
  double* X;
  double* Lam;
};
struct Finish2JobHost {
  const double* Tu;
  const double* Llam;
  const double* Tdl;
  const double* r;
  const double* logs;
  int64_t nch;
  const double* a2part;
  int64_t npart;
  int64_t n;
  const int* status;
  double* out;
  double* me;
};
constexpr int kDenseNB = 64;
void launch_chol_blocked(hipStream_t st, const CholJob2Host* jobs_dev, int njobs, int64_t ld,
                         int nb, bool want_t);
void launch_tgt(hipStream_t st, const TgtJobHost* jobs_dev, int njobs, int64_t ld, int nb);
void launch_finish2(hipStream_t st, const Finish2JobHost* jobs_dev, int njobs, int64_t ld, int nb);
// X = T G only (tgt mode 0): V = L_D^-1 L_u^-1 from the two inverses
void launch_tg(hipStream_t st, const TgtJobHost* jobs_dev, int njobs, int64_t ld, int nb);
void launch_gemv_tn_lower(hipStream_t st, const double* T, int64_t ld, int mp, const double* x,
                          double* y);

}  // namespace gpar
