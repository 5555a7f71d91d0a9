// nelder_mead.hpp -- Optim.jl NelderMead() as an ask/tell state machine.
//
// Restates the optimiser the reference calls at dtc.jl:58-61 (and
// temporal_gp_inference.jl:82, optimized.jl:45,164): AffineSimplexer(a = 0.025, b = 0.5),
// AdaptiveParameters (alpha = 1, beta = 1 + 2/n, gamma = 0.75 - 1/(2n), delta = 1 - 1/n),
// convergence on the simplex value spread (g_tol), iteration cap, wall-clock time_limit,
// and Optim's after_while! (evaluate the centroid, keep the better of it and the best
// vertex).  `max_evals` is the build's reproducible evaluation budget (includes the final
// centroid evaluation); an iteration that would exceed it is abandoned with the simplex
// consistent.  The same machine is restated in oracle/gpar_oracle.py (NelderMead) and the
// two take identical steps given identical objective values (tests/test_host.py).
//
// Being a state machine, one GPU evaluation round can serve the pending points of many
// independent optimisations (one per GPAR output).
#pragma once
#include <algorithm>
#include <chrono>
#include <cmath>
#include <numeric>
#include <vector>

namespace gpar {

class NelderMead {
 public:
  NelderMead(std::vector<double> x0, int max_evals, int max_iterations, double g_tol,
             double time_limit)
      : n_((int)x0.size()), x0_(std::move(x0)), max_evals_(max_evals),
        max_iter_(max_iterations), g_tol_(g_tol), time_limit_(time_limit) {
    const double n = (double)n_;
    alpha_ = 1.0;
    beta_ = 1.0 + 2.0 / n;
    gamma_ = 0.75 - 1.0 / (2.0 * n);
    delta_ = 1.0 - 1.0 / n;
    m_ = n_ + 1;
    simplex_.assign(m_, x0_);
    for (int j = 0; j < n_; ++j) simplex_[j + 1][j] = (1.0 + 0.5) * simplex_[j + 1][j] + 0.025;
    fs_.assign(m_, 0.0);
    t0_ = std::chrono::steady_clock::now();
    init_i_ = 0;
    if (!can_eval()) {
      // no budget at all
      x_min_ = x0_;
      f_min_ = NAN;
      st_ = St::Done;
    } else {
      pending_ = simplex_[0];
      st_ = St::Init;
    }
  }

  bool done() const { return st_ == St::Done; }
  const std::vector<double>& ask() const { return pending_; }
  int evals() const { return evals_; }
  int iterations() const { return iters_; }
  const std::vector<double>& x_min() const { return x_min_; }
  double f_min() const { return f_min_; }

  void tell(double f) {
    ++evals_;
    switch (st_) {
      case St::Init:
        fs_[init_i_] = f;
        ++init_i_;
        if (init_i_ < m_) {
          if (!can_eval()) {
            m_ = init_i_;
            simplex_.resize(m_);
            fs_.resize(m_);
            finish();
            return;
          }
          pending_ = simplex_[init_i_];
          return;
        }
        order_ = argsort(fs_);
        converged_ = nm_obj() <= g_tol_;
        begin_iteration();
        return;
      case St::Reflect: on_reflect(f); return;
      case St::Expand: on_expand(f); return;
      case St::ContractOut:
        if (f < f_ref_) {
          accept(x_c_, f);
          order_ = argsort(fs_);
          end_iteration();
        } else {
          start_shrink();
        }
        return;
      case St::ContractIn:
        if (f < f_hi_) {
          accept(x_c_, f);
          order_ = argsort(fs_);
          end_iteration();
        } else {
          start_shrink();
        }
        return;
      case St::Shrink:
        simplex_[shrink_o_] = pending_;
        fs_[shrink_o_] = f;
        ++shrink_i_;
        next_shrink();
        return;
      case St::Centroid:
        if (f < f_min_) {
          x_min_ = pending_;
          f_min_ = f;
        }
        st_ = St::Done;
        return;
      case St::Done: return;
    }
  }

 private:
  enum class St { Init, Reflect, Expand, ContractOut, ContractIn, Shrink, Centroid, Done };

  bool can_eval() const { return max_evals_ <= 0 || evals_ < max_evals_ - 1; }
  bool out_of_time() const {
    if (time_limit_ <= 0) return false;
    const double el =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0_).count();
    return el > time_limit_;
  }

  std::vector<int> argsort(const std::vector<double>& v) const {
    std::vector<int> idx(v.size());
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return v[a] < v[b]; });
    return idx;
  }

  double nm_obj() const {
    double c = 0.0;
    for (double f : fs_) c += f;
    c /= (double)fs_.size();
    double s = 0.0;
    for (double f : fs_) s += (f - c) * (f - c);
    return std::sqrt(s / (double)n_);
  }

  std::vector<double> centroid_excluding(int hi) const {
    std::vector<double> c(n_, 0.0);
    for (int i = 0; i < m_; ++i)
      if (i != hi)
        for (int j = 0; j < n_; ++j) c[j] += simplex_[i][j];
    for (int j = 0; j < n_; ++j) c[j] /= (double)(m_ - 1);
    return c;
  }

  void begin_iteration() {
    if (converged_ || iters_ >= max_iter_ || m_ != n_ + 1 || out_of_time()) {
      finish();
      return;
    }
    ++iters_;
    hi_ = order_[m_ - 1];
    cen_ = centroid_excluding(hi_);
    x_lo_ = simplex_[order_[0]];
    f_lo_ = fs_[order_[0]];
    f_2hi_ = fs_[order_[n_ - 1]];
    f_hi_ = fs_[hi_];
    x_ref_.assign(n_, 0.0);
    for (int j = 0; j < n_; ++j) x_ref_[j] = cen_[j] + alpha_ * (cen_[j] - simplex_[hi_][j]);
    if (!can_eval()) {
      finish();
      return;
    }
    pending_ = x_ref_;
    st_ = St::Reflect;
  }

  void on_reflect(double f) {
    f_ref_ = f;
    if (f < f_lo_) {
      std::vector<double> xe(n_);
      for (int j = 0; j < n_; ++j) xe[j] = cen_[j] + beta_ * (x_ref_[j] - cen_[j]);
      if (!can_eval()) {
        finish();
        return;
      }
      pending_ = xe;
      st_ = St::Expand;
    } else if (f < f_2hi_) {
      accept(x_ref_, f);
      order_ = argsort(fs_);
      end_iteration();
    } else {
      x_c_.assign(n_, 0.0);
      const bool outside = f < f_hi_;
      for (int j = 0; j < n_; ++j)
        x_c_[j] = outside ? cen_[j] + gamma_ * (x_ref_[j] - cen_[j])
                          : cen_[j] - gamma_ * (x_ref_[j] - cen_[j]);
      if (!can_eval()) {
        finish();
        return;
      }
      pending_ = x_c_;
      st_ = outside ? St::ContractOut : St::ContractIn;
    }
  }

  void on_expand(double f) {
    if (f < f_ref_)
      accept(pending_, f);
    else
      accept(x_ref_, f_ref_);
    std::vector<int> o(m_);
    o[0] = hi_;
    for (int i = 1; i < m_; ++i) o[i] = order_[i - 1];
    order_ = o;
    end_iteration();
  }

  void accept(const std::vector<double>& x, double f) {
    simplex_[hi_] = x;
    fs_[hi_] = f;
  }

  void start_shrink() {
    shrink_i_ = 1;
    next_shrink();
  }

  void next_shrink() {
    if (shrink_i_ == m_) {
      order_ = argsort(fs_);
      end_iteration();
      return;
    }
    shrink_o_ = order_[shrink_i_];
    std::vector<double> xs(n_);
    for (int j = 0; j < n_; ++j) xs[j] = x_lo_[j] + delta_ * (simplex_[shrink_o_][j] - x_lo_[j]);
    if (!can_eval()) {
      finish();
      return;
    }
    pending_ = xs;
    st_ = St::Shrink;
  }

  void end_iteration() {
    converged_ = nm_obj() <= g_tol_;
    begin_iteration();
  }

  void finish() {
    order_ = argsort(fs_);
    const int hi = order_[m_ - 1];
    int imin = 0;
    for (int i = 1; i < m_; ++i)
      if (fs_[i] < fs_[imin]) imin = i;
    x_min_ = simplex_[imin];
    f_min_ = fs_[imin];
    if (m_ > 1) {
      pending_ = centroid_excluding(hi);
      st_ = St::Centroid;
    } else {
      st_ = St::Done;
    }
  }

  int n_, m_;
  std::vector<double> x0_;
  int max_evals_, max_iter_;
  double g_tol_, time_limit_;
  double alpha_, beta_, gamma_, delta_;
  std::vector<std::vector<double>> simplex_;
  std::vector<double> fs_;
  std::vector<int> order_;
  std::vector<double> pending_, cen_, x_lo_, x_ref_, x_c_, x_min_;
  double f_lo_ = 0, f_2hi_ = 0, f_hi_ = 0, f_ref_ = 0, f_min_ = NAN;
  int hi_ = 0, init_i_ = 0, shrink_i_ = 0, shrink_o_ = 0;
  int evals_ = 0, iters_ = 0;
  bool converged_ = false;
  St st_ = St::Init;
  std::chrono::steady_clock::time_point t0_;
};

}  // namespace gpar
