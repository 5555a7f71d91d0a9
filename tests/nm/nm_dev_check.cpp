// Steps NelderMead (nelder_mead.hpp, the host machine) and NmDev (nm_dev.hpp, the record the
// device steps) side by side on the same objective values; exits non-zero at the first point,
// state or result that differs in any bit.  Built and run by tests/test_nm_dev.py (g++ on the
// CPU; the device build of nm_dev.hpp is the same source with FMA contraction off).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "nelder_mead.hpp"
#include "nm_dev.hpp"

using namespace gpar;

static bool same(double a, double b) { return std::memcmp(&a, &b, sizeof(double)) == 0; }

static uint64_t rng_state = 88172645463325252ull;
static double urand() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return (double)(rng_state >> 11) * (1.0 / 9007199254740992.0);
}

// objective families: a shifted quadratic, Rosenbrock, and a noisy one with occasional +inf
static double objective(int fam, const std::vector<double>& x) {
  if (fam == 0) {
    double s = 0.0;
    for (size_t j = 0; j < x.size(); ++j) s += (x[j] - 0.3 * j) * (x[j] - 0.3 * j) * (1.0 + j);
    return s;
  }
  if (fam == 1) {
    double s = 0.0;
    for (size_t j = 0; j + 1 < x.size(); ++j)
      s += 100.0 * (x[j + 1] - x[j] * x[j]) * (x[j + 1] - x[j] * x[j]) + (1 - x[j]) * (1 - x[j]);
    return s;
  }
  if (urand() < 0.05) return INFINITY;
  double s = 0.0;
  for (double v : x) s += std::fabs(v - 0.5);
  return s + 0.01 * urand();
}

int main() {
  int cases = 0, steps = 0;
  const int budgets[] = {0, 1, 2, 3, 4, 5, 7, 12, 50, 200};
  const double tols[] = {-1.0, 1e-8, 1e-3};
  const int iters[] = {1000, 3, 0};
  for (int fam = 0; fam < 3; ++fam)
    for (int me : budgets)
      for (double tol : tols)
        for (int mi : iters)
          for (int rep = 0; rep < 3; ++rep) {
            std::vector<double> x0(3);
            for (double& v : x0) v = 2.0 * urand() - 1.0;
            NelderMead h(x0, me, mi, tol, 0.0);
            NmDev<3> d;
            nm_init(d, x0.data(), me, mi, tol);
            ++cases;
            for (int k = 0; k < 20000; ++k) {
              const bool hd = h.done(), dd = d.st == NmDev<3>::Done;
              if (hd != dd) { std::printf("done differs: fam %d me %d step %d\n", fam, me, k); return 1; }
              if (hd) break;
              const std::vector<double>& p = h.ask();
              for (int j = 0; j < 3; ++j)
                if (!same(p[j], d.pending[j])) {
                  std::printf("pending differs: fam %d me %d tol %g step %d\n", fam, me, tol, k);
                  return 1;
                }
              const double f = objective(fam, p);
              h.tell(f);
              nm_tell(d, f);
              ++steps;
              if (h.evals() != d.evals || h.iterations() != d.iters) {
                std::printf("counters differ: fam %d me %d step %d\n", fam, me, k);
                return 1;
              }
            }
            if (!h.done()) { std::printf("not done after 20000 steps\n"); return 1; }
            for (int j = 0; j < 3; ++j)
              if (!same(h.x_min()[j], d.x_min[j])) { std::printf("x_min differs\n"); return 1; }
            if (!same(h.f_min(), d.f_min) && !(std::isnan(h.f_min()) && std::isnan(d.f_min))) {
              std::printf("f_min differs\n");
              return 1;
            }
          }
  std::printf("ok %d cases %d steps\n", cases, steps);
  return 0;
}
