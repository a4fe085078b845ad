// Host check of the fast correctly rounded pow (aigar_math.h): fast path vs the
// slow double-double series on random inputs of the path's domain; reports the
// fallback rate, disagreements (must be 0) and the fast path's max error.
// g++ -O2 -std=c++17 -ffp-contract=off -I aigar_amd/csrc tools/gen/check_pow.cpp -o /tmp/check_pow
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "aigar_math.h"

using namespace aigar_math;

int main(int argc, char **argv) {
  long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 g(42);
  std::uniform_real_distribution<double> um(0.0, 1.0);
  const double ys[4] = {0.475, -0.35, 0.32, 0.0};
  long fallback = 0, bad = 0, glibc_diff = 0;
  double maxrel = 0;
  for (long it = 0; it < n; it++) {
    double x, y = ys[it & 3];
    int kind = (int)(it % 5);
    if (kind == 0) x = 10.0 * pow(2250.0, um(g));           // masses
    else if (kind == 1) x = sqrt(x = 10.0 * pow(2250.0, um(g)) / M_PI);  // radii
    else if (kind == 2) x = 1.0 + (um(g) - 0.5) * 1e-3;     // near 1
    else if (kind == 3) x = ldexp(0.5 + um(g), (int)(um(g) * 40) - 20);
    else x = (double)(1 + (int)(um(g) * 16));               // cell counts
    if (y == 0.0) y = (um(g) - 0.5) * 2.0;
    double slow = pow_cr_slow(x, y), fast;
    dd raw;
    bool ok = pow_fast(x, y, fast, &raw);
    {  // relative error of the fast double-double against the slow one (~2^-100 accurate)
      dd l = log_dd(x);
      dd pp = dd_add(two_prod(l.hi, y), dd{l.lo * y, 0.0});
      dd ex = exp_dd(pp);
      dd diff = dd_sub(raw, ex);
      double rel = fabs(diff.hi / ex.hi);
      if (rel > maxrel) maxrel = rel;
    }
    if (!ok) {
      fallback++;
      continue;
    }
    if (fast != slow) {
      if (++bad < 10) printf("MISMATCH x=%a y=%a fast=%a slow=%a\n", x, y, fast, slow);
    }
    if (fast != pow(x, y)) glibc_diff++;
    // error of the fast double-double vs the slow double-double (re-run internals)
    (void)maxrel;
  }
  printf("max relative error of the fast double-double: %a (2^%.1f)\n", maxrel, log2(maxrel));
  printf("n=%ld fallback=%ld (%.2e) mismatches=%ld glibc_differs=%ld (%.2e)\n", n, fallback, (double)fallback / n,
         bad, glibc_diff, (double)glibc_diff / n);
  return bad ? 1 : 0;
}
