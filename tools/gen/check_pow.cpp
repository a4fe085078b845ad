// Host check of aigar_math::pow_glibc (the device's restatement of glibc 2.35's
// pow) against the C library's pow, which is what the reference's float power
// calls: the path's domain (masses^-0.35, radii^0.475, cell counts^0.32),
// values near 1, and random x over 2^+-40 with random |y| <= 2.  Any mismatch
// fails.  Host libm must be the glibc whose tables aigar_glibc_pow_tables.h holds.
// g++ -O2 -std=c++17 -ffp-contract=off -I aigar_amd/csrc tools/gen/check_pow.cpp -o /tmp/check_pow
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "aigar_math.h"

using namespace aigar_math;

int main(int argc, char **argv) {
  long n = argc > 1 ? atol(argv[1]) : 10000000;
  std::mt19937_64 g(42);
  std::uniform_real_distribution<double> um(0.0, 1.0);
  const double ys[4] = {0.475, -0.35, 0.32, 0.0};
  long bad = 0;
  for (long it = 0; it < n; it++) {
    double x, y = ys[it & 3];
    int kind = (int)(it % 6);
    if (kind == 0) x = 10.0 * pow(2250.0, um(g));                     // masses
    else if (kind == 1) x = sqrt(10.0 * pow(2250.0, um(g)) / M_PI);   // radii
    else if (kind == 2) x = 1.0 + (um(g) - 0.5) * 1e-3;               // near 1
    else if (kind == 3) x = ldexp(0.5 + um(g), (int)(um(g) * 80) - 40);
    else if (kind == 4) x = (double)(1 + (int)(um(g) * 16));          // cell counts
    else x = 1.0 + (double)(g() >> 40) * 0x1p-24;                     // dense near [1, 2)
    if (y == 0.0) y = (um(g) - 0.5) * 4.0;
    const double a = pow_glibc(x, y), b = pow(x, y);
    if (a != b && !(a != a && b != b)) {
      if (++bad < 10) printf("MISMATCH x=%a y=%a pow_glibc=%a libm=%a\n", x, y, a, b);
    }
  }
  printf("n=%ld mismatches=%ld\n", n, bad);
  return bad ? 1 : 0;
}
