// Host check: aigar_math::mod_pos(a, b, 1/b) == Python's a % b (fmod, +0 for a
// zero remainder) for a >= 0, b > 0: random values, exact multiples and their
// neighbours, for the bucket size 20 and random grid-square sizes.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "aigar_math.h"

static double py_mod(double a, double b) {
  double m = std::fmod(a, b);
  if (m != 0.0) {
    if ((b < 0) != (m < 0)) m += b;
  } else {
    m = std::copysign(0.0, b);
  }
  return m;
}

int main(int argc, char **argv) {
  long n = argc > 1 ? atol(argv[1]) : 1000000;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> ua(0.0, 6000.0), ub(0.05, 400.0), uu(0.0, 1.0);
  long bad = 0, checked = 0;
  auto check = [&](double a, double b) {
    if (!(a >= 0) || !(b > 0)) return;
    double want = py_mod(a, b), got = aigar_math::mod_pos(a, b, 1.0 / b);
    checked++;
    if (std::memcmp(&want, &got, 8) != 0) {
      if (bad < 10) printf("mismatch a=%.17g b=%.17g want=%.17g got=%.17g\n", a, b, want, got);
      bad++;
    }
  };
  for (long i = 0; i < n; i++) {
    double b = (i & 1) ? 20.0 : ub(rng);
    double a = ua(rng);
    check(a, b);
    // exact and near multiples of b, the rounding-sensitive cases
    double k = std::floor(uu(rng) * 300);
    double m = k * b;
    check(m, b);
    check(std::nextafter(m, 0.0), b);
    check(std::nextafter(m, 1e9), b);
    check(std::nextafter(std::nextafter(m, 1e9), 1e9), b);
    // cl - fmod(cl, gs) then + gs steps (the axis-mask loop's values)
    double x = a - py_mod(a, b);
    check(x, b);
    check(x + b, b);
    check(std::fmax(0.0, a - 0.5 * b), b);
  }
  check(0.0, 20.0);
  printf("checked=%ld mismatches=%ld\n", checked, bad);
  return bad != 0;
}
