// Host check of aigar_trig.h: sin_cr / cos_cr / atan2_cr against the quad
// precision (libquadmath, 113 bits) value rounded to double, on inputs shaped
// like the stepper's (move directions from coordinate differences, split
// angles in [-pi, pi], explosion angles deg2rad(0..359)).  Also reports how
// often glibc differs from that rounding.  Adversarial sets too: arguments at
// the j/64 table seams, next to multiples of pi/2, ratios at the seams, and
// huge / tiny / subnormal atan2 operands.  Prints "mismatches=<n>" for ours.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <quadmath.h>

#include "aigar_trig.h"

using namespace aigar_math;

static bool same(double a, double b) { return memcmp(&a, &b, sizeof a) == 0; }

int main(int argc, char **argv) {
  const long n = argc > 1 ? atol(argv[1]) : 200000;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> coord(-1000.0, 1000.0), small(-1e-3, 1e-3), ang(-3.2, 3.2), wide(-8.0, 8.0);
  long bad = 0, glibc_bad = 0, total = 0;
  auto check_sc = [&](double a) {
    const double qs = (double)sinq((__float128)a), qc = (double)cosq((__float128)a);
    const double s = sin_cr(a), c = cos_cr(a);
    if (!same(s, qs) || !same(c, qc)) {
      if (bad < 10) printf("sin/cos(%a): %a %a vs %a %a\n", a, s, c, qs, qc);
      bad++;
    }
    glibc_bad += !same(sin(a), qs) + !same(cos(a), qc);
    total += 2;
  };
  auto check_at = [&](double y, double x) {
    const double q = (double)atan2q((__float128)y, (__float128)x);
    const double v = atan2_cr(y, x);
    if (!same(v, q)) {
      if (bad < 10) printf("atan2(%a, %a): %a vs %a\n", y, x, v, q);
      bad++;
    }
    glibc_bad += !same(atan2(y, x), q);
    total++;
  };
  for (int k = 0; k < 360; k++) check_sc(k * (3.14159265358979323846 / 180.0));
  const double edge[] = {0.0, -0.0, 1.0, -1.0, 1e-300, -1e-300, 5e-324, 1000.0, -1000.0};
  for (double y : edge)
    for (double x : edge) check_at(y, x);
  std::uniform_real_distribution<double> unit(-1.0, 1.0);
  for (long i = 0; i < n / 8; i++) {
    const int j = (int)(i % 52), k = (int)(i % 6) - 1;
    const double e = unit(rng) * 0x1p-9;
    check_sc(j / 64.0 + 1 / 128.0 + e * 0x1p-20);  // the seam between table rows
    check_sc(k * 1.5707963267948966 + e);           // near k pi/2
    check_sc(k * 1.5707963267948966 + j / 64.0 + e);
    const double den = coord(rng);
    check_at((j / 64.0 + 1 / 128.0 + e * 0x1p-20) * den, den);  // ratio at a seam
    check_at(den, (j / 64.0 + e) * den);
    check_at(ldexp(unit(rng), -1060), ldexp(unit(rng), -1050));  // subnormal operands
    check_at(ldexp(unit(rng), 1020), ldexp(unit(rng), 1023));    // near overflow
    check_at(ldexp(unit(rng), -700), ldexp(unit(rng), 300));     // tiny ratio
    check_at(ldexp(unit(rng), 200), ldexp(unit(rng), -950));
  }
  for (long i = 0; i < n; i++) {
    check_at(coord(rng), coord(rng));
    check_at(small(rng), coord(rng));
    check_at(coord(rng), small(rng));
    const double a = ang(rng);
    check_sc(a);
    check_sc(wide(rng));
    check_sc(atan2_cr(coord(rng), coord(rng)));
  }
  printf("calls=%ld mismatches=%ld glibc_mismatches=%ld (%.4f%%)\n", total, bad, glibc_bad,
         100.0 * glibc_bad / total);
  return bad != 0;
}
