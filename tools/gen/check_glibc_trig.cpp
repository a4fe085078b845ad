// Host check of aigar_glibc_trig.h (the device's restatement of glibc 2.35's
// sin / cos / atan2) against
//   * the C library's sin / cos / atan2 -- what the reference's math module calls;
//   * with -DAIGAR_LINK_FMA_VARIANTS, the FMA variants themselves (__sin_fma,
//     __cos_fma, __ieee754_atan2_fma, linked from libm-2.35.a), whatever this
//     host's CPU dispatch picks.
// Inputs shaped like the path's: move / split / eject directions from coordinate
// differences (small, large, mixed magnitudes, exact zeros, signed zeros), the
// angles atan2 returns, deg2rad(0..359), every sin / cos range boundary of
// s_sin.c (2^-27, 2^-26, 0.126, 0.855469, 2.426265), sincostab seams (k/128 +- ulps),
// atan2 ratios at 1/16 and at the cij seams, |y| ~ |x|, huge / tiny / subnormal
// and infinite operands.  Prints "mismatches=<n>"; any mismatch fails.
// g++ -O2 -std=c++17 -ffp-contract=off -I aigar_amd/csrc tools/gen/check_glibc_trig.cpp -o /tmp/cgt
//   [-DAIGAR_LINK_FMA_VARIANTS /usr/lib/x86_64-linux-gnu/libm-2.35.a]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "aigar_glibc_trig.h"

using namespace aigar_math;

#ifdef AIGAR_LINK_FMA_VARIANTS
extern "C" double __sin_fma(double);
extern "C" double __cos_fma(double);
extern "C" double __ieee754_atan2_fma(double, double);
#endif

static bool same(double a, double b) { return memcmp(&a, &b, sizeof a) == 0 || (a != a && b != b); }

static long bad = 0, total = 0;

static void check_sc(double a) {
  const double s = sin_glibc(a), c = cos_glibc(a);
  double fs, fc;
  sincos_glibc(a, fs, fc);  // (the wavefront-shaped form the device runs)
  total++;
  if (!same(s, fs) || !same(c, fc)) {
    if (++bad < 12) printf("sincos_glibc(%a): %a %a vs sin/cos_glibc %a %a\n", a, fs, fc, s, c);
  }
  if (!same(s, sin(a)) || !same(c, cos(a))) {
    if (++bad < 12) printf("sin/cos(%a): %a %a vs libm %a %a\n", a, s, c, sin(a), cos(a));
  }
#ifdef AIGAR_LINK_FMA_VARIANTS
  if (!same(s, __sin_fma(a)) || !same(c, __cos_fma(a))) {
    if (++bad < 12) printf("sin/cos(%a): %a %a vs __sin_fma %a %a\n", a, s, c, __sin_fma(a), __cos_fma(a));
  }
#endif
}

static void check_at(double y, double x) {
  const double r = atan2_glibc(y, x);
  total++;
  if (!same(r, atan2_glibc_flat(y, x))) {
    if (++bad < 12) printf("atan2_glibc_flat(%a, %a): %a vs atan2_glibc %a\n", y, x, atan2_glibc_flat(y, x), r);
  }
  if (!same(r, atan2(y, x))) {
    if (++bad < 12) printf("atan2(%a, %a): %a vs libm %a\n", y, x, r, atan2(y, x));
  }
#ifdef AIGAR_LINK_FMA_VARIANTS
  if (!same(r, __ieee754_atan2_fma(y, x))) {
    if (++bad < 12) printf("atan2(%a, %a): %a vs __ieee754_atan2_fma %a\n", y, x, r, __ieee754_atan2_fma(y, x));
  }
#endif
  check_sc(r);  // (the path takes cos / sin of every angle atan2 returns)
}

int main(int argc, char **argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  const double specials[] = {0.0, -0.0, 1.0, -1.0, INFINITY, -INFINITY, NAN, 0x1p-1074, -0x1p-1074, 0x1p-1022,
                             0x1.fffffffffffffp+1023, -0x1.fffffffffffffp+1023, 1e-300, 1e300, 3.0, -7.5};
  for (double y : specials)
    for (double x : specials) check_at(y, x);
  // range boundaries of s_sin.c and the sincostab seams
  const double bounds[] = {0x1p-27, 0x1p-26, 0.126, 0.855469, 2.426265, 3.14159, 6.2831853, 105414350.0};
  for (double b : bounds)
    for (int k = -300; k <= 300; k++) {
      const double a = b + k * ldexp(b, -52);
      check_sc(a);
      check_sc(-a);
    }
  for (int k = 0; k < 110; k++)
    for (int e = -64; e <= 64; e++) check_sc(k / 128.0 + e * 0x1p-53);
  for (int d = 0; d < 360; d++) check_sc(d * (M_PI / 180.0));  // numpy.deg2rad(randint(0, 360)) (field.py:363)
  for (long it = 0; it < n; it++) {
    const int kind = (int)(it % 8);
    double x, y;
    if (kind == 0) {  // cell -> command point differences (field-sized)
      x = (u01(g) - 0.5) * 9600.0;
      y = (u01(g) - 0.5) * 9600.0;
    } else if (kind == 1) {  // tiny differences (command point next to the centre)
      x = (u01(g) - 0.5) * 1e-3;
      y = (u01(g) - 0.5) * 1e-3;
    } else if (kind == 2) {  // mixed magnitudes
      x = ldexp(u01(g) - 0.5, (int)(u01(g) * 60) - 30);
      y = ldexp(u01(g) - 0.5, (int)(u01(g) * 60) - 30);
    } else if (kind == 3) {  // one axis zero or an integer grid point
      x = std::floor((u01(g) - 0.5) * 200.0);
      y = (it & 8) ? 0.0 : std::floor((u01(g) - 0.5) * 200.0);
    } else if (kind == 4) {  // |y| / |x| near 1/16 and the cij seams (i + 16) / 256
      const double r = (16 + (int)(u01(g) * 241)) / 256.0 * (1.0 + (u01(g) - 0.5) * 1e-12);
      x = (u01(g) + 0.1) * 1000.0 * ((it & 16) ? -1 : 1);
      y = x * r * ((it & 32) ? -1 : 1);
      if (it & 64) std::swap(x, y);
    } else if (kind == 5) {  // |y| ~ |x|
      x = (u01(g) + 0.01) * 500.0 * ((it & 16) ? -1 : 1);
      y = x * (1.0 + (u01(g) - 0.5) * 1e-9) * ((it & 32) ? -1 : 1);
    } else if (kind == 6) {  // exponent differences near the 57 * 16^5 cut-offs
      x = ldexp(1.0 + u01(g), (int)(u01(g) * 140) - 70);
      y = ldexp(1.0 + u01(g), (int)(u01(g) * 140) - 70) * ((it & 16) ? -1 : 1);
      if (it & 32) x = -x;
    } else {  // huge / tiny operands (the 2^+-500 rescaling)
      x = ldexp(u01(g) - 0.5, (int)(u01(g) * 2000) - 1000);
      y = ldexp(u01(g) - 0.5, (int)(u01(g) * 2000) - 1000);
    }
    check_at(y, x);
    if ((it & 3) == 0) check_sc((u01(g) - 0.5) * 16.0);  // wider angles
  }
  printf("n=%ld checks=%ld mismatches=%ld\n", n, total, bad);
  return bad ? 1 : 0;
}
