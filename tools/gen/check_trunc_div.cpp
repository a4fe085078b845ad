// Host check of aigar_math::trunc_div_pos against int(x / b), on the operands the
// observation's mask loops produce (bot.py:389-398's float-hash insertion: x runs
// from a multiple of the square size b by repeated addition, so x / b sits next
// to an integer every time), and on adversarial operands: k * b +- a few ulps,
// the midpoints between an integer and its predecessor, powers of two.
// Prints "checks=<n> fallbacks=<f> mismatches=<m>"; any mismatch fails.
// g++ -O2 -std=c++17 -ffp-contract=off -I aigar_amd/csrc tools/gen/check_trunc_div.cpp -o /tmp/ctd
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "aigar_math.h"

using namespace aigar_math;

static long checks = 0, bad = 0, fallbacks = 0;

static void check(double x, double b) {
  const double inv_b = 1.0 / b;
  const int want = (int)(x / b);
  const int got = trunc_div_pos(x, b, inv_b);
  // (a fallback: the residual landed on the midpoint)
  const double n = rint(x * inv_b);
  if (n > 0) {
    const double below = std::nextafter(n, 0.0);
    if (std::fma(-n, b, x) == -((n - below) * 0.5 * b)) fallbacks++;
  }
  checks++;
  if (want != got && ++bad < 12) printf("x=%a b=%a: int(x / b)=%d trunc_div_pos=%d\n", x, b, want, got);
}

int main(int argc, char **argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  std::mt19937_64 g(11);
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  for (long it = 0; it < n; it++) {
    // a FOV size as player.py:163-167 makes them, a grid of G squares
    const double fs = std::pow(0.5 + u01(g) * 60.0, 0.475) * std::pow(1 + (int)(u01(g) * 16), 0.32) * 35;
    const int G = (it & 7) == 0 ? 3 + (int)(u01(g) * 60) : 11;
    const double gs = fs / G, inv_gs = 1.0 / gs, lim = fs - 1;
    // a candidate's axis: position relative to the view's edge, radius
    const double r = (it & 1) ? std::sqrt((1 + (int)(u01(g) * 3)) / M_PI) : u01(g) * fs * 0.3;
    const double p = -r + u01(g) * (fs + 2 * r);
    const double cl = std::fmax(0.0, p - r);
    const double bl = cl - mod_pos(cl, gs, inv_gs);
    const double lx = std::fmin(lim, p + r);
    for (double x = bl; x <= lx; x += gs) check(x, gs);
    // adversarial: next to k * b
    const int k = (int)(u01(g) * 140);
    const double xk = k * gs;
    double x = xk;
    for (int s = 0; s < 4; s++) x = std::nextafter(x, 0.0);
    for (int s = 0; s < 9; s++, x = std::nextafter(x, 1e300))
      if (x >= 0) check(x, gs);
  }
  // midpoints: x / b == m - ulp/2 exactly is not representable in general; sweep
  // b = powers of two and small integers, where the quotients are exact
  for (int e = -8; e <= 8; e++) {
    const double b = std::ldexp(1.0, e);
    for (int k = 1; k < 4096; k++) {
      double x = k * b;
      for (int s = 0; s < 3; s++) x = std::nextafter(x, 0.0);
      for (int s = 0; s < 7; s++, x = std::nextafter(x, 1e300)) check(x, b);
    }
  }
  for (int bi = 1; bi < 200; bi++) {
    const double b = bi * 0.1 + 0.013;
    for (int k = 0; k < 200; k++) {
      double x = k * b;
      for (int s = 0; s < 3; s++) x = std::nextafter(x, 0.0);
      for (int s = 0; s < 7; s++, x = std::nextafter(x, 1e300))
        if (x >= 0) check(x, b);
    }
  }
  printf("checks=%ld fallbacks=%ld mismatches=%ld\n", checks, fallbacks, bad);
  return bad ? 1 : 0;
}
