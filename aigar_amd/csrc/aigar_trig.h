// aigar_trig.h -- correctly rounded sin, cos and atan2 (host + device).
//
// Why: every cell's move direction is atan2 -> cos / sin each tick
// (cell.py:47-57), splits and ejections aim the same way (cell.py:72-103) and
// virus explosions take sin / cos of integer-degree angles (field.py:363).
// The reference runs glibc, whose sin / cos / atan2 agree with the correctly
// rounded result on ~99.9 % of inputs; OCML's differ in the last bit on 27 %
// (atan2) and 4 % (sin, cos) of the stepper's inputs
// (tools/micro/trig_vs_glibc.hip), and in crowded worlds those ulps grow
// through the push-apart dynamics.  These evaluate in double-double (~100
// correct bits) and return the rounding to nearest of that value.
// Domain: sin / cos for |a| <= 8 (the path's angles lie in [-pi, 2 pi)),
// larger |a| fall back to the libm function; atan2 for all finite inputs
// (C99 signed-zero conventions), non-finite ones fall back to libm.
#pragma once
#include "aigar_math.h"
#include "aigar_trig_tables.h"

namespace aigar_math {

AIGAR_HD dd kdd(const double (&c)[2]) { return dd{c[0], c[1]}; }

// sin r and cos r for |r| <= pi/4 + tiny (r as double-double): Taylor series in
// s = -r^2, Horner over 15 terms (the first neglected one is < 2^-110 r)
AIGAR_HD void sincos_dd_small(dd r, dd &sn, dd &cs) {
  const dd s = dd_neg(dd_mul(r, r));
  dd as = kdd(kInvFact[29]), ac = kdd(kInvFact[28]);
  for (int n = 13; n >= 0; n--) {
    as = dd_add(dd_mul(as, s), kdd(kInvFact[2 * n + 1]));
    ac = dd_add(dd_mul(ac, s), kdd(kInvFact[2 * n]));
  }
  sn = dd_mul(as, r);
  cs = ac;
}

// a = k pi/2 + r, |r| <= pi/4: r in double-double (pi/2 as three doubles; k <= 5)
AIGAR_HD dd reduce_pio2(double a, int &q) {
  const double k = rint(a * 0x1.45f306dc9c883p-1);  // a * 2/pi
  q = ((int)k) & 3;
  const dd t = dd_add(two_prod(k, kPio2T[0]), dd_add(two_prod(k, kPio2T[1]), dd{k * kPio2T[2], 0.0}));
  return dd_sub(dd{a, 0.0}, t);
}

AIGAR_HD double sin_cr(double a) {
  if (a == 0) return a;  // +-0 keeps its sign
  if (!(fabs(a) <= 8.0)) return sin(a);
  int q;
  dd sn, cs;
  sincos_dd_small(reduce_pio2(a, q), sn, cs);
  const dd v = q == 0 ? sn : q == 1 ? cs : q == 2 ? dd_neg(sn) : dd_neg(cs);
  return v.hi + v.lo;
}

AIGAR_HD double cos_cr(double a) {
  if (a == 0) return 1.0;
  if (!(fabs(a) <= 8.0)) return cos(a);
  int q;
  dd sn, cs;
  sincos_dd_small(reduce_pio2(a, q), sn, cs);
  const dd v = q == 0 ? cs : q == 1 ? dd_neg(sn) : q == 2 ? dd_neg(cs) : sn;
  return v.hi + v.lo;
}

// s = sin_cr(a), c = cos_cr(a) from one reduction and one series pass
AIGAR_HD void sincos_cr(double a, double &s, double &c) {
  if (a == 0 || !(fabs(a) <= 8.0)) {
    s = sin_cr(a);
    c = cos_cr(a);
    return;
  }
  int q;
  dd sn, cs;
  sincos_dd_small(reduce_pio2(a, q), sn, cs);
  const dd vs = q == 0 ? sn : q == 1 ? cs : q == 2 ? dd_neg(sn) : dd_neg(cs);
  const dd vc = q == 0 ? cs : q == 1 ? dd_neg(sn) : q == 2 ? dd_neg(cs) : sn;
  s = vs.hi + vs.lo;
  c = vc.hi + vc.lo;
}

// atan t for 0 <= t <= 1 (double-double): atan t = atan(j/16) + atan u,
// u = (t - j/16) / (1 + t j/16), |u| <= 1/32; atan u by 12 terms of its series
AIGAR_HD dd atan_dd_unit(dd t) {
  const int j = (int)rint(t.hi * 16.0);
  const double c = j * 0.0625;
  const dd u = dd_div(dd_sub(t, dd{c, 0.0}), dd_add(dd{1.0, 0.0}, dd_mul_d(t, c)));
  const dd s = dd_neg(dd_mul(u, u));
  dd acc = kdd(kInvOdd[11]);
  for (int n = 10; n >= 0; n--) acc = dd_add(dd_mul(acc, s), kdd(kInvOdd[n]));
  return dd_add(kdd(kAtanJ16[j]), dd_mul(acc, u));
}

AIGAR_HD double atan2_cr(double y, double x) {
  if (!(fabs(x) <= 1.7e308) || !(fabs(y) <= 1.7e308)) return atan2(y, x);  // inf / nan: libm
  const bool xneg = __builtin_signbit(x), yneg = __builtin_signbit(y);
  if (y == 0) {  // atan2(+-0, x): +-0 for x > 0 or x = +0, +-pi for x < 0 or x = -0
    const double v = xneg ? kPiDD[0] : 0.0;
    return yneg ? -v : v;
  }
  if (x == 0) return yneg ? -kPio2T[0] : kPio2T[0];  // +-pi/2
  const double ax = fabs(x), ay = fabs(y);
  const bool swap = ay > ax;
  const double num = swap ? ax : ay, den = swap ? ay : ax;
  const double q = num / den;
  const dd t = fast_two_sum(q, fma(-q, den, num) / den);  // num / den in double-double
  dd th = atan_dd_unit(t);
  const dd pi = kdd(kPiDD), pio2 = dd{kPio2T[0], kPio2T[1]};
  if (swap) th = dd_sub(pio2, th);
  if (xneg) th = dd_sub(pi, th);
  const double v = th.hi + th.lo;
  return yneg ? -v : v;
}

// the stepper's trig entry points (AIGAR_LIBM_TRIG: OCML instead, A/B builds only)
AIGAR_HD double trig_atan2(double y, double x) {
#ifdef AIGAR_LIBM_TRIG
  return atan2(y, x);
#else
  return atan2_cr(y, x);
#endif
}
AIGAR_HD void trig_sincos(double a, double &s, double &c) {
#ifdef AIGAR_LIBM_TRIG
  s = sin(a);
  c = cos(a);
#else
  sincos_cr(a, s, c);
#endif
}
}  // namespace aigar_math
