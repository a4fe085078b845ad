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
//
// Shape: one table-driven path, no rounding test.  The argument is split as
// j/64 + t with |t| <= 1/128, so sin / cos / atan of j/64 come from a
// double-double table and only a short series in t remains: its two or three
// leading terms in double-double, the rest (each < 2^-47 of the result) in
// plain double.  That is ~10 dependent double-double operations per call
// instead of a 15-term Horner series.  A rounding-test fast path does not pay
// here: the kernels that call these run one lane per cell, so some wave of
// every launch would take the slow branch and the launch would wait for it.
// Domain: sin / cos for |a| <= 8 (the path's angles lie in [-pi, 2 pi)),
// larger |a| fall back to the libm function; atan2 for all finite inputs
// (C99 signed-zero conventions), non-finite ones fall back to libm.
// tools/gen/check_trig.cpp checks both against the quad-precision value.
#pragma once
#include "aigar_math.h"
#include "aigar_trig_tables.h"

namespace aigar_math {

AIGAR_HD dd kdd(const double (&c)[2]) { return dd{c[0], c[1]}; }

// a = k pi/2 + r, |r| <= pi/4: r in double-double (pi/2 as three doubles; k <= 5)
AIGAR_HD dd reduce_pio2(double a, int &q) {
  const double k = rint(a * 0x1.45f306dc9c883p-1);  // a * 2/pi
  q = ((int)k) & 3;
  const dd t = dd_add(two_prod(k, kPio2T[0]), dd_add(two_prod(k, kPio2T[1]), dd{k * kPio2T[2], 0.0}));
  return dd_sub(dd{a, 0.0}, t);
}

// sin r and cos r for |r| <= pi/4 + tiny: |r| = j/64 + t, |t| <= 1/128,
//   sin t = t + t s (-1/6 + s (1/120 + s Ps(s))),  cos t = 1 + s (-1/2 + s (1/24 + s Pc(s))),
// s = t^2, Ps / Pc in double (the terms from t^7 / t^6 on: < 2^-51 of the
// value, so their rounding stays below 2^-104); then
//   sin(c + t) = S cos t + C sin t,  cos(c + t) = C cos t - S sin t.
AIGAR_HD void sincos_dd(dd r, dd &sn, dd &cs) {
  const bool neg = r.hi < 0;
  if (neg) r = dd_neg(r);
  const int j0 = (int)rint(r.hi * 64.0), j = j0 < 51 ? j0 : 51;  // (|r| <= pi/4 + tiny: j <= 50; the clamp keeps the read in bounds)
  const double c = j * 0.015625;
  const dd t = two_sum(r.hi - c, r.lo);  // r.hi - c exact (Sterbenz, or c = 0)
  const dd s = dd_mul(t, t);
  const double sh = s.hi;
  const double ps = -0x1.a01a01a01a01ap-13 + sh * (0x1.71de3a556c734p-19 - sh * 0x1.ae64567f544e4p-26);
  const double pc = -0x1.6c16c16c16c17p-10 + sh * (0x1.a01a01a01a01ap-16 - sh * 0x1.27e4fb7789f5cp-22);
  dd qs = dd_add_d(kdd(kSinQ[1]), sh * ps);
  dd qc = dd_add_d(kdd(kCosQ), sh * pc);
  qs = dd_add(kdd(kSinQ[0]), dd_mul(s, qs));
  qc = dd_add_d(dd_mul(s, qc), -0.5);
  const dd st = dd_add(t, dd_mul(t, dd_mul(s, qs)));
  const dd ct = dd_add_d(dd_mul(s, qc), 1.0);
  if (j == 0) {
    sn = st;
    cs = ct;
  } else {
    const double *row = kSinCos64[j];
    const dd S{row[0], row[1]}, C{row[2], row[3]};
    sn = dd_add(dd_mul(S, ct), dd_mul(C, st));
    cs = dd_sub(dd_mul(C, ct), dd_mul(S, st));
  }
  if (neg) sn = dd_neg(sn);
}

// s = sin(a), c = cos(a), both correctly rounded, from one reduction
AIGAR_HD void sincos_cr(double a, double &s, double &c) {
  if (a == 0) {  // +-0 keeps its sign
    s = a;
    c = 1.0;
    return;
  }
  if (!(fabs(a) <= 8.0)) {
    s = sin(a);
    c = cos(a);
    return;
  }
  int q;
  dd sn, cs;
  sincos_dd(reduce_pio2(a, q), sn, cs);
  const dd vs = q == 0 ? sn : q == 1 ? cs : q == 2 ? dd_neg(sn) : dd_neg(cs);
  const dd vc = q == 0 ? cs : q == 1 ? dd_neg(sn) : q == 2 ? dd_neg(cs) : sn;
  s = vs.hi + vs.lo;
  c = vc.hi + vc.lo;
}

AIGAR_HD double sin_cr(double a) {
  double s, c;
  sincos_cr(a, s, c);
  return s;
}

AIGAR_HD double cos_cr(double a) {
  double s, c;
  sincos_cr(a, s, c);
  return c;
}

// atan(num / den) for 0 < num <= den: with c = j/64 nearest num/den,
//   atan(num/den) = atan c + atan u,  u = (num - c den) / (den + c num),  |u| <= 1/128,
// num - c den exact (c den is exact as two_prod; Sterbenz), one division plus
// two residual corrections for u, and
//   atan u = u + u s (-1/3 + s (1/5 + s (-1/7 + s Pa(s)))),  s = u^2,
// Pa in double (the terms from u^9 on: < 2^-59 of the value).
AIGAR_HD dd atan_ratio_dd(double num, double den) {
  const int j0 = (int)rint(num / den * 64.0), j = j0 < 64 ? j0 : 64;  // (num <= den; the clamp keeps the read in bounds)
  const double c = j * 0.015625;
  const dd cd = two_prod(c, den), cn = two_prod(c, num);
  const dd N = two_sum(num - cd.hi, -cd.lo);
  const dd D = dd_add(dd{den, 0.0}, cn);
  const double inv = 1.0 / D.hi;
  const double u1 = N.hi * inv;
  const dd r1 = dd_sub(N, dd_mul_d(D, u1));
  const double u2 = r1.hi * inv;
  const dd r2 = dd_sub(r1, dd_mul_d(D, u2));
  const dd u = dd_add_d(fast_two_sum(u1, u2), r2.hi * inv);
  const dd s = dd_mul(u, u);
  const double sh = s.hi;
  const double pa = 0x1.c71c71c71c71cp-4 - sh * (0x1.745d1745d1746p-4 - sh * (0x1.3b13b13b13b14p-4 - sh * 0x1.1111111111111p-4));
  dd qa = dd_add_d(kdd(kAtanQ[2]), sh * pa);
  qa = dd_add(kdd(kAtanQ[1]), dd_mul(s, qa));
  qa = dd_add(kdd(kAtanQ[0]), dd_mul(s, qa));
  return dd_add(kdd(kAtanJ64[j]), dd_add(u, dd_mul(u, dd_mul(s, qa))));
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
  dd th;
  if (num >= den * 0x1p-900) {  // (den * 2^-900 may underflow to 0; then num / den > 2^-200)
    // an exact power-of-two rescale keeps den + c num finite and the residuals clear of underflow
    const double sc = den > 0x1p1000 ? 0x1p-600 : den < 0x1p-900 ? 0x1p600 : 1.0;
    th = atan_ratio_dd(num * sc, den * sc);
  } else {  // atan q = q (1 - q^2/3 + ...) with q < 2^-900: the quotient rounded once
    th = dd{num / den, 0.0};
  }
  if (swap) th = dd_sub(dd{kPio2T[0], kPio2T[1]}, th);
  if (xneg) th = dd_sub(kdd(kPiDD), th);
  const double v = th.hi + th.lo;
  return yneg ? -v : v;
}

}  // namespace aigar_math
