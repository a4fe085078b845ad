// aigar_math.h -- correctly rounded pow(x, y) for the stepper (host + device).
//
// Why: the reference's observation grid has a quirk (spatialHashTable.py:19 vs
// bot.py:389): cols = ceil(fov / (fov / 11)) is 12 instead of 11 for ~3% of
// fov sizes, and fov = r^0.475 * n^0.32 * 35 (player.py:163-167).  Whether the
// quirk fires depends on the LAST BIT of fov, i.e. of libm's pow.  The
// reference runs glibc pow (correctly rounded except ~0.1% of inputs); OCML's
// pow differs far more often.  This double-double pow (~96 correct bits before
// the final rounding) returns the correctly rounded result, so it agrees with
// glibc wherever glibc is correctly rounded.
// Domain used by the path: x > 0 finite, |y| < 1 (also fine for moderate y).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define AIGAR_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define AIGAR_HD static inline
#endif

namespace aigar_math {

struct dd {
  double hi, lo;
};
AIGAR_HD dd two_sum(double a, double b) {
  double s = a + b;
  double bb = s - a;
  double e = (a - (s - bb)) + (b - bb);
  return {s, e};
}
AIGAR_HD dd fast_two_sum(double a, double b) {  // |a| >= |b|
  double s = a + b;
  double e = b - (s - a);
  return {s, e};
}
AIGAR_HD dd two_prod(double a, double b) {
  double p = a * b;
  double e = fma(a, b, -p);
  return {p, e};
}
AIGAR_HD dd dd_add(dd a, dd b) {
  dd s = two_sum(a.hi, b.hi);
  dd t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = fast_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return fast_two_sum(s.hi, s.lo);
}
AIGAR_HD dd dd_neg(dd a) { return {-a.hi, -a.lo}; }
AIGAR_HD dd dd_sub(dd a, dd b) { return dd_add(a, dd_neg(b)); }
AIGAR_HD dd dd_mul(dd a, dd b) {
  dd p = two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return fast_two_sum(p.hi, p.lo);
}
AIGAR_HD dd dd_mul_d(dd a, double b) {
  dd p = two_prod(a.hi, b);
  p.lo += a.lo * b;
  return fast_two_sum(p.hi, p.lo);
}
AIGAR_HD dd dd_div(dd a, dd b) {
  double q1 = a.hi / b.hi;
  dd r = dd_sub(a, dd_mul_d(b, q1));
  double q2 = r.hi / b.hi;
  r = dd_sub(r, dd_mul_d(b, q2));
  double q3 = r.hi / b.hi;
  dd q = fast_two_sum(q1, q2);
  return dd_add(q, dd{q3, 0.0});
}


// ln 2 = LN2_HI + LN2_LO
#define AIGAR_LN2_HI 6.93147180559945286227e-01
#define AIGAR_LN2_LO 2.31904681384629955842e-17

// log(x) in double-double: x = 2^k m, m in [sqrt(1/2), sqrt(2)),
// log m = 2 atanh(s), s = (m-1)/(m+1), |s| <= 0.1716
AIGAR_HD dd log_dd(double x) {
  int k;
  double m = frexp(x, &k);
  if (m < 0.70710678118654752440) {
    m *= 2;
    k -= 1;
  }
  dd num = two_sum(m, -1.0);
  dd den = two_sum(m, 1.0);
  dd s = dd_div(num, den);
  dd s2 = dd_mul(s, s);
  // 1/(2j+1) as double-double (generated with 80-digit decimal arithmetic)
  constexpr double kOddInv[25][2] = {{0x1.0000000000000p+0, 0x0.0p+0}, {0x1.5555555555555p-2, 0x1.5555555555555p-56}, {0x1.999999999999ap-3, -0x1.999999999999ap-57}, {0x1.2492492492492p-3, 0x1.2492492492492p-57}, {0x1.c71c71c71c71cp-4, 0x1.c71c71c71c71cp-58}, {0x1.745d1745d1746p-4, -0x1.745d1745d1746p-59}, {0x1.3b13b13b13b14p-4, -0x1.3b13b13b13b14p-58}, {0x1.1111111111111p-4, 0x1.1111111111111p-60}, {0x1.e1e1e1e1e1e1ep-5, 0x1.e1e1e1e1e1e1ep-61}, {0x1.af286bca1af28p-5, 0x1.af286bca1af28p-59}, {0x1.8618618618618p-5, 0x1.8618618618618p-59}, {0x1.642c8590b2164p-5, 0x1.642c8590b2164p-60}, {0x1.47ae147ae147bp-5, -0x1.eb851eb851eb8p-61}, {0x1.2f684bda12f68p-5, 0x1.2f684bda12f68p-59}, {0x1.1a7b9611a7b96p-5, 0x1.1a7b9611a7b96p-61}, {0x1.0842108421084p-5, 0x1.0842108421084p-60}, {0x1.f07c1f07c1f08p-6, -0x1.f07c1f07c1f08p-61}, {0x1.d41d41d41d41dp-6, 0x1.0750750750750p-60}, {0x1.bacf914c1bad0p-6, -0x1.bacf914c1bad0p-60}, {0x1.a41a41a41a41ap-6, 0x1.0690690690690p-60}, {0x1.8f9c18f9c18fap-6, -0x1.f3831f3831f38p-61}, {0x1.7d05f417d05f4p-6, 0x1.7d05f417d05f4p-62}, {0x1.6c16c16c16c17p-6, -0x1.f49f49f49f49fp-61}, {0x1.5c9882b931057p-6, 0x1.310572620ae4cp-61}, {0x1.4e5e0a72f0539p-6, 0x1.e0a72f0539783p-60}};
  dd acc = dd{kOddInv[24][0], kOddInv[24][1]};
  for (int j = 23; j >= 0; j--) acc = dd_add(dd_mul(acc, s2), dd{kOddInv[j][0], kOddInv[j][1]});
  dd lm = dd_mul_d(dd_mul(s, acc), 2.0);
  dd kl = dd_add(two_prod((double)k, AIGAR_LN2_HI), dd{(double)k * AIGAR_LN2_LO, 0.0});
  return dd_add(kl, lm);
}

// exp(p) in double-double: p = k ln2 + r, exp(r) = (Taylor(r / 2^10))^(2^10)
AIGAR_HD dd exp_dd(dd p) {
  double kd = rint(p.hi / AIGAR_LN2_HI);
  dd kl = dd_add(two_prod(kd, AIGAR_LN2_HI), two_prod(kd, AIGAR_LN2_LO));
  dd r = dd_sub(p, kl);
  r.hi *= 0x1p-10;
  r.lo *= 0x1p-10;
  // 1/n as double-double
  constexpr double kInvN[15][2] = {{0.0, 0.0}, {0x1.0000000000000p+0, 0x0.0p+0}, {0x1.0000000000000p-1, 0x0.0p+0}, {0x1.5555555555555p-2, 0x1.5555555555555p-56}, {0x1.0000000000000p-2, 0x0.0p+0}, {0x1.999999999999ap-3, -0x1.999999999999ap-57}, {0x1.5555555555555p-3, 0x1.5555555555555p-57}, {0x1.2492492492492p-3, 0x1.2492492492492p-57}, {0x1.0000000000000p-3, 0x0.0p+0}, {0x1.c71c71c71c71cp-4, 0x1.c71c71c71c71cp-58}, {0x1.999999999999ap-4, -0x1.999999999999ap-58}, {0x1.745d1745d1746p-4, -0x1.745d1745d1746p-59}, {0x1.5555555555555p-4, 0x1.5555555555555p-58}, {0x1.3b13b13b13b14p-4, -0x1.3b13b13b13b14p-58}, {0x1.2492492492492p-4, 0x1.2492492492492p-58}};
  dd acc = dd{1.0, 0.0};
  for (int n = 14; n >= 1; n--) acc = dd_add(dd{1.0, 0.0}, dd_mul(dd_mul(acc, r), dd{kInvN[n][0], kInvN[n][1]}));
  for (int i = 0; i < 10; i++) acc = dd_mul(acc, acc);
  int ki = (int)kd;
  acc.hi = ldexp(acc.hi, ki);
  acc.lo = ldexp(acc.lo, ki);
  return acc;
}

// correctly rounded x^y (x > 0)
AIGAR_HD double pow_cr(double x, double y) {
  if (y == 0.0 || x == 1.0) return 1.0;
  if (x == 0.0) return y > 0 ? 0.0 : __builtin_inf();
  dd l = log_dd(x);
  dd p = dd_add(two_prod(l.hi, y), dd{l.lo * y, 0.0});
  dd e = exp_dd(p);
  return e.hi + e.lo;
}

}  // namespace aigar_math
