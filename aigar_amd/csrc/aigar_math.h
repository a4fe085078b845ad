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
#include "aigar_pow_tables.h"

namespace aigar_math {

// fmod(a, b) for a >= 0, b > 0, a / b < 2^50 (bucket and grid-square offsets),
// exactly, without the long fmod routine: q = trunc(a * inv_b) is within one
// of floor(a / b); when q is right, a - q*b is the exact remainder (always
// representable) and the single-rounding fma returns it unchanged; a q one too
// large (small too) shows as r < 0 (r >= b) and the fma is redone with q -/+ 1.
// Returns +0 for a zero remainder, as Python's float % does for b > 0.
AIGAR_HD double mod_pos(double a, double b, double inv_b) {
  double q = trunc(a * inv_b);
  double r = fma(-q, b, a);
  if (r < 0) {
    r = fma(-(q - 1), b, a);
  } else if (r >= b) {
    r = fma(-(q + 1), b, a);
  }
  return r == 0 ? 0.0 : r;
}

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

// ---------------------------------------------------------------- fast path
// Table-driven x^y with ~2^-70 relative error as a double-double, plus Ziv's
// rounding test: when the error interval rounds to one double, that double is
// the correctly rounded result; otherwise (about 1 call in 2^16) the slow
// series above decides.  log: x = 2^E m, m in [1,2), t = m r_i - 1 exact
// (r_i has 8 significant bits, |t| < 2^-7), log1p(t) = t - t^2/2 + t^3 P(t).
// exp: p = (128 kk + j) ln2/128 + r, |r| < 2^-8, 2^(j/128) from a table.
struct PowLogEnt {
  double r, lh, ll;
};
struct PowExpEnt {
  double h, l;
};
#ifdef __HIPCC__
static __constant__ PowLogEnt kPowLogDev[128] = AIGAR_POW_LOG_TABLE;
static __constant__ PowExpEnt kPowExpDev[128] = AIGAR_POW_EXP_TABLE;
#endif
static const PowLogEnt kPowLogHost[128] = AIGAR_POW_LOG_TABLE;
static const PowExpEnt kPowExpHost[128] = AIGAR_POW_EXP_TABLE;
AIGAR_HD PowLogEnt pow_log_ent(int i) {
#ifdef __HIP_DEVICE_COMPILE__
  return kPowLogDev[i];
#else
  return kPowLogHost[i];
#endif
}
AIGAR_HD PowExpEnt pow_exp_ent(int j) {
#ifdef __HIP_DEVICE_COMPILE__
  return kPowExpDev[j];
#else
  return kPowExpHost[j];
#endif
}
AIGAR_HD dd dd_add_d(dd a, double b) {
  dd s = two_sum(a.hi, b);
  s.lo += a.lo;
  return fast_two_sum(s.hi, s.lo);
}
// relative error bound of the fast double-double result (measured max 2^-75.7 over
// 3M samples of the path's domain, tools/gen/check_pow.cpp; 2^5.7 margin)
#define AIGAR_POW_FAST_ERR 0x1p-70
AIGAR_HD bool pow_fast(double x, double y, double &res, dd *raw = nullptr) {
  uint64_t bits;
  __builtin_memcpy(&bits, &x, 8);
  int E = (int)((bits >> 52) & 0x7ff);
  if (E == 0 || E == 0x7ff || (bits >> 63)) return false;  // zero/subnormal/inf/nan/negative
  E -= 1023;
  const int i = (int)((bits >> 45) & 127);
  const uint64_t mb = (bits & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
  double m;
  __builtin_memcpy(&m, &mb, 8);
  const PowLogEnt L = pow_log_ent(i);
  const double t = fma(m, L.r, -1.0);  // exact
  const dd t2 = two_prod(t, t);
  double P = -0x1.999999999999ap-4;  // -1/10
  P = fma(P, t, 0x1.c71c71c71c71cp-4);   // 1/9
  P = fma(P, t, -0x1.0000000000000p-3);  // -1/8
  P = fma(P, t, 0x1.2492492492492p-3);   // 1/7
  P = fma(P, t, -0x1.5555555555555p-3);  // -1/6
  P = fma(P, t, 0x1.999999999999ap-3);   // 1/5
  P = fma(P, t, -0x1.0000000000000p-2);  // -1/4
  P = fma(P, t, 0x1.5555555555555p-2);   // 1/3
  const double ln2[3] = AIGAR_POW_LN2;
  const double Ed = (double)E;
  // small terms first (all << 2^-20 in magnitude)
  const double small = Ed * ln2[1] + Ed * ln2[2] + L.ll - 0.5 * t2.lo + t * t2.hi * P;
  dd lg = two_sum(Ed * ln2[0], L.lh);  // E ln2_hi is exact
  lg = dd_add_d(lg, t);
  lg = dd_add_d(lg, -0.5 * t2.hi);
  lg = dd_add_d(lg, small);
  // p = y log x
  dd p = two_prod(y, lg.hi);
  p.lo += y * lg.lo;
  p = fast_two_sum(p.hi, p.lo);
  if (!(p.hi > -700.0 && p.hi < 700.0)) return false;
  const double l128[3] = AIGAR_POW_LN2_128;
  const double kd = rint(p.hi * AIGAR_POW_INV_LN2_128);
  const int k = (int)kd;
  dd r = two_sum(p.hi, -kd * l128[0]);  // kd * ln2/128_hi is exact
  double rl = r.lo + p.lo - kd * l128[1] - kd * l128[2];
  r = two_sum(r.hi, rl);
  const double rh = r.hi;
  rl = r.lo;
  const dd r2 = two_prod(rh, rh);
  double Q = 0x1.a01a01a01a01ap-16;  // 1/40320
  Q = fma(Q, rh, 0x1.a01a01a01a01ap-13);  // 1/5040
  Q = fma(Q, rh, 0x1.6c16c16c16c17p-10);  // 1/720
  Q = fma(Q, rh, 0x1.1111111111111p-7);   // 1/120
  Q = fma(Q, rh, 0x1.5555555555555p-5);   // 1/24
  Q = fma(Q, rh, 0x1.5555555555555p-3);   // 1/6
  const double tail = rl + 0.5 * r2.lo + rh * rl + rh * r2.hi * Q;
  dd e = fast_two_sum(1.0, rh);
  e = dd_add_d(e, 0.5 * r2.hi);
  e = dd_add_d(e, tail);
  const PowExpEnt T = pow_exp_ent(k & 127);
  e = dd_mul(e, dd{T.h, T.l});
  if (raw) *raw = dd{ldexp(e.hi, k >> 7), ldexp(e.lo, k >> 7)};  // (diagnostics: tools/gen/check_pow.cpp)
  const double err = fabs(e.hi) * AIGAR_POW_FAST_ERR;
  const double u1 = e.hi + (e.lo - err), u2 = e.hi + (e.lo + err);
  if (u1 != u2) return false;
  res = ldexp(u1, k >> 7);  // (arithmetic shift: k = 128 (k >> 7) + (k & 127))
  return true;
}

// correctly rounded x^y (x > 0)
AIGAR_HD double pow_cr_slow(double x, double y) {
  dd l = log_dd(x);
  dd p = dd_add(two_prod(l.hi, y), dd{l.lo * y, 0.0});
  dd e = exp_dd(p);
  return e.hi + e.lo;
}
AIGAR_HD double pow_cr(double x, double y) {
  if (y == 0.0 || x == 1.0) return 1.0;
  if (x == 0.0) return y > 0 ? 0.0 : __builtin_inf();
  double r;
  if (pow_fast(x, y, r)) return r;
  return pow_cr_slow(x, y);
}

}  // namespace aigar_math
