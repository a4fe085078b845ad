// aigar_math.h -- pow(x, y) exactly as the reference's glibc computes it, and
// an exact non-negative fmod, for the stepper (host + device).
//
// Why: the reference's observation grid has a quirk (spatialHashTable.py:19 vs
// bot.py:389): cols = ceil(fov / (fov / 11)) is 12 instead of 11 for ~3% of
// fov sizes, and fov = r^0.475 * n^0.32 * 35 (player.py:163-167).  Whether the
// quirk fires depends on the LAST BIT of fov, i.e. of libm's pow, which
// CPython's float power calls.  glibc 2.35's pow is not correctly rounded
// (< 0.52 ulp), so the device restates glibc's algorithm itself: same tables
// (aigar_glibc_pow_tables.h, dumped from the host's libm by
// tools/gen/glibc_pow_tables.c), same operation sequence, and the same fused
// multiply-adds as the x86-64 FMA variant the reference's host dispatches to
// (glibc's __ieee754_pow_fma, whose contractions were read off its object code;
// sysdeps/ieee754/dbl-64/e_pow.c).  tests/test_pow_host.py checks the host
// build against libm's pow on 10^7 inputs; tests/test_gpu_parity.py the device.
#pragma once
#include <stdint.h>
#include <string.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define AIGAR_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define AIGAR_HD static inline
#endif
#include "aigar_glibc_pow_tables.h"

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

// int(x / b) for x >= 0, b > 0 (inv_b = 1 / b), exactly, without the division
// (an fp64 divide is ~10 VALU with a transcendental rcp in its chain; the
// observation's mask loops ran one per candidate and axis: 2.5 of k_observe's
// 19 us in round 6).  n = the integer nearest x * inv_b is within a few ulps of
// x / b, so int(x / b) is n or n - 1: fl(x / b) >= n iff x / b lies above the
// midpoint between n and its predecessor, i.e. iff D = x - n * b >= -t with
// t = b * (n - pred(n)) / 2 (exact: a power-of-two scaling of b).  fma gives
// fl(D); rounding is monotone and -t is a double, so fl(D) > -t implies D > -t
// and fl(D) < -t implies D < -t; fl(D) == -t (D on or next to the midpoint,
// where ties-to-even decides) takes the division itself.  x / b < 2^31.
// (tools/gen/check_trunc_div.cpp, tests/test_pow_host.py)
AIGAR_HD int trunc_div_pos(double x, double b, double inv_b) {
  const double n = rint(x * inv_b);
  if (n <= 0.0) return 0;
  int64_t bits;
  memcpy(&bits, &n, sizeof bits);
  bits -= 1;
  double below;
  memcpy(&below, &bits, sizeof below);
  const double t = (n - below) * 0.5 * b;
  const double d = fma(-n, b, x);
  if (d > -t) return (int)n;
  if (d < -t) return (int)n - 1;
  return (int)(x / b);
}

// double-double helpers (aigar_trig.h)
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


AIGAR_HD dd dd_add_d(dd a, double b) {
  dd s = two_sum(a.hi, b);
  s.lo += a.lo;
  return fast_two_sum(s.hi, s.lo);
}

// ------------------------------------------------------------ glibc pow
#ifdef __HIPCC__
static __constant__ uint64_t kGlibcPowLogDev[521] = AIGAR_GLIBC_POW_LOG_DATA;
static __constant__ uint64_t kGlibcExpDev[270] = AIGAR_GLIBC_EXP_DATA;
#endif
static const uint64_t kGlibcPowLogHost[521] = AIGAR_GLIBC_POW_LOG_DATA;
static const uint64_t kGlibcExpHost[270] = AIGAR_GLIBC_EXP_DATA;

AIGAR_HD double as_double(uint64_t u) {
  double d;
  __builtin_memcpy(&d, &u, 8);
  return d;
}
AIGAR_HD uint64_t as_u64(double d) {
  uint64_t u;
  __builtin_memcpy(&u, &d, 8);
  return u;
}
// __pow_log_data: [0] ln2hi [1] ln2lo [2..8] poly A[0..6] [9 + 4i] {invc, pad, logc, logctail}
AIGAR_HD double glog_data(int i) {
#ifdef __HIP_DEVICE_COMPILE__
  return as_double(kGlibcPowLogDev[i]);
#else
  return as_double(kGlibcPowLogHost[i]);
#endif
}
// __exp_data: [0] invln2N [1] shift [2] negln2hiN [3] negln2loN [4..7] C2..C5 ... [14 + j] tab
AIGAR_HD uint64_t gexp_data(int i) {
#ifdef __HIP_DEVICE_COMPILE__
  return kGlibcExpDev[i];
#else
  return kGlibcExpHost[i];
#endif
}

// log(x) as hi + tail for the bit pattern ix of a positive normal x
// (glibc e_pow.c log_inline, __FP_FAST_FMA branch).
AIGAR_HD double glibc_log_inline(uint64_t ix, double *tail) {
  const uint64_t OFF = 0x3fe6955500000000ull;
  const uint64_t tmp = ix - OFF;
  const int i = (int)((tmp >> 45) & 127);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double z = as_double(iz);
  const double kd = (double)k;
  const double invc = glog_data(9 + 4 * i), logc = glog_data(11 + 4 * i), logctail = glog_data(12 + 4 * i);
  const double ln2hi = glog_data(0), ln2lo = glog_data(1);
  const double A0 = glog_data(2), A1 = glog_data(3), A2 = glog_data(4), A3 = glog_data(5), A4 = glog_data(6),
               A5 = glog_data(7), A6 = glog_data(8);
  const double r = fma(z, invc, -1.0);  // exact: 1/c is j/128 or j/256
  const double t1 = fma(kd, ln2hi, logc);
  const double t2 = t1 + r;
  const double lo1 = fma(kd, ln2lo, logctail);
  const double lo2 = t1 - t2 + r;
  const double ar = A0 * r;
  const double ar2 = r * ar;
  const double ar3 = r * ar2;
  const double hi = t2 + ar2;
  const double lo3 = fma(ar, r, -ar2);
  const double lo4 = t2 - hi + ar2;
  // p = ar3 * (A1 + r A2 + ar2 (A3 + r A4 + ar2 (A5 + r A6))), folded into lo by one fma
  const double q = fma(ar2, fma(ar2, fma(r, A6, A5), fma(r, A4, A3)), fma(r, A2, A1));
  const double lo = fma(ar3, q, lo1 + lo2 + lo3 + lo4);
  const double y = hi + lo;
  *tail = hi - y + lo;
  return y;
}

// exp(x + xtail) for the pow result, sign_bias 0 (glibc e_pow.c exp_inline).
AIGAR_HD double glibc_exp_inline(double x, double xtail) {
  uint32_t abstop = (uint32_t)(as_u64(x) >> 52) & 0x7ff;
  if (abstop - 0x3c9u >= 0x3fu) {
    if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + x;  // |x| < 2^-54
    if (abstop >= 0x409u) return (as_u64(x) >> 63) ? 0.0 : __builtin_inf();  // __math_uflow / oflow
    abstop = 0;  // large |x| below the overflow bound: specialcase below
  }
  const double InvLn2N = as_double(gexp_data(0)), Shift = as_double(gexp_data(1));
  const double NegLn2hiN = as_double(gexp_data(2)), NegLn2loN = as_double(gexp_data(3));
  const double C2 = as_double(gexp_data(4)), C3 = as_double(gexp_data(5)), C4 = as_double(gexp_data(6)),
               C5 = as_double(gexp_data(7));
  double kd = fma(x, InvLn2N, Shift);  // z + Shift, contracted
  const uint64_t ki = as_u64(kd);
  kd -= Shift;
  double r = fma(kd, NegLn2loN, fma(kd, NegLn2hiN, x));
  r = xtail + r;
  const uint64_t idx = 2 * (ki % 128);
  const uint64_t top = ki << 45;
  const double tail = as_double(gexp_data(14 + (int)idx));
  uint64_t sbits = gexp_data(15 + (int)idx) + top;
  const double r2 = r * r;
  const double tmp = fma(fma(r, C5, C4), r2 * r2, fma(fma(r, C3, C2), r2, r + tail));
  if (abstop == 0) {  // glibc specialcase (results near overflow / underflow; not on the stepper's path)
    if ((ki & 0x80000000ull) == 0) {
      sbits -= 1009ull << 52;
      const double scale = as_double(sbits);
      return 0x1p1009 * fma(tmp, scale, scale);
    }
    sbits += 1022ull << 52;
    const double scale = as_double(sbits);
    return 0x1p-1022 * (scale + scale * tmp);  // (subnormal double rounding not restated)
  }
  const double scale = as_double(sbits);
  return fma(tmp, scale, scale);
}

// pow(x, y) bit-identical to glibc 2.35 for x >= 0 finite and 2^-65 <= |y| < 2^63
// (fovSize, move speed; other inputs are outside the stepper's domain).
AIGAR_HD double pow_glibc(double x, double y) {
  if (x == 1.0 || y == 0.0) return 1.0;
  if (x == 0.0) return y > 0 ? 0.0 : __builtin_inf();
  uint64_t ix = as_u64(x);
  if ((ix >> 52) == 0) ix = as_u64(x * 0x1p52) - (52ull << 52);  // subnormal x
  double lo;
  const double hi = glibc_log_inline(ix, &lo);
  const double ehi = y * hi;
  const double elo = fma(y, lo, fma(y, hi, -ehi));
  return glibc_exp_inline(ehi, elo);
}

}  // namespace aigar_math
