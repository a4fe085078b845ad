// aigar_glibc_trig.h -- sin, cos and atan2 exactly as the reference's glibc
// computes them (host + device).
//
// Why: every cell's move direction is atan2 -> cos / sin each tick
// (cell.py:47-57), splits and ejections aim the same way (cell.py:67-103) and
// virus explosions take cos / sin of integer-degree angles (field.py:363-365).
// CPython's math module calls the C library: on the reference's x86-64 host,
// glibc 2.35's FMA variants __sin_fma / __cos_fma (sysdeps/ieee754/dbl-64/
// s_sin.c) and __ieee754_atan2_fma (e_atan2.c, whose multi-precision slow
// paths glibc had removed by 2.35).  Those are NOT correctly rounded (~0.1 % of
// the path's inputs differ from the correct rounding in the last bit), so a
// correctly rounded device function (aigar_trig.h) left positions within ~1e-16
// of the reference, not equal to it.  This header restates glibc's algorithms:
// the same tables (aigar_glibc_trig_tables.h: __sincostab and the atan2 cij
// table, dumped from the host's static libm by tools/gen/glibc_trig_tables.py),
// the same constants (the object code's literal pool), the same operation order,
// and a fused multiply-add exactly where the FMA variants' object code has one
// (read off `objdump -d` of s_sin-fma.o and e_atan2-fma.o; e.g. reduce_sincos's
// t = x * hpinv + toint is one fma there).  The file compiles with
// -ffp-contract=off, so no other operation fuses.
// tools/gen/check_glibc_trig.cpp checks the host build against libm and against
// the FMA variants themselves (linked from libm-2.35.a) on 10^7 inputs shaped
// like the path's; tests/test_gpu_parity.py checks the device.
// Domain: sin / cos for |x| < 105414350 (s_sin.c's __branred range beyond is
// never reached by the path's angles, |x| < 2 pi; it falls back to the
// correctly rounded aigar_trig.h), atan2 for all inputs.
#pragma once
#include "aigar_math.h"
#include "aigar_glibc_trig_tables.h"
#include "aigar_trig.h"

namespace aigar_math {

#ifdef __HIPCC__
static __constant__ uint64_t kGlibcSinCosTabDev[440] = AIGAR_GLIBC_SINCOSTAB;
static __constant__ uint64_t kGlibcAtanCijDev[241 * 7] = AIGAR_GLIBC_ATAN2_CIJ;
#endif
static const uint64_t kGlibcSinCosTabHost[440] = AIGAR_GLIBC_SINCOSTAB;
static const uint64_t kGlibcAtanCijHost[241 * 7] = AIGAR_GLIBC_ATAN2_CIJ;

AIGAR_HD double gsct(int i) {
#ifdef __HIP_DEVICE_COMPILE__
  return as_double(kGlibcSinCosTabDev[i]);
#else
  return as_double(kGlibcSinCosTabHost[i]);
#endif
}
AIGAR_HD double gcij(int i, int j) {
#ifdef __HIP_DEVICE_COMPILE__
  return as_double(kGlibcAtanCijDev[i * 7 + j]);
#else
  return as_double(kGlibcAtanCijHost[i * 7 + j]);
#endif
}

namespace gsin {
// s_sin.c / usncs.h constants (the literal pool of s_sin-fma.o)
constexpr double big = 0x1.8p+45;
constexpr double sn3 = -0x1.5555555555515p-3, sn5 = 0x1.11110e829872fp-7;
constexpr double cs2 = 0x1p-1, cs4 = -0x1.5555555555535p-5, cs6 = 0x1.6c16bedd9e239p-10;
constexpr double s1 = -0x1.5555555555555p-3, s2 = 0x1.1111111110ecep-7, s3 = -0x1.a01a019db08b8p-13;
constexpr double s4 = 0x1.71de27b9a7ed9p-19, s5 = -0x1.addffc2fcdf59p-26;
constexpr double hp0 = 0x1.921fb54442d18p+0, hp1 = 0x1.1a62633145c07p-54;
constexpr double hpinv = 0x1.45f306dc9c883p-1, toint = 0x1.8p+52;
constexpr double mp1 = 0x1.921fb58p+0, mp2 = -0x1.dde973cp-27;
constexpr double pp3 = -0x1.cb3b398p-55, pp4 = -0x1.d747f23e32ed7p-83;
constexpr double t126 = 0x1.020c49ba5e354p-3;  // 0.126

AIGAR_HD uint32_t hi32(double x) { return (uint32_t)(as_u64(x) >> 32); }
AIGAR_HD uint32_t lo32(double x) { return (uint32_t)as_u64(x); }

// TAYLOR_SIN(xx, a, da): ((POLYNOMIAL(xx) * a - 0.5 * da) * xx + da) + a
AIGAR_HD double taylor_sin(double a, double da) {
  const double xx = a * a;
  const double p = fma(fma(fma(fma(s5, xx, s4), xx, s3), xx, s2), xx, s1);
  const double t = fma(xx, fma(p, a, -(0.5 * da)), da);
  return a + t;
}
// do_sin(x, dx) for |x| < 0.855469
AIGAR_HD double do_sin(double x, double dx) {
  if (fabs(x) < t126) return taylor_sin(x, dx);
  if (x <= 0) dx = -dx;
  const double u = big + fabs(x);
  const double xr = fabs(x) - (u - big);
  const double xx = xr * xr;
  const double s = xr + fma(xr * xx, fma(xx, sn5, sn3), dx);
  const double c = fma(xr, dx, xx * fma(fma(xx, cs6, cs4), xx, cs2));
  const int k = (int)(lo32(u) << 2);
  const double sn = gsct(k), ssn = gsct(k + 1), cs = gsct(k + 2), ccs = gsct(k + 3);
  const double cor = fma(s, cs, fma(-c, sn, fma(s, ccs, ssn)));
  return copysign(sn + cor, x);
}
// do_cos(x, dx) for |x| < 0.855469
AIGAR_HD double do_cos(double x, double dx) {
  if (x < 0) dx = -dx;
  const double u = big + fabs(x);
  const double xr = (fabs(x) - (u - big)) + dx;
  const double xx = xr * xr;
  const double s = fma(xr * xx, fma(xx, sn5, sn3), xr);
  const double c = xx * fma(fma(xx, cs6, cs4), xx, cs2);
  const int k = (int)(lo32(u) << 2);
  const double sn = gsct(k), ssn = gsct(k + 1), cs = gsct(k + 2), ccs = gsct(k + 3);
  const double cor = fma(-s, sn, fma(-c, cs, fma(-s, ssn, ccs)));
  return cs + cor;
}
// reduce_sincos: x = n * pi/2 + (a + da), |x| < 105414350
AIGAR_HD int reduce(double x, double &a, double &da) {
  const double t = fma(x, hpinv, toint);
  const double xn = t - toint;
  const double y = fma(-xn, mp2, fma(-xn, mp1, x));
  const double t2 = fma(-xn, pp3, y);
  const double db1 = fma(-pp3, xn, y - t2);
  const double b = fma(-xn, pp4, t2);
  const double db2 = fma(-xn, pp4, t2 - b);
  a = b;
  da = db1 + db2;
  return (int)(lo32(t) & 3);
}
AIGAR_HD double do_sincos(double a, double da, int n) {
  const double r = (n & 1) ? do_cos(a, da) : do_sin(a, da);
  return (n & 2) ? -r : r;
}
}  // namespace gsin

// __sin_fma
AIGAR_HD double sin_glibc(double x) {
  using namespace gsin;
  const uint32_t k = hi32(x) & 0x7fffffffu;
  if (k < 0x3e500000u) return x;                                    // |x| < 2^-26
  if (k < 0x3feb6000u) return do_sin(x, 0.0);                       // |x| < 0.855469
  if (k < 0x400368fdu) return copysign(do_cos(hp0 - fabs(x), hp1), x);  // |x| < 2.426265
  if (k < 0x419921fbu) {                                            // |x| < 105414350
    double a, da;
    const int n = reduce(x, a, da);
    return do_sincos(a, da, n);
  }
  if (k < 0x7ff00000u) return sin_cr(x);  // (__branred range: not on the path)
  return x - x;                            // inf, nan -> nan
}
// __cos_fma
AIGAR_HD double cos_glibc(double x) {
  using namespace gsin;
  const uint32_t k = hi32(x) & 0x7fffffffu;
  if (k < 0x3e400000u) return 1.0;                  // |x| < 2^-27
  if (k < 0x3feb6000u) return do_cos(x, 0.0);       // |x| < 0.855469
  if (k < 0x400368fdu) {                            // |x| < 2.426265
    const double y = hp0 - fabs(x);
    const double a = y + hp1;
    const double da = (y - a) + hp1;
    return do_sin(a, da);
  }
  if (k < 0x419921fbu) {  // |x| < 105414350
    double a, da;
    const int n = reduce(x, a, da);
    return do_sincos(a, da, n + 1);
  }
  if (k < 0x7ff00000u) return cos_cr(x);
  return x - x;
}

// sin and cos of one angle, shaped for a wavefront: the same operations as
// sin_glibc / cos_glibc, but every lane runs ONE do_sin and ONE do_cos whose
// inputs the range selects (|x| < 0.855469: (x, 0) both; < 2.426265: the
// hp0 - |x| forms; else reduce_sincos's (a, da) and the quadrant picks which
// core is which), the Taylor / table choice of do_sin a select, and both
// sincostab rows loaded in one round.  Branching per lane -- the stepper's
// angles span every range in one wave -- serialised the paths and their table
// loads (measured: 44.6 -> 31.8 M env-steps/s at C3).  Results are identical
// (tools/gen/check_glibc_trig.cpp checks both shapes against libm).
namespace gsin {
AIGAR_HD int row_of(double u) { const uint32_t k = lo32(u); return (int)(k < 109u ? k : 109u) << 2; }  // (109: the last row; NaN / inf lanes)
}  // namespace gsin
AIGAR_HD void sincos_glibc(double x, double &sv, double &cv) {
  using namespace gsin;
  const uint32_t k = hi32(x) & 0x7fffffffu;
  const double ax = fabs(x);
  const double y = hp0 - ax, am = y + hp1, dam = (y - am) + hp1;  // (2.426265 range)
  double ar, dar;
  const int n = reduce(x, ar, dar);  // (105414350 range)
  const bool r1 = k < 0x3feb6000u, r2 = !r1 && k < 0x400368fdu;
  const double XS = r1 ? x : (r2 ? am : ar), DXS0 = r1 ? 0.0 : (r2 ? dam : dar);
  const double XC = r1 ? x : (r2 ? y : ar), DXC0 = r1 ? 0.0 : (r2 ? hp1 : dar);
  // the two table rows (one load round)
  const double uS = big + fabs(XS), uC = big + fabs(XC);
  const int kS = row_of(uS), kC = row_of(uC);
  const double snS = gsct(kS), ssnS = gsct(kS + 1), csS = gsct(kS + 2), ccsS = gsct(kS + 3);
  const double snC = gsct(kC), ssnC = gsct(kC + 1), csC = gsct(kC + 2), ccsC = gsct(kC + 3);
  // do_sin (XS, DXS0): TAYLOR_SIN below 0.126, else the table form
  double S;
  {
    const double xx = XS * XS;
    const double p = fma(fma(fma(fma(s5, xx, s4), xx, s3), xx, s2), xx, s1);
    const double St = XS + fma(xx, fma(p, XS, -(0.5 * DXS0)), DXS0);
    const double dx = XS <= 0 ? -DXS0 : DXS0;
    const double xr = fabs(XS) - (uS - big), x2 = xr * xr;
    const double ss = xr + fma(xr * x2, fma(x2, sn5, sn3), dx);
    const double cc = fma(xr, dx, x2 * fma(fma(x2, cs6, cs4), x2, cs2));
    const double cor = fma(ss, csS, fma(-cc, snS, fma(ss, ccsS, ssnS)));
    S = fabs(XS) < t126 ? St : copysign(snS + cor, XS);
  }
  // do_cos (XC, DXC0)
  double C;
  {
    const double dx = XC < 0 ? -DXC0 : DXC0;
    const double xr = (fabs(XC) - (uC - big)) + dx, x2 = xr * xr;
    const double ss = fma(xr * x2, fma(x2, sn5, sn3), xr);
    const double cc = x2 * fma(fma(x2, cs6, cs4), x2, cs2);
    const double cor = fma(-ss, snC, fma(-cc, csC, fma(-ss, ssnC, ccsC)));
    C = csC + cor;
  }
  if (r1) {
    sv = S;
    cv = C;
  } else if (r2) {
    sv = copysign(C, x);
    cv = S;
  } else {  // do_sincos (a, da, n) and (a, da, n + 1)
    const double s0 = (n & 1) ? C : S, c0 = (n & 1) ? S : C;
    sv = (n & 2) ? -s0 : s0;
    cv = ((n + 1) & 2) ? -c0 : c0;
  }
  if (k < 0x3e500000u) sv = x;    // |x| < 2^-26
  if (k < 0x3e400000u) cv = 1.0;  // |x| < 2^-27
  if (k >= 0x419921fbu) {         // (__branred range: not on the path) and inf / nan
    sv = k < 0x7ff00000u ? sin_cr(x) : x - x;
    cv = k < 0x7ff00000u ? cos_cr(x) : x - x;
  }
}

namespace gatan {
constexpr double hpi = 0x1.921fb54442d18p+0, hpi1 = 0x1.1a62633145c07p-54;
constexpr double opi = 0x1.921fb54442d18p+1, opi1 = 0x1.1a62633145c07p-53;
constexpr double qpi = 0x1.921fb54442d18p-1, tqpi = 0x1.2d97c7f3321d2p+1;
constexpr double d3 = -0x1.5555555555555p-2, d5 = 0x1.99999999997fdp-3, d7 = -0x1.24924923f7603p-3;
constexpr double d9 = 0x1.c71c6e5129a3bp-4, d11 = -0x1.7458022b13c25p-4, d13 = 0x1.375f08b31cbcep-4;
constexpr double inv16 = 0x1p-4, two8 = 0x1p+8, two52 = 0x1p+52;
constexpr double twom500 = 0x1p-500, two500 = 0x1p+500;
constexpr int ep = 59768832, em = -59768832;  // +-57 * 16^5

// d3 + v (d5 + v (d7 + v (d9 + v (d11 + v d13))))
AIGAR_HD double poly_d(double v) { return fma(v, fma(v, fma(v, fma(v, fma(v, d13, d11), d9), d7), d5), d3); }
// cij[i][2] + v (cij[i][3] + v (cij[i][4] + v (cij[i][5] + v cij[i][6])))
AIGAR_HD double poly_c2(int i, double v) {
  return fma(v, fma(v, fma(v, fma(v, gcij(i, 6), gcij(i, 5)), gcij(i, 4)), gcij(i, 3)), gcij(i, 2));
}
// i = (TWO52 + TWO8 * u) - TWO52 - 16
AIGAR_HD int row(double u) { return (int)(fma(u, two8, two52) - two52) - 16; }
}  // namespace gatan

// __ieee754_atan2_fma
AIGAR_HD double atan2_glibc(double y, double x) {
  using namespace gatan;
  const uint64_t bx = as_u64(x), by = as_u64(y);
  const uint32_t ux = (uint32_t)(bx >> 32), dx = (uint32_t)bx, uy = (uint32_t)(by >> 32), dy = (uint32_t)by;
  // NaN operands
  if ((ux & 0x7ff00000u) == 0x7ff00000u && (((ux & 0x000fffffu) | dx) != 0)) return x + y;
  if ((uy & 0x7ff00000u) == 0x7ff00000u && (((uy & 0x000fffffu) | dy) != 0)) return y + y;
  // y = +-0
  if (uy == 0x00000000u && dy == 0) return (ux & 0x80000000u) == 0 ? 0.0 : opi;
  if (uy == 0x80000000u && dy == 0) return (ux & 0x80000000u) == 0 ? -0.0 : -opi;
  // x = +-0
  if (x == 0) return (uy & 0x80000000u) == 0 ? hpi : -hpi;
  // x = +-inf
  if (ux == 0x7ff00000u && dx == 0) {
    if (uy == 0x7ff00000u && dy == 0) return qpi;
    if (uy == 0xfff00000u && dy == 0) return -qpi;
    return (uy & 0x80000000u) == 0 ? 0.0 : -0.0;
  }
  if (ux == 0xfff00000u && dx == 0) {
    if (uy == 0x7ff00000u && dy == 0) return tqpi;
    if (uy == 0xfff00000u && dy == 0) return -tqpi;
    return (uy & 0x80000000u) == 0 ? opi : -opi;
  }
  // y = +-inf
  if (uy == 0x7ff00000u && dy == 0) return hpi;
  if (uy == 0xfff00000u && dy == 0) return -hpi;

  double ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
  const int de = (int)(uy & 0x7ff00000u) - (int)(ux & 0x7ff00000u);
  if (de >= ep) return y > 0 ? hpi : -hpi;
  if (de <= em) {
    if (x > 0) return copysign(ay / ax, y);  // signArctan2 (y, ay / ax)
    return y > 0 ? opi : -opi;
  }
  if (ax < twom500 || ay < twom500) {
    ax *= two500;
    ay *= two500;
  }
  if (ax > two500 || ay > two500) {
    ax *= twom500;
    ay *= twom500;
  }
  double u, du;
  if (ay < ax) {
    u = ay / ax;
    const double v = ax * u, vv = fma(ax, u, -v);  // EMULV
    du = ((ay - v) - vv) / ax;
  } else {
    u = ax / ay;
    const double v = ay * u, vv = fma(ay, u, -v);
    du = ((ax - v) - vv) / ay;
  }
  double z;
  if (x > 0) {
    if (ay < ax) {  // (i) atan(ay / ax)
      if (u < inv16) {
        const double v = u * u;
        const double zz = fma(u * v, poly_d(v), du);
        z = u + zz;
      } else {
        const int i = row(u);
        const double t3 = u - gcij(i, 0);
        const double v = t3 + du;  // EADD (t3, du, v, dv)
        const double dv = fabs(t3) > fabs(du) ? (t3 - v) + du : (du - v) + t3;
        const double t1 = gcij(i, 1), t2 = gcij(i, 2);
        const double p = fma(v, fma(v, fma(v, gcij(i, 6), gcij(i, 5)), gcij(i, 4)), gcij(i, 3));
        const double zz = fma(v, t2, fma(dv, t2, (v * v) * p));
        z = zz + t1;
      }
    } else {  // (ii) pi/2 - atan(ax / ay)
      if (u < inv16) {
        const double v = u * u;
        const double zz = (u * v) * poly_d(v);
        const double t2 = hpi - u;  // ESUB (hpi, u, t2, cor)
        const double cor = fabs(hpi) > fabs(u) ? (hpi - t2) - u : hpi - (u + t2);
        const double t3 = ((cor + hpi1) - du) - zz;
        z = t3 + t2;
      } else {
        const int i = row(u);
        const double v = (u - gcij(i, 0)) + du;
        const double zz = fma(-v, poly_c2(i, v), hpi1);
        const double t1 = hpi - gcij(i, 1);
        z = t1 + zz;
      }
    }
  } else if (ax < ay) {  // (iii) pi/2 + atan(ax / ay)
    if (u < inv16) {
      const double v = u * u;
      const double zz = (v * u) * poly_d(v);
      const double t2 = u + hpi;  // EADD (hpi, u, t2, cor)
      const double cor = fabs(hpi) > fabs(u) ? (hpi - t2) + u : (u - t2) + hpi;
      const double t3 = ((cor + hpi1) + du) + zz;
      z = t3 + t2;
    } else {
      const int i = row(u);
      const double v = (u - gcij(i, 0)) + du;
      const double zz = fma(v, poly_c2(i, v), hpi1);
      const double t1 = hpi + gcij(i, 1);
      z = t1 + zz;
    }
  } else {  // (iv) pi - atan(ay / ax)
    if (u < inv16) {
      const double v = u * u;
      const double zz = (v * u) * poly_d(v);
      const double t2 = opi - u;  // ESUB (opi, u, t2, cor)
      const double cor = fabs(opi) > fabs(u) ? (opi - t2) - u : opi - (u + t2);
      const double t3 = ((cor + opi1) - du) - zz;
      z = t3 + t2;
    } else {
      const int i = row(u);
      const double v = (u - gcij(i, 0)) + du;
      const double zz = fma(-v, poly_c2(i, v), opi1);
      const double t1 = opi - gcij(i, 1);
      z = t1 + zz;
    }
  }
  return copysign(z, y);  // signArctan2
}

// atan2 shaped for a wavefront, as sincos_glibc: the four quadrant cases share
// their forms (ii)-(iv) are K + s u with K = pi/2 or pi and s = +-1, whose
// ESUB / EADD corrections take their first branch since |u| < 1/16 < K), the
// Taylor and table forms are both evaluated and selected, and the cij row is
// loaded in one round; the special operands replace the result at the end, in
// e_atan2.c's order.  Identical results to atan2_glibc.
AIGAR_HD double atan2_glibc_flat(double y, double x) {
  using namespace gatan;
  const uint64_t bx = as_u64(x), by = as_u64(y);
  const uint32_t ux = (uint32_t)(bx >> 32), dx = (uint32_t)bx, uy = (uint32_t)(by >> 32), dy = (uint32_t)by;
  const double ax0 = x < 0 ? -x : x, ay0 = y < 0 ? -y : y;
  const int de = (int)(uy & 0x7ff00000u) - (int)(ux & 0x7ff00000u);
  // the regular path
  const bool sml = ax0 < twom500 || ay0 < twom500;
  double ax = ax0 * (sml ? two500 : 1.0), ay = ay0 * (sml ? two500 : 1.0);
  const bool lrg = ax > two500 || ay > two500;
  ax *= lrg ? twom500 : 1.0;
  ay *= lrg ? twom500 : 1.0;
  const bool yx = ay < ax, xpos = x > 0, c1 = xpos && yx, c3 = !xpos && ax < ay;
  const double num = yx ? ay : ax, den = yx ? ax : ay;
  const double u = num / den;
  const double v0 = den * u, vv = fma(den, u, -v0);  // EMULV
  const double du = ((num - v0) - vv) / den;
  const bool c4 = !xpos && !c3;
  const double K = c4 ? opi : hpi, K1 = c4 ? opi1 : hpi1, sg = c3 ? 1.0 : -1.0;
  // the cij row (its load first)
  double ri = fma(u, two8, two52) - two52;
  ri = (ri >= 16.0 && ri <= 256.0) ? ri : 16.0;  // (u < 1/16, nan: a row that is not used)
  const int i = (int)ri - 16;
  const double cj0 = gcij(i, 0), cj1 = gcij(i, 1), cj2 = gcij(i, 2), cj3 = gcij(i, 3), cj4 = gcij(i, 4),
               cj5 = gcij(i, 5), cj6 = gcij(i, 6);
  // Taylor, u < 1/16
  const double v = u * u, pd = poly_d(v);
  const double zTi = u + fma(u * v, pd, du);
  const double zz = (u * v) * pd;
  const double t2 = K + sg * u;
  const double cor = (K - t2) + sg * u;
  const double zTr = (((cor + K1) + sg * du) + sg * zz) + t2;
  // table
  const double t3 = u - cj0, vi = t3 + du;
  const double dvi = fabs(t3) > fabs(du) ? (t3 - vi) + du : (du - vi) + t3;
  const double p4 = fma(vi, fma(vi, fma(vi, cj6, cj5), cj4), cj3);
  const double zBi = fma(vi, cj2, fma(dvi, cj2, (vi * vi) * p4)) + cj1;
  const double pc = fma(vi, fma(vi, fma(vi, fma(vi, cj6, cj5), cj4), cj3), cj2);
  const double zBr = (K + sg * cj1) + fma(sg * vi, pc, K1);
  const double z = u < inv16 ? (c1 ? zTi : zTr) : (c1 ? zBi : zBr);
  double res = copysign(z, y);
  // e_atan2.c's special operands, last-checked first
  if (de <= em) res = x > 0 ? copysign(ay0 / ax0, y) : (y > 0 ? opi : -opi);
  if (de >= ep) res = y > 0 ? hpi : -hpi;
  if (uy == 0xfff00000u && dy == 0) res = -hpi;
  if (uy == 0x7ff00000u && dy == 0) res = hpi;
  if (ux == 0xfff00000u && dx == 0)
    res = (uy == 0x7ff00000u && dy == 0) ? tqpi : (uy == 0xfff00000u && dy == 0) ? -tqpi : ((uy & 0x80000000u) == 0 ? opi : -opi);
  if (ux == 0x7ff00000u && dx == 0)
    res = (uy == 0x7ff00000u && dy == 0) ? qpi : (uy == 0xfff00000u && dy == 0) ? -qpi : ((uy & 0x80000000u) == 0 ? 0.0 : -0.0);
  if (x == 0) res = (uy & 0x80000000u) == 0 ? hpi : -hpi;
  if (uy == 0x80000000u && dy == 0) res = (ux & 0x80000000u) == 0 ? -0.0 : -opi;
  if (uy == 0x00000000u && dy == 0) res = (ux & 0x80000000u) == 0 ? 0.0 : opi;
  if ((uy & 0x7ff00000u) == 0x7ff00000u && (((uy & 0x000fffffu) | dy) != 0)) res = y + y;
  if ((ux & 0x7ff00000u) == 0x7ff00000u && (((ux & 0x000fffffu) | dx) != 0)) res = x + y;
  return res;
}

// the stepper's trig entry points: glibc's functions (AIGAR_CR_TRIG: the
// correctly rounded aigar_trig.h versions, AIGAR_LIBM_TRIG: OCML -- A/B builds only)
AIGAR_HD double trig_atan2(double y, double x) {
#if defined(AIGAR_LIBM_TRIG)
  return atan2(y, x);
#elif defined(AIGAR_CR_TRIG)
  return atan2_cr(y, x);
#else
  return atan2_glibc_flat(y, x);
#endif
}
AIGAR_HD void trig_sincos(double a, double &s, double &c) {
#if defined(AIGAR_LIBM_TRIG)
  s = sin(a);
  c = cos(a);
#elif defined(AIGAR_CR_TRIG)
  sincos_cr(a, s, c);
#else
  sincos_glibc(a, s, c);
#endif
}

}  // namespace aigar_math
