// aigar_sem.h -- per-entity semantics of the reference tick as __device__
// functions (gfx950).  Every formula keeps the reference's operation order so
// that fp64 results round identically; the file:line each follows is cited.
// Compiled with -ffp-contract=off (no FMA contraction).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aigar_math.h"
#include "aigar_glibc_trig.h"

#define AIGAR_D __device__ __forceinline__

namespace aigar {

// ---------------------------------------------------------- parameters.py
constexpr double kFPS = 30, kGameSpeed = 1;
constexpr double kSpeedModifier = kGameSpeed / kFPS;
constexpr int kBucket = 20;                                  // HASH_BUCKET_SIZE
constexpr double kStartMass = 10;                            // START_MASS
constexpr double kVirusBase = 100;                           // VIRUS_BASE_SIZE
constexpr double kVirusEatFactor = 0.5;                      // VIRUS_EAT_FACTOR
constexpr double kExplosionProp = 0.6;                       // VIRUS_EXPLOSION_CELL_MASS_PROPORTION
constexpr double kEjectMass = 18;                            // EJECTEDBLOB_BASE_MASS
constexpr double kMaxMass = 22500;                           // MAX_MASS_SINGLE_CELL
constexpr double kBaseMerge = 25, kMergeMassFactor = 0.0233; // BASE_MERGE_TIME, MERGE_TIME_MASS_FACTOR
constexpr double kMergeVirusFactor = 0.85;                   // MERGE_TIME_VIRUS_FACTOR
constexpr double kMoveSpeed = 90 * kSpeedModifier;           // CELL_MOVE_SPEED
constexpr double kDecay = 1 - (0.01 * kSpeedModifier);       // CELL_MASS_DECAY_RATE
constexpr double kPi = 3.141592653589793;                    // numpy.pi
constexpr int kMaxCells = 16;

enum : uint32_t { F_ALIVE = 1u, F_INHASH = 2u, F_EJECT = 4u, F_NEW = 8u };

// ------------------------------------------------- python number helpers
AIGAR_D double py_max(double a, double b) { return (b > a) ? b : a; }  // builtin max(a, b)
AIGAR_D double py_min(double a, double b) { return (b < a) ? b : a; }  // builtin min(a, b)
AIGAR_D double py_mod(double a, double b) {                            // float % float
  double m = fmod(a, b);
  if (m != 0.0) {
    if ((b < 0) != (m < 0)) m += b;
  } else {
    m = copysign(0.0, b);
  }
  return m;
}
AIGAR_D double radius_of(double m) { return (m > 0) ? sqrt(m / kPi) : 0.0; }  // cell.py:210-212
// A pellet's radius: spawned pellets weigh 1, 2 or 3 (field.py:20-26), whose
// radii fold to constants -- radius_of is correctly rounded (IEEE division and
// square root), and these are Python's math.sqrt(m / math.pi)
// (tests/test_pow_host.py::test_pellet_radius_constants); other masses
// (converted blobs) take the formula.  Saves a division and a square root per
// pellet candidate.
constexpr double kPelletR1 = 0x1.20dd750429b6dp-1, kPelletR2 = 0x1.9884533d43651p-1,
                 kPelletR3 = 0x1.f45437857749ap-1;
AIGAR_D double pellet_radius(double m) {
  if (m == 1.0) return kPelletR1;
  if (m == 2.0) return kPelletR2;
  if (m == 3.0) return kPelletR3;
  return radius_of(m);
}
AIGAR_D double grow_mass(double m, double food) { return py_min(kMaxMass, m + food); }  // cell.py:119-121

// overlap (cell.py:143-152): bigger = strictly larger mass, else the argument
AIGAR_D bool overlap(double ax, double ay, double am, double ar, double bx, double by, double bm, double br) {
  bool a_big = am > bm;
  double sx = a_big ? ax : bx, sy = a_big ? ay : by, R = a_big ? ar : br;
  double ox = a_big ? bx : ax, oy = a_big ? by : ay;
  double d2 = (sx - ox) * (sx - ox) + (sy - oy) * (sy - oy);  // bigger.squaredDistance(smaller)
  return d2 * 1.1 < R * R;
}
AIGAR_D bool can_eat(double m, double other) { return m > 1.25 * other; }  // cell.py:163-164
// Cell.isInFov.  The reference's FOV queries (getPelletsInFov & co.,
// field.py:434-456) are a hash query around the FOV box -- objects whose bucket
// footprint meets Q = footprint(fx, fy, fs / 2) -- filtered by isInFov, and
// isInFov IMPLIES that overlap, so the queries test isInFov alone: per axis,
// x - r <= xmax gives floor(max(0, x - r) / 20) <= floor(xmax / 20) = Q's last
// bucket, and x + r >= xmin gives Q's first bucket floor(max(0, xmin) / 20) <=
// floor((x + r) / 20) = the footprint's last (the same rounded x - r, x + r and
// fx -+ fs / 2 on both sides; the field-size clamps only pull both last buckets
// to (size - 1) / 20).  tests/test_fov_membership.py checks it against the
// reference's getIdsForArea on 2 M random and bucket-edge cases.
AIGAR_D bool in_fov(double x, double y, double r, double fx, double fy, double fs) {  // cell.py:169-177
  double h = fs / 2, xmin = fx - h, xmax = fx + h, ymin = fy - h, ymax = fy + h;
  return !(x + r < xmin || x - r > xmax || y + r < ymin || y - r > ymax);
}

// cell.py:105-116
AIGAR_D void update_momentum(int &svc, double &svx, double &svy) {
  if (svc == -1) return;
  if (svc > 0) {
    svc -= 1;
    double ratio = svc / 15.0;
    if (ratio < 0.1) {
      svx *= (1 - ratio);
      svy *= (1 - ratio);
    }
  } else {
    svx = 0;
    svy = 0;
    svc = -1;
  }
}
// cell.py:132-141 (note the precedence quirk of the bounce test)
AIGAR_D void update_pos(double &x, double &y, double vx, double vy, double &svx, double &svy, int svc, double mx,
                        double my) {
  double xs = vx + svx, ys = vy + svy;
  x = py_min(mx, py_max(0.0, x + xs));
  y = py_min(my, py_max(0.0, y + ys));
  if ((svc != 0 && x == mx) || x == 0) svx *= -1;
  if ((svc != 0 && y == my) || y == 0) svy *= -1;
}
// cell.py:47-57
// (c, s: cos / sin of the angle to the command point -- Cell.split's angle too, cell.py:76-78)
AIGAR_D void set_move_direction(double x, double y, double m, double r, double cpx, double cpy, double &vx,
                                double &vy, double &c, double &s) {
  double xd = cpx - x, yd = cpy - y;
  double hyp = xd * xd + yd * yd, r2 = r * r;
  double mod = hyp >= r2 ? 1.0 : hyp / r2;  // min(hyp, r2) / r2 (r2 / r2 is exactly 1: no division then)
  double ang = aigar_math::trig_atan2(yd, xd);  // glibc's atan2, bit for bit (aigar_glibc_trig.h)
  double sp = kMoveSpeed * aigar_math::pow_glibc(m, -0.35);  // glibc pow, bit for bit (aigar_math.h)
  aigar_math::trig_sincos(ang, s, c);
  vx = sp * mod * c;
  vy = sp * mod * s;
}
AIGAR_D void set_move_direction(double x, double y, double m, double r, double cpx, double cpy, double &vx,
                                double &vy) {
  double c, s;
  set_move_direction(x, y, m, r, cpx, cpy, vx, vy, c, s);
}
// cell.py:96-103 (orig_r = radius of the originating cell)
AIGAR_D void add_momentum(double x, double y, double cpx, double cpy, double w, double h, double orig_r,
                          double &svx, double &svy, int &svc) {
  double cx = py_max(0.0, py_min(w, cpx)), cy = py_max(0.0, py_min(h, cpy));
  double ang = aigar_math::trig_atan2(cy - y, cx - x);
  double sp = 2 + orig_r * 0.05;
  double c, s;
  aigar_math::trig_sincos(ang, s, c);
  svx = c * sp;
  svy = s * sp;
  svc = 15;
}
// cell.py:154-155
AIGAR_D double merge_time_for(double f, double m) { return f * (kBaseMerge + m * kMergeMassFactor) * kFPS / 2 / kGameSpeed; }

// numpy pairwise sum for n <= 16 (player.py:129,158; numpy loops_utils.h)
AIGAR_D double np_sum(const double *a, int n) {
  if (n < 8) {
    double r = 0.;
    for (int i = 0; i < n; i++) r += a[i];
    return r;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; j++) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; j++) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += a[i];
  return res;
}

// Python round(v, 3) (bot.py:450): round-half-even of the exact binary value
// to a multiple of 1/1000, returned as the double nearest to k/1000 (what
// float(repr) of the decimal gives); a zero result keeps the sign of v.
AIGAR_D double py_round3(double v) {
  // |1000 v| < 0.4: rounds to k = 0, i.e. a zero with v's sign -- the common
  // case of the wall channel, whose 1 - freeA / (gs * gs) is a few ulps for a
  // square inside the field (no floor / fmod / division then)
  if (fabs(v) < 0.0004) return copysign(0.0, v);
  double p = v * 1000.0;
  double e = fma(v, 1000.0, -p);  // p + e == 1000 * v exactly
  double k0 = floor(p), f, d;
  if (p == k0 && e < 0) {  // exact value just below the integer p
    f = k0 - 1;
    d = 1.0;
  } else {
    f = k0;
    d = p - k0;  // exact
  }
  double g = d - 0.5;  // exact where it matters; |e| < |g| whenever g != 0
  int s = (g != 0) ? (g > 0 ? 1 : -1) : (e > 0 ? 1 : (e < 0 ? -1 : 0));
  double k = (s > 0) ? f + 1 : (s < 0) ? f : ((fmod(f, 2.0) == 0.0) ? f : f + 1);
  double r = k / 1000.0;
  if (r == 0.0) r = copysign(0.0, v);
  return r;
}

// ------------------------------------------------ spatial hash footprint
// getIdsForArea (int variant, spatialHashTable.py:70-83) as a bucket rectangle
// [x0, x1] x [y0, y1] (inclusive); empty when x1 < x0 or y1 < y0.
struct Rect {
  int x0, x1, y0, y1;
};
// floor(c / 20) of the exact quotient, c >= 0 (< 2^31): one multiply and two
// exact corrections (20 q is an exact double) -- what c - py_mod(c, 20) / 20 is
AIGAR_D int bucket_floor(double c) {
  int q = (int)(c * 0.05);
  q += ((double)(q + 1) * kBucket <= c) ? 1 : 0;
  q -= ((double)q * kBucket > c) ? 1 : 0;
  return q;
}
// floor(c / 20) for any sign, = floor of the rounded quotient (see center_bucket_coord)
AIGAR_D int bucket_floor_s(double c) {
  int q = (int)floor(c * 0.05);
  q += ((double)(q + 1) * kBucket <= c) ? 1 : 0;
  q -= ((double)q * kBucket > c) ? 1 : 0;
  return q;
}
AIGAR_D Rect footprint(double px, double py, double rad, int size) {
  double cl = py_max(0.0, px - rad), ct = py_max(0.0, py - rad);
  // bl = cl - cl % 20 = 20 * floor(cl / 20) exactly (Python's float modulo), so
  // the first bucket is floor(cl / 20); range(bl, lx, 20)'s last value
  // bl + 20 * floor((lx - 1 - bl) / 20) lies in bucket floor((lx - 1) / 20)
  // (32-bit integers: coordinates are bounded by the field size)
  const int kx = bucket_floor(cl), ky = bucket_floor(ct);
  int lx = (int)py_min((double)size, px + rad + 1), ly = (int)py_min((double)size, py + rad + 1);
  Rect r;
  r.x0 = kx;
  r.y0 = ky;
  r.x1 = (lx > kx * kBucket) ? (lx - 1) / kBucket : kx - 1;
  r.y1 = (ly > ky * kBucket) ? (ly - 1) / kBucket : ky - 1;
  return r;
}
AIGAR_D bool rect_hit(const Rect &a, const Rect &b) {
  return a.x0 <= a.x1 && a.y0 <= a.y1 && b.x0 <= b.x1 && b.y0 <= b.y1 && a.x0 <= b.x1 && b.x0 <= a.x1 &&
         a.y0 <= b.y1 && b.y0 <= a.y1;
}
// storage bucket of a centre coordinate: int(v / 20) of the rounded quotient,
// which is the exact floor -- the round-up window below an integer k + 1
// (20 x half the spacing of doubles below k + 1) is narrower than the spacing
// of doubles near v = 20 (k + 1), so no v rounds up -- hence bucket_floor
AIGAR_D int center_bucket_coord(double v, int cols) {
  const int b = v < 0 ? 0 : bucket_floor(v);
  return b < cols ? b : cols - 1;
}

// ------------------------------------------------------- Philox4x64-10
AIGAR_D void philox(uint64_t c0, uint64_t c1, uint64_t c2, uint64_t c3, uint64_t k0, uint64_t k1, uint64_t out[4]) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    uint64_t hi0 = __umul64hi(0xD2E7470EE14C6C93ull, c0), lo0 = 0xD2E7470EE14C6C93ull * c0;
    uint64_t hi1 = __umul64hi(0xCA5A826395121157ull, c2), lo1 = 0xCA5A826395121157ull * c2;
    uint64_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B97F4A7C15ull;
    k1 += 0xBB67AE8584CAA73Bull;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}
AIGAR_D uint64_t mulhi(uint64_t a, uint64_t b) { return __umul64hi(a, b); }
AIGAR_D int64_t ph_randint(uint64_t u, double lo, double hi) {  // randint(lo, hi), int() truncation
  int64_t l = (int64_t)lo, h = (int64_t)hi;
  if (h <= l) return l;
  return l + (int64_t)mulhi(u, (uint64_t)(h - l));
}
AIGAR_D double u01(uint64_t u) { return (double)(u >> 11) * (1.0 / 9007199254740992.0); }
enum : uint64_t {
  ST_PELLET = 1, ST_VIRUS = 2, ST_PLAYER = 3, ST_ANGLE = 4, ST_INIT_PLAYER = 5, ST_POLICY = 6, ST_GREEDY = 7,
  ST_GREEDY_LH = 8, ST_REFRANDOM = 9
};

}  // namespace aigar
