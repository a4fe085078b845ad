// obs.hip -- Bot.getStateRepresentation() (bot.py:272-497) for every bot, one
// 64-lane wavefront per bot, plus the synthetic-population policy and the
// per-player summary (player.py:129-167).
//
// Per bot: the FOV query runs on the field's centre-bucket grids with the
// reference's exact bucket-footprint membership (spatialHashTable.py:70-83)
// and isInFov (cell.py:169-177).  The per-bot float hash of the reference
// (spatialHashTable.py:85-108, including the cols==12 quirk and the size-1
// limit) is reproduced as a pair of 16-bit masks per object: the x- and
// y-indices its accumulation loops visit; grid square t = r + c*G reads the
// bucket id t, i.e. (t % cols, t / cols).  Visible objects are compacted into
// LDS with ballot + prefix-sum; pellets are ranked by creation sequence so
// every pellet-mass sum runs in the reference's order.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "aigar_dev.h"
#include "aigar_sem.h"
#include "aigar_wave.h"

#ifndef AIGAR_OBS_PAIR
#define AIGAR_OBS_PAIR 1  // the fast path scans each list once for both of a lane's squares
#endif
namespace aigar {

#define GTID ((int)(blockIdx.x * blockDim.x + threadIdx.x))

#ifndef AIGAR_OBS_PCAP
#define AIGAR_OBS_PCAP 256
#endif
constexpr int OBS_PCAP = AIGAR_OBS_PCAP;  // visible pellets per bot kept in LDS
constexpr int OBS_CCAP = 64;   // visible player cells
constexpr int OBS_VCAP = 32;   // visible viruses

#ifdef AIGAR_OBS_TIMING  // diagnostics build: per-wave phase timestamps (tools/micro/obs_timing.py)
constexpr int OBS_TS = 8;
__device__ unsigned long long g_obs_ts[65536 * OBS_TS];
#define OBS_STAMP(k) \
  if (lane == 0) obs_ts_l[k] = wall_clock64()
#else
#define OBS_STAMP(k)
#endif

// x / y index masks of the reference's float-hash insertion loops
__device__ __forceinline__ uint32_t axis_mask(double p, double r, double gs, double inv_gs, double lim) {
#ifdef AIGAR_OBS_DIAG_NOMASK  // (cost diagnostics only, results invalid)
  return p > r ? 2u : 1u;
#endif
  double cl = py_max(0.0, p - r);
  double bl = cl - aigar_math::mod_pos(cl, gs, inv_gs);  // (cl >= 0, gs > 0)
  double lx = py_min(lim, p + r);
  uint32_t m = 0;
  for (double x = bl; x <= lx; x += gs) m |= 1u << min(31, aigar_math::trunc_div_pos(x, gs, inv_gs));
  return m;
}

// lane k's value, broadcast to the wave (v_readlane into scalar registers; k is wave-uniform)
__device__ __forceinline__ double readlane_d(double v, int k) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)b, k);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), k);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ int64_t readlane_i64(int64_t v, int k) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)v, k);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(v >> 32), k);
  return (int64_t)(((unsigned long long)hi << 32) | lo);
}

// getAdditionalFeatures (bot.py:302-323) in two halves.  extra_load, with the
// kernel's first load round: lane k loads input k (0 lastFovSize, 1 total mass,
// 2-5 the last action, 6-9 the one before) -- loaded at the end, lane 0's loads
// waited behind the wave's row stores (vmcnt counts stores too on gfx9) and added
// a dependent memory round to every wave's tail.  extra_store, at the end: each
// lane writes its own feature (lane 10 the current fov size, which it records as
// the next lastFovSize).
__device__ __forceinline__ double extra_load(const Dev &d, int gp, int lane) {
  const uint32_t ex = d.obs_ex;
  const double *src = nullptr;
  if (lane == 0 && (ex & AIGAR_EX_LAST_FOV)) src = d.o_lastfov + gp;
  else if (lane == 1 && (ex & AIGAR_EX_MASS)) src = d.p_mass + gp;
  else if (lane >= 2 && lane < 6 && (ex & AIGAR_EX_LAST_ACT)) src = d.o_act_cur + (size_t)gp * 4 + (lane - 2);
  else if (lane >= 6 && lane < 10 && (ex & AIGAR_EX_2LAST_ACT)) src = d.o_act_prev + (size_t)gp * 4 + (lane - 6);
  return src ? *src : 0.0;
}
template <typename OutT>
__device__ __forceinline__ void extra_store(const Dev &d, int gp, int lane, OutT *row, int off, double fs, double xin) {
  const uint32_t ex = d.obs_ex;
  const int lf = (ex & AIGAR_EX_LAST_FOV) ? 1 : 0, fv = (ex & AIGAR_EX_FOV) ? 1 : 0;
  const int ms = (ex & AIGAR_EX_MASS) ? 1 : 0, la = (ex & AIGAR_EX_LAST_ACT) ? 4 : 0;
  int o = -1;
  double v = xin;
  if (lane == 0 && lf) o = off;
  else if (lane == 1 && ms) o = off + lf + fv;
  else if (lane >= 2 && lane < 6 && la) o = off + lf + fv + ms + (lane - 2);
  else if (lane >= 6 && lane < 10 && (ex & AIGAR_EX_2LAST_ACT)) o = off + lf + fv + ms + la + (lane - 6);
  else if (lane == 10 && fv) {
    o = off + lf;
    v = fs;
    d.o_lastfov[gp] = fs;
  }
  if (o >= 0) row[o] = (OutT)v;
}

// Python round(v, 5) (getRelativeCellPos, bot.py:16-21): round-half-even of
// the exact binary value to a multiple of 1e-5, as the double nearest k/1e5
__device__ __forceinline__ double py_round5(double v) {
  double p = v * 100000.0;
  double e = fma(v, 100000.0, -p);  // p + e == 1e5 * v exactly
  double k0 = floor(p), f, dd;
  if (p == k0 && e < 0) {
    f = k0 - 1;
    dd = 1.0;
  } else {
    f = k0;
    dd = p - k0;
  }
  double g = dd - 0.5;
  int sgn = (g != 0) ? (g > 0 ? 1 : -1) : (e > 0 ? 1 : (e < 0 ? -1 : 0));
  double k = (sgn > 0) ? f + 1 : (sgn < 0) ? f : ((fmod(f, 2.0) == 0.0) ? f : f + 1);
  double r = k / 100000.0;
  if (r == 0.0) r = copysign(0.0, v);
  return r;
}

// make_greedy_bot_move (bot.py:579-633) in three parts, shared by k_policy_greedy
// and the observation that computes the next tick's Greedy moves on its own walk
// (k_observe<..., GREEDY>: aigar_run with the Greedy population).
// (1) the biggest own cell: max(playerCells, key=mass) keeps the first maximum;
// lane k holds cell k's (mass, x, y) (mass -1 past the list), all lanes get the winner
__device__ __forceinline__ void greedy_own_best(double &bm, double &bx, double &by) {
  const int lane = threadIdx.x & 63;
  int bl = lane;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double om = __shfl_xor(bm, off);
    int ol = __shfl_xor(bl, off);
    if (om > bm || (om == bm && ol < bl)) {
      bm = om;
      bl = ol;
    }
  }
  bx = __shfl(bx, bl);
  by = __shfl(by, bl);
}
// (2) per lane: the best mass / distance^2 candidate seen, ties to the first in list
// order (pellets, enemy cells, viruses, each by creation sequence); a candidate has
// passed the liveness, own-cell and isInFov tests
struct GreedyAcc {
  double best = -1;
  uint64_t bord = ~0ull;
  double tx = 0, ty = 0;
  __device__ __forceinline__ void consider(int kd, double x, double y, double m, int64_t seq, double bm, double bx,
                                           double by) {
    if (kd != 0 && !(bm > 1.25 * m)) return;  // the biggest own cell must be able to eat it
    const double sd = (x - bx) * (x - bx) + (y - by) * (y - by);
    const double k = m / (sd != 0 ? sd : 1);
    const uint64_t ord = ((uint64_t)kd << 56) | (uint64_t)seq;
    if (k > best || (k == best && ord < bord)) {
      best = k;
      bord = ord;
      tx = x;
      ty = y;
    }
  }
};
// (3) the wave's best, then set_command_point (bot.py:550-577) by lane 0
__device__ __forceinline__ void greedy_commit(const Dev &d, int gp, GreedyAcc acc, double fx, double fy, double fs,
                                              int greedy_split) {
  const int lane = threadIdx.x & 63, a = gp / d.B, p = gp - a * d.B;
  double best = acc.best, tx = acc.tx, ty = acc.ty;
  uint64_t bord = acc.bord;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double ok = __shfl_xor(best, off);
    uint64_t oo = __shfl_xor(bord, off);
    double ox = __shfl_xor(tx, off), oy = __shfl_xor(ty, off);
    if (ok > best || (ok == best && oo < bord)) {
      best = ok;
      bord = oo;
      tx = ox;
      ty = oy;
    }
  }
  if (lane != 0) return;
  const ArenaCtl &ctl = d.ctl[a];
  const int64_t ix = (int64_t)fx, iy = (int64_t)fy;
  const int64_t left = ix - (int64_t)(fs / 2), top = iy - (int64_t)(fs / 2);
  uint64_t u[4];
  philox((uint64_t)p, ST_GREEDY, (uint64_t)ctl.tick, 0, ctl.key0, ctl.key1, u);
  double a0, a1;
  if (bord != ~0ull) {  // getRelativeCellPos(bestCell, left, top, size)
    a0 = py_round5((tx - (double)left) / fs);
    a1 = py_round5((ty - (double)top) / fs);
  } else {
    a0 = u01(u[0]);
    a1 = u01(u[1]);
  }
  int split = 0, eject = 0;
  if (greedy_split) {  // ENABLE_GREEDY_SPLIT: randint(0, 10000) > splitLikelihood
    int lh = d.p_split_lh[gp];
    if (lh <= 0) {
      uint64_t v[4];
      philox((uint64_t)p, ST_GREEDY_LH, 0, 0, ctl.key0, ctl.key1, v);
      lh = (int)ph_randint(v[0], 9950, 10000);
    }
    split = ph_randint(u[2], 0, 10000) > lh;
    eject = ph_randint(u[3], 0, 10000) > 100000;  // ejectLikelihood (bot.py:94)
  }
  const int64_t isz = (int64_t)fs;  // set_command_point: left + action * int(size)
  d.p_cmdx[gp] = (double)left + a0 * (double)isz;
  d.p_cmdy[gp] = (double)top + a1 * (double)isz;
  d.p_split[gp] = split;
  d.p_eject[gp] = eject;
}

// One list of visible objects (structure of arrays).  Lives in LDS; when a
// bot sees more objects than the LDS list holds, the same scan is repeated
// into a slice of the global overflow pool (exact, only slower).
struct ObjList {
  int64_t *seq;
  double *m, *r;
  uint32_t *mask;
  uint8_t *own;
  int *perm;
};
struct Cand {
  bool keep;
  int64_t seq;
  double m, r;
  uint32_t mask;
  uint8_t own;
};

// wave-wide append (ballot + prefix count); count is wave-uniform and keeps the true total
__device__ __forceinline__ void list_append(const Cand &c, ObjList &L, int cap, int &count) {
#ifdef AIGAR_OBS_DIAG_NOAPPEND  // (cost diagnostics only, results invalid)
  count += c.keep ? 1 : 0;
  return;
#endif
  unsigned long long bal = __ballot(c.keep);
  int slot = count + __popcll(bal & ((1ull << __lane_id()) - 1));
  if (c.keep && slot < cap) {
    if (L.seq) L.seq[slot] = c.seq;
    if (L.m) L.m[slot] = c.m;
    if (L.r) L.r[slot] = c.r;
    L.mask[slot] = c.mask;
    if (L.own) L.own[slot] = c.own;
  }
  count += __popcll(bal);
}

// claim n overflow slots; the pool word carries the observe-call epoch, so the
// first claim of a call restarts it (no reset pass, no end-of-launch ticket)
__device__ __forceinline__ int obs_claim(const Dev &d, uint32_t epoch, int n) {
  unsigned long long old = *(volatile unsigned long long *)d.ob_used, assumed;
  do {
    assumed = old;
    unsigned long long used = ((uint32_t)(assumed >> 32) == epoch) ? (assumed & 0xFFFFFFFFull) : 0;
    unsigned long long nv = ((unsigned long long)epoch << 32) | (used + (unsigned long long)n);
    old = atomicCAS(d.ob_used, assumed, nv);
  } while (old != assumed);
  return ((uint32_t)(assumed >> 32) == epoch) ? (int)(assumed & 0xFFFFFFFFull) : 0;
}

// The FOV queries of the reference -- getPelletsInFov, getEnemyPlayerCellsInFov,
// getVirusesInFov (field.py:434-456): hash lookup around the FOV box, then
// Cell.isInFov -- as ONE wave-wide walk: every grid row the box touches (pellet,
// cell and virus grids) gets a lane that fetches its item range, the ranges
// are flattened with a prefix sum, and each step hands 64 candidates of any
// kind to f(valid, kind, g) (kind 0 pellet slot, 1 cell pool index, 2 virus
// slot; g is the global index), so the three queries share their memory
// latency instead of chaining it.  f is called by every lane (it may ballot).
// pre() runs once, after the row-range loads are issued and before they are
// used (the caller's own-cell appends overlap that latency).
// The hash query's centre-bucket span, cut to the centre buckets an object of
// radius <= R can occupy and still pass isInFov (cell.py:169-177): its centre
// lies within R of the FOV box (+1 unit against rounding at the box edge).
// Exact -- every candidate is still tested -- and it drops the ring of buckets
// the hash expansion adds whenever the FOV edge sits away from a bucket edge.
__device__ __forceinline__ Span clip_to_fov(Span s, double fx, double fy, double h, double R, int cols, int shift) {
  const double m = h + R + 1.0;
  const int x0 = max(0, bucket_floor_s(fx - m)) >> shift, x1 = min(cols - 1, bucket_floor_s(fx + m));
  const int y0 = max(0, bucket_floor_s(fy - m)) >> shift, y1 = min(cols - 1, bucket_floor_s(fy + m));
  s.bx0 = max(s.bx0, x0);
  s.bx1 = min(s.bx1, x1 < 0 ? -1 : x1 >> shift);
  s.by0 = max(s.by0, y0);
  s.by1 = min(s.by1, y1 < 0 ? -1 : y1 >> shift);
  return s;
}
__device__ __forceinline__ int span_rows(const Span &s) { return (s.bx1 >= s.bx0 && s.by1 >= s.by0) ? s.by1 - s.by0 + 1 : 0; }

template <class P, class F>
// rmax_c / rmax_v: the arena's largest cell / virus radius (ArenaCtl), read by
// the caller together with its first loads
__device__ __forceinline__ void wave_fov_walk_k(const Dev &d, int a, Rect Q, double fx, double fy, double fs,
                                                double rmax_c, double rmax_v, bool want_p, bool want_c, bool want_v,
                                                P pre, F f) {
  const int lane = threadIdx.x & 63;
  const bool qok = Q.x1 >= Q.x0 && Q.y1 >= Q.y0;
  const double rc = fmax(rmax_c, radius_of(kStartMass)), rv = fmax(rmax_v, radius_of(kVirusBase));
  const int Ec = (int)ceil((rc + 1.0) / kBucket) + 1;
  const int Ev = (int)ceil((rv + 1.0) / kBucket) + 1;
  const double h = fs / 2;
  // pellets weigh 1-3, or 14.4 when converted from a blob: radius < 2.2
  Span sp = clip_to_fov(grid_span(Q, 1, d.cols, 0), fx, fy, h, 2.2, d.cols, 0);
  sp.stride = d.cols + 1;  // (pellet rows keep one more entry: the row's end)
#ifdef AIGAR_OBS_CLIP_ALL
  const Span sc = clip_to_fov(grid_span(Q, Ec, d.cols, d.cshift_c), fx, fy, h, rc, d.cols, d.cshift_c);
  const Span sv = clip_to_fov(grid_span(Q, Ev, d.cols, d.cshift), fx, fy, h, rv, d.cols, d.cshift);
#else  // (the coarse cell / virus grids gain little from the cut; it cost registers)
  const Span sc = grid_span(Q, Ec, d.cols, d.cshift_c), sv = grid_span(Q, Ev, d.cols, d.cshift);
#endif
  const int np_rows = (qok && want_p) ? span_rows(sp) : 0;
  const int nc_rows = (qok && want_c) ? span_rows(sc) : 0;
  const int nv_rows = (qok && want_v) ? span_rows(sv) : 0;
  const int nrows = np_rows + nc_rows + nv_rows;
  const size_t H1 = (size_t)a * (d.H + 1);
  const int *pst = d.pstart + (size_t)a * d.PH1, *cst = d.cstart + H1, *vst = d.vstart + H1;
  const int *cit = d.citems + (size_t)a * kMaxCells * d.B, *vit = d.vitems + (size_t)a * d.Vcap;
  if (nrows <= 0) pre();
  for (int r0 = 0; r0 < nrows; r0 += 64) {
    const int R = r0 + lane, nr = min(64, nrows - r0);
    int lo = 0, hi = 0, kind = 0;
    if (R < nrows) {
      const int *st;
      int row, bx0, bx1, stride;
      if (R < np_rows) {
        st = pst; row = sp.by0 + R; bx0 = sp.bx0; bx1 = sp.bx1; stride = sp.stride;
      } else if (R < np_rows + nc_rows) {
        kind = 1; st = cst; row = sc.by0 + (R - np_rows); bx0 = sc.bx0; bx1 = sc.bx1; stride = sc.stride;
      } else {
        kind = 2; st = vst; row = sv.by0 + (R - np_rows - nc_rows); bx0 = sv.bx0; bx1 = sv.bx1; stride = sv.stride;
      }
      lo = st[row * stride + bx0];
      hi = st[row * stride + bx1 + 1];
    }
    if (r0 == 0) pre();
    const int len = hi - lo;
    int inc = len;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      int y = __shfl_up(inc, off);
      if (lane >= off) inc += y;
    }
    const int excl = inc - len, total = __shfl(inc, 63);
    for (int t0 = 0; t0 < total; t0 += 64) {
      const int t = t0 + lane;
      // the batch's items lie in rows kb .. ke-1 (excl is non-decreasing): kb holds
      // item t0, ke is the first row starting at or after t0 + 64; only those rows
      // are searched, not all nr
      const int kb = __popcll(__ballot(lane < nr && excl <= t0)) - 1;
      const int ke = __popcll(__ballot(lane < nr && excl < t0 + 64));
      int rw = kb;
      for (int k = kb + 1; k < ke; k++) rw = (__builtin_amdgcn_readlane(excl, k) <= t) ? k : rw;  // (k uniform: v_readlane)
      const int idx = __shfl(lo, rw) + (t - __shfl(excl, rw));
      const int kd = __shfl(kind, rw);
      const bool valid = t < total;
      size_t g = 0;
      if (valid) g = kd == 0 ? (size_t)a * d.PS + idx : (kd == 1 ? (size_t)cit[idx] : (size_t)a * d.Vcap + vit[idx]);
      f(valid, kd, g);
    }
  }
}

// (every kind's rows: pellets and viruses as asked, player cells always)
template <class P, class F>
__device__ __forceinline__ void wave_fov_walk(const Dev &d, int a, Rect Q, double fx, double fy, double fs,
                                              double rmax_c, double rmax_v, bool want_p, bool want_v, P pre, F f) {
  wave_fov_walk_k(d, a, Q, fx, fy, fs, rmax_c, rmax_v, want_p, true, want_v, pre, f);
}

#ifdef AIGAR_OBS_WPE
#define OBS_ATTR __attribute__((amdgpu_waves_per_eu(AIGAR_OBS_WPE, 8)))
#else
// 4 waves/SIMD: 4096 bots = 16 waves per CU, one residency round on 256 CUs.
// The streaming variant (!WT, many arenas) ran at 5 waves/SIMD for a while (96
// VGPRs, 36 B per lane spilled: 37.3 -> 39.4 % of HBM peak at 16 C3 arenas);
// with the order-free pellet sums it spilled 72 B and 4 waves measured better
// again (38.5 -> 40.0 %, profiles/r04_ab_notes.txt)
#define OBS_ATTR __attribute__((amdgpu_waves_per_eu(4, 8)))
#endif
// WT: the store policy of the row and the history (below), chosen per launch by
// the number of bots (launch_observe)
// GREEDY (aigar_run with the Greedy population): the walk also picks every bot's
// next Greedy move (make_greedy_bot_move, bot.py:579-633: it reads the world this
// observation reads -- nothing changes before the next tick's policy), so that
// tick needs no k_policy_greedy launch; greedy_split as for k_policy_greedy
template <typename OutT, bool WT, bool GREEDY>
__global__ void __launch_bounds__(64) OBS_ATTR k_observe(Dev d, OutT *out, uint32_t epoch, const uint8_t *mask,
                                                         int greedy_split) {
  FLOOR(9);
  // p_seq / p_perm are reused, once the pellets are ranked, for the masses and
  // masks in creation order (no indirection in the per-square sums)
  __shared__ union {
    int64_t seq;
    double m;
  } p_sx[OBS_PCAP];
  __shared__ double p_m[OBS_PCAP];
  __shared__ uint32_t p_mask[OBS_PCAP];
  __shared__ union {
    int perm;
    uint32_t mask;
  } p_px[OBS_PCAP];
  __shared__ double c_mass[OBS_CCAP];
  __shared__ uint32_t c_mask[OBS_CCAP];
  __shared__ uint8_t c_own[OBS_CCAP];
  __shared__ double v_rad[OBS_VCAP], v_mass[OBS_VCAP];
  __shared__ int64_t v_seqs[OBS_VCAP];
  __shared__ uint32_t v_mask[OBS_VCAP];

  const int gp = xcd_block(blockIdx.x, gridDim.x), lane = threadIdx.x;
  const int NP = d.NP, a = gp / d.B, G = d.G, GG = G * G, L = d.L;
  // a masked-out bot does not compute its state this tick: no row, no history update
  // (the reference's getStateRepresentation runs only for NN bots that are not skipping)
  if (mask && !mask[gp]) return;
  if (epoch == 0) epoch = *d.ob_epoch;  // graph replay (aigar_run): the tick's closing kernel set it
#ifdef AIGAR_OBS_TIMING
  __shared__ unsigned long long obs_ts_l[OBS_TS];
  if (lane == 0) obs_ts_l[5] = (unsigned long long)__smid();
#endif
  OBS_STAMP(0);
  OutT *row = out + (size_t)gp * L;
  // the output row is written once and read by the host / learner, never by
  // the next tick, and the history grids are read back one observation later.
  // WT (one arena, a launch of a few thousand bots beside a latency-bound
  // tick): both are stored write-through (sc1: the line leaves the XCD's L2 with
  // the store), so they neither evict the world state (the next tick's working
  // set) from the L2s nor leave dirty lines for the end-of-launch write-back;
  // A/B on MI355X (profiles/r03_ab_notes.txt): +6.5 % per C3 step against
  // non-temporal rows and plain history (tick 96 -> 92 us).  !WT (many arenas:
  // a streaming launch of hundreds of MB): non-temporal rows, plain history --
  // write-through stores lost a quarter of the bandwidth there (16 arenas:
  // 2.66 -> 1.85 TB/s).
#ifdef AIGAR_OBS_DIAG_NOSTORE  // (cost diagnostics only, results invalid: one store per lane at the end)
  double diag_sum = 0;
  auto hist_st = [&](double *p, unsigned t, double v) __attribute__((always_inline)) { diag_sum += v; };
  auto row_st = [&](int o, unsigned t, OutT v) __attribute__((always_inline)) { diag_sum += (double)v; };
#else
  // element t of a wave-uniform base (the base in SGPRs, the lane's byte offset a
  // 32-bit VGPR: the store's saddr form, no 64-bit address arithmetic per store)
  auto at = [](auto *base, unsigned t) __attribute__((always_inline)) {
    using E = std::remove_pointer_t<decltype(base)>;
    return reinterpret_cast<E *>(reinterpret_cast<char *>(base) + t * (unsigned)sizeof(E));
  };
  auto hist_st = [&](double *base, unsigned t, double v) __attribute__((always_inline)) {
    if constexpr (WT) __hip_atomic_store(at(base, t), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *at(base, t) = v;
  };
  auto row_st = [&](int o, unsigned t, OutT v) __attribute__((always_inline)) {
    OutT *const p = reinterpret_cast<OutT *>(reinterpret_cast<char *>(row) + (unsigned)o * (unsigned)sizeof(OutT) +
                                              t * (unsigned)sizeof(OutT));
    if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __builtin_nontemporal_store(v, p);
  };
#endif
  // one round of independent loads: liveness, the FOV cache written at the end
  // of the tick (store_player_fov) and the own cells' slots
  const bool alive = d.p_alive[gp];
  const double fx = d.p_fx[gp], fy = d.p_fy[gp], fs = d.p_fs[gp];
  const int ncell = d.p_ncells[gp];
  const int oslot = lane < kMaxCells ? (int)d.p_list[lane * NP + gp] : 0;
  const ArenaCtl &ctl = d.ctl[a];
  const double rmax_c = ctl.rmax_cell, rmax_v = ctl.rmax_virus;  // (the walk's grid expansions)
  const double xin = extra_load(d, gp, lane);
  if (!alive) {  // getStateRepresentation returns None for dead players
    for (int i = lane; i < L; i += 64) row_st(0, i, (OutT)__builtin_nan(""));
    return;
  }
  if (d.tiled) {  // C4: one tile observes the bot -- its history holder, else its view centre's tile (tile_plan_thread)
    const int hold = d.t_holder[gp];
    const int by = hold >= 0 ? hold : tile_of(d, fx, fy);
    if (lane == 0) d.t_obsby[gp] = by;  // (every tile records the same observer)
    if (by != d.tile_id) return;
  }
  // own cells (getPortionOfCellsInFov(player.getCells())), loaded up front
  double ox = 0, oy = 0, orad = 0, omass = 0;
  if (lane < ncell) {
    const size_t ci = (size_t)oslot * NP + gp;
    ox = d.c_x[ci];
    oy = d.c_y[ci];
    orad = d.c_r[ci];
    omass = d.c_m[ci];
  }
  // GREEDY: the biggest own cell (greedy_own_best) from the same loads
  double g_bm = lane < ncell ? omass : -1.0, g_bx = ox, g_by = oy;
  if constexpr (GREEDY) greedy_own_best(g_bm, g_bx, g_by);
  GreedyAcc gacc_best;
  bool gacc = GREEDY;  // (the first walk only: an overflow walk sees the same candidates again)
  const double left = fx - fs / 2, top = fy - fs / 2, gs = fs / G, inv_gs = 1.0 / gs;
  const int cols = (int)ceil(fs / gs);
  const double lim = fs - 1;
  const Rect Q = footprint(fx, fy, fs / 2, d.size);
  // C4 tiles: the observing tile must hold every pellet the view can see; one
  // that does not (a halo below the view's reach) is an error, and the pellet
  // channel is NaN
  const bool held = tile_holds_rect(d, rect_grow(Q, 1, d.cols));
  if (!held && lane == wave_leader()) atomicOr(&d.ctl[a].err, ERR_TILE_OBS);
  // owner of cell pool index g = slot * NP + player, without a 64-bit modulo
  const double inv_np = 1.0 / NP;
  auto pool_owner = [&](size_t g) {
    const int gi = (int)g;
    int o = gi - (int)((double)gi * inv_np) * NP;
    o += o < 0 ? NP : 0;
    return o >= NP ? o - NP : o;
  };
  // last-frame history grids: independent of the queries
  // (first two squares of each lane; larger grids read the rest in the loop)
  // (GG <= 128: the loop below then issues no load, so no wait on its own stores)
  double h_slf0 = 0, h_slf1 = 0, h_elf0 = 0, h_elf1 = 0;  // (scalars: no stack slot)
  double h_sslf0 = 0, h_sslf1 = 0, h_eslf0 = 0, h_eslf1 = 0;
  auto load_hist = [&]() __attribute__((always_inline)) {
    const uint32_t och = d.obs_ch;
    const bool pslf = och & (AIGAR_OBS_SELF_LF | AIGAR_OBS_SELF_SLF), pelf = och & (AIGAR_OBS_ENEMY_LF | AIGAR_OBS_ENEMY_SLF);
    const bool psslf = och & AIGAR_OBS_SELF_SLF, peslf = och & AIGAR_OBS_ENEMY_SLF;
    const size_t hb = (size_t)gp * GG + lane;
    const bool in0 = lane < GG, in1 = lane + 64 < GG;
    if (pslf && in0) h_slf0 = d.o_self_lf[hb];
    if (pelf && in0) h_elf0 = d.o_en_lf[hb];
    if (pslf && in1) h_slf1 = d.o_self_lf[hb + 64];
    if (pelf && in1) h_elf1 = d.o_en_lf[hb + 64];
    if (psslf && in0) h_sslf0 = d.o_self_slf[hb];
    if (peslf && in0) h_eslf0 = d.o_en_slf[hb];
    if (psslf && in1) h_sslf1 = d.o_self_slf[hb + 64];
    if (peslf && in1) h_eslf1 = d.o_en_slf[hb + 64];
  };
// (their loads issued after the walk: early, the eight doubles stayed live through
// the walk -- 127 VGPRs; late, 110 -- and the A/B favoured late, profiles/r04_ab_notes.txt)

  // ---- getPelletsInFov / getEnemyPlayerCellsInFov / getVirusesInFov
  // (field.py:434-456) as ONE walk: every grid row the FOV touches (pellet,
  // cell and virus grids) gets a lane that fetches its item range, the ranges
  // are flattened with a prefix sum, and each step inspects 64 candidates of any
  // kind with a single round of loads (per-lane base pointers), so the three
  // queries share their memory latency instead of chaining it.

  auto walk = [&](ObjList &PLx, int capP, ObjList &CLx, int capC, ObjList &VLx, int capV, int &np, int &nc,
                  int &nv) __attribute__((always_inline)) {
    np = nc = nv = 0;
    auto own_cells = [&]() {  // own cells first: getPortionOfCellsInFov(player.getCells())
      Cand c{false, 0, 0, 0, 0, 1};
      if (lane < ncell && in_fov(ox, oy, orad, fx, fy, fs)) {
        uint32_t ix = axis_mask(ox - left, orad, gs, inv_gs, lim), iy = axis_mask(oy - top, orad, gs, inv_gs, lim);
        if (ix && iy) c = Cand{true, 0, omass, orad, ix | (iy << 16), 1};
      }
      list_append(c, CLx, capC, nc);
    };
    wave_fov_walk(d, a, Q, fx, fy, fs, rmax_c, rmax_v, held && (d.obs_ch & AIGAR_OBS_PELLET), d.virus_enabled, own_cells,
                  [&](bool valid, int kd, size_t g) {
      // per-lane base and stride: a pellet is one 32-byte record (x, y, m, seq), the
      // other kinds structure-of-arrays -- one load instruction per field either way
      const PelRec *PR = d.pel;
      const double *X = kd == 0 ? &PR->x : (kd == 1 ? d.c_x : d.v_x);
      const double *Y = kd == 0 ? &PR->y : (kd == 1 ? d.c_y : d.v_y);
      const double *M = kd == 0 ? &PR->m : (kd == 1 ? d.c_m : d.v_m);
      const double *RR = kd == 1 ? d.c_r : d.v_r;
      const int64_t *S = kd == 0 ? &PR->seq : (kd == 1 ? d.c_seq : d.v_seq);
      const uint32_t *FL = kd == 1 ? d.c_flags : d.v_flags;
      const size_t gr = kd == 0 ? g * kPelStride : g;
      bool ok = false;
      double x = 0, y = 0, m = 0, r = 0;
      int64_t sq = 0;
      if (valid) {
        x = X[gr];
        y = Y[gr];
        m = M[gr];
        r = kd == 0 ? 0.0 : RR[g];
        sq = (kd == 1 && !GREEDY) ? 0 : S[gr];
        uint32_t fl = kd == 0 ? (F_ALIVE | F_INHASH) : FL[g];
        if (kd == 0) r = pellet_radius(m);
        // (the hash query's footprint test is implied by isInFov: aigar_sem.h in_fov)
        ok = (fl & (F_ALIVE | F_INHASH)) == (F_ALIVE | F_INHASH) && !(kd == 1 && pool_owner(g) == gp) &&
             in_fov(x, y, r, fx, fy, fs);
        if constexpr (GREEDY)  // (k_policy_greedy's filter exactly: liveness, not its own cell, isInFov)
          if (gacc && ok) gacc_best.consider(kd, x, y, m, sq, g_bm, g_bx, g_by);
      }
      uint32_t msk = 0;
      if (ok) {
        uint32_t ix = axis_mask(x - left, r, gs, inv_gs, lim), iy = axis_mask(y - top, r, gs, inv_gs, lim);
        ok = ix && iy;
        msk = ix | (iy << 16);
      }
      list_append(Cand{ok && kd == 0, sq, m, r, msk, 0}, PLx, capP, np);
      list_append(Cand{ok && kd == 1, sq, m, r, msk, 0}, CLx, capC, nc);
      list_append(Cand{ok && kd == 2, sq, m, r, msk, 0}, VLx, capV, nv);
    });
  };
  int np, nc, nv;
  OBS_STAMP(1);
#if defined(AIGAR_OBS_STOP) && AIGAR_OBS_STOP == 1  // per-phase cost variants (timing only, results invalid)
  if (fx + fy + fs + left + ox + h_slf0 + h_elf0 == -1.2345) row_st(0, 0, (OutT)0);
  return;
#endif
  {  // (lists known to be the LDS arrays here: ds_write appends)
    ObjList P0{&p_sx[0].seq, p_m, nullptr, p_mask, nullptr, nullptr};
    ObjList C0{nullptr, c_mass, nullptr, c_mask, c_own, nullptr};
    ObjList V0{v_seqs, v_mass, v_rad, v_mask, nullptr, nullptr};
    walk(P0, OBS_PCAP, C0, OBS_CCAP, V0, OBS_VCAP, np, nc, nv);
  }
  if constexpr (GREEDY) {
    greedy_commit(d, gp, gacc_best, fx, fy, fs, greedy_split);
    gacc = false;
  }
  OBS_STAMP(2);
#if defined(AIGAR_OBS_STOP) && AIGAR_OBS_STOP == 2
  if (np + nc + nv == -12345 || h_slf0 + h_elf0 == -1.2345) row_st(0, 0, (OutT)0);
  return;
#endif
  ObjList PL{&p_sx[0].seq, p_m, nullptr, p_mask, nullptr, &p_px[0].perm};
  ObjList CL{nullptr, c_mass, nullptr, c_mask, c_own, nullptr};
  ObjList VL{v_seqs, v_mass, v_rad, v_mask, nullptr, nullptr};
  if (np > OBS_PCAP || nc > OBS_CCAP || nv > OBS_VCAP) {
    // a list outgrew LDS: claim slices of the global pool for the overflowing
    // lists and walk again (exact, only slower)
    const int need = (np > OBS_PCAP ? np : 0) + (nc > OBS_CCAP ? nc : 0) + (nv > OBS_VCAP ? nv : 0);
    int b = 0;
    const int ld = wave_leader();
    if (lane == ld) b = obs_claim(d, epoch, need);
    b = __builtin_amdgcn_readlane(b, ld);
    if (b + need > d.OBcap) {
      if (lane == ld) atomicOr(&d.ctl[a].err, ERR_OBS_CAP);
      np = min(np, OBS_PCAP);
      nc = min(nc, OBS_CCAP);
      nv = min(nv, OBS_VCAP);
    } else {
      auto slice = [&](ObjList Lg, bool over, ObjList Ll, int n, int &cap) {
        if (!over) return Ll;
        if (Lg.seq) Lg.seq += b;
        if (Lg.m) Lg.m += b;
        if (Lg.r) Lg.r += b;
        Lg.mask += b;
        if (Lg.own) Lg.own += b;
        if (Lg.perm) Lg.perm += b;
        b += n;
        cap = n;
        return Lg;
      };
      int cp = OBS_PCAP, cc = OBS_CCAP, cv = OBS_VCAP;
      PL = slice(ObjList{d.ob_seq, d.ob_m, nullptr, d.ob_mask, nullptr, d.ob_perm}, np > OBS_PCAP, PL, np, cp);
      CL = slice(ObjList{nullptr, d.ob_m, nullptr, d.ob_mask, d.ob_own, nullptr}, nc > OBS_CCAP, CL, nc, cc);
      VL = slice(ObjList{d.ob_seq, d.ob_m, d.ob_r, d.ob_mask, nullptr, nullptr}, nv > OBS_VCAP, VL, nv, cv);
      wave_fence();
      walk(PL, cp, CL, cc, VL, cv, np, nc, nv);
    }
  }
  wave_fence();  // lists written by all lanes -> read by all lanes
  load_hist();
  const bool in_lds = PL.seq == &p_sx[0].seq;  // (else the list overflowed into the global pool)
  // Every visible pellet weighing a whole number of units (spawns weigh 1-3; a
  // blob conversion need not): the pellet channel's sums are then exact in any
  // order, so each pellet adds its mass into the squares it covers (LDS integer
  // atomics below) -- no ranking by creation sequence, no per-square scan over
  // the list.  Otherwise the reference's creation-order sums.
  // A list in the overflow pool takes the same order-free sums (np * 65536 stays
  // below 2^31): its creation-order scan reads the pool per square, and its
  // ranking is quadratic -- the crowded Greedy worlds' wide views spent most of
  // the launch there (tools/clustered.py).
  bool pint = false;
#ifndef AIGAR_OBS_ORDERED_ONLY  // (A/B builds: the creation-order scan for every bot)
  if (GG <= OBS_PCAP && G <= 16 && np <= 32767) {
    bool bad = false;
    if (in_lds) {
      for (int i = lane; i < np; i += 64) {
        const double m = p_m[i];
        bad |= !(m >= 1.0 && m <= 65536.0 && m == floor(m));
      }
    } else {
      for (int i = lane; i < np; i += 64) {
        const double m = PL.m[i];
        bad |= !(m >= 1.0 && m <= 65536.0 && m == floor(m));
      }
    }
    pint = __ballot(bad) == 0;
  }
#endif
  // rank pellets by creation sequence (the sum order of the reference)
  const double *sm = nullptr;
  const uint32_t *smk = nullptr;
  if (in_lds && !pint) {  // np <= OBS_PCAP = 4 x 64: keep (rank, m, mask) in registers, then store in order
    int rk4[OBS_PCAP / 64];
    double m4[OBS_PCAP / 64];
    uint32_t k4[OBS_PCAP / 64];
#pragma unroll
    for (int j = 0; j < OBS_PCAP / 64; j++) {
      const int i = lane + 64 * j;
      rk4[j] = -1;
      if (i < np) {
        int64_t sq = p_sx[i].seq;
        int rk = 0;
        for (int q = 0; q < np; q++) rk += (p_sx[q].seq < sq);
        rk4[j] = rk;
        m4[j] = p_m[i];
        k4[j] = p_mask[i];
      }
    }
    wave_fence();
#pragma unroll
    for (int j = 0; j < OBS_PCAP / 64; j++)
      if (rk4[j] >= 0) {
        p_sx[rk4[j]].m = m4[j];
        p_px[rk4[j]].mask = k4[j];
      }
    sm = &p_sx[0].m;
    smk = &p_px[0].mask;
  } else if (!in_lds && !pint) {
    for (int i = lane; i < np; i += 64) {
      int64_t sq = PL.seq[i];
      int rk = 0;
      for (int j = 0; j < np; j++) rk += (PL.seq[j] < sq);
      PL.perm[rk] = i;
    }
  }
  wave_fence();
  OBS_STAMP(3);
#if defined(AIGAR_OBS_STOP) && AIGAR_OBS_STOP == 3
  if (np + nc + nv == -12345 || h_slf0 + h_elf0 == -1.2345 || (sm && sm[0] == -1.0)) row_st(0, 0, (OutT)0);
  return;
#endif
#ifdef AIGAR_OBS_TIMING
  if (lane == 0) obs_ts_l[6] = (unsigned long long)np | ((unsigned long long)nc << 20) | ((unsigned long long)nv << 40);
#endif

  // ---- per grid square (bot.py:387-456); lane owns squares t = lane + 64*j
  const uint32_t ch = d.obs_ch;
  const double fieldSize = (double)d.size;
  int off = 0;
  int o_pel = -1, o_self = -1, o_wall = -1, o_enemy = -1, o_all = -1, o_vir = -1;
  int o_sslf = -1, o_slf = -1, o_eslf = -1, o_elf = -1;
  if (ch & AIGAR_OBS_PELLET) { o_pel = off; off += GG; }
  if (ch & AIGAR_OBS_SELF) { o_self = off; off += GG; }
  if (ch & AIGAR_OBS_WALL) { o_wall = off; off += GG; }
  if (ch & AIGAR_OBS_ENEMY) { o_enemy = off; off += GG; }
  if (ch & AIGAR_OBS_ALL) { o_all = off; off += GG; }
  if (ch & AIGAR_OBS_VIRUS) { o_vir = off; off += GG; }
  if (ch & AIGAR_OBS_SELF_SLF) { o_sslf = off; off += GG; }
  if (ch & AIGAR_OBS_SELF_LF) { o_slf = off; off += GG; }
  if (ch & AIGAR_OBS_ENEMY_SLF) { o_eslf = off; off += GG; }
  if (ch & AIGAR_OBS_ENEMY_LF) { o_elf = off; off += GG; }
  double *slf = d.o_self_lf + (size_t)gp * GG, *sslf = d.o_self_slf + (size_t)gp * GG;
  double *elf = d.o_en_lf + (size_t)gp * GG, *eslf = d.o_en_slf + (size_t)gp * GG;
  // square centres, accumulated as the reference does (mx += gs per column,
  // bot.py:389-398): lane j holds column / row j's, read back by shuffle
  double colx = left + gs / 2, rowy = top + gs / 2;
  if (G <= 64)
    for (int i = 0; i < min(lane, G - 1); i++) {
      colx += gs;
      rowy += gs;
    }
  // per column / row (lane j): the wall channel's clipped extents -- a square's
  // free area is (rb - lb) * (bb - tb) of its column's and its row's values,
  // the same doubles (bot.py:444-450) -- and whether the square lies inside
  // the field (bits of a ballot per axis): one multiply and a few integer ops
  // per square instead of eight clamps and four compares
  const double wcol = py_max(py_min(colx + gs / 2, fieldSize), 0.0) - py_min(py_max(colx - gs / 2, 0.0), fieldSize);
  const double hrow = py_max(py_min(rowy + gs / 2, fieldSize), 0.0) - py_min(py_max(rowy - gs / 2, 0.0), fieldSize);
  const unsigned long long in_col = __ballot(!(colx + gs / 2 < 0 || colx - gs / 2 > fieldSize));
  const unsigned long long in_row = __ballot(!(rowy + gs / 2 < 0 || rowy - gs / 2 > fieldSize));
  const double inv_G = 1.0 / G, inv_cols = 1.0 / cols;
  // t / n for 0 <= t, n < 2^20: double reciprocal, then one correction step
  auto idiv = [](int t, int n, double inv_n) {
    int q = (int)((double)t * inv_n);
    q -= (q * n > t) ? 1 : 0;
    q += ((q + 1) * n <= t) ? 1 : 0;
    return q;
  };
  // t / n for 0 <= t < 512, 1 <= n <= 128: (t * ceil(2^16 / n)) >> 16 is exact
  // (checked for every such pair) -- a 24-bit multiply and a shift
  const bool small = GG <= 512 && G <= 127;  // (wave-uniform; cols <= G + 1)
  const int Mg = (65536 + G - 1) / G, Mc = (65536 + cols - 1) / cols;
  auto sdiv = [](int t, int M) { return (int)(((unsigned)t * (unsigned)M) >> 16); };
  // the whole-unit pellets' sums (pint): square t = iy * cols + ix of every
  // (column bit ix, row bit iy) of a pellet's mask -- the squares whose `need`
  // bits the mask holds -- inside the field and with ix < 16, as in the scan
  int *const s_pcnt = &p_px[0].perm;  // (the ranking's slots: unused on this path)
  if (pint) {
    for (int t = lane; t < GG; t += 64) s_pcnt[t] = 0;
    wave_fence();
    auto scatter = [&](const uint32_t *pmk, const double *pmm) __attribute__((always_inline)) {
      for (int i = lane; i < np; i += 64) {
        const uint32_t mk = pmk[i];
        const int mi = (int)pmm[i];
        for (uint32_t X = mk & 0xFFFFu; X; X &= X - 1) {
          const int ix = __ffs(X) - 1;
          if (ix >= cols) break;  // (bits ascend)
          for (uint32_t Y = mk >> 16; Y; Y &= Y - 1) {
            const int t = (__ffs(Y) - 1) * cols + ix;
            if (t >= GG) break;
            const int c = sdiv(t, Mg), r = t - c * G;  // (GG <= 256 here)
            if ((in_col >> r) & (in_row >> c) & 1) atomicAdd(&s_pcnt[t], mi);
          }
        }
      }
    };
#ifdef AIGAR_OBS_DIAG_NOPINT  // (cost diagnostics only, results invalid)
    if (np > 0 && p_m[0] == -1.2345)
#endif
    {
      if (in_lds) scatter(p_mask, p_m);  // (LDS addresses: ds_read)
      else scatter(PL.mask, PL.m);       // (the overflow pool)
    }
    wave_fence();
  }
  // instantiated twice: with the LDS lists themselves (ds_read, no wait on the
  // row stores in flight) and with generic pointers (a list in the overflow pool)
  // The per-square scans read list entry k through accessors: PEL(k) -> (mass,
  // mask) of the k-th pellet in creation order, CEL(k) -> (mass, mask, own),
  // VIR(k) -> (radius, mass, seq, mask).
  // pre (true_type): the scans ran already for both of the lane's squares
  // (squares t = lane, lane + 64: one pass over each list, vp0 / vp1 ...)
  double vp0 = 0, vp1 = 0, vs0 = 0, vs1 = 0, ve0 = 0, ve1 = 0, vv0 = 0, vv1 = 0;
  auto squares = [&](auto hist_regs, auto pre, auto PEL, auto CEL, auto VIR) __attribute__((always_inline)) {
  for (int t0 = 0; t0 < GG; t0 += 64) {
    // every lane runs the shuffles (a shuffle from a lane outside the loop's
    // active set reads 0): lanes past the grid take the last square and store nothing
    const int t = min(t0 + lane, GG - 1);
    const bool act = t0 + lane < GG;
    const int c = small ? sdiv(t, Mg) : idiv(t, G, inv_G), r = t - c * G;
    double mx, my, freeA = 0;
    if (G <= 64) {  // (wave-uniform)
      mx = __shfl(colx, r);
      my = __shfl(rowy, c);
      freeA = __shfl(wcol, r) * __shfl(hrow, c);
    } else {
      mx = left + gs / 2;
      my = top + gs / 2;
      for (int i = 0; i < r; i++) mx += gs;
      for (int i = 0; i < c; i++) my += gs;
    }
    if (!act) continue;
    const int iy = small ? sdiv(t, Mc) : idiv(t, cols, inv_cols), ix = t - iy * cols;
    uint32_t need = (1u << ix) | (1u << (16 + iy));
    double vp = 0, ve = 0, vs = 0, vv = 0;
    const bool within = G <= 64 ? ((in_col >> r) & (in_row >> c) & 1) != 0
                                : !(mx + gs / 2 < 0 || mx - gs / 2 > fieldSize || my + gs / 2 < 0 || my - gs / 2 > fieldSize);
    if constexpr (decltype(pre)::value) {
      vp = t < 64 ? vp0 : vp1;
      vs = t < 64 ? vs0 : vs1;
      ve = t < 64 ? ve0 : ve1;
      vv = t < 64 ? vv0 : vv1;
    } else if (within && ix < 16) {
      if (pint) {
        vp = (double)s_pcnt[t];
      } else {
        double s = 0;
        bool anyp = false;
        for (int k = 0; k < np; k++) {  // creation order
          double m;
          uint32_t mk;
          PEL(k, m, mk);
          const bool hit = (mk & need) == need;
          s = hit ? s + m : s;
          anyp |= hit;
        }
        if (anyp) vp = s;
      }
      bool fe = false, fo = false;
      for (int k = 0; k < nc; k++) {
        double m;
        uint32_t mk;
        bool own;
        CEL(k, m, mk, own);
        if ((mk & need) != need) continue;
        if (own) {
          if (!fo || m > vs) vs = m;
          fo = true;
        } else {
          if (!fe || m > ve) ve = m;
          fe = true;
        }
      }
      bool fv = false;
      double br = 0;
      int64_t bs = 0;
      for (int k = 0; k < nv; k++) {
        double rr, vmk;
        int64_t sq;
        uint32_t mk;
        VIR(k, rr, vmk, sq, mk);
        if ((mk & need) != need) continue;
        if (!fv || rr > br || (rr == br && sq < bs)) {
          br = rr;
          bs = sq;
          vv = vmk;
        }
        fv = true;
      }
    }
#ifdef AIGAR_OBS_DIAG_NOWALL  // (cost diagnostics only, results invalid)
    double vw = 0.0;
#else
    if (G > 64) {
      double lb = py_min(py_max(mx - gs / 2, 0.0), fieldSize), tb = py_min(py_max(my - gs / 2, 0.0), fieldSize);
      double rb = py_max(py_min(mx + gs / 2, fieldSize), 0.0), bb = py_max(py_min(my + gs / 2, fieldSize), 0.0);
      freeA = (rb - lb) * (bb - tb);
    }
    // round(1 - freeA / (gs*gs), 3).  A square inside the field has freeA within
    // a few ulps of gs*gs, and the result is a zero whose sign is that of
    // 1 - fl(freeA / gs2): negative iff fl(freeA / gs2) > 1, i.e. iff the exact
    // quotient exceeds 1 + 2^-53 (the midpoint rounds to even, 1), i.e. iff
    // freeA - gs2 > gs2 * 2^-53 -- exact: the difference of two doubles within a
    // factor 2 (Sterbenz), a power-of-two scaling.  No division then.
    const double gs2 = gs * gs, dlt = freeA - gs2;
    double vw;
    if (freeA == gs2) vw = 0.0;
    else if (fabs(dlt) < 0.0003 * gs2) vw = dlt > gs2 * 0x1p-53 ? -0.0 : 0.0;
    else vw = py_round3(1 - (freeA / gs2));
#endif
    if (o_pel >= 0) row_st(o_pel, t, held ? (OutT)vp : (OutT)__builtin_nan(""));
    if (o_self >= 0) row_st(o_self, t, (OutT)vs);
    if (o_wall >= 0) row_st(o_wall, t, (OutT)vw);
    if (o_enemy >= 0) row_st(o_enemy, t, (OutT)ve);
    if (o_all >= 0) row_st(o_all, t, (OutT)py_max(ve, vs));
    if (o_vir >= 0) row_st(o_vir, t, (OutT)vv);
    double o_sl, o_ss, o_el, o_es;  // history before this frame
    if constexpr (decltype(hist_regs)::value) {
      o_sl = t < 64 ? h_slf0 : h_slf1;
      o_ss = t < 64 ? h_sslf0 : h_sslf1;
      o_el = t < 64 ? h_elf0 : h_elf1;
      o_es = t < 64 ? h_eslf0 : h_eslf1;
    } else {
      o_sl = (o_slf >= 0 || o_sslf >= 0) ? slf[t] : 0.0;
      o_ss = o_sslf >= 0 ? sslf[t] : 0.0;
      o_el = (o_elf >= 0 || o_eslf >= 0) ? elf[t] : 0.0;
      o_es = o_eslf >= 0 ? eslf[t] : 0.0;
    }
    if (o_sslf >= 0) {
      row_st(o_sslf, t, (OutT)o_ss);
      hist_st(sslf, t, o_sl);
    }
    if (o_slf >= 0) {
      row_st(o_slf, t, (OutT)o_sl);
      hist_st(slf, t, vs);
    }
    if (o_eslf >= 0) {
      row_st(o_eslf, t, (OutT)o_es);
      hist_st(eslf, t, o_el);
    }
    if (o_elf >= 0) {
      row_st(o_elf, t, (OutT)o_el);
      hist_st(elf, t, ve);
    }
  }
  };
#ifdef AIGAR_OBS_DIAG_NOCV  // (cost diagnostics only, results invalid: no cell / virus scans)
  nc = 0;
  nv = 0;
#endif
  const bool all_lds = (in_lds || pint) && CL.mask == c_mask && VL.mask == v_mask;  // (pint: no pellet list read)
  if (all_lds && (pint || np <= 64) && nc <= 64 && nv <= 64 && GG <= 128) {
    // common case: entry k of every list sits in lane k's registers and is read
    // with v_readlane into scalar registers (no LDS round trip per entry)
    const bool rp = !pint && lane < np;
    const double rpm = rp ? sm[lane] : 0.0, rcm = lane < nc ? c_mass[lane] : 0.0;
    const uint32_t rpk = rp ? smk[lane] : 0u, rck = lane < nc ? c_mask[lane] : 0u;
    const int rco = lane < nc ? c_own[lane] : 0;
    const double rvr = lane < nv ? v_rad[lane] : 0.0, rvm = lane < nv ? v_mass[lane] : 0.0;
    const int64_t rvs = lane < nv ? v_seqs[lane] : 0;
    const uint32_t rvk = lane < nv ? v_mask[lane] : 0u;
#if AIGAR_OBS_PAIR
    if (GG > 64) {  // both squares of a lane in one pass over each list
      bool ok0, ok1;
      uint32_t nd0, nd1;
      {
        auto sq = [&](int t, bool &ok, uint32_t &need) {
          const int c = sdiv(t, Mg), r = t - c * G;  // (GG <= 128 here)
          const int iy = sdiv(t, Mc), ix = t - iy * cols;
          need = (1u << ix) | (1u << (16 + iy));
          ok = t < GG && ix < 16 && ((in_col >> r) & (in_row >> c) & 1) != 0;
        };
        sq(lane, ok0, nd0);
        sq(lane + 64, ok1, nd1);
      }
      if (pint) {  // (GG <= 128 here; the counts of squares outside the field or past ix 15 stayed 0)
        vp0 = (double)s_pcnt[lane];
        vp1 = lane + 64 < GG ? (double)s_pcnt[lane + 64] : 0.0;
      } else {
        double s0 = 0, s1 = 0;
        bool a0 = false, a1 = false;
        for (int k = 0; k < np; k++) {  // creation order
          const double m = readlane_d(rpm, k);
          const uint32_t mk = (uint32_t)__builtin_amdgcn_readlane((int)rpk, k);
          const bool h0 = ok0 && (mk & nd0) == nd0, h1 = ok1 && (mk & nd1) == nd1;
          s0 = h0 ? s0 + m : s0;
          s1 = h1 ? s1 + m : s1;
          a0 |= h0;
          a1 |= h1;
        }
        vp0 = a0 ? s0 : 0.0;
        vp1 = a1 ? s1 : 0.0;
      }
      bool fe0 = false, fo0 = false, fe1 = false, fo1 = false;
      for (int k = 0; k < nc; k++) {
        const double m = readlane_d(rcm, k);
        const uint32_t mk = (uint32_t)__builtin_amdgcn_readlane((int)rck, k);
        const bool own = __builtin_amdgcn_readlane(rco, k) != 0;
        const bool h0 = ok0 && (mk & nd0) == nd0, h1 = ok1 && (mk & nd1) == nd1;
        if (own) {
          if (h0 && (!fo0 || m > vs0)) vs0 = m;
          if (h1 && (!fo1 || m > vs1)) vs1 = m;
          fo0 |= h0;
          fo1 |= h1;
        } else {
          if (h0 && (!fe0 || m > ve0)) ve0 = m;
          if (h1 && (!fe1 || m > ve1)) ve1 = m;
          fe0 |= h0;
          fe1 |= h1;
        }
      }
      bool fv0 = false, fv1 = false;
      double br0 = 0, br1 = 0;
      int64_t bs0 = 0, bs1 = 0;
      for (int k = 0; k < nv; k++) {
        const double rr = readlane_d(rvr, k), vmk = readlane_d(rvm, k);
        const int64_t sq = readlane_i64(rvs, k);
        const uint32_t mk = (uint32_t)__builtin_amdgcn_readlane((int)rvk, k);
        const bool h0 = ok0 && (mk & nd0) == nd0, h1 = ok1 && (mk & nd1) == nd1;
        if (h0 && (!fv0 || rr > br0 || (rr == br0 && sq < bs0))) {
          br0 = rr;
          bs0 = sq;
          vv0 = vmk;
        }
        if (h1 && (!fv1 || rr > br1 || (rr == br1 && sq < bs1))) {
          br1 = rr;
          bs1 = sq;
          vv1 = vmk;
        }
        fv0 |= h0;
        fv1 |= h1;
      }
      auto none = [](auto...) {};
#if defined(AIGAR_OBS_STOP) && AIGAR_OBS_STOP == 4  // (after the pellet counts and the list scans)
      if (vp0 + vp1 + vs0 + vs1 + ve0 + ve1 + vv0 + vv1 + h_slf0 + h_elf0 == -1.2345) row_st(0, 0, (OutT)0);
      return;
#endif
      squares(std::true_type{}, std::true_type{}, none, none, none);
    } else
#endif
    squares(
        std::true_type{}, std::false_type{},
        [&](int k, double &m, uint32_t &mk) {
          m = readlane_d(rpm, k);
          mk = (uint32_t)__builtin_amdgcn_readlane((int)rpk, k);
        },
        [&](int k, double &m, uint32_t &mk, bool &own) {
          m = readlane_d(rcm, k);
          mk = (uint32_t)__builtin_amdgcn_readlane((int)rck, k);
          own = __builtin_amdgcn_readlane(rco, k) != 0;
        },
        [&](int k, double &rr, double &vmk, int64_t &sq, uint32_t &mk) {
          rr = readlane_d(rvr, k);
          vmk = readlane_d(rvm, k);
          sq = readlane_i64(rvs, k);
          mk = (uint32_t)__builtin_amdgcn_readlane((int)rvk, k);
        });
  } else {
    const double *pm = in_lds ? sm : PL.m;
    const uint32_t *pk = in_lds ? smk : PL.mask;
    const int *pperm = in_lds ? nullptr : PL.perm;
    squares(
        std::false_type{}, std::false_type{},
        [&](int k, double &m, uint32_t &mk) {
          const int e = pperm ? pperm[k] : k;
          m = pm[e];
          mk = pk[e];
        },
        [&](int k, double &m, uint32_t &mk, bool &own) {
          m = CL.m[k];
          mk = CL.mask[k];
          own = CL.own[k] != 0;
        },
        [&](int k, double &rr, double &vmk, int64_t &sq, uint32_t &mk) {
          rr = VL.r[k];
          vmk = VL.m[k];
          sq = VL.seq[k];
          mk = VL.mask[k];
        });
  }
  OBS_STAMP(4);
#ifdef AIGAR_OBS_DIAG_NOSTORE
  if (diag_sum == -1.2345) row[lane] = (OutT)diag_sum;
#endif
#ifdef AIGAR_OBS_TIMING
  if (lane < OBS_TS && gp < 65536) g_obs_ts[(size_t)gp * OBS_TS + lane] = obs_ts_l[lane];
#endif
  extra_store(d, gp, lane, row, off, fs, xin);  // getAdditionalFeatures (bot.py:302-323)
}


// Model.takeBotActions for Greedy bots (bot.py:252-269): make_greedy_bot_move
// (bot.py:579-633) then set_command_point (bot.py:550-577).  One wavefront per
// bot: the three FOV queries in one walk, every lane keeps its best
// mass/distance^2 candidate, a wave reduction picks the maximum with the
// reference's tie rule (first in list order: pellets, enemy cells, viruses,
// each by creation sequence).  mask (optional): which players are Greedy bots.
// mask: NULL = every player; want < 0: players with mask != 0; else mask == want
__global__ void __launch_bounds__(64) k_policy_greedy(Dev d, int greedy_split, const uint8_t *mask, int want) {
  const int gp = xcd_block(blockIdx.x, gridDim.x), lane = threadIdx.x, NP = d.NP, a = gp / d.B;
  if (!d.p_alive[gp] || (mask && (want < 0 ? !mask[gp] : mask[gp] != want))) return;  // (dead players keep their command)
  const ArenaCtl &ctl = d.ctl[a];
  const double fx = d.p_fx[gp], fy = d.p_fy[gp], fs = d.p_fs[gp];
  // biggest own cell: max(playerCells, key=mass) keeps the first maximum
  const int ncell = d.p_ncells[gp];
  double bm = -1, bx = 0, by = 0;
  if (lane < ncell) {
    size_t ci = (size_t)d.p_list[lane * NP + gp] * NP + gp;
    bm = d.c_m[ci];
    bx = d.c_x[ci];
    by = d.c_y[ci];
  }
  greedy_own_best(bm, bx, by);
  const Rect Q = footprint(fx, fy, fs / 2, d.size);
  // C4 (aigar_tile_policy): the tile taking this bot's move must hold every pellet of its view
  if (d.tiled && !tile_holds_rect(d, rect_grow(Q, 1, d.cols)) && lane == wave_leader()) atomicOr(&d.ctl[a].err, ERR_TILE_OBS);
  GreedyAcc acc;
  wave_fov_walk(d, a, Q, fx, fy, fs, ctl.rmax_cell, ctl.rmax_virus, true, d.virus_enabled, [] {},
                [&](bool valid, int kd, size_t g) {
    if (!valid) return;
    const PelRec *PR = d.pel;
    const double *X = kd == 0 ? &PR->x : (kd == 1 ? d.c_x : d.v_x);
    const double *Y = kd == 0 ? &PR->y : (kd == 1 ? d.c_y : d.v_y);
    const double *M = kd == 0 ? &PR->m : (kd == 1 ? d.c_m : d.v_m);
    const double *RR = kd == 1 ? d.c_r : d.v_r;
    const int64_t *S = kd == 0 ? &PR->seq : (kd == 1 ? d.c_seq : d.v_seq);
    const uint32_t *FL = kd == 1 ? d.c_flags : d.v_flags;
    const size_t gr = kd == 0 ? g * kPelStride : g;
    const double x = X[gr], y = Y[gr], m = M[gr];
    const double r = kd == 0 ? pellet_radius(m) : RR[g];
    const uint32_t fl = kd == 0 ? (F_ALIVE | F_INHASH) : FL[g];
    if ((fl & (F_ALIVE | F_INHASH)) != (F_ALIVE | F_INHASH)) return;
    if (kd == 1 && (int)(g % NP) == gp) return;
    if (!in_fov(x, y, r, fx, fy, fs)) return;  // (implies the hash query's footprint test: aigar_sem.h)
    acc.consider(kd, x, y, m, S[gr], bm, bx, by);
  });
  greedy_commit(d, gp, acc, fx, fy, fs, greedy_split);
}
void launch_policy_greedy(const Dev &d, hipStream_t s, int greedy_split, const uint8_t *mask, int want) {
  hipLaunchKernelGGL(k_policy_greedy, dim3(d.NP), dim3(64), 0, s, d, greedy_split, mask, want);
}

// Random bots (bot.py:243-249 make_random_bot_move + makeMove's set_command_point,
// bot.py:252-269): every FRAME_SKIP_RATE of its moves the bot draws a new action
// (two uniforms; split / eject uniforms when enabled, else False), and every tick
// it steers by that action -- split / eject whenever the held value is > 0.5.
// Draws are Philox-keyed by (player, move counter, salt) instead of numpy's stream.
__global__ void k_policy_refrandom(Dev d, int skip_rate, int enable_split, int enable_eject, uint64_t salt) {
  const int gp = GTID;
  if (gp >= d.NP || d.p_role[gp] != AIGAR_ROLE_RANDOM || !d.p_alive[gp]) return;
  const int a = gp / d.B;
  double *cur = d.o_act_cur + (size_t)gp * 4;
  const int t = d.p_time[gp];
  if (skip_rate <= 0 || t % skip_rate == 0) {
    uint64_t u[4];
    philox((uint64_t)gp, ST_REFRANDOM, (uint64_t)t, salt, d.ctl[a].key0, d.ctl[a].key1, u);
    cur[0] = u01(u[0]);
    cur[1] = u01(u[1]);
    cur[2] = enable_split ? u01(u[2]) : 0.0;
    cur[3] = enable_eject ? u01(u[3]) : 0.0;
  }
  d.p_time[gp] = t + 1;
  const int64_t x = (int64_t)d.p_fx[gp], y = (int64_t)d.p_fy[gp];
  const double fs = d.p_fs[gp];
  const int64_t left = x - (int64_t)(fs / 2), top = y - (int64_t)(fs / 2), size = (int64_t)fs;
  d.p_cmdx[gp] = (double)left + cur[0] * (double)size;
  d.p_cmdy[gp] = (double)top + cur[1] * (double)size;
  d.p_split[gp] = cur[2] > 0.5;
  d.p_eject[gp] = cur[3] > 0.5;
}
void launch_policy_refrandom(const Dev &d, hipStream_t s, int skip_rate, int enable_split, int enable_eject,
                             uint64_t salt) {
  hipLaunchKernelGGL(k_policy_refrandom, dim3((d.NP + 255) / 256), dim3(256), 0, s, d, skip_rate, enable_split,
                     enable_eject, salt);
}

// synthetic bot population: random action in [0,1]^2 through set_command_point
// (bot.py:550-577), split/eject with the given probabilities
__global__ void k_policy_random(Dev d, double p_split, double p_eject, uint64_t salt) {
  int gp = GTID;
  if (gp >= d.NP || !d.p_alive[gp]) return;
  const Command c = random_command(d, gp, RandomPolicy{1, p_split, p_eject, salt});
  d.p_cmdx[gp] = c.x;
  d.p_cmdy[gp] = c.y;
  d.p_split[gp] = c.split;
  d.p_eject[gp] = c.eject;
}

// set_command_point (bot.py:550-577) for external actions act[NP][n_act]
// (n_act 2, 3 or 4); during skipped frames split/eject are dropped (bot.py:266-267).
// record: updateValues (bot.py:180-193) -- lastAction <- currentAction <- act.
__global__ void k_apply_actions(Dev d, const double *act, int n_act, int enable_split, int skipping, int record) {
  int gp = GTID;
  if (gp >= d.NP || !d.p_alive[gp]) return;  // makeMove: dead players do not move
  if (d.p_role[gp] != AIGAR_ROLE_NN) return;  // Greedy / Random bots steer themselves
  const double *ac = act + (size_t)gp * n_act;
  const double a0 = ac[0], a1 = ac[1];
  int split = 0, eject = 0;
  if (!skipping && n_act == 4) {
    split = ac[2] > 0.5;
    eject = ac[3] > 0.5;
  } else if (!skipping && n_act == 3 && enable_split) {
    split = ac[2] > 0.5;
  }
  const int64_t x = (int64_t)d.p_fx[gp], y = (int64_t)d.p_fy[gp];
  const double fs = d.p_fs[gp];
  const int64_t left = x - (int64_t)(fs / 2), top = y - (int64_t)(fs / 2), size = (int64_t)fs;
  d.p_cmdx[gp] = (double)left + a0 * (double)size;
  d.p_cmdy[gp] = (double)top + a1 * (double)size;
  d.p_split[gp] = split;
  d.p_eject[gp] = eject;
  if (record)
    for (int k = 0; k < 4; k++) {
      d.o_act_prev[(size_t)gp * 4 + k] = d.o_act_cur[(size_t)gp * 4 + k];
      d.o_act_cur[(size_t)gp * 4 + k] = k < n_act ? ac[k] : 0.0;
    }
}
void launch_apply_actions(const Dev &d, hipStream_t s, const double *act, int n_act, int enable_split, int skipping,
                          int record) {
  hipLaunchKernelGGL(k_apply_actions, dim3((d.NP + 255) / 256), dim3(256), 0, s, d, act, n_act, enable_split,
                     skipping, record);
}

// Bot.getReward (bot.py:654-667) for every player; NaN where the reference
// returns None (no lastMass yet).  update_last: the end of move_NN on a
// decision frame (bot.py:229-230) -- lastMass <- total mass of live players.
// mode 0: out = r (NaN = None); 1: out = r, None -> 0; 2: out += r, None -> 0 (the
// cumulative reward of a frame-skip window, bot.py:166-168,220-228)
__global__ void k_rewards(Dev d, double *out, aigar_reward_params prm, int update_last, int mode) {
  int gp = GTID;
  if (gp >= d.NP) return;
  const bool alive = d.p_alive[gp];
  const double mass = alive ? d.p_mass[gp] : 0.0, last = d.o_last_mass[gp];
  double r;
  if (prm.mass_as_reward) {
    r = alive ? mass - prm.reward_term : prm.death_term - prm.reward_term;
  } else if (isnan(last)) {
    r = __builtin_nan("");
  } else {
    double rw = alive ? mass - last : -1 * last * prm.death_factor + prm.death_term;
    r = rw * prm.reward_scale - prm.reward_term;
  }
  if (mode != 0 && isnan(r)) r = 0;
  out[gp] = mode == 2 ? out[gp] + r : r;
  if (update_last && alive) d.o_last_mass[gp] = mass;
}
void launch_rewards(const Dev &d, hipStream_t s, double *out, const aigar_reward_params &p, int update_last,
                    int mode) {
  hipLaunchKernelGGL(k_rewards, dim3((d.NP + 255) / 256), dim3(256), 0, s, d, out, p, update_last, mode);
}

__global__ void k_player_stats(Dev d, double *out) {
  int gp = GTID;
  if (gp >= d.NP) return;
  double *o = out + (size_t)gp * 5;
  if (!d.p_alive[gp]) {
    o[0] = 0;
    o[1] = 0;
    o[2] = o[3] = o[4] = __builtin_nan("");
    return;
  }
  const Fov f{d.p_fx[gp], d.p_fy[gp], d.p_fs[gp], d.p_mass[gp], 0};
  o[0] = 1;
  o[1] = f.mass;
  o[2] = f.fx;
  o[3] = f.fy;
  o[4] = f.fs;
}

__global__ void k_set_commands(Dev d, const double *cmd) {
  int gp = GTID;
  if (gp >= d.NP) return;
  d.p_cmdx[gp] = cmd[4 * (size_t)gp];
  d.p_cmdy[gp] = cmd[4 * (size_t)gp + 1];
  d.p_split[gp] = cmd[4 * (size_t)gp + 2] != 0;
  d.p_eject[gp] = cmd[4 * (size_t)gp + 3] != 0;
}

// FOV cache of every live player, and the arena's largest cell radius (bounds
// the cell-grid expansion of the observation and the next greedy moves)
__global__ void __launch_bounds__(256) k_player_fov(Dev d) { fov_cache_thread(d, GTID); }
void launch_player_fov(const Dev &d, hipStream_t s) {
  hipLaunchKernelGGL(k_player_fov, dim3((d.NP + 255) / 256), dim3(256), 0, s, d);
}
// ---------------------------------------------------- pixel observation
// RGBGenerator.get_cnn_inputRGB (rgbGenerator.py:95-110) for every player: a
// white side x side frame, every pellet / blob / virus / player cell in the FOV
// (drawAllCells, rgbGenerator.py:60-68) stable-sorted by mass and drawn in
// that order, then numpy.average(weights=[0.298, 0.587, 0.114]) grayscale.
// pygame's primitives follow the published SDL_gfx 2.0 algorithms (see
// oracle/oracle.c pixels_one; pygame itself is absent, parity with it is
// unpinned): rad >= 4 filledCircle + aacircle rim (black for viruses), else
// pygame.draw.circle as filledEllipse spans.
// One 64-lane block per player, the frame in LDS (packed 0x00RRGGBB): the FOV
// objects are gathered by the observation walk (+ the arena's blob slots),
// culled to those that touch the frame, bitonic-sorted by (mass, kind, seq),
// then drawn one by one: lane 0 runs the span recurrence into a half-width
// table, all lanes fill the spans, lane 0 runs the anti-aliased rim (its
// blends are order-dependent).
#include "pixels.inc"

#include "obs_wide.inc"

constexpr int kObsWtBots = 16384;  // k_observe's store policy switch (bots per launch)
// the state representation the configuration asks for (bot.py:272-299): the
// default grid (<= 16 squares per side), the wide grid (CNN grid view), or the
// simple representation (GRID_VIEW_ENABLED = False)
// whether the observation can also pick the next tick's Greedy moves (k_observe's
// GREEDY mode: the grid observation with its pellet channel, which walks every
// candidate the Greedy policy reads)
bool observe_fuses_greedy(const Dev &d) {
  return !(d.obs_ch & AIGAR_OBS_SIMPLE) && d.G <= 16 && (d.obs_ch & AIGAR_OBS_PELLET) && !d.tiled;
}
// greedy_next >= 0 (observe_fuses_greedy): also the next tick's Greedy moves, with greedy_split = greedy_next
void launch_observe(const Dev &d, hipStream_t s, void *out, int dtype, uint32_t epoch, const uint8_t *mask,
                    int greedy_next) {
  if (greedy_next >= 0 && observe_fuses_greedy(d) && !mask) {
    const bool wt = d.NP <= kObsWtBots;
    if (dtype == 0) {
      if (wt) hipLaunchKernelGGL((k_observe<double, true, true>), dim3(d.NP), dim3(64), 0, s, d, (double *)out, epoch, mask, greedy_next);
      else hipLaunchKernelGGL((k_observe<double, false, true>), dim3(d.NP), dim3(64), 0, s, d, (double *)out, epoch, mask, greedy_next);
    } else {
      if (wt) hipLaunchKernelGGL((k_observe<float, true, true>), dim3(d.NP), dim3(64), 0, s, d, (float *)out, epoch, mask, greedy_next);
      else hipLaunchKernelGGL((k_observe<float, false, true>), dim3(d.NP), dim3(64), 0, s, d, (float *)out, epoch, mask, greedy_next);
    }
    return;
  }
  if (greedy_next >= 0) launch_policy_greedy(d, s, greedy_next, nullptr, -1);  // (cannot fuse: its own launch, first)
  if (d.obs_ch & AIGAR_OBS_SIMPLE) {
    if (dtype == 0) hipLaunchKernelGGL(k_observe_simple<double>, dim3(d.NP), dim3(64), 0, s, d, (double *)out, mask);
    else hipLaunchKernelGGL(k_observe_simple<float>, dim3(d.NP), dim3(64), 0, s, d, (float *)out, mask);
  } else if (d.G > 16) {
    if (dtype == 0) hipLaunchKernelGGL(k_observe_wide<double>, dim3(d.NP), dim3(64), 0, s, d, (double *)out, epoch, mask);
    else hipLaunchKernelGGL(k_observe_wide<float>, dim3(d.NP), dim3(64), 0, s, d, (float *)out, epoch, mask);
  } else {
    // write-through stores up to a few arenas' worth of bots (a latency-bound
    // launch), non-temporal beyond (a streaming one); see k_observe
    const bool wt = d.NP <= kObsWtBots;
    if (dtype == 0) {
      if (wt) hipLaunchKernelGGL((k_observe<double, true, false>), dim3(d.NP), dim3(64), 0, s, d, (double *)out, epoch, mask, 0);
      else hipLaunchKernelGGL((k_observe<double, false, false>), dim3(d.NP), dim3(64), 0, s, d, (double *)out, epoch, mask, 0);
    } else {
      if (wt) hipLaunchKernelGGL((k_observe<float, true, false>), dim3(d.NP), dim3(64), 0, s, d, (float *)out, epoch, mask, 0);
      else hipLaunchKernelGGL((k_observe<float, false, false>), dim3(d.NP), dim3(64), 0, s, d, (float *)out, epoch, mask, 0);
    }
  }
}
void launch_policy(const Dev &d, hipStream_t s, double ps, double pe, uint64_t salt) {
  hipLaunchKernelGGL(k_policy_random, dim3((d.NP + 255) / 256), dim3(256), 0, s, d, ps, pe, salt);
}
void launch_player_stats(const Dev &d, hipStream_t s, double *out) {
  hipLaunchKernelGGL(k_player_stats, dim3((d.NP + 255) / 256), dim3(256), 0, s, d, out);
}
void launch_set_commands(const Dev &d, hipStream_t s, const double *cmd) {
  hipLaunchKernelGGL(k_set_commands, dim3((d.NP + 255) / 256), dim3(256), 0, s, d, cmd);
}

}  // namespace aigar

#ifdef AIGAR_OBS_TIMING
extern "C" int aigar_debug_obs_ts(unsigned long long *out, int n) {
  n = n < 65536 ? n : 65536;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(aigar::g_obs_ts), sizeof(unsigned long long) * n * aigar::OBS_TS) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif
