// aigar_wave.h -- wavefront-level helpers shared by the tick and observation
// kernels (one 64-lane wavefront cooperating on one query).
#pragma once
#include <hip/hip_runtime.h>

#include "aigar_dev.h"
#include "aigar_math.h"
#include "aigar_sem.h"

namespace aigar {

// XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md, workgroup dispatch), so block b and b + 1 sit on
// different L2s.  Kernels with one wave per player remap b so that the players
// of consecutive logical blocks -- whose per-player words share 128-B lines
// (p_fx, c_x[slot * NP + gp], ...) -- are served by one XCD's L2.  Placement
// is only observed, never guaranteed: a bijection, correct for any placement.
__device__ __forceinline__ int xcd_block(int b, int nb) {
  const int per = nb >> 3, rem = nb & 7, x = b & 7, i = b >> 3;
  return x < rem ? x * (per + 1) + i : rem * (per + 1) + (x - rem) * per + i;
}

// a wave-uniform value moved to SGPRs (the compiler keeps a uniform value that
// came from a vector load in VGPRs; in a register-bound kernel that costs waves)
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// the wave's first active lane: a claim or an error bit written by "lane 0" is lost
// when lane 0 is inactive (the round-5 hang: a lane-0 atomic that never ran)
__device__ __forceinline__ int wave_leader() { return __ffsll((long long)__ballot(1)) - 1; }
__device__ __forceinline__ int64_t uni(int64_t v) {
  const int lo = __builtin_amdgcn_readfirstlane((int)v), hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double uni(double v) { return __longlong_as_double(uni((int64_t)__double_as_longlong(v))); }
__device__ __forceinline__ Rect uni(Rect r) {
  r.x0 = uni(r.x0);
  r.x1 = uni(r.x1);
  r.y0 = uni(r.y0);
  r.y1 = uni(r.y1);
  return r;
}

__device__ __forceinline__ void atomic_max_pos(double *addr, double v) {  // v >= 0
  atomicMax((unsigned long long *)addr, (unsigned long long)__double_as_longlong(v));
}
// max over the wavefront, then one atomic per wave (all lanes must call; invalid
// lanes pass 0).  A wave whose lanes target different arenas falls back to per-lane atomics.
__device__ __forceinline__ void wave_atomic_max_pos(double *addr, double v) {
  unsigned long long ad = (unsigned long long)addr, a0 = __shfl(ad, 0);
  if (__all(ad == a0)) {
    double m = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off));
    if (__lane_id() == 0 && m > 0) atomic_max_pos(addr, m);
  } else if (v > 0) {
    atomic_max_pos(addr, v);
  }
}

// C4 tiles (aigar_dev.h): ownership by centre bucket; a tile holds the pellets of
// its owned range grown by the halo.  Untiled handles own and hold everything.
__device__ __forceinline__ bool tile_owns(const Dev &d, double x, double y) {
  if (!d.tiled) return true;
  const int bx = center_bucket_coord(x, d.cols), by = center_bucket_coord(y, d.cols);
  return bx >= d.own_bx0 && bx < d.own_bx1 && by >= d.own_by0 && by < d.own_by1;
}
__device__ __forceinline__ bool tile_holds_bucket(const Dev &d, int bx, int by) {
  return !d.tiled || (bx >= d.loc_bx0 && bx < d.loc_bx1 && by >= d.loc_by0 && by < d.loc_by1);
}
// bucket rectangle r (inclusive) grown by e buckets, clamped to the field
__device__ __forceinline__ Rect rect_grow(Rect r, int e, int cols) {
  return Rect{max(0, r.x0 - e), min(cols - 1, r.x1 + e), max(0, r.y0 - e), min(cols - 1, r.y1 + e)};
}
// every bucket of r lies in the held range
__device__ __forceinline__ bool tile_holds_rect(const Dev &d, Rect r) {
  return !d.tiled || r.x1 < r.x0 || r.y1 < r.y0 ||
         (r.x0 >= d.loc_bx0 && r.x1 < d.loc_bx1 && r.y0 >= d.loc_by0 && r.y1 < d.loc_by1);
}
// r touches the held range grown by e buckets
__device__ __forceinline__ bool tile_near_rect(const Dev &d, Rect r, int e) {
  return !d.tiled || (r.x0 <= r.x1 && r.y0 <= r.y1 && r.x1 >= d.loc_bx0 - e && r.x0 < d.loc_bx1 + e &&
                      r.y1 >= d.loc_by0 - e && r.y0 < d.loc_by1 + e);
}
// the tile owning the centre bucket of (x, y) (tile k owns buckets
// [k * cols / n, (k + 1) * cols / n) along each axis, as aigar_create cuts them)
__device__ __forceinline__ int tile_of(const Dev &d, double x, double y) {
  const int bx = center_bucket_coord(x, d.cols), by = center_bucket_coord(y, d.cols);
  int ix = 0, iy = 0;
  for (int i = 1; i < d.tile_nx; i++) ix = bx >= i * d.cols / d.tile_nx ? i : ix;
  for (int i = 1; i < d.tile_ny; i++) iy = by >= i * d.cols / d.tile_ny ? i : iy;
  return iy * d.tile_nx + ix;
}
// the j-th observation-history grid a bot keeps (the ones the channels need, in
// the order self LF, self SLF, enemy LF, enemy SLF): the hand-off slot layout
__device__ __forceinline__ double *hist_grid(const Dev &d, int j) {
  const uint32_t ch = d.obs_ch;
  const int s = (ch & (AIGAR_OBS_SELF_LF | AIGAR_OBS_SELF_SLF)) ? 1 : 0, ss = (ch & AIGAR_OBS_SELF_SLF) ? 1 : 0;
  const int e = (ch & (AIGAR_OBS_ENEMY_LF | AIGAR_OBS_ENEMY_SLF)) ? 1 : 0;
  if (s && j == 0) return d.o_self_lf;
  j -= s;
  if (ss && j == 0) return d.o_self_slf;
  j -= ss;
  if (e && j == 0) return d.o_en_lf;
  return d.o_en_slf;
}

// Wave-parallel walk over the grid rows around q (expanded by E): the rows'
// item ranges are loaded by one lane each and flattened with a prefix sum, so
// 64 items are inspected per step whatever the row layout.  f(valid, item) is
// called by every lane (it may ballot); valid is false on padding lanes.
// Buckets of a centre-bucket grid covering footprint q grown by E fine
// buckets.  Grids of the small entity sets (viruses, blobs) are coarsened by
// 2^shift fine buckets per side (Dev::cshift); every consumer still applies
// the exact reference membership test, so coarsening only adds candidates.
struct Span {
  int bx0, bx1, by0, by1, stride;
};
__device__ __forceinline__ Span grid_span(Rect q, int E, int cols, int shift) {
  Span s;
  s.bx0 = max(0, q.x0 - E) >> shift;
  s.bx1 = min(cols - 1, q.x1 + E) >> shift;
  s.by0 = max(0, q.y0 - E) >> shift;
  s.by1 = min(cols - 1, q.y1 + E) >> shift;
  s.stride = (cols + (1 << shift) - 1) >> shift;
  return s;
}

// xlo/xlen: one extra range of item indices [xlo, xlo + xlen) walked in the same
// steps (valid only without an items array: f receives xlo + k)
template <class F>
// stride: entries per grid row of st (0: the grid's own width; the pellet rows keep
// one more, the row's end)
__device__ __forceinline__ void wave_grid_for(const int *st, const int *items, int cols, Rect q, int E, F f,
                                              int shift = 0, int xlo = 0, int xlen = 0, int stride = 0) {
  if (q.x1 < q.x0 || q.y1 < q.y0) return;
  const Span g = grid_span(q, E, cols, shift);
  const int bx0 = g.bx0, bx1 = g.bx1, by0 = g.by0, cols_ = stride ? stride : g.stride;
  const int lane = threadIdx.x & 63, ngrid = g.by1 - by0 + 1, nrows = ngrid + (xlen > 0 ? 1 : 0);
  for (int r0 = 0; r0 < nrows; r0 += 64) {
    const int r = r0 + lane, nr = min(64, nrows - r0);
    int lo = 0, len = 0;
    if (r < ngrid) {
      int b = (by0 + r) * cols_;
      lo = st[b + bx0];
      len = st[b + bx1 + 1] - lo;
    } else if (r == ngrid && xlen > 0) {
      lo = xlo;
      len = xlen;
    }
    int inc = len;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      int y = __shfl_up(inc, off);
      if (lane >= off) inc += y;
    }
    const int excl = inc - len, total = __shfl(inc, 63);
    for (int t0 = 0; t0 < total; t0 += 64) {
      const int t = t0 + lane;
      int row = 0;
      for (int k = 1; k < nr; k++) row = (__builtin_amdgcn_readlane(excl, k) <= t) ? k : row;  // (k uniform: v_readlane)
      const int idx = __shfl(lo, row) + (t - __shfl(excl, row));
      const bool valid = t < total;
      f(valid, valid ? (items ? items[idx] : idx) : -1);
    }
  }
}
__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// getFovSize / getFovPos / getTotalMass of one player (player.py:129,156-167),
// sequential over its cells in list order (numpy pairwise sums below 128)
struct Fov {
  double fx, fy, fs, mass, rmax;
  int n;
};
__device__ inline Fov player_fov(const Dev &d, int gp) {
  const int NP = d.NP;
  Fov f;
  int n = d.p_ncells[gp];
  f.n = n;
  double ms[kMaxCells], xs[kMaxCells], ys[kMaxCells];
  double rb = -1;
  for (int k = 0; k < n; k++) {
    size_t ci = (size_t)d.p_list[k * NP + gp] * NP + gp;
    double m = d.c_m[ci], r = d.c_r[ci];
    ms[k] = m;
    xs[k] = d.c_x[ci] * m;
    ys[k] = d.c_y[ci] * m;
    if (k == 0 || r > rb) rb = r;
  }
  f.mass = n ? np_sum(ms, n) : 0.0;
  f.fs = aigar_math::pow_glibc(rb, 0.475) * d.pow_n032[n] * 35;  // (table: same glibc pow values)
  f.fx = np_sum(xs, n) / f.mass;
  f.fy = np_sum(ys, n) / f.mass;
  f.rmax = rb;
  return f;
}
// per-player FOV cache, refreshed once the world state of a tick is final
__device__ inline void store_player_fov(const Dev &d, int gp) {
  if (!d.p_alive[gp]) return;
  Fov f = player_fov(d, gp);
  d.p_fx[gp] = f.fx;
  d.p_fy[gp] = f.fy;
  d.p_fs[gp] = f.fs;
  d.p_mass[gp] = f.mass;
}
// one thread of the end-of-tick FOV cache pass (every thread of the wave calls
// it): getFovPos / getFovSize / getTotalMass (player.py:129,156-167) for the
// observation and the policies, the largest cell radius for their grid walks,
// and a fresh overflow-pool epoch for an observe replayed from a graph (epoch
// argument 0; host-issued observes pass epochs below 2^31, these sit above)
__device__ inline void fov_cache_thread(const Dev &d, int gp) {
  const bool live = gp < d.NP && d.p_alive[gp];
  double rb = 0;
  const int a = gp < d.NP ? gp / d.B : 0;
  if (live) {
    const Fov f = player_fov(d, gp);
    d.p_fx[gp] = f.fx;
    d.p_fy[gp] = f.fy;
    d.p_fs[gp] = f.fs;
    d.p_mass[gp] = f.mass;
    rb = f.rmax;
  }
  wave_atomic_max_pos(&d.ctl[a].rmax_cell, rb);  // (per-lane atomics when a wave spans arenas)
  if (gp == 0) *d.ob_epoch = 0x80000000u | ((*d.ob_epoch + 1) & 0x7FFFFFFFu);
}

// The synthetic bot population's command for live player gp (bench / smoke
// driver): an action in [0,1]^2 through set_command_point (bot.py:550-577),
// split / eject with probabilities ps / pe; Philox-keyed by (player, tick, salt).
struct Command {
  double x, y;
  int split, eject;
};
__device__ inline Command random_command(const Dev &d, int gp, const RandomPolicy &rp) {
  const int a = gp / d.B;
  const double fx = d.p_fx[gp], fy = d.p_fy[gp], fs = d.p_fs[gp];
  uint64_t u[4];
  philox((uint64_t)gp, ST_POLICY, (uint64_t)d.ctl[a].tick, rp.salt, d.ctl[a].key0, d.ctl[a].key1, u);
  const double a0 = u01(u[0]), a1 = u01(u[1]);
  const int64_t x = (int64_t)fx, y = (int64_t)fy;
  const int64_t left = x - (int64_t)(fs / 2), top = y - (int64_t)(fs / 2), size = (int64_t)fs;
  return Command{(double)left + a0 * (double)size, (double)top + a1 * (double)size, u01(u[2]) < rp.ps,
                 u01(u[3]) < rp.pe};
}

}  // namespace aigar
