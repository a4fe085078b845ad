// tick.hip -- Field.update() (field.py:85-92) as a sequence of gfx950 kernels.
//
// Phase map (kernel <- reference), in launch order:
//   k_players                 one block per 256 players, one per arena and one per 512 blob
//                             slots: updateViruses + updateBlobs (field.py:94-110) and the
//                             tick's bookkeeping in the extra blocks, the player blocks first the per-cell part
//                             of Player.update (player.py:39-44), then the
//                             rest of updatePlayers (split, eject, move, push-apart) +
//                             creation-sequence numbers (canonical order) + blob append
//                             field.py:112-181, player.py:30-72; + updateHashTables for
//                             blobs and viruses (field.py:121-132; centre-bucket counting
//                             sort, membership tested exactly per query)
//   k_merge_pv                mergePlayerCells + virus<-blob activity + cell<-virus activity
//                             field.py:183-198, 246-253, 225-231 (a player's thread merges,
//                             then tests its cells); its last block: virusBlobOverlap's and
//                             playerVirusOverlap's serial passes (field.py:316-325, 333-370)
//                             (k_merge_vb: the merges alone, viruses disabled)
//   k_food_prep/commit        playerPelletOverlap + playerBlobOverlap field.py:207-222 as one
//                             "deterministic reservations" pass: each cell reserves the foods
//                             it could ever eat; a cell commits once it owns them all (=> every
//                             earlier conflicting cell has committed); leftovers run serially
//                             in priority order in the last commit round's last block.  Extra
//                             blocks of rounds 1 / 2 build the player-cell grid.
//   k_pp_active               playerPlayerOverlap      field.py:233-244
//                             parallel activity test; its serial pass (one wavefront per
//                             arena walks the active players in order: live-list semantics
//                             incl. skip-after-removal, re-activating neighbours on growth)
//                             opens k_spawn_plan
//   k_spawn_plan/all          spawnStuff               field.py:256-313
//   k_pel_update              closing pellet update: the bucket rows whose pellets changed are
//                             rewritten; extra blocks respawn players (FOV cache) and spawn viruses
// "last block" = the block that draws the last ticket (last_block): an idle
// serial pass then costs a ticket, not a dependent launch.
#include <hip/hip_runtime.h>

#include "aigar_dev.h"
#include "aigar_sem.h"
#include "aigar_wave.h"

namespace aigar {

#define GTID ((int)(blockIdx.x * blockDim.x + threadIdx.x))
// C4: a later eat pass issued without a host decision (aigar_tile_apply with no
// readback) does nothing once the last exchange left no owned cell undone on any
// tile -- the count is in every tile's ArenaCtl, written by k_tile_apply
#define TILE_GATE(d)                                          \
  do {                                                        \
    if ((d).tile_gate && (d).ctl[0].n_undone_glob == 0) return; \
  } while (0)

// Diagnostics build only (-DAIGAR_PHASE_TIMING, tools/phase_timing.py): per
// wave, its start time (slot 0, low 32 bits of the 100 MHz wall clock) and the
// time from its start to each mark, after its outstanding loads have landed
// (plain stores to the wave's own slots: no contention).  The product build
// compiles these to nothing.
#ifdef AIGAR_PHASE_TIMING
constexpr int kPtWaves = 8192;
__device__ unsigned int g_ptw[9][kPtWaves][8];
__device__ unsigned int g_ptid[9][kPtWaves][2];  // HW_ID, XCC_ID of the wave
__device__ __forceinline__ void pt_ids(unsigned *o) {
  unsigned a, b;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(a));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(b));
  o[0] = a;
  o[1] = b;
}
#define PT_BEGIN(PT_K)                                                                              \
  const unsigned long long pt0_ = wall_clock64();                                                   \
  const int pt_w_ = (blockIdx.x + blockIdx.y * gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); \
  if ((threadIdx.x & 63) == 0 && pt_w_ < kPtWaves) {                                                \
    g_ptw[PT_K][pt_w_][0] = (unsigned)pt0_;                                                         \
    pt_ids(g_ptid[PT_K][pt_w_]);                                                                    \
  }
#define PT_MARK(k, m)                                                                               \
  do {                                                                                              \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                     \
    if ((threadIdx.x & 63) == 0 && pt_w_ < kPtWaves) g_ptw[k][pt_w_][m] = (unsigned)(wall_clock64() - pt0_); \
  } while (0)
#define PT_PARAMS , unsigned long long pt0_, int pt_w_
// a mark in divergent code: recorded by the first active lane (the latest pass wins)
#define PT_MARKW(k, m)                                                                              \
  do {                                                                                              \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                     \
    if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1 && pt_w_ < kPtWaves)         \
      g_ptw[k][pt_w_][m] = (unsigned)(wall_clock64() - pt0_);                                       \
  } while (0)
// accumulating buckets for a serial loop (g_ptw[6][a][k]: wall-clock ticks, [7][a][k]: counts)
#define PA_DECL                                   \
  unsigned long long pa_t_ = wall_clock64();      \
  unsigned pa_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pa_cnt_[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define PA_T(k)                                                         \
  do {                                                                  \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");         \
    const unsigned long long pa_n_ = wall_clock64();                    \
    pa_acc_[k] += (unsigned)(pa_n_ - pa_t_);                            \
    pa_t_ = pa_n_;                                                      \
  } while (0)
#define PA_C(k) (pa_cnt_[k]++)
#define PA_ADD(k, v) (pa_cnt_[k] += (v))
#define PA_STORE(a)                                                             \
  if ((threadIdx.x & 63) == 0 && (a) < kPtWaves)                                \
    for (int k_ = 0; k_ < 8; k_++) {                                            \
      g_ptw[6][a][k_] += pa_acc_[k_];                                           \
      g_ptw[7][a][k_] += pa_cnt_[k_];                                           \
    }
// (the parallel pp groups' waves: summed over the waves, at index 1024 + a)
#define PA_STORE_GROUP(a)                                                       \
  if ((threadIdx.x & 63) == 0 && 1024 + (a) < kPtWaves)                         \
    for (int k_ = 0; k_ < 8; k_++) {                                            \
      atomicAdd(&g_ptw[6][1024 + (a)][k_], pa_acc_[k_]);                        \
      atomicAdd(&g_ptw[7][1024 + (a)][k_], pa_cnt_[k_]);                        \
    }
#define PT_ARGS , pt0_, pt_w_
// block-level sub-marks of k_spawn_plan's pp pass (g_ptw[6][2048 + block][k]: time from the wave's start)
#define PT_SUB(k)                                                                                 \
  do {                                                                                            \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                   \
    if (threadIdx.x == 0 && 2048 + blockIdx.x < kPtWaves)                                         \
      g_ptw[6][2048 + blockIdx.x][k] = (unsigned)(wall_clock64() - pt0_);                         \
  } while (0)
#else
#define PT_SUB(k)
#define PT_BEGIN(k)
#define PT_MARK(k, m)
#define PT_MARKW(k, m)
#define PT_PARAMS
#define PT_ARGS
#define PA_DECL
#define PA_STORE_GROUP(a)
#define PA_T(k)
#define PA_C(k)
#define PA_ADD(k, v)
#define PA_STORE(a)
#endif

__device__ __forceinline__ void set_err(const Dev &d, int a, uint32_t bit) { atomicOr(&d.ctl[a].err, bit); }

constexpr int SG_CAP = 4096;           // cells of a coarse grid (small entity sets, player cells)
constexpr int CG_STRIDE = SG_CAP + 4;  // per-arena, per-parity stride of Dev::cgcnt (16-byte aligned rows)
template <int KIND>
__device__ __forceinline__ void grid_small_build(const Dev &d, int a, int *cnt, int *sh);

// Last-block ticket (cdna_hip_programming.md, the in-launch reduction recipe):
// each of the nblocks participating blocks publishes its writes (every wave's
// stores drained, one agent-scope release) and takes a ticket; the block that
// draws the last one returns true in all its threads and, after its acquire,
// sees every participant's writes.  The last block resets the counter, so it is
// 0 between launches (dalloc zeroes it).  Correct for any block placement.
// (acquire false: the caller acquires itself, and only when it reads other
// blocks' plain stores -- agent_acquire_block below)
__device__ bool last_block(int *ticket, int nblocks, bool acquire = true) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == nblocks - 1;
    if (t == nblocks - 1) {
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (acquire) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
  }
  __syncthreads();
  return s_last;
}
// the last block's deferred acquire (every thread of the block calls it; `need`
// block-uniform): one lane's agent-scope acquire, its wait, then the barrier
__device__ void agent_acquire_block(bool need) {
  if (!need) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}
// a work counter other blocks raise with atomics, read without an acquire
__device__ __forceinline__ int agent_load(const int *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The same without the fences (each ~0.7 us on the kernel's tail, A/B r06):
// for a last block that reads only words the other blocks stored or added with
// agent-scope atomics (sc1), loading them with agent-scope atomic loads -- the
// ticket's add comes after every storing wave's vmcnt(0), so the last block's
// loads after its add returned see them (MI355X_MICROARCH.md, hand-off table)
__device__ bool last_block_relaxed(int *ticket, int nblocks) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == nblocks - 1;
    if (t == nblocks - 1) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return s_last;
}
// The same for a wide grid: the tickets are sharded by blockIdx % 8 (tk[0..7]),
// the last block of each shard takes a ticket of tk[8], so no counter sees more
// than ~nblocks / 8 arrivals (one device-scope counter serialises them at
// ~12 ns each, MI355X_MICROARCH.md row fanin).  Acquire / release between the
// two levels chain the visibility from every block to the last one.
__device__ bool last_block_sharded(int *tk, int nblocks) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int sh = blockIdx.x & 7, members = (nblocks - sh + 7) / 8, shards = min(8, nblocks);
    int last = 0;
    if (__hip_atomic_fetch_add(&tk[sh], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == members - 1) {
      __hip_atomic_store(&tk[sh], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (__hip_atomic_fetch_add(&tk[8], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == shards - 1) {
        __hip_atomic_store(&tk[8], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = 1;
      }
    }
    s_last = last;
  }
  __syncthreads();
  return s_last;
}

__device__ __forceinline__ void tile_out(const Dev &d, int32_t kind, int32_t idx, int64_t seq, double x, double y) {
  const int i = atomicAdd(&d.ctl[0].n_out, 1);
  if (i >= d.tcap) {
    atomicOr(&d.ctl[0].err, (uint32_t)ERR_TILE_CAP);
    return;
  }
  if (kind == TR_PELLET) atomicAdd(&d.ctl[0].n_out_pel, 1);
  TileRec &r = d.outbox[1 + i];
  r.kind = kind;
  r.idx = idx;
  r.seq = seq;
  r.x = x;
  r.y = y;
}

__device__ void ev_push_at(const Dev &d, int a, int64_t tick, uint32_t phase, uint64_t order, int code, int64_t x,
                           int64_t y) {
  if (!(d.flags & 1)) return;
  // tiles: the replicated phases are logged by tile 0, the eat phases by the cell's owner
  if (d.tiled && d.tile_id != 0 && phase != PH_PELLET && phase != PH_BLOB) return;
  int i = atomicAdd(&d.ctl[a].n_ev, 1);
  if (i >= d.EVcap) {
    set_err(d, a, ERR_EVENT_CAP);
    return;
  }
  int64_t *e = d.ev + ((size_t)a * d.EVcap + i) * 5;
  e[0] = (tick << 8) | phase;
  e[1] = (int64_t)order;
  e[2] = code;
  e[3] = x;
  e[4] = y;
}
__device__ void ev_push(const Dev &d, int a, uint32_t phase, uint64_t order, int code, int64_t x, int64_t y) {
  ev_push_at(d, a, d.ctl[a].tick, phase, order, code, x, y);
}

// centre-bucket grid iteration: every entity whose centre bucket lies in the
// query rectangle grown by E buckets (E covers the largest footprint).
template <class F>
__device__ __forceinline__ void grid_visit(const int *start, const int *items, int cols, Rect q, int E, F f,
                                           int shift = 0) {
  if (q.x1 < q.x0 || q.y1 < q.y0) return;
  const Span g = grid_span(q, E, cols, shift);
  for (int by = g.by0; by <= g.by1; by++) {
    int lo = start[by * g.stride + g.bx0], hi = start[by * g.stride + g.bx1 + 1];
    for (int t = lo; t < hi; t++) f(items ? items[t] : t);
  }
}
__device__ __forceinline__ int expand_for(double rmax) { return (int)ceil((rmax + 1.0) / kBucket) + 1; }

// ------------------------------------------------------------ T1 viruses
__device__ __forceinline__ void update_virus(const Dev &d, int gi) {
  int a = gi / d.Vcap, i = gi - a * d.Vcap;
  if (i >= d.ctl[a].n_vir || !(d.v_flags[gi] & F_ALIVE)) return;
  int svc = d.v_svc[gi];
  double svx = d.v_svx[gi], svy = d.v_svy[gi], x = d.v_x[gi], y = d.v_y[gi];
  update_momentum(svc, svx, svy);
  update_pos(x, y, d.v_vx[gi], d.v_vy[gi], svx, svy, svc, (double)d.size, (double)d.size);
  d.v_svc[gi] = svc;
  d.v_svx[gi] = svx;
  d.v_svy[gi] = svy;
  d.v_x[gi] = x;
  d.v_y[gi] = y;
  d.v_flags[gi] |= F_INHASH;  // updateHashTables (later this tick) inserts every virus
}

// ------------------------------------------------------------ T2 blobs
// (returns whether the blob lives on as a blob, with its new position in x, y)
__device__ __forceinline__ bool update_blob(const Dev &d, int gi, double &x, double &y) {
  int a = gi / d.Ecap, i = gi - a * d.Ecap;
  if (i >= d.ctl[a].n_blob || !(d.b_flags[gi] & F_ALIVE)) return false;
  if (d.b_svc[gi] == 0) {  // stopped blob becomes a pellet (addPellet)
    int j = atomicAdd(&d.ctl[a].n_pnew, 1);
    if (j >= d.Pcap) {  // (the staging list; eat-phase index PS + j, see Food)
      set_err(d, a, ERR_PELLET_CAP);
      return false;
    }
    size_t pj = (size_t)a * d.Pcap + j;
    d.pn[pj] = PelRec{d.b_x[gi], d.b_y[gi], d.b_m[gi], d.b_seq[gi]};
    d.pn_col[pj] = d.b_col[gi];  // (addPellet(blob): the same object, its colour kept)
    d.b_flags[gi] = 0;
    atomicOr(&d.ctl[a].dirty, DIRTY_BLOB);
    return false;
  }
  int svc = d.b_svc[gi];
  double svx = d.b_svx[gi], svy = d.b_svy[gi];
  x = d.b_x[gi];
  y = d.b_y[gi];
  update_momentum(svc, svx, svy);
  update_pos(x, y, d.b_vx[gi], d.b_vy[gi], svx, svy, svc, (double)d.size, (double)d.size);
  d.b_svc[gi] = svc;
  d.b_svx[gi] = svx;
  d.b_svy[gi] = svy;
  d.b_x[gi] = x;
  d.b_y[gi] = y;
  return true;
}
// The blob grid (coarse, 2^cshift fine buckets per side) is built in two steps:
// each blob takes its rank in a per-arena count array (cgrid_counts row 1) where its
// position is final -- k_players' blob blocks (updateBlobs) and the ejecting
// player's thread -- and an extra block per arena of the merge launch scans the
// counts (re-zeroing them) and places the items (blob_grid_place).
__device__ __forceinline__ int blob_cell(const Dev &d, double x, double y) {
  const int s = d.cshift, cc = (d.cols + (1 << s) - 1) >> s;
  return (center_bucket_coord(y, d.cols) >> s) * cc + (center_bucket_coord(x, d.cols) >> s);
}
__device__ __forceinline__ int *cgrid_counts(const Dev &d, int a, int row);
__device__ __forceinline__ void blob_count(const Dev &d, int a, size_t g, double x, double y) {
  const int b = blob_cell(d, x, y);
  d.b_rank[g] = (b << 12) | atomicAdd(&cgrid_counts(d, a, 1)[b], 1);  // rank < 4096 (else ERR_SLOT)
}

// ------------------------------------------------------------ T4 players
// Player.decayMass + updateCellProperties for one cell (player.py:39-44,
// cell.py:105-130,47-57): independent per cell, so one thread per pool slot --
// the correctly rounded pow of the move speed no longer chains per player
// rp.on: the synthetic population's policy is evaluated here (every cell of a
// player computes the same command; slot 0 stores it for k_players), which
// saves the policy launch of aigar_run's step
// What update_player will create (k_players' look-back scan publishes it before
// the player chains run): Cell.split makes a cell of every cell heavier than 36
// after decay, the heaviest first, while the player has fewer than 16 cells
// (player.py:46-52), and Player.eject then ejects from every cell of at least 35
// (player.py:54-58; a split cell weighs half, m / 2 exactly).  Every live cell of
// at least 35 after decay adds its class to its player's word p_heavy (update_cell,
// one atomic per heavy cell): bits 0-7 cells > 36, 8-15 cells >= 70 (both halves
// eject), 16-23 cells in [35, 36].  Ties split in list order, but tied cells weigh
// the same, so the counts do not depend on which.  k_players reads and clears the
// word and checks the chain's own counts against it (ERR_PREDICT).
__device__ __forceinline__ void predicted_counts(int heavy, int n0, bool split, bool eject, int &nsplit, int &nb) {
  const int c36 = heavy & 0xFF, c70 = (heavy >> 8) & 0xFF, c35 = (heavy >> 16) & 0xFF;
  nsplit = split ? min(c36, kMaxCells - n0) : 0;
  nb = eject ? 2 * min(nsplit, c70) + (c36 - nsplit) + c35 : 0;
}
// one live cell ci of a live player (k_players' cell phase), the player's command given;
// heavy: the player's predicted-count word in LDS
// every load of a cell up front, before any store: one memory round trip, not
// one per store the compiler cannot prove disjoint (and a thread's two cells
// load together)
struct CellIn {
  double m, r, svx, svy, mt, x, y;
  int svc;
};
__device__ __forceinline__ CellIn load_cell(const Dev &d, size_t ci) {
  return CellIn{d.c_m[ci], d.c_r[ci], d.c_svx[ci], d.c_svy[ci], d.c_mt[ci], d.c_x[ci], d.c_y[ci], d.c_svc[ci]};
}
__device__ __forceinline__ void update_cell(const Dev &d, size_t ci, const CellIn &in, double cmdx, double cmdy,
                                            bool split, int *heavy) {
  double m = in.m, r = in.r, svx = in.svx, svy = in.svy;
  const double mt = in.mt, x = in.x, y = in.y;
  int svc = in.svc;
  if (m >= 4) {  // Cell.decayMass (cell.py:123-126)
    m = m * kDecay;
    r = radius_of(m);
    d.c_m[ci] = m;
    d.c_r[ci] = r;
  }
  if (m >= 35)  // k_players' predicted counts (predicted_counts)
    atomicAdd(heavy, (m > 36 ? 1 : 0) | (m >= 70 ? 1 << 8 : 0) | (m > 36 ? 0 : 1 << 16));
  update_momentum(svc, svx, svy);
  d.c_svc[ci] = svc;
  d.c_svx[ci] = svx;
  d.c_svy[ci] = svy;
  if (mt > 0) d.c_mt[ci] = mt - 1;
  double vx, vy, ca, sa;
  set_move_direction(x, y, m, r, cmdx, cmdy, vx, vy, ca, sa);
  d.c_vx[ci] = vx;
  d.c_vy[ci] = vy;
  if (split && m > 36) {  // Cell.split's geometry (cell.py:72-85), for update_player's split
    const double W = (double)d.size, nr = radius_of(m / 2);
    const double xp = ca * nr * 4.5 + x, yp = sa * nr * 4.5 + y;
    double svx2, svy2;
    int svc2;
    add_momentum(x, y, xp, yp, W, W, r, svx2, svy2, svc2);
    d.sp_r[ci] = nr;
    d.sp_svx[ci] = svx2;
    d.sp_svy[ci] = svy2;
  }
}

// adjustCellPositions (field.py:161-181) for the pair (a, b), a the bigger
__device__ __forceinline__ void adjust_pair(double &bx, double &by, double bm, double &sx, double &sy, double sm,
                                            double dist, double sr, double W) {
  double ds = (sr - dist) / dist, mds = sm / bm;
  double xd = (bx - sx) * ds, yd = (by - sy) * ds;
  double nbx = bx + xd * mds, nby = by + yd * mds;
  double nsx = sx - xd * (1 - mds), nsy = sy - yd * (1 - mds);
  bx = py_min(W, py_max(0.0, nbx));
  by = py_min(W, py_max(0.0, nby));
  sx = py_min(W, py_max(0.0, nsx));
  sy = py_min(W, py_max(0.0, nsy));
}
// The eject flags, updateCellsMovement, performEjections and
// handlePlayerCollisions of update_player below for a player with n <= N
// cells, on registers: every field of the n cells is loaded in ONE round
// (fully unrolled, constant indices), the phases run in the same order on the
// copies, and only what changed is stored.  The memory version re-loads
// across each phase's stores (one dependent round per phase and cell).
constexpr int kTailRegs = 4;
template <int N>
__device__ __forceinline__ int player_tail_regs(const Dev &d, int gp, const uint8_t *lst, int n, bool eject,
                                                double cpx, double cpy, double W PT_PARAMS) {
  const int NP = d.NP;
  double x[N], y[N], vx[N], vy[N], svx[N], svy[N], m[N], r[N], mt[N];
  int svc[N];
  uint32_t fl[N];
  bool ej[N];
#pragma unroll
  for (int k = 0; k < N; k++) {
    x[k] = y[k] = vx[k] = vy[k] = svx[k] = svy[k] = m[k] = r[k] = mt[k] = 0;
    svc[k] = 0;
    fl[k] = 0;
    if (k < n) {
      const size_t ci = (size_t)lst[k] * NP + gp;
      x[k] = d.c_x[ci];
      y[k] = d.c_y[ci];
      vx[k] = d.c_vx[ci];
      vy[k] = d.c_vy[ci];
      svx[k] = d.c_svx[ci];
      svy[k] = d.c_svy[ci];
      m[k] = d.c_m[ci];
      r[k] = d.c_r[ci];
      mt[k] = d.c_mt[ci];
      svc[k] = d.c_svc[ci];
      fl[k] = d.c_flags[ci];
    }
  }
  PT_MARK(1, 2);
#pragma unroll
  for (int k = 0; k < N; k++) {
    if (eject && k < n && m[k] >= 35) fl[k] |= F_EJECT;  // Player.eject (player.py:54-58)
    ej[k] = k < n && (fl[k] & F_EJECT);
  }
#pragma unroll
  for (int k = 0; k < N; k++)  // updateCellsMovement
    if (k < n) update_pos(x[k], y[k], vx[k], vy[k], svx[k], svy[k], svc[k], W, W);
  int nb = 0;
#pragma unroll
  for (int k = 0; k < N; k++) {  // performEjections (field.py:134-146)
    if (!ej[k]) continue;
    m[k] = m[k] - kEjectMass;  // Cell.eject: radius stays stale (cell.py:90-94)
    double bsvx, bsvy;
    int bsvc;
    add_momentum(x[k], y[k], cpx, cpy, W, W, r[k], bsvx, bsvy, bsvc);
    const size_t si = (size_t)nb * NP + gp;
    d.sb_x[si] = x[k];
    d.sb_y[si] = y[k];
    d.sb_svx[si] = bsvx;
    d.sb_svy[si] = bsvy;
    d.sb_slot[si] = lst[k];
    nb++;
  }
#pragma unroll
  for (int i = 0; i < N; i++) {  // handlePlayerCollisions (field.py:149-159)
    if (i >= n || svc[i] > 0) continue;
#pragma unroll
    for (int j = 0; j < N; j++) {
      if (j >= n || i == j || svc[j] > 0 || (mt[i] <= 0 && mt[j] <= 0)) continue;
      double dist = sqrt((x[i] - x[j]) * (x[i] - x[j]) + (y[i] - y[j]) * (y[i] - y[j]));
      double sr = r[i] + r[j];
      if (dist < sr && dist != 0) {
        if (m[i] > m[j])
          adjust_pair(x[i], y[i], m[i], x[j], y[j], m[j], dist, sr, W);
        else
          adjust_pair(x[j], y[j], m[j], x[i], y[i], m[i], dist, sr, W);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < N; k++) {
    if (k >= n) continue;
    const size_t ci = (size_t)lst[k] * NP + gp;
    d.c_x[ci] = x[k];
    d.c_y[ci] = y[k];
    d.c_svx[ci] = svx[k];
    d.c_svy[ci] = svy[k];
    if (ej[k]) d.c_m[ci] = m[k];
    // the flags as k_players leaves them: updateHashTables inserts every cell, and a
    // new cell stops being new (the seq pass then only numbers the new cells)
    d.c_flags[ci] = (fl[k] & ~(F_EJECT | F_NEW)) | F_INHASH;
  }
  return nb;
}

// the rest of Player.update (split, eject, move) + performEjections +
// handlePlayerCollisions, one thread per player (list order matters)
// The player's fields update_player starts from, loaded by k_players in the
// kernel's first round (beside the predicted counts, before the block scan)
struct PlayerHead {
  uint8_t lst[kTailRegs];  // the list's first rows (the rows past the count exist, unused)
  bool alive, split, eject;
  int n;
  double cpx, cpy;
};
__device__ __forceinline__ PlayerHead player_head(const Dev &d, int gp) {
  PlayerHead h;
#pragma unroll
  for (int k = 0; k < kTailRegs; k++) h.lst[k] = d.p_list[k * d.NP + gp];
  h.alive = d.p_alive[gp] != 0;
  h.n = d.p_ncells[gp];
  h.split = d.p_split[gp] != 0;
  h.eject = d.p_eject[gp] != 0;
  h.cpx = d.p_cmdx[gp];
  h.cpy = d.p_cmdy[gp];
  return h;
}
// nn / nb_out: the new cells and blobs it made (k_players' scans take them from registers)
// fast: the player took the register tail, its flags are final and its list is
// in lst_out (n_out cells; k_players' seq pass then needs no loads)
__device__ __forceinline__ void update_player(const Dev &d, int gp, const PlayerHead &ph, int &nn, int &nb_out,
                                              bool &fast, uint8_t (&lst_out)[kTailRegs], int &n_out PT_PARAMS) {
  const int NP = d.NP;
  // the cell arrays never alias: let the compiler keep values in registers across stores
  double *__restrict__ cx = d.c_x, *__restrict__ cy = d.c_y, *__restrict__ cm = d.c_m, *__restrict__ cr = d.c_r;
  double *__restrict__ cvx = d.c_vx, *__restrict__ cvy = d.c_vy, *__restrict__ csvx = d.c_svx;
  double *__restrict__ csvy = d.c_svy, *__restrict__ cmt = d.c_mt;
  int *__restrict__ csvc = d.c_svc;
  uint32_t *__restrict__ cfl = d.c_flags;
  // the list's first rows are loaded with the player's fields (one round; the
  // rows past the cell count are allocated and simply unused)
  uint8_t lst[kMaxCells];
#pragma unroll
  for (int k = 0; k < kTailRegs; k++) lst[k] = ph.lst[k];
  int n = ph.n;
  nn = nb_out = 0;
  fast = false;
  if (!ph.alive) {  // updateRespawnTime (player.py:74-75)
    d.p_respawn[gp] -= 1;
    return;
  }
  const double W = (double)d.size;
  const double cpx = ph.cpx, cpy = ph.cpy;
  for (int k = kTailRegs; k < n; k++) lst[k] = d.p_list[k * NP + gp];
  PT_MARK(1, 1);
  // (decay, momentum, merge timer and direction already ran per cell: update_cell)
  int n_new = 0;
  if (ph.split) {  // Player.split (player.py:46-52): stable sort by mass desc, split the snapshot
    for (int i = 1; i < n; i++) {
      uint8_t key = lst[i];
      double km = cm[(size_t)key * NP + gp];
      int j = i - 1;
      while (j >= 0 && km > cm[(size_t)lst[j] * NP + gp]) {
        lst[j + 1] = lst[j];
        j--;
      }
      lst[j + 1] = key;
    }
    uint32_t used = 0;
    for (int k = 0; k < n; k++) used |= 1u << lst[k];
    int n0 = n;
    uint8_t snap[kMaxCells];
    for (int k = 0; k < n0; k++) snap[k] = lst[k];
    for (int k = 0; k < n0; k++) {
      size_t ci = (size_t)snap[k] * NP + gp;
      if (!(cm[ci] > 36 && n < kMaxCells)) continue;
      int slot = __ffs(~used) - 1;
      used |= 1u << slot;
      size_t ni = (size_t)slot * NP + gp;
      // Cell.split (cell.py:72-85); its angle, radius and momentum were computed by
      // the cell's own update_cell thread (the same values, bit for bit)
      double x = cx[ci], y = cy[ci];
      double nm = cm[ci] / 2, nr = d.sp_r[ci];
      double svx = d.sp_svx[ci], svy = d.sp_svy[ci];
      int svc = 15;
      cx[ni] = x;
      cy[ni] = y;
      cm[ni] = nm;
      cr[ni] = nr;
      cvx[ni] = 0;
      cvy[ni] = 0;
      csvx[ni] = svx;
      csvy[ni] = svy;
      csvc[ni] = svc;
      cmt[ni] = merge_time_for(1, nm);
      cfl[ni] = F_ALIVE | F_NEW;
      cm[ci] = nm;  // (the parent keeps the other half: the same mass and radius)
      cr[ci] = nr;
      lst[n++] = (uint8_t)slot;
      n_new++;
    }
  }
  if (n <= kTailRegs) {  // the common case: the rest runs on registers, one load round
    const int nb = player_tail_regs<kTailRegs>(d, gp, lst, n, ph.eject, cpx, cpy, W PT_ARGS);
    PT_MARK(1, 3);
    for (int k = 0; k < n; k++) d.p_list[k * NP + gp] = lst[k];
    d.p_ncells[gp] = n;
    nn = n_new;
    nb_out = nb;
    fast = true;
    n_out = n;
#pragma unroll
    for (int k = 0; k < kTailRegs; k++) lst_out[k] = lst[k];
    return;
  }
  if (ph.eject)  // Player.eject (player.py:54-58)
    for (int k = 0; k < n; k++) {
      size_t ci = (size_t)lst[k] * NP + gp;
      if (cm[ci] >= 35) cfl[ci] |= F_EJECT;
    }
  for (int k = 0; k < n; k++) {  // updateCellsMovement
    size_t ci = (size_t)lst[k] * NP + gp;
    double x = cx[ci], y = cy[ci], svx = csvx[ci], svy = csvy[ci];
    update_pos(x, y, cvx[ci], cvy[ci], svx, svy, csvc[ci], W, W);
    cx[ci] = x;
    cy[ci] = y;
    csvx[ci] = svx;
    csvy[ci] = svy;
  }
  int nb = 0;
  for (int k = 0; k < n; k++) {  // performEjections (field.py:134-146)
    size_t ci = (size_t)lst[k] * NP + gp;
    if (!(cfl[ci] & F_EJECT)) continue;
    cm[ci] = cm[ci] - kEjectMass;  // Cell.eject: radius stays stale (cell.py:90-94)
    cfl[ci] &= ~F_EJECT;
    double bx = cx[ci], by = cy[ci], svx, svy;
    int svc;
    add_momentum(bx, by, cpx, cpy, W, W, cr[ci], svx, svy, svc);
    size_t si = (size_t)nb * NP + gp;
    d.sb_x[si] = bx;
    d.sb_y[si] = by;
    d.sb_svx[si] = svx;
    d.sb_svy[si] = svy;
    d.sb_slot[si] = lst[k];
    nb++;
  }
  for (int i = 0; i < n; i++) {  // handlePlayerCollisions (field.py:149-159)
    size_t ci = (size_t)lst[i] * NP + gp;
    if (csvc[ci] > 0) continue;
    for (int j = 0; j < n; j++) {
      size_t cj = (size_t)lst[j] * NP + gp;
      if (i == j || csvc[cj] > 0 || (cmt[ci] <= 0 && cmt[cj] <= 0)) continue;
      double x1 = cx[ci], y1 = cy[ci], x2 = cx[cj], y2 = cy[cj];
      double dist = sqrt((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2));
      double sr = cr[ci] + cr[cj];
      if (dist < sr && dist != 0) {  // adjustCellPositions (field.py:161-181)
        bool one_big = cm[ci] > cm[cj];
        size_t bi = one_big ? ci : cj, si = one_big ? cj : ci;
        double bx = cx[bi], by = cy[bi], sx = cx[si], sy = cy[si];
        double ds = (sr - dist) / dist, mds = cm[si] / cm[bi];
        double xd = (bx - sx) * ds, yd = (by - sy) * ds;
        double nbx = bx + xd * mds, nby = by + yd * mds;
        double nsx = sx - xd * (1 - mds), nsy = sy - yd * (1 - mds);
        cx[bi] = py_min(W, py_max(0.0, nbx));
        cy[bi] = py_min(W, py_max(0.0, nby));
        cx[si] = py_min(W, py_max(0.0, nsx));
        cy[si] = py_min(W, py_max(0.0, nsy));
      }
    }
  }
  for (int k = 0; k < n; k++) d.p_list[k * NP + gp] = lst[k];
  d.p_ncells[gp] = n;
  nn = n_new;
  nb_out = nb;
}

// lane k's double / int, k wave-uniform
__device__ __forceinline__ double lane_d(double v, int k) {
  const int64_t b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, k), hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
  return __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ int lane_i(int v, int k) { return __builtin_amdgcn_readlane(v, k); }

// update_player for a player that has more than kTailRegs cells after its split,
// on one wavefront (k_players' helper waves): lane k holds list row k's cell in
// registers, so the phases run without the memory version's reload per cell and
// pair (a 16-cell player's handlePlayerCollisions was 256 dependent pairs of
// global loads -- ~270 us per crowded Greedy tick, profiles/r06_clustered.txt).
// The same phases in the same order as update_player:
//  * Player.split: the stable sort by mass (descending) as a rank per lane, the
//    snapshot's qualifying cells in sorted order take the lowest free slots;
//  * the eject flags, updateCellsMovement (independent per cell);
//  * performEjections in list order (a ballot prefix numbers the blobs);
//  * handlePlayerCollisions: for each i in list order, the lanes j test the pair
//    (i, j) together and the first hit at or after the last one is adjusted --
//    an adjustment moves only i and j, so the later pairs of the same i need
//    only i's new position: the serial loop's outcome exactly.
// Results: the cells (flags final), the list and count, the blob staging rows;
// the list also into LDS (hl, hn: the seq pass numbers the new cells from it).
// cnt = pn | pb << 8: the predicted counts, checked (ERR_PREDICT).
__device__ void player_wave(const Dev &d, int a, int gp, double cpx, double cpy, bool split, bool eject, int cnt,
                            uint8_t *hl, uint8_t *hn) {
  const int lane = threadIdx.x & 63, NP = d.NP;
  const unsigned long long lt = (1ull << lane) - 1;
  const double W = (double)d.size;
  const int n0 = uni(d.p_ncells[gp]);
  int slot = 0, svc = 0;
  uint32_t fl = 0;
  double x = 0, y = 0, vx = 0, vy = 0, svx = 0, svy = 0, m = 0, r = 0, mt = 0, spr = 0, spsvx = 0, spsvy = 0;
  if (lane < n0) {
    slot = d.p_list[lane * NP + gp];
    const size_t ci = (size_t)slot * NP + gp;
    x = d.c_x[ci];
    y = d.c_y[ci];
    vx = d.c_vx[ci];
    vy = d.c_vy[ci];
    svx = d.c_svx[ci];
    svy = d.c_svy[ci];
    m = d.c_m[ci];
    r = d.c_r[ci];
    mt = d.c_mt[ci];
    svc = d.c_svc[ci];
    fl = d.c_flags[ci];
    if (split) {  // (update_cell's split geometry; read only for the cells that split)
      spr = d.sp_r[ci];
      spsvx = d.sp_svx[ci];
      spsvy = d.sp_svy[ci];
    }
  }
  int n = n0, n_new = 0;
  bool touched = false;  // mass / radius / fresh fields changed (stored below)
  if (split) {  // Player.split (player.py:46-52)
    int rk = 0;
    for (int j = 0; j < n0; j++) {
      const double mj = lane_d(m, j);
      rk += (mj > m || (mj == m && j < lane)) ? 1 : 0;
    }
    int src = lane;
    for (int k = 0; k < n0; k++)
      if (lane_i(rk, k) == lane) src = k;
    slot = __shfl(slot, src);
    x = __shfl(x, src);
    y = __shfl(y, src);
    vx = __shfl(vx, src);
    vy = __shfl(vy, src);
    svx = __shfl(svx, src);
    svy = __shfl(svy, src);
    m = __shfl(m, src);
    r = __shfl(r, src);
    mt = __shfl(mt, src);
    svc = __shfl(svc, src);
    fl = (uint32_t)__shfl((int)fl, src);
    spr = __shfl(spr, src);
    spsvx = __shfl(spsvx, src);
    spsvy = __shfl(spsvy, src);
    uint32_t used = 0;
    for (int j = 0; j < n0; j++) used |= 1u << lane_i(slot, j);
    const unsigned long long qb = __ballot(lane < n0 && m > 36);
    n_new = min(__popcll(qb), kMaxCells - n0);
    // new cell t (lane n0 + t): the t-th qualifying cell's other half, the t-th free slot
    int par = lane;
    uint32_t u = used;
    for (int t = 0; t < n_new; t++) {
      const int s = __ffs(~u) - 1;
      u |= 1u << s;
      if (lane == n0 + t) slot = s;
    }
    for (int k = 0; k < n0; k++) {
      if (!((qb >> k) & 1)) continue;
      const int t = __popcll(qb & ((1ull << k) - 1));
      if (t < n_new && lane == n0 + t) par = k;
    }
    const double px = __shfl(x, par), py = __shfl(y, par), pm = __shfl(m, par);
    const double pr = __shfl(spr, par), psx = __shfl(spsvx, par), psy = __shfl(spsvy, par);
    const bool is_par = ((qb >> lane) & 1) && __popcll(qb & lt) < n_new;
    const bool is_new = lane >= n0 && lane < n0 + n_new;
    if (is_par) {  // Cell.split: the parent keeps the other half (same mass and radius)
      m = m / 2;
      r = spr;
    }
    if (is_new) {
      x = px;
      y = py;
      m = pm / 2;
      r = pr;
      vx = vy = 0;
      svx = psx;
      svy = psy;
      svc = 15;
      mt = merge_time_for(1, m);
      fl = F_ALIVE | F_NEW;
    }
    touched = is_par || is_new;
    n = n0 + n_new;
  }
  const bool fresh = lane >= n0 && lane < n;
  if (eject && lane < n && m >= 35) fl |= F_EJECT;  // Player.eject (player.py:54-58)
  const bool ej = lane < n && (fl & F_EJECT);
  if (lane < n) update_pos(x, y, vx, vy, svx, svy, svc, W, W);  // updateCellsMovement
  const unsigned long long eb = __ballot(ej);  // performEjections (field.py:134-146), list order
  if (ej) {
    m = m - kEjectMass;  // Cell.eject: radius stays stale (cell.py:90-94)
    double bsvx, bsvy;
    int bsvc;
    add_momentum(x, y, cpx, cpy, W, W, r, bsvx, bsvy, bsvc);
    const size_t si = (size_t)__popcll(eb & lt) * NP + gp;
    d.sb_x[si] = x;
    d.sb_y[si] = y;
    d.sb_svx[si] = bsvx;
    d.sb_svy[si] = bsvy;
    d.sb_slot[si] = (uint8_t)slot;
  }
  const int nb = __popcll(eb);
  for (int i = 0; i < n; i++) {  // handlePlayerCollisions (field.py:149-159)
    if (lane_i(svc, i) > 0) continue;
    const double mti = lane_d(mt, i), mi = lane_d(m, i), ri = lane_d(r, i);
    const bool cand = lane < n && lane != i && svc <= 0 && !(mti <= 0 && mt <= 0);
    int j0 = 0;
    for (;;) {
      const double xi = lane_d(x, i), yi = lane_d(y, i);
      double dist = 0, sr = 0;
      bool hit = false;
      if (cand && lane >= j0) {
        dist = sqrt((xi - x) * (xi - x) + (yi - y) * (yi - y));
        sr = ri + r;
        hit = dist < sr && dist != 0;
      }
      const unsigned long long hb = __ballot(hit);
      if (!hb) break;
      const int j = __ffsll((long long)hb) - 1;
      double bx = xi, by = yi, sx = lane_d(x, j), sy = lane_d(y, j);
      const double mj = lane_d(m, j), dj = lane_d(dist, j), sj = lane_d(sr, j);
      if (mi > mj) {  // adjustCellPositions (field.py:161-181), the bigger first
        adjust_pair(bx, by, mi, sx, sy, mj, dj, sj, W);
      } else {
        adjust_pair(sx, sy, mj, bx, by, mi, dj, sj, W);
      }
      if (lane == i) {
        x = bx;
        y = by;
      }
      if (lane == j) {
        x = sx;
        y = sy;
      }
      j0 = j + 1;
    }
  }
  if (lane < n) {
    const size_t ci = (size_t)slot * NP + gp;
    d.c_x[ci] = x;
    d.c_y[ci] = y;
    d.c_svx[ci] = svx;
    d.c_svy[ci] = svy;
    if (ej || touched) d.c_m[ci] = m;
    if (touched) d.c_r[ci] = r;
    if (fresh) {
      d.c_vx[ci] = 0;
      d.c_vy[ci] = 0;
      d.c_svc[ci] = svc;
      d.c_mt[ci] = mt;
    }
    // the flags as k_players leaves them (player_tail_regs)
    d.c_flags[ci] = (fl & ~(F_EJECT | F_NEW)) | F_INHASH;
    d.p_list[lane * NP + gp] = (uint8_t)slot;
    hl[lane] = (uint8_t)slot;
  }
  if (lane == 0) {
    d.p_ncells[gp] = n;
    *hn = (uint8_t)n;
    if (n_new != (cnt & 0xFF) || nb != (cnt >> 8)) set_err(d, a, ERR_PREDICT);
  }
}

// updateViruses + updateBlobs + the per-cell part of updatePlayers in one
// launch: thread ranges [cell slots | viruses | blobs] (independent, field.py:94-119)
// the first kSpawnAhead pellet spawns of this tick, drawn now: their counter
// (ctr_pellet) is fixed before spawnStuff counts them, and a 64-bit Philox on the
// closing update's path would cost more than all its loads
constexpr int kSpawnAhead = 64;
__device__ void spawn_ahead(const Dev &d, int a, int j) {
  const ArenaCtl &c = d.ctl[a];
  uint64_t u[4];
  philox(c.ctr_pellet + j, ST_PELLET, 0, 0, c.key0, c.key1, u);
  const int64_t sr = (int64_t)mulhi(u[2], 50);
  const size_t o = (size_t)a * kSpawnAhead + j;
  d.spec_x[o] = (double)(int64_t)mulhi(u[0], (uint64_t)d.size);
  d.spec_y[o] = (double)(int64_t)mulhi(u[1], (uint64_t)d.size);
  d.spec_m[o] = (sr > 50 - 4) ? (double)(50 - sr) : 1.0;  // randomSize (field.py:20-26)
}
// per-tick resets, by k_players' arena block (in the cell threads their loads
// delayed every cell's first round): the spawn
// occupancy restarts (k_pp_active rebuilds it; its last reader was the previous
// tick's spawns); the dead flags of the last closing update's blob conversions
// (that update's blocks read them while building their lists, so none of them
// may clear one) are cleared
// (arena a; part k of nk: the occupancy is one bucket count per fine bucket --
// 320k at C3, ~14 us for one block's stores -- so every extra block of the
// arena zeroes a slice of it)
__device__ void tick_zero(const Dev &d, int a, int k, int nk) {
  const int T = blockDim.x;
  const int h0 = (int)((long)d.H * k / nk), h1 = (int)((long)d.H * (k + 1) / nk);
  for (int i = h0 + threadIdx.x; i < h1; i += T) d.occ_cnt[(size_t)a * d.H + i] = 0;
  const int w0 = (int)((long)d.occ_words * k / nk), w1 = (int)((long)d.occ_words * (k + 1) / nk);
  for (int i = w0 + threadIdx.x; i < w1; i += T) d.occ[(size_t)a * d.occ_words + i] = 0;
  if (k == 0) {
    const int nconv = d.ctl[a].pu_nconv;
    for (int j = threadIdx.x; j < nconv; j += T) d.pel_dead[(size_t)a * d.PD + d.PS + j] = 0;
  }
}
// C4: the tick's first pass opens with the observation hand-off plan: extra
// threads of k_players' arena block, one per player.  A bot's history is current on
// t_holder (-1: on every tile), or on the tile that observed it since the last
// plan (t_obsby) -- that update is replicated, every tile makes it.  The holder
// hands the history off when the bot is dead (it respawns anywhere at the end of
// this tick) or its view centre (the FOV cache, end of the last tick) lies in
// another tile, in a slot of its first-pass message; every other tile drops the
// holder for the slots it receives (k_tile_apply), so the holders stay identical
// on every tile.  Dead bots come first: they take slots here (more than hcap in
// one tick is ERR_TILE_HANDOFF, never a silent deferral -- the stale holder could
// not observe a bot respawned outside its pellets).  Live bots only queue here
// (t_holive, room for every player); tile_plan_live, in the message's last block,
// gives them the slots the dead left, and the rest keep their holder a tick
// longer: their centre moved at most one tick's distance from the tile, which the
// halo covers, and they go first at the next plan (t_hodefer), so none waits long.
__device__ void tile_plan_thread(const Dev &d, int gp) {
  ArenaCtl &c = d.ctl[0];
  if (gp == 0) {  // the first pass's counters
    c.n_out = c.n_out_pel = c.n_undone = 0;
    c.n_eaten_glob = 0;
  }
  if (gp >= d.NP) return;
  int h = d.t_holder[gp];
  const int ob = d.t_obsby[gp];
  if (ob >= 0) {
    h = ob;
    d.t_obsby[gp] = -1;
    d.t_holder[gp] = h;
  }
  // (a bot that does not queue for a live hand-off keeps no waiting priority)
  if (h != d.tile_id || !d.p_alive[gp] || tile_of(d, d.p_fx[gp], d.p_fy[gp]) == h) {
    if (d.t_hodefer[gp]) d.t_hodefer[gp] = 0;
    if (h != d.tile_id || d.p_alive[gp]) return;
  } else {
    const int q = atomicAdd(&c.n_ho_live, 1);
    if (q < d.NP) d.t_holive[q] = gp;
    return;
  }
  const int sl = atomicAdd(&c.n_ho, 1);
  if (sl >= d.hcap) {
    set_err(d, 0, ERR_TILE_HANDOFF);
    return;
  }
  d.t_holder[gp] = -1;
  d.t_hoslot[sl] = gp;  // (its history is copied into the slot by tile_plan_live, block-parallel)
}
// The first pass's hand-off slots, in the message's last block: the live bots
// take the slots the dead left -- every queued bot is ranked, the ones that
// waited at an earlier plan first, then by player index (the choice does not
// depend on atomic order, and a bot passed over goes first next tick) -- then
// the whole block copies every slot's history -- [TR_HIST record: player,
// lastFovSize][nh grids] -- element by element (a thread per bot copying its
// ~250 doubles serially took ~4 us)
constexpr int kHoLds = 2048;  // queued live bots ranked in LDS (more: ranked from global memory)
__device__ void tile_plan_live(const Dev &d) {
  ArenaCtl &c = d.ctl[0];
  __shared__ int s_q[kHoLds];
  const int nd = min(c.n_ho, d.hcap), nq = min(c.n_ho_live, d.NP), room = d.hcap - nd;
  // key: (did not wait before) << 30 | player
  auto key_of = [&](int gp) { return (d.t_hodefer[gp] ? 0 : 1 << 30) | gp; };
  const bool lds = nq <= kHoLds;
  for (int i = threadIdx.x; i < nq; i += blockDim.x) {  // (the keys first: the ranking below updates t_hodefer)
    const int k = key_of(d.t_holive[i]);
    if (lds) s_q[i] = k;
    else d.t_holive[i] = k;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nq; i += blockDim.x) {
    const int k = lds ? s_q[i] : d.t_holive[i], gp = k & ((1 << 30) - 1);
    int r = 0;
    for (int j = 0; j < nq; j++) r += (lds ? s_q[j] : d.t_holive[j]) < k;
    if (r < room) {
      d.t_holder[gp] = -1;
      d.t_hoslot[nd + r] = gp;
      d.t_hodefer[gp] = 0;
    } else {
      d.t_hodefer[gp] = (uint8_t)min(255, d.t_hodefer[gp] + 1);
    }
  }
  __syncthreads();
  const int ns = nd + min(nq, room), GG = d.G * d.G, per = 1 + d.nh * GG;
  for (int e = threadIdx.x; e < ns * per; e += blockDim.x) {
    const int sl = e / per, j = e - sl * per, gp = d.t_hoslot[sl];
    TileRec *slot = d.outbox + 1 + d.tcap + (size_t)sl * d.hrec;
    if (j == 0) {
      slot->kind = TR_HIST;
      slot->idx = gp;
      slot->seq = 0;
      slot->x = d.o_lastfov[gp];
      slot->y = 0;
    } else {
      const int q = j - 1, g = q / GG, t = q - g * GG;
      ((double *)(slot + 1))[q] = hist_grid(d, g)[(size_t)gp * GG + t];
    }
  }
  if (threadIdx.x == 0) c.n_ho = ns;
}
// rank of this thread among the flagged threads of the block (thread order);
// *total = number flagged.  Ballot per wave + one pass over <= 16 wave counts.
__device__ __forceinline__ int block_rank(bool flag, int *sh, int *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  unsigned long long b = __ballot(flag);
  int before = __popcll(b & ((1ull << lane) - 1));
  if (lane == 0) sh[w] = __popcll(b);
  __syncthreads();
  int off = 0, tot = 0;
  for (int k = 0; k < nw; k++) {
    int v = sh[k];
    off += k < w ? v : 0;
    tot += v;
  }
  __syncthreads();
  *total = tot;
  return off + before;
}

// block-wide exclusive scan of in[0..n) into out (may alias; any multiple of 64
// threads up to 1024; sh >= 17 ints); each thread scans a consecutive chunk,
// per-thread sums go through a shuffle scan per wave and one across waves.
// Returns the total.
__device__ int block_scan_excl(const int *in, int *out, int n, int *sh) {
  const int T = blockDim.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = T >> 6;
  int per = (n + T - 1) / T, lo = min(n, tid * per), hi = min(n, lo + per);
  int s = 0;
  for (int i = lo; i < hi; i++) s += in[i];
  int inc = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  if (w == 0) {
    int v = lane < nw ? sh[lane] : 0, vi = v;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      int y = __shfl_up(vi, off);
      if (lane >= off) vi += y;
    }
    if (lane < nw) sh[lane] = vi - v;
    if (lane == nw - 1) sh[16] = vi;
  }
  __syncthreads();
  int run = sh[w] + inc - s;
  const int total = sh[16];
  for (int i = lo; i < hi; i++) {
    int v = in[i];
    out[i] = run;
    run += v;
  }
  __syncthreads();
  return total;
}

// updatePlayers' per-player part + the creation-sequence numbering + the blob
// append, in ONE launch.  Grid (tiles, arenas) of 256 players; each tile scans
// its (new cells + new blobs, new blobs) counts, then a decoupled look-back
// over the arena's tiles (one 64-bit word per tile: status 2 | epoch 14 |
// seq 24 | blobs 24) gives every player its offsets, and the player assigns its
// new cells' seqs and writes its blobs right away (field.py:112-146,121-132).
// The bases (seq_next, n_blob) are read by every tile before it publishes; the
// last tile, whose look-back proves all tiles have published, advances them.
constexpr unsigned long long PL_AGG = 1ull << 62, PL_INC = 2ull << 62;
__device__ __forceinline__ unsigned long long pl_word(unsigned long long st, uint32_t ep, uint32_t vs, uint32_t vb) {
  return st | ((unsigned long long)(ep & 0x3FFFu) << 48) | ((unsigned long long)(vs & 0xFFFFFFu) << 24) |
         (unsigned long long)(vb & 0xFFFFFFu);
}
// The tick opens here too (round 5: the per-cell part of updatePlayers was a
// launch of its own, k_tick_begin, one thread per pool slot over the whole GPU):
// a player tile's cells depend only on their own players' commands, so the
// block updates them itself before its player chains -- its 256 player threads
// take the commands (the synthetic policy, rp.on) and queue their live cells in
// LDS, all 512 threads then run the queue (decay, momentum, merge timer, move
// direction with its correctly rounded pow / atan2 / sincos: one chain per cell,
// a few hundred cells per tile), and the predicted counts collect in LDS.
// The arena's extra blocks: the first (tile == ntiles) runs updateViruses
// (field.py:94-100), the pellet spawns drawn ahead and the virus grid; the rest
// updateBlobs (field.py:102-110), one blob slot per thread, and the per-tick
// resets.  updateHashTables for viruses and blobs rides along: the virus grid
// in the arena block, the blob grid's counts where each blob's position is final
// (blob_count: the blob blocks, the ejecting players), its placement in the
// merge launch (blob_grid_place).
constexpr int kPlT = 512;  // threads per k_players block: 256 player threads + 256 cell helpers
__global__ void __launch_bounds__(512) k_players(Dev d, RandomPolicy rp) {
  FLOOR(1);
  __shared__ int ws[4], wb[4];
  __shared__ int s_ps, s_pb, s_ts, s_tb, s_blob0;
  __shared__ int64_t s_seq0;
  __shared__ uint32_t s_epoch;
  __shared__ int g_cnt[SG_CAP + 1], g_sh[32];  // (the small grids' counting sort)
  __shared__ int s_nq, s_heavy[256];
  __shared__ double s_cx[256], s_cy[256];
  __shared__ uint8_t s_csp[256];
  __shared__ uint16_t s_q[256 * (kMaxCells - 1)];  // the tile's queued cells: local player << 4 | slot
  // players of more than kTailRegs cells after the split: queued for the helper
  // waves (player_wave); entry = local player | predicted counts << 8
  __shared__ int s_nh, s_hq[256];
  __shared__ uint8_t s_cej[256], s_hn[256], s_hl[256][kMaxCells];
  PT_BEGIN(1);
#ifdef AIGAR_PHASE_TIMING  // (the cell phase and the extra blocks mark under slot 2)
  if ((threadIdx.x & 63) == 0 && pt_w_ < kPtWaves) g_ptw[2][pt_w_][0] = (unsigned)pt0_;
#endif
  const int tile = blockIdx.x, a = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ntiles = d.pl_tiles, NP = d.NP;
  ArenaCtl &c = d.ctl[a];
  // every block of the arena draws a ticket; the last one bumps the look-back
  // epoch and sets the blob count
  auto finish = [&]() __attribute__((always_inline)) {
    // (the last block reads only the two blob words, stored atomically below)
    if (last_block_relaxed(&c.pl_ticket, (int)gridDim.x) && tid == 0) {
      __hip_atomic_fetch_add(&c.pl_epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // the blob count moves only now: the blob blocks bound their slots by it
      const int nb = __hip_atomic_load(&c.n_blob_base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
                     __hip_atomic_load(&c.n_blob_add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (nb > d.Ecap) set_err(d, a, ERR_BLOB_CAP);
      c.n_blob = min(nb, d.Ecap);
    }
  };
  if (tile > ntiles) {  // updateBlobs: one blob slot per thread (a loop over the pool
    // in one block was the kernel's longest chain, ~15 us at C3), + the resets
    const int k = tile - ntiles - 1, i = k * kPlT + tid;
    if (i < c.n_blob) {  // (the count at the tick's start: it moves in the last block)
      const size_t g = (size_t)a * d.Ecap + i;
      double x, y;
      if (update_blob(d, (int)g, x, y)) blob_count(d, a, g, x, y);
      else d.b_rank[g] = -1;
    }
    tick_zero(d, a, k, gridDim.x - ntiles - 1);
    PT_MARK(2, 4);
    finish();
    return;
  }
  if (tile == ntiles) {  // the arena block
    if (d.virus_enabled)
      for (int i = tid; i < d.Vcap; i += kPlT) update_virus(d, a * d.Vcap + i);
    for (int j = tid; j < kSpawnAhead; j += kPlT) spawn_ahead(d, a, j);
    __syncthreads();  // (the virus updates -> the virus grid, in this block)
    if (d.virus_enabled) grid_small_build<2>(d, a, g_cnt, g_sh);  // (+ its radius bound and lightest mass)
    PT_MARK(2, 3);
    finish();
    return;
  }
  unsigned long long *st = d.pl_state + (size_t)a * ntiles;
  // ---- the cell phase (Player.decayMass + updateCellProperties, player.py:39-44)
  const int p = tile * 256 + (tid & 255), gp = a * d.B + p;
  PlayerHead ph{};
  // a player's first cell is updated by its own thread, its record loaded beside
  // the command's inputs; the other cells (multi-cell players) queue in LDS for
  // the block's other threads
  CellIn own{};
  size_t own_ci = 0;
  bool own_ok = false;
  if (tid == 0) s_nq = s_nh = 0;
  if (tid < 256) s_heavy[tid] = 0;
  __syncthreads();
  if (tid < 256 && p < d.B) {
    ph = player_head(d, gp);  // (update_player's first round)
    if (d.tiled) tile_plan_thread(d, gp);  // C4: the observation hand-off plan
    if (ph.alive) {
      own_ok = ph.n > 0;
      if (own_ok) {
        own_ci = (size_t)ph.lst[0] * NP + gp;
        own = load_cell(d, own_ci);
      }
      if (rp.on) {  // the synthetic population's move (makeMove; dead players keep their command)
        const Command cm = random_command(d, gp, rp);
        d.p_cmdx[gp] = ph.cpx = cm.x;
        d.p_cmdy[gp] = ph.cpy = cm.y;
        d.p_split[gp] = cm.split;
        d.p_eject[gp] = cm.eject;
        ph.split = cm.split != 0;
        ph.eject = cm.eject != 0;
      }
      s_cx[tid] = ph.cpx;
      s_cy[tid] = ph.cpy;
      s_csp[tid] = ph.split ? 1 : 0;
      s_cej[tid] = ph.eject ? 1 : 0;
      if (ph.n > 1) {
        const int q = atomicAdd(&s_nq, ph.n - 1);
        for (int k = 1; k < ph.n; k++)
          s_q[q + k - 1] = (uint16_t)((tid << 4) | (k < kTailRegs ? ph.lst[k] : d.p_list[k * NP + gp]));
      }
    }
  }
  __syncthreads();
  PT_MARK(2, 1);
  if (own_ok) update_cell(d, own_ci, own, ph.cpx, ph.cpy, ph.split, &s_heavy[tid]);
  {  // the queued cells: the helper threads take the first 256, the player threads the rest
    const int nq = s_nq, pb = a * d.B + tile * 256;
    for (int i = tid >= 256 ? tid - 256 : tid + 256; i < nq; i += kPlT) {
      const int e = s_q[i], lp = e >> 4;
      update_cell(d, (size_t)(e & 15) * NP + (pb + lp), load_cell(d, (size_t)(e & 15) * NP + (pb + lp)), s_cx[lp],
                  s_cy[lp], s_csp[lp] != 0, &s_heavy[lp]);
    }
  }
  __syncthreads();
  PT_MARK(2, 2);
  if (tid >= 256) {  // (the helpers join the player part's three barriers and the last-block ticket)
    __syncthreads();
    __syncthreads();
    // the queued many-cell players, one per helper wave, beside the player
    // threads' chains and look-back (their results are read after the third barrier)
    for (int h = (tid - 256) >> 6; h < s_nh; h += (kPlT - 256) / 64) {
      const int e = s_hq[h], lp = e & 0xFF;
      player_wave(d, a, a * d.B + tile * 256 + lp, s_cx[lp], s_cy[lp], s_csp[lp] != 0, s_cej[lp] != 0, e >> 8,
                  s_hl[h], &s_hn[h]);
    }
    __syncthreads();
    finish();
    return;
  }
  if (tid == 0) {
    s_epoch = __hip_atomic_load(&c.pl_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_seq0 = c.seq_next;
    s_blob0 = c.n_blob;
    if (tile == 0) {
      c.rmax_cell = 0;  // the cell grid's radius bound restarts (re-maxed by its build)
      c.n_kill = 0;     // this tick's pellet kills (read by the last tick's closing update, done by now)
    }
  }
  // the new cells / blobs each player will create, predicted by the cell phase
  // (predicted_counts): the block scan and the tile's aggregate for the
  // look-back are published before the player chains run, so the look-back after
  // them finds every predecessor's aggregate instead of waiting for the slowest tile
  int pn = 0, pb = 0;
  if (p < d.B && ph.alive) predicted_counts(s_heavy[tid], ph.n, ph.split, ph.eject, pn, pb);
  int hslot = -1;  // (queued for a helper wave: its list in s_hl[hslot])
  if (p < d.B && ph.alive && ph.n + pn > kTailRegs) {
    hslot = atomicAdd(&s_nh, 1);
    s_hq[hslot] = tid | pn << 8 | pb << 16;
  }
  const int vs = pn + pb, vb = pb;
  int is = vs, ib = vb;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int y1 = __shfl_up(is, off), y2 = __shfl_up(ib, off);
    if (lane >= off) {
      is += y1;
      ib += y2;
    }
  }
  if (lane == 63) {
    ws[w] = is;
    wb[w] = ib;
  }
  __syncthreads();
  if (tid == 0) {
    int ts = 0, tb = 0;
    for (int k = 0; k < 4; k++) {
      int x1 = ws[k], x2 = wb[k];
      ws[k] = ts;
      wb[k] = tb;
      ts += x1;
      tb += x2;
    }
    s_ts = ts;
    s_tb = tb;
  }
  __syncthreads();
  const uint32_t ep = s_epoch;
  if (w == 0 && lane == 0) {
    const uint32_t ts = s_ts, tb = s_tb;
    if (tile == 0) {
      __hip_atomic_store(&st[0], pl_word(PL_INC, ep, ts, tb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_ps = s_pb = 0;
    } else {
      __hip_atomic_store(&st[tile], pl_word(PL_AGG, ep, ts, tb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  int nn = 0, nb = 0, fn = 0;
  bool fast = false;
  uint8_t flst[kTailRegs];
  if (hslot >= 0) {  // (player_wave checks its counts)
    nn = pn;
    nb = pb;
  } else if (p < d.B) {
    update_player(d, gp, ph, nn, nb, fast, flst, fn PT_ARGS);  // (its counts from registers, not re-loaded)
    if (nn != pn || nb != pb) set_err(d, a, ERR_PREDICT);
  }
  PT_MARK(1, 4);
  if (w == 0) {
    const uint32_t ts = s_ts, tb = s_tb;
    if (tile != 0) {
      int run_s = 0, run_b = 0, hi = tile - 1;
      for (;;) {
        int t = hi - lane;
        unsigned long long word = 0;
        bool ready = true;
        if (t >= 0) {
          word = __hip_atomic_load(&st[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ready = (word >> 62) != 0 && (uint32_t)((word >> 48) & 0x3FFFu) == (ep & 0x3FFFu);
        }
        if (!__all(ready)) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        unsigned long long incmask = __ballot(t >= 0 && (word >> 62) == 2);
        int stop = incmask ? __ffsll((long long)incmask) - 1 : 64;
        bool take = t >= 0 && lane <= stop;
        int v1 = take ? (int)((word >> 24) & 0xFFFFFFu) : 0, v2 = take ? (int)(word & 0xFFFFFFu) : 0;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          v1 += __shfl_xor(v1, off);
          v2 += __shfl_xor(v2, off);
        }
        run_s += v1;
        run_b += v2;
        if (incmask || hi - 63 < 0) break;
        hi -= 64;
      }
      if (lane == 0) {
        __hip_atomic_store(&st[tile], pl_word(PL_INC, ep, run_s + ts, run_b + tb), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        s_ps = run_s;
        s_pb = run_b;
      }
    }
  }
  __syncthreads();
  PT_MARK(1, 5);
  const int64_t seq0 = s_seq0;
  const int blob0 = s_blob0;
  if (tile == ntiles - 1 && tid == 0) {  // arena totals are known: advance the bases
    const int tot = s_ps + s_ts, totb = s_pb + s_tb;
    c.seq_base_upd = seq0;
    c.seq_next = seq0 + tot;
    __hip_atomic_store(&c.n_blob_base, blob0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&c.n_blob_add, totb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (n_blob moves in the last block)
  }
  // the seq pass: a register-tail player's flags are final already and its list
  // is in flst (fn cells): only its new cells (the last nn) are numbered here
  if (p < d.B && (fast || hslot >= 0 ? nb > 0 || nn > 0 : d.p_alive[gp] != 0)) {
    const int64_t s0 = seq0 + s_ps + ws[w] + (is - vs);
    const int boff = s_pb + wb[w] + (ib - vb);
    if (hslot >= 0) {  // (player_wave: flags final, the list in LDS)
      const int n = s_hn[hslot];
      for (int k = n - nn; k < n; k++) d.c_seq[(size_t)s_hl[hslot][k] * NP + gp] = s0 + (k - (n - nn));
    } else if (fast) {
#pragma unroll
      for (int k = 0; k < kTailRegs; k++)
        if (k >= fn - nn && k < fn) d.c_seq[(size_t)flst[k] * NP + gp] = s0 + (k - (fn - nn));
    } else {
      const int n = d.p_ncells[gp];
      for (int k = 0; k < n; k++) {
        size_t ci = (size_t)d.p_list[k * NP + gp] * NP + gp;
        if (k >= n - nn) d.c_seq[ci] = s0 + (k - (n - nn));
        d.c_flags[ci] = (d.c_flags[ci] & ~F_NEW) | F_INHASH;  // updateHashTables inserts every cell
      }
    }
    for (int j = 0; j < nb; j++) {
      int bi = blob0 + boff + j;
      if (bi >= d.Ecap) break;  // ERR_BLOB_CAP set in the last block
      size_t g = (size_t)a * d.Ecap + bi, si = (size_t)j * NP + gp;
      const double bm = kEjectMass * 0.8, bx = d.sb_x[si], by = d.sb_y[si];
      d.b_x[g] = bx;
      d.b_y[g] = by;
      d.b_m[g] = bm;
      d.b_r[g] = radius_of(bm);
      d.b_vx[g] = 0;
      d.b_vy[g] = 0;
      d.b_svx[g] = d.sb_svx[si];
      d.b_svy[g] = d.sb_svy[si];
      d.b_svc[g] = 15;
      d.b_seq[g] = s0 + nn + j;
      d.b_ej[g] = d.c_seq[(size_t)d.sb_slot[si] * NP + gp];
      d.b_col[g] = p;
      d.b_flags[g] = F_ALIVE;
      blob_count(d, a, g, bx, by);
    }
  }
  PT_MARK(1, 6);
  finish();
}

// ------------------------------------------------------------ grids

// block-wide exclusive scan of one int per thread (1024 threads); returns the
// exclusive prefix and writes the block total to *total (shared)
__device__ __forceinline__ int block_excl_1024(int x, int *wsum, int *total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  int inc = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  if (w == 0) {
    int v = lane < nw ? wsum[lane] : 0, vi = v;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      int y = __shfl_up(vi, off);
      if (lane >= off) vi += y;
    }
    if (lane < nw) wsum[lane] = vi - v;  // exclusive wave offsets
    if (lane == nw - 1) *total = vi;
  }
  __syncthreads();
  return inc - x + wsum[w];
}


// Grids of the small entity sets (blobs, viruses): one block per arena (any
// multiple of 64 threads) runs the whole counting sort in LDS on a grid
// coarsened by 2^cshift (<= SG_CAP cells, chosen at create): LDS-atomic ranks,
// block scan, coalesced start[] store, scatter.  The virus grid also sets the
// radius bound and the lightest mass (the block is their only writer then).
template <int KIND>
__device__ __forceinline__ void grid_small_build(const Dev &d, int a, int *cnt, int *sh) {
  __shared__ double vmin_w[32];  // per wave (<= 16): lightest mass, then largest radius
  const int tid = threadIdx.x, T = blockDim.x, s = d.cshift;
  const int cc = (d.cols + (1 << s) - 1) >> s, Hc = cc * cc;
  ArenaCtl &c = d.ctl[a];
  const int per = KIND == 1 ? d.Ecap : d.Vcap;
  const int n = KIND == 1 ? c.n_blob : c.n_vir;
  __syncthreads();
  int *start = (KIND == 1 ? d.bstart : d.vstart) + (size_t)a * (d.H + 1);
  int *items = (KIND == 1 ? d.bitems : d.vitems) + (size_t)a * per;
  int *rank = (KIND == 1 ? d.b_rank : d.v_rank) + (size_t)a * per;
  for (int i = tid; i <= Hc; i += T) cnt[i] = 0;
  __syncthreads();
  double rloc = 0;
  for (int i = tid; i < n; i += T) {
    size_t g = (size_t)a * per + i;
    bool ok = (KIND == 1 ? d.b_flags[g] : d.v_flags[g]) & F_ALIVE;
    int rk = -1;
    if (ok) {
      double x = KIND == 1 ? d.b_x[g] : d.v_x[g], y = KIND == 1 ? d.b_y[g] : d.v_y[g];
      if (KIND == 2) rloc = fmax(rloc, d.v_r[g]);
      int b = (center_bucket_coord(y, d.cols) >> s) * cc + (center_bucket_coord(x, d.cols) >> s);
      rk = (b << 12) | atomicAdd(&cnt[b], 1);  // rank < 4096 per coarse cell (else ERR_SLOT)
    }
    rank[i] = rk;
  }
  if (KIND == 2) {
    // lightest virus (bounds who can eat one in playerVirusOverlap)
    double mn = __builtin_inf();
    for (int i = tid; i < n; i += T) {
      size_t g = (size_t)a * per + i;
      if (d.v_flags[g] & F_ALIVE) mn = fmin(mn, d.v_m[g]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      mn = fmin(mn, __shfl_xor(mn, off));
      rloc = fmax(rloc, __shfl_xor(rloc, off));
    }
    if ((tid & 63) == 0) {
      vmin_w[tid >> 6] = mn;
      vmin_w[16 + (tid >> 6)] = rloc;
    }
  }
  __syncthreads();
  if (KIND == 2 && tid == 0) {
    double mn = vmin_w[0], rm = vmin_w[16];
    for (int k = 1; k < T >> 6; k++) {
      mn = fmin(mn, vmin_w[k]);
      rm = fmax(rm, vmin_w[16 + k]);
    }
    c.vmin_mass = mn;
    c.rmax_virus = rm;
  }
  block_scan_excl(cnt, cnt, Hc + 1, sh);  // in place: bucket starts
  for (int i = tid; i <= Hc; i += T) start[i] = cnt[i];
  for (int i = tid; i < n; i += T) {
    int rk = rank[i];
    if (rk < 0) continue;
    int b = rk >> 12, r = rk & 4095;
    if (r == 4095) set_err(d, a, ERR_SLOT);
    items[cnt[b] + r] = i;
  }
  __syncthreads();
}
// Player-cell grid, coarse (2^cshift_c fine buckets per side, <= SG_CAP cells).
// Atomic ranks go into a small count array per arena; one block re-scans those
// <= SG_CAP + 1 counts in LDS, so the grid needs no multi-block scan.
// Consumers apply the exact footprint test, so the coarser buckets only add
// candidates.
__device__ __forceinline__ int cgrid_cols(const Dev &d) { return (d.cols + (1 << d.cshift_c) - 1) >> d.cshift_c; }
__device__ __forceinline__ int cgrid_bucket(const Dev &d, double x, double y) {
  const int sh = d.cshift_c;
  return (center_bucket_coord(y, d.cols) >> sh) * cgrid_cols(d) + (center_bucket_coord(x, d.cols) >> sh);
}
// row 0: the player-cell grid's counts, row 1: the blob grid's (blob_count)
__device__ __forceinline__ int *cgrid_counts(const Dev &d, int a, int row) {
  return d.cgcnt + ((size_t)a * 2 + row) * CG_STRIDE;
}
// The player-cell grid is built in three steps, none of them a launch of its own:
//  1. counts: every live cell takes an atomic rank in its coarse bucket where its
//     position and list are final -- mergePlayerCells' / the virus test's player
//     threads of k_merge_pv (k_merge_vb), explosion children in its serial pass
//     (cgrid_count_cell); the grid's radius bound is maxed there too;
//  2. scan: the first block of k_food_prep per arena turns the counts into
//     the bucket starts (cgrid_scan_block) and zeroes them for the next tick,
//     before its own players;
//  3. placement: each player's thread of k_food_commit round 1 writes its cells'
//     items (start of the bucket + rank).
// Eating changes masses and radii, never positions (a cell that eats reports its
// grown radius itself), and the grid is first read by playerPlayerOverlap.
// (Until round 5 the counts were extra blocks of commit round 1 and the scatter
// extra blocks of round 2, which made a second commit launch necessary.)
// c_rank holds (bucket << 17) | rank: bucket < SG_CAP + 1 <= 2^13, rank < 16 * B <= 2^17
__device__ __forceinline__ void cgrid_count_cell(const Dev &d, int a, size_t ci, double x, double y) {
  const int per = kMaxCells * d.B, slot = (int)(ci / d.NP), p = (int)(ci - (size_t)slot * d.NP) - a * d.B;
  const int b = cgrid_bucket(d, x, y);
  d.c_rank[(size_t)a * per + (size_t)slot * d.B + p] = (b << 17) | atomicAdd(&cgrid_counts(d, a, 0)[b], 1);
}
// one block per arena: bucket starts from the counts (exclusive scan of <= SG_CAP + 1
// values in LDS), and the counts back to zero for the next tick
// (256 threads) bucket starts of n <= SG_CAP counts (16-byte aligned, kept in
// registers: 16 per thread, one int4 load round), written to start[0..n] and,
// when lds is given, to lds[0..n]; the counts are re-zeroed for the next tick;
// bits (optional): one bit per non-empty bucket, 16 per thread (bucket b at bit
// b % 16 of bits[b / 16]: a little-endian bitmap)
__device__ void count_scan_256(int *cnt, int n, int *start, int *lds, uint16_t *bits) {
  __shared__ int wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int4 *c4 = reinterpret_cast<const int4 *>(cnt);
  int v[16], sum = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int j = tid * 16 + 4 * k;
    int4 q = j < n ? c4[j >> 2] : make_int4(0, 0, 0, 0);
    v[4 * k] = j < n ? q.x : 0;
    v[4 * k + 1] = j + 1 < n ? q.y : 0;
    v[4 * k + 2] = j + 2 < n ? q.z : 0;
    v[4 * k + 3] = j + 3 < n ? q.w : 0;
  }
#pragma unroll
  for (int k = 0; k < 16; k++) sum += v[k];
  if (bits) {
    uint32_t bm = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) bm |= (v[k] != 0 ? 1u : 0u) << k;
    bits[tid] = (uint16_t)bm;
  }
  int inc = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int t = __shfl_up(inc, off);
    if (lane >= off) inc += t;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int run = inc - sum;
  for (int k = 0; k < w; k++) run += wsum[k];
  const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int j = tid * 16 + k;
    if (j < n) {
      start[j] = run;
      if (lds) lds[j] = run;
      cnt[j] = 0;
    }
    run += v[k];
  }
  if (tid == 0) {
    start[n] = total;
    if (lds) lds[n] = total;
  }
}
__device__ void cgrid_scan_block(const Dev &d, int a) {
  const int cc = cgrid_cols(d);
  count_scan_256(cgrid_counts(d, a, 0), cc * cc, d.cstart + (size_t)a * (d.H + 1), nullptr, nullptr);
}
// step 3 for player gp's n cells (k_food_commit round 1)
__device__ __forceinline__ void cgrid_place_player(const Dev &d, int gp, int n) {
  const int NP = d.NP, a = gp / d.B, p = gp - a * d.B, per = kMaxCells * d.B;
  const int *start = d.cstart + (size_t)a * (d.H + 1);
  int *items = d.citems + (size_t)a * per;
  for (int k = 0; k < n; k++) {
    const int slot = d.p_list[k * NP + gp];
    const int br = d.c_rank[(size_t)a * per + (size_t)slot * d.B + p];
    items[start[br >> 17] + (br & 0x1FFFF)] = slot * NP + gp;
  }
}

// blocks [0, A): blob grids; [A, 2A): virus grids (when enabled)

// ------------------------------------------------------------ pellet rows
// The pellet store (aigar_dev.h): bucket rows with two homes each.  Reset
// (Field.initialize's spawnPellets, field.py:57-67, 303-313) places the staged
// spawns by a counting sort -- atomic ranks per bucket, one block per row for
// the row's bucket starts, then the records -- into home 0.  A tick changes a
// few pellets (eaten: field.py:327-344; blob conversions: :99-110; spawns): the
// closing update (k_pel_update) rewrites only the rows they touch.
__device__ __forceinline__ int prow_entry(const Dev &d, int bx, int by) { return by * (d.cols + 1) + bx; }
// staged record j: its rank in its bucket (tiles: -1 outside the held range)
__global__ void k_prow_count(Dev d) {
  const int gi = GTID;
  if (gi >= d.A * d.Pcap) return;
  const int a = gi / d.Pcap, j = gi - a * d.Pcap;
  ArenaCtl &c = d.ctl[a];
  if (j == 0) c.n_pel = 0;  // (k_prow_scan adds the rows' counts)
  if (j >= c.n_pnew) return;
  const PelRec r = d.pn[gi];
  const int bx = center_bucket_coord(r.x, d.cols), by = center_bucket_coord(r.y, d.cols);
  d.pel_rank[gi] = tile_holds_bucket(d, bx, by) ? atomicAdd(&d.pncnt[(size_t)a * d.PH1 + prow_entry(d, bx, by)], 1) : -1;
}
// block-wide exclusive scan of up to 4 values per thread (256 threads); returns the total
__device__ __forceinline__ int block_scan4(int *v, int *wsum) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int sum = v[0] + v[1] + v[2] + v[3], inc = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int before = 0, total = 0;
  for (int k = 0; k < 4; k++) {
    before += k < w ? wsum[k] : 0;
    total += wsum[k];
  }
  __syncthreads();
  int run = before + inc - sum;
  for (int k = 0; k < 4; k++) {
    const int x = v[k];
    v[k] = run;
    run += x;
  }
  return total;
}
// one block per (row, arena): the row's bucket starts in home 0 (cols <= 1024)
__global__ void __launch_bounds__(256) k_prow_scan(Dev d) {
  __shared__ int wsum[4];
  const int r = blockIdx.x, a = blockIdx.y, tid = threadIdx.x, C = d.cols;
  ArenaCtl &c = d.ctl[a];
  int *cnt = d.pncnt + (size_t)a * d.PH1 + (size_t)r * (C + 1);
  int *st = d.pstart + (size_t)a * d.PH1 + (size_t)r * (C + 1);
  int v[4];
  for (int k = 0; k < 4; k++) {
    const int bx = tid * 4 + k;
    v[k] = bx < C ? cnt[bx] : 0;
  }
  const int total = block_scan4(v, wsum), base = r * d.PR;
  for (int k = 0; k < 4; k++) {
    const int bx = tid * 4 + k;
    if (bx < C) {
      st[bx] = base + min(v[k], d.PR);
      cnt[bx] = 0;  // (re-zeroed for the next reset)
    }
  }
  if (tid == 0) {
    st[C] = base + min(total, d.PR);
    if (total > d.PR) set_err(d, a, ERR_PELLET_CAP);
    atomicAdd(&c.n_pel, min(total, d.PR));
    if (r == 0) {
      c.src_n_stage = c.n_pnew;  // (k_prow_scatter's bound; nothing here reads n_pnew)
      c.n_pnew = 0;
      c.n_pel_eaten = 0;
    }
  }
}
__global__ void k_prow_scatter(Dev d) {
  const int gi = GTID;
  if (gi >= d.A * d.Pcap) return;
  const int a = gi / d.Pcap, j = gi - a * d.Pcap;
  if (j >= d.ctl[a].src_n_stage) return;
  const int rk = d.pel_rank[gi];
  if (rk < 0) return;  // (tiles: not held here)
  const PelRec r = d.pn[gi];
  const int bx = center_bucket_coord(r.x, d.cols), by = center_bucket_coord(r.y, d.cols);
  const int e = (int)((size_t)a * d.PH1) + prow_entry(d, bx, by);
  const int pos = d.pstart[e] + rk;
  if (pos >= d.pstart[e + 1]) return;  // (row overflow: ERR_PELLET_CAP is set)
  const size_t o = (size_t)a * d.PS + pos;
  d.pel[o] = r;
  d.pel_col[o] = d.pn_col[gi];
}
// ------------------------------------------------------------ T10 merge
__device__ __forceinline__ void merge_player(const Dev &d, int gp) {
  if (gp >= d.NP) return;
  const int NP = d.NP, a = gp / d.B;
  // liveness, count and the list's first rows in one load round (rows past
  // the count are allocated and unused), then the first cells' timers in one
  uint8_t l4[kTailRegs];
#pragma unroll
  for (int k = 0; k < kTailRegs; k++) l4[k] = d.p_list[k * NP + gp];
  const bool alive = d.p_alive[gp];
  const int n = d.p_ncells[gp];
  if (!alive) return;
  uint8_t cs[kMaxCells];
  int nm = 0;
  double mt4[kTailRegs];
#pragma unroll
  for (int k = 0; k < kTailRegs; k++) mt4[k] = k < n ? d.c_mt[(size_t)l4[k] * NP + gp] : 1.0;
#pragma unroll
  for (int k = 0; k < kTailRegs; k++)  // getMergableCells (player.py:144-149)
    if (k < n && mt4[k] <= 0) cs[nm++] = l4[k];
  for (int k = kTailRegs; k < n; k++) {
    uint8_t s = d.p_list[k * NP + gp];
    if (d.c_mt[(size_t)s * NP + gp] <= 0) cs[nm++] = s;
  }
  if (nm <= 1) return;
  for (int i = 1; i < nm; i++) {  // stable sort by mass desc
    uint8_t key = cs[i];
    double km = d.c_m[(size_t)key * NP + gp];
    int j = i - 1;
    while (j >= 0 && km > d.c_m[(size_t)cs[j] * NP + gp]) {
      cs[j + 1] = cs[j];
      j--;
    }
    cs[j + 1] = key;
  }
  uint32_t order = 0;
  for (int i = 0; i < nm; i++) {
    size_t c1 = (size_t)cs[i] * NP + gp;
    if (!(d.c_flags[c1] & F_ALIVE)) continue;
    for (int j = 0; j < nm; j++) {
      size_t c2 = (size_t)cs[j] * NP + gp;
      if (!(d.c_flags[c2] & F_ALIVE) || c2 == c1) continue;
      if (!overlap(d.c_x[c1], d.c_y[c1], d.c_m[c1], d.c_r[c1], d.c_x[c2], d.c_y[c2], d.c_m[c2], d.c_r[c2]))
        continue;
      // mergeCells (field.py:372-380)
      bool first_big = d.c_m[c1] > d.c_m[c2];
      size_t bi = first_big ? c1 : c2, si = first_big ? c2 : c1;
      ev_push(d, a, PH_MERGE, ((uint64_t)(gp - a * d.B) << 20) | order++, 1, d.c_seq[bi], d.c_seq[si]);
      double m = grow_mass(d.c_m[bi], d.c_m[si]);
      d.c_m[bi] = m;
      d.c_r[bi] = radius_of(m);
      d.c_flags[si] = 0;  // deletePlayerCell: removeCell
      uint8_t sslot = (uint8_t)(si / NP);
      int cur = d.p_ncells[gp], w = 0;
      for (int k = 0; k < cur; k++) {
        uint8_t s = d.p_list[k * NP + gp];
        if (s != sslot) d.p_list[(w++) * NP + gp] = s;
      }
      d.p_ncells[gp] = w;
      if (!(d.c_flags[c1] & F_ALIVE)) break;
    }
  }
}

// step 1 of the player-cell grid for player gp's cells after its merges, when no
// virus test visits them (k_merge_vb); returns its largest cell radius
__device__ double cgrid_count_player(const Dev &d, int gp) {
  const int NP = d.NP, a = gp / d.B;
  uint8_t l4[kTailRegs];
#pragma unroll
  for (int k = 0; k < kTailRegs; k++) l4[k] = d.p_list[k * NP + gp];
  const bool alive = d.p_alive[gp];
  const int n = d.p_ncells[gp];
  if (!alive) return 0.0;
  double rmax = 0;
  for (int k = 0; k < n; k++) {
    const size_t ci = (size_t)(k < kTailRegs ? l4[k] : d.p_list[k * NP + gp]) * NP + gp;
    cgrid_count_cell(d, a, ci, d.c_x[ci], d.c_y[ci]);
    rmax = fmax(rmax, d.c_r[ci]);
  }
  return rmax;
}

// ------------------------------------------------------------ serial-phase helpers
// insertion sort of (key, val) pairs, single thread (worklists are short)
__device__ void isort_kv(int64_t *key, int *val, int n) {
  for (int i = 1; i < n; i++) {
    int64_t k = key[i];
    int v = val[i];
    int j = i - 1;
    while (j >= 0 && key[j] > k) {
      key[j + 1] = key[j];
      val[j + 1] = val[j];
      j--;
    }
    key[j + 1] = k;
    val[j + 1] = v;
  }
}

// ------------------------------------------------------------ T11 virus <- blob
// virusBlobOverlap's activity test (field.py:316-325) from the blob side: one
// thread per blob slot walks the virus grid around the blob's footprint and
// marks every virus it overlaps -- the same pairs as the virus side's walk of the
// blob grid (both tests are symmetric: footprint-rect hit, then overlap), but
// without the blob grid, which is built in the same launch.  A virus joins the
// work list once (v_active: set here, cleared by the serial pass).
__device__ __forceinline__ void vb_active_blob(const Dev &d, int gb) {
  if (gb >= d.A * d.Ecap) return;
  const int a = gb / d.Ecap, j = gb - a * d.Ecap;
  const ArenaCtl &c = d.ctl[a];
  if (j >= c.n_blob || !(d.b_flags[gb] & F_ALIVE)) return;
  const double bx = d.b_x[gb], by = d.b_y[gb], bm = d.b_m[gb], br = d.b_r[gb];
  const Rect qb = footprint(bx, by, br, d.size);
  const int *st = d.vstart + (size_t)a * (d.H + 1);
  const int *it = d.vitems + (size_t)a * d.Vcap;
  const int nv = c.n_vir;
  grid_visit(st, it, d.cols, qb, expand_for(c.rmax_virus), [&](int i) {
    const size_t g = (size_t)a * d.Vcap + i;
    if (i >= nv || !(d.v_flags[g] & F_ALIVE)) return;
    const double vx = d.v_x[g], vy = d.v_y[g], vr = d.v_r[g];
    if (!rect_hit(footprint(vx, vy, vr, d.size), qb)) return;
    if (!overlap(vx, vy, d.v_m[g], vr, bx, by, bm, br)) return;
    if (atomicExch(&d.v_active[g], 1) != 0) return;
    const int w = atomicAdd(&d.ctl[a].n_pend, 1);
    if (w < d.Wcap) d.work[(size_t)a * d.Wcap + w] = i;
    else set_err(d, a, ERR_WORK_CAP);
  }, d.cshift);
}
// the blob grid's second step (blob_count): one block per arena loads the
// counts (re-zeroing them for the next tick), scans them in LDS, stores the
// bucket starts and places every ranked blob
__device__ void count_scan_256(int *cnt, int n, int *start, int *lds, uint16_t *bits);
__device__ void blob_grid_place(const Dev &d, int a, int *cnt) {
  const int tid = threadIdx.x, T = blockDim.x, s = d.cshift;
  const int cc = (d.cols + (1 << s) - 1) >> s;
  const int n = d.ctl[a].n_blob;
  int *items = d.bitems + (size_t)a * d.Ecap;
  const int *rank = d.b_rank + (size_t)a * d.Ecap;
  // (+ the non-empty buckets as a bitmap, which k_food_prep keeps in LDS to
  // skip the blob walk of a box that holds none)
  count_scan_256(cgrid_counts(d, a, 1), cc * cc, d.bstart + (size_t)a * (d.H + 1), cnt,
                 reinterpret_cast<uint16_t *>(d.bmap + (size_t)a * 64));
  __syncthreads();
  if (tid == 0) d.ctl[a].n_blob_live = cnt[cc * cc];  // (k_spawn_plan: whether the list needs compacting)
  for (int i = tid; i < n; i += T) {
    const int rk = rank[i];
    if (rk < 0) continue;
    const int b = rk >> 12, r = rk & 4095;
    if (r == 4095) set_err(d, a, ERR_SLOT);
    items[cnt[b] + r] = i;
  }
}
// the serial passes are device bodies run by one wavefront per arena: as their
// own launches (k_*_serial) or in the tail / head of a neighbouring kernel
// (launch_tick: fold), which saves a dependent launch per idle pass
// (returns, on lane 0, whether the pass had work: a virus may then have grown or split)
__device__ bool vb_serial_body(const Dev &d, int a, int64_t *scr_k, int *scr_v) {
  if ((threadIdx.x & 63) != 0) return false;
  ArenaCtl &c = d.ctl[a];
  int nw = min(agent_load(&c.n_pend), d.Wcap);
  c.n_pend = 0;
  c.stat[0] += nw;
  int *w = d.work + (size_t)a * d.Wcap;
  int64_t *ck = scr_k + (size_t)a * d.Wcap;
  int *cv = scr_v + (size_t)a * d.Wcap;
  if (nw == 0) return false;
  // active viruses in list order; viruses appended by splits are visited too
  for (int k = 0; k < nw; k++) {
    ck[k] = w[k];
    d.v_active[(size_t)a * d.Vcap + w[k]] = 0;  // (vb_active_blob's marks)
  }
  isort_kv(ck, w, nw);
  const int *st = d.bstart + (size_t)a * (d.H + 1);
  const int *it = d.bitems + (size_t)a * d.Ecap;
  int wk = 0;
  uint64_t order = 0;
  const double thr = kVirusBase + 7 * kEjectMass * 0.8;
  for (int i = w[0]; i < c.n_vir; i++) {
    if (i < c.n_vir_start) {
      if (wk < nw && w[wk] == i) wk++;
      else continue;
    }
    size_t gv = (size_t)a * d.Vcap + i;
    double vx = d.v_x[gv], vy = d.v_y[gv];
    Rect q = footprint(vx, vy, d.v_r[gv], d.size);
    int nc = 0;
    grid_visit(st, it, d.cols, q, 1, [&](int j) {
      size_t g = (size_t)a * d.Ecap + j;
      if (!(d.b_flags[g] & F_ALIVE)) return;
      if (!rect_hit(footprint(d.b_x[g], d.b_y[g], d.b_r[g], d.size), q)) return;
      if (nc < d.Wcap) {
        ck[nc] = d.b_seq[g];
        cv[nc] = j;
        nc++;
      }
    }, d.cshift);
    isort_kv(ck, cv, nc);
    for (int t = 0; t < nc; t++) {
      size_t g = (size_t)a * d.Ecap + cv[t];
      if (!(d.b_flags[g] & F_ALIVE)) continue;
      if (!overlap(d.v_x[gv], d.v_y[gv], d.v_m[gv], d.v_r[gv], d.b_x[g], d.b_y[g], d.b_m[g], d.b_r[g])) continue;
      if (i >= c.n_vir_start) c.warn |= WARN_NEW_VIRUS_EATS;  // reference: deleteObject raises
      ev_push(d, a, PH_VB, order++, 2, d.v_seq[gv], d.b_seq[g]);
      double m = grow_mass(d.v_m[gv], d.b_m[g]);
      d.v_m[gv] = m;
      d.v_r[gv] = radius_of(m);
      c.rmax_virus = fmax(c.rmax_virus, d.v_r[gv]);
      d.b_flags[g] = 0;
      atomicOr(&d.ctl[a].dirty, DIRTY_BLOB);
      if (m >= thr) {  // virus split (field.py:318-325, cell.py:72-85)
        if (c.n_vir >= d.Vcap) {
          c.err |= ERR_VIRUS_CAP;
          continue;
        }
        double ox = 2 * d.v_x[gv] - d.b_x[g], oy = 2 * d.v_y[gv] - d.b_y[g];
        size_t gn = (size_t)a * d.Vcap + c.n_vir;
        double x = d.v_x[gv], y = d.v_y[gv], nm = m / 2, nr = radius_of(nm);
        double ang = aigar_math::trig_atan2(oy - y, ox - x);
        double ca, sa;
        aigar_math::trig_sincos(ang, sa, ca);
        double xp = ca * nr * 4.5 + x, yp = sa * nr * 4.5 + y;
        double svx, svy;
        int svc;
        add_momentum(x, y, xp, yp, (double)d.size, (double)d.size, d.v_r[gv], svx, svy, svc);
        d.v_x[gn] = x;
        d.v_y[gn] = y;
        d.v_m[gn] = nm;
        d.v_r[gn] = nr;
        d.v_vx[gn] = 0;
        d.v_vy[gn] = 0;
        d.v_svx[gn] = svx;
        d.v_svy[gn] = svy;
        d.v_svc[gn] = svc;
        d.v_seq[gn] = c.seq_next++;
        d.v_flags[gn] = F_ALIVE;  // addVirus does not hash it
        double pm = d.v_m[gv] / 2;
        d.v_m[gv] = pm;
        d.v_r[gv] = radius_of(pm);
        ev_push(d, a, PH_VB, order++, 3, d.v_seq[gv], d.v_seq[gn]);
        c.n_vir++;
      }
    }
  }
  return true;
}

// mergePlayerCells (per player) and the virus<-blob activity test (per virus)
// in one launch: merging touches only player cells, the test only viruses/blobs
// fold: virusBlobOverlap's serial pass runs in the last block (one wave per arena)
// (+ one block per arena at the end: the blob grid's placement, blob_grid_place)
__global__ void __launch_bounds__(256) k_merge_vb(Dev d, int64_t *scr_k, int *scr_v, int fold) {
  FLOOR(2);
  __shared__ int g_cnt[SG_CAP + 1];
  const int nbP = (d.NP + 255) / 256;
  if ((int)blockIdx.x >= nbP) {
    blob_grid_place(d, blockIdx.x - nbP, g_cnt);
  } else {
    const int gi = GTID;
    double rg = 0;
    if (gi < d.NP) {
      merge_player(d, gi);
      rg = cgrid_count_player(d, gi);
    }
    wave_atomic_max_pos(&d.ctl[min(gi, d.NP - 1) / d.B].rmax_cell, rg);
  }
  if (fold && last_block(d.ticket + 0, gridDim.x))
    for (int a = threadIdx.x >> 6; a < d.A; a += blockDim.x >> 6) vb_serial_body(d, a, scr_k, scr_v);
}

// ------------------------------------------------------------ T12 cell <- virus
// wave-wide "does any entity in the grid rows around q satisfy pred"
template <class Pred>
__device__ __forceinline__ bool wave_any_in_grid(const int *st, const int *items, int cols, Rect q, int E, Pred pred,
                                                 int shift = 0) {
  if (q.x1 < q.x0 || q.y1 < q.y0) return false;
  const Span g = grid_span(q, E, cols, shift);
  const int bx0 = g.bx0, bx1 = g.bx1, by0 = g.by0;
  const int lane = threadIdx.x & 63, nrows = g.by1 - by0 + 1;
  for (int r0 = 0; r0 < nrows; r0 += 64) {  // rows flattened as in wave_grid_for
    const int r = r0 + lane, nr = min(64, nrows - r0);
    int lo = 0, len = 0;
    if (r < nrows) {
      int b = (by0 + r) * g.stride;
      lo = st[b + bx0];
      len = st[b + bx1 + 1] - lo;
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
      bool hit = t < total && pred(items ? items[idx] : idx);
      if (__ballot(hit)) return true;
    }
  }
  return false;
}

// one thread per player: its cells that overlap an edible virus at phase start
// (c_active; the player joins the serial pass's work list).  Cells lighter than
// 1.25 x the lightest virus have nothing to eat and skip the grid; the rest
// walk the coarse virus grid serially (a few viruses per neighbourhood).  One
// thread per player keeps the grid at NP/256 blocks, so the serial pass runs
// in the last block (fold) for the price of a small ticket fan-in.
// count: also take the cells' ranks in the player-cell grid (step 1 of its
// build; not in pv_redo) -- returns the player's largest cell radius (0: none)
__device__ double pv_player(const Dev &d, int gp, bool count = true) {
  const int NP = d.NP, a = gp / d.B;
  const int *st = d.vstart + (size_t)a * (d.H + 1);
  const int *it = d.vitems + (size_t)a * d.Vcap;
  const int E = expand_for(d.ctl[a].rmax_virus);
  // lightest virus at the grid build (k_players); viruses split during
  // virusBlobOverlap are >= (VIRUS_BASE_SIZE + 7 * 14.4) / 2, so VIRUS_BASE_SIZE bounds them
  const double vmin = fmin(d.ctl[a].vmin_mass, kVirusBase);
  uint8_t l4[kTailRegs];  // (the list's first rows with the count: one load round)
#pragma unroll
  for (int k = 0; k < kTailRegs; k++) l4[k] = d.p_list[k * NP + gp];
  const bool alive = d.p_alive[gp];
  const int n = d.p_ncells[gp];
  if (!alive) return 0.0;
  bool anyp = false;
  double rmax = 0;
  // the first cells' records in one round, before any grid walk
  double x4[kTailRegs], y4[kTailRegs], m4[kTailRegs], r4[kTailRegs];
#pragma unroll
  for (int k = 0; k < kTailRegs; k++) {
    x4[k] = y4[k] = m4[k] = r4[k] = 0;
    if (k < n) {
      const size_t ci = (size_t)l4[k] * NP + gp;
      x4[k] = d.c_x[ci];
      y4[k] = d.c_y[ci];
      m4[k] = d.c_m[ci];
      r4[k] = d.c_r[ci];
    }
  }
  for (int k = 0; k < n; k++) {
    size_t ci;
    double x, y, m, r;
    if (k < kTailRegs) {  // (select from the registers: no dynamic index)
      uint8_t s = l4[0];
      x = x4[0], y = y4[0], m = m4[0], r = r4[0];
#pragma unroll
      for (int j = 1; j < kTailRegs; j++)
        if (k == j) s = l4[j], x = x4[j], y = y4[j], m = m4[j], r = r4[j];
      ci = (size_t)s * NP + gp;
    } else {
      ci = (size_t)d.p_list[k * NP + gp] * NP + gp;
      x = d.c_x[ci], y = d.c_y[ci], m = d.c_m[ci], r = d.c_r[ci];
    }
    rmax = fmax(rmax, r);
    bool any = false;
    if (m > 1.25 * vmin) {
      const Rect q = footprint(x, y, r, d.size);
      grid_visit(st, it, d.cols, q, E, [&](int j) {
        const size_t g = (size_t)a * d.Vcap + j;
        if (any || (d.v_flags[g] & (F_ALIVE | F_INHASH)) != (F_ALIVE | F_INHASH)) return;
        if (!rect_hit(footprint(d.v_x[g], d.v_y[g], d.v_r[g], d.size), q)) return;
        any = overlap(x, y, m, r, d.v_x[g], d.v_y[g], d.v_m[g], d.v_r[g]) && m > 1.25 * d.v_m[g];
      }, d.cshift);
    }
    d.c_active[ci] = any;
    anyp |= any;
  }
  if (anyp) {  // (its own work list: virusBlobOverlap's runs in the same launch)
    const int w = atomicAdd(&d.ctl[a].n_pend2, 1);
    if (w < d.Wcap) d.work2[(size_t)a * d.Wcap + w] = gp - a * d.B;
    else set_err(d, a, ERR_WORK_CAP);
  }
  if (count) {  // (last: the returning atomics delay no load of the activity test)
#pragma unroll
    for (int k = 0; k < kTailRegs; k++)
      if (k < n) cgrid_count_cell(d, a, (size_t)l4[k] * NP + gp, x4[k], y4[k]);
    for (int k = kTailRegs; k < n; k++) {
      const size_t ci = (size_t)d.p_list[k * NP + gp] * NP + gp;
      cgrid_count_cell(d, a, ci, d.c_x[ci], d.c_y[ci]);
    }
  }
  return rmax;
}
// The activity test again for every player of arena a, by one wavefront, after
// virusBlobOverlap's serial pass had work: a virus that grew or split changes
// which cells overlap an edible virus at playerVirusOverlap's start.
__device__ void pv_redo(const Dev &d, int a) {
  const int lane = threadIdx.x & 63;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (lane 0's virus writes)
  if (lane == 0) __hip_atomic_store(&d.ctl[a].n_pend2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int p = lane; p < d.B; p += 64) pv_player(d, a * d.B + p, false);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (the lanes' work-list writes, read by lane 0)
}
__device__ void pv_serial_body(const Dev &d, int a, int64_t *scr_k, int *scr_v);
// mergePlayerCells, the virus<-blob activity test and the cell<-virus activity
// test in ONE launch (field.py:183-198, 246-253, 225-231): a player's thread
// merges its cells, then tests them against the viruses -- a player's merges
// touch only its own cells, and the virus test reads only its own cells and
// the viruses.  The viruses are those of the phase's start unless
// virusBlobOverlap's serial pass (the last block) had work, which is rare (0
// per tick at C3, random or Greedy bots): then the arena's test runs again
// (pv_redo) before playerVirusOverlap's serial pass.
// Blocks: the players' (merges + the virus test), the blob slots' (the
// virus<-blob activity test from the blob side) and one per arena placing the
// blob grid (read first by virusBlobOverlap's serial pass, in the last block).
__global__ void __launch_bounds__(256) k_merge_pv(Dev d, int64_t *scr_k, int *scr_v) {
  FLOOR(2);
  __shared__ int g_cnt[SG_CAP + 1];
  const int nbP = (d.NP + 255) / 256, nbB = (d.A * d.Ecap + 255) / 256, b = blockIdx.x;
  if (b < nbP) {
    const int gi = GTID;
    double rg = 0;
    if (gi < d.NP) {
#ifndef AIGAR_DIAG_NO_MERGE  // (cost diagnostics only, results invalid)
      merge_player(d, gi);
#endif
      rg = pv_player(d, gi);
    }
    // the player-cell grid's radius bound (pre-eat radii; eaters report their growth)
    wave_atomic_max_pos(&d.ctl[min(gi, d.NP - 1) / d.B].rmax_cell, rg);
  } else if (b < nbP + nbB) {
    vb_active_blob(d, (b - nbP) * 256 + threadIdx.x);
  } else {
    const int a = b - nbP - nbB;
    if (threadIdx.x == 0) d.ctl[a].n_vir_start = d.ctl[a].n_vir;  // (splits append past it)
    blob_grid_place(d, a, g_cnt);
  }
  // the serial passes read the other blocks' plain stores only when they have
  // work: the last block acquires only then (random C3: ~1 tick in 100)
  if (last_block(d.ticket + 0, gridDim.x, false)) {
    __shared__ int s_work;
    if (threadIdx.x == 0) {
      int w = 0;
      for (int a = 0; a < d.A; a++) w |= agent_load(&d.ctl[a].n_pend) | agent_load(&d.ctl[a].n_pend2);
      s_work = w;
    }
    __syncthreads();
    agent_acquire_block(s_work != 0);
    for (int a = threadIdx.x >> 6; a < d.A; a += blockDim.x >> 6) {
      const bool vb = vb_serial_body(d, a, scr_k, scr_v);
      if (__shfl(vb ? 1 : 0, 0)) pv_redo(d, a);
#ifndef AIGAR_DIAG_NO_PV_SERIAL  // (cost diagnostics only, results invalid)
      pv_serial_body(d, a, scr_k, scr_v);
#endif
    }
  }
}
// playerVirusOverlap's serial pass, one wavefront per arena: every lane runs
// the same serial code (the same loads and plain stores, in program order, as
// pp_turns), the atomics and the event log on lane 0, and each active cell's
// virus candidates are gathered by the lanes together (wave_grid_for; the list
// is then sorted by creation sequence as before, so its order is the same)
__device__ void pv_serial_body(const Dev &d, int a, int64_t *scr_k, int *scr_v) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lt = (1ull << lane) - 1;
  ArenaCtl &c = d.ctl[a];
  int nw = min(agent_load(&c.n_pend2), d.Wcap);
  wave_fence();
  if (lane == 0) {
    c.n_pend2 = 0;
    c.stat[1] += nw;
  }
  if (nw == 0) return;
  const int NP = d.NP;
  int *w = d.work2 + (size_t)a * d.Wcap;
  int64_t *ck = scr_k + (size_t)a * d.Wcap;
  int *cv = scr_v + (size_t)a * d.Wcap;
  for (int k = 0; k < nw; k++) ck[k] = w[k];
  isort_kv(ck, w, nw);
  const int *st = d.vstart + (size_t)a * (d.H + 1);
  const int *it = d.vitems + (size_t)a * d.Vcap;
  const double W = (double)d.size;
  uint64_t order = 0;
  for (int wi = 0; wi < nw; wi++) {
    int gp = a * d.B + w[wi];
    if (!d.p_alive[gp]) continue;
    for (int i = 0; i < d.p_ncells[gp];) {  // live list: explosion children are visited too
      size_t ci = (size_t)d.p_list[i * NP + gp] * NP + gp;
      i++;
      if (!d.c_active[ci] && !(d.c_flags[ci] & F_NEW)) continue;
      int E = expand_for(c.rmax_virus);
      Rect q = footprint(d.c_x[ci], d.c_y[ci], d.c_r[ci], d.size);
      int nc = 0;
      wave_grid_for(st, it, d.cols, q, E, [&](bool valid, int j) {
        bool keep = false;
        int64_t sq = 0;
        if (valid) {
          const size_t g = (size_t)a * d.Vcap + j;
          keep = (d.v_flags[g] & (F_ALIVE | F_INHASH)) == (F_ALIVE | F_INHASH) &&
                 rect_hit(footprint(d.v_x[g], d.v_y[g], d.v_r[g], d.size), q);
          if (keep) sq = d.v_seq[g];
        }
        const unsigned long long bal = __ballot(keep);
        const int slot = nc + __popcll(bal & lt);
        if (keep && slot < d.Wcap) {
          ck[slot] = sq;
          cv[slot] = j;
        }
        nc += __popcll(bal);
      }, d.cshift);
      nc = min(nc, d.Wcap);
      wave_fence();  // (the lanes' candidates -> every lane's sort)
      isort_kv(ck, cv, nc);
      for (int t = 0; t < nc; t++) {
        size_t g = (size_t)a * d.Vcap + cv[t];
        if (!(d.v_flags[g] & F_ALIVE)) continue;
        double cm = d.c_m[ci];
        if (!(overlap(d.c_x[ci], d.c_y[ci], cm, d.c_r[ci], d.v_x[g], d.v_y[g], d.v_m[g], d.v_r[g]) &&
              cm > 1.25 * d.v_m[g]))
          continue;
        // eatVirus -> eatCell(..., isVirus=True) (field.py:333-344)
        if (lane == 0) ev_push(d, a, PH_PV, order, 4, d.c_seq[ci], d.v_seq[g]);
        order++;
        double m = grow_mass(cm, d.v_m[g] * kVirusEatFactor);
        d.c_m[ci] = m;
        d.c_r[ci] = radius_of(m);
        if (lane == 0) {
          atomic_max_pos(&c.rmax_cell, d.c_r[ci]);  // (the player-cell grid's radius bound)
          atomicOr(&d.ctl[a].dirty, DIRTY_VIRUS);
        }
        d.v_flags[g] = 0;
        // playerCellAteVirus (field.py:350-370)
        int ncur = d.p_ncells[gp];
        int n_new = kMaxCells - ncur;
        if (lane == 0) ev_push(d, a, PH_PV, order, 5, d.c_seq[ci], n_new);
        order++;
        if (n_new == 0) continue;
        double dist = d.c_m[ci] * kExplosionProp;
        double mpc = dist / n_new;
        d.c_mt[ci] = merge_time_for(kMergeVirusFactor, d.c_m[ci]);
        double m2 = grow_mass(d.c_m[ci], -1 * mpc * n_new);
        d.c_m[ci] = m2;
        d.c_r[ci] = radius_of(m2);
        uint32_t used = 0;
        for (int k = 0; k < ncur; k++) used |= 1u << d.p_list[k * NP + gp];
        double px = d.c_x[ci], py = d.c_y[ci], pr = d.c_r[ci];
        for (int k = 0; k < n_new; k++) {
          int slot = __ffs(~used) - 1;
          used |= 1u << slot;
          size_t ni = (size_t)slot * NP + gp;
          int64_t seq = c.seq_next++;
          double nr = radius_of(mpc);
          uint64_t u[4];
          philox((uint64_t)seq, ST_ANGLE, 0, 0, c.key0, c.key1, u);
          int64_t deg = (int64_t)mulhi(u[0], 360);
          double ang = (double)deg * (kPi / 180.0);  // numpy.deg2rad
          double ca, sa;
          aigar_math::trig_sincos(ang, sa, ca);
          double xp = ca * pr * 12 + px, yp = sa * pr * 12 + py;
          double vx, vy, svx, svy;
          int svc;
          set_move_direction(px, py, mpc, nr, xp, yp, vx, vy);
          add_momentum(px, py, xp, yp, W, W, pr, svx, svy, svc);
          d.c_x[ni] = px;
          d.c_y[ni] = py;
          d.c_m[ni] = mpc;
          d.c_r[ni] = nr;
          d.c_vx[ni] = vx;
          d.c_vy[ni] = vy;
          d.c_svx[ni] = svx;
          d.c_svy[ni] = svy;
          d.c_svc[ni] = svc;
          d.c_mt[ni] = merge_time_for(0.8, mpc);
          d.c_seq[ni] = seq;
          d.c_flags[ni] = F_ALIVE | F_INHASH | F_NEW;  // addPlayerCell hashes it
          d.c_active[ni] = 0;
          if (lane == 0) cgrid_count_cell(d, a, ni, px, py);  // (step 1 of the player-cell grid)
          d.p_list[(ncur + k) * NP + gp] = (uint8_t)slot;
        }
        d.p_ncells[gp] = ncur + n_new;
      }
    }
    for (int k = 0; k < d.p_ncells[gp]; k++) d.c_flags[(size_t)d.p_list[k * NP + gp] * NP + gp] &= ~F_NEW;
  }
}

// ------------------------------------------------------------ T14/T15 food
// playerPelletOverlap then playerBlobOverlap (field.py:200-222) as ONE
// reservation pass.  The reference eats every pellet (all players, all cells)
// before any blob, but a cell's blob turn depends only on its own mass after
// its pellet turn and on the blobs lower-priority cells ate: no pellet turn of
// another cell and no blob turn of any other cell touches either.  So the
// sequential order "per cell (player order, list order): its pellets, then its
// blobs" gives the same world, and one reservation pass with a combined
// per-cell food list (pellets by creation sequence, then blobs by creation
// sequence) resolves both phases.  Events keep their reference phase keys.
//
// Foods are coded j: pellets j in [0, n0) (the current bucket-sorted buffer)
// and [n0, n0 + nst) (this tick's blob conversions, addPellet in updateBlobs,
// still in the staging list -- they join the sorted buffer at the closing
// rebuild, so no rebuild runs before the eat phase); blobs kBlobBit | slot.
// Pellet dead flags and reservation words are indexed by a * PD + j.
constexpr int kBlobBit = 1 << 30;
// a store pellet killed this tick, for the closing update (each once: a tile
// applying another tile's kill notes it only if its own eat phase did not)
__device__ __forceinline__ void note_kill(const Dev &d, int a, int j) {
  const int k = atomicAdd(&d.ctl[a].n_kill, 1);
  if (k < d.Pcap) d.kill_list[(size_t)a * d.Pcap + k] = j;
  else set_err(d, a, ERR_PELLET_CAP);
}
struct Food {
  const Dev &d;
  int a;
  int n0, nst;  // n0: the store's slots (PS); staged records (this tick's blob conversions) follow
  int nblob;  // (the blob list's length is fixed during the eat phase: loaded with the rest, no round of its own)
  __device__ Food(const Dev &dd, int aa) : d(dd), a(aa), n0(dd.PS), nst(dd.ctl[aa].n_pnew), nblob(dd.ctl[aa].n_blob) {}
  __device__ static bool blob(int j) { return (j & kBlobBit) != 0; }
  __device__ size_t g(int j) const { return (size_t)a * d.PD + j; }                 // pellet j's flag / key
  __device__ size_t gp(int j) const { return (size_t)a * d.PS + j; }                // store pellet j's record
  __device__ size_t gs(int j) const { return (size_t)a * d.Pcap + (j - n0); }       // staged pellet j
  __device__ size_t gb(int j) const { return (size_t)a * d.Ecap + (j & ~kBlobBit); }  // blob
  __device__ double x(int j) const { return blob(j) ? d.b_x[gb(j)] : (j < n0 ? d.pel[gp(j)].x : d.pn[gs(j)].x); }
  __device__ double y(int j) const { return blob(j) ? d.b_y[gb(j)] : (j < n0 ? d.pel[gp(j)].y : d.pn[gs(j)].y); }
  __device__ double m(int j) const { return blob(j) ? d.b_m[gb(j)] : (j < n0 ? d.pel[gp(j)].m : d.pn[gs(j)].m); }
  __device__ double r(int j) const { return blob(j) ? d.b_r[gb(j)] : pellet_radius(m(j)); }
  __device__ int64_t seq(int j) const {
    return blob(j) ? d.b_seq[gb(j)] : (j < n0 ? d.pel[gp(j)].seq : d.pn[gs(j)].seq);
  }
  // the whole food record in one round of loads (a pellet: its 32-byte record)
  __device__ void load(int j, double &x, double &y, double &m, int64_t &sq) const {
    if (blob(j)) {
      const size_t b = gb(j);
      x = d.b_x[b];
      y = d.b_y[b];
      m = d.b_m[b];
      sq = d.b_seq[b];
    } else {
      const PelRec r = j < n0 ? d.pel[gp(j)] : d.pn[gs(j)];
      x = r.x;
      y = r.y;
      m = r.m;
      sq = r.seq;
    }
  }
  __device__ double rad(int j, double m) const { return blob(j) ? d.b_r[gb(j)] : pellet_radius(m); }
  __device__ bool alive(int j) const { return blob(j) ? (d.b_flags[gb(j)] & F_ALIVE) != 0 : !d.pel_dead[g(j)]; }
  __device__ int64_t ej(int j) const { return blob(j) ? d.b_ej[gb(j)] : -2; }
  // the dead flag alone (food_eat_loop notes its pellet kills in batches)
  __device__ void mark_dead(int j) const {
    if (!blob(j)) {
      d.pel_dead[g(j)] = 1;
    } else {
      d.b_flags[gb(j)] = 0;
      atomicOr(&d.ctl[a].dirty, DIRTY_BLOB);
    }
  }
  __device__ void kill(int j) const {
    if (!blob(j)) {
      d.pel_dead[g(j)] = 1;
      if (j < n0) note_kill(d, a, j);  // (a staged record is dropped by its flag)
    } else {
      d.b_flags[gb(j)] = 0;
      atomicOr(&d.ctl[a].dirty, DIRTY_BLOB);
    }
  }
  __device__ uint64_t *owner(int j) const { return blob(j) ? d.b_owner + gb(j) : d.pel_owner + g(j); }
  __device__ bool any_blobs() const { return nblob > 0; }
  // every pellet / blob whose footprint may touch q: f(valid, j) on all lanes (wave-uniform calls)
  template <class Fn>
  __device__ void walk_pellets(Rect q, Fn f) const {
    wave_grid_for(d.pstart + (size_t)a * d.PH1, nullptr, d.cols, q, 1, f, 0, n0, nst, d.cols + 1);  // (+ staged)
  }
  template <class Fn>
  __device__ void walk_blobs(Rect q, Fn f) const {
    if (any_blobs())
      wave_grid_for(d.bstart + (size_t)a * (d.H + 1), d.bitems + (size_t)a * d.Ecap, d.cols, q, 1,
                    [&](bool valid, int j) { f(valid, valid ? (j | kBlobBit) : -1); }, d.cshift);
  }
  // whether the blob grid's buckets around q (the walk's own span) hold any blob,
  // from the bitmap bm (the arena's 64 words, in LDS): every lane tests one bucket
  __device__ bool blobs_near(Rect q, const uint64_t *bm) const {
    if (!any_blobs() || q.x1 < q.x0 || q.y1 < q.y0) return false;
    const Span g = grid_span(q, 1, d.cols, d.cshift);
    const int w = g.bx1 - g.bx0 + 1, nb = w * (g.by1 - g.by0 + 1);
    bool any = false;
    for (int i = threadIdx.x & 63; i < nb; i += 64) {
      const int b = (g.by0 + i / w) * g.stride + g.bx0 + i % w;
      any |= (bm[b >> 6] >> (b & 63)) & 1;
    }
    return __ballot(any) != 0;
  }
  // order of a cell's food list: pellets by creation sequence, then blobs
  __device__ static int64_t order_key(int j, int64_t sq) { return sq | (blob(j) ? (1ll << 62) : 0); }
};
// reservation key: higher round wins, within a round the lower priority wins.
// Rounds are global per arena and only grow (ArenaCtl::food_round), so stale
// keys of earlier phases never need clearing.
__device__ __forceinline__ uint64_t food_key(uint32_t round, uint32_t prio) {
  return ((uint64_t)round << 32) | (0xFFFFFFFFull - prio);
}
constexpr uint8_t kOverflow = 255;

// wave-level helpers (one player per wavefront; no block barriers inside)
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// For every cell, the foods it could possibly eat this phase (R set, pellets
// then blobs, each by creation sequence) and the round-1 reservation.  One
// wavefront per player: lanes scan the candidate buckets in parallel,
// ballot-compact into LDS, rank by (kind, sequence).  Cells with more than
// PREP_CAND candidates or FCAP foods in reach reserve everything they may touch
// with a key that dominates all rounds and are resolved by the serial pass.
constexpr int PREP_CAND = 128;
constexpr int PREP_WAVES = 1;  // wavefronts per player (wave h takes cells h, h + PREP_WAVES, ...; 2 measured slower)
// C4 tiles: a cell whose boxes reach beyond the held pellets is EXCLUDED -- it
// reserves what it can see with a key that dominates every round and never eats
// here; cells sharing a food with it go to the serial pass, which lets the
// higher-priority ones eat and TAINTS the rest (left undone, resolved by a later
// pass once the owners' outcomes arrived).  Cells that cannot touch a held food
// are skipped.  resume: only cells not yet final (f_done != 1) are prepared.
__device__ __forceinline__ double tile_rall() { return sqrt(kMaxMass / kPi) * (1 + 1e-9); }  // any cell's radius bound
template <bool SHARE>
__global__ void __launch_bounds__(256, 4) k_food_prep(Dev d, int rounds, int resume) {
  FLOOR(4);
  TILE_GATE(d);
  __shared__ int64_t s_seq[4][PREP_CAND];
  __shared__ double s_x[4][PREP_CAND], s_y[4][PREP_CAND], s_m[4][PREP_CAND];
  __shared__ int s_idx[4][PREP_CAND];
  __shared__ uint8_t s_sel[4][PREP_CAND];
  __shared__ uint64_t s_bm[4][64];  // each wave's arena blob bitmap (blob_grid_place)
  // blocks [0, A) when not resuming first run the player-cell grid's scan for
  // arena blockIdx.x (cgrid_scan_block; read by the commit round), then their
  // players: as extra blocks they were the 1025th block of a launch whose 1024
  // fill the GPU once, and started ~5 us late
  if (!resume && (int)blockIdx.x < d.A) cgrid_scan_block(d, blockIdx.x);
  PT_BEGIN(0);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wi = xcd_block(blockIdx.x, gridDim.x) * 4 + w, gp = wi / PREP_WAVES,
            h = wi - gp * PREP_WAVES;
  static_assert(PREP_WAVES == 1, "the block's cell sharing assumes one wave per player");
  // SHARE (Greedy populations, many multi-cell players): a block's four players
  // share their further cells -- a wave prepares its player's first cell, then
  // claims cells 1 .. n-1 of its own player and of the block's other players of
  // the same arena (q_next: LDS claim counters), so a multi-cell player's cells
  // run side by side on the waves whose players had one (cells are independent
  // here: each reserves with its own priority).  A wave that reads a count before
  // its owner published it skips that player; the owner then claims its cells
  // itself.  (Under the random population few players have several cells and the
  // claims cost more than they save: ~1.5 us on this kernel, r05 v41.)
  __shared__ int q_n[4], q_next[4], q_a[4];
  if constexpr (SHARE) {
    if (lane == 0) {
      q_n[w] = 0;
      q_next[w] = 1;  // (cell 0: its owner, unclaimed)
    }
    __syncthreads();
  }
  if (gp < d.NP && gp % d.B == 0 && h == 0 && lane == 0) d.ctl[gp / d.B].food_undone[1] = 0;  // round 1's failure count
  if (gp >= d.NP) return;
  // this wave's first list row rides the liveness / count load round (the row
  // exists whatever the count: h < PREP_WAVES <= kMaxCells)
  const int s_first = uni((int)d.p_list[h * d.NP + gp]);
  s_bm[w][lane] = d.bmap[(size_t)(gp / d.B) * 64 + lane];  // (read after the pellet walk: its waits cover it)
  const bool alive = d.p_alive[gp];
  const int NP = d.NP, a = gp / d.B;
  Food F(d, a);
  const uint32_t base = d.ctl[a].food_round;
  const int n0 = uni(d.p_ncells[gp]);  // (wave-uniform values kept in SGPRs: 4 waves per SIMD fit in 128 VGPRs)
  const int n = alive ? n0 : 0;
  if (SHARE && lane == 0) {
    q_a[w] = a;
    __hip_atomic_store(&q_n[w], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  PT_MARK(0, 1);
  // cell k of player gpc (arena a), pool index ci
  auto prep_cell = [&](const int gpc, const int k, const size_t ci) {
    const int p = gpc - a * d.B;
    uint32_t prio = (uint32_t)p * kMaxCells + k;
    const size_t kc = (size_t)k * NP + gpc;  // (food counts and lists by list position: see food_commit_player)
    if (resume && d.f_done[ci] == 1) return;  // final (here or by its owner's message)
    double x = uni(d.c_x[ci]), y = uni(d.c_y[ci]), m = uni(d.c_m[ci]), r = uni(d.c_r[ci]);
    int64_t cseq = uni(d.c_seq[ci]);
    PT_MARK(0, 2);
    Rect q = uni(footprint(x, y, r, d.size));
    if (d.tiled && !tile_near_rect(d, rect_grow(footprint(x, y, fmax(r, tile_rall()), d.size), 1, d.cols), 2)) {
      if (lane == 0) {  // cannot compete for any held food: its owner decides it
        d.f_cnt[kc] = 0;
        d.f_done[ci] = 2;
      }
      return;
    }
    int cnt = 0;
    double lsum = 0;
    auto visit = [&](bool valid, int j) {
      bool keep = false;
      double fx = 0, fy = 0, fm = 0;
      int64_t fsq = 0;
      if (valid) {
        F.load(j, fx, fy, fm, fsq);
        // (a pellet's liveness: every pellet in the store and the staging list is
        // alive when a tick's first eat pass begins -- the closing update drops the
        // eaten, tick_zero clears the staged records' flags -- so only a later pass
        // of a tiled tick, after other tiles' kills arrived, loads it)
        keep = (!resume || F.alive(j)) && rect_hit(footprint(fx, fy, pellet_radius(fm), d.size), q);
      }
      unsigned long long bal = __ballot(keep);
      int slot = cnt + __popcll(bal & ((1ull << lane) - 1));
      if (keep) {
        lsum += fm;
        if (slot < PREP_CAND) {
          s_seq[w][slot] = Food::order_key(j, fsq);
          s_x[w][slot] = fx;
          s_y[w][slot] = fy;
          s_m[w][slot] = fm;
          s_idx[w][slot] = j;
        }
      }
      cnt += __popcll(bal);
    };
    F.walk_pellets(q, visit);
    PT_MARK(0, 3);
    // The blob turn's candidates are the blobs hashed in the buckets of the
    // cell's box AFTER its pellet turn (field.py:215-222): walk the box of the
    // largest radius the pellets can give (the eat loop applies the exact box).
    const double Rp = fmax(r, radius_of(py_min(kMaxMass, (m + wave_sum(lsum)) * (1 + 1e-9))) * (1 + 1e-9));
    const Rect qb = uni(footprint(x, y, Rp, d.size));
    auto visit_b = [&](bool valid, int j) {  // as visit, against the blob-turn box bound
      bool keep = false;
      double fx = 0, fy = 0, fm = 0;
      int64_t fsq = 0;
      if (valid) {  // the record and the liveness in one round of loads
        F.load(j, fx, fy, fm, fsq);
        // a blob's own ejecter cell skips it (field.py:219)
        keep = F.alive(j) && F.ej(j) != cseq && rect_hit(footprint(fx, fy, F.rad(j, fm), d.size), qb);
      }
      unsigned long long bal = __ballot(keep);
      int slot = cnt + __popcll(bal & ((1ull << lane) - 1));
      if (keep) {
        lsum += fm;
        if (slot < PREP_CAND) {
          s_seq[w][slot] = Food::order_key(j, fsq);
          s_x[w][slot] = fx;
          s_y[w][slot] = fy;
          s_m[w][slot] = fm;
          s_idx[w][slot] = j;
        }
      }
      cnt += __popcll(bal);
    };
    if (F.blobs_near(qb, s_bm[w])) F.walk_blobs(qb, visit_b);  // (most boxes hold no blob: no row round)
    PT_MARK(0, 4);
    // upper bound of the mass / radius this cell can reach while eating (grow is monotone);
    // before its first bite the radius may still be the stale pre-eject one (cell.py:90-94)
    double sum = wave_sum(lsum);
    double M = uni(py_min(kMaxMass, (m + sum) * (1 + 1e-9)));
    double Rm = uni(fmax(r, radius_of(M)) * (1 + 1e-9));
    wave_sync_lds();
    if (d.tiled && (!(tile_holds_rect(d, rect_grow(q, 1, d.cols)) && tile_holds_rect(d, rect_grow(qb, 1, d.cols))) ||
                    ((d.tile_flags & AIGAR_TILE_OWNED_ONLY) && !tile_owns(d, x, y)))) {
      const uint64_t key = food_key(base + rounds + 2, prio);  // excluded: dominates overflow keys too
      const Rect qm = footprint(x, y, fmax(r, tile_rall()), d.size);
      if (lane == 0) {
        d.f_cnt[kc] = kOverflow;
        d.f_done[ci] = 2;
      }
      F.walk_pellets(q, [&](bool valid, int j) {
        if (valid && F.alive(j) && rect_hit(footprint(F.x(j), F.y(j), F.r(j), d.size), q))
          atomicMax((unsigned long long *)F.owner(j), (unsigned long long)key);
      });
      F.walk_blobs(qm, [&](bool valid, int j) {
        if (valid && F.alive(j) && F.ej(j) != cseq && rect_hit(footprint(F.x(j), F.y(j), F.r(j), d.size), qm))
          atomicMax((unsigned long long *)F.owner(j), (unsigned long long)key);
      });
      return;
    }
    int nsel = 0;
    bool ovf = cnt > PREP_CAND;
    if (!ovf) {
      for (int i0 = 0; i0 < cnt; i0 += 64) {
        int i = i0 + lane;
        bool sel = false;
        if (i < cnt) {
          double fx = s_x[w][i], fy = s_y[w][i];
          sel = (M > 1.25 * s_m[w][i]) && ((x - fx) * (x - fx) + (y - fy) * (y - fy) < Rm * Rm);
          s_sel[w][i] = sel;
        }
        nsel += __popcll(__ballot(sel));
      }
      ovf = nsel > FCAP;
    }
    wave_sync_lds();
    PT_MARK(0, 5);
    if (ovf) {  // reserve everything the cell may touch, resolved serially in priority order
      uint64_t key = food_key(base + rounds + 1, prio);
      if (lane == 0) {
        d.f_cnt[kc] = kOverflow;
        d.f_done[ci] = 0;
        int wi = atomicAdd(&d.ctl[a].n_pend, 1);  // straight to the serial pass
        if (wi < d.Wcap) {
          d.work[(size_t)a * d.Wcap + wi] = (int)ci;
          d.work2[(size_t)a * d.Wcap + wi] = (int)prio;
        } else {
          set_err(d, a, ERR_WORK_CAP);
        }
      }
      F.walk_pellets(q, [&](bool valid, int j) {
        if (valid && F.alive(j) && rect_hit(footprint(F.x(j), F.y(j), F.r(j), d.size), q))
          atomicMax((unsigned long long *)F.owner(j), (unsigned long long)key);
      });
      F.walk_blobs(qb, [&](bool valid, int j) {
        if (valid && F.alive(j) && rect_hit(footprint(F.x(j), F.y(j), F.r(j), d.size), qb))
          atomicMax((unsigned long long *)F.owner(j), (unsigned long long)key);
      });
      return;
    }
    int *lst = d.f_list + kc * FCAP;
    uint64_t key = food_key(base + 1, prio);
    for (int i0 = 0; i0 < cnt; i0 += 64) {
      int i = i0 + lane;
      if (i < cnt && s_sel[w][i]) {
        int64_t sq = s_seq[w][i];
        int rk = 0;
        for (int jj = 0; jj < cnt; jj++) rk += (s_sel[w][jj] && s_seq[w][jj] < sq);
        lst[rk] = s_idx[w][i];
        atomicMax((unsigned long long *)F.owner(s_idx[w][i]), (unsigned long long)key);
      }
    }
    if (lane == 0) {
      d.f_cnt[kc] = (uint8_t)nsel;
      d.f_done[ci] = (nsel == 0);
    }
    wave_sync_lds();
    PT_MARK(0, 6);
  };
  // its own first cell (the slot arrived with the count) unclaimed, then claims of
  // the block's further cells, its own player's first; one call site (two
  // inlined copies of the cell spilled VGPRs)
  if constexpr (!SHARE) {  // the player's cells one after the other
    for (int k = 0; k < n; k++) prep_cell(gp, k, (size_t)(k == 0 ? s_first : uni((int)d.p_list[k * NP + gp])) * NP + gp);
    return;
  }
  const int g0 = xcd_block(blockIdx.x, gridDim.x) * 4;
  int gpc = gp, kc = n > 0 ? 0 : -1, sc = s_first;
  int step = 0;
  for (; step <= 4 * kMaxCells; step++) {
    if (kc < 0) {  // the next claim: a player of the block (same arena) with a cell left
      for (int t = 0; t < 4 && kc < 0; t++) {
        const int w2 = (w + t) & 3;
        const int n2 = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&q_n[w2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (n2 <= 1 || __builtin_amdgcn_readfirstlane(q_a[w2]) != a) continue;
        const int leader = __ffsll((long long)__ballot(1)) - 1;  // (the claim by the first active lane)
        int k = 0;
        if (lane == leader) k = atomicAdd(&q_next[w2], 1);
        k = __builtin_amdgcn_readlane(k, leader);
        if (k >= n2) continue;
        gpc = __builtin_amdgcn_readfirstlane(g0 + w2);
        kc = k;
        sc = __builtin_amdgcn_readfirstlane((int)d.p_list[k * NP + gpc]);
      }
      if (kc < 0) break;
    }
    prep_cell(gpc, kc, (size_t)sc * NP + gpc);
    kc = -1;
  }
  // (a block holds at most 4 x kMaxCells cells: the bound is never reached unless the
  // claim counters are corrupt -- then cells went unprepared, which must not pass silently)
  if (step > 4 * kMaxCells && lane == wave_leader()) set_err(d, a, ERR_CLAIM);
}
// one eaten food: the event (in its reference phase), kill, growth
// (eatCell -> adjustCellSize -> grow, field.py:327-344)
// (tiles: only the cell's owner logs and reports it; fx, fy locate a pellet on the other tiles)
__device__ __forceinline__ void food_eat(const Dev &d, const Food &F, int a, int j, uint32_t prio, int t,
                                         int64_t cseq, int64_t fseq, double fm, double &m, double &r, int &eaten,
                                         bool own, double fx, double fy) {
  const bool bl = Food::blob(j);
  if (own) {
    ev_push(d, a, bl ? PH_BLOB : PH_PELLET, ((uint64_t)prio << 16) | (uint64_t)t, bl ? 7 : 6, cseq, fseq);
    if (d.tiled) {
      if (bl) tile_out(d, TR_BLOB, j & ~kBlobBit, fseq, 0.0, 0.0);
      else tile_out(d, TR_PELLET, 0, fseq, fx, fy);
    }
  }
  m = grow_mass(m, fm);
  r = radius_of(m);
  F.kill(j);
  eaten += bl ? 0 : 1;
}
// A committing cell's foods, kTailRegs at a time: the liveness and record of a
// batch in one round of loads (the cell holds every reservation, so nothing
// else eats them this round), the eats decided in list order on registers,
// and the batch's pellet kills noted with one atomic (the kill list takes them
// in any order: k_spawn_plan sorts it).  The first batch arrives preloaded.
struct FoodBatch {
  int j[kTailRegs];
  bool al[kTailRegs];
  double x[kTailRegs], y[kTailRegs], m[kTailRegs], r[kTailRegs];
  int64_t sq[kTailRegs];
  __device__ void load(const Dev &d, const Food &F, const int *jv, int n) {
#pragma unroll
    for (int k = 0; k < kTailRegs; k++) {
      j[k] = jv[k];
      al[k] = false;
      x[k] = y[k] = m[k] = r[k] = 0;
      sq[k] = 0;
      if (k < n) {
        al[k] = F.alive(j[k]);
        F.load(j[k], x[k], y[k], m[k], sq[k]);
        r[k] = Food::blob(j[k]) ? d.b_r[F.gb(j[k])] : 0.0;  // (a pellet's radius follows from its mass)
      }
    }
  }
};
// returns the cell's radius if it ate, else 0
struct EaterIn {  // a committing cell's state, loaded with its reservation keys
  double x, y, m, r;
  int64_t seq;
};
__device__ double food_eat_loop(const Dev &d, const Food &F, int a, size_t ci, const EaterIn &cell, uint32_t prio,
                                const int *lst, int cnt, FoodBatch &fb) {
  const double x = cell.x, y = cell.y;
  double m = cell.m, r = cell.r;
  const int64_t cseq = cell.seq;
  const bool own = tile_owns(d, x, y);
  int eaten = 0;
  bool blobs = false, ate = false;
  Rect qb{};
  for (int t0 = 0; t0 < cnt; t0 += kTailRegs) {
    if (t0 > 0) {
      int jv[kTailRegs];
#pragma unroll
      for (int k = 0; k < kTailRegs; k++) jv[k] = t0 + k < cnt ? lst[t0 + k] : 0;
      fb.load(d, F, jv, cnt - t0);
    }
    int kp[kTailRegs], nkp = 0;
#pragma unroll
    for (int k = 0; k < kTailRegs; k++) {
      kp[k] = -1;
      const int t = t0 + k, j = fb.j[k];
      if (t >= cnt) continue;
      if (Food::blob(j) && !blobs) {  // the blob turn: candidates from the box after the pellet turn
        blobs = true;
        qb = footprint(x, y, r, d.size);
      }
      if (!fb.al[k]) continue;
      const double fm = fb.m[k], fx = fb.x[k], fy = fb.y[k], fr = Food::blob(j) ? fb.r[k] : pellet_radius(fm);
      if (blobs && !rect_hit(footprint(fx, fy, fr, d.size), qb)) continue;
      if (!(overlap(x, y, m, r, fx, fy, fm, fr) && can_eat(m, fm))) continue;
      // eatCell (field.py:337-344): the event, the kill, the growth
      if (own) {
        const bool bl = Food::blob(j);
        ev_push(d, a, bl ? PH_BLOB : PH_PELLET, ((uint64_t)prio << 16) | (uint64_t)t, bl ? 7 : 6, cseq, fb.sq[k]);
        if (d.tiled) {
          if (bl) tile_out(d, TR_BLOB, j & ~kBlobBit, fb.sq[k], 0.0, 0.0);
          else tile_out(d, TR_PELLET, 0, fb.sq[k], fx, fy);
        }
      }
      m = grow_mass(m, fm);
      r = radius_of(m);
      F.mark_dead(j);
      if (!Food::blob(j)) {
        eaten++;
        if (j < F.n0) {
          kp[k] = j;
          nkp++;
        }
      }
      ate = true;
    }
    if (nkp) {  // note_kill for the batch
      int b = atomicAdd(&d.ctl[a].n_kill, nkp);
#pragma unroll
      for (int k = 0; k < kTailRegs; k++)
        if (kp[k] >= 0) {
          if (b < d.Pcap) d.kill_list[(size_t)a * d.Pcap + b] = kp[k];
          else set_err(d, a, ERR_PELLET_CAP);
          b++;
        }
    }
  }
  d.c_m[ci] = m;
  d.c_r[ci] = r;
  if (d.tiled && own && ate) tile_out(d, TR_CELL, (int32_t)ci, cseq, m, r);
  if (eaten) atomicAdd(&d.ctl[a].n_pel_eaten, eaten);
  return ate ? r : 0.0;
}
// one player's cells in reservation round `round`; returns the largest radius
// of its cells that ate (0: none) -- the player-cell grid's radius bound
__device__ double food_commit_player(const Dev &d, int gp, int round, int last, int place PT_PARAMS) {
  const int NP = d.NP, a = gp / d.B, p = gp - a * d.B;
  ArenaCtl &c = d.ctl[a];
  // round r reads how many cells failed round r-1 (nothing left: skip), counts
  // its own failures, and clears the counter round r+1 will use.
  // ONE load round: liveness, cell count, the list's first row, and the first
  // cell's food count and list -- k_food_prep keeps those by list position
  // (k * NP + gp), so they need no slot first (FCAP slots exist; entries past
  // the count are never used)
  const bool alive = d.p_alive[gp];
  const int n = d.p_ncells[gp];
  const int s_first = d.p_list[gp];
  const int cnt_first = d.f_cnt[gp];
  int l4_first[kTailRegs];
#pragma unroll
  for (int t = 0; t < kTailRegs; t++) l4_first[t] = d.f_list[(size_t)gp * FCAP + t];
  if (place && alive) cgrid_place_player(d, gp, n);  // (independent of the eats: its loads overlap theirs)
  if (round > 1 && c.food_undone[(round - 1) % 3] == 0) return 0;
  if (p == 0) c.food_undone[(round + 1) % 3] = 0;
  if (!alive) return 0;
  double rgrow = 0;
  Food F(d, a);
  for (int k = 0; k < n; k++) {
    const size_t kc = (size_t)k * NP + gp;
    const int *lst = d.f_list + kc * FCAP;
    int slot = s_first, cnt = cnt_first, l4[kTailRegs];
#pragma unroll
    for (int t = 0; t < kTailRegs; t++) l4[t] = l4_first[t];
    if (k > 0) {  // (a further cell: its slot, count and list in one round)
      slot = d.p_list[kc];
      cnt = d.f_cnt[kc];
#pragma unroll
      for (int t = 0; t < kTailRegs; t++) l4[t] = lst[t];
    }
    PT_MARKW(4, 2);
    if (cnt == 0 || cnt == kOverflow) continue;  // nothing to eat / already in the serial work list (k_food_prep)
    const size_t ci = (size_t)slot * NP + gp;
    uint32_t prio = (uint32_t)p * kMaxCells + k;
    bool own = true;
    FoodBatch fb;
    EaterIn cell;
    bool done;
    {  // ONE round: the cell's done flag and state, every reservation key of the
       // list (the first entries) and the first entries' records, which the eats
       // use if it won
      done = d.f_done[ci];
      cell.x = d.c_x[ci];
      cell.y = d.c_y[ci];
      cell.m = d.c_m[ci];
      cell.r = d.c_r[ci];
      cell.seq = d.c_seq[ci];
      uint64_t key = food_key(d.ctl[a].food_round + round, prio);
      uint64_t kw[kTailRegs];
#pragma unroll
      for (int t = 0; t < kTailRegs; t++) kw[t] = t < cnt ? *F.owner(l4[t]) : key;
      fb.load(d, F, l4, cnt);
#pragma unroll
      for (int t = 0; t < kTailRegs; t++) own &= kw[t] == key;
      if (done) continue;  // (an earlier round's, or a tile's final cell)
      for (int t = kTailRegs; t < cnt && own; t++) own = (*F.owner(lst[t]) == key);
    }
    PT_MARKW(4, 3);
    if (own) {
      rgrow = fmax(rgrow, food_eat_loop(d, F, a, ci, cell, prio, lst, cnt, fb));
      d.f_done[ci] = 1;
      PT_MARKW(4, 4);
    } else if (!last) {
      // reserve for the next round right away.  Safe without a separate pass: a
      // cell that still has to wait for a lower-priority neighbour made its
      // round-(r+1) reservation no later than this kernel, so the neighbour's
      // key dominates at the next commit; a cell whose round-r check races with
      // a round-(r+1) key only loses a round (it re-reserves and wins next time).
      uint64_t key = food_key(d.ctl[a].food_round + round + 1, prio);
      for (int t = 0; t < cnt; t++) atomicMax((unsigned long long *)F.owner(lst[t]), (unsigned long long)key);
      atomicAdd(&c.food_undone[round % 3], 1);
    } else {
      int w = atomicAdd(&d.ctl[a].n_pend, 1);
      if (w < d.Wcap) {
        d.work[(size_t)a * d.Wcap + w] = (int)ci;
        d.work2[(size_t)a * d.Wcap + w] = (int)prio;
      } else {
        set_err(d, a, ERR_WORK_CAP);
      }
    }
  }
  return rgrow;
}
__device__ void food_serial_body(const Dev &d, int a, int64_t *scr_k, int *scr_v, int rounds);
// fold (last round only): the serial pass runs in the last of the player blocks
// (wave 0, arena after arena; the grid's extra blocks do not take part)
// place: the player-cell grid's placement (round 1 of a tick's first eat pass)
__global__ void __launch_bounds__(256) k_food_commit(Dev d, int round, int last, int64_t *scr_k, int *scr_v,
                                                     int rounds, int fold, int place) {
  FLOOR(5);
  TILE_GATE(d);
  const int ncommit = (d.NP + 255) / 256;
  PT_BEGIN(4);
  const int gp = GTID;
  const double rg = gp < d.NP ? food_commit_player(d, gp, round, last, place PT_ARGS) : 0.0;
  PT_MARK(4, round < 7 ? round : 7);
  wave_atomic_max_pos(&d.ctl[min(gp, d.NP - 1) / d.B].rmax_cell, rg);
  PT_MARK(4, 5);
  if (fold && last_block(d.ticket + 1, ncommit, false)) {  // (acquires only when a cell waits: as k_merge_pv)
    __shared__ int s_work;
    if (threadIdx.x == 0) {
      int w = 0;
      for (int a = 0; a < d.A; a++) w |= agent_load(&d.ctl[a].n_pend);
      s_work = w;
    }
    __syncthreads();
    agent_acquire_block(s_work != 0);
    if (threadIdx.x < 64)
      for (int a = 0; a < d.A; a++) food_serial_body(d, a, scr_k, scr_v, rounds);
    PT_MARK(4, 6);
  }
}
// Cells the reservation rounds could not settle, in priority order (player,
// list position), one wavefront per arena.  The sequential eat loop runs on
// all lanes uniformly; each cell's candidates are gathered lane-parallel with
// their state into LDS (within one cell's turn only that cell changes them).
constexpr int FS_CAP = 512;
__device__ void food_serial_body(const Dev &d, int a, int64_t *scr_k, int *scr_v, int rounds) {
  __shared__ int64_t s_key[FS_CAP];
  __shared__ int s_val[FS_CAP], s_srt[FS_CAP];
  __shared__ double s_x[FS_CAP], s_y[FS_CAP], s_m[FS_CAP], s_r[FS_CAP];
  const int lane = threadIdx.x & 63;
  ArenaCtl &c = d.ctl[a];
  const int nw = min(agent_load(&c.n_pend), d.Wcap);
  const uint32_t excl_round = c.food_round + rounds + 2;  // tiles: excluded / tainted keys (k_food_prep)
  wave_fence();
  if (lane == 0) {
    c.n_pend = 0;
    c.stat[2] += nw;
    c.food_round += rounds + 2;  // next phase's keys dominate every key written in this one
  }
  if (nw == 0) return;
  Food F(d, a);
  int *w = d.work + (size_t)a * d.Wcap;
  int *wp = d.work2 + (size_t)a * d.Wcap;
  if (nw <= FS_CAP) {  // priority order: rank sort in LDS (priorities are unique)
    for (int k = lane; k < nw; k += 64) {
      s_val[k] = w[k];
      s_key[k] = wp[k];
    }
    wave_fence();
    for (int k = lane; k < nw; k += 64) {
      int64_t key = s_key[k];
      int rk = 0;
      for (int y = 0; y < nw; y++) rk += s_key[y] < key;
      s_srt[rk] = k;
    }
    wave_fence();
    for (int k = lane; k < nw; k += 64) {  // (w, wp are free now: write back sorted)
      w[k] = s_val[s_srt[k]];
      wp[k] = (int)s_key[s_srt[k]];
    }
  } else if (lane == 0) {
    int64_t *ck = scr_k + (size_t)a * d.Wcap;
    for (int k = 0; k < nw; k++) ck[k] = wp[k];
    isort_kv(ck, w, nw);
    for (int k = 0; k < nw; k++) wp[k] = (int)ck[k];
  }
  wave_fence();
  const unsigned long long lt = (1ull << lane) - 1;
  for (int wi = 0; wi < nw; wi++) {
    const size_t ci = (size_t)w[wi];
    const uint32_t prio = (uint32_t)wp[wi];
    const double x = d.c_x[ci], y = d.c_y[ci];
    double m = d.c_m[ci], r = d.c_r[ci];
    const int64_t cseq = d.c_seq[ci];
    const bool own = tile_owns(d, x, y);
    if (d.tiled) {
      // taint: a higher-priority excluded or tainted cell may eat one of this cell's
      // foods; its outcome is not known here, so neither is this cell's (left undone)
      const Rect q = footprint(x, y, r, d.size), qm = footprint(x, y, fmax(r, tile_rall()), d.size);
      bool taint = false;
      Rect box = q;
      auto check = [&](bool valid, int j) {
        bool hit = valid && F.alive(j) && F.ej(j) != cseq && rect_hit(footprint(F.x(j), F.y(j), F.r(j), d.size), box);
        if (hit) {
          const uint64_t w = *F.owner(j);
          hit = (uint32_t)(w >> 32) == excl_round && (0xFFFFFFFFu - (uint32_t)w) < prio;
        }
        if (__ballot(hit)) taint = true;
      };
      auto mark = [&](bool valid, int j) {
        if (valid && F.alive(j) && F.ej(j) != cseq && rect_hit(footprint(F.x(j), F.y(j), F.r(j), d.size), box))
          atomicMax((unsigned long long *)F.owner(j), (unsigned long long)food_key(excl_round, prio));
      };
      F.walk_pellets(q, check);
      box = qm;
      F.walk_blobs(qm, check);
      if (taint) {
        box = q;
        F.walk_pellets(q, mark);
        box = qm;
        F.walk_blobs(qm, mark);
        wave_fence();
        continue;
      }
    }
    int eaten = 0, t_base = 0;
    bool ate = false;
    for (int kind = 0; kind < 2; kind++) {  // pellet turn, then blob turn (box after the pellets)
    const Rect q = footprint(x, y, r, d.size);
    int nc = 0;
    auto gather = [&](bool valid, int j) {
      double fx = 0, fy = 0, fm = 0, fr = 0;
      bool keep = valid && F.alive(j) && F.ej(j) != cseq;
      if (keep) {
        fx = F.x(j);
        fy = F.y(j);
        fm = F.m(j);
        fr = F.r(j);
        keep = rect_hit(footprint(fx, fy, fr, d.size), q);
      }
      unsigned long long bal = __ballot(keep);
      int slot = nc + __popcll(bal & lt);
      if (keep && slot < FS_CAP) {
        s_key[slot] = Food::order_key(j, F.seq(j));
        s_val[slot] = j;
        s_x[slot] = fx;
        s_y[slot] = fy;
        s_m[slot] = fm;
        s_r[slot] = fr;
      }
      nc += __popcll(bal);
    };
    if (kind == 0) F.walk_pellets(q, gather);
    else F.walk_blobs(q, gather);
    if (nc > FS_CAP) {
      set_err(d, a, ERR_CAND_CAP);
      nc = FS_CAP;
    }
    wave_fence();
    for (int k = lane; k < nc; k += 64) {  // candidate order: pellets, then blobs, each by creation sequence
      int64_t key = s_key[k];
      int rk = 0;
      for (int y = 0; y < nc; y++) rk += s_key[y] < key;
      s_srt[rk] = k;
    }
    wave_fence();
    for (int t = 0; t < nc; t++) {  // food_eat_loop, on the turn-start snapshot
      const int k = s_srt[t];
      const double fm = s_m[k];
      if (!(overlap(x, y, m, r, s_x[k], s_y[k], fm, s_r[k]) && can_eat(m, fm))) continue;
      const int j = s_val[k];
      const int64_t fseq = s_key[k] & ~(1ll << 62);
      ate = true;
      if (lane == 0) {
        food_eat(d, F, a, j, prio, t_base + t, cseq, fseq, fm, m, r, eaten, own, s_x[k], s_y[k]);
      } else {
        m = grow_mass(m, fm);
        r = radius_of(m);
      }
    }
    t_base += nc;
    wave_fence();  // this sub-turn's kills are read by the next gather
    }
    if (lane == 0) {
      d.c_m[ci] = m;
      d.c_r[ci] = r;
      d.f_done[ci] = 1;
      if (d.tiled && own && ate) tile_out(d, TR_CELL, (int32_t)ci, cseq, m, r);
      if (eaten) atomicAdd(&d.ctl[a].n_pel_eaten, eaten);
      atomic_max_pos(&c.rmax_cell, r);  // (radii only grow while eating)
    }
    wave_fence();  // kills and the new mass are read by the next cell's gather
  }
}
__global__ void __launch_bounds__(64) k_food_serial(Dev d, int64_t *scr_k, int *scr_v, int rounds) {
  TILE_GATE(d);
  food_serial_body(d, blockIdx.x, scr_k, scr_v, rounds);
}

// ------------------------------------------------------------ T16 player <- player
__device__ __forceinline__ Rect cell_rect(const Dev &d, size_t ci) { return footprint(d.c_x[ci], d.c_y[ci], d.c_r[ci], d.size); }

// getSpawnPos's occupancy (field.py:283-301: the buckets of the player hash that
// hold a cell) as a per-bucket cell count plus the bit words spawn_pos scans.
// k_pp_active adds every live cell's footprint; the pp pass keeps it exact
// (a removed cell leaves its buckets, a grown one adds the buckets it reached),
// so it describes the cells left when spawnStuff runs.  One bucket per lane.
__device__ __forceinline__ void occ_add(const Dev &d, int a, Rect q) {
  int *cnt = d.occ_cnt + (size_t)a * d.H;
  unsigned long long *occ = d.occ + (size_t)a * d.occ_words;
  const int w = q.x1 - q.x0 + 1, n = w * (q.y1 - q.y0 + 1);
  for (int t = threadIdx.x & 63; t < n; t += 64) {
    const int b = (q.y0 + t / w) * d.cols + q.x0 + t % w;
    atomicAdd(&cnt[b], 1);
    atomicOr(&occ[b >> 6], 1ull << (b & 63));
  }
}
// the buckets of q that old does not hold (old inside q: a radius grew in place)
__device__ __forceinline__ void occ_grow(const Dev &d, int a, Rect old, Rect q) {
  int *cnt = d.occ_cnt + (size_t)a * d.H;
  unsigned long long *occ = d.occ + (size_t)a * d.occ_words;
  const int w = q.x1 - q.x0 + 1, n = w * (q.y1 - q.y0 + 1);
  for (int t = threadIdx.x & 63; t < n; t += 64) {
    const int bx = q.x0 + t % w, by = q.y0 + t / w;
    if (bx >= old.x0 && bx <= old.x1 && by >= old.y0 && by <= old.y1) continue;
    const int b = by * d.cols + bx;
    if (atomicAdd(&cnt[b], 1) == 0) atomicOr(&occ[b >> 6], 1ull << (b & 63));
  }
}
__device__ __forceinline__ void occ_remove(const Dev &d, int a, Rect q) {
  int *cnt = d.occ_cnt + (size_t)a * d.H;
  unsigned long long *occ = d.occ + (size_t)a * d.occ_words;
  const int w = q.x1 - q.x0 + 1, n = w * (q.y1 - q.y0 + 1);
  for (int t = threadIdx.x & 63; t < n; t += 64) {
    const int b = (q.y0 + t / w) * d.cols + q.x0 + t % w;
    if (atomicSub(&cnt[b], 1) == 1) atomicAnd(&occ[b >> 6], ~(1ull << (b & 63)));
  }
}

// The pp pass's occupancy updates, deferred: counts by non-returning atomics
// (no round trip per eat), the touched bit words marked in an LDS bitmap and
// rebuilt from the final counts once the pass is over (occ_rebuild_dirty).
// Counts are sums, so the order of the updates does not matter.
constexpr int OCC_DW = 64;  // dirty-word bitmap: up to 2048 occupancy words (C3: 900)
#ifndef AIGAR_OCC_BATCH
#define AIGAR_OCC_BATCH 1
#endif
__device__ __forceinline__ void occ_mark(uint32_t *dirty, int b) {
  const int wd = b >> 6;
  atomicOr(&dirty[wd >> 5], 1u << (wd & 31));
}
__device__ __forceinline__ void occ_remove_def(const Dev &d, int a, Rect q, uint32_t *dirty) {
  int *cnt = d.occ_cnt + (size_t)a * d.H;
  const int w = q.x1 - q.x0 + 1, n = w * (q.y1 - q.y0 + 1);
  for (int t = threadIdx.x & 63; t < n; t += 64) {
    const int b = (q.y0 + t / w) * d.cols + q.x0 + t % w;
    (void)__hip_atomic_fetch_add(&cnt[b], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    occ_mark(dirty, b);
  }
}
__device__ __forceinline__ void occ_grow_def(const Dev &d, int a, Rect old, Rect q, uint32_t *dirty) {
  int *cnt = d.occ_cnt + (size_t)a * d.H;
  const int w = q.x1 - q.x0 + 1, n = w * (q.y1 - q.y0 + 1);
  for (int t = threadIdx.x & 63; t < n; t += 64) {
    const int bx = q.x0 + t % w, by = q.y0 + t / w;
    if (bx >= old.x0 && bx <= old.x1 && by >= old.y0 && by <= old.y1) continue;
    const int b = by * d.cols + bx;
    (void)__hip_atomic_fetch_add(&cnt[b], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    occ_mark(dirty, b);
  }
}
// every wave of the block: the k-th dirty word goes to wave k % waves; its 64
// counts are read at device scope (past L1) and the word is their ballot
__device__ __forceinline__ void occ_rebuild_dirty(const Dev &d, int a, const uint32_t *dirty) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int *cnt = d.occ_cnt + (size_t)a * d.H;
  unsigned long long *occ = d.occ + (size_t)a * d.occ_words;
  static_assert(OCC_DW == 64, "one bitmap word per lane");
  const uint32_t mine = dirty[lane];
  unsigned long long nz = __ballot(mine != 0);  // (usually none: no pp eat this tick)
  int k = 0;
#if AIGAR_OCC_BATCH
  // a wave's words four at a time: their count loads in one round
  int q0 = -1, q1 = -1, q2 = -1, q3 = -1;
  auto word = [&](int wd, int c) {
    const unsigned long long bits = __ballot(c > 0);
    if (lane == 0) occ[wd] = bits;
  };
  auto flush = [&]() {
    auto ld = [&](int wd) {
      const int b = wd * 64 + lane;
      return wd >= 0 && b < d.H ? __hip_atomic_load(&cnt[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    };
    const int c0 = ld(q0), c1 = ld(q1), c2 = ld(q2), c3 = ld(q3);
    if (q0 >= 0) word(q0, c0);
    if (q1 >= 0) word(q1, c1);
    if (q2 >= 0) word(q2, c2);
    if (q3 >= 0) word(q3, c3);
    q0 = q1 = q2 = q3 = -1;
  };
#endif
  while (nz) {
    const int i = __ffsll((long long)nz) - 1;
    nz &= nz - 1;
    uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)mine, i);
    while (m) {
      const int wd = i * 32 + __ffs(m) - 1;
      m &= m - 1;
      if (k++ % nw != w) continue;
#if AIGAR_OCC_BATCH
      if (q0 < 0) q0 = wd;
      else if (q1 < 0) q1 = wd;
      else if (q2 < 0) q2 = wd;
      else {
        q3 = wd;
        flush();
      }
#else
      const int b = wd * 64 + lane;
      const int c = b < d.H ? __hip_atomic_load(&cnt[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
      const unsigned long long bits = __ballot(c > 0);
      if (lane == 0) occ[wd] = bits;
#endif
    }
  }
#if AIGAR_OCC_BATCH
  if (q0 >= 0) flush();
#endif
}

// one wavefront per player: cells with an overlapping enemy cell at phase start
// (+ the player's cells into the spawn occupancy)
// (!SHARE: each wave tests its own player's cells in order)
__device__ __forceinline__ void pp_active_own(const Dev &d PT_PARAMS) {
  const int lane = threadIdx.x & 63;
  const int gp = xcd_block(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
  // C4, device-bounded eat passes: the tick may go on only if no owned cell is undone
  if (d.tiled && gp == 0 && lane == 0 && d.ctl[0].n_undone_glob != 0) atomicOr(&d.ctl[0].err, ERR_TILE_PASSES);
  if (gp >= d.NP) return;
  const int s_first = d.p_list[gp];  // (list row 0 rides the liveness / count load round)
  if (!d.p_alive[gp]) return;
  const int NP = d.NP, a = gp / d.B;
  const int *st = d.cstart + (size_t)a * (d.H + 1);
  const int *it = d.citems + (size_t)a * kMaxCells * d.B;
  int E = expand_for(d.ctl[a].rmax_cell);
  int n = d.p_ncells[gp];
  bool anyp = false;
  PT_MARK(3, 1);
  for (int k = 0; k < n; k++) {
    size_t ci = (size_t)(k == 0 ? s_first : d.p_list[k * NP + gp]) * NP + gp;
    double x = d.c_x[ci], y = d.c_y[ci], m = d.c_m[ci], r = d.c_r[ci];
    PT_MARK(3, 2);
    Rect q = footprint(x, y, r, d.size);
    occ_add(d, a, q);
    bool any = wave_any_in_grid(st, it, d.cols, q, E, [&](int e) {
      // only the LOWER-index player of a pair is marked: its turn comes first
      // and resolves the pair ("the one that can eat does", field.py:238-243).
      // The higher-index side's turn could only see a changed pair, and every
      // change re-activates it: a growth re-activates the cells overlapping the
      // grown one; a cell skipped by the live-list quirk re-activates its partners.
      if (!(d.c_flags[e] & F_ALIVE) || (int)(e % NP) <= gp) return false;
      if (!rect_hit(cell_rect(d, e), q)) return false;
      // a pair where neither side can eat stays inert until one of them grows
      double me = d.c_m[e];
      return overlap(x, y, m, r, d.c_x[e], d.c_y[e], me, d.c_r[e]) && (can_eat(m, me) || can_eat(me, m));
    }, d.cshift_c);
    if (lane == 0) d.c_active[ci] = any;
    anyp |= any;
    PT_MARK(3, 3);
  }
  if (anyp && lane == 0) {
    int w = atomicAdd(&d.ctl[a].n_pend, 1);
    if (w < d.Wcap) d.work[(size_t)a * d.Wcap + w] = gp - a * d.B;
    else set_err(d, a, ERR_WORK_CAP);
  }
}
// SHARE (Greedy populations): a block's four players share their cells as in
// k_food_prep -- a wave tests its own player's first cell, then claims the
// remaining cells of the block's players of its arena (q_next).  A one-cell
// player is queued by its own wave; for a player with more cells every tested
// cell marks q_any and counts in q_done, and the wave that tests the last one
// queues the player if marked.
template <bool SHARE>
__global__ void __launch_bounds__(256) k_pp_active(Dev d) {
  FLOOR(6);
  PT_BEGIN(3);
  if constexpr (!SHARE) {
    pp_active_own(d PT_ARGS);
    return;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g0 = xcd_block(blockIdx.x, gridDim.x) * 4, gp = g0 + w;
  __shared__ int q_n[4], q_next[4], q_done[4], q_any[4], q_a[4];
  if (lane == 0) {
    q_n[w] = 0;
    q_next[w] = 1;  // (cell 0: its owner, unclaimed)
    q_done[w] = 0;
    q_any[w] = 0;
  }
  __syncthreads();
  // C4, device-bounded eat passes: the tick may go on only if no owned cell is undone
  if (d.tiled && gp == 0 && lane == 0 && d.ctl[0].n_undone_glob != 0) atomicOr(&d.ctl[0].err, ERR_TILE_PASSES);
  if (gp >= d.NP) return;
  const int s_first = d.p_list[gp];  // (list row 0 rides the liveness / count load round)
  const bool alive = d.p_alive[gp];
  const int NP = d.NP, a = gp / d.B;
  const int *st = d.cstart + (size_t)a * (d.H + 1);
  const int *it = d.citems + (size_t)a * kMaxCells * d.B;
  const int E = expand_for(d.ctl[a].rmax_cell);
  const int n = alive ? d.p_ncells[gp] : 0;
  if (lane == 0) {
    q_a[w] = a;
    __hip_atomic_store(&q_n[w], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  PT_MARK(3, 1);
  int wc = w, kc = n > 0 ? 0 : -1, nc = n, sc = s_first;
  int step = 0;
  for (; step <= 4 * kMaxCells; step++) {
    if (kc < 0) {  // the next claim: a player of the block (same arena) with a cell left
      for (int t = 0; t < 4 && kc < 0; t++) {
        const int w2 = (w + t) & 3;
        const int n2 = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&q_n[w2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (n2 <= 1 || __builtin_amdgcn_readfirstlane(q_a[w2]) != a) continue;
        const int leader = __ffsll((long long)__ballot(1)) - 1;  // (the claim by the first active lane)
        int k = 0;
        if (lane == leader) k = atomicAdd(&q_next[w2], 1);
        k = __builtin_amdgcn_readlane(k, leader);
        if (k >= n2) continue;
        wc = w2;
        kc = k;
        nc = n2;
        sc = __builtin_amdgcn_readfirstlane((int)d.p_list[k * NP + g0 + w2]);
      }
      if (kc < 0) break;
    }
    const int gpc = __builtin_amdgcn_readfirstlane(g0 + wc);
    const size_t ci = (size_t)sc * NP + gpc;
    double x = d.c_x[ci], y = d.c_y[ci], m = d.c_m[ci], r = d.c_r[ci];
    PT_MARK(3, 2);
    Rect q = footprint(x, y, r, d.size);
    occ_add(d, a, q);
    bool any = wave_any_in_grid(st, it, d.cols, q, E, [&](int e) {
      // only the LOWER-index player of a pair is marked: its turn comes first
      // and resolves the pair ("the one that can eat does", field.py:238-243).
      // The higher-index side's turn could only see a changed pair, and every
      // change re-activates it: a growth re-activates the cells overlapping the
      // grown one; a cell skipped by the live-list quirk re-activates its partners.
      if (!(d.c_flags[e] & F_ALIVE) || (int)(e % NP) <= gpc) return false;
      if (!rect_hit(cell_rect(d, e), q)) return false;
      // a pair where neither side can eat stays inert until one of them grows
      double me = d.c_m[e];
      return overlap(x, y, m, r, d.c_x[e], d.c_y[e], me, d.c_r[e]) && (can_eat(m, me) || can_eat(me, m));
    }, d.cshift_c);
    const int leader = __ffsll((long long)__ballot(1)) - 1;
    if (lane == leader) {
      d.c_active[ci] = any;
      bool push = any;
      if (nc > 1) {
        if (any) atomicOr(&q_any[wc], 1);
        push = atomicAdd(&q_done[wc], 1) == nc - 1 &&  // (after the mark: LDS atomics of a CU apply in order)
               __hip_atomic_load(&q_any[wc], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
      }
      if (push) {
        const int wq = atomicAdd(&d.ctl[a].n_pend, 1);
        if (wq < d.Wcap) d.work[(size_t)a * d.Wcap + wq] = gpc - a * d.B;
        else set_err(d, a, ERR_WORK_CAP);
      }
    }
    PT_MARK(3, 3);
    kc = -1;
  }
  if (step > 4 * kMaxCells && lane == wave_leader()) set_err(d, a, ERR_CLAIM);  // (as in k_food_prep)
}

// removes cell e (pool index) from its player's list; returns true if the player died
__device__ __forceinline__ bool remove_cell(const Dev &d, int a, size_t e, uint64_t &order, bool writer = true) {
  const int NP = d.NP;
  int gp = (int)(e % NP);
  uint8_t slot = (uint8_t)(e / NP);
  // the count and every list row in one load round (all kMaxCells rows exist),
  // then the compacted list is written back
  uint8_t l[kMaxCells];
#pragma unroll
  for (int k = 0; k < kMaxCells; k++) l[k] = d.p_list[k * NP + gp];
  const int n = d.p_ncells[gp];
  d.c_flags[e] = 0;
  int w = 0;
#pragma unroll
  for (int k = 0; k < kMaxCells; k++)
    if (k < n && l[k] != slot) d.p_list[(w++) * NP + gp] = l[k];
  d.p_ncells[gp] = w;
  if (w == 0) {  // deletePlayerCell: last cell -> deadPlayers, setDead (field.py:386-388)
    ArenaCtl &c = d.ctl[a];
    d.p_alive[gp] = 0;
    d.p_respawn[gp] = 1;
    d.dead[(size_t)a * d.B + c.n_dead++] = gp - a * d.B;
    if (writer) ev_push(d, a, PH_PP, order, 9, gp - a * d.B, d.c_seq[e]);
    order++;
    return true;
  }
  return false;
}

__device__ __forceinline__ uint8_t active_ld(const Dev &d, size_t i) {
  return __hip_atomic_load(&d.c_active[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void active_st(const Dev &d, size_t i, uint8_t v) {
  __hip_atomic_store(&d.c_active[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// playerPlayerOverlap (field.py:233-244) for the players k_pp_active marked, in
// player order, one wavefront per arena.  The sequential semantics (live cell
// list, skip-next after a removal, break when the current cell is eaten) are
// executed uniformly by all 64 lanes -- every lane performs the same loads and
// stores, so program order alone orders them -- while the grid queries
// (candidate gathering, re-activation after growth) are spread over the lanes.
// Cross-lane data: the LDS candidate lists, the pending bitmap and c_active.
// Event / death order keys are (player << 32 | step of its turn): turns run in
// increasing player order, so the keys sort into the serial order whether the
// turns ran in one wave or in independent groups (pp_pass).
constexpr int PP_LCAP = 512;
struct PPL {  // a turn's candidate lists (LDS) and their capacity
  int64_t *key;
  int *val, *srt;
  double *x, *y, *m, *r;
  int cap;
};
// A parallel group's cell table (LDS, one per group wave): every live cell of
// the group's closure -- pool index, position, current mass and radius, seq,
// liveness -- kept current by the group's own eats.  The closure holds every
// cell a turn of the group can gather, eat, be eaten by or re-activate (the
// closure's definition, pp_closure), so the group's candidate gathers and
// re-activation walks scan this table instead of walking the grid (three
// dependent global rounds each).
constexpr int PPT_CAP = 64;  // (= PPG_CELLS: a closure holds at most that many cells)
struct PPT {
  int *e;                       // [row] pool index
  double *x, *y, *m, *r;        // [row] position, mass, radius
  int64_t *seq;                 // [row] creation sequence
  uint8_t *al, *act;            // [row] alive, active (c_active)
  int *pid;                     // [member] arena player index
  uint8_t *pn, *pal, *pl;       // [member] live count, alive; [member][k] live list (slots)
  int8_t *row;                  // [member][slot] the slot's table row, -1 if not live
  int n, np;                    // rows, members
};
// the first pending player at or after q: one bitmap word per lane, a ballot
// picks the first non-empty one (a turn's scan is one LDS round, not one per word)
__device__ __forceinline__ int pend_next(const uint32_t *pend, int NW, int q) {
  const int lane = threadIdx.x & 63;
  for (int wb = q >> 5; wb < NW; wb += 64) {
    const int wd = wb + lane;
    uint32_t bits = wd < NW ? pend[wd] : 0u;
    if (wd == (q >> 5)) bits &= (q & 31) ? ~((1u << (q & 31)) - 1) : 0xFFFFFFFFu;
    const unsigned long long bal = __ballot(bits != 0);
    if (bal) {
      const int l = __ffsll((long long)bal) - 1;
      const uint32_t bw = (uint32_t)__builtin_amdgcn_readlane((int)bits, l);
      return (wb + l) * 32 + __ffs(bw) - 1;
    }
  }
  return -1;
}
// srt[rank] = index, ranks by creation sequence (keys are unique)
__device__ __forceinline__ void rank_by_key(const int64_t *key, int *srt, int nc) {
  for (int x = threadIdx.x & 63; x < nc; x += 64) {
    const int64_t k = key[x];
    int rk = 0;
    for (int y = 0; y < nc; y++) rk += key[y] < k;
    srt[rk] = x;
  }
  wave_fence();
}
// odirty: the deferred occupancy's dirty-word bitmap (LDS, zeroed), or NULL for
// immediate updates
__device__ __forceinline__ void pp_turns(const Dev &d, int a, uint32_t *pend, const PPL &L, uint32_t *odirty, double &rmax) {
  const int lane = threadIdx.x & 63;
  PA_DECL;
  const int B = d.B, NW = (B + 31) / 32;
  const int NP = d.NP;
  const int *st = d.cstart + (size_t)a * (d.H + 1);
  const int *it = d.citems + (size_t)a * kMaxCells * B;
  const unsigned long long lt = (1ull << lane) - 1;
  int64_t *s_key = L.key;
  int *s_val = L.val, *s_srt = L.srt;
  double *s_x = L.x, *s_y = L.y, *s_m = L.m, *s_r = L.r;
  PA_T(0);
  int P = -1;
  for (;;) {
    const int found = pend_next(pend, NW, P + 1);
    if (found < 0) break;
    P = found;
    wave_fence();
    if (lane == 0) pend[P >> 5] &= ~(1u << (P & 31));
    wave_fence();
    const int gp = a * B + P;
    uint64_t order = (uint64_t)P << 32;  // this turn's event / death keys
    PA_C(0);
    // liveness, count and the list's first row in one load round
    // (the list's rows ride the same round: all kMaxCells rows exist)
    const int kslot = lane < kMaxCells ? (int)d.p_list[lane * NP + gp] : 0;
    const int n_first = d.p_ncells[gp];
    if (!d.p_alive[gp]) continue;
    // every cell of the turn, one lane each (lane = the row at the turn's start):
    // its list row, then its state and activity in one round (two rounds per turn,
    // not two per cell).  A turn cell eats only other players' cells, and the
    // re-activation after its eat skips the eater's owner, so the player's own
    // cells and activity change only when the turn cell is eaten: the list then
    // closes up (the cell that moves into its row is skipped, player.py:97 -- the
    // next lane but one), and the eater's re-activation may wake own cells (their
    // activity is loaded again).
    double kx = 0, ky = 0, km = 0, kr = 0;
    int64_t kseq = 0;
    bool kact = false;
    if (lane < n_first) {
      const size_t kc = (size_t)kslot * NP + gp;
      kx = d.c_x[kc];
      ky = d.c_y[kc];
      kseq = d.c_seq[kc];
      km = d.c_m[kc];
      kr = d.c_r[kc];
      kact = active_ld(d, kc) != 0;
    }
    unsigned long long amask = __ballot(kact);
    int nrem = 0;  // own cells removed this turn (rows closed up)
    for (int kn = 0;;) {  // for playerCell in player.getCells(): live list (its active cells)
      const unsigned long long rest = kn < 64 ? amask & (~0ull << kn) : 0;
      if (!rest) break;
      const int kl = __ffsll((long long)rest) - 1;
      kn = kl + 1;
      const int i = kl - nrem + 1;  // (the list row after pc's, as the reference's loop counts)
      const size_t pc = (size_t)lane_i(kslot, kl) * NP + gp;
      const double px = lane_d(kx, kl), py = lane_d(ky, kl);
      const int64_t pseq = (int64_t)__double_as_longlong(lane_d(__longlong_as_double(kseq), kl));
      double pm = lane_d(km, kl), pr = lane_d(kr, kl);
      active_st(d, pc, 0);
      const Rect q0 = footprint(px, py, pr, d.size);  // (cell_rect)
      PA_T(1);
      int nc = 0;
      wave_grid_for(st, it, d.cols, q0, expand_for(rmax), [&](bool valid, int e) {
        double ex = 0, ey = 0, er = 0;
        bool keep = valid && (d.c_flags[e] & F_ALIVE) && (e % NP) != gp;
        if (keep) {
          ex = d.c_x[e];
          ey = d.c_y[e];
          er = d.c_r[e];
          keep = rect_hit(footprint(ex, ey, er, d.size), q0);
        }
        unsigned long long bal = __ballot(keep);
        int slot = nc + __popcll(bal & lt);
        if (keep && slot < L.cap) {
          s_key[slot] = d.c_seq[e];
          s_val[slot] = e;
          s_x[slot] = ex;
          s_y[slot] = ey;
          s_m[slot] = d.c_m[e];
          s_r[slot] = er;
        }
        nc += __popcll(bal);
      }, d.cshift_c);
      if (nc > L.cap) {
        set_err(d, a, ERR_CAND_CAP);
        nc = L.cap;
      }
      PA_T(2);
      PA_C(1);
      PA_ADD(4, nc);
      wave_fence();
      rank_by_key(s_key, s_srt, nc);
      PA_T(3);
      for (int t = 0; t < nc; t++) {
        const int k = s_srt[t];
        const size_t o = (size_t)s_val[k];
        const double ox = s_x[k], oy = s_y[k], om = s_m[k], orr = s_r[k];
        if (!overlap(px, py, pm, pr, ox, oy, om, orr)) continue;
        size_t g, v;
        const bool pc_eats = can_eat(pm, om);
        if (pc_eats) {
          g = pc;
          v = o;
        } else if (can_eat(om, pm)) {
          g = o;
          v = pc;
        } else {
          continue;
        }
        // eatPlayerCell (field.py:346-348)
        if (lane == 0) ev_push(d, a, PH_PP, order, 8, pc_eats ? pseq : s_key[k], pc_eats ? s_key[k] : pseq);
        order++;
        const double m = pc_eats ? grow_mass(pm, om) : grow_mass(om, pm);
        const double mr = radius_of(m);
        d.c_m[g] = m;
        d.c_r[g] = mr;
        // the spawn occupancy follows: the eaten cell leaves, the eater's footprint grows
        if (odirty) {
          occ_remove_def(d, a, pc_eats ? footprint(ox, oy, orr, d.size) : footprint(px, py, pr, d.size), odirty);
          if (pc_eats) occ_grow_def(d, a, footprint(px, py, pr, d.size), footprint(px, py, mr, d.size), odirty);
          else occ_grow_def(d, a, footprint(ox, oy, orr, d.size), footprint(ox, oy, mr, d.size), odirty);
        } else {
          occ_remove(d, a, pc_eats ? footprint(ox, oy, orr, d.size) : footprint(px, py, pr, d.size));
          wave_fence();
          if (pc_eats) occ_grow(d, a, footprint(px, py, pr, d.size), footprint(px, py, mr, d.size));
          else occ_grow(d, a, footprint(ox, oy, orr, d.size), footprint(ox, oy, mr, d.size));
        }
        if (pc_eats) {
          pm = m;
          pr = mr;
        }
        rmax = fmax(rmax, mr);
        remove_cell(d, a, v, order, lane == 0);
        // re-activate every later turn whose outcome the growth of g may change
        const int gpl = (int)(g % NP);
        const double gx = pc_eats ? px : ox, gy = pc_eats ? py : oy, gm = m, gr = mr;
        wave_fence();  // (the removal above is read by the re-activation walk)
        PA_T(4);
        PA_C(2);
        // (cell_rect(d, g) from the registers: g's position and its new radius)
        wave_grid_for(st, it, d.cols, footprint(gx, gy, gr, d.size), expand_for(rmax), [&](bool valid, int e) {
          if (!valid || (int)(e % NP) == gpl || !(d.c_flags[e] & F_ALIVE)) return;
          if (!overlap(gx, gy, gm, gr, d.c_x[e], d.c_y[e], d.c_m[e], d.c_r[e])) return;
          active_st(d, (size_t)e, 1);
          int pe = (int)(e % NP) - a * B;
          if (pe > P) atomicOr(&pend[pe >> 5], 1u << (pe & 31));
        }, d.cshift_c);
        active_st(d, g, 1);
        if (gpl - a * B > P && lane == 0) atomicOr(&pend[(gpl - a * B) >> 5], 1u << ((gpl - a * B) & 31));
        wave_fence();
        PA_T(5);
        if (!pc_eats) {
          // pc left the live list: the cell that moved into its place is skipped
          // this turn (field.py:236 + player.py:97).  Its pairs with later
          // players are then theirs to resolve: activate those partners.
          if (i - 1 < d.p_ncells[gp]) {
            const size_t sk = (size_t)d.p_list[(i - 1) * NP + gp] * NP + gp;
            const double sx = d.c_x[sk], sy = d.c_y[sk], sm = d.c_m[sk], sr = d.c_r[sk];
            wave_grid_for(st, it, d.cols, footprint(sx, sy, sr, d.size), expand_for(rmax), [&](bool valid, int e) {
              if (!valid || (int)(e % NP) == gp || !(d.c_flags[e] & F_ALIVE)) return;
              const double me = d.c_m[e];
              if (!(overlap(sx, sy, sm, sr, d.c_x[e], d.c_y[e], me, d.c_r[e]) && (can_eat(sm, me) || can_eat(me, sm))))
                return;
              int pe = (int)(e % NP) - a * B;
              if (pe <= P) return;
              active_st(d, (size_t)e, 1);
              atomicOr(&pend[pe >> 5], 1u << (pe & 31));
            }, d.cshift_c);
            wave_fence();
          }
          PA_T(6);
          PA_C(3);
          nrem++;
          kn = kl + 2;  // (the skipped row's cell)
          bool re = lane >= kn && lane < n_first && active_ld(d, (size_t)kslot * NP + gp) != 0;
          amask = __ballot(re);
          break;
        }
      }
    }
  }
  PA_T(7);
  PA_STORE(a);
}

// The turns of one parallel group, entirely on its LDS table: the members' live
// lists, counts and liveness, and every live cell of the closure with its
// activity (the closure holds every cell a turn of the group can gather, eat, be
// eaten by or re-activate -- pp_closure).  The same sequence of turns, eats and
// re-activations as pp_turns; global memory is only written (the eats' mass,
// list and liveness stores, the occupancy counts), never read, so a turn waits
// on no load.  The group's deaths take slots of the pass's death list (dpl /
// dkey, counted in *s_nd) for the sort into turn order after the pass.
__device__ __forceinline__ void pp_group_turns(const Dev &d, int a, uint32_t *pend, int64_t *s_key, int *s_val,
                                               int *s_srt, uint32_t *odirty, double &rmax, int *dpl, int64_t *dkey,
                                               int *s_nd, const PPT &tab) {
  const int lane = threadIdx.x & 63;
  PA_DECL;
  const int B = d.B, NW = (B + 31) / 32, NP = d.NP;
  const unsigned long long lt = (1ull << lane) - 1;
  auto member = [&](int p) {  // the member index of arena player p (every pp partner is a member)
    const unsigned long long b = __ballot(lane < tab.np && tab.pid[lane] == p);
    return b ? __ffsll((long long)b) - 1 : -1;
  };
  // removePlayerCell on the table (remove_cell's semantics): row's cell leaves
  // its player's list, which closes up; the last cell's removal kills the player
  auto remove = [&](int row, uint64_t &order) {
    const size_t e = (size_t)tab.e[row];
    const int gpv = (int)(e % NP), pv = gpv - a * B, jv = member(pv);
    const int slot = (int)(e / NP);
    const int n = tab.pn[jv];
    const int l = lane < kMaxCells ? tab.pl[jv * kMaxCells + lane] : 0;
    const bool keep = lane < n && l != slot;
    const unsigned long long kb = __ballot(keep);
    const int pos = __popcll(kb & lt), w = __popcll(kb);
    wave_fence();  // (the list is read before it is rewritten)
    if (keep) {
      tab.pl[jv * kMaxCells + pos] = (uint8_t)l;
      d.p_list[(size_t)pos * NP + gpv] = (uint8_t)l;
    }
    if (lane == 0) {
      tab.pn[jv] = (uint8_t)w;
      tab.al[row] = 0;
      d.p_ncells[gpv] = w;
      d.c_flags[e] = 0;
    }
    if (w == 0) {  // deletePlayerCell: last cell -> deadPlayers, setDead (field.py:386-388)
      if (lane == 0) {
        tab.pal[jv] = 0;
        d.p_alive[gpv] = 0;
        d.p_respawn[gpv] = 1;
        const int sl = atomicAdd(s_nd, 1);
        dpl[sl] = pv;
        dkey[sl] = (int64_t)order;
        ev_push(d, a, PH_PP, order, 9, pv, tab.seq[row]);
      }
      order++;
    }
    wave_fence();
  };
  PA_T(0);
  int P = -1;
  for (;;) {
    const int found = pend_next(pend, NW, P + 1);
    if (found < 0) break;
    P = found;
    wave_fence();
    if (lane == 0) pend[P >> 5] &= ~(1u << (P & 31));
    wave_fence();
    const int gp = a * B + P, j = member(P);
    uint64_t order = (uint64_t)P << 32;  // this turn's event / death keys
    PA_C(0);
    if (j < 0 || !tab.pal[j]) continue;
    for (int i = 0;;) {  // for playerCell in player.getCells(): live list
      if (i >= tab.pn[j]) break;
      const int prow = tab.row[j * kMaxCells + tab.pl[j * kMaxCells + i]];
      i++;
      if (prow < 0 || !tab.act[prow]) continue;
      wave_fence();
      if (lane == 0) tab.act[prow] = 0;
      const size_t pc = (size_t)tab.e[prow];
      const double px = tab.x[prow], py = tab.y[prow];
      const int64_t pseq = tab.seq[prow];
      double pm = tab.m[prow], pr = tab.r[prow];
      const Rect q0 = footprint(px, py, pr, d.size);  // (cell_rect)
      PA_T(1);
      // candidates: the table rows of other players' live cells whose footprint meets q0
      int nc = 0;
      for (int r0 = 0; r0 < tab.n; r0 += 64) {
        const int t = r0 + lane;
        bool keep = false;
        if (t < tab.n && tab.al[t])
          keep = (tab.e[t] % NP) != gp && rect_hit(footprint(tab.x[t], tab.y[t], tab.r[t], d.size), q0);
        const unsigned long long bal = __ballot(keep);
        const int slot = nc + __popcll(bal & lt);
        if (keep) {
          s_key[slot] = tab.seq[t];
          s_val[slot] = t;
        }
        nc += __popcll(bal);
      }
      PA_T(2);
      PA_C(1);
      PA_ADD(4, nc);
      wave_fence();
      rank_by_key(s_key, s_srt, nc);
      PA_T(3);
      for (int t = 0; t < nc; t++) {
        // (a candidate's row holds its state at turn start: only pc's row, and a
        // victim's liveness, change before every candidate was visited)
        const int k = s_srt[t], ro = s_val[k];
        const double ox = tab.x[ro], oy = tab.y[ro], om = tab.m[ro], orr = tab.r[ro];
        if (!overlap(px, py, pm, pr, ox, oy, om, orr)) continue;
        const bool pc_eats = can_eat(pm, om);
        if (!pc_eats && !can_eat(om, pm)) continue;
        const int gi = pc_eats ? prow : ro, vi = pc_eats ? ro : prow;
        const size_t g = (size_t)tab.e[gi];
        // eatPlayerCell (field.py:346-348)
        if (lane == 0) ev_push(d, a, PH_PP, order, 8, pc_eats ? pseq : s_key[k], pc_eats ? s_key[k] : pseq);
        order++;
        const double m = pc_eats ? grow_mass(pm, om) : grow_mass(om, pm);
        const double mr = radius_of(m);
        if (lane == 0) {
          d.c_m[g] = m;
          d.c_r[g] = mr;
        }
        // the spawn occupancy follows: the eaten cell leaves, the eater's footprint grows
        occ_remove_def(d, a, pc_eats ? footprint(ox, oy, orr, d.size) : footprint(px, py, pr, d.size), odirty);
        if (pc_eats) occ_grow_def(d, a, footprint(px, py, pr, d.size), footprint(px, py, mr, d.size), odirty);
        else occ_grow_def(d, a, footprint(ox, oy, orr, d.size), footprint(ox, oy, mr, d.size), odirty);
        if (pc_eats) {
          pm = m;
          pr = mr;
        }
        rmax = fmax(rmax, mr);
        wave_fence();
        if (lane == 0) {
          tab.m[gi] = m;
          tab.r[gi] = mr;
        }
        remove(vi, order);
        PA_T(4);
        PA_C(2);
        // re-activate every later turn whose outcome the growth of g may change
        const int gpl = (int)(g % NP);
        const double gx = pc_eats ? px : ox, gy = pc_eats ? py : oy;
        for (int t2 = lane; t2 < tab.n; t2 += 64) {
          if (!tab.al[t2] || (int)(tab.e[t2] % NP) == gpl) continue;
          if (!overlap(gx, gy, m, mr, tab.x[t2], tab.y[t2], tab.m[t2], tab.r[t2])) continue;
          tab.act[t2] = 1;
          const int pe = (int)(tab.e[t2] % NP) - a * B;
          if (pe > P) atomicOr(&pend[pe >> 5], 1u << (pe & 31));
        }
        if (lane == 0) {
          tab.act[gi] = 1;
          if (gpl - a * B > P) atomicOr(&pend[(gpl - a * B) >> 5], 1u << ((gpl - a * B) & 31));
        }
        wave_fence();
        PA_T(5);
        if (!pc_eats) {
          // pc left the live list: the cell that moved into its place is skipped
          // this turn (field.py:236 + player.py:97).  Its pairs with later
          // players are then theirs to resolve: activate those partners.
          if (i - 1 < tab.pn[j]) {
            const int sr_ = tab.row[j * kMaxCells + tab.pl[j * kMaxCells + i - 1]];
            const double sx = tab.x[sr_], sy = tab.y[sr_], sm = tab.m[sr_], sr = tab.r[sr_];
            for (int t2 = lane; t2 < tab.n; t2 += 64) {
              if (!tab.al[t2] || (int)(tab.e[t2] % NP) == gp) continue;
              const double me = tab.m[t2];
              if (!(overlap(sx, sy, sm, sr, tab.x[t2], tab.y[t2], me, tab.r[t2]) && (can_eat(sm, me) || can_eat(me, sm))))
                continue;
              const int pe = (int)(tab.e[t2] % NP) - a * B;
              if (pe <= P) continue;
              tab.act[t2] = 1;
              atomicOr(&pend[pe >> 5], 1u << (pe & 31));
            }
            wave_fence();
          }
          PA_T(6);
          PA_C(3);
          break;
        }
      }
    }
  }
  // (the activity marks leave with the group, as the serial pass leaves them)
  for (int t = lane; t < tab.n; t += 64) d.c_active[tab.e[t]] = tab.act[t];
  PA_T(7);
  PA_STORE_GROUP(a);
}
// the whole pass in one wavefront (nw pending players in d.work)
// L: the candidates of the current turn, with their state at turn start (only
// the turn's own cell changes them: what it eats dies, and it stops when eaten)
// -- LDS shared with the parallel groups' lists (the two paths never run together)
__device__ __forceinline__ void pp_serial_body(const Dev &d, int a, uint32_t *pend, uint32_t *odirty, int nw,
                                               const PPL &L) {
  const int lane = threadIdx.x & 63, NW = (d.B + 31) / 32;
  for (int i = lane; i < NW; i += 64) pend[i] = 0;
  wave_fence();
  for (int i = lane; i < nw; i += 64) {
    int p = d.work[(size_t)a * d.Wcap + i];
    atomicOr(&pend[p >> 5], 1u << (p & 31));
  }
  wave_fence();
  if (nw == 0) return;
  ArenaCtl &c = d.ctl[a];
  double rmax = c.rmax_cell;
  pp_turns(d, a, pend, L, odirty, rmax);
  c.rmax_cell = rmax;
}

// ---- independent pp groups
// A turn reads and changes only cells near the turning player's cells, but a
// growth re-activates the partners of the grown cell, whose turns walk their
// whole lists, and so on.  The closure of a seed player bounds that: no cell
// of a group eats outside it, so no radius in it exceeds R = radius_of(min(cap,
// group mass)) (or a cell's own, possibly stale, radius); every cell whose
// footprint at max(its radius, R) meets the union U of the group cells'
// footprints at R could be a candidate, a victim, an eater or a re-activated
// partner, so its player joins -- with all its cells, which its turn walks --
// and R, U are recomputed, to a fixed point.  Seeds whose closures share no
// player commute: cells of two such groups never meet, so each group can run
// its turns in its own wavefront, in player order, on the pass's state.  (A cell
// of another group can only be read while a grid walk filters it out: its
// footprint misses every footprint of this group, whatever its current radius.)
#ifdef AIGAR_PP_DIAG  // diagnostics build: why the parallel pass fell back (tools/var/pp_diag.py)
__device__ unsigned long long g_ppdiag[16];
#define PP_DIAG(k) atomicAdd(&g_ppdiag[k], 1ull)
extern "C" int aigar_debug_ppdiag(unsigned long long *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ppdiag), sizeof(g_ppdiag)) == hipSuccess ? 0 : -1;
}
#else
#define PP_DIAG(k)
#endif
constexpr int PPG_SEEDS = 64;  // most pending players for the parallel pass
constexpr int PPG_PL = 16;     // players per closure (32 measured: the crowded world's overflowing closures exceed it too)
constexpr int PPG_CELLS = 64;  // cells per closure (also the turn candidate cap)
#ifndef AIGAR_PPG_WAVES
#define AIGAR_PPG_WAVES 16
#endif
constexpr int PPG_WAVES = AIGAR_PPG_WAVES;  // wavefronts running groups
constexpr int PP_LOWN_MAX = 8192;  // arenas up to this many players keep the pass's player owners in LDS
constexpr int PPG_MIN = 3;     // fewer pending players: the serial pass (closures cost ~10 us)
// (pl[0..npl): the starting players -- a seed, or merged closures)
__device__ __forceinline__ bool pp_closure(const Dev &d, int a, int *pl, int &npl) {
  const int lane = threadIdx.x & 63, NP = d.NP, B = d.B;
  const int *st = d.cstart + (size_t)a * (d.H + 1);
  const int *it = d.citems + (size_t)a * kMaxCells * B;
  const double rmax0 = d.ctl[a].rmax_cell;
  wave_fence();
  for (int iter = 0; iter < 12; iter++) {
    // the group's cells: (player j, slot k) pairs, four per lane, one load round
    uint32_t fl[4];
    double cx[4], cy[4], cm[4], cr[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int pr = lane + 64 * k, j = pr >> 4;
      fl[k] = 0;
      cx[k] = cy[k] = cm[k] = cr[k] = 0;
      if (j < npl) {
        const size_t ci = (size_t)(pr & 15) * NP + (size_t)a * B + pl[j];
        fl[k] = d.c_flags[ci];
        cx[k] = d.c_x[ci];
        cy[k] = d.c_y[ci];
        cm[k] = d.c_m[ci];
        cr[k] = d.c_r[ci];
      }
    }
    double M = 0, rr = 0;
    int n = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (fl[k] & F_ALIVE) {
        M += cm[k];
        rr = fmax(rr, cr[k]);
        n++;
      }
    M = wave_sum(M);
    for (int o = 32; o > 0; o >>= 1) {
      rr = fmax(rr, __shfl_xor(rr, o));
      n += __shfl_xor(n, o);
    }
    if (n > PPG_CELLS) {
      if (lane == 0) PP_DIAG(3);
      return false;
    }
    const double R = fmax(radius_of(py_min(kMaxMass, M)), rr) * (1 + 1e-9) + 1e-9;
    Rect U{INT_MAX, -1, INT_MAX, -1};
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (fl[k] & F_ALIVE) {
        const Rect q = footprint(cx[k], cy[k], R, d.size);
        U.x0 = min(U.x0, q.x0);
        U.x1 = max(U.x1, q.x1);
        U.y0 = min(U.y0, q.y0);
        U.y1 = max(U.y1, q.y1);
      }
    for (int o = 32; o > 0; o >>= 1) {
      U.x0 = min(U.x0, __shfl_xor(U.x0, o));
      U.x1 = max(U.x1, __shfl_xor(U.x1, o));
      U.y0 = min(U.y0, __shfl_xor(U.y0, o));
      U.y1 = max(U.y1, __shfl_xor(U.y1, o));
    }
    bool added = false;
    // the members in registers (lane j holds pl[j]): membership tests are
    // readlane compares, not LDS round trips; pl[] is written back at the end
    int mine = lane < min(npl, PPG_PL) ? pl[lane] : -1;
    const int npl0 = npl;
    wave_grid_for(st, it, d.cols, U, expand_for(fmax(rmax0, R)), [&](bool valid, int e) {
      int q = -1;
      if (valid && (d.c_flags[e] & F_ALIVE) &&
          rect_hit(footprint(d.c_x[e], d.c_y[e], fmax(d.c_r[e], R), d.size), U))
        q = e % NP - a * B;
      for (int j = 0; j < min(npl, PPG_PL); j++)  // (j uniform)
        if (__builtin_amdgcn_readlane(mine, j) == q) q = -1;  // already in
      unsigned long long nb = __ballot(q >= 0);
      while (nb) {  // new players, deduplicated in lane order
        const int l = __ffsll((long long)nb) - 1;
        const int qq = __builtin_amdgcn_readlane(q, l);
        nb &= ~__ballot(q == qq);  // (every lane holding the same player)
        if (npl < PPG_PL && lane == npl) mine = qq;
        npl++;
        added = true;
      }
    }, d.cshift_c);
    if (npl > npl0) {
      if (lane < min(npl, PPG_PL) && lane >= npl0) pl[lane] = mine;
      wave_fence();
    }
    if (npl > PPG_PL) {
      if (lane == 0) PP_DIAG(2);
      return false;
    }
    if (!added) {
      if (lane == 0) PP_DIAG(8 + min(npl, 7));
      return true;
    }
  }
  if (lane == 0) PP_DIAG(4);
  return false;
}
// playerPlayerOverlap for the block: the serial pass in wave 0, or -- with at
// least PPG_MIN pending players whose closures are pairwise disjoint -- one
// group per seed, PPG_WAVES wavefronts each running its seeds' turns (their
// pending bits together: disjoint groups interleave freely), then the pass's
// deaths sorted into turn order by their keys.  Called by every thread.
__device__ __forceinline__ void pp_pass(const Dev &d, int a, int64_t *scr_k, int *scr_v, uint32_t *pend, uint32_t *odirty PT_PARAMS) {
  __shared__ int s_nw, s_dead0, s_bad, s_nd;
  __shared__ int s_pl[PPG_SEEDS][PPG_PL], s_npl[PPG_SEEDS];
  __shared__ double s_rmax[PPG_WAVES];
  // the group waves' candidate lists (key, table row, rank)
  __shared__ int64_t g_key[PPG_WAVES][PPG_CELLS];
  __shared__ int g_val[PPG_WAVES][PPG_CELLS], g_srt[PPG_WAVES][PPG_CELLS];
  // the group waves' tables (PPT); the serial pass's candidate states use the rows' arrays
  __shared__ int t_e[PPG_WAVES][PPT_CAP];
  __shared__ double t_x[PPG_WAVES][PPT_CAP], t_y[PPG_WAVES][PPT_CAP], t_m[PPG_WAVES][PPT_CAP], t_r[PPG_WAVES][PPT_CAP];
  __shared__ int64_t t_seq[PPG_WAVES][PPT_CAP];
  __shared__ uint8_t t_al[PPG_WAVES][PPT_CAP], t_act[PPG_WAVES][PPT_CAP];
  __shared__ int t_pid[PPG_WAVES][PPG_PL];
  __shared__ uint8_t t_pn[PPG_WAVES][PPG_PL], t_pal[PPG_WAVES][PPG_PL], t_pl[PPG_WAVES][PPG_PL * kMaxCells];
  __shared__ int8_t t_row[PPG_WAVES][PPG_PL * kMaxCells];
  ArenaCtl &c = d.ctl[a];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nwv = blockDim.x >> 6, T = blockDim.x;
  // each wave's first seed, loaded beside the count (in bounds whatever the count)
  const int p_first = w < d.Wcap ? d.work[(size_t)a * d.Wcap + w] : 0;
  if (tid == 0) {  // (every thread reads the count before it is reset)
    s_nw = min(c.n_pend, d.Wcap);
    s_dead0 = c.n_dead;
    s_bad = 0;
    s_nd = 0;
    c.n_pend = 0;
    c.stat[4] += s_nw;
    c.stat[7] += 1;
  }
  __syncthreads();
  const int nw = s_nw, dead0 = s_dead0;
  const bool par = d.pp_par && odirty && nw >= PPG_MIN && nw <= PPG_SEEDS && nwv >= PPG_WAVES;
  static_assert(PPG_WAVES * PPG_CELLS >= PP_LCAP && PPG_WAVES * PPT_CAP >= PP_LCAP,
                "the serial pass's candidate lists live in the groups' LDS");
  static_assert(PPT_CAP <= 127 && PPG_PL <= 64, "table rows as int8, members one per lane");
  const PPL serial_l{&g_key[0][0], &g_val[0][0], &g_srt[0][0], &t_x[0][0], &t_y[0][0], &t_m[0][0], &t_r[0][0], PP_LCAP};
  if (!par) {
    if (tid == 0 && nw > 0) PP_DIAG(nw < PPG_MIN ? 0 : 1);
    if (tid < 64) pp_serial_body(d, a, pend, odirty, nw, serial_l);
    return;
  }
  // closures; per player the lowest seed whose closure holds it
  // (in the dynamic LDS after the pending bitmaps when the arena is small enough:
  // the label propagation and the owner checks are then LDS rounds)
  const bool lown = d.B <= PP_LOWN_MAX;
  int *g_pown = scr_v + (size_t)a * d.Wcap, *s_pown = reinterpret_cast<int *>(pend + PPG_WAVES * ((d.B + 31) / 32));
  auto pown_st = [&](int i, int v) {
    if (lown) s_pown[i] = v;
    else __hip_atomic_store(&g_pown[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto pown_min = [&](int i, int v) {
    if (lown) atomicMin(&s_pown[i], v);
    else atomicMin(&g_pown[i], v);
  };
  auto pown_ld = [&](int i) {
    return lown ? __hip_atomic_load(&s_pown[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                : __hip_atomic_load(&g_pown[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  for (int i = tid; i < d.B; i += T) pown_st(i, INT_MAX);
  __syncthreads();
  PT_SUB(0);
  for (int sd = w; sd < nw; sd += nwv) {
    const int P = sd == w ? p_first : d.work[(size_t)a * d.Wcap + sd];
    if (lane == 0) s_pl[sd][0] = P;
    int npl = 1;
    const bool ok = pp_closure(d, a, s_pl[sd], npl);
    if (lane == 0) s_npl[sd] = ok ? npl : 0;
    if (!ok) {
      if (lane == 0) s_bad = 1;
      continue;
    }
    for (int j = lane; j < npl; j += 64) pown_min(s_pl[sd][j], sd);
  }
  __syncthreads();
  PT_SUB(1);
  // closures that share a player merge: their seeds' components (label = the
  // lowest seed, propagated along every shared player to a fixed point), each
  // component's players united in its root's list and closed again from there;
  // the groups are then the roots' closures, checked pairwise disjoint as above
  __shared__ int s_lab[PPG_SEEDS], s_root[PPG_SEEDS];
  if (!s_bad) {
    for (int i = tid; i < nw; i += T) s_lab[i] = i;
    __syncthreads();
    for (int iter = 0; iter < PPG_SEEDS; iter++) {
      int chg = 0;
      for (int sd = w; sd < nw; sd += nwv)
        for (int j = lane; j < s_npl[sd]; j += 64) {
          const int o = pown_ld(s_pl[sd][j]);
          if (o == sd) continue;
          const int lo = min(s_lab[sd], s_lab[o]);
          chg |= atomicMin(&s_lab[sd], lo) > lo;
          chg |= atomicMin(&s_lab[o], lo) > lo;
        }
      if (!__syncthreads_or(chg)) break;
    }
    for (int i = tid; i < nw; i += T) s_root[i] = s_lab[i];
    __syncthreads();
    PT_SUB(2);
    for (int rt = w; rt < nw; rt += nwv) {
      if (s_root[rt] != rt) continue;
      int npl = s_npl[rt];
      bool more = false;
      for (int sd = rt + 1; sd < nw && npl <= PPG_PL; sd++) {
        if (s_root[sd] != rt) continue;
        more = true;
        for (int j = 0; j < s_npl[sd] && npl <= PPG_PL; j++) {
          const int q = s_pl[sd][j];
          bool dup = false;
          for (int k = lane; k < npl; k += 64) dup |= s_pl[rt][k] == q;
          if (__ballot(dup)) continue;
          if (npl < PPG_PL && lane == 0) s_pl[rt][npl] = q;
          npl++;
          wave_fence();
        }
      }
      if (!more) continue;
      bool ok = npl <= PPG_PL;
      if (ok) ok = pp_closure(d, a, s_pl[rt], npl);
      if (lane == 0) s_npl[rt] = ok ? npl : 0;
      if (!ok && lane == 0) s_bad = 1;
    }
    __syncthreads();
    PT_SUB(3);
    if (!s_bad) {
      for (int i = tid; i < d.B; i += T) pown_st(i, INT_MAX);
      __syncthreads();
      for (int rt = w; rt < nw; rt += nwv)
        if (s_root[rt] == rt)
          for (int j = lane; j < s_npl[rt]; j += 64) pown_min(s_pl[rt][j], rt);
      __syncthreads();
    }
  }
  if (!s_bad)
    for (int sd = w; sd < nw; sd += nwv)
      if (s_root[sd] == sd)
        for (int j = lane; j < s_npl[sd]; j += 64)
          if (pown_ld(s_pl[sd][j]) != sd) s_bad = 1;
  __syncthreads();
  PT_SUB(4);
  PT_MARK(5, 6);
  if (tid == 0) PP_DIAG(s_bad ? 5 : 6);
  if (s_bad) {  // a closure overflowed, or two groups may meet: the serial pass
    if (tid < 64) pp_serial_body(d, a, pend, odirty, nw, serial_l);
    return;
  }
  if (w < PPG_WAVES) {
    const int NW = (d.B + 31) / 32;
    uint32_t *mine = pend + (size_t)w * NW;
    for (int i = lane; i < NW; i += 64) mine[i] = 0;
    wave_fence();
    // group g (the g-th root) runs in wave g % PPG_WAVES, one group after the
    // other (groups are independent): its seeds' pending bits, its table (every
    // (member, slot) pair's cell state, list entry and activity, and each
    // member's count and liveness: one load round), its turns
    double rmax = c.rmax_cell;
    int g = 0;  // roots before rt
    for (int rt = 0; rt < nw; rt++) {
      if (s_root[rt] != rt) continue;
      const bool mineg = g % PPG_WAVES == w;
      g++;
      if (!mineg) continue;
      for (int sd = rt; sd < nw; sd++)
        if (s_root[sd] == rt && lane == 0) {
          const int P = d.work[(size_t)a * d.Wcap + sd];
          mine[P >> 5] |= 1u << (P & 31);
        }
      const int npl = s_npl[rt];
      PPT tab{t_e[w], t_x[w], t_y[w], t_m[w], t_r[w], t_seq[w], t_al[w], t_act[w], t_pid[w], t_pn[w], t_pal[w],
              t_pl[w], t_row[w], 0, npl};
      int nt = 0;
#pragma unroll
      for (int kk = 0; kk < 4; kk++) {  // (member j, slot k) pairs, four per lane
        const int pr = lane + 64 * kk, j = pr >> 4, k = pr & 15;
        bool keep = false;
        size_t ci = 0;
        double x = 0, y = 0, m = 0, r = 0;
        int64_t sq = 0;
        int pj = 0, pn = 0, pal = 0;
        uint8_t act = 0, li = 0;
        if (j < npl) {
          pj = s_pl[rt][j];
          const int gpj = a * d.B + pj;
          ci = (size_t)k * d.NP + gpj;
          keep = (d.c_flags[ci] & F_ALIVE) != 0;
          x = d.c_x[ci];
          y = d.c_y[ci];
          m = d.c_m[ci];
          r = d.c_r[ci];
          sq = d.c_seq[ci];
          act = d.c_active[ci];
          li = d.p_list[ci];  // (p_list rows share the cells' (slot, player) layout)
          if (k == 0) {
            pn = d.p_ncells[gpj];
            pal = d.p_alive[gpj];
          }
        }
        const unsigned long long bal = __ballot(keep);
        const int slot = nt + __popcll(bal & ((1ull << lane) - 1));
        if (keep && slot < PPT_CAP) {
          tab.e[slot] = (int)ci;
          tab.x[slot] = x;
          tab.y[slot] = y;
          tab.m[slot] = m;
          tab.r[slot] = r;
          tab.seq[slot] = sq;
          tab.al[slot] = 1;
          tab.act[slot] = act;
        }
        if (j < npl) {
          tab.pl[pr] = li;
          tab.row[pr] = (int8_t)(keep && slot < PPT_CAP ? slot : -1);
          if (k == 0) {
            tab.pid[j] = pj;
            tab.pn[j] = (uint8_t)pn;
            tab.pal[j] = (uint8_t)pal;
          }
        }
        nt += __popcll(bal);
      }
      if (nt > PPT_CAP) {  // (a closure holds at most PPG_CELLS cells: cannot happen)
        if (lane == 0) set_err(d, a, ERR_CAND_CAP);
        nt = PPT_CAP;
      }
      tab.n = nt;
      wave_fence();
      pp_group_turns(d, a, mine, g_key[w], g_val[w], g_srt[w], odirty, rmax, d.dead + (size_t)a * d.B + dead0,
                     scr_k + (size_t)a * d.Wcap, &s_nd, tab);
    }
    if (lane == 0) s_rmax[w] = rmax;
  }
  __syncthreads();
  PT_SUB(5);
  PT_MARK(5, 7);
  // the pass's deaths (slots taken in completion order) into turn order: rank by key
  const int nd = s_nd;
  const int64_t *dk = scr_k + (size_t)a * d.Wcap;
  int *dl = d.dead + (size_t)a * d.B + dead0;
  int rk[2], pv[2];
  for (int k = 0; k < 2; k++) {
    const int i = tid + k * T;
    rk[k] = -1;
    if (i < nd) {
      const int64_t key = dk[i];
      int r = 0;
      for (int j = 0; j < nd; j++) r += dk[j] < key;
      rk[k] = r;
      pv[k] = dl[i];
    }
  }
  if (nd > 2 * T && tid == 0) set_err(d, a, ERR_WORK_CAP);
  __syncthreads();
  for (int k = 0; k < 2; k++)
    if (rk[k] >= 0) dl[rk[k]] = pv[k];
  if (tid == 0) {
    double r = c.rmax_cell;
    for (int k = 0; k < PPG_WAVES; k++) r = fmax(r, s_rmax[k]);
    c.rmax_cell = r;
    c.n_dead = dead0 + nd;
    c.stat[6] += 1;
  }
  PT_SUB(6);
}

// ------------------------------------------------------------ T18 spawn
// getSpawnPos (field.py:283-301) with the player-hash occupancy bitmap
__device__ void spawn_pos(const Dev &d, int a, double radius, const uint64_t u[4], double &ox, double &oy) {
  const int cols = d.cols, total = d.H;
  const unsigned long long *occ = d.occ + (size_t)a * d.occ_words;
  int sb = (int)mulhi(u[0], (uint64_t)total);
  int found = -1;
  // first non-occupied bucket at or after sb, cyclically
  for (int pass = 0; pass < 2 && found < 0; pass++) {
    int lo = pass == 0 ? sb : 0, hi = pass == 0 ? total : sb;
    for (int b = lo; b < hi && found < 0;) {
      int wd = b >> 6;
      unsigned long long free_bits = ~occ[wd];
      free_bits &= (~0ull) << (b & 63);
      int wend = (wd + 1) << 6;
      if (wend > hi) free_bits &= (hi - (wd << 6)) >= 64 ? ~0ull : ((1ull << (hi - (wd << 6))) - 1);
      if (free_bits) found = (wd << 6) + __ffsll((long long)free_bits) - 1;
      b = wend;
    }
  }
  int64_t xp, yp;
  if (found < 0) {
    xp = ph_randint(u[1], 0, d.size);
    yp = ph_randint(u[2], 0, d.size);
  } else {
    int64_t x = found % cols;
    double y = (double)(found - x) / cols;
    int64_t left = (x - 1) * kBucket;
    double top = y * kBucket;
    xp = ph_randint(u[1], left + radius, (double)(left + kBucket) - radius);
    yp = ph_randint(u[2], top + radius, top + kBucket - radius);
  }
  ox = (double)xp;
  oy = (double)yp;
}

// the arena fields spawn_counts reads, loaded by its thread before the dead
// list's partition (their load round overlaps it)
struct SpawnIn {
  int n_pel, n_pel_eaten, n_pnew, n_pel_glob, n_eaten_glob, n_vir;
  int64_t seq_next, tick, stat3, stat5;
  uint64_t ctr_pellet, ctr_virus;
};
__device__ __forceinline__ SpawnIn spawn_in(const ArenaCtl &c) {
  return SpawnIn{c.n_pel,    c.n_pel_eaten, c.n_pnew,    c.n_pel_glob, c.n_eaten_glob, c.n_vir,
                 c.seq_next, c.tick,        c.stat[3],   c.stat[5],    c.ctr_pellet,   c.ctr_virus};
}
__device__ __forceinline__ void spawn_counts(const Dev &d, int a, int init, int n_resp, int n_wait, const SpawnIn &in);
// ---------------------------------------------------- closing pellet update
// Pellets never move and only a few change per tick (eaten, spawned, converted
// from blobs): the closing update (k_pel_update) rewrites only the bucket rows
// those touch, each into its other home.  Step 1, by the arena's block of
// k_spawn_plan after the spawn counts: this tick's pellet spawns are staged
// (spawnPellets, field.py:303-313) -- the first kSpawnAhead were drawn by
// k_players' arena block already (spec_*) -- and the tick's pellet bookkeeping closes.
__device__ void spawn_pellet_at(const Dev &d, int a, int j, double *px, double *py);
__device__ __forceinline__ void pellet_close_prep(const Dev &d, int a) {
  ArenaCtl &c = d.ctl[a];
  const int nconv = c.n_pnew, nsp = c.n_spawn_p;
  const bool spec = nsp <= kSpawnAhead;
  if (!spec)  // into the staging list after the conversions (pn[nconv + j])
    for (int j = threadIdx.x; j < nsp; j += blockDim.x) spawn_pellet_at(d, a, j, nullptr, nullptr);
  __syncthreads();  // (spawn_pellet_at reads n_pnew)
  if (threadIdx.x == 0) {
    c.pu_nconv = nconv;
    c.pu_nsp = nsp;
    c.pu_spec = spec ? 1 : 0;
    c.n_pnew = 0;
    c.n_pel_eaten = 0;  // (n_pel: the rewritten rows add their change)
  }
}
// pp (tick only): playerPlayerOverlap's serial pass first, by wave 0 of the
// arena's block (its pending bitmap in the dynamic LDS)
// close (tick only): then the closing pellet update's step 1 (pellet_close_prep)
__global__ void __launch_bounds__(1024) k_spawn_plan(Dev d, int init, int64_t *scr_k, int *scr_v, int pp,
                                                     int close) {
  FLOOR(7);
  __shared__ int sflag[1024];
  __shared__ int gcnt[SG_CAP + 1];
  PT_BEGIN(5);
  int a = blockIdx.x;
  if (pp) {
    extern __shared__ uint32_t pend[];
    __shared__ uint32_t s_odirty[OCC_DW];
    const bool defer = d.occ_words <= OCC_DW * 32;
    for (int i = threadIdx.x; i < OCC_DW; i += blockDim.x) s_odirty[i] = 0;
    __syncthreads();
    // (the barrier's workgroup release waits for wave 0's count atomics; the
    // rebuild reads the counts at device scope, from L2)
    pp_pass(d, a, scr_k, scr_v, pend, defer ? s_odirty : nullptr PT_ARGS);
    __syncthreads();
    if (defer) occ_rebuild_dirty(d, a, s_odirty);
    __syncthreads();
    PT_SUB(7);
  }
  PT_MARK(5, 1);
  ArenaCtl &c = d.ctl[a];
  const int T = blockDim.x, tid = threadIdx.x;
  // order-preserving compaction of viruses and blobs (list order == creation order),
  // only for lists that lost an entity this tick
  const uint32_t dirty = c.dirty;
  for (int kind = 0; kind < 2; kind++) {
    if (!(dirty & (kind == 0 ? DIRTY_VIRUS : DIRTY_BLOB))) continue;
    // blobs die every tick (stopped ones turn into pellets): the list keeps its
    // holes -- every consumer tests F_ALIVE and orders by seq -- until they are
    // half of it or it nears its capacity, so most ticks skip this pass -- but
    // never when the next tick's ejections could overflow the holes' list: every
    // player cell may eject once (field.py:134-146), and a split may double the
    // cells first, so the bound is 2 x this tick's cell-grid total
    if (kind == 1 && c.n_blob < 2 * c.n_blob_live + 256 && c.n_blob < d.Ecap / 2) {
      const int cc = cgrid_cols(d);
      const int ncell = d.cstart[(size_t)a * (d.H + 1) + cc * cc];
      if (c.n_blob + min(2 * ncell, kMaxCells * d.B) <= d.Ecap) continue;
    }
    int n = kind == 0 ? c.n_vir : c.n_blob;
    int cap = kind == 0 ? d.Vcap : d.Ecap;
    int out = 0;
    for (int base = 0; base < n; base += T) {
      int i = base + tid;
      size_t g = (size_t)a * cap + i;
      bool alive = i < n && ((kind == 0 ? d.v_flags[g] : d.b_flags[g]) & F_ALIVE);
      double f0 = 0, f1 = 0, f2 = 0, f3 = 0, f4 = 0, f5 = 0, f6 = 0, f7 = 0;
      int svc = 0, col = -1;
      int64_t s = 0, e = 0;
      uint32_t fl = 0;
      if (alive) {
        if (kind == 0) {
          f0 = d.v_x[g]; f1 = d.v_y[g]; f2 = d.v_m[g]; f3 = d.v_r[g]; f4 = d.v_vx[g]; f5 = d.v_vy[g];
          f6 = d.v_svx[g]; f7 = d.v_svy[g]; svc = d.v_svc[g]; s = d.v_seq[g]; fl = d.v_flags[g];
        } else {
          f0 = d.b_x[g]; f1 = d.b_y[g]; f2 = d.b_m[g]; f3 = d.b_r[g]; f4 = d.b_vx[g]; f5 = d.b_vy[g];
          f6 = d.b_svx[g]; f7 = d.b_svy[g]; svc = d.b_svc[g]; s = d.b_seq[g]; e = d.b_ej[g]; fl = d.b_flags[g];
          col = d.b_col[g];
        }
      }
      int chunk;
      const int pos = out + block_rank(alive, sflag, &chunk);  // (all loads of this chunk are done)
      if (alive) {
        size_t o = (size_t)a * cap + pos;
        if (kind == 0) {
          d.v_x[o] = f0; d.v_y[o] = f1; d.v_m[o] = f2; d.v_r[o] = f3; d.v_vx[o] = f4; d.v_vy[o] = f5;
          d.v_svx[o] = f6; d.v_svy[o] = f7; d.v_svc[o] = svc; d.v_seq[o] = s; d.v_flags[o] = fl;
        } else {
          d.b_x[o] = f0; d.b_y[o] = f1; d.b_m[o] = f2; d.b_r[o] = f3; d.b_vx[o] = f4; d.b_vy[o] = f5;
          d.b_svx[o] = f6; d.b_svy[o] = f7; d.b_svc[o] = svc; d.b_seq[o] = s; d.b_ej[o] = e; d.b_flags[o] = fl;
          d.b_col[o] = col;
        }
      }
      out += chunk;
      __syncthreads();
    }
    // clear the tail flags
    for (int i = out + tid; i < n; i += T) {
      size_t g = (size_t)a * cap + i;
      if (kind == 0) d.v_flags[g] = 0;
      else d.b_flags[g] = 0;
    }
    __syncthreads();
    if (tid == 0) {
      if (kind == 0) c.n_vir = out;
      else c.n_blob = out;
    }
    __syncthreads();
  }
  // the virus list is compacted: re-index the virus grid for the observations
  // (membership stays the F_INHASH flag; the viruses spawned below are not hashed)
  // (unchanged otherwise: viruses do not move after updateViruses, and the ones
  // appended by splits or spawns are not hashed this tick)
  PT_MARK(5, 2);
  if (d.virus_enabled && (dirty & DIRTY_VIRUS)) grid_small_build<2>(d, a, gcnt, sflag);
  PT_MARK(5, 3);
  // (the spawn occupancy is built by k_pp_active and kept by the pp pass above)
  // spawnPlayers' dead list (deadPlayers in order; respawnTime == 0 respawns):
  // partitioned by the whole block, a chunk of T players per round (a serial
  // loop was one load chain per dead player: ~8 us per greedy tick); every dead
  // player's respawn slot (its place in the respawn order, -1 = waits) is
  // what k_pel_update's player threads read
  int n_resp = 0, n_wait = 0;
  SpawnIn sin{};
  if (tid == 0) sin = spawn_in(c);  // (spawn_counts' fields: their round overlaps the partition's)
  if (!init) {
    const int nd = c.n_dead;
    int *dl = d.dead + (size_t)a * d.B, *rl = d.resp_slot + (size_t)a * d.B;
    for (int base = 0; base < nd; base += T) {
      const int i = base + tid;
      int p = -1;
      bool rsp = false;
      if (i < nd) {
        p = dl[i];
        rsp = d.p_respawn[(size_t)a * d.B + p] == 0;
      }
      int tr, tw;
      const int rr = block_rank(i < nd && rsp, sflag, &tr);
      const int rw = block_rank(i < nd && !rsp, sflag, &tw);  // (every read of this chunk is done)
      if (i < nd) rl[p] = rsp ? n_resp + rr : -1;
      if (i < nd && !rsp) dl[n_wait + rw] = p;  // (n_wait + rw <= i: never ahead of an unread entry)
      n_resp += tr;
      n_wait += tw;
    }
  }
  if (tid == 0) spawn_counts(d, a, init, n_resp, n_wait, sin);
  __syncthreads();
  PT_MARK(5, 4);
  if (close) {
    __syncthreads();
    pellet_close_prep(d, a);
  }
  PT_MARK(5, 5);
}

// spawnStuff's counts (field.py:227-280): pellets and viruses to add, players to respawn
// (n_resp / n_wait: the dead list's partition, done by the caller's block when !init)
// in: every field it reads, loaded in ONE round (spawn_in) before the arithmetic
// and the stores (read-modify-writes of the struct in place cost a round each: a
// load after a store to the same struct cannot move above it)
__device__ __forceinline__ void spawn_counts(const Dev &d, int a, int init, int n_resp, int n_wait, const SpawnIn &in) {
  ArenaCtl &c = d.ctl[a];
  const int n_pel = in.n_pel, n_pel_eaten = in.n_pel_eaten, n_pnew = in.n_pnew;
  const int n_pel_glob = in.n_pel_glob, n_eaten_glob = in.n_eaten_glob, n_vir = in.n_vir;
  const int64_t seq_next = in.seq_next, tick = in.tick, stat3 = in.stat3, stat5 = in.stat5;
  const uint64_t ctr_pellet = in.ctr_pellet, ctr_virus = in.ctr_virus;
  uint32_t err = 0;
  // spawnPellets: while len(pellets) < maxCollectibleCount
  // (tiles: the global count -- every tile spawns the same global list and keeps what it holds)
  const int alive_p = d.tiled ? n_pel_glob - n_eaten_glob + n_pnew : n_pel - n_pel_eaten + n_pnew;
  int kp = 0;
  if ((double)alive_p < d.max_pellets) kp = (int)ceil(d.max_pellets) - alive_p;
  if (alive_p + kp > d.Pcap || n_pnew + kp > d.Pcap) {
    err |= ERR_PELLET_CAP;
    kp = max(0, min(d.Pcap - alive_p, d.Pcap - n_pnew));
  }
  // spawnViruses
  int kv = 0;
  if (d.virus_enabled && (double)n_vir < d.max_viruses) kv = (int)ceil(d.max_viruses) - n_vir;
  if (n_vir + kv > d.Vcap) {
    err |= ERR_VIRUS_CAP;
    kv = d.Vcap - n_vir;
  }
  // spawnPlayers: deadPlayers in order, respawnTime == 0 (init: every player, in order)
  const int np = init ? d.B : n_resp;
  c.dirty = 0;
  if (err) c.err |= err;
  c.seq_base_spawn = seq_next;
  c.ctr_pellet_base = ctr_pellet;
  c.ctr_pellet = ctr_pellet + kp;
  c.n_spawn_p = kp;
  c.n_pel_glob = alive_p + kp;
  if (!init) {  // diagnostics: pellets eaten / respawned this tick (whole arena)
    c.stat[3] = stat3 + (d.tiled ? n_eaten_glob : n_pel_eaten);
    c.stat[5] = stat5 + kp;
  }
  c.ctr_virus_base = ctr_virus;
  c.ctr_virus = ctr_virus + kv;
  c.vir_base_spawn = n_vir;
  c.n_spawn_v = kv;
  c.n_vir = n_vir + kv;
  if (!init) {
    c.n_dead = n_wait;
    c.tick_sp = tick;
  }
  c.n_spawn_pl = np;
  // (at initialize() players already own seqs 0..B-1)
  c.seq_next = seq_next + kp + kv + (init ? 0 : np);
}

__global__ void k_pnew_commit(Dev d) {
  int a = GTID;
  if (a >= d.A) return;
  d.ctl[a].n_pnew += d.ctl[a].n_spawn_p;
}

// spawn j of this tick (j < n_spawn_p): its record, a function of (key, counter) only
__device__ __forceinline__ void spawn_pellet_rec(const Dev &d, const ArenaCtl &c, int j, double &x, double &y,
                                                 double &m, int64_t &seq) {
  uint64_t u[4];
  philox(c.ctr_pellet_base + j, ST_PELLET, 0, 0, c.key0, c.key1, u);
  x = (double)(int64_t)mulhi(u[0], (uint64_t)d.size);
  y = (double)(int64_t)mulhi(u[1], (uint64_t)d.size);
  const int64_t sr = (int64_t)mulhi(u[2], 50);
  m = (sr > 50 - 4) ? (double)(50 - sr) : 1.0;  // randomSize (field.py:20-26)
  seq = c.seq_base_spawn + j;
}
// ... into the staging list; its position also to *px, *py
__device__ void spawn_pellet_at(const Dev &d, int a, int j, double *px, double *py) {
  const ArenaCtl &c = d.ctl[a];
  double x, y, m;
  int64_t seq;
  spawn_pellet_rec(d, c, j, x, y, m, seq);
  size_t o = (size_t)a * d.Pcap + c.n_pnew + j;
  d.pn[o] = PelRec{x, y, m, seq};
  d.pn_col[o] = -1;  // Cell(..., None): a colour of its own
  if (px) {
    *px = x;
    *py = y;
  }
}
__device__ __forceinline__ void spawn_pellet(const Dev &d, int gi) {
  if (gi >= d.A * d.Pcap) return;
  int a = gi / d.Pcap, j = gi - a * d.Pcap;
  ArenaCtl &c = d.ctl[a];
  if (j >= c.n_spawn_p) return;
  uint64_t u[4];
  philox(c.ctr_pellet_base + j, ST_PELLET, 0, 0, c.key0, c.key1, u);
  int64_t x = (int64_t)mulhi(u[0], (uint64_t)d.size), y = (int64_t)mulhi(u[1], (uint64_t)d.size);
  int64_t sr = (int64_t)mulhi(u[2], 50);
  double m = (sr > 50 - 4) ? (double)(50 - sr) : 1.0;  // randomSize (field.py:20-26)
  size_t o = (size_t)a * d.Pcap + c.n_pnew + j;
  d.pn[o] = PelRec{(double)x, (double)y, m, c.seq_base_spawn + j};
  d.pn_col[o] = -1;  // Cell(..., None): a colour of its own
}
__global__ void k_spawn_pellets(Dev d) { spawn_pellet(d, GTID); }
__device__ __forceinline__ void spawn_virus(const Dev &d, int gi) {
  if (gi >= d.A * d.Vcap) return;
  int a = gi / d.Vcap, j = gi - a * d.Vcap;
  ArenaCtl &c = d.ctl[a];
  if (j >= c.n_spawn_v) return;
  uint64_t u[4], u2[4];
  philox(c.ctr_virus_base + j, ST_VIRUS, 0, 0, c.key0, c.key1, u);
  philox(c.ctr_virus_base + j, ST_VIRUS, 1, 0, c.key0, c.key1, u2);
  const double vr = radius_of(kVirusBase);
  double x, y;
  spawn_pos(d, a, vr, u, x, y);
  double rng = kBucket - vr;
  x += (double)ph_randint(u2[0], (-1) * rng / 2, rng / 2);
  y += (double)ph_randint(u2[1], (-1) * rng / 2, rng / 2);
  size_t o = (size_t)a * d.Vcap + c.vir_base_spawn + j;
  d.v_x[o] = x;
  d.v_y[o] = y;
  d.v_m[o] = kVirusBase;
  d.v_r[o] = vr;
  d.v_vx[o] = 0;
  d.v_vy[o] = 0;
  d.v_svx[o] = 0;
  d.v_svy[o] = 0;
  d.v_svc[o] = 0;
  d.v_seq[o] = c.seq_base_spawn + c.n_spawn_p + j;
  d.v_flags[o] = F_ALIVE;  // addVirus: not hashed until the next rebuild
}
__global__ void k_spawn_viruses(Dev d) { spawn_virus(d, GTID); }
// player gp (= arena a's player p) spawns j-th in spawnPlayers' order
__device__ __forceinline__ void spawn_player(const Dev &d, int gp, int j, int init) {
  const int a = gp / d.B, p = gp - a * d.B;
  ArenaCtl &c = d.ctl[a];
  const int NP = d.NP;
  uint64_t u[4];
  if (init) philox((uint64_t)p, ST_INIT_PLAYER, 0, 0, c.key0, c.key1, u);
  else philox((uint64_t)p, ST_PLAYER, (uint64_t)c.tick_sp, 0, c.key0, c.key1, u);
  const double sr = radius_of(kStartMass);
  double x, y;
  spawn_pos(d, a, sr, u, x, y);
  int64_t seq = init ? (int64_t)j : c.seq_base_spawn + c.n_spawn_p + c.n_spawn_v + j;
  if (init) seq = (int64_t)j;  // Field.initialize: players first
  for (int k = 0; k < kMaxCells; k++) d.c_flags[(size_t)k * NP + gp] = 0;
  size_t ci = (size_t)gp;  // slot 0
  d.c_x[ci] = x;
  d.c_y[ci] = y;
  d.c_m[ci] = kStartMass;
  d.c_r[ci] = sr;
  d.c_vx[ci] = 0;
  d.c_vy[ci] = 0;
  d.c_svx[ci] = 0;
  d.c_svy[ci] = 0;
  d.c_svc[ci] = 0;
  d.c_mt[ci] = 0;
  d.c_seq[ci] = seq;
  d.c_flags[ci] = F_ALIVE;  // initializePlayer does not hash the cell
  d.p_list[gp] = 0;
  d.p_ncells[gp] = 1;
  d.p_alive[gp] = 1;
  d.p_respawn[gp] = 0;
  if (!init) ev_push_at(d, a, c.tick_sp, PH_SPAWN, (uint64_t)j, 10, p, seq);
}
__global__ void k_spawn_players(Dev d, int init) {  // Field.initialize: every player, in order
  const int gp = GTID;
  if (gp < d.NP) spawn_player(d, gp, gp % d.B, init);
}
// the end of spawnStuff for live-or-dead player gp: a dead player whose respawn
// slot k_spawn_plan set respawns, then the FOV cache of the end-of-tick state
// (one thread per player, so the respawn and its cache need no ordering)
__device__ __forceinline__ void respawn_fov_thread(const Dev &d, int gp) {
  if (gp < d.NP && !d.p_alive[gp]) {
    const int j = d.resp_slot[gp];
    if (j >= 0) spawn_player(d, gp, j, 0);
  }
  fov_cache_thread(d, gp);
}

// Step 2 of the closing pellet update (see pellet_close_prep): one block per
// bucket row of every arena, + extra blocks for the rest of spawnStuff, which
// reads nothing this launch writes: the player respawns with the FOV cache
// (respawn_fov_thread), then the virus spawns.  A row block finds whether a
// killed slot (kill_list) lies in its row or a joining staged record (a blob
// conversion nobody ate, a spawn; tiles: in the held range) has its centre in
// it; if so it writes the row anew -- survivors by bucket in their old order,
// each bucket's new records behind them (consumers rank candidates by creation
// sequence, so order inside a bucket carries no meaning) -- and the row's bucket
// starts.  Only the suffix from the first changed slot (the first kill, or the
// old end of the first bucket a record joins) moves: it is parked in LDS and
// written back in the row's home, the slots before it untouched; a suffix
// longer than PU_LDS slots moves the whole row into its other home instead.
// Rows nothing touched are left alone (their bucket starts not even read).
constexpr int PU_ROW_STG = 512;  // joining records per row and tick (more: ERR_PELLET_CAP)
constexpr int kPelRowCols = 1024;  // buckets per row the update handles (aigar_create checks)
__device__ __forceinline__ int block_excl1(int v, int *wsum, int &total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int before = 0;
  total = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); k++) {
    before += k < w ? wsum[k] : 0;
    total += wsum[k];
  }
  __syncthreads();
  return before + inc - v;
}
// two exclusive block scans in one pass (one barrier): a, one value per thread
// in thread order, and p[0..3], four per thread (thread t holds items 4t .. 4t+3);
// tp = p's total.  wsum: 8 entries.
__device__ __forceinline__ void block_scan_pair(int &a, int64_t *p, int64_t *wsum, int64_t &tp) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  const int sa = a;
  const int64_t sp = p[0] + p[1] + p[2] + p[3];
  int ia = sa;
  int64_t ip = sp;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int ya = __shfl_up(ia, off);
    const int64_t yp = __shfl_up(ip, off);
    if (lane >= off) {
      ia += ya;
      ip += yp;
    }
  }
  if (lane == 63) {
    wsum[w] = ia;
    wsum[4 + w] = ip;
  }
  __syncthreads();
  int64_t ba = 0, bp = 0;
  tp = 0;
  for (int k = 0; k < nw; k++) {
    ba += k < w ? wsum[k] : 0;
    bp += k < w ? wsum[4 + k] : 0;
    tp += wsum[4 + k];
  }
  a = (int)ba + ia - sa;
  int64_t run = bp + ip - sp;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int64_t x = p[k];
    p[k] = run;
    run += x;
  }
}
constexpr int PU_JREC = 64;  // joining records per row kept whole in LDS (beyond: loaded again)
constexpr int PU_LDS = 512;  // row slots whose records the update parks in LDS (longer rows: two rounds)
constexpr int PU_K = PU_LDS / 256;  // consecutive slots per thread
__device__ void pel_row_update(const Dev &d, int a, int r PT_PARAMS) {
  __shared__ int s_flag[3];
  __shared__ int s_sj[PU_ROW_STG];
  __shared__ short s_sbx[PU_ROW_STG];
  __shared__ PelRec s_jrec[PU_JREC];
  __shared__ int s_jcol[PU_JREC];
  __shared__ PelRec s_rec[PU_LDS];
  __shared__ int s_rcol[PU_LDS];
  __shared__ int s_ost[kPelRowCols + 1];  // the row's old bucket starts (absolute slots)
  __shared__ int s_live[kPelRowCols], s_stc[kPelRowCols];  // per bucket: survivors, joining records
  __shared__ int s_lpre[kPelRowCols], s_nofs[kPelRowCols];  // survivors before the bucket; its new start - row base
  __shared__ int wsum[4];
  __shared__ int64_t wsum2[8];
  __shared__ short s_slotb[PU_LDS];  // a parked suffix slot's old bucket
  const int tid = threadIdx.x, C = d.cols;
  ArenaCtl &c = d.ctl[a];
  const int nconv = c.pu_nconv, nst = nconv + c.pu_nsp, spec = c.pu_spec;
  const int nk = min(c.n_kill, d.Pcap);
  int *e0 = d.pstart + (size_t)a * d.PH1 + (size_t)r * (C + 1);
  const size_t S0 = (size_t)a * d.PS, D0 = (size_t)a * d.PD, Q0 = (size_t)a * d.Pcap;
  // round 1, ONE round of independent loads: the row's bucket starts, the
  // tick's first kills and staged records (a staged record joining the row is
  // kept whole in LDS: it is there when the row is written)
  const int *kl = d.kill_list + Q0;
  if (tid == 0) {
    s_flag[0] = s_flag[1] = 0;
    s_flag[2] = INT_MAX;  // the row's first changed slot
  }
  for (int bx = tid; bx <= C; bx += blockDim.x) {
    s_ost[bx] = e0[bx];
    if (bx < C) s_stc[bx] = 0;
  }
  const int kill0 = tid < nk ? kl[tid] : -1;
  // staged record j: whether it joins this row (its centre bucket's column, or -1)
  auto staged = [&](int j, PelRec &rec, int &col) {
    col = -1;
    bool live = true;
    if (j < nconv) {
      rec = d.pn[Q0 + j];
      col = d.pn_col[Q0 + j];
      live = !d.pel_dead[D0 + d.PS + j];  // (a conversion eaten this tick does not join)
    } else if (spec) {  // a spawn drawn ahead by k_players' arena block
      const size_t o = (size_t)a * kSpawnAhead + (j - nconv);
      rec = PelRec{d.spec_x[o], d.spec_y[o], d.spec_m[o], c.seq_base_spawn + (j - nconv)};
    } else {
      rec = d.pn[Q0 + j];
      col = d.pn_col[Q0 + j];
    }
    const int by = center_bucket_coord(rec.y, C);
    if (!live || by != r) return -1;
    const int bx = center_bucket_coord(rec.x, C);
    return tile_holds_bucket(d, bx, by) ? bx : -1;
  };
  auto stage = [&](int j, int bx, const PelRec &rec, int col) {
    const int k = atomicAdd(&s_flag[1], 1);
    if (k < PU_ROW_STG) {
      s_sj[k] = j;
      s_sbx[k] = (short)bx;
      if (k < PU_JREC) {
        s_jrec[k] = rec;
        s_jcol[k] = col;
      }
    }
  };
  PelRec rec0;
  int col0 = -1, bx0 = -1;
  if (tid < nst) bx0 = staged(tid, rec0, col0);
  __syncthreads();
  PT_MARK(8, 1);
  const int lo = s_ost[0], hi = s_ost[C];
  auto kill = [&](int k) {
    if (k >= lo && k < hi) {
      s_flag[0] = 1;
      atomicMin(&s_flag[2], k);
    }
  };
  kill(kill0);
  for (int t = tid + blockDim.x; t < nk; t += blockDim.x) kill(kl[t]);
  if (bx0 >= 0) stage(tid, bx0, rec0, col0);
  for (int j = tid + blockDim.x; j < nst; j += blockDim.x) {
    PelRec rec;
    int col;
    const int bx = staged(j, rec, col);
    if (bx >= 0) stage(j, bx, rec, col);
  }
  __syncthreads();
  PT_MARK(8, 2);
  const int ns_all = s_flag[1];
  if (!s_flag[0] && ns_all == 0) return;  // (uniform) untouched row
  // More joining records than the LDS list holds (a large refill, e.g. the first
  // tick after load_state of a depleted world): the list is dropped and the
  // staged records are walked again, counted here and placed in chunks below.
  const bool over = ns_all > PU_ROW_STG;  // (uniform)
  const int ns = over ? 0 : ns_all;
  // a join goes behind its bucket's survivors: the row changes from that bucket's old end
  for (int k = tid; k < ns; k += blockDim.x) {
    atomicAdd(&s_stc[s_sbx[k]], 1);
    atomicMin(&s_flag[2], s_ost[s_sbx[k] + 1]);
  }
  if (over) {
    for (int j = tid; j < nst; j += blockDim.x) {
      PelRec rec;
      int col;
      const int bx = staged(j, rec, col);
      if (bx >= 0) {
        atomicAdd(&s_stc[bx], 1);
        atomicMin(&s_flag[2], s_ost[bx + 1]);
      }
    }
  }
  __syncthreads();
  const int f = min(s_flag[2], hi);
  // in place (the row's home) when the changed suffix [f, hi) fits LDS: the slots
  // before f keep their records and bucket starts and are neither read nor
  // written; else the whole row into its other home
  const bool inplace = hi - f <= PU_LDS;
  const int home = C * d.PR, nb = inplace ? lo : lo >= home ? lo - home : lo + home;
  auto bucket_of = [&](int i) {  // old bucket of slot i: s_ost[bx] <= i < s_ost[bx + 1]
    int l = 0, h = C;  // invariant: s_ost[l] <= i < s_ost[h]
    while (h - l > 1) {
      const int m = (l + h) >> 1;
      if (s_ost[m] <= i) l = m;
      else h = m;
    }
    return l;
  };
  const int lim = nb + d.PR;
  // the row's bucket starts from per-bucket survivor + join counts (s_live / s_stc
  // complete: the caller's scan begins with a barrier)
  auto bucket_scans = [&]() {
    int v[4], w[4];
    for (int k = 0; k < 4; k++) {
      const int bx = tid * 4 + k;
      v[k] = bx < C ? s_live[bx] + s_stc[bx] : 0;
      w[k] = bx < C ? s_live[bx] : 0;
    }
    const int total = block_scan4(v, wsum);
    (void)block_scan4(w, wsum);
    for (int k = 0; k < 4; k++) {
      const int bx = tid * 4 + k;
      if (bx < C) {
        s_nofs[bx] = v[k];
        s_lpre[bx] = w[k];
      }
    }
    if (total > d.PR && tid == 0) set_err(d, a, ERR_PELLET_CAP);
    __syncthreads();
    return total;
  };
  int total;
  if (inplace) {
    // round 2: thread t's PU_K consecutive suffix slots -- liveness, records,
    // colours in ONE round of loads, parked in LDS (the suffix is rewritten in
    // place: every record is read before any is written)
    const int i0 = f + PU_K * tid;
    uint32_t livem = 0;
#pragma unroll
    for (int k = 0; k < PU_K; k++) {
      const int i = i0 + k;
      if (i < hi) {
        livem |= d.pel_dead[D0 + i] ? 0u : 1u << k;
        s_rec[i - f] = d.pel[S0 + i];
        s_rcol[i - f] = d.pel_col[S0 + i];
      }
    }
    // meanwhile, with LDS alone: every suffix slot's old bucket (scattered by
    // bucket: buckets are a few slots long), the survivors before f
    for (int bx = tid; bx < C; bx += blockDim.x) {
      const int s0 = s_ost[bx], s1 = s_ost[bx + 1];
      for (int i = max(s0, f); i < s1; i++) s_slotb[i - f] = (short)bx;
      s_live[bx] = max(0, min(s1, f) - s0);
    }
    __syncthreads();
    int bk[PU_K];
#pragma unroll
    for (int k = 0; k < PU_K; k++) {
      const int i = i0 + k;
      bk[k] = 0;
      if (i >= hi) continue;
      bk[k] = s_slotb[i - f];
      if ((livem >> k) & 1) atomicAdd(&s_live[bk[k]], 1);
      else d.pel_dead[D0 + i] = 0;  // eaten: dropped, and its flag clean for whatever lands on the slot
    }
    __syncthreads();
    // ONE pass of scans: the survivors' order over the suffix, the new bucket starts
    int pk[4];
    int64_t pb[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int bx = tid * 4 + k;
      pk[k] = bx < C ? s_live[bx] : 0;
      pb[k] = bx < C ? ((int64_t)s_stc[bx] << 32) | (uint32_t)pk[k] : 0;
    }
    int ex = __popc(livem);
    int64_t tb;
    block_scan_pair(ex, pb, wsum2, tb);
    ex += f - lo;
    total = (int)(tb >> 32) + (int)(uint32_t)tb;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int bx = tid * 4 + k;
      if (bx < C) {
        const int lp = (int)(uint32_t)pb[k];
        s_nofs[bx] = lp + (int)(pb[k] >> 32);
        s_lpre[bx] = lp;
      }
    }
    if (total > d.PR && tid == 0) set_err(d, a, ERR_PELLET_CAP);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PU_K; k++)
      if ((livem >> k) & 1) {
        const int bx = bk[k], pos = nb + s_nofs[bx] + (ex - s_lpre[bx]);
        ex++;
        if (pos < lim && pos != i0 + k) {
          d.pel[S0 + pos] = s_rec[i0 + k - f];
          d.pel_col[S0 + pos] = s_rcol[i0 + k - f];
        }
      }
  } else {  // (longer rows: the same in chunks of 256 slots, the records loaded after the count)
    for (int bx = tid; bx < C; bx += blockDim.x) s_live[bx] = 0;
    __syncthreads();
    for (int i = lo + tid; i < hi; i += blockDim.x)
      if (!d.pel_dead[D0 + i]) atomicAdd(&s_live[bucket_of(i)], 1);
    __syncthreads();
    total = bucket_scans();
    // survivors: slot i of bucket bx -> nb + new start + (survivors of bx before i)
    int carry = 0;
    for (int c0 = lo; c0 < hi; c0 += blockDim.x) {
      const int i = c0 + tid;
      bool live = false;
      if (i < hi) live = !d.pel_dead[D0 + i];
      int tot;
      const int ex = carry + block_excl1(live ? 1 : 0, wsum, tot);
      carry += tot;
      if (i < hi) {
        if (live) {
          const int bx = bucket_of(i);
          const int pos = nb + s_nofs[bx] + (ex - s_lpre[bx]);
          if (pos < lim) {
            d.pel[S0 + pos] = d.pel[S0 + i];
            d.pel_col[S0 + pos] = d.pel_col[S0 + i];
          }
        } else {
          d.pel_dead[D0 + i] = 0;
        }
      }
    }
  }
  // joining records: behind the bucket's survivors, in staging order
  for (int k = tid; k < ns; k += blockDim.x) {
    const int j = s_sj[k], bx = s_sbx[k];
    int rk = 0;
    for (int q = 0; q < ns; q++) rk += s_sbx[q] == bx && s_sj[q] < j;
    const int pos = nb + s_nofs[bx] + s_live[bx] + rk;
    if (pos >= lim) continue;
    PelRec rec;
    int col = -1;
    if (k < PU_JREC) {
      rec = s_jrec[k];
      col = s_jcol[k];
    } else if (j >= nconv && spec) {
      const size_t o = (size_t)a * kSpawnAhead + (j - nconv);
      rec = PelRec{d.spec_x[o], d.spec_y[o], d.spec_m[o], c.seq_base_spawn + (j - nconv)};
    } else {
      rec = d.pn[Q0 + j];
      col = d.pn_col[Q0 + j];
    }
    d.pel[S0 + pos] = rec;
    d.pel_col[S0 + pos] = col;
  }
  if (over) {
    // the overflow's joins in chunks of blockDim staged records, in staging order:
    // a record's rank in its bucket = the bucket's joins of earlier chunks
    // (s_lpre, free once the survivors are placed) + its bucket mates earlier in
    // its chunk (s_sbx, free once the list is dropped)
    __syncthreads();
    for (int bx = tid; bx < C; bx += blockDim.x) s_lpre[bx] = 0;
    for (int c0 = 0; c0 < nst; c0 += blockDim.x) {
      const int j = c0 + tid;
      PelRec rec;
      int col = -1, bx = -1;
      if (j < nst) bx = staged(j, rec, col);
      s_sbx[tid] = (short)bx;
      __syncthreads();
      if (bx >= 0) {
        int rk = 0;
        for (int q = 0; q < tid; q++) rk += s_sbx[q] == bx;
        const int pos = nb + s_nofs[bx] + s_live[bx] + s_lpre[bx] + rk;
        if (pos < lim) {
          d.pel[S0 + pos] = rec;
          d.pel_col[S0 + pos] = col;
        }
      }
      __syncthreads();
      if (bx >= 0) atomicAdd(&s_lpre[bx], 1);
      __syncthreads();
    }
  }
  for (int bx = tid; bx < C; bx += blockDim.x) {
    const int st = nb + min(s_nofs[bx], d.PR);
    if (st != s_ost[bx]) e0[bx] = st;  // (in place: the starts up to f's bucket stay)
  }
  if (tid == 0) {
    e0[C] = nb + min(total, d.PR);
    atomicAdd(&c.n_pel, min(total, d.PR) - (hi - lo));
  }
}
__global__ void __launch_bounds__(256) k_pel_update(Dev d, int nbF) {
  FLOOR(8);
  PT_BEGIN(8);
  const int nup = d.A * d.cols;
  if ((int)blockIdx.x >= nup + nbF) {
    spawn_virus(d, (blockIdx.x - nup - nbF) * 256 + threadIdx.x);
    PT_MARK(8, 5);
    return;
  }
  if ((int)blockIdx.x >= nup) {
    respawn_fov_thread(d, (blockIdx.x - nup) * 256 + threadIdx.x);
    PT_MARK(8, 4);
    return;
  }
  const int a = blockIdx.x / d.cols, r = blockIdx.x - a * d.cols;
  if (r == 0 && threadIdx.x == 0) d.ctl[a].tick += 1;  // (nothing in this launch reads it)
  pel_row_update(d, a, r PT_ARGS);
  PT_MARK(8, 3);
}

// aigar_get_state's pellet records: every row's live range [start of bucket 0,
// end of the last bucket) of arena a, packed in row order into the staging list
// (free between ticks), so one copy of the live records leaves the device instead
// of the whole two-home row store.  One block per row; its offset is the sum of
// the earlier rows' lengths.
__global__ void __launch_bounds__(256) k_pel_gather(Dev d, int a) {
  __shared__ int wsum[4];
  const int r = blockIdx.x, C = d.cols, tid = threadIdx.x;
  const int *pst = d.pstart + (size_t)a * d.PH1;
  int part = 0;
  for (int q = tid; q < r; q += blockDim.x) part += pst[(size_t)q * (C + 1) + C] - pst[(size_t)q * (C + 1)];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
  if ((tid & 63) == 0) wsum[tid >> 6] = part;
  __syncthreads();
  const int off = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  const int lo = pst[(size_t)r * (C + 1)], hi = pst[(size_t)r * (C + 1) + C];
  const size_t S0 = (size_t)a * d.PS, Q0 = (size_t)a * d.Pcap;
  for (int i = lo + tid; i < hi; i += blockDim.x) {
    const int o = off + (i - lo);
    if (o >= d.Pcap) break;  // (the caller checks the total)
    d.pn[Q0 + o] = d.pel[S0 + i];
    d.pn_col[Q0 + o] = d.pel_col[S0 + i];
  }
}
void launch_pel_gather(const Dev &d, hipStream_t s, int a) {
  hipLaunchKernelGGL(k_pel_gather, dim3(d.cols), dim3(256), 0, s, d, a);
}

// ------------------------------------------------------------ init helpers
__global__ void k_init_ctl(Dev d, uint64_t seed) {
  int a = GTID;
  if (a >= d.A) return;
  ArenaCtl &c = d.ctl[a];
  c.seq_next = d.B;  // players take 0..B-1 (Field.initialize order)
  c.tick = 0;
  c.key0 = seed;
  c.key1 = ((uint64_t)a << 32) | 0x9E3779B9ull;
  c.ctr_pellet = c.ctr_virus = 0;
  c.n_pel = c.n_pnew = c.n_pel_eaten = 0;
  c.n_blob = c.n_blob_base = 0;
  c.n_vir = c.n_vir_start = 0;
  c.n_dead = 0;
  c.n_ev = 0;
  c.n_pend = c.n_pend2 = 0;
  c.n_kill = 0;
  c.pu_nconv = c.pu_nsp = c.pu_spec = 0;
  c.err = c.warn = 0;
  c.rmax_cell = radius_of(kStartMass);
  c.rmax_virus = radius_of(kVirusBase);
  c.food_round = 1;
  c.scan_epoch[0] = c.scan_epoch[1] = 0;
  c.pl_epoch = 0;
  c.dirty = 0;
  c.pl_ticket = 0;
  c.scan_ticket[0] = c.scan_ticket[1] = 0;
  c.n_pel_glob = c.n_eaten_glob = c.n_out = c.n_out_pel = c.n_undone = c.n_undone_glob = 0;
  c.n_ho = c.n_ho_live = 0;
  for (int k = 0; k < 8; k++) c.stat[k] = 0;
}

// ------------------------------------------------------------ launch sequences
static inline int nblk(long n, int t) { return (int)((n + t - 1) / t); }

struct Scratch {
  int64_t *k;
  int *v;
};

// Field.initialize's pellets: the staging list -> home 0 of every row (counting sort)
void launch_pellet_rows(const Dev &d, hipStream_t s) {
  const long n = (long)d.A * d.Pcap;
  hipLaunchKernelGGL(k_prow_count, dim3(nblk(n, 256)), dim3(256), 0, s, d);
  hipLaunchKernelGGL(k_prow_scan, dim3(d.cols, d.A), dim3(256), 0, s, d);
  hipLaunchKernelGGL(k_prow_scatter, dim3(nblk(n, 256)), dim3(256), 0, s, d);
}


// playerPelletOverlap + playerBlobOverlap: prep, reservation rounds (>= 1),
// serial rest; the player-cell grid's scan rides along as the prep's head
// blocks and its placement in round 1's player threads (cgrid_count_cell).
// (resume: a further eat pass of a tiled tick -- the cell grid is built already)
static void launch_food(const Dev &d, hipStream_t s, int rounds, Scratch scr, int resume = 0, int fold = 0) {
  rounds = std::max(rounds, 1);
  const int g = nblk(d.NP, 256);
  if (d.share_cells)
    hipLaunchKernelGGL(k_food_prep<true>, dim3(std::max(nblk((long)d.NP * PREP_WAVES, 4), resume ? 0 : d.A)), dim3(256),
                       0, s, d, rounds, resume);
  else
    hipLaunchKernelGGL(k_food_prep<false>, dim3(std::max(nblk((long)d.NP * PREP_WAVES, 4), resume ? 0 : d.A)), dim3(256),
                       0, s, d, rounds, resume);
  for (int r = 1; r <= rounds; r++) {
    hipLaunchKernelGGL(k_food_commit, dim3(g), dim3(256), 0, s, d, r, r == rounds ? 1 : 0, scr.k, scr.v, rounds,
                       fold && r == rounds ? 1 : 0, r == 1 && !resume ? 1 : 0);
  }
  if (!fold) hipLaunchKernelGGL(k_food_serial, dim3(d.A), dim3(64), 0, s, d, scr.k, scr.v, rounds);
}

void launch_player_fov(const Dev &d, hipStream_t s);
// One Field.update(): a single stream of dependent launches (captured once into a
// hipGraph by api.hip).  Forking independent phases onto a second stream was
// measured slower on MI355X (cross-queue dependencies cost more than the
// overlap gains at this kernel size), so the graph stays linear.
// the phases before the eat phase (field.py:94-198, 225-231, 246-253)
void launch_tick_pre(const Dev &d, hipStream_t s, int64_t *scr_k, int *scr_v, const RandomPolicy *rp) {
  // the tick's first launch: per player tile its cells, then the players (+ C4:
  // the observation hand-off plan); per arena one block for the viruses, spawns
  // drawn ahead and the virus grid, and blocks for the blobs and the resets
  hipLaunchKernelGGL(k_players, dim3(d.pl_tiles + 1 + (d.Ecap + kPlT - 1) / kPlT, d.A), dim3(kPlT), 0, s, d, rp ? *rp : RandomPolicy{0, 0, 0, 0});
  if (d.virus_enabled)  // merges, both virus activity tests, the blob grid, both serial passes (last block)
    hipLaunchKernelGGL(k_merge_pv, dim3(nblk(d.NP, 256) + nblk((long)d.A * d.Ecap, 256) + d.A), dim3(256), 0, s, d,
                       scr_k, scr_v);
  else
    hipLaunchKernelGGL(k_merge_vb, dim3(nblk(d.NP, 256) + d.A), dim3(256), 0, s, d, scr_k, scr_v, 0);
}
// the phases after it: playerPlayerOverlap, spawnStuff, closing rebuild (field.py:233-313)
void launch_tick_post(const Dev &d, hipStream_t s, int64_t *scr_k, int *scr_v) {
  if (d.share_cells) hipLaunchKernelGGL(k_pp_active<true>, dim3(nblk(d.NP, 4)), dim3(256), 0, s, d);
  else hipLaunchKernelGGL(k_pp_active<false>, dim3(nblk(d.NP, 4)), dim3(256), 0, s, d);
  // playerPlayerOverlap's serial pass + spawnStuff's plan + the end-of-tick virus
  // grid + the closing pellet update's sorted kill / join lists (and the pellet spawns)
  hipLaunchKernelGGL(k_spawn_plan, dim3(d.A), dim3(1024),
                     sizeof(uint32_t) * ((d.B + 31) / 32) * PPG_WAVES + (d.B <= PP_LOWN_MAX ? sizeof(int) * d.B : 0), s, d, 0,
                     scr_k, scr_v, 1, 1);  // (pending bitmaps: one per parallel pp group wave)
  // the closing pellet update (survivors U joining staged records -> the new
  // current buffer) + the rest of spawnStuff as extra blocks: player respawns
  // with the FOV cache, virus spawns (fused into the pellet threads the FOV
  // cache stretched the kernel; as separate blocks they only add to the grid)
  const int nbF = nblk(d.NP, 256);
  const int nbV = d.virus_enabled ? nblk((long)d.A * d.Vcap, 256) : 0;
  hipLaunchKernelGGL(k_pel_update, dim3(d.A * d.cols + nbF + nbV), dim3(256), 0, s, d, nbF);
}
void launch_tick(const Dev &d, hipStream_t s, int rounds, int64_t *scr_k, int *scr_v, const RandomPolicy *rp) {
  launch_tick_pre(d, s, scr_k, scr_v, rp);
  launch_food(d, s, rounds, Scratch{scr_k, scr_v}, 0, 1);
  launch_tick_post(d, s, scr_k, scr_v);
}

// ------------------------------------------------------------ C4 tile passes
// One eat pass of a tiled tick: (first: the tick's pellet-kill total restarts)
// the eat phase for the not-yet-final cells, then the message -- records were
// appended by the eat loops; the bitmap marks the owned cells now final; the
// header carries the record count, the owned cells left undone and the pellet
// kills.
__global__ void k_tile_pass_begin(Dev d) {  // a later pass
  ArenaCtl &c = d.ctl[0];
  c.n_out = c.n_out_pel = c.n_undone = 0;
  c.n_ho = c.n_ho_live = 0;
  // a fresh, empty header: when the pass is gated (no undone cell anywhere) the
  // collect kernel returns before writing one, and the previous pass's header
  // (its pellet kills) must not be exchanged and summed a second time
  TileRec &hd = d.outbox[0];
  hd.kind = TR_HDR;
  hd.idx = 0;
  hd.seq = 0;
  hd.x = hd.y = 0.0;
}
__device__ void tile_header(const Dev &d);
__global__ void __launch_bounds__(256) k_tile_collect(Dev d, int with_bitmap) {
  TILE_GATE(d);
  const int gp = GTID;
  if (gp < d.NP && d.p_alive[gp]) {
    unsigned long long *bm = (unsigned long long *)(d.outbox + 1 + d.tcap);
    const int NP = d.NP, n = d.p_ncells[gp];
    int und = 0;
    for (int k = 0; k < n; k++) {
      const size_t ci = (size_t)d.p_list[k * NP + gp] * NP + gp;
      if (!tile_owns(d, d.c_x[ci], d.c_y[ci])) continue;
      if (d.f_done[ci] != 1) und++;
      else if (with_bitmap) atomicOr(&bm[ci >> 6], 1ull << (ci & 63));
    }
    if (und) atomicAdd(&d.ctl[0].n_undone, und);
  }
  // the message header, once every owned cell is counted (the last block); on
  // the first pass, first the live bots' history hand-offs
  if (last_block(d.ticket + 3, gridDim.x)) {
    if (!with_bitmap) tile_plan_live(d);
    if (threadIdx.x == 0) tile_header(d);
  }
}
__device__ void tile_header(const Dev &d) {
  const ArenaCtl &c = d.ctl[0];
  TileRec &h = d.outbox[0];
  h.kind = TR_HDR;
  h.idx = min(c.n_out, d.tcap);
  h.seq = c.n_undone;
  h.x = (double)c.n_out_pel;
  h.y = (double)min(c.n_ho, d.hcap);
}
// The first pass's message has no bitmap: a tick that needs a second pass
// learns the other tiles' non-eating final cells from the second pass's
// bitmaps (it may take one pass longer; ticks rarely need a second at all).
// A later pass is gated (Dev::tile_gate): issued without asking the host whether
// it is needed, its kernels return at once when no owned cell is undone.
// The first pass's bookkeeping (counters, the hand-off plan) ran in k_players.
void launch_tile_pass(const Dev &d0, hipStream_t s, int rounds, int64_t *scr_k, int *scr_v, int first) {
  Dev d = d0;
  d.tile_gate = first ? 0 : 1;
  if (!first) hipLaunchKernelGGL(k_tile_pass_begin, dim3(1), dim3(1), 0, s, d);
  launch_food(d, s, rounds, Scratch{scr_k, scr_v}, first ? 0 : 1, 1);  // (serial rest in the last commit block)
  if (!first) (void)hipMemsetAsync(d.outbox + 1 + d.tcap, 0, 8 * (size_t)d.bm_words, s);
  hipLaunchKernelGGL(k_tile_collect, dim3(nblk(d.NP, 256)), dim3(256), 0, s, d, first ? 0 : 1);
}
// the other tiles' messages: their owned cells' outcomes (pellet and blob kills,
// new masses), their final cells, and the totals (thread 0)
// box_recs: records per inbox slot (the pass's message size); bitmaps only when
// the messages carry them (box_recs covers them)
// One block per source tile k (first: the messages carry the observation-
// history hand-off slots instead of bitmaps); the block of this tile's own
// message sums the headers.
__global__ void __launch_bounds__(256) k_tile_apply(Dev d, int box_recs, int first) {
  const int T = d.ntiles, k = blockIdx.x, tid = threadIdx.x;
  ArenaCtl &c = d.ctl[0];
  const TileRec *box = d.inbox + (size_t)k * box_recs;
  if (k == d.tile_id) {
    if (tid == 0) {
      int kills = 0, und = 0;
      for (int t = 0; t < T; t++) {
        const TileRec &h = d.inbox[(size_t)t * box_recs];
        kills += (int)h.x;
        und += (int)h.seq;
      }
      c.n_eaten_glob += kills;
      c.n_undone_glob = und;
      if (first) c.n_ho = c.n_ho_live = 0;  // (the header holds this tick's hand-offs; the next plan counts afresh)
    }
    return;
  }
  const int nrec = min(box[0].idx, d.tcap);
  for (int i = tid; i < nrec; i += blockDim.x) {
    const TileRec r = box[1 + i];
    if (r.kind == TR_PELLET) {
      const int bx = center_bucket_coord(r.x, d.cols), by = center_bucket_coord(r.y, d.cols);
      if (!tile_holds_bucket(d, bx, by)) continue;
      const Food F(d, 0);
      const int e = by * (d.cols + 1) + bx, lo = d.pstart[e], hi = d.pstart[e + 1];
      bool found = false;
      for (int t = lo; t < hi && !found; t++)
        if (d.pel[F.gp(t)].seq == r.seq) {
          uint8_t *pd = d.pel_dead + F.g(t);  // (flag set through its 32-bit word: the first setter notes the kill)
          unsigned *w = (unsigned *)((uintptr_t)pd & ~(uintptr_t)3);
          const unsigned sh = (unsigned)((uintptr_t)pd & 3) * 8;
          if (!((atomicOr(w, 1u << sh) >> sh) & 0xFFu)) note_kill(d, 0, t);
          found = true;
        }
      for (int j = F.n0; j < F.n0 + F.nst && !found; j++)  // this tick's blob conversions (staged)
        if (d.pn[F.gs(j)].seq == r.seq) {
          d.pel_dead[F.g(j)] = 1;
          found = true;
        }
      if (!found) set_err(d, 0, ERR_TILE_LOOKUP);
    } else if (r.kind == TR_BLOB) {
      if (d.b_seq[r.idx] != r.seq) {
        set_err(d, 0, ERR_TILE_LOOKUP);
        continue;
      }
      d.b_flags[r.idx] = 0;
      atomicOr(&c.dirty, DIRTY_BLOB);
    } else if (r.kind == TR_CELL) {
      if (d.c_seq[r.idx] != r.seq) {
        set_err(d, 0, ERR_TILE_LOOKUP);
        continue;
      }
      d.c_m[r.idx] = r.x;
      d.c_r[r.idx] = r.y;
      d.f_done[r.idx] = 1;
      atomic_max_pos(&c.rmax_cell, r.y);
    }
  }
  if (first) {  // hand-off slots: every tile takes the sender's history copy (tile_plan_thread)
    const int GG = d.G * d.G, per = d.nh * GG, slot_e = 1 + per, ns = min((int)box[0].y, d.hcap);
    for (int e = tid; e < ns * slot_e; e += blockDim.x) {
      const int sl = e / slot_e, j = e - sl * slot_e;
      const TileRec *slot = box + 1 + d.tcap + (size_t)sl * d.hrec;
      const int gp = slot->idx;
      if (slot->kind != TR_HIST || gp < 0 || gp >= d.NP) {
        set_err(d, 0, ERR_TILE_LOOKUP);
        continue;
      }
      if (j == 0) {
        d.o_lastfov[gp] = slot->x;
        d.t_holder[gp] = -1;  // every tile's copy is current again (as the sender's plan set)
      } else {
        const int q = j - 1, g = q / GG, t = q - g * GG;
        hist_grid(d, g)[(size_t)gp * GG + t] = ((const double *)(slot + 1))[q];
      }
    }
  } else {  // the sender's owned cells now final
    const unsigned long long *bmw = (const unsigned long long *)(box + 1 + d.tcap);
    for (int w = tid; w < d.bm_words; w += blockDim.x) {
      unsigned long long b = bmw[w];
      while (b) {
        const int t = __ffsll((long long)b) - 1;
        b &= b - 1;
        d.f_done[(size_t)w * 64 + t] = 1;
      }
    }
  }
}
// C4 with the reference's Greedy bots (bot.py:579-633, aigar_tile_policy): a
// Greedy move reads every pellet of the bot's view, which only the tile that
// observes the bot is sure to hold -- the observation's own rule, the history
// holder (the last observer until this tick's plan folds it in,
// tile_plan_thread), else the tile of the view centre (its view was checked against the
// held pellets when it was last observed; k_policy_greedy checks it again).  So
// each tile takes the moves of the bots it observes (k_policy_greedy under this
// mask) and the commands are all-gathered before the tick: one message of
// TR_CMD records (player, command point, split | eject << 1).  The policy's
// random draws are Philox-keyed by (player, tick): the same on every tile.
__global__ void k_tile_cmd_mask(Dev d, uint8_t *mask) {
  const int gp = GTID;
  if (gp >= d.NP) return;
  bool mine = false;
  if (d.p_alive[gp]) {  // (before this tick's hand-off plan: the last observer, if any, holds the history)
    const int ob = d.t_obsby[gp], hold = ob >= 0 ? ob : d.t_holder[gp];
    mine = (hold >= 0 ? hold : tile_of(d, d.p_fx[gp], d.p_fy[gp])) == d.tile_id;
  }
  mask[gp] = mine ? 1 : 0;
}
// cap: command records a message holds (the message buffer less its header)
__global__ void __launch_bounds__(256) k_tile_cmd_collect(Dev d, const uint8_t *mask, int cap) {
  const int gp = GTID;
  ArenaCtl &c = d.ctl[0];
  if (gp < d.NP && mask[gp]) {
    const int k = atomicAdd(&c.n_cmd, 1);
    if (k < cap) {
      TileRec r;
      r.kind = TR_CMD;
      r.idx = gp;
      r.seq = (int64_t)(d.p_split[gp] ? 1 : 0) | ((int64_t)(d.p_eject[gp] ? 1 : 0) << 1);
      r.x = d.p_cmdx[gp];
      r.y = d.p_cmdy[gp];
      d.outbox[1 + k] = r;
    } else {
      set_err(d, 0, ERR_TILE_CAP);
    }
  }
  if (last_block(d.ticket + 4, gridDim.x) && threadIdx.x == 0) {
    TileRec &h = d.outbox[0];
    h.kind = TR_HDR;
    h.idx = min(c.n_cmd, cap);
    h.seq = 0;
    h.x = h.y = 0.0;
    c.n_cmd = 0;
  }
}
// one block per source tile: the other tiles' commands (box_recs: records per inbox slot)
__global__ void __launch_bounds__(256) k_tile_cmd_apply(Dev d, int box_recs) {
  const int k = blockIdx.x;
  if (k == d.tile_id) return;
  const TileRec *box = d.inbox + (size_t)k * box_recs;
  const int n = min(box[0].idx, box_recs - 1);
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const TileRec r = box[1 + i];
    if (r.kind != TR_CMD || r.idx < 0 || r.idx >= d.NP) {
      set_err(d, 0, ERR_TILE_LOOKUP);
      continue;
    }
    d.p_cmdx[r.idx] = r.x;
    d.p_cmdy[r.idx] = r.y;
    d.p_split[r.idx] = (int)(r.seq & 1);
    d.p_eject[r.idx] = (int)((r.seq >> 1) & 1);
  }
}
void launch_policy_greedy(const Dev &d, hipStream_t s, int greedy_split, const uint8_t *mask, int want);
void launch_tile_policy(const Dev &d, hipStream_t s, int greedy_split, uint8_t *mask, int cap) {
  hipLaunchKernelGGL(k_tile_cmd_mask, dim3(nblk(d.NP, 256)), dim3(256), 0, s, d, mask);
  launch_policy_greedy(d, s, greedy_split, mask, 1);
  hipLaunchKernelGGL(k_tile_cmd_collect, dim3(nblk(d.NP, 256)), dim3(256), 0, s, d, (const uint8_t *)mask, cap);
}
void launch_tile_cmd_apply(const Dev &d, hipStream_t s, int box_recs) {
  hipLaunchKernelGGL(k_tile_cmd_apply, dim3(d.ntiles), dim3(256), 0, s, d, box_recs);
}
void launch_tile_apply(const Dev &d, hipStream_t s, int box_recs, int first) {
  hipLaunchKernelGGL(k_tile_apply, dim3(d.ntiles), dim3(256), 0, s, d, box_recs, first);
}

// Field.initialize()/reset() (field.py:57-83): players first (seq 0..B-1, empty
// player hash), then spawnStuff's pellets and viruses.
void launch_reset(const Dev &d, hipStream_t s, uint64_t seed) {
  (void)hipMemsetAsync(d.c_flags, 0, sizeof(uint32_t) * (size_t)kMaxCells * d.NP, s);
  (void)hipMemsetAsync(d.v_flags, 0, sizeof(uint32_t) * (size_t)d.A * d.Vcap, s);
  (void)hipMemsetAsync(d.b_flags, 0, sizeof(uint32_t) * (size_t)d.A * d.Ecap, s);
  (void)hipMemsetAsync(d.p_split, 0, sizeof(int) * d.NP, s);
  (void)hipMemsetAsync(d.p_eject, 0, sizeof(int) * d.NP, s);
  (void)hipMemsetAsync(d.pel_owner, 0, sizeof(uint64_t) * (size_t)d.A * d.PD, s);
  (void)hipMemsetAsync(d.pel_dead, 0, (size_t)d.A * d.PD, s);
  (void)hipMemsetAsync(d.b_owner, 0, sizeof(uint64_t) * (size_t)d.A * d.Ecap, s);
  (void)hipMemsetAsync(d.scan_state, 0, sizeof(unsigned long long) * 2 * (size_t)d.A * d.scan_tiles, s);
  (void)hipMemsetAsync(d.pl_state, 0, sizeof(unsigned long long) * (size_t)d.A * d.pl_tiles, s);
  hipLaunchKernelGGL(k_init_ctl, dim3(nblk(d.A, 64)), dim3(64), 0, s, d, seed);
  (void)hipMemsetAsync(d.occ, 0, sizeof(unsigned long long) * (size_t)d.A * d.occ_words, s);
  hipLaunchKernelGGL(k_spawn_plan, dim3(d.A), dim3(1024), 0, s, d, 1, (int64_t *)nullptr, (int *)nullptr, 0, 0);
  hipLaunchKernelGGL(k_spawn_players, dim3(nblk(d.NP, 256)), dim3(256), 0, s, d, 1);
  hipLaunchKernelGGL(k_spawn_pellets, dim3(nblk((long)d.A * d.Pcap, 256)), dim3(256), 0, s, d);
  if (d.virus_enabled) hipLaunchKernelGGL(k_spawn_viruses, dim3(nblk((long)d.A * d.Vcap, 256)), dim3(256), 0, s, d);
  hipLaunchKernelGGL(k_pnew_commit, dim3(nblk(d.A, 64)), dim3(64), 0, s, d);
  launch_pellet_rows(d, s);  // staging -> the row store
  launch_player_fov(d, s);
}

#ifdef AIGAR_PHASE_TIMING
// out: [9][kPtWaves][8] wave records, ids: [9][kPtWaves][2] (see PT_BEGIN); *khz: the wall clock's rate
extern "C" int aigar_debug_phase_times(unsigned int *out, unsigned int *ids, int *khz, int reset) {
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ptw), sizeof(g_ptw)) != hipSuccess) return -1;
  if (ids && hipMemcpyFromSymbol(ids, HIP_SYMBOL(g_ptid), sizeof(g_ptid)) != hipSuccess) return -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return -1;
  if (reset) {
    void *p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_ptw)) != hipSuccess || hipMemset(p, 0, sizeof(g_ptw)) != hipSuccess)
      return -1;
  }
  return 0;
}
#endif
}  // namespace aigar
