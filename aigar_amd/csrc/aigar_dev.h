// aigar_dev.h -- HBM layout of the stepper (all arenas of one handle).
//
// Structure-of-arrays, fp64 state (the reference computes in Python floats).
// Index conventions (A arenas, B players per arena, NP = A*B):
//   player  gp = a*B + p
//   cell    pool index ci = slot*NP + gp, slot in [0,16): the 16 pool slots
//           owned by a player; the player's cell *list* (order matters:
//           player.py:22,48-61) is p_list[k*NP + gp] = slot of the k-th cell.
//           Slot-major layout makes per-player loops coalesce across lanes.
//   pellet  a*PS + slot: bucket rows with two homes each (slot = home * cols * PR
//           + row * PR + k); a row's live records are contiguous in its current
//           home, sorted by centre bucket, so bucket (bx, by) is the range
//           [pstart[a*PH1 + by*(cols+1) + bx], the next entry) and a grid row's
//           buckets bx0..bx1 are ONE range (entry cols of a row = the row's end).
//           The closing update rewrites only the rows whose pellets changed, from
//           the first changed slot on, in place (a long suffix: the whole row into
//           its other home) (field.py:303-313, 327-344 change a few per tick).
//           Dead flags / reservation keys: a*PD + slot, staged records a*PD + PS + j.
//   blob    a*Ecap + i,   virus a*Vcap + i   (list order == creation order)
//   grids   a*(H+1) + bucket   (H = cols*cols, 20-unit buckets)
#pragma once
#include <stdint.h>

#include "../../include/aigar.h"

namespace aigar {

// Timing experiments only (tools/build_variant.sh + prof_ab.sh, results invalid): a kernel
// whose bit is set in AIGAR_FLOOR returns at entry.  With AIGAR_FLOOR_OPAQUE the
// test reads a kernel argument, so the compiler keeps the body (same registers,
// LDS and code size); without it the body is compiled out.  Product builds: nothing.
#ifdef AIGAR_FLOOR
#ifdef AIGAR_FLOOR_OPAQUE
#define FLOOR(k) \
  if ((((AIGAR_FLOOR) >> (k)) & 1) && d.A > 0) return
#else
#define FLOOR(k) \
  if (((AIGAR_FLOOR) >> (k)) & 1) return
#endif
#else
#define FLOOR(k)
#endif

struct ArenaCtl {
  int64_t seq_next;  // next Cell creation sequence number
  int64_t tick;      // completed Field.update() calls since reset
  int64_t tick_sp;   // the tick spawnStuff runs in (k_pel_update advances tick beside its respawns)
  uint64_t key0, key1, ctr_pellet, ctr_virus;
  int64_t seq_base_upd;  // seq_next before updatePlayers' creations (this tick)
  int64_t seq_base_spawn;
  uint64_t ctr_pellet_base, ctr_virus_base;
  int n_pel;          // pellets in the store (a tile: those it holds)
  int n_pnew;         // staged pellets (blob conversions, spawns)
  int n_pel_eaten;    // eaten in this tick's eat phase
  int n_blob;         // blob slots in use
  int n_blob_base;    // blob count before this tick's ejections
  int n_blob_add;     // this tick's ejections (n_blob moves in k_players' last block)
  int n_blob_live;    // live blobs at this tick's blob grid (blob_grid_place): the holes' share
  int n_vir;          // virus slots in use
  int n_vir_start;    // viruses that existed when virusBlobOverlap started
  int n_dead;         // deadPlayers list length
  int n_ev;           // events recorded this step
  int n_pend;         // worklist length (serial phases)
  int n_pend2;
  int n_spawn_p, n_spawn_v, n_spawn_pl;
  int vir_base_spawn;
  uint32_t err;   // sticky error bits (capacity overflow ...)
  uint32_t warn;  // sticky quirk bits (reference would raise)
  double rmax_cell, rmax_virus;
  double vmin_mass;  // lightest virus at the mid-tick virus grid build
  uint64_t ev_order;     // serial-phase event counter
  uint32_t food_round;   // reservation epoch (grows every eat phase)
  uint32_t scan_epoch[2];  // decoupled look-back epoch per scan slot (grows every launch)
  int scan_ticket[2];      // slot 0: pellet rebuilds, slot 1: cell grid (may run concurrently)
  int src_n_stage;  // reset: the staged records the row build places
  int n_kill;      // buffer pellets killed this tick (kill_list; sorted + unique after k_spawn_plan)
  int pu_nconv;   // the closing update: this tick's blob conversions (staged records 0 .. pu_nconv - 1)
  int pu_nsp, pu_spec;  // the closing update: this tick's pellet spawns, drawn ahead (spec_*) or staged (pn)
  uint32_t dirty;     // DIRTY_*: a virus / blob died this tick (k_spawn_plan compacts)
  int food_undone[3];  // cells that failed reservation round r (index r % 3)
  uint32_t pl_epoch;  // k_players look-back epoch / finished-tile ticket
  int pl_ticket;  // pellet rebuild: source counts snapshotted by the scan epilogue
  // C4 tiling (Dev::tiled): global pellet count at the tick's start, pellets every
  // tile ate this tick, this pass's outbox fill / pellet kills / undone owned
  // cells, and the undone owned cells of all tiles after the last exchange
  int n_pel_glob, n_eaten_glob, n_out, n_out_pel, n_undone, n_undone_glob;
  int n_ho;       // observation history hand-off slots in this tile's first-pass message (dead bots first)
  int n_ho_live;  // live bots whose view centre left this tile: hand-off candidates (t_holive)
  int n_cmd;      // Greedy commands in this tile's command message (aigar_tile_policy)
  // diagnostics, accumulated since reset (aigar_counters): serial work-list sizes of
  // virus<-blob, cell<-virus, pellet, blob, player<-player; then ticks seen
  int64_t stat[8];
};

enum : uint32_t {
  ERR_PELLET_CAP = 1, ERR_BLOB_CAP = 2, ERR_VIRUS_CAP = 4, ERR_EVENT_CAP = 8, ERR_WORK_CAP = 16,
  ERR_OBS_CAP = 32, ERR_CAND_CAP = 64, ERR_SLOT = 128, ERR_PIX_CAP = 256, ERR_TILE_CAP = 512, ERR_TILE_LOOKUP = 1024,
  ERR_TILE_OBS = 2048,    // a tile observed a bot whose view reaches beyond its held pellets
  ERR_TILE_PASSES = 4096,  // a device-bounded tiled tick ended with owned cells undone
  ERR_PREDICT = 8192,      // updatePlayers made other counts than k_players' arena block predicted (head_counts)
  ERR_TILE_HANDOFF = 16384,  // more dead bots to hand off in one tick than a message has hand-off slots
  ERR_CLAIM = 32768  // a bounded cell-claim loop (shared-cell kernels) ran out with claims left
};
enum : uint32_t { WARN_NEW_VIRUS_EATS = 1, WARN_DEAD_VIRUS = 2, WARN_TILE_OBS = 4 };
enum : uint32_t { DIRTY_VIRUS = 1, DIRTY_BLOB = 2 };

// event phases (sort key high word), in reference order within a tick
enum : uint32_t { PH_MERGE = 0, PH_VB = 1, PH_PV = 2, PH_PELLET = 3, PH_BLOB = 4, PH_PP = 5, PH_SPAWN = 6 };

// C4: one arena tiled 2-D over tile_x * tile_y handles (one per GPU).  Every
// handle holds a replica of the players, cells, blobs and viruses (a few
// thousand records: the player-ordered phases then need no exchange) and only
// the pellets whose centre bucket lies in its tile plus a halo.  The eat phase
// is resolved per tile; the outcomes of the cells a tile owns (centre bucket in
// the tile) travel in one all-gathered message per pass:
//   first pass of a tick: [TR_HDR][tcap records][hcap hand-off slots of hrec records]
//   later passes:         [TR_HDR][tcap records][final-cell bitmap, 16 * NP bits]
// Observation ownership: a bot is observed by ONE tile; its last-frame history
// grids (bot.py:480-495) live there.  t_holder[gp] names the tile whose copy is
// current (-1: every tile's copy is); a bot whose view centre left its holder's
// tile, or that died, has its history handed off in the next tick's first
// message (slot = [TR_HIST rec: idx = player, x = lastFovSize][nh grids]) and
// every tile applies it, so any tile can take the bot over.
struct TileRec {
  int32_t kind, idx;  // TR_*; idx: blob slot / cell pool index / player / (header) record count
  int64_t seq;        // pellet creation sequence / (header) undone owned cells
  double x, y;        // pellet position / cell mass, radius / lastFovSize / (header) pellet kills, hand-off slots
};
enum : int32_t { TR_HDR = 0, TR_PELLET = 1, TR_BLOB = 2, TR_CELL = 3, TR_HIST = 4, TR_CMD = 5 };
constexpr int kHcapMax = 256;  // hand-off slots per message (LDS list of the plan kernel)

// a pellet (field.py:303-313, 107-110): position, mass and creation sequence
struct alignas(32) PelRec {
  double x, y, m;
  int64_t seq;
};
constexpr int kPelStride = 4;  // PelRec in 8-byte words (per-lane strided loads of one field)
// the closing pellet update's record store (AIGAR_PEL_WT: write-through, timing variant)
__device__ __forceinline__ void pel_store(PelRec *p, const PelRec &r) {
#ifdef AIGAR_PEL_WT
  __hip_atomic_store(&p->x, r.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&p->y, r.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&p->m, r.m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&p->seq, r.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  *p = r;
#endif
}

struct Dev {
  int A, B, NP, size, cols, H;
  int tiled, tile_id, ntiles, tcap, bm_words;  // tcap: records per outbox; bm_words: u64 words of the bitmap
  int tile_flags;                              // AIGAR_TILE_*
  int tile_nx, tile_ny;                        // tile grid (tile_id = iy * tile_nx + ix)
  int tile_gate;  // a later eat pass issued without a host decision: its kernels do nothing once no owned cell is undone
  int hcap, hrec, nh;  // hand-off slots per message, records per slot, history grids per bot (0..4)
  int *t_holder;  // [NP] tile holding the bot's current observation history, -1: every tile
  int *t_obsby;   // [NP] tile that observed the bot since the last plan, -1: none
  int *t_holive;  // [NP] live bots waiting for a hand-off slot this tick (slots left after the dead ones)
  uint8_t *t_hodefer;  // [NP] ticks a live bot has waited for a hand-off slot (waiters go first)
  int *t_hoslot;  // [hcap] the player of each hand-off slot of this tick's first message
  int own_bx0, own_bx1, own_by0, own_by1;      // owned centre buckets [x0, x1) x [y0, y1)
  int loc_bx0, loc_bx1, loc_by0, loc_by1;      // held pellets: owned range + halo
  TileRec *outbox;       // [1 + tcap] records + bitmap
  const TileRec *inbox;  // [ntiles] outboxes (the transport fills it)
  int *ticket;  // finished-block counters of kernels whose last block runs an epilogue
  // closing pellet update (k_pel_update): the store slots killed this tick (their rows
  // are rewritten), and this tick's first pellet spawns, drawn ahead by k_players
  int *kill_list;     // [A][Pcap]
  double *spec_x, *spec_y, *spec_m;  // [A][64]
  double pow_n032[17];  // pow_glibc(n, 0.32) for n = 0..16 cells (getFovSize, player.py:163-167)
  int cshift;  // blob/virus grids: 2^cshift x 2^cshift fine buckets per cell (grid_span)
  int cshift_c;  // player-cell grid: smallest shift with <= 4096 cells (k_cgrid_count / k_cgrid_scatter)
  int Pcap, Ecap, Vcap, Wcap, EVcap;
  int PR;   // pellet slots per row home
  int PS;   // pellet store slots per arena: 2 homes x cols rows x PR
  int PD;   // dead-flag / reservation index space per arena: PS + Pcap (staged records j at PS + j)
  int PH1;  // pstart entries per arena: cols * (cols + 1) + 1
  int virus_enabled;
  double max_pellets, max_viruses;
  int G, L;
  uint32_t obs_ch, obs_ex;
  int flags;
  int pp_par;  // playerPlayerOverlap may run as independent groups (pp_pass; AIGAR_PP_SERIAL=1: never)
  int share_cells;  // launch choice: k_food_prep / k_pp_active share a block's cells (Greedy populations)
  ArenaCtl *ctl;
  // players [NP]
  int *p_alive, *p_respawn, *p_ncells, *p_split, *p_eject, *p_pend;
  double *p_cmdx, *p_cmdy;
  double *p_fx, *p_fy, *p_fs, *p_mass;  // FOV cache (getFovPos/getFovSize/getTotalMass at tick end)
  int *p_split_lh;       // Greedy bots' splitLikelihood (bot.py:93); <= 0: derived from the Philox key
  uint8_t *p_role;       // AIGAR_ROLE_*: NN / external actions, Greedy, Random bot (batched populations)
  int *p_time;           // Random bots' move counter (bot.py:243-249: a new action every FRAME_SKIP_RATE)
  double *o_last_mass;  // NN bots' lastMass (bot.py:229-230); NaN = None
  uint8_t *p_list;  // [16][NP]
  int *p_newc, *p_newb, *p_seqoff, *p_bloboff;
  int *p_heavy;  // per player: classes of its heavy cells this tick (update_cell -> k_players)
  // cells [16*NP]
  double *c_x, *c_y, *c_m, *c_r, *c_vx, *c_vy, *c_svx, *c_svy, *c_mt;
  int *c_svc;
  uint32_t *c_flags;
  int64_t *c_seq;
  uint8_t *c_active;
  // Cell.split geometry of a splitting player's cells [16*NP], computed by the
  // cell's own update_cell thread (the new cell's radius and momentum): the
  // split in k_players' per-player chain then loads it instead of evaluating
  // two atan2 / sincos pairs per cell
  double *sp_r, *sp_svx, *sp_svy;
  // per-player blob staging [16][NP]
  double *sb_x, *sb_y, *sb_svx, *sb_svy;
  uint8_t *sb_slot;
  // pellets: the row store + staging
  PelRec *pel;      // [A*PS] one 32-byte record per pellet: a bucket row's gather touches whole lines
  int *pel_col;     // [A*PS] colour owner: the player whose colour a blob-made pellet carries, -1: its own
  PelRec *pn;       // [A*Pcap] staging: this tick's blob conversions, then (closing update) spawns
  int *pn_col;
  uint8_t *pel_dead;  // [A*PD] eaten this tick (store slots, then staged records)
  int *pel_rank;      // [A*Pcap] reset: a staged record's rank in its bucket
  int *pstart;        // [A*PH1] bucket starts in the store, rows of cols + 1 entries
  int *pncnt;         // [A*PH1] reset: staged records per bucket
  uint64_t *pel_owner;  // reservation keys [A*PD]
  // blobs [A*Ecap]
  double *b_x, *b_y, *b_m, *b_r, *b_vx, *b_vy, *b_svx, *b_svy;
  int *b_svc;
  int64_t *b_seq, *b_ej;
  int *b_col;  // the ejecting player (field.py:141 blob.setColor(player.getColor()))
  uint32_t *b_flags;
  uint64_t *b_owner;
  int *bstart, *bitems, *b_rank;
  uint64_t *bmap;  // [A][64] the blob grid's non-empty coarse buckets (one bit each; blob_grid_place)
  // viruses [A*Vcap]
  double *v_x, *v_y, *v_m, *v_r, *v_vx, *v_vy, *v_svx, *v_svy;
  int *v_svc;
  int64_t *v_seq;
  uint32_t *v_flags;
  int *v_active;  // virusBlobOverlap's work-list marks (vb_active_blob; cleared by the serial pass)
  int *vcnt, *vstart, *vitems, *v_rank;
  // cell grid
  int *ccnt, *cstart, *citems, *c_rank;
  int *cgcnt;  // [A][2][4100] coarse grid counts (<= 4096 cells): the player cells', the blobs'
  // occupancy bitmap of the player hash [A][ceil(H/64)]
  unsigned long long *occ;  // getSpawnPos occupancy: one bit per fine bucket a live player cell touches
  int *occ_cnt;             // ... and the number of such cells per bucket (k_pp_active, kept by the pp pass)
  int occ_words;
  // dead list [NP], worklists [A*Wcap]
  int *dead;
  int *work, *work2;
  // food-phase per-cell candidate lists [16*NP][FCAP]
  int *f_list;
  uint8_t *f_cnt;
  uint8_t *f_done;
  // spawn staging
  int *resp_slot;  // [NP] a dead player's place in this tick's respawn order, -1 = waits
  // events [A*EVcap][5]: key_hi, key_lo, code, a, b
  int64_t *ev;
  // observation state
  double *o_lastfov;                             // [NP]
  double *o_self_lf, *o_self_slf, *o_en_lf, *o_en_slf;  // [NP][G*G]
  double *o_act_cur, *o_act_prev;                // [NP][4]
  // decoupled look-back tile states [A][scan_tiles]
  unsigned long long *scan_state;  // [2 slots][A][scan_tiles]
  unsigned long long *pl_state;    // [A][pl_tiles] (k_players)
  int pl_tiles;
  int scan_tiles;
  // observation overflow pool (bots that see more objects than their LDS lists hold)
  int OBcap;
  unsigned long long *ob_used;  // {observe call epoch:32 | overflow slots taken:32}
  uint32_t *ob_epoch;  // device-side epoch for graph-replayed observes (bumped by k_player_fov)
  int64_t *ob_seq;
  double *ob_m, *ob_r;
  uint32_t *ob_mask;
  uint8_t *ob_own;
  int *ob_perm;
  uint64_t *ob_wmask;  // [OBcap][4] x / y index masks of the wide grid (grid_squares > 16)
};

constexpr int FCAP = 32;  // stored candidate foods per cell (overflow -> serial)

// the synthetic population's policy when it is evaluated inside the tick
// (aigar_run, AIGAR_POLICY_RANDOM): probabilities and Philox salt
struct RandomPolicy {
  int on;
  double ps, pe;
  uint64_t salt;
};

}  // namespace aigar
