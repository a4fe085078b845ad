// api.hip -- host implementation of include/aigar.h (libaigar_hip.so).
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/aigar.h"
#include "aigar_dev.h"
#include "aigar_sem.h"

namespace aigar {
void launch_tick(const Dev &d, hipStream_t s, int rounds, int64_t *scr_k, int *scr_v,
                 const RandomPolicy *rp = nullptr);
void launch_tick_pre(const Dev &d, hipStream_t s, int64_t *scr_k, int *scr_v, const RandomPolicy *rp);
void launch_tick_post(const Dev &d, hipStream_t s, int64_t *scr_k, int *scr_v);
void launch_tile_pass(const Dev &d, hipStream_t s, int rounds, int64_t *scr_k, int *scr_v, int first);
void launch_tile_policy(const Dev &d, hipStream_t s, int greedy_split, uint8_t *mask, int cap);
void launch_tile_cmd_apply(const Dev &d, hipStream_t s, int box_recs);
void launch_pel_gather(const Dev &d, hipStream_t s, int a);
void launch_tile_apply(const Dev &d, hipStream_t s, int box_recs, int first);
void launch_reset(const Dev &d, hipStream_t s, uint64_t seed);
void launch_observe(const Dev &d, hipStream_t s, void *out, int dtype, uint32_t epoch,
                    const uint8_t *mask = nullptr, int greedy_next = -1);
bool observe_fuses_greedy(const Dev &d);
void launch_policy_refrandom(const Dev &d, hipStream_t s, int skip_rate, int enable_split, int enable_eject,
                             uint64_t salt);
int launch_observe_pixels(const Dev &d, hipStream_t s, void *out, int dtype, int side, uint64_t seed, uint8_t *ovf);
void launch_policy(const Dev &d, hipStream_t s, double ps, double pe, uint64_t salt);
void launch_player_stats(const Dev &d, hipStream_t s, double *out);
void launch_player_fov(const Dev &d, hipStream_t s);
void launch_apply_actions(const Dev &d, hipStream_t s, const double *act, int n_act, int enable_split, int skipping,
                          int record);
void launch_rewards(const Dev &d, hipStream_t s, double *out, const aigar_reward_params &p, int update_last,
                    int mode);
void launch_policy_greedy(const Dev &d, hipStream_t s, int greedy_split, const uint8_t *mask, int want = -1);
void launch_set_commands(const Dev &d, hipStream_t s, const double *cmd);
}  // namespace aigar

using namespace aigar;

static thread_local std::string g_err;
static int fail(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return -1;
}
#define HIPCHK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) return fail("%s failed: %s", #x, hipGetErrorString(e_));       \
  } while (0)

// librccl.so, bound at run time (C4 over RCCL, below)
namespace {
struct RcclId {
  char b[128];  // ncclUniqueId (rccl.h: NCCL_UNIQUE_ID_BYTES)
};
constexpr int kNcclUint8 = 1;  // ncclDataType_t ncclUint8 (rccl.h)
struct Rccl {
  void *so = nullptr;
  int (*get_unique_id)(RcclId *) = nullptr;
  int (*comm_init_rank)(void **, int, RcclId, int) = nullptr;
  int (*all_gather)(const void *, void *, size_t, int, void *, hipStream_t) = nullptr;
  int (*comm_destroy)(void *) = nullptr;
  const char *(*error_string)(int) = nullptr;
};
Rccl g_rccl;
int rccl_load(const char *path) {
  if (g_rccl.so) return 0;
  void *so = dlopen(path && *path ? path : "librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (!so) return fail("RCCL: dlopen(%s) failed: %s", path ? path : "librccl.so", dlerror());
  Rccl r;
  r.so = so;
  r.get_unique_id = (int (*)(RcclId *))dlsym(so, "ncclGetUniqueId");
  r.comm_init_rank = (int (*)(void **, int, RcclId, int))dlsym(so, "ncclCommInitRank");
  r.all_gather = (int (*)(const void *, void *, size_t, int, void *, hipStream_t))dlsym(so, "ncclAllGather");
  r.comm_destroy = (int (*)(void *))dlsym(so, "ncclCommDestroy");
  r.error_string = (const char *(*)(int))dlsym(so, "ncclGetErrorString");
  if (!r.get_unique_id || !r.comm_init_rank || !r.all_gather || !r.comm_destroy || !r.error_string)
    return fail("RCCL: %s lacks an nccl* entry point", path ? path : "librccl.so");
  g_rccl = r;
  return 0;
}
}  // namespace

struct aigar_handle {
  aigar_config cfg;
  Dev d;
  hipStream_t stream = nullptr;
  bool own_stream = true;
  uint32_t obs_calls = 0;
  // reservation rounds of the eat phase before the serial fallback (food_rounds):
  // 0 = by population -- 1 until the handle's Greedy policy ran, then 2 (Greedy
  // bots crowd the same pellets: 18 cells per C3 tick failed a single round and
  // took the serial pass, 0.9 with two rounds, profiles/r05_v2g_*); an empty
  // round exits at once but costs a dependent launch
  int rounds = 0;
  bool greedy_seen = false;
  int graph_rounds = 0;  // the rounds the step graph was captured with
  int64_t *scr_k = nullptr;
  int *scr_v = nullptr;
  double *d_cmd = nullptr, *d_stats = nullptr;
  uint8_t *d_mask = nullptr;
  uint8_t *d_nnmask = nullptr;  // 1 for the players of role NN (the env step's observations)
  int n_greedy = 0, n_random = 0;  // role counts (aigar_set_roles)
  aigar_env_params envp{};
  void *d_obs = nullptr;
  void *d_pix = nullptr;  // host-destination staging for aigar_observe_pixels
  uint8_t *d_pix_ovf = nullptr;  // per player: frame left to the pixel kernel's second pass
  size_t pix_bytes = 0;
  std::vector<void *> allocs;
  char *arena = nullptr;  // aigar_create's arrays (dalloc); freed through allocs
  size_t arena_size = 0, arena_used = 0;
  bool arena_sizing = false;
  int box_recs = 0;   // C4: TileRec slots of a full exchange message (header + records + bitmap)
  int pass_recs = 0;  // ... of the current pass's message (the first pass sends no bitmap)
  int first_pass = 0;  // the current pass is the tick's first (its message carries the history hand-off)
  hipEvent_t ev_x = nullptr;  // in-process transport: this handle's outbox is written / its inbox is filled
  // C4: the tick up to the first exchange and the tick after the last one, as
  // graphs (re-captured when the policy, the observation buffer or the message
  // buffers change)
  hipGraphExec_t tb_graph = nullptr, te_graph = nullptr;
  aigar_run_params tb_key{};
  const void *tb_box[2] = {nullptr, nullptr}, *te_box[2] = {nullptr, nullptr};
  void *te_out = nullptr;
  int te_dtype = -2;
  bool profile = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // timer name -> recorded (start, stop) event pairs, resolved lazily
  std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> marks;
  std::vector<hipEvent_t> event_pool;
  hipGraphExec_t graph = nullptr;
  hipStream_t cap_stream = nullptr;  // private stream graphs are captured on (the caller's may be the null stream)
  bool use_graph = true;  // AIGAR_NO_GRAPH=1 disables (direct launches)
  // C4 tile phases as graphs (AIGAR_TILE_GRAPH=1): measured no faster than direct
  // launches on a tile's own GPU (tools/c4_tile_timing.py), and slower in the
  // 1-GPU gloo rehearsal, so off by default
  bool tile_graph = false;
  bool graph_failed = false;
  // C4 over RCCL (aigar_tile_comm_init / aigar_tile_run)
  void *rccl_comm = nullptr;
  int rccl_ranks = 0;
  bool rccl_bad = false;  // an all-gather failed while a graph was captured
  bool loopback = false;  // timing rehearsal: the exchange copies this tile's message to its own slot only
  bool cmd_ready = false;  // this tick's Greedy commands were exchanged and applied (aigar_tile_apply_commands)
  bool cmd_pending = false;  // aigar_tile_policy wrote a command message that was not applied yet
  hipGraphExec_t tr_graph = nullptr;
  aigar_run_params tr_key{};
  void *tr_out = nullptr;
  int tr_dtype = -2, tr_extra = -1;
  bool tr_failed = false;
  // aigar_run: one whole env step (policy + Field.update + observation) as a graph
  hipGraphExec_t run_graph = nullptr;
  hipGraphExec_t run_graph_u = nullptr;  // run_unroll steps in one graph (same key)
  // AIGAR_RUN_UNROLL (default 4): each graph launch costs an inter-graph gap on
  // the device that a node boundary inside a graph does not (C3 A/B,
  // profiles/r05_ab_notes.txt v30: 1 -> 4 steps per graph 42.5 -> 44.4 M env-steps/s)
  int run_unroll = 4;
  bool run_u_tried = false;  // the unrolled graph of this key was captured (or its capture failed)
  aigar_run_params run_key{};
  void *run_out = nullptr;
  int run_dtype = -1;
  // aigar_env_step: one learner decision (skip + 1 ticks) as a graph
  hipGraphExec_t env_graph = nullptr;
  struct EnvKey {
    const double *act;
    int n_act, enable_split, skip, dtype;
    aigar_reward_params prm;
    double *reward;
    void *obs;
    aigar_env_params envp;
    int n_greedy, n_random;
  } env_key{};
};

extern "C" const char *aigar_last_error(void) { return g_err.c_str(); }
extern "C" int aigar_abi_version(void) { return AIGAR_ABI_VERSION; }

// Device arrays.  aigar_create carves the world's ~120 arrays out of ONE
// allocation (arena_*: a sizing pass, one hipMalloc, a carving pass) instead of a
// hipMalloc each: one large allocation is mapped with large pages, so the tick's
// kernels, which touch tens of arrays per load round, need far fewer address
// translations.  Every array starts on a 256-byte boundary.  Later allocations
// (pixel buffers) are separate.
template <class T>
static T *dalloc(aigar_handle *h, size_t n) {
  void *p = nullptr;
  if (n == 0) n = 1;
  const size_t bytes = (n * sizeof(T) + 255) & ~(size_t)255;
  if (h->arena_sizing) {  // sizing pass: a placeholder (never dereferenced)
    const size_t off = h->arena_used;
    h->arena_used += bytes;
    return (T *)(uintptr_t)(256 + off);
  }
  if (h->arena) {
    if (h->arena_used + bytes > h->arena_size) return nullptr;
    p = h->arena + h->arena_used;
    h->arena_used += bytes;
    return (T *)p;  // (zeroed with the whole arena)
  }
  if (hipMalloc(&p, n * sizeof(T)) != hipSuccess) return nullptr;
  (void)hipMemset(p, 0, n * sizeof(T));
  h->allocs.push_back(p);
  return (T *)p;
}

static int obs_len_of(const aigar_config &c) {
  int G = c.grid_squares ? c.grid_squares : 11, n = 0, e = 0;
  if (c.obs_channels & AIGAR_OBS_SIMPLE) return 12;  // getSimpleStateRepresentation (bot.py:511-547)
  for (int b = 0; b < 10; b++) n += (c.obs_channels >> b) & 1;
  e += (c.obs_extras & AIGAR_EX_LAST_FOV) ? 1 : 0;
  e += (c.obs_extras & AIGAR_EX_FOV) ? 1 : 0;
  e += (c.obs_extras & AIGAR_EX_MASS) ? 1 : 0;
  e += (c.obs_extras & AIGAR_EX_LAST_ACT) ? 4 : 0;
  e += (c.obs_extras & AIGAR_EX_2LAST_ACT) ? 4 : 0;
  return G * G * n + e;
}

static void free_all(aigar_handle *h) {
  if (h->graph) (void)hipGraphExecDestroy(h->graph);
  if (h->run_graph) (void)hipGraphExecDestroy(h->run_graph);
  if (h->run_graph_u) (void)hipGraphExecDestroy(h->run_graph_u);
  if (h->env_graph) (void)hipGraphExecDestroy(h->env_graph);
  for (void *p : h->allocs) (void)hipFree(p);
  h->allocs.clear();
  if (h->d_pix) (void)hipFree(h->d_pix);
  h->d_pix = nullptr;
  h->d_pix_ovf = nullptr;  // (one of allocs)
  h->pix_bytes = 0;
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  if (h->ev_x) (void)hipEventDestroy(h->ev_x);
  if (h->tb_graph) (void)hipGraphExecDestroy(h->tb_graph);
  if (h->te_graph) (void)hipGraphExecDestroy(h->te_graph);
  if (h->tr_graph) (void)hipGraphExecDestroy(h->tr_graph);
  if (h->rccl_comm && g_rccl.comm_destroy) (void)g_rccl.comm_destroy(h->rccl_comm);
  h->rccl_comm = nullptr;
  for (auto &m : h->marks) {
    (void)hipEventDestroy(m.second.first);
    (void)hipEventDestroy(m.second.second);
  }
  for (hipEvent_t e : h->event_pool) (void)hipEventDestroy(e);
  if (h->stream && h->own_stream) (void)hipStreamDestroy(h->stream);
  if (h->cap_stream) (void)hipStreamDestroy(h->cap_stream);
}

static hipEvent_t pool_event(aigar_handle *h) {
  hipEvent_t e = nullptr;
  if (!h->event_pool.empty()) {
    e = h->event_pool.back();
    h->event_pool.pop_back();
  } else {
    (void)hipEventCreate(&e);
  }
  return e;
}
struct Mark {  // records a (start, stop) event pair around a launch group when profiling
  aigar_handle *h;
  const char *name;
  hipEvent_t a = nullptr;
  Mark(aigar_handle *hh, const char *n) : h(hh), name(n) {
    if (h->profile) {
      a = pool_event(h);
      (void)hipEventRecord(a, h->stream);
    }
  }
  ~Mark() {
    if (!a) return;
    hipEvent_t b = pool_event(h);
    (void)hipEventRecord(b, h->stream);
    h->marks.push_back({name, {a, b}});
  }
};

extern "C" int aigar_create(const aigar_config *cfg, aigar_handle **out) {
  if (!cfg || !out) return fail("aigar_create: null argument");
  if (cfg->n_arenas < 1 || cfg->bots_per_arena < 1) return fail("aigar_create: need n_arenas >= 1 and bots >= 1");
  if (cfg->rng_mode != AIGAR_RNG_PHILOX)
    return fail("aigar_create: the device stepper runs AIGAR_RNG_PHILOX only (MT19937 lives in the CPU oracle)");
  int G = cfg->grid_squares ? cfg->grid_squares : 11;
  if (G < 1 || G > 127) return fail("aigar_create: grid_squares must be in [1, 127]");
  if (cfg->obs_channels & AIGAR_OBS_ALL &&
      cfg->obs_channels & (AIGAR_OBS_SELF_LF | AIGAR_OBS_SELF_SLF | AIGAR_OBS_ENEMY_LF | AIGAR_OBS_ENEMY_SLF))
    return fail("aigar_create: ALL_PLAYER_GRID with last-frame grids is undefined in the reference");
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (cfg->device < 0 || cfg->device >= ndev) return fail("aigar_create: device %d not present (%d devices)", cfg->device, ndev);
  HIPCHK(hipSetDevice(cfg->device));
  aigar_handle *h = new aigar_handle();
  h->cfg = *cfg;
  if (getenv("AIGAR_NO_GRAPH")) h->use_graph = false;
  if (const char *u = getenv("AIGAR_RUN_UNROLL")) h->run_unroll = std::max(1, std::min(64, atoi(u)));
  if (getenv("AIGAR_TILE_GRAPH")) h->tile_graph = true;
  h->d.pp_par = getenv("AIGAR_PP_SERIAL") ? 0 : 1;
  h->d.share_cells = 0;  // (aigar_run sets it in the graph it captures for the Greedy population)
  // tuning knob: a fixed number of reservation rounds for every population
  if (const char *r = getenv("AIGAR_FOOD_ROUNDS")) h->rounds = std::max(1, std::min(16, atoi(r)));
  Dev &d = h->d;
  d.A = cfg->n_arenas;
  d.B = cfg->bots_per_arena;
  d.NP = d.A * d.B;
  d.size = cfg->field_size > 0 ? cfg->field_size : (int)(75 * std::sqrt((double)d.B));
  d.cols = (int)std::ceil(d.size / 20.0);
  d.H = d.cols * d.cols;
  d.virus_enabled = cfg->virus_enabled ? 1 : 0;
  d.max_pellets = cfg->max_pellets >= 0 ? cfg->max_pellets : (double)d.size * d.size * 0.015;
  d.max_viruses = cfg->max_viruses >= 0 ? cfg->max_viruses : (double)d.size * d.size * 0.00005;
  if (!d.virus_enabled) d.max_viruses = 0;
  auto r64 = [](int v) { return (v + 63) / 64 * 64; };  // a wavefront never straddles two arenas
  d.Ecap = r64(cfg->blob_cap > 0 ? cfg->blob_cap : 4 * d.B + 256);
  d.Pcap = r64(cfg->pellet_cap > 0 ? cfg->pellet_cap : (int)std::ceil(d.max_pellets) + d.Ecap + 64);
  d.Vcap = r64(cfg->virus_cap > 0 ? cfg->virus_cap : 2 * (int)std::ceil(d.max_viruses) + 64);
  // the pellet row store (aigar_dev.h): per bucket row a home of PR slots, twice;
  // PR leaves a quarter of headroom over the row's share of Pcap (uniform spawns
  // put ~Pcap / cols pellets in a row) plus 64
  if (d.cols > 1024) {
    delete h;
    return fail("aigar_create: field size %d: more than 1024 bucket rows", d.size);
  }
  d.PR = r64((int)std::ceil(1.25 * d.Pcap / d.cols) + 64);
  d.PS = 2 * d.cols * d.PR;
  d.PD = d.PS + d.Pcap;
  d.PH1 = d.cols * (d.cols + 1) + 1;
  d.Wcap = std::max(kMaxCells * d.B, std::max(d.Ecap, 4096));
  d.EVcap = cfg->event_cap > 0 ? cfg->event_cap : 65536;
  d.G = G;
  d.L = obs_len_of(*cfg);
  d.obs_ch = cfg->obs_channels;
  d.obs_ex = cfg->obs_extras;
  d.flags = cfg->flags;
  d.occ_words = (d.H + 63) / 64;
  d.scan_tiles = (d.H + 2047) / 2048;
  d.pl_tiles = (d.B + 255) / 256;
  // C4 tiles: bucket-aligned tiles, ownership by centre bucket
  const int tx = std::max(1, cfg->tile_x), ty = std::max(1, cfg->tile_y);
  d.ntiles = tx * ty;
  d.tiled = d.ntiles > 1 || (cfg->tile_flags & AIGAR_TILE_FORCE);
  d.own_bx0 = d.own_by0 = d.loc_bx0 = d.loc_by0 = 0;
  d.own_bx1 = d.own_by1 = d.loc_bx1 = d.loc_by1 = d.cols;
  if (d.tiled) {
    auto bad = [&](const char *m) {
      delete h;
      return fail("aigar_create: %s", m);
    };
    if (d.A != 1) return bad("a tiled handle steps one arena (n_arenas must be 1)");
    if (cfg->tile_id < 0 || cfg->tile_id >= d.ntiles) return bad("tile_id out of range");
    if (tx > d.cols || ty > d.cols) return bad("more tiles than hash buckets along a side");
    const int ix = cfg->tile_id % tx, iy = cfg->tile_id / tx;
    const int halo = cfg->tile_halo > 0 ? cfg->tile_halo : 400;
    // an owned cell's boxes (pellet turn, blob turn, one bucket of food footprint)
    // reach <= 6 buckets from its centre bucket at the mass cap: with 7 its owner
    // holds every food it can touch, so every cell is decidable somewhere
    const int hb = std::max(7, (halo + kBucket - 1) / kBucket);
    if (d.ntiles > 64) return bad("at most 64 tiles");
    d.tile_id = cfg->tile_id;
    d.tile_flags = cfg->tile_flags;
    d.own_bx0 = ix * d.cols / tx;
    d.own_bx1 = (ix + 1) * d.cols / tx;
    d.own_by0 = iy * d.cols / ty;
    d.own_by1 = (iy + 1) * d.cols / ty;
    d.loc_bx0 = std::max(0, d.own_bx0 - hb);
    d.loc_bx1 = std::min(d.cols, d.own_bx1 + hb);
    d.loc_by0 = std::max(0, d.own_by0 - hb);
    d.loc_by1 = std::min(d.cols, d.own_by1 + hb);
  }
  d.tile_nx = tx;
  d.tile_ny = ty;
  d.tile_gate = 0;
  d.tcap = cfg->tile_cap > 0 ? cfg->tile_cap : 2048;
  d.bm_words = (int)(((size_t)kMaxCells * d.NP + 255) / 256 * 4);  // 16 * NP bits, whole TileRecs
  // observation-history hand-off: the grids the observation keeps per bot
  // (self / enemy, last / second-last frame), 4 doubles per 32-byte record
  {
    const uint32_t ch = cfg->obs_channels;
    d.nh = ((ch & (AIGAR_OBS_SELF_LF | AIGAR_OBS_SELF_SLF)) ? 1 : 0) + ((ch & AIGAR_OBS_SELF_SLF) ? 1 : 0) +
           ((ch & (AIGAR_OBS_ENEMY_LF | AIGAR_OBS_ENEMY_SLF)) ? 1 : 0) + ((ch & AIGAR_OBS_ENEMY_SLF) ? 1 : 0);
    d.hrec = 1 + (d.nh * G * G + 3) / 4;
    d.hcap = std::min(kHcapMax, std::max(16, d.tcap / 64));
  }
  h->box_recs = 1 + d.tcap + std::max(d.bm_words / 4, d.hcap * d.hrec);
  for (int k = 0; k <= kMaxCells; k++) d.pow_n032[k] = aigar_math::pow_glibc((double)k, 0.32);
  d.cshift = 3;  // coarse blob/virus grids: 160 x 160 field units per cell, <= 4096 cells (grid_small_build)
  while ((((d.cols + (1 << d.cshift) - 1) >> d.cshift) * ((d.cols + (1 << d.cshift) - 1) >> d.cshift)) > 4096)
    d.cshift++;
  d.cshift_c = 0;  // player-cell grid: as fine as one block's LDS histogram allows
  while ((((d.cols + (1 << d.cshift_c) - 1) >> d.cshift_c) * ((d.cols + (1 << d.cshift_c) - 1) >> d.cshift_c)) > 4096)
    d.cshift_c++;
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return fail("hipStreamCreate failed");
  }
  const size_t A = d.A, NP = d.NP, C = (size_t)kMaxCells * NP, H1 = (size_t)d.H + 1, GG = (size_t)G * G;
  bool ok = true;
#define AL(field, T, n)                     \
  do {                                      \
    d.field = dalloc<T>(h, (n));            \
    ok = ok && d.field != nullptr;          \
  } while (0)
#ifndef AIGAR_NO_ARENA
  for (int pass = 0; pass < 2; pass++) {  // 0: size the arena, 1: carve it
    h->arena_sizing = pass == 0;
    if (pass == 1) {
      h->arena_size = h->arena_used;
      h->arena_used = 0;
      void *base = nullptr;
      if (hipMalloc(&base, h->arena_size) != hipSuccess) {
        ok = false;
        break;
      }
      h->allocs.push_back(base);
      (void)hipMemset(base, 0, h->arena_size);
      h->arena = (char *)base;
    }
#endif
  AL(ctl, ArenaCtl, A);
  AL(p_alive, int, NP); AL(p_respawn, int, NP); AL(p_ncells, int, NP); AL(p_split, int, NP); AL(p_eject, int, NP);
  AL(p_pend, int, NP); AL(p_cmdx, double, NP); AL(p_cmdy, double, NP); AL(p_list, uint8_t, C);
  AL(p_newc, int, NP); AL(p_heavy, int, NP); AL(p_newb, int, NP); AL(p_seqoff, int, NP); AL(p_bloboff, int, NP);
  AL(c_x, double, C); AL(c_y, double, C); AL(c_m, double, C); AL(c_r, double, C); AL(c_vx, double, C);
  AL(c_vy, double, C); AL(c_svx, double, C); AL(c_svy, double, C); AL(c_mt, double, C); AL(c_svc, int, C);
  AL(c_flags, uint32_t, C); AL(c_seq, int64_t, C); AL(c_active, uint8_t, C);
  AL(sp_r, double, C); AL(sp_svx, double, C); AL(sp_svy, double, C);
  AL(sb_x, double, C); AL(sb_y, double, C); AL(sb_svx, double, C); AL(sb_svy, double, C); AL(sb_slot, uint8_t, C);
  const size_t P = A * d.Pcap, PSA = A * d.PS, PDA = A * d.PD, PHA = A * d.PH1;
  AL(pel, PelRec, PSA); AL(pel_col, int, PSA);
  AL(pn, PelRec, P); AL(pn_col, int, P);
  AL(pel_dead, uint8_t, PDA); AL(pel_rank, int, P); AL(pncnt, int, PHA); AL(pstart, int, PHA);
  AL(pel_owner, uint64_t, PDA);
  const size_t E = A * d.Ecap, V = A * d.Vcap;
  AL(b_x, double, E); AL(b_y, double, E); AL(b_m, double, E); AL(b_r, double, E); AL(b_vx, double, E);
  AL(b_vy, double, E); AL(b_svx, double, E); AL(b_svy, double, E); AL(b_svc, int, E); AL(b_seq, int64_t, E);
  AL(b_ej, int64_t, E); AL(b_flags, uint32_t, E); AL(b_owner, uint64_t, E); AL(b_col, int, E);
  AL(bstart, int, A * H1); AL(bitems, int, E); AL(b_rank, int, E); AL(bmap, uint64_t, A * 64);
  AL(v_x, double, V); AL(v_y, double, V); AL(v_m, double, V); AL(v_r, double, V); AL(v_vx, double, V);
  AL(v_vy, double, V); AL(v_svx, double, V); AL(v_svy, double, V); AL(v_svc, int, V); AL(v_seq, int64_t, V);
  AL(v_flags, uint32_t, V); AL(v_active, int, V);
  AL(vcnt, int, A * H1); AL(vstart, int, A * H1); AL(vitems, int, V); AL(v_rank, int, V);
  AL(ccnt, int, A * H1); AL(cstart, int, A * H1); AL(citems, int, C); AL(c_rank, int, C);
  AL(cgcnt, int, A * 2 * 4100);
  AL(occ, unsigned long long, A * d.occ_words); AL(occ_cnt, int, A * d.H);
  AL(dead, int, NP); AL(work, int, A * d.Wcap); AL(work2, int, A * d.Wcap);
  AL(f_list, int, C * FCAP); AL(f_cnt, uint8_t, C); AL(f_done, uint8_t, C);
  AL(resp_slot, int, NP);
  AL(ev, int64_t, A * d.EVcap * 5);
  AL(o_lastfov, double, NP); AL(o_self_lf, double, NP * GG); AL(o_self_slf, double, NP * GG);
  AL(o_en_lf, double, NP * GG); AL(o_en_slf, double, NP * GG); AL(o_act_cur, double, NP * 4);
  AL(o_act_prev, double, NP * 4);
  d.OBcap = (int)std::min<size_t>(std::max<size_t>(1u << 20, 64 * NP), (size_t)1 << 24);
  AL(scan_state, unsigned long long, 2 * A * d.scan_tiles);
  AL(pl_state, unsigned long long, A * d.pl_tiles);
  AL(ticket, int, 16);
  AL(kill_list, int, P); AL(spec_x, double, A * 64); AL(spec_y, double, A * 64); AL(spec_m, double, A * 64); 
  AL(ob_used, unsigned long long, 1);
  AL(ob_epoch, uint32_t, 1);
  AL(p_split_lh, int, NP);
  AL(p_role, uint8_t, NP);
  AL(p_time, int, NP);
  AL(o_last_mass, double, NP);
  if (d.tiled) {
    AL(t_holder, int, NP);
    AL(t_obsby, int, NP);
    AL(t_holive, int, NP);
    AL(t_hodefer, uint8_t, NP);
    AL(t_hoslot, int, d.hcap);
    AL(outbox, TileRec, h->box_recs);
    TileRec *ib = nullptr;
    ib = dalloc<TileRec>(h, (size_t)h->box_recs * d.ntiles);
    ok = ok && ib != nullptr;
    d.inbox = ib;
  }
  AL(p_fx, double, NP); AL(p_fy, double, NP); AL(p_fs, double, NP); AL(p_mass, double, NP); AL(ob_seq, int64_t, d.OBcap); AL(ob_m, double, d.OBcap); AL(ob_r, double, d.OBcap);
  AL(ob_mask, uint32_t, d.OBcap); AL(ob_own, uint8_t, d.OBcap); AL(ob_perm, int, d.OBcap);
  d.ob_wmask = nullptr;
  if (G > 16) AL(ob_wmask, uint64_t, 4 * (size_t)d.OBcap);
#undef AL
  h->scr_k = dalloc<int64_t>(h, A * d.Wcap);
  h->scr_v = dalloc<int>(h, A * d.Wcap);
  h->d_cmd = dalloc<double>(h, NP * 4);
  h->d_mask = dalloc<uint8_t>(h, NP);
  h->d_nnmask = dalloc<uint8_t>(h, NP);
  h->d_stats = dalloc<double>(h, NP * 5);
  h->d_obs = dalloc<double>(h, NP * (size_t)d.L);
  ok = ok && h->scr_k && h->scr_v && h->d_cmd && h->d_stats && h->d_obs && h->d_mask && h->d_nnmask;
#ifndef AIGAR_NO_ARENA
  }
  h->arena_sizing = false;
  h->arena = nullptr;  // later dalloc calls (pixel buffers) allocate on their own
#endif
  if (ok) (void)hipMemset(h->d_nnmask, 1, NP);  // every player is NN until aigar_set_roles
  (void)hipEventCreate(&h->ev0);
  (void)hipEventCreate(&h->ev1);
  if (!ok) {
    free_all(h);
    delete h;
    return fail("aigar_create: device allocation failed");
  }
  if (hipDeviceSynchronize() != hipSuccess) {
    free_all(h);
    delete h;
    return fail("aigar_create: device synchronize failed");
  }
  *out = h;
  return 0;
}

extern "C" int aigar_destroy(aigar_handle *h) {
  if (!h) return 0;
  (void)hipSetDevice(h->cfg.device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  free_all(h);
  delete h;
  return 0;
}

static int check_device_errors(aigar_handle *h) {
  std::vector<ArenaCtl> ctl(h->d.A);
  HIPCHK(hipMemcpyAsync(ctl.data(), h->d.ctl, sizeof(ArenaCtl) * h->d.A, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  for (int a = 0; a < h->d.A; a++)
    if (ctl[a].err)
      return fail("device error bits 0x%x in arena %d (1 pellet cap, 2 blob cap, 4 virus cap, 8 event cap, "
                  "16 worklist cap, 32 observation cap, 64 candidate cap, 128 slot, 256 pixel-frame object cap, "
                  "512 tile message cap, 1024 tile record lookup, 2048 tile view beyond the held pellets, "
                  "4096 tiled tick ended with undone cells, 8192 new-cell / blob counts not as predicted, "
                  "16384 more dead bots to hand off than hand-off slots, 32768 cell claims left at the claim bound)",
                  ctl[a].err, a);
  return 0;
}

__global__ void k_fill_d(double *p, size_t n, double v) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

extern "C" int aigar_reset(aigar_handle *h, uint64_t seed) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  Dev &d = h->d;
  const size_t NP = d.NP, GG = (size_t)d.G * d.G, A = d.A, H1 = (size_t)d.H + 1;
  hipLaunchKernelGGL(k_fill_d, dim3((NP + 255) / 256), dim3(256), 0, h->stream, d.p_cmdx, NP, -1.0);
  hipLaunchKernelGGL(k_fill_d, dim3((NP + 255) / 256), dim3(256), 0, h->stream, d.p_cmdy, NP, -1.0);
  hipLaunchKernelGGL(k_fill_d, dim3((NP + 255) / 256), dim3(256), 0, h->stream, d.o_last_mass, NP,
                     __builtin_nan(""));  // NN bots' lastMass = None (bot.py:125-130)
  HIPCHK(hipMemsetAsync(d.cstart, 0, sizeof(int) * A * H1, h->stream));
  HIPCHK(hipMemsetAsync(d.cgcnt, 0, sizeof(int) * A * 2 * 4100, h->stream));
  HIPCHK(hipMemsetAsync(d.vstart, 0, sizeof(int) * A * H1, h->stream));
  HIPCHK(hipMemsetAsync(d.bstart, 0, sizeof(int) * A * H1, h->stream));
  HIPCHK(hipMemsetAsync(d.bmap, 0, sizeof(uint64_t) * A * 64, h->stream));
  HIPCHK(hipMemsetAsync(d.v_active, 0, sizeof(int) * A * d.Vcap, h->stream));
  HIPCHK(hipMemsetAsync(d.o_lastfov, 0, sizeof(double) * NP, h->stream));
  // Bot.reset (bot.py:125-164): currentAction None (NN) / [0, 0, 0, 0] (Greedy, Random)
  HIPCHK(hipMemsetAsync(d.o_act_cur, 0, sizeof(double) * NP * 4, h->stream));
  for (double *p : {d.o_self_lf, d.o_self_slf, d.o_en_lf, d.o_en_slf})
    HIPCHK(hipMemsetAsync(p, 0, sizeof(double) * NP * GG, h->stream));
  if (d.tiled) {  // every tile's history copy is current (all zero)
    HIPCHK(hipMemsetAsync(d.t_holder, 0xFF, sizeof(int) * NP, h->stream));
    HIPCHK(hipMemsetAsync(d.t_obsby, 0xFF, sizeof(int) * NP, h->stream));
    HIPCHK(hipMemsetAsync(d.t_hodefer, 0, NP, h->stream));  // (hand-off priorities restart)
  }
  launch_reset(d, h->stream, seed);
  HIPCHK(hipGetLastError());
  return check_device_errors(h);
}

extern "C" int aigar_set_commands(aigar_handle *h, const double *cmd, int on_device) {
  if (!h || !cmd) return fail("null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  const double *src = cmd;
  if (!on_device) {
    HIPCHK(hipMemcpyAsync(h->d_cmd, cmd, sizeof(double) * 4 * h->d.NP, hipMemcpyHostToDevice, h->stream));
    src = h->d_cmd;
  }
  launch_set_commands(h->d, h->stream, src);
  HIPCHK(hipGetLastError());
  if (!on_device) HIPCHK(hipStreamSynchronize(h->stream));  // caller may reuse its buffer
  return 0;
}

extern "C" int aigar_policy_random(aigar_handle *h, double p_split, double p_eject, uint64_t seed) {
  if (!h) return fail("null handle");
  Mark m(h, "policy");
  launch_policy(h->d, h->stream, p_split, p_eject, seed);  // draws keyed by (seed, tick, player)
  HIPCHK(hipGetLastError());
  return 0;
}

// Capture launch(stream) into an executable graph on the handle's private
// capture stream: graphs are then replayed on whatever stream the caller gave
// (torch's default stream is the legacy null stream, which cannot capture).
template <class F>
static hipGraphExec_t capture_graph(aigar_handle *h, F launch) {
  if (!h->cap_stream && hipStreamCreateWithFlags(&h->cap_stream, hipStreamNonBlocking) != hipSuccess) {
    h->cap_stream = nullptr;
    return nullptr;
  }
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  bool ok = hipStreamBeginCapture(h->cap_stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
  if (ok) {
    launch(h->cap_stream);
    ok = hipStreamEndCapture(h->cap_stream, &g) == hipSuccess && g;
  }
  if (ok) ok = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) == hipSuccess;
  if (g) (void)hipGraphDestroy(g);
  if (!ok) {
    if (ge) (void)hipGraphExecDestroy(ge);
    (void)hipGetLastError();
    return nullptr;
  }
  return ge;
}

__global__ void k_step_begin(Dev d) {
  int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a < d.A) d.ctl[a].n_ev = 0;
}

static int food_rounds(const aigar_handle *h) { return h->rounds > 0 ? h->rounds : (h->greedy_seen ? 2 : 1); }

// food_rounds() follows the handle's history: when a Greedy policy first runs, the
// graphs captured with the old round count are dropped (recaptured at their next
// call), so a step graph and the tile passes never mix round counts.  (The
// Field.update graph of aigar_step keeps its own graph_rounds check.)
static void note_greedy(aigar_handle *h) {
  if (h->greedy_seen) return;
  h->greedy_seen = true;
  if (h->rounds > 0) return;  // (the round count is fixed: nothing changes)
  (void)hipStreamSynchronize(h->stream);  // (no replay of a graph being destroyed is pending)
  for (hipGraphExec_t *g : {&h->run_graph, &h->run_graph_u, &h->env_graph, &h->tb_graph, &h->te_graph, &h->tr_graph}) {
    if (*g) (void)hipGraphExecDestroy(*g);
    *g = nullptr;
  }
  h->run_u_tried = false;
}

extern "C" int aigar_step(aigar_handle *h, int n_ticks) {
  if (!h) return fail("null handle");
  if (n_ticks < 0) return fail("n_ticks < 0");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (h->d.flags & AIGAR_FLAG_EVENTS)  // the event log restarts every step
    hipLaunchKernelGGL(k_step_begin, dim3((h->d.A + 63) / 64), dim3(64), 0, h->stream, h->d);
  const int rounds = food_rounds(h);
  if (h->graph && h->graph_rounds != rounds) {  // (the population changed the eat phase's rounds)
    (void)hipGraphExecDestroy(h->graph);
    h->graph = nullptr;
  }
  if (h->use_graph && !h->graph && !h->graph_failed && n_ticks > 0) {
    // capture one Field.update() (~25 kernel launches) once; replay it per tick
    h->graph = capture_graph(h, [&](hipStream_t cs) { launch_tick(h->d, cs, rounds, h->scr_k, h->scr_v); });
    if (!h->graph) h->graph_failed = true;
    h->graph_rounds = rounds;
  }
  for (int t = 0; t < n_ticks; t++) {
    Mark m(h, "tick");
    if (h->graph) HIPCHK(hipGraphLaunch(h->graph, h->stream));
    else launch_tick(h->d, h->stream, rounds, h->scr_k, h->scr_v);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

// One batched env step -- Model.update's takeBotActions + Field.update + every
// bot's getStateRepresentation (model.py:100-112, bot.py:272-299) -- captured
// once as a single hipGraph and replayed n_steps times: no host round trip
// between the policy, the tick's ~25 kernels and the observation.
// policy_done: this step's Greedy moves were picked by the previous step's
// observation (fuse_next there); fuse_next: this step's observation also picks the
// next step's Greedy moves (observe_fuses_greedy) -- one launch fewer per step
static void launch_env_step(aigar_handle *h, hipStream_t s, const aigar_run_params &p, void *out, int dtype,
                            bool policy_done = false, bool fuse_next = false) {
  // the random population's policy runs inside the tick's first kernel (same draws as aigar_policy_random)
#ifdef AIGAR_NO_POLICY_FOLD  // (diagnostics build: the policy as its own launch)
  const RandomPolicy rp{0, 0, 0, 0};
  if (p.policy == AIGAR_POLICY_RANDOM) launch_policy(h->d, s, p.p_split, p.p_eject, p.seed);
#else
  const RandomPolicy rp{p.policy == AIGAR_POLICY_RANDOM, p.p_split, p.p_eject, p.seed};
#endif
  if (p.policy == AIGAR_POLICY_GREEDY && !policy_done) launch_policy_greedy(h->d, s, p.greedy_split ? 1 : 0, nullptr, -1);
  // a Greedy population splits by choice: many players hold several cells, and the
  // eat-phase preparation and the pp activity test share a block's cells among its
  // waves (r05 v41: greedy 16.9 -> 18.2 M env-steps/s; the random population keeps
  // the one-wave-per-player kernels, for which the sharing cost ~2 %)
  Dev dt = h->d;
  dt.share_cells = p.policy == AIGAR_POLICY_GREEDY ? 1 : 0;
  launch_tick(dt, s, food_rounds(h), h->scr_k, h->scr_v, &rp);
  if (out) launch_observe(h->d, s, out, dtype, 0, nullptr, fuse_next ? (p.greedy_split ? 1 : 0) : -1);  // epoch 0: the device-side epoch
}
// aigar_run's unrolled graph may carry each step's Greedy moves in the step before
static bool run_fuses_greedy(const aigar_handle *h, const aigar_run_params &p, const void *out) {
  return p.policy == AIGAR_POLICY_GREEDY && out && observe_fuses_greedy(h->d) &&
         !getenv("AIGAR_NO_GREEDY_FUSE");
}

extern "C" int aigar_run(aigar_handle *h, int n_steps, const aigar_run_params *p, void *obs_out, int dtype) {
  if (!h || !p) return fail("null argument");
  if (n_steps < 0) return fail("n_steps < 0");
  if (p->policy < AIGAR_POLICY_NONE || p->policy > AIGAR_POLICY_GREEDY) return fail("unknown policy %d", p->policy);
  if (obs_out && dtype != 0 && dtype != 1) return fail("dtype must be 0 (float64) or 1 (float32)");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (h->d.flags & AIGAR_FLAG_EVENTS)  // the event log restarts every call (all n_steps accumulate)
    hipLaunchKernelGGL(k_step_begin, dim3((h->d.A + 63) / 64), dim3(64), 0, h->stream, h->d);
  if (p->policy == AIGAR_POLICY_GREEDY) note_greedy(h);  // (food_rounds)
  const bool same = h->run_graph && memcmp(&h->run_key, p, sizeof *p) == 0 && h->run_out == obs_out &&
                    h->run_dtype == (obs_out ? dtype : -1);
  if (h->use_graph && !same && n_steps > 0) {
    if (h->run_graph) (void)hipGraphExecDestroy(h->run_graph);
    if (h->run_graph_u) (void)hipGraphExecDestroy(h->run_graph_u);
    h->run_graph = capture_graph(h, [&](hipStream_t cs) { launch_env_step(h, cs, *p, obs_out, dtype); });
    if (!h->run_graph) return fail("aigar_run: graph capture failed");
    h->run_graph_u = nullptr;
    h->run_u_tried = false;
    h->run_key = *p;
    h->run_out = obs_out;
    h->run_dtype = obs_out ? dtype : -1;
  }
  // run_unroll > 1: the same step captured that many times in one graph -- one
  // graph launch, and one inter-graph gap, per run_unroll steps.  Captured at the
  // first call of the key that can use it; if that capture fails, the one-step
  // graph serves alone.
  if (h->run_graph && !h->run_graph_u && !h->run_u_tried && h->run_unroll > 1 && n_steps >= h->run_unroll &&
      !h->profile) {
    h->run_u_tried = true;
    // (the Greedy population: steps 1.. of the graph take the moves their previous
    // step's observation picked -- the first step, and the one-step graph, run the policy)
    const bool fuse = run_fuses_greedy(h, *p, obs_out);
    h->run_graph_u = capture_graph(h, [&](hipStream_t cs) {
      for (int k = 0; k < h->run_unroll; k++)
        launch_env_step(h, cs, *p, obs_out, dtype, fuse && k > 0, fuse && k + 1 < h->run_unroll);
    });
  }
  int t = 0;
  if (h->run_graph_u && !h->profile)
    for (; t + h->run_unroll <= n_steps; t += h->run_unroll) HIPCHK(hipGraphLaunch(h->run_graph_u, h->stream));
  for (; t < n_steps; t++) {
    Mark m(h, "run");
    if (h->run_graph) HIPCHK(hipGraphLaunch(h->run_graph, h->stream));
    else launch_env_step(h, h->stream, *p, obs_out, dtype);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- C4 tiles
static int need_tiled(aigar_handle *h) {
  if (!h) return fail("null handle");
  if (!h->d.tiled) return fail("not a tiled handle (tile_x * tile_y must be > 1, or AIGAR_TILE_FORCE)");
  return 0;
}
extern "C" int aigar_tile_info(aigar_handle *h, int32_t *info, void **outbox, void **inbox, int64_t *msg_bytes) {
  if (need_tiled(h)) return -1;
  const Dev &d = h->d;
  if (info) {
    const int32_t v[14] = {d.ntiles, d.tile_id, d.own_bx0, d.own_bx1, d.own_by0, d.own_by1,
                           d.loc_bx0, d.loc_bx1, d.loc_by0, d.loc_by1, d.tcap, d.bm_words, d.hcap, d.hrec};
    memcpy(info, v, sizeof v);
  }
  if (outbox) *outbox = d.outbox;
  if (inbox) *inbox = (void *)d.inbox;
  if (msg_bytes) *msg_bytes = (int64_t)h->box_recs * (int64_t)sizeof(TileRec);
  return 0;
}
extern "C" int aigar_tile_msg_bytes(aigar_handle *h, int64_t *bytes) {
  if (need_tiled(h) || !bytes) return bytes ? -1 : fail("null argument");
  if (!h->pass_recs) return fail("tile_msg_bytes: no pass begun");
  *bytes = (int64_t)h->pass_recs * (int64_t)sizeof(TileRec);
  return 0;
}
extern "C" int aigar_tile_set_buffers(aigar_handle *h, void *outbox, void *inbox) {
  if (need_tiled(h)) return -1;
  if (!outbox || !inbox) return fail("tile_set_buffers: null buffer");
  HIPCHK(hipStreamSynchronize(h->stream));
  h->d.outbox = (TileRec *)outbox;
  h->d.inbox = (const TileRec *)inbox;
  return 0;
}
// Greedy bots on tiles: each tile moves the bots it observes, the commands go
// round in their own message (k_tile_cmd_collect / k_tile_cmd_apply, tick.hip)
extern "C" int aigar_tile_policy(aigar_handle *h, int greedy_split) {
  if (need_tiled(h)) return -1;
  HIPCHK(hipSetDevice(h->cfg.device));
  note_greedy(h);  // (food_rounds)
  {
    Mark m(h, "policy");
    launch_tile_policy(h->d, h->stream, greedy_split ? 1 : 0, h->d_mask, h->box_recs - 1);
  }
  h->pass_recs = h->box_recs;  // (the command message: the whole buffer is exchanged)
  h->cmd_ready = false;
  h->cmd_pending = true;
  HIPCHK(hipGetLastError());
  return 0;
}
extern "C" int aigar_tile_apply_commands(aigar_handle *h) {
  if (need_tiled(h)) return -1;
  // (a flag of its own: pass_recs alone can equal box_recs after an eat pass)
  if (!h->cmd_pending || h->pass_recs != h->box_recs)
    return fail("tile_apply_commands: no aigar_tile_policy before it");
  HIPCHK(hipSetDevice(h->cfg.device));
  launch_tile_cmd_apply(h->d, h->stream, h->box_recs);
  HIPCHK(hipGetLastError());
  h->pass_recs = 0;
  h->cmd_pending = false;
  h->cmd_ready = true;
  return 0;
}
extern "C" int aigar_tile_begin(aigar_handle *h, const aigar_run_params *p) {
  if (need_tiled(h) || !p) return p ? -1 : fail("null argument");
  if (p->policy == AIGAR_POLICY_GREEDY && !h->cmd_ready)
    return fail("tile_begin: GREEDY needs this tick's commands (aigar_tile_policy, all-gather, "
                "aigar_tile_apply_commands): no tile holds every pellet a Greedy move reads");
  if (p->policy != AIGAR_POLICY_NONE && p->policy != AIGAR_POLICY_RANDOM && p->policy != AIGAR_POLICY_GREEDY)
    return fail("tile_begin: unknown policy %d", p->policy);
  h->cmd_ready = false;
  HIPCHK(hipSetDevice(h->cfg.device));
  if (h->d.flags & AIGAR_FLAG_EVENTS)  // the event log holds this tick
    hipLaunchKernelGGL(k_step_begin, dim3(1), dim3(64), 0, h->stream, h->d);
  const RandomPolicy rp{p->policy == AIGAR_POLICY_RANDOM, p->p_split, p->p_eject, p->seed};  // (GREEDY: set already)
  auto issue = [&](hipStream_t s) {
    launch_tick_pre(h->d, s, h->scr_k, h->scr_v, &rp);
    launch_tile_pass(h->d, s, food_rounds(h), h->scr_k, h->scr_v, 1);
  };
  const bool same = h->tb_graph && memcmp(&h->tb_key, p, sizeof *p) == 0 && h->tb_box[0] == h->d.outbox &&
                    h->tb_box[1] == h->d.inbox;
  if (h->tile_graph && !same) {
    if (h->tb_graph) (void)hipGraphExecDestroy(h->tb_graph);
    h->tb_graph = capture_graph(h, issue);
    h->tb_key = *p;
    h->tb_box[0] = h->d.outbox;
    h->tb_box[1] = h->d.inbox;
  }
  {
    Mark m(h, "tile_begin");
    if (h->tile_graph && h->tb_graph) HIPCHK(hipGraphLaunch(h->tb_graph, h->stream));
    else issue(h->stream);
  }
  h->pass_recs = 1 + h->d.tcap + h->d.hcap * h->d.hrec;  // (+ the observation-history hand-off slots)
  h->cmd_pending = false;
  h->first_pass = 1;
  HIPCHK(hipGetLastError());
  return 0;
}
extern "C" int aigar_tile_apply(aigar_handle *h, int *undone) {
  if (need_tiled(h)) return -1;
  if (!h->pass_recs) return fail("tile_apply: no pass begun");
  HIPCHK(hipSetDevice(h->cfg.device));
  {
    Mark m(h, "tile_apply");
    launch_tile_apply(h->d, h->stream, h->pass_recs, h->first_pass);
  }
  HIPCHK(hipGetLastError());
  if (!undone) return 0;  // device-decided passes: no host round trip (aigar_tile_resume gates itself)
  ArenaCtl c;
  HIPCHK(hipMemcpyAsync(&c, h->d.ctl, sizeof c, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (c.err) return check_device_errors(h);
  *undone = c.n_undone_glob;
  return 0;
}
extern "C" int aigar_tile_resume(aigar_handle *h) {
  if (need_tiled(h)) return -1;
  HIPCHK(hipSetDevice(h->cfg.device));
  Mark m(h, "tile_resume");
  launch_tile_pass(h->d, h->stream, food_rounds(h), h->scr_k, h->scr_v, 0);
  h->pass_recs = 1 + h->d.tcap + h->d.bm_words / 4;
  h->cmd_pending = false;
  h->first_pass = 0;
  HIPCHK(hipGetLastError());
  return 0;
}
extern "C" int aigar_tile_end(aigar_handle *h, void *obs_out, int dtype) {
  if (need_tiled(h)) return -1;
  if (obs_out && dtype != 0 && dtype != 1) return fail("dtype must be 0 (float64) or 1 (float32)");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (h->profile || !h->tile_graph) {  // separate launches (the post phases and the observation timed apart)
    {
      Mark m(h, "tile_end");
      launch_tick_post(h->d, h->stream, h->scr_k, h->scr_v);
    }
    if (obs_out) {
      Mark m(h, "observe");
      launch_observe(h->d, h->stream, obs_out, dtype, 0);
    }
    HIPCHK(hipGetLastError());
    return 0;
  }
  auto issue = [&](hipStream_t s) {
    launch_tick_post(h->d, s, h->scr_k, h->scr_v);
    if (obs_out) launch_observe(h->d, s, obs_out, dtype, 0);
  };
  const bool same = h->te_graph && h->te_out == obs_out && h->te_dtype == (obs_out ? dtype : -1) &&
                    h->te_box[0] == h->d.outbox && h->te_box[1] == h->d.inbox;
  if (h->use_graph && !same) {
    if (h->te_graph) (void)hipGraphExecDestroy(h->te_graph);
    h->te_graph = capture_graph(h, issue);
    h->te_out = obs_out;
    h->te_dtype = obs_out ? dtype : -1;
    h->te_box[0] = h->d.outbox;
    h->te_box[1] = h->d.inbox;
  }
  if (h->use_graph && h->te_graph) HIPCHK(hipGraphLaunch(h->te_graph, h->stream));
  else issue(h->stream);
  HIPCHK(hipGetLastError());
  return 0;
}
// in-process transport: every handle's outbox into every handle's inbox slot
// No host synchronisation: each source's outbox is complete when its stream
// reaches the recorded event (every destination waits for it before copying),
// and every source's later work (the next pass rewrites its outbox) waits for
// all destinations' copies.
extern "C" int aigar_tile_exchange_local(aigar_handle **hs, int n) {
  if (!hs || n < 1) return fail("null argument");
  uint64_t seen = 0;
  for (int i = 0; i < n; i++) {
    if (need_tiled(hs[i])) return -1;
    if (hs[i]->d.ntiles != n || hs[i]->pass_recs != hs[0]->pass_recs || hs[i]->pass_recs == 0)
      return fail("tile_exchange_local: tiles are not at the same pass");
    const uint64_t bit = 1ull << hs[i]->d.tile_id;
    if (seen & bit) return fail("tile_exchange_local: tile %d appears twice", hs[i]->d.tile_id);
    seen |= bit;
    HIPCHK(hipSetDevice(hs[i]->cfg.device));
    if (!hs[i]->ev_x) HIPCHK(hipEventCreateWithFlags(&hs[i]->ev_x, hipEventDisableTiming));
    HIPCHK(hipEventRecord(hs[i]->ev_x, hs[i]->stream));  // outbox written
  }
  const size_t bytes = (size_t)hs[0]->pass_recs * sizeof(TileRec);
  for (int i = 0; i < n; i++) {
    HIPCHK(hipSetDevice(hs[i]->cfg.device));
    for (int k = 0; k < n; k++)
      if (k != i) HIPCHK(hipStreamWaitEvent(hs[i]->stream, hs[k]->ev_x, 0));
  }
  for (int i = 0; i < n; i++) {
    HIPCHK(hipSetDevice(hs[i]->cfg.device));
    for (int k = 0; k < n; k++) {
      const aigar_handle *src = hs[k];
      HIPCHK(hipMemcpyAsync((char *)hs[i]->d.inbox + (size_t)src->d.tile_id * bytes, src->d.outbox, bytes,
                            hipMemcpyDeviceToDevice, hs[i]->stream));
    }
  }
  for (int i = 0; i < n; i++) {  // inbox i filled (re-recorded: the outbox events are waited on already)
    HIPCHK(hipSetDevice(hs[i]->cfg.device));
    HIPCHK(hipEventRecord(hs[i]->ev_x, hs[i]->stream));
  }
  for (int k = 0; k < n; k++) {
    HIPCHK(hipSetDevice(hs[k]->cfg.device));
    for (int i = 0; i < n; i++)
      if (i != k) HIPCHK(hipStreamWaitEvent(hs[k]->stream, hs[i]->ev_x, 0));
  }
  return 0;
}

// ---------------------------------------------------------------- C4 over RCCL
// The exchange is ncclAllGather over the tiles' communicator (xGMI between the
// GPUs of a node).  librccl.so is bound at run time (dlopen of the file the
// caller names -- torch's, so one HIP runtime serves both -- and dlsym of the
// five entry points used); the library itself does not link RCCL.

extern "C" int aigar_rccl_unique_id(const char *path, void *id) {
  if (!id) return fail("null argument");
  if (rccl_load(path)) return -1;
  RcclId u;
  const int r = g_rccl.get_unique_id(&u);
  if (r) return fail("ncclGetUniqueId: %s", g_rccl.error_string(r));
  memcpy(id, &u, sizeof u);
  return 0;
}

extern "C" int aigar_tile_comm_init(aigar_handle *h, const char *path, const void *id, int nranks, int rank) {
  if (need_tiled(h)) return -1;
  if (!id) return fail("null argument");
  if (nranks != h->d.ntiles || rank != h->d.tile_id)
    return fail("tile_comm_init: %d ranks / rank %d for %d tiles / tile %d (one rank per tile, rank = tile id)",
                nranks, rank, h->d.ntiles, h->d.tile_id);
  if (rccl_load(path)) return -1;
  HIPCHK(hipSetDevice(h->cfg.device));
  if (h->rccl_comm) {
    (void)g_rccl.comm_destroy(h->rccl_comm);
    h->rccl_comm = nullptr;
  }
  RcclId u;
  memcpy(&u, id, sizeof u);
  const int r = g_rccl.comm_init_rank(&h->rccl_comm, nranks, u, rank);
  if (r) {
    h->rccl_comm = nullptr;
    return fail("ncclCommInitRank(%d ranks, rank %d): %s", nranks, rank, g_rccl.error_string(r));
  }
  h->rccl_ranks = nranks;
  return 0;
}

// every tile's current-pass message into every tile's inbox (tile k at k * bytes)
static int tile_allgather(aigar_handle *h, hipStream_t s, int recs) {
  if (h->loopback) {  // (aigar_tile_loopback: the other slots hold empty messages)
    const size_t bytes = (size_t)recs * sizeof(TileRec);
    HIPCHK(hipMemcpyAsync((char *)h->d.inbox + (size_t)h->d.tile_id * bytes, h->d.outbox, bytes,
                          hipMemcpyDeviceToDevice, s));
    return 0;
  }
  const int r = g_rccl.all_gather(h->d.outbox, (void *)h->d.inbox, (size_t)recs * sizeof(TileRec), kNcclUint8,
                                  h->rccl_comm, s);
  if (r) {
    h->rccl_bad = true;
    return fail("ncclAllGather: %s", g_rccl.error_string(r));
  }
  return 0;
}

// One tiled step (the rank-side sequence of include/aigar.h's aigar_tile_* calls)
static int issue_tile_step(aigar_handle *h, hipStream_t s, const aigar_run_params &p, int extra, void *obs,
                           int dtype) {
  const RandomPolicy rp{p.policy == AIGAR_POLICY_RANDOM, p.p_split, p.p_eject, p.seed};
  const int first_recs = 1 + h->d.tcap + h->d.hcap * h->d.hrec, later_recs = 1 + h->d.tcap + h->d.bm_words / 4;
  if (p.policy == AIGAR_POLICY_GREEDY) {  // each tile moves the bots it observes; the commands go round first
    Mark m(h, "policy");
    launch_tile_policy(h->d, s, p.greedy_split ? 1 : 0, h->d_mask, h->box_recs - 1);
    if (tile_allgather(h, s, h->box_recs)) return -1;
    launch_tile_cmd_apply(h->d, s, h->box_recs);
  }
  {
    Mark m(h, "tile_begin");
    launch_tick_pre(h->d, s, h->scr_k, h->scr_v, &rp);
    launch_tile_pass(h->d, s, food_rounds(h), h->scr_k, h->scr_v, 1);
  }
  for (int k = 0; k <= extra; k++) {
    {
      Mark m(h, "exchange");
      if (tile_allgather(h, s, k == 0 ? first_recs : later_recs)) return -1;
    }
    {
      Mark m(h, "tile_apply");
      launch_tile_apply(h->d, s, k == 0 ? first_recs : later_recs, k == 0 ? 1 : 0);
    }
    if (k < extra) {
      Mark m(h, "tile_resume");
      launch_tile_pass(h->d, s, food_rounds(h), h->scr_k, h->scr_v, 0);
    }
  }
  {
    Mark m(h, "tile_end");
    launch_tick_post(h->d, s, h->scr_k, h->scr_v);
  }
  if (obs) {
    Mark m(h, "observe");
    launch_observe(h->d, s, obs, dtype, 0);
  }
  return 0;
}

extern "C" int aigar_tile_run(aigar_handle *h, int n_steps, const aigar_run_params *p, int extra_passes,
                              void *obs_out, int dtype) {
  if (need_tiled(h) || !p) return p ? -1 : fail("null argument");
  if (!h->rccl_comm && !h->loopback) return fail("tile_run: no RCCL communicator (aigar_tile_comm_init)");
  if (n_steps < 0 || extra_passes < 0 || extra_passes > 64) return fail("tile_run: bad n_steps / extra_passes");
  if (p->policy < AIGAR_POLICY_NONE || p->policy > AIGAR_POLICY_GREEDY) return fail("tile_run: unknown policy %d", p->policy);
  if (p->policy == AIGAR_POLICY_GREEDY) note_greedy(h);  // (food_rounds)
  if (obs_out && dtype != 0 && dtype != 1) return fail("dtype must be 0 (float64) or 1 (float32)");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (h->d.flags & AIGAR_FLAG_EVENTS)  // the event log restarts every call (all n_steps accumulate)
    hipLaunchKernelGGL(k_step_begin, dim3(1), dim3(64), 0, h->stream, h->d);
  h->pass_recs = 0;  // (the aigar_tile_* call sequence restarts at a tile_begin)
  h->cmd_pending = false;
  const bool same = h->tr_graph && memcmp(&h->tr_key, p, sizeof *p) == 0 && h->tr_out == obs_out &&
                    h->tr_dtype == (obs_out ? dtype : -1) && h->tr_extra == extra_passes;
  if (h->use_graph && !h->profile && !same && !h->tr_failed && n_steps > 0) {
    if (h->tr_graph) (void)hipGraphExecDestroy(h->tr_graph);
    h->rccl_bad = false;
    h->tr_graph = capture_graph(h, [&](hipStream_t cs) { (void)issue_tile_step(h, cs, *p, extra_passes, obs_out, dtype); });
    if (h->rccl_bad && h->tr_graph) {  // an all-gather refused the capture: direct launches from now on
      (void)hipGraphExecDestroy(h->tr_graph);
      h->tr_graph = nullptr;
    }
    if (!h->tr_graph) h->tr_failed = true;
    h->tr_key = *p;
    h->tr_out = obs_out;
    h->tr_dtype = obs_out ? dtype : -1;
    h->tr_extra = extra_passes;
  }
  for (int t = 0; t < n_steps; t++) {
    if (h->tr_graph && !h->profile) {
      Mark m(h, "tile_step");
      HIPCHK(hipGraphLaunch(h->tr_graph, h->stream));
    } else if (issue_tile_step(h, h->stream, *p, extra_passes, obs_out, dtype)) {
      return -1;
    }
  }
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int aigar_tile_run_graphed(aigar_handle *h) { return h && h->tr_graph ? 1 : 0; }

extern "C" int aigar_tile_loopback(aigar_handle *h) {
  if (need_tiled(h)) return -1;
  HIPCHK(hipSetDevice(h->cfg.device));
  // every slot an empty message (kind TR_HDR, no records, nothing undone, no kills)
  HIPCHK(hipMemsetAsync((void *)h->d.inbox, 0, (size_t)h->box_recs * h->d.ntiles * sizeof(TileRec), h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->loopback = true;
  if (h->tr_graph) (void)hipGraphExecDestroy(h->tr_graph);
  h->tr_graph = nullptr;
  h->tr_failed = false;
  return 0;
}

// the tile that computed each bot's row at the last observation (-1: dead /
// not observed); every tile computes the same assignment
extern "C" int aigar_tile_observers(aigar_handle *h, int32_t *out) {
  if (need_tiled(h) || !out) return out ? -1 : fail("null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  HIPCHK(hipMemcpyAsync(out, h->d.t_obsby, sizeof(int32_t) * h->d.NP, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return check_device_errors(h);
}

// One learner decision for every player (bot.py:166-233 batched, the loop of
// aigar.py:performModelSteps): the action through set_command_point, held for
// skip + 1 ticks with split/eject dropped on the skipped ones, the rewards of
// the window summed, then every bot's observation -- one graph replay.
// Mixed populations (aigar_set_roles): per tick, the NN bots' held action, then
// the Greedy and Random bots' moves (Model.takeBotActions, model.py:113-115; the
// moves are independent of each other), then Field.update; the observation is
// computed for the NN bots only.
static void launch_env_decision(aigar_handle *h, hipStream_t s, const aigar_handle::EnvKey &k) {
  for (int t = 0; t <= k.skip; t++) {
    if (t > 0) launch_rewards(h->d, s, k.reward, k.prm, 0, t == 1 ? 1 : 2);  // updateRewards (bot.py:166-168)
    launch_apply_actions(h->d, s, k.act, k.n_act, k.enable_split, t > 0, t == 0);
    if (k.n_greedy) launch_policy_greedy(h->d, s, k.envp.greedy_split, h->d.p_role, AIGAR_ROLE_GREEDY);
    if (k.n_random)
      launch_policy_refrandom(h->d, s, k.envp.random_skip, k.envp.random_split, k.envp.random_eject, k.envp.salt);
    launch_tick(h->d, s, food_rounds(h), h->scr_k, h->scr_v);
  }
  launch_rewards(h->d, s, k.reward, k.prm, 1, k.skip == 0 ? 1 : 2);  // end of move_NN (bot.py:220-230)
  launch_observe(h->d, s, k.obs, k.dtype, 0, (k.n_greedy || k.n_random) ? h->d_nnmask : nullptr);
}

extern "C" int aigar_env_step(aigar_handle *h, const double *act, int n_act, int enable_split, int skip,
                              const aigar_reward_params *p, double *reward_out, void *obs_out, int dtype) {
  if (!h || !act || !p || !reward_out || !obs_out) return fail("null argument");
  if (n_act < 2 || n_act > 4) return fail("env_step: n_act must be 2, 3 or 4");
  if (skip < 0) return fail("env_step: skip < 0");
  if (dtype != 0 && dtype != 1) return fail("dtype must be 0 (float64) or 1 (float32)");
  HIPCHK(hipSetDevice(h->cfg.device));
  aigar_handle::EnvKey k{};
  k.act = act;
  k.n_act = n_act;
  k.enable_split = enable_split ? 1 : 0;
  k.skip = skip;
  k.dtype = dtype;
  k.prm = *p;
  k.reward = reward_out;
  k.obs = obs_out;
  k.envp = h->envp;
  k.n_greedy = h->n_greedy;
  k.n_random = h->n_random;
  if (h->d.flags & AIGAR_FLAG_EVENTS)  // the event log holds the window's ticks
    hipLaunchKernelGGL(k_step_begin, dim3((h->d.A + 63) / 64), dim3(64), 0, h->stream, h->d);
  if (!h->use_graph) {
    launch_env_decision(h, h->stream, k);
  } else {
    if (!h->env_graph || memcmp(&h->env_key, &k, sizeof k) != 0) {
      if (h->env_graph) (void)hipGraphExecDestroy(h->env_graph);
      h->env_graph = capture_graph(h, [&](hipStream_t cs) { launch_env_decision(h, cs, k); });
      if (!h->env_graph) return fail("env_step: graph capture failed");
      h->env_key = k;
    }
    Mark m(h, "env_step");
    HIPCHK(hipGraphLaunch(h->env_graph, h->stream));
  }
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int aigar_set_roles(aigar_handle *h, const uint8_t *roles, int on_device) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  const int NP = h->d.NP;
  std::vector<uint8_t> r(NP, AIGAR_ROLE_NN);
  if (roles) {
    if (on_device) HIPCHK(hipMemcpy(r.data(), roles, NP, hipMemcpyDeviceToHost));
    else memcpy(r.data(), roles, NP);
  }
  std::vector<uint8_t> nn(NP);
  int ng = 0, nr = 0;
  for (int i = 0; i < NP; i++) {
    if (r[i] > AIGAR_ROLE_RANDOM) return fail("set_roles: role %d of player %d is not an AIGAR_ROLE_*", r[i], i);
    ng += r[i] == AIGAR_ROLE_GREEDY;
    nr += r[i] == AIGAR_ROLE_RANDOM;
    nn[i] = r[i] == AIGAR_ROLE_NN;
  }
  HIPCHK(hipMemcpyAsync(h->d.p_role, r.data(), NP, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d_nnmask, nn.data(), NP, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->n_greedy = ng;
  h->n_random = nr;
  if (ng) note_greedy(h);  // (food_rounds)
  return 0;
}
extern "C" int aigar_env_config(aigar_handle *h, const aigar_env_params *p) {
  if (!h || !p) return fail("null argument");
  h->envp = *p;
  return 0;
}
extern "C" int aigar_policy_random_bots(aigar_handle *h) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  launch_policy_refrandom(h->d, h->stream, h->envp.random_skip, h->envp.random_split, h->envp.random_eject,
                          h->envp.salt);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int aigar_obs_len(aigar_handle *h) { return h ? h->d.L : -1; }

extern "C" int aigar_observe(aigar_handle *h, void *out, int dtype, int on_device) {
  return aigar_observe_masked(h, out, dtype, on_device, nullptr, 0);
}
extern "C" int aigar_observe_masked(aigar_handle *h, void *out, int dtype, int on_device, const uint8_t *mask,
                                    int mask_on_device) {
  if (!h || !out) return fail("null argument");
  if (dtype != 0 && dtype != 1) return fail("dtype must be 0 (float64) or 1 (float32)");
  HIPCHK(hipSetDevice(h->cfg.device));
  void *dst = on_device ? out : h->d_obs;
  const uint8_t *m = mask;
  if (mask && !mask_on_device) {
    HIPCHK(hipMemcpyAsync(h->d_mask, mask, (size_t)h->d.NP, hipMemcpyHostToDevice, h->stream));
    m = h->d_mask;
  }
  if (!on_device && mask) {  // rows of masked-out bots are left as the caller's buffer has them
    size_t bytes = (size_t)h->d.NP * h->d.L * (dtype == 0 ? 8 : 4);
    HIPCHK(hipMemcpyAsync(h->d_obs, out, bytes, hipMemcpyHostToDevice, h->stream));
  }
  {
    Mark mk(h, "observe");
    launch_observe(h->d, h->stream, dst, dtype, ++h->obs_calls, m);
  }
  HIPCHK(hipGetLastError());
  if (!on_device) {
    size_t bytes = (size_t)h->d.NP * h->d.L * (dtype == 0 ? 8 : 4);
    HIPCHK(hipMemcpyAsync(out, h->d_obs, bytes, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return check_device_errors(h);
  }
  return 0;
}

extern "C" int aigar_observe_pixels(aigar_handle *h, void *out, int side, uint64_t color_seed, int dtype,
                                    int on_device) {
  if (!h || !out) return fail("null argument");
  if (side < 1 || side > 84) return fail("pixel frame side must be in [1, 84], got %d", side);
  if (dtype < 0 || dtype > 2) return fail("dtype must be 0 (float64 gray), 1 (float32 gray) or 2 (uint8 rgb)");
  HIPCHK(hipSetDevice(h->cfg.device));
  const size_t bytes = (size_t)h->d.NP * side * side * (dtype == 0 ? 8 : dtype == 1 ? 4 : 3);
  if (!h->d_pix_ovf) {
    h->d_pix_ovf = dalloc<uint8_t>(h, h->d.NP);
    if (!h->d_pix_ovf) return fail("out of device memory");
  }
  void *dst = out;
  if (!on_device) {
    if (bytes > h->pix_bytes) {
      if (h->d_pix) HIPCHK(hipFree(h->d_pix));
      h->d_pix = nullptr;
      h->pix_bytes = 0;
      HIPCHK(hipMalloc(&h->d_pix, bytes));
      h->pix_bytes = bytes;
    }
    dst = h->d_pix;
  }
  {
    Mark m(h, "observe_pixels");
    if (launch_observe_pixels(h->d, h->stream, dst, dtype, side, color_seed, h->d_pix_ovf)) return fail("bad pixel launch");
  }
  HIPCHK(hipGetLastError());
  if (!on_device) {
    HIPCHK(hipMemcpyAsync(out, h->d_pix, bytes, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return check_device_errors(h);
  }
  return 0;
}

__global__ void k_set_actions(Dev d, const double *cur, const double *prev) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (size_t)d.NP * 4) return;
  if (cur) d.o_act_cur[i] = cur[i];
  if (prev) d.o_act_prev[i] = prev[i];
}

extern "C" int aigar_set_actions(aigar_handle *h, const double *cur, const double *prev, int on_device) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  size_t n = (size_t)h->d.NP * 4;
  if (on_device) {
    hipLaunchKernelGGL(k_set_actions, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->d, cur, prev);
  } else {
    if (cur) HIPCHK(hipMemcpyAsync(h->d.o_act_cur, cur, n * 8, hipMemcpyHostToDevice, h->stream));
    if (prev) HIPCHK(hipMemcpyAsync(h->d.o_act_prev, prev, n * 8, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  return 0;
}

// Bot.reset (bot.py:125-164) for the masked players: an NN bot's last /
// second-last self and enemy grids restart at zero and fovSize / lastFovSize at
// 0 (the collector calls model.resetBots() every FRAME_SKIP_RATE + 2 updates,
// aigar.py:845-852).  C4: every tile's copy is then current (all zero).
__global__ void k_reset_bots(Dev d, const uint8_t *mask) {
  const int GG = d.G * d.G;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (size_t)d.NP * GG) return;
  const int gp = (int)(i / GG);
  if (mask && !mask[gp]) return;
  d.o_self_lf[i] = d.o_self_slf[i] = d.o_en_lf[i] = d.o_en_slf[i] = 0.0;
  if (i % GG == 0) {
    d.o_lastfov[gp] = 0.0;
    if (d.tiled) d.t_holder[gp] = -1;
  }
}

extern "C" int aigar_reset_bots(aigar_handle *h, const uint8_t *mask, int on_device) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  const uint8_t *m = mask;
  if (mask && !on_device) {
    HIPCHK(hipMemcpyAsync(h->d_mask, mask, (size_t)h->d.NP, hipMemcpyHostToDevice, h->stream));
    m = h->d_mask;
  }
  const size_t n = (size_t)h->d.NP * h->d.G * h->d.G;
  hipLaunchKernelGGL(k_reset_bots, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream, h->d, m);
  HIPCHK(hipGetLastError());
  if (mask && !on_device) HIPCHK(hipStreamSynchronize(h->stream));  // caller may reuse its buffer
  return 0;
}

extern "C" int aigar_player_stats(aigar_handle *h, double *out, int on_device) {
  if (!h || !out) return fail("null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  launch_player_stats(h->d, h->stream, on_device ? out : h->d_stats);
  if (!on_device) {
    HIPCHK(hipMemcpyAsync(out, h->d_stats, sizeof(double) * 5 * h->d.NP, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  return 0;
}

extern "C" int aigar_set_stream(aigar_handle *h, void *s) {
  if (!h) return fail("null handle");
  HIPCHK(hipStreamSynchronize(h->stream));
  if (h->own_stream) (void)hipStreamDestroy(h->stream);
  h->stream = (hipStream_t)s;
  h->own_stream = false;
  return 0;
}

extern "C" int aigar_sync(aigar_handle *h) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  return check_device_errors(h);
}

// diagnostics: the first list row (the slot of every player's first cell) and
// the cell counts, [NP] bytes and [NP] ints (tools/first_slot.py)
extern "C" int aigar_debug_first_slots(aigar_handle *h, uint8_t *slot0, int *ncells) {
  if (!h || !slot0 || !ncells) return fail("null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpy(slot0, h->d.p_list, h->d.NP, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(ncells, h->d.p_ncells, sizeof(int) * h->d.NP, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int aigar_profile(aigar_handle *h, int enable) {
  if (!h) return fail("null handle");
  HIPCHK(hipStreamSynchronize(h->stream));
  for (auto &m : h->marks) {
    h->event_pool.push_back(m.second.first);
    h->event_pool.push_back(m.second.second);
  }
  h->marks.clear();
  h->profile = enable != 0;
  return 0;
}
// total HIP-event time (ms) and launch count of a timer since aigar_profile(h, 1):
// "tick" (one Field.update), "observe" (k_observe), "policy" (k_policy_random)
extern "C" int aigar_kernel_time(aigar_handle *h, const char *name, double *ms, int *launches) {
  if (!h || !name || !ms || !launches) return fail("null argument");
  HIPCHK(hipStreamSynchronize(h->stream));
  double tot = 0;
  int n = 0;
  for (auto &m : h->marks) {
    if (m.first != name) continue;
    float t = 0;
    HIPCHK(hipEventElapsedTime(&t, m.second.first, m.second.second));
    tot += t;
    n++;
  }
  *ms = tot;
  *launches = n;
  return 0;
}

// ---------------------------------------------------------------- snapshots
template <class T>
static int d2h(aigar_handle *h, std::vector<T> &v, const T *src, size_t n) {
  v.resize(n);
  if (n) HIPCHK(hipMemcpyAsync(v.data(), src, n * sizeof(T), hipMemcpyDeviceToHost, h->stream));
  return 0;
}
template <class T>
static int h2d(aigar_handle *h, T *dst, const std::vector<T> &v) {
  if (!v.empty()) HIPCHK(hipMemcpyAsync(dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, h->stream));
  return 0;
}

extern "C" int aigar_get_state(aigar_handle *h, int arena, aigar_state *st) {
  if (!h || !st) return fail("null argument");
  Dev &d = h->d;
  if (arena < 0 || arena >= d.A) return fail("arena %d out of range", arena);
  HIPCHK(hipSetDevice(h->cfg.device));
  if (check_device_errors(h)) return -1;
  ArenaCtl c;
  HIPCHK(hipMemcpy(&c, d.ctl + arena, sizeof c, hipMemcpyDeviceToHost));
  const int B = d.B, NP = d.NP;
  const size_t p0 = (size_t)arena * B;
  std::vector<int> alive, resp, ncells, split, eject, dead;
  std::vector<double> cmdx, cmdy;
  if (d2h(h, alive, d.p_alive + p0, B) || d2h(h, resp, d.p_respawn + p0, B) || d2h(h, ncells, d.p_ncells + p0, B) ||
      d2h(h, split, d.p_split + p0, B) || d2h(h, eject, d.p_eject + p0, B) || d2h(h, cmdx, d.p_cmdx + p0, B) ||
      d2h(h, cmdy, d.p_cmdy + p0, B) || d2h(h, dead, d.dead + p0, c.n_dead))
    return -1;
  // cells: 16 slot rows of this arena's players
  std::vector<uint8_t> lst((size_t)kMaxCells * B);
  std::vector<double> cf[9];
  std::vector<int> csvc((size_t)kMaxCells * B);
  std::vector<uint32_t> cfl((size_t)kMaxCells * B);
  std::vector<int64_t> cseq((size_t)kMaxCells * B);
  double *cfs[9] = {d.c_x, d.c_y, d.c_m, d.c_r, d.c_vx, d.c_vy, d.c_svx, d.c_svy, d.c_mt};
  for (int f = 0; f < 9; f++) cf[f].resize((size_t)kMaxCells * B);
  for (int s = 0; s < kMaxCells; s++) {
    size_t o = (size_t)s * NP + p0, ho = (size_t)s * B;
    HIPCHK(hipMemcpyAsync(lst.data() + ho, d.p_list + o, B, hipMemcpyDeviceToHost, h->stream));
    for (int f = 0; f < 9; f++)
      HIPCHK(hipMemcpyAsync(cf[f].data() + ho, cfs[f] + o, 8 * B, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(csvc.data() + ho, d.c_svc + o, 4 * B, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(cfl.data() + ho, d.c_flags + o, 4 * B, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(cseq.data() + ho, d.c_seq + o, 8 * B, hipMemcpyDeviceToHost, h->stream));
  }
  const size_t po = (size_t)arena * d.PS, bo = (size_t)arena * d.Ecap, vo = (size_t)arena * d.Vcap;
  std::vector<double> px, py, pm, bf[8], vf[8];
  std::vector<int64_t> ps, bseq, bej, vseq;
  std::vector<int> bsvc, vsvc, pcol, bcol;
  std::vector<uint32_t> bfl, vfl;
  int n_pel = 0;
  {  // the row store: each row's live records [entry 0, entry cols) of its current home,
     // packed on the device (k_pel_gather) so only the live records are copied
    std::vector<int> pst;
    std::vector<PelRec> store;
    std::vector<int> scol;
    if (d2h(h, pst, d.pstart + (size_t)arena * d.PH1, d.PH1)) return -1;
    HIPCHK(hipStreamSynchronize(h->stream));
    long tot = 0;
    for (int r = 0; r < d.cols; r++) tot += pst[(size_t)r * (d.cols + 1) + d.cols] - pst[(size_t)r * (d.cols + 1)];
    if (tot > d.Pcap) return fail("get_state: %ld live pellet records exceed the capacity %d", tot, d.Pcap);
    launch_pel_gather(d, h->stream, arena);
    HIPCHK(hipGetLastError());
    if (d2h(h, store, d.pn + (size_t)arena * d.Pcap, (int)tot) || d2h(h, scol, d.pn_col + (size_t)arena * d.Pcap, (int)tot))
      return -1;
    HIPCHK(hipStreamSynchronize(h->stream));  // (unpacked below)
    for (long i = 0; i < tot; i++) {
      px.push_back(store[i].x); py.push_back(store[i].y); pm.push_back(store[i].m); ps.push_back(store[i].seq);
      pcol.push_back(scol[i]);
    }
    n_pel = (int)px.size();
  }
  double *bfs[8] = {d.b_x, d.b_y, d.b_m, d.b_r, d.b_vx, d.b_vy, d.b_svx, d.b_svy};
  double *vfs[8] = {d.v_x, d.v_y, d.v_m, d.v_r, d.v_vx, d.v_vy, d.v_svx, d.v_svy};
  for (int f = 0; f < 8; f++)
    if (d2h(h, bf[f], bfs[f] + bo, c.n_blob) || d2h(h, vf[f], vfs[f] + vo, c.n_vir)) return -1;
  if (d2h(h, bsvc, d.b_svc + bo, c.n_blob) || d2h(h, bseq, d.b_seq + bo, c.n_blob) ||
      d2h(h, bej, d.b_ej + bo, c.n_blob) || d2h(h, bfl, d.b_flags + bo, c.n_blob) || d2h(h, bcol, d.b_col + bo, c.n_blob) ||
      d2h(h, vsvc, d.v_svc + vo, c.n_vir) || d2h(h, vseq, d.v_seq + vo, c.n_vir) ||
      d2h(h, vfl, d.v_flags + vo, c.n_vir))
    return -1;
  HIPCHK(hipStreamSynchronize(h->stream));

  int nc = 0;
  for (int p = 0; p < B; p++) nc += ncells[p];
  std::vector<int> bl, vl;
  for (int i = 0; i < c.n_blob; i++)
    if (bfl[i] & F_ALIVE) bl.push_back(i);
  for (int i = 0; i < c.n_vir; i++)
    if (vfl[i] & F_ALIVE) vl.push_back(i);
  std::sort(bl.begin(), bl.end(), [&](int x, int y) { return bseq[x] < bseq[y]; });
  std::sort(vl.begin(), vl.end(), [&](int x, int y) { return vseq[x] < vseq[y]; });
  std::vector<int> pord;
  for (int i = 0; i < n_pel; i++) {
    const int bx = std::min(d.cols - 1, std::max(0, (int)(px[i] / kBucket)));
    const int by = std::min(d.cols - 1, std::max(0, (int)(py[i] / kBucket)));
    if (bx >= d.own_bx0 && bx < d.own_bx1 && by >= d.own_by0 && by < d.own_by1) pord.push_back(i);  // (tiles: owned)
  }
  std::sort(pord.begin(), pord.end(), [&](int x, int y) { return ps[x] < ps[y]; });
  int caps[5] = {st->n_cells, st->n_pellets, st->n_blobs, st->n_viruses, st->n_dead};
  st->n_players = B;
  st->field_size = d.size;
  st->virus_enabled = d.virus_enabled;
  st->rng_mode = AIGAR_RNG_PHILOX;
  st->seq_next = c.seq_next;
  st->tick = c.tick;
  st->max_pellets = d.max_pellets;
  st->max_viruses = d.max_viruses;
  st->philox_key[0] = c.key0;
  st->philox_key[1] = c.key1;
  st->ctr_pellet = c.ctr_pellet;
  st->ctr_virus = c.ctr_virus;
  memset(st->mt_key, 0, sizeof st->mt_key);
  st->mt_pos = 0;
  st->n_cells = nc;
  st->n_pellets = (int)pord.size();
  st->n_blobs = (int)bl.size();
  st->n_viruses = (int)vl.size();
  st->n_dead = c.n_dead;
  if (!st->cells_f) return 0;
  if (caps[0] < nc || caps[1] < (int)pord.size() || caps[2] < (int)bl.size() || caps[3] < (int)vl.size() || caps[4] < c.n_dead)
    return fail("get_state: caller arrays too small");
  for (int p = 0; p < B; p++) {
    st->players_f[2 * p] = cmdx[p];
    st->players_f[2 * p + 1] = cmdy[p];
    int64_t *q = st->players_i + 5 * p;
    q[0] = alive[p]; q[1] = resp[p]; q[2] = split[p]; q[3] = eject[p]; q[4] = ncells[p];
  }
  int k = 0;
  for (int p = 0; p < B; p++)
    for (int j = 0; j < ncells[p]; j++, k++) {
      size_t hi = (size_t)lst[(size_t)j * B + p] * B + p;
      for (int f = 0; f < 9; f++) st->cells_f[9 * k + f] = cf[f][hi];
      int64_t *q = st->cells_i + 4 * k;
      q[0] = p; q[1] = csvc[hi]; q[2] = cseq[hi]; q[3] = (cfl[hi] & F_INHASH) ? 1 : 0;
    }
  for (size_t i = 0; i < pord.size(); i++) {
    int j = pord[i];
    double *f = st->pellets_f + 4 * i;
    f[0] = px[j]; f[1] = py[j]; f[2] = pm[j]; f[3] = pm[j] > 0 ? std::sqrt(pm[j] / 3.141592653589793) : 0.0;
    st->pellets_seq[i] = ps[j];
    if (st->pellets_col) st->pellets_col[i] = pcol[j];
  }
  for (size_t i = 0; i < bl.size(); i++) {
    int j = bl[i];
    for (int f = 0; f < 8; f++) st->blobs_f[8 * i + f] = bf[f][j];
    st->blobs_i[3 * i] = bsvc[j]; st->blobs_i[3 * i + 1] = bseq[j]; st->blobs_i[3 * i + 2] = bej[j];
    if (st->blobs_col) st->blobs_col[i] = bcol[j];
  }
  for (size_t i = 0; i < vl.size(); i++) {
    int j = vl[i];
    for (int f = 0; f < 8; f++) st->viruses_f[8 * i + f] = vf[f][j];
    st->viruses_i[3 * i] = vsvc[j]; st->viruses_i[3 * i + 1] = vseq[j];
    st->viruses_i[3 * i + 2] = (vfl[j] & F_INHASH) ? 1 : 0;
  }
  for (int i = 0; i < c.n_dead; i++) st->dead[i] = dead[i];
  return 0;
}

// counting sort of items by centre bucket (host side, used by load_state)
static void host_grid(int cols, const std::vector<double> &x, const std::vector<double> &y, std::vector<int> &start,
                      std::vector<int> &order, int shift = 0) {
  const int cc = (cols + (1 << shift) - 1) >> shift;
  int H = cc * cc;
  start.assign(H + 1, 0);
  std::vector<int> b(x.size());
  for (size_t i = 0; i < x.size(); i++) {
    auto cb = [&](double v) {
      int q = (int)(v / 20);
      if (v < 0) q = 0;
      return (q < cols ? q : cols - 1) >> shift;
    };
    b[i] = cb(y[i]) * cc + cb(x[i]);
    start[b[i] + 1]++;
  }
  for (int i = 0; i < H; i++) start[i + 1] += start[i];
  std::vector<int> cur(start.begin(), start.end() - 1);
  order.assign(x.size(), 0);
  for (size_t i = 0; i < x.size(); i++) order[cur[b[i]]++] = (int)i;
}

extern "C" int aigar_load_state(aigar_handle *h, int arena, const aigar_state *st) {
  if (!h || !st) return fail("null argument");
  Dev &d = h->d;
  if (arena < 0 || arena >= d.A) return fail("arena %d out of range", arena);
  if (st->n_players != d.B) return fail("load_state: n_players %d != bots_per_arena %d", st->n_players, d.B);
  if (st->field_size != d.size) return fail("load_state: field_size %d != %d", st->field_size, d.size);
  if (!!st->virus_enabled != !!d.virus_enabled) return fail("load_state: virus_enabled mismatch");
  if (st->n_pellets > d.Pcap || st->n_blobs > d.Ecap || st->n_viruses > d.Vcap)
    return fail("load_state: snapshot exceeds capacities (pellets %d/%d blobs %d/%d viruses %d/%d)", st->n_pellets,
                d.Pcap, st->n_blobs, d.Ecap, st->n_viruses, d.Vcap);
  HIPCHK(hipSetDevice(h->cfg.device));
  HIPCHK(hipStreamSynchronize(h->stream));
  const int B = d.B, NP = d.NP;
  const size_t p0 = (size_t)arena * B, GG = (size_t)d.G * d.G;
  std::vector<int> alive(B), resp(B), ncells(B, 0), split(B), eject(B), dead(st->n_dead);
  std::vector<double> cmdx(B), cmdy(B);
  for (int p = 0; p < B; p++) {
    cmdx[p] = st->players_f[2 * p];
    cmdy[p] = st->players_f[2 * p + 1];
    const int64_t *q = st->players_i + 5 * p;
    alive[p] = (int)q[0]; resp[p] = (int)q[1]; split[p] = (int)q[2]; eject[p] = (int)q[3];
  }
  const size_t CB = (size_t)kMaxCells * B;
  std::vector<uint8_t> lst(CB, 0);
  std::vector<double> cf[9];
  for (int f = 0; f < 9; f++) cf[f].assign(CB, 0.0);
  std::vector<int> csvc(CB, 0);
  std::vector<uint32_t> cfl(CB, 0);
  std::vector<int64_t> cseq(CB, 0);
  std::vector<double> gx, gy;
  std::vector<int> gid;
  double rmax_c = 0;
  for (int k = 0; k < st->n_cells; k++) {
    const int64_t *q = st->cells_i + 4 * k;
    int p = (int)q[0];
    if (p < 0 || p >= B) return fail("load_state: cell owner %d out of range", p);
    int j = ncells[p]++;
    if (j >= kMaxCells) return fail("load_state: player %d has more than 16 cells", p);
    lst[(size_t)j * B + p] = (uint8_t)j;  // slot j == list position j
    size_t hi = (size_t)j * B + p;
    for (int f = 0; f < 9; f++) cf[f][hi] = st->cells_f[9 * k + f];
    csvc[hi] = (int)q[1];
    cseq[hi] = q[2];
    cfl[hi] = F_ALIVE | (q[3] ? F_INHASH : 0);
    gx.push_back(cf[0][hi]);
    gy.push_back(cf[1][hi]);
    gid.push_back((int)((size_t)j * NP + p0 + p));
    rmax_c = std::max(rmax_c, cf[3][hi]);
  }
  for (int i = 0; i < st->n_dead; i++) dead[i] = (int)st->dead[i];
  if (h2d(h, d.p_alive + p0, alive) || h2d(h, d.p_respawn + p0, resp) || h2d(h, d.p_ncells + p0, ncells) ||
      h2d(h, d.p_split + p0, split) || h2d(h, d.p_eject + p0, eject) || h2d(h, d.p_cmdx + p0, cmdx) ||
      h2d(h, d.p_cmdy + p0, cmdy) || h2d(h, d.dead + p0, dead))
    return -1;
  double *cfs[9] = {d.c_x, d.c_y, d.c_m, d.c_r, d.c_vx, d.c_vy, d.c_svx, d.c_svy, d.c_mt};
  for (int s = 0; s < kMaxCells; s++) {
    size_t o = (size_t)s * NP + p0, ho = (size_t)s * B;
    HIPCHK(hipMemcpyAsync(d.p_list + o, lst.data() + ho, B, hipMemcpyHostToDevice, h->stream));
    for (int f = 0; f < 9; f++)
      HIPCHK(hipMemcpyAsync(cfs[f] + o, cf[f].data() + ho, 8 * B, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(d.c_svc + o, csvc.data() + ho, 4 * B, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(d.c_flags + o, cfl.data() + ho, 4 * B, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(d.c_seq + o, cseq.data() + ho, 8 * B, hipMemcpyHostToDevice, h->stream));
  }
  // cell grid (for observations before the next tick)
  std::vector<int> start, order;
  host_grid(d.cols, gx, gy, start, order, d.cshift_c);
  std::vector<int> items(order.size());
  for (size_t i = 0; i < order.size(); i++) items[i] = gid[order[i]];
  const size_t H1 = (size_t)d.H + 1;
  HIPCHK(hipMemcpyAsync(d.cstart + arena * H1, start.data(), 4 * start.size(), hipMemcpyHostToDevice, h->stream));
  if (!items.empty())
    HIPCHK(hipMemcpyAsync(d.citems + (size_t)arena * CB, items.data(), 4 * items.size(), hipMemcpyHostToDevice,
                          h->stream));
  // pellets -> P0 sorted by bucket
  // (tiles: only the pellets in the held range)
  std::vector<double> px, py, pm;
  std::vector<int64_t> ps;
  std::vector<int> pc;
  for (int i = 0; i < st->n_pellets; i++) {
    const double x = st->pellets_f[4 * i], y = st->pellets_f[4 * i + 1];
    const int bx = std::min(d.cols - 1, std::max(0, (int)(x / kBucket)));
    const int by = std::min(d.cols - 1, std::max(0, (int)(y / kBucket)));
    if (bx < d.loc_bx0 || bx >= d.loc_bx1 || by < d.loc_by0 || by >= d.loc_by1) continue;
    px.push_back(x);
    py.push_back(y);
    pm.push_back(st->pellets_f[4 * i + 2]);
    ps.push_back(st->pellets_seq[i]);
    pc.push_back(st->pellets_col ? (int)st->pellets_col[i] : -1);
  }
  host_grid(d.cols, px, py, start, order);
  {  // the row store, every row in home 0 (aigar_dev.h)
    const int C = d.cols;
    std::vector<PelRec> sr(d.PS);
    std::vector<int> sc(d.PS, -1), pst(d.PH1, 0);
    for (int r = 0; r < C; r++) {
      const int b0 = start[(size_t)r * C], n = start[(size_t)(r + 1) * C] - b0, base = r * d.PR;
      if (n > d.PR) return fail("load_state: %d pellets in bucket row %d, more than its %d slots", n, r, d.PR);
      for (int bx = 0; bx <= C; bx++) pst[(size_t)r * (C + 1) + bx] = base + (start[(size_t)r * C + bx] - b0);
      for (int k = 0; k < n; k++) {
        const int i = order[b0 + k];
        sr[base + k] = PelRec{px[i], py[i], pm[i], ps[i]};
        sc[base + k] = pc[i];
      }
    }
    const size_t po = (size_t)arena * d.PS;
    if (h2d(h, d.pel + po, sr) || h2d(h, d.pel_col + po, sc) || h2d(h, d.pstart + (size_t)arena * d.PH1, pst))
      return -1;
    HIPCHK(hipStreamSynchronize(h->stream));  // (the host records go out of scope)
  }
  // blobs and viruses in list order; blob grid for completeness, virus grid for observations
  const size_t bo = (size_t)arena * d.Ecap, vo = (size_t)arena * d.Vcap;
  double *bfs[8] = {d.b_x, d.b_y, d.b_m, d.b_r, d.b_vx, d.b_vy, d.b_svx, d.b_svy};
  double *vfs[8] = {d.v_x, d.v_y, d.v_m, d.v_r, d.v_vx, d.v_vy, d.v_svx, d.v_svy};
  for (int f = 0; f < 8; f++) {
    std::vector<double> bv(st->n_blobs), vv(st->n_viruses);
    for (int i = 0; i < st->n_blobs; i++) bv[i] = st->blobs_f[8 * i + f];
    for (int i = 0; i < st->n_viruses; i++) vv[i] = st->viruses_f[8 * i + f];
    if (h2d(h, bfs[f] + bo, bv) || h2d(h, vfs[f] + vo, vv)) return -1;
  }
  std::vector<int> bsvc(st->n_blobs), vsvc(st->n_viruses), bcol(st->n_blobs);
  std::vector<int64_t> bseq(st->n_blobs), bej(st->n_blobs), vseq(st->n_viruses);
  std::vector<uint32_t> bfl(d.Ecap, 0), vfl(d.Vcap, 0);
  std::vector<double> vgx, vgy;
  double rmax_v = 0;
  for (int i = 0; i < st->n_blobs; i++) {
    bsvc[i] = (int)st->blobs_i[3 * i]; bseq[i] = st->blobs_i[3 * i + 1]; bej[i] = st->blobs_i[3 * i + 2];
    bcol[i] = st->blobs_col ? (int)st->blobs_col[i] : -1;
    bfl[i] = F_ALIVE;
  }
  std::vector<int> vg_ids;
  for (int i = 0; i < st->n_viruses; i++) {
    vsvc[i] = (int)st->viruses_i[3 * i]; vseq[i] = st->viruses_i[3 * i + 1];
    vfl[i] = F_ALIVE | (st->viruses_i[3 * i + 2] ? F_INHASH : 0);
    vgx.push_back(st->viruses_f[8 * i]);
    vgy.push_back(st->viruses_f[8 * i + 1]);
    rmax_v = std::max(rmax_v, st->viruses_f[8 * i + 3]);
  }
  if (h2d(h, d.b_svc + bo, bsvc) || h2d(h, d.b_seq + bo, bseq) || h2d(h, d.b_ej + bo, bej) || h2d(h, d.b_col + bo, bcol) ||
      h2d(h, d.b_flags + bo, bfl) || h2d(h, d.v_svc + vo, vsvc) || h2d(h, d.v_seq + vo, vseq) ||
      h2d(h, d.v_flags + vo, vfl))
    return -1;
  host_grid(d.cols, vgx, vgy, start, order, d.cshift);
  HIPCHK(hipMemcpyAsync(d.vstart + arena * H1, start.data(), 4 * start.size(), hipMemcpyHostToDevice, h->stream));
  if (!order.empty()) HIPCHK(hipMemcpyAsync(d.vitems + vo, order.data(), 4 * order.size(), hipMemcpyHostToDevice, h->stream));
  // control block
  ArenaCtl c;
  memset(&c, 0, sizeof c);
  c.seq_next = st->seq_next;
  c.tick = st->tick;
  c.key0 = st->philox_key[0];
  c.key1 = st->philox_key[1];
  c.ctr_pellet = st->ctr_pellet;
  c.ctr_virus = st->ctr_virus;
  c.n_pel = (int)px.size();
  c.n_pel_glob = st->n_pellets;
  c.n_blob = st->n_blobs;
  c.n_vir = st->n_viruses;
  c.n_dead = st->n_dead;
  c.rmax_cell = std::max(rmax_c, std::sqrt(10.0 / 3.141592653589793));
  c.rmax_virus = std::max(rmax_v, std::sqrt(100.0 / 3.141592653589793));
  c.food_round = 1;  // reservation epochs restart: clear this arena's keys
  HIPCHK(hipMemsetAsync(d.pel_owner + (size_t)arena * d.PD, 0, 8 * (size_t)d.PD, h->stream));
  HIPCHK(hipMemsetAsync(d.b_owner + (size_t)arena * d.Ecap, 0, 8 * (size_t)d.Ecap, h->stream));
  // look-back epochs restart too: clear this arena's tile states
  HIPCHK(hipMemsetAsync(d.pl_state + (size_t)arena * d.pl_tiles, 0, 8 * (size_t)d.pl_tiles, h->stream));
  HIPCHK(hipMemsetAsync(d.pel_dead + (size_t)arena * d.PD, 0, (size_t)d.PD, h->stream));
  HIPCHK(hipMemsetAsync(d.cgcnt + (size_t)arena * 2 * 4100, 0, sizeof(int) * 2 * 4100, h->stream));
  for (int sl = 0; sl < 2; sl++)
    HIPCHK(hipMemsetAsync(d.scan_state + ((size_t)sl * d.A + arena) * d.scan_tiles, 0, 8 * (size_t)d.scan_tiles,
                          h->stream));
  HIPCHK(hipMemcpyAsync(d.ctl + arena, &c, sizeof c, hipMemcpyHostToDevice, h->stream));
  // bot-side observation history restarts (NN bot reset, bot.py:151-158)
  HIPCHK(hipMemsetAsync(d.o_lastfov + p0, 0, 8 * B, h->stream));
  HIPCHK(hipMemsetAsync(d.o_act_cur + p0 * 4, 0, 8 * 4 * (size_t)B, h->stream));  // currentAction reset
  hipLaunchKernelGGL(k_fill_d, dim3((B + 255) / 256), dim3(256), 0, h->stream, d.o_last_mass + p0, (size_t)B,
                     __builtin_nan(""));
  for (double *p : {d.o_self_lf, d.o_self_slf, d.o_en_lf, d.o_en_slf})
    HIPCHK(hipMemsetAsync(p + p0 * GG, 0, 8 * B * GG, h->stream));
  if (d.tiled) {
    HIPCHK(hipMemsetAsync(d.t_holder, 0xFF, sizeof(int) * d.NP, h->stream));
    HIPCHK(hipMemsetAsync(d.t_obsby, 0xFF, sizeof(int) * d.NP, h->stream));
    HIPCHK(hipMemsetAsync(d.t_hodefer, 0, d.NP, h->stream));
  }
  launch_player_fov(d, h->stream);  // FOV cache of the loaded players
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

extern "C" int aigar_policy_greedy(aigar_handle *h, int greedy_split, const uint8_t *mask, int on_device) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  const uint8_t *m = mask;
  if (mask && !on_device) {
    HIPCHK(hipMemcpyAsync(h->d_mask, mask, (size_t)h->d.NP, hipMemcpyHostToDevice, h->stream));
    m = h->d_mask;
  }
  note_greedy(h);  // (food_rounds)
  {
    Mark mk(h, "policy");
    launch_policy_greedy(h->d, h->stream, greedy_split ? 1 : 0, m, -1);
  }
  HIPCHK(hipGetLastError());
  if (mask && !on_device) HIPCHK(hipStreamSynchronize(h->stream));  // (host mask buffer reused next call)
  return 0;
}

extern "C" int aigar_set_split_likelihood(aigar_handle *h, int arena, const int32_t *lh) {
  if (!h) return fail("null handle");
  if (arena < 0 || arena >= h->d.A) return fail("arena out of range");
  HIPCHK(hipSetDevice(h->cfg.device));
  int *dst = h->d.p_split_lh + (size_t)arena * h->d.B;
  if (!lh) {
    HIPCHK(hipMemsetAsync(dst, 0, sizeof(int) * h->d.B, h->stream));
  } else {
    HIPCHK(hipMemcpyAsync(dst, lh, sizeof(int) * h->d.B, hipMemcpyHostToDevice, h->stream));
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

extern "C" int aigar_apply_actions(aigar_handle *h, const double *act, int n_act, int enable_split, int skipping,
                                   int record, int on_device) {
  if (!h || !act) return fail("null argument");
  if (n_act < 2 || n_act > 4) return fail("apply_actions: n_act must be 2, 3 or 4");
  HIPCHK(hipSetDevice(h->cfg.device));
  const double *src = act;
  if (!on_device) {
    HIPCHK(hipMemcpyAsync(h->d_cmd, act, sizeof(double) * n_act * h->d.NP, hipMemcpyHostToDevice, h->stream));
    src = h->d_cmd;
  }
  launch_apply_actions(h->d, h->stream, src, n_act, enable_split, skipping, record);
  HIPCHK(hipGetLastError());
  if (!on_device) HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

extern "C" int aigar_rewards(aigar_handle *h, double *out, const aigar_reward_params *p, int update_last,
                             int on_device) {
  if (!h || !out || !p) return fail("null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  double *dst = on_device ? out : h->d_stats;
  launch_rewards(h->d, h->stream, dst, *p, update_last, 0);
  HIPCHK(hipGetLastError());
  if (!on_device) {
    HIPCHK(hipMemcpyAsync(out, h->d_stats, sizeof(double) * h->d.NP, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  return 0;
}

extern "C" int aigar_counters(aigar_handle *h, int arena, int64_t *out, int n) {
  if (!h) return fail("null handle");
  if (arena < 0 || arena >= h->d.A) return fail("arena out of range");
  if (!out || n < 0 || n > 8) return fail("counters: need 0 <= n <= 8 and an output array");
  HIPCHK(hipSetDevice(h->cfg.device));
  ArenaCtl c;
  HIPCHK(hipMemcpyAsync(&c, h->d.ctl + arena, sizeof c, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  for (int k = 0; k < n; k++) out[k] = c.stat[k];
  return 0;
}

extern "C" int aigar_get_events(aigar_handle *h, int arena, int64_t *out, int cap, int *n) {
  if (!h || !n) return fail("null argument");
  Dev &d = h->d;
  if (arena < 0 || arena >= d.A) return fail("arena %d out of range", arena);
  HIPCHK(hipSetDevice(h->cfg.device));
  if (check_device_errors(h)) return -1;
  ArenaCtl c;
  HIPCHK(hipMemcpy(&c, d.ctl + arena, sizeof c, hipMemcpyDeviceToHost));
  int ne = std::min(c.n_ev, d.EVcap);
  *n = ne;
  if (!out) return 0;
  if (cap < ne) return fail("get_events: cap %d < %d events", cap, ne);
  std::vector<int64_t> ev((size_t)ne * 5);
  if (ne) HIPCHK(hipMemcpy(ev.data(), d.ev + (size_t)arena * d.EVcap * 5, ev.size() * 8, hipMemcpyDeviceToHost));
  std::vector<int> ord(ne);
  for (int i = 0; i < ne; i++) ord[i] = i;
  std::sort(ord.begin(), ord.end(), [&](int x, int y) {
    if (ev[5 * x] != ev[5 * y]) return ev[5 * x] < ev[5 * y];
    return (uint64_t)ev[5 * x + 1] < (uint64_t)ev[5 * y + 1];
  });
  for (int i = 0; i < ne; i++) {
    const int64_t *e = &ev[5 * (size_t)ord[i]];
    out[4 * i] = e[0] >> 8;
    out[4 * i + 1] = e[2];
    out[4 * i + 2] = e[3];
    out[4 * i + 3] = e[4];
  }
  return 0;
}

// the raw event rows (sort keys kept) -- tiles merge their logs by key
extern "C" int aigar_get_events_raw(aigar_handle *h, int arena, int64_t *out, int cap, int *n) {
  if (!h || !n) return fail("null argument");
  Dev &d = h->d;
  if (arena < 0 || arena >= d.A) return fail("arena %d out of range", arena);
  HIPCHK(hipSetDevice(h->cfg.device));
  if (check_device_errors(h)) return -1;
  ArenaCtl c;
  HIPCHK(hipMemcpy(&c, d.ctl + arena, sizeof c, hipMemcpyDeviceToHost));
  const int ne = std::min(c.n_ev, d.EVcap);
  *n = ne;
  if (!out) return 0;
  if (cap < ne) return fail("get_events_raw: cap %d < %d events", cap, ne);
  if (ne) HIPCHK(hipMemcpy(out, d.ev + (size_t)arena * d.EVcap * 5, (size_t)ne * 5 * 8, hipMemcpyDeviceToHost));
  return 0;
}

__global__ void k_selftest_pow(const double *x, const double *y, double *out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = aigar_math::pow_glibc(x[i], y[i]);
}

extern "C" int aigar_selftest_pow(const double *x, const double *y, double *out, int n) {
  if (!x || !y || !out || n < 0) return fail("null argument");
  double *dx = nullptr, *dy = nullptr, *dz = nullptr;
  size_t b = sizeof(double) * (size_t)(n > 0 ? n : 1);
  HIPCHK(hipMalloc(&dx, b));
  HIPCHK(hipMalloc(&dy, b));
  HIPCHK(hipMalloc(&dz, b));
  HIPCHK(hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dy, y, sizeof(double) * n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_selftest_pow, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dy, dz, n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dz, sizeof(double) * n, hipMemcpyDeviceToHost));
  (void)hipFree(dx);
  (void)hipFree(dy);
  (void)hipFree(dz);
  return 0;
}

// out[0, n): atan2(y, x); out[n, 2n): sin(x); out[2n, 3n): cos(x) -- the stepper's trig
// entry points (aigar_glibc_trig.h), one thread per element
__global__ void k_selftest_trig(const double *y, const double *x, double *out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = aigar_math::trig_atan2(y[i], x[i]);
  double s, c;
  aigar_math::trig_sincos(x[i], s, c);
  out[n + i] = s;
  out[2 * (size_t)n + i] = c;
}

extern "C" int aigar_selftest_trig(const double *y, const double *x, double *out, int n) {
  if (!x || !y || !out || n < 0) return fail("null argument");
  double *dx = nullptr, *dy = nullptr, *dz = nullptr;
  const size_t b = sizeof(double) * (size_t)(n > 0 ? n : 1);
  HIPCHK(hipMalloc(&dx, b));
  HIPCHK(hipMalloc(&dy, b));
  HIPCHK(hipMalloc(&dz, 3 * b));
  HIPCHK(hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dy, y, sizeof(double) * n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_selftest_trig, dim3((n + 255) / 256), dim3(256), 0, 0, dy, dx, dz, n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dz, 3 * sizeof(double) * n, hipMemcpyDeviceToHost));
  (void)hipFree(dx);
  (void)hipFree(dy);
  (void)hipFree(dz);
  return 0;
}
