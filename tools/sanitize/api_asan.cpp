// Host-side sanitizer run of libaigar_hip: the library's host
// code (api.hip: argument checks, snapshot marshalling, event sorting, tile
// plumbing, graph capture) built with -Xarch_host -fsanitize=address,undefined
// (device code is not instrumented: GPU ASan is not available on this pool)
// and driven through the C-ABI: create / reset / steps / run (graph) /
// observe / pixels / env calls / snapshot round trip / events / tiles (2x1,
// in-process exchange) / the documented error paths, then destroy.
// Build + run on the GPU box: bash tools/sanitize/api_asan.sh
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/aigar.h"

#define CHK(x)                                                                  \
  do {                                                                          \
    if ((x) < 0) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, aigar_last_error()); \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)
#define MUST_FAIL(x)                                                            \
  do {                                                                          \
    if ((x) >= 0) {                                                             \
      fprintf(stderr, "%s:%d %s should have failed\n", __FILE__, __LINE__, #x); \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)

static aigar_config cfg(int arenas, int bots, int field, double pellets, int virus) {
  aigar_config c;
  memset(&c, 0, sizeof c);
  c.n_arenas = arenas;
  c.bots_per_arena = bots;
  c.field_size = field;
  c.virus_enabled = virus;
  c.max_pellets = pellets;
  c.max_viruses = virus ? -1.0 : 0.0;
  c.grid_squares = 11;
  c.obs_channels = 0x3FF & ~AIGAR_OBS_ALL;  /* (ALL_PLAYER_GRID excludes the last-frame grids) */
  c.obs_extras = AIGAR_EX_LAST_FOV | AIGAR_EX_FOV | AIGAR_EX_MASS | AIGAR_EX_LAST_ACT | AIGAR_EX_2LAST_ACT;
  c.rng_mode = AIGAR_RNG_PHILOX;
  c.flags = 1;  // events
  return c;
}

struct Snap {
  aigar_state st;
  std::vector<double> pf, cf, pelf, bf, vf;
  std::vector<int64_t> pi, ci, ps, pc, bi, bc, vi, dead;
};
static void get_snap(aigar_handle *h, int arena, Snap &s) {
  memset(&s.st, 0, sizeof s.st);
  CHK(aigar_get_state(h, arena, &s.st));
  aigar_state &t = s.st;
  s.pf.assign((size_t)t.n_players * 2 + 1, 0); s.pi.assign((size_t)t.n_players * 5 + 1, 0);
  s.cf.assign((size_t)t.n_cells * 9 + 1, 0); s.ci.assign((size_t)t.n_cells * 4 + 1, 0);
  s.pelf.assign((size_t)t.n_pellets * 4 + 1, 0); s.ps.assign((size_t)t.n_pellets + 1, 0);
  s.pc.assign((size_t)t.n_pellets + 1, 0);
  s.bf.assign((size_t)t.n_blobs * 8 + 1, 0); s.bi.assign((size_t)t.n_blobs * 3 + 1, 0);
  s.bc.assign((size_t)t.n_blobs + 1, 0);
  s.vf.assign((size_t)t.n_viruses * 8 + 1, 0); s.vi.assign((size_t)t.n_viruses * 3 + 1, 0);
  s.dead.assign((size_t)t.n_dead + 1, 0);
  t.players_f = s.pf.data(); t.players_i = s.pi.data(); t.cells_f = s.cf.data(); t.cells_i = s.ci.data();
  t.pellets_f = s.pelf.data(); t.pellets_seq = s.ps.data(); t.pellets_col = s.pc.data();
  t.blobs_f = s.bf.data(); t.blobs_i = s.bi.data(); t.blobs_col = s.bc.data();
  t.viruses_f = s.vf.data(); t.viruses_i = s.vi.data(); t.dead = s.dead.data();
  CHK(aigar_get_state(h, arena, &t));
}

static void exercise(int arenas, int bots, int field, double pellets, int virus, int ticks) {
  aigar_config c = cfg(arenas, bots, field, pellets, virus);
  aigar_handle *h = nullptr;
  CHK(aigar_create(&c, &h));
  CHK(aigar_reset(h, 11));
  const int n = arenas * bots, L = aigar_obs_len(h);
  std::vector<double> obs((size_t)n * L), cmd((size_t)n * 4), act((size_t)n * 4), stats((size_t)n * 5), rw(n);
  std::vector<uint8_t> pix((size_t)n * 42 * 42 * 3), mask(n, 1), roles(n);
  for (int i = 0; i < n; i++) roles[i] = (uint8_t)(i % 3);
  aigar_run_params rp;
  memset(&rp, 0, sizeof rp);
  rp.policy = AIGAR_POLICY_RANDOM;
  rp.greedy_split = 1;
  rp.p_split = 0.02;
  rp.p_eject = 0.05;
  rp.seed = 5;
  for (int t = 0; t < ticks; t++) {
    if (t % 4 == 0) {
      CHK(aigar_policy_random(h, 0.02, 0.05, t));
    } else if (t % 4 == 1) {
      CHK(aigar_policy_greedy(h, 1, nullptr, 0));
    } else {
      for (int i = 0; i < n; i++) {
        cmd[4 * i] = (i * 37 + t * 11) % field;
        cmd[4 * i + 1] = (i * 53 + t * 7) % field;
        cmd[4 * i + 2] = (i + t) % 17 == 0;
        cmd[4 * i + 3] = (i + t) % 5 == 0;
      }
      CHK(aigar_set_commands(h, cmd.data(), 0));
    }
    CHK(aigar_step(h, 1));
    int ne = 0;
    for (int a = 0; a < arenas; a++) {
      CHK(aigar_get_events(h, a, nullptr, 0, &ne));
      std::vector<int64_t> ev((size_t)ne * 4 + 4);
      CHK(aigar_get_events(h, a, ev.data(), ne, &ne));
    }
    if (t % 5 == 0) CHK(aigar_observe(h, obs.data(), 0, 0));
    if (t % 7 == 0) CHK(aigar_observe_pixels(h, pix.data(), 42, 3, 2, 0));
    if (t % 9 == 0) {
      CHK(aigar_player_stats(h, stats.data(), 0));
      for (int a = 0; a < arenas; a++) {
        Snap s;
        get_snap(h, a, s);
        CHK(aigar_load_state(h, a, &s.st));
      }
    }
  }
  // the graph path and the env / learner glue
  CHK(aigar_run(h, 3, &rp, nullptr, 0));
  CHK(aigar_set_roles(h, roles.data(), 0));
  for (int i = 0; i < n * 4; i++) act[i] = (i % 7) / 7.0;
  CHK(aigar_set_actions(h, act.data(), act.data(), 0));
  CHK(aigar_observe_masked(h, obs.data(), 0, 0, mask.data(), 0));
  aigar_reward_params rwp;
  memset(&rwp, 0, sizeof rwp);
  rwp.death_factor = 1.5;
  rwp.reward_scale = 2.0;
  CHK(aigar_rewards(h, rw.data(), &rwp, 1, 0));
  std::vector<int64_t> ctr(8);
  CHK(aigar_counters(h, 0, ctr.data(), 8));
  // documented error paths: bad arguments fail cleanly
  MUST_FAIL(aigar_get_state(h, arenas, nullptr));
  MUST_FAIL(aigar_observe_pixels(h, pix.data(), 0, 0, 2, 0));
  MUST_FAIL(aigar_step(nullptr, 1));
  CHK(aigar_destroy(h));
}

static void tiles() {
  aigar_config c = cfg(1, 64, 600, 3000, 1);
  aigar_handle *hs[2] = {nullptr, nullptr};
  for (int k = 0; k < 2; k++) {
    aigar_config ck = c;
    ck.tile_x = 2;
    ck.tile_y = 1;
    ck.tile_id = k;
    CHK(aigar_create(&ck, &hs[k]));
    CHK(aigar_reset(hs[k], 3));
  }
  aigar_run_params rp;
  memset(&rp, 0, sizeof rp);
  rp.policy = AIGAR_POLICY_RANDOM;
  rp.p_split = 0.05;
  rp.p_eject = 0.05;
  for (int t = 0; t < 20; t++) {
    for (auto *h : hs) CHK(aigar_tile_begin(h, &rp));
    int u = 0;
    for (int pass = 0;; pass++) {
      CHK(aigar_tile_exchange_local(hs, 2));
      for (auto *h : hs) CHK(aigar_tile_apply(h, &u));
      if (u == 0 || pass > 32) break;
      for (auto *h : hs) CHK(aigar_tile_resume(h));
    }
    for (auto *h : hs) CHK(aigar_tile_end(h, nullptr, 0));
  }
  for (auto *h : hs) {
    Snap s;
    get_snap(h, 0, s);
    CHK(aigar_destroy(h));
  }
}

int main() {
  aigar_config bad = cfg(0, 4, 100, 10, 0);
  aigar_handle *h = nullptr;
  MUST_FAIL(aigar_create(&bad, &h));
  MUST_FAIL(aigar_create(nullptr, &h));
  exercise(1, 1, 1000, 100, 0, 30);     // C1
  exercise(1, 48, 200, 800, 1, 60);     // crowded, viruses
  exercise(4, 24, 300, 1000, 0, 40);    // batched arenas
  exercise(1, 512, 1697, 43200, 0, 10); // a C5 arena
  tiles();
  printf("host sanitizer run: clean\n");
  return 0;
}
