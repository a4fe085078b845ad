/* CPU sanitizer run of the oracle ("race detection / sanitizers"):
 * built with -fsanitize=address,undefined -fno-sanitize-recover=all together
 * with oracle/oracle.c, it drives every entry point the tests use -- reset,
 * commands / actions, steps, the Greedy policy, observations (every channel and
 * extra), pixel frames, events, player stats, snapshot round trips, MT stream
 * positioning -- over several configurations (crowded, viruses, several
 * arenas, a one-bot field) and exits 0 when the sanitizers found nothing.
 * tests/test_sanitize.py builds and runs it. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/aigar.h"

void *oracle_create(const aigar_config *cfg);
void oracle_destroy(void *h);
int oracle_reset(void *h, uint64_t seed);
int oracle_set_commands(void *h, const double *cmd);
int oracle_set_actions(void *h, const double *cur, const double *prev);
int oracle_step(void *h, int n);
int oracle_obs_len(void *h);
int oracle_observe(void *h, double *out);
int oracle_observe_one(void *h, int arena, int p, double *out);
int oracle_player_stats(void *h, double *out);
int oracle_get_events(void *h, int arena, int64_t *out, int cap);
int oracle_reset_obs_state(void *h);
int oracle_get_state(void *h, int arena, aigar_state *st);
int oracle_load_state(void *h, int arena, const aigar_state *st);
int oracle_policy_greedy(void *h, int greedy_split);
int oracle_pixels(void *h, int L, uint64_t seed, uint8_t *out);
const char *oracle_last_error(void);

static uint64_t rng = 88172645463325252ull;
static double urand(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (double)(rng >> 11) * 0x1p-53;
}

#define CHK(x)                                                                 \
  do {                                                                         \
    if ((x) < 0) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, oracle_last_error()); \
      exit(2);                                                                 \
    }                                                                          \
  } while (0)

/* get_state into freshly sized arrays (the counts query first), then load it back */
static void round_trip(void *h, int arena) {
  aigar_state st;
  memset(&st, 0, sizeof st);
  CHK(oracle_get_state(h, arena, &st));
  aigar_state s2 = st;
  s2.players_f = calloc((size_t)st.n_players * 2 + 1, 8);
  s2.players_i = calloc((size_t)st.n_players * 5 + 1, 8);
  s2.cells_f = calloc((size_t)st.n_cells * 9 + 1, 8);
  s2.cells_i = calloc((size_t)st.n_cells * 4 + 1, 8);
  s2.pellets_f = calloc((size_t)st.n_pellets * 4 + 1, 8);
  s2.pellets_seq = calloc((size_t)st.n_pellets + 1, 8);
  s2.pellets_col = calloc((size_t)st.n_pellets + 1, 8);
  s2.blobs_f = calloc((size_t)st.n_blobs * 8 + 1, 8);
  s2.blobs_i = calloc((size_t)st.n_blobs * 3 + 1, 8);
  s2.blobs_col = calloc((size_t)st.n_blobs + 1, 8);
  s2.viruses_f = calloc((size_t)st.n_viruses * 8 + 1, 8);
  s2.viruses_i = calloc((size_t)st.n_viruses * 3 + 1, 8);
  s2.dead = calloc((size_t)st.n_dead + 1, 8);
  CHK(oracle_get_state(h, arena, &s2));
  CHK(oracle_load_state(h, arena, &s2));
  void *ps[] = {s2.players_f, s2.players_i, s2.cells_f, s2.cells_i, s2.pellets_f, s2.pellets_seq, s2.pellets_col,
                s2.blobs_f, s2.blobs_i, s2.blobs_col, s2.viruses_f, s2.viruses_i, s2.dead};
  for (size_t i = 0; i < sizeof ps / sizeof ps[0]; i++) free(ps[i]);
}

static void run(int arenas, int bots, int field, double pellets, int virus, double viruses, int ticks, int rng_mode,
                double ps, double pe) {
  aigar_config c;
  memset(&c, 0, sizeof c);
  c.n_arenas = arenas;
  c.bots_per_arena = bots;
  c.field_size = field;
  c.virus_enabled = virus;
  c.max_pellets = pellets;
  c.max_viruses = viruses;
  c.grid_squares = 11;
  c.obs_channels = 0x3FF & ~AIGAR_OBS_ALL;  /* (ALL_PLAYER_GRID excludes the last-frame grids) */
  c.obs_extras = AIGAR_EX_LAST_FOV | AIGAR_EX_FOV | AIGAR_EX_MASS | AIGAR_EX_LAST_ACT | AIGAR_EX_2LAST_ACT;
  c.rng_mode = rng_mode;
  c.flags = 1;
  void *h = oracle_create(&c);
  if (!h) {
    fprintf(stderr, "create: %s\n", oracle_last_error());
    exit(2);
  }
  CHK(oracle_reset(h, 7));
  const int n = arenas * bots, L = oracle_obs_len(h);
  double *cmd = malloc(sizeof(double) * 4 * n), *act = malloc(sizeof(double) * 4 * n);
  double *obs = malloc(sizeof(double) * (size_t)L * n), *stats = malloc(sizeof(double) * 5 * n);
  uint8_t *pix = malloc((size_t)n * 42 * 42 * 3);
  int64_t *ev = malloc(sizeof(int64_t) * 4 * 100000);
  for (int t = 0; t < ticks; t++) {
    if (t % 3 == 0) {
      CHK(oracle_policy_greedy(h, 1));
    } else {
      for (int i = 0; i < n; i++) {
        cmd[4 * i] = urand() * field;
        cmd[4 * i + 1] = urand() * field;
        cmd[4 * i + 2] = urand() < ps;
        cmd[4 * i + 3] = urand() < pe;
        for (int k = 0; k < 4; k++) act[4 * i + k] = urand();
      }
      CHK(oracle_set_commands(h, cmd));
      CHK(oracle_set_actions(h, act, act));
    }
    CHK(oracle_step(h, 1));
    for (int a = 0; a < arenas; a++) CHK(oracle_get_events(h, a, ev, 100000));
    if (t % 4 == 0) CHK(oracle_observe(h, obs));
    if (t % 9 == 0) CHK(oracle_pixels(h, 42, 3, pix));
    if (t % 11 == 0) {
      CHK(oracle_observe_one(h, 0, 0, obs));
      CHK(oracle_player_stats(h, stats));
      for (int a = 0; a < arenas; a++) round_trip(h, a);
    }
  }
  CHK(oracle_reset_obs_state(h));
  free(cmd);
  free(act);
  free(obs);
  free(stats);
  free(pix);
  free(ev);
  oracle_destroy(h);
}

int main(void) {
  run(1, 1, 1000, 100, 0, 0, 60, AIGAR_RNG_MT19937, 0.0, 0.0);       /* C1: the reference's own CPU case */
  run(1, 48, 150, 600, 0, 0, 120, AIGAR_RNG_PHILOX, 0.05, 0.05);     /* crowded: splits, ejections, deaths */
  run(1, 32, 400, 2000, 1, 30, 150, AIGAR_RNG_PHILOX, 0.05, 0.1);    /* viruses: feeding, explosions */
  run(3, 16, 300, 800, 1, 10, 80, AIGAR_RNG_MT19937, 0.02, 0.05);    /* several arenas, MT stream */
  printf("oracle sanitizer run: clean\n");
  return 0;
}
