/*
 * oracle.c -- CPU restatement of the reference agar.io tick and grid
 * observation.  TEST INFRASTRUCTURE ONLY: used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg as the checker /
 * CPU baseline.  The product (aigar_amd/, libaigar_hip.so) never links it.
 *
 * Parity pinned against golden vectors produced by running the reference
 * itself (tools/golden/gen_golden.py, fixtures under tests/golden) in AIGAR_RNG_MT19937
 * mode; AIGAR_RNG_PHILOX mode is the same code with the counter-based draws the
 * GPU uses (keyed by site), so GPU == oracle(philox) is checked bit-exactly on
 * events.
 *
 * Structure follows the reference file by file: fp64 everywhere, Python list
 * semantics (live-list iteration, list.remove, stable sort), real bucket-list
 * spatial hashes with insert/delete (spatialHashTable.py), creation-sequence
 * ordered candidate sets (the canonical-order shim), numpy's
 * pairwise sum (player.py:129,158-159) and Python's round(x, 3) (bot.py:450).
 * Build: -O2 -ffp-contract=off (no FMA contraction; IEEE per operation).
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/aigar.h"

#define PI M_PI /* numpy.pi */

/* ---------------------------------------------------------- parameters.py */
static const double FPS = 30, GAME_SPEED = 1;
#define SPEED_MODIFIER (GAME_SPEED / FPS)
static const int HASH_BUCKET_SIZE = 20;
static const double START_MASS = 10;
#define START_RADIUS sqrt(START_MASS / PI)
static const double VIRUS_BASE_SIZE = 100;
static const double VIRUS_EAT_FACTOR = 0.5;
#define VIRUS_BASE_RADIUS sqrt(VIRUS_BASE_SIZE / PI)
static const double VIRUS_EXPLOSION_CELL_MASS_PROPORTION = 0.6;
static const double EJECTEDBLOB_BASE_MASS = 18;
static const double MAX_MASS_SINGLE_CELL = 22500;
static const double BASE_MERGE_TIME = 25;
static const double MERGE_TIME_MASS_FACTOR = 0.0233;
static const double MERGE_TIME_VIRUS_FACTOR = 0.85;
#define CELL_MOVE_SPEED (90 * SPEED_MODIFIER)
#define CELL_MASS_DECAY_RATE (1 - (0.01 * SPEED_MODIFIER))

/* philox streams (shared definition with aigar_amd/csrc/aigar_rng.h) */
enum { ST_PELLET = 1, ST_VIRUS = 2, ST_PLAYER = 3, ST_ANGLE = 4, ST_INIT_PLAYER = 5, ST_POLICY = 6, ST_GREEDY = 7,
       ST_GREEDY_LH = 8 };

/* ------------------------------------------------------------ errors ---- */
static __thread char g_err[512];
static void set_err(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}
const char *oracle_last_error(void) { return g_err; }

/* ------------------------------------------------ python number helpers */
/* builtin max(a, b): keeps a unless b > a; min(a, b): keeps a unless b < a */
static inline double py_max(double a, double b) { return (b > a) ? b : a; }
static inline double py_min(double a, double b) { return (b < a) ? b : a; }
/* float % positive float (Python float_rem for non-negative operands) */
static inline double py_mod(double a, double b) {
  double m = fmod(a, b);
  if (m != 0.0) {
    if ((b < 0) != (m < 0)) m += b;
  } else {
    m = copysign(0.0, b);
  }
  return m;
}

/* numpy pairwise summation for n <= 128 (numpy/_core/src/umath/loops_utils.h) */
double oracle_np_sum(const double *a, int n) {
  if (n < 8) {
    double r = 0.;
    for (int i = 0; i < n; i++) r += a[i];
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; j++) r[j] = a[j];
  int i;
  for (i = 8; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; j++) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += a[i];
  return res;
}

/* Python round(x, 3): correctly rounded decimal, half-even on exact ties */
double oracle_py_round3(double v) {
  char buf[64];
  snprintf(buf, sizeof buf, "%.3f", v);
  return strtod(buf, NULL);
}
/* Python round(v, 5) (bot.py:16-21 getRelativeCellPos) */
double oracle_py_round5(double v) {
  char buf[64];
  snprintf(buf, sizeof buf, "%.5f", v);
  return strtod(buf, NULL);
}

/* --------------------------------------------------- numpy MT19937 ---- */
typedef struct { uint32_t key[624]; int pos; } MT;

static void mt_gen(MT *s) {
  const uint32_t UP = 0x80000000u, LO = 0x7fffffffu, A = 0x9908b0dfu;
  int i;
  uint32_t y;
  for (i = 0; i < 624 - 397; i++) {
    y = (s->key[i] & UP) | (s->key[i + 1] & LO);
    s->key[i] = s->key[i + 397] ^ (y >> 1) ^ ((uint32_t)(-(int32_t)(y & 1)) & A);
  }
  for (; i < 623; i++) {
    y = (s->key[i] & UP) | (s->key[i + 1] & LO);
    s->key[i] = s->key[i + (397 - 624)] ^ (y >> 1) ^ ((uint32_t)(-(int32_t)(y & 1)) & A);
  }
  y = (s->key[623] & UP) | (s->key[0] & LO);
  s->key[623] = s->key[396] ^ (y >> 1) ^ ((uint32_t)(-(int32_t)(y & 1)) & A);
  s->pos = 0;
}
static uint32_t mt_next32(MT *s) {
  if (s->pos == 624) mt_gen(s);
  uint32_t y = s->key[s->pos++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
static void mt_seed(MT *s, uint32_t seed) { /* init_genrand (numpy.random.seed(int)) */
  s->key[0] = seed;
  for (int i = 1; i < 624; i++)
    s->key[i] = 1812433253u * (s->key[i - 1] ^ (s->key[i - 1] >> 30)) + (uint32_t)i;
  s->pos = 624;
}
/* RandomState.randint(low, high): int() truncation of float bounds, then masked
 * rejection on raw 32-bit words (numpy/random/_bounded_integers.pyx) */
static int64_t mt_randint(MT *s, double lo, double hi) {
  int64_t l = (int64_t)lo, h = (int64_t)hi - 1;
  uint64_t rng = (uint64_t)(h - l);
  if (h < l) return l; /* numpy raises ValueError; never reached by the tick */
  if (rng == 0) return l;
  uint32_t mask = (uint32_t)rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
  if (rng == 0xffffffffu) return l + (int64_t)mt_next32(s);
  uint32_t v;
  while ((v = (mt_next32(s) & mask)) > (uint32_t)rng) {
  }
  return l + (int64_t)v;
}
static double mt_random(MT *s) {
  int32_t a = (int32_t)(mt_next32(s) >> 5), b = (int32_t)(mt_next32(s) >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}
void oracle_mt_seed(uint32_t seed, uint32_t *key, int *pos) {
  MT m;
  mt_seed(&m, seed);
  memcpy(key, m.key, sizeof m.key);
  *pos = m.pos;
}
int64_t oracle_mt_randint(uint32_t *key, int *pos, double lo, double hi) {
  MT m;
  memcpy(m.key, key, sizeof m.key);
  m.pos = *pos;
  int64_t r = mt_randint(&m, lo, hi);
  memcpy(key, m.key, sizeof m.key);
  *pos = m.pos;
  return r;
}
double oracle_mt_random(uint32_t *key, int *pos) {
  MT m;
  memcpy(m.key, key, sizeof m.key);
  m.pos = *pos;
  double r = mt_random(&m);
  memcpy(key, m.key, sizeof m.key);
  *pos = m.pos;
  return r;
}

/* ------------------------------------------------- Philox4x64-10 ------ */
static inline uint64_t mulhi64(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }
void oracle_philox(const uint64_t ctr_in[4], const uint64_t key_in[2], uint64_t out[4]) {
  uint64_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint64_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; r++) {
    uint64_t hi0 = mulhi64(0xD2E7470EE14C6C93ull, c0), lo0 = 0xD2E7470EE14C6C93ull * c0;
    uint64_t hi1 = mulhi64(0xCA5A826395121157ull, c2), lo1 = 0xCA5A826395121157ull * c2;
    uint64_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B97F4A7C15ull;
    k1 += 0xBB67AE8584CAA73Bull;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
static void philox_site(const uint64_t key[2], uint64_t a, uint64_t stream, uint64_t b, uint64_t c, uint64_t out[4]) {
  uint64_t ctr[4] = {a, stream, b, c};
  oracle_philox(ctr, key, out);
}
/* randint(lo, hi) in philox mode: int() truncation, multiply-high mapping */
static inline int64_t ph_randint(uint64_t u, double lo, double hi) {
  int64_t l = (int64_t)lo, h = (int64_t)hi;
  if (h <= l) return l;
  return l + (int64_t)mulhi64(u, (uint64_t)(h - l));
}

/* -------------------------------------------------------------- Cell -- */
typedef struct Cell {
  double x, y, mass, radius, vx, vy, svx, svy, merge_time;
  int svc;
  int64_t seq;
  int player; /* -1: pellet / blob / virus */
  int alive;
  int blob_to_eject;
  int64_t ejecter_seq;
  int col;  /* colour owner: the player whose colour an ejected blob (and the
               pellet it becomes) carries (field.py:141, cell.py:219), else -1 */
  int mark; /* scratch for snapshot hash membership */
} Cell;

typedef struct { Cell **a; int n, cap; } CVec;
static void cv_push(CVec *v, Cell *c) {
  if (v->n == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 4;
    v->a = (Cell **)realloc(v->a, sizeof(Cell *) * v->cap);
  }
  v->a[v->n++] = c;
}
static int cv_remove(CVec *v, Cell *c) { /* list.remove: first occurrence, stable */
  for (int i = 0; i < v->n; i++)
    if (v->a[i] == c) {
      memmove(v->a + i, v->a + i + 1, sizeof(Cell *) * (v->n - i - 1));
      v->n--;
      return 0;
    }
  return -1;
}
static void cv_free(CVec *v) { free(v->a); v->a = NULL; v->n = v->cap = 0; }

/* cell.py:210-212 */
static inline void cell_set_mass(Cell *c, double v) {
  c->mass = v;
  c->radius = (v > 0) ? sqrt(v / PI) : 0;
}

/* ----------------------------------------------------------- World ---- */
typedef struct Hash {
  double size, bucket, left, top; /* spatialHashTable.py:15-23 */
  int rows, cols;
  CVec *b;
} Hash;

typedef struct Player {
  CVec cells;
  int alive, respawn;
  double cmdx, cmdy;
  int do_split, do_eject;
  double fov_x, fov_y, fov_size; /* cached (player.py:156-167) */
} Player;

typedef struct Arena {
  int idx, B, size, virus_enabled, G;
  double max_pellets, max_viruses;
  Player *pl;
  CVec pellets, blobs, viruses, grave;
  int *dead, n_dead;
  Hash ph, bh, plh, vh; /* pellet, blob, player, virus hashes */
  int64_t seq_next, tick;
  int rng_mode;
  MT mt;
  uint64_t key[2], ctr_pellet, ctr_virus;
  /* bot-side observation state (bot.py:81-121, reset for NN bots) */
  double *obs_fov, *self_lf, *self_slf, *enemy_lf, *enemy_slf, *act_cur, *act_prev;
  int64_t *ev;
  int n_ev, cap_ev;
  int err;
  int *split_lh; /* Greedy bots' splitLikelihood (bot.py:93); NULL: derived from the Philox key */
} Arena;

typedef struct Oracle {
  aigar_config cfg;
  int A, L;
  Arena *ar;
} Oracle;

static void ev_push(Arena *A, int code, int64_t a, int64_t b) {
  if (A->n_ev == A->cap_ev) {
    A->cap_ev = A->cap_ev ? 2 * A->cap_ev : 1024;
    A->ev = (int64_t *)realloc(A->ev, sizeof(int64_t) * 4 * A->cap_ev);
  }
  int64_t *e = A->ev + 4 * A->n_ev++;
  e[0] = A->tick; e[1] = code; e[2] = a; e[3] = b;
}

/* Cell.__init__ (cell.py:21-45).  Colour draws: 3 x randint(50, 200) when the
 * cell has no player, in MT mode only (colours never feed the dynamics). */
static Cell *new_cell(Arena *A, double x, double y, double mass, int player) {
  Cell *c = (Cell *)calloc(1, sizeof(Cell));
  c->seq = A->seq_next++;
  c->player = player;
  cell_set_mass(c, mass);
  c->x = x;
  c->y = y;
  if (player < 0 && A->rng_mode == AIGAR_RNG_MT19937) {
    mt_randint(&A->mt, 50, 200);
    mt_randint(&A->mt, 50, 200);
    mt_randint(&A->mt, 50, 200);
  }
  c->svc = 0;
  c->merge_time = 0;
  c->alive = 1;
  c->ejecter_seq = -1;
  c->col = -1;
  return c;
}

/* ------------------------------------------------------ spatial hash -- */
static void hash_init(Hash *h, double size, double bucket, double left, double top) {
  h->size = size; h->bucket = bucket; h->left = left; h->top = top;
  h->rows = (int)ceil(size / bucket);
  h->cols = h->rows;
  h->b = (CVec *)calloc((size_t)h->rows * h->cols, sizeof(CVec));
}
static void hash_free(Hash *h) {
  if (!h->b) return;
  for (int i = 0; i < h->rows * h->cols; i++) cv_free(&h->b[i]);
  free(h->b);
  h->b = NULL;
}
static void hash_clear(Hash *h) { /* clearBuckets (spatialHashTable.py:45-47) */
  for (int i = 0; i < h->rows * h->cols; i++) h->b[i].n = 0;
}
/* getIdsForArea, int variant (spatialHashTable.py:70-83); returns #ids.
 * The id set is enumerated without duplicates (x, y strides are disjoint). */
static int hash_ids(const Hash *h, double px, double py, double rad, int **ids, int *cap) {
  int bs = (int)h->bucket;
  double cl = py_max(0, px - rad), ct = py_max(0, py - rad);
  long bl = (long)(cl - py_mod(cl, bs)), bt = (long)(ct - py_mod(ct, bs));
  long lx = (long)py_min(h->size, px + rad + 1), ly = (long)py_min(h->size, py + rad + 1);
  int n = 0;
  for (long x = bl; x < lx; x += bs)
    for (long y = bt; y < ly; y += bs) {
      if (n == *cap) {
        *cap = *cap ? *cap * 2 : 64;
        *ids = (int *)realloc(*ids, sizeof(int) * *cap);
      }
      (*ids)[n++] = (int)(long)((double)x / bs) + (int)(long)((double)y / bs) * h->cols;
    }
  return n;
}
static __thread int *t_ids;
static __thread int t_ids_cap;
static void hash_insert(Hash *h, Cell *c) {
  int n = hash_ids(h, c->x, c->y, c->radius, &t_ids, &t_ids_cap);
  for (int i = 0; i < n; i++) cv_push(&h->b[t_ids[i]], c);
}
static int hash_delete(Arena *A, Hash *h, Cell *c) { /* list.remove raises when missing */
  int n = hash_ids(h, c->x, c->y, c->radius, &t_ids, &t_ids_cap);
  for (int i = 0; i < n; i++)
    if (cv_remove(&h->b[t_ids[i]], c)) {
      set_err("spatial hash delete of an object that is not hashed (reference raises ValueError), seq %lld",
              (long long)c->seq);
      A->err = 1;
      return -1;
    }
  return 0;
}
static int cmp_seq(const void *a, const void *b) {
  int64_t x = (*(Cell *const *)a)->seq, y = (*(Cell *const *)b)->seq;
  return (x > y) - (x < y);
}
/* getObjectsFromBuckets with the canonical-order shim: unique, seq-sorted */
static void hash_query(const Hash *h, double px, double py, double rad, CVec *out) {
  out->n = 0;
  int n = hash_ids(h, px, py, rad, &t_ids, &t_ids_cap);
  for (int i = 0; i < n; i++) {
    CVec *b = &h->b[t_ids[i]];
    for (int j = 0; j < b->n; j++) cv_push(out, b->a[j]);
  }
  if (out->n > 1) {
    qsort(out->a, out->n, sizeof(Cell *), cmp_seq);
    int m = 1;
    for (int i = 1; i < out->n; i++)
      if (out->a[i] != out->a[m - 1]) out->a[m++] = out->a[i];
    out->n = m;
  }
}
/* adjustCellSize (field.py:14-17) */
static void adjust_cell_size(Arena *A, Cell *c, double mass, Hash *h) {
  hash_delete(A, h, c);
  cell_set_mass(c, py_min(MAX_MASS_SINGLE_CELL, c->mass + mass)); /* Cell.grow cell.py:119-121 */
  hash_insert(h, c);
}

/* -------------------------------------------------- Cell methods ------ */
static inline double sqdist(const Cell *a, const Cell *b) { /* cell.py:158-160 */
  return (a->x - b->x) * (a->x - b->x) + (a->y - b->y) * (a->y - b->y);
}
static inline int overlap(const Cell *a, const Cell *b) { /* cell.py:143-152 */
  const Cell *big = a, *small = b;
  if (!(a->mass > b->mass)) { big = b; small = a; }
  return sqdist(big, small) * 1.1 < big->radius * big->radius;
}
static inline int can_eat(const Cell *a, const Cell *b) { return a->mass > 1.25 * b->mass; } /* cell.py:163 */
static inline int in_fov(const Cell *c, double fx, double fy, double fs) { /* cell.py:169-177 */
  double h = fs / 2, xmin = fx - h, xmax = fx + h, ymin = fy - h, ymax = fy + h;
  return !(c->x + c->radius < xmin || c->x - c->radius > xmax || c->y + c->radius < ymin || c->y - c->radius > ymax);
}
static void set_move_direction(Cell *c, double cpx, double cpy) { /* cell.py:47-57 */
  double xd = cpx - c->x, yd = cpy - c->y;
  double hyp = xd * xd + yd * yd, r2 = c->radius * c->radius;
  double mod = py_min(hyp, r2) / r2;
  double ang = atan2(yd, xd);
  double sp = CELL_MOVE_SPEED * pow(c->mass, -0.35);
  c->vx = sp * mod * cos(ang);
  c->vy = sp * mod * sin(ang);
}
static void add_momentum(Cell *c, double cpx, double cpy, double w, double h, const Cell *orig) { /* cell.py:96-103 */
  double cx = py_max(0, py_min(w, cpx)), cy = py_max(0, py_min(h, cpy));
  double ang = atan2(cy - c->y, cx - c->x);
  double sp = 2 + orig->radius * 0.05;
  c->svx = cos(ang) * sp;
  c->svy = sin(ang) * sp;
  c->svc = 15;
}
static void update_momentum(Cell *c) { /* cell.py:105-116 */
  if (c->svc == -1) return;
  if (c->svc > 0) {
    c->svc -= 1;
    double ratio = c->svc / 15.0;
    if (ratio < 0.1) {
      c->svx *= (1 - ratio);
      c->svy *= (1 - ratio);
    }
  } else {
    c->svx = 0;
    c->svy = 0;
    c->svc = -1;
  }
}
static void reset_merge_time(Cell *c, double f) { /* cell.py:154-155 */
  c->merge_time = f * (BASE_MERGE_TIME + c->mass * MERGE_TIME_MASS_FACTOR) * FPS / 2 / GAME_SPEED;
}
static void update_pos(Cell *c, double mx, double my) { /* cell.py:132-141 */
  double xs = c->vx + c->svx, ys = c->vy + c->svy;
  c->x = py_min(mx, py_max(0, c->x + xs));
  c->y = py_min(my, py_max(0, c->y + ys));
  if ((c->svc != 0 && c->x == mx) || c->x == 0) c->svx *= -1;
  if ((c->svc != 0 && c->y == my) || c->y == 0) c->svy *= -1;
}
static Cell *cell_split(Arena *A, Cell *c, double cpx, double cpy, double w, double h) { /* cell.py:72-85 */
  double x = c->x, y = c->y;
  Cell *n = new_cell(A, x, y, c->mass / 2, c->player);
  double ang = atan2(cpy - n->y, cpx - n->x);
  double xp = cos(ang) * n->radius * 4.5 + x, yp = sin(ang) * n->radius * 4.5 + y;
  add_momentum(n, xp, yp, w, h, c);
  reset_merge_time(n, 1);
  cell_set_mass(c, c->mass / 2);
  return n;
}

/* ------------------------------------------------------ Player ------- */
static double player_total_mass(const Player *P) { /* player.py:129-130 */
  if (P->cells.n == 0) return 0;
  double tmp[16] = {0};
  int n = P->cells.n;
  double *m = n <= 16 ? tmp : (double *)malloc(sizeof(double) * n);
  for (int i = 0; i < n; i++) m[i] = P->cells.a[i]->mass;
  double s = oracle_np_sum(m, n);
  if (m != tmp) free(m);
  return s;
}
static void player_fov_pos(Player *P, double *fx, double *fy) { /* player.py:156-161 */
  if (P->alive && player_total_mass(P) != 0) {
    int n = P->cells.n;
    double ax[64], ay[64];
    for (int i = 0; i < n; i++) {
      ax[i] = P->cells.a[i]->x * P->cells.a[i]->mass;
      ay[i] = P->cells.a[i]->y * P->cells.a[i]->mass;
    }
    double tm = player_total_mass(P);
    P->fov_x = oracle_np_sum(ax, n) / tm;
    P->fov_y = oracle_np_sum(ay, n) / tm;
  }
  *fx = P->fov_x;
  *fy = P->fov_y;
}
static double player_fov_size(Player *P) { /* player.py:163-167 */
  if (P->alive && P->cells.n > 0) {
    const Cell *b = P->cells.a[0];
    for (int i = 1; i < P->cells.n; i++)
      if (P->cells.a[i]->radius > b->radius) b = P->cells.a[i];
    P->fov_size = pow(b->radius, 0.475) * pow((double)P->cells.n, 0.32) * 35;
  }
  return P->fov_size;
}
static void player_set_dead(Player *P) { P->alive = 0; P->respawn = 1; } /* player.py:110-112, stepsUntilRespawn */
static void player_set_alive(Player *P) { P->alive = 1; P->respawn = 0; }

/* player.py:30-72 */
static void player_update(Arena *A, Player *P, double w, double h) {
  if (!P->alive) return;
  for (int i = 0; i < P->cells.n; i++) { /* decayMass, cell.py:123-126 */
    Cell *c = P->cells.a[i];
    if (c->mass >= 4) cell_set_mass(c, c->mass * CELL_MASS_DECAY_RATE);
  }
  for (int i = 0; i < P->cells.n; i++) { /* updateCellProperties */
    Cell *c = P->cells.a[i];
    update_momentum(c);
    if (c->merge_time > 0) c->merge_time -= 1; /* updateMerge cell.py:128-130 */
    set_move_direction(c, P->cmdx, P->cmdy);
  }
  if (P->do_split) { /* Player.split: stable sort by mass desc, then split the snapshot */
    for (int i = 1; i < P->cells.n; i++) {
      Cell *k = P->cells.a[i];
      int j = i - 1;
      while (j >= 0 && k->mass > P->cells.a[j]->mass) {
        P->cells.a[j + 1] = P->cells.a[j];
        j--;
      }
      P->cells.a[j + 1] = k;
    }
    int n0 = P->cells.n;
    Cell *snap[16];
    for (int i = 0; i < n0; i++) snap[i] = P->cells.a[i];
    for (int i = 0; i < n0; i++) {
      Cell *c = snap[i];
      if (c->mass > 36 && P->cells.n < 16) cv_push(&P->cells, cell_split(A, c, P->cmdx, P->cmdy, w, h));
    }
  }
  if (P->do_eject) /* Player.eject */
    for (int i = 0; i < P->cells.n; i++)
      if (P->cells.a[i]->mass >= 35) P->cells.a[i]->blob_to_eject = 1;
  for (int i = 0; i < P->cells.n; i++) update_pos(P->cells.a[i], w, h);
}

/* ------------------------------------------------------ Field -------- */
/* getSpawnPos (field.py:283-301) */
static void get_spawn_pos(Arena *A, double radius, const uint64_t *u, double *ox, double *oy) {
  int cols = A->plh.cols, total = A->plh.rows * cols;
  int64_t sb = (A->rng_mode == AIGAR_RNG_MT19937) ? mt_randint(&A->mt, 0, total) : (int64_t)mulhi64(u[0], (uint64_t)total);
  int count = 0;
  while (A->plh.b[sb].n > 0 && count < total) {
    sb = (sb + 1) % total;
    count++;
  }
  int64_t xp, yp;
  if (count == total) {
    if (A->rng_mode == AIGAR_RNG_MT19937) {
      xp = mt_randint(&A->mt, 0, A->size);
      yp = mt_randint(&A->mt, 0, A->size);
    } else {
      xp = ph_randint(u[1], 0, A->size);
      yp = ph_randint(u[2], 0, A->size);
    }
  } else {
    int64_t x = sb % cols;
    double y = (double)(sb - x) / cols;
    int64_t left = (x - 1) * HASH_BUCKET_SIZE;
    double top = y * HASH_BUCKET_SIZE;
    if (A->rng_mode == AIGAR_RNG_MT19937) {
      xp = mt_randint(&A->mt, left + radius, left + HASH_BUCKET_SIZE - radius);
      yp = mt_randint(&A->mt, top + radius, top + HASH_BUCKET_SIZE - radius);
    } else {
      xp = ph_randint(u[1], left + radius, left + HASH_BUCKET_SIZE - radius);
      yp = ph_randint(u[2], top + radius, top + HASH_BUCKET_SIZE - radius);
    }
  }
  *ox = (double)xp;
  *oy = (double)yp;
}

static void add_player_cell(Arena *A, Player *P, Cell *c) { /* field.py:402-404 */
  hash_insert(&A->plh, c);
  cv_push(&P->cells, c);
}

/* initializePlayer (field.py:49-55) */
static void initialize_player(Arena *A, int p, int is_respawn) {
  Player *P = &A->pl[p];
  for (int i = 0; i < P->cells.n; i++) cv_push(&A->grave, P->cells.a[i]);
  P->cells.n = 0;
  uint64_t u[4] = {0, 0, 0, 0};
  if (A->rng_mode == AIGAR_RNG_PHILOX) {
    if (is_respawn)
      philox_site(A->key, (uint64_t)p, ST_PLAYER, (uint64_t)A->tick, 0, u);
    else
      philox_site(A->key, (uint64_t)p, ST_INIT_PLAYER, 0, 0, u);
  }
  double x, y;
  get_spawn_pos(A, START_RADIUS, u, &x, &y);
  Cell *c = new_cell(A, x, y, START_MASS, p);
  cv_push(&P->cells, c);
  player_set_alive(P);
}

static void delete_player_cell(Arena *A, Cell *c) { /* field.py:382-388 */
  hash_delete(A, &A->plh, c);
  Player *P = &A->pl[c->player];
  c->alive = 0;
  cv_remove(&P->cells, c);
  cv_push(&A->grave, c);
  if (P->cells.n == 0) {
    A->dead[A->n_dead++] = c->player;
    player_set_dead(P);
    ev_push(A, AIGAR_EV_PLAYER_DEATH, c->player, c->seq);
  }
}

/* eatCell (field.py:337-344) */
static void eat_cell(Arena *A, Cell *eater, Hash *eh, Cell *c, Hash *ch, CVec *list, int is_virus) {
  double mass = c->mass;
  if (is_virus) mass *= VIRUS_EAT_FACTOR;
  adjust_cell_size(A, eater, mass, eh);
  if (cv_remove(list, c)) {
    set_err("list.remove of a missing entity (reference raises ValueError), seq %lld", (long long)c->seq);
    A->err = 1;
  }
  hash_delete(A, ch, c);
  c->alive = 0;
  cv_push(&A->grave, c);
}

static void spawn_pellets(Arena *A) { /* field.py:303-313, randomSize field.py:20-26 */
  while (A->pellets.n < A->max_pellets) {
    int64_t x, y, sr;
    if (A->rng_mode == AIGAR_RNG_MT19937) {
      x = mt_randint(&A->mt, 0, A->size);
      y = mt_randint(&A->mt, 0, A->size);
      sr = mt_randint(&A->mt, 0, 50);
    } else {
      uint64_t u[4];
      philox_site(A->key, A->ctr_pellet++, ST_PELLET, 0, 0, u);
      x = (int64_t)mulhi64(u[0], (uint64_t)A->size);
      y = (int64_t)mulhi64(u[1], (uint64_t)A->size);
      sr = (int64_t)mulhi64(u[2], 50);
    }
    double m = (sr > 50 - 4) ? (double)(50 - sr) : 1.0;
    Cell *c = new_cell(A, (double)x, (double)y, m, -1);
    hash_insert(&A->ph, c); /* addPellet field.py:390-392 */
    cv_push(&A->pellets, c);
  }
}
static void spawn_viruses(Arena *A) { /* field.py:262-275 */
  while (A->viruses.n < A->max_viruses) {
    uint64_t u[4] = {0, 0, 0, 0}, u2[4] = {0, 0, 0, 0};
    if (A->rng_mode == AIGAR_RNG_PHILOX) {
      philox_site(A->key, A->ctr_virus, ST_VIRUS, 0, 0, u);
      philox_site(A->key, A->ctr_virus, ST_VIRUS, 1, 0, u2);
      A->ctr_virus++;
    }
    double x, y;
    get_spawn_pos(A, VIRUS_BASE_RADIUS, u, &x, &y);
    double rng = HASH_BUCKET_SIZE - VIRUS_BASE_RADIUS;
    if (A->rng_mode == AIGAR_RNG_MT19937) {
      x += (double)mt_randint(&A->mt, (-1) * rng / 2, rng / 2);
      y += (double)mt_randint(&A->mt, (-1) * rng / 2, rng / 2);
    } else {
      x += (double)ph_randint(u2[0], (-1) * rng / 2, rng / 2);
      y += (double)ph_randint(u2[1], (-1) * rng / 2, rng / 2);
    }
    Cell *v = new_cell(A, x, y, VIRUS_BASE_SIZE, -1);
    cv_push(&A->viruses, v); /* addVirus: not hashed (field.py:398-400) */
  }
}
static void spawn_players(Arena *A) { /* field.py:277-281 */
  int nd = A->n_dead;
  int *snap = (int *)malloc(sizeof(int) * (nd + 1));
  memcpy(snap, A->dead, sizeof(int) * nd);
  for (int i = 0; i < nd; i++) {
    int p = snap[i];
    if (A->pl[p].respawn == 0) {
      for (int j = 0; j < A->n_dead; j++)
        if (A->dead[j] == p) {
          memmove(A->dead + j, A->dead + j + 1, sizeof(int) * (A->n_dead - j - 1));
          A->n_dead--;
          break;
        }
      initialize_player(A, p, 1);
      ev_push(A, AIGAR_EV_RESPAWN, p, A->pl[p].cells.a[0]->seq);
    }
  }
  free(snap);
}
static void spawn_stuff(Arena *A) { /* field.py:256-260 */
  spawn_pellets(A);
  if (A->virus_enabled) spawn_viruses(A);
  spawn_players(A);
}

/* --- tick phases (field.py:85-92) --- */
static void update_viruses(Arena *A) { /* field.py:94-97 */
  for (int i = 0; i < A->viruses.n; i++) {
    update_momentum(A->viruses.a[i]);
    update_pos(A->viruses.a[i], A->size, A->size);
  }
}
static void update_blobs(Arena *A) { /* field.py:99-110 */
  CVec stop = {0};
  for (int i = 0; i < A->blobs.n; i++) {
    Cell *b = A->blobs.a[i];
    if (b->svc == 0) {
      cv_push(&stop, b);
      continue;
    }
    update_momentum(b);
    update_pos(b, A->size, A->size);
  }
  for (int i = 0; i < stop.n; i++) {
    Cell *b = stop.a[i];
    cv_remove(&A->blobs, b);
    hash_delete(A, &A->bh, b);
    hash_insert(&A->ph, b); /* addPellet */
    cv_push(&A->pellets, b);
  }
  cv_free(&stop);
}
static void adjust_cell_positions(Arena *A, Cell *c1, Cell *c2, double d, double sr) { /* field.py:161-181 */
  Cell *big = c1, *small = c2;
  if (!(c1->mass > c2->mass)) { big = c2; small = c1; }
  double bx = big->x, by = big->y, sx = small->x, sy = small->y;
  double ds = (sr - d) / d, mds = small->mass / big->mass;
  double xd = (bx - sx) * ds, yd = (by - sy) * ds;
  double nbx = bx + xd * mds, nby = by + yd * mds;
  double nsx = sx - xd * (1 - mds), nsy = sy - yd * (1 - mds);
  big->x = py_min(A->size, py_max(0, nbx)); /* adjustCellPos field.py:406-410 */
  big->y = py_min(A->size, py_max(0, nby));
  small->x = py_min(A->size, py_max(0, nsx));
  small->y = py_min(A->size, py_max(0, nsy));
}
static void update_players(Arena *A) { /* field.py:112-119 */
  for (int p = 0; p < A->B; p++) {
    Player *P = &A->pl[p];
    if (!P->alive) {
      P->respawn -= 1; /* updateRespawnTime */
      continue;
    }
    player_update(A, P, A->size, A->size);
    for (int i = 0; i < P->cells.n; i++) { /* performEjections field.py:134-146 */
      Cell *c = P->cells.a[i];
      if (!c->blob_to_eject) continue;
      c->mass -= EJECTEDBLOB_BASE_MASS; /* Cell.eject: radius left stale (cell.py:90-94) */
      c->blob_to_eject = 0;
      Cell *b = new_cell(A, c->x, c->y, EJECTEDBLOB_BASE_MASS * 0.8, -1);
      add_momentum(b, P->cmdx, P->cmdy, A->size, A->size, c);
      cv_push(&A->blobs, b);
      b->ejecter_seq = c->seq;
      b->col = c->player; /* blob.setColor(player.getColor()); setEjecterCell (field.py:141-146) */
    }
    for (int i = 0; i < P->cells.n; i++) { /* handlePlayerCollisions field.py:149-159 */
      Cell *c = P->cells.a[i];
      if (c->svc > 0) continue;
      for (int j = 0; j < P->cells.n; j++) {
        Cell *o = P->cells.a[j];
        if (c == o || o->svc > 0 || (c->merge_time <= 0 && o->merge_time <= 0)) continue;
        double d = sqrt(sqdist(c, o));
        double sr = c->radius + o->radius;
        if (d < sr && d != 0) adjust_cell_positions(A, c, o, d, sr);
      }
    }
  }
}
static void update_hash_tables(Arena *A) { /* field.py:121-132 */
  hash_clear(&A->plh);
  for (int p = 0; p < A->B; p++)
    if (A->pl[p].alive)
      for (int i = 0; i < A->pl[p].cells.n; i++) hash_insert(&A->plh, A->pl[p].cells.a[i]);
  hash_clear(&A->bh);
  for (int i = 0; i < A->blobs.n; i++) hash_insert(&A->bh, A->blobs.a[i]);
  hash_clear(&A->vh);
  for (int i = 0; i < A->viruses.n; i++) hash_insert(&A->vh, A->viruses.a[i]);
}
static void merge_cells(Arena *A, Cell *a, Cell *b) { /* field.py:372-380 */
  Cell *big = a, *small = b;
  if (!(a->mass > b->mass)) { big = b; small = a; }
  ev_push(A, AIGAR_EV_MERGE, big->seq, small->seq);
  adjust_cell_size(A, big, small->mass, &A->plh);
  delete_player_cell(A, small);
}
static void merge_player_cells(Arena *A) { /* field.py:183-198 */
  for (int p = 0; p < A->B; p++) {
    Player *P = &A->pl[p];
    if (!P->alive) continue;
    Cell *cs[64];
    int n = 0;
    for (int i = 0; i < P->cells.n; i++)
      if (P->cells.a[i]->merge_time <= 0) cs[n++] = P->cells.a[i];
    if (n <= 1) continue;
    for (int i = 1; i < n; i++) { /* stable sort, mass descending */
      Cell *k = cs[i];
      int j = i - 1;
      while (j >= 0 && k->mass > cs[j]->mass) {
        cs[j + 1] = cs[j];
        j--;
      }
      cs[j + 1] = k;
    }
    for (int i = 0; i < n; i++) {
      Cell *c1 = cs[i];
      if (!c1->alive) continue;
      for (int j = 0; j < n; j++) {
        Cell *c2 = cs[j];
        if (!c2->alive || c2 == c1) continue;
        if (overlap(c1, c2)) {
          merge_cells(A, c1, c2);
          if (!c1->alive) break;
        }
      }
    }
  }
}
static void virus_blob_overlap(Arena *A) { /* field.py:246-253, virusEatBlob :316-325 */
  CVec near = {0};
  for (int i = 0; i < A->viruses.n; i++) {
    Cell *v = A->viruses.a[i];
    hash_query(&A->bh, v->x, v->y, v->radius, &near);
    for (int j = 0; j < near.n; j++) {
      Cell *b = near.a[j];
      if (!overlap(v, b)) continue;
      ev_push(A, AIGAR_EV_VIRUS_EAT_BLOB, v->seq, b->seq);
      eat_cell(A, v, &A->vh, b, &A->bh, &A->blobs, 0);
      if (v->mass >= VIRUS_BASE_SIZE + 7 * EJECTEDBLOB_BASE_MASS * 0.8) {
        double ox = 2 * v->x - b->x, oy = 2 * v->y - b->y;
        Cell *nv = cell_split(A, v, ox, oy, A->size, A->size);
        cv_push(&A->viruses, nv);
        ev_push(A, AIGAR_EV_VIRUS_SPLIT, v->seq, nv->seq);
      }
    }
  }
  cv_free(&near);
}
static void player_cell_ate_virus(Arena *A, Cell *pc) { /* field.py:350-370 */
  Player *P = &A->pl[pc->player];
  int n_new = 16 - P->cells.n;
  ev_push(A, AIGAR_EV_EXPLODE, pc->seq, n_new);
  if (n_new == 0) return;
  double dist = pc->mass * VIRUS_EXPLOSION_CELL_MASS_PROPORTION;
  double mpc = dist / n_new;
  reset_merge_time(pc, MERGE_TIME_VIRUS_FACTOR);
  adjust_cell_size(A, pc, -1 * mpc * n_new, &A->plh);
  for (int k = 0; k < n_new; k++) {
    double x = pc->x, y = pc->y;
    Cell *nc = new_cell(A, x, y, mpc, pc->player);
    int64_t deg;
    if (A->rng_mode == AIGAR_RNG_MT19937) {
      deg = mt_randint(&A->mt, 0, 360);
    } else {
      uint64_t u[4];
      philox_site(A->key, (uint64_t)nc->seq, ST_ANGLE, 0, 0, u);
      deg = (int64_t)mulhi64(u[0], 360);
    }
    double ang = (double)deg * (PI / 180.0); /* numpy.deg2rad */
    double xp = cos(ang) * pc->radius * 12 + x, yp = sin(ang) * pc->radius * 12 + y;
    set_move_direction(nc, xp, yp);
    add_momentum(nc, xp, yp, A->size, A->size, pc);
    reset_merge_time(nc, 0.8);
    add_player_cell(A, P, nc);
  }
}
static void player_virus_overlap(Arena *A) { /* field.py:225-231 */
  CVec near = {0};
  for (int p = 0; p < A->B; p++) {
    Player *P = &A->pl[p];
    if (!P->alive) continue;
    for (int i = 0; i < P->cells.n;) {
      Cell *c = P->cells.a[i++];
      hash_query(&A->vh, c->x, c->y, c->radius, &near);
      for (int j = 0; j < near.n; j++) {
        Cell *v = near.a[j];
        if (overlap(c, v) && c->mass > 1.25 * v->mass) {
          ev_push(A, AIGAR_EV_CELL_EAT_VIRUS, c->seq, v->seq); /* eatVirus field.py:333-335 */
          eat_cell(A, c, &A->plh, v, &A->vh, &A->viruses, 1);
          player_cell_ate_virus(A, c);
        }
      }
    }
  }
  cv_free(&near);
}
static void player_food_overlap(Arena *A, int blobs) { /* field.py:207-222 */
  CVec near = {0};
  Hash *h = blobs ? &A->bh : &A->ph;
  CVec *list = blobs ? &A->blobs : &A->pellets;
  for (int p = 0; p < A->B; p++) {
    Player *P = &A->pl[p];
    if (!P->alive) continue;
    for (int i = 0; i < P->cells.n;) {
      Cell *c = P->cells.a[i++];
      hash_query(h, c->x, c->y, c->radius, &near);
      for (int j = 0; j < near.n; j++) {
        Cell *f = near.a[j];
        if (!overlap(c, f)) continue;
        if (blobs && f->ejecter_seq == c->seq) continue;
        if (!can_eat(c, f)) continue;
        ev_push(A, blobs ? AIGAR_EV_CELL_EAT_BLOB : AIGAR_EV_CELL_EAT_PELLET, c->seq, f->seq);
        eat_cell(A, c, &A->plh, f, h, list, 0);
      }
    }
  }
  cv_free(&near);
}
static void player_player_overlap(Arena *A) { /* field.py:233-244 */
  CVec near = {0};
  for (int p = 0; p < A->B; p++) {
    Player *P = &A->pl[p];
    if (!P->alive) continue;
    for (int i = 0; i < P->cells.n;) {
      Cell *pc = P->cells.a[i++];
      hash_query(&A->plh, pc->x, pc->y, pc->radius, &near); /* getNearbyEnemyObjects */
      for (int j = 0; j < near.n; j++) {
        Cell *o = near.a[j];
        if (o->player == p) continue;
        if (!overlap(pc, o)) continue;
        if (can_eat(pc, o)) {
          ev_push(A, AIGAR_EV_CELL_EAT_CELL, pc->seq, o->seq); /* eatPlayerCell field.py:346-348 */
          adjust_cell_size(A, pc, o->mass, &A->plh);
          delete_player_cell(A, o);
        } else if (can_eat(o, pc)) {
          ev_push(A, AIGAR_EV_CELL_EAT_CELL, o->seq, pc->seq);
          adjust_cell_size(A, o, pc->mass, &A->plh);
          delete_player_cell(A, pc);
          break;
        }
      }
    }
  }
  cv_free(&near);
}
static void field_update(Arena *A) { /* field.py:85-92 */
  update_viruses(A);
  update_blobs(A);
  update_players(A);
  update_hash_tables(A);
  /* dead entities may still sit in stale virus-hash buckets until this rebuild
   * (a split virus is not re-hashed, field.py:322): free them only now */
  for (int i = 0; i < A->grave.n; i++) free(A->grave.a[i]);
  A->grave.n = 0;
  merge_player_cells(A);
  virus_blob_overlap(A); /* checkOverlaps field.py:200-205 */
  player_virus_overlap(A);
  player_food_overlap(A, 0);
  player_food_overlap(A, 1);
  player_player_overlap(A);
  spawn_stuff(A);
  A->tick++;
}

/* --------------------------------------------------- observation ----- */
/* float-variant spatial hash (spatialHashTable.py:85-108) */
/* ------------------------------------------------------ Greedy bot ---- */
static inline double u01(uint64_t u) { return (double)(u >> 11) * (1.0 / 9007199254740992.0); }
/* splitLikelihood = numpy.random.randint(9950, 10000) at bot creation (bot.py:93) */
static int greedy_split_likelihood(const Arena *A, int p) {
  if (A->split_lh) return A->split_lh[p];
  uint64_t u[4];
  philox_site(A->key, (uint64_t)p, ST_GREEDY_LH, 0, 0, u);
  return (int)ph_randint(u[0], 9950, 10000);
}
/* Bot.makeMove for a Greedy bot (bot.py:252-269): make_greedy_bot_move
 * (bot.py:579-633) then set_command_point (bot.py:550-577).  Candidates come
 * in the reference's list order -- pellets, then enemy cells, then viruses,
 * each in (canonical) set order -- and max() keeps the first maximum. */
static void greedy_move(Arena *A, int p, int greedy_split) {
  Player *P = &A->pl[p];
  if (!P->alive) return;
  double fx, fy;
  player_fov_pos(P, &fx, &fy);
  const double size = player_fov_size(P);
  const int64_t x = (int64_t)fx, y = (int64_t)fy;
  const int64_t left = x - (int64_t)(size / 2), top = y - (int64_t)(size / 2);
  CVec q = {0}, cand = {0};
  hash_query(&A->ph, fx, fy, size / 2, &q); /* getPelletsInFov */
  for (int i = 0; i < q.n; i++)
    if (in_fov(q.a[i], fx, fy, size)) cv_push(&cand, q.a[i]);
  Cell *big = P->cells.a[0]; /* max(playerCells, key=mass): first maximum */
  for (int k = 1; k < P->cells.n; k++)
    if (P->cells.a[k]->mass > big->mass) big = P->cells.a[k];
  hash_query(&A->plh, fx, fy, size / 2, &q); /* getEnemyPlayerCellsInFov */
  for (int i = 0; i < q.n; i++)
    if (in_fov(q.a[i], fx, fy, size) && q.a[i]->player != p && big->mass > 1.25 * q.a[i]->mass)
      cv_push(&cand, q.a[i]);
  if (A->virus_enabled) { /* getVirusesInFov */
    hash_query(&A->vh, fx, fy, size / 2, &q);
    for (int i = 0; i < q.n; i++)
      if (in_fov(q.a[i], fx, fy, size) && big->mass > 1.25 * q.a[i]->mass) cv_push(&cand, q.a[i]);
  }
  uint64_t u[4] = {0, 0, 0, 0};
  if (A->rng_mode != AIGAR_RNG_MT19937) philox_site(A->key, (uint64_t)p, ST_GREEDY, (uint64_t)A->tick, 0, u);
  double a0, a1;
  if (cand.n) {
    Cell *best = NULL;
    double bk = 0;
    for (int i = 0; i < cand.n; i++) {
      Cell *c = cand.a[i];
      double sd = sqdist(c, big);
      double k = c->mass / (sd != 0 ? sd : 1);
      if (!best || k > bk) {
        best = c;
        bk = k;
      }
    }
    a0 = oracle_py_round5((best->x - (double)left) / size); /* getRelativeCellPos (bot.py:16-21) */
    a1 = oracle_py_round5((best->y - (double)top) / size);
  } else if (A->rng_mode == AIGAR_RNG_MT19937) {
    a0 = mt_random(&A->mt);
    a1 = mt_random(&A->mt);
  } else {
    a0 = u01(u[0]);
    a1 = u01(u[1]);
  }
  int split = 0, eject = 0;
  if (greedy_split) {
    int64_t rs, re;
    if (A->rng_mode == AIGAR_RNG_MT19937) {
      rs = mt_randint(&A->mt, 0, 10000);
      re = mt_randint(&A->mt, 0, 10000);
    } else {
      rs = ph_randint(u[2], 0, 10000);
      re = ph_randint(u[3], 0, 10000);
    }
    split = rs > greedy_split_likelihood(A, p);
    eject = re > 100000; /* ejectLikelihood (bot.py:94) */
  }
  /* set_command_point (bot.py:550-577) with the 4-element action */
  const int64_t isz = (int64_t)size;
  P->cmdx = (double)left + a0 * (double)isz;
  P->cmdy = (double)top + a1 * (double)isz;
  P->do_split = split;
  P->do_eject = eject;
  cv_free(&q);
  cv_free(&cand);
}

typedef struct { int cols, rows; CVec *b; } FHash;
static void fh_insert_all(FHash *fh, double size, double gs, double left, double top, Cell **objs, int n) {
  for (int k = 0; k < n; k++) {
    Cell *o = objs[k];
    double px = o->x - left, py = o->y - top, r = o->radius;
    double cl = py_max(0, px - r), ct = py_max(0, py - r);
    double bl = cl - py_mod(cl, gs), bt = ct - py_mod(ct, gs);
    double lx = py_min(size - 1, px + r), ly = py_min(size - 1, py + r);
    /* the ids form a set (spatialHashTable.py:89): an object enters a bucket once
     * (at 42 / 84 squares per side a cell covers thousands of them) */
    int nb = fh->cols * fh->rows;
    unsigned char *seen = (unsigned char *)calloc((size_t)nb, 1);
    for (double x = bl; x <= lx; x += gs)
      for (double y = bt; y <= ly; y += gs) {
        int id = (int)(long)(x / gs) + (int)(long)(y / gs) * fh->cols;
        if (seen[id]) continue;
        seen[id] = 1;
        cv_push(&fh->b[id], o);
      }
    free(seen);
  }
}

/* Bot.getSimpleStateRepresentation (bot.py:511-547; GRID_VIEW_ENABLED = False):
 * the first own cell, the closest enemy cell and the closest pellet relative to
 * the integer view box, then the distances to the visible field edges -- 12
 * values.  The enemy query uses the real fovSize, the pellet query the
 * truncated one (bot.py:531 passes size = int(size)); "closest" is min() over
 * the query's list (creation order), first one on ties. */
static void rel_cell(const Cell *c, int64_t left, int64_t top, int64_t size, double *o, int with_r) {
  if (!c) { /* getRelativeCellPos -> [0, 0] (+ [0]) */
    o[0] = o[1] = 0;
    if (with_r) o[2] = 0;
    return;
  }
  o[0] = oracle_py_round5((c->x - (double)left) / (double)size);
  o[1] = oracle_py_round5((c->y - (double)top) / (double)size);
  if (with_r) o[2] = oracle_py_round5(c->radius <= (double)size ? c->radius / (double)size : 1.0);
}
static void simple_one(Arena *A, int p, double *out) {
  Player *P = &A->pl[p];
  if (!P->alive) {
    for (int i = 0; i < 12; i++) out[i] = NAN;
    return;
  }
  double fs = player_fov_size(P), fx, fy;
  player_fov_pos(P, &fx, &fy);
  const int64_t x = (int64_t)fx, y = (int64_t)fy;
  const int64_t left = x - (int64_t)(fs / 2), top = y - (int64_t)(fs / 2), size = (int64_t)fs;
  const Cell *first = P->cells.a[0];
  rel_cell(first, left, top, size, out, 1);
  CVec q = {0};
  const Cell *best = NULL;
  double bd = 0;
  hash_query(&A->plh, fx, fy, fs / 2, &q); /* getEnemyPlayerCellsInFov (field.py:434-436) */
  for (int i = 0; i < q.n; i++) {
    const Cell *c = q.a[i];
    if (c->player == p || !in_fov(c, fx, fy, fs)) continue;
    const double dd = sqdist(c, first);
    if (!best || dd < bd) { best = c; bd = dd; }
  }
  rel_cell(best, left, top, size, out + 3, 1);
  best = NULL;
  hash_query(&A->ph, fx, fy, (double)size / 2, &q); /* getPelletsInFov(midPoint, int size) */
  for (int i = 0; i < q.n; i++) {
    const Cell *c = q.a[i];
    if (!in_fov(c, fx, fy, (double)size)) continue;
    const double dd = sqdist(c, first);
    if (!best || dd < bd) { best = c; bd = dd; }
  }
  rel_cell(best, left, top, size, out + 6, 0);
  const double w = (double)A->size, sz = (double)size;
  out[8] = left <= 0 ? (double)x / sz : 1.0;
  out[9] = left + size >= A->size ? (w - (double)x) / sz : 1.0;
  out[10] = top <= 0 ? (double)y / sz : 1.0;
  out[11] = top + size >= A->size ? (w - (double)y) / sz : 1.0;
  cv_free(&q);
}

static void observe_one(Oracle *O, Arena *A, int p, double *out) {
  const uint32_t ch = O->cfg.obs_channels, ex = O->cfg.obs_extras;
  if (ch & AIGAR_OBS_SIMPLE) {
    simple_one(A, p, out);
    return;
  }
  const int G = A->G, GG = G * G;
  Player *P = &A->pl[p];
  if (!P->alive) {
    for (int i = 0; i < O->L; i++) out[i] = NAN;
    return;
  }
  double fieldSize = A->size;
  double fovSize = player_fov_size(P);
  double fx, fy;
  player_fov_pos(P, &fx, &fy);
  double left = fx - fovSize / 2, top = fy - fovSize / 2;
  double gs = fovSize / G;
  FHash fh[4]; /* pellet, own, enemy, virus */
  int rows = (int)ceil(fovSize / gs);
  for (int k = 0; k < 4; k++) {
    fh[k].rows = fh[k].cols = rows;
    fh[k].b = (CVec *)calloc((size_t)rows * rows, sizeof(CVec));
  }
  CVec q = {0}, sel = {0};
  /* pellets: getPelletsInFov (field.py:442-444) */
  hash_query(&A->ph, fx, fy, fovSize / 2, &q);
  for (int i = 0; i < q.n; i++)
    if (in_fov(q.a[i], fx, fy, fovSize)) cv_push(&sel, q.a[i]);
  fh_insert_all(&fh[0], fovSize, gs, left, top, sel.a, sel.n);
  /* enemy cells: getEnemyPlayerCellsInFov (field.py:434-436) */
  player_fov_pos(P, &fx, &fy);
  hash_query(&A->plh, fx, fy, player_fov_size(P) / 2, &q);
  sel.n = 0;
  for (int i = 0; i < q.n; i++)
    if (in_fov(q.a[i], fx, fy, fovSize) && q.a[i]->player != p) cv_push(&sel, q.a[i]);
  fh_insert_all(&fh[2], fovSize, gs, left, top, sel.a, sel.n);
  /* own cells: getPortionOfCellsInFov(player.getCells()) */
  sel.n = 0;
  for (int i = 0; i < P->cells.n; i++)
    if (in_fov(P->cells.a[i], fx, fy, fovSize)) cv_push(&sel, P->cells.a[i]);
  fh_insert_all(&fh[1], fovSize, gs, left, top, sel.a, sel.n);
  if (A->virus_enabled) { /* getVirusesInFov */
    hash_query(&A->vh, fx, fy, fovSize / 2, &q);
    sel.n = 0;
    for (int i = 0; i < q.n; i++)
      if (in_fov(q.a[i], fx, fy, fovSize)) cv_push(&sel, q.a[i]);
    fh_insert_all(&fh[3], fovSize, gs, left, top, sel.a, sel.n);
  }
  double *gP = (double *)calloc(GG, sizeof(double)), *gW = (double *)calloc(GG, sizeof(double));
  double *gE = (double *)calloc(GG, sizeof(double)), *gS = (double *)calloc(GG, sizeof(double));
  double *gV = (double *)calloc(GG, sizeof(double));
  double mx = left + gs / 2, my = top + gs / 2;
  for (int c = 0; c < G; c++) {
    for (int r = 0; r < G; r++) {
      int cnt = r + c * G;
      if (!(mx + gs / 2 < 0 || mx - gs / 2 > fieldSize || my + gs / 2 < 0 || my - gs / 2 > fieldSize)) {
        CVec *b = &fh[0].b[cnt];
        if (b->n) {
          double s = 0;
          for (int i = 0; i < b->n; i++) s += b->a[i]->mass;
          gP[c * G + r] = s;
        }
        b = &fh[2].b[cnt];
        if (b->n) {
          const Cell *m = b->a[0];
          for (int i = 1; i < b->n; i++)
            if (b->a[i]->mass > m->mass) m = b->a[i];
          gE[c * G + r] = m->mass;
        }
        b = &fh[1].b[cnt];
        if (b->n) {
          const Cell *m = b->a[0];
          for (int i = 1; i < b->n; i++)
            if (b->a[i]->mass > m->mass) m = b->a[i];
          gS[c * G + r] = m->mass;
        }
        if (A->virus_enabled) {
          b = &fh[3].b[cnt];
          if (b->n) {
            const Cell *m = b->a[0];
            for (int i = 1; i < b->n; i++)
              if (b->a[i]->radius > m->radius) m = b->a[i];
            gV[c * G + r] = m->mass;
          }
        }
      }
      double lb = py_min(py_max(mx - gs / 2, 0), fieldSize), tb = py_min(py_max(my - gs / 2, 0), fieldSize);
      double rb = py_max(py_min(mx + gs / 2, fieldSize), 0), bb = py_max(py_min(my + gs / 2, fieldSize), 0);
      double freeA = (rb - lb) * (bb - tb);
      gW[c * G + r] = oracle_py_round3(1 - (freeA / pow(gs, 2)));
      mx += gs;
    }
    mx = left + gs / 2;
    my += gs;
  }
  /* stack channels (bot.py:459-495) */
  double *o = out;
  double *sl = A->self_lf + (size_t)p * GG, *ssl = A->self_slf + (size_t)p * GG;
  double *el = A->enemy_lf + (size_t)p * GG, *esl = A->enemy_slf + (size_t)p * GG;
#define PUT(src) do { memcpy(o, (src), sizeof(double) * GG); o += GG; } while (0)
  if (ch & AIGAR_OBS_PELLET) PUT(gP);
  if (ch & AIGAR_OBS_SELF) PUT(gS);
  if (ch & AIGAR_OBS_WALL) PUT(gW);
  if (ch & AIGAR_OBS_ENEMY) PUT(gE);
  if (ch & AIGAR_OBS_ALL) { /* ALL_PLAYER_GRID: biggest of own+enemy */
    double *gA = (double *)calloc(GG, sizeof(double));
    for (int i = 0; i < GG; i++) gA[i] = py_max(gE[i], gS[i]);
    PUT(gA);
    free(gA);
  }
  if (ch & AIGAR_OBS_VIRUS) PUT(gV);
  if (ch & AIGAR_OBS_SELF_SLF) { PUT(ssl); memcpy(ssl, sl, sizeof(double) * GG); }
  if (ch & AIGAR_OBS_SELF_LF) { PUT(sl); memcpy(sl, gS, sizeof(double) * GG); }
  if (ch & AIGAR_OBS_ENEMY_SLF) { PUT(esl); memcpy(esl, el, sizeof(double) * GG); }
  if (ch & AIGAR_OBS_ENEMY_LF) { PUT(el); memcpy(el, gE, sizeof(double) * GG); }
#undef PUT
  /* extras (bot.py:302-323) */
  if (ex & AIGAR_EX_LAST_FOV) *o++ = A->obs_fov[p];
  if (ex & AIGAR_EX_FOV) { A->obs_fov[p] = player_fov_size(P); *o++ = A->obs_fov[p]; }
  if (ex & AIGAR_EX_MASS) *o++ = player_total_mass(P);
  if (ex & AIGAR_EX_LAST_ACT) for (int k = 0; k < 4; k++) *o++ = A->act_cur[4 * p + k];
  if (ex & AIGAR_EX_2LAST_ACT) for (int k = 0; k < 4; k++) *o++ = A->act_prev[4 * p + k];
  for (int k = 0; k < 4; k++) {
    for (int i = 0; i < rows * rows; i++) cv_free(&fh[k].b[i]);
    free(fh[k].b);
  }
  cv_free(&q);
  cv_free(&sel);
  free(gP); free(gW); free(gE); free(gS); free(gV);
}

/* ------------------------------------------------ pixel observation ---- */
/* RGBGenerator.get_cnn_inputRGB (rgbGenerator.py:95-110): white frame, every
 * pellet / blob / virus / player cell in the FOV (rgbGenerator.py:60-68),
 * stable-sorted by mass, drawn with pygame's primitives.  pygame (1.9.4,
 * src/pip.txt) is not in this image, so the primitives are restated from the
 * published SDL_gfx 2.0 algorithms: filledCircleColor (midpoint spans),
 * aacircleColor = aaellipseColor (Wu-style weighted rim) with
 * pixelColorWeight blending, and pygame.draw.circle (width 0) as
 * filledEllipseColor spans.  Parity with pygame itself is UNPINNED.
 * Frame: RGB bytes, surfarray order [x][y][3]. */
typedef struct { uint8_t *px; int L; } Frame; /* px[(y * L + x) * 3 + c] */
static void fr_put(Frame *f, int x, int y, const uint8_t *c) {
  if (x < 0 || y < 0 || x >= f->L || y >= f->L) return; /* clip rect = surface */
  uint8_t *p = f->px + ((size_t)y * f->L + x) * 3;
  p[0] = c[0]; p[1] = c[1]; p[2] = c[2];
}
static void fr_hline(Frame *f, int x1, int x2, int y, const uint8_t *c) { /* hlineColor, opaque */
  if (x1 > x2) { int t = x1; x1 = x2; x2 = t; }
  for (int x = x1; x <= x2; x++) fr_put(f, x, y, c);
}
/* pixelColorWeight: alpha = (255 * weight) >> 8, then the 32-bpp blend
 * d + ((s - d) * alpha >> 8) per channel (alpha 255: plain store) */
static void fr_weight(Frame *f, int x, int y, const uint8_t *c, int weight) {
  int alpha = (255 * weight) >> 8;
  if (x < 0 || y < 0 || x >= f->L || y >= f->L) return;
  uint8_t *p = f->px + ((size_t)y * f->L + x) * 3;
  for (int k = 0; k < 3; k++) {
    int d = p[k];
    p[k] = (uint8_t)(alpha == 255 ? c[k] : d + (((c[k] - d) * alpha) >> 8));
  }
}
static void sdl_filled_circle(Frame *f, int x, int y, int rad, const uint8_t *c) { /* filledCircleColor */
  if (rad == 0) { fr_put(f, x, y, c); return; }
  int cx = 0, cy = rad, ocx = -1, ocy = -1, df = 1 - rad, d_e = 3, d_se = -2 * rad + 5;
  do {
    if (ocy != cy) {
      if (cy > 0) { fr_hline(f, x - cx, x + cx, y + cy, c); fr_hline(f, x - cx, x + cx, y - cy, c); }
      else fr_hline(f, x - cx, x + cx, y, c);
      ocy = cy;
    }
    if (ocx != cx) {
      if (cx != cy) {
        if (cx > 0) { fr_hline(f, x - cy, x + cy, y - cx, c); fr_hline(f, x - cy, x + cy, y + cx, c); }
        else fr_hline(f, x - cy, x + cy, y, c);
      }
      ocx = cx;
    }
    if (df < 0) { df += d_e; d_e += 2; d_se += 2; }
    else { df += d_se; d_e += 2; d_se += 4; cy--; }
    cx++;
  } while (cx <= cy);
}
static void sdl_filled_ellipse(Frame *f, int x, int y, int rx, int ry, const uint8_t *c) { /* filledEllipseColor */
  if (rx == 0) { for (int yy = y - ry; yy <= y + ry; yy++) fr_put(f, x, yy, c); return; }
  if (ry == 0) { fr_hline(f, x - rx, x + rx, y, c); return; }
  int oh = 0xFFFF, oi = 0xFFFF, oj = 0xFFFF, ok = 0xFFFF, ix, iy, h, i, j, k;
  if (rx > ry) {
    ix = 0; iy = rx * 64;
    do {
      h = (ix + 32) >> 6; i = (iy + 32) >> 6; j = (h * ry) / rx; k = (i * ry) / rx;
      if (ok != k && oj != k) {
        if (k > 0) { fr_hline(f, x - h, x + h, y + k, c); fr_hline(f, x - h, x + h, y - k, c); }
        else fr_hline(f, x - h, x + h, y, c);
        ok = k;
      }
      if (oj != j && ok != j && k != j) {
        if (j > 0) { fr_hline(f, x - i, x + i, y + j, c); fr_hline(f, x - i, x + i, y - j, c); }
        else fr_hline(f, x - i, x + i, y, c);
        oj = j;
      }
      ix = ix + iy / rx; iy = iy - ix / rx;
    } while (i > h);
  } else {
    ix = 0; iy = ry * 64;
    do {
      h = (ix + 32) >> 6; i = (iy + 32) >> 6; j = (h * rx) / ry; k = (i * rx) / ry;
      if (oi != i && oh != i) {
        if (i > 0) { fr_hline(f, x - j, x + j, y + i, c); fr_hline(f, x - j, x + j, y - i, c); }
        else fr_hline(f, x - j, x + j, y, c);
        oi = i;
      }
      if (oh != h && oi != h && i != h) {
        if (h > 0) { fr_hline(f, x - k, x + k, y + h, c); fr_hline(f, x - k, x + k, y - h, c); }
        else fr_hline(f, x - k, x + k, y, c);
        oh = h;
      }
      ix = ix + iy / ry; iy = iy - ix / ry;
    } while (i > h);
  }
}
static void sdl_aa_ellipse(Frame *f, int xc, int yc, int rx, int ry, const uint8_t *c) { /* aaellipseColor */
  int a2 = rx * rx, b2 = ry * ry, ds = 2 * a2, dt = 2 * b2, xc2 = 2 * xc, yc2 = 2 * yc;
  double sab = sqrt((double)(a2 + b2));
  int od = (int)lrint(sab * 0.01) + 1;
  int dxt = (int)lrint((double)a2 / sab) + od;
  int t = 0, s = -2 * a2 * ry, d = 0, x = xc, y = yc - ry, xs, ys, xx, yy;
  fr_put(f, x, y, c); fr_put(f, xc2 - x, y, c); fr_put(f, x, yc2 - y, c); fr_put(f, xc2 - x, yc2 - y, c);
  for (int i = 1; i <= dxt; i++) {
    x--;
    d += t - b2;
    if (d >= 0) ys = y - 1;
    else if ((d - s - a2) > 0) {
      if ((2 * d - s - a2) >= 0) ys = y + 1;
      else { ys = y; y++; d -= s + a2; s += ds; }
    } else { y++; ys = y + 1; d -= s + a2; s += ds; }
    t -= dt;
    float cp = s != 0 ? (float)abs(d) / (float)abs(s) : 1.0f;
    if (cp > 1.0f) cp = 1.0f;
    int weight = (uint8_t)(cp * 255), iweight = 255 - weight;
    xx = xc2 - x;
    fr_weight(f, x, y, c, iweight); fr_weight(f, xx, y, c, iweight);
    fr_weight(f, x, ys, c, weight); fr_weight(f, xx, ys, c, weight);
    yy = yc2 - y;
    fr_weight(f, x, yy, c, iweight); fr_weight(f, xx, yy, c, iweight);
    yy = yc2 - ys;
    fr_weight(f, x, yy, c, weight); fr_weight(f, xx, yy, c, weight);
  }
  int dyt = (int)lrint((double)b2 / sab) + od;
  for (int i = 1; i <= dyt; i++) {
    y++;
    d -= s + a2;
    if (d <= 0) xs = x + 1;
    else if ((d + t - b2) < 0) {
      if ((2 * d + t - b2) <= 0) xs = x - 1;
      else { xs = x; x--; d += t - b2; t -= dt; }
    } else { x--; xs = x - 1; d += t - b2; t -= dt; }
    s += ds;
    float cp = t != 0 ? (float)abs(d) / (float)abs(t) : 1.0f;
    if (cp > 1.0f) cp = 1.0f;
    int weight = (uint8_t)(cp * 255), iweight = 255 - weight;
    xx = xc2 - x; yy = yc2 - y;
    fr_weight(f, x, y, c, iweight); fr_weight(f, xx, y, c, iweight);
    fr_weight(f, x, yy, c, iweight); fr_weight(f, xx, yy, c, iweight);
    xx = xc2 - xs;
    fr_weight(f, xs, y, c, weight); fr_weight(f, xx, y, c, weight);
    fr_weight(f, xs, yy, c, weight); fr_weight(f, xx, yy, c, weight);
  }
}

/* colours: the facade's deterministic stand-ins for the reference's random
 * draws (aigar_amd/model.py player_color / pellet_color; splitmix64 finaliser) */
static uint64_t mix64(uint64_t v) {
  v += 0x9E3779B97F4A7C15ull;
  v = (v ^ (v >> 30)) * 0xBF58476D1CE4E5B9ull;
  v = (v ^ (v >> 27)) * 0x94D049BB133111EBull;
  return v ^ (v >> 31);
}
static void player_rgb(int index, uint64_t seed, uint8_t *c) { /* Player.randomizeColor (player.py:38-41) */
  for (uint64_t k = 0;; k++) {
    uint64_t h = mix64((seed << 32) ^ ((uint64_t)index << 8) ^ k);
    c[0] = h & 255; c[1] = (h >> 8) & 255; c[2] = (h >> 16) & 255;
    if (c[0] + c[1] + c[2] <= 600) return;
  }
}
static void pellet_rgb(int64_t seq, uint64_t seed, uint8_t *c) { /* cell.py:31 (also blobs: Cell(..., None)) */
  uint64_t h = mix64((seed << 40) ^ (uint64_t)seq ^ 0x5E11E7ull);
  c[0] = 50 + h % 150; c[1] = 50 + (h >> 16) % 150; c[2] = 50 + (h >> 32) % 150;
}

typedef struct { const Cell *c; int kind; } PixObj; /* kind: 0 pellet, 1 blob, 2 virus, 3 player cell */
static int cmp_pix(const void *pa, const void *pb) {
  const PixObj *a = (const PixObj *)pa, *b = (const PixObj *)pb;
  /* list.sort(key=mass) is stable over pellets + blobs + viruses + playerCells,
   * each in canonical (creation sequence) order */
  if (a->c->mass != b->c->mass) return a->c->mass < b->c->mass ? -1 : 1;
  if (a->kind != b->kind) return a->kind - b->kind;
  return a->c->seq < b->c->seq ? -1 : (a->c->seq > b->c->seq);
}

static void pixels_one(Arena *A, int p, int L, uint64_t seed, uint8_t *out) {
  Player *P = &A->pl[p];
  memset(out, 0, (size_t)L * L * 3);
  if (!P->alive) return;
  double fx, fy, fs = player_fov_size(P);
  player_fov_pos(P, &fx, &fy);
  CVec q = {0};
  PixObj *objs = NULL;
  int n = 0, cap = 0;
  const Hash *hs[4] = {&A->ph, &A->bh, &A->vh, &A->plh}; /* drawAllCells (rgbGenerator.py:60-68) */
  for (int k = 0; k < 4; k++) {
    hash_query(hs[k], fx, fy, fs / 2, &q);
    for (int i = 0; i < q.n; i++) {
      if (!in_fov(q.a[i], fx, fy, fs)) continue;
      if (n == cap) { cap = cap ? 2 * cap : 64; objs = (PixObj *)realloc(objs, sizeof(PixObj) * cap); }
      objs[n].c = q.a[i];
      objs[n++].kind = k;
    }
  }
  if (n > 1) qsort(objs, n, sizeof(PixObj), cmp_pix);
  Frame f = {(uint8_t *)malloc((size_t)L * L * 3), L};
  memset(f.px, 255, (size_t)L * L * 3); /* screen.fill(WHITE) */
  const double scale = (double)L / fs;  /* screenDims / fovSize */
  for (int i = 0; i < n; i++) { /* drawSingleCell (rgbGenerator.py:36-53) */
    const Cell *c = objs[i].c;
    uint8_t col[3], rim[3];
    if (objs[i].kind == 3) player_rgb(c->player, seed, col);
    else if (objs[i].kind == 2) { col[0] = 0; col[1] = 255; col[2] = 0; }
    else if (c->col >= 0) player_rgb(c->col, seed, col); /* a blob / blob-made pellet: its player's */
    else pellet_rgb(c->seq, seed, col);
    int rad = (int)(c->radius * scale);
    int x = (int)(int64_t)(((c->x - fx) + fs / 2) * scale), y = (int)(int64_t)(((c->y - fy) + fs / 2) * scale);
    if (rad >= 4) {
      sdl_filled_circle(&f, x, y, rad, col);
      if (objs[i].kind == 2) { rim[0] = rim[1] = rim[2] = 0; } /* viruses: black rim */
      else memcpy(rim, col, 3);
      sdl_aa_ellipse(&f, x, y, rad, rad, rim);
    } else {
      sdl_filled_ellipse(&f, x, y, rad, rad, col); /* pygame.draw.circle(width 0) */
    }
  }
  for (int x = 0; x < L; x++) /* surfarray.array3d: [x][y][rgb] */
    for (int y = 0; y < L; y++) memcpy(out + ((size_t)x * L + y) * 3, f.px + ((size_t)y * L + x) * 3, 3);
  free(f.px);
  free(objs);
  cv_free(&q);
}

/* ------------------------------------------------------------ API ---- */
int oracle_pixels(void *h, int L, uint64_t seed, uint8_t *out) {
  Oracle *O = (Oracle *)h;
  for (int a = 0; a < O->A; a++) {
    Arena *A = &O->ar[a];
    for (int p = 0; p < A->B; p++) pixels_one(A, p, L, seed, out + (size_t)L * L * 3 * ((size_t)a * A->B + p));
  }
  return 0;
}

static int obs_len(const aigar_config *c) {
  int G = c->grid_squares ? c->grid_squares : 11, n = 0, e = 0;
  if (c->obs_channels & AIGAR_OBS_SIMPLE) return 12;
  for (int b = 0; b < 10; b++) n += (c->obs_channels >> b) & 1;
  e += (c->obs_extras & AIGAR_EX_LAST_FOV) ? 1 : 0;
  e += (c->obs_extras & AIGAR_EX_FOV) ? 1 : 0;
  e += (c->obs_extras & AIGAR_EX_MASS) ? 1 : 0;
  e += (c->obs_extras & AIGAR_EX_LAST_ACT) ? 4 : 0;
  e += (c->obs_extras & AIGAR_EX_2LAST_ACT) ? 4 : 0;
  return G * G * n + e;
}

static void arena_free_world(Arena *A) {
  for (int p = 0; p < A->B; p++) {
    for (int i = 0; i < A->pl[p].cells.n; i++) free(A->pl[p].cells.a[i]);
    A->pl[p].cells.n = 0;
  }
  for (int i = 0; i < A->pellets.n; i++) free(A->pellets.a[i]);
  for (int i = 0; i < A->blobs.n; i++) free(A->blobs.a[i]);
  for (int i = 0; i < A->viruses.n; i++) free(A->viruses.a[i]);
  for (int i = 0; i < A->grave.n; i++) free(A->grave.a[i]);
  A->pellets.n = A->blobs.n = A->viruses.n = A->grave.n = 0;
  A->n_dead = 0;
  hash_free(&A->ph); hash_free(&A->bh); hash_free(&A->plh); hash_free(&A->vh);
}
static void arena_new_hashes(Arena *A) {
  hash_free(&A->ph); hash_free(&A->bh); hash_free(&A->plh); hash_free(&A->vh);
  hash_init(&A->ph, A->size, HASH_BUCKET_SIZE, 0, 0);
  hash_init(&A->bh, A->size, HASH_BUCKET_SIZE, 0, 0);
  hash_init(&A->plh, A->size, HASH_BUCKET_SIZE, 0, 0);
  hash_init(&A->vh, A->size, HASH_BUCKET_SIZE, 0, 0);
}
static void arena_reset_obs_state(Oracle *O, Arena *A) {
  size_t GG = (size_t)A->G * A->G;
  memset(A->obs_fov, 0, sizeof(double) * A->B);
  memset(A->self_lf, 0, sizeof(double) * GG * A->B);
  memset(A->self_slf, 0, sizeof(double) * GG * A->B);
  memset(A->enemy_lf, 0, sizeof(double) * GG * A->B);
  memset(A->enemy_slf, 0, sizeof(double) * GG * A->B);
  (void)O;
}

void *oracle_create(const aigar_config *cfg) {
  if (!cfg || cfg->n_arenas < 1 || cfg->bots_per_arena < 1) {
    set_err("bad config");
    return NULL;
  }
  Oracle *O = (Oracle *)calloc(1, sizeof(Oracle));
  O->cfg = *cfg;
  O->A = cfg->n_arenas;
  O->L = obs_len(cfg);
  O->ar = (Arena *)calloc(O->A, sizeof(Arena));
  for (int a = 0; a < O->A; a++) {
    Arena *A = &O->ar[a];
    A->idx = a;
    A->B = cfg->bots_per_arena;
    A->size = cfg->field_size > 0 ? cfg->field_size : (int)(75 * sqrt((double)A->B));
    A->virus_enabled = cfg->virus_enabled;
    A->G = cfg->grid_squares ? cfg->grid_squares : 11;
    A->max_pellets = cfg->max_pellets >= 0 ? cfg->max_pellets : (double)A->size * A->size * 0.015;
    A->max_viruses = cfg->max_viruses >= 0 ? cfg->max_viruses : (double)A->size * A->size * 0.00005;
    A->rng_mode = cfg->rng_mode;
    A->pl = (Player *)calloc(A->B, sizeof(Player));
    A->dead = (int *)malloc(sizeof(int) * (A->B + 1));
    size_t GG = (size_t)A->G * A->G;
    A->obs_fov = (double *)calloc(A->B, sizeof(double));
    A->self_lf = (double *)calloc(GG * A->B, sizeof(double));
    A->self_slf = (double *)calloc(GG * A->B, sizeof(double));
    A->enemy_lf = (double *)calloc(GG * A->B, sizeof(double));
    A->enemy_slf = (double *)calloc(GG * A->B, sizeof(double));
    A->act_cur = (double *)calloc(4 * (size_t)A->B, sizeof(double));
    A->act_prev = (double *)calloc(4 * (size_t)A->B, sizeof(double));
    for (int p = 0; p < A->B; p++) {
      A->pl[p].alive = 1; /* Field.addPlayer -> setAlive (field.py:414-416) */
      A->pl[p].cmdx = -1;
      A->pl[p].cmdy = -1;
    }
    arena_new_hashes(A);
  }
  return O;
}
void oracle_destroy(void *h) {
  Oracle *O = (Oracle *)h;
  if (!O) return;
  for (int a = 0; a < O->A; a++) {
    Arena *A = &O->ar[a];
    arena_free_world(A);
    for (int p = 0; p < A->B; p++) cv_free(&A->pl[p].cells);
    cv_free(&A->pellets); cv_free(&A->blobs); cv_free(&A->viruses); cv_free(&A->grave);
    free(A->pl); free(A->dead); free(A->ev); free(A->split_lh);
    free(A->obs_fov); free(A->self_lf); free(A->self_slf); free(A->enemy_lf); free(A->enemy_slf);
    free(A->act_cur); free(A->act_prev);
  }
  free(O->ar);
  free(O);
}

/* Field.initialize()/reset() (field.py:57-83) after numpy.random.seed(seed) */
int oracle_reset(void *h, uint64_t seed) {
  Oracle *O = (Oracle *)h;
  for (int a = 0; a < O->A; a++) {
    Arena *A = &O->ar[a];
    arena_free_world(A);
    arena_new_hashes(A);
    A->seq_next = 0;
    A->tick = 0;
    A->n_ev = 0;
    A->err = 0;
    mt_seed(&A->mt, (uint32_t)(seed + (uint64_t)a));
    A->key[0] = seed;
    A->key[1] = ((uint64_t)a << 32) | 0x9E3779B9ull;
    A->ctr_pellet = A->ctr_virus = 0;
    for (int p = 0; p < A->B; p++) initialize_player(A, p, 0);
    spawn_stuff(A);
    arena_reset_obs_state(O, A);
  }
  return 0;
}

int oracle_set_commands(void *h, const double *cmd) { /* Player.setCommands */
  Oracle *O = (Oracle *)h;
  for (int a = 0; a < O->A; a++)
    for (int p = 0; p < O->ar[a].B; p++) {
      const double *c = cmd + 4 * ((size_t)a * O->ar[a].B + p);
      Player *P = &O->ar[a].pl[p];
      P->cmdx = c[0];
      P->cmdy = c[1];
      P->do_split = c[2] != 0;
      P->do_eject = c[3] != 0;
    }
  return 0;
}
int oracle_set_actions(void *h, const double *cur, const double *prev) {
  Oracle *O = (Oracle *)h;
  for (int a = 0; a < O->A; a++) {
    Arena *A = &O->ar[a];
    size_t off = 4 * (size_t)a * A->B;
    if (cur) memcpy(A->act_cur, cur + off, sizeof(double) * 4 * A->B);
    if (prev) memcpy(A->act_prev, prev + off, sizeof(double) * 4 * A->B);
  }
  return 0;
}
int oracle_step(void *h, int n) {
  Oracle *O = (Oracle *)h;
  for (int a = 0; a < O->A; a++) {
    Arena *A = &O->ar[a];
    A->n_ev = 0;
    for (int t = 0; t < n; t++) {
      field_update(A);
      if (A->err) return -1;
    }
  }
  return 0;
}
int oracle_obs_len(void *h) { return ((Oracle *)h)->L; }
int oracle_observe(void *h, double *out) {
  Oracle *O = (Oracle *)h;
  for (int a = 0; a < O->A; a++) {
    Arena *A = &O->ar[a];
    for (int p = 0; p < A->B; p++) observe_one(O, A, p, out + (size_t)O->L * ((size_t)a * A->B + p));
  }
  return 0;
}
int oracle_observe_one(void *h, int arena, int p, double *out) {
  Oracle *O = (Oracle *)h;
  observe_one(O, &O->ar[arena], p, out);
  return 0;
}
int oracle_player_stats(void *h, double *out) {
  Oracle *O = (Oracle *)h;
  for (int a = 0; a < O->A; a++) {
    Arena *A = &O->ar[a];
    for (int p = 0; p < A->B; p++) {
      double *o = out + 5 * ((size_t)a * A->B + p);
      Player *P = &A->pl[p];
      o[0] = P->alive;
      o[1] = player_total_mass(P);
      if (P->alive) {
        player_fov_pos(P, &o[2], &o[3]);
        o[4] = player_fov_size(P);
      } else {
        o[2] = o[3] = o[4] = NAN;
      }
    }
  }
  return 0;
}
int oracle_get_events(void *h, int arena, int64_t *out, int cap) {
  Arena *A = &((Oracle *)h)->ar[arena];
  const int n = A->n_ev < cap ? A->n_ev : cap;
  if (out && n > 0) memcpy(out, A->ev, sizeof(int64_t) * 4 * (size_t)n);  /* (no events: A->ev may be NULL) */
  return A->n_ev;
}
int oracle_reset_obs_state(void *h) {
  Oracle *O = (Oracle *)h;
  for (int a = 0; a < O->A; a++) arena_reset_obs_state(O, &O->ar[a]);
  return 0;
}
/* Bot.reset (bot.py:125-164, NN branch) for the players with mask[p] != 0 of
 * every arena (player index a * B + p): the history grids restart at zero and
 * fovSize / lastFovSize at 0.  NULL mask: every player. */
int oracle_reset_bots(void *h, const uint8_t *mask) {
  Oracle *O = (Oracle *)h;
  for (int a = 0; a < O->A; a++) {
    Arena *A = &O->ar[a];
    const size_t GG = (size_t)A->G * A->G;
    for (int p = 0; p < A->B; p++) {
      if (mask && !mask[(size_t)a * A->B + p]) continue;
      A->obs_fov[p] = 0;
      memset(A->self_lf + p * GG, 0, sizeof(double) * GG);
      memset(A->self_slf + p * GG, 0, sizeof(double) * GG);
      memset(A->enemy_lf + p * GG, 0, sizeof(double) * GG);
      memset(A->enemy_slf + p * GG, 0, sizeof(double) * GG);
    }
  }
  return 0;
}

static void mark_hashed(const Hash *h) {
  for (int i = 0; i < h->rows * h->cols; i++)
    for (int j = 0; j < h->b[i].n; j++) h->b[i].a[j]->mark = 1;
}

int oracle_get_state(void *h, int arena, aigar_state *st) {
  Oracle *O = (Oracle *)h;
  Arena *A = &O->ar[arena];
  int nc = 0;
  for (int p = 0; p < A->B; p++) nc += A->pl[p].cells.n;
  int cap_c = st->n_cells, cap_p = st->n_pellets, cap_b = st->n_blobs, cap_v = st->n_viruses, cap_d = st->n_dead;
  st->n_players = A->B;
  st->field_size = A->size;
  st->virus_enabled = A->virus_enabled;
  st->rng_mode = A->rng_mode;
  st->seq_next = A->seq_next;
  st->tick = A->tick;
  st->max_pellets = A->max_pellets;
  st->max_viruses = A->max_viruses;
  st->philox_key[0] = A->key[0];
  st->philox_key[1] = A->key[1];
  st->ctr_pellet = A->ctr_pellet;
  st->ctr_virus = A->ctr_virus;
  memcpy(st->mt_key, A->mt.key, sizeof A->mt.key);
  st->mt_pos = A->mt.pos;
  st->n_cells = nc;
  st->n_pellets = A->pellets.n;
  st->n_blobs = A->blobs.n;
  st->n_viruses = A->viruses.n;
  st->n_dead = A->n_dead;
  if (!st->cells_f) return 0;
  if (cap_c < nc || cap_p < A->pellets.n || cap_b < A->blobs.n || cap_v < A->viruses.n || cap_d < A->n_dead) {
    set_err("get_state: caller arrays too small");
    return -1;
  }
  for (int p = 0; p < A->B; p++)
    for (int i = 0; i < A->pl[p].cells.n; i++) A->pl[p].cells.a[i]->mark = 0;
  for (int i = 0; i < A->viruses.n; i++) A->viruses.a[i]->mark = 0;
  mark_hashed(&A->plh);
  mark_hashed(&A->vh);
  for (int p = 0; p < A->B; p++) {
    Player *P = &A->pl[p];
    st->players_f[2 * p] = P->cmdx;
    st->players_f[2 * p + 1] = P->cmdy;
    int64_t *pi = st->players_i + 5 * p;
    pi[0] = P->alive; pi[1] = P->respawn; pi[2] = P->do_split; pi[3] = P->do_eject; pi[4] = P->cells.n;
  }
  int k = 0;
  for (int p = 0; p < A->B; p++)
    for (int i = 0; i < A->pl[p].cells.n; i++, k++) {
      Cell *c = A->pl[p].cells.a[i];
      double *f = st->cells_f + 9 * k;
      f[0] = c->x; f[1] = c->y; f[2] = c->mass; f[3] = c->radius; f[4] = c->vx; f[5] = c->vy;
      f[6] = c->svx; f[7] = c->svy; f[8] = c->merge_time;
      int64_t *q = st->cells_i + 4 * k;
      q[0] = p; q[1] = c->svc; q[2] = c->seq; q[3] = c->mark;
    }
  Cell **ps = (Cell **)malloc(sizeof(Cell *) * (A->pellets.n + 1));
  memcpy(ps, A->pellets.a, sizeof(Cell *) * A->pellets.n);
  qsort(ps, A->pellets.n, sizeof(Cell *), cmp_seq);
  for (int i = 0; i < A->pellets.n; i++) {
    double *f = st->pellets_f + 4 * i;
    f[0] = ps[i]->x; f[1] = ps[i]->y; f[2] = ps[i]->mass; f[3] = ps[i]->radius;
    st->pellets_seq[i] = ps[i]->seq;
    if (st->pellets_col) st->pellets_col[i] = ps[i]->col;
  }
  free(ps);
  for (int i = 0; i < A->blobs.n; i++) {
    Cell *c = A->blobs.a[i];
    double *f = st->blobs_f + 8 * i;
    f[0] = c->x; f[1] = c->y; f[2] = c->mass; f[3] = c->radius; f[4] = c->vx; f[5] = c->vy; f[6] = c->svx; f[7] = c->svy;
    int64_t *q = st->blobs_i + 3 * i;
    q[0] = c->svc; q[1] = c->seq; q[2] = c->ejecter_seq;
    if (st->blobs_col) st->blobs_col[i] = c->col;
  }
  for (int i = 0; i < A->viruses.n; i++) {
    Cell *c = A->viruses.a[i];
    double *f = st->viruses_f + 8 * i;
    f[0] = c->x; f[1] = c->y; f[2] = c->mass; f[3] = c->radius; f[4] = c->vx; f[5] = c->vy; f[6] = c->svx; f[7] = c->svy;
    int64_t *q = st->viruses_i + 3 * i;
    q[0] = c->svc; q[1] = c->seq; q[2] = c->mark;
  }
  for (int i = 0; i < A->n_dead; i++) st->dead[i] = A->dead[i];
  return 0;
}

/* Rebuild an arena from a snapshot.  Hash contents are reconstructed the way
 * the reference has them between ticks: pellets all hashed; player / virus
 * hash = entities flagged in_hash (footprints from current pos/radius); blob
 * hash = every blob (rebuilt each tick after creation). */
int oracle_load_state(void *h, int arena, const aigar_state *st) {
  Oracle *O = (Oracle *)h;
  Arena *A = &O->ar[arena];
  if (st->n_players != A->B) {
    set_err("load_state: n_players %d != %d", st->n_players, A->B);
    return -1;
  }
  arena_free_world(A);
  A->size = st->field_size;
  A->virus_enabled = st->virus_enabled;
  A->rng_mode = st->rng_mode;
  A->max_pellets = st->max_pellets;
  A->max_viruses = st->max_viruses;
  arena_new_hashes(A);
  A->seq_next = st->seq_next;
  A->tick = st->tick;
  A->key[0] = st->philox_key[0];
  A->key[1] = st->philox_key[1];
  A->ctr_pellet = st->ctr_pellet;
  A->ctr_virus = st->ctr_virus;
  memcpy(A->mt.key, st->mt_key, sizeof A->mt.key);
  A->mt.pos = st->mt_pos;
  A->n_ev = 0;
  A->err = 0;
  for (int p = 0; p < A->B; p++) {
    Player *P = &A->pl[p];
    P->cmdx = st->players_f[2 * p];
    P->cmdy = st->players_f[2 * p + 1];
    const int64_t *pi = st->players_i + 5 * p;
    P->alive = (int)pi[0]; P->respawn = (int)pi[1]; P->do_split = (int)pi[2]; P->do_eject = (int)pi[3];
    P->cells.n = 0;
  }
  for (int k = 0; k < st->n_cells; k++) {
    const double *f = st->cells_f + 9 * k;
    const int64_t *q = st->cells_i + 4 * k;
    Cell *c = (Cell *)calloc(1, sizeof(Cell));
    c->x = f[0]; c->y = f[1]; c->mass = f[2]; c->radius = f[3]; c->vx = f[4]; c->vy = f[5];
    c->svx = f[6]; c->svy = f[7]; c->merge_time = f[8];
    c->player = (int)q[0]; c->svc = (int)q[1]; c->seq = q[2]; c->alive = 1; c->ejecter_seq = -1;
    cv_push(&A->pl[c->player].cells, c);
    if (q[3]) hash_insert(&A->plh, c);
  }
  for (int i = 0; i < st->n_pellets; i++) {
    const double *f = st->pellets_f + 4 * i;
    Cell *c = (Cell *)calloc(1, sizeof(Cell));
    c->x = f[0]; c->y = f[1]; c->mass = f[2]; c->radius = f[3]; c->seq = st->pellets_seq[i];
    c->player = -1; c->alive = 1; c->ejecter_seq = -1;
    c->col = st->pellets_col ? (int)st->pellets_col[i] : -1;
    cv_push(&A->pellets, c);
    hash_insert(&A->ph, c);
  }
  for (int i = 0; i < st->n_blobs; i++) {
    const double *f = st->blobs_f + 8 * i;
    const int64_t *q = st->blobs_i + 3 * i;
    Cell *c = (Cell *)calloc(1, sizeof(Cell));
    c->x = f[0]; c->y = f[1]; c->mass = f[2]; c->radius = f[3]; c->vx = f[4]; c->vy = f[5]; c->svx = f[6]; c->svy = f[7];
    c->svc = (int)q[0]; c->seq = q[1]; c->ejecter_seq = q[2]; c->player = -1; c->alive = 1;
    c->col = st->blobs_col ? (int)st->blobs_col[i] : -1;
    cv_push(&A->blobs, c);
    hash_insert(&A->bh, c);
  }
  for (int i = 0; i < st->n_viruses; i++) {
    const double *f = st->viruses_f + 8 * i;
    const int64_t *q = st->viruses_i + 3 * i;
    Cell *c = (Cell *)calloc(1, sizeof(Cell));
    c->x = f[0]; c->y = f[1]; c->mass = f[2]; c->radius = f[3]; c->vx = f[4]; c->vy = f[5]; c->svx = f[6]; c->svy = f[7];
    c->svc = (int)q[0]; c->seq = q[1]; c->ejecter_seq = -1; c->player = -1; c->alive = 1;
    cv_push(&A->viruses, c);
    if (q[2]) hash_insert(&A->vh, c);
  }
  A->n_dead = st->n_dead;
  for (int i = 0; i < st->n_dead; i++) A->dead[i] = (int)st->dead[i];
  return 0;
}

/* overwrite the MT19937 stream (bots draw from the same numpy stream outside
 * Field.update in the reference; the harness replays their consumption) */
int oracle_set_mt(void *h, int arena, const uint32_t *key, int pos) {
  Arena *A = &((Oracle *)h)->ar[arena];
  memcpy(A->mt.key, key, sizeof A->mt.key);
  A->mt.pos = pos;
  return 0;
}

/* Model.takeBotActions for an all-Greedy population (bot.py:252-269) */
int oracle_policy_greedy(void *h, int greedy_split) {
  Oracle *O = (Oracle *)h;
  for (int a = 0; a < O->A; a++)
    for (int p = 0; p < O->ar[a].B; p++) greedy_move(&O->ar[a], p, greedy_split);
  return 0;
}
/* explicit splitLikelihoods (e.g. replayed from numpy's stream); NULL restores the Philox-derived ones */
int oracle_set_split_likelihood(void *h, int arena, const int *lh) {
  Arena *A = &((Oracle *)h)->ar[arena];
  if (!lh) {
    free(A->split_lh);
    A->split_lh = NULL;
    return 0;
  }
  if (!A->split_lh) A->split_lh = (int *)malloc(sizeof(int) * A->B);
  memcpy(A->split_lh, lh, sizeof(int) * A->B);
  return 0;
}
