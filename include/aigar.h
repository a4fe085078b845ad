/*
 * aigar.h -- C-ABI of the MI355X agar.io environment stepper (libaigar_hip.so).
 *
 * Drop-in boundary for the reference's hot path.  The
 * reference has no FFI: its boundary is the Python object API of
 * src/model/{field,model,player,cell,bot}.py.  Each entry point below names the
 * reference call it replaces; the Python facade in aigar_amd/ binds them with
 * ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every call returns int: 0 = OK, < 0 = error; aigar_last_error() gives the
 *    message (thread-local).  No C++ exception crosses the ABI.
 *  - One handle = one HIP device + one HIP stream.  Calls on a handle are
 *    serialised by the caller.  Handles on different devices may run
 *    concurrently (one process per GPU).
 *  - A handle owns n_arenas independent arenas ("fields") of bots_per_arena
 *    players each; arrays that span all arenas are arena-major:
 *    index = arena * bots_per_arena + player.
 *  - on_device = 0: caller passes host pointers (copied during the call);
 *    on_device = 1: device pointers on the handle's stream (e.g. torch tensors
 *    via data_ptr(); adopt torch's stream with aigar_set_stream()).
 *  - All state is fp64, like the reference (Python floats / numpy float64).
 */
#ifndef AIGAR_H
#define AIGAR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AIGAR_ABI_VERSION 5

/* random number stream of the world (spawns, explosion angles) */
#define AIGAR_RNG_PHILOX 0   /* Philox4x64-10 keyed by (seed, site, index): device + oracle */
#define AIGAR_RNG_MT19937 1  /* numpy legacy MT19937 stream, reference-exact: oracle only */

/* observation channels, in the reference's stacking order (bot.py:459-495) */
#define AIGAR_OBS_PELLET     0x001u  /* PELLET_GRID: pellet mass sum      */
#define AIGAR_OBS_SELF       0x002u  /* SELF_GRID: biggest own cell mass  */
#define AIGAR_OBS_WALL       0x004u  /* WALL_GRID: wall fraction (3 dp)   */
#define AIGAR_OBS_ENEMY      0x008u  /* ENEMY_GRID: biggest enemy mass    */
#define AIGAR_OBS_ALL        0x010u  /* ALL_PLAYER_GRID                   */
#define AIGAR_OBS_VIRUS      0x020u  /* VIRUS_GRID                        */
#define AIGAR_OBS_SELF_SLF   0x040u  /* SELF_GRID_SLF  (second-last frame)*/
#define AIGAR_OBS_SELF_LF    0x080u  /* SELF_GRID_LF   (last frame)       */
#define AIGAR_OBS_ENEMY_SLF  0x100u  /* ENEMY_GRID_SLF                    */
#define AIGAR_OBS_ENEMY_LF   0x200u  /* ENEMY_GRID_LF                     */
/* GRID_VIEW_ENABLED = False (networkParameters.py:119): getSimpleStateRepresentation
 * (bot.py:511-547) instead of the grids -- 12 values per bot (first own cell,
 * closest enemy cell, closest pellet, visible field edges); no grids, no extras */
#define AIGAR_OBS_SIMPLE     0x400u
/* extra inputs, in getAdditionalFeatures order (bot.py:302-323) */
#define AIGAR_EX_LAST_FOV    0x01u
#define AIGAR_EX_FOV         0x02u
#define AIGAR_EX_MASS        0x04u
#define AIGAR_EX_LAST_ACT    0x08u
#define AIGAR_EX_2LAST_ACT   0x10u

/* event codes (tick-ordered the way the reference performs them) */
#define AIGAR_EV_MERGE           1  /* (bigger seq, smaller seq)     field.py:372  */
#define AIGAR_EV_VIRUS_EAT_BLOB  2  /* (virus seq, blob seq)         field.py:316  */
#define AIGAR_EV_VIRUS_SPLIT     3  /* (virus seq, new virus seq)    field.py:318  */
#define AIGAR_EV_CELL_EAT_VIRUS  4  /* (cell seq, virus seq)         field.py:333  */
#define AIGAR_EV_EXPLODE         5  /* (cell seq, n new cells)       field.py:350  */
#define AIGAR_EV_CELL_EAT_PELLET 6  /* (cell seq, pellet seq)        field.py:327  */
#define AIGAR_EV_CELL_EAT_BLOB   7  /* (cell seq, blob seq)          field.py:330  */
#define AIGAR_EV_CELL_EAT_CELL   8  /* (eater seq, eaten seq)        field.py:346  */
#define AIGAR_EV_PLAYER_DEATH    9  /* (player index, last cell seq) field.py:386  */
#define AIGAR_EV_RESPAWN        10  /* (player index, new cell seq)  field.py:277  */

#define AIGAR_FLAG_EVENTS 0x1       /* record the event log of each step */
/* tile_flags: decide only the cells this tile owns (the others wait for their
 * owners' messages) -- the strictest exchange pattern, used by the tests */
#define AIGAR_TILE_OWNED_ONLY 0x1
/* a 1 x 1 "tiled" handle: the whole field is one tile that still runs the tile
 * passes and the exchange (a 1-rank RCCL communicator: the one-GPU test of the
 * C4 exchange path) */
#define AIGAR_TILE_FORCE 0x2

typedef struct aigar_handle aigar_handle;

typedef struct aigar_config {
  int32_t n_arenas;        /* independent fields per handle (batched-env mode)        */
  int32_t bots_per_arena;  /* players per field                                       */
  int32_t field_size;      /* 0 -> int(75 * sqrt(bots)) (field.py:58)                 */
  int32_t virus_enabled;   /* Field(virusEnabled) (field.py:30, VIRUS_SPAWN)          */
  double max_pellets;      /* < 0 -> size*size*0.015 (field.py:65, parameters.py:16)  */
  double max_viruses;      /* < 0 -> size*size*5e-5 (field.py:66, parameters.py:17)   */
  int32_t grid_squares;    /* GRID_SQUARES_PER_FOV (networkParameters.py:97), or the CNN
                            * grid view's CNN_INPUT_DIM_* (bot.py:103-111: 42 / 84);
                            * 0 -> 11; at most 127                                     */
  uint32_t obs_channels;   /* AIGAR_OBS_* mask (networkParameters.py:76-96)           */
  uint32_t obs_extras;     /* AIGAR_EX_* mask (networkParameters.py:91-95)            */
  int32_t rng_mode;        /* AIGAR_RNG_*                                             */
  int32_t device;          /* HIP device ordinal                                      */
  int32_t pellet_cap;      /* 0 -> max_pellets + blob_cap + 64                        */
  int32_t blob_cap;        /* 0 -> 4 * bots + 256                                     */
  int32_t virus_cap;       /* 0 -> 2 * max_viruses + 64                               */
  int32_t event_cap;       /* events kept per arena per step (0 -> 65536)             */
  int32_t flags;           /* AIGAR_FLAG_*                                            */
  /* C4: one arena tiled 2-D over tile_x * tile_y handles, one per GPU (SURVEY.md
   * §8e).  1 x 1 (or 0 x 0) = untiled.  A tiled handle needs n_arenas == 1.     */
  int32_t tile_x, tile_y;  /* tiles along x and y                                     */
  int32_t tile_id;         /* this handle's tile, row-major: ty * tile_x + tx         */
  int32_t tile_halo;       /* pellets held beyond the tile, field units (0 -> 400;    *
                            * at least 140: an owned cell's reach; 370 covers any view) */
  int32_t tile_cap;        /* records per exchange message (0 -> 2048)                */
  int32_t tile_flags;      /* AIGAR_TILE_*                                            */
} aigar_config;

/*
 * Snapshot of one arena, the unit of parity.  Record layouts (row-major):
 *   players_f [n_players][2]  command point x, y          (player.py:99-102)
 *   players_i [n_players][5]  alive, respawnTime, doSplit, doEject, #cells
 *   cells_f   [n_cells][9]    x y mass radius vx vy svx svy mergeTime (cell.py:21-45)
 *   cells_i   [n_cells][4]    owner, splitVelocityCounter, seq, in_player_hash
 *             cells are grouped by owner in player order, each group in the
 *             player's cell-list order
 *   pellets_f [n_pellets][4]  x y mass radius, sorted by seq
 *   pellets_seq [n_pellets]
 *   blobs_f   [n_blobs][8]    x y mass radius vx vy svx svy (list order)
 *   blobs_i   [n_blobs][3]    svc, seq, ejecter cell seq
 *   viruses_f [n_viruses][8]  as blobs
 *   viruses_i [n_viruses][3]  svc, seq, in_virus_hash
 *   dead      [n_dead]        deadPlayers list (player indices, in order)
 * seq = creation sequence number of the Cell object (canonical order).
 * aigar_get_state: with NULL arrays only the counts are filled; otherwise the
 * n_* fields give the capacities of the caller's arrays on input.
 */
typedef struct aigar_state {
  int32_t n_players, field_size, virus_enabled, rng_mode;
  int64_t seq_next, tick;
  double max_pellets, max_viruses;
  uint64_t philox_key[2];
  uint64_t ctr_pellet, ctr_virus;
  uint32_t mt_key[624];
  int32_t mt_pos;
  int32_t n_cells, n_pellets, n_blobs, n_viruses, n_dead;
  double *players_f;
  int64_t *players_i;
  double *cells_f;
  int64_t *cells_i;
  double *pellets_f;
  int64_t *pellets_seq;
  double *blobs_f;
  int64_t *blobs_i;
  double *viruses_f;
  int64_t *viruses_i;
  int64_t *dead;
  /* optional (NULL: not exported / -1 on import): the player whose colour the
   * object carries -- an ejected blob its ejecting player's (field.py:141,
   * cell.py:219), a pellet made from a blob the blob's (field.py:110) -- or -1
   * for a pellet's / orphan blob's colour of its own (cell.py:31) */
  int64_t *pellets_col;  /* [n_pellets], in pellets_seq order */
  int64_t *blobs_col;    /* [n_blobs] */
} aigar_state;

const char *aigar_last_error(void);
int aigar_abi_version(void);

/* Field(virusEnabled) + Model bookkeeping: allocate all device buffers.
 * replaces model.py:51-73 / field.py:30-46 */
int aigar_create(const aigar_config *cfg, aigar_handle **out);
int aigar_destroy(aigar_handle *h);

/* Field.initialize()/Field.reset(): spawn every player, pellets, viruses.
 * replaces field.py:57-83 (model.py:90-98) */
int aigar_reset(aigar_handle *h, uint64_t seed);

/* Player.setCommands(x, y, split, eject) for every player: cmd[A*B][4].
 * replaces player.py:99-102 (called from bot.py:550-577) */
int aigar_set_commands(aigar_handle *h, const double *cmd, int on_device);

/* Synthetic bot population on the device (benchmark / smoke driver): every
 * alive player draws an action in [0,1]^2 mapped through the reference's
 * set_command_point (bot.py:550-577) and splits/ejects with p_split/p_eject.
 * The draws are Philox-keyed by (world key, seed, tick, player): a function of
 * the state, not of how many times the policy was called. */
int aigar_policy_random(aigar_handle *h, double p_split, double p_eject, uint64_t seed);

/* Model.takeBotActions for Greedy bots (bot.py:252-269 -> make_greedy_bot_move
 * bot.py:579-633 -> set_command_point bot.py:550-577): sets the command of every
 * alive player whose mask byte is non-zero (mask NULL: every player).
 * greedy_split = ENABLE_GREEDY_SPLIT (networkParameters.py:17).  Random draws
 * (fallback target, split dice) come from the Philox stream. */
int aigar_policy_greedy(aigar_handle *h, int greedy_split, const uint8_t *mask, int on_device);
/* Greedy bots' splitLikelihood (bot.py:93), [bots_per_arena] for one arena;
 * NULL: derive them from the Philox key (the default). */
int aigar_set_split_likelihood(aigar_handle *h, int arena, const int32_t *lh);

/* External (learner) actions for every player: act[A*B][n_act], n_act = 2, 3 or 4,
 * mapped through set_command_point (bot.py:550-577).  skipping: a frame-skip
 * frame, split/eject dropped (bot.py:266-267); record: a decision frame, the
 * observation's last / second-last action extras advance (bot.py:180-193). */
int aigar_apply_actions(aigar_handle *h, const double *act, int n_act, int enable_split, int skipping, int record,
                        int on_device);

/* Bot.getReward (bot.py:654-667) for every player into out[A*B] (NaN = None);
 * update_last: lastMass <- total mass for live players (end of move_NN). */
typedef struct aigar_reward_params {
  int32_t mass_as_reward;  /* MASS_AS_REWARD (networkParameters.py:50) */
  int32_t pad;
  double reward_term;      /* REWARD_TERM  */
  double death_term;       /* DEATH_TERM   */
  double death_factor;     /* DEATH_FACTOR */
  double reward_scale;     /* REWARD_SCALE */
} aigar_reward_params;
int aigar_rewards(aigar_handle *h, double *out, const aigar_reward_params *p, int update_last, int on_device);

/* One learner decision for every player -- the NN bots' move_NN / updateRewards
 * / frame skipping (bot.py:166-233) batched, as aigar.py:performModelSteps
 * drives them: act[A*B][n_act] (n_act 2..4, DEVICE pointer) goes through
 * set_command_point (as aigar_apply_actions) and is held for skip + 1 ticks
 * (FRAME_SKIP_RATE; split/eject dropped on the skipped ticks), reward_out[A*B]
 * (DEVICE) gets the window's summed getReward (None counts 0; lastMass advances
 * at the end), obs_out (DEVICE, as aigar_observe) every bot's observation.  The
 * whole decision is one hipGraph replay (re-captured when a pointer or a
 * parameter changes). */
int aigar_env_step(aigar_handle *h, const double *act, int n_act, int enable_split, int skip,
                   const aigar_reward_params *p, double *reward_out, void *obs_out, int dtype);

/* n_ticks x Field.update() with the current commands (field.py:85-92). */
int aigar_step(aigar_handle *h, int n_ticks);

/* One whole batched env step, n_steps times: the bot policy (Model.takeBotActions,
 * model.py:100-105), Field.update() (field.py:85-92) and, when obs_out is not
 * NULL, every bot's getStateRepresentation (bot.py:272-299) into the DEVICE
 * buffer obs_out[A*B][aigar_obs_len()] (dtype as aigar_observe).  The step is
 * captured once as a single hipGraph (re-captured when the parameters or the
 * buffer change) and replayed, so no host round trip separates the phases;
 * a second graph holds AIGAR_RUN_UNROLL copies of the step (environment,
 * read at aigar_create; default 4) and carries n_steps / 4 of them (the rest
 * one step per replay) -- the same kernels in the same order, one graph launch
 * per 4 steps.
 * policy: AIGAR_POLICY_NONE keeps the current commands; RANDOM is
 * aigar_policy_random(p_split, p_eject, seed);
 * GREEDY is aigar_policy_greedy for every player.  With AIGAR_FLAG_EVENTS the
 * event log holds the events of all n_steps of the call. */
/* player roles of a batched population (aigar_set_roles) */
#define AIGAR_ROLE_NN     0  /* actions from the caller (learner): aigar_apply_actions / aigar_env_step */
#define AIGAR_ROLE_GREEDY 1  /* Greedy bot on the device (bot.py:579-633)                              */
#define AIGAR_ROLE_RANDOM 2  /* Random bot on the device (bot.py:243-249)                              */
#define AIGAR_POLICY_NONE   0
#define AIGAR_POLICY_RANDOM 1
#define AIGAR_POLICY_GREEDY 2
typedef struct aigar_run_params {
  int32_t policy;        /* AIGAR_POLICY_*                                   */
  int32_t greedy_split;  /* ENABLE_GREEDY_SPLIT (networkParameters.py:17)    */
  double p_split;        /* RANDOM: split probability per bot-tick           */
  double p_eject;        /* RANDOM: eject probability per bot-tick           */
  uint64_t seed;         /* RANDOM: Philox salt                              */
} aigar_run_params;
int aigar_run(aigar_handle *h, int n_steps, const aigar_run_params *p, void *obs_out, int dtype);

/* Bot.getStateRepresentation() for every player (bot.py:272-497):
 * out[A*B][aigar_obs_len()] (dtype 0 = float64, 1 = float32); dead players get NaN.
 * Updates each bot's last-frame history grids like the reference does. */
int aigar_obs_len(aigar_handle *h);
int aigar_observe(aigar_handle *h, void *out, int dtype, int on_device);
/* The same for the players whose mask byte is non-zero only (mask on the host, or on
 * the device when mask_on_device): the others' rows stay as they are in out and
 * their last-frame history does not advance -- the reference computes a state only
 * for the NN bots that are not skipping a frame (bot.py:195-202). */
int aigar_observe_masked(aigar_handle *h, void *out, int dtype, int on_device, const uint8_t *mask,
                         int mask_on_device);

/* Mixed populations (aigar.py:767-780: NN bots trained among Greedy and Random
 * bots): roles[A*B] of AIGAR_ROLE_* (NULL: every player NN).  aigar_env_step then
 * moves the Greedy and Random bots itself every tick (the learner's actions apply to
 * the NN players only) and observes the NN players only. */
int aigar_set_roles(aigar_handle *h, const uint8_t *roles, int on_device);
typedef struct aigar_env_params {
  int32_t greedy_split;   /* ENABLE_GREEDY_SPLIT (networkParameters.py:17)            */
  int32_t random_skip;    /* Random bots draw a new action every FRAME_SKIP_RATE moves */
  int32_t random_split;   /* ENABLE_SPLIT: Random bots draw a split value             */
  int32_t random_eject;   /* ENABLE_EJECT: Random bots draw an eject value            */
  uint64_t salt;          /* Philox salt of the Random bots' draws                    */
} aigar_env_params;
int aigar_env_config(aigar_handle *h, const aigar_env_params *p);
/* One Model.takeBotActions for the Random bots only (make_random_bot_move +
 * set_command_point, bot.py:243-269), with the aigar_env_config parameters. */
int aigar_policy_random_bots(aigar_handle *h);
/* RGBGenerator.get_cnn_inputRGB (rgbGenerator.py:95-110) for every player: a
 * side x side frame (side <= 84; CNN_INPUT_DIM_* of networkParameters.py) of
 * the player's FOV, objects drawn in stable mass order with SDL_gfx circle
 * primitives.  dtype 2: uint8 RGB out[A*B][side][side][3] in pygame surfarray
 * order [x][y][rgb]; 0 / 1: float64 / float32 grayscale out[A*B][side][side]
 * (numpy.average with weights 0.298, 0.587, 0.114).  color_seed picks the
 * per-player / per-pellet colours (the reference draws them from numpy RNG,
 * cell.py:31, player.py:39).  Dead players get zeros (uint8) / NaN (gray). */
int aigar_observe_pixels(aigar_handle *h, void *out, int side, uint64_t color_seed, int dtype, int on_device);
/* bot.currentAction / bot.lastAction used by the action extras: [A*B][4] each (may be NULL). */
int aigar_set_actions(aigar_handle *h, const double *cur, const double *prev, int on_device);
/* Bot.reset (bot.py:125-164) for the players with mask[i] != 0 (NULL: all): the
 * NN bot's last / second-last self and enemy grids restart at zero and its
 * lastFovSize at 0, as model.resetBots() does between the collector's windows
 * (aigar.py:845-852, 833-838).  mask: NP bytes, host or (on_device) device. */
int aigar_reset_bots(aigar_handle *h, const uint8_t *mask, int on_device);

/* per-player summary [A*B][5]: alive, total mass (player.py:129), fov x, fov y, fov size
 * (player.py:156-167). */
int aigar_player_stats(aigar_handle *h, double *out, int on_device);

/* Snapshot / restore one arena (parity harness, checkpoint/resume). */
int aigar_get_state(aigar_handle *h, int arena, aigar_state *st);
int aigar_load_state(aigar_handle *h, int arena, const aigar_state *st);

/* Event log of the last aigar_step (AIGAR_FLAG_EVENTS): rows of (tick, code, a, b)
 * in reference order.  *n gets the count; returns < 0 if cap is too small. */
int aigar_get_events(aigar_handle *h, int arena, int64_t *out, int cap, int *n);

/*
 * C4 tiled arena (field.py:85-92, 200-253, 256-313).  Every tile
 * handle replays the whole tick on its replica of the players, cells, blobs and
 * viruses; it holds only the pellets of its tile plus the halo.  The eat phase
 * (field.py:207-222) is resolved per tile; the cells a tile owns (centre bucket
 * in the tile) report their outcomes in ONE message per pass, and the caller's
 * transport all-gathers the messages (RCCL all-gather over xGMI; in-process
 * device copies for tests):
 *   [Greedy bots (bot.py:579-633): aigar_tile_policy(h, greedy_split), the
 *    all-gather, aigar_tile_apply_commands(h) -- each tile moves the bots it
 *    observes (it holds their whole view) and sends their commands]
 *   aigar_tile_begin(h, p)  policy (NONE / RANDOM; GREEDY once the commands of
 *                           this tick were applied) + the tick up to the first
 *                           eat pass; the outbox holds the message
 *   <all-gather every tile's outbox into every tile's inbox>
 *   aigar_tile_apply(h, &u) the other tiles' outcomes; u = owned cells still
 *                           undone on all tiles (same value on every tile)
 *   while (u > 0) { aigar_tile_resume(h); <all-gather>; aigar_tile_apply(h, &u); }
 *   aigar_tile_end(h, obs, dtype)  playerPlayerOverlap .. spawnStuff; then, if obs
 *                           (DEVICE) is given, the observations of the bots THIS
 *                           tile observes (bot.py:272-497; the other rows are left
 *                           as they are, dead bots get NaN on every tile)
 * Without host round trips: aigar_tile_apply(h, NULL) returns at once, and a
 * fixed number K of further (aigar_tile_resume, all-gather, aigar_tile_apply)
 * rounds follow; a resume pass does nothing on the device once no owned cell is
 * undone, and aigar_tile_end raises error bit 4096 if cells are still undone
 * after the K passes (K = 0 with the default halo in practice: one pass).
 * Observation: each bot is observed by ONE tile -- the one holding its
 * last-frame history grids (bot.py:480-495), else the tile of its view centre.
 * A bot whose view centre moved to another tile, or that died, has its history
 * handed off in the next tick's first message and every tile takes it, so the
 * next observation is made by the view centre's tile; a view the observing
 * tile does not hold sets error bit 2048.  aigar_tile_observers: per player,
 * the observing tile of the last observation (-1: dead), identical on every tile.
 * The spawn deficit is global: each tile's message carries its pellet kills.
 * aigar_tile_info: info[14] = ntiles, tile_id, owned bucket range x0, x1, y0, y1
 * (half-open), held range x0, x1, y0, y1, records per message, bitmap words,
 * hand-off slots per message, records per hand-off slot;
 * the device outbox / inbox and the bytes of one message (the inbox holds
 * ntiles messages, tile k at k * bytes).  A message is 32-byte records:
 * [header: kind 0, record count, undone owned cells, pellet kills as double,
 * hand-off slots as double] [records: kind 1 pellet kill (seq, x, y) | 2 blob
 * kill (slot, seq) | 3 cell outcome (pool index, seq, mass, radius)] and, in
 * the tick's first pass, [hand-off slots: kind 4 (player, lastFovSize) + the
 * bot's history grids as doubles], in later passes [bitmap: owned cells now final].
 * aigar_tile_set_buffers: use caller-owned device buffers instead (e.g. torch
 * tensors that RCCL fills); aigar_tile_exchange_local: the in-process transport
 * -- copies every handle's outbox into every handle's inbox (same process).
 * aigar_get_state on a tiled handle returns the pellets the tile OWNS; the
 * union over the tiles is the arena's pellet list.
 */
int aigar_tile_info(aigar_handle *h, int32_t *info, void **outbox, void **inbox, int64_t *msg_bytes);
int aigar_tile_set_buffers(aigar_handle *h, void *outbox, void *inbox);
/* bytes of the current pass's message: the first pass of a tick sends the header
 * and records only (no bitmap); the inbox then holds tile k's at k * these bytes */
int aigar_tile_msg_bytes(aigar_handle *h, int64_t *bytes);
int aigar_tile_begin(aigar_handle *h, const aigar_run_params *p);
/* Greedy moves of the bots this tile observes (the observation's rule: history
 * holder, else the view centre's tile) into a command message [header: kind 0,
 * count][kind 5 records: player, split | eject << 1, command x, y]; after the
 * all-gather aigar_tile_apply_commands takes the other tiles' commands.  Replaces
 * Bot.make_greedy_bot_move + set_command_point (bot.py:579-633, 550-577) for a
 * tiled arena, where no tile holds every pellet. */
int aigar_tile_policy(aigar_handle *h, int greedy_split);
int aigar_tile_apply_commands(aigar_handle *h);
int aigar_tile_apply(aigar_handle *h, int *undone);
int aigar_tile_resume(aigar_handle *h);
int aigar_tile_end(aigar_handle *h, void *obs_out, int dtype);
int aigar_tile_exchange_local(aigar_handle **hs, int n);
int aigar_tile_observers(aigar_handle *h, int32_t *out);

/* C4 over RCCL (xGMI): the tile's exchange as ncclAllGather(outbox -> inbox) on
 * the handle's stream, so a whole tiled step -- policy, the tick with its eat
 * passes and exchanges, the observation of this tile's bots -- is one hipGraph
 * replay with no host round trip (the rank-side loop of the aigar_tile_* calls
 * above, with the caller's transport replaced by RCCL).
 *   aigar_rccl_unique_id(path, id)   rank 0: a fresh ncclUniqueId (128 bytes),
 *                                    which the caller broadcasts to every rank
 *   aigar_tile_comm_init(h, path, id, nranks, rank)  ncclCommInitRank; nranks
 *                                    must be the tile count and rank the tile id
 *   aigar_tile_run(h, n, p, extra_passes, obs, dtype)  n tiled steps: per step
 *       (policy GREEDY: aigar_tile_policy, all-gather, aigar_tile_apply_commands)
 *       aigar_tile_begin, all-gather, aigar_tile_apply, extra_passes gated
 *       (resume, all-gather, apply) rounds, aigar_tile_end (obs: DEVICE buffer
 *       or NULL) -- captured once as a hipGraph (RCCL is captured with it),
 *       direct launches if the capture fails or while profiling
 * path: the librccl.so to bind (the one the process's torch loaded, so that one
 * HIP runtime serves both), or NULL for "librccl.so" on the loader path. */
int aigar_rccl_unique_id(const char *path, void *id);
int aigar_tile_comm_init(aigar_handle *h, const char *path, const void *id, int nranks, int rank);
int aigar_tile_run(aigar_handle *h, int n_steps, const aigar_run_params *p, int extra_passes, void *obs_out,
                   int dtype);
/* 1 if aigar_tile_run replays a captured graph, 0 if it launches directly */
int aigar_tile_run_graphed(aigar_handle *h);
/* Timing rehearsal only (tools/c4_solo.py): aigar_tile_run without a
 * communicator, the exchange replaced by a copy of this tile's message into its
 * own inbox slot, every other tile's slot an empty message.  The tile then steps
 * alone on its GPU -- the per-GPU cost of a tiled step without the all-gather;
 * its world is not the tiled arena's (no other tile's outcomes arrive). */
int aigar_tile_loopback(aigar_handle *h);

/* The event log as raw rows (key_hi = tick << 8 | phase, key_lo = order within the
 * phase, code, a, b), unsorted: tiled arenas merge their tiles' logs by key. */
int aigar_get_events_raw(aigar_handle *h, int arena, int64_t *out, int cap, int *n);

/* Stream control. */
int aigar_set_stream(aigar_handle *h, void *hip_stream);
int aigar_sync(aigar_handle *h);

/* Timing support for bench.py: HIP-event time of the named kernel's launches
 * on the handle's stream during the last step (ms total, launch count). */
int aigar_profile(aigar_handle *h, int enable);
int aigar_kernel_time(aigar_handle *h, const char *kernel, double *ms, int *launches);

/* Diagnostics: per-arena work counters accumulated since reset/load_state --
 * out[0..n) of: serial work-list entries of virusBlobOverlap, playerVirusOverlap,
 * pellet + blob eating (cells), pellets eaten, playerPlayerOverlap (players),
 * pellets respawned, ticks whose playerPlayerOverlap ran as independent
 * groups (see tick.hip pp_pass), ticks.  n <= 8. */
int aigar_counters(aigar_handle *h, int arena, int64_t *out, int n);

/* Diagnostics: evaluate the device's pow (aigar_math.h: glibc 2.35's pow, bit
 * for bit) on host arrays of n (x, y) pairs -- used by the parity tests. */
int aigar_selftest_pow(const double *x, const double *y, double *out, int n);

/* Diagnostics: evaluate the device's trig (aigar_glibc_trig.h: glibc 2.35's
 * __ieee754_atan2_fma / __sin_fma / __cos_fma, bit for bit) on host arrays:
 * out[0, n) = atan2(y, x), out[n, 2n) = sin(x), out[2n, 3n) = cos(x). */
int aigar_selftest_trig(const double *y, const double *x, double *out, int n);

#ifdef __cplusplus
}
#endif
#endif /* AIGAR_H */
