#!/usr/bin/env python3
"""Golden-vector generator for the agar.io tick + grid observation.

CONTAINER-ONLY TEST INFRASTRUCTURE.  This script imports the read-only
reference (`/root/reference/src/model`) and runs it; it never runs on the GPU
box and nothing in the product imports it.  It writes `tests/golden/*.npz`
fixtures that hold numbers only (states, commands, RNG states, event logs,
observations) -- no reference source.

Shims (all live here; reference files are untouched), see SURVEY.md §8c:
  * a stub `pygame` module (`model/rgbGenerator.py:1-3` imports it; unused
    unless CNN_P_REPR);
  * canonical order: every `Cell.__init__` is stamped with a creation
    sequence number and `spatialHashTable.getObjectsFromBuckets`
    (`spatialHashTable.py:38-43`) returns a seq-sorted list instead of a set
    (CPython set order follows object addresses -> non-deterministic);
  * observers wrapping `Field.eatCell/eatPlayerCell/mergeCells/...` that append
    to an event log (they call the original method unchanged).

Determinism: `Field.__init__` reseeds numpy from time/pid (`field.py:32`), so
we reseed `numpy.random` immediately after `Model(...)`.

Usage:  python tools/golden/gen_golden.py [--out tests/golden] [--only NAME]
"""
import argparse
import math
import os
import random
import sys
import time
import tracemalloc
import types

import numpy as np

REF_SRC = "/root/reference/src"

# event codes (shared with oracle/ and the HIP library, see include/aigar.h)
EV_MERGE, EV_VIRUS_EAT_BLOB, EV_VIRUS_SPLIT, EV_CELL_EAT_VIRUS, EV_EXPLODE = 1, 2, 3, 4, 5
EV_CELL_EAT_PELLET, EV_CELL_EAT_BLOB, EV_CELL_EAT_CELL, EV_PLAYER_DEATH, EV_RESPAWN = 6, 7, 8, 9, 10


def import_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    pg = types.ModuleType("pygame")
    pg.gfxdraw = types.ModuleType("pygame.gfxdraw")
    sys.modules.setdefault("pygame", pg)
    sys.modules.setdefault("pygame.gfxdraw", pg.gfxdraw)
    if REF_SRC not in sys.path:
        sys.path.insert(0, REF_SRC)
    import model.cell as mcell
    import model.field as mfield
    import model.spatialHashTable as msht
    import model.model as mmodel
    import model.bot as mbot
    import model.player as mplayer
    import model.networkParameters as mnp
    return types.SimpleNamespace(cell=mcell, field=mfield, sht=msht, model=mmodel,
                                 bot=mbot, player=mplayer, np=mnp)


class Recorder:
    def __init__(self):
        self.seq = 0
        self.events = []
        self.field = None


def install_shims(ref, rec):
    Cell = ref.cell.Cell
    orig_init = Cell.__init__

    def init(self, *a, **k):
        self._seq = rec.seq
        rec.seq += 1
        orig_init(self, *a, **k)
    Cell.__init__ = init

    def get_objects_from_buckets(self, cellIds):
        s = set()
        for cid in cellIds:
            for c in self.buckets[cid]:
                s.add(c)
        return sorted(s, key=lambda c: c._seq)
    ref.sht.spatialHashTable.getObjectsFromBuckets = get_objects_from_buckets

    F = ref.field.Field
    o_eatCell, o_eatPC, o_merge = F.eatCell, F.eatPlayerCell, F.mergeCells
    o_del, o_vEB, o_expl, o_init_pl = F.deletePlayerCell, F.virusEatBlob, F.playerCellAteVirus, F.initializePlayer
    o_spawnPlayers = F.spawnPlayers

    def eatCell(self, eating, eh, cell, ch, lst, isVirus=None):
        if lst is self.pellets:
            code = EV_CELL_EAT_PELLET
        elif lst is self.viruses:
            code = EV_CELL_EAT_VIRUS
        elif eating.getPlayer() is None:
            code = EV_VIRUS_EAT_BLOB
        else:
            code = EV_CELL_EAT_BLOB
        rec.events.append((code, eating._seq, cell._seq))
        return o_eatCell(self, eating, eh, cell, ch, lst, isVirus)

    def eatPlayerCell(self, larger, smaller):
        rec.events.append((EV_CELL_EAT_CELL, larger._seq, smaller._seq))
        return o_eatPC(self, larger, smaller)

    def mergeCells(self, a, b):
        big, small = (a, b) if a.getMass() > b.getMass() else (b, a)
        rec.events.append((EV_MERGE, big._seq, small._seq))
        return o_merge(self, a, b)

    def deletePlayerCell(self, cell):
        r = o_del(self, cell)
        pl = cell.getPlayer()
        if not pl.getCells():
            rec.events.append((EV_PLAYER_DEATH, self.players.index(pl), cell._seq))
        return r

    def virusEatBlob(self, virus, blob):
        n0 = len(self.viruses)
        r = o_vEB(self, virus, blob)
        if len(self.viruses) > n0:
            rec.events.append((EV_VIRUS_SPLIT, virus._seq, self.viruses[-1]._seq))
        return r

    def playerCellAteVirus(self, cell):
        n_new = 16 - len(cell.getPlayer().getCells())
        rec.events.append((EV_EXPLODE, cell._seq, n_new))
        return o_expl(self, cell)

    def spawnPlayers(self):
        self._in_respawn = True
        try:
            return o_spawnPlayers(self)
        finally:
            self._in_respawn = False

    def initializePlayer(self, player):
        r = o_init_pl(self, player)
        if getattr(self, "_in_respawn", False):
            rec.events.append((EV_RESPAWN, self.players.index(player), player.getCells()[0]._seq))
        return r

    F.eatCell, F.eatPlayerCell, F.mergeCells = eatCell, eatPlayerCell, mergeCells
    F.deletePlayerCell, F.virusEatBlob, F.playerCellAteVirus = deletePlayerCell, virusEatBlob, playerCellAteVirus
    F.spawnPlayers, F.initializePlayer = spawnPlayers, initializePlayer


# ---------------------------------------------------------------- params ----
def make_params(ref, n_bots, virus, split, eject, overrides=None):
    """Copy of networkParameters with the derived obs sizes recomputed the way
    `networkParameters.py:74-102` does at import time."""
    p = types.ModuleType("golden_params")
    for k, v in vars(ref.np).items():
        if not k.startswith("__"):
            setattr(p, k, v)
    p.GATHER_EXP = False
    p.VIRUS_SPAWN = virus
    p.ENABLE_SPLIT = split
    p.ENABLE_EJECT = eject
    multi = n_bots > 1
    p.MULTIPLE_BOTS_PRESENT = multi
    p.NORMALIZE_GRID_BY_MAX_MASS = False
    p.PELLET_GRID = True
    p.SELF_GRID = split or virus
    p.SELF_GRID_LF = split
    p.SELF_GRID_SLF = False
    p.WALL_GRID = multi
    p.VIRUS_GRID = virus
    p.ENEMY_GRID = multi
    p.ENEMY_GRID_LF = split
    p.ENEMY_GRID_SLF = False
    p.SIZE_GRID = False
    p.ALL_PLAYER_GRID = False
    p.USE_FOVSIZE = True
    p.USE_LAST_FOVSIZE = split
    p.USE_TOTALMASS = True
    p.USE_LAST_ACTION = split
    p.USE_SECOND_LAST_ACTION = False
    p.GRID_SQUARES_PER_FOV = 11
    for k, v in (overrides or {}).items():
        setattr(p, k, v)
    if p.ALL_PLAYER_GRID:
        p.SELF_GRID = False
        p.ENEMY_GRID = False
    p.NUM_OF_GRIDS = (p.PELLET_GRID + p.SELF_GRID + p.WALL_GRID + p.VIRUS_GRID + p.ENEMY_GRID
                      + p.SIZE_GRID + p.SELF_GRID_LF + p.SELF_GRID_SLF + p.ENEMY_GRID_LF
                      + p.ENEMY_GRID_SLF + p.ALL_PLAYER_GRID)
    p.EXTRA_INPUT = (p.USE_FOVSIZE + p.USE_TOTALMASS + p.USE_LAST_ACTION * 4
                     + p.USE_SECOND_LAST_ACTION * 4 + p.USE_LAST_FOVSIZE)
    p.STATE_REPR_LEN = p.GRID_SQUARES_PER_FOV ** 2 * p.NUM_OF_GRIDS + p.EXTRA_INPUT
    return p


# obs channel bits (canonical order, bot.py:459-495) and extra bits (bot.py:302-323)
OBS_PELLET, OBS_SELF, OBS_WALL, OBS_ENEMY, OBS_ALL, OBS_VIRUS = 1, 2, 4, 8, 16, 32
OBS_SELF_SLF, OBS_SELF_LF, OBS_ENEMY_SLF, OBS_ENEMY_LF = 64, 128, 256, 512
EX_LAST_FOV, EX_FOV, EX_MASS, EX_LAST_ACT, EX_2LAST_ACT = 1, 2, 4, 8, 16


def obs_masks(p):
    ch = 0
    for flag, bit in ((p.PELLET_GRID, OBS_PELLET), (p.SELF_GRID, OBS_SELF), (p.WALL_GRID, OBS_WALL),
                      (p.ENEMY_GRID, OBS_ENEMY), (p.ALL_PLAYER_GRID, OBS_ALL), (p.VIRUS_GRID, OBS_VIRUS),
                      (p.SELF_GRID_SLF, OBS_SELF_SLF), (p.SELF_GRID_LF, OBS_SELF_LF),
                      (p.ENEMY_GRID_SLF, OBS_ENEMY_SLF), (p.ENEMY_GRID_LF, OBS_ENEMY_LF)):
        if flag:
            ch |= bit
    ex = 0
    for flag, bit in ((p.USE_LAST_FOVSIZE, EX_LAST_FOV), (p.USE_FOVSIZE, EX_FOV), (p.USE_TOTALMASS, EX_MASS),
                      (p.USE_LAST_ACTION, EX_LAST_ACT), (p.USE_SECOND_LAST_ACTION, EX_2LAST_ACT)):
        if flag:
            ex |= bit
    return ch, ex


# -------------------------------------------------------------- snapshot ----
def f(v):
    return float(v)


def snapshot(field):
    players = field.players
    hashed_cells = {id(o) for b in field.playerHashTable.buckets.values() for o in b}
    hashed_vir = {id(o) for b in field.virusHashTable.buckets.values() for o in b}
    pl_f = np.array([[f(p.commandPoint[0]), f(p.commandPoint[1])] for p in players], np.float64).reshape(-1, 2)
    pl_i = np.array([[int(p.isAlive), int(p.respawnTime), int(bool(p.doSplit)), int(bool(p.doEject)),
                      len(p.cells)] for p in players], np.int64).reshape(-1, 5)
    cf, ci = [], []
    for pi, p in enumerate(players):
        for c in p.cells:
            cf.append([f(c.x), f(c.y), f(c.mass), f(c.radius), f(c.velocity[0]), f(c.velocity[1]),
                       f(c.splitVelocity[0]), f(c.splitVelocity[1]), f(c.mergeTime)])
            ci.append([pi, int(c.splitVelocityCounter), c._seq, int(id(c) in hashed_cells)])
    pel = sorted(field.pellets, key=lambda c: c._seq)
    pf = [[f(c.x), f(c.y), f(c.mass), f(c.radius)] for c in pel]
    ps = [c._seq for c in pel]
    bf, bi = [], []
    for c in field.blobs:
        bf.append([f(c.x), f(c.y), f(c.mass), f(c.radius), f(c.velocity[0]), f(c.velocity[1]),
                   f(c.splitVelocity[0]), f(c.splitVelocity[1])])
        bi.append([int(c.splitVelocityCounter), c._seq, c.ejecterCell._seq if c.ejecterCell is not None else -1])
    vf, vi = [], []
    for c in field.viruses:
        vf.append([f(c.x), f(c.y), f(c.mass), f(c.radius), f(c.velocity[0]), f(c.velocity[1]),
                   f(c.splitVelocity[0]), f(c.splitVelocity[1])])
        vi.append([int(c.splitVelocityCounter), c._seq, int(id(c) in hashed_vir)])
    dead = [players.index(p) for p in field.deadPlayers]
    return {
        "players_f": pl_f, "players_i": pl_i,
        "cells_f": np.array(cf, np.float64).reshape(-1, 9), "cells_i": np.array(ci, np.int64).reshape(-1, 4),
        "pellets_f": np.array(pf, np.float64).reshape(-1, 4), "pellets_seq": np.array(ps, np.int64),
        "blobs_f": np.array(bf, np.float64).reshape(-1, 8), "blobs_i": np.array(bi, np.int64).reshape(-1, 3),
        "viruses_f": np.array(vf, np.float64).reshape(-1, 8), "viruses_i": np.array(vi, np.int64).reshape(-1, 3),
        "dead": np.array(dead, np.int64),
    }


def mt_state():
    st = np.random.get_state(legacy=True)
    assert st[0] == "MT19937"
    return np.asarray(st[1], np.uint32).copy(), int(st[2])


def digest(field):
    """Cheap per-tick fingerprint (exact float sums in a fixed order)."""
    s = snapshot(field)
    out = [len(s["cells_f"]), len(s["pellets_f"]), len(s["blobs_f"]), len(s["viruses_f"]), len(s["dead"])]
    vals = [float(np.sum(s[k][:, :3])) if len(s[k]) else 0.0 for k in ("cells_f", "pellets_f", "blobs_f", "viruses_f")]
    return out, vals


# ------------------------------------------------------------- scenarios ----
SCENARIOS = {
    # C1: BASELINE.json configs[0] -- 1 greedy bot, 1000x1000, 100 pellets
    "c1_greedy": dict(n=1, driver="greedy", size_per_player=1000, max_pellets=100, virus=False,
                      split=False, eject=False, ticks=1000, ck_every=100, obs=True, seed=0),
    # 16 greedy bots, default size 75*sqrt(16)=300, density 0.015 (1350 pellets)
    "greedy16": dict(n=16, driver="greedy", virus=False, split=False, eject=False, ticks=200,
                     ck_every=40, obs=True, seed=1),
    # greedy with viruses + greedy split (the C3 flavour, small)
    "greedy16_virus_split": dict(n=16, driver="greedy", virus=True, virus_density=4e-4, split=True,
                                 eject=False, greedy_split=True, ticks=200, ck_every=40, obs=True, seed=2),
    # scripted stress: viruses, split, eject, big cells -> explosions, blobs, eating, deaths, respawns
    "stress_virus": dict(n=16, driver="scripted", virus=True, virus_density=5e-4, split=True, eject=True,
                         p_split=0.06, p_eject=0.08, ticks=260, ck_every=20, obs=True, seed=3,
                         boost=[(0, 600.0), (1, 400.0), (2, 260.0), (3, 180.0), (4, 150.0), (5, 90.0)],
                         obs_over=dict(SELF_GRID_SLF=True, ENEMY_GRID_SLF=True, USE_SECOND_LAST_ACTION=True)),
    # crowded field: many collisions, deaths and respawns with hash-occupancy probing
    "crowd32": dict(n=32, driver="scripted", size_per_player=30, density=0.015, virus=False, split=True,
                    eject=True, p_split=0.03, p_eject=0.03, ticks=220, ck_every=20, obs=True, seed=4,
                    center_bias=0.7, boost=[(i, 20.0 + 9.0 * i) for i in range(32)]),
    # merges early: players start with several cells whose merge timers are ~0
    "merge8": dict(n=8, driver="scripted", virus=False, split=True, eject=False, p_split=0.02, p_eject=0.0,
                   ticks=120, ck_every=20, obs=True, seed=5, multi_cells=True),
    # virus feeding: a big player ejects toward viruses until they split (virus-blob path)
    "virus_feed": dict(n=4, driver="feed", virus=True, virus_density=4e-4, split=False, eject=True,
                       ticks=160, ck_every=20, obs=True, seed=6),
    # 64 reference Random bots (split + eject enabled via their own policy)
    "random64": dict(n=64, driver="random", size_per_player=75, density=0.0083, virus=False, split=True,
                     eject=True, ticks=120, ck_every=30, obs=False, seed=7),
    # GRID_VIEW_ENABLED = False: getSimpleStateRepresentation (bot.py:511-547), 12 values per bot;
    # big players see the field edges, small ones not
    "simple16": dict(n=16, driver="scripted", virus=True, virus_density=4e-4, split=True, eject=True,
                     p_split=0.03, p_eject=0.03, ticks=120, ck_every=20, obs=True, seed=8,
                     boost=[(0, 900.0), (1, 300.0), (2, 120.0)], obs_over=dict(GRID_VIEW_ENABLED=False),
                     obs_kind="simple"),
    # CNN over the grid view (bot.py:103-111, 284: CNN_REPR without CNN_P_REPR): 42 squares per side,
    # every channel incl. viruses and the last-frame grids, no extra inputs
    "cnn42": dict(n=12, driver="scripted", virus=True, virus_density=4e-4, split=True, eject=True,
                  p_split=0.03, p_eject=0.03, ticks=80, ck_every=40, obs=True, seed=9, boost=[(0, 400.0)],
                  obs_over=dict(CNN_REPR=True, CNN_P_REPR=False, CNN_USE_L1=True), obs_kind="cnn"),
    # ... and 84 squares per side (CNN_USE_L2) with Greedy bots that split
    "cnn84": dict(n=6, driver="greedy", virus=False, split=True, eject=False, greedy_split=True, ticks=60,
                  ck_every=30, obs=True, seed=10,
                  obs_over=dict(CNN_REPR=True, CNN_P_REPR=False, CNN_USE_L1=False, CNN_USE_L2=True),
                  obs_kind="cnn"),
    # BASELINE.json configs[1] (C2): 256 reference Greedy bots, default field 75*sqrt(256) = 1200,
    # 10,000 pellets, every bot's observation at every checkpoint
    "c2_greedy256": dict(n=256, driver="greedy", max_pellets=10000, virus=False, split=False, eject=False,
                         ticks=150, ck_every=50, obs=True, seed=11),
    # BASELINE.json configs[2] (C3, the headline world): 4096 bots, field 4800, 100k pellets, 1152 viruses,
    # split + eject on, started from the bench's own matured world (data/c3_t50.npz, loaded into the
    # reference object by object) and driven like bench.py's synthetic policy: a uniform point of the
    # bot's FOV through the reference's own Bot.set_command_point (bot.py:550-577), split p = 2.5e-3,
    # eject p = 1e-2 per bot-tick.  Every bot is observed every tick (its last-frame
    # grids evolve as in the device / oracle runs); the full 854-value rows are kept at the last tick.
    "c3_4096": dict(n=4096, driver="bench", load="data/c3_t50.npz", virus=True, split=True, eject=True,
                    p_split=2.5e-3, p_eject=1e-2, ticks=10, ck_every=5, obs=True, obs_init_stored=False, seed=12),
    # the same world size from the late matured world (data/c3_t600.npz: 6233 cells, 580 past mass 125,
    # 673 multi-cell players) with more splits and ejections, so that the headline size also pins
    # splits, ejected blobs, virus eating and explosions
    "c3_4096_t600": dict(n=4096, driver="bench", load="data/c3_t600.npz", virus=True, split=True, eject=True,
                         p_split=0.03, p_eject=0.05, ticks=4, ck_every=4, obs=True, obs_init_stored=False,
                         seed=13),
    # the headline world with every event kind: the tick-600 world with a few players set up
    # next to viruses -- 400-mass cells on 100-mass viruses (playerVirusOverlap + the explosion,
    # field.py:225-231, 350-370), 150-mass cells ejecting at 195-mass viruses (virusBlobOverlap + the
    # virus split, field.py:246-253, 315-324), multi-cell players whose merge timers ran out steered to
    # their centre (mergePlayerCells) -- everyone else on bench.py's policy
    "c3_4096_virus": dict(n=4096, driver="bench", load="data/c3_t600.npz", virus=True, split=True, eject=True,
                          p_split=2.5e-3, p_eject=1e-2, ticks=16, ck_every=8, obs=True, obs_init_stored=False,
                          seed=14, setup="virus_events"),
    # the headline start world with the reference's own Greedy bots (bot.py:579-633, ENABLE_GREEDY_SPLIT)
    "c3_greedy4096": dict(n=4096, driver="greedy", load="data/c3_t50.npz", virus=True, split=True, eject=True,
                          greedy_split=True, ticks=4, ck_every=4, obs=True, obs_init_stored=False, seed=15),
}


def setup_virus_events(field):
    """c3_4096_virus: mutate the loaded world before tick 1 (the snapshot "init/" is taken after it,
    so the fixture's start world holds the mutations); returns per-player command overrides
    [(player, (x, y), eject)] applied on top of the bench policy every tick."""
    size = field.size
    vir = [v for v in field.viruses if 80 < v.x < size - 80 and 80 < v.y < size - 80]
    singles = [i for i, p in enumerate(field.players) if p.getIsAlive() and len(p.cells) == 1]
    multis = [i for i, p in enumerate(field.players) if p.getIsAlive() and len(p.cells) >= 3]
    # spread the picks over the lists (neighbouring indices are unrelated places on the field)
    pick = lambda lst, k, n: lst[(k * len(lst)) // n]
    over = []
    for k in range(6):  # eaters: overlap (cell.py:143-152) and mass > 1.25 x virus mass at tick 1
        v, i = vir[k * 7], pick(singles, k, 12)
        c = field.players[i].cells[0]
        c.setMass(400.0)
        c.setPos([float(v.x) + 4.0, float(v.y) - 3.0])
        over.append((i, (float(v.x), float(v.y)), False))
    for k in range(6, 12):  # feeders: one 14.4-mass blob takes a 195-mass virus past 200.8
        v, i = vir[k * 7], pick(singles, k, 12)
        v.setMass(195.0)
        c = field.players[i].cells[0]
        c.setMass(150.0)
        c.setPos([float(v.x) - 20.0, float(v.y)])
        over.append((i, (float(v.x), float(v.y)), True))
    for k in range(8):  # mergers
        i = pick(multis, k, 8)
        cells = field.players[i].cells
        for c in cells:
            c.mergeTime = 0.0
        cx = sum(float(c.x) for c in cells) / len(cells)
        cy = sum(float(c.y) for c in cells) / len(cells)
        over.append((i, (cx, cy), False))
    return over
OBS_SIMPLE = 0x400  # include/aigar.h AIGAR_OBS_SIMPLE


def scripted_commands(field, rng, sc):
    size = field.size
    cmds = []
    for p in field.players:
        if rng.random() < sc.get("center_bias", 0.3):
            x, y = size / 2 + rng.normal() * size / 8, size / 2 + rng.normal() * size / 8
        else:
            x, y = rng.random() * size, rng.random() * size
        s = rng.random() < sc.get("p_split", 0.0)
        e = rng.random() < sc.get("p_eject", 0.0)
        cmds.append((x, y, s, e))
    return cmds


def feed_commands(field, rng, tick):
    """Player 0 (huge) sits near virus 0 and ejects toward it every tick."""
    cmds = []
    for i, p in enumerate(field.players):
        if i == 0 and field.viruses:
            v = field.viruses[0]
            cmds.append((float(v.x), float(v.y), False, True))
        else:
            cmds.append((rng.random() * field.size, rng.random() * field.size, False, False))
    return cmds


def bench_commands(field, bots, rng, sc):
    """bench.py's synthetic policy restated over the reference's own objects: an action drawn
    uniformly in [0,1]^2 mapped through Bot.set_command_point (bot.py:550-577), split / eject with
    p_split / p_eject.  Dead players keep their command point (they have no FOV position)."""
    for b in bots:
        a0, a1 = rng.random(), rng.random()
        s = 1.0 if rng.random() < sc["p_split"] else 0.0
        e = 1.0 if rng.random() < sc["p_eject"] else 0.0
        if b.player.getIsAlive():
            b.set_command_point([a0, a1, s, e])


def load_world(ref, rec, model, path):
    """Load a world written by tools/mature.py (the oracle's get_state layout) into the reference's
    objects, reproducing what a reference run that reached this state would hold:
      * `Field` sizes, counts and the four hashes (`field.py:57-66`): pellets and blobs hashed at
        their positions, player cells and viruses as the snapshot's `hashed` flag says (respawned
        cells and new viruses are not hashed until the next `updateHashTables`, `field.py:121-132`);
      * cells in each player's list order with every field the tick reads, the stored (possibly
        stale, `cell.py:90-94`) radius kept as is; the dead-player list in its order;
      * the creation sequence continues at `seq_next`.
    Cells are constructed before numpy is reseeded (a cell without a player draws its colour)."""
    z = np.load(path)
    field = model.field
    Cell = ref.cell.Cell
    SHT = ref.sht.spatialHashTable
    size = int(z["field_size"])
    field.size = size
    bucket = ref.field.HASH_BUCKET_SIZE
    field.pelletHashTable = SHT(size, bucket)
    field.blobHashTable = SHT(size, bucket)
    field.playerHashTable = SHT(size, bucket)
    field.virusHashTable = SHT(size, bucket)
    field.maxCollectibleCount = float(z["max_pellets"])
    field.maxVirusCount = float(z["max_viruses"])
    players = field.players
    pf, pi = z["players_f"], z["players_i"]
    assert len(players) == len(pf)
    for i, p in enumerate(players):
        p.commandPoint = [float(pf[i, 0]), float(pf[i, 1])]
        p.isAlive = bool(pi[i, 0])
        p.respawnTime = int(pi[i, 1])
        p.doSplit = bool(pi[i, 2])
        p.doEject = bool(pi[i, 3])
        p.cells = []

    def fill(c, row_f, counter, seq):
        c.radius = float(row_f[3])
        c.velocity = [float(row_f[4]), float(row_f[5])]
        c.splitVelocity = [float(row_f[6]), float(row_f[7])]
        c.splitVelocityCounter = int(counter)
        c._seq = int(seq)

    by_seq = {}
    cf, ci = z["cells_f"], z["cells_i"]
    for k in range(len(cf)):
        p = players[int(ci[k, 0])]
        c = Cell(float(cf[k, 0]), float(cf[k, 1]), float(cf[k, 2]), p)
        fill(c, cf[k], ci[k, 1], ci[k, 2])
        c.mergeTime = float(cf[k, 8])
        p.cells.append(c)
        by_seq[c._seq] = c
        if ci[k, 3]:
            field.playerHashTable.insertObject(c)
    for k in range(len(pi)):
        assert len(players[k].cells) == int(pi[k, 4])
    vf, vi = z["viruses_f"], z["viruses_i"]
    field.viruses = []
    for k in range(len(vf)):
        v = Cell(float(vf[k, 0]), float(vf[k, 1]), float(vf[k, 2]), None)
        v.setName("Virus")
        fill(v, vf[k], vi[k, 0], vi[k, 1])
        field.viruses.append(v)
        if vi[k, 2]:
            field.virusHashTable.insertObject(v)
    bf, bi = z["blobs_f"], z["blobs_i"]
    field.blobs = []
    for k in range(len(bf)):
        b = Cell(float(bf[k, 0]), float(bf[k, 1]), float(bf[k, 2]), None)
        fill(b, bf[k], bi[k, 0], bi[k, 1])
        b.ejecterCell = by_seq.get(int(bi[k, 2]))
        field.blobs.append(b)
        field.blobHashTable.insertObject(b)
    plf, pls = z["pellets_f"], z["pellets_seq"]
    field.pellets = []
    for k in np.argsort(pls, kind="stable"):
        c = Cell(float(plf[k, 0]), float(plf[k, 1]), float(plf[k, 2]), None)
        c.setName("Pellet")
        c.radius = float(plf[k, 3])
        c._seq = int(pls[k])
        field.pellets.append(c)
        field.pelletHashTable.insertObject(c)
    field.deadPlayers = [players[int(d)] for d in z["dead"]]
    rec.seq = int(z["seq_next"])
    return field


def run_scenario(ref, rec, name, sc):
    n = sc["n"]
    mf = ref.field
    # world size / densities via module globals of model.field
    mf.SIZE_INCREASE_PER_PLAYER = sc.get("size_per_player", 75)
    size = int(mf.SIZE_INCREASE_PER_PLAYER * math.sqrt(n))
    if "max_pellets" in sc:
        mf.MAX_COLLECTIBLE_DENSITY = sc["max_pellets"] / (size * size)
    else:
        mf.MAX_COLLECTIBLE_DENSITY = sc.get("density", 0.015)
    mf.MAX_VIRUS_DENSITY = sc.get("virus_density", 0.00005)

    params = make_params(ref, n, sc["virus"], sc["split"], sc["eject"], sc.get("obs_over"))
    params.ENABLE_GREEDY_SPLIT = sc.get("greedy_split", False)
    model = ref.model.Model(False, False, params)
    tracemalloc.stop()
    np.random.seed(sc["seed"])
    random.seed(sc["seed"])
    rec.seq = 0  # creation sequence restarts per scenario (only relative order matters)
    driver = sc["driver"]
    if driver in ("greedy", "random"):
        for _ in range(n):
            model.createBot("Greedy" if driver == "greedy" else "Random", None, params)
    else:
        for i in range(n):
            model.createPlayer("P%d" % i)
    if sc.get("load"):
        field = load_world(ref, rec, model, os.path.join(os.path.dirname(__file__), "..", "..", sc["load"]))
        np.random.seed(sc["seed"])  # the loader's colour draws are not part of the run
        model.resetBots()
    else:
        model.initialize()
    field = model.field
    rng = np.random.default_rng(1000 + sc["seed"])  # scenario driver RNG (not the field's MT stream)

    # stress mutations before tick 1 (hash rebuild at tick 1 picks them up)
    for pi, m in sc.get("boost", []):
        field.players[pi].cells[0].setMass(m)
    if sc.get("multi_cells"):
        for pi, p in enumerate(field.players):
            c0 = p.cells[0]
            c0.setMass(120.0 + 10 * pi)
            for k in range(3):
                ang = 2 * math.pi * k / 3
                c = ref.cell.Cell(min(field.size, max(0, c0.x + 6 * math.cos(ang))),
                                  min(field.size, max(0, c0.y + 6 * math.sin(ang))), 40.0 + 5 * k, p)
                c.mergeTime = float(k)
                p.addCell(c)
    overrides = []
    if sc.get("setup") == "virus_events":
        overrides = setup_virus_events(field)
    if driver == "feed":
        v = field.viruses[0]
        big = field.players[0].cells[0]
        big.setMass(3000.0)
        big.setPos([min(field.size, float(v.x) + 45.0), float(v.y)])

    obs_bots = []
    if sc.get("obs"):
        for p in field.players:
            obs_bots.append(ref.bot.Bot(p, field, "NN", None, params))
    ch_mask, ex_mask = obs_masks(params)
    kind = sc.get("obs_kind", "grid")
    G, L = params.GRID_SQUARES_PER_FOV, params.STATE_REPR_LEN
    if kind == "simple":  # no grids, no extra inputs
        ch_mask, ex_mask, L = OBS_SIMPLE, 0, 12
    elif kind == "cnn":  # the grid view alone, [NUM_OF_GRIDS, G, G] with the bot's CNN side
        G = obs_bots[0].gridSquaresPerFov if obs_bots else G
        ex_mask, L = 0, params.NUM_OF_GRIDS * G * G

    out = {
        "n_players": np.int64(n), "size": np.int64(field.size),
        "max_pellets": np.float64(field.maxCollectibleCount), "max_viruses": np.float64(field.maxVirusCount),
        "virus_enabled": np.int64(int(field.virusEnabled)),
        "obs_channels": np.int64(ch_mask), "obs_extras": np.int64(ex_mask),
        "obs_len": np.int64(L), "obs_grids": np.int64(params.NUM_OF_GRIDS), "grid_squares": np.int64(G),
        "ticks": np.int64(sc["ticks"]),
    }
    for k, v in snapshot(field).items():
        out["init/" + k] = v
    out["init/seq_next"] = np.int64(rec.seq)
    keys, pos = mt_state()
    out["init/mt_key"], out["init/mt_pos"] = keys, np.int64(pos)

    T = sc["ticks"]
    cmds_all = np.zeros((T, n, 4), np.float64)
    mt_keys = np.zeros((T, 624), np.uint32)
    mt_pos = np.zeros(T, np.int64)
    ev_rows, ev_off = [], [0]
    dig_i, dig_f = [], []
    ck_ticks = []

    def record_obs(tag):
        arr = np.full((n, L), np.nan)
        for i, b in enumerate(obs_bots):
            s = b.getStateRepresentation()
            if s is not None:
                arr[i] = np.asarray(s, np.float64).reshape(-1)
        return arr

    if obs_bots:
        obs0 = record_obs("init")  # (also advances the bots' last-frame grids, as the test's first observe)
        if sc.get("obs_init_stored", True):
            out["obs/init"] = obs0
    for t in range(T):
        if driver in ("greedy", "random"):
            model.takeBotActions()
        elif driver == "bench":
            bench_commands(field, obs_bots, rng, sc)
            for i, (x, y), e in overrides:
                p = field.players[i]
                if p.getIsAlive():
                    p.setCommands(x, y, False, e)
        else:
            cmds = scripted_commands(field, rng, sc) if driver == "scripted" else feed_commands(field, rng, t)
            for p, (x, y, s, e) in zip(field.players, cmds):
                p.setCommands(x, y, s, e)
        for i, p in enumerate(field.players):
            cmds_all[t, i] = (f(p.commandPoint[0]), f(p.commandPoint[1]), float(bool(p.doSplit)), float(bool(p.doEject)))
        mt_keys[t], mt_pos[t] = mt_state()
        rec.events = []
        field.update()
        ev_rows.extend(rec.events)
        ev_off.append(len(ev_rows))
        di, dfv = digest(field)
        dig_i.append(di)
        dig_f.append(dfv)
        obs_now = record_obs("t") if obs_bots else None
        if (t + 1) % sc["ck_every"] == 0 or t == T - 1:
            ck_ticks.append(t + 1)
            for k, v in snapshot(field).items():
                out["ck%d/%s" % (t + 1, k)] = v
            out["ck%d/seq_next" % (t + 1)] = np.int64(rec.seq)
            kk, pp = mt_state()
            out["ck%d/mt_key" % (t + 1)], out["ck%d/mt_pos" % (t + 1)] = kk, np.int64(pp)
            if obs_now is not None:
                out["obs/ck%d" % (t + 1)] = obs_now
    out["cmds"] = cmds_all
    out["mt_keys"], out["mt_pos"] = mt_keys, mt_pos
    out["events"] = np.array(ev_rows, np.int64).reshape(-1, 3)
    out["events_off"] = np.array(ev_off, np.int64)
    out["digest_i"] = np.array(dig_i, np.int64)
    out["digest_f"] = np.array(dig_f, np.float64)
    out["ck_ticks"] = np.array(ck_ticks, np.int64)
    ev = out["events"]
    counts = {c: int(np.sum(ev[:, 0] == c)) for c in range(1, 11)} if len(ev) else {}
    return out, counts


def rng_kats():
    """Known-answer vectors for the numpy legacy MT19937 draws the tick uses
    (randint with int and float bounds, random())."""
    rs = np.random.RandomState(12345)
    st = rs.get_state(legacy=True)
    spec = [(0, 1000), (0, 50), (50, 200), (0, 360), (-7.18, 7.18), (101.784, 118.216), (-18.2, -1.7),
            (0, 57600), (0, 3), (9950, 10000), (0, 1 << 31)]
    seq_i, seq_lo, seq_hi = [], [], []
    for _ in range(400):
        for lo, hi in spec:
            seq_lo.append(lo)
            seq_hi.append(hi)
            seq_i.append(int(rs.randint(lo, hi)))
    randoms = np.array([rs.random() for _ in range(200)], np.float64)
    end = rs.get_state(legacy=True)
    return {"mt_key": np.asarray(st[1], np.uint32), "mt_pos": np.int64(st[2]),
            "lo": np.array(seq_lo, np.float64), "hi": np.array(seq_hi, np.float64),
            "val": np.array(seq_i, np.int64), "random": randoms,
            "end_key": np.asarray(end[1], np.uint32), "end_pos": np.int64(end[2])}


def numeric_kats():
    """numpy pairwise sum, Python round(x, 3), deg2rad, pow as used by the path."""
    rng = np.random.default_rng(99)
    sums_in, sums_off, sums_out = [], [0], []
    for n in range(1, 40):
        for _ in range(20):
            a = list(rng.random(n) * rng.choice([1.0, 100.0, 5000.0]))
            sums_in.extend(a)
            sums_off.append(len(sums_in))
            sums_out.append(float(np.sum(a)))
    rv = np.concatenate([rng.random(4000) * 2 - 0.5, np.arange(-5, 2005) / 2000.0,
                         np.array([-2e-16, 2e-16, 0.0005, 0.0015, 0.0025, 1 - 1e-16])])
    rounded = np.array([round(float(v), 3) for v in rv], np.float64)
    return {"sum_in": np.array(sums_in), "sum_off": np.array(sums_off, np.int64), "sum_out": np.array(sums_out),
            "round_in": rv, "round_out": rounded,
            "deg2rad": np.array([np.deg2rad(d) for d in range(360)], np.float64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden"))
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    ref = import_reference()
    rec = Recorder()
    install_shims(ref, rec)
    if args.only in (None, "kats"):
        np.savez_compressed(os.path.join(args.out, "kat_rng.npz"), **rng_kats())
        np.savez_compressed(os.path.join(args.out, "kat_numeric.npz"), **numeric_kats())
    for name, sc in SCENARIOS.items():
        if args.only not in (None, name):
            continue
        if args.only is None and sc.get("load"):
            continue  # the BASELINE-size worlds take minutes: generate them with --only NAME
        t0 = time.time()
        out, counts = run_scenario(ref, rec, name, sc)
        np.savez_compressed(os.path.join(args.out, name + ".npz"), **out)
        print(name, "events:", counts, "final counts:", out["digest_i"][-1].tolist(), "%.0f s" % (time.time() - t0),
              flush=True)


if __name__ == "__main__":
    main()
