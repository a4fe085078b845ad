"""Python facade with the reference's object API over the device stepper.

Mirrors the names and behaviour of the reference's hot-path objects so its
drivers keep working:

  Field   src/model/field.py     (addPlayer, initialize, reset, update, FOV/list getters)
  Player  src/model/player.py    (setCommands, getCells, getFovPos/Size, getTotalMass, ...)
  Cell    src/model/cell.py      (read-only view: getters and predicates)
  Bot     src/model/bot.py       (Greedy / Random / NN bots: makeMove,
                                  set_command_point, getStateRepresentation)
  Model   src/model/model.py     (createPlayer, createBot, initialize, resetModel, update)

The world lives on the GPU.  `Field.update()` pushes every player's command and
runs one `aigar_step`; getters read a snapshot (`aigar_get_state`) taken lazily
once per tick, so the per-object API is a compatibility path.  The batched
fast path is `Field.set_commands(cmd[B,4])`, `Field.step(n)` and
`Field.observe_all(out)` (device tensors accepted).

Differences a caller can see:
 - object identity: Cell views are rebuilt each tick (compare `getId()`, the
   creation sequence number, instead of `is`);
 - canonical order: every set-derived list (FOV queries) is ordered by creation
   sequence instead of CPython object addresses;
 - randomness comes from the device's Philox stream (seeded by `seed`), not from
   numpy's global MT19937; Random bots still draw from numpy like the reference;
 - colours (for a View: view.py:164-215) follow the reference's rules with
   hashed instead of drawn values: a player's colour is three bytes with a sum
   <= 600 (player.py:38-41), its cells and its ejected blobs take it
   (cell.py:35, field.py:141), viruses are (0, 255, 0) (field.py:274) and
   pellets three values in [50, 200) (cell.py:31), each keyed by the object;
 - Greedy bots move on the device, all in one launch per tick
   (`Model.takeBotActions`); their splitLikelihood comes from the Philox stream
   unless set with `Field.set_split_likelihood`.
"""
import math

import numpy as np

from . import _abi
from ._lib import Stepper

HASH_BUCKET_SIZE = 20  # parameters.py: HASH_BUCKET_SIZE
START_MASS = 10
MAX_COLLECTIBLE_DENSITY = 0.015
MAX_VIRUS_DENSITY = 0.00005
SIZE_INCREASE_PER_PLAYER = 75

# reference flag name -> observation channel bit (stacking order bot.py:459-495)
_CHANNEL_FLAGS = (
    ("PELLET_GRID", _abi.OBS_PELLET), ("SELF_GRID", _abi.OBS_SELF), ("WALL_GRID", _abi.OBS_WALL),
    ("ENEMY_GRID", _abi.OBS_ENEMY), ("ALL_PLAYER_GRID", _abi.OBS_ALL), ("VIRUS_GRID", _abi.OBS_VIRUS),
    ("SELF_GRID_SLF", _abi.OBS_SELF_SLF), ("SELF_GRID_LF", _abi.OBS_SELF_LF),
    ("ENEMY_GRID_SLF", _abi.OBS_ENEMY_SLF), ("ENEMY_GRID_LF", _abi.OBS_ENEMY_LF),
)
_EXTRA_FLAGS = (
    ("USE_LAST_FOVSIZE", _abi.EX_LAST_FOV), ("USE_FOVSIZE", _abi.EX_FOV), ("USE_TOTALMASS", _abi.EX_MASS),
    ("USE_LAST_ACTION", _abi.EX_LAST_ACT), ("USE_SECOND_LAST_ACTION", _abi.EX_2LAST_ACT),
)


def obs_masks(parameters):
    """(channels, extras, grid squares) of a reference networkParameters-like object."""
    if parameters is None:  # networkParameters.py defaults for one NN bot
        return _abi.OBS_PELLET, _abi.EX_FOV | _abi.EX_MASS, 11
    if not getattr(parameters, "GRID_VIEW_ENABLED", True):  # bot.py:296-297: getSimpleStateRepresentation
        return _abi.OBS_SIMPLE, 0, 11
    if getattr(parameters, "SIZE_GRID", False):
        raise NotImplementedError("SIZE_GRID observations are not implemented")
    cnn_grid = getattr(parameters, "CNN_REPR", False) and not getattr(parameters, "CNN_P_REPR", False)
    ch = 0
    for name, bit in _CHANNEL_FLAGS:
        if getattr(parameters, name, False):
            ch |= bit
    if ch & _abi.OBS_ALL:  # networkParameters.py: ALL_PLAYER_GRID disables SELF/ENEMY
        ch &= ~(_abi.OBS_SELF | _abi.OBS_ENEMY)
    ex = 0
    if getattr(parameters, "EXTRA_INPUT", True) and not cnn_grid:
        for name, bit in _EXTRA_FLAGS:
            if getattr(parameters, name, False):
                ex |= bit
    if cnn_grid:  # bot.py:103-111, 284: the grid view alone, CNN_INPUT_DIM_* squares per side (42 / 84)
        if getattr(parameters, "CNN_USE_L1", False):
            g = parameters.CNN_INPUT_DIM_1
        elif getattr(parameters, "CNN_USE_L2", False):
            g = parameters.CNN_INPUT_DIM_2
        else:
            g = parameters.CNN_INPUT_DIM_3
        return ch, 0, int(g)
    return ch, ex, int(getattr(parameters, "GRID_SQUARES_PER_FOV", 11))


def reference_parameters():
    """The reference's networkParameters module when its code is loaded in this
    process (model.py imports it, then builds Field(virusEnabled) without passing
    it), else None (the single-NN-bot defaults of obs_masks)."""
    import sys
    for name, mod in list(sys.modules.items()):
        if name.split(".")[-1] == "networkParameters" and hasattr(mod, "GRID_SQUARES_PER_FOV"):
            return mod
    return None


def _mix(v):
    """splitmix64 finaliser: the hash behind the (deterministic) colours."""
    v = (v + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    v = ((v ^ (v >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    v = ((v ^ (v >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return v ^ (v >> 31)


def player_color(index, seed=0):
    """Player.randomizeColor (player.py:38-41): (0..255)^3, redrawn while the sum exceeds 600."""
    k = 0
    while True:
        h = _mix((int(seed) << 32) ^ (int(index) << 8) ^ k)
        c = (h & 255, (h >> 8) & 255, (h >> 16) & 255)
        if sum(c) <= 600:
            return c
        k += 1


def pellet_color(seq, seed=0):
    """cell.py:31: three numpy.random.randint(50, 200) draws (hashed from the creation sequence)."""
    h = _mix((int(seed) << 40) ^ int(seq) ^ 0x5E11E7)
    return (50 + h % 150, 50 + (h >> 16) % 150, 50 + (h >> 32) % 150)


VIRUS_COLOR = (0, 255, 0)  # field.py:274


def _footprint(x, y, r, size):
    """Bucket rectangle of spatialHashTable.getIdsForArea (int variant,
    spatialHashTable.py:70-83); arrays in, (x0, x1, y0, y1) out (x1 < x0: empty)."""
    b = HASH_BUCKET_SIZE
    cl, ct = np.maximum(0.0, x - r), np.maximum(0.0, y - r)
    bl = np.trunc(cl - np.mod(cl, b)).astype(np.int64)
    bt = np.trunc(ct - np.mod(ct, b)).astype(np.int64)
    lx = np.trunc(np.minimum(float(size), x + r + 1)).astype(np.int64)
    ly = np.trunc(np.minimum(float(size), y + r + 1)).astype(np.int64)
    x0, y0 = bl // b, bt // b
    x1 = np.where(lx > bl, (bl + b * ((lx - 1 - bl) // b)) // b, x0 - 1)
    y1 = np.where(ly > bt, (bt + b * ((ly - 1 - bt) // b)) // b, y0 - 1)
    return x0, x1, y0, y1


def _in_area(x, y, r, size, fov_pos, fov_size):
    """hash.getNearbyObjectsInArea(pos, fov/2) then Cell.isInFov (field.py:422-456,
    cell.py:169-177), as a boolean mask."""
    if len(x) == 0:
        return np.zeros(0, bool)
    qx0, qx1, qy0, qy1 = _footprint(np.float64(fov_pos[0]), np.float64(fov_pos[1]), np.float64(fov_size / 2), size)
    x0, x1, y0, y1 = _footprint(x, y, r, size)
    near = (x0 <= x1) & (y0 <= y1) & (qx0 <= qx1) & (qy0 <= qy1) & (x0 <= qx1) & (qx0 <= x1) & (y0 <= qy1) & \
        (qy0 <= y1)
    h = fov_size / 2
    inside = ~((x + r < fov_pos[0] - h) | (x - r > fov_pos[0] + h) | (y + r < fov_pos[1] - h) |
               (y - r > fov_pos[1] + h))
    return near & inside


class Cell:
    """Read-only view of one entity of a tick snapshot (cell.py:7-260)."""
    __slots__ = ("x", "y", "mass", "radius", "velocity", "splitVelocity", "splitVelocityCounter", "mergeTime",
                 "player", "id", "kind", "alive", "pos", "color")

    def __init__(self, kind, f, seq, svc, player=None, merge_time=0.0, color=(0, 0, 0)):
        self.kind = kind
        self.x, self.y, self.mass, self.radius = float(f[0]), float(f[1]), float(f[2]), float(f[3])
        self.pos = [self.x, self.y]
        self.velocity = [float(f[4]), float(f[5])] if len(f) > 5 else [0.0, 0.0]
        self.splitVelocity = [float(f[6]), float(f[7])] if len(f) > 7 else [0.0, 0.0]
        self.splitVelocityCounter = int(svc)
        self.mergeTime = float(merge_time)
        self.player = player
        self.id = int(seq)
        self.alive = True
        self.color = color

    def __repr__(self):
        return "Cell(%s #%d m=%.3f @ %.2f,%.2f)" % (self.kind, self.id, self.mass, self.x, self.y)

    # getters (cell.py:222-260)
    def getX(self): return self.x
    def getY(self): return self.y
    def getPos(self): return self.pos
    def getMass(self): return self.mass
    def getRadius(self): return self.radius
    def getPlayer(self): return self.player
    def getId(self): return self.id
    def getMergeTime(self): return self.mergeTime
    def getSplitVelocityCounter(self): return self.splitVelocityCounter
    def getVelocity(self): return self.velocity
    def getSplitVelocity(self): return self.splitVelocity
    def getReducedSpeed(self): return 3.0 * math.pow(self.mass, -0.35)
    def getName(self): return self.player.getName() if self.player is not None else ""
    def getColor(self): return self.color

    # predicates (cell.py:143-189)
    def isAlive(self): return self.alive
    def justEjected(self): return self.splitVelocityCounter > 0
    def canSplit(self): return self.mass > 36
    def canEject(self): return self.mass >= 35
    def canMerge(self): return self.mergeTime <= 0
    def canEat(self, cell): return self.mass > 1.25 * cell.getMass()

    def squaredDistance(self, cell):
        p = cell.getPos()
        return (self.x - p[0]) * (self.x - p[0]) + (self.y - p[1]) * (self.y - p[1])

    def overlap(self, cell):
        big, small = (self, cell) if self.getMass() > cell.getMass() else (cell, self)
        return big.squaredDistance(small) * 1.1 < big.getRadius() * big.getRadius()

    def isInFov(self, fovPos, fovSize):
        h = fovSize / 2
        return not (self.x + self.radius < fovPos[0] - h or self.x - self.radius > fovPos[0] + h or
                    self.y + self.radius < fovPos[1] - h or self.y - self.radius > fovPos[1] + h)


class Player:
    """player.py:4-184 -- commands go to the device at the next Field.update()."""

    def __init__(self, name):
        self.name = name
        self.field = None
        self.index = -1
        self.exploring = False
        self.selected = False
        self.commandPoint = [-1, -1]
        self.doSplit = False
        self.doEject = False
        self._alive = False

    def __repr__(self):
        return "Player(%s)" % self.name

    def setCommands(self, x, y, split, eject):  # player.py:99-102
        self.commandPoint = [x, y]
        self.doSplit = bool(split)
        self.doEject = bool(eject)
        if self.field is not None and self.field.stepper is not None:
            self.field._cmd[self.index] = (x, y, float(bool(split)), float(bool(eject)))

    def setSplit(self, val): self.setCommands(self.commandPoint[0], self.commandPoint[1], val, self.doEject)
    def setEject(self, val): self.setCommands(self.commandPoint[0], self.commandPoint[1], self.doSplit, val)
    def setMoveTowards(self, pos): self.setCommands(pos[0], pos[1], self.doSplit, self.doEject)
    def setExploring(self, val): self.exploring = val
    def setSelected(self, val): self.selected = val
    def setAlive(self): self._alive = True

    def _stats(self):
        return self.field._player_stats()[self.index]

    def getIsAlive(self):
        if self.field is None or self.field.stepper is None:
            return self._alive
        return bool(self._stats()[0] > 0)

    def getTotalMass(self):  # player.py:129-130
        return float(self._stats()[1]) if self.getIsAlive() else 0.0

    def getFovPos(self):  # player.py:156-161
        s = self._stats()
        return [float(s[2]), float(s[3])]

    def getFovSize(self):  # player.py:163-167
        return float(self._stats()[4])

    def getFov(self):
        return self.getFovPos(), self.getFovSize()

    def getCells(self):
        return self.field._player_cells(self.index)

    def getMergableCells(self):
        return [c for c in self.getCells() if c.canMerge()]

    def getCanSplit(self):
        cells = self.getCells()
        return len(cells) < 16 and any(c.canSplit() for c in cells)

    def getCanEject(self):
        return any(c.canEject() for c in self.getCells())

    def getRespawnTime(self):
        return int(self.field._snapshot()["players_i"][self.index][1])

    def getCommandPoint(self): return self.commandPoint
    def getName(self): return self.name
    def getSelected(self): return self.selected
    def isExploring(self): return self.exploring

    def getColor(self):  # player.py:174
        seed = self.field.seed if self.field is not None else 0
        return player_color(self.index, seed)


class Field:
    """field.py:28-487 over one device arena."""

    def __init__(self, virusEnabled, parameters=None, seed=0, device=0, field_size=0, max_pellets=-1.0,
                 max_viruses=-1.0, record_events=False):
        self.virusEnabled = bool(virusEnabled)
        self.parameters = parameters
        self.seed = int(seed)
        self.device = device
        self.field_size = field_size
        self.max_pellets, self.max_viruses = max_pellets, max_viruses
        self.record_events = record_events
        self.players = []
        self.stepper = None
        self.size = 0
        self._resets = 0
        self._cache = {}

    # ---- lifecycle
    def addPlayer(self, player):  # field.py:414-416
        if self.stepper is not None:
            raise RuntimeError("players must be added before initialize() (the device world is sized then)")
        player.setAlive()
        player.field = self
        player.index = len(self.players)
        self.players.append(player)

    def _config(self):
        if self.parameters is None:  # the reference's model.py builds Field(virusEnabled) without them
            self.parameters = reference_parameters()
        ch, ex, g = obs_masks(self.parameters)
        if not self.virusEnabled:
            ch &= ~_abi.OBS_VIRUS
        c = _abi.Config()
        c.n_arenas, c.bots_per_arena = 1, len(self.players)
        c.field_size = int(self.field_size)
        c.virus_enabled = int(self.virusEnabled)
        c.max_pellets, c.max_viruses = float(self.max_pellets), float(self.max_viruses)
        c.grid_squares, c.obs_channels, c.obs_extras = g, ch, ex
        self.grid_squares = g
        c.rng_mode, c.device = _abi.RNG_PHILOX, self.device
        c.flags = _abi.FLAG_EVENTS if self.record_events else 0
        return c

    def initialize(self):  # field.py:57-67
        if not self.players:
            raise RuntimeError("Field.initialize() needs at least one player")
        if self.stepper is None:
            self.stepper = Stepper(self._config())
            self._cmd = np.zeros((len(self.players), 4))
            self._cmd[:, :2] = -1
        self.stepper.reset(self.seed)
        self.size = int(self.stepper.get_state()["field_size"])
        self._cache = {}

    def reset(self):  # field.py:69-83
        self._resets += 1
        self.stepper.reset(self.seed + 7919 * self._resets)
        # the reference's players survive Field.reset with their commandPoint and
        # split / eject flags (initializePlayer only gives them new cells)
        self.stepper.set_commands(self._cmd)
        self._cache = {}

    def update(self):  # field.py:85-92
        self.stepper.set_commands(self._cmd)
        self.stepper.step(1)
        self._cache = {}

    # ---- batched fast path
    def set_commands(self, cmd):
        """cmd[B, 4] = (x, y, split, eject) for every player (numpy or device tensor)."""
        self.stepper.set_commands(cmd)

    def step(self, n=1):
        self.stepper.step(n)
        self._cache = {}

    def observe_all(self, out=None, dtype=np.float64):
        """Bot.getStateRepresentation() of every player, [B, L] (NaN rows for dead players)."""
        return self.stepper.observe(out, dtype)

    def events(self):
        """Ordered (tick, code, a, b) rows of the last step (record_events=True)."""
        return self.stepper.events()

    def observe_pixels_all(self, side=42, rgb=False, out=None, color_seed=None):
        """RGBGenerator.get_cnn_inputRGB of every player in one launch: uint8 [B, side, side, 3]
        (rgb) or float64 grayscale [B, side, side]; surfarray order [x][y]."""
        return self.stepper.observe_pixels(side, self.seed if color_seed is None else color_seed, rgb=rgb, out=out)

    # ---- snapshot-backed compatibility getters
    def _snapshot(self):
        if "state" not in self._cache:
            self._cache["state"] = self.stepper.get_state()
        return self._cache["state"]

    def _player_stats(self):
        if "stats" not in self._cache:
            self._cache["stats"] = self.stepper.player_stats()
        return self._cache["stats"]

    def _views(self):
        if "views" in self._cache:
            return self._cache["views"]
        st = self._snapshot()
        per_player = [[] for _ in self.players]
        cells = []
        pcol = [p.getColor() for p in self.players]
        for f, i in zip(st["cells_f"], st["cells_i"]):
            c = Cell("player", f[:8], i[2], i[1], self.players[int(i[0])], f[8], pcol[int(i[0])])
            per_player[int(i[0])].append(c)
            cells.append(c)
        # an ejected blob carries its player's colour (field.py:141, cell.py:219), and so
        # does the pellet it becomes (addPellet(blob), field.py:110): the state's colour owners
        colour = lambda owner, seq: pcol[int(owner)] if owner >= 0 else pellet_color(seq, self.seed)  # noqa: E731
        pel = [Cell("pellet", f, s, 0, color=colour(c, s))
               for f, s, c in zip(st["pellets_f"], st["pellets_seq"], st["pellets_col"])]
        blobs = [Cell("blob", f, i[1], i[0], color=colour(c, i[1]))
                 for f, i, c in zip(st["blobs_f"], st["blobs_i"], st["blobs_col"])]
        vir = [Cell("virus", f, i[1], i[0], color=VIRUS_COLOR) for f, i in zip(st["viruses_f"], st["viruses_i"])]
        v = {"per_player": per_player, "cells": cells, "pellets": pel, "blobs": blobs, "viruses": vir,
             "cell_hashed": np.asarray(st["cells_i"])[:, 3] != 0 if len(cells) else np.zeros(0, bool),
             "virus_hashed": np.asarray(st["viruses_i"])[:, 2] != 0 if len(vir) else np.zeros(0, bool)}
        self._cache["views"] = v
        return v

    def _player_cells(self, index):
        return list(self._views()["per_player"][index])

    def _query(self, objs, fov_pos, fov_size, member=None):
        if not objs:
            return []
        x = np.array([o.x for o in objs])
        y = np.array([o.y for o in objs])
        r = np.array([o.radius for o in objs])
        m = _in_area(x, y, r, self.size, fov_pos, fov_size)
        if member is not None:
            m &= member
        sel = [objs[k] for k in np.nonzero(m)[0]]
        sel.sort(key=lambda o: o.id)  # canonical order of the hash's set
        return sel

    # getters (field.py:418-487)
    def getVirusEnabled(self): return self.virusEnabled
    def getWidth(self): return self.size
    def getHeight(self): return self.size
    def getPlayers(self): return self.players
    def getPellets(self): return self._views()["pellets"]
    def getBlobs(self): return self._views()["blobs"]
    def getViruses(self): return self._views()["viruses"]
    def getPlayerCells(self): return list(self._views()["cells"])

    def getDeadPlayers(self):
        return [self.players[int(p)] for p in self._snapshot()["dead"]]

    @staticmethod
    def getPortionOfCellsInFov(cells, fovPos, fovSize):
        return [c for c in cells if c.isInFov(fovPos, fovSize)]

    def getPlayerCellsInFov(self, fovPos, fovSize):
        v = self._views()
        return self._query(v["cells"], fovPos, fovSize, v["cell_hashed"])

    def getFoVPlayerCellsInFov(self, fovPlayer):
        return [c for c in self.getPlayerCellsInFov(fovPlayer.getFovPos(), fovPlayer.getFovSize())
                if c.getPlayer() is fovPlayer]

    def getEnemyPlayerCellsInFov(self, fovPlayer):
        return [c for c in self.getPlayerCellsInFov(fovPlayer.getFovPos(), fovPlayer.getFovSize())
                if c.getPlayer() is not fovPlayer]

    def getEnemyPlayerCellsInGivenFov(self, fovPlayer, fovPos, fovSize):
        return [c for c in self.getPlayerCellsInFov(fovPos, fovSize) if c.getPlayer() is not fovPlayer]

    def getPelletsInFov(self, fovPos, fovSize):
        return self._query(self._views()["pellets"], fovPos, fovSize)

    def getVirusesInFov(self, fovPos, fovSize):
        v = self._views()
        return self._query(v["viruses"], fovPos, fovSize, v["virus_hashed"])

    def getBlobsInFov(self, fovPos, fovSize):
        return self._query(self._views()["blobs"], fovPos, fovSize)

    @staticmethod
    def getReward(player):
        return player.getTotalMass()

    # observation for the NN bots: getStateRepresentation advances a bot's last-frame
    # history only when that bot computes its state (bot.py:195-202), so the device
    # observes exactly the bots asked for (aigar_observe_masked); Model.takeBotActions
    # asks for all NN bots of a tick in one call
    def _prefetch_states(self, indices):
        idx = [i for i in indices if i not in self._cache.get("obs_rows", {})]
        if not idx:
            return
        mask = np.zeros(len(self.players), np.uint8)
        mask[idx] = 1
        if "obs_buf" not in self._cache:
            self._cache["obs_buf"] = np.zeros((len(self.players), self.stepper.obs_len))
        buf = self.stepper.observe(self._cache["obs_buf"], mask=mask)
        rows = self._cache.setdefault("obs_rows", {})
        for i in idx:
            rows[i] = buf[i].copy()

    def _state_row(self, index):
        self._prefetch_states([index])
        return self._cache["obs_rows"][index]

    def _greedy_moves(self, mask, greedy_split):
        """make_greedy_bot_move + set_command_point on the device for the masked players;
        the resulting commands replace theirs in the host command buffer."""
        self.stepper.set_commands(self._cmd)  # keep the other players' commands
        self.stepper.policy_greedy(greedy_split, mask)
        st = self.stepper.get_state()
        pf, pi = np.asarray(st["players_f"]), np.asarray(st["players_i"])
        sel = np.asarray(mask, bool)
        self._cmd[sel, 0], self._cmd[sel, 1] = pf[sel, 0], pf[sel, 1]
        self._cmd[sel, 2], self._cmd[sel, 3] = pi[sel, 2], pi[sel, 3]
        for p in self.players:
            if sel[p.index]:
                p.commandPoint = [float(self._cmd[p.index, 0]), float(self._cmd[p.index, 1])]
                p.doSplit, p.doEject = bool(self._cmd[p.index, 2]), bool(self._cmd[p.index, 3])
        self._cache.pop("state", None)
        self._cache.pop("views", None)

    def set_split_likelihood(self, lh):
        """Greedy bots' splitLikelihood per player (bot.py:93); None: Philox-derived."""
        self.stepper.set_split_likelihood(lh)

    def _set_actions(self, bots):
        cur = np.zeros((len(self.players), 4))
        prev = np.zeros((len(self.players), 4))
        for b in bots:
            for arr, act in ((cur, b.currentAction), (prev, b.lastAction)):
                if act is not None:
                    a = list(act)[:4]
                    arr[b.player.index, :len(a)] = a
        self.stepper.set_actions(cur, prev)


class Bot:
    """bot.py:23-710.  Greedy bots move on the device (k_policy_greedy, batched
    over all Greedy bots by Model.takeBotActions); Random bots draw from numpy
    like the reference; NN bots run the reference's move_NN (bot.py:194-233):
    cumulative reward over the frame-skip window, frame skipping, the state from
    the device (grid view, or the pixel frame for CNN_P_REPR), the learner's
    decideMove(state), the experience tuples."""

    def __init__(self, player, field, bot_type, learningAlg=None, parameters=None, rgbGenerator=None):
        if bot_type not in ("Greedy", "Random", "NN"):
            raise NotImplementedError("bot type %r is not one of Greedy, Random, NN" % bot_type)
        self.player, self.field, self.type = player, field, bot_type
        self.learningAlg = learningAlg
        self.parameters = parameters
        self.rgbGenerator = rgbGenerator
        self.gatherExperiences = self._param("GATHER_EXP", True)
        self.experiences = []
        self.memories = []
        self.lastMass = None
        self.lastReward = None
        self.lastAction = None
        self.fovSize = None
        self.lastFovSize = None
        self.currentAction = None
        self.lastPixelGrid = None
        self.time = 0
        self.totalMasses = []
        self.reset()

    def __repr__(self):
        return "%s bot (%s)" % (self.type, self.player)

    def _param(self, name, default):
        return getattr(self.parameters, name, default) if self.parameters is not None else default

    def reset(self, _device=True):  # bot.py:125-164
        if self.learningAlg is not None and hasattr(self.learningAlg, "reset"):
            self.learningAlg.reset()
        self.lastMass = None
        self.oldState = None
        self.lastMemory = None
        self.skipFrames = 0
        self.cumulativeReward = 0
        self.lastReward = 0
        self.rewardAvgOfEpisode = 0
        self.rewardLenOfEpisode = 0
        self.currentlySkipping = False
        if self.type == "NN":
            self.currentActionIdx = None
            self.currentAction = None
            if len(self.memories) > 0:
                self.memories[-1][-1] = True
            self.fovSize = 0
            self.lastFovSize = 0
            # the history grids and lastFovSize live on the device (Model.resetBots batches this)
            st = self.field.stepper if self.field is not None else None
            if _device and st is not None:
                mask = np.zeros(len(self.field.players), np.uint8)
                mask[self.player.index] = 1
                st.reset_bots(mask)
                self.field._cache.pop("obs_rows", None)
        else:
            self.currentAction = [0, 0, 0, 0]
        self.experiences = []

    # ---- NN bots (bot.py:166-233)
    def getReward(self):  # bot.py:654-667
        p = self.parameters
        if getattr(p, "MASS_AS_REWARD", False):
            if self.player.getIsAlive():
                return self.player.getTotalMass() - p.REWARD_TERM
            return p.DEATH_TERM - p.REWARD_TERM
        if self.lastMass is None:
            return None
        if not self.player.getIsAlive():
            reward = -1 * self.lastMass * p.DEATH_FACTOR + p.DEATH_TERM
        else:
            reward = self.player.getTotalMass() - self.lastMass
        return reward * p.REWARD_SCALE - p.REWARD_TERM

    def updateRewards(self):  # bot.py:166-168
        self.cumulativeReward += self.getReward() if self.lastMass else 0
        self.lastReward = self.cumulativeReward

    def updateFrameSkip(self):  # bot.py:171-178
        if self.skipFrames > 0:
            self.skipFrames -= 1
            self.latestTDerror = None
            if self.player.getIsAlive():
                return True
        return False

    def updateValues(self, extraInfo, newAction, newState, newLastMemory=None):  # bot.py:180-192
        if newLastMemory is not None:
            self.lastMemory = newLastMemory
        self.cumulativeReward = 0
        self.skipFrames = self._param("FRAME_SKIP_RATE", 0)
        self.oldState = newState
        self.lastAction = self.currentAction
        self.currentAction = newAction
        if str(self.learningAlg) == "Q-learning":
            self.currentActionIdx = extraInfo
        else:
            self.currentRawAction = extraInfo

    def _move_nn_pre(self):  # bot.py:196-199
        self.currentlySkipping = False
        if self.learningAlg is None:
            return
        if self.currentAction is not None:
            self.updateRewards()
            self.currentlySkipping = self.updateFrameSkip()

    def _move_nn_post(self):  # bot.py:201-229
        if self.learningAlg is None:  # (facade: an NN bot without a learner steers by the
            return                    #  currentAction its caller sets -- the reference would raise)
        if self.currentlySkipping:
            return
        newState = self.getStateRepresentation()
        if self.gatherExperiences and self.oldState is not None:
            self.time += 1
            action = self.currentActionIdx if getattr(self.learningAlg, "discrete", False) else self.currentAction
            if str(self.learningAlg) != "Q-learning" and self._param("ALGORITHM", "") == "CACLA":
                self.experiences.append((self.oldState, action, self.lastReward, newState, self.currentRawAction))
            else:
                self.experiences.append((self.oldState, action, self.lastReward, newState, None))
            self.lastMemory = ([self.oldState], [action], [self.lastReward], [newState], [newState is not None])
            if self.player.getSelected():
                print("Reward: ", self.cumulativeReward)
        if self.player.getIsAlive():
            extraInfo, new_action = self.learningAlg.decideMove(newState)
            self.updateValues(extraInfo, new_action, newState)
        if self.player.getIsAlive():
            self.lastMass = self.player.getTotalMass()

    def move_NN(self):  # bot.py:194-233
        self._move_nn_pre()
        self._move_nn_post()

    def make_random_bot_move(self):  # bot.py:243-249
        if self.time % self._param("FRAME_SKIP_RATE", 7) == 0:
            self.currentAction[0] = np.random.random()
            self.currentAction[1] = np.random.random()
            self.currentAction[2] = np.random.random() if self._param("ENABLE_SPLIT", False) else False
            self.currentAction[3] = np.random.random() if self._param("ENABLE_EJECT", False) else False
        self.time += 1

    def makeMove(self, _prepared=False):  # bot.py:252-269
        if not _prepared:
            self.totalMasses.append(self.player.getTotalMass())
            if self.type == "NN":
                self._move_nn_pre()
        if self.type == "NN":
            self._move_nn_post()
        if not self.player.getIsAlive():
            return
        if self.type == "Greedy":  # one bot at a time (Model.takeBotActions batches them)
            mask = np.zeros(len(self.field.players), np.uint8)
            mask[self.player.index] = 1
            self.field._greedy_moves(mask, self._param("ENABLE_GREEDY_SPLIT", False))
            return
        if self.type == "Random":
            self.make_random_bot_move()
        if self.currentAction is None:
            return
        action = list(self.currentAction)
        if self.currentlySkipping:
            action[2:] = [0, 0]
        self.set_command_point(action)

    def set_command_point(self, action):  # bot.py:550-577
        mid = self.player.getFovPos()
        size = self.player.getFovSize()
        x, y = int(mid[0]), int(mid[1])
        left, top = x - int(size / 2), y - int(size / 2)
        size = int(size)
        split = eject = False
        if len(action) > 2:
            if len(action) == 3:
                if self._param("ENABLE_SPLIT", False):
                    split = action[2] > 0.5
                elif self._param("ENABLE_EJECT", False):
                    # the reference evaluates `[3] > 0.5` here (bot.py:568): a TypeError in Python 3
                    raise TypeError("'>' not supported between instances of 'list' and 'float'")
            else:
                split, eject = action[2] > 0.5, action[3] > 0.5
        self.player.setCommands(left + action[0] * size, top + action[1] * size, split, eject)

    def getStateRepresentation(self):  # bot.py:272-299
        if not self.player.getIsAlive():
            return None
        if not self._param("GRID_VIEW_ENABLED", True):  # getSimpleStateRepresentation (bot.py:511-547): a list
            return [float(v) for v in self.field._state_row(self.player.index)]
        if self._param("CNN_REPR", False):
            if not self._param("CNN_P_REPR", False):  # bot.py:284: the grid view [NUM_OF_GRIDS, G, G]
                row = self.field._state_row(self.player.index)
                g = self.field.grid_squares
                return row.reshape(-1, g, g).copy()
            rgb_values = self.rgbGenerator.get_cnn_inputRGB(self.player)
            stateRepr = (rgb_values - 255) / 100  # bot.py:279
            if self._param("CNN_LAST_GRID", False):
                # bot.py:281 (lastPixelGrid starts as None: the reference raises here on the first frame)
                stateRepr = np.concatenate((stateRepr, self.lastPixelGrid), axis=2)
                self.lastPixelGrid = stateRepr
            return stateRepr
        row = self.field._state_row(self.player.index)  # grid view + extras, flattened (bot.py:286-295)
        return row.reshape(1, -1).copy()

    # the parts of getStateRepresentation by their public names (bot.py:302-323,
    # 326-497, 511-547).  All read the one device observation this bot computes in
    # a tick (its history grids and last fov size advance once per tick, as they do
    # when the reference's getStateRepresentation calls them in sequence).
    def _grid_len(self):
        g = self.field.grid_squares
        return bin(int(self.field.stepper.cfg.obs_channels) & 0x3FF).count("1") * g * g

    def getGridStateRepresentation(self):  # bot.py:326-497: gridView [NUM_OF_GRIDS, G, G]
        if not self._param("GRID_VIEW_ENABLED", True):
            raise RuntimeError("getGridStateRepresentation: the field was built for the simple "
                               "representation (GRID_VIEW_ENABLED = False)")
        if not self.player.getIsAlive():
            raise RuntimeError("getGridStateRepresentation: the player is dead (the reference reads a "
                               "dead player's FOV and fails)")
        g = self.field.grid_squares
        row = self.field._state_row(self.player.index)
        return row[:self._grid_len()].reshape(-1, g, g).copy()

    def getAdditionalFeatures(self):  # bot.py:302-323: [lastFovSize, fovSize, mass, action(4), action(4)]
        if not self._param("GRID_VIEW_ENABLED", True) or not self.player.getIsAlive():
            raise RuntimeError("getAdditionalFeatures: no grid observation for this bot")
        row = self.field._state_row(self.player.index)
        return [float(v) for v in row[self._grid_len():]]

    def getSimpleStateRepresentation(self):  # bot.py:511-547: 12 values
        if self._param("GRID_VIEW_ENABLED", True):
            raise NotImplementedError("getSimpleStateRepresentation: the device computes it when the field is "
                                      "built with GRID_VIEW_ENABLED = False (one observation layout per field)")
        return [float(v) for v in self.field._state_row(self.player.index)]

    def getCoorConvGrids(self):  # bot.py:500-508
        g = self.field.grid_squares
        row, col = np.meshgrid(np.arange(g, dtype=np.float64), np.arange(g, dtype=np.float64), indexing="ij")
        return row, col

    # bookkeeping (bot.py:115-123, 235-241)
    def saveInitialModels(self, path):
        if self.learningAlg is not None:
            self.learningAlg.save(path, "init_")

    def saveModel(self, path):
        self.learningAlg.save(path)

    def resetMassList(self): self.totalMasses = []
    def setMassesOverTime(self, array): self.totalMasses = array
    def setExploring(self, val): self.player.setExploring(val)

    def getPlayer(self): return self.player
    def getType(self): return self.type
    def getLearningAlg(self): return self.learningAlg
    def getCurrentAction(self): return self.currentAction
    def getCurrentActionIdx(self): return self.currentActionIdx
    def getMassOverTime(self): return self.totalMasses
    def getAvgReward(self): return self.rewardAvgOfEpisode
    def getLastReward(self): return self.lastReward
    def getCumulativeReward(self): return self.cumulativeReward
    def getLastState(self): return self.oldState
    def getLastMemory(self): return self.lastMemory
    def getExperiences(self): return self.experiences
    def getFrameSkipRate(self): return self._param("FRAME_SKIP_RATE", 0)
    def getTrainMode(self): return getattr(self, "trainMode", None)
    def getExpRepEnabled(self): return self._param("EXP_REPLAY_ENABLED", False)
    # (the reference's getGridSquaresPerFov calls itself and never returns, bot.py:702-703)
    def getGridSquaresPerFov(self): return self.field.grid_squares


class RGBGenerator:
    """rgbGenerator.py:10-110 -- pixel observations, drawn on the device for every player at once
    (aigar_observe_pixels); get_cnn_inputRGB(player) returns one player's frame of that launch.
    Colours come from player_color / pellet_color (seeded) rather than numpy's global RNG
    (cell.py:31, player.py:39)."""

    def __init__(self, field, parameters=None):
        self.field = field
        self.parameters = parameters

        def prm(name, default):
            return getattr(parameters, name, default) if parameters is not None else default
        if prm("CNN_USE_L1", True):
            self.length = int(prm("CNN_INPUT_DIM_1", 42))
        elif prm("CNN_USE_L2", True):
            self.length = int(prm("CNN_INPUT_DIM_2", 84))
        else:
            self.length = int(prm("CNN_INPUT_DIM_3", 42))
        self.rgb = bool(prm("CNN_P_RGB", False))
        self.screenDims = np.array([self.length, self.length])

    def modelToViewScaling(self, pos, fovPos, fovSize):  # rgbGenerator.py:80-83
        return (np.asarray(pos) - fovPos + (fovSize / 2)) * (self.screenDims / fovSize)

    def viewToModelScaling(self, pos, fovPos, fovSize):  # rgbGenerator.py:86-89
        return np.asarray(pos) / (self.screenDims / fovSize) + fovPos - (fovSize / 2)

    def modelToViewScaleRadius(self, rad, fovSize):  # rgbGenerator.py:92-93
        return rad * (self.screenDims[0] / fovSize)

    def get_all_inputs(self):
        """Every player's frame: uint8 [B, L, L, 3] (CNN_P_RGB) or float64 [B, L, L, 1]."""
        f = self.field.observe_pixels_all(self.length, rgb=self.rgb)
        return f if self.rgb else f[..., None]

    def get_cnn_inputRGB(self, player):  # rgbGenerator.py:95-100
        key = ("pixels", self.length, self.rgb)  # Field drops its cache at every update / reset
        if key not in self.field._cache:
            self.field._cache[key] = self.get_all_inputs()
        return self.field._cache[key][player.index]

    @staticmethod
    def grayscale(arr):  # rgbGenerator.py:102-106
        arr = np.average(arr, axis=2, weights=[0.298, 0.587, 0.114])
        return arr.reshape(list(np.shape(arr)) + [1])


class Model:
    """model.py:48-200: the tick driver."""

    def __init__(self, guiEnabled=False, viewEnabled=False, parameters=None, seed=0, device=0, **field_kw):
        self.guiEnabled, self.viewEnabled = guiEnabled, viewEnabled
        self.parameters = parameters
        self.virusEnabled = bool(getattr(parameters, "VIRUS_SPAWN", False)) if parameters is not None else False
        self.resetLimit = getattr(parameters, "RESET_LIMIT", 20000) if parameters is not None else 20000
        self.players, self.bots, self.humans = [], [], []
        self.listeners = []
        self.playerSpectator = None
        self.spectatedPlayer = None
        self.path = None
        self.screenWidth = self.screenHeight = None
        self._field_kw = dict(field_kw)  # (kept for initParameters: a rebuilt Field keeps the sizes / flags)
        self.field = Field(self.virusEnabled, parameters, seed=seed, device=device, **field_kw)
        self.counter = 0
        # model.py:67-71: the pixel generator exists when the CNN reads pixels
        self.rgbGenerator = RGBGenerator(self.field, parameters) if (
            parameters is not None and getattr(parameters, "CNN_REPR", False) and
            getattr(parameters, "CNN_P_REPR", False)) else None

    def createPlayer(self, name):  # model.py:149-152
        p = Player(name)
        self.addPlayer(p)
        return p

    def createBot(self, botType, learningAlg=None, parameters=None):  # model.py:154-162
        name = botType + str(len(self.bots))
        p = self.createPlayer(name)
        bot = Bot(p, self.field, botType, learningAlg, parameters if parameters is not None else self.parameters,
                  self.rgbGenerator)
        self.addBot(bot)
        return bot

    def addPlayer(self, player):
        self.players.append(player)
        self.field.addPlayer(player)

    def addBot(self, bot):
        self.bots.append(bot)

    def initialize(self):  # model.py:89-92
        self.field.initialize()
        self.resetBots()

    def resetModel(self):  # model.py:94-96
        self.field.reset()
        self.counter = 0

    def takeBotActions(self):  # model.py:113-115
        """Every bot's makeMove, in list order for the ones that draw from numpy
        (Random bots, and learners that may); the world does not change between the
        moves, so the parts that read it are batched: every Greedy bot's move in one
        device launch, every NN bot's state in one masked observation."""
        for bot in self.bots:
            bot.totalMasses.append(bot.player.getTotalMass())
            if bot.type == "NN":
                bot._move_nn_pre()
        need = [b.player.index for b in self.bots if b.type == "NN" and b.learningAlg is not None and
                not b.currentlySkipping and b.player.getIsAlive() and not b._param("CNN_REPR", False)]
        if need:
            self.field._prefetch_states(need)
        greedy = [b for b in self.bots if b.type == "Greedy"]
        if greedy:  # (their moves are independent of each other and of the other bots')
            mask = np.zeros(len(self.players), np.uint8)
            for b in greedy:
                mask[b.player.index] = 1
            self.field._greedy_moves(mask, bool(getattr(self.parameters, "ENABLE_GREEDY_SPLIT", False)))
        for bot in self.bots:
            if bot.type != "Greedy":
                bot.makeMove(_prepared=True)

    def resetBots(self):  # model.py:117-119 (the NN bots' device history in one call)
        for bot in self.bots:
            bot.reset(_device=False)
        nn = [b.player.index for b in self.bots if b.type == "NN"]
        if nn and self.field.stepper is not None:
            mask = np.zeros(len(self.players), np.uint8)
            mask[nn] = 1
            self.field.stepper.reset_bots(mask)
            self.field._cache.pop("obs_rows", None)

    def update(self):  # model.py:98-111
        self.counter += 1
        nn = [b for b in self.bots if b.type == "NN"]
        if nn and self.parameters is not None and (getattr(self.parameters, "USE_LAST_ACTION", False) or
                                                   getattr(self.parameters, "USE_SECOND_LAST_ACTION", False)):
            self.field._set_actions(nn)
        self.takeBotActions()
        self.field.update()
        if self.guiEnabled and self.viewEnabled:  # model.py:107-108
            self.notify()

    def initParameters(self, parameters):  # model.py:79-84 (before initialize: the world is sized then)
        if self.field.stepper is not None:
            raise RuntimeError("initParameters after initialize(): the device world is already built")
        self.parameters = parameters
        self.virusEnabled = bool(getattr(parameters, "VIRUS_SPAWN", False))
        self.resetLimit = getattr(parameters, "RESET_LIMIT", self.resetLimit)
        self.field = Field(self.virusEnabled, parameters, seed=self.field.seed, device=self.field.device,
                           **self._field_kw)
        for p in self.players:
            p.field = None
            self.field.addPlayer(p)
        for b in self.bots:
            b.field = self.field

    def modifySettings(self, reset_time):  # model.py:87-88
        self.resetLimit = reset_time

    def printBotMasses(self):  # model.py:139-142
        for bot in self.bots:
            mass = bot.getPlayer().getTotalMass()
            print("Mass of ", bot.getPlayer(), ": ", round(mass, 1) if mass is not None else "Dead")

    def createHuman(self, name):  # model.py:165-167
        self.addHuman(self.createPlayer(name))

    def addHuman(self, human): self.humans.append(human)

    def addPlayerSpectator(self):  # model.py:181-183
        self.playerSpectator = True
        self.setSpectatedPlayer(self.players[0])

    def setPath(self, path): self.path = path
    def setSpectatedPlayer(self, player): self.spectatedPlayer = player
    def setViewEnabled(self, boolean): self.viewEnabled = boolean

    def setScreenSize(self, width, height):
        self.screenWidth, self.screenHeight = width, height

    # checks (model.py:201-205)
    def hasHuman(self): return bool(self.humans)
    def hasPlayerSpectator(self): return self.playerSpectator is not None

    # getters (model.py:208-270)
    def getNNBot(self):
        for bot in self.bots:
            if bot.getType() == "NN":
                return bot
        return None

    def getNNBots(self): return [bot for bot in self.bots if bot.getType() == "NN"]

    def getTopTenPlayers(self):  # stable sort by total mass, descending (list.sort is stable)
        players = self.getPlayers()[:]
        players.sort(key=lambda p: p.getTotalMass(), reverse=True)
        return players[0:10]

    def getFovPos(self, humanNr):
        if self.hasHuman():
            return np.array(self.humans[humanNr].getFovPos())
        if self.hasPlayerSpectator():
            return np.array(self.spectatedPlayer.getFovPos())
        return np.array([self.field.getWidth() / 2, self.field.getHeight() / 2])

    def getFovSize(self, humanNr):
        if self.hasHuman():
            return self.humans[humanNr].getFovSize()
        if self.hasPlayerSpectator():
            return self.spectatedPlayer.getFovSize()
        return self.field.getWidth()

    def getSpectatedPlayer(self):
        if self.hasHuman():
            return self.humans
        if self.hasPlayerSpectator():
            return self.spectatedPlayer
        return None

    def getField(self): return self.field
    def getPellets(self): return self.field.getPellets()
    def getViruses(self): return self.field.getViruses()
    def getPlayerCells(self): return self.field.getPlayerCells()
    def getPlayers(self): return self.players
    def getBots(self): return self.bots
    def getHumans(self): return self.humans
    def getParameters(self): return self.parameters
    def getVirusEnabled(self): return self.virusEnabled

    # MVC (model.py:273-281)
    def set_GUI(self, value): self.guiEnabled = value
    def register_listener(self, listener): self.listeners.append(listener)

    def notify(self):
        for listener in self.listeners:
            listener()
