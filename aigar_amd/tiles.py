"""C4: one arena tiled 2-D over several stepper handles.

The reference steps one `Field` (field.py:85-92) in one process.  Here the
arena's field is cut into `tile_x * tile_y` bucket-aligned tiles, one handle
each (one GPU each in production).  Every handle replays the whole tick on its
replica of the players, cells, blobs and viruses -- a few thousand records, so
the player-ordered phases (updatePlayers, merges, virus phases,
playerPlayerOverlap, spawns) need no exchange -- and holds only the pellets of
its tile plus a halo.  The eat phase (playerPelletOverlap + playerBlobOverlap,
field.py:207-222) is resolved per tile in the reference's global priority order
(player, cell list position, food creation sequence); the cells a tile owns
(centre bucket in the tile) report their outcomes -- pellet and blob kills, new
masses, which cells are final -- in one message per pass that every tile
all-gathers (`include/aigar.h`, aigar_tile_*).  The spawn deficit is global:
the messages carry each tile's pellet kills.

The observation (bot.py:272-497) is divided: every bot is observed by ONE tile
-- the one holding its last-frame history grids, else the tile of its view
centre -- and a bot whose view centre changed tile (or that died) has its
history handed off in the next tick's first message.  Every tile computes the
same assignment (`aigar_tile_observers`).

Transports:
  - RCCL inside the library (`rccl_comm` + `Stepper.tile_run`): one tile per rank,
    the exchange an ncclAllGather on the tile's stream, the whole tiled step one
    hipGraph replay -- the production path (bench.py on the nccl backend).
  - `LocalTransport`: all tiles in this process (one GPU): device copies.
  - `TorchTransport`: one tile per rank; `torch.distributed.all_gather_into_tensor`
    over the process group (RCCL over xGMI on the `nccl` backend; gloo on CPU
    for the exchange-layer tests).
"""
import ctypes as C

import numpy as np

from . import _abi
from . import _lib


def tile_grid(n):
    """tiles (x, y) for n tiles: 1 -> 1x1, 2 -> 2x1, 4 -> 2x2, 8 -> 4x2."""
    return {1: (1, 1), 2: (2, 1), 4: (2, 2), 8: (4, 2)}.get(n) or (n, 1)


def tile_config(cfg, tx, ty, tile_id, halo=0, cap=0, flags=0):
    c = _abi.Config()
    C.memmove(C.byref(c), C.byref(cfg), C.sizeof(_abi.Config))
    c.tile_x, c.tile_y, c.tile_id, c.tile_halo, c.tile_cap = tx, ty, tile_id, int(halo), int(cap)
    c.tile_flags = int(flags)
    return c


def merge_events(raws):
    """Merge the tiles' raw event logs (key_hi, key_lo, code, a, b) into the
    reference-ordered rows (tick, code, a, b), as aigar_get_events sorts one log."""
    rows = np.concatenate([r for r in raws if len(r)] or [np.zeros((0, 5), np.int64)])
    if not len(rows):
        return np.zeros((0, 4), np.int64)
    lo = rows[:, 1].view(np.uint64)
    order = np.lexsort((lo, rows[:, 0]))
    r = rows[order]
    return np.stack([r[:, 0] >> 8, r[:, 2], r[:, 3], r[:, 4]], axis=1)


def merge_states(states):
    """Snapshot of the whole arena from the tiles' snapshots: the replicated part
    from tile 0 (every tile holds the same), the pellets as the union of what each
    tile owns, sorted by creation sequence."""
    d = dict(states[0])
    pf = np.concatenate([s["pellets_f"] for s in states])
    ps = np.concatenate([s["pellets_seq"] for s in states])
    o = np.argsort(ps, kind="stable")
    d["pellets_f"], d["pellets_seq"] = pf[o], ps[o]
    if all("pellets_col" in s for s in states):
        d["pellets_col"] = np.concatenate([s["pellets_col"] for s in states])[o]
    d["n_pellets"] = len(ps)
    return d


def tiled_tick(tiles, transport, policy="none", p_split=0.0, p_eject=0.0, seed=0, obs=None, extra_passes=None,
               greedy_split=False):
    """One tick of the tiles in `tiles` (all of them, or this rank's one): begin,
    then exchange / apply passes until no owned cell is undone on any tile (the
    count comes with the messages, so every tile takes the same decision), then
    the rest of the tick.  Returns the number of eat passes issued.

    extra_passes=K (an int): no host round trip -- K further passes are issued
    whatever happens and do nothing on the device once every cell is final; the
    tick raises (device error bit) if cells are still undone after them.  With
    the default halo every cell is decided by the first pass (K = 0).

    policy "greedy": the reference's Greedy bots (bot.py:579-633) -- each tile
    moves the bots it observes (it holds their whole view), and the commands go
    round in one exchange before the tick."""
    if policy == "greedy":
        for t in tiles:
            t.tile_policy(greedy_split)
        transport.exchange(tiles)
        for t in tiles:
            t.tile_apply_commands()
    for t in tiles:
        t.tile_begin(policy, p_split, p_eject, seed)
    passes = 1
    transport.exchange(tiles)
    if extra_passes is not None:
        for t in tiles:
            t.tile_apply(wait=False)
        for _ in range(int(extra_passes)):
            for t in tiles:
                t.tile_resume()
            transport.exchange(tiles)
            for t in tiles:
                t.tile_apply(wait=False)
            passes += 1
        for k, t in enumerate(tiles):
            t.tile_end(None if obs is None else obs[k])
        return passes
    undone = [t.tile_apply() for t in tiles]
    while undone[0] > 0:
        if len(set(undone)) != 1:
            raise RuntimeError("tiles disagree on the undone count: %r" % undone)
        for t in tiles:
            t.tile_resume()
        transport.exchange(tiles)
        undone = [t.tile_apply() for t in tiles]
        passes += 1
        if passes > 64:
            raise RuntimeError("tiled eat phase did not converge")
    for k, t in enumerate(tiles):
        t.tile_end(None if obs is None else obs[k])
    return passes


def rccl_comm(stepper, dist=None, group=None):
    """Give this rank's tile handle an RCCL communicator over all the tiles (rank =
    tile id): rank 0 makes the ncclUniqueId, the process group broadcasts it.
    Then `stepper.tile_run` steps the tile with the exchange as an RCCL all-gather
    inside the step's hipGraph (no Python, no host round trip per tick)."""
    info = stepper.tile_info()
    n, k = info["ntiles"], info["tile_id"]
    uid = _lib.rccl_unique_id() if k == 0 else None
    if n > 1:
        box = [uid]
        dist.broadcast_object_list(box, src=0, group=group)
        uid = box[0]
    stepper.tile_comm_init(uid, n, k)


class LocalTransport:
    """All tiles in one process: every outbox copied into every inbox on the device."""

    def exchange(self, steppers):
        _lib.tile_exchange_local(steppers)


class TiledArena:
    """One arena over tile_x * tile_y tile handles in this process (one GPU):
    the parity tests' and the single-box benchmark's driver of the tiled tick."""

    def __init__(self, cfg, tx, ty, halo=0, cap=0, flags=0, transport=None):
        if cfg.n_arenas != 1:
            raise ValueError("a tiled arena is one arena")
        self.tx, self.ty = tx, ty
        self.tiles = [_lib.Stepper(tile_config(cfg, tx, ty, k, halo, cap, flags)) for k in range(tx * ty)]
        self.transport = transport or LocalTransport()
        self.NP = cfg.bots_per_arena
        self.obs_len = self.tiles[0].obs_len
        self.passes = []  # eat passes of each tick (1 unless a cross-tile chain needed more)

    def close(self):
        for t in self.tiles:
            t.close()

    def reset(self, seed=0):
        for t in self.tiles:
            t.reset(seed)

    def load_state(self, d):
        for t in self.tiles:
            t.load_state(d)

    def set_commands(self, cmd):
        for t in self.tiles:
            t.set_commands(cmd)

    def tick(self, policy="none", p_split=0.0, p_eject=0.0, seed=0, obs=None, extra_passes=None, greedy_split=False):
        """One Field.update() of the tiled arena; obs: per-tile device tensors
        (each tile writes the rows of the bots it observes)."""
        self.passes.append(tiled_tick(self.tiles, self.transport, policy, p_split, p_eject, seed, obs, extra_passes,
                                      greedy_split))

    def step(self, n=1, **kw):
        for _ in range(n):
            self.tick(**kw)

    def get_state(self):
        return merge_states([t.get_state() for t in self.tiles])

    def events(self):
        return merge_events([t.events_raw() for t in self.tiles])

    def _geometry(self):
        if not hasattr(self, "_geo"):
            self._geo = [t.tile_info() for t in self.tiles]
        return self._geo

    def owner(self, x, y):
        """Tile owning the centre bucket of each (x, y); -1 where x or y is NaN
        (a dead player's FOV)."""
        x, y = np.asarray(x, np.float64), np.asarray(y, np.float64)
        ok = np.isfinite(x) & np.isfinite(y)
        cols = max(g["own"][1] for g in self._geometry())
        bx = np.clip(np.where(ok, x, 0.0) // 20, 0, cols - 1).astype(np.int64)
        by = np.clip(np.where(ok, y, 0.0) // 20, 0, cols - 1).astype(np.int64)
        own = np.full(bx.shape, -1, np.int64)
        for k, g in enumerate(self._geometry()):
            x0, x1, y0, y1 = g["own"]
            own[ok & (bx >= x0) & (bx < x1) & (by >= y0) & (by < y1)] = k
        return own

    def observe(self):
        """Every bot's observation: each tile computes the rows of the bots it
        observes (aigar_tile_observers: the same assignment on every tile); dead
        bots get NaN rows."""
        rows = [t.observe() for t in self.tiles]
        by = self.tiles[0].tile_observers()
        for t in self.tiles[1:]:
            if not np.array_equal(t.tile_observers(), by):
                raise RuntimeError("tiles disagree on the observation owners")
        self.last_observers = by
        out = np.full((self.NP, self.obs_len), np.nan)
        for k in range(len(self.tiles)):
            sel = by == k
            out[sel] = rows[k][sel]
        return out

    def player_stats(self):
        return self.tiles[0].player_stats()


class TorchTransport:
    """One tile per rank: the exchange is one all-gather of fixed-size messages
    over the process group (RCCL on `nccl`, gloo on CPU).  The tile's outbox /
    inbox are torch tensors the collective writes in place; `for_stepper` hands
    them to the tile handle (and the handle adopts torch's stream, so the
    collective and the tile kernels are ordered on one queue).  staged: the
    process group cannot take device tensors (gloo rehearsal on GPUs): the
    message goes through host copies."""

    def __init__(self, msg_bytes, ntiles, device, group=None, staged=False):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.msg_bytes, self.ntiles = int(msg_bytes), int(ntiles)
        self.outbox = torch.zeros(self.msg_bytes, dtype=torch.uint8, device=device)
        self.inbox = torch.zeros(self.ntiles * self.msg_bytes, dtype=torch.uint8, device=device)
        self.staged = bool(staged) and self.outbox.is_cuda
        if self.staged:
            self._ho = torch.zeros(self.msg_bytes, dtype=torch.uint8)
            self._hi = torch.zeros(self.ntiles * self.msg_bytes, dtype=torch.uint8)
        self._marks = []

    @classmethod
    def for_stepper(cls, stepper, group=None, staged=False):
        import torch
        info = stepper.tile_info()
        dev = torch.device("cuda", torch.cuda.current_device())
        t = cls(info["msg_bytes"], info["ntiles"], dev, group, staged)
        stepper.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        stepper.tile_set_buffers(t.outbox.data_ptr(), t.inbox.data_ptr())
        return t

    def exchange(self, steppers=None):
        """All-gather this pass's messages (steppers: this rank's tile, whose current
        message size is taken; default: the full message)."""
        torch = self.torch
        n = steppers[0].tile_msg_bytes() if steppers else self.msg_bytes
        nt = self.ntiles * n
        timed = self.outbox.is_cuda
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        if self.staged:
            self._ho[:n].copy_(self.outbox[:n])
            self.dist.all_gather_into_tensor(self._hi[:nt], self._ho[:n], group=self.group)
            self.inbox[:nt].copy_(self._hi[:nt])
        else:
            self.dist.all_gather_into_tensor(self.inbox[:nt], self.outbox[:n], group=self.group)
        if timed:
            e1.record()
            self._marks.append((e0, e1))

    def reset_timing(self):
        self._marks = []

    def avg_exchange_ms(self):
        """Average device time of one exchange since reset_timing (CUDA events)."""
        if not self._marks:
            return None
        self.torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self._marks) / len(self._marks)


# ---- message layout (include/aigar.h aigar_tile_info; aigar_dev.h TileRec)
TILE_REC = np.dtype([("kind", "<i4"), ("idx", "<i4"), ("seq", "<i8"), ("x", "<f8"), ("y", "<f8")])
TR_HDR, TR_PELLET, TR_BLOB, TR_CELL = 0, 1, 2, 3


def pack_message(records, undone, tcap, bm_words, final_cells=()):
    """Host image of one tile's message: header, records (a TILE_REC array), the
    final-cell bitmap; the header counts the pellet kills among the records."""
    recs = np.zeros(1 + tcap + bm_words // 4, TILE_REC)
    n = len(records)
    if n > tcap:
        raise ValueError("message overflow: %d records > %d" % (n, tcap))
    recs[1:1 + n] = records
    recs[0] = (TR_HDR, n, undone, float(np.sum(np.asarray(records["kind"]) == TR_PELLET)) if n else 0.0, 0.0)
    bm = recs[1 + tcap:].view(np.uint64)
    for c in final_cells:
        bm[c >> 6] |= np.uint64(1) << np.uint64(c & 63)
    return recs.view(np.uint8)


def unpack_message(buf, tcap, bm_words):
    """(header dict, records, final cells) of one message image."""
    recs = np.frombuffer(np.ascontiguousarray(buf, np.uint8).tobytes(), TILE_REC)
    h = recs[0]
    n = int(h["idx"])
    bm = recs[1 + tcap:1 + tcap + bm_words // 4].view(np.uint64)
    bits = np.unpackbits(bm.view(np.uint8), bitorder="little")
    return ({"records": n, "undone": int(h["seq"]), "pellet_kills": int(h["x"])}, recs[1:1 + n].copy(),
            np.nonzero(bits)[0])
