"""GPU: C4 -- one arena tiled 2-D over tile handles (aigar_amd/tiles.py, the
aigar_tile_* C-ABI) against the UNTILED oracle.

Every tile replays the tick on its replica of the players, cells, blobs and
viruses and holds only its tile's pellets plus a halo; the eat phase
(field.py:207-222) is resolved per tile and the owners' outcomes are
all-gathered (in-process device copies here; RCCL in production).  The bar is
the untiled one: the merged event log (every eat / merge / split / explosion /
death / respawn, indices and order) equals the oracle's exactly, the merged
state (replicated part from tile 0, pellets as the union of the owned sets)
within 1e-5, observations within 1e-5 for every bot.  Small halos force the
cross-tile paths: cells whose reach leaves the held pellets (excluded), the
taint of cells that share a food with them, and further exchange passes.
"""
import numpy as np
import pytest

from aigar_amd import _abi
from oracle_lib import Oracle, make_config
import parity

pytestmark = pytest.mark.gpu
_lib = pytest.importorskip("aigar_amd._lib")
from aigar_amd.tiles import TiledArena  # noqa: E402

C3_CH = (_abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_VIRUS | _abi.OBS_SELF_LF
         | _abi.OBS_ENEMY_LF)


def run(cfg, tx, ty, ticks, seed, cmd_fn, halo=0, obs_every=0, check_every=10, ftol=parity.FTOL, flags=0,
        start=None, extra_passes=None):
    ta, o = TiledArena(cfg, tx, ty, halo=halo, flags=flags), Oracle(cfg)
    if start is None:
        ta.reset(seed)
        o.reset(seed)
    else:  # a matured world (tools/mature.py): every tile keeps the pellets it holds
        ta.load_state(start)
        o.load_state(start)
    dif = parity.diff_states(ta.get_state(), o.get_state())
    assert not dif, dif
    kinds, nev = set(), 0
    prev_by, moved, per_tile = None, 0, np.zeros(tx * ty, np.int64)
    for t in range(ticks):
        cmd = cmd_fn(t, o)
        ta.set_commands(cmd)
        o.set_commands(cmd)
        ta.tick(extra_passes=extra_passes)
        o.step(1)
        eg, eo = ta.events(), o.events()
        if not np.array_equal(eg, eo):
            n = min(len(eg), len(eo))
            bad = next((i for i in range(n) if not np.array_equal(eg[i], eo[i])), n)
            raise AssertionError("tick %d: event %d differs (tiles %d events, oracle %d): %s vs %s" % (
                t, bad, len(eg), len(eo), eg[bad:bad + 2].tolist(), eo[bad:bad + 2].tolist()))
        kinds |= set(eo[:, 1].tolist())
        nev += len(eo)
        if (t + 1) % check_every == 0 or t == ticks - 1:
            dif = parity.diff_states(ta.get_state(), o.get_state(), ftol)
            assert not dif, "tick %d: %s" % (t, dif[:3])
        if obs_every and (t + 1) % obs_every == 0:
            og, oo = ta.observe(), o.observe()
            assert parity.obs_close(og, oo), "tick %d: observations differ" % t
            by = ta.last_observers
            alive = o.player_stats()[:, 0] > 0
            assert np.array_equal(by >= 0, alive), "tick %d: observed set != alive set" % t
            per_tile += np.bincount(by[by >= 0], minlength=tx * ty)
            if prev_by is not None:  # a bot observed by another tile than last time: its history was handed off
                moved += int(np.sum((by >= 0) & (prev_by >= 0) & (by != prev_by)))
            prev_by = by
    stats = {"kinds": kinds, "events": nev, "passes": list(ta.passes), "moved": moved, "per_tile": per_tile}
    ta.close()
    o.close()
    return stats


def synthetic(n, size, ps, pe, seed):
    rng = np.random.default_rng(seed)
    return lambda t, o: parity.synthetic_commands(rng, None, n, size, ps, pe)


def greedy(gsplit):
    def f(t, o):
        o.policy_greedy(gsplit)
        return o.commands()
    return f


def c3_config(**kw):
    return make_config(bots=4096, field_size=4800, virus=True, max_pellets=100000.0, channels=C3_CH, extras=0x1F,
                       **kw)


@pytest.mark.parametrize("tx,ty", [(2, 1), (2, 2), (4, 2)])
def test_c3_tiled_matches_untiled_oracle(tx, ty):
    """C3 (4096 bots, 100k pellets, 1152 viruses, split p 2.5e-3 / eject p 1e-2)
    from the matured tick-600 world (cells past 125, multi-cell players), 200 ticks:
    splits, ejections, blob eating, explosions, merges, cell-eats-cell across the
    tile borders.  (4, 2) is C4's own layout (tiles 1200 x 2400).
    Every 25 ticks every bot's observation, each from the one tile that observes
    it (its history holder or its view centre's tile): bots that crossed a border
    in between arrive with their history handed off."""
    st = run(c3_config(), tx, ty, 200, 31, synthetic(4096, 4800, 2.5e-3, 1e-2, 31), obs_every=25, check_every=25,
             start=parity.load_snapshot("c3_t600"))
    assert st["events"] > 10000
    assert {_abi.EV_CELL_EAT_PELLET, _abi.EV_CELL_EAT_BLOB, _abi.EV_RESPAWN, _abi.EV_MERGE, _abi.EV_EXPLODE,
            _abi.EV_CELL_EAT_CELL, _abi.EV_CELL_EAT_VIRUS} <= st["kinds"], st["kinds"]
    assert st["moved"] > 0, "no bot changed its observing tile"
    # the observation is divided: every tile observes its share (~1/N of the bots)
    share = st["per_tile"] / st["per_tile"].sum()
    assert share.max() < 2.0 / (tx * ty), share


def test_c3_4x2_history_handoff_every_tick():
    """C4 layout, observation EVERY tick for 60 ticks (the last-frame channels
    compare each bot's history): a bot whose view centre crosses into another
    tile, or that dies and respawns anywhere, is observed next by a tile that got
    its history in that tick's first message; no host round trip per pass
    (extra_passes=0: the device-bounded path the benchmark runs)."""
    st = run(c3_config(), 4, 2, 60, 33, synthetic(4096, 4800, 2.5e-3, 1e-2, 33), obs_every=1, check_every=20,
             start=parity.load_snapshot("c3_t600"), extra_passes=0)
    assert st["moved"] >= 10, st["moved"]
    assert set(st["passes"]) == {1}


def test_device_bounded_passes_raise_when_cells_stay_undone():
    """extra_passes=0 with a small halo deciding only owned cells: a tick that needs
    a second exchange pass must fail loudly (device error bit), not go on."""
    with pytest.raises(RuntimeError, match="device error bits"):
        run(c3_config(), 2, 2, 60, 32, synthetic(4096, 4800, 2.5e-3, 1e-2, 32), halo=140, check_every=10,
            flags=_abi.TILE_OWNED_ONLY, start=parity.load_snapshot("c3_t600"), extra_passes=0)


def test_view_beyond_the_held_pellets_is_refused():
    """A view the observing tile does not hold (here: a cell at the mass cap on a
    tile border, view ~287 wide, with the smallest halo, 7 buckets) must raise
    instead of returning a row with pellets missing."""
    cfg = make_config(bots=256, channels=C3_CH, extras=0x1F)
    o = Oracle(cfg)
    o.reset(3)
    snap = o.get_state()
    o.close()
    owner = np.asarray(snap["cells_i"])[:, 0]
    k = int(np.nonzero(owner == 0)[0][0])
    cf = np.array(snap["cells_f"], copy=True)
    cf[k, 0] = cf[k, 1] = 600.5
    cf[k, 2] = 22500.0
    cf[k, 3] = np.sqrt(22500.0 / np.pi)
    snap["cells_f"] = cf
    ta = TiledArena(cfg, 2, 2, halo=140)
    ta.load_state(snap)
    with pytest.raises(RuntimeError, match="device error bits"):
        ta.observe()
    ta.close()


def test_c3_small_halo_forces_cross_tile_passes():
    """2 x 2 tiles with the smallest halo (an owned cell's reach) deciding only the
    cells they own (AIGAR_TILE_OWNED_ONLY): every cell near a border that shares a
    food with a higher-priority cell of another tile is tainted and waits for that
    tile's message, so ticks take several exchange passes; the result must still
    be the untiled world."""
    st = run(c3_config(), 2, 2, 60, 32, synthetic(4096, 4800, 2.5e-3, 1e-2, 32), halo=140, check_every=20,
             flags=_abi.TILE_OWNED_ONLY, start=parity.load_snapshot("c3_t600"))
    assert st["events"] > 3000
    assert max(st["passes"]) > 1


@pytest.mark.parametrize("tx,ty,flags,seed", [(2, 2, _abi.TILE_OWNED_ONLY, 4), (2, 1, _abi.TILE_OWNED_ONLY, 5),
                                               (2, 2, 0, 6)])
def test_border_crowded_greedy_tiles(tx, ty, flags, seed):
    """64 greedy bots in a 250-unit field cut into 2 x 2 (or 2 x 1) tiles: bots
    chase each other across the tile edges, cells eat pellets, blobs and each
    other there and explode on viruses near them; 300 ticks against the untiled
    oracle.  With AIGAR_TILE_OWNED_ONLY every tile decides only its own cells,
    so contested border foods go through the taint / extra-pass exchange."""
    cfg = make_config(bots=64, virus=True, max_viruses=30, field_size=250,
                      channels=_abi.OBS_PELLET | _abi.OBS_WALL | _abi.OBS_ENEMY, extras=0x3)
    st = run(cfg, tx, ty, 300, seed, greedy(True), check_every=10, ftol=1e-9, flags=flags)
    assert {_abi.EV_CELL_EAT_CELL, _abi.EV_PLAYER_DEATH, _abi.EV_CELL_EAT_PELLET,
            _abi.EV_EXPLODE} <= st["kinds"], st["kinds"]
    if flags:
        assert max(st["passes"]) > 1, "the scenario never needed a second exchange pass"


def test_tiled_load_state_continues_like_the_oracle():
    """A tiled arena loaded from a mid-run oracle snapshot (each tile keeps its
    held pellets) continues exactly like the oracle."""
    cfg = make_config(bots=256, virus=True, max_viruses=40, channels=C3_CH, extras=0x1F)
    o = Oracle(cfg)
    o.reset(9)
    rng = np.random.default_rng(9)
    for _ in range(40):
        o.set_commands(parity.synthetic_commands(rng, None, 256, 1200, 0.02, 0.05))
        o.step(1)
    snap = o.get_state()
    ta = TiledArena(cfg, 2, 2, halo=100)
    ta.load_state(snap)
    dif = parity.diff_states(ta.get_state(), snap)
    assert not dif, dif
    for t in range(60):
        cmd = parity.synthetic_commands(rng, None, 256, 1200, 0.02, 0.05)
        ta.set_commands(cmd)
        o.set_commands(cmd)
        ta.tick()
        o.step(1)
        assert np.array_equal(ta.events(), o.events()), "tick %d" % t
    dif = parity.diff_states(ta.get_state(), o.get_state())
    assert not dif, dif
    ta.close()
    o.close()


def test_c3_4x2_gated_extra_pass_matches_oracle():
    """extra_passes=1 (the bench's fallback): the second pass is issued blindly
    and gated on the device.  With the default halo every cell is final after
    the first pass, so the second is gated on every tick; its message must be an
    empty header (k_tile_pass_begin), not the first pass's header again -- a
    stale one would add every tile's pellet kills twice and over-spawn pellets
    (n_pellets and ctr_pellet drift from the oracle within a tick)."""
    st = run(c3_config(), 4, 2, 40, 35, synthetic(4096, 4800, 2.5e-3, 1e-2, 35), obs_every=5, check_every=1,
             start=parity.load_snapshot("c3_t600"), extra_passes=1)
    assert set(st["passes"]) == {2}
    assert _abi.EV_CELL_EAT_PELLET in st["kinds"] and _abi.EV_RESPAWN in st["kinds"]


def _crossing_world(n_move=64, seed=11):
    """A 256-bot reset world (field 1200, 2 x 1 tiles: tile 0 holds x < 600) with
    bots 0..n_move-1 moved to x = 595 in a column, one cell each."""
    cfg = make_config(bots=256, channels=C3_CH, extras=0x1F)
    o = Oracle(cfg)
    o.reset(seed)
    snap = o.get_state()
    o.close()
    cf = np.array(snap["cells_f"], copy=True)
    owner = np.asarray(snap["cells_i"])[:, 0]
    for p in range(n_move):
        k = int(np.nonzero(owner == p)[0][0])
        cf[k, 0], cf[k, 1] = 595.0, 80.0 + 16.0 * p
        cf[k, 4:8] = 0.0
    snap["cells_f"] = cf
    return cfg, snap, owner


def test_many_bots_crossing_a_border_in_one_tick():
    """64 bots observed by tile 0 cross into tile 1 in the same tick: more than
    the hand-off slots of one message (16 at tile_cap 512).  The lowest player
    indices are handed off first, the rest stay with tile 0 a tick longer (their
    view is inside its halo) and follow in the next messages; every bot's
    observation, history channels included, equals the oracle's every tick."""
    cfg, snap, _ = _crossing_world()
    ta, o = TiledArena(cfg, 2, 1, cap=512), Oracle(cfg)
    assert ta.tiles[0].tile_info()["hcap"] == 16
    ta.load_state(snap)
    o.load_state(snap)
    rng = np.random.default_rng(3)
    moves, moved_sets = [], []
    prev = None
    for t in range(14):
        cmd = parity.synthetic_commands(rng, None, 256, 1200)
        cmd[:64, 0], cmd[:64, 1] = 1190.0, 80.0 + 16.0 * np.arange(64)  # straight across the border
        ta.set_commands(cmd)
        o.set_commands(cmd)
        ta.tick(extra_passes=0)
        o.step(1)
        assert np.array_equal(ta.events(), o.events()), "tick %d" % t
        og, oo = ta.observe(), o.observe()
        assert parity.obs_close(og, oo), "tick %d: observations differ" % t
        by = ta.last_observers[:64].copy()
        if prev is not None:
            moves.append(int(np.sum((prev == 0) & (by == 1))))
            if moves[-1]:
                moved_sets.append(np.nonzero((prev == 0) & (by == 1))[0])
        prev = by
    dif = parity.diff_states(ta.get_state(), o.get_state())
    assert not dif, dif
    assert np.all(prev == 1), prev
    # the crossing happened in one tick but the hand-offs were spread over several,
    # in a fixed order: the lowest player indices first, and a bot passed over goes
    # before any newcomer (the choice never depends on atomic order)
    assert max(moves) == 16 and sum(moves) == 64, moves
    assert np.array_equal(np.concatenate(moved_sets), np.arange(64)), moved_sets
    ta.close()
    o.close()


def test_dead_bots_beyond_the_hand_off_slots_raise():
    """More bots held by one tile die in one tick than its message has hand-off
    slots: a dead bot respawns anywhere, so its history may not wait for a later
    message -- the tick must fail with its own error bit (16384), not defer."""
    cfg, snap, owner = _crossing_world(n_move=0)
    cf = np.array(snap["cells_f"], copy=True)
    big = int(np.nonzero(owner == 100)[0][0])
    cf[big, 0], cf[big, 1], cf[big, 2] = 400.0, 600.0, 20000.0
    cf[big, 3] = np.sqrt(20000.0 / np.pi)
    ang = np.arange(64) * 2 * np.pi / 64
    for p in range(64):  # a ring around the big cell, just out of its reach
        k = int(np.nonzero(owner == p)[0][0])
        cf[k, 0], cf[k, 1] = 400.0 + 84.0 * np.cos(ang[p]), 600.0 + 84.0 * np.sin(ang[p])
        cf[k, 4:8] = 0.0
    snap["cells_f"] = cf
    ta = TiledArena(cfg, 2, 1, cap=512)
    ta.load_state(snap)
    ta.observe()  # tile 0 becomes the ring bots' history holder
    cmd = np.zeros((256, 4))
    cmd[:, 0], cmd[:, 1] = 400.0, 600.0
    with pytest.raises(RuntimeError, match=r"device error bits 0x4[0-9a-f]{3} "):
        for _ in range(12):
            ta.set_commands(cmd)
            ta.tick(extra_passes=0)
            ta.observe()
    ta.close()


def _commands(st):
    pf, pi = np.asarray(st["players_f"]), np.asarray(st["players_i"])
    return np.c_[pf[:, 0], pf[:, 1], pi[:, 2], pi[:, 3]].astype(np.float64)


def test_c3_4x2_greedy_bots_on_tiles():
    """the reference's Greedy bots (bot.py:579-633 with
    ENABLE_GREEDY_SPLIT) driving C4's own layout.  No tile holds every pellet, so
    each tile moves the bots it observes (their history holder, else their view
    centre's tile: it holds the whole view) and the commands are all-gathered
    before the tick (aigar_tile_policy / aigar_tile_apply_commands).  From the
    matured tick-50 world, 40 ticks: every bot's command equals the oracle's own
    Greedy move, the merged events every tick, the state every 10 ticks, every
    bot's observation every 5 (observations hand histories, and with them the
    moving tile, from tile to tile)."""
    cfg = c3_config()
    start = parity.load_snapshot("c3_t50")
    ta, o = TiledArena(cfg, 4, 2), Oracle(cfg)
    ta.load_state(start)
    o.load_state(start)
    nev, splits = 0, 0
    for t in range(40):
        o.policy_greedy(True)
        want = o.commands()
        ta.tick(policy="greedy", greedy_split=True)
        for k, tile in enumerate(ta.tiles):
            got = _commands(tile.get_state())
            bad = np.argwhere(got != want)
            assert not len(bad), "tick %d tile %d bot %d: %s vs oracle %s" % (t, k, bad[0][0], got[bad[0][0]],
                                                                              want[bad[0][0]])
        splits += int(want[:, 2].sum())
        o.step(1)
        eg, eo = ta.events(), o.events()
        assert np.array_equal(eg, eo), "tick %d: events differ (%d vs %d)" % (t, len(eg), len(eo))
        nev += len(eo)
        if (t + 1) % 10 == 0:
            dif = parity.diff_states(ta.get_state(), o.get_state())
            assert not dif, "tick %d: %s" % (t, dif[:3])
        if (t + 1) % 5 == 0:
            assert parity.obs_close(ta.observe(), o.observe()), "tick %d: observations differ" % t
    assert nev > 5000 and splits > 0, (nev, splits)
    ta.close()
    o.close()
