"""GPU: the state-representation variants of Bot.getStateRepresentation
(bot.py:272-299) beside the default grid (a25 of SURVEY.md §8):

  * getSimpleStateRepresentation (GRID_VIEW_ENABLED = False, bot.py:511-547):
    k_observe_simple, 12 values per bot;
  * the CNN over the grid view (CNN_REPR without CNN_P_REPR, bot.py:103-111, 284)
    at CNN_INPUT_DIM 42 and 84 squares per side: k_observe_wide.

The oracle's restatements reproduce the reference's own states bit-exactly
(tests/test_oracle_golden.py: simple16, cnn42, cnn84, MT mode).  Here the device
runs the same scenarios re-keyed to Philox and matches the oracle: events
exact, every bot's state every tick within 1e-5 (fov sizes and view boxes
exactly equal)."""
import numpy as np
import pytest

from aigar_amd import _abi
from oracle_lib import Oracle, make_config
import parity

pytestmark = pytest.mark.gpu
_lib = pytest.importorskip("aigar_amd._lib")


def _run(cfg, ticks, seed, ps, pe, obs_every=1):
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    g.reset(seed)
    o.reset(seed)
    assert g.obs_len == o.obs_len
    rng = np.random.default_rng(seed)
    size = g.get_state()["field_size"]
    n = cfg.bots_per_arena
    seen = []
    for t in range(ticks):
        cmd = parity.synthetic_commands(rng, None, n, size, ps, pe)
        g.set_commands(cmd)
        o.set_commands(cmd)
        g.step(1)
        o.step(1)
        assert np.array_equal(g.events(), o.events()), "events differ at tick %d" % t
        if (t + 1) % obs_every == 0:
            og, oo = g.observe(), o.observe()
            assert parity.obs_close(og, oo), "tick %d: states differ (max %g)" % (
                t, np.nanmax(np.abs(np.nan_to_num(og, nan=0) - np.nan_to_num(oo, nan=0))))
            seen.append(oo)
    dif = parity.diff_states(g.get_state(), o.get_state())
    assert not dif, dif
    g.close()
    o.close()
    return np.concatenate(seen)


@pytest.mark.parametrize("bots,field,virus,seed", [(16, 0, True, 8), (64, 600, True, 3), (128, 0, False, 4)])
def test_simple_state_matches_oracle(bots, field, virus, seed):
    cfg = make_config(bots=bots, field_size=field, virus=virus, max_viruses=20 if virus else -1.0,
                      channels=_abi.OBS_SIMPLE, extras=0)
    states = _run(cfg, 80, seed, 0.03, 0.03)
    assert states.shape == (80 * bots, 12)
    live = states[~np.isnan(states[:, 0])]
    # over the run, bots saw enemy cells, pellets and field edges
    assert (live[:, 3:6] != 0).any() and (live[:, 6:8] != 0).any() and (live[:, 8:12] != 1).any()


@pytest.mark.parametrize("G,bots,seed", [(42, 24, 9), (84, 12, 10), (17, 32, 11)])
def test_wide_grid_matches_oracle(G, bots, seed):
    ch = (_abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_VIRUS | _abi.OBS_SELF_LF
          | _abi.OBS_ENEMY_LF | _abi.OBS_SELF_SLF | _abi.OBS_ENEMY_SLF)
    cfg = make_config(bots=bots, virus=True, max_viruses=12, channels=ch, extras=0, grid_squares=G)
    states = _run(cfg, 40, seed, 0.04, 0.04, obs_every=5)
    assert states.shape == (8 * bots, 9 * G * G)


@pytest.mark.parametrize("G,seed", [(8, 21), (13, 22), (14, 23), (16, 24)])
def test_default_kernel_other_grid_sizes(G, seed):
    """k_observe (16-bit square masks) at grid sizes beside the default 11: the
    paired-square fast path (GG <= 128) and the generic loop (up to 4 squares per
    lane; G = 14 leaves 4 lanes in the last round, whose shuffles must still read
    the column / row values of the other lanes)."""
    ch = (_abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_VIRUS | _abi.OBS_SELF_LF
          | _abi.OBS_ENEMY_LF)
    cfg = make_config(bots=48, virus=True, max_viruses=12, channels=ch, extras=0x1F, grid_squares=G)
    states = _run(cfg, 30, seed, 0.04, 0.04, obs_every=3)
    assert states.shape == (10 * 48, 7 * G * G + 11)


def test_wide_grid_overflow_pool_and_big_views():
    """Big cells (wide views, thousands of visible pellets: the lists leave LDS for
    the global pool) at 42 squares per side."""
    ch = _abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_ENEMY | _abi.OBS_WALL
    cfg = make_config(bots=8, field_size=500, channels=ch, extras=_abi.EX_FOV | _abi.EX_MASS, grid_squares=42)
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    o.reset(12)
    st = o.get_state()
    cf = np.array(st["cells_f"], copy=True)
    cf[:3, 2] = [9000.0, 3000.0, 800.0]
    cf[:3, 3] = np.sqrt(cf[:3, 2] / np.pi)
    st["cells_f"] = cf
    o.load_state(st)
    g.load_state(st)
    rng = np.random.default_rng(12)
    for t in range(10):
        cmd = parity.synthetic_commands(rng, None, 8, 500, 0.0, 0.0)
        g.set_commands(cmd)
        o.set_commands(cmd)
        g.step(1)
        o.step(1)
        assert parity.obs_close(g.observe(), o.observe()), "tick %d" % t
    g.close()
    o.close()


@pytest.mark.parametrize("converted", [False, True])
def test_default_grid_overflow_pool(converted):
    """k_observe at the default 11 squares with views of over a thousand pellets
    (the lists leave LDS for the overflow pool): whole-unit pellets take the
    order-free sums from the pool, a view holding a blob-made pellet the ranked
    creation-order scan.  Pellet channel EXACT, the rest within 1e-5."""
    ch = _abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_ENEMY | _abi.OBS_WALL | _abi.OBS_SELF_LF | _abi.OBS_ENEMY_LF
    cfg = make_config(bots=16, field_size=400, max_pellets=4000.0, channels=ch, extras=_abi.EX_FOV | _abi.EX_MASS)
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    o.reset(41)
    st = o.get_state()
    cf = np.array(st["cells_f"], copy=True)
    cf[:4, 2] = [9000.0, 4000.0, 2500.0, 1200.0]
    cf[:4, 3] = np.sqrt(cf[:4, 2] / np.pi)
    st["cells_f"] = cf
    if converted:
        pf = np.array(st["pellets_f"], copy=True)
        sel = np.arange(len(pf)) % 7 == 0
        pf[sel, 2] = 18 * 0.8
        pf[sel, 3] = np.sqrt(pf[sel, 2] / np.pi)
        st["pellets_f"] = pf
    o.load_state(st)
    g.load_state(st)
    rng = np.random.default_rng(41)
    big = 0
    for t in range(5):
        og, oo = g.observe(), o.observe()
        assert np.array_equal(np.isnan(og), np.isnan(oo))
        pg, po = np.nan_to_num(og[:, :121]), np.nan_to_num(oo[:, :121])
        assert np.array_equal(pg, po), "tick %d: pellet channel differs (max %g)" % (t, np.abs(pg - po).max())
        assert parity.obs_close(og, oo), "tick %d" % t
        big += int((po.sum(axis=1) > 300).sum())  # (views over the LDS list's 256 pellets)
        cmd = parity.synthetic_commands(rng, None, 16, 400, 0.0, 0.0)
        g.set_commands(cmd)
        o.set_commands(cmd)
        g.step(1)
        o.step(1)
    assert big > 0
    g.close()
    o.close()


def test_pellet_sums_whole_units_and_converted():
    """k_observe's pellet channel takes two paths: when every pellet a bot sees
    weighs whole units (spawns, 1-3) the sums are scattered into the squares in
    any order (exact: integer sums); a bot that sees a blob-made pellet (14.4)
    keeps the creation-order scan.  Both must give the reference's doubles
    bit for bit, so the pellet channel is compared EXACTLY here (not within
    1e-5): a world where the left half of the field holds converted pellets
    among the spawned ones, many of them per square, observed as loaded and
    after a few ticks."""
    cfg = make_config(bots=24, field_size=400, max_pellets=4000.0, channels=_abi.OBS_PELLET | _abi.OBS_SELF,
                      extras=0)
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    o.reset(31)
    st = o.get_state()
    pf = np.array(st["pellets_f"], copy=True)
    conv = pf[:, 0] < 200
    sel = conv & (np.arange(len(pf)) % 3 == 0)  # a third of the left half's pellets are blob-made
    pf[sel, 2] = 18 * 0.8
    pf[sel, 3] = np.sqrt(pf[sel, 2] / np.pi)
    st["pellets_f"] = pf
    o.load_state(st)
    g.load_state(st)
    GG = 121
    rng = np.random.default_rng(31)
    n_mixed = n_whole = 0
    for t in range(4):
        og, oo = g.observe(), o.observe()
        assert np.array_equal(np.isnan(og), np.isnan(oo))
        pg, po = np.nan_to_num(og[:, :GG]), np.nan_to_num(oo[:, :GG])
        assert np.array_equal(pg, po), "tick %d: pellet channel differs (max %g)" % (t, np.abs(pg - po).max())
        assert parity.obs_close(og, oo)
        frac = np.abs(po - np.round(po)) > 0
        n_mixed += int(frac.any(axis=1).sum())
        n_whole += int(((po > 0).any(axis=1) & ~frac.any(axis=1)).sum())
        cmd = parity.synthetic_commands(rng, None, 24, 400, 0.0, 0.0)
        g.set_commands(cmd)
        o.set_commands(cmd)
        g.step(1)
        o.step(1)
    assert n_mixed > 0 and n_whole > 0, (n_mixed, n_whole)  # both paths ran
    g.close()
    o.close()
