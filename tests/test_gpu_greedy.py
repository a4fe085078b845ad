"""GPU: the device Greedy bot policy (k_policy_greedy) against the oracle's
(pinned to the reference by test_oracle_greedy.py), and directly against the
reference's own greedy commands where they do not depend on a random draw."""
import os

import numpy as np
import pytest

from aigar_amd import _abi
from oracle_lib import Oracle, golden_state, make_config
import parity
from test_oracle_greedy import GREEDY, split_likelihoods

pytestmark = pytest.mark.gpu
_lib = pytest.importorskip("aigar_amd._lib")


def commands(st):
    pf, pi = np.asarray(st["players_f"]), np.asarray(st["players_i"])
    return np.c_[pf[:, 0], pf[:, 1], pi[:, 2], pi[:, 3]].astype(np.float64)


@pytest.mark.parametrize("bots,virus,gsplit,seed,field,ticks", [
    (16, False, False, 1, 0, 120), (48, True, True, 2, 0, 120), (200, True, True, 3, 0, 120),
    # crowded: greedy bots hunt each other (playerPlayerOverlap turns, respawns); with correctly rounded device
    # atan2/sin/cos (aigar_trig.h) the world stays within 1e-9 of the oracle for 600 ticks (OCML trig: 1e-5 is
    # exceeded at tick ~277)
    (64, True, True, 4, 250, 600), (64, True, True, 5, 250, 600),
])
def test_greedy_population_matches_oracle(bots, virus, gsplit, seed, field, ticks):
    cfg = make_config(bots=bots, virus=virus, max_viruses=30 if virus else -1.0, field_size=field,
                      channels=_abi.OBS_PELLET | _abi.OBS_WALL | _abi.OBS_ENEMY, extras=0x3)
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    g.reset(seed)
    o.reset(seed)
    kinds = set()
    for t in range(ticks):
        g.policy_greedy(gsplit)
        o.policy_greedy(gsplit)
        cg, co = commands(g.get_state()), commands(o.get_state())
        bad = np.argwhere(cg != co)
        assert not len(bad), "tick %d bot %d: gpu %s oracle %s" % (t, bad[0][0], cg[bad[0][0]], co[bad[0][0]])
        g.step(1)
        o.step(1)
        ev = g.events()
        assert np.array_equal(ev, o.events()), "events differ at tick %d" % t
        kinds |= set(ev[:, 1].tolist())
    dif = parity.diff_states(g.get_state(), o.get_state(), ftol=1e-9 if field else parity.FTOL)
    assert not dif, dif
    if field:  # the crowded world must have exercised cell-eats-cell and deaths
        assert {_abi.EV_CELL_EAT_CELL, _abi.EV_PLAYER_DEATH} <= kinds, kinds
    g.close()
    o.close()


@pytest.mark.parametrize("name,seed,gsplit", GREEDY)
def test_greedy_matches_reference_commands_at_checkpoints(name, seed, gsplit, golden_dir):
    """At every reference checkpoint state, the device's greedy command equals
    the reference bot's for every bot whose move involved no random draw
    (the MT- and Philox-mode oracles agree on exactly those)."""
    z = np.load(os.path.join(golden_dir, name + ".npz"))
    n = int(z["n_players"])
    lh = split_likelihoods(seed, n)
    cfg_mt = make_config(bots=n, field_size=int(z["size"]), virus=bool(z["virus_enabled"]),
                         max_pellets=float(z["max_pellets"]), max_viruses=float(z["max_viruses"]),
                         channels=int(z["obs_channels"]), extras=int(z["obs_extras"]), rng_mode=_abi.RNG_MT19937)
    cfg_ph = parity.golden_config(z)
    g, om, op = _lib.Stepper(cfg_ph), Oracle(cfg_mt), Oracle(cfg_ph)
    for orc in (om, op):
        orc.set_split_likelihood(lh)
    g.set_split_likelihood(lh)
    checked = 0
    for ck in [0] + [int(t) for t in z["ck_ticks"] if int(t) < int(z["ticks"])]:
        pre = "init" if ck == 0 else "ck%d" % ck
        st_mt = golden_state(z, pre)
        st_ph = parity.philox_dict(z, pre)
        om.load_state(st_mt)
        op.load_state(st_ph)
        g.load_state(st_ph)
        om.policy_greedy(gsplit)
        op.policy_greedy(gsplit)
        g.policy_greedy(gsplit)
        ref = z["cmds"][ck]
        cm, cp, cg = om.commands(), op.commands(), commands(g.get_state())
        assert np.array_equal(cm, ref), "MT oracle vs reference at tick %d" % ck
        det = np.all(cm == cp, axis=1)  # no random draw involved
        assert np.array_equal(cg[det], ref[det]), "device vs reference at tick %d" % ck
        assert np.array_equal(cg, cp), "device vs Philox oracle at tick %d" % ck
        checked += int(det.sum())
    if n > 1:  # (the lone C1 bot mostly sees no pellet and moves at random)
        assert checked > 0
    for x in (g, om, op):
        x.close()


def test_c2_greedy_population_matches_oracle():
    """BASELINE configs[1] / SURVEY.md §8d C2 at its stated population: 256 Greedy
    bots, field 1200 (75 * sqrt(256)), 10,000 pellets, no viruses / split / eject,
    250 ticks (the survey's 100-tick warm-up and 150 more): every command, every
    event and the world against the oracle, and every bot's observation
    (pellet, wall and enemy grids + fov extras) every 25 ticks."""
    cfg = make_config(bots=256, virus=False, field_size=0, max_pellets=10000.0,
                      channels=_abi.OBS_PELLET | _abi.OBS_WALL | _abi.OBS_ENEMY, extras=0x3)
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    g.reset(21)
    o.reset(21)
    assert g.get_state()["field_size"] == 1200
    eaten = 0
    for t in range(250):
        g.policy_greedy(False)
        o.policy_greedy(False)
        cg, co = commands(g.get_state()), commands(o.get_state())
        assert np.array_equal(cg, co), "tick %d: greedy commands differ" % t
        g.step(1)
        o.step(1)
        ev = g.events()
        assert np.array_equal(ev, o.events()), "events differ at tick %d" % t
        eaten += int(np.sum(ev[:, 1] == _abi.EV_CELL_EAT_PELLET))
        if (t + 1) % 25 == 0:
            assert parity.obs_close(g.observe(), o.observe()), "observations differ at tick %d" % t
            dif = parity.diff_states(g.get_state(), o.get_state())
            assert not dif, "tick %d: %s" % (t, dif[:3])
    assert eaten > 1000  # greedy bots converge on the pellets
    g.close()
    o.close()
