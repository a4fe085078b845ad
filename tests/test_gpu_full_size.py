"""GPU vs oracle at BASELINE.json's full C3 size (4096 bots, field 4800, 100k
pellets, 1152 viruses): every event, the whole state and every bot's
observation, tick by tick -- for the synthetic C3 population and for the
reference's Greedy bots.  Plus run-to-run determinism of the device."""
import numpy as np
import pytest

from aigar_amd import _abi
from oracle_lib import Oracle, make_config
import parity

pytestmark = pytest.mark.gpu
_lib = pytest.importorskip("aigar_amd._lib")

C3_CH = (_abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_VIRUS | _abi.OBS_SELF_LF
         | _abi.OBS_ENEMY_LF)
C3_EX = _abi.EX_LAST_FOV | _abi.EX_FOV | _abi.EX_MASS | _abi.EX_LAST_ACT


def c3():
    return make_config(bots=4096, field_size=4800, virus=True, max_pellets=100000.0, channels=C3_CH, extras=C3_EX)


def test_c3_synthetic_population_matches_oracle():
    cfg = c3()
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    g.reset(21)
    o.reset(21)
    rng = np.random.default_rng(21)
    err, stats = parity.run_pair(g, o, 25, lambda t: parity.synthetic_commands(rng, None, 4096, 4800, 2.5e-3, 1e-2),
                                 obs=True)
    assert err is None, err
    assert stats["events"] > 1000
    g.close()
    o.close()


def test_c3_greedy_population_matches_oracle():
    cfg = c3()
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    g.reset(22)
    o.reset(22)
    for t in range(15):
        g.policy_greedy(True)
        o.policy_greedy(True)
        g.step(1)
        o.step(1)
        assert np.array_equal(g.events(), o.events()), "tick %d" % t
    dif = parity.diff_states(g.get_state(), o.get_state())
    assert not dif, dif
    g.close()
    o.close()


def test_device_is_deterministic_at_full_size():
    cfg = c3()
    outs = []
    for _ in range(2):
        g = _lib.Stepper(cfg)
        g.reset(5)
        for _ in range(40):
            g.policy_random(2.5e-3, 1e-2, 7)
            g.step(1)
        st = g.get_state()
        outs.append((st, g.observe()))
        g.close()
    (a, oa), (b, ob) = outs
    for k in _abi.LAYOUT:
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert parity.obs_close(oa, ob, 0.0)


@pytest.mark.parametrize("policy", ["synthetic", "greedy"])
def test_c3_matured_world_matches_oracle(policy):
    """C3 from the matured tick-600 world (tools/mature.py: cells past 36 and 125,
    673 multi-cell players): 60 ticks, every event, state and observation.  Split,
    eject, blob eating, virus explosions, merges and cell-eats-cell all happen at
    full size (field.py:200-253)."""
    cfg = c3()
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    snap = parity.load_snapshot("c3_t600")
    g.load_state(snap)
    o.load_state(snap)
    rng = np.random.default_rng(23)
    kinds = set()
    for t in range(60):
        if policy == "greedy":
            o.policy_greedy(True)
            cmd = o.commands()
        else:
            cmd = parity.synthetic_commands(rng, None, 4096, 4800, 2.5e-3, 1e-2)
        err, st = parity.run_pair(g, o, 1, lambda _: cmd, obs=(t % 10 == 9))
        assert err is None, "tick %d: %s" % (t, err)
        kinds |= set(o.events()[:, 1].tolist())
    want = {_abi.EV_MERGE, _abi.EV_CELL_EAT_VIRUS, _abi.EV_EXPLODE, _abi.EV_CELL_EAT_PELLET, _abi.EV_CELL_EAT_CELL}
    if policy == "synthetic":  # (the greedy bots never eject, bot.py:94)
        want |= {_abi.EV_CELL_EAT_BLOB}
    assert want <= kinds, kinds
    s = g.get_state()
    assert np.sum(s["players_i"][:, 4] > 1) > 100  # multi-cell players
    g.close()
    o.close()


@pytest.mark.parametrize("A,ticks,every", [(8, 60, 20), (40, 20, 10)])
def test_c5_gpu_slice_matches_eight_oracles(A, ticks, every):
    """C5's per-GPU slice: 8 independent arenas x 512 bots, field
    1697, 43,200 pellets, viruses off, stepped by the same launches; each arena
    against its own single-arena oracle (loaded from the arena's reset state, so
    it carries that arena's Philox key) for 60 ticks: events every tick, states
    and observations every 20.  A = 40 (20,480 bots) puts more than 16,384 bots in
    one observation launch, where k_observe switches to its streaming (non-temporal)
    store variant (obs.hip kObsWtBots): that variant against the oracles too."""
    B = 512
    ch, ex = _abi.OBS_PELLET | _abi.OBS_WALL | _abi.OBS_ENEMY, _abi.EX_FOV | _abi.EX_MASS
    g = _lib.Stepper(make_config(n_arenas=A, bots=B, field_size=1697, max_pellets=43200.0, channels=ch, extras=ex))
    g.reset(40)
    orcs = []
    for a in range(A):
        o = Oracle(make_config(bots=B, field_size=1697, max_pellets=43200.0, channels=ch, extras=ex))
        o.load_state(g.get_state(a))
        orcs.append(o)
    rng = np.random.default_rng(40)
    nev = 0
    for t in range(ticks):
        cmd = parity.synthetic_commands(rng, None, A * B, 1697, 0.01, 0.02)
        g.set_commands(cmd)
        g.step(1)
        for a, o in enumerate(orcs):
            o.set_commands(cmd[a * B:(a + 1) * B])
            o.step(1)
            ev = o.events()
            assert np.array_equal(g.events(a), ev), "tick %d arena %d" % (t, a)
            nev += len(ev)
        if t % every == every - 1:
            obs = g.observe()
            for a, o in enumerate(orcs):
                dif = parity.diff_states(g.get_state(a), o.get_state())
                assert not dif, (t, a, dif[:3])
                assert parity.obs_close(obs[a * B:(a + 1) * B], o.observe()), (t, a)
    assert nev > A * ticks * 5
    g.close()
    for o in orcs:
        o.close()


def test_parallel_pp_groups_match_the_serial_pass_and_the_oracle():
    """playerPlayerOverlap as independent groups (tick.hip pp_pass: seeds whose
    closures share no player run their turns in separate wavefronts, deaths
    re-sorted into turn order): the bench's tick-50 C3 world with the
    reference's Greedy bots (~6 pending players per tick), 40 ticks -- every
    event and the state against the oracle and against the same device forced
    to the serial pass (AIGAR_PP_SERIAL), and most ticks must have taken the
    parallel path.  (The tick-600 world's greedy ticks, ~33 pending players,
    mostly fall back to the serial pass: test_c3_matured_world_matches_oracle.)"""
    import os
    cfg = c3()
    snap = parity.load_snapshot("c3_t50")
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    os.environ["AIGAR_PP_SERIAL"] = "1"
    try:
        s = _lib.Stepper(cfg)
    finally:
        del os.environ["AIGAR_PP_SERIAL"]
    for x in (g, o, s):
        x.load_state(snap)
    w0, s0 = g.counters(), s.counters()
    for t in range(40):
        o.policy_greedy(True)
        cmd = o.commands()
        for x in (g, o, s):
            x.set_commands(cmd)
            x.step(1)
        eo = o.events()
        assert np.array_equal(g.events(), eo), "tick %d: parallel groups vs oracle" % t
        assert np.array_equal(s.events(), eo), "tick %d: serial pass vs oracle" % t
    for x in (g, s):
        dif = parity.diff_states(x.get_state(), o.get_state())
        assert not dif, dif[:3]
    w1, s1 = g.counters(), s.counters()
    assert s1["pp_parallel_ticks"] == s0["pp_parallel_ticks"]
    par = w1["pp_parallel_ticks"] - w0["pp_parallel_ticks"]
    assert par >= 20, "only %d of 40 ticks ran the groups in parallel" % par
    for x in (g, o, s):
        x.close()
