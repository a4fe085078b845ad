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
