"""GPU vs oracle on edge cases of the world: no pellets at all, a tiny field
where players split repeatedly against the walls, a cell at the mass
cap (grow stops at 22500, parameters.py:30) and a heavy cell dropped on a virus
(eatVirus + the 16 - n explosion, field.py:333-370).  Events exact, floats
within 1e-5 (parity.FTOL)."""
import math

import numpy as np
import pytest

from aigar_amd import _abi
from oracle_lib import Oracle, make_config
import parity

pytestmark = pytest.mark.gpu
_lib = pytest.importorskip("aigar_amd._lib")

CH = (_abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_VIRUS | _abi.OBS_SELF_LF
      | _abi.OBS_ENEMY_LF)


def _pair(cfg, seed):
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    g.reset(seed)
    o.reset(seed)
    assert parity.diff_states(g.get_state(), o.get_state()) == []
    return g, o


def _run(g, o, ticks, bots, size, ps, pe, seed):
    rng = np.random.default_rng(seed)
    err, stats = parity.run_pair(g, o, ticks, lambda t: parity.synthetic_commands(rng, None, bots, size, ps, pe),
                                 obs=True)
    assert err is None, err
    return stats


def test_world_without_pellets():
    cfg = make_config(bots=32, virus=True, max_viruses=30, max_pellets=0.0, channels=CH, extras=0x1F)
    g, o = _pair(cfg, 31)
    assert g.get_state()["n_pellets"] == 0
    _run(g, o, 80, 32, g.get_state()["field_size"], 0.05, 0.05, 31)
    assert g.get_state()["n_pellets"] == 0


def test_tiny_field_splits_and_walls():
    cfg = make_config(bots=8, field_size=60, max_pellets=200.0, channels=CH & ~_abi.OBS_VIRUS, extras=0x1F)
    g, o = _pair(cfg, 32)
    most = 0
    for k in range(12):
        _run(g, o, 10, 8, 60, 0.5, 0.2, 32 + k)
        most = max(most, int(np.max(g.get_state()["players_i"][:, 4])))
    assert most >= 4  # repeated splits, squeezed against the walls


def _load_both(g, o, d):
    g.load_state(d)
    o.load_state(d)
    assert parity.diff_states(g.get_state(), o.get_state()) == []


def test_mass_cap_and_virus_explosion():
    cfg = make_config(bots=16, virus=True, max_viruses=40, channels=CH, extras=0x1F)
    g, o = _pair(cfg, 33)
    d = o.get_state()
    cf, ci = d["cells_f"].copy(), d["cells_i"]
    vf = d["viruses_f"]
    # cell of player 0 just under the mass cap: every pellet it eats is capped by grow()
    cf[0, 2] = 22490.0
    cf[0, 3] = math.sqrt(22490.0 / math.pi)
    # cell of player 1 heavy enough to eat a virus, dropped on the first one
    k = int(np.nonzero(ci[:, 0] == 1)[0][0])
    cf[k, 0], cf[k, 1] = vf[0, 0] + 0.5, vf[0, 1] - 0.5
    cf[k, 2] = 400.0
    cf[k, 3] = math.sqrt(400.0 / math.pi)
    d = dict(d)
    d["cells_f"] = cf
    _load_both(g, o, d)
    size = d["field_size"]
    most, events = 0, 0
    for k in range(8):
        events += _run(g, o, 5, 16, size, 0.0, 0.0, 33 + k)["events"]
        st = g.get_state()
        assert float(np.max(st["cells_f"][:, 2])) <= 22500.0
        most = max(most, int(np.max(st["players_i"][:, 4])))
    assert events > 0
    assert most == 16  # the explosion fills the player up to the 16-cell cap (field.py:354)


def test_eject_burst_near_blob_capacity():
    """the blob list keeps its holes between compactions
    (k_spawn_plan); a tick on which every cell ejects (field.py:134-146) must
    still find room when the live blobs plus its ejections fit the capacity.
    40 players split to 16 cells each, a trickle of ejections leaves holes, then
    every player ejects from all of its cells at once (~640 blobs, capacity 1024)."""
    B, size = 40, 600
    cfg = make_config(bots=B, field_size=size, max_pellets=300.0, channels=CH & ~_abi.OBS_VIRUS, extras=0x1F,
                      blob_cap=1024)
    g, o = _pair(cfg, 35)
    d = dict(o.get_state())
    cf = d["cells_f"].copy()
    cf[:, 2] = 1500.0
    cf[:, 3] = math.sqrt(1500.0 / math.pi)
    d["cells_f"] = cf
    _load_both(g, o, d)
    _run(g, o, 5, B, size, 1.0, 0.0, 35)  # every player splits up to the 16-cell cap
    assert int(np.min(g.get_state()["players_i"][:, 4])) >= 8
    _run(g, o, 24, B, size, 0.0, 0.04, 36)  # a trickle: blobs die after 15 ticks and leave holes
    _run(g, o, 1, B, size, 0.0, 1.0, 37)  # the burst
    assert g.get_state()["n_blobs"] >= 300
    _run(g, o, 12, B, size, 0.0, 0.04, 38)
    g.sync()  # no ERR_BLOB_CAP


def test_refill_of_a_depleted_world_in_one_tick():
    """a tick whose spawns put more joining records into one bucket row
    than the closing update's LDS list holds (512; field 1000 = 50 rows, 40,000
    pellets: ~800 joins per row) -- the whole refill lands, in order, and the world
    stays the oracle's; it keeps stepping from the refilled rows."""
    cfg = make_config(bots=16, field_size=1000, max_pellets=40000.0, channels=CH & ~_abi.OBS_VIRUS, extras=0x1F)
    g, o = _pair(cfg, 33)
    d = g.get_state()
    assert d["n_pellets"] == 40000
    for k in ("pellets_f", "pellets_col"):
        if k in d:
            d[k] = d[k][:100]
    d["pellets_seq"] = d["pellets_seq"][:100]
    d["n_pellets"] = 100
    _load_both(g, o, d)
    st = _run(g, o, 1, 16, 1000, 0.0, 0.0, 33)
    assert g.get_state()["n_pellets"] == 40000
    _run(g, o, 20, 16, 1000, 0.05, 0.05, 34)
    assert st["ticks"] == 1
