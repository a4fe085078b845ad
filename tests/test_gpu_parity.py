"""GPU parity: libaigar_hip.so (HIP, gfx950) vs the CPU oracle in Philox mode.

Bar (north_star): events -- every eat / merge / split / explosion / death /
respawn, with its indices (creation sequence numbers) and its ORDER -- are
bit-exact; float state within 1e-5 (observed: <= 1e-11); fov sizes exactly
equal (the device pow is glibc's, bit for bit, so the reference's cols==12
quirk fires on the same bots); observations within 1e-5 for every bot.
"""
import math

import numpy as np
import pytest

from aigar_amd import _abi
from oracle_lib import Oracle, make_config
import parity

pytestmark = pytest.mark.gpu

_lib = pytest.importorskip("aigar_amd._lib")

FULL_CH = (_abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_VIRUS | _abi.OBS_SELF_SLF
           | _abi.OBS_SELF_LF | _abi.OBS_ENEMY_SLF | _abi.OBS_ENEMY_LF)


def pair(cfg, seed):
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    g.reset(seed)
    o.reset(seed)
    return g, o


def check(err, stats, n_bot_obs=None):
    assert err is None, err


def test_device_pow_is_glibc_pow():
    rng = np.random.default_rng(0)
    n = 200000
    x = np.concatenate([np.sqrt(rng.uniform(0.01, 22500, n) / math.pi), rng.uniform(0.5, 22500, n),
                        np.arange(1, 17, dtype=np.float64), 1.0 + rng.random(n)])
    y = np.concatenate([np.full(n, 0.475), np.full(n, -0.35), np.full(16, 0.32), rng.uniform(-2, 2, n)])
    dev = _lib.selftest_pow(x, y)
    glibc = np.array([math.pow(a, b) for a, b in zip(x, y)])
    assert np.array_equal(dev, glibc), np.argwhere(dev != glibc)[:5]  # bit for bit (aigar_math.h)


def test_device_trig_is_glibc_trig():
    """The device's atan2 / sin / cos (aigar_glibc_trig.h) equal the C library's -- what the
    reference's math.atan2 / math.sin / math.cos call (cell.py:47-103, field.py:363-365) -- bit
    for bit: move directions from coordinate differences, the angles atan2 returns, integer
    degrees, and the s_sin.c / e_atan2.c range seams."""
    rng = np.random.default_rng(1)
    n = 100000
    x = np.concatenate([rng.uniform(-4800, 4800, n), rng.uniform(-1e-3, 1e-3, n),
                        np.ldexp(rng.uniform(-1, 1, n), rng.integers(-40, 40, n)), [0.0, -0.0, 0.0, -0.0, 5.0]])
    y = np.concatenate([rng.uniform(-4800, 4800, n), rng.uniform(-1e-3, 1e-3, n),
                        np.ldexp(rng.uniform(-1, 1, n), rng.integers(-40, 40, n)), [0.0, 0.0, -0.0, -0.0, 0.0]])
    at, _, _ = _lib.selftest_trig(y, x)
    ref = np.array([math.atan2(b, a) for b, a in zip(y, x)])
    assert np.array_equal(at.view(np.int64), ref.view(np.int64)), np.argwhere(at != ref)[:5]
    seams = np.concatenate([b * (1 + np.arange(-200, 201) * 2.0 ** -52)
                            for b in (2.0 ** -26, 0.126, 0.855469, 2.426265, math.pi, 2 * math.pi)])
    a = np.concatenate([ref, np.deg2rad(np.arange(360)), rng.uniform(-7, 7, n), seams, -seams])
    _, s, c = _lib.selftest_trig(np.zeros_like(a), a)
    rs = np.array([math.sin(v) for v in a])
    rc = np.array([math.cos(v) for v in a])
    assert np.array_equal(s.view(np.int64), rs.view(np.int64)), np.argwhere(s != rs)[:5]
    assert np.array_equal(c.view(np.int64), rc.view(np.int64)), np.argwhere(c != rc)[:5]


def test_reset_is_identical():
    cfg = make_config(bots=64, virus=True, max_viruses=20, channels=FULL_CH, extras=0x1F)
    g, o = pair(cfg, 11)
    assert parity.diff_states(g.get_state(), o.get_state()) == []
    ob_g, ob_o = g.observe(), o.observe()
    assert parity.obs_close(ob_g, ob_o)


@pytest.mark.parametrize("bots,ticks,seed,kw", [
    (1, 300, 1, dict(max_pellets=100, field_size=1000)),                      # C1 shape
    (64, 120, 2, dict(p_split=0.03, p_eject=0.03)),
    (64, 120, 3, dict(virus=True, max_viruses=60, p_split=0.03, p_eject=0.05)),
    (48, 150, 4, dict(field_size=120, p_split=0.05, p_eject=0.05)),           # crowded: deaths, respawns
    (256, 40, 5, dict(max_pellets=10000, field_size=1200)),                   # C2
])
def test_random_population(bots, ticks, seed, kw):
    kw = dict(kw)
    ps, pe = kw.pop("p_split", 0.0), kw.pop("p_eject", 0.0)
    virus = kw.pop("virus", False)
    cfg = make_config(bots=bots, virus=virus, channels=FULL_CH if virus else FULL_CH & ~_abi.OBS_VIRUS,
                      extras=0x1F, **kw)
    g, o = pair(cfg, seed)
    rng = np.random.default_rng(seed)
    size = g.get_state()["field_size"]
    err, stats = parity.run_pair(g, o, ticks, lambda t: parity.synthetic_commands(rng, None, bots, size, ps, pe),
                                 obs=True)
    check(err, stats, bots * ticks)


@pytest.mark.parametrize("name", ["stress_virus", "crowd32", "merge8", "virus_feed", "greedy16_virus_split",
                                  "greedy16", "random64",
                                  # BASELINE configs[1] and [2] at full size (reference-generated fixtures)
                                  "c2_greedy256", "c3_4096", "c3_4096_t600",
                                  # the C3 world with every event kind; the C3 start with reference Greedy bots
                                  "c3_4096_virus", "c3_greedy4096"])
def test_reference_states(name):
    """Start both from the reference's own initial world (tests/golden), replay its commands."""
    z = parity.load_golden(name)
    cfg = parity.golden_config(z)
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    d = parity.philox_dict(z, "init")
    g.load_state(d)
    o.load_state(d)
    T = int(z["ticks"])
    err, stats = parity.run_pair(g, o, T, lambda t: z["cmds"][t], obs=True)
    check(err, stats, int(z["n_players"]) * T)


def test_every_event_kind_on_device():
    seen = set()
    for name in ("stress_virus", "crowd32", "merge8", "virus_feed"):
        z = parity.load_golden(name)
        g = _lib.Stepper(parity.golden_config(z))
        g.load_state(parity.philox_dict(z, "init"))
        for t in range(int(z["ticks"])):
            g.set_commands(z["cmds"][t])
            g.step(1)
            ev = g.events()
            seen |= set(ev[:, 1].tolist())
    assert seen == set(range(1, 11))


def test_batched_arenas_match_independent_oracles():
    A, B = 4, 24
    cfg = make_config(n_arenas=A, bots=B, virus=True, max_viruses=30, channels=FULL_CH, extras=0x1F,
                      field_size=200)
    g, o = pair(cfg, 21)
    rng = np.random.default_rng(21)
    for t in range(60):
        cmd = parity.synthetic_commands(rng, None, A * B, 200, 0.05, 0.05)
        g.set_commands(cmd)
        o.set_commands(cmd)
        g.step(1)
        o.step(1)
        for a in range(A):
            assert np.array_equal(g.events(a), o.events(a)), (t, a)
            assert parity.diff_states(g.get_state(a), o.get_state(a)) == [], (t, a)


def test_state_roundtrip_and_float32_observation():
    cfg = make_config(bots=32, virus=True, max_viruses=20, channels=FULL_CH, extras=0x1F)
    g = _lib.Stepper(cfg)
    g.reset(3)
    rng = np.random.default_rng(3)
    for t in range(30):
        g.set_commands(parity.synthetic_commands(rng, None, 32, 424, 0.05, 0.05))
        g.step(1)
    s1 = g.get_state()
    g.load_state(s1)
    assert parity.diff_states(g.get_state(), s1, ftol=0.0) == []
    o64 = g.observe(dtype=np.float64)
    g.load_state(s1)  # resets the history grids
    o32 = g.observe(out=np.zeros((32, g.obs_len), np.float32))
    assert np.allclose(np.nan_to_num(o32), np.nan_to_num(o64.astype(np.float32)), rtol=1e-6, atol=1e-6)


def test_torch_device_buffers_and_stream():
    torch = pytest.importorskip("torch")
    cfg = make_config(bots=64, channels=FULL_CH & ~_abi.OBS_VIRUS, extras=0x1F)
    g, o = pair(cfg, 8)
    g.set_stream(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(8)
    for t in range(10):
        cmd = parity.synthetic_commands(rng, None, 64, 600, 0.0, 0.0)
        g.set_commands(torch.tensor(cmd, device="cuda"))
        o.set_commands(cmd)
        g.step(1)
        o.step(1)
    out = torch.zeros((64, g.obs_len), dtype=torch.float64, device="cuda")
    g.observe(out)
    torch.cuda.synchronize()
    assert parity.obs_close(out.cpu().numpy(), o.observe())
    assert parity.diff_states(g.get_state(), o.get_state()) == []


def test_policy_is_deterministic_and_uses_set_command_point():
    cfg = make_config(bots=128, channels=_abi.OBS_PELLET, extras=0x6)
    runs = []
    for _ in range(2):
        g = _lib.Stepper(cfg)
        g.reset(9)
        for t in range(20):
            g.policy_random(0.1, 0.1, 77)
            g.step(1)
        runs.append(g.get_state())
    assert parity.diff_states(runs[0], runs[1], ftol=0.0) == []
    pf = runs[0]["players_f"]
    assert np.all(pf[:, 0] >= -400) and np.all(pf[:, 0] <= 1250)
