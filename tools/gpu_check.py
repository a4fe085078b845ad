#!/usr/bin/env python3
"""Quick GPU-vs-oracle diagnostic (prints the first divergence per scenario).

Run on the GPU box:  python tools/gpu_check.py [scenario ...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from aigar_amd import _abi, _lib  # noqa: E402
from oracle_lib import Oracle, make_config  # noqa: E402
import parity  # noqa: E402


def fresh(cfg, seed):
    g = _lib.Stepper(cfg)
    o = Oracle(cfg)
    g.reset(seed)
    o.reset(seed)
    return g, o


def scen_reset():
    cfg = make_config(bots=64, virus=True, max_viruses=20, channels=0x3FF & ~0x10, extras=0x1F)
    g, o = fresh(cfg, 11)
    dif = parity.diff_states(g.get_state(), o.get_state())
    return dif[0] if dif else None, {}


def scen_random(bots, ticks, seed, virus=False, p_split=0.0, p_eject=0.0, obs=False, **kw):
    ch = _abi.OBS_PELLET | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_SELF | (_abi.OBS_VIRUS if virus else 0) \
        | _abi.OBS_SELF_LF | _abi.OBS_ENEMY_LF
    cfg = make_config(bots=bots, virus=virus, channels=ch, extras=0x1F, **kw)
    g, o = fresh(cfg, seed)
    rng = np.random.default_rng(seed)
    size = g.get_state()["field_size"]
    return parity.run_pair(g, o, ticks,
                           lambda t: parity.synthetic_commands(rng, None, bots, size, p_split, p_eject), obs=obs)


def scen_golden(name, ticks=None, obs=True):
    z = parity.load_golden(name)
    cfg = parity.golden_config(z)
    g, o = _lib.Stepper(cfg), Oracle(cfg)
    d = parity.philox_dict(z, "init")
    g.load_state(d)
    o.load_state(d)
    T = int(z["ticks"]) if ticks is None else ticks
    return parity.run_pair(g, o, T, lambda t: z["cmds"][t], obs=obs)


def scen_pow():
    import math
    rng = np.random.default_rng(0)
    x = np.concatenate([np.sqrt(rng.uniform(0.01, 22500, 20000) / math.pi), rng.uniform(0.5, 22500, 20000)])
    y = np.concatenate([np.full(20000, 0.475), np.full(20000, -0.35)])
    sys.path.insert(0, "/tmp/mt")
    g = _lib.selftest_pow(x, y)
    glibc = np.array([math.pow(a, b) for a, b in zip(x, y)])
    return None, {"device_vs_glibc_mismatch": int(np.sum(g != glibc)), "n": len(x)}


SCEN = {
    "pow": scen_pow,
    "reset": scen_reset,
    "c1": lambda: scen_random(1, 300, 1, max_pellets=100, field_size=1000, obs=True),
    "b64": lambda: scen_random(64, 120, 2, p_split=0.03, p_eject=0.03, obs=True),
    "b64v": lambda: scen_random(64, 120, 3, virus=True, max_viruses=60, p_split=0.03, p_eject=0.05, obs=True),
    "crowd": lambda: scen_random(48, 150, 4, field_size=120, p_split=0.05, p_eject=0.05, obs=True),
    "g_stress": lambda: scen_golden("stress_virus"),
    "g_crowd": lambda: scen_golden("crowd32"),
    "g_merge": lambda: scen_golden("merge8"),
    "g_feed": lambda: scen_golden("virus_feed"),
    "g_greedyv": lambda: scen_golden("greedy16_virus_split"),
    "c2": lambda: scen_random(256, 60, 5, max_pellets=10000, field_size=1200, obs=True),
}

if __name__ == "__main__":
    names = sys.argv[1:] or list(SCEN)
    fails = 0
    for n in names:
        t0 = time.time()
        try:
            err, stats = SCEN[n]()
        except Exception as e:  # report and continue with the next scenario
            err, stats = "EXCEPTION %r" % (e,), {}
        dt = time.time() - t0
        print("%-10s %-6s %5.1fs %s %s" % (n, "OK" if err is None else "FAIL", dt, stats, err or ""), flush=True)
        fails += err is not None
    sys.exit(1 if fails else 0)
