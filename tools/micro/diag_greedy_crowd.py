"""Parity horizon of the crowded greedy world (64 bots, 250-unit field): steps
the device and the oracle side by side, prints the max |cell float diff| every
50 ticks and stops at the first differing greedy command.
usage: python tools/micro/diag_greedy_crowd.py [ticks=600] [seed=4]"""
import sys

import numpy as np

sys.path[:0] = ['.', 'tests']
from aigar_amd import _abi, _lib  # noqa: E402
from oracle_lib import Oracle, make_config  # noqa: E402
import parity  # noqa: E402

ticks = int(sys.argv[1]) if len(sys.argv) > 1 else 600
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 4
cfg = make_config(bots=64, virus=True, max_viruses=30, field_size=250,
                  channels=_abi.OBS_PELLET | _abi.OBS_WALL | _abi.OBS_ENEMY, extras=0x3)
g, o = _lib.Stepper(cfg), Oracle(cfg)
g.reset(seed)
o.reset(seed)


def cmds(st):
    pf, pi = np.asarray(st["players_f"]), np.asarray(st["players_i"])
    return np.c_[pf[:, 0], pf[:, 1], pi[:, 2], pi[:, 3]]


def cell_diff(sg, so):
    a, b = np.asarray(sg["cells_f"]), np.asarray(so["cells_f"])
    if a.shape != b.shape or not np.array_equal(np.asarray(sg["cells_i"]), np.asarray(so["cells_i"])):
        return float("inf")
    return float(np.max(np.abs(a - b))) if a.size else 0.0


for t in range(ticks):
    g.policy_greedy(True)
    o.policy_greedy(True)
    sg, so = g.get_state(), o.get_state()
    cg, co = cmds(sg), cmds(so)
    bad = np.nonzero(np.any(cg != co, axis=1))[0]
    if len(bad):
        print("tick", t, "first differing greedy command: bot", bad[0], cg[bad[0]], co[bad[0]],
              "max cell diff", cell_diff(sg, so))
        break
    if t % 50 == 0:
        print("tick", t, "max cell diff", cell_diff(sg, so), flush=True)
    g.step(1)
    o.step(1)
    if not np.array_equal(g.events(), o.events()):
        print("tick", t, "events differ")
        break
else:
    sg, so = g.get_state(), o.get_state()
    print("completed", ticks, "ticks; max cell diff", cell_diff(sg, so),
          "diffs at 1e-5:", parity.diff_states(sg, so)[:3])
