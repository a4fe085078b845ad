"""Write matured C3 snapshots (SURVEY.md §8d warm distribution) for bench.py
and the full-size parity tests.

The reference's C3 numbers are quoted on a world that has been played: after
50 ticks of Greedy bots (bot.py:579-633, ENABLE_GREEDY_SPLIT) its cells average
mass 17.4 (max 54.2) and players own several cells.  A fresh reset has every
cell at START_MASS 10, where split (m > 36), eject (m >= 35) and virus
explosions (m > 125) cannot happen.  This script plays C3 from reset with the
Greedy policy of the CPU oracle (oracle/oracle.c, Philox stream; the device
matches it event for event) and saves the state at the requested ticks:

  data/c3_t50.npz   the bench's start (the survey's warm distribution)
  data/c3_t600.npz  a late world (580 cells past 125, 673 multi-cell players) for parity

usage: python tools/mature.py [ticks...]   (default 50 600)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

from aigar_amd import _abi  # noqa: E402
from oracle_lib import Oracle, make_config  # noqa: E402  (CPU oracle: generator only)

C3_CH = (_abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_VIRUS | _abi.OBS_SELF_LF
         | _abi.OBS_ENEMY_LF)
SEED = 20251016


def stats(st):
    cf, ci = st["cells_f"], st["cells_i"]
    pl = st["players_i"]
    return {"tick": int(st["tick"]), "cells": int(st["n_cells"]), "mean_mass": float(cf[:, 2].mean()),
            "max_mass": float(cf[:, 2].max()), "multi_cell_players": int(np.sum(pl[:, 4] > 1)),
            "cells_over_36": int(np.sum(cf[:, 2] > 36)), "cells_over_125": int(np.sum(cf[:, 2] > 125)),
            "blobs": int(st["n_blobs"]), "pellets": int(st["n_pellets"]), "viruses": int(st["n_viruses"])}


def main():
    want = sorted(int(a) for a in sys.argv[1:]) or [50, 600]
    cfg = make_config(bots=4096, field_size=4800, virus=True, max_pellets=100000.0, channels=C3_CH, extras=0x1F)
    o = Oracle(cfg)
    o.reset(SEED)
    os.makedirs(os.path.join(ROOT, "data"), exist_ok=True)
    t0 = time.time()
    for t in range(1, want[-1] + 1):
        o.policy_greedy(True)
        o.step(1)
        if t in want:
            st = o.get_state()
            keep = {k: v for k, v in st.items() if k != "mt_key"}
            path = os.path.join(ROOT, "data", "c3_t%d.npz" % t)
            np.savez_compressed(path, **keep)
            print(path, stats(st), "%.0f s" % (time.time() - t0), flush=True)
    o.close()


if __name__ == "__main__":
    main()
