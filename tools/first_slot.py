#!/usr/bin/env python3
"""How often a player's first cell sits in pool slot 0 (GPU box): the bench's C3
world, stepped with the random and the Greedy population; after each step the
first list row and the cell counts are read back (aigar_debug_first_slots).
A kernel that loaded slot 0's record beside the player's list row would skip a
dependent load round for those players.
usage: python tools/first_slot.py [steps]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(steps):
    import torch
    import bench
    from aigar_amd import _lib
    out = {}
    for policy, snap in (("random", "c3"), ("greedy", "c3")):
        bots, field, pellets, virus, ps, pe, ch, ex, arenas = bench.WORKLOADS["c3"]
        stp = _lib.Stepper(bench.make_cfg("c3", device=0, arenas=1))
        obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
        bench.start_world(stp, snap, 1234, 1)
        L = stp.L
        L.aigar_debug_first_slots.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        s0 = np.zeros(bots, np.uint8)
        nc = np.zeros(bots, np.int32)
        rows = []
        for t in range(steps):
            stp.run(1, policy, obs, p_split=ps, p_eject=pe, seed=99, greedy_split=True)
            stp.sync()
            assert L.aigar_debug_first_slots(stp.h, s0.ctypes.data, nc.ctypes.data) == 0
            alive = nc > 0
            rows.append([int(alive.sum()), int((alive & (s0 == 0)).sum()), int((nc == 1).sum()),
                         int(((nc == 1) & (s0 == 0)).sum())])
        r = np.asarray(rows, dtype=np.float64)
        out[policy] = {"steps": steps, "alive": r[:, 0].mean(), "first_cell_in_slot0": r[:, 1].mean(),
                       "one_cell": r[:, 2].mean(), "one_cell_in_slot0": r[:, 3].mean(),
                       "frac_first_in_slot0": float(r[:, 1].sum() / r[:, 0].sum()),
                       "frac_first_in_slot0_last10": float(r[-10:, 1].sum() / r[-10:, 0].sum())}
        stp.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 100)
