#!/usr/bin/env python3
"""Greedy ticks from a clustered world (GPU box): the late-Greedy regime of
tools/long_run.py without its 3000 lead-in ticks.  The start is the world
tools/long_prof.py saved after 1500 random + 1500 Greedy ticks
(data/c3_greedy_late.npz); the variant library is picked by AIGAR_SO as in
tools/abn.sh.

  python tools/clustered.py [ticks] [snapshot]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(ticks=200, snap=os.path.join(ROOT, "data", "c3_greedy_late.npz")):
    import numpy as np
    import torch
    import bench
    from aigar_amd import _lib
    bots, field, pellets, virus, ps, pe, ch, ex, arenas = bench.WORKLOADS["c3"]
    stp = _lib.Stepper(bench.make_cfg("c3", device=0, arenas=1))
    obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
    z = np.load(snap)
    stp.reset(1234)
    stp.load_state({k: z[k] for k in z.files}, 0)
    run = lambda n, s: stp.run(n, "greedy", obs, p_split=ps, p_eject=pe, seed=s, greedy_split=True)
    run(20, 3)
    stp.sync()
    c0 = stp.counters()
    t0 = time.perf_counter()
    run(ticks, 4)
    stp.sync()
    dt = time.perf_counter() - t0
    c1 = stp.counters()
    cnt = {k: round((c1[k] - c0[k]) / ticks, 2) for k in c1 if k != "ticks"}
    print("clustered greedy: %.3f ms/tick over %d ticks %s" % (dt / ticks * 1e3, ticks, cnt), flush=True)
    stp.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200, *sys.argv[2:3])
