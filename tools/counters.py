#!/usr/bin/env python3
"""Per-tick work counters of the C3 bench step (GPU box): how many cells / players
each serial pass took, pellets eaten and spawned, from the matured start.

  python tools/counters.py [steps] [random|greedy]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(steps=200, policy="random"):
    import torch
    import bench
    from aigar_amd import _lib
    name = "c3"
    bots, field, pellets, virus, ps, pe, ch, ex, arenas = bench.WORKLOADS[name]
    stp = _lib.Stepper(bench.make_cfg(name, device=0, arenas=arenas))
    obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
    print(bench.start_world(stp, name, 1234, arenas))
    stp.run(20, policy, obs, p_split=ps, p_eject=pe, seed=1234, greedy_split=True)
    stp.sync()
    c0 = stp.counters()
    stp.run(steps, policy, obs, p_split=ps, p_eject=pe, seed=99, greedy_split=True)
    stp.sync()
    c1 = stp.counters()
    print("%s, %d ticks: per tick" % (policy, steps))
    for k in c1:
        print("  %-20s %10.3f" % (k, (c1[k] - c0[k]) / steps))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200, sys.argv[2] if len(sys.argv) > 2 else "random")
