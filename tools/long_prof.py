#!/usr/bin/env python3
"""The clustered Greedy regime (GPU box, under rocprofv3): 1500 random ticks
then 1500 Greedy ticks from the matured start, so a kernel trace shows where a
late Greedy tick's time goes (tools/long_run.py for the timing alone).

  rocprofv3 --kernel-trace --stats -- python3 tools/long_prof.py [state.npz]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from aigar_amd import _lib
    bots, field, pellets, virus, ps, pe, ch, ex, arenas = bench.WORKLOADS["c3"]
    stp = _lib.Stepper(bench.make_cfg("c3", device=0, arenas=arenas))
    obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
    print(bench.start_world(stp, "c3", 1234, arenas), flush=True)
    stp.run(1500, "random", obs, p_split=ps, p_eject=pe, seed=7, greedy_split=True)
    stp.sync()
    stp.run(1400, "greedy", obs, p_split=ps, p_eject=pe, seed=8, greedy_split=True)
    stp.sync()
    c0 = stp.counters()
    stp.run(100, "greedy", obs, p_split=ps, p_eject=pe, seed=9, greedy_split=True)
    stp.sync()
    c1 = stp.counters()
    print({k: round((c1[k] - c0[k]) / 100, 3) for k in c1}, flush=True)
    if len(sys.argv) > 1:  # keep the clustered world (a start for short Greedy A/B runs)
        import numpy as np
        st = stp.get_state(0)
        np.savez_compressed(sys.argv[1], **st)
        cf = np.asarray(st["cells_f"])
        print("saved", sys.argv[1], "cells", len(cf), "max mass", float(cf[:, 2].max()), flush=True)
    stp.close()


if __name__ == "__main__":
    main()
