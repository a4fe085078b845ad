#!/usr/bin/env python3
"""Robustness run (GPU box): the bench's C3 step graph for many ticks from the
matured start, random then Greedy population, checking the device error bits
after every chunk (Stepper.sync raises on any) and printing the work counters.

  python tools/long_run.py [ticks] [chunk]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(ticks=3000, chunk=250):
    import torch
    import bench
    from aigar_amd import _lib
    name = "c3"
    bots, field, pellets, virus, ps, pe, ch, ex, arenas = bench.WORKLOADS[name]
    stp = _lib.Stepper(bench.make_cfg(name, device=0, arenas=arenas))
    obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
    print(bench.start_world(stp, name, 1234, arenas), flush=True)
    for policy in ("random", "greedy"):
        c0 = stp.counters()
        t0 = time.perf_counter()
        done = 0
        while done < ticks:
            n = min(chunk, ticks - done)
            stp.run(n, policy, obs, p_split=ps, p_eject=pe, seed=7 + done, greedy_split=True)
            stp.sync()  # (raises on a device error bit)
            done += n
            assert torch.isfinite(obs[:, :8]).any(), "observations all NaN"
            print("%s: %d ticks ok (%.1f s)" % (policy, done, time.perf_counter() - t0), flush=True)
        c1 = stp.counters()
        print(policy, {k: round((c1[k] - c0[k]) / ticks, 3) for k in c1}, flush=True)
    stp.close()
    print("long run ok")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3000, int(sys.argv[2]) if len(sys.argv) > 2 else 250)
