#!/usr/bin/env python3
"""Fixed cost of one aigar_run call around the timed steps (GPU box): host
time of the call, and wall time of run(n) + synchronize for several n from the
matured C3 start, after a long warm-up (clocks and graph settled)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from aigar_amd import _lib
    bots, field, pellets, virus, ps, pe, ch, ex, arenas = bench.WORKLOADS["c3"]
    stp = _lib.Stepper(bench.make_cfg("c3", device=0, arenas=arenas))
    stp.set_stream(torch.cuda.current_stream().cuda_stream)
    obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
    bench.start_world(stp, "c3", 1234, arenas)

    def run(n):
        stp.run(n, "random", obs, p_split=ps, p_eject=pe, seed=1234, greedy_split=True)
    run(200)
    torch.cuda.synchronize()
    for n in (1, 2, 5, 20, 100, 1, 20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(n)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("n %4d: host call %7.1f us (%.1f per step), wall %8.1f us = %.1f us per step" %
              (n, (t1 - t0) * 1e6, (t1 - t0) * 1e6 / n, (t2 - t0) * 1e6, (t2 - t0) * 1e6 / n))
    # idle gap then 20 steps (as the driver's run: the GPU idles while the host prepares)
    time.sleep(0.5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(20)
    torch.cuda.synchronize()
    print("after 0.5 s idle, n 20: %.1f us per step" % ((time.perf_counter() - t0) * 1e6 / 20))
    stp.close()


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def chunks():
    """Fresh C3 world, GPU kept busy right before by another stepper: 20-step
    chunks timed one after the other (is the early slowness the world, or the GPU?)."""
    import torch
    import bench
    from aigar_amd import _lib
    bots, field, pellets, virus, ps, pe, ch, ex, arenas = bench.WORKLOADS["c3"]
    cfg = bench.make_cfg("c3", device=0, arenas=arenas)
    hot = _lib.Stepper(cfg)
    hot.set_stream(torch.cuda.current_stream().cuda_stream)
    ho = torch.empty((bots, hot.obs_len), dtype=torch.float64, device="cuda")
    bench.start_world(hot, "c3", 99, arenas)
    stp = _lib.Stepper(cfg)
    stp.set_stream(torch.cuda.current_stream().cuda_stream)
    obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
    bench.start_world(stp, "c3", 1234, arenas)
    hot.run(300, "random", ho, p_split=ps, p_eject=pe, seed=99, greedy_split=True)  # GPU busy, clocks up
    torch.cuda.synchronize()
    row = []
    for c in range(8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        stp.run(20, "random", obs, p_split=ps, p_eject=pe, seed=1234, greedy_split=True)
        torch.cuda.synchronize()
        row.append((time.perf_counter() - t0) * 1e6 / 20)
    print("fresh world after a busy GPU, 20-step chunks (us per step):", " ".join("%.1f" % v for v in row))
    hot.run(300, "random", ho, p_split=ps, p_eject=pe, seed=99, greedy_split=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stp.run(20, "random", obs, p_split=ps, p_eject=pe, seed=1234, greedy_split=True)
    torch.cuda.synchronize()
    print("the same stepper after 300 more steps of the other: %.1f us per step" % ((time.perf_counter() - t0) * 1e6 / 20))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "chunks":
    chunks()
