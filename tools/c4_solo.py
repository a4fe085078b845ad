#!/usr/bin/env python3
"""Per-GPU cost of a C4 tile step, each tile alone on the GPU (timing rehearsal).

bench.py's C4 leg steps one tile per rank with aigar_tile_run: the whole tiled
step -- policy, the tick with its eat-phase all-gather, the observation of the
tile's bots -- as ONE hipGraph replay.  On a one-GPU box the 8 tiles of the 4x2
layout cannot each have a GPU, and tools/c4_tile_timing.py runs them one after
the other with a sync between phases: every tile's kernels then find the other
tiles' worlds in the caches and no graph, which inflates every kernel.  Here
each tile k runs alone: its own handle, the matured C3 world, aigar_tile_loopback
(the all-gather replaced by a copy of its own message; the other tiles' slots
are empty messages), and aigar_tile_run's graph replayed for `steps` steps,
timed with HIP events on the tile's stream.  That is the tile's GPU time per
step WITHOUT the exchange (its world drifts from the tiled arena's: no other
tile's outcomes arrive).  The untiled step (aigar_run, the bench's N = 1 graph)
is timed the same way on the same box.

  python tools/c4_solo.py [ntiles] [steps]      (GPU box)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(torch, fn, steps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    fn(steps)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps * 1e3  # us per step


def main():
    import torch
    import bench
    from aigar_amd import _lib, tiles
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    tx, ty = tiles.tile_grid(n)
    bots, field, pellets, virus, ps, pe, ch, ex, _ = bench.WORKLOADS["c3"]
    cfg = bench.make_cfg("c3")
    stream = torch.cuda.current_stream()
    rows = []
    for k in range(n):
        t = _lib.Stepper(tiles.tile_config(cfg, tx, ty, k, cap=512))  # (bench.py's C4 message)
        t.set_stream(stream.cuda_stream)
        bench.start_world(t, "c3", 1, 1)
        t.tile_loopback()
        obs = torch.empty((bots, t.obs_len), dtype=torch.float64, device="cuda")

        def run(m):
            t.tile_run(m, "random", obs, p_split=ps, p_eject=pe, seed=7, extra_passes=0)
        run(20)
        us = timed(torch, run, steps)
        graphed = t.tile_run_graphed()
        # phase breakdown: the same steps as direct launches, HIP events per phase
        t.profile(True)
        run(30)
        torch.cuda.synchronize()
        br = {nm: t.kernel_time(nm)[0] / 30 * 1e3 for nm in ("tile_begin", "exchange", "tile_apply", "tile_end",
                                                               "observe")}
        t.profile(False)
        t.sync()
        rows.append({"tile": k, "us_per_step_graph": us, "graphed": graphed,
                     "bots_observed": int(np.sum(t.tile_observers() == k)), "phases_us_direct": br})
        t.close()
        del obs
    u = _lib.Stepper(cfg)
    u.set_stream(stream.cuda_stream)
    bench.start_world(u, "c3", 1, 1)
    uo = torch.empty((bots, u.obs_len), dtype=torch.float64, device="cuda")

    def urun(m):
        u.run(m, "random", uo, p_split=ps, p_eject=pe, seed=7)
    urun(20)
    uus = timed(torch, urun, steps)
    u.sync()
    u.close()
    out = {"ntiles": n, "layout": "%dx%d" % (tx, ty), "steps": steps, "per_tile": rows,
           "max_tile_us_per_step": max(r["us_per_step_graph"] for r in rows),
           "untiled_us_per_step": uus,
           "note": "each tile alone on the GPU, aigar_tile_run graph, exchange = a copy of its own message "
                   "(aigar_tile_loopback); untiled = aigar_run graph (bench.py N = 1), same box"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
