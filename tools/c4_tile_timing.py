#!/usr/bin/env python3
"""Per-tile kernel time of the C4 tiled tick with the tiles run one at a time.

The 1-GPU rehearsal of bench.py --gpus N puts N ranks on one card, so every
tile's kernels share the GPU with the others' and the gloo exchange is staged
through host memory: neither is the per-tile cost on its own GPU.  Here all
tile handles of one arena live in this process (LocalTransport) and each
phase of each tile is issued and synchronised alone, HIP events around it (the
handle's own marks): the time a tile's GPU would spend per tick, without the
exchange (RCCL, measured only on a multi-GPU node).

  python tools/c4_tile_timing.py [ntiles] [ticks]      (GPU box)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from aigar_amd import _lib, tiles
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    tx, ty = tiles.tile_grid(n)
    cfg = bench.make_cfg("c3")
    bots, field, pellets, virus, ps, pe, ch, ex, _ = bench.WORKLOADS["c3"]
    ts = [_lib.Stepper(tiles.tile_config(cfg, tx, ty, k, cap=512)) for k in range(n)]  # (bench.py's C4 message)
    for t in ts:
        bench.start_world(t, "c3", 1, 1)
    obs = [torch.empty((bots, t.obs_len), dtype=torch.float64, device="cuda") for t in ts]

    def tick(seed):
        for t in ts:
            t.tile_begin("random", ps, pe, seed)
            t.sync()
        _lib.tile_exchange_local(ts)
        for t in ts:
            t.sync()
        for t in ts:
            t.tile_apply(wait=False)
            t.sync()
        for k, t in enumerate(ts):
            t.tile_end(obs[k])
            t.sync()

    for _ in range(5):
        tick(7)
    for t in ts:
        t.profile(True)
    for _ in range(ticks):
        tick(7)
    names = ("tile_begin", "tile_apply", "tile_end", "observe")
    rows = []
    for k, t in enumerate(ts):
        r = {nm: t.kernel_time(nm)[0] / ticks * 1e3 for nm in names}
        r["tile"] = k
        r["bots_observed"] = int(np.sum(t.tile_observers() == k))
        r["total_us"] = sum(r[nm] for nm in names)
        rows.append(r)
        t.profile(False)
    # the untiled step's phases on the same box for comparison
    u = _lib.Stepper(cfg)
    bench.start_world(u, "c3", 1, 1)
    uo = torch.empty((bots, u.obs_len), dtype=torch.float64, device="cuda")
    for _ in range(5):
        u.policy_random(ps, pe, 7)
        u.step(1)
        u.observe(uo)
    u.profile(True)
    for _ in range(ticks):
        u.policy_random(ps, pe, 7)
        u.step(1)
        u.observe(uo)
        u.sync()
    un = {nm: u.kernel_time(nm)[0] / ticks * 1e3 for nm in ("policy", "tick", "observe")}
    out = {"ntiles": n, "layout": "%dx%d" % (tx, ty), "ticks": ticks, "per_tile_us": rows, "untiled_us": un,
           "max_tile_total_us": max(r["total_us"] for r in rows),
           "message_bytes_first_pass": ts[0].tile_info()["msg_bytes"]}
    print(json.dumps(out))
    for t in ts:
        t.close()
    u.close()


if __name__ == "__main__":
    main()
