"""Per-wave phase timing of k_observe (diagnostics build, -DAIGAR_OBS_TIMING).

Build here:  python tools/micro/obs_timing.py --build
Run on GPU:  python tools/micro/obs_timing.py [--workload c3]
Stamps (wall_clock64, 100 MHz): 0 wave start, 1 FOV cache read, 2 walk done,
3 pellets ranked, 4 squares done.
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SO = os.path.join(ROOT, "tools", "micro", "libaigar_hip_ts%s.so")
sys.path.insert(0, ROOT)


def build(tag, defines):
    from aigar_amd import _build
    cmd = ["hipcc"] + _build.FLAGS + ["-DAIGAR_OBS_TIMING"] + ["-D" + x for x in defines]
    cmd += [os.path.join(_build.CSRC, s) for s in _build.SOURCES]
    subprocess.check_call(cmd + ["-o", SO % tag], cwd=_build.CSRC)
    print(SO % tag)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--tag", default="")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    args = ap.parse_args()
    if args.build:
        return build(args.tag, args.defines)
    os.environ["AIGAR_SO"] = SO % args.tag
    import torch
    import bench
    from aigar_amd import _lib
    name = args.workload
    bots, field, pellets, virus, ps, pe, ch, ex, arenas = bench.WORKLOADS[name]
    stp = _lib.Stepper(bench.make_cfg(name))
    stp.set_stream(torch.cuda.current_stream().cuda_stream)
    obs = torch.empty((bots * arenas, stp.obs_len), dtype=torch.float64, device="cuda")
    stp.reset(1)
    for _ in range(args.warmup):
        stp.policy_random(ps, pe, 1)
        stp.step(1)
        stp.observe(obs)
    torch.cuda.synchronize()
    L = _lib.load()
    n = bots * arenas
    ts = np.zeros((n, 8), np.uint64)
    assert L.aigar_debug_obs_ts(ts.ctypes.data_as(C.c_void_p), n) == 0
    smid = ts[:, 5].astype(np.int64)
    cnt6 = ts[:, 6].astype(np.int64)
    ts = ts[:, :5].astype(np.int64)
    alive = ts[:, 4] > 0
    ts = ts[alive]
    smid = smid[alive]
    cnt6 = cnt6[alive]
    npel, ncel, nvir = cnt6 & 0xFFFFF, (cnt6 >> 20) & 0xFFFFF, cnt6 >> 40
    qq = lambda v: "mean %.1f p50 %d p90 %d max %d" % (v.mean(), *np.percentile(v, [50, 90, 100]))
    print("visible pellets", qq(npel))
    print("visible cells  ", qq(ncel))
    print("visible viruses", qq(nvir))
    t0 = ts[:, 0].min()
    ns = lambda v: v * 10.0  # 100 MHz -> ns
    start = ns(ts[:, 0] - t0) / 1000
    end = ns(ts[:, 4] - t0) / 1000
    print("waves", len(ts), "span us %.2f" % end.max())
    q = lambda v: "p10 %.2f p50 %.2f p90 %.2f max %.2f" % tuple(np.percentile(v, [10, 50, 90, 100]))
    print("start offset us ", q(start))
    print("end us          ", q(end))
    names = ["prologue", "walk", "rank", "squares"]
    for k in range(4):
        print("%-15s" % names[k], q(ns(ts[:, k + 1] - ts[:, k]) / 1000))
    print("total per wave  ", q(ns(ts[:, 4] - ts[:, 0]) / 1000))
    late_m = start > 3.0
    print("late starters: %d of %d" % (late_m.sum(), len(ts)))
    u, cnt = np.unique(smid, return_counts=True)
    print("distinct smid %d, waves per smid: min %d max %d" % (len(u), cnt.min(), cnt.max()))
    ul, cl = np.unique(smid[~late_m], return_counts=True)
    print("first round: distinct smid %d, waves per smid min %d max %d" % (len(ul), cl.min(), cl.max()))
    print("smid samples", [hex(x) for x in u[:8]], [hex(x) for x in u[-8:]])
    gp = np.nonzero(alive)[0]
    print("late gp by residue mod 8:", np.bincount(gp[late_m] % 8, minlength=8))
    # does the kernel span come from late starts or long waves?
    late = np.argsort(end)[-10:]
    for i in late:
        print("slow wave: start %.2f dur %.2f" % (start[i], (end[i] - start[i])), ns(np.diff(ts[i])) / 1000)
    st = stp.get_state()
    print("pellets", st["n_pellets"], "cells", st["n_cells"])


if __name__ == "__main__":
    main()
