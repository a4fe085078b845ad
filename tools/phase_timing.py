#!/usr/bin/env python3
"""Where a latency-bound kernel's time goes: the diagnostics build of the
stepper (-DAIGAR_PHASE_TIMING, tick.hip PT_MARK) records, for every 8th wave,
the time from the wave's first instruction to each mark.  Runs the bench's C3
step (matured start, graph replays) and prints mean / max per mark in us.

  python tools/phase_timing.py build          # here: hipcc the diagnostics .so
  python tools/phase_timing.py run [steps] [random|greedy]   # GPU box (AIGAR_PT_START=world.npz: that start)
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.environ.get("AIGAR_PT_SO") or os.path.join(ROOT, "aigar_amd", "libaigar_hip_pt.so")
KERNELS = {0: ("k_food_prep", ["", "player", "cell", "pellet walk", "blob walk", "select", "reserve"]),
           1: ("k_players", ["", "player loads", "tail loads", "tail done", "update_player", "look-back", "seq + blobs"]),
           2: ("k_players/x", ["", "head+policy+queue", "cell updates", "arena block", "blob block", "last-block grid"]),
           3: ("k_pp_active", ["", "player", "cell", "grid test"]),
           4: ("k_food_commit", ["", "round 1", "r2 | cell list", "r3 | keys+recs", "r4 | eat loop", "rmax atomic", "serial (fold)", "round 7+"]),
           5: ("k_spawn_plan", ["", "pp serial", "compaction", "virus grid", "spawn counts", "pellet close", "pp closures", "pp turns"]),
           8: ("k_pel_update", ["", "first loads", "kill / join lists", "pellets + buckets", "fov cache", "virus spawns", "suffix loaded", "scans done"])}


def build():
    sys.path.insert(0, ROOT)
    from aigar_amd import _build
    cmd = ["hipcc"] + _build.FLAGS + ["-DAIGAR_PHASE_TIMING"] + [os.path.join(_build.CSRC, s) for s in _build.SOURCES]
    subprocess.check_call(cmd + ["-o", SO], cwd=_build.CSRC)
    print(SO)


def run(steps, policy="random"):
    os.environ["AIGAR_SO"] = SO
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from aigar_amd import _lib
    name = "c3"
    bots, field, pellets, virus, ps, pe, ch, ex, arenas = bench.WORKLOADS[name]
    stp = _lib.Stepper(bench.make_cfg(name, device=0, arenas=arenas))
    obs = torch.empty((bots, stp.obs_len), dtype=torch.float64, device="cuda")
    start = os.environ.get("AIGAR_PT_START")  # (a saved world instead, e.g. data/c3_greedy_late.npz)
    if start:
        import numpy as np
        z = np.load(start)
        stp.reset(1234)
        stp.load_state({k: z[k] for k in z.files}, 0)
        print(start)
    else:
        print(bench.start_world(stp, name, 1234, arenas))
    stp.run(20, policy, obs, p_split=ps, p_eject=pe, seed=1234, greedy_split=True)
    stp.sync()
    import numpy as np
    L = C.CDLL(SO)
    W = 8192
    buf = np.zeros((9, W, 8), dtype=np.uint32)
    ids = np.zeros((9, W, 2), dtype=np.uint32)
    khz = C.c_int(0)
    ptr = buf.ctypes.data_as(C.POINTER(C.c_uint))
    iptr = ids.ctypes.data_as(C.POINTER(C.c_uint))
    rec = {}
    placement = {}
    for _ in range(steps):  # one step per snapshot: every wave's slots are written once per step
        assert L.aigar_debug_phase_times(None, None, C.byref(khz), 1) == 0
        stp.run(1, policy, obs, p_split=ps, p_eject=pe, seed=99, greedy_split=True)
        stp.sync()
        assert L.aigar_debug_phase_times(ptr, iptr, C.byref(khz), 0) == 0
        pa_acc = pa_acc + buf[6, 0, :].astype(np.float64) if "pa_acc" in dir() else buf[6, 0, :].astype(np.float64)
        pa_cnt = pa_cnt + buf[7, 0, :].astype(np.float64) if "pa_cnt" in dir() else buf[7, 0, :].astype(np.float64)
        pg_acc = pg_acc + buf[6, 1024, :].astype(np.float64) if "pg_acc" in dir() else buf[6, 1024, :].astype(np.float64)
        pg_cnt = pg_cnt + buf[7, 1024, :].astype(np.float64) if "pg_cnt" in dir() else buf[7, 1024, :].astype(np.float64)
        sub = buf[6, 2048:2048 + 64, :].astype(np.float64)  # pp pass block sub-marks, per arena block
        sub_ok = sub[:, 6] > 0  # (blocks that ran the parallel pass this step)
        if sub_ok.any():
            sb_acc = (sb_acc if "sb_acc" in dir() else 0) + sub[sub_ok].sum(axis=0)
            sb_n = (sb_n if "sb_n" in dir() else 0) + int(sub_ok.sum())
        for k in KERNELS:
            started = buf[k, :, 0] != 0
            if not started.any():
                continue
            t0 = buf[k, started, 0].astype(np.int64)
            skew = (t0 - t0.min()) % (1 << 32)
            rec.setdefault((k, 0), []).extend(skew.tolist())
            widx = np.nonzero(started)[0]
            dec = (widx * 10 // max(1, widx.max() + 1))
            for q in range(10):
                sel = dec == q
                if sel.any():
                    rec.setdefault((k, "dec", q), []).extend(skew[sel].tolist())
            hw, xcc = ids[k, started, 0], ids[k, started, 1]
            cu = (xcc.astype(np.int64) << 8) | ((hw >> 8) & 0xFF)  # XCC | SE, SH, CU
            placement.setdefault(k, []).append((cu, skew))
            for m in range(1, 8):
                v = buf[k, started, m]
                done = v != 0
                if done.any():
                    rec.setdefault((k, m), []).extend(v[done].tolist())
                    rec.setdefault((k, m, "end"), []).append(int((skew[done] + v[done]).max()))
    us = 1e3 / khz.value
    print("wall clock %d kHz; %d steps; us from each wave's own start (start: skew after the first wave)"
          % (khz.value, steps))
    print("%-14s %-14s %9s %8s %8s %8s %8s %10s" % ("kernel", "mark", "waves/st", "mean", "p50", "p90", "max",
                                                   "span max"))
    for k, (kn, marks) in KERNELS.items():
        for m in range(0, len(marks)):
            v = np.asarray(rec.get((k, m), []), dtype=np.float64) * us
            if not len(v):
                continue
            span = np.asarray(rec.get((k, m, "end"), [0]), dtype=np.float64) * us
            print("%-14s %-14s %9.1f %8.2f %8.2f %8.2f %8.2f %10.2f" % (
                kn, marks[m] or "start", len(v) / steps, v.mean(), np.percentile(v, 50), np.percentile(v, 90),
                v.max(), span.mean() if m else 0.0))
    if "pa_acc" in dir():  # the pp serial pass, arena 0: accumulated buckets per step
        names = ["setup", "turn start", "gather walk", "rank", "eat", "re-activation walk", "skip+reload", "rest"]
        print("pp serial pass (arena 0, per step): " + ", ".join(
            "%s %.2f us" % (nm, pa_acc[k] * us / steps) for k, nm in enumerate(names)))
        print("pp serial pass counts per step: turns %.2f, gathers %.2f, eats %.2f, pc eaten %.2f, candidates %.2f" % tuple(
            pa_cnt[k] / steps for k in (0, 1, 2, 3, 4)))
    if "pg_acc" in dir():  # the parallel groups' waves, arena 0, summed over waves
        names = ["setup", "turn start", "gather walk", "rank", "eat", "re-activation walk", "skip+reload", "rest"]
        print("pp group waves (arena 0, per step, summed over waves): " + ", ".join(
            "%s %.2f us" % (nm, pg_acc[k] * us / steps) for k, nm in enumerate(names)))
        print("pp group waves counts per step: turns %.2f, gathers %.2f, eats %.2f, pc eaten %.2f, candidates %.2f" % tuple(
            pg_cnt[k] / steps for k in (0, 1, 2, 3, 4)))
    if "sb_acc" in dir():
        names = ["pown init", "seed closures", "labels", "merged closures", "owner check", "turns", "death sort",
                 "occ rebuild"]
        print("pp parallel pass block marks (mean over %d block-steps, us from kernel start): " % sb_n + ", ".join(
            "%s %.2f" % (nm, sb_acc[k] * us / sb_n) for k, nm in enumerate(names)))
    khz_ = khz.value / 1e3
    for k in KERNELS:
        row = []
        for q in range(10):
            v = np.asarray(rec.get((k, "dec", q), []), dtype=np.float64) * us
            row.append("%5.1f/%5.1f" % (np.median(v), v.max()) if len(v) else "-")
        print("%-14s start skew (median/max us) by wave-index decile: %s" % (KERNELS[k][0], " ".join(row)))
    for k, lst in placement.items():
        cus, late = {}, {}
        for cu, skew in lst:
            for c, sk in zip(cu.tolist(), skew.tolist()):
                cus[c] = cus.get(c, 0) + 1
                late[c] = late.get(c, 0) + (sk / khz_ > 4.0)
        n = len(lst)
        per = np.array(list(cus.values())) / n
        lt = np.array([late[c] for c in cus]) / n
        print("%-14s waves per CU per step: %d CUs used, mean %.1f, min %.1f, max %.1f; waves starting >4 us late "
              "per CU: mean %.2f, max %.1f; late waves on the CUs holding the most waves: %.2f" % (
                  KERNELS[k][0], len(cus), per.mean(), per.min(), per.max(), lt.mean(), lt.max(),
                  lt[per >= np.percentile(per, 75)].mean()))
    stp.close()


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 50, sys.argv[3] if len(sys.argv) > 3 else "random")
