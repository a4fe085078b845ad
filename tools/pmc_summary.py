#!/usr/bin/env python3
"""Per-launch and per-step HBM-side bytes of every kernel from `tools/gpu.sh TAG pmc` output.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts
128-B read requests as 64 B (MI355X_MICROARCH.md, HBM section), so the read
figure is doubled; Infinity-Cache hits are included (the C3 world is ~10 MB).
The step totals count the kernels of the timed env step only: launches per
step = launches / steps (steps = the k_players launches: the tick's first kernel); the snapshot load
before the timed region (`__amd_rocclr_*` copies and fills, the one-off
reset / load kernels, < 1 launch per step) is reported apart.
usage: pmc_summary.py DIR_FETCH DIR_WRITE [out.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(list)
    for row in csv.DictReader(open(f[0])):
        if row["Counter_Name"] != counter:
            continue
        acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return acc


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    steps = max((len(v) for k, v in fetch.items() if "k_players" in k), default=1)
    out, step = {}, {"read_bytes": 0.0, "write_bytes": 0.0, "traffic_bytes": 0.0, "kernels": 0, "steps": steps}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fr = 2 * 1024 * sum(f) / max(1, len(f))
        wr = 1024 * sum(w) / max(1, len(w))
        per_step = len(f) / steps
        in_step = per_step >= 0.5 and not k.startswith("__amd_rocclr")
        out[k] = {"launches": len(f), "launches_per_step": per_step, "in_step": in_step,
                  "fetch_bytes_raw": 1024 * sum(f) / max(1, len(f)), "read_bytes": fr, "write_bytes": wr,
                  "traffic_bytes": fr + wr}
        if in_step:
            step["read_bytes"] += fr * per_step
            step["write_bytes"] += wr * per_step
            step["traffic_bytes"] += (fr + wr) * per_step
            step["kernels"] += 1
        print("%-60s n=%4d /step %4.2f read %12.0f B  write %12.0f B  total %12.0f B%s" % (
            k[:60], len(f), per_step, fr, wr, fr + wr, "" if in_step else "  (outside the step)"))
    print("step (%d kernels, %d steps): read %.0f B  write %.0f B  total %.0f B per step" % (
        step["kernels"], steps, step["read_bytes"], step["write_bytes"], step["traffic_bytes"]))
    out["_step"] = step
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
