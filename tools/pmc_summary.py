#!/usr/bin/env python3
"""Per-launch HBM-side bytes of each kernel from tools/pmc.sh output.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts
128-B read requests as 64 B (MI355X_MICROARCH.md, HBM section), so the read
figure is doubled; Infinity-Cache hits are included (the C3 world is ~10 MB).
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
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fr = 2 * 1024 * sum(f) / max(1, len(f))
        wr = 1024 * sum(w) / max(1, len(w))
        out[k] = {"launches": len(f), "fetch_bytes_raw": 1024 * sum(f) / max(1, len(f)), "read_bytes": fr,
                  "write_bytes": wr, "traffic_bytes": fr + wr}
        print("%-60s n=%4d read %12.0f B  write %12.0f B  total %12.0f B" % (k[:60], len(f), fr, wr, fr + wr))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
