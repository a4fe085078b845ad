#!/usr/bin/env python3
"""Per-kernel average duration from a rocprofv3 kernel trace, split by grid size
(the C4 tile timing runs tiled and untiled handles in one process: the same
kernel with different launch geometry is listed apart) and by phase of the run.

  python tools/trace_split.py run_kernel_trace.csv [skip_first_n_dispatches]"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
agg = defaultdict(list)
for r in rows[skip:]:
    nm = r["Kernel_Name"].split("(")[0].replace("aigar::", "")
    if nm.startswith("__amd"):
        continue
    key = (nm, r["Grid_Size_X"], r["Grid_Size_Y"])
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print("%-34s %9s %5s %6s %8s %8s" % ("kernel", "grid_x", "gy", "calls", "avg_us", "max_us"))
for (nm, gx, gy), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print("%-34s %9s %5s %6d %8.2f %8.2f" % (nm[:34], gx, gy, len(v), sum(v) / len(v), max(v)))
