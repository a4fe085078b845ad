#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV: per-kernel avg us, calls/step, us/step.
Kernels of less than half a launch per step (the snapshot load before the timed
region: `__amd_rocclr_*` copies / fills, reset / load kernels) are listed apart
and left out of the per-step total."""
import csv
import sys

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
# steps: given, else the number of ticks (k_players launches: the tick's first kernel) in the trace
steps = float(sys.argv[2]) if len(sys.argv) > 2 else float(
    next((r["Calls"] for r in rows if "k_players" in r["Name"]), 110.0))
fmt = "%-58s %7.2f %8.2f %9.2f"
print("%-58s %7s %8s %9s" % ("kernel", "calls/s", "avg_us", "us/step"))
tot, other = 0.0, []
for r in rows:
    n = float(r["Calls"])
    if n / steps < 0.5 or r["Name"].startswith("__amd_rocclr"):
        other.append(r)
        continue
    tot += float(r["TotalDurationNs"])
    print(fmt % (r["Name"][:58], n / steps, float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3 / steps))
print("total kernel time per step: %.1f us (%d steps)" % (tot / 1e3 / steps, steps))
if other:
    print("outside the timed step (snapshot load before it):")
    for r in other:
        print("  %-56s calls %5d avg_us %8.2f" % (r["Name"][:56], int(float(r["Calls"])), float(r["AverageNs"]) / 1e3))
