#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV: per-kernel avg us, calls/step, us/step."""
import csv
import sys

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
# steps: given, else the number of ticks (k_tick_begin launches) in the trace
steps = float(sys.argv[2]) if len(sys.argv) > 2 else float(
    next((r["Calls"] for r in rows if "k_tick_begin" in r["Name"]), 110.0))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("%-58s %7s %8s %9s %6s" % ("kernel", "calls/s", "avg_us", "us/step", "%"))
for r in rows:
    n = float(r["Calls"])
    print("%-58s %7.2f %8.2f %9.2f %6.1f" % (r["Name"][:58], n / steps, float(r["AverageNs"]) / 1e3,
                                            float(r["TotalDurationNs"]) / 1e3 / steps, float(r["Percentage"])))
print("total kernel time per step: %.1f us" % (tot / 1e3 / steps))
