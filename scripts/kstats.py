#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: per-kernel calls, mean us, total ms, share (top N)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
div = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0  # e.g. steps: per-step ms
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.3f} ms ({tot / 1e6 / div:.3f} ms per unit of {div:g})")
for r in rows[:n]:
    print(f"{float(r['Percentage']):6.2f}%  {int(r['Calls']):6d}  {float(r['AverageNs']) / 1e3:9.2f} us  "
          f"{float(r['TotalDurationNs']) / 1e6 / div:8.3f} ms  {r['Name'][:110]}")
