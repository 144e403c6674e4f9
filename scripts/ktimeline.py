#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel_trace.csv: one line per dispatch (start / end relative to
the first listed dispatch, duration, stream), from dispatch index A to B."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
a = int(sys.argv[2]) if len(sys.argv) > 2 else 0
b = int(sys.argv[3]) if len(sys.argv) > 3 else len(rows)
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
    print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f}  q{r['Queue_Id']} s{r['Stream_Id']}  "
          f"grid {int(r['Grid_Size_X']) // max(int(r['Workgroup_Size_X']), 1):6d}  {name}")
