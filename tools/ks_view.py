#!/usr/bin/env python3
"""Print the last step's MSM-related dispatches of a rocprofv3 kernel trace."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
pats = sys.argv[3].split(",") if len(sys.argv) > 3 else None
for r in rows[-n:]:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if pats and not any(p in k for p in pats):
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(f"{k[:60]:60s} {d:9.3f} ms  vgpr {r['VGPR_Count']:>4s} scratch {r['Scratch_Size']:>5s} grid {r['Grid_Size_X']}")
