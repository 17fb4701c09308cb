#!/usr/bin/env python3
"""Kernel durations of the last MSM in a rocprofv3 kernel trace (from its last k_scalar_bits on),
summed per kernel and grid size: tools/last_msm.py <run_kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
start = max(i for i, x in enumerate(rows) if "k_scalar_bits" in x["Kernel_Name"])
t0 = int(rows[start]["Start_Timestamp"])
end = int(rows[-1]["End_Timestamp"])
agg = {}
for x in rows[start:]:
    d = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
    key = (x["Kernel_Name"].split("(")[0].replace("tns::", "")[:40], x["Grid_Size_X"])
    agg[key] = agg.get(key, 0) + d
for (name, g), d in sorted(agg.items(), key=lambda kv: -kv[1]):
    if d >= 0.02:
        print(f"   {d:7.3f} ms  g{g:>10s} {name}")
print(f"   wall {(end - t0) / 1e6:.3f} ms")
