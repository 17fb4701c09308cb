"""Print the kernel timeline of the last `--from` kernel occurrence group in a rocprofv3 kernel trace.
    python3 tools/trace_tail.py <run_kernel_trace.csv> <first-kernel-substring> [min_ms]
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
first = sys.argv[2]
min_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
idx = [i for i, x in enumerate(rows) if first in x["Kernel_Name"]]
start = idx[-1]
t0 = int(rows[start]["Start_Timestamp"])
tot = {}
for x in rows[start:]:
    s = (int(x["Start_Timestamp"]) - t0) / 1e6
    d = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
    name = x["Kernel_Name"].split("(")[0]
    tot[name] = tot.get(name, 0) + d
    if d >= min_ms:
        print(f"{s:8.3f} {d:7.3f} q{x['Queue_Id']} g{x['Grid_Size_X']:>9s} lds{x['LDS_Block_Size']:>6s} v{x['VGPR_Count']:>4s} {name}")
print("--- totals")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{v:8.3f} {k}")
