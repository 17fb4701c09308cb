#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats kernel_stats.csv: tools/ks_top.py <csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{r['Name'][:58]:58s} {int(r['Calls']):5d} tot {float(r['TotalDurationNs']) / 1e6:9.3f} "
          f"avg {float(r['AverageNs']) / 1e6:8.3f} ms")
