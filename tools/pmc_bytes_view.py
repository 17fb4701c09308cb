#!/usr/bin/env python3
"""Per-kernel FETCH_SIZE / WRITE_SIZE (KiB counters -> GB) of the last step from tools/pmc_bytes.sh:
    python3 tools/pmc_bytes_view.py gpurun_out/pmcb_<tag>_FETCH_SIZE gpurun_out/pmcb_<tag>_WRITE_SIZE
Raw values (no gfx950 doubling); dispatch counts per kernel."""
import collections
import csv
import glob
import sys

tot = collections.defaultdict(lambda: [0.0, 0.0, 0])
for k, d in enumerate(sys.argv[1:3]):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tns::", "")[:44]
        tot[name][k] += float(r["Counter_Value"]) * 1024 / 1e9
        if k == 0:
            tot[name][2] += 1
for name, (fe, wr, n) in sorted(tot.items(), key=lambda kv: -(kv[1][0] + kv[1][1])):
    if fe + wr > 0.05:
        print(f"{name:44s} n={n:4d}  fetch {fe:7.2f} GB  write {wr:7.2f} GB")
