#!/usr/bin/env python3
"""Per-kernel SQ counter summary (sums over dispatches): tools/pmc_view.py <counter_collection.csv> [kernel-substr,...]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pats = sys.argv[2].split(",") if len(sys.argv) > 2 else None
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if pats and not any(p in k for p in pats):
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k[:40]:40s} waves {c.get('SQ_WAVES',0):10.0f} valu_inst/wave {c.get('SQ_INSTS_VALU',0)/max(1,c.get('SQ_WAVES',1)):9.0f} "
          f"active_valu {c.get('SQ_ACTIVE_INST_VALU',0)/wc:5.2f} active_any {c.get('SQ_ACTIVE_INST_ANY',0)/wc:5.2f} "
          f"wait_any {c.get('SQ_WAIT_ANY',0)/wc:5.2f} wait_inst {c.get('SQ_WAIT_INST_ANY',0)/wc:5.2f}")
    extra = {n: v for n, v in c.items() if n not in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY",
                                                     "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES")}
    if extra:
        print("    " + "  ".join(f"{n} {v:.4g}" for n, v in sorted(extra.items())))
