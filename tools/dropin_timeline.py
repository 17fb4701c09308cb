#!/usr/bin/env python3
"""Merged kernel + memory-copy timeline of the LAST drop-in proof in a rocprofv3 run of
tools/dropin_trace.py (--kernel-trace --memory-copy-trace): from the last proof's first H2D copy
to its last kernel.  Copies are summed into runs (consecutive copies of one direction).
    python3 tools/dropin_timeline.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv> [min_ms]
"""
import csv
import glob
import os
import sys

d = sys.argv[1]
min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.03
kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
mt = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)[0]
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"].split("(")[0], r.get("Queue_Id", ""))
      for r in csv.DictReader(open(kt))]
ms = []
for r in csv.DictReader(open(mt)):
    kind = r.get("Direction") or r.get("Operation") or "COPY"
    ms.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M", kind.replace("MEMORY_COPY_", ""),
               r.get("Size") or "0"))
ms.sort()
# the last proof: copies of >= 0.1 ms (the 16 MiB staged chunks; this rocprofv3 records no sizes);
# a proof's uploads are separated from the previous proof's by > 5 ms
big = [m for m in ms if m[1] - m[0] >= 100_000 and "HOST_TO_DEVICE" in m[3]]
starts = [big[0][0]] + [b[0] for a, b in zip(big, big[1:]) if b[0] - a[1] > 5_000_000]
t0 = starts[-1]
ev = sorted([k for k in ks if k[0] >= t0] + [m for m in ms if m[0] >= t0])
# copy runs
out, run = [], None
for e in ev:
    if e[2] == "M":
        if run and run[3] == e[3] and e[0] - run[1] < 200_000:
            run[1] = max(run[1], e[1]); run[4] += int(e[4] or 0); run[5] += 1
        else:
            if run: out.append(tuple(run))
            run = [e[0], e[1], "M", e[3], int(e[4] or 0), 1]
    else:
        out.append(e)
if run: out.append(tuple(run))
out.sort()
end = max(e[1] for e in out)
for e in out:
    s, dur = (e[0] - t0) / 1e6, (e[1] - e[0]) / 1e6
    if e[2] == "M":
        print(f"{s:8.3f} {dur:7.3f} COPY {e[3]} x{e[5]}")
    elif dur >= min_ms:
        print(f"{s:8.3f} {dur:7.3f} q{e[4]} {e[3]}")
print(f"--- last proof span {(end - t0) / 1e6:.3f} ms")
