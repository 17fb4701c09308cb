#!/usr/bin/env python3
"""Time the tau-free Lagrange basis build (tns_srs_prepare_lagrange_from_powers, tfree.hip) at
2^lo .. 2^hi nodes on one GPU, check each against the tau-derived basis, and extrapolate the
one-time setup cost to C4 (2^24) and C5 (2^26) with the algorithm's N log^2 N law fitted to the
two largest sizes.  One JSON line on stdout.

    python tools/tfree_bench.py --lo 10 --hi 18
"""
import argparse
import json
import math
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "multilinear-map-cryptography_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

import twist_and_shout as ts  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lo", type=int, default=10)
    ap.add_argument("--hi", type=int, default=18)
    args = ap.parse_args()
    t_start = time.perf_counter()

    def heartbeat():  # a long build prints nothing else for minutes
        while True:
            time.sleep(30)
            print(f"[tfree_bench] running, {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    pts = []
    for k in range(args.lo, args.hi + 1):
        n = 1 << k
        pp, _ = ts.setup_params(max(2, k - 2))
        want = pp.commitment_params.srs.lagrange_points(n)
        limbs = pp.commitment_params.srs.download(n)
        cp = ts.CommitmentParams.from_g1_limbs(limbs)
        t0 = time.perf_counter()
        cp.srs.prepare_lagrange_from_powers(n)
        dt = time.perf_counter() - t0
        ok = bool(np.array_equal(cp.srs.lagrange_points(n), want))
        pts.append({"log_n": k, "s": round(dt, 4), "equals_tau_basis": ok})
        print(json.dumps(pts[-1]), file=sys.stderr, flush=True)
        del cp, pp, want, limbs
    law = lambda k: (1 << k) * k * k  # noqa: E731
    b = pts[-1]
    scale = b["s"] / law(b["log_n"])
    ratio = None
    if len(pts) > 1:
        a = pts[-2]
        ratio = round((b["s"] / a["s"]) / (law(b["log_n"]) / law(a["log_n"])), 3)
    out = {"measured": pts, "law": "t = a N log2(N)^2 (fitted to the largest size)",
           "law_check_last_two": ratio,
           "extrapolated_s": {f"2^{k}": round(scale * law(k), 1) for k in (20, 22, 24, 26)},
           "note": "EXTRAPOLATED one-time setup per (SRS, N), one GPU; the tau-derived basis takes ~58 ms at 2^24"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
