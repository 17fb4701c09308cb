"""The generic sum-check extra of bench.py alone (SumCheck::prove of the Twist-shaped degree-3
composition over three resident 2^k tables):  python3 tools/sc_bench.py 20,24"""
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multilinear-map-cryptography_amd"))
import bench  # noqa: E402
import twist_and_shout as ts  # noqa: E402

logs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "20,24").split(",")]
ctx = ts.Context.get(0)
print(json.dumps(bench.sumcheck_generic(ts, ctx, logs)), flush=True)
