"""bench.py's C2 and C3 extras alone (setup_params(18) + its 2^20 Lagrange basis, as the bench
prepares them): KZG MSM of 2^20 Fr::rand scalars ([7;32]) and Shout::prove of the 2^20 squares
table with 2^20 lookups; one JSON line.
    python3 tools/c2c3_bench.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multilinear-map-cryptography_amd"))
import twist_and_shout as ts  # noqa: E402


def timed(fn, reps, warm=1):
    for _ in range(warm):
        fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps


ctx = ts.Context.get(0)
n = 1 << 20
pp18, _ = ts.setup_params(18)
pp18.commitment_params.srs.prepare_lagrange(n)
sc = ts.DeviceBuffer(ctx, ts.fr_rand_batch(bytes([7] * 32), n))
out = {}
ref = ts.msm_resident(pp18.commitment_params, sc, n)
out["msm_ms_2^20"] = round(timed(lambda: ts.msm_resident(pp18.commitment_params, sc, n), 20) * 1e3, 3)
out["msm_commitment_hash"] = int(ref[0] ^ ref[4])
T = 1 << 20
entries = ts.fr_from_u64_array(np.arange(T, dtype=np.uint64) ** 2)
d_e, d_i = ts.DeviceBuffer(ctx, entries), ts.DeviceBuffer(ctx, np.arange(T, dtype=np.uint64))
out["shout_ms_2^20"] = round(timed(lambda: ts.shout_prove_resident(pp18, d_e, T, d_i, T), 10) * 1e3, 3)
print(json.dumps(out), flush=True)
