"""C2 (2^20-scalar KZG MSM over setup_params(18)) in three orders of setup work -- does the time
depend on what was allocated before the SRS window table (built lazily at the first MSM)?
    python3 tools/c2_alloc.py {none|lagrange_first|table_first}"""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multilinear-map-cryptography_amd"))
import twist_and_shout as ts  # noqa: E402

mode = sys.argv[1]
ctx = ts.Context.get(0)
n = 1 << 20
pp18, _ = ts.setup_params(18)
sc = ts.DeviceBuffer(ctx, ts.fr_rand_batch(bytes([7] * 32), n))
if mode == "lagrange_first":
    pp18.commitment_params.srs.prepare_lagrange(n)
ts.msm_resident(pp18.commitment_params, sc, n)  # builds the SRS window table
if mode == "table_first":
    pp18.commitment_params.srs.prepare_lagrange(n)
t = time.perf_counter()
for _ in range(20):
    ts.msm_resident(pp18.commitment_params, sc, n)
dt = (time.perf_counter() - t) / 20
print(json.dumps({"mode": mode, "contig": os.environ.get("TNS_TABLE_CONTIG"), "msm_ms_2^20": round(dt * 1e3, 3)}), flush=True)
