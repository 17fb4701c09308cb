"""C2 (KZG MSM of 2^20 Fr::rand scalars, setup_params(18)) timed in a fresh process, then again after
the C4 work the bench does before it (resident proofs, drop-in proofs, coefficient-route proofs):
does the bench's C2 figure depend on what ran before it in the process?
    python3 tools/c2_state.py"""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multilinear-map-cryptography_amd"))
import twist_and_shout as ts  # noqa: E402

ctx = ts.Context.get(0)
n = 1 << 20
pp18, _ = ts.setup_params(18)
pp18.commitment_params.srs.prepare_lagrange(n)
sc = ts.DeviceBuffer(ctx, ts.fr_rand_batch(bytes([7] * 32), n))


def c2(tag, reps=10):
    ts.msm_resident(pp18.commitment_params, sc, n)
    t = time.perf_counter()
    for _ in range(reps):
        ts.msm_resident(pp18.commitment_params, sc, n)
    dt = (time.perf_counter() - t) / reps
    print(json.dumps({"after": tag, "msm_ms_2^20": round(dt * 1e3, 3)}), flush=True)


c2("fresh process")
pp, _ = ts.setup_params(22)
N = 1 << 24
pp.commitment_params.srs.prepare_lagrange(N)
addr, val, isw = ts.bench_trace(1 << 22, N)
d = [ts.DeviceBuffer(ctx, x) for x in (addr, val, isw)]
for _ in range(5):
    ts.twist_prove_resident(pp, d[0], d[1], d[2], N)
c2("5 resident C4 proofs")
for _ in range(3):
    ts.twist_prove_host_raw(pp, addr, val, isw)
c2("3 drop-in C4 proofs")
ctx.set_commit_basis(False)
ts.twist_prove_resident(pp, d[0], d[1], d[2], N)
ctx.set_commit_basis(True)
c2("1 coefficient-route C4 proof")
c2("again")
