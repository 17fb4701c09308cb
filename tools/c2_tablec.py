"""C2 (MSM of 2^20 Fr::rand scalars over setup_params(18)) per fixed-base table window:
    python3 tools/c2_tablec.py 20 19 18 17 16
Each c builds a fresh SRS + window table with TNS_TABLE_C=c; prints ms per MSM (host-timed, like bench.py)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multilinear-map-cryptography_amd"))
import twist_and_shout as ts  # noqa: E402

n = 1 << 20
ctx = ts.Context.get(0)
sc = ts.DeviceBuffer(ctx, ts.fr_rand_batch(bytes([7] * 32), n))
ref = None
for c in sys.argv[1:]:
    os.environ["TNS_TABLE_C"] = c
    pp, _ = ts.setup_params(18)
    out = ts.msm_resident(pp.commitment_params, sc, n)
    if ref is None:
        ref = out
    assert (out == ref).all()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(10):
            ts.msm_resident(pp.commitment_params, sc, n)
        best = min(best, (time.perf_counter() - t) / 10)
    print(f"TNS_TABLE_C={c}: {best * 1e3:.3f} ms  {n / best / 1e6:.1f} M pairs/s", flush=True)
    del pp
