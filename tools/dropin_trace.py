"""Drop-in Twist::prove at C4 (host trace buffers through the C ABI) next to the resident prove,
repeated, with the ABI's per-phase timings: for kernel + memory-copy traces of the H2D overlap.
    rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/di -o run -- python3 tools/dropin_trace.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multilinear-map-cryptography_amd"))
import twist_and_shout as ts  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 22
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
n = 1 << (L + 2)
pp, _ = ts.setup_params(L)
ctx = pp.commitment_params.srs.ctx
pp.commitment_params.srs.prepare_lagrange(n)
addr, val, isw = ts.bench_trace(1 << L, n)
d = [ts.DeviceBuffer(ctx, x) for x in (addr, val, isw)]
tw = ts.Twist(pp)
ref = tw.prove_soa(addr, val, isw)
ts.twist_prove_resident(pp, *d, n)
for name, fn in (("resident", lambda: ts.twist_prove_resident(pp, *d, n)), ("dropin", lambda: tw.prove_soa(addr, val, isw))):
    ts_ = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts_.append((time.perf_counter() - t) * 1e3)
    print(name, " ".join("%.2f" % x for x in ts_), "ms; last phases", ctx.timing(), flush=True)
assert tw.prove_soa(addr, val, isw) == ref
