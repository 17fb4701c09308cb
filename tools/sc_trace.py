"""Where a generic sum-check proof's time goes (2^k tables, the bench's Twist-shaped composition):
wall per call through the Python mirror vs the bare C call, and -- under rocprofv3 --kernel-trace --
the kernels of the last proof.   python3 tools/sc_trace.py [k] [reps] [noprio]
(noprio: a private context created without stream priorities)"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multilinear-map-cryptography_amd"))
import twist_and_shout as ts  # noqa: E402
from twist_and_shout import _native as N  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
R = ts.R_MOD
terms = [(1, [0, 1]), (R - 1, [2, 2, 1]), (2, [2])]
ctx = ts.Context(0, stream_priorities=False) if "noprio" in sys.argv[3:] else ts.Context.get(0)
rng = np.random.default_rng(9)
n = 1 << k
tabs = []
for _ in range(3):
    t = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64) * np.uint64(2)
    t[:, 3] &= np.uint64((1 << 60) - 1)
    tabs.append(ts.DeviceBuffer(ctx, t))
claim = ts.SumCheck.composition_sum_resident(k, tabs, terms)
sc = ts.SumCheck(k, claim)
sc.prove_resident(tabs, terms, ts.Transcript(bytes(32)), raw=True)
t0 = time.perf_counter()
for _ in range(reps):
    sc.prove_resident(tabs, terms, ts.Transcript(bytes(32)), raw=True)
py = (time.perf_counter() - t0) / reps
# the bare C call with every argument prepared once
ptrs = (C.c_void_p * 3)(*[t.ptr for t in tabs])
cl = ts.to_mont([claim])[0]
rounds = np.zeros((k, 4, 4), dtype=np.uint64)
fin = np.zeros(4, dtype=np.uint64)
ch = np.zeros((k, 4), dtype=np.uint64)
tm = sc._terms(terms)
trs = [ts.Transcript(bytes(32)) for _ in range(reps)]
lib = N.load()
t0 = time.perf_counter()
for i in range(reps):
    lib.tns_sumcheck_prove_device(ctx.handle, ptrs, 3, k, N.p64(cl), tm, len(terms), trs[i]._h, N.p64(rounds),
                                  N.p64(fin), N.p64(ch))
cc = (time.perf_counter() - t0) / reps
import hashlib  # noqa: E402

digest = hashlib.sha256(rounds.tobytes() + fin.tobytes() + ch.tobytes()).hexdigest()[:16]
print(f"2^{k}: python mirror {py * 1e3:.3f} ms per proof, bare C call {cc * 1e3:.3f} ms, proof {digest}", flush=True)
