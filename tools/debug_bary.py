"""Debug: Lagrange commit (trapdoor) and single-vector opening value (barycentric) at 2^k."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "multilinear-map-cryptography_amd"))
sys.path.insert(0, ROOT)
import twist_and_shout as ts  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

k = int(sys.argv[1])
n = 1 << k
pp, _ = ts.setup_params(k - 2)
cp = pp.commitment_params
cp.srs.prepare_lagrange(n)
rng = np.random.default_rng(5)
ys = [int(x) for x in rng.integers(0, 1 << 60, size=n)]
y = ts.to_mont(ys)
C = ts.KZGCommitment.commit_evaluations(cp, y).commitment
tau = cp.tau
print("commit trapdoor", C == po.affine_mul(po.G1_GEN, po.barycentric_eval(ys, tau)))
z = 0xABCDEF12345 * 7 + (1 << 200)
v, pi = ts.KZGCommitment.open_evaluations(cp, y, z)
print("open value", v == po.barycentric_eval(ys, z))
# the Twist pair path (k_node_finish2)
L = k - 2
addr, val, isw = ts.bench_trace(1 << L, n)
g = ts.Twist(pp).prove_soa(addr, val, isw)
zt = g.opening_point
va = po.barycentric_eval([int(a) for a in addr], zt)
vv = po.barycentric_eval(ts.from_mont(val) if hasattr(ts, "from_mont") else [], zt)
print("twist final_evaluations[0]", g.final_evaluations[0] == va)
print("twist final_evaluations[1]", g.final_evaluations[1] == vv)
pa, pv = ts.to_mont([int(a) for a in addr]), val
v2a, _ = ts.KZGCommitment.open_evaluations(cp, pa, zt)
v2v, _ = ts.KZGCommitment.open_evaluations(cp, pv, zt)
print("single-open addr / val", v2a == va, v2v == vv)
