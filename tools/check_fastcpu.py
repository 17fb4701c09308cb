"""GPU Twist proof vs oracle/fastcpu.c at 2^k ops (setup_params(k-2)), field by field:
    python3 tools/check_fastcpu.py 20"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "multilinear-map-cryptography_amd"))
sys.path.insert(0, ROOT)
import twist_and_shout as ts  # noqa: E402
from oracle import coracle as co  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 1 << k
L = k - 2
pp, _ = ts.setup_params(L)
pp.commitment_params.srs.prepare_lagrange(n)
addr, val, isw = ts.bench_trace(1 << L, n)
lag = pp.commitment_params.srs.lagrange_points(n)
w = co.bary_weights(n)
st, proof = co.fast_twist_prove(lag, w, pp.max_operations, addr, val, isw, 16)
g = ts.Twist(pp).prove_soa(addr, val, isw)
print("address_commitment", g.address_commitment.commitment == proof["address_commitment"])
print("value_commitment", g.value_commitment.commitment == proof["value_commitment"])
print("opening_point", g.opening_point == proof["opening_point"])
for j, q in enumerate(g.opening_proofs):
    print("opening_proof", j, q.proof == proof["opening_proofs"][j])
if "final_evaluations" in proof:
    print("final_evaluations", g.final_evaluations == proof["final_evaluations"])
