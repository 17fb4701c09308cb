"""Root-cause run for the withdrawn fused chain inversion (df7fe42): a Twist proof at 2^k ops with
the library build in <pkgdir> (tools/df7/<variant>, built from a git worktree) against
oracle/fastcpu.c and the trapdoor identities.  python3 tools/df7_check.py <pkgdir> <k>"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.abspath(sys.argv[1]))
import twist_and_shout as ts  # noqa: E402
from oracle import coracle as co  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

k = int(sys.argv[2])
n, L = 1 << k, k - 2
pp, _ = ts.setup_params(L)
pp.commitment_params.srs.prepare_lagrange(n)
addr, val, isw = ts.bench_trace(1 << L, n)
g = ts.Twist(pp).prove_soa(addr, val, isw)
lag = pp.commitment_params.srs.lagrange_points(n)
w = co.bary_weights(n)
st, want = co.fast_twist_prove(lag, w, pp.max_operations, addr, val, isw, 16)
tau = pp.commitment_params.tau
z = g.opening_point
fa_z, fv_z, _ = co.bary_eval2(w, ts.fr_from_u64_array(addr), val, z, 16)
print(sys.argv[1], "k=%d" % k,
      "commitments", [g.address_commitment.commitment, g.value_commitment.commitment] ==
      [want["address_commitment"], want["value_commitment"]],
      "z", z == want["opening_point"],
      "values", g.final_evaluations == [fa_z, fv_z],
      "proofs", [q.proof for q in g.opening_proofs] == want["opening_proofs"], flush=True)
