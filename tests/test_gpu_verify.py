"""prove -> verify on the MI355X prover (the loop of the reference's integration tests,
tests/integration_tests.rs:37, :74, tests/shout_tests.rs): GPU proofs must pass the host
verifier (BN254 pairing checks), sharded proofs included; tampered ones must not."""
import numpy as np
import pytest

import twist_and_shout as ts

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("logn", [1, 6, 12])
def test_twist_prove_then_verify(logn):
    L = max(1, logn - 2)
    pp, vp = ts.setup_params(L)
    addr, val, isw = ts.bench_trace(1 << L, (1 << logn) - 1)
    proof = ts.Twist(pp).prove_soa(addr, val, isw)
    assert ts.Twist.verify(proof, vp)
    if proof.final_evaluations:  # a 1-op trace has no openings
        proof.final_evaluations[1] = (proof.final_evaluations[1] + 1) % ts.R_MOD
        assert not ts.Twist.verify(proof, vp)


def test_shout_prove_then_verify():
    pp, vp = ts.setup_params(10)
    rng = np.random.default_rng(5)
    t = ts.LookupTable([int(x) for x in rng.integers(0, 2**60, size=300)])
    for i in rng.integers(0, 300, size=777):
        t.lookup(int(i))
    proof = ts.Shout(pp).prove(t)
    assert ts.Shout.verify(proof, vp)


def test_coefficient_route_proof_verifies():
    pp, vp = ts.setup_params(6)
    ctx = ts.Context.get(0)
    addr, val, isw = ts.bench_trace(64, 200)
    ctx.set_commit_basis(False)
    try:
        proof = ts.Twist(pp).prove_soa(addr, val, isw)
    finally:
        ctx.set_commit_basis(True)
    assert ts.Twist.verify(proof, vp)
