"""GPU parity of the Lagrange-basis commit/open path (lagrange.hip).

Twist/Shout::prove commit to vector_to_polynomial(v) and open it (src/twist.rs:151-243,
src/shout.rs:120-211).  With the setup's tau the prover does both straight from the
evaluations through [L_j(tau)]G; these tests pin that path to the oracle's
interpolate-then-commit restatement and to the device coefficient path, including its
fallbacks (uploaded SRS without tau, tau a node, challenge z a node).
"""
import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyoracle as po

import twist_and_shout as ts

pytestmark = pytest.mark.gpu
R = po.R_MOD

_PARAMS = {}


def params(L):
    if L not in _PARAMS:
        _PARAMS[L] = ts.setup_params(L)
    return _PARAMS[L]


_G1 = {}


def g1_limbs(L):
    if L not in _G1:
        _G1[L] = co.setup_params(L)["g1_limbs"]
    return _G1[L]


def rand_vals(n, seed):
    rng = np.random.default_rng(seed)
    return [int.from_bytes(rng.bytes(32), "little") % R for _ in range(n)]


def oracle_commit_evals(L, ys):
    coeffs = co.interpolate(co.fr_array(ys))
    st, P = co.commit(g1_limbs(L), coeffs)
    assert st == 0
    return co.g1_from_limbs(P)


def oracle_open_evals(L, ys, z):
    coeffs = co.interpolate(co.fr_array(ys))
    st, v, pi = co.open_(g1_limbs(L), coeffs, co.fr_array([z]))
    assert st == 0
    return co.fr_ints(v)[0], co.g1_from_limbs(pi)


@pytest.mark.parametrize("n", [1, 2, 4, 8, 64, 256])
def test_commit_evaluations_matches_oracle(n):
    pp, _ = params(8)
    ys = rand_vals(n, seed=n)
    got = ts.KZGCommitment.commit_evaluations(pp.commitment_params, ys).commitment
    assert got == oracle_commit_evals(8, ys)


@pytest.mark.parametrize("n", [1, 2, 8, 128])
def test_open_evaluations_matches_oracle(n):
    pp, _ = params(8)
    ys = rand_vals(n, seed=100 + n)
    z = rand_vals(1, seed=7)[0]
    v, pi = ts.KZGCommitment.open_evaluations(pp.commitment_params, ys, z)
    wv, wpi = oracle_open_evals(8, ys, z)
    assert v == wv and pi.proof == wpi


@pytest.mark.parametrize("z", [0, 3, 7])
def test_open_at_a_node_falls_back_to_coefficients(z):
    pp, _ = params(8)
    ys = rand_vals(8, seed=z)
    v, pi = ts.KZGCommitment.open_evaluations(pp.commitment_params, ys, z)
    wv, wpi = oracle_open_evals(8, ys, z)
    assert v == wv == ys[z] and pi.proof == wpi


def test_open_just_outside_the_nodes():
    pp, _ = params(8)
    ys = rand_vals(16, seed=3)
    for z in (16, R - 1):
        v, pi = ts.KZGCommitment.open_evaluations(pp.commitment_params, ys, z)
        wv, wpi = oracle_open_evals(8, ys, z)
        assert v == wv and pi.proof == wpi


@pytest.mark.parametrize("logn", [12, 16, 20])
def test_lagrange_equals_coefficient_path_large(logn):
    pp, _ = params(max(8, logn - 2))
    rng = np.random.default_rng(logn)
    y = rng.integers(0, 2**63, size=(1 << logn, 4), dtype=np.uint64)
    y[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
    z = rand_vals(1, seed=logn)[0]
    cp = pp.commitment_params
    a = ts.KZGCommitment.commit_evaluations(cp, y).commitment
    va, pa = ts.KZGCommitment.open_evaluations(cp, y, z)
    ctx = ts.Context.get(0)
    ctx.set_commit_basis(False)
    try:
        b = ts.KZGCommitment.commit_evaluations(cp, y).commitment
        vb, pb = ts.KZGCommitment.open_evaluations(cp, y, z)
    finally:
        ctx.set_commit_basis(True)
    assert a == b and va == vb and pa.proof == pb.proof
    # trapdoor identity pi * (tau - z) = C - v G
    tau = cp.tau
    lhs = po.affine_mul(pa.proof, (tau - z) % R)
    rhs = po.affine_add(a, po.g1_neg(po.affine_mul(po.G1_GEN, va)))
    assert lhs == rhs


@pytest.mark.parametrize("logn", [4, 10, 14])
def test_twist_proof_identical_on_both_paths(logn):
    L = max(2, logn - 2)
    pp, _ = params(L)
    addr, val, isw = ts.bench_trace(1 << L, (1 << logn) - 3)
    a = ts.Twist(pp).prove_soa(addr, val, isw)
    ctx = ts.Context.get(0)
    ctx.set_commit_basis(False)
    try:
        b = ts.Twist(pp).prove_soa(addr, val, isw)
    finally:
        ctx.set_commit_basis(True)
    assert a == b


def test_chain_inverse_openings_match_coefficient_route():
    """The openings' batch chain inversion (k_chain_inv: one inversion per block of 256 chains,
    chains of several nodes from 2^18 on) against the coefficient route (interpolation +
    coefficient KZG, no inversion at all): Twist at 2^18 (the two-vector k_node_finish2) and Shout
    with T != M (two single-vector openings) give the same proofs."""
    pp, _ = params(17)  # SRS 2^19 + 1 points
    n = 1 << 18
    pp.commitment_params.srs.prepare_lagrange(n)
    addr, val, isw = ts.bench_trace(1 << 16, n)
    T, M = 1 << 18, 3 << 16
    rng = np.random.default_rng(5)
    entries = ts.to_mont(rand_vals(T, seed=11))
    idx = rng.integers(0, T, size=M, dtype=np.uint64)
    a = (ts.Twist(pp).prove_soa(addr, val, isw), ts.Shout(pp).prove_arrays(entries, idx))
    ctx = pp.commitment_params.srs.ctx
    ctx.set_commit_basis(False)
    try:
        b = (ts.Twist(pp).prove_soa(addr, val, isw), ts.Shout(pp).prove_arrays(entries, idx))
    finally:
        ctx.set_commit_basis(True)
    assert a == b


@pytest.mark.parametrize("T,M", [(5, 3), (64, 1000), (4096, 17)])
def test_shout_proof_identical_on_both_paths(T, M):
    pp, _ = params(10)  # SRS 4097 points
    rng = np.random.default_rng(T * 7 + M)
    entries = ts.to_mont(rand_vals(T, seed=T))
    idx = rng.integers(0, T, size=M, dtype=np.uint64)
    a = ts.Shout(pp).prove_arrays(entries, idx)
    ctx = ts.Context.get(0)
    ctx.set_commit_basis(False)
    try:
        b = ts.Shout(pp).prove_arrays(entries, idx)
    finally:
        ctx.set_commit_basis(True)
    assert a == b


def _srs_from_tau(tau, n):
    return [po.affine_mul(po.G1_GEN, pow(tau, i, R)) for i in range(n)]


def test_uploaded_srs_with_small_tau_uses_coefficients_on_nodes():
    tau = 5  # a node of every N > 5: the Lagrange basis does not exist there
    cp = ts.CommitmentParams.from_g1_powers(_srs_from_tau(tau, 17), tau=tau)
    for n in (4, 8, 16):  # 4: basis path (5 is not a node); 8, 16: coefficient path
        ys = rand_vals(n, seed=n)
        C = ts.KZGCommitment.commit_evaluations(cp, ys).commitment
        assert C == po.affine_mul(po.G1_GEN, po.barycentric_eval(ys, tau))
        z = 1234567
        v, pi = ts.KZGCommitment.open_evaluations(cp, ys, z)
        assert v == po.barycentric_eval(ys, z)
        q_tau = (po.barycentric_eval(ys, tau) - v) * po.fr_inv((tau - z) % R) % R
        assert pi.proof == po.affine_mul(po.G1_GEN, q_tau)


def test_uploaded_srs_rejects_mismatched_tau():
    # the Lagrange basis is derived from tau: a tau that is not the powers' trapdoor would
    # give silently wrong commitments, so set_tau checks g1_powers[1] == tau * G1
    with pytest.raises(ts.InvalidParameters):
        ts.CommitmentParams.from_g1_powers(_srs_from_tau(5, 8), tau=6)
    pp, _ = params(3)
    with pytest.raises(ts.InvalidParameters):
        ts.CommitmentParams.from_g1_powers(pp.commitment_params.g1_powers, tau=pp.commitment_params.tau + 1)
    cp = ts.CommitmentParams.from_g1_powers(pp.commitment_params.g1_powers, tau=pp.commitment_params.tau)
    ys = rand_vals(8, seed=3)
    assert ts.KZGCommitment.commit_evaluations(cp, ys).commitment == oracle_commit_evals(3, ys)
    # a one-point SRS (g1_powers[0] = G1 only) cannot contradict tau
    ts.CommitmentParams.from_g1_powers(_srs_from_tau(5, 1), tau=6)


def test_uploaded_srs_without_tau_matches_setup_srs():
    pp, _ = params(3)
    pts = pp.commitment_params.g1_powers
    cp = ts.CommitmentParams.from_g1_powers(pts)  # no tau: interpolation path
    ys = rand_vals(16, seed=11)
    a = ts.KZGCommitment.commit_evaluations(cp, ys).commitment
    b = ts.KZGCommitment.commit_evaluations(pp.commitment_params, ys).commitment
    assert a == b == oracle_commit_evals(3, ys)


def test_prepare_lagrange_errors():
    pp, _ = params(3)
    with pytest.raises(ts.InvalidParameters):
        pp.commitment_params.srs.prepare_lagrange(3)
    cp = ts.CommitmentParams.from_g1_powers(pp.commitment_params.g1_powers)
    with pytest.raises(ts.InvalidParameters):
        cp.srs.prepare_lagrange(8)
    pp.commitment_params.srs.prepare_lagrange(16)


def test_non_power_of_two_needs_tau_basis():
    pp, _ = params(3)
    ys = [1, 2, 3]
    got = ts.KZGCommitment.commit_evaluations(pp.commitment_params, ys).commitment
    assert got == po.affine_mul(po.G1_GEN, po.barycentric_eval(ys, pp.commitment_params.tau))
    cp = ts.CommitmentParams.from_g1_powers(pp.commitment_params.g1_powers)  # no tau: interpolation only
    with pytest.raises(ts.PolynomialError):
        ts.KZGCommitment.commit_evaluations(cp, ys)
