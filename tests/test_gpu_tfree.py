"""The Lagrange basis from g1_powers alone (tns_srs_prepare_lagrange_from_powers, tfree.hip): an
SRS without tau (src/utils.rs:61, :107 mark tau test-only; commit/open read only g1_powers,
src/commitments.rs:162-199) gets the same basis [L_j(tau)]G, j < N, as the tau-derived one
(lagrange.hip, itself pinned by test_gpu_lagrange.py / test_gpu_configs.py), and the provers then
take the Lagrange route on it with identical proofs."""
import dataclasses

import numpy as np
import pytest

import twist_and_shout as ts

pytestmark = pytest.mark.gpu

_PARAMS = {}


def params(L):
    if L not in _PARAMS:
        _PARAMS[L] = ts.setup_params(L)
    return _PARAMS[L]


def tau_free(pp, n_points):
    """The same g1_powers[0..n_points) uploaded WITHOUT tau."""
    limbs = pp.commitment_params.srs.download(n_points)
    return ts.CommitmentParams.from_g1_limbs(limbs)


@pytest.mark.parametrize("logn", [0, 1, 2, 3, 4, 5, 6, 8, 10, 12])
def test_basis_from_powers_equals_tau_basis(logn):
    n = 1 << logn
    pp, _ = params(max(2, logn))  # SRS of 4 * 2^L + 1 >= n points
    want = pp.commitment_params.srs.lagrange_points(n)
    cp = tau_free(pp, len(pp.commitment_params.srs))
    with pytest.raises(ts.InvalidParameters):  # no tau, nothing prepared yet
        cp.srs.lagrange_points(n)
    cp.srs.prepare_lagrange_from_powers(n)
    got = cp.srs.lagrange_points(n)
    assert np.array_equal(got, want)


def test_basis_from_powers_2e14_and_proofs():
    """2^14 nodes, then Twist::prove of a 2^14-op trace on the tau-less SRS: the same proof as on the
    setup SRS (both through the Lagrange route) and as the coefficient route."""
    logn, L = 14, 12
    n = 1 << logn
    pp, _ = params(L)
    cp = tau_free(pp, len(pp.commitment_params.srs))
    cp.srs.prepare_lagrange_from_powers(n)
    assert np.array_equal(cp.srs.lagrange_points(n), pp.commitment_params.srs.lagrange_points(n))
    pp_free = dataclasses.replace(pp, commitment_params=cp, _raw=None)
    addr, val, isw = ts.bench_trace(1 << L, n)
    want = ts.Twist(pp).prove_soa(addr, val, isw)
    assert ts.Twist(pp_free).prove_soa(addr, val, isw) == want
    ctx = cp.srs.ctx
    ctx.set_commit_basis(False)
    try:
        assert ts.Twist(pp_free).prove_soa(addr, val, isw) == want
    finally:
        ctx.set_commit_basis(True)


def test_basis_from_powers_errors():
    pp, _ = params(3)
    cp = tau_free(pp, 8)
    with pytest.raises(ts.InvalidParameters):
        cp.srs.prepare_lagrange_from_powers(16)  # more nodes than held powers
    with pytest.raises(ts.InvalidParameters):
        cp.srs.prepare_lagrange_from_powers(6)  # not a power of two
