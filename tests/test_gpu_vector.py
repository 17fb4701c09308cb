"""KZGVectorCommitment (src/commitments.rs:408-483) on the device: commit to
the interpolant of a vector of any length through the Lagrange basis, open at an index (a
node: value = the entry, quotient values via the barycentric derivative), verify with the
pairing.  Pinned to the oracle's interpolate-then-KZG restatement (small n) and to the
trapdoor identities C = f(tau) G, pi (tau - i) = C - v G (larger n)."""
import numpy as np
import pytest

from oracle import pyoracle as po

import twist_and_shout as ts

pytestmark = pytest.mark.gpu
R = po.R_MOD

_P = {}


def params(L):
    if L not in _P:
        _P[L] = ts.setup_params(L)
    return _P[L]


def rand_vals(n, seed):
    rng = np.random.default_rng(seed)
    return [int.from_bytes(rng.bytes(32), "little") % R for _ in range(n)]


@pytest.mark.parametrize("n", [1, 2, 3, 5, 17, 40])
def test_vector_commit_open_matches_oracle(n):
    pp, vp = params(6)
    cp = pp.commitment_params
    vec = rand_vals(n, seed=n)
    C = ts.KZGVectorCommitment.commit(cp, vec)
    poly = po.lagrange_interpolate([(i, v) for i, v in enumerate(vec)])
    g1 = cp.g1_powers
    assert C.commitment == po.kzg_commit(g1, poly)
    for idx in sorted({0, n - 1, n // 2}):
        v, pi = ts.KZGVectorCommitment.open(cp, vec, idx)
        wv, wpi = po.kzg_open(g1, poly, idx)
        assert v == vec[idx] == wv and pi.proof == wpi
        assert ts.KZGVectorCommitment.verify(vp.commitment_vk, C, idx, v, pi)
        assert not ts.KZGVectorCommitment.verify(vp.commitment_vk, C, idx, (v + 1) % R, pi)


@pytest.mark.parametrize("n", [1000, 4097, 1 << 16])
def test_vector_commit_open_trapdoor_large(n):
    pp, vp = params(15)
    cp = pp.commitment_params
    tau = cp.tau
    vec = rand_vals(n, seed=n)
    C = ts.KZGVectorCommitment.commit(cp, vec).commitment
    assert C == po.affine_mul(po.G1_GEN, po.barycentric_eval(vec, tau))
    for idx in (0, n // 3, n - 1):
        v, pi = ts.KZGVectorCommitment.open(cp, vec, idx)
        assert v == vec[idx]
        lhs = po.affine_mul(pi.proof, (tau - idx) % R)
        rhs = po.affine_add(C, po.g1_neg(po.affine_mul(po.G1_GEN, v))) if v else C
        assert lhs == rhs


def test_vector_open_index_out_of_bounds():
    pp, _ = params(4)
    with pytest.raises(ts.CommitmentError):
        ts.KZGVectorCommitment.open(pp.commitment_params, [1, 2, 3], 3)
