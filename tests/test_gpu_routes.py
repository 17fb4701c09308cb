"""Every benchmarked route pinned at the size it is benchmarked.

* The coefficient route -- vector_to_polynomial (src/twist.rs:151-152, src/polynomials.rs:301-352)
  + coefficient KZG over g1_powers (src/commitments.rs:162-199), the only route for an SRS without
  tau -- is timed by bench.py at C4 (2^24 ops).  Its whole Twist proof must equal the Lagrange
  route's proof at 2^20 and at 2^24 (the Lagrange route itself is pinned at those sizes by the
  trapdoor identities of test_gpu_configs.py).
* setup_params' g1_powers (src/utils.rs:89-96: g1_powers[i] = tau^i G1) at L = 22 (C4) and
  L = 24 (C5): 64 random indices plus both ends against the C oracle's double-and-add of tau^i.
  The Lagrange route never reads them, so a wrong large SRS would otherwise pass every proof test.
* The C5 shards of setup_params_shard(24, r, 8): contiguous, disjoint, covering all 2^26 + 1
  powers, and every shard's points are the same tau^i G1 (spot checks at both shard edges).
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


@pytest.mark.parametrize("logn", [20, 24])
def test_twist_coefficient_route_equals_lagrange_route(logn):
    """The bench's two routes prove the same statement: identical TwistProof (commitments,
    round polynomials, challenges, openings, final evaluations) on the ProtocolBenchmarks trace."""
    n, L = 1 << logn, logn - 2
    pp, _ = params(L)
    pp.commitment_params.srs.prepare_lagrange(n)
    addr, val, isw = ts.bench_trace(1 << L, n)
    ctx = pp.commitment_params.srs.ctx
    lag = ts.Twist(pp).prove_soa(addr, val, isw)
    ctx.set_commit_basis(False)
    try:
        coef = ts.Twist(pp).prove_soa(addr, val, isw)
        d = [ts.DeviceBuffer(ctx, x) for x in (addr, val, isw)]
        coef_resident = ts.twist_proof_from_raw(ts.twist_prove_resident(pp, *d, n))  # the bench's call
    finally:
        ctx.set_commit_basis(True)
    assert coef == lag
    assert coef_resident == lag


def _spot_indices(first, held, k, seed):
    rng = np.random.default_rng(seed)
    last = first + held - 1
    edges = {first, min(first + 1, last), last, max(first, last - 1)}
    return sorted(edges | {int(i) for i in rng.integers(first, last + 1, size=k)})


def _check_points(srs, tau, idx):
    got = srs.points_at(idx)
    for i, row in zip(idx, got):
        assert co.g1_from_limbs(row) == co.g1_mul_gen(pow(tau, int(i), R)), i


@pytest.mark.parametrize("L", [22, 24])
def test_g1_powers_spot_check_large(L):
    """setup_params(22) (C4, 2^24 + 1 points) and setup_params(24) (C5, 2^26 + 1 points):
    g1_powers[i] == tau^i G1 at 64 random indices and both ends."""
    pp, _ = ts.setup_params(L)  # not cached: the 4.3 GB C5 SRS goes with this test
    srs, tau = pp.commitment_params.srs, pp.commitment_params.tau
    assert len(srs) == (1 << (L + 2)) + 1
    assert srs.share() == (0, len(srs))
    _check_points(srs, tau, _spot_indices(0, len(srs), 64, seed=L))
    with pytest.raises(ts.InvalidParameters):
        srs.points_at([len(srs)])


def test_c5_srs_shards_partition_g1_powers():
    """setup_params_shard(24, r, 8) for r < 8 (the per-GPU SRS of bench.py --gpus 8): the shares
    are contiguous, disjoint and cover the 2^26 + 1 powers; each shard holds tau^i G1."""
    L, size = 24, 8
    n = (1 << (L + 2)) + 1
    ctx = ts.Context(0)  # private: every shard goes with it
    nxt = 0
    for r in range(size):
        pp, _ = ts.setup_params_shard(L, r, size, ctx=ctx)
        srs, tau = pp.commitment_params.srs, pp.commitment_params.tau
        assert len(srs) == n
        first, held = srs.share()
        assert first == nxt and held > 0
        nxt = first + held
        _check_points(srs, tau, _spot_indices(first, held, 8, seed=r))
        with pytest.raises(ts.InvalidParameters):
            srs.points_at([first + held])
        if first:
            with pytest.raises(ts.InvalidParameters):
                srs.points_at([first - 1])
        del pp, srs
    assert nxt == n


@pytest.mark.parametrize("big", [None, (1 << 28) + 3, (1 << 40) + 5, (1 << 24) - 1])
def test_dropin_address_narrowing(big):
    """The drop-in prover sends u64 addresses over PCIe as packed 24-bit values when every address
    is below 2^24, as u32 when one is not but all fit 32 bits, and as u64 otherwise (HostUpload
    add_narrow; widened on the device); every form equals the device-resident proof.  2^20 + 3 ops
    (8 MB of addresses: the staged path, a ragged last group of the 24-bit packing)."""
    L = 19  # max_operations 2^21: the trace pads to 2^21
    n = (1 << 20) + 3
    pp, _ = params(L)
    addr, val, isw = ts.bench_trace(1 << L, n)
    if big is not None:
        addr = addr.copy()
        addr[n // 3] = big  # past 24 bits: the u32 fallback; past 32 bits: u64; 2^24 - 1: still 24-bit
        addr[n - 1] = big
    ctx = pp.commitment_params.srs.ctx
    d = [ts.DeviceBuffer(ctx, x) for x in (addr, val, isw)]
    want = ts.twist_proof_from_raw(ts.twist_prove_resident(pp, *d, n))
    assert ts.Twist(pp).prove_soa(addr, val, isw) == want
    assert ts.twist_proof_from_raw(ts.twist_prove_host_raw(pp, addr, val, isw)) == want  # the bench's drop-in call


def test_dropin_shout_index_narrowing():
    L, T, M = 18, 1 << 20, 1 << 20
    pp, _ = params(L)
    entries = ts.fr_from_u64_array(np.arange(T, dtype=np.uint64) * 3)
    idx = (np.arange(M, dtype=np.uint64) * 7) % T
    ctx = pp.commitment_params.srs.ctx
    raw = ts.shout_prove_resident(pp, ts.DeviceBuffer(ctx, entries), T, ts.DeviceBuffer(ctx, idx), M)
    assert ts.Shout(pp).prove_arrays(entries, idx) == ts.shout_proof_from_raw(raw)
