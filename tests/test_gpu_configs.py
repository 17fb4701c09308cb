"""BASELINE's configurations at their full sizes on the GPU, checked independently of the
device's own setup artefacts.

C4 (Twist::prove, 2^24 ops, setup_params(22)) and C3 (Shout::prove, 2^20-entry squares table,
2^20 lookups i % 2^20, setup_params(18); src/benchmarks.rs:88-99, :167-177) are too large for
the reference-algorithm oracle, so the proofs are pinned by size-independent identities that
use nothing the GPU computed except the proof itself:

* commitments: C = f(tau) G, with f(tau) the barycentric evaluation of the padded vector at the
  setup's tau (CommitmentParams.tau, src/utils.rs:84, :107) -- O(N) in the C oracle
  (oracle/fastcpu.c fc_bary_eval2), G f(tau) by the oracle's double-and-add;
* transcript: the Fiat-Shamir replay of src/twist.rs:170-219 / src/shout.rs:140-190 in the Python
  oracle (zero round polynomials, challenges, opening point z);
* openings: v = f(z) (same barycentric evaluation) and pi (tau - z) = C - v G
  (src/commitments.rs:201-228 without the pairing);
* the device Lagrange basis itself: 64 points Lambda_j = L_j(tau) G, L_j(tau) = ell(tau) w_j / (tau - j).
The device-resident entry points (the bench's path) must return the same proof as the host ones.
C5 (one 2^26-op proof sharded over 8 ranks) is in test_gpu_sharded.py.
"""
import os

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


def host_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(64, n))


def replay(seed, labels, C0, C1, nv):
    """Sum-check challenges and the opening point of a zero-closure proof (src/twist.rs:170-219)."""
    t = po.Transcript(seed)
    t.append_field_element(labels[0], po.commitment_hash(C0))
    t.append_field_element(labels[1], po.commitment_hash(C1))
    chals = []
    for r in range(nv):
        t.append_field_elements(b"sumcheck_round_%d" % r, [0, 0, 0, 0])
        chals.append(t.challenge_field_element(b"sumcheck_challenge_%d" % r))
    return chals, t.challenge_field_element(b"opening_challenges_0")


def check_pair(tau, n, y0, y1, commitments, z, values, proofs):
    """Both commitments and both openings of a proof against the trapdoor identities; returns the
    barycentric weights and ell(tau) for the basis spot check."""
    w = co.bary_weights(n)
    T = host_threads()
    f0t, f1t, ell_t = co.bary_eval2(w, y0, y1, tau, T)
    assert commitments[0] == co.g1_mul_gen(f0t)
    assert commitments[1] == co.g1_mul_gen(f1t)
    f0z, f1z, _ = co.bary_eval2(w, y0, y1, z, T)
    assert list(values) == [f0z, f1z]
    for C, v, pi in zip(commitments, values, proofs):
        assert co.g1_mul(pi, (tau - z) % R) == po.affine_add(C, po.g1_neg(co.g1_mul_gen(v)))
    return w, ell_t


def spot_check_basis(pp, n, w, ell_t, k=64, seed=0):
    tau = pp.commitment_params.tau
    lag = pp.commitment_params.srs.lagrange_points(n)
    rng = np.random.default_rng(seed)
    js = sorted({0, 1, n - 1, *(int(j) for j in rng.integers(0, n, size=k - 3))})
    wj = co.fr_ints(w[js])
    for j, wv in zip(js, wj):
        Lj = ell_t * wv % R * pow((tau - j) % R, -1, R) % R
        assert co.g1_from_limbs(lag[j]) == co.g1_mul_gen(Lj), j


@pytest.mark.parametrize("logn", [18, 20, 24])
def test_twist_full_size_trapdoor(logn):
    """Twist::prove of the ProtocolBenchmarks trace at 2^18, 2^20 and 2^24 operations (C4);
    from 2^18 nodes the barycentric batch inversion runs chains of >= 2 nodes."""
    n = 1 << logn
    L = logn - 2
    pp, _ = params(L)
    pp.commitment_params.srs.prepare_lagrange(n)
    addr, val, isw = ts.bench_trace(1 << L, n)
    g = ts.Twist(pp).prove_soa(addr, val, isw)
    ctx = pp.commitment_params.srs.ctx
    d = [ts.DeviceBuffer(ctx, x) for x in (addr, val, isw)]
    assert ts.twist_proof_from_raw(ts.twist_prove_resident(pp, *d, n)) == g
    Ca, Cv = g.address_commitment.commitment, g.value_commitment.commitment
    chals, z = replay(pp.fiat_shamir_seed, (b"address_commitment", b"value_commitment"), Ca, Cv, logn)
    assert g.consistency_proof.round_polynomials == [[0, 0, 0, 0]] * logn
    assert g.consistency_proof.final_evaluation == 0
    assert g.sumcheck_challenges == chals and g.opening_point == z
    tau = pp.commitment_params.tau
    w, ell_t = check_pair(tau, n, ts.fr_from_u64_array(addr), val, (Ca, Cv), z, g.final_evaluations,
                          [p.proof for p in g.opening_proofs])
    spot_check_basis(pp, n, w, ell_t, seed=logn)
    if logn <= 20:  # and the fast-CPU restatement (oracle/fastcpu.c) on the same basis
        st, want = co.fast_twist_prove(pp.commitment_params.srs.lagrange_points(n), w, pp.max_operations, addr,
                                       val, isw, host_threads())
        assert st == 0
        assert [Ca, Cv] == [want["address_commitment"], want["value_commitment"]]
        assert [q.proof for q in g.opening_proofs] == want["opening_proofs"]
        assert g.final_evaluations == want["final_evaluations"]


def test_shout_c3_full_size_trapdoor():
    """C3: Shout::prove over the 2^20-entry table of squares with 2^20 lookups i % 2^20
    (src/benchmarks.rs:167-177), setup_params(18)."""
    L, T, M = 18, 1 << 20, 1 << 20
    pp, _ = params(L)
    entries = ts.fr_from_u64_array(np.arange(T, dtype=np.uint64) ** 2)
    idx = np.arange(M, dtype=np.uint64) % T
    g = ts.Shout(pp).prove_arrays(entries, idx)
    ctx = pp.commitment_params.srs.ctx
    raw = ts.shout_prove_resident(pp, ts.DeviceBuffer(ctx, entries), T, ts.DeviceBuffer(ctx, idx), M)
    assert ts.shout_proof_from_raw(raw) == g
    Ct, Ci = g.table_commitment.commitment, g.index_commitment.commitment
    chals, z = replay(pp.fiat_shamir_seed, (b"table_commitment", b"index_commitment"), Ct, Ci, 20)
    assert g.lookup_proof.round_polynomials == [[0, 0, 0, 0]] * 20
    assert g.sumcheck_challenges == chals and g.opening_point == z
    w, ell_t = check_pair(pp.commitment_params.tau, T, entries, ts.fr_from_u64_array(idx), (Ct, Ci), z,
                          g.final_evaluations, [p.proof for p in g.opening_proofs])
    spot_check_basis(pp, T, w, ell_t, seed=3)


def test_twist_shout_msm_tables_off_same_proof():
    """MSMs without the window tables (tns_ctx_set_msm_tables(0): per-window buckets, no
    precomputation, as the reference's commit, /root/reference/src/commitments.rs:173-177) give
    the same Twist and Shout proofs as the shared-bucket table plans."""
    L = 14
    pp, _ = params(L)
    addr, val, isw = ts.bench_trace(1 << L, 1 << (L + 2))
    entries = ts.to_mont([i * i for i in range(5000)])
    idx = (np.arange(3 << 12, dtype=np.uint64) * 7) % 5000
    a = ts.Twist(pp).prove_soa(addr, val, isw)
    s_tab = ts.Shout(pp).prove_arrays(entries, idx)
    ctx = pp.commitment_params.srs.ctx
    ctx.set_msm_tables(False)
    try:
        b = ts.Twist(pp).prove_soa(addr, val, isw)
        s_plain = ts.Shout(pp).prove_arrays(entries, idx)
    finally:
        ctx.set_msm_tables(True)
    assert a == b
    assert s_tab == s_plain


@pytest.mark.parametrize("chunks", [1, 3, 4, 7])
def test_twist_dropin_chunked_value_commitment(chunks):
    """The drop-in prover commits the value vector chunk by chunk as its upload lands
    (tns_ctx_set_upload_chunks node ranges; one MSM each, summed): full-width values take the
    window-table plan at each chunk's offset, the bench trace's narrow values the per-window plan;
    both equal the device-resident proof (one MSM over the whole vector)."""
    L = 16
    pp, _ = params(L)
    n = 1 << (L + 2)
    addr, val, isw = ts.bench_trace(1 << L, n)
    rng = np.random.default_rng(11)
    wide = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64) * 2 + rng.integers(0, 2, size=(n, 4), dtype=np.uint64)
    wide[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
    ctx = pp.commitment_params.srs.ctx
    ctx.set_upload_chunks(chunks)
    try:
        for v in (val, wide):
            d = [ts.DeviceBuffer(ctx, x) for x in (addr, v, isw)]
            want = ts.twist_proof_from_raw(ts.twist_prove_resident(pp, *d, n))
            assert ts.Twist(pp).prove_soa(addr, v, isw) == want
    finally:
        ctx.set_upload_chunks(4)


def test_upload_chunks_out_of_range():
    pp, _ = params(10)
    ctx = pp.commitment_params.srs.ctx
    for bad in (0, -1, 65):
        with pytest.raises(ts.InvalidParameters):
            ctx.set_upload_chunks(bad)


def test_context_without_stream_priorities_same_proofs():
    """tns_ctx_create_ex(TNS_CTX_NO_STREAM_PRIORITIES) (processes sharing a GPU): a private context
    with every stream at the default priority gives the same resident and drop-in Twist proofs and
    Shout proofs as the default context (the pair accumulations' stream priority only changes the
    order blocks dispatch in)."""
    L = 14
    pp, _ = params(L)
    n = 1 << (L + 2)
    addr, val, isw = ts.bench_trace(1 << L, n)
    entries = ts.to_mont([i * i for i in range(1 << 10)])
    idx = (np.arange(1 << 12, dtype=np.uint64) * 7) % (1 << 10)
    want = ts.Twist(pp).prove_soa(addr, val, isw)
    want_s = ts.Shout(pp).prove_arrays(entries, idx)
    ctx = ts.Context(0, stream_priorities=False)
    assert not ctx.stream_priorities
    pq, _ = ts.setup_params_shard(L, 0, 1, ctx=ctx)
    d = [ts.DeviceBuffer(ctx, x) for x in (addr, val, isw)]
    assert ts.twist_proof_from_raw(ts.twist_prove_resident(pq, *d, n)) == want
    assert ts.Twist(pq).prove_soa(addr, val, isw) == want
    assert ts.Shout(pq).prove_arrays(entries, idx) == want_s
