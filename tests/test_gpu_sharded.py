"""One Twist / Shout proof sharded over ranks (BASELINE C5) on one MI355X.

The ranks are threads, each with its own tns context, SRS shard (setup_params_shard) and
slice of the trace; the allgather runs through the host-callback communicator, so the
exchange protocol of the multi-GPU prover (partial MSM sums, barycentric partials, folded
table values) is exercised end to end.  Every rank must return exactly the unsharded proof.
The RCCL transport is covered with one rank (more need more GPUs).
"""
import threading

import numpy as np
import pytest

import twist_and_shout as ts

pytestmark = pytest.mark.gpu

_PARAMS = {}


def params(L):
    """The unsharded ProverParams for setup_params(L)."""
    if L not in _PARAMS:
        _PARAMS[L] = ts.setup_params(L)[0]
    return _PARAMS[L]


class ThreadGather:
    def __init__(self, size):
        self.size = size
        self.bar = threading.Barrier(size, timeout=120)
        self.slots = [None] * size

    def fn(self, rank):
        def f(data):
            self.slots[rank] = data
            self.bar.wait()
            out = b"".join(self.slots)
            self.bar.wait()
            return out
        return f


def run_ranks(size, body):
    g = ThreadGather(size)
    results, errors = [None] * size, [None] * size

    def worker(r):
        try:
            comm = ts.Comm.from_allgather(r, size, g.fn(r))
            results[r] = body(r, comm, ts.Context(0))
        except BaseException as e:  # noqa: BLE001 -- surfaced below
            errors[r] = e
            g.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(size)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    return results, errors


def sharded_twist(L, size, addr, val, isw):
    n_total = len(addr)

    def body(r, comm, ctx):
        pp, _ = ts.setup_params_shard(L, r, size, ctx=ctx)
        first, count = ts.shard_slice(n_total, r, size)
        return ts.Twist(pp).prove_sharded(comm, addr[first:first + count], val[first:first + count],
                                          isw[first:first + count], n_total)
    return run_ranks(size, body)


@pytest.mark.parametrize("logn,size", [(3, 2), (3, 8), (4, 4), (10, 2), (10, 4), (12, 8), (14, 2)])
def test_twist_sharded_equals_unsharded(logn, size):
    L = max(1, logn - 2)
    addr, val, isw = ts.bench_trace(1 << L, 1 << logn)
    want = ts.Twist(params(L)).prove_soa(addr, val, isw)
    got, errs = sharded_twist(L, size, addr, val, isw)
    assert errs == [None] * size
    for p in got:
        assert p == want


@pytest.mark.parametrize("n_total,size", [(1000, 4), (513, 2), (5, 4)])
def test_twist_sharded_ragged_trace(n_total, size):
    L = max(1, (n_total - 1).bit_length() - 2 + 1)
    addr, val, isw = ts.bench_trace(1 << max(1, L - 1), n_total)
    want = ts.Twist(params(L)).prove_soa(addr, val, isw)
    got, errs = sharded_twist(L, size, addr, val, isw)
    assert errs == [None] * size
    assert all(p == want for p in got)


def test_bench_trace_slices_concatenate():
    a, v, w = ts.bench_trace(1 << 6, 3000)
    parts = [ts.bench_trace_slice(1 << 6, 3000, f, c) for f, c in ((0, 1000), (1000, 1500), (2500, 500))]
    assert np.array_equal(np.concatenate([p[0] for p in parts]), a)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), v)
    assert np.array_equal(np.concatenate([p[2] for p in parts]), w)


@pytest.mark.parametrize("T,M,size", [(8, 8, 2), (5, 3, 2), (64, 1000, 4), (4096, 17, 8), (1000, 4096, 4)])
def test_shout_sharded_equals_unsharded(T, M, size):
    L = 10
    rng = np.random.default_rng(T + 7 * M)
    entries = ts.to_mont([int(x) for x in rng.integers(0, 2**62, size=T)])
    idx = rng.integers(0, T, size=M, dtype=np.uint64)
    want = ts.Shout(params(L)).prove_arrays(entries, idx)

    def body(r, comm, ctx):
        pp, _ = ts.setup_params_shard(L, r, size, ctx=ctx)
        fe, ce = ts.shard_slice(T, r, size)
        fi, ci = ts.shard_slice(M, r, size)
        return ts.Shout(pp).prove_sharded(comm, entries[fe:fe + ce], T, idx[fi:fi + ci], M)
    got, errs = run_ranks(size, body)
    assert errs == [None] * size
    assert all(p == want for p in got)


def test_shout_sharded_bad_index_fails_on_every_rank():
    L, T, M, size = 6, 16, 16, 2
    entries = ts.to_mont(list(range(T)))
    idx = np.arange(M, dtype=np.uint64)
    idx[3] = T  # out of bounds, held by rank 0 only

    def body(r, comm, ctx):
        pp, _ = ts.setup_params_shard(L, r, size, ctx=ctx)
        fe, ce = ts.shard_slice(T, r, size)
        fi, ci = ts.shard_slice(M, r, size)
        return ts.Shout(pp).prove_sharded(comm, entries[fe:fe + ce], T, idx[fi:fi + ci], M)
    _, errs = run_ranks(size, body)
    assert all(isinstance(e, ts.InvalidParameters) for e in errs)


def test_sharded_shape_errors():
    L = 4
    addr, val, isw = ts.bench_trace(16, 64)

    def wrong_count(r, comm, ctx):
        pp, _ = ts.setup_params_shard(L, r, 2, ctx=ctx)
        return ts.Twist(pp).prove_sharded(comm, addr[:10], val[:10], isw[:10], 64)
    _, errs = run_ranks(2, wrong_count)
    assert all(isinstance(e, ts.InvalidParameters) for e in errs)

    def three_ranks(r, comm, ctx):
        pp, _ = ts.setup_params_shard(L, r, 3, ctx=ctx)
        return ts.Twist(pp).prove_sharded(comm, addr[:22], val[:22], isw[:22], 64)
    _, errs = run_ranks(3, three_ranks)
    assert all(isinstance(e, ts.InvalidParameters) for e in errs)


def test_setup_params_shard_splits_the_srs():
    L, size = 3, 4
    full = params(L).commitment_params.g1_powers  # 33 points
    got = []
    for r in range(size):
        pp, _ = ts.setup_params_shard(L, r, size)
        assert len(pp.commitment_params.srs) == len(full)
        assert pp.commitment_params.tau == params(L).commitment_params.tau
        got.append(pp)
    # shards are disjoint and cover g1_powers (downloads are only allowed on the rank-0 shard)
    first = got[0].commitment_params.srs
    pts = first.download(8)
    assert [(ts.from_mont(pts[i:i + 1, :4], ts.P_MOD)[0], ts.from_mont(pts[i:i + 1, 4:], ts.P_MOD)[0])
            for i in range(8)] == full[:8]


@pytest.mark.parametrize("L,n_total,size", [(18, 1 << 20, 2), (18, 1 << 20, 8), (10, 3000, 4), (6, 200, 8)])
def test_msm_sharded_equals_unsharded(L, n_total, size):
    """The C2 MSM at N ranks (tns_msm_sharded): each rank commits its coefficient slice against its
    own SRS share (setup_params_shard), the 96-byte partials are allgathered; every rank returns
    the unsharded KZGCommitment::commit (src/commitments.rs:162-180)."""
    sc = ts.fr_rand_batch(bytes([7] * 32), n_total)
    sc[5] = 0  # a zero scalar and a ragged tail
    pp = params(L)
    want = ts.msm_resident(pp.commitment_params, ts.DeviceBuffer(pp.commitment_params.srs.ctx, sc), n_total)

    def body(r, comm, ctx):
        sp, _ = ts.setup_params_shard(L, r, size, ctx=ctx)
        first, count = ts.shard_slice(n_total, r, size)
        held_first, held = sp.commitment_params.srs.share()
        assert held_first <= first and first + count <= held_first + held
        d = ts.DeviceBuffer(ctx, sc[first:first + count] if count else np.zeros((1, 4), dtype=np.uint64))
        return ts.msm_sharded_resident(sp.commitment_params, comm, d, count, n_total), comm.info()
    got, errs = run_ranks(size, body)
    assert errs == [None] * size
    for r, (g, info) in enumerate(got):
        assert np.array_equal(g, want)
        assert info == {"rank": r, "size": size, "seen_size": size, "kind": "callback"}


def test_msm_sharded_rejects_wrong_slice():
    L, size, n_total = 8, 2, 512
    sc = ts.fr_rand_batch(bytes([7] * 32), n_total)

    def body(r, comm, ctx):
        sp, _ = ts.setup_params_shard(L, r, size, ctx=ctx)
        d = ts.DeviceBuffer(ctx, sc[:100])
        return ts.msm_sharded_resident(sp.commitment_params, comm, d, 100, n_total)
    _, errs = run_ranks(size, body)
    assert all(isinstance(e, ts.InvalidParameters) for e in errs)


def test_rccl_communicator_one_rank():
    L = 6
    addr, val, isw = ts.bench_trace(1 << L, 1 << (L + 2))
    want = ts.Twist(params(L)).prove_soa(addr, val, isw)
    ctx = ts.Context(0)
    comm = ts.Comm.rccl(ctx, 0, 1, ts.Comm.unique_id())
    assert comm.info() == {"rank": 0, "size": 1, "seen_size": 1, "kind": "rccl"}  # ncclCommCount
    pp, _ = ts.setup_params_shard(L, 0, 1, ctx=ctx)
    assert ts.Twist(pp).prove_sharded(comm, addr, val, isw, len(addr)) == want


def test_c5_one_2e26_proof_over_8_ranks():
    """BASELINE C5: ONE Twist::prove of the 2^26-operation ProtocolBenchmarks trace,
    setup_params(24), sharded over 8 ranks (threads on one GPU here, one process per GPU in
    bench.py): every rank returns the unsharded proof, and that proof passes the trapdoor
    identities (C = f(tau) G, pi (tau - z) = C - v G, v = f(z); f by the C oracle's O(N)
    barycentric evaluation) and the transcript replay."""
    from test_gpu_configs import check_pair, replay

    logn, size = 26, 8
    n, L = 1 << logn, logn - 2
    addr, val, isw = ts.bench_trace(1 << L, n)
    ctx = ts.Context(0)  # private: its SRS, window table and workspaces go with it
    pp, _ = ts.setup_params_shard(L, 0, 1, ctx=ctx)
    want = ts.Twist(pp).prove_soa(addr, val, isw)
    seed, tau = pp.fiat_shamir_seed, pp.commitment_params.tau
    del pp, ctx
    got, errs = sharded_twist(L, size, addr, val, isw)
    assert errs == [None] * size
    assert all(p == want for p in got)
    Ca, Cv = want.address_commitment.commitment, want.value_commitment.commitment
    chals, z = replay(seed, (b"address_commitment", b"value_commitment"), Ca, Cv, logn)
    assert want.sumcheck_challenges == chals and want.opening_point == z
    assert want.consistency_proof.round_polynomials == [[0, 0, 0, 0]] * logn
    check_pair(tau, n, ts.fr_from_u64_array(addr), val, (Ca, Cv), z, want.final_evaluations,
               [p.proof for p in want.opening_proofs])


@pytest.mark.skipif(ts.device_count() < 2, reason="needs 2 visible GPUs")
def test_rccl_communicator_two_devices():
    """The library's own RCCL communicator (ncclAllGather over xGMI) with 2 ranks on 2 GPUs,
    one thread per rank: the sharded proof equals the unsharded one."""
    L, size = 10, 2
    addr, val, isw = ts.bench_trace(1 << L, 1 << (L + 2))
    want = ts.Twist(params(L)).prove_soa(addr, val, isw)
    uid = ts.Comm.unique_id()
    out, errs = [None] * size, [None] * size

    def worker(r):
        try:
            ctx = ts.Context(r)
            comm = ts.Comm.rccl(ctx, r, size, uid)
            pp, _ = ts.setup_params_shard(L, r, size, ctx=ctx)
            first, count = ts.shard_slice(len(addr), r, size)
            out[r] = ts.Twist(pp).prove_sharded(comm, addr[first:first + count], val[first:first + count],
                                                isw[first:first + count], len(addr))
        except BaseException as e:  # noqa: BLE001 -- surfaced below
            errs[r] = e

    th = [threading.Thread(target=worker, args=(r,)) for r in range(size)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert errs == [None] * size
    assert all(p == want for p in out)
