"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact for every output (all hot-path arithmetic is integer / modular).  Small sizes
compare with the oracle's restatement of the reference algorithms and the committed
golden fixtures; large sizes use size-independent properties (trapdoor identities
C = f(tau) G and pi (tau - z) = C - v G, interpolant round trips, transcript replay).
"""
import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyoracle as po

import twist_and_shout as ts

pytestmark = pytest.mark.gpu
R = po.R_MOD


def h(x):
    return int(x, 16)


def g1h(P):
    return None if P is None else (h(P[0]), h(P[1]))


def rand_fr_mont(n, seed):
    """Uniform random Fr (Montgomery limbs < r: top limb masked below r's top limb)."""
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64) * 2 + rng.integers(0, 2, size=(n, 4), dtype=np.uint64)
    a[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
    return a


_PARAMS = {}


def params(L):
    if L not in _PARAMS:
        _PARAMS[L] = ts.setup_params(L)
    return _PARAMS[L]


_CPARAMS = {}


def cparams(L):
    if L not in _CPARAMS:
        _CPARAMS[L] = co.setup_params(L)
    return _CPARAMS[L]


# ---------------------------------------------------------------- setup_params / SRS
def test_setup_params_matches_golden(golden):
    for L, s in golden["setup_params"].items():
        pp, vp = params(int(L))
        assert pp.commitment_params.tau == h(s["tau"])
        assert pp.fiat_shamir_seed.hex() == s["fiat_shamir_seed"]
        assert pp.max_operations == s["max_operations"] == vp.max_operations
        assert pp.commitment_params.g1_powers == [g1h(P) for P in s["g1_powers"]]


def test_setup_params_L8_matches_c_oracle():
    pp, _ = params(8)
    got = pp.commitment_params.srs.download()
    want = cparams(8)["g1_limbs"]
    assert got.shape == want.shape and np.array_equal(got, want)


# ---------------------------------------------------------------- MSM / KZG commit
@pytest.mark.parametrize("n", [1, 2, 5, 64, 65, 127, 128, 129, 1000, 1025])
def test_msm_random_matches_oracle(n):
    pp, _ = params(8)
    c = rand_fr_mont(n, seed=n)
    got = ts.KZGCommitment.commit(pp.commitment_params, c).commitment
    st, want = co.commit(cparams(8)["g1_limbs"], c)
    assert st == 0 and got == co.g1_from_limbs(want)


@pytest.mark.parametrize("pattern", ["zeros", "ones", "minus_one", "small", "last_only", "equal", "neg_pairs"])
def test_msm_structured_scalars(pattern):
    pp, _ = params(8)
    n = 777
    if pattern == "zeros":
        vals = [0] * n
    elif pattern == "ones":
        vals = [1] * n
    elif pattern == "minus_one":
        vals = [R - 1] * n
    elif pattern == "small":
        vals = [i % 17 for i in range(n)]
    elif pattern == "last_only":
        vals = [0] * (n - 1) + [123456789]
    elif pattern == "equal":
        vals = [2**200 + 12345] * n
    else:
        vals = [(i if i % 2 == 0 else R - i) for i in range(n)]
    c = ts.to_mont(vals)
    got = ts.KZGCommitment.commit(pp.commitment_params, c).commitment
    st, want = co.commit(cparams(8)["g1_limbs"], c)
    assert st == 0 and got == co.g1_from_limbs(want)


@pytest.mark.parametrize("L", [14, 18])
def test_msm_large_trapdoor(L):
    """2^16 / 2^20 pairs: C == (sum c_i tau^i) G (the C2 configuration at L = 18)."""
    pp, _ = params(L)
    n = 1 << (L + 2)
    c = rand_fr_mont(n, seed=L)
    got = ts.msm(pp.commitment_params, c)
    tau = pp.commitment_params.tau
    s = 0
    for v in reversed(ts.from_mont(c)):
        s = (s * tau + v) % R
    assert got == po.affine_mul(po.G1_GEN, s)


@pytest.mark.parametrize("pattern", ["equal", "tiny", "addr22", "flags", "half_equal", "pow2"])
def test_msm_skewed_scalars_large(pattern):
    """Heavy buckets (one bucket holding up to all 2^20 entries) and narrow scalars (the
    bit-length-adaptive window plan) -- the shapes Twist commits produce."""
    pp, _ = params(18)
    n = 1 << 20
    rng = np.random.default_rng(hash(pattern) % 2**32)
    if pattern == "equal":
        vals = [2**200 + 12345] * n
    elif pattern == "tiny":
        vals = [int(x) for x in rng.integers(0, 3, size=n)]
    elif pattern == "addr22":
        vals = [int(x) for x in rng.integers(0, 1 << 22, size=n)]
    elif pattern == "flags":
        vals = [int(x) for x in rng.integers(0, 2, size=n)]
    elif pattern == "half_equal":
        r = rand_fr_mont(n // 2, seed=5)
        vals = [R - 7] * (n // 2) + ts.from_mont(r)
    else:  # powers of two: one nonzero digit per scalar, spread over every window
        vals = [1 << int(x) for x in rng.integers(0, 254, size=n)]
    c = ts.to_mont(vals)
    got = ts.msm(pp.commitment_params, c)
    tau = pp.commitment_params.tau
    s = 0
    for v in reversed(vals):
        s = (s * tau + v) % R
    assert got == po.affine_mul(po.G1_GEN, s)


@pytest.mark.parametrize("logn", [16, 20])
def test_msm_window_tables_equal_per_window_layout(logn):
    """Shared-bucket MSM (fixed-base window table) == per-window MSM, full-width and
    narrow scalars."""
    pp, _ = params(logn - 2)
    n = 1 << logn
    ctx = ts.Context.get(0)
    for c in (rand_fr_mont(n, seed=logn + 1), ts.to_mont([i * 7919 % (1 << 40) for i in range(n)])):
        a = ts.msm(pp.commitment_params, c)
        ctx.set_msm_tables(False)
        try:
            b = ts.msm(pp.commitment_params, c)
        finally:
            ctx.set_msm_tables(True)
        assert a == b


def trapdoor_commitment(tau, vals):
    """(sum_i c_i tau^i) G -- the commitment by the SRS's retained tau (oracle side)."""
    s = 0
    for v in reversed(vals):
        s = (s * tau + v) % R
    return po.affine_mul(po.G1_GEN, s)


@pytest.mark.parametrize("tables", [True, False])
@pytest.mark.parametrize("pattern", ["full", "addr21", "addr22", "val30", "equal"])
def test_msm_sort_shapes_trapdoor(pattern, tables):
    """The bucket sort's plans at 2^20 pairs, each against the trapdoor identity (not against
    another HIP path): full-width scalars (the c = 20, W = 13 table plan, or 13 per-window
    buckets sets without the table: the runtime-plan pass-1 kernels), 21- and 22-bit scalars (the
    single 22/23-bit window: 2^21/2^22 buckets, the per-window packed tail), 30-bit values (W = 2,
    c = 16: the per-window compile-time plan and its heavy buckets across many chunks), and one
    value repeated (every entry of a window in one bucket: the fixup's wave-summed runs)."""
    pp, _ = params(18)
    n = 1 << 20
    rng = np.random.default_rng(len(pattern))
    if pattern == "full":
        c = rand_fr_mont(n, seed=77)
        vals = ts.from_mont(c)
    elif pattern == "equal":
        vals = [R - 12345] * n
        c = ts.to_mont(vals)
    else:
        bits = int(pattern[-2:])
        u = rng.integers(0, 1 << bits, size=n, dtype=np.uint64)
        vals = [int(x) for x in u]
        c = ts.fr_from_u64_array(u)
    ctx = pp.commitment_params.srs.ctx
    ctx.set_msm_tables(tables)
    try:
        got = ts.msm(pp.commitment_params, c)
    finally:
        ctx.set_msm_tables(True)
    assert got == trapdoor_commitment(pp.commitment_params.tau, vals)


@pytest.mark.parametrize("tables", [True, False])
def test_msm_c2_bench_workload_trapdoor(tables):
    """The exact C2 bench input -- Fr::rand from ChaCha20Rng([7; 32]), 2^20 scalars
    (ts.fr_rand_batch, the reference's UniformRand restated) over setup_params(18), device-resident
    as bench.py passes them -- against C == (sum c_i tau^i) G, with the SRS window table and
    without it (/root/reference/src/commitments.rs:162-180)."""
    pp, _ = params(18)
    n = 1 << 20
    sc = ts.fr_rand_batch(bytes([7] * 32), n)
    ctx = pp.commitment_params.srs.ctx
    d = ts.DeviceBuffer(ctx, sc)
    ctx.set_msm_tables(tables)
    try:
        got = ts.msm_resident(pp.commitment_params, d, n)
    finally:
        ctx.set_msm_tables(True)
    assert ts._g1_from_proj(got) == trapdoor_commitment(pp.commitment_params.tau, ts.from_mont(sc))


def test_commit_beyond_srs_is_commitment_error():
    pp, _ = params(1)  # 9 SRS points
    with pytest.raises(ts.CommitmentError):
        ts.KZGCommitment.commit(pp.commitment_params, list(range(10)))


# ---------------------------------------------------------------- KZG open
@pytest.mark.parametrize("n", [0, 1, 2, 3, 17, 64, 65, 256, 1025])
def test_kzg_open_matches_oracle(n):
    pp, _ = params(8)
    c = rand_fr_mont(n, seed=100 + n) if n else np.zeros((0, 4), dtype=np.uint64)
    z = 0xDEADBEEF * (n + 3) + 2**190
    v, pi = ts.KZGCommitment.open(pp.commitment_params, c, z)
    if n == 0:
        assert v == 0 and pi.proof is None
        return
    st, vw, pw = co.open_(cparams(8)["g1_limbs"], c, co.fr_array([z])[0])
    assert st == 0
    assert v == co.fr_ints(vw)[0]
    assert pi.proof == co.g1_from_limbs(pw)


def test_kzg_demo_polynomial():
    # examples/demo.rs / src/commitments.rs:491-533: 3x^2 + 2x + 1 opened at 5 -> 86
    pp, _ = params(4)
    v, pi = ts.KZGCommitment.open(pp.commitment_params, [1, 2, 3], 5)
    assert v == 86
    C = ts.KZGCommitment.commit(pp.commitment_params, [1, 2, 3]).commitment
    tau = pp.commitment_params.tau
    assert po.affine_mul(pi.proof, (tau - 5) % R) == po.affine_add(C, po.g1_neg(po.affine_mul(po.G1_GEN, 86)))


# ---------------------------------------------------------------- interpolation
@pytest.mark.parametrize("logn", list(range(0, 10)))
def test_interpolate_matches_oracle(logn):
    n = 1 << logn
    y = rand_fr_mont(n, seed=logn)
    got = ts.poly_utils.interpolate_consecutive(y)
    want = co.interpolate(y)
    assert np.array_equal(got, want)


def test_interpolate_reference_kat():
    # tests/polynomial_tests.rs:195-207 (x^2 through (0,0),(1,1),(2,4)); padded to 4 nodes: (3,9)
    assert ts.poly_utils.lagrange_interpolate([(0, 0), (1, 1), (2, 4), (3, 9)]) == [0, 0, 1, 0]


@pytest.mark.parametrize("logn", [12, 16, 20])
def test_interpolate_large_roundtrip(logn):
    """Interpolant reproduces the values at sampled nodes and matches barycentric at a far point."""
    n = 1 << logn
    y = rand_fr_mont(n, seed=1000 + logn)
    coeffs = ts.poly_utils.interpolate_consecutive(y)
    rng = np.random.default_rng(logn)
    nodes = [0, 1, n - 1] + [int(x) for x in rng.integers(0, n, size=5)]
    for i in nodes:
        assert np.array_equal(co.horner(coeffs, co.fr_array([i])[0]), y[i])
    if logn <= 16:
        z = 2**250 + 77
        ys = ts.from_mont(y)
        assert co.fr_ints(co.horner(coeffs, co.fr_array([z])[0]))[0] == po.barycentric_eval(ys, z)


def test_interpolate_structured_inputs():
    for logn in (4, 8):
        n = 1 << logn
        for vals in ([0] * n, [1] * n, list(range(n)), [i * i for i in range(n)], [R - 1] * n):
            y = ts.to_mont(vals)
            assert np.array_equal(ts.poly_utils.interpolate_consecutive(y), co.interpolate(y))


# ---------------------------------------------------------------- MLE
def test_mle_reference_kats():
    m = ts.MultilinearExtension.from_evaluations([1, 2, 3, 4])
    assert [m.evaluate(p) for p in ([0, 0], [1, 0], [0, 1], [1, 1])] == [1, 2, 3, 4]
    half = pow(2, -1, R)
    assert m.evaluate([half, half]) == 10 * pow(4, -1, R) % R
    p = m.partial_evaluate([1])
    assert p.num_vars == 1 and p.evaluations == [2, 4]
    s = ts.MultilinearExtension.from_sparse(3, [(0, 100), (7, 700)])
    assert s.evaluate([0, 0, 0]) == 100 and s.evaluate([1, 1, 1]) == 700 and s.evaluate([1, 1, 0]) == 0


def test_mle_struct_with_any_entry_count():
    # the struct's fields are public (src/polynomials.rs:18-24): evaluate sums over the entries
    # held, each at its low num_vars index bits (:91-122) -- short and long vectors included
    pt = [5, 7, 11]
    short = ts.MultilinearExtension(3, [1, 2])
    assert short.evaluate(pt) == po.mle_evaluate([1, 2] + [0] * 6, pt)
    long_ = ts.MultilinearExtension(2, list(range(1, 11)))
    folded = [sum(v for i, v in enumerate(range(1, 11)) if i % 4 == j) % R for j in range(4)]
    assert long_.evaluate(pt[:2]) == po.mle_evaluate(folded, pt[:2])
    assert short.partial_evaluate([3]).evaluations == ts.MultilinearExtension(3, [1, 2] + [0] * 6).partial_evaluate(
        [3]).evaluations
    assert ts.MultilinearExtension(2, []).evaluate([1, 2]) == 0
    import twist_and_shout._native as N
    ev = ts.to_mont([1, 2, 3, 4, 5])
    out = np.zeros(4, dtype=np.uint64)
    st = N.load().tns_mle_evaluate(ts.Context.get(0).handle, N.p64(ev), 5, 2, N.p64(ts.to_mont([1, 2])), N.p64(out))
    assert st == 1  # more entries than 2^nv: InvalidParameters at the C ABI


@pytest.mark.parametrize("nv", [0, 1, 2, 5, 10, 14])
def test_mle_evaluate_matches_oracle(nv):
    ev = rand_fr_mont(1 << nv, seed=nv)
    pt = rand_fr_mont(max(nv, 1), seed=50 + nv)[:nv]
    import twist_and_shout._native as N
    import ctypes as C
    out = np.zeros(4, dtype=np.uint64)
    st = N.load().tns_mle_evaluate(ts.Context.get(0).handle, N.p64(ev), len(ev), nv,
                                   N.p64(np.ascontiguousarray(pt) if nv else np.zeros((1, 4), dtype=np.uint64)),
                                   N.p64(out))
    assert st == 0
    if nv <= 10:
        assert np.array_equal(out, co.mle_evaluate(ev, pt))
    else:  # oracle evaluate is O(N n); check linearity-free property: fold == partial chain
        want = ts.from_mont(ev)
        for j, r in enumerate(ts.from_mont(pt)):
            want = [(want[2 * s] + r * (want[2 * s + 1] - want[2 * s])) % R for s in range(len(want) // 2)]
        assert ts.from_mont(out)[0] == want[0]


@pytest.mark.parametrize("nv,k", [(3, 1), (6, 3), (8, 8), (9, 0)])
def test_mle_partial_evaluate_matches_oracle(nv, k):
    vals = ts.from_mont(rand_fr_mont(1 << nv, seed=nv * 7 + k))
    fixed = ts.from_mont(rand_fr_mont(max(k, 1), seed=k + 99))[:k]
    got = ts.MultilinearExtension(nv, vals).partial_evaluate(fixed).evaluations
    want = co.fr_ints(co.mle_partial_evaluate(ts.to_mont(vals), ts.to_mont(fixed) if k else np.zeros((0, 4), dtype=np.uint64)))
    assert got == want


# ---------------------------------------------------------------- sum-check
def test_sumcheck_x1x2_golden(golden):
    # src/sumcheck.rs:221-245: f(x1, x2) = x1 * x2, claim 1
    sc = ts.SumCheck(2, 1)
    tr = ts.Transcript(bytes([42] * 32))
    proof, chals = sc.prove([[0, 1, 0, 1], [0, 0, 1, 1]], [(1, [0, 1])], tr, return_challenges=True)
    g = golden["sumcheck_x1x2"]
    assert proof.round_polynomials == [[h(c) for c in r] for r in g["rounds"]]
    assert proof.final_evaluation == h(g["final"])
    assert chals == [h(c) for c in g["challenges"]]


COMPOSITIONS = {
    "abc": [(1, [0, 1, 2])],
    "mixed": [(3, [0, 1, 2]), (R - 5, [1]), (7, [0, 0]), (11, [])],
    "twist_like": [(1, [0, 1]), (R - 1, [2, 2, 1]), (2, [2])],
    # every coefficient kind (1, -1, 2, general) at every nesting depth, repeated tables, terms that
    # combine (the two [1, 2] terms) and a constant: the round kernel's nested form (sc_poly)
    "kinds": [(1, [0]), (R - 1, [1, 2]), (2, [0, 1, 2]), (5, [2, 2]), (R - 1, [0, 0, 0]), (3, [2, 1]), (R - 2, [])],
    # all 19 monomials of degree 1..3 over 3 tables with general coefficients (the most products)
    "dense": [(1000003 * (i + 1) % R, ix) for i, ix in enumerate(
        [[a] for a in range(3)] + [[a, b] for a in range(3) for b in range(a, 3)]
        + [[a, b, c] for a in range(3) for b in range(a, 3) for c in range(b, 3)])],
}


@pytest.mark.parametrize("name", list(COMPOSITIONS))
@pytest.mark.parametrize("nv", [0, 1, 3, 6])
def test_sumcheck_matches_oracle(name, nv):
    terms = COMPOSITIONS[name]
    tabs = [rand_fr_mont(1 << nv, seed=nv * 31 + i) for i in range(3)]
    ints = [ts.from_mont(t) for t in tabs]
    claim = 0
    for x in range(1 << nv):
        for c, ix in terms:
            p = c
            for j in ix:
                p = p * ints[j][x] % R
            claim = (claim + p) % R
    tr = ts.Transcript(bytes(32))
    proof, chals = ts.SumCheck(nv, claim).prove(tabs, terms, tr, return_challenges=True)
    st, rounds, fin, chal = co.sumcheck_prove(tabs, nv, claim, terms)
    assert st == 0
    assert proof.round_polynomials == [co.fr_ints(r) for r in rounds]
    assert proof.final_evaluation == co.fr_ints(fin)[0]
    assert chals == co.fr_ints(chal)


def test_sumcheck_wrong_claim_is_sumcheck_error():
    tabs = [rand_fr_mont(8, seed=3)]
    with pytest.raises(ts.SumCheckError):
        ts.SumCheck(3, 12345).prove(tabs, [(1, [0])], ts.Transcript(bytes(32)))


# ---------------------------------------------------------------- Twist / Shout
def _twist_from_golden(case):
    pp, _ = params(case["log_size"])
    addr = np.array([a for (_, a, _) in case["ops"]], dtype=np.uint64)
    val = ts.to_mont([h(v) for (_, _, v) in case["ops"]]) if case["ops"] else np.zeros((0, 4), dtype=np.uint64)
    isw = np.array([w for (w, _, _) in case["ops"]], dtype=np.uint8)
    return ts.Twist(pp).prove_soa(addr, val, isw)


def _assert_twist_equal(pr, want):
    assert pr.address_commitment.commitment == g1h(want["address_commitment"])
    assert pr.value_commitment.commitment == g1h(want["value_commitment"])
    assert pr.consistency_proof.round_polynomials == [[h(c) for c in r] for r in want["round_polynomials"]]
    assert pr.consistency_proof.final_evaluation == h(want["final_evaluation"])
    assert [p.proof for p in pr.opening_proofs] == [g1h(P) for P in want["opening_proofs"]]
    assert pr.final_evaluations == [h(v) for v in want["final_evaluations"]]
    assert pr.opening_point == (None if want["opening_point"] is None else h(want["opening_point"]))
    assert pr.sumcheck_challenges == [h(c) for c in want["sumcheck_challenges"]]


@pytest.mark.parametrize("name", ["demo_L3", "small_trace_L3", "empty_L2", "only_reads_L2", "only_writes_L2",
                                  "repeated_L2", "max_ops_L2", "unit_L4", "single_op_L2"])
def test_twist_matches_golden(golden, name):
    case = golden["twist"][name]
    _assert_twist_equal(_twist_from_golden(case), case["proof"])


def test_twist_c1_256_ops_matches_golden(golden):
    """C1: setup_params(8), 256 benchmark ops (src/benchmarks.rs:88-99)."""
    case = golden["twist"]["C1_bench_256_L8"]
    pp, _ = params(8)
    pr = ts.Twist(pp).prove_soa(*ts.bench_trace(256, 256))
    _assert_twist_equal(pr, case["proof"])


def test_twist_via_memory_trace_api(golden):
    pp, _ = params(3)
    tr = ts.MemoryTrace(8)  # examples/demo.rs:32-62
    tr.write(0, 42)
    tr.write(1, 100)
    tr.read(0)
    tr.read(1)
    tr.write(0, 43)
    assert tr.read(0) == 43
    _assert_twist_equal(ts.Twist(pp).prove(tr), golden["twist"]["demo_L3"]["proof"])


def test_twist_too_many_operations():
    pp, _ = params(1)  # max 8 (tests/twist_tests.rs:180-196)
    tr = ts.MemoryTrace(2)
    for i in range(10):
        tr.write(i % 2, i + 1)
    with pytest.raises(ts.InvalidParameters):
        ts.Twist(pp).prove(tr)


@pytest.mark.parametrize("name", ["demo_squares_L3", "single_entry_L2", "no_lookups_L2", "ragged_table_L3",
                                  "sixteen_L4"])
def test_shout_matches_golden(golden, name):
    case = golden["shout"][name]
    pp, _ = params(case["log_size"])
    t = ts.LookupTable([h(e) for e in case["entries"]])
    for i in case["lookups"]:
        t.lookup(i)
    pr = ts.Shout(pp).prove(t)
    want = case["proof"]
    assert pr.table_commitment.commitment == g1h(want["table_commitment"])
    assert pr.index_commitment.commitment == g1h(want["index_commitment"])
    assert pr.lookup_proof.round_polynomials == [[h(c) for c in r] for r in want["round_polynomials"]]
    assert [p.proof for p in pr.opening_proofs] == [g1h(P) for P in want["opening_proofs"]]
    assert pr.final_evaluations == [h(v) for v in want["final_evaluations"]]
    assert pr.opening_point == (None if want["opening_point"] is None else h(want["opening_point"]))


def test_shout_table_larger_than_srs_is_commitment_error():
    pp, _ = params(1)  # 9 SRS points; the table size is not checked up front (src/shout.rs:97-133)
    t = ts.LookupTable(list(range(16)))
    t.lookup(3)
    with pytest.raises(ts.CommitmentError):
        ts.Shout(pp).prove(t)


def _check_twist_properties(pp, addr, val_mont, isw, pr):
    """Size-independent checks: trapdoor identities + transcript replay + MLE values."""
    n = len(addr)
    N = 1 << max(0, (n - 1).bit_length())
    tau = pp.commitment_params.tau
    ys_a = [int(a) for a in addr] + [0] * (N - n)
    ys_v = ts.from_mont(val_mont) + [0] * (N - n)
    Ca = pr.address_commitment.commitment
    Cv = pr.value_commitment.commitment
    assert Ca == po.affine_mul(po.G1_GEN, po.barycentric_eval(ys_a, tau))
    assert Cv == po.affine_mul(po.G1_GEN, po.barycentric_eval(ys_v, tau))
    # transcript replay (src/twist.rs:170-219) with the all-zero round polynomials
    t = po.Transcript(pp.fiat_shamir_seed)
    t.append_field_element(b"address_commitment", po.commitment_hash(Ca))
    t.append_field_element(b"value_commitment", po.commitment_hash(Cv))
    nv = N.bit_length() - 1
    chals = []
    for r in range(nv):
        assert pr.consistency_proof.round_polynomials[r] == [0, 0, 0, 0]
        t.append_field_elements(b"sumcheck_round_%d" % r, [0, 0, 0, 0])
        chals.append(t.challenge_field_element(b"sumcheck_challenge_%d" % r))
    assert pr.sumcheck_challenges == chals
    z = t.challenge_field_element(b"opening_challenges_0")
    assert pr.opening_point == z
    for ys, C, v, pi in zip((ys_a, ys_v), (Ca, Cv), pr.final_evaluations, pr.opening_proofs):
        assert v == po.barycentric_eval(ys, z)
        assert po.affine_mul(pi.proof, (tau - z) % R) == po.affine_add(C, po.g1_neg(po.affine_mul(po.G1_GEN, v)))
    return chals


# 10: the whole fold chain runs in k_sc_fold_tail; 13 / 14: one / two k_sc_round folds first
# (the tail then starts from the scratch / the caller's buffers); 15 / 16: one three-round
# k_sc_fold3 pass (then nothing / one k_sc_round) before the tail
@pytest.mark.parametrize("logn", [10, 13, 14, 15, 16])
def test_twist_bench_trace_properties(logn):
    L = logn - 2
    pp, _ = params(L)
    addr, val, isw = ts.bench_trace(1 << L, 1 << logn)
    pr = ts.Twist(pp).prove_soa(addr, val, isw)
    chals = _check_twist_properties(pp, addr, val, isw, pr)
    # the sum-check fold chain ends at the MLE values at the challenge point
    want = [co.fr_ints(co.mle_evaluate(t, ts.to_mont(chals)))[0]
            for t in (ts.fr_from_u64_array(addr), val, ts.fr_from_u64_array(isw.astype(np.uint64)))]
    assert pr.final_mle_evals == want


@pytest.mark.parametrize("n_ops", [(1 << 15) + 1, (1 << 16) - 13])
def test_twist_ragged_fold_chain_from_flag_bytes(n_ops):
    """From 2^15 padded operations the op-type table's first fold reads the is_write bytes (zero
    beyond the trace, an unaligned tail); the bound values still equal the padded tables' MLEs."""
    n = 1 << (n_ops - 1).bit_length()
    L = n.bit_length() - 3
    pp, _ = params(L)
    addr, val, isw = ts.bench_trace(1 << L, n_ops)
    pr = ts.Twist(pp).prove_soa(addr, val, isw)
    chals = _check_twist_properties(pp, addr, val, isw, pr)
    pad = n - n_ops
    cols = (np.concatenate([addr, np.zeros(pad, np.uint64)]), np.concatenate([val, np.zeros((pad, 4), np.uint64)]),
            np.concatenate([isw.astype(np.uint64), np.zeros(pad, np.uint64)]))
    want = [co.fr_ints(co.mle_evaluate(t, ts.to_mont(chals)))[0]
            for t in (ts.fr_from_u64_array(cols[0]), cols[1], ts.fr_from_u64_array(cols[2]))]
    assert pr.final_mle_evals == want


def test_twist_ragged_trace_properties():
    pp, _ = params(8)  # max_operations 1024
    addr, val, isw = ts.bench_trace(256, 1000)  # pads to 1024
    pr = ts.Twist(pp).prove_soa(addr, val, isw)
    _check_twist_properties(pp, addr, val, isw, pr)
