"""The fast CPU baseline (oracle/fastcpu.c: the GPU path's algorithms on host threads) against
the reference-algorithm restatement (oracle/oracle.c): identical Twist proofs."""
import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyoracle as po


def _trace(n_ops, mem, seed):
    rng = np.random.default_rng(seed)
    addr = rng.integers(0, mem, size=n_ops).astype(np.uint64)
    vals = [int(x) for x in rng.integers(0, 1 << 40, size=n_ops)]
    isw = rng.integers(0, 2, size=n_ops).astype(np.uint8)
    return addr, vals, isw


@pytest.mark.parametrize("n_ops,threads", [(2, 1), (8, 3), (13, 4), (64, 8), (100, 5)])
def test_fast_cpu_twist_matches_reference_algorithms(n_ops, threads):
    p = co.setup_params(5)  # max_operations 128, SRS 129 points
    addr, vals, isw = _trace(n_ops, 16, n_ops)
    N = 1 << max(1, (n_ops - 1).bit_length())
    lag = co.lagrange_basis(p["tau_limbs"], N)
    w = co.bary_weights(N)
    st, got = co.fast_twist_prove(lag, w, p["max_operations"], addr, co.fr_array(vals), isw, threads)
    assert st == 0
    ops = [(int(isw[i]), int(addr[i]), vals[i]) for i in range(n_ops)]
    st2, want = co.twist_prove(p, ops)
    assert st2 == 0
    for k in ("address_commitment", "value_commitment", "opening_proofs", "final_evaluations", "opening_point",
              "round_polynomials", "final_evaluation", "sumcheck_challenges"):
        assert got[k] == want[k], k


def test_fast_cpu_bench_trace_and_errors():
    p = co.setup_params(4)
    ops = po.benchmark_trace(16, 48)
    N = 64
    lag, w = co.lagrange_basis(p["tau_limbs"], N), co.bary_weights(N)
    addr = np.array([a for (_, a, _) in ops], dtype=np.uint64)
    isw = np.array([k for (k, _, _) in ops], dtype=np.uint8)
    vals = co.fr_array([v for (_, _, v) in ops])
    st, got = co.fast_twist_prove(lag, w, p["max_operations"], addr, vals, isw, 4)
    st2, want = co.twist_prove(p, ops)
    assert st == st2 == 0 and got == want
    # too many operations (src/twist.rs:108-112) -> InvalidParameters
    st, _ = co.fast_twist_prove(lag, w, 32, addr, vals, isw, 2)
    assert st == 1


def test_bary_weights_identity():
    # sum_j L_j(x) = 1: ell(x) sum_j w_j / (x - j) = 1 at a random x
    N, x = 16, 123456789
    w = co.fr_ints(co.bary_weights(N))
    ell = 1
    for j in range(N):
        ell = ell * (x - j) % po.R_MOD
    s = sum(wj * pow(x - j, -1, po.R_MOD) for j, wj in enumerate(w)) % po.R_MOD
    assert ell * s % po.R_MOD == 1


SC_COMPOSITIONS = {
    "abc": [(1, [0, 1, 2])],
    "mixed": [(3, [0, 1, 2]), (po.R_MOD - 5, [1]), (7, [0, 0]), (11, [])],
    "twist_like": [(1, [0, 1]), (po.R_MOD - 1, [2, 2, 1]), (2, [2])],
    "cube": [(5, [1, 1, 1]), (9, [3])],
}


def _rand_tables(k, nv, seed):
    rng = np.random.default_rng(seed)
    return [co.fr_array([int.from_bytes(rng.bytes(32), "little") % po.R_MOD for _ in range(1 << nv)])
            for _ in range(k)]


@pytest.mark.parametrize("name", list(SC_COMPOSITIONS))
@pytest.mark.parametrize("nv,threads", [(0, 1), (1, 2), (3, 3), (6, 4), (8, 5)])
def test_fast_sumcheck_matches_reference_algorithm(name, nv, threads):
    """fc_sumcheck_prove (table folds, O(N) per round) == orc_sumcheck_prove (the reference's
    closure sum-check, src/sumcheck.rs:56-110, O(N n) per hypercube point) with the transcript
    prefix of a caller."""
    terms = SC_COMPOSITIONS[name]
    tabs = _rand_tables(4, nv, seed=nv * 13 + len(name))
    claim = co.fast_composition_sum(tabs, nv, terms, threads)
    want = co.sumcheck_prove(tabs, nv, claim, terms, prefix=b"prefix")
    got = co.fast_sumcheck_prove(tabs, nv, claim, terms, prefix=b"prefix", threads=threads)
    assert want[0] == got[0] == 0
    for a, b in zip(want[1:], got[1:]):
        assert np.array_equal(a, b)


def test_fast_sumcheck_wrong_claim_and_bad_table():
    tabs = _rand_tables(3, 4, seed=1)
    terms = SC_COMPOSITIONS["twist_like"]
    claim = co.fast_composition_sum(tabs, 4, terms, 2)
    assert co.fast_sumcheck_prove(tabs, 4, claim + 1, terms, threads=2)[0] == 6
    assert co.sumcheck_prove(tabs, 4, claim + 1, terms)[0] == 6
    assert co.fast_sumcheck_prove(tabs, 4, claim, [(1, [3])], threads=2)[0] == 1
