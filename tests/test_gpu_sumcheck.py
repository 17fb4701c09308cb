"""SumCheck::prove with a non-zero composition (src/sumcheck.rs:56-110, :156-212) on the GPU at
the sizes the bench times it (2^20, 2^24) and between, against the C oracle's O(N)-per-round fold
restatement (oracle/fastcpu.c fc_sumcheck_prove), which tests/test_fastcpu.py pins to the
reference's closure algorithm (oracle.c orc_sumcheck_prove).  Round polynomials, challenges and
the final evaluation must be bit-identical; host-buffer and device-resident entry points agree."""
import os

import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyoracle as po

import twist_and_shout as ts

pytestmark = pytest.mark.gpu
R = po.R_MOD

COMPOSITIONS = {
    # the Twist MLE shapes (address A, value V, op flag O): A V - O^2 V + 2 O, degree 3
    "twist_like": [(1, [0, 1]), (R - 1, [2, 2, 1]), (2, [2])],
    "mixed": [(3, [0, 1, 2]), (R - 5, [1]), (7, [0, 0]), (11, [])],
    "cube4": [(5, [1, 1, 1]), (9, [3]), (1, [0, 2, 3])],
    # four tables, general coefficients at every depth (the K = 4 round kernel's most products)
    "dense4": [(17, [0, 1, 2]), (R - 3, [3, 3]), (5, [1, 2, 3]), (R - 1, [0]), (2, [2, 3]), (7, [])],
    # one and two tables (the K = 1 / 2 kernels and the host rounds' smallest table sets)
    "single": [(3, [0, 0, 0]), (R - 2, [0]), (5, [])],
    "pair2": [(1, [0, 1]), (4, [1, 1])],
}


def host_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(64, n))


def rand_tables(k, nv, seed):
    """k tables of 2^nv Montgomery Fr (limbs below r: top limb < 2^60)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        t = rng.integers(0, 2**63, size=(1 << nv, 4), dtype=np.uint64) * np.uint64(2)
        t += rng.integers(0, 2, size=(1 << nv, 4), dtype=np.uint64)
        t[:, 3] &= np.uint64((1 << 60) - 1)
        out.append(t)
    return out


@pytest.mark.parametrize("nv,name", [(14, "twist_like"), (14, "mixed"), (14, "cube4"), (14, "dense4"), (18, "twist_like"),
                                     (20, "twist_like"), (24, "twist_like")])
def test_generic_sumcheck_matches_fold_oracle(nv, name):
    terms = COMPOSITIONS[name]
    k = 1 + max(max(ix) for _, ix in terms if ix)
    tabs = rand_tables(k, nv, seed=nv * 7 + k)
    T = host_threads()
    claim = co.fast_composition_sum(tabs, nv, terms, T)
    st, rounds, fin, chal = co.fast_sumcheck_prove(tabs, nv, claim, terms, threads=T)
    assert st == 0
    want_rounds = [co.fr_ints(r) for r in rounds]
    proof, chals = ts.SumCheck(nv, claim).prove(tabs, terms, ts.Transcript(bytes(32)), return_challenges=True)
    assert proof.round_polynomials == want_rounds
    assert proof.final_evaluation == co.fr_ints(fin)[0]
    assert chals == co.fr_ints(chal)
    ctx = ts.Context.get(0)
    d = [ts.DeviceBuffer(ctx, t) for t in tabs]
    assert ts.SumCheck.composition_sum_resident(nv, d, terms) == claim
    p2, c2 = ts.SumCheck(nv, claim).prove_resident(d, terms, ts.Transcript(bytes(32)))
    assert p2 == proof and c2 == chals
    for t, dt in zip(tabs, d):  # the inputs are only read
        back = np.empty_like(t)
        ts.buffer_download(dt, back)
        assert np.array_equal(back, t)


def test_generic_sumcheck_wrong_claim_at_scale():
    nv = 18
    terms = COMPOSITIONS["twist_like"]
    tabs = rand_tables(3, nv, seed=5)
    claim = co.fast_composition_sum(tabs, nv, terms, host_threads())
    ctx = ts.Context.get(0)
    d = [ts.DeviceBuffer(ctx, t) for t in tabs]
    with pytest.raises(ts.SumCheckError):
        ts.SumCheck(nv, claim + 1).prove_resident(d, terms, ts.Transcript(bytes(32)))
    with pytest.raises(ts.InvalidParameters):
        ts.SumCheck(nv + 1, claim).prove_resident(d, terms, ts.Transcript(bytes(32)))
    # the failed proofs released the round kernels queued behind their challenges: the context
    # proves the true claim afterwards (the prover's final-value check would catch stale state)
    ts.SumCheck(nv, claim).prove_resident(d, terms, ts.Transcript(bytes(32)))


@pytest.mark.parametrize("name", ["twist_like", "dense4"])
@pytest.mark.parametrize("nv", [0, 1, 2, 3, 4, 5, 13, 14, 15, 16])
def test_generic_sumcheck_schedule_regimes(name, nv):
    _regime(name, nv)


@pytest.mark.parametrize("name", ["single", "pair2", "mixed", "cube4"])
@pytest.mark.parametrize("nv", [3, 7, 9, 12])
def test_generic_sumcheck_host_rounds(name, nv):
    """The last rounds on the host (from the first round of <= 64 pairs, mle.hip SC_HOST_PAIRS)
    for one to four tables: at nv = 3 / 7 / 9 the device runs rounds 0-1 and the persistent tail's
    first round is the hand-over; at nv = 12 the tail runs rounds 2-4 first (512 .. 128 pairs) and
    the host takes rounds 5-11."""
    _regime(name, nv)


def _regime(name, nv):
    """Every regime of the round schedule against the fold oracle: nv = 0 (the final kernel reads
    the caller's tables as they are), nv = 1 (round 0 then the final fold of the caller's
    tables), 2..5 (the persistent tail from round 2 on), 13..16 (split four-lanes-a-pair rounds up
    to 2^13 pairs, the pairs-per-lane kernel above, the tail taking over at 2^13 pairs) -- host
    and device-resident entry points alike."""
    terms = COMPOSITIONS[name]
    k = 1 + max(max(ix) for _, ix in terms if ix)
    tabs = rand_tables(k, nv, seed=41 + k + nv)
    T = host_threads()
    claim = co.fast_composition_sum(tabs, nv, terms, T)
    st, rounds, fin, chal = co.fast_sumcheck_prove(tabs, nv, claim, terms, threads=T)
    assert st == 0
    ctx = ts.Context.get(0)
    d = [ts.DeviceBuffer(ctx, t) for t in tabs]
    for proof, chals in (ts.SumCheck(nv, claim).prove(tabs, terms, ts.Transcript(bytes(32)), return_challenges=True),
                         ts.SumCheck(nv, claim).prove_resident(d, terms, ts.Transcript(bytes(32)))):
        assert proof.round_polynomials == [co.fr_ints(r) for r in rounds]
        assert proof.final_evaluation == co.fr_ints(fin)[0]
        assert chals == co.fr_ints(chal)
