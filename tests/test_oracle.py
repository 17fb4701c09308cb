"""CPU tests of the oracle: pin it to the reference's KATs, the published ChaCha20 /
SipHash vectors, algebraic identities, and cross-check the Python and C restatements."""
import struct

import pytest

from oracle import coracle as co
from oracle import pyoracle as po

R = po.R_MOD


def h(x):
    return int(x, 16)


# ---------------------------------------------------------------- primitives vs published vectors
def test_chacha20_zero_key_keystream():
    # DJB ChaCha20, key = 0, nonce = 0, block 0: the whole 64-byte keystream block
    w = po.chacha20_block([0] * 8, 0)
    assert b"".join(x.to_bytes(4, "little") for x in w) == bytes.fromhex(
        "76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
        "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586")
    out = (co.C.c_uint32 * 16)()
    co.lib().orc_chacha20_block((co.C.c_uint32 * 8)(*[0] * 8), co.C.c_uint64(0), out)
    assert list(out) == w


def test_chacha20_rfc8439_block():
    # RFC 8439 section 2.3.2 (key 00..1f, nonce 00000009 0000004a 00000000, counter 1)
    key = list(struct.unpack("<8I", bytes(range(32))))
    st = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + key + [1, 0x09000000, 0x4A000000, 0]
    out = po.chacha20_block_raw(st)
    assert out == [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204,
                   0x4E6CD4C3, 0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE,
                   0xE883D0CB, 0x4E3C50A2]


# SipHash-2-4 reference-implementation vectors (key 00..0f, message 00..(n-1)), n = 0..15: every
# tail length of the last block, one- and two-block messages -- the block loop, tail packing and
# finalisation that SipHash-1-3 shares, pinned independently of the round counts
SIPHASH24_VECTORS = [
    0x726FDB47DD0E0E31, 0x74F839C593DC67FD, 0x0D6C8009D9A94F5A, 0x85676696D7FB7E2D,
    0xCF2794E0277187B7, 0x18765564CD99A68D, 0xCBC9466E58FEE3CE, 0xAB0200F58B01D137,
    0x93F5F5799A932462, 0x9E0082DF0BA9E4B0, 0x7A5DBBC594DDB9F3, 0xF4B32F46226BADA7,
    0x751E8FBC860EE5FB, 0x14EA5627C0843D90, 0xF723CA908E7AF2EE, 0xA129CA6149BE45E5,
]


def test_siphash24_reference_vectors():
    k0, k1 = struct.unpack("<QQ", bytes(range(16)))
    L = co.lib()
    for n, want in enumerate(SIPHASH24_VECTORS):
        m = bytes(range(n))
        buf = (co.C.c_uint8 * max(1, n)).from_buffer_copy(m or b"\0")
        assert po.siphash(m, k0, k1, 2, 4) == want, n
        assert L.orc_siphash(buf, n, k0, k1, 2, 4) == want, n
    for n in (0, 1, 7, 8, 9, 15, 16, 63):
        m = bytes(range(n))
        buf = (co.C.c_uint8 * max(1, n)).from_buffer_copy(m or b"\0")
        assert L.orc_siphash(buf, n, k0, k1, 2, 4) == po.siphash(m, k0, k1, 2, 4)
        assert L.orc_siphash(buf, n, 0, 0, 1, 3) == po.siphash(m, 0, 0, 1, 3)


def test_siphash13_known_answer():
    # SipHash-1-3 (Rust std DefaultHasher's compression/finalisation rounds), key 00..0f, empty
    # message: the first vector of Rust's own SipHasher13 suite (library/core/tests/hash/sip.rs,
    # test_siphash_1_3), bytes dc c4 0f 05 58 01 ac ab.  Both restatements must hit it.
    k0, k1 = struct.unpack("<QQ", bytes(range(16)))
    want = int.from_bytes(bytes.fromhex("dcc40f055801acab"), "little")
    assert po.siphash(b"", k0, k1, 1, 3) == want
    buf = (co.C.c_uint8 * 1)(0)
    assert co.lib().orc_siphash(buf, 0, k0, k1, 1, 3) == want


def test_fr_rand_rejection_and_montgomery_semantics():
    rng = po.ChaCha20Rng(bytes([42] * 32))
    t = po.fr_rand(rng)
    assert 0 < t < R
    # limbs are taken as the Montgomery representation: re-derive by hand
    rng2 = po.ChaCha20Rng(bytes([42] * 32))
    while True:
        limbs = [rng2.next_u64() for _ in range(4)]
        limbs[3] &= (1 << 62) - 1
        v = sum(l << (64 * i) for i, l in enumerate(limbs))
        if v < R:
            break
    assert t == v * pow(1 << 256, -1, R) % R


# ---------------------------------------------------------------- reference KATs
def test_reference_kats(golden):
    k = golden["kats"]
    # tests/polynomial_tests.rs:195-207
    assert [h(c) for c in k["lagrange_x2"]] == [0, 0, 1]
    # tests/polynomial_tests.rs:221-224, src/commitments.rs:509
    assert h(k["horner_3x2_2x_1_at_5"]) == 86
    # src/commitments.rs:570-586
    assert [h(c) for c in k["division_x2m1_by_xm1"]] == [1, 1]
    # tests/polynomial_tests.rs:103-111
    assert h(k["mle_1234_half_half"]) == 10 * pow(4, -1, R) % R
    # tests/polynomial_tests.rs:126-130
    assert [h(c) for c in k["mle_1234_partial_1"]] == [2, 4]
    # tests/polynomial_tests.rs:86-89
    for i, pt in enumerate(([0, 0], [1, 0], [0, 1], [1, 1])):
        assert po.mle_evaluate([1, 2, 3, 4], pt) == i + 1


def test_setup_sizes():
    p = po.setup_params(4, with_srs=False)
    assert p["max_operations"] == 64  # src/utils.rs:282
    assert p["n_powers"] == 65


# ---------------------------------------------------------------- golden fixtures == oracle
def test_golden_setup_params(golden):
    for L, s in golden["setup_params"].items():
        p = po.setup_params(int(L))
        assert hex(p["tau"]) == hex(h(s["tau"]))
        assert p["fiat_shamir_seed"].hex() == s["fiat_shamir_seed"]
        g = [None if P is None else (h(P[0]), h(P[1])) for P in s["g1_powers"]]
        assert g == p["g1_powers"]
        assert all(po.g1_is_on_curve(P) for P in g)
        tau = p["tau"]
        for i in (0, 1, len(g) - 1):
            assert g[i] == po.affine_mul(po.G1_GEN, pow(tau, i, R))


def _check_kzg_identities(tau, poly, C, z, v, pi):
    """C = P(tau) G and pi (tau - z) = C - v G (the pairing equation, via the trapdoor)."""
    assert C == po.affine_mul(po.G1_GEN, po.horner_eval(poly, tau))
    assert v == po.horner_eval(poly, z)
    lhs = po.affine_mul(pi, (tau - z) % R) if pi is not None else None
    assert lhs == po.affine_add(C, po.g1_neg(po.affine_mul(po.G1_GEN, v)))


@pytest.mark.parametrize("name", ["demo_L3", "small_trace_L3", "empty_L2", "max_ops_L2", "single_op_L2"])
def test_golden_twist_identities(golden, name):
    case = golden["twist"][name]
    p = po.setup_params(case["log_size"], with_srs=False)
    pr = case["proof"]
    ap = [h(c) for c in case["address_poly"]]
    vp = [h(c) for c in case["value_poly"]]
    # interpolants reproduce the padded vectors at the nodes
    ops = case["ops"]
    n = len(ap)
    addrs = [a for (_, a, _) in ops] + [0] * (n - len(ops))
    vals = [h(v) for (_, _, v) in ops] + [0] * (n - len(ops))
    assert [po.horner_eval(ap, i) for i in range(n)] == addrs
    assert [po.horner_eval(vp, i) for i in range(n)] == vals
    for r in pr["round_polynomials"]:
        assert [h(c) for c in r] == [0, 0, 0, 0]
    assert h(pr["final_evaluation"]) == 0
    if pr["opening_point"] is not None:
        z = h(pr["opening_point"])
        for poly, C, v, pi in zip((ap, vp), (pr["address_commitment"], pr["value_commitment"]),
                                  pr["final_evaluations"], pr["opening_proofs"]):
            Cp = None if C is None else (h(C[0]), h(C[1]))
            pip = None if pi is None else (h(pi[0]), h(pi[1]))
            _check_kzg_identities(p["tau"], poly, Cp, z, h(v), pip)


def test_python_and_c_oracles_agree(golden):
    for L in (2, 3):
        pp = po.setup_params(L)
        cp = co.setup_params(L)
        assert pp["tau"] == cp["tau"] and pp["fiat_shamir_seed"] == cp["fiat_shamir_seed"]
        assert [co.g1_from_limbs(r) for r in cp["g1_limbs"]] == pp["g1_powers"]
    for name in ("demo_L3", "repeated_L2", "only_reads_L2"):
        case = golden["twist"][name]
        cp = co.setup_params(case["log_size"])
        ops = [(w, a, h(v)) for (w, a, v) in case["ops"]]
        st, pr = co.twist_prove(cp, ops)
        assert st == 0
        g = case["proof"]
        assert pr["address_commitment"] == (None if g["address_commitment"] is None else
                                            tuple(h(x) for x in g["address_commitment"]))
        assert [hex(v) for v in pr["final_evaluations"]] == [hex(h(v)) for v in g["final_evaluations"]]
        assert pr["opening_point"] == (None if g["opening_point"] is None else h(g["opening_point"]))
    for name, case in golden["shout"].items():
        cp = co.setup_params(case["log_size"])
        st, pr = co.shout_prove(cp, [h(e) for e in case["entries"]], case["lookups"])
        assert st == 0
        g = case["proof"]
        assert pr["index_commitment"] == (None if g["index_commitment"] is None else
                                          tuple(h(x) for x in g["index_commitment"]))
        assert pr["opening_proofs"] == [None if P is None else (h(P[0]), h(P[1])) for P in g["opening_proofs"]]


def test_c_oracle_sumcheck_matches_python(golden):
    x1 = co.fr_array([0, 1, 0, 1])
    x2 = co.fr_array([0, 0, 1, 1])
    st, rounds, fin, chal = co.sumcheck_prove([x1, x2], 2, 1, [(1, [0, 1])], prefix=b"")
    assert st == 0
    g = golden["sumcheck_x1x2"]
    assert [co.fr_ints(r) for r in rounds] == [[h(c) for c in r] for r in g["rounds"]]
    assert co.fr_ints(fin)[0] == h(g["final"])
    assert co.fr_ints(chal) == [h(c) for c in g["challenges"]]


def test_c_oracle_error_paths():
    cp = co.setup_params(1)  # max 8 ops (tests/twist_tests.rs:180-196)
    ops = [(1, i % 2, i + 1) for i in range(10)]
    st, _ = co.twist_prove(cp, ops)
    assert st == 1
    # commit beyond the SRS: Commitment error (src/commitments.rs:166-170)
    st, _ = co.commit(cp["g1_limbs"], co.fr_array(list(range(cp["n_powers"] + 1))))
    assert st == 4
