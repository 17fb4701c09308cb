"""Proof wire format: G1 / Fr canonical encodings and whole proofs,
product (csrc/serialize.cpp) against the oracle restatement of ark-serialize 0.4 semantics,
round trips, and rejection of malformed bytes.  Host only (no GPU)."""
import pytest

from oracle import pyoracle as po

import twist_and_shout as ts

R, P = po.R_MOD, po.P_MOD


def h(x):
    return int(x, 16)


def g1h(Pt):
    return None if Pt is None else (h(Pt[0]), h(Pt[1]))


POINTS = [None, po.G1_GEN, po.g1_neg(po.G1_GEN), po.affine_mul(po.G1_GEN, 123456789),
          po.affine_mul(po.G1_GEN, R - 5)]


@pytest.mark.parametrize("compressed", [True, False])
def test_g1_encoding_matches_oracle_and_round_trips(compressed):
    for Pt in POINTS:
        b = ts.g1_serialize(Pt, compressed)
        assert b == po.g1_serialize(Pt, compressed)
        assert ts.g1_deserialize(b, compressed) == Pt


def test_generator_encoding():
    # x = 1 little-endian, y = 2 <= -2: no flag
    assert ts.g1_serialize(po.G1_GEN) == bytes([1]) + bytes(31)
    assert ts.g1_serialize(None) == bytes(31) + bytes([0x40])


def test_malformed_g1_rejected():
    bad_x = (P).to_bytes(32, "little")  # x = p (not canonical)
    with pytest.raises(ts.InvalidParameters):
        ts.g1_deserialize(bad_x)
    with pytest.raises(ts.InvalidParameters):
        ts.g1_deserialize(bytes(31) + bytes([0xC0]))  # both flags
    not_on_curve = (0).to_bytes(32, "little")  # x = 0: 3 is not a square mod p
    with pytest.raises(ts.InvalidParameters):
        ts.g1_deserialize(not_on_curve)
    unc = bytearray(ts.g1_serialize(po.G1_GEN, False))
    unc[32] ^= 1  # y = 3
    with pytest.raises(ts.InvalidParameters):
        ts.g1_deserialize(bytes(unc), False)


def _twist(case):
    pr = case["proof"]
    return ts.TwistProof(
        ts.KZGCommitmentValue(g1h(pr["address_commitment"])), ts.KZGCommitmentValue(g1h(pr["value_commitment"])),
        ts.SumCheckProof([[h(c) for c in r] for r in pr["round_polynomials"]], h(pr["final_evaluation"])),
        [ts.KZGProof(g1h(p)) for p in pr["opening_proofs"]], [h(v) for v in pr["final_evaluations"]])


@pytest.mark.parametrize("compressed", [True, False])
def test_proof_bytes_match_oracle_and_round_trip(golden, compressed):
    for name, case in golden["twist"].items():
        pf = _twist(case)
        b = pf.serialize(compressed)
        want = po.proof_serialize([pf.address_commitment.commitment, pf.value_commitment.commitment],
                                  pf.consistency_proof.round_polynomials, pf.consistency_proof.final_evaluation,
                                  [p.proof for p in pf.opening_proofs], pf.final_evaluations, compressed)
        assert b == want, name
        assert ts.TwistProof.deserialize(b, compressed) == pf, name
    for name, case in golden["shout"].items():
        pr = case["proof"]
        sp = ts.ShoutProof(
            ts.KZGCommitmentValue(g1h(pr["table_commitment"])), ts.KZGCommitmentValue(g1h(pr["index_commitment"])),
            ts.SumCheckProof([[h(c) for c in r] for r in pr["round_polynomials"]], h(pr["final_evaluation"])),
            [ts.KZGProof(g1h(p)) for p in pr["opening_proofs"]], [h(v) for v in pr["final_evaluations"]])
        assert ts.ShoutProof.deserialize(sp.serialize(compressed), compressed) == sp, name


def test_truncated_and_trailing_bytes_rejected(golden):
    b = _twist(golden["twist"]["demo_L3"]).serialize()
    with pytest.raises(ts.InvalidParameters):
        ts.TwistProof.deserialize(b[:-1])
    with pytest.raises(ts.InvalidParameters):
        ts.TwistProof.deserialize(b + b"\0")
