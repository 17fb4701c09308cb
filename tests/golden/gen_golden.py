"""Generate tests/golden/*.json from the CPU oracle (oracle/pyoracle.py, oracle/liboracle.so).

There is no runnable reference here (Rust crate, no toolchain), so these fixtures are the
oracle's outputs on the reference's own test inputs (tests/*.rs, examples/demo.rs,
src/benchmarks.rs generators).  The oracle itself is pinned by the reference KATs and the
published ChaCha20 / SipHash vectors (tests/test_oracle.py).

Run:  python tests/golden/gen_golden.py     (a few seconds; C1 uses the C oracle)
"""

from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import coracle as co  # noqa: E402
from oracle import pyoracle as po  # noqa: E402


def hx(x: int) -> str:
    return "0x%064x" % x


def g1hex(P):
    return None if P is None else [hx(P[0]), hx(P[1])]


def proof_json(pr: dict, names):
    return {
        names[0]: g1hex(pr[names[0]]),
        names[1]: g1hex(pr[names[1]]),
        "round_polynomials": [[hx(c) for c in r] for r in pr["round_polynomials"]],
        "final_evaluation": hx(pr["final_evaluation"]),
        "opening_proofs": [g1hex(p) for p in pr["opening_proofs"]],
        "final_evaluations": [hx(v) for v in pr["final_evaluations"]],
        "opening_point": None if pr["opening_point"] is None else hx(pr["opening_point"]),
        "sumcheck_challenges": [hx(c) for c in pr["sumcheck_challenges"]],
    }


# traces from /root/reference/tests/twist_tests.rs, src/twist.rs tests, examples/demo.rs
TWIST_CASES = {
    "demo_L3": (3, 8, [("w", 0, 42), ("w", 1, 100), ("r", 0), ("r", 1), ("w", 0, 43), ("r", 0)]),
    "small_trace_L3": (3, 8, [("w", 0, 10), ("w", 1, 20), ("r", 0), ("w", 2, 30), ("r", 1), ("r", 2)]),
    "empty_L2": (2, 4, []),
    "only_reads_L2": (2, 4, [("r", 0), ("r", 1), ("r", 2), ("r", 3)]),
    "only_writes_L2": (2, 4, [("w", 0, 1), ("w", 1, 2), ("w", 2, 3), ("w", 3, 4)]),
    "repeated_L2": (2, 4, [("w", 0, 100), ("r", 0), ("w", 0, 200), ("r", 0), ("w", 0, 300), ("r", 0)]),
    "max_ops_L2": (2, 4, [("w", i % 4, i + 1) for i in range(15)]),
    "unit_L4": (4, 16, [("w", 0, 42), ("w", 1, 73), ("r", 0)]),
    "single_op_L2": (2, 4, [("w", 3, 7)]),
}

# tables from tests/shout_tests.rs and examples/demo.rs
SHOUT_CASES = {
    "demo_squares_L3": (3, [i * i for i in range(8)], [3, 5, 0, 7]),
    "single_entry_L2": (2, [99], [0, 0, 0]),
    "no_lookups_L2": (2, [1, 2, 3], []),
    "ragged_table_L3": (3, [5, 10, 15, 20, 25], [4, 0, 2, 2, 1]),
    "sixteen_L4": (4, [i * 3 + 1 for i in range(16)], [i % 16 for i in range(16)]),
}


def main():
    out = {}
    # setup_params: tau, seed and SRS heads
    setups = {}
    params_cache = {}
    for L in (1, 2, 3, 4):
        p = po.setup_params(L)
        params_cache[L] = p
        setups[str(L)] = {
            "tau": hx(p["tau"]),
            "fiat_shamir_seed": p["fiat_shamir_seed"].hex(),
            "max_operations": p["max_operations"],
            "n_powers": p["n_powers"],
            "g1_powers": [g1hex(P) for P in p["g1_powers"]],
        }
    out["setup_params"] = setups
    # KATs restated from the reference tests
    out["kats"] = {
        "lagrange_x2": [hx(c) for c in po.lagrange_interpolate([(0, 0), (1, 1), (2, 4)])],
        "horner_3x2_2x_1_at_5": hx(po.horner_eval([1, 2, 3], 5)),
        "division_x2m1_by_xm1": [hx(c) for c in po.polynomial_division([po.R_MOD - 1, 0, 1], [po.R_MOD - 1, 1])],
        "mle_1234_half_half": hx(po.mle_evaluate([1, 2, 3, 4], [po.fr_inv(2)] * 2)),
        "mle_1234_partial_1": [hx(c) for c in po.mle_partial_evaluate([1, 2, 3, 4], [1])],
    }
    twist = {}
    for name, (L, msz, script) in TWIST_CASES.items():
        ops = po.memory_trace_ops(msz, script)
        pr = po.twist_prove(params_cache[L], ops)
        twist[name] = {"log_size": L, "memory_size": msz,
                       "ops": [[w, a, hx(v)] for (w, a, v) in ops],
                       "proof": proof_json(pr, ("address_commitment", "value_commitment")),
                       "address_poly": [hx(c) for c in pr["address_poly"]],
                       "value_poly": [hx(c) for c in pr["value_poly"]]}
    # C1: setup_params(8), MemoryTrace::new(256), 256 benchmark ops (C oracle: O(N^3) ~5 s)
    cp8 = co.setup_params(8)
    ops = po.benchmark_trace(256, 256)
    st, pr = co.twist_prove(cp8, ops)
    assert st == 0
    twist["C1_bench_256_L8"] = {"log_size": 8, "memory_size": 256, "generator": "benchmarks.rs:88-99",
                                "n_ops": 256,
                                "proof": proof_json(pr, ("address_commitment", "value_commitment"))}
    out["twist"] = twist
    shout = {}
    for name, (L, entries, lookups) in SHOUT_CASES.items():
        pr = po.shout_prove(params_cache[L], entries, lookups)
        shout[name] = {"log_size": L, "entries": [hx(e) for e in entries], "lookups": lookups,
                       "proof": proof_json(pr, ("table_commitment", "index_commitment"))}
    out["shout"] = shout
    # sum-check of f = x1 * x2 over 2 vars, claim 1 (src/sumcheck.rs:221-245) as MLE tables
    tr = po.Transcript(bytes([42] * 32))
    x1 = [0, 1, 0, 1]
    x2 = [0, 0, 1, 1]
    rounds, final, chals = po.sumcheck_prove(
        2, 1, lambda v: po.mle_evaluate(x1, v) * po.mle_evaluate(x2, v) % po.R_MOD, tr)
    out["sumcheck_x1x2"] = {"rounds": [[hx(c) for c in r] for r in rounds], "final": hx(final),
                            "challenges": [hx(c) for c in chals]}
    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
