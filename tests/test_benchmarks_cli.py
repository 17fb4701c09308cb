"""ProtocolBenchmarks / comprehensive_benchmarks parity: schedules,
estimates and CLI validation on CPU (src/benchmarks.rs, examples/comprehensive_benchmarks.rs);
the dev suite end to end (GPU prove, host verify) under the gpu marker."""
import pytest

from twist_and_shout import benchmarks as B


def test_operation_schedule_matches_reference():
    # src/benchmarks.rs:55-62: size/2 up to 64, size/4 up to 512, size/8 beyond
    assert [B._scaled_ops(1 << k) for k in range(4, 12)] == [8, 16, 32, 32, 64, 128, 128, 256]


def test_estimates_match_reference_formulas():
    assert B.ProtocolBenchmarks.estimate_proof_size(5, 2) == 128 + 5 * 128 + 2 * 64
    assert B.ProtocolBenchmarks.estimate_memory_usage(16, 8) == 16 * 32 + 8 * 96
    r = B.BenchmarkResults(0.5, 2.0, 0.25, 10, 100, 0)
    assert r.prove_ops_per_second() == 50 and r.verify_ops_per_second() == 400 and r.total_time() == 2.75


@pytest.mark.parametrize("args,want", [
    ([], (4, 8, 256)),
    (["--min-log-size", "3", "--max-log-size", "9", "--operations", "77"], (3, 9, 77)),
    (["--operations"], (4, 8, 256)),  # a trailing flag without a value is ignored, as in the reference
])
def test_parse_options(args, want):
    assert B.parse_options(args) == want


@pytest.mark.parametrize("args,msg", [
    (["--min-log-size", "9", "--max-log-size", "5"], "cannot be greater"),
    (["--min-log-size", "1"], "between 2 and 20"),
    (["--max-log-size", "21"], "between 2 and 20"),
    (["--operations", "x"], "Invalid operations value"),
    (["--bogus"], "Unknown argument"),
])
def test_parse_options_rejects(args, msg):
    with pytest.raises(B.CliError, match=msg):
        B.parse_options(args)


def test_cli_help_and_unknown_mode(capsys):
    assert B.main(["help"]) == 0
    out = capsys.readouterr().out
    for mode in ("quick", "full", "default", "dev", "custom", "twist-only", "shout-only"):
        assert mode in out
    assert B.main(["nope"]) == 1
    assert B.main(["custom", "--min-log-size", "7", "--max-log-size", "4"]) == 1


def test_ratio_prints_like_f64_division():
    assert B._ratio(3, 2) == 1.5 and B._ratio(3, 0) == float("inf")
    assert B._ratio(0, 0) != B._ratio(0, 0)  # NaN


@pytest.mark.gpu
def test_dev_suite_end_to_end(capsys):
    tw, sh, (t, s) = B.ProtocolBenchmarks.run_dev_benchmark()
    out = capsys.readouterr().out
    assert "Twist Protocol Scaling Analysis" in out and "Performance Ratios" in out
    assert [sz for sz, _ in tw] == [16, 32] and [sz for sz, _ in sh] == [16, 32]
    assert [r.num_operations for _, r in tw] == [8, 16]
    assert t.num_operations == 32 and s.num_operations == 32
    # log2(next_pow2(n_ops)) sum-check rounds, two openings: Twist 2^4 with 8 ops -> 3 rounds
    assert tw[0][1].proof_size == B.ProtocolBenchmarks.estimate_proof_size(3, 2)
    assert all(r.prove_time > 0 and r.verify_time > 0 for _, r in tw + sh)


@pytest.mark.gpu
def test_optimized_and_single_mode_cli(capsys):
    out = B.ProtocolBenchmarks.run_optimized_benchmark(6, 7)
    assert [(ls, t.num_operations, s.num_operations) for ls, t, s in out] == [(6, 128, 128), (7, 64, 64)]
    # at 2^4 the schedule asks 512 ops > max_operations = 64 (src/utils.rs:80): the reference's
    # prove returns InvalidParameters there (src/twist.rs:108) and its unwrap panics
    with pytest.raises(B.TwistAndShoutError):
        B.ProtocolBenchmarks.run_optimized_benchmark(4, 4)
    t, s = B.run_demo()
    assert t.num_operations == s.num_operations == 16
    assert B.main(["twist-only", "--min-log-size", "4", "--max-log-size", "4"]) == 0
    assert B.main(["shout-only", "--min-log-size", "4", "--max-log-size", "4"]) == 0
