"""ProtocolBenchmarks (src/benchmarks.rs:46-366) and the comprehensive_benchmarks CLI
(examples/comprehensive_benchmarks.rs) on the MI355X prover -- SURVEY 8(f) row 4.

Same schedules, traces and tables as the reference: setup_params(log_size) per size, the
ProtocolBenchmarks trace (writes i*42 at i % mem on every third op, reads (i/2) % mem), the
squares lookup table, prove then verify (asserting validity), proof size and memory usage
estimated as the reference estimates them.  Run as

    python -m twist_and_shout.benchmarks [quick|full|dev|custom|twist-only|shout-only|help]
        [--min-log-size N] [--max-log-size N] [--operations N]
"""
import sys
import time
from dataclasses import dataclass
from typing import List, Tuple

from . import LookupTable, Shout, Twist, TwistAndShoutError, bench_trace, setup_params


@dataclass
class BenchmarkResults:
    """src/benchmarks.rs:8-22 (times in seconds)."""
    setup_time: float
    prove_time: float
    verify_time: float
    proof_size: int
    num_operations: int
    memory_usage: int

    def prove_ops_per_second(self) -> float:
        return self.num_operations / self.prove_time if self.prove_time > 0 else float("inf")

    def verify_ops_per_second(self) -> float:
        return self.num_operations / self.verify_time if self.verify_time > 0 else float("inf")

    def total_time(self) -> float:
        return self.setup_time + self.prove_time + self.verify_time


def _scaled_ops(size: int) -> int:
    """src/benchmarks.rs:55-62, :133-140: 50 % / 25 % / 12.5 % utilisation by size."""
    if size <= 64:
        return size // 2
    if size <= 512:
        return size // 4
    return size // 8


def _ratio(a: int, b: int) -> float:
    """f64 division as the reference prints it (x/0 -> inf, 0/0 -> NaN)."""
    if b:
        return a / b
    return float("nan") if a == 0 else float("inf")


def _ms(t: float) -> int:
    return int(t * 1000)  # Duration::as_millis truncates


class ProtocolBenchmarks:
    @staticmethod
    def benchmark_twist_single(log_size: int, num_operations: int) -> BenchmarkResults:
        t0 = time.perf_counter()
        pp, vp = setup_params(log_size)
        twist = Twist(pp)
        setup_time = time.perf_counter() - t0
        memory_size = 1 << log_size
        addr, val, isw = bench_trace(memory_size, num_operations)
        t1 = time.perf_counter()
        proof = twist.prove_soa(addr, val, isw)
        prove_time = time.perf_counter() - t1
        t2 = time.perf_counter()
        ok = Twist.verify(proof, vp)
        verify_time = time.perf_counter() - t2
        assert ok, "Proof verification failed"
        return BenchmarkResults(setup_time, prove_time, verify_time,
                                ProtocolBenchmarks.estimate_proof_size(len(proof.consistency_proof.round_polynomials),
                                                                       len(proof.opening_proofs)),
                                num_operations, ProtocolBenchmarks.estimate_memory_usage(memory_size, num_operations))

    @staticmethod
    def benchmark_shout_single(log_size: int, num_lookups: int) -> BenchmarkResults:
        t0 = time.perf_counter()
        pp, vp = setup_params(log_size)
        shout = Shout(pp)
        setup_time = time.perf_counter() - t0
        table_size = 1 << log_size
        table = LookupTable([i * i for i in range(table_size)])
        for i in range(num_lookups):
            table.lookup(i % table_size)
        t1 = time.perf_counter()
        proof = shout.prove(table)
        prove_time = time.perf_counter() - t1
        t2 = time.perf_counter()
        ok = Shout.verify(proof, vp)
        verify_time = time.perf_counter() - t2
        assert ok, "Proof verification failed"
        return BenchmarkResults(setup_time, prove_time, verify_time,
                                ProtocolBenchmarks.estimate_proof_size(len(proof.lookup_proof.round_polynomials),
                                                                       len(proof.opening_proofs)),
                                len(table.lookups), ProtocolBenchmarks.estimate_memory_usage(table_size, num_lookups))

    @staticmethod
    def benchmark_twist_scaling_range(min_log_size: int, max_log_size: int) -> List[Tuple[int, BenchmarkResults]]:
        out = []
        for log_size in range(min_log_size, max_log_size + 1):
            size = 1 << log_size
            n = _scaled_ops(size)
            print(f"  Testing Twist with memory size: {size} (2^{log_size}), operations: {n}")
            out.append((size, ProtocolBenchmarks.benchmark_twist_single(log_size, n)))
        return out

    @staticmethod
    def benchmark_shout_scaling_range(min_log_size: int, max_log_size: int) -> List[Tuple[int, BenchmarkResults]]:
        out = []
        for log_size in range(min_log_size, max_log_size + 1):
            size = 1 << log_size
            n = _scaled_ops(size)
            print(f"  Testing Shout with table size: {size} (2^{log_size}), lookups: {n}")
            out.append((size, ProtocolBenchmarks.benchmark_shout_single(log_size, n)))
        return out

    @staticmethod
    def benchmark_twist_scaling():
        return ProtocolBenchmarks.benchmark_twist_scaling_range(4, 8)

    @staticmethod
    def benchmark_shout_scaling():
        return ProtocolBenchmarks.benchmark_shout_scaling_range(4, 8)

    @staticmethod
    def comparative_benchmark(log_size: int, num_operations: int):
        return (ProtocolBenchmarks.benchmark_twist_single(log_size, num_operations),
                ProtocolBenchmarks.benchmark_shout_single(log_size, num_operations))

    @staticmethod
    def run_comprehensive_benchmark_with_params(min_log_size: int, max_log_size: int, num_ops: int):
        print("Twist and Shout Protocol Benchmark Suite")
        print("============================================\n")
        print("Twist Protocol Scaling Analysis:")
        tw = ProtocolBenchmarks.benchmark_twist_scaling_range(min_log_size, max_log_size)
        ProtocolBenchmarks.print_scaling_results("Twist", tw)
        print("\nShout Protocol Scaling Analysis:")
        sh = ProtocolBenchmarks.benchmark_shout_scaling_range(min_log_size, max_log_size)
        ProtocolBenchmarks.print_scaling_results("Shout", sh)
        cmp_log = (min_log_size + max_log_size) // 2
        print(f"\nComparative Analysis (Memory/Table Size: {1 << cmp_log}):")
        t, s = ProtocolBenchmarks.comparative_benchmark(cmp_log, num_ops)
        ProtocolBenchmarks.print_comparative_results(t, s)
        return tw, sh, (t, s)

    @staticmethod
    def run_comprehensive_benchmark():
        return ProtocolBenchmarks.run_comprehensive_benchmark_with_params(4, 8, 256)

    @staticmethod
    def run_quick_benchmark():
        return ProtocolBenchmarks.run_comprehensive_benchmark_with_params(4, 6, 64)

    @staticmethod
    def run_dev_benchmark():
        return ProtocolBenchmarks.run_comprehensive_benchmark_with_params(4, 5, 32)

    @staticmethod
    def run_optimized_benchmark(min_log_size: int, max_log_size: int):
        print("Optimized Twist and Shout Protocol Benchmark Suite")
        print("======================================================\n")
        out = []
        for log_size in range(min_log_size, max_log_size + 1):
            if log_size < 4:  # the reference's usize shift underflows below 2^4
                raise ValueError("run_optimized_benchmark needs log sizes >= 4")
            n = max(32, 512 // (1 << (log_size - 4)))
            print(f"Protocol Comparison at size {1 << log_size} (2^{log_size}) with {n} operations:")
            t, s = ProtocolBenchmarks.comparative_benchmark(log_size, n)
            print("Protocol | Prove(ms) | Verify(ms) | Proof(KB) | Ops/sec | Memory(KB)")
            print("---------|-----------|------------|-----------|---------|----------")
            for name, r in (("Twist", t), ("Shout", s)):
                print(f"{name:<8} | {_ms(r.prove_time)}      | {_ms(r.verify_time)}       | "
                      f"{r.proof_size / 1024.0:.2f}      | {r.prove_ops_per_second():.0f}     | "
                      f"{r.memory_usage / 1024.0:.1f}")
            print()
            out.append((log_size, t, s))
        return out

    @staticmethod
    def print_scaling_results(protocol: str, results):
        print("Size\t| Setup(ms)\t| Prove(ms)\t| Verify(ms)\t| Proof(KB)\t| Ops/sec")
        print("--------|---------------|---------------|---------------|---------------|--------")
        for size, r in results:
            print(f"{size}\t| {_ms(r.setup_time)}\t\t| {_ms(r.prove_time)}\t\t| {_ms(r.verify_time)}\t\t| "
                  f"{r.proof_size / 1024.0:.2f}\t\t| {r.prove_ops_per_second():.0f}")

    @staticmethod
    def print_comparative_results(twist: BenchmarkResults, shout: BenchmarkResults):
        print("Protocol | Prove(ms) | Verify(ms) | Proof(KB) | Ops/sec | Total(ms)")
        print("---------|-----------|------------|-----------|---------|----------")
        for name, r in (("Twist", twist), ("Shout", shout)):
            print(f"{name:<8} | {_ms(r.prove_time)}      | {_ms(r.verify_time)}       | {r.proof_size / 1024.0:.2f}      "
                  f"| {r.prove_ops_per_second():.0f}     | {_ms(r.total_time())}")
        pr = _ratio(_ms(twist.prove_time), _ms(shout.prove_time))
        vr = _ratio(_ms(twist.verify_time), _ms(shout.verify_time))
        print("\nPerformance Ratios (Twist/Shout):")
        print(f"Proving: {pr:.2f}x, Verification: {vr:.2f}x")

    @staticmethod
    def estimate_proof_size(n_rounds: int, n_openings: int) -> int:
        """src/benchmarks.rs:337-353: 2 x 64 + 128 per round + 64 per opening."""
        return 2 * 64 + n_rounds * 128 + n_openings * 64

    @staticmethod
    def estimate_memory_usage(table_size: int, num_operations: int) -> int:
        """src/benchmarks.rs:355-362"""
        return table_size * 32 + num_operations * 32 * 3


def run_demo():
    """examples/benchmark.rs: comparative_benchmark(6, 16) with per-protocol summaries."""
    print("Twist and Shout Protocol Performance Demo")
    print("=============================================\n")
    print("Quick Performance Test (Memory/Table Size: 64, Operations: 16):")
    t, s = ProtocolBenchmarks.comparative_benchmark(6, 16)
    for title, r in (("Twist Protocol (Memory Consistency)", t), ("Shout Protocol (Lookup Verification)", s)):
        print(f"\n{title}:")
        print(f"  Setup Time:       {_ms(r.setup_time)} ms")
        print(f"  Proving Time:     {_ms(r.prove_time)} ms")
        print(f"  Verification Time: {_ms(r.verify_time)} ms")
        print(f"  Operations/sec:    {r.prove_ops_per_second():.0f}")
        print(f"  Proof Size:        {r.proof_size / 1024.0:.2f} KB")
    return t, s


# ----------------------------------------------------------------------------- CLI
HELP = """Twist and Shout comprehensive benchmarks (MI355X prover)

USAGE:
    python -m twist_and_shout.benchmarks [MODE] [OPTIONS]

MODES:
    quick          Quick benchmark (log sizes 4-6, 64 operations)
    full           Full benchmark (log sizes 4-10, 256 operations)
    default        Default benchmark (log sizes 4-8, 256 operations)
    dev            Development mode (log sizes 4-5, 32 operations)
    custom         Custom parameters (use with --min-log-size, --max-log-size, --operations)
    twist-only     Only Twist protocol benchmarks
    shout-only     Only Shout protocol benchmarks
    demo           examples/benchmark.rs: one comparative run at size 64 with 16 operations
    help           Show this help message

OPTIONS:
    --min-log-size N    Minimum log2(table size) (default: 4, min: 2, max: 20)
    --max-log-size N    Maximum log2(table size) (default: 8, min: 2, max: 20)
    --operations N      Number of operations per table size (default: 256)
"""


class CliError(Exception):
    pass


def parse_options(args: List[str]) -> Tuple[int, int, int]:
    """examples/comprehensive_benchmarks.rs:91-152: option parsing and validation."""
    mn, mx, ops = 4, 8, 256
    i = 0
    while i < len(args):
        a = args[i]
        if a in ("--min-log-size", "--max-log-size", "--operations"):
            if i + 1 < len(args):
                try:
                    v = int(args[i + 1])
                except ValueError:
                    raise CliError(f"Invalid {a[2:]} value: {args[i + 1]}") from None
                if a == "--min-log-size":
                    mn = v
                elif a == "--max-log-size":
                    mx = v
                else:
                    ops = v
                i += 1
        else:
            raise CliError(f"Unknown argument: {a}")
        i += 1
    if mn > mx:
        raise CliError(f"min-log-size ({mn}) cannot be greater than max-log-size ({mx})")
    if mn < 2 or mx > 20:
        raise CliError("Log sizes must be between 2 and 20 (table sizes 4 to 1M)")
    return mn, mx, ops


def main(argv: List[str]) -> int:
    if not argv:
        print("Running default comprehensive benchmarks (log sizes 4-8, 256 operations)")
        ProtocolBenchmarks.run_comprehensive_benchmark()
        return 0
    mode, rest = argv[0], argv[1:]
    try:
        if mode in ("help", "--help", "-h"):
            print(HELP)
        elif mode == "demo":
            run_demo()
        elif mode == "quick":
            ProtocolBenchmarks.run_quick_benchmark()
        elif mode == "full":
            ProtocolBenchmarks.run_comprehensive_benchmark_with_params(4, 10, 256)
        elif mode == "default":
            ProtocolBenchmarks.run_comprehensive_benchmark()
        elif mode == "dev":
            ProtocolBenchmarks.run_dev_benchmark()
        elif mode == "custom":
            ProtocolBenchmarks.run_comprehensive_benchmark_with_params(*parse_options(rest))
        elif mode == "twist-only":
            mn, mx, _ = parse_options(rest)
            ProtocolBenchmarks.print_scaling_results("Twist", ProtocolBenchmarks.benchmark_twist_scaling_range(mn, mx))
        elif mode == "shout-only":
            mn, mx, _ = parse_options(rest)
            ProtocolBenchmarks.print_scaling_results("Shout", ProtocolBenchmarks.benchmark_shout_scaling_range(mn, mx))
        else:
            print(f"Unknown mode: {mode}")
            print(HELP)
            return 1
    except CliError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
