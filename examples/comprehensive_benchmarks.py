"""examples/comprehensive_benchmarks.rs on the MI355X prover: the same modes and flags.

    python examples/comprehensive_benchmarks.py [quick|full|default|dev|custom|twist-only|shout-only|help]
        [--min-log-size N] [--max-log-size N] [--operations N]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "multilinear-map-cryptography_amd"))

from twist_and_shout.benchmarks import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
