"""The drop-in boundary driven from plain C (examples/twist_prove.c: no Python, no torch in the
process) -- the calls a Rust binding of Twist::prove makes.  Its
serialized proof must equal, byte for byte, the Python mirror's proof of the same
ProtocolBenchmarks trace (src/benchmarks.rs:88-99), which test_gpu_parity.py pins to the golden
C1 proof and test_gpu_configs.py to the trapdoor identities at C4; the C host's verifier call
(Twist::verify, src/twist.rs:255-304) must accept it."""
import json
import os
import subprocess

import pytest

import twist_and_shout as ts

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "multilinear-map-cryptography_amd", "examples", "twist_prove")


def run_c_host(*args, timeout=240):
    assert os.path.exists(EXE), "build() builds examples/twist_prove"
    r = subprocess.run([EXE] + [str(a) for a in args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("L,n,mem", [(3, 0, 8), (8, 256, 256), (8, 1000, 256), (14, 1 << 16, 1 << 14)])
def test_c_host_proof_equals_python_mirror(L, n, mem):
    d = run_c_host(L, n, mem)
    assert d["ok"] == 1 and d["n_ops"] == n
    pp, _ = ts.setup_params(L)
    want = ts.Twist(pp).prove_soa(*ts.bench_trace(mem, n)).serialize(True)
    assert bytes.fromhex(d["proof"]) == want


def test_c_host_c4_dropin_rate():
    """C4 from C: setup_params(22), 2^24 ProtocolBenchmarks ops on host buffers, 3 proves (the
    first untimed); the proof verifies and equals the Python mirror's."""
    d = run_c_host(22, 1 << 24, 1 << 22, 3)
    assert d["ok"] == 1
    print(f"C host drop-in C4: {d['prove_ms']:.2f} ms = {d['ops_per_sec'] / 1e6:.1f} M ops/s")
    pp, _ = ts.setup_params(22)
    want = ts.Twist(pp).prove_soa(*ts.bench_trace(1 << 22, 1 << 24)).serialize(True)
    assert bytes.fromhex(d["proof"]) == want
