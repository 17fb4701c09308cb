"""The drop-in boundary driven from plain C (examples/prove.c: no Python, no torch in the process)
-- the calls a Rust binding of Twist::prove / Shout::prove makes (INTEGRATION.md sections 1, 2b).
Its serialized proofs must equal, byte for byte, the Python mirror's proofs of the same
ProtocolBenchmarks workloads (src/benchmarks.rs:88-99 trace, :167-177 lookups), which
test_gpu_parity.py pins to the golden proofs and test_gpu_configs.py to the trapdoor identities
at C3 / C4; the C host's verifier call (Twist::verify / Shout::verify, src/twist.rs:255-304,
src/shout.rs:225-274) must accept them."""
import json
import os
import subprocess

import numpy as np
import pytest

import twist_and_shout as ts

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "multilinear-map-cryptography_amd", "examples", "prove")


def run_c_host(*args, timeout=240):
    assert os.path.exists(EXE), "build() builds examples/prove"
    r = subprocess.run([EXE] + [str(a) for a in args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def python_twist(L, n, mem):
    pp, _ = ts.setup_params(L)
    return ts.Twist(pp).prove_soa(*ts.bench_trace(mem, n)).serialize(True)


def python_shout(L, T, m):
    pp, _ = ts.setup_params(L)
    entries = ts.fr_from_u64_array(np.arange(T, dtype=np.uint64) ** 2)
    idx = np.arange(m, dtype=np.uint64) % np.uint64(max(T, 1))
    return ts.Shout(pp).prove_arrays(entries, idx).serialize(True)


@pytest.mark.parametrize("L,n,mem", [(3, 0, 8), (8, 256, 256), (8, 1000, 256), (14, 1 << 16, 1 << 14)])
def test_c_host_twist_equals_python_mirror(L, n, mem):
    d = run_c_host("twist", L, n, mem)
    assert d["ok"] == 1 and d["n"] == n
    assert bytes.fromhex(d["proof"]) == python_twist(L, n, mem)


@pytest.mark.parametrize("L,T,m", [(3, 8, 8), (8, 256, 256), (8, 100, 1000), (14, 1 << 12, 1 << 16)])
def test_c_host_shout_equals_python_mirror(L, T, m):
    d = run_c_host("shout", L, T, m)
    assert d["ok"] == 1 and d["m"] == m
    assert bytes.fromhex(d["proof"]) == python_shout(L, T, m)


def test_c_host_c4_twist_dropin_rate():
    """C4 from C: setup_params(22), 2^24 ProtocolBenchmarks ops on host buffers, 3 proves (the
    first untimed); the proof verifies and equals the Python mirror's."""
    d = run_c_host("twist", 22, 1 << 24, 1 << 22, 3)
    assert d["ok"] == 1
    print(f"C host drop-in C4: {d['prove_ms']:.2f} ms = {d['per_sec'] / 1e6:.1f} M ops/s")
    assert bytes.fromhex(d["proof"]) == python_twist(22, 1 << 24, 1 << 22)


def test_c_host_c3_shout_dropin_rate():
    """C3 from C: setup_params(18), a 2^20-entry table of squares, 2^20 lookups i % 2^20 on host
    buffers, 6 proves (the first untimed)."""
    d = run_c_host("shout", 18, 1 << 20, 1 << 20, 6)
    assert d["ok"] == 1
    print(f"C host drop-in C3: {d['prove_ms']:.2f} ms = {d['per_sec'] / 1e6:.1f} M lookups/s")
    assert bytes.fromhex(d["proof"]) == python_shout(18, 1 << 20, 1 << 20)
