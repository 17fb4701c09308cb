"""The radix-2^29 field arithmetic of the accumulation experiment (tools/f29.hpp) checked on the host:
tests/native/f29_host_check.cpp compares its mixed addition with bn254.hpp's radix-2^32 one on
20000 chains that include coordinates next to the modulus (the case a too-small subtraction offset
got wrong)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_f29_madd_matches_radix32(tmp_path):
    exe = str(tmp_path / "f29_host_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "multilinear-map-cryptography_amd", "csrc"), "-I", os.path.join(ROOT, "tools"),
                           "-o", exe, os.path.join(ROOT, "tests", "native", "f29_host_check.cpp")])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad 0 of 20000" in out.stdout
