"""Host build of tests/cpp/test_math.cpp: the shared index arithmetic the
kernels use (bloom_math.h: reciprocal remainder, incremental indices, word-stream
hashing with the seed-prefix splice, every misalignment; the Merkle decimal
conversion and parent hash) against plain 64-bit arithmetic and the oracle."""
import os
import subprocess

from conftest import ORACLE, REPO


def test_bloom_math_host(tmp_path, built):
    exe = tmp_path / "test_math"
    src = os.path.join(REPO, "tests", "cpp", "test_math.cpp")
    subprocess.check_call(["gcc", "-O2", "-c", os.path.join(ORACLE, "bloom_oracle.c"),
                           "-o", str(tmp_path / "bo.o")])
    subprocess.check_call(["g++", "-O2", "-std=c++17", src, str(tmp_path / "bo.o"), "-o", str(exe), "-lm"])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "hash mismatches: 0" in out.stdout
    assert "merkle mismatches: 0" in out.stdout
