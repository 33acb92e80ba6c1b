"""The C++ drop-in class (host/BloomFilter.h): it compiles and links against the
C ABI library on CPU; on the GPU box tests/cpp/test_dropin.cpp runs the
reference callers' usage patterns and checks every image against the oracle."""
import os
import subprocess

import pytest

from conftest import ORACLE, PKG, REPO


def build_dropin(tmp_path):
    exe = tmp_path / "test_dropin"
    bo = tmp_path / "bo.o"
    subprocess.check_call(["gcc", "-O2", "-c", os.path.join(ORACLE, "bloom_oracle.c"), "-o", str(bo)])
    libdir = os.path.join(PKG, "build")
    subprocess.check_call([
        "g++", "-O2", "-std=c++17", "-Wall",
        os.path.join(REPO, "tests", "cpp", "test_dropin.cpp"),
        os.path.join(PKG, "host", "BloomFilter.cpp"), str(bo),
        "-L" + libdir, "-lnasp_bloom", "-Wl,-rpath," + libdir, "-o", str(exe)])
    return exe


def test_dropin_compiles_and_links(tmp_path, built):
    assert build_dropin(tmp_path).exists()


@pytest.mark.gpu
def test_dropin_on_gpu(tmp_path, built):
    exe = build_dropin(tmp_path)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    if out.returncode == 77:
        pytest.skip("no GPU")
    assert out.returncode == 0, out.stdout + out.stderr
    assert "drop-in OK" in out.stdout
