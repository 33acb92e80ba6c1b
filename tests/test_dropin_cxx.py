"""The C++ drop-in class (host/BloomFilter.h): tests/cpp/test_dropin.cpp runs the
reference callers' usage patterns and checks every image against the oracle --
on the CPU box with no device visible (every batch then built on the host, large
ones after a std::cerr line: SURVEY §8(b)'s fallback), and on the GPU box, where
large batches must reach the device and small ones must not."""
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


def test_dropin_without_gpu(tmp_path, built):
    """HIP_VISIBLE_DEVICES= (empty): no device; the class still produces the
    reference bytes, and says on stderr that it built on the host."""
    exe = build_dropin(tmp_path)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "devices: 0" in out.stdout and "drop-in OK" in out.stdout
    assert "[BloomFilter] GPU build failed (no HIP device visible)" in out.stderr
    assert out.stderr.count("GPU build failed") == 1, "one note per process, not one per filter"


@pytest.mark.gpu
def test_dropin_on_gpu(tmp_path, built):
    exe = build_dropin(tmp_path)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "devices: 0" not in out.stdout, "the GPU test ran without a device"
    assert "drop-in OK" in out.stdout
    # the only device failures are the injected ones (NB_FAIL_BUILDS, section 9)
    fails = [l for l in out.stderr.splitlines() if "GPU build failed" in l]
    assert len(fails) == 2 and all("injected" in l for l in fails), out.stderr
