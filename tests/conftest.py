import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "nasp-key-value-engine_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, ORACLE, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def built():
    """Make sure the product library and the oracle library exist (both build on CPU)."""
    subprocess.check_call(["make", "-s", "-C", PKG])
    subprocess.check_call(["make", "-s", "-C", ORACLE, "all"])
    return True


@pytest.fixture(scope="session")
def oracle(built):
    from oracle_ctypes import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(GOLDEN, "libstdcxx_vectors.json")) as f:
        lib = json.load(f)
    with open(os.path.join(GOLDEN, "msvc_filters.json")) as f:
        msvc = json.load(f)
    return lib, msvc
