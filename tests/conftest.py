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


@pytest.fixture
def knobs(built):
    """Set library knobs (nb_set_knob) for one test; the previous values come back
    afterwards.  knobs(NB_BUILD_PATH="tiled", NB_CHUNK_KEYS=70000)."""
    import nasp_bloom as nbm
    saved = {}

    def set_(**kv):
        for k, v in kv.items():
            saved.setdefault(k, nbm.get_knob(k))
            nbm.set_knob(k, v)
    yield set_
    for k, v in saved.items():
        nbm.set_knob(k, v)
