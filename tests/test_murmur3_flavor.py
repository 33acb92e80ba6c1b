"""The optional, non-parity NB_FLAVOR_MURMUR3_X64_128 (include/nasp_bloom.h): the
north star's "k MurmurHash3_x64_128 hashes" wording, with h1, h2 = the two halves
of MurmurHash3_x64_128(key, len, (uint32_t)h2_seed) and the reference's
(h1 + i*h2) % m closure.  It is NOT the reference filter (BloomFilter.cpp uses
std::hash); parity here means: the oracle restatement equals the REAL reference
MurmurHash3.cpp (tests/golden/murmur3_vectors.json, made by
tests/golden/gen_murmur3_golden.py from oracle/_ref/libref_murmur3.so), and the
library's host path equals the oracle.  The device path is in test_gpu_parity.py."""
import json
import os

import numpy as np

from conftest import GOLDEN

FLAVOR = 2


def test_oracle_murmur3_vs_reference_vectors(oracle):
    from oracle_ctypes import murmur3_x64_128
    v = json.load(open(os.path.join(GOLDEN, "murmur3_vectors.json")))
    assert len(v["cases"]) > 200
    for c in v["cases"]:
        got = murmur3_x64_128(oracle.lib, bytes.fromhex(c["key"]), c["seed"])
        assert got == (int(c["h1"]), int(c["h2"])), c


def test_oracle_murmur3_vs_compiled_reference(oracle):
    """Directly against the reference build when oracle/_ref is present (here)."""
    import pytest
    from oracle_ctypes import RefMurmur3, murmur3_x64_128
    try:
        ref = RefMurmur3()
    except FileNotFoundError:
        pytest.skip("oracle/_ref/libref_murmur3.so not built")
    rng = np.random.default_rng(5)
    for n in range(0, 300):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        seed = int(rng.integers(0, 2**32))
        assert murmur3_x64_128(oracle.lib, data, seed) == \
            murmur3_x64_128(ref.lib, data, seed, "ref_murmur3_x64_128")


def test_host_build_and_probe_murmur3(built, oracle):
    """nb_build_cpu / nb_probe_cpu with the Murmur3 flavour vs the oracle, fixed-
    and variable-length keys (every tail length), several seeds."""
    import nasp_bloom as nbm
    from nasp_bloom import synth
    m, k = 1_000_003, 7
    for seed in (0, 5, 17027509906831645879):
        buf, offs = synth.var_keys(20_000, 0, 70, seed=seed & 0xFFFF)
        w = np.zeros(nbm.nwords(m), np.uint64)
        nbm.build_cpu(buf, offs, 0, 20_000, m, k, seed, FLAVOR, w)
        want = oracle.build(FLAVOR, buf, offs, 0, 20_000, m, k, seed)
        np.testing.assert_array_equal(w, want)
        assert nbm.probe_cpu(buf, offs, 0, 20_000, m, k, seed, FLAVOR, w).min() == 1
        fk = synth.fixed_keys(10_000, 16)
        w2 = np.zeros(nbm.nwords(m), np.uint64)
        nbm.build_cpu(fk, None, 16, 10_000, m, k, seed, FLAVOR, w2)
        np.testing.assert_array_equal(w2, oracle.build(FLAVOR, fk, None, 16, 10_000, m, k, seed))


def test_std_hash_murmur3_is_first_half(built, oracle):
    import nasp_bloom as nbm
    from oracle_ctypes import murmur3_x64_128
    for n in (0, 1, 15, 16, 17, 40):
        data = bytes(range(n))
        assert nbm.std_hash(data, FLAVOR) == murmur3_x64_128(oracle.lib, data, 0)[0]
