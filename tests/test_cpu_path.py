"""The host build/probe path of the C ABI (nb_build_cpu / nb_probe_cpu): what the
drop-in classes use for small batches and on hosts without a usable GPU (SURVEY
§8(b)).  It runs the kernels' own index arithmetic (csrc/bloom_math.h) on the CPU,
so it is checked here, without a GPU, against every golden vector and against
the oracle on random fixed- and variable-length keys, both flavours."""
import struct

import numpy as np
import pytest

from golden_util import image_of, keys_of, pack, words_of_bits

SEED = 17027509906831645879


def test_cpu_build_golden_cases(built, golden):
    import nasp_bloom as nbm
    lib, _ = golden
    for c in lib["build_cases"]:
        keys = keys_of(lib, c["keys"])
        buf, offs = pack(keys)
        seed = int(c["seed"])
        w = np.zeros(max(nbm.nwords(c["m"]), 1), np.uint64)
        nbm.build_cpu(buf, offs, 0, len(keys), c["m"], c["k"], seed, 0, w)
        assert nbm.serialize(c["m"], c["k"], c["p"], c["time_const"], seed, w) == image_of(c)


def test_cpu_build_msvc_filters(built, golden):
    import nasp_bloom as nbm
    _, msvc = golden
    for f in msvc["filters"]:
        img = bytes.fromhex(f["bytes_hex"])[8:]
        m, k, p, tc, seed, _ = nbm.deserialize(img)
        buf, offs = pack([bytes.fromhex(h) for h in f["keys_hex"]])
        w = np.zeros(max(nbm.nwords(m), 1), np.uint64)
        nbm.build_cpu(buf, offs, 0, len(f["keys_hex"]), m, k, seed, 1, w)
        assert nbm.serialize(m, k, p, tc, seed, w) == img, f["file"]


def test_cpu_probe_golden_cases(built, golden):
    import nasp_bloom as nbm
    lib, _ = golden
    for c in lib["probe_cases"]:
        img = image_of(c)
        m, k = struct.unpack("<II", img[:8])
        (seed,) = struct.unpack("<Q", img[20:28])
        words = words_of_bits(m, c["bits"])
        q = [bytes.fromhex(h) for h in c["query_hex"]]
        buf, offs = pack(q)
        assert nbm.probe_cpu(buf, offs, 0, len(q), m, k, seed, 0, words).tolist() == c["answer"]


def test_cpu_accumulate_golden(built, golden):
    import nasp_bloom as nbm
    lib, _ = golden
    keys = keys_of(lib, "var8_64")
    for c in lib["accumulate_cases"]:
        m, k = c["m"], c["k"]
        w = words_of_bits(m, c["first"]["bits"])
        b2, o2 = pack(keys[100:])
        nbm.build_cpu(b2, o2, 0, len(keys) - 100, m, k, SEED, 0, w)
        np.testing.assert_array_equal(w, words_of_bits(m, c["final"]["bits"]))


@pytest.mark.parametrize("flavor", [0, 1])
@pytest.mark.parametrize("key_len", [0, 1, 7, 16, 33])
def test_cpu_build_matches_oracle(built, oracle, flavor, key_len):
    import nasp_bloom as nbm
    from nasp_bloom import synth
    n, m, k = 20_000, 191_701, 7
    if key_len:
        buf, offs = synth.fixed_keys(n, key_len), None
    else:
        buf, offs = synth.var_keys(n, 0, 70)
    for shift in (0, 3):  # misaligned key base
        b = np.zeros(buf.size + shift + 8, np.uint8)
        b[shift:shift + buf.size] = buf
        view = b[shift:]
        w = np.zeros(nbm.nwords(m), np.uint64)
        nbm.build_cpu(view, offs, key_len, n, m, k, SEED, flavor, w)
        want = oracle.build(flavor, buf, offs, key_len, n, m, k, SEED)
        np.testing.assert_array_equal(w, want)
        probe_keys, probe_offs = synth.var_keys(2000, 1, 40, seed=99)
        got = nbm.probe_cpu(probe_keys, probe_offs, 0, 2000, m, k, SEED, flavor, w)
        np.testing.assert_array_equal(got, oracle.probe(flavor, probe_keys, probe_offs, 0, 2000, m, k,
                                                        SEED, want))


def test_cpu_edges(built):
    import nasp_bloom as nbm
    w = np.zeros(4, np.uint64)
    nbm.build_cpu(np.zeros(16, np.uint8), None, 16, 0, 200, 3, SEED, 0, w)  # no keys: no-op
    assert not w.any()
    with pytest.raises(nbm.NaspBloomError, match="m == 0"):
        nbm.build_cpu(np.zeros(16, np.uint8), None, 8, 1, 0, 3, SEED, 0, w)
    with pytest.raises(nbm.NaspBloomError, match="flavor"):
        nbm.build_cpu(np.zeros(16, np.uint8), None, 8, 1, 64, 3, SEED, 7, w)
    # k == 0 (no closures): nothing set, every probe true (BloomFilter.cpp:26,67-80)
    nbm.build_cpu(np.zeros(16, np.uint8), None, 8, 1, 64, 0, SEED, 0, w)
    assert not w.any()
    assert nbm.probe_cpu(np.zeros(16, np.uint8), None, 8, 2, 64, 0, SEED, 0, w).tolist() == [1, 1]


def test_python_mirror_small_batches_stay_on_host(built):
    """The Python BloomFilter mirror builds small batches with nb_build_cpu: no
    device needed, no device build counted."""
    import nasp_bloom as nbm
    before = nbm.device_build_count()
    bf = nbm.BloomFilter(1000, 0.01, time_const=1748963255)
    for i in range(100):
        bf.add(f"user{i:08d}")
    img = bf.serialize()
    again = nbm.BloomFilter.deserialize(img)
    again.add("one more")
    assert again.possiblyContains("one more") and again.possiblyContains("user00000007")
    assert not again.last_on_device and nbm.device_build_count() == before
