"""C ABI checks that need no GPU: the library loads, exports every symbol the
header declares, and its host-only functions (formulas, seed, serialize,
deserialize) agree with the golden vectors.  No compute entry point is called."""
import os
import re
import struct

import numpy as np
import pytest

from conftest import REPO
from golden_util import image_of, words_of_bits


def header_symbols():
    text = open(os.path.join(REPO, "include", "nasp_bloom.h")).read()
    return sorted(set(re.findall(r"\b(nb_[a-z_0-9]+)\s*\(", text)))


def test_exports_every_header_symbol(built):
    import nasp_bloom
    from nasp_bloom import _lib
    h = nasp_bloom.lib()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(h, s), s
        assert s in _lib._SIGS, f"{s} has no ctypes signature"
    assert h.nb_abi_version() == 1


def test_no_device_is_reported_not_faked(built):
    import nasp_bloom
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = nasp_bloom.lib()
    assert h.nb_device_count() == 0
    # every building entry point fails loudly (NB_ERR_NODEV), none falls back to the CPU
    import numpy as np
    keys = np.zeros(160, np.uint8)
    words = np.zeros(nasp_bloom.nwords(1000), np.uint64)
    for call in (lambda: nasp_bloom.build_host(keys, None, 16, 10, 1000, 7, 1, 0, words),
                 lambda: nasp_bloom.build_host_sharded(keys, None, 16, 10, 1000, 7, 1, 0, words, 2),
                 lambda: nasp_bloom.probe_host(keys, None, 16, 10, 1000, 7, 1, 0, words),
                 lambda: nasp_bloom.Builder(1000, 7, 1, 0)):
        with pytest.raises(nasp_bloom.NaspBloomError, match="device"):
            call()
    assert not words.any()


def test_formulas_and_seed(built, golden):
    import nasp_bloom as nbm
    lib, msvc = golden
    for f in lib["formulas"]:
        assert nbm.size_of_bitset(f["n"], f["p"]) == f["m"]
        if f["k"] is not None:
            assert nbm.num_hashes(f["n"], f["m"]) == f["k"]
    for f in msvc["filters"]:
        raw = bytes.fromhex(f["bytes_hex"])
        tc, seed = struct.unpack("<IQ", raw[8 + 16:8 + 28])
        assert nbm.seed_from_time(tc) == seed


def test_serialize_roundtrip_golden(built, golden):
    import nasp_bloom as nbm
    lib, msvc = golden
    for c in lib["build_cases"][:40]:
        img = image_of(c)
        m, k, p, tc, seed, words = nbm.deserialize(img)
        assert (m, k) == (c["m"], c["k"])
        assert nbm.serialize(m, k, p, tc, seed, words) == img
        np.testing.assert_array_equal(words[:(m + 63) // 64], words_of_bits(m, c["bits"])[:(m + 63) // 64])
    for f in msvc["filters"]:
        img = bytes.fromhex(f["bytes_hex"])[8:]
        assert nbm.serialize(*nbm.deserialize(img)) == img


def test_deserialize_rejects_short_image(built):
    import nasp_bloom as nbm
    with pytest.raises(nbm.NaspBloomError):
        nbm.deserialize(b"\x01" * 10)
    hdr = struct.pack("<IIdIQ", 1000, 3, 0.01, 1, 5)
    with pytest.raises(nbm.NaspBloomError):
        nbm.deserialize(hdr + b"\0" * 10)  # needs 125 payload bytes


def test_serialized_size_wraps_like_reference(built):
    import nasp_bloom as nbm
    h = nbm.lib()
    assert h.nb_serialized_size(20) == 31
    assert h.nb_serialized_size(2**32 - 8) == 28 + (2**32 - 1) // 8
    assert h.nb_serialized_size(2**32 - 1) == 28  # (m+7) wraps in unsigned int


def test_default_filter_contains_everything(built):
    import nasp_bloom as nbm
    bf = nbm.BloomFilter()
    assert bf.possiblyContains(b"anything")  # no closures -> true (no device needed)
    assert bf.serialize()[:8] == b"\0" * 8


def test_knobs_set_get_and_reject_unknown(built):
    """The library's switches (nb_set_knob / nb_get_knob): read from the environment
    once, then set through the ABI -- no getenv at build time."""
    import nasp_bloom as nbm
    assert nbm.get_knob("NB_PACK") in (0, 1)
    with nbm.knobs(NB_BUILD_PATH="tiled", NB_CHUNK_KEYS=70000):
        assert nbm.get_knob("NB_BUILD_PATH") == 2 and nbm.get_knob("NB_CHUNK_KEYS") == 70000
    assert nbm.get_knob("NB_CHUNK_KEYS") == 0
    with pytest.raises(nbm.NaspBloomError):
        nbm.set_knob("NB_NO_SUCH_KNOB", 1)
    with pytest.raises(nbm.NaspBloomError):
        nbm.get_knob("NB_NO_SUCH_KNOB")


def test_knobs_read_from_environment_once(built):
    """A fresh process sees NB_* variables as the knobs' initial values."""
    import subprocess
    import sys
    code = ("import nasp_bloom as n; print(n.get_knob('NB_BUILD_PATH'), n.get_knob('NB_TILE_BITS'), "
            "n.get_knob('NB_PROBE_PATH'))")
    env = dict(os.environ, NB_BUILD_PATH="atomic", NB_TILE_BITS="18", NB_PROBE_PATH="lane",
               PYTHONPATH=os.path.join(REPO, "nasp-key-value-engine_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                         timeout=120)
    assert out.stdout.split() == ["1", "18", "1"], out.stderr


def test_std_hash_unknown_flavor(built):
    import nasp_bloom as nbm
    h = nbm.lib()
    assert h.nb_std_hash(b"abc", 3, 7) == 0
    assert b"flavor" in h.nb_last_error()


def test_cpu_paths_read_only_key_bytes(built, oracle):
    """nb_build_cpu / nb_probe_cpu at every misalignment of a buffer that ends at
    its last key byte (no slack): same bits as the oracle."""
    import nasp_bloom as nbm
    rng = np.random.default_rng(11)
    m, k, seed = 50_021, 7, 17027509906831645879
    for shift in range(8):
        n, kl = 301, 13
        raw = rng.integers(0, 256, shift + n * kl, dtype=np.uint8)
        keys = raw[shift:]
        pad = np.concatenate([keys, np.zeros(16, np.uint8)])
        for fl in (0, 1, 2):
            w = np.zeros(nbm.nwords(m), np.uint64)
            nbm.build_cpu(keys, None, kl, n, m, k, seed, fl, w)
            np.testing.assert_array_equal(w, oracle.build(fl, pad, None, kl, n, m, k, seed))
            np.testing.assert_array_equal(nbm.probe_cpu(keys, None, kl, n, m, k, seed, fl, w),
                                          np.ones(n, np.uint8))


def test_knob_defaults(built):
    """The switches keep their product defaults: the counted-tile policy
    (NB_TILE_COUNT 0), the sub-pass policy (NB_SUBPASSES 0: 2 for multi-pass builds, 1
    for a single pass -- 0 is the policy, not one sub-pass), the tiled probe's pass
    policy (NB_PROBE_CHUNK 0), auto's tiled threshold (NB_PROBE_TILED_PCT 0: the policy) and its
    split-path threshold (NB_PROBE_SPLIT_PCT 0: the policy) --
    unless the environment of this process set them.  The switches of the variants
    round 5 removed (measured slower) are refused as unknown names."""
    import nasp_bloom as nbm
    for name in ("NB_TILE_COUNT", "NB_SUBPASSES", "NB_PROBE_CHUNK"):
        if name not in os.environ:
            assert nbm.get_knob(name) == 0, name
    if "NB_PROBE_TILED_PCT" not in os.environ:
        assert nbm.get_knob("NB_PROBE_TILED_PCT") == 0
    if "NB_PROBE_SPLIT_PCT" not in os.environ:
        assert nbm.get_knob("NB_PROBE_SPLIT_PCT") == 0
    with nbm.knobs(NB_TILE_COUNT=768):
        assert nbm.get_knob("NB_TILE_COUNT") == 768
    for gone in ("NB_BIN_PIPE", "NB_BIN_MIX", "NB_BUCKET_GMAJOR", "NB_FINE_BITS"):
        with pytest.raises(nbm.NaspBloomError):
            nbm.get_knob(gone)
        with pytest.raises(nbm.NaspBloomError):
            nbm.set_knob(gone, 1)
