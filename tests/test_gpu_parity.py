"""GPU parity: the HIP build/probe path (through the C ABI) against the oracle
and the golden vectors.  Integer/byte work: the bar is bit-exact.

Sizes: the golden vectors, C1 and C2 in full (10M x 16B, oracle ~1 s), C3's
shape at 2M keys against the oracle, and C3 at its full 100M keys through
size-independent properties (shard-OR equals whole build, no false negatives,
subset filters contained in the full filter)."""
import struct

import numpy as np
import pytest

from golden_util import image_of, keys_of, pack, words_of_bits

pytestmark = pytest.mark.gpu

SEED = 17027509906831645879
TC = 1748963255


@pytest.fixture(scope="module")
def dev(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import nasp_bloom
    assert nasp_bloom.lib().nb_device_count() >= 1
    return torch.device("cuda:0")


@pytest.fixture(params=["auto", "atomic", "tiled"])
def build_path(request, knobs):
    """Run a test through each build path of the library (NB_BUILD_PATH)."""
    knobs(NB_BUILD_PATH=request.param)
    return request.param


def t_u8(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def t_u64(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)


def dev_build(dev, buf, offs, key_len, n, m, k, seed, flavor=0, words=None, byte_shift=0):
    """Build on the device; returns host uint64 words. byte_shift misaligns the key base."""
    import torch
    import nasp_bloom as nbm
    if byte_shift:
        big = np.zeros(buf.size + byte_shift, dtype=np.uint8)
        big[byte_shift:] = buf
        kt = t_u8(big, dev)[byte_shift:]
    else:
        kt = t_u8(buf, dev)
    ot = t_u64(offs, dev) if offs is not None else None
    nw = max(nbm.nwords(m), 1)
    wt = t_u64(words, dev) if words is not None else torch.zeros(nw, dtype=torch.int64, device=dev)
    nbm.build_device(kt, ot, key_len, n, m, k, seed, flavor, wt)
    torch.cuda.synchronize()
    return wt.cpu().numpy().view(np.uint64)


def dev_probe(dev, buf, offs, key_len, n, m, k, seed, words, flavor=0):
    import torch
    import nasp_bloom as nbm
    kt = t_u8(buf, dev)
    ot = t_u64(offs, dev) if offs is not None else None
    wt = t_u64(words, dev)
    out = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
    nbm.probe_device(kt, ot, key_len, n, m, k, seed, flavor, wt, out)
    torch.cuda.synchronize()
    return out.cpu().numpy()[:n]


def oracle_build_threaded(oracle, flavor, buf, offs, key_len, n, m, k, seed, threads=16):
    """The oracle over n keys in `threads` key ranges at once (its C build releases
    the GIL), ORed: exact full-size parity in seconds.  16 threads = one GPU's CPU
    share on the box."""
    import threading
    parts = [None] * threads

    def run(t):
        b, e = n * t // threads, n * (t + 1) // threads
        if offs is not None:
            parts[t] = oracle.build(flavor, buf, offs[b:e + 1], 0, e - b, m, k, seed)
        else:
            parts[t] = oracle.build(flavor, buf[b * key_len:], None, key_len, e - b, m, k, seed)
    th = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    out = parts[0]
    for p_ in parts[1:]:
        out |= p_
    return out


def set_bits(words):
    """Sorted indices of the set bits; expands only the non-zero words (a 2^32-bit
    filter with a handful of bits set stays cheap)."""
    nz = np.flatnonzero(words)
    sub = np.unpackbits(words[nz].view(np.uint8), bitorder="little").reshape(len(nz), 64)
    r, b = np.nonzero(sub)
    return (nz[r].astype(np.int64) * 64 + b).tolist()


# ---------------------------------------------------------------- golden --

def test_golden_build_cases(dev, golden, build_path):
    import nasp_bloom as nbm
    lib, _ = golden
    for c in lib["build_cases"]:
        keys = keys_of(lib, c["keys"])
        buf, offs = pack(keys)
        seed = int(c["seed"])
        w = dev_build(dev, buf, offs, 0, len(keys), c["m"], c["k"], seed)
        img = nbm.serialize(c["m"], c["k"], c["p"], c["time_const"], seed, w)
        assert img == image_of(c), (c["keys"], c["m"], c["k"])


def test_golden_msvc_filters_device(dev, golden, build_path):
    import nasp_bloom as nbm
    _, msvc = golden
    for f in msvc["filters"]:
        raw = bytes.fromhex(f["bytes_hex"])
        img = raw[8:]
        m, k, p, tc, seed, _ = nbm.deserialize(img)
        keys = [bytes.fromhex(h) for h in f["keys_hex"]]
        buf, offs = pack(keys)
        w = dev_build(dev, buf, offs, 0, len(keys), m, k, seed, flavor=1)
        assert nbm.serialize(m, k, p, tc, seed, w) == img, f["file"]


def test_golden_probe_cases(dev, golden):
    lib, _ = golden
    for c in lib["probe_cases"]:
        img = image_of(c)
        m, k = struct.unpack("<II", img[:8])
        (seed,) = struct.unpack("<Q", img[20:28])
        words = words_of_bits(m, c["bits"])
        q = [bytes.fromhex(h) for h in c["query_hex"]]
        buf, offs = pack(q)
        assert dev_probe(dev, buf, offs, 0, len(q), m, k, seed, words).tolist() == c["answer"]


def test_golden_accumulate(dev, golden, build_path):
    """add() after deserialize() ORs into the existing bits (TypesManager.cpp:84-86)."""
    lib, _ = golden
    keys = keys_of(lib, "var8_64")
    for c in lib["accumulate_cases"]:
        m, k = c["m"], c["k"]
        first = words_of_bits(m, c["first"]["bits"])
        b2, o2 = pack(keys[100:])
        w = dev_build(dev, b2, o2, 0, len(keys) - 100, m, k, SEED, words=first)
        np.testing.assert_array_equal(w, words_of_bits(m, c["final"]["bits"]))


def test_golden_large_m(dev, golden, build_path):
    lib, _ = golden
    for c in lib["large_m"]:
        key = bytes.fromhex(c["key_hex"])
        buf, offs = pack([key])
        w = dev_build(dev, buf, offs, 0, 1, c["m"], c["k"], int(c["seed"]))
        assert set_bits(w) == c["bits"], c


# ------------------------------------------------------ configs vs oracle --

@pytest.mark.parametrize("cfg", ["c1", "c2"])
def test_fixed16_configs_full_size(dev, oracle, cfg, build_path):
    from nasp_bloom import synth
    w = synth.WORKLOADS[cfg]
    buf, offs, kl = synth.keys_for(w)
    got = dev_build(dev, buf, offs, kl, w.n, w.m, w.k, SEED)
    want = oracle.build(0, buf, offs, kl, w.n, w.m, w.k, SEED)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("flavor", [0, 1])
@pytest.mark.parametrize("shift", [0, 3])
def test_varlen_c3_shape(dev, oracle, flavor, shift, build_path):
    from nasp_bloom import synth
    n = 2_000_000 if flavor == 0 else 500_000
    buf, offs = synth.var_keys(n)
    got = dev_build(dev, buf, offs, 0, n, synth.C3.m, 7, SEED, flavor=flavor, byte_shift=shift)
    want = oracle.build(flavor, buf, offs, 0, n, synth.C3.m, 7, SEED)
    np.testing.assert_array_equal(got, want)


def test_fnv_c2_full_size(dev, oracle):
    """The MSVC FNV-1a flavour at C2's full size (10M x 16 B, k = 7), bit-exact."""
    from nasp_bloom import synth
    w = synth.C2
    buf, offs, kl = synth.keys_for(w)
    got = dev_build(dev, buf, offs, kl, w.n, w.m, w.k, SEED, flavor=1)
    np.testing.assert_array_equal(got, oracle_build_threaded(oracle, 1, buf, offs, kl, w.n, w.m,
                                                             w.k, SEED))


@pytest.mark.parametrize("key_len,shift", [(16, 4), (32, 0), (7, 1), (1, 0), (64, 5), (100, 0)])
def test_fixed_stride_layouts(dev, oracle, key_len, shift, build_path):
    from nasp_bloom import synth
    n = 200_003
    buf = synth.fixed_keys(n, key_len, seed=key_len)
    for flavor in (0, 1):
        got = dev_build(dev, buf, None, key_len, n, 1_000_003, 7, SEED, flavor=flavor,
                        byte_shift=shift)
        want = oracle.build(flavor, buf, None, key_len, n, 1_000_003, 7, SEED)
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("layout", ["fixed16", "fixed32", "stride7", "varlen"])
def test_murmur3_flavor_device(dev, oracle, layout, build_path):
    """The optional non-parity NB_FLAVOR_MURMUR3_X64_128 (h1, h2 = the halves of
    MurmurHash3_x64_128(key, len, (uint32_t)seed)) on the device against the
    oracle (itself pinned to the compiled reference MurmurHash3.cpp), every key
    layout path, build and probe."""
    from nasp_bloom import synth
    n, m, k = 200_003, 4_000_037, 7
    if layout == "varlen":
        buf, offs = synth.var_keys(n, 0, 70)
        kl = 0
    else:
        kl = {"fixed16": 16, "fixed32": 32, "stride7": 7}[layout]
        buf, offs = synth.fixed_keys(n, kl), None
    want = oracle.build(2, buf, offs, kl, n, m, k, SEED)
    got = dev_build(dev, buf, offs, kl, n, m, k, SEED, flavor=2)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(dev_probe(dev, buf, offs, kl, n, m, k, SEED, want, 2),
                                  oracle.probe(2, buf, offs, kl, n, m, k, SEED, want))


# D % 8 = 1, 0, 4, 5, 7, 3: every prefix class of the register-resident 32-byte path
@pytest.mark.parametrize("seed", [7, 12345678, 12345678901234567890, 1234567890123,
                                  123456789012345, 123])
def test_fixed32_vector_path(dev, oracle, seed, build_path):
    """32-byte keys at a 16-byte-aligned base (C5's shape) are hashed from two dwordx4
    loads in registers (kFixed32); every seed-prefix class, both flavours, build and
    probe, bit-exact; NB_FIXED32=0 keeps the LDS-staged path for the same keys."""
    import os
    from nasp_bloom import synth
    n, m = 300_001, 4_000_037
    buf = synth.fixed_keys(n, 32, seed=32)
    for flavor in (0, 1):
        want = oracle.build(flavor, buf, None, 32, n, m, 10, seed)
        got = dev_build(dev, buf, None, 32, n, m, 10, seed, flavor=flavor)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(oracle.probe(flavor, buf, None, 32, n, m, 10, seed, want),
                                      dev_probe(dev, buf, None, 32, n, m, 10, seed, want, flavor))
    import nasp_bloom as nbm
    with nbm.knobs(NB_FIXED32=0):
        got = dev_build(dev, buf, None, 32, n, m, 10, seed)
    np.testing.assert_array_equal(got, oracle.build(0, buf, None, 32, n, m, 10, seed))


@pytest.mark.parametrize("seed", [0, 7, 12345678, 123456789, 1234567890123456789, 2**64 - 1])
def test_seed_prefix_lengths(dev, oracle, seed, build_path):
    """to_string(seed) of 1..20 digits changes how the prefix splices into h2."""
    from nasp_bloom import synth
    buf, offs = synth.var_keys(100_000, 0, 40)
    for flavor in (0, 1):
        got = dev_build(dev, buf, offs, 0, 100_000, 4_000_037, 5, seed, flavor=flavor)
        want = oracle.build(flavor, buf, offs, 0, 100_000, 4_000_037, 5, seed)
        np.testing.assert_array_equal(got, want)


def test_c5_shape_sample(dev, oracle):
    """C5's m = 2^32-1, k = 10, 32-byte keys (a 2M-key sample of one shard)."""
    from nasp_bloom import synth
    w = synth.C5
    n = 2_000_000
    buf = synth.fixed_keys(n, 32)
    got = dev_build(dev, buf, None, 32, n, w.m, w.k, SEED)
    want = oracle.build(0, buf, None, 32, n, w.m, w.k, SEED)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("m", [1, 2, 63, 64, 65, 2**31, 2**32 - 8, 2**32 - 1])
def test_edge_m(dev, oracle, m, build_path):
    from nasp_bloom import synth
    buf, offs = synth.var_keys(20_000, 0, 24)
    for k in (1, 10):
        got = dev_build(dev, buf, offs, 0, 20_000, m, k, SEED)
        want = oracle.build(0, buf, offs, 0, 20_000, m, k, SEED)
        np.testing.assert_array_equal(got, want)


def test_empty_and_degenerate(dev, oracle, build_path):
    import nasp_bloom as nbm
    import torch
    # n = 0: no-op
    w = dev_build(dev, np.zeros(16, np.uint8), np.zeros(1, np.uint64), 0, 0, 1000, 7, SEED)
    assert not w.any()
    # all-empty keys: every key hashes identically
    offs = np.zeros(1001, dtype=np.uint64)
    w = dev_build(dev, np.zeros(16, np.uint8), offs, 0, 1000, 1000, 7, SEED)
    want = oracle.build(0, np.zeros(16, np.uint8), offs, 0, 1000, 1000, 7, SEED)
    np.testing.assert_array_equal(w, want)
    # m == 0 with keys is an argument error (the reference divides by zero)
    kt = torch.zeros(32, dtype=torch.uint8, device=dev)
    wt = torch.zeros(1, dtype=torch.int64, device=dev)
    with pytest.raises(nbm.NaspBloomError):
        nbm.build_device(kt, None, 16, 1, 0, 7, SEED, 0, wt)
    # k == 0: nothing set, probe answers true
    w0 = dev_build(dev, np.zeros(48, np.uint8), None, 16, 3, 1000, 0, SEED)
    assert not w0.any()
    assert dev_probe(dev, np.zeros(48, np.uint8), None, 16, 3, 1000, 0, SEED, w0).tolist() == [1, 1, 1]


def test_device_shape_checks(dev):
    """Tensors too small for (n, key_len, m) are refused on the host, before any
    kernel could read past them."""
    import nasp_bloom as nbm
    import torch
    kt = torch.zeros(16 * 10, dtype=torch.uint8, device=dev)
    wt = torch.zeros(nbm.nwords(1000), dtype=torch.int64, device=dev)
    out = torch.zeros(11, dtype=torch.uint8, device=dev)
    offs = torch.zeros(11, dtype=torch.int64, device=dev)
    for call in (lambda: nbm.build_device(kt, None, 16, 11, 1000, 7, SEED, 0, wt),
                 lambda: nbm.build_device(kt, offs[:10], 0, 10 + 1, 1000, 7, SEED, 0, wt),
                 lambda: nbm.build_device(kt, offs.to(torch.int32), 0, 10, 1000, 7, SEED, 0, wt),
                 lambda: nbm.build_device(kt, None, 16, 10, 100_000, 7, SEED, 0, wt),
                 lambda: nbm.probe_device(kt, None, 16, 11, 1000, 7, SEED, 0, wt, out),
                 lambda: nbm.probe_device(kt, None, 16, 10, 1000, 7, SEED, 0, wt, out[:9]),
                 lambda: nbm.probe_device(kt, None, 16, 10, 100_000, 7, SEED, 0, wt, out)):
        with pytest.raises(nbm.NaspBloomError):
            call()
    nbm.build_device(kt, None, 16, 10, 1000, 7, SEED, 0, wt)  # exact sizes are fine
    nbm.build_device(kt, offs, 0, 10, 1000, 7, SEED, 0, wt)
    for o, kl in ((None, 16), (offs, 0)):
        out.zero_()
        nbm.probe_device(kt, o, kl, 10, 1000, 7, SEED, 0, wt, out)
        torch.cuda.synchronize()
        assert int(out[:10].min()) == 1


@pytest.mark.parametrize("k", [1, 8, 9, 16, 17, 24, 32, 33])
def test_k_range_tiled(dev, oracle, k, knobs):
    """k selects the tiled kernel's keys per block (<=8, <=16, <=32) or the atomic path (>32)."""
    from nasp_bloom import synth
    knobs(NB_BUILD_PATH="tiled")
    buf, offs = synth.var_keys(300_000, 4, 40)
    got = dev_build(dev, buf, offs, 0, 300_000, 7_000_003, k, SEED)
    want = oracle.build(0, buf, offs, 0, 300_000, 7_000_003, k, SEED)
    np.testing.assert_array_equal(got, want)


def test_tiled_bucket_overflow_spill(dev, oracle, knobs):
    """Massively duplicated keys overflow the per-tile buckets; the spill path must
    still give the exact filter (SSTable keys are unique, but the API allows this)."""
    from nasp_bloom import synth
    knobs(NB_BUILD_PATH="tiled")
    n = 400_000
    buf = np.zeros(n * 16 + 16, np.uint8)  # 400k identical all-zero 16-byte keys
    buf[: 16 * 1000] = synth.fixed_keys(1000, 16)[: 16 * 1000]  # + 1000 distinct ones
    got = dev_build(dev, buf, None, 16, n, 95_850_584, 7, SEED)
    want = oracle.build(0, buf, None, 16, n, 95_850_584, 7, SEED)
    np.testing.assert_array_equal(got, want)


# Tile policy boundaries (bloom_kernels.hip choose_tiles): u16 entries up to
# m = 2^27 (ts 16, T 2048); above it 32-bit entries with the largest tiles that
# leave >= 512 of them -- 2^27+1 -> ts 18 / T 513, 2^28-1 -> ts 19 / T 512,
# C3/C4's m -> ts 20 / T 915, 2^30+7 -> T 1025 (packed entries: two bin blocks
# still fit a CU's LDS), 2^31-1 -> ts 20 / T 2048 (32-bit entries: the pad slots
# would not fit two blocks; last single-level m), 2^31+1 -> two-level.  Ragged
# last tiles included.
@pytest.mark.parametrize("m", [2**27, 2**27 + 1, 2**28 - 1, 300_000_001, 958_505_838,
                               2**30 + 7, 2**31 - 1, 2**31 + 1])
def test_tile_policy_boundaries(dev, oracle, m, knobs):
    from nasp_bloom import synth
    knobs(NB_BUILD_PATH="tiled")
    n = 300_000
    buf = synth.fixed_keys(n, 16)
    got = dev_build(dev, buf, None, 16, n, m, 7, SEED)
    want = oracle.build(0, buf, None, 16, n, m, 7, SEED)
    np.testing.assert_array_equal(got, want)
    vbuf, voffs = synth.var_keys(n, 8, 64)
    got = dev_build(dev, vbuf, voffs, 0, n, m, 7, SEED, flavor=1)
    want = oracle.build(1, vbuf, voffs, 0, n, m, 7, SEED)
    np.testing.assert_array_equal(got, want)


def test_packed_entries_past_4gib(dev, knobs):
    """Packed bucket words past 4 GiB of buckets (word-indexed write-out): 120M
    keys x k = 16 into m = 900 x 2^20 (900 2^20-bit tiles, packed while two bin
    blocks fit a CU's LDS; 1.92G entries = 5.1 GB of packed words in one chunk) must give the same filter as 32-bit entries
    (NB_PACK=0, checked against the oracle elsewhere), with no false negatives."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    knobs(NB_BUILD_PATH="tiled")
    n, m, k = 120_000_000, 900 << 20, 16
    kt = t_u8(synth.fixed_keys(n, 16), dev)
    out = []
    for pack in ("1", "0"):
        knobs(NB_PACK=pack)
        wt = torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev)
        nbm.build_device(kt, None, 16, n, m, k, SEED, 0, wt)
        torch.cuda.synchronize()
        out.append(wt)
    assert torch.equal(out[0], out[1])
    res = torch.empty(n, dtype=torch.uint8, device=dev)
    nbm.probe_device(kt, None, 16, n, m, k, SEED, 0, out[0], res)
    torch.cuda.synchronize()
    assert int(res.min()) == 1


def test_tiled_overflow_spill_large_tiles(dev, oracle, knobs):
    """The spill path with 32-bit entries and 2^20-bit tiles (C4's m)."""
    from nasp_bloom import synth
    knobs(NB_BUILD_PATH="tiled")
    n = 400_000
    buf = np.zeros(n * 16 + 16, np.uint8)
    buf[: 16 * 1000] = synth.fixed_keys(1000, 16)[: 16 * 1000]
    got = dev_build(dev, buf, None, 16, n, 958_505_838, 7, SEED)
    want = oracle.build(0, buf, None, 16, n, 958_505_838, 7, SEED)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("two_level", ["1", "0"])
@pytest.mark.parametrize("chunk", ["0", "300000"])
def test_two_level_build_large_m(dev, oracle, two_level, chunk, knobs):
    """m > 2^31 (C5's 2^32-1): 4 096 fine tiles, built through super tiles + re-bin
    (NB_TWO_LEVEL=1, the default) or binned straight into the fine tiles; chunked
    builds accumulate across chunks; k = 10 and k = 7 (rank paths KR=16 / KR=8)."""
    from nasp_bloom import synth
    knobs(NB_BUILD_PATH="tiled")
    knobs(NB_TWO_LEVEL=two_level)
    if chunk != "0":
        knobs(NB_CHUNK_KEYS=chunk)
    n = 1_000_003
    buf = synth.fixed_keys(n, 32, seed=77)
    for m, k in ((2**32 - 1, 10), (3_000_000_019, 7)):
        got = dev_build(dev, buf, None, 32, n, m, k, SEED)
        want = oracle.build(0, buf, None, 32, n, m, k, SEED)
        np.testing.assert_array_equal(got, want)
    vb, vo = synth.var_keys(300_000)
    got = dev_build(dev, vb, vo, 0, 300_000, 2**32 - 1, 10, SEED)
    np.testing.assert_array_equal(got, oracle.build(0, vb, vo, 0, 300_000, 2**32 - 1, 10, SEED))


def test_two_level_overflow_spill(dev, oracle, knobs):
    """Duplicated keys overflow both the super-tile and the fine-tile buckets of the
    two-level build: pass 1 spills by fine tile, the re-bin spills too."""
    from nasp_bloom import synth
    knobs(NB_BUILD_PATH="tiled")
    n = 400_000
    buf = np.zeros(n * 32 + 16, np.uint8)
    buf[: 32 * 5000] = synth.fixed_keys(5000, 32)[: 32 * 5000]
    got = dev_build(dev, buf, None, 32, n, 2**32 - 1, 10, SEED)
    want = oracle.build(0, buf, None, 32, n, 2**32 - 1, 10, SEED)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("overlap,sub", [("1", "1"), ("2", "2"), ("6", "3"), ("0", "3"), ("6", "1"),
                                         ("2", "5")])
def test_two_level_overlap(dev, oracle, overlap, sub, knobs):
    """NB_OVERLAP: the two-level sub-passes pipelined over two streams (a re-bin
    beside the next bin kernel; & 4: a tile kernel beside the next pass's bin kernel;
    sub-pass- and pass-parity scratch); NB_SUBPASSES: bin + re-bin sub-passes sharing
    one tile pass.  Odd and even pass counts, overwrite over stale words, duplicated keys
    spilling in every pass, and an exact normal build afterwards (scratch clean)."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    knobs(NB_BUILD_PATH="tiled", NB_OVERLAP=overlap, NB_SUBPASSES=sub)
    m, k = 2**32 - 1, 10
    n = 700_001
    buf = synth.fixed_keys(n, 32, seed=91)
    want = oracle.build(0, buf, None, 32, n, m, k, SEED)
    for chunk in ("150000", "240000", "350001"):  # 5, 3 and 2 passes
        knobs(NB_CHUNK_KEYS=chunk)
        words = torch.full((nbm.nwords(m),), -1, dtype=torch.int64, device=dev)
        nbm.build_device(t_u8(buf, dev), None, 32, n, m, k, SEED, 0, words, overwrite=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(words.cpu().numpy().view(np.uint64), want)
    dup = np.zeros(400_000 * 32 + 16, np.uint8)
    dup[: 32 * 5000] = synth.fixed_keys(5000, 32)[: 32 * 5000]
    knobs(NB_CHUNK_KEYS="90000")
    got = dev_build(dev, dup, None, 32, 400_000, m, k, SEED)
    np.testing.assert_array_equal(got, oracle.build(0, dup, None, 32, 400_000, m, k, SEED))
    vb, vo = synth.var_keys(300_000)
    got = dev_build(dev, vb, vo, 0, 300_000, m, k, SEED)
    np.testing.assert_array_equal(got, oracle.build(0, vb, vo, 0, 300_000, m, k, SEED))
    knobs(NB_OVERLAP="0", NB_SUBPASSES="1")
    got = dev_build(dev, buf, None, 32, n, m, k, SEED)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("chunk", ["4096", "100000", "999999"])
def test_tiled_chunking(dev, oracle, chunk, knobs):
    from nasp_bloom import synth
    knobs(NB_BUILD_PATH="tiled")
    knobs(NB_CHUNK_KEYS=chunk)
    buf, offs = synth.var_keys(1_000_000)
    got = dev_build(dev, buf, offs, 0, 1_000_000, 9_585_059, 7, SEED)
    want = oracle.build(0, buf, offs, 0, 1_000_000, 9_585_059, 7, SEED)
    np.testing.assert_array_equal(got, want)
    fixed = synth.fixed_keys(700_001, 16)
    got = dev_build(dev, fixed, None, 16, 700_001, 95_850_584, 7, SEED)
    np.testing.assert_array_equal(got, oracle.build(0, fixed, None, 16, 700_001, 95_850_584, 7, SEED))


@pytest.mark.parametrize("path", ["atomic", "tiled"])
def test_overwrite_mode(dev, oracle, path, knobs):
    """NB_BUILD_OVERWRITE: the words become the batch's filter whatever they held
    before -- including when buckets spill (duplicated keys) and across chunks."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    knobs(NB_BUILD_PATH=path)
    m, k = 9_585_059, 7
    buf, offs = synth.var_keys(500_000)
    kt, ot = t_u8(buf, dev), t_u64(offs, dev)
    stale = torch.full((nbm.nwords(m),), -1, dtype=torch.int64, device=dev)  # all ones
    nbm.build_device(kt, ot, 0, 500_000, m, k, SEED, 0, stale, overwrite=True)
    torch.cuda.synchronize()
    want = oracle.build(0, buf, offs, 0, 500_000, m, k, SEED)
    np.testing.assert_array_equal(stale.cpu().numpy().view(np.uint64), want)
    # duplicated keys (spill path) into stale words, then a second chunked batch
    dup = np.zeros(300_000 * 16 + 16, np.uint8)
    dup[:16 * 500] = synth.fixed_keys(500, 16)[:16 * 500]
    stale.fill_(-1)
    knobs(NB_CHUNK_KEYS="70000")
    nbm.build_device(t_u8(dup, dev), None, 16, 300_000, m, k, SEED, 0, stale, overwrite=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(stale.cpu().numpy().view(np.uint64),
                                  oracle.build(0, dup, None, 16, 300_000, m, k, SEED))
    # the spill bitmap and cursors were left clean: a normal build is exact again
    fresh = torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev)
    nbm.build_device(kt, ot, 0, 500_000, m, k, SEED, 0, fresh)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(fresh.cpu().numpy().view(np.uint64), want)


def test_probe_parity(dev, oracle):
    from nasp_bloom import synth
    buf, offs = synth.var_keys(1_000_000)
    m, k = 9_585_059, 7
    # filter from the even keys only -> probes hit on even keys, rare FPs on odd ones
    sub = np.arange(0, 1_000_000, 2)
    sub_buf = np.concatenate([buf[int(offs[i]):int(offs[i + 1])] for i in sub[:200_000]] + [np.zeros(16, np.uint8)])
    sub_offs = np.zeros(200_001, np.uint64)
    sub_offs[1:] = np.cumsum([int(offs[i + 1] - offs[i]) for i in sub[:200_000]])
    words = oracle.build(0, sub_buf, sub_offs, 0, 200_000, m, k, SEED)
    got = dev_probe(dev, buf, offs, 0, 1_000_000, m, k, SEED, words)
    want = oracle.probe(0, buf, offs, 0, 1_000_000, m, k, SEED, words)
    np.testing.assert_array_equal(got, want)
    assert got[0:400_000:2].all()


def test_deterministic(dev):
    from nasp_bloom import synth
    buf, offs, kl = synth.keys_for(synth.C2, n=3_000_000)
    a = dev_build(dev, buf, offs, kl, 3_000_000, synth.C2.m, 7, SEED)
    b = dev_build(dev, buf, offs, kl, 3_000_000, synth.C2.m, 7, SEED)
    np.testing.assert_array_equal(a, b)


# --------------------------------------------------------- full-size C3 --

def test_c3_full_size_properties(dev, oracle):
    """100M var-length keys: (1) OR of 4 shard builds == whole build,
    (2) every key probes positive, (3) an oracle filter of a 1M-key subset is
    contained in the full filter, and the oracle's own bits for the first 200k keys
    all appear.  Bit-exact parity of the whole filter at this size is implied by
    the shard/subset identities plus the 2M-key exact test above."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    w = synth.C3
    buf, offs = synth.var_keys(w.n)
    kt = t_u8(buf, dev)
    ot = t_u64(offs, dev)
    nw = nbm.nwords(w.m)
    full = torch.zeros(nw, dtype=torch.int64, device=dev)
    nbm.build_device(kt, ot, 0, w.n, w.m, w.k, SEED, 0, full)
    parts = torch.zeros(nw, dtype=torch.int64, device=dev)
    q = w.n // 4
    for s in range(4):
        e = w.n if s == 3 else (s + 1) * q
        part = torch.zeros(nw, dtype=torch.int64, device=dev)
        nbm.build_device(kt, ot[s * q:], 0, e - s * q, w.m, w.k, SEED, 0, part)
        parts |= part
        del part
    torch.cuda.synchronize()
    assert torch.equal(full, parts)
    out = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    nbm.probe_device(kt, ot, 0, w.n, w.m, w.k, SEED, 0, full, out)
    torch.cuda.synchronize()
    assert int(out.min()) == 1
    del out
    fh = full.cpu().numpy().view(np.uint64)
    n_sub = 1_000_000
    sub = oracle.build(0, buf, offs, 0, n_sub, w.m, w.k, SEED)  # first 1M keys
    assert not (sub & ~fh).any()
    # popcount sanity vs the expected fill 1 - exp(-kn/m) (~50% for p=0.01)
    fill = float(np.bitwise_count(fh).sum(dtype=np.int64)) / w.m
    assert 0.45 < fill < 0.55
    # and bit-exact at full size: the oracle over all 100M keys, 16 threads
    np.testing.assert_array_equal(fh, oracle_build_threaded(oracle, 0, buf, offs, 0, w.n, w.m,
                                                            w.k, SEED))


def test_fnv_c3_full_size(dev, oracle):
    """The MSVC FNV-1a flavour at C3's full size (100M var-length 8-64 B keys),
    bit-exact against the oracle run over 16 key ranges."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    w = synth.C3
    buf, offs = synth.var_keys(w.n)
    kt = t_u8(buf, dev)
    ot = t_u64(offs, dev)
    full = torch.zeros(nbm.nwords(w.m), dtype=torch.int64, device=dev)
    nbm.build_device(kt, ot, 0, w.n, w.m, w.k, SEED, 1, full)
    torch.cuda.synchronize()
    del kt, ot
    fh = full.cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(fh, oracle_build_threaded(oracle, 1, buf, offs, 0, w.n, w.m,
                                                            w.k, SEED))


def test_c4_full_size_properties(dev, oracle):
    """C4's per-GPU shard at full size: 100M x 16 B keys, k = 7, m = 958 505 838
    (2^19-bit tiles, 32-bit bucket entries): shard-OR identity, no false negatives,
    fill ~ 50 %, and bit-exact against the (threaded) oracle."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    w = synth.C4
    g = torch.Generator(device=dev).manual_seed(synth.SEED + 4)
    kt = torch.randint(0, 256, (w.n * 16,), dtype=torch.uint8, device=dev, generator=g)
    nw = nbm.nwords(w.m)
    full = torch.zeros(nw, dtype=torch.int64, device=dev)
    nbm.build_device(kt, None, 16, w.n, w.m, w.k, SEED, 0, full, overwrite=True)
    parts = torch.zeros(nw, dtype=torch.int64, device=dev)
    q = w.n // 3
    for s in range(3):
        e = w.n if s == 2 else (s + 1) * q
        nbm.build_device(kt[s * q * 16:], None, 16, e - s * q, w.m, w.k, SEED, 0, parts)
    torch.cuda.synchronize()
    assert torch.equal(full, parts)
    del parts
    out = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    nbm.probe_device(kt, None, 16, w.n, w.m, w.k, SEED, 0, full, out)
    torch.cuda.synchronize()
    assert int(out.min()) == 1
    del out
    fh = full.cpu().numpy().view(np.uint64)
    fill = float(np.bitwise_count(fh).sum(dtype=np.int64)) / w.m
    assert abs(fill - (1.0 - np.exp(-w.k * w.n / w.m))) < 0.005
    # bit-exact at full size: the oracle over all 100M keys, 16 threads
    keys_h = kt.cpu().numpy()
    np.testing.assert_array_equal(fh, oracle_build_threaded(oracle, 0, keys_h, None, 16, w.n, w.m,
                                                            w.k, SEED))


def test_c5_full_size_properties(dev, oracle):
    """C5 at its full size on one GPU: 1B x 32 B keys, k = 10, m = 2^32 - 1 (the
    two-level path in eight 125M-key passes).  (1) OR of 4 shard builds == whole
    build, (2) every key probes positive, (3) fill matches 1 - exp(-kn/m), (4)
    bit-exact against the (threaded) oracle."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    w = synth.C5
    g = torch.Generator(device=dev).manual_seed(synth.SEED)
    kt = torch.randint(0, 256, (w.n * w.key_len,), dtype=torch.uint8, device=dev, generator=g)
    nw = nbm.nwords(w.m)
    full = torch.zeros(nw, dtype=torch.int64, device=dev)
    nbm.build_device(kt, None, w.key_len, w.n, w.m, w.k, SEED, 0, full, overwrite=True)
    parts = torch.zeros(nw, dtype=torch.int64, device=dev)
    q = w.n // 4
    for s in range(4):
        e = w.n if s == 3 else (s + 1) * q
        nbm.build_device(kt[s * q * w.key_len:], None, w.key_len, e - s * q, w.m, w.k, SEED, 0,
                         parts)
    torch.cuda.synchronize()
    assert torch.equal(full, parts)
    del parts
    out = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    nbm.probe_device(kt, None, w.key_len, w.n, w.m, w.k, SEED, 0, full, out)
    torch.cuda.synchronize()
    assert int(out.min()) == 1
    del out
    fh = full.cpu().numpy().view(np.uint64)
    fill = float(np.bitwise_count(fh).sum(dtype=np.int64)) / w.m
    expect = 1.0 - np.exp(-w.k * w.n / w.m)  # 0.903
    assert abs(fill - expect) < 0.005
    # bit-exact at full size: the oracle over all 1B keys (32 GB on the host),
    # 16 threads with a 512 MB filter each, ORed
    keys_h = kt.cpu().numpy()
    del kt
    np.testing.assert_array_equal(fh, oracle_build_threaded(oracle, 0, keys_h, None, w.key_len, w.n,
                                                            w.m, w.k, SEED))


# --------------------------------------------------------- host entry points --

def test_host_entry_points(dev, oracle):
    import nasp_bloom as nbm
    from nasp_bloom import synth
    buf, offs = synth.var_keys(300_000)
    m, k = 2_875_518, 7
    words = np.zeros(nbm.nwords(m), np.uint64)
    nbm.build_host(buf, offs, 0, 300_000, m, k, SEED, 0, words)
    want = oracle.build(0, buf, offs, 0, 300_000, m, k, SEED)
    np.testing.assert_array_equal(words, want)
    ans = nbm.probe_host(buf, offs, 0, 300_000, m, k, SEED, 0, words)
    assert ans.all()
    fixed = synth.fixed_keys(100_000, 16)
    w2 = np.zeros(nbm.nwords(m), np.uint64)
    nbm.build_host(fixed, None, 16, 100_000, m, k, SEED, 1, w2)
    np.testing.assert_array_equal(w2, oracle.build(1, fixed, None, 16, 100_000, m, k, SEED))


def test_bloomfilter_class_mirror(dev, oracle, golden):
    """The reference test program's flow (BloomFilter/main.cpp:28-117) through the
    mirror class, checked against the oracle bit for bit."""
    import nasp_bloom as nbm
    added = ["Ana", "Marko", "Jelena", "Nikola", "Maja", "Stefan", "Marina", "Petar", "Ivana", "Luka"]
    bf = nbm.BloomFilter(20, 0.05, time_const=TC)
    for e in added:
        bf.add(e)
    assert all(bf.possiblyContains(e) for e in added)
    img = bf.serialize()
    keys = [e.encode() for e in added]
    buf, offs = pack(keys)
    w = oracle.build(0, buf, offs, 0, len(keys), bf.m, bf.k, bf.h2_seed)
    assert img == oracle.serialize(bf.m, bf.k, 0.05, TC, bf.h2_seed, w)
    # serialize / deserialize round trip; add after deserialize accumulates
    bf2 = nbm.BloomFilter.deserialize(img)
    assert bf2.serialize() == img
    bf2.add("Bogdan")
    assert bf2.possiblyContains("Bogdan") and all(bf2.possiblyContains(e) for e in added)
    # default filter: everything "possibly" present
    assert nbm.BloomFilter().possiblyContains("x")


# ------------------------------------------------------------ multi-GPU --

def test_or_merge_kernel(dev):
    import torch
    import nasp_bloom as nbm
    g = torch.Generator(device="cpu").manual_seed(5)
    for nsrc, nw in ((1, 1), (3, 1000), (8, 65_537)):
        src = torch.randint(-2**62, 2**62, (nsrc, nw + 3), generator=g, dtype=torch.int64)
        dst = torch.randint(-2**62, 2**62, (nw,), generator=g, dtype=torch.int64)
        want = dst.clone()
        for s in range(nsrc):
            want |= src[s, :nw]
        d_dst, d_src = dst.to(dev), src.to(dev)
        nbm.or_merge_device(d_dst, d_src, nw, nsrc, nw + 3)
        torch.cuda.synchronize()
        assert torch.equal(d_dst.cpu(), want)


def test_cooperative_build_single_rank(dev, oracle):
    """The cooperative (C5) path end to end on one GPU through RCCL (world size 1):
    partial build + all-to-all + HIP OR-merge + all-gather (forced), and the
    one-rank shortcut that returns the partial itself."""
    import os
    import torch
    import torch.distributed as dist
    from nasp_bloom import distributed as D
    from nasp_bloom import synth
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    n = 1_000_000
    buf = synth.fixed_keys(n, 32)
    want = oracle.build(0, buf, None, 32, n, synth.C5.m, synth.C5.k, SEED)
    for exchange in (True, False):  # through RCCL, then the one-rank shortcut
        full = D.build_cooperative(t_u8(buf, dev), None, 32, n, synth.C5.m, synth.C5.k, SEED, 0,
                                   exchange_single=exchange)
        torch.cuda.synchronize()
        got = full.cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(got[: want.size], want)
    # the build on a caller's non-current stream: it waits for the keys' producer on the
    # current stream (here a copy queued behind ~10 ms of matmuls, no host
    # synchronisation: ADVICE r05), and the merge (on the current stream) joins it
    # before the exchange; the phase marks bracket the build on that stream
    side = torch.cuda.Stream(device=dev)
    src = t_u8(buf, dev)
    torch.cuda.synchronize()
    keys = torch.zeros_like(src)
    busy = torch.rand(4096, 4096, device=dev)
    for _ in range(12):
        busy = busy @ busy * 1e-3
    keys.copy_(src)
    marks = []
    full = D.build_cooperative(keys, None, 32, n, synth.C5.m, synth.C5.k, SEED, 0, exchange_single=True,
                               stream=side, marks=marks)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(full.cpu().numpy().view(np.uint64)[: want.size], want)
    ph = D.phase_ms(marks)
    assert ph["build"] > 0 and set(ph) >= {"build", "all_to_all", "or_merge", "all_gather"}
    dist.destroy_process_group()


@pytest.mark.parametrize("kexact,wide", [(0, 0), (1, 0), (1, 1), (1, 2), (1, 3), (1, 4)])
def test_exact_k_kernels(dev, oracle, knobs, kexact, wide):
    """The bin kernels specialised for k = 7 (16-byte and variable-length keys;
    NB_BIN_WIDE=1: 2 304-key blocks, or 1 024-key blocks three per CU for filters
    of <= 384 tiles, 2 / 3 forcing either) and k = 10 (32-byte keys; NB_BIN_WIDE:
    1 792-key blocks, or 1 152-key blocks three per CU for few tiles and two-level
    pass 1, 4 forcing them), and the general
    k <= 8 / k <= 16 kernels they replace (NB_KEXACT=0), give the same bits as the
    oracle -- both flavours, chunked, single- and two-level."""
    from nasp_bloom import synth
    knobs(NB_KEXACT=kexact, NB_BIN_WIDE=wide, NB_BUILD_PATH="tiled", NB_CHUNK_KEYS=400_000)
    n = 1_000_003
    f16 = synth.fixed_keys(n, 16, seed=21)
    vb, vo = synth.var_keys(n)
    f32 = synth.fixed_keys(n, 32, seed=22)
    for flavor in (0, 1):
        for buf, offs, kl, m, k in ((f16, None, 16, 958_505_838, 7), (vb, vo, 0, 95_850_584, 7),
                                    (f32, None, 32, 2**32 - 1, 10), (f16, None, 16, 9_585_059, 7),
                                    (f32, None, 32, 95_850_584, 10), (f32, None, 32, 2**31 - 1, 10)):
            got = dev_build(dev, buf, offs, kl, n, m, k, SEED, flavor=flavor)
            np.testing.assert_array_equal(got, oracle.build(flavor, buf, offs, kl, n, m, k, SEED))
    # duplicated keys: one block's indices pile into a few tiles (ranks up to
    # KPT * NT * k - 1, the placement handles' widest case)
    dup16 = np.zeros(300_000 * 16 + 16, np.uint8)
    dup32 = np.zeros(300_000 * 32 + 16, np.uint8)
    for buf, kl, m, k in ((dup16, 16, 1_000_003, 7), (dup32, 32, 1_000_003, 10),
                          (dup32, 32, 2**32 - 1, 10)):
        got = dev_build(dev, buf, None, kl, 300_000, m, k, SEED)
        np.testing.assert_array_equal(got, oracle.build(0, buf, None, kl, 300_000, m, k, SEED))
