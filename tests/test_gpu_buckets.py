"""GPU parity of every path that writes or reads the shard-major buckets
(bloom_kernels.hip bucket_region, [G][T][cap]) -- the single-level bin kernel (packed
21-bit and 32-bit entries, counted and power-of-two tiles, spill), the two-level build
(pass-1 Pack5 units, re-bin, fine tiles) and the tiled probe in several key-range
passes (NB_PROBE_CHUNK) -- and, since round 5, counted tiles on every single-level
bin tail: round 4's unpacked tails found a tile by shifting, so a counted TileCfg that
reached one scattered out of range and needed a run-time refusal; every tail now maps
an index through the TileCfg's multiplier.  Bit-exact against the oracle
(BloomFilter::add / possiblyContains, BloomFilter.cpp:67-86)."""
import numpy as np
import pytest

from test_gpu_parity import SEED, dev_probe, t_u64, t_u8

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def build_into(dev, words_np, buf, offs, key_len, n, m, k, overwrite, flavor=0):
    import torch
    import nasp_bloom as nbm
    wt = t_u64(words_np, dev)
    nbm.build_device(t_u8(buf, dev), t_u64(offs, dev) if offs is not None else None, key_len, n, m, k,
                     SEED, flavor, wt, overwrite=overwrite)
    torch.cuda.synchronize()
    return wt.cpu().numpy().view(np.uint64)


# (m, k, key_len, extra knobs): counted tiles (C4's m, the packed two-tile tail), power-
# of-two tiles with 32-bit entries, a C2-sized filter, the two-level build (C5's m,
# k = 10, several passes); then counted tiles on the unpacked tails: 32-bit entries in
# the two-tile tail (NB_PACK=0 with an explicit tile count), the general tail with
# regenerated indices (NB_RANK=0), and k = 20 (> 16: no rank registers)
CASES = [
    (958_505_838, 7, 16, {}),
    (958_505_838, 7, 16, {"NB_TILE_COUNT": "1", "NB_PACK": "0"}),
    (95_850_584, 7, 16, {"NB_CHUNK_KEYS": "70000"}),
    (2**32 - 1, 10, 32, {"NB_CHUNK_KEYS": "100000"}),
    (958_505_838, 7, 16, {"NB_TILE_COUNT": "701", "NB_PACK": "0"}),
    (958_505_838, 7, 16, {"NB_TILE_COUNT": "1531", "NB_PACK": "0", "NB_RANK": "0"}),
    (958_505_838, 20, 16, {"NB_TILE_COUNT": "997", "NB_PACK": "0"}),
    (300_000_007, 7, 16, {"NB_TILE_COUNT": "333"}),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_buckets_build(dev, oracle, knobs, case):
    from nasp_bloom import synth
    import nasp_bloom as nbm
    m, k, kl, extra = CASES[case]
    knobs(NB_BUILD_PATH="tiled", **extra)
    n = 300_000
    buf = synth.fixed_keys(2 * n, kl, seed=31)
    stale = np.full(nbm.nwords(m), np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64)
    got = build_into(dev, stale, buf, None, kl, n, m, k, overwrite=True)
    np.testing.assert_array_equal(got, oracle.build(0, buf, None, kl, n, m, k, SEED))
    got2 = build_into(dev, got, buf[kl * n:], None, kl, n, m, k, overwrite=False)
    np.testing.assert_array_equal(got2, oracle.build(0, buf, None, kl, 2 * n, m, k, SEED))
    vbuf, voffs = synth.var_keys(n, 8, 64)
    got = build_into(dev, stale, vbuf, voffs, 0, n, m, k, overwrite=True, flavor=1)
    np.testing.assert_array_equal(got, oracle.build(1, vbuf, voffs, 0, n, m, k, SEED))


@pytest.mark.parametrize("m,k,kl,extra", [(958_505_838, 7, 16, {}), (2**32 - 1, 10, 32, {}),
                                          (958_505_838, 7, 16, {"NB_TILE_COUNT": "701", "NB_PACK": "0"}),
                                          (958_505_838, 7, 16, {"NB_TILE_COUNT": "1531", "NB_RANK": "0"})])
def test_buckets_spill(dev, oracle, knobs, m, k, kl, extra):
    """Duplicated keys past the buckets' capacity (spill bitmap, folded per counted
    or power-of-two tile), then a normal build is exact again (cursors and spill
    scratch clean)."""
    from nasp_bloom import synth
    import nasp_bloom as nbm
    knobs(NB_BUILD_PATH="tiled", NB_CHUNK_KEYS="70000", **extra)
    stale = np.full(nbm.nwords(m), np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64)
    n = 300_000
    dup = np.zeros(n * kl + 16, np.uint8)
    dup[: kl * 500] = synth.fixed_keys(500, kl)[: kl * 500]
    got = build_into(dev, stale, dup, None, kl, n, m, k, overwrite=True)
    np.testing.assert_array_equal(got, oracle.build(0, dup, None, kl, n, m, k, SEED))
    buf = synth.fixed_keys(n, kl, seed=32)
    got = build_into(dev, stale, buf, None, kl, n, m, k, overwrite=True)
    np.testing.assert_array_equal(got, oracle.build(0, buf, None, kl, n, m, k, SEED))


@pytest.mark.parametrize("entry", [32, 64])
@pytest.mark.parametrize("path", ["tiled", "split"])
@pytest.mark.parametrize("chunk", ["0", "1000000", "777777"])
def test_buckets_tiled_probe(dev, oracle, knobs, chunk, path, entry):
    """The tiled probe in key-range passes: a filter of 60 % of 4.5M keys probed
    over all of them, bit-exact; the split path's second round runs each pass over
    that pass's compacted survivors (ids relative to the pass)."""
    import torch
    import nasp_bloom as nbm
    n, m, k, kl = 4_500_000, 958_505_838, 7, 16
    from nasp_bloom import synth
    buf = synth.fixed_keys(n, kl, seed=33)
    npres = int(n * 0.6)
    wt = torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev)
    nbm.build_device(t_u8(buf, dev), None, kl, npres, m, k, SEED, 0, wt)
    torch.cuda.synchronize()
    words = wt.cpu().numpy().view(np.uint64)
    knobs(NB_PROBE_PATH=path, NB_PROBE_CHUNK=chunk, NB_PROBE_ENTRY=entry)
    got = dev_probe(dev, buf, None, kl, n, m, k, SEED, words, 0)
    np.testing.assert_array_equal(got, oracle.probe(0, buf, None, kl, n, m, k, SEED, words))
    assert got[:npres].all()


@pytest.mark.parametrize("chunk", ["0", "900001"])
def test_split_probe_unaligned_answers(dev, oracle, knobs, chunk):
    """The split probe's survivor compaction reads the answers four bytes at a time
    only when they are 4-byte aligned: an answer buffer starting one byte into its
    allocation, an odd key count and key-range passes of an odd size (so every pass
    after the first starts unaligned too) take the byte-wise path, bit-exact against
    the oracle (BloomFilter::possiblyContains, BloomFilter.cpp:67-80)."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    n, m, k, kl = 4_500_003, 958_505_838, 7, 16
    buf = synth.fixed_keys(n, kl, seed=34)
    npres = int(n * 0.3)
    wt = torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev)
    nbm.build_device(t_u8(buf, dev), None, kl, npres, m, k, SEED, 0, wt)
    torch.cuda.synchronize()
    words = wt.cpu().numpy().view(np.uint64)
    knobs(NB_PROBE_PATH="split", NB_PROBE_CHUNK=chunk)
    backing = torch.full((n + 8,), 7, dtype=torch.uint8, device=dev)
    out = backing[1:n + 1]
    nbm.probe_device(t_u8(buf, dev), None, kl, n, m, k, SEED, 0, wt, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got, oracle.probe(0, buf, None, kl, n, m, k, SEED, words))
    assert got[:npres].all()
    b = backing.cpu().numpy()
    assert b[0] == 7 and (b[n + 1:] == 7).all()  # nothing written outside the answers
