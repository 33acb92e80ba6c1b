"""GPU parity of the counted-tile build (round 4, bloom_kernels.hip TileCfg /
counted_tiles): the single-level packed path cut into any number of tiles, T a whole
number of tile-kernel rounds by default (C3 / C4's m: 768 tiles instead of 915), so
tile boundaries fall inside filter words and the two words holding a boundary are
ORed in atomically -- zeroed first by the bin kernel when the build overwrites.
Bit-exact against the oracle (BloomFilter::add, BloomFilter.cpp:82-86) in overwrite
mode over stale words, in accumulate mode over loaded words, across chunks, and with
duplicated keys that spill past the buckets' capacity."""
import numpy as np
import pytest

from test_gpu_parity import SEED, t_u64, t_u8

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


# (m, NB_TILE_COUNT): 0 = the policy (C4's m: 768; 2^31 - 1: too many tiles for the
# wide bin kernel, so power-of-two tiles), else exactly that many tiles -- odd
# counts, a C2-sized m the policy leaves alone, ragged last tiles
CASES = [(958_505_838, "0"), (958_505_838, "733"), (958_505_838, "1000"), (300_000_001, "300"),
         (2**30 + 7, "1024"), (95_850_584, "300"), (2**31 - 1, "0")]


@pytest.mark.parametrize("m,tiles", CASES)
def test_counted_tiles_overwrite_and_accumulate(dev, oracle, knobs, m, tiles):
    from nasp_bloom import synth
    import nasp_bloom as nbm
    knobs(NB_BUILD_PATH="tiled", NB_TILE_COUNT=tiles)
    n, k = 300_000, 7
    buf = synth.fixed_keys(2 * n, 16, seed=21)
    stale = np.full(nbm.nwords(m), np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64)
    got = build_into(dev, stale, buf, None, 16, n, m, k, overwrite=True)
    want = oracle.build(0, buf, None, 16, n, m, k, SEED)
    np.testing.assert_array_equal(got, want)
    # accumulate: the second half ORed into the first half's words (deserialize + add)
    got2 = build_into(dev, got, buf[16 * n:], None, 16, n, m, k, overwrite=False)
    np.testing.assert_array_equal(got2, oracle.build(0, buf, None, 16, 2 * n, m, k, SEED))
    # variable-length keys, MSVC flavour, overwrite over stale words
    vbuf, voffs = synth.var_keys(n, 8, 64)
    got = build_into(dev, stale, vbuf, voffs, 0, n, m, k, overwrite=True, flavor=1)
    np.testing.assert_array_equal(got, oracle.build(1, vbuf, voffs, 0, n, m, k, SEED))


@pytest.mark.parametrize("tiles", ["0", "733"])
def test_counted_tiles_chunks_and_spill(dev, oracle, knobs, tiles):
    """Several bin/tile passes (the first overwrites, the rest OR in) and duplicated
    keys past the buckets' capacity (the spill bitmap, folded per tile with boundary
    words shared between two tiles' blocks) over stale words; afterwards a normal
    build is exact again (cursors and spill scratch left clean)."""
    from nasp_bloom import synth
    import nasp_bloom as nbm
    m, k = 958_505_838, 7
    knobs(NB_BUILD_PATH="tiled", NB_TILE_COUNT=tiles, NB_CHUNK_KEYS="70000")
    stale = np.full(nbm.nwords(m), np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64)
    n = 300_000
    dup = np.zeros(n * 16 + 16, np.uint8)
    dup[: 16 * 500] = synth.fixed_keys(500, 16)[: 16 * 500]
    got = build_into(dev, stale, dup, None, 16, n, m, k, overwrite=True)
    np.testing.assert_array_equal(got, oracle.build(0, dup, None, 16, n, m, k, SEED))
    buf, offs = synth.var_keys(250_000, 4, 40)
    got = build_into(dev, stale, buf, offs, 0, 250_000, m, k, overwrite=True)
    np.testing.assert_array_equal(got, oracle.build(0, buf, offs, 0, 250_000, m, k, SEED))
