"""GPU parity of the pipelined bin kernel (round 4, bloom_kernels.hip
bloom_bin_pipe_kernel, NB_BIN_PIPE=1; off by default: measured 1.52 vs 0.96 ms for
C4's bin pass): one persistent block per CU, two LDS batch buffers,
hashing of batch i overlapped with the write-out of batch i-1.  Bit-exact against the oracle
(BloomFilter::add, BloomFilter.cpp:82-86) for C4-shaped builds (16-byte keys, k = 7,
385-1 024 tiles) with one batch per block and with many (both LDS buffers in turn),
ragged last batches, overwrite over stale words, accumulate, chunks and duplicated
keys past the buckets' capacity (the spill path of its write-out)."""
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


def build_into(dev, words_np, buf, n, m, k, overwrite):
    import torch
    import nasp_bloom as nbm
    wt = t_u64(words_np, dev)
    nbm.build_device(t_u8(buf, dev), None, 16, n, m, k, SEED, 0, wt, overwrite=overwrite)
    torch.cuda.synchronize()
    return wt.cpu().numpy().view(np.uint64)


# n: one key, one batch +- 1 (2 304 keys), one batch per block of the 256-block grid
# and several per block (the second LDS buffer), ragged
@pytest.mark.parametrize("n,tiles", [(2305, "0"), (1_500_001, "0"), (3_000_000, "1")])  # "0" counted
# (768) tiles, "1" power-of-two (915) tiles
def test_bin_pipe_c4_shape(dev, oracle, knobs, n, tiles):
    from nasp_bloom import synth
    import nasp_bloom as nbm
    knobs(NB_BUILD_PATH="tiled", NB_BIN_PIPE="1", NB_TILE_COUNT=tiles)
    m, k = 958_505_838, 7
    buf = synth.fixed_keys(n + 300_000, 16, seed=31)
    stale = np.full(nbm.nwords(m), np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64)
    got = build_into(dev, stale, buf, n, m, k, overwrite=True)
    np.testing.assert_array_equal(got, oracle.build(0, buf, None, 16, n, m, k, SEED))
    got2 = build_into(dev, got, buf[16 * n:], 300_000, m, k, overwrite=False)
    np.testing.assert_array_equal(got2, oracle.build(0, buf, None, 16, n + 300_000, m, k, SEED))


def test_bin_pipe_spill_chunks_and_other_m(dev, oracle, knobs):
    """Duplicated keys past the capacity (spills) over stale words, in chunks; and a
    filter of 2^30 + 7 bits (1 024 counted tiles)."""
    from nasp_bloom import synth
    import nasp_bloom as nbm
    knobs(NB_BUILD_PATH="tiled", NB_BIN_PIPE="1", NB_CHUNK_KEYS="700000")
    m, k = 958_505_838, 7
    n = 1_600_000
    dup = np.zeros(n * 16 + 16, np.uint8)
    dup[: 16 * 800] = synth.fixed_keys(800, 16)[: 16 * 800]
    stale = np.full(nbm.nwords(m), np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64)
    got = build_into(dev, stale, dup, n, m, k, overwrite=True)
    np.testing.assert_array_equal(got, oracle.build(0, dup, None, 16, n, m, k, SEED))
    knobs(NB_CHUNK_KEYS="0", NB_TILE_COUNT="1024")
    m2 = 2**30 + 7
    buf = synth.fixed_keys(1_200_000, 16, seed=32)
    got = build_into(dev, np.zeros(nbm.nwords(m2), np.uint64), buf, 1_200_000, m2, k, overwrite=False)
    np.testing.assert_array_equal(got, oracle.build(0, buf, None, 16, 1_200_000, m2, k, SEED))


@pytest.mark.parametrize("n", [2305, 30_721, 1_500_001])
def test_bin_mix_c4_shape(dev, oracle, knobs, n):
    """NB_BIN_MIX: bin blocks of two sizes (2 304 / 1 536 keys; 16-block groups, the
    last group ragged and partly empty) give the same filter, overwrite and
    accumulate."""
    from nasp_bloom import synth
    import nasp_bloom as nbm
    knobs(NB_BUILD_PATH="tiled", NB_BIN_MIX="1")
    m, k = 958_505_838, 7
    buf = synth.fixed_keys(n + 100_000, 16, seed=33)
    stale = np.full(nbm.nwords(m), np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64)
    got = build_into(dev, stale, buf, n, m, k, overwrite=True)
    np.testing.assert_array_equal(got, oracle.build(0, buf, None, 16, n, m, k, SEED))
    got2 = build_into(dev, got, buf[16 * n:], 100_000, m, k, overwrite=False)
    np.testing.assert_array_equal(got2, oracle.build(0, buf, None, 16, n + 100_000, m, k, SEED))
