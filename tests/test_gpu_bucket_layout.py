"""GPU parity of both bucket layouts (round 4, bloom_kernels.hip bucket_region):
shard-major [G][T] (NB_BUCKET_GMAJOR=1, the default) and tile-major [T][G] (0), on
every path that writes or reads buckets -- the single-level bin kernel
(packed 21-bit and 32-bit entries, counted and power-of-two tiles, spill), the
two-level build (pass-1 Pack5 units, re-bin, fine tiles), the pipelined bin kernel and
the tiled probe in several key-range passes (NB_PROBE_CHUNK).  Bit-exact against the
oracle (BloomFilter::add / possiblyContains, BloomFilter.cpp:67-86)."""
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


# (m, k, key_len, extra knobs): counted tiles (C4's m), power-of-two tiles with 32-bit
# entries, a C2-sized filter, the two-level build (C5's m, k = 10, several passes)
CASES = [
    (958_505_838, 7, 16, {}),
    (958_505_838, 7, 16, {"NB_TILE_COUNT": "1", "NB_PACK": "0"}),
    (95_850_584, 7, 16, {"NB_CHUNK_KEYS": "70000"}),
    (2**32 - 1, 10, 32, {"NB_CHUNK_KEYS": "100000"}),
    (958_505_838, 7, 16, {"NB_BIN_PIPE": "1"}),
]


@pytest.mark.parametrize("gmajor", ["0", "1"])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_gmajor_build(dev, oracle, knobs, case, gmajor):
    from nasp_bloom import synth
    import nasp_bloom as nbm
    m, k, kl, extra = CASES[case]
    knobs(NB_BUILD_PATH="tiled", NB_BUCKET_GMAJOR=gmajor, **extra)
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


@pytest.mark.parametrize("gmajor", ["0", "1"])
@pytest.mark.parametrize("m,k,kl", [(958_505_838, 7, 16), (2**32 - 1, 10, 32)])
def test_gmajor_spill(dev, oracle, knobs, m, k, kl, gmajor):
    """Duplicated keys past the buckets' capacity (spill bitmap) in either layout,
    then a normal build is exact again (cursors and spill scratch clean)."""
    from nasp_bloom import synth
    import nasp_bloom as nbm
    knobs(NB_BUILD_PATH="tiled", NB_BUCKET_GMAJOR=gmajor, NB_CHUNK_KEYS="70000")
    stale = np.full(nbm.nwords(m), np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64)
    n = 300_000
    dup = np.zeros(n * kl + 16, np.uint8)
    dup[: kl * 500] = synth.fixed_keys(500, kl)[: kl * 500]
    got = build_into(dev, stale, dup, None, kl, n, m, k, overwrite=True)
    np.testing.assert_array_equal(got, oracle.build(0, dup, None, kl, n, m, k, SEED))
    buf = synth.fixed_keys(n, kl, seed=32)
    got = build_into(dev, stale, buf, None, kl, n, m, k, overwrite=True)
    np.testing.assert_array_equal(got, oracle.build(0, buf, None, kl, n, m, k, SEED))


@pytest.mark.parametrize("gmajor", ["0", "1"])
@pytest.mark.parametrize("chunk", ["0", "1000000"])
def test_gmajor_tiled_probe(dev, oracle, knobs, gmajor, chunk):
    """The tiled probe in either layout and in key-range passes: a filter of
    60 % of 4.5M keys probed over all of them, bit-exact."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    n, m, k, kl = 4_500_000, 958_505_838, 7, 16
    buf = synth.fixed_keys(n, kl, seed=33)
    npres = int(n * 0.6)
    wt = torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev)
    nbm.build_device(t_u8(buf, dev), None, kl, npres, m, k, SEED, 0, wt)
    torch.cuda.synchronize()
    words = wt.cpu().numpy().view(np.uint64)
    knobs(NB_PROBE_PATH="tiled", NB_BUCKET_GMAJOR=gmajor, NB_PROBE_CHUNK=chunk)
    got = dev_probe(dev, buf, None, kl, n, m, k, SEED, words, 0)
    np.testing.assert_array_equal(got, oracle.probe(0, buf, None, kl, n, m, k, SEED, words))
    assert got[:npres].all()
