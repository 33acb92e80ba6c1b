"""nb_build_sharded: the single-process multi-GPU build (keys split into shard
ranges, one streaming builder and host thread per shard, partials OR-merged by
owner slices over peer copies).  Parity with the oracle's one-filter build is the
bar (bit-exact).  On a one-GPU box every shard runs on device 0 (shard s on device
s % device_count), which still exercises the split, the concurrent builders and
the slice-wise merge; only the xGMI copies themselves become local ones."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 17027509906831645879


@pytest.fixture(scope="module")
def nbm(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import nasp_bloom
    return nasp_bloom


@pytest.mark.parametrize("nshards", [0, 1, 2, 3, 8])
@pytest.mark.parametrize("flavor", [0, 1])
def test_sharded_varlen_matches_oracle(nbm, oracle, nshards, flavor):
    from nasp_bloom import synth
    n = 400_003
    buf, offs = synth.var_keys(n)
    m, k = 3_834_023, 7
    words = np.zeros(nbm.nwords(m), np.uint64)
    nbm.build_host_sharded(buf, offs, 0, n, m, k, SEED, flavor, words, nshards)
    np.testing.assert_array_equal(words, oracle.build(flavor, buf, offs, 0, n, m, k, SEED))


@pytest.mark.parametrize("nshards", [2, 5])
def test_sharded_fixed16_c2_full_size(nbm, oracle, nshards):
    from nasp_bloom import synth
    w = synth.WORKLOADS["c2"]
    buf, offs, kl = synth.keys_for(w)
    words = np.zeros(nbm.nwords(w.m), np.uint64)
    nbm.build_host_sharded(buf, offs, kl, w.n, w.m, w.k, SEED, 0, words, nshards)
    np.testing.assert_array_equal(words, oracle.build(0, buf, offs, kl, w.n, w.m, w.k, SEED))


def test_sharded_accumulates_and_edges(nbm, oracle):
    from nasp_bloom import synth
    buf, offs = synth.var_keys(50_000)
    m, k = 479_253, 7
    # OR-accumulate onto the caller's bits (add() after deserialize())
    first = oracle.build(0, buf, offs[:20_001], 0, 20_000, m, k, SEED)
    words = first.copy()
    tail = offs[20_000:]
    nbm.build_host_sharded(buf, tail, 0, 30_000, m, k, SEED, 0, words, 4)
    np.testing.assert_array_equal(words, oracle.build(0, buf, offs, 0, 50_000, m, k, SEED))
    # fewer keys than shards, and fewer words than shards
    few = np.zeros(nbm.nwords(m), np.uint64)
    nbm.build_host_sharded(buf, offs[:4], 0, 3, m, k, SEED, 0, few, 8)
    np.testing.assert_array_equal(few, oracle.build(0, buf, offs[:4], 0, 3, m, k, SEED))
    tiny = np.zeros(1, np.uint64)
    nbm.build_host_sharded(buf, offs[:101], 0, 100, 20, 3, SEED, 1, tiny, 6)
    np.testing.assert_array_equal(tiny, oracle.build(1, buf, offs[:101], 0, 100, 20, 3, SEED))
    # no keys / k == 0: words untouched
    keep = first.copy()
    nbm.build_host_sharded(buf, offs[:1], 0, 0, m, k, SEED, 0, keep, 4)
    nbm.build_host_sharded(buf, offs, 0, 50_000, m, 0, SEED, 0, keep, 4)
    np.testing.assert_array_equal(keep, first)
    # errors reported, not thrown across the ABI
    with pytest.raises(nbm.NaspBloomError):
        nbm.build_host_sharded(buf, offs, 0, 10, 0, 3, SEED, 0, np.zeros(1, np.uint64), 2)
    with pytest.raises(nbm.NaspBloomError):
        nbm.build_host_sharded(buf, offs, 0, 10, m, 3, SEED, 7, words, 2)


@pytest.mark.parametrize("nshards", [2, 3, 8])
def test_sharded_forced_staging(nbm, oracle, knobs, nshards):
    """NB_SHARDED_STAGE=1: every source of the slice merge goes through the
    blocking hipMemcpyPeer staging branch (taken for real only between devices
    without peer access), bit-exact against the oracle, both key layouts."""
    from nasp_bloom import synth
    knobs(NB_SHARDED_STAGE=1)
    n = 300_007
    buf, offs = synth.var_keys(n)
    m, k = 2_875_519, 7
    words = np.zeros(nbm.nwords(m), np.uint64)
    nbm.build_host_sharded(buf, offs, 0, n, m, k, SEED, 0, words, nshards)
    np.testing.assert_array_equal(words, oracle.build(0, buf, offs, 0, n, m, k, SEED))
    fb = synth.fixed_keys(n, 16)
    fw = np.zeros(nbm.nwords(m), np.uint64)
    nbm.build_host_sharded(fb, None, 16, n, m, k, SEED, 1, fw, nshards)
    np.testing.assert_array_equal(fw, oracle.build(1, fb, None, 16, n, m, k, SEED))
