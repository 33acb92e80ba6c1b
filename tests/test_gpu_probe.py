"""GPU parity of the batch probe (BloomFilter::possiblyContains, BloomFilter.cpp:67-80,
callers SSTManager.cpp:203,224) on every path: the lane kernel (one lane per key,
early exit), the tiled path (probe_bin_kernel + probe_tile_kernel: lookups binned by
filter tile and tested in LDS), the split tiled path (round 5: two rounds, the
second over the keys the first one's two indices left at 1) and auto (a sampled
prefix picks the path on the device).  Bit-exact against oracle.probe on mixed present / absent batches; the
tiled and lane answers equal each other at C4's full size."""
import numpy as np
import pytest

from test_gpu_parity import SEED, dev_probe, t_u8, t_u64  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def device_words(dev, buf, offs, key_len, n, m, k, flavor=0):
    """The filter of the first n keys, built on the device (its parity is tested
    elsewhere), as host words."""
    import torch
    import nasp_bloom as nbm
    wt = torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev)
    nbm.build_device(t_u8(buf, dev), t_u64(offs[:n + 1], dev) if offs is not None else None, key_len, n,
                     m, k, SEED, flavor, wt)
    torch.cuda.synchronize()
    return wt.cpu().numpy().view(np.uint64)


def shapes():
    from nasp_bloom import synth
    n = 4_500_000
    f16 = synth.fixed_keys(n, 16, seed=5)
    var, voffs = synth.var_keys(n, 8, 64)
    f32 = synth.fixed_keys(n, 32, seed=6)
    return {
        "c4_fixed16": (f16, None, 16, n, 958_505_838, 7, 0),
        "c3_varlen": (var, voffs, 0, n, 958_505_838, 7, 0),
        "c3_varlen_fnv": (var, voffs, 0, n, 958_505_838, 7, 1),
        "c2_fixed16_fnv": (f16, None, 16, n, 95_850_584, 7, 1),
        "c5_fixed32_k10": (f32, None, 32, n, 2**32 - 1, 10, 0),
    }


@pytest.fixture(scope="module")
def probe_shapes():
    return shapes()


@pytest.mark.parametrize("path", ["lane", "tiled", "split", "auto"])
@pytest.mark.parametrize("shape", ["c4_fixed16", "c3_varlen", "c3_varlen_fnv", "c2_fixed16_fnv", "c5_fixed32_k10"])
@pytest.mark.parametrize("present_first", [True, False])
def test_probe_paths_match_oracle(dev, oracle, knobs, probe_shapes, path, shape, present_first):
    """A filter of 60 % of the batch's keys, probed over all of them: present keys,
    absent keys and the filter's false positives, bit-exact on every path.  With the
    present keys first, auto's sample sees hits (tiled); absent first, misses (lane)."""
    buf, offs, kl, n, m, k, fl = probe_shapes[shape]
    knobs(NB_PROBE_PATH=path)
    npres = int(n * 0.6)
    if present_first:
        words = device_words(dev, buf, offs, kl, npres, m, k, fl)
    else:  # the filter of the last 60 % of the keys
        if offs is None:
            words = device_words(dev, buf[(n - npres) * kl:], None, kl, npres, m, k, fl)
        else:
            sh = offs[n - npres:] - offs[n - npres]
            words = device_words(dev, buf[int(offs[n - npres]):], sh, 0, npres, m, k, fl)
    got = dev_probe(dev, buf, offs, kl, n, m, k, SEED, words, fl)
    want = oracle.probe(fl, buf, offs, kl, n, m, k, SEED, words)
    np.testing.assert_array_equal(got, want)
    lo, hi = (0, npres) if present_first else (n - npres, n)
    assert got[lo:hi].all()
    assert got.mean() - 0.6 < 0.02  # the absent 40 %: false positives only


@pytest.mark.parametrize("entry", [32, 64])
@pytest.mark.parametrize("path", ["tiled", "split"])
@pytest.mark.parametrize("shape", ["c4_fixed16", "c3_varlen", "c3_varlen_fnv", "c2_fixed16_fnv", "c5_fixed32_k10"])
def test_probe_entry_formats(dev, oracle, knobs, probe_shapes, path, shape, entry):
    """Both tiled-probe bucket formats (NB_PROBE_ENTRY): 32-bit entries behind run
    headers (round 6, the default) and round 3-5's key << 32 | offset words, on every
    shape of both tiled paths, bit-exact against the oracle; the 32-bit tile kernel's
    segments start inside runs and find their header by a backward look."""
    buf, offs, kl, n, m, k, fl = probe_shapes[shape]
    knobs(NB_PROBE_PATH=path, NB_PROBE_ENTRY=entry)
    npres = int(n * 0.3)
    words = device_words(dev, buf, offs, kl, npres, m, k, fl)
    got = dev_probe(dev, buf, offs, kl, n, m, k, SEED, words, fl)
    np.testing.assert_array_equal(got, oracle.probe(fl, buf, offs, kl, n, m, k, SEED, words))
    assert got[:npres].all()


@pytest.mark.parametrize("entry", [32, 64])
@pytest.mark.parametrize("path", ["tiled", "split"])
def test_tiled_probe_overflow_and_small_filter(dev, oracle, knobs, path, entry):
    """Duplicated keys overflow the probe's buckets (those entries are tested in the
    bin kernel instead; with 32-bit entries a truncated run keeps its header and a run
    of one key's thousand copies is ~7 000 words long, so segments look back far); a
    small filter (few, small tiles); k = 1 (the split path then runs one round), k = 3
    and k = 8."""
    knobs(NB_PROBE_PATH=path, NB_PROBE_ENTRY=entry)
    from nasp_bloom import synth
    n = 400_000
    dup = np.zeros(n * 16 + 16, np.uint8)
    dup[: 16 * 1000] = synth.fixed_keys(1000, 16)[: 16 * 1000]
    for m, k in ((958_505_838, 7), (1_000_003, 8), (2**20 + 5, 1), (3_000_017, 3)):
        words = oracle.build(0, dup, None, 16, 2000, m, k, SEED)  # 1000 distinct + zero keys
        got = dev_probe(dev, dup, None, 16, n, m, k, SEED, words)
        np.testing.assert_array_equal(got, oracle.probe(0, dup, None, 16, n, m, k, SEED, words))
        assert got.all()
    vb, vo = synth.var_keys(300_000, 0, 70)  # empty keys included
    words = oracle.build(1, vb, vo, 0, 150_000, 5_000_011, 7, SEED)
    np.testing.assert_array_equal(dev_probe(dev, vb, vo, 0, 300_000, 5_000_011, 7, SEED, words, 1),
                                  oracle.probe(1, vb, vo, 0, 300_000, 5_000_011, 7, SEED, words))


def test_tiled_probe_c4_full_size(dev, knobs):
    """C4's 100M-key filter probed with 100M present keys and 100M absent ones: the
    tiled path answers 1 for every present key and exactly what the lane path
    answers for the absent ones (the filter's false positives)."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    w = synth.C4
    g = torch.Generator(device=dev).manual_seed(synth.SEED + 9)
    kt = torch.randint(0, 256, (2 * w.n * 16,), dtype=torch.uint8, device=dev, generator=g)
    words = torch.zeros(nbm.nwords(w.m), dtype=torch.int64, device=dev)
    nbm.build_device(kt, None, 16, w.n, w.m, w.k, SEED, 0, words, overwrite=True)
    outs = {}
    for path in ("tiled", "split", "lane"):
        knobs(NB_PROBE_PATH=path)
        out = torch.zeros(2 * w.n, dtype=torch.uint8, device=dev)
        nbm.probe_device(kt, None, 16, 2 * w.n, w.m, w.k, SEED, 0, words, out)
        torch.cuda.synchronize()
        outs[path] = out
    assert int(outs["tiled"][: w.n].min()) == 1
    assert torch.equal(outs["tiled"], outs["lane"])
    assert torch.equal(outs["split"], outs["lane"])
    fp = float(outs["lane"][w.n:].float().mean())
    assert 0.008 < fp < 0.012


@pytest.mark.parametrize("m, k, n", [(2**25, 4, 4_500_000), (2**25 + 1, 4, 4_500_000),
                                     (40_250_003, 3, 16_800_000), (95_850_584, 5, 16_800_000)])
@pytest.mark.parametrize("pc", [0, 30, 100])
def test_auto_policy_boundaries(dev, oracle, knobs, m, k, n, pc):
    """Auto at the shape rules' edges (round 6, profiles/r06sh_auto_shapes.txt): a
    filter of 2^25 bits (lane, no sample) and one bit more (lane / tiled at 10 %);
    k = 3 (no split round) and k = 5 at 2^24 + 22 784 keys (split back in the choice),
    each on absent, 30 % present and present batches, bit-exact against the oracle."""
    from nasp_bloom import synth
    knobs(NB_PROBE_PATH="auto", NB_PROBE_SPLIT_PCT="0", NB_PROBE_TILED_PCT="0")
    base = synth.fixed_keys(n, 16, seed=31)
    words = oracle.build(0, base, None, 16, n // 2, m, k, SEED)
    batch = synth.fixed_keys(n, 16, seed=32)
    idx = np.nonzero(np.arange(n) % 10 < pc // 10)[0]
    bv, pv = batch[: n * 16].reshape(n, 16), base[: n * 16].reshape(n, 16)
    bv[idx] = pv[idx % (n // 2)]
    got = dev_probe(dev, batch, None, 16, n, m, k, SEED, words)
    np.testing.assert_array_equal(got, oracle.probe(0, batch, None, 16, n, m, k, SEED, words))
    assert got[idx].all()


@pytest.mark.parametrize("path", ["tiled", "split", "auto"])
@pytest.mark.parametrize("k", [11, 12, 16])
def test_probe_32byte_keys_large_k_full_filter(dev, oracle, knobs, path, k):
    """32-byte keys at k = 11..16 over m = 2^32 - 1 (4 096 probe tiles): the tiled bin
    kernel's LDS (sorted indices + their keys) fits a workgroup's 160 KiB up to k = 11
    and not from k = 12 on (163 968 B), so those batches must take the lane path --
    before the auto sample writes anything -- and still answer bit-exactly (ADVICE
    r03: the tiled launch used to fail with NB_ERR_HIP)."""
    from nasp_bloom import synth
    knobs(NB_PROBE_PATH=path)
    n, m = 4_200_000, 2**32 - 1
    buf = synth.fixed_keys(n, 32, seed=11)
    npres = int(n * 0.6)
    words = device_words(dev, buf, None, 32, npres, m, k)
    got = dev_probe(dev, buf, None, 32, n, m, k, SEED, words)
    want = oracle.probe(0, buf, None, 32, n, m, k, SEED, words)
    np.testing.assert_array_equal(got, want)
    assert got[:npres].all()


@pytest.mark.parametrize("shape", ["c4_fixed16", "c5_fixed32_k10"])
@pytest.mark.parametrize("split_pct", ["0", "7", "101"])
@pytest.mark.parametrize("pc", [5, 30, 70])
def test_auto_mixed_batches(dev, oracle, knobs, probe_shapes, pc, split_pct, shape):
    """Auto on batches whose sample sees pc % present keys (every key i with
    i % 20 < pc / 5 present): lane, split (NB_PROBE_SPLIT_PCT=7: from 7 % to 65 % / 55 %)
    or tiled, bit-exact against the oracle whichever it picks; NB_PROBE_SPLIT_PCT 0 is
    the policy, which at 4.5M keys (< 2^24) leaves the split path out (lane / tiled at
    10 %), as does NB_PROBE_SPLIT_PCT=101."""
    from nasp_bloom import synth
    buf, offs, kl, n, m, k, fl = probe_shapes[shape]
    knobs(NB_PROBE_PATH="auto", NB_PROBE_SPLIT_PCT=split_pct)
    npres = n // 2
    words = device_words(dev, buf, None, kl, npres, m, k, fl)
    absent = synth.fixed_keys(n, kl, seed=77)
    mixed = absent.copy()
    idx = np.nonzero(np.arange(n) % 20 < pc // 5)[0]
    mv, bv = mixed[: n * kl].reshape(n, kl), buf[: n * kl].reshape(n, kl)
    mv[idx] = bv[idx % npres]
    got = dev_probe(dev, mixed, None, kl, n, m, k, SEED, words, fl)
    want = oracle.probe(fl, mixed, None, kl, n, m, k, SEED, words)
    np.testing.assert_array_equal(got, want)
    assert got[idx].all()


@pytest.mark.parametrize("pc", [5, 30, 70])
def test_auto_mixed_batches_varlen(dev, oracle, knobs, probe_shapes, pc):
    """The same for variable-length keys (C3's shape): the filter of all the keys, the
    batch the same keys with the first byte changed except where i % 20 < pc / 5 --
    lane, split (NB_PROBE_SPLIT_PCT=18, the policy's threshold on larger batches: 18-40 %;
    its second round hashes the listed keys straight from HBM) or tiled, bit-exact
    against the oracle."""
    buf, offs, kl, n, m, k, fl = probe_shapes["c3_varlen"]
    knobs(NB_PROBE_PATH="auto", NB_PROBE_SPLIT_PCT="18")
    words = device_words(dev, buf, offs, kl, n, m, k, fl)
    keep = np.arange(n) % 20 < pc // 5
    mixed = buf.copy()
    starts = offs[:-1].astype(np.int64)
    mixed[starts[~keep]] ^= 0x5A
    got = dev_probe(dev, mixed, offs, kl, n, m, k, SEED, words, fl)
    want = oracle.probe(fl, mixed, offs, kl, n, m, k, SEED, words)
    np.testing.assert_array_equal(got, want)
    assert got[keep].all()
