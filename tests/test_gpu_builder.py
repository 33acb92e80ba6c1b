"""GPU parity of the streaming host builder (nb_builder_*, the host side of
SSTable::build's filter block, reference SSTable/SSTable.cpp:28-35): per-key adds
packed into pinned chunks, batch adds uploaded chunk by chunk, accumulation into
loaded bits, chunk-boundary and oversized keys -- all bit-exact against the
oracle (integer work: the bar is equality)."""
import numpy as np
import pytest

from golden_util import pack

pytestmark = pytest.mark.gpu

SEED = 17027509906831645879
CHUNK_KEYS = 1 << 20  # bloom_stream.cpp kChunkKeys
CHUNK_BYTES = 16 << 20  # bloom_stream.cpp kChunkBytes


@pytest.fixture(scope="module")
def dev(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return 0


def keys_list(buf, offs):
    return [bytes(buf[int(offs[i]):int(offs[i + 1])]) for i in range(len(offs) - 1)]


@pytest.mark.parametrize("flavor", [0, 1])
def test_builder_per_key_mixed_lengths(dev, oracle, flavor):
    """Per-key adds (BloomFilter::add), lengths 0..40 incl. empty keys and NULs."""
    import nasp_bloom as nbm
    from nasp_bloom import synth
    buf, offs = synth.var_keys(30_000, 0, 40)
    m, k = 300_007, 7
    with nbm.Builder(m, k, SEED, flavor) as b:
        for key in keys_list(buf, offs):
            b.add(key)
        got = b.finish()
    want = oracle.build(flavor, buf, offs, 0, 30_000, m, k, SEED)
    np.testing.assert_array_equal(got[: nbm.nwords(m)], want)


def test_builder_per_key_crosses_chunks_fixed16(dev, oracle):
    """More than one chunk of 16-byte keys added one by one: the fixed-length
    chunks travel without offsets and take the dwordx4 path; slots are reused."""
    import nasp_bloom as nbm
    from nasp_bloom import synth
    n = CHUNK_KEYS + 12_345
    buf = synth.fixed_keys(n, 16, seed=99)
    m, k = 9_585_059, 7
    raw = buf.tobytes()
    with nbm.Builder(m, k, SEED) as b:
        for i in range(n):
            b.add(raw[16 * i:16 * i + 16])
        got = b.finish()
    want = oracle.build(0, buf, None, 16, n, m, k, SEED)
    np.testing.assert_array_equal(got[: nbm.nwords(m)], want)


def test_builder_accumulates_into_init_words_and_continues(dev, oracle):
    """init_words = loaded bits (add-after-deserialize, TypesManager.cpp:84-86);
    finish() then more adds keep OR-ing into the same filter."""
    import nasp_bloom as nbm
    from nasp_bloom import synth
    buf, offs = synth.var_keys(60_000, 1, 50, seed=5)
    m, k = 1_000_003, 5
    first = oracle.build(0, buf, offs[:20_001], 0, 20_000, m, k, SEED)
    keys = keys_list(buf, offs)
    with nbm.Builder(m, k, SEED, init_words=first.copy()) as b:
        for key in keys[20_000:40_000]:
            b.add(key)
        mid = b.finish()
        for key in keys[40_000:]:
            b.add(key)
        got = b.finish()
    want_mid = oracle.build(0, buf, offs[:40_001], 0, 40_000, m, k, SEED)
    want = oracle.build(0, buf, offs, 0, 60_000, m, k, SEED)
    np.testing.assert_array_equal(mid[: nbm.nwords(m)], want_mid)
    np.testing.assert_array_equal(got[: nbm.nwords(m)], want)


def test_builder_add_batch_c2_full_size(dev, oracle):
    """C2 (10M x 16 B) through add_batch: ten chunks uploaded straight from the
    caller's buffer, each build overlapping the next upload."""
    import nasp_bloom as nbm
    from nasp_bloom import synth
    w = synth.C2
    buf, offs, kl = synth.keys_for(w)
    with nbm.Builder(w.m, w.k, SEED) as b:
        b.add_batch(buf, offs, kl, w.n)
        got = b.finish()
    want = oracle.build(0, buf, offs, kl, w.n, w.m, w.k, SEED)
    np.testing.assert_array_equal(got[: nbm.nwords(w.m)], want)


def test_builder_add_batch_async_buffers_kept(dev, oracle):
    """nb_builder_add_batch_async: many batches from distinct buffers (fixed and
    variable-length), enqueued without waiting for their uploads, a sync_uploads in
    the middle, then finish: bit-exact with the oracle; a second finish after more
    async batches accumulates."""
    import nasp_bloom as nbm
    from nasp_bloom import synth
    m, k = synth.C3.m, 7
    n = 1_200_000
    parts = [synth.fixed_keys(n, 16, seed=400 + i) for i in range(3)]
    vb, vo = synth.var_keys(900_000)
    with nbm.Builder(m, k, SEED) as b:
        for i, buf in enumerate(parts):
            b.add_batch_async(buf, None, 16, n)
            if i == 1:
                b.sync_uploads()
        got = b.finish()
        want = np.zeros(nbm.nwords(m), np.uint64)
        for buf in parts:
            want |= oracle.build(0, buf, None, 16, n, m, k, SEED)
        np.testing.assert_array_equal(got[: nbm.nwords(m)], want)
        b.add_batch_async(vb, vo, 0, 900_000)
        got = b.finish()
    want |= oracle.build(0, vb, vo, 0, 900_000, m, k, SEED)
    np.testing.assert_array_equal(got[: nbm.nwords(m)], want)


@pytest.mark.parametrize("flavor", [0, 1])
def test_builder_add_batch_varlen_byte_chunks(dev, oracle, flavor):
    """C3's shape (8-64 B keys): chunks cut by bytes, each copied from a 16-byte
    aligned start so the kernel's aligned staging reads stay inside the copy;
    a per-key add before the batch is flushed first."""
    import nasp_bloom as nbm
    from nasp_bloom import synth
    n = 1_500_000 if flavor == 0 else 300_000
    buf, offs = synth.var_keys(n)
    m, k = synth.C3.m, 7
    head = bytes(buf[int(offs[0]):int(offs[1])])
    with nbm.Builder(m, k, SEED, flavor) as b:
        b.add(head)
        b.add_batch(buf, offs, 0, n)
        got = b.finish()
    want = oracle.build(flavor, buf, offs, 0, n, m, k, SEED)
    np.testing.assert_array_equal(got[: nbm.nwords(m)], want)


def test_builder_oversized_and_empty_keys(dev, oracle):
    """A key longer than a chunk takes its own synchronous upload; empty keys
    alone make an offsets chunk (no zero-length fixed stride)."""
    import nasp_bloom as nbm
    rng = np.random.default_rng(3)
    big = rng.integers(0, 256, CHUNK_BYTES + 1000, dtype=np.uint8).tobytes()
    keys = [b"", b"", b"a", big, b"", b"tail-key"]
    buf, offs = pack(keys)
    m, k = 50_021, 4
    with nbm.Builder(m, k, SEED) as b:
        for key in keys:
            b.add(key)
        got = b.finish()
    want = oracle.build(0, buf, offs, 0, len(keys), m, k, SEED)
    np.testing.assert_array_equal(got[: nbm.nwords(m)], want)
    with nbm.Builder(m, k, SEED) as b:  # only empty keys
        for _ in range(3):
            b.add(b"")
        got = b.finish()
    buf, offs = pack([b""] * 3)
    np.testing.assert_array_equal(got[: nbm.nwords(m)],
                                  oracle.build(0, buf, offs, 0, 3, m, k, SEED))


def test_builder_k0_and_errors(dev):
    import nasp_bloom as nbm
    init = np.arange(1, 17, dtype=np.uint64)
    with nbm.Builder(1000, 0, SEED, init_words=init.copy()) as b:  # no closures: adds set nothing
        b.add(b"abc")
        np.testing.assert_array_equal(b.finish()[:16], init)
    with nbm.Builder(0, 3, SEED) as b:  # the reference divides by zero; the ABI refuses
        with pytest.raises(nbm.NaspBloomError, match="m == 0"):  # at add(), before any build
            b.add(b"abc")
        with pytest.raises(nbm.NaspBloomError):
            b.add_batch(np.zeros(32, np.uint8), None, 16, 2)
    with pytest.raises(nbm.NaspBloomError):
        nbm.Builder(100, 3, SEED, flavor=7)


def test_nb_build_fixed_key_longer_than_a_chunk(dev, oracle):
    """Fixed-length keys longer than the builder's 16 MiB chunk (nb_build ->
    add_batch) take the oversized-key path instead of overrunning the chunk."""
    import nasp_bloom as nbm
    kl = (16 << 20) + 1000
    n = 2
    buf = np.random.default_rng(5).integers(0, 256, n * kl + 16, dtype=np.uint8)
    m, k = 4099, 5
    w = np.zeros(nbm.nwords(m), np.uint64)
    nbm.build_host(buf, None, kl, n, m, k, SEED, 0, w)
    np.testing.assert_array_equal(w, oracle.build(0, buf, None, kl, n, m, k, SEED))


def test_python_mirror_places_batches(dev, oracle):
    """The Python BloomFilter mirror: a batch of >= HOST_BATCH_LIMIT keys is built
    on the device (a device build is counted), a smaller one on the host; both
    bit-exact with the oracle."""
    import nasp_bloom as nbm
    from golden_util import pack
    for n, on_dev in ((nbm.BloomFilter.HOST_BATCH_LIMIT - 1, False),
                      (nbm.BloomFilter.HOST_BATCH_LIMIT, True)):
        keys = [b"user%012d" % i for i in range(n)]
        bf = nbm.BloomFilter(n, 0.01, time_const=1748963255)
        before = nbm.device_build_count()
        bf.add_batch(keys)
        img = bf.serialize()
        assert bf.last_on_device == on_dev and (nbm.device_build_count() > before) == on_dev
        buf, offs = pack(keys)
        want = oracle.build(0, buf, offs, 0, n, bf.m, bf.k, bf.h2_seed)
        assert img == nbm.serialize(bf.m, bf.k, bf.p, bf.timeConst, bf.h2_seed, want)
