"""hipGraph capture of the device build (include/nasp_bloom.h: "warm a stream up with
its largest shape before capturing it into a hipGraph"): the captured bin + tile
launches replayed on new keys written into the same buffers give the oracle's
filter, bit-exact, for the fixed-16 and the variable-length paths."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 17027509906831645879


@pytest.fixture(scope="module")
def dev(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("var", [False, True])
def test_build_replayed_from_graph(dev, oracle, var):
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    n, m, k = 500_000, 4_792_530, 7
    if var:
        sets = [synth.var_keys(n, seed=synth.SEED + s) for s in range(3)]
        ot = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    else:
        sets = [(synth.fixed_keys(n, 16, seed=synth.SEED + s), None) for s in range(3)]
        ot = None
    # one key buffer large enough for every set (replays reuse the captured pointers)
    kt = torch.zeros(max(b.size for b, _ in sets), dtype=torch.uint8, device=dev)
    words = torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev)
    kl = 0 if var else 16
    st = torch.cuda.Stream(device=dev)

    def load(i):
        buf, offs = sets[i]
        kt[:buf.size].copy_(torch.from_numpy(buf))
        if var:
            ot.copy_(torch.from_numpy(offs.view(np.int64)))

    def build():
        nbm.build_device(kt, ot, kl, n, m, k, SEED, 0, words, stream=st, overwrite=True)

    load(0)
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        build()  # warm-up: sizes the stream's workspace
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        build()
    for i in (1, 2, 0):
        load(i)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        buf, offs = sets[i]
        want = oracle.build(0, buf, offs, kl, n, m, k, SEED)
        np.testing.assert_array_equal(words.cpu().numpy().view(np.uint64), want)


def test_auto_probe_replayed_from_graph(dev, oracle):
    """The auto probe under stream capture: its sample's count stays on the device,
    every path (lane, tiled, split) is captured and gated on it.  One captured graph
    replayed on present keys (tiled chosen), absent keys (lane), 30 % present (split:
    its compaction's count and the second round's list come from the replay) and 80 %
    present (tiled) gives the oracle's answers every time (the split
    sequence was never the open path on a replay).  NB_PROBE_SPLIT_PCT=7 keeps the split
    path in the choice at this size (the policy leaves it out below 2^24 keys)."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    n, m, k = 4_200_000, 40_250_003, 7
    base = synth.fixed_keys(n, 16, seed=71)
    words_np = oracle.build(0, base, None, 16, n, m, k, SEED)
    other = synth.fixed_keys(n, 16, seed=72)

    def mixed(pc):  # keys i with i % 10 < pc / 10 present
        b = other.copy()
        bv, pv = b[:n * 16].reshape(n // 10, 10, 16), base[:n * 16].reshape(n // 10, 10, 16)
        bv[:, :pc // 10] = pv[:, :pc // 10]
        return b
    kt = torch.from_numpy(base).to(dev)
    words = torch.from_numpy(words_np.view(np.int64)).to(dev)
    out = torch.zeros(n, dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(device=dev)
    with nbm.knobs(NB_PROBE_PATH="auto", NB_PROBE_SPLIT_PCT=7, NB_PROBE_TILED_PCT=0):
        with torch.cuda.stream(st):  # warm-up: sizes the workspace for every path
            nbm.probe_device(kt, None, 16, n, m, k, SEED, 0, words, out, stream=st)
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            nbm.probe_device(kt, None, 16, n, m, k, SEED, 0, words, out, stream=st)
        for name, keys in (("present", base), ("absent", other), ("p30", mixed(30)), ("p80", mixed(80)),
                           ("p30 again", mixed(30))):
            kt.copy_(torch.from_numpy(keys))
            out.fill_(7)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            np.testing.assert_array_equal(got, oracle.probe(0, keys, None, 16, n, m, k, SEED, words_np),
                                          err_msg=name)


def test_auto_probe_does_not_wait_on_the_host(dev):
    """nb_probe_device's contract (include/nasp_bloom.h): no host synchronisation once
    the workspace is sized -- auto's choice is made on the device.
    Behind ~tens of ms of queued matmuls the auto call returns at once; with
    NB_PROBE_HOST_PICK=1 (rounds 3-5's host read-back) it waits for the queue."""
    import time
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    n, m, k = 4_200_000, 40_250_003, 7
    kt = torch.from_numpy(synth.fixed_keys(n, 16, seed=73)).to(dev)
    words = torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev)
    nbm.build_device(kt, None, 16, n, m, k, SEED, 0, words)
    out = torch.zeros(n, dtype=torch.uint8, device=dev)
    a = torch.rand(4096, 4096, device=dev)
    secs = {}
    for hp in (0, 1):
        with nbm.knobs(NB_PROBE_PATH="auto", NB_PROBE_HOST_PICK=hp):
            nbm.probe_device(kt, None, 16, n, m, k, SEED, 0, words, out)  # sized, warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            b = a
            for _ in range(40):
                b = b @ a * 1e-3
            t1 = time.perf_counter()
            nbm.probe_device(kt, None, 16, n, m, k, SEED, 0, words, out)
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            secs[hp] = (t2 - t1, t3 - t0)
            assert int(out.min()) == 1
    call0, total0 = secs[0]
    call1, total1 = secs[1]
    assert call0 < 0.25 * total0, secs  # enqueued behind the matmuls, not waited for
    assert call1 > 0.5 * total1, secs   # the host pick waits for the queue and its sample


def test_two_level_pipelined_build_replayed_from_graph(dev, oracle, knobs):
    """The two-level build pipelined over two streams (NB_OVERLAP, the default for
    T > 2 048 tiles) under stream capture: the aux stream joins the capture through
    the first event and rejoins the build stream at the end (fork / join), so the
    captured graph holds every pass's bin, re-bin, cursor reset and tile kernels;
    replays on new keys give the oracle's filter, bit-exact."""
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    knobs(NB_BUILD_PATH="tiled", NB_CHUNK_KEYS="300000")  # 3 passes x 2 sub-passes
    assert nbm.get_knob("NB_OVERLAP") != 0
    n, m, k = 700_001, 2**32 - 1, 10
    sets = [synth.fixed_keys(n, 32, seed=300 + s) for s in range(2)]
    kt = torch.zeros(sets[0].size, dtype=torch.uint8, device=dev)
    words = torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev)
    st = torch.cuda.Stream(device=dev)

    def build():
        nbm.build_device(kt, None, 32, n, m, k, SEED, 0, words, stream=st, overwrite=True)

    kt.copy_(torch.from_numpy(sets[0]))
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        build()  # warm-up: sizes the workspace, creates the aux stream
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        build()
    for i in (1, 0):
        kt.copy_(torch.from_numpy(sets[i]))
        words.fill_(-1)  # overwrite mode: stale words must not survive
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        want = oracle.build(0, sets[i], None, 32, n, m, k, SEED)
        np.testing.assert_array_equal(words.cpu().numpy().view(np.uint64), want)
