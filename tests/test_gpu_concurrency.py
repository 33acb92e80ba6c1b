"""Re-entrancy of the C ABI (SURVEY §8(b) "Threading"): host threads building and
probing distinct filters at the same time on one device.  Each nb_build takes its
own pooled slot set (own streams, own per-stream workspace); nb_probe shares the
device scratch under its lock; device builds on distinct torch streams use
distinct workspaces.  Every result must equal the oracle's (bit-exact), and a
failing call in one thread must not leak its error into another."""
import threading

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


def _run_threads(fns):
    errors = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001 -- reported below
            errors.append(e)
    th = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errors:
        raise errors[0]


def test_concurrent_host_builds_and_probes(nbm, oracle):
    from nasp_bloom import synth
    jobs = []
    for t in range(8):
        n = 150_000 + 7_919 * t
        if t % 2:
            (buf, offs), kl = synth.var_keys(n, t, 40 + t, seed=synth.SEED + t), 0
        else:
            buf, offs, kl = synth.fixed_keys(n, 16, seed=synth.SEED + t), None, 16
        m = nbm.size_of_bitset(n, 0.01)
        jobs.append((buf, offs, kl, n, m, nbm.num_hashes(n, m), t % 2))
    got = [None] * len(jobs)
    hits = [None] * len(jobs)

    def job(i):
        buf, offs, kl, n, m, k, flavor = jobs[i]

        def f():
            w = np.zeros(nbm.nwords(m), np.uint64)
            for _ in range(3):  # repeated builds OR into the same words
                nbm.build_host(buf, offs, kl, n, m, k, SEED, flavor, w)
            got[i] = w
            hits[i] = nbm.probe_host(buf, offs, kl, n, m, k, SEED, flavor, w)
        return f
    _run_threads([job(i) for i in range(len(jobs))])
    for i, (buf, offs, kl, n, m, k, flavor) in enumerate(jobs):
        np.testing.assert_array_equal(got[i], oracle.build(flavor, buf, offs, kl, n, m, k, SEED))
        assert hits[i].all()


def test_concurrent_device_builds_on_streams(nbm, oracle):
    import torch
    from nasp_bloom import synth
    dev = torch.device("cuda", 0)
    n, m, k = 400_000, 3_834_023, 7
    keysets = [synth.fixed_keys(n, 16, seed=synth.SEED + 100 + t) for t in range(4)]
    words = [torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev) for _ in keysets]

    def job(i):
        def f():
            st = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(st):  # the upload is ordered on the build stream too
                kt = torch.from_numpy(keysets[i]).to(dev)
                for _ in range(5):
                    nbm.build_device(kt, None, 16, n, m, k, SEED, 0, words[i], stream=st,
                                     overwrite=True)
            st.synchronize()
        return f
    _run_threads([job(i) for i in range(len(keysets))])
    torch.cuda.synchronize()
    for i, ks in enumerate(keysets):
        np.testing.assert_array_equal(words[i].cpu().numpy().view(np.uint64),
                                      oracle.build(0, ks, None, 16, n, m, k, SEED))


def test_two_threads_one_stream(nbm, oracle):
    """Two host threads building different filters on the SAME stream: the
    per-(device, stream) workspace is held for a whole build, so the kernels of
    the two builds never interleave over one set of buckets and cursors."""
    import torch
    from nasp_bloom import synth
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    n, m, k = 300_000, 2_875_519, 7
    keysets = [synth.fixed_keys(n, 16, seed=synth.SEED + 200 + t) for t in range(2)]
    with torch.cuda.stream(st):
        kts = [torch.from_numpy(ks).to(dev) for ks in keysets]
    st.synchronize()
    words = [torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev) for _ in keysets]

    def job(i):
        def f():
            for _ in range(20):
                nbm.build_device(kts[i], None, 16, n, m, k, SEED, 0, words[i], stream=st,
                                 overwrite=True)
        return f
    _run_threads([job(i) for i in range(2)])
    st.synchronize()
    for i, ks in enumerate(keysets):
        np.testing.assert_array_equal(words[i].cpu().numpy().view(np.uint64),
                                      oracle.build(0, ks, None, 16, n, m, k, SEED))


def test_errors_stay_in_their_thread(nbm):
    """nb_last_error is per thread: a failing call does not change another
    thread's successful call's message state."""
    lib = nbm.lib()
    results = {}
    barrier = threading.Barrier(2)

    def bad():
        rc = lib.nb_build(None, None, 16, 10, 1000, 7, SEED, 9, None, 0)  # unknown flavor
        barrier.wait()
        results["bad"] = (rc, (lib.nb_last_error() or b"").decode())

    def good():
        w = np.zeros(nbm.nwords(1000), np.uint64)
        keys = np.zeros(160, np.uint8)
        barrier.wait()
        nbm.build_host(keys, None, 16, 10, 1000, 7, SEED, 0, w)
        results["good"] = int(w.any())
    _run_threads([bad, good])
    assert results["bad"][0] != 0 and "flavor" in results["bad"][1]
    assert results["good"] == 1
