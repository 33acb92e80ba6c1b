#!/usr/bin/env python3
"""Device-resident build time of the atomic and the tiled path across batch sizes
(p = 0.01 filters, 16-byte keys): where the auto path should switch.  Run on the
GPU box:  python tools/small_n_sweep.py > gpurun_out/small_n.txt"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nasp-key-value-engine_amd"))
import nasp_bloom as nbm  # noqa: E402
from nasp_bloom import synth  # noqa: E402


def time_build(keys, n, m, k, words, stream, reps=50):
    def one():
        with torch.cuda.stream(stream):
            nbm.build_device(keys, None, 16, n, m, k, synth.H2_SEED, 0, words, stream=stream,
                             overwrite=True)
    for _ in range(5):
        one()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        one()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    print("n, m, k, atomic_us, tiled_us")
    for n in (1_000, 4_000, 16_000, 64_000, 256_000, 1_000_000, 4_000_000):
        m = nbm.size_of_bitset(n, 0.01)
        k = nbm.num_hashes(n, m)
        keys = torch.from_numpy(synth.fixed_keys(n, 16)).to(dev)
        words = torch.zeros(nbm.nwords(m), dtype=torch.int64, device=dev)
        res = {}
        for path in ("atomic", "tiled"):
            os.environ["NB_BUILD_PATH"] = path
            res[path] = time_build(keys, n, m, k, words, stream) * 1e3
        os.environ.pop("NB_BUILD_PATH")
        print(f"{n}, {m}, {k}, {res['atomic']:.1f}, {res['tiled']:.1f}", flush=True)


if __name__ == "__main__":
    np.random.seed(0)
    main()
