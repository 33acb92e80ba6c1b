#!/usr/bin/env python3
"""Per-build device time of back-to-back C4 builds (100M x 16 B keys, k = 7), each
build bracketed by its own HIP events on the build stream, after different
preludes: a cold start, an idle gap of 50 ms / 500 ms, and the bench's own sequence
(warmup builds, the probe guard, then the timed builds).  Shows how the build time
follows the chip's clock as the power controller settles ("clock").
usage: python tools/clock_ramp.py [builds per run]"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nasp-key-value-engine_amd"))


def main():
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 80
    wl = synth.C4
    dev = torch.device("cuda", 0)
    keys_np, _, kl = synth.keys_for(wl)
    keys = torch.from_numpy(keys_np).to(dev)
    words = torch.zeros(nbm.nwords(wl.m), dtype=torch.int64, device=dev)
    st = torch.cuda.Stream(device=dev)

    def run(n):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        with torch.cuda.stream(st):
            evs[0].record(st)
            for i in range(n):
                nbm.build_device(keys, None, kl, wl.n, wl.m, wl.k, synth.H2_SEED, 0, words, stream=st,
                                 overwrite=True)
                evs[i + 1].record(st)
        torch.cuda.synchronize(dev)
        return [round(evs[i].elapsed_time(evs[i + 1]), 4) for i in range(n)]

    def probe_guard():
        out = torch.empty(wl.n, dtype=torch.uint8, device=dev)
        nbm.probe_device(keys, None, kl, wl.n, wl.m, wl.k, synth.H2_SEED, 0, words, out)
        torch.cuda.synchronize(dev)

    res = {}
    res["cold"] = run(nb)
    for gap in (0.05, 0.5):
        time.sleep(gap)
        res[f"after_idle_{int(gap * 1000)}ms"] = run(nb)
    time.sleep(0.5)
    w = run(5)          # bench: 5 warmup builds,
    probe_guard()       # the false-negative guard,
    res["bench_sequence"] = w + run(nb)  # then the timed builds
    for name, ms in res.items():
        a = np.array(ms)
        print(f"{name:>20}: first5 {a[:5].mean():.3f}  builds 6-25 {a[5:25].mean():.3f}  "
              f"26-50 {a[25:50].mean():.3f}  last20 {a[-20:].mean():.3f}  min {a.min():.3f} ms", flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
