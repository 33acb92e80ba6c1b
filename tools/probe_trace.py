#!/usr/bin/env python3
"""Back-to-back batch probes on C4's filter for a kernel trace (diagnostic; run
under `rocprofv3 --kernel-trace`): the auto path (sample -> host decision -> chosen
path) and the lane path, 5 calls each on 100M absent keys, so tools/timeline.py
shows where the auto path's extra time per call goes."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "nasp-key-value-engine_amd")
import nasp_bloom as nbm  # noqa: E402
from nasp_bloom import synth  # noqa: E402

w = synth.C4
dev = torch.device("cuda", 0)
keys = torch.from_numpy(synth.fixed_keys(w.n, 16)).to(dev)
absent = torch.from_numpy(synth.fixed_keys(w.n, 16, seed=synth.SEED + 1000)).to(dev)
words = torch.zeros(nbm.nwords(w.m), dtype=torch.int64, device=dev)
out = torch.empty(w.n, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream(dev)
nbm.build_device(keys, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, overwrite=True)
torch.cuda.synchronize()
for path in ("auto", "lane"):
    with nbm.knobs(NB_PROBE_PATH=path):
        nbm.probe_device(absent, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            nbm.probe_device(absent, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, out)
        torch.cuda.synchronize()
        print(path, f"{(time.perf_counter() - t0) / 5 * 1e3:.3f} ms per call (host clock)", flush=True)
