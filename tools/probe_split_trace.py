#!/usr/bin/env python3
"""Split vs one-round tiled probe on C4's filter, for a kernel trace (diagnostic; run
under `rocprofv3 --kernel-trace --stats`): 3 calls each of the tiled and the split
path on 100M present, 30 %-present and absent keys, so the per-kernel times show
where the split path's rounds spend their time."""
import sys
import time

import torch

sys.path.insert(0, "nasp-key-value-engine_amd")
import nasp_bloom as nbm  # noqa: E402
from nasp_bloom import synth  # noqa: E402

w = synth.C4
dev = torch.device("cuda", 0)
keys = torch.from_numpy(synth.fixed_keys(w.n, 16)).to(dev)
absent = torch.from_numpy(synth.fixed_keys(w.n, 16, seed=synth.SEED + 1000)).to(dev)
p30 = absent.clone()
p30[:w.n * 16].view(w.n // 10, 10, 16)[:, :3] = keys[:w.n * 16].view(w.n // 10, 10, 16)[:, :3]
words = torch.zeros(nbm.nwords(w.m), dtype=torch.int64, device=dev)
out = torch.empty(w.n, dtype=torch.uint8, device=dev)
nbm.build_device(keys, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, overwrite=True)
torch.cuda.synchronize()
for name, batch in (("present", keys), ("p30", p30), ("absent", absent)):
    for path in ("tiled", "split"):
        with nbm.knobs(NB_PROBE_PATH=path):
            nbm.probe_device(batch, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, out)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                nbm.probe_device(batch, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, out)
            torch.cuda.synchronize()
            print(name, path, f"{(time.perf_counter() - t0) / 3 * 1e3:.3f} ms per call (host clock)", flush=True)
