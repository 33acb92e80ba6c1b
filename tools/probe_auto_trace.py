#!/usr/bin/env python3
"""Auto's device-gated choice against the host pick (diagnostic; run under
`rocprofv3 --kernel-trace`): C4's filter, `--reps` auto calls per batch kind and per
NB_PROBE_HOST_PICK value, each call bracketed by a device synchronisation and a 2 ms
host sleep, so that tools/trace_calls.py can cut the kernel trace into calls and show
what the gated paths' closed launches cost on the device.

  python tools/probe_auto_trace.py --batches present,p30,absent --reps 3
"""
import argparse
import sys
import time

import torch

sys.path.insert(0, "nasp-key-value-engine_amd")
import nasp_bloom as nbm  # noqa: E402
from nasp_bloom import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batches", default="present,p30,absent")
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
w = synth.C4
dev = torch.device("cuda", 0)
keys = torch.from_numpy(synth.fixed_keys(w.n, 16)).to(dev)
absent = torch.from_numpy(synth.fixed_keys(w.n, 16, seed=synth.SEED + 1000)).to(dev)
p30 = absent.clone()
p30[:w.n * 16].view(w.n // 10, 10, 16)[:, :3] = keys[:w.n * 16].view(w.n // 10, 10, 16)[:, :3]
batches = {"present": keys, "p30": p30, "absent": absent}
words = torch.zeros(nbm.nwords(w.m), dtype=torch.int64, device=dev)
out = torch.empty(w.n, dtype=torch.uint8, device=dev)
nbm.build_device(keys, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, overwrite=True)
torch.cuda.synchronize()
for name in args.batches.split(","):
    for hp in (0, 1):
        with nbm.knobs(NB_PROBE_PATH="auto", NB_PROBE_HOST_PICK=hp):
            for r in range(args.reps + 1):
                time.sleep(0.002)
                t0 = time.perf_counter()
                nbm.probe_device(batches[name], None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, out)
                torch.cuda.synchronize()
                print(f"call {name} host_pick={hp} rep {r}: {(time.perf_counter() - t0) * 1e3:.3f} ms (host clock)",
                      flush=True)
