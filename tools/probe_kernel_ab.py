#!/usr/bin/env python3
"""Per-kernel A/B of the tiled-probe entry formats (diagnostic; run under
`rocprofv3 --kernel-trace --stats`): C4's filter, one batch kind, `--reps` calls of
the chosen path per NB_PROBE_ENTRY format.  The two formats' bin / tile kernels are
distinct template instances, so the stats file separates them (the compaction
kernel is shared).

  python tools/probe_kernel_ab.py --batch p30 --path split --entries 32,64
"""
import argparse
import sys
import time

import torch

sys.path.insert(0, "nasp-key-value-engine_amd")
import nasp_bloom as nbm  # noqa: E402
from nasp_bloom import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", default="p30", choices=["present", "p30", "absent"])
ap.add_argument("--path", default="split")
ap.add_argument("--entries", default="32,64")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--chunk", default="0")
ap.add_argument("--kpts", default="0", help="NB_PROBE_KPT values (one-round E32 keys per bin thread)")
args = ap.parse_args()
w = synth.C4
dev = torch.device("cuda", 0)
keys = torch.from_numpy(synth.fixed_keys(w.n, 16)).to(dev)
batch = keys
if args.batch != "present":
    absent = torch.from_numpy(synth.fixed_keys(w.n, 16, seed=synth.SEED + 1000)).to(dev)
    batch = absent
    if args.batch == "p30":
        batch = absent.clone()
        batch[:w.n * 16].view(w.n // 10, 10, 16)[:, :3] = keys[:w.n * 16].view(w.n // 10, 10, 16)[:, :3]
words = torch.zeros(nbm.nwords(w.m), dtype=torch.int64, device=dev)
out = torch.empty(w.n, dtype=torch.uint8, device=dev)
nbm.build_device(keys, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, overwrite=True)
torch.cuda.synchronize()
ref = None
for e, kpt in [(e, q) for e in map(int, args.entries.split(",")) for q in map(int, args.kpts.split(","))]:
    with nbm.knobs(NB_PROBE_PATH=args.path, NB_PROBE_ENTRY=e, NB_PROBE_CHUNK=args.chunk, NB_PROBE_KPT=kpt):
        nbm.probe_device(batch, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, out)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        assert torch.equal(out, ref), "answers differ between entry formats"
        t0 = time.perf_counter()
        for _ in range(args.reps):
            nbm.probe_device(batch, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, out)
        torch.cuda.synchronize()
        print(args.batch, args.path, f"e{e}", f"kpt{kpt}", f"{(time.perf_counter() - t0) / args.reps * 1e3:.3f} ms per call",
              flush=True)
