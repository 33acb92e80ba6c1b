#!/usr/bin/env python3
"""The batch probe's profiled workload (run under rocprofv3 by tools/profile_probe.sh):
C4's filter (100M x 16 B keys, k = 7), one batch kind, `--calls` calls of each
explicit path -- lane, tiled, split -- whose kernels are distinct template instances
(lane: bloom_probe_kernel; tiled: the E32 probe_bin_kernel + probe_tile32_kernel;
split: the 64-bit-entry rounds, probe_tile_kernel, probe_compact_kernel), so the
counters separate by path.  Answers are checked against the lane path.

  python tools/probe_pmc.py --batch present|p30|absent [--calls 3]
"""
import argparse
import sys

import torch

sys.path.insert(0, "nasp-key-value-engine_amd")
import nasp_bloom as nbm  # noqa: E402
from nasp_bloom import synth  # noqa: E402

PATHS = ("lane", "tiled", "split")


def batch_of(name, w, dev):
    keys = torch.from_numpy(synth.fixed_keys(w.n, 16)).to(dev)
    if name == "present":
        return keys, keys
    absent = torch.from_numpy(synth.fixed_keys(w.n, 16, seed=synth.SEED + 1000)).to(dev)
    if name == "absent":
        return keys, absent
    b = absent.clone()  # p30: keys 0-2 of every 10 present
    b[:w.n * 16].view(w.n // 10, 10, 16)[:, :3] = keys[:w.n * 16].view(w.n // 10, 10, 16)[:, :3]
    return keys, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", default="present", choices=["present", "p30", "absent"])
    ap.add_argument("--calls", type=int, default=3)
    args = ap.parse_args()
    w = synth.C4
    dev = torch.device("cuda", 0)
    keys, batch = batch_of(args.batch, w, dev)
    words = torch.zeros(nbm.nwords(w.m), dtype=torch.int64, device=dev)
    nbm.build_device(keys, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, overwrite=True)
    out = torch.empty(w.n, dtype=torch.uint8, device=dev)
    ref = None
    for path in PATHS:
        with nbm.knobs(NB_PROBE_PATH=path):
            for _ in range(args.calls):
                nbm.probe_device(batch, None, 16, w.n, w.m, w.k, synth.H2_SEED, 0, words, out)
            torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        elif not torch.equal(out, ref):
            raise SystemExit(f"{path}: answers differ from the lane path")
    print(f"probe_pmc {args.batch}: {args.calls} calls per path, answers identical", flush=True)


if __name__ == "__main__":
    main()
