#!/usr/bin/env python3
"""C5 per-rank share (125M x 32 B keys into the 2^32-1-bit partial, k = 10, one pass)
under several two-level settings, same box, interleaved after a settle.

  python tools/c5_rank_sweep.py [--reps R] [--configs "SUB:OVL[:TWO],..."]

Each config sets NB_SUBPASSES (bin + re-bin sub-passes sharing one tile pass),
NB_OVERLAP (the sub-passes pipelined over a second stream) and, optionally,
NB_TWO_LEVEL (0: the single-level build straight into the 4 096 fine tiles, no
re-bin round trip; default 1).  Many small sub-passes
keep each sub-pass's pass-1 buckets (~32 B per key) inside the 256 MiB Infinity Cache
between the bin kernel that writes them and the re-bin that reads them back
(MI355X_MICROARCH.md: a line stays resident while the bytes moved between its two
uses fit ~256 MiB).  Every config's filter is compared with the first one's."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nasp-key-value-engine_amd"))


def main():
    import torch
    import nasp_bloom as nbm
    from nasp_bloom import synth
    from nasp_bloom import distributed as D
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--configs", default="1:6,2:6,8:6,16:6,32:6,64:6,16:0")
    args = ap.parse_args()
    wl = synth.C5
    b, e = D.shard_range(wl.n, 0, 8)
    n = e - b
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    k_np, _, kl = synth.keys_for(wl, n=n)
    keys = torch.from_numpy(k_np).to(dev)
    words = torch.empty(nbm.nwords(wl.m), dtype=torch.int64, device=dev)
    cfgs = [tuple(int(x) for x in (c + ":1").split(":")[:3]) for c in args.configs.split(",")]

    def build():
        nbm.build_device(keys, None, kl, n, wl.m, wl.k, synth.H2_SEED, 0, words, stream=st, overwrite=True)

    ref = None
    times = {c: [] for c in cfgs}
    ok = {c: True for c in cfgs}
    with nbm.knobs(NB_SUBPASSES=cfgs[0][0], NB_OVERLAP=cfgs[0][1], NB_TWO_LEVEL=cfgs[0][2]):
        for _ in range(8):  # settle + workspace growth
            build()
        torch.cuda.synchronize(dev)
        ref = words.clone()
    for r in range(args.reps):
        for c in cfgs:
            with nbm.knobs(NB_SUBPASSES=c[0], NB_OVERLAP=c[1], NB_TWO_LEVEL=c[2]):
                build()  # first build of a config grows its workspace
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(3):
                    build()
                e1.record(st)
                torch.cuda.synchronize(dev)
                times[c].append(e0.elapsed_time(e1) / 3)
                if r == 0:
                    ok[c] = bool(torch.equal(words, ref))
        print(f"rep {r}: " + "  ".join(f"{c[0]}:{c[1]}:{c[2]} {times[c][-1]:.3f}" for c in cfgs), flush=True)
    for c in cfgs:
        t = sorted(times[c])
        print(f"NB_SUBPASSES={c[0]:3d} NB_OVERLAP={c[1]} NB_TWO_LEVEL={c[2]}: per-rank share min {t[0]:.3f} med {t[len(t) // 2]:.3f} ms"
              f"  {'bit-exact' if ok[c] else 'MISMATCH'}", flush=True)


if __name__ == "__main__":
    main()
