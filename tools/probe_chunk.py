#!/usr/bin/env python3
"""Tiled batch probe by key-range passes (NB_PROBE_CHUNK), same box, interleaved.

A miss in the tiled probe is a byte store into the key's answer (≈ k/2 per absent
key).  Over 100M keys those stores land anywhere in a 100 MB answer
array; split into passes of C keys, a pass's stores stay inside C bytes, which the
XCDs' 4 MiB L2s can hold -- at the price of one read of the filter per pass.  This
times the tiled path at several C against the lane path on C4's filter, for present,
absent and half-present batches, and checks every answer against the lane path's.

  python tools/probe_chunk.py [--reps R] [--chunks 0,25000000,...] [--batches present,absent,mixed]
                               [--no-lane]
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--chunks", default="0,25000000,12500000,6250000,3125000")
    ap.add_argument("--batches", default="present,absent,mixed")
    ap.add_argument("--no-lane", action="store_true")
    ap.add_argument("--split", action="store_true", help="also the split tiled probe (two rounds)")
    ap.add_argument("--auto-pct", default="", help="auto path at these NB_PROBE_TILED_PCT values ('policy' = 0)")
    ap.add_argument("--workload", default="c4", choices=["c4", "c5", "c3", "shape"],
                    help="c4: C4's filter from the 100M probed present keys; c5: C5's shape "
                         "(m = 2^32-1, k = 10, 32-byte keys), --n probed keys, the filter built "
                         "from --fill-keys device-random keys (the present keys among them); c3: "
                         "C3's 100M variable-length keys (8-64 B) and filter, the absent keys "
                         "the same keys with their first byte changed (same offsets); shape: "
                         "as c5 at --m / --k / --key-len, the filter half full unless --fill-keys")
    ap.add_argument("--entries", default="0",
                    help="tiled / split variants at these NB_PROBE_ENTRY formats (0: the policy -- "
                         "32-bit one-round, 64-bit split; 32,64: an A/B forcing either)")
    ap.add_argument("--variant", action="append", default=[],
                    help="extra variant LABEL:PATH:KNOB=V,KNOB=V (repeatable), e.g. "
                         "'auto-host:auto:NB_PROBE_HOST_PICK=1'")
    ap.add_argument("--n", type=int, default=50_000_000)
    ap.add_argument("--fill-keys", type=int, default=0, help="c5 / shape (0: 400M for c5, m ln2 / k for shape)")
    ap.add_argument("--m", type=int, default=0)
    ap.add_argument("--k", type=int, default=0)
    ap.add_argument("--key-len", type=int, default=0)
    args = ap.parse_args()
    if args.workload == "shape" and not (args.m and args.k and args.key_len):
        ap.error("--workload shape needs --m, --k and --key-len")
    reps = args.reps
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    fill = None
    offs = None
    if args.workload == "c3":
        wl = synth.C3
        p_np, o_np, kl = synth.keys_for(wl)
        present = torch.from_numpy(p_np).to(dev)
        offs = torch.from_numpy(o_np.view(np.int64)).to(dev)
        starts = offs[:-1]

        def flipped(mask):  # the keys where mask holds, first byte changed
            b = present.clone()
            sel = starts[mask]
            b[sel] = b[sel] ^ 0x5A
            return b
        keyno = torch.arange(wl.n, device=dev)
        absent = flipped(torch.ones(wl.n, dtype=torch.bool, device=dev))
    elif args.workload == "c4":
        wl = synth.C4
        p_np, _, kl = synth.keys_for(wl)
        a_np, _, _ = synth.keys_for(wl, seed=synth.SEED + 1000)
        # (the generator's buffers keep their tail padding: kernels may read past a key)
        present = torch.from_numpy(p_np).to(dev)
        absent = torch.from_numpy(a_np).to(dev)
    else:
        if args.workload == "c5":
            wl = synth.Workload("c5_shape_probe", args.n, 32, synth.C5.m, synth.C5.k, 0.01)
            args.fill_keys = args.fill_keys or 400_000_000
        else:  # (p is a label only: the probe takes m and k)
            wl = synth.Workload(f"shape_m{args.m}_k{args.k}_L{args.key_len}", args.n, args.key_len,
                                args.m, args.k, 0.01)
            args.fill_keys = args.fill_keys or int(args.m * np.log(2) / args.k)
        kl = wl.key_len
        g = torch.Generator(device=dev)
        g.manual_seed(5)
        fill = torch.randint(0, 256, (args.fill_keys * kl + 64,), dtype=torch.uint8, device=dev, generator=g)
        if args.fill_keys >= wl.n:
            present = fill[:wl.n * kl + 64].clone()
        else:  # (a filter smaller than the batch: the filled keys, repeated)
            rep = -(-wl.n // args.fill_keys)
            present = torch.cat([fill[:args.fill_keys * kl].repeat(rep)[:wl.n * kl],
                                 torch.zeros(64, dtype=torch.uint8, device=dev)])
        absent = torch.randint(0, 256, (wl.n * kl + 64,), dtype=torch.uint8, device=dev, generator=g)
    want_b = args.batches.split(",")
    if offs is not None:
        batches = {"present": present, "absent": absent, "mixed": flipped(keyno % 2 == 1)}
        for pc in range(10, 100, 10):
            if f"p{pc}" in want_b:
                batches[f"p{pc}"] = flipped(keyno % 10 >= pc // 10)
    else:
        mixed = present.clone()
        mv = mixed[:wl.n * kl].view(wl.n, kl)
        mv[1::2] = absent[:wl.n * kl].view(wl.n, kl)[1::2]
        batches = {"present": present, "absent": absent, "mixed": mixed}
    for pc in range(10, 100, 10):  # pc % present: keys i with i % 10 < pc / 10 (the sample sees the same mix)
        if f"p{pc}" not in want_b or offs is not None:
            continue
        b = absent.clone()
        bv, pv = b[:wl.n * kl].view(wl.n // 10, 10, kl), present[:wl.n * kl].view(wl.n // 10, 10, kl)
        bv[:, :pc // 10] = pv[:, :pc // 10]
        batches[f"p{pc}"] = b
    batches = {b: batches[b] for b in args.batches.split(",")}
    words = torch.zeros(nbm.nwords(wl.m), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)  # (the keys and the zeroed words, made on the current stream, before st uses them)
    if fill is None:
        nbm.build_device(present, offs, kl, wl.n, wl.m, wl.k, synth.H2_SEED, 0, words, stream=st,
                         overwrite=True)
    else:
        nbm.build_device(fill, None, kl, args.fill_keys, wl.m, wl.k, synth.H2_SEED, 0, words, stream=st,
                         overwrite=True)
        del fill
    torch.cuda.synchronize(dev)
    ones = int(np.unpackbits(words.view(torch.uint8)[:1 << 20].cpu().numpy()).sum())
    print(f"{wl.name}: n={wl.n} m={wl.m} k={wl.k} key_len={kl}, filter fill ~{ones / (8 << 20):.3f} "
          f"(first MiB)", flush=True)
    out = torch.empty(wl.n, dtype=torch.uint8, device=dev)
    ref = {}
    with nbm.knobs(NB_PROBE_PATH="lane"):
        for name, b in batches.items():
            nbm.probe_device(b, offs, kl, wl.n, wl.m, wl.k, synth.H2_SEED, 0, words, out, stream=st)
            torch.cuda.synchronize(dev)
            ref[name] = out.clone()
            torch.cuda.synchronize(dev)  # (the copy, on the current stream, before st writes out again)
    ents = [int(e) for e in args.entries.split(",")]

    def ent(e):
        return "" if len(ents) == 1 else f" e{e}"
    variants = ([] if args.no_lane else [("lane", "lane", 0, "0", {})]) + [
        (f"tiled C={c / 1e6 if c else 'policy'}M{ent(e)}", "tiled", c, "0", {"NB_PROBE_ENTRY": e})
        for c in map(int, args.chunks.split(",") if args.chunks else []) for e in ents
    ] + ([(f"split{ent(e)}", "split", 0, "0", {"NB_PROBE_ENTRY": e}) for e in ents] if args.split else []) + [
        (f"auto pct={p}", "auto", 0, "0" if p == "policy" else p, {})
        for p in filter(None, args.auto_pct.split(","))]
    for v in args.variant:
        label, path, kv = (v.split(":", 2) + [""])[:3]
        variants.append((label, path, 0, "0", {a.split("=")[0]: int(a.split("=")[1]) for a in kv.split(",") if a}))
    table = {}
    bad = 0
    for rep in range(reps):
        for label, path, chunk, pct, extra in variants:
            with nbm.knobs(**{"NB_PROBE_PATH": path, "NB_PROBE_CHUNK": str(chunk), "NB_PROBE_TILED_PCT": pct,
                              **extra}):
                for name, b in batches.items():
                    nbm.probe_device(b, offs, kl, wl.n, wl.m, wl.k, synth.H2_SEED, 0, words, out, stream=st)
                    torch.cuda.synchronize(dev)
                    if not torch.equal(out, ref[name]):
                        bad += 1
                        d = torch.nonzero(out != ref[name]).flatten()
                        print(f"MISMATCH {label} {name}: {d.numel()} answers, first at "
                              f"{d[:4].tolist()} (got {out[d[:4]].tolist()}, lane {ref[name][d[:4]].tolist()})",
                              flush=True)
                    t0 = time.perf_counter()
                    for _ in range(5):
                        nbm.probe_device(b, offs, kl, wl.n, wl.m, wl.k, synth.H2_SEED, 0, words, out,
                                         stream=st)
                    torch.cuda.synchronize(dev)
                    ms = (time.perf_counter() - t0) * 1e3 / 5
                    table.setdefault((label, name), []).append(ms)
                    print(f"rep {rep} {label:>16} {name:>8} {ms:8.3f} ms  {wl.n / ms / 1e6:7.2f} Gkeys/s",
                          flush=True)
    print(f"summary (ms per {wl.n / 1e6:.0f}M-key call, wall clock over 5 calls; min over reps):")
    for label, _, _, _, _ in variants:
        print(f"  {label:>16} " + "  ".join(f"{n} {min(table[(label, n)]):7.3f}" for n in batches))
    print(f"answers identical to the lane path: {'yes' if bad == 0 else f'NO ({bad} mismatches)'}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
