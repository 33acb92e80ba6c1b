#!/usr/bin/env python3
"""Recompute a bench line's roofline figures from the committed profiles (no GPU).

  python tools/roofline_check.py <tag> <workload> [bench json]
  e.g. python tools/roofline_check.py r04f c4 profiles/r04f_bench_c4.json

From profiles/<tag>_kernel_stats_<wl>.csv (rocprofv3 --kernel-trace --stats) and
profiles/<tag>_pmc_<wl>.json (tools/pmc_traffic.py): the build's kernels per step
(dispatches per step as pmc_traffic counted them), their traced time per step, the
algorithmic bytes per step (bench.py algorithmic_bytes) over that time
as a fraction of the 8 TB/s HBM peak, and the measured HBM bytes per step against the
algorithmic ones.  With a bench line it also prints the line's own (untraced,
HIP-event) kernel_ms and frac beside the traced ones, and checks that the profiles'
kernel-source hash is the current one.
"""
import csv
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 8000.0


def kernel_sha():
    h = hashlib.sha256()
    for f in ("csrc/bloom_kernels.hip", "csrc/bloom_math.h"):
        h.update(open(os.path.join(REPO, "nasp-key-value-engine_amd", f), "rb").read())
    return h.hexdigest()[:16]


def short(name):
    import re
    m = re.search(r"([A-Za-z_][A-Za-z_0-9]*(<[^()]*>)?)\(", name)
    return m.group(1) if m else name


def main(tag, wl_key, bench=None):
    sys.path.insert(0, os.path.join(REPO, "nasp-key-value-engine_amd"))
    sys.path.insert(0, REPO)
    from nasp_bloom import synth
    from bench import algorithmic_bytes
    wl = synth.WORKLOADS[wl_key]
    pmc = json.load(open(os.path.join(REPO, "profiles", f"{tag}_pmc_{wl_key}.json")))
    stats = {}
    for r in csv.DictReader(open(os.path.join(REPO, "profiles", f"{tag}_kernel_stats_{wl_key}.csv"))):
        stats[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]))
    var_len = wl_key == "c3"
    if var_len:
        _, offs, _ = synth.keys_for(wl)
        key_bytes = int(offs[-1])
    else:
        key_bytes = wl.n * wl.key_len
    B = algorithmic_bytes(wl.n, wl.key_len if not var_len else 0, key_bytes, wl.m, var_len)
    t_ns = 0.0
    print(f"{tag} {wl.name}: kernel-source sha {pmc['kernel_source_sha']} "
          f"({'current' if pmc['kernel_source_sha'] == kernel_sha() else 'STALE: ' + kernel_sha()})")
    for k, part in pmc["per_kernel"].items():
        per_step = part.get("dispatches_per_step", 1.0)
        calls, avg = stats.get(k, (0, 0.0))
        t_ns += avg * per_step
        print(f"  {k[:70]:70s} x{per_step:5.2f}  {avg / 1e3:9.2f} us  {part['hbm_bytes'] / 1e9:7.3f} GB/dispatch")
    t_ms = t_ns / 1e6
    frac = B / (t_ms * 1e-3) / 1e9 / PEAK
    traffic = pmc["hbm_bytes_per_launch"]
    if wl_key == "c5":
        print("  (C5's bin and re-bin / tile kernels run on two streams and overlap: the traced sum "
              "over-counts the step, whose own time is the bench line's ms_per_step)")
    print(f"  traced build time {t_ms:.4f} ms per step; algorithmic {B / 1e9:.3f} GB -> "
          f"{B / (t_ms * 1e-3) / 1e9:.1f} GB/s, frac {frac:.4f}")
    print(f"  measured HBM traffic {traffic / 1e9:.3f} GB per step = {traffic / B:.2f}x algorithmic; "
          f"at the measured attainable 6.0 TB/s read rate that traffic alone takes {traffic / 6e12 * 1e3:.3f} ms")
    if bench:
        lines = [ln for ln in open(bench) if ln.startswith("{")]
        d = json.loads(lines[-1])
        rl = d["roofline"]
        print(f"  bench line: kernel_ms {rl.get('kernel_ms')} (untraced HIP events), frac {rl['frac']}, "
              f"traffic {rl.get('traffic')}; ms_per_step {d['ms_per_step']}"
              + (f"; settled {d['steady_state']['last20_mean_ms']} ms" if "steady_state" in d else ""))


if __name__ == "__main__":
    main(*sys.argv[1:4])
