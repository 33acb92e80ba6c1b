#!/usr/bin/env python3
"""tools/profile_probe.sh output -> profiles/<tag>_pmc_probe_c4.json: per batch kind
and probe path, the device time and the HBM bytes of one 100M-key call of C4's
filter, against the algorithmic bytes (keys read once, the filter read once, one
answer byte written per key: SURVEY §8(d)'s probe row).

HBM bytes per call = Σ over the path's kernels of (2 x FETCH_SIZE + WRITE_SIZE) x
dispatches / calls (KB x 1024; the x2 is the gfx950 correction for 16 B/lane
streaming reads, MI355X_MICROARCH.md §HBM -- the split path's 8 B/lane bucket reads
are uncalibrated, so its figure is approximate).  Device time per call = Σ of the
kernels' trace durations / calls.

  python tools/pmc_probe.py <tag> <profile dir> <calls per path>
"""
import csv
import hashlib
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_PEAK_GBS = 8000.0


def path_of(name):
    if "bloom_probe_kernel" in name:
        return "lane"
    if "probe_tile32_kernel" in name:
        return "tiled"
    if "probe_bin_kernel" in name:
        args = re.search(r"probe_bin_kernel<([^>]*)>", name).group(1).split(",")
        return "tiled" if args[-1].strip() == "true" else "split"
    if "probe_tile_kernel" in name or "probe_compact_kernel" in name:
        return "split"
    return None


def sums(path, counter=None):
    """{probe path: (sum of the counter or of durations over its dispatches, dispatches)}"""
    acc = defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        p = path_of(r["Kernel_Name"])
        if p is None:
            continue
        if counter is None:
            acc[p][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        elif r["Counter_Name"] == counter:
            acc[p][0] += float(r["Counter_Value"])
        else:
            continue
        acc[p][1] += 1
    return acc


def kernel_sha():
    h = hashlib.sha256()
    for f in ("csrc/bloom_kernels.hip", "csrc/bloom_math.h"):
        h.update(open(os.path.join(REPO, "nasp-key-value-engine_amd", f), "rb").read())
    return h.hexdigest()[:16]


def main(tag, prof, calls):
    sys.path.insert(0, os.path.join(REPO, "nasp-key-value-engine_amd"))
    from nasp_bloom import synth
    w = synth.C4
    algo = w.n * 16 + (w.m + 7) // 8 + w.n
    res = {}
    for b in ("present", "p30", "absent"):
        t = sums(os.path.join(prof, b, "trace", "run_kernel_trace.csv"))
        f = sums(os.path.join(prof, b, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
        wr = sums(os.path.join(prof, b, "write", "run_counter_collection.csv"), "WRITE_SIZE")
        for p in ("lane", "tiled", "split"):
            if p not in t:
                continue
            us = t[p][0] / calls
            hbm = (2 * f[p][0] + wr[p][0]) * 1024 / calls if p in f and p in wr else None
            res.setdefault(p, {})[b] = {
                "device_us_per_call": round(us, 1),
                "hbm_bytes_per_call": int(hbm) if hbm is not None else None,
                "traffic_over_algorithmic": round(hbm / algo, 2) if hbm is not None else None,
                "frac_device": round(algo / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
    out = {"workload": "c4_probe", "kernel_source_sha": kernel_sha(), "algorithmic_bytes_per_call": algo,
           "calls_per_path": calls, "paths": res,
           "source": f"profiles/{tag}_pmc_probe_c4.json (tools/profile_probe.sh: tools/probe_pmc.py under "
                     "rocprofv3 --kernel-trace, --pmc FETCH_SIZE and --pmc WRITE_SIZE passes; "
                     "2 x FETCH_SIZE + WRITE_SIZE)"}
    dst = os.path.join(REPO, "profiles", f"{tag}_pmc_probe_c4.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(dst)
    for p, v in res.items():
        for b, x in v.items():
            print(f"  {p:6s} {b:8s} {x}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]))
