#!/usr/bin/env python3
"""Turn tools/profile_round.sh output into profiles/<tag>_pmc_<workload>.json.

HBM bytes per build call = Σ over the build's kernels (bin + tile) of
  2 x FETCH_SIZE + WRITE_SIZE   (KB, x1024)
The 2x: on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced
streaming reads (MI355X_MICROARCH.md §HBM); the build's reads are the 16 B/lane
key stream and bucket stream.  FETCH_SIZE and WRITE_SIZE come from separate
--pmc passes (they do not fit one TCC pass).  Also copies the kernel-trace stats.
"""
import csv
import hashlib
import json
import os
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def short(name):
    """'void (anonymous namespace)::bloom_bin_kernel<0, 2, ...>(args)' -> 'bloom_bin_kernel<0, 2, ...>'"""
    import re
    m = re.search(r"([A-Za-z_][A-Za-z_0-9]*(<[^()]*>)?)\(", name)
    return m.group(1) if m else name


def kernel_sha():
    h = hashlib.sha256()
    for f in ("csrc/bloom_kernels.hip", "csrc/bloom_math.h"):
        h.update(open(os.path.join(REPO, "nasp-key-value-engine_amd", f), "rb").read())
    return h.hexdigest()[:16]


def main(tag, wl_key, prof_dir):
    sys.path.insert(0, os.path.join(REPO, "nasp-key-value-engine_amd"))
    from nasp_bloom import synth
    wl = synth.WORKLOADS[wl_key]
    fetch = per_kernel(os.path.join(prof_dir, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(prof_dir, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    parts = {}
    for name in fetch:
        if any(x in name for x in ("bloom_bin_kernel", "bloom_tile_or_kernel", "bloom_rebin_kernel")):
            f, w = fetch[name], write.get(name, 0.0)
            parts[short(name)] = {"FETCH_SIZE_KB": round(f, 1), "WRITE_SIZE_KB": round(w, 1),
                                  "hbm_bytes": int((2 * f + w) * 1024)}
    stats = {}
    for r in csv.DictReader(open(os.path.join(prof_dir, "trace", "run_kernel_stats.csv"))):
        stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    # one bench step = one build call: exactly one overwrite-mode tile kernel (the
    # first tile pass), plus per step the same number of bin / re-bin / OR-mode tile
    # launches (C4: bin + tile; C5: 16 bin + 16 re-bin + 1 overwrite + 7 OR-mode tile
    # passes).  Per-step bytes = sum over those kernels of the per-dispatch average x
    # dispatches / steps (the profiled runs skip bench's host-path and probe legs)
    used = [k for k in parts if k in stats]
    ow = [k for k in used if "tile_or" in k and "true" in k]
    steps = sum(stats[k]["calls"] for k in ow) or 1
    total = sum(parts[k]["hbm_bytes"] * stats[k]["calls"] / steps for k in used)
    for k in used:
        parts[k]["dispatches_per_step"] = round(stats[k]["calls"] / steps, 3)
    out = {"workload": wl.name, "kernel_source_sha": kernel_sha(),
           "hbm_bytes_per_launch": int(total), "build_kernels": used, "per_kernel": parts,
           "kernel_stats": stats,
           "source": f"profiles/{tag}_pmc_{wl_key}.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                     "separate passes, FETCH_SIZE x2 gfx950 correction)"}
    dst = os.path.join(REPO, "profiles", f"{tag}_pmc_{wl_key}.json")
    json.dump(out, open(dst, "w"), indent=1)
    shutil.copy(os.path.join(prof_dir, "trace", "run_kernel_stats.csv"),
                os.path.join(REPO, "profiles", f"{tag}_kernel_stats_{wl_key}.csv"))
    print(dst, int(total))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
