#!/usr/bin/env python3
"""Per-phase instruction counts of the bin kernel from tools/pmc_phase.sh output
(gpurun_out/pp/<workload>/run_counter_collection.csv): the ubench_tiled `pmc`
mode dispatches the kernel stopped after each phase (hash only, + count,
+ scan/reservations, + placement, full), so successive differences price a phase.
usage: python tools/pmc_phase_summary.py [dir] > profiles/<tag>_phase_counts.txt"""
import collections
import csv
import os
import sys

N = {"c2": 10e6, "c4": 100e6, "c3": 100e6, "c5": 200e6}  # c5: one 200M-key pass
LABELS = ["hash+index", "+count", "+scan/res", "+placement", "+write-out"]


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pp"
    for w, n in N.items():
        f = os.path.join(root, w, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg, names = collections.defaultdict(float), {}
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            agg[(d, r["Counter_Name"])] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
        bins = [d for d in sorted(names) if "bloom_bin" in names[d]]
        print(f"{w}: per key (n = {n:.0f}); {names[bins[0]][:90]}")
        prev = None
        for lab, d in zip(LABELS, bins):
            v = agg[(d, "SQ_INSTS_VALU")] * 64 / n
            l = agg[(d, "SQ_INSTS_LDS")] * 64 / n
            sa = agg[(d, "SQ_INSTS_SALU")] * 64 / n
            dv = f"(+{v - prev[0]:6.1f})" if prev else " " * 9
            dl = f"(+{l - prev[1]:5.2f})" if prev else " " * 8
            print(f"  {lab:11s} VALU {v:7.1f} {dv}  LDS {l:6.2f} {dl}  SALU {sa:6.1f}")
            prev = (v, l)


if __name__ == "__main__":
    main()
