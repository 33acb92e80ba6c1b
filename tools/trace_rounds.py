#!/usr/bin/env python3
"""Average kernel time per probe round from a rocprofv3 kernel trace: each tile-kernel
dispatch is labelled by the bin kernel launched right before it (its template
arguments name the round and the entry format), so the split path's round-one and
round-two tile kernels -- one template instance for 64-bit entries -- are told apart.

  python tools/trace_rounds.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(probe_\w+|bloom_\w+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    acc = defaultdict(list)
    last_bin = "-"
    for r in rows:
        nm = short(r["Kernel_Name"])
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if nm.startswith("probe_bin"):
            last_bin = nm
            acc[nm].append(us)
        elif nm.startswith("probe_tile"):
            acc[f"{nm}  after {last_bin}"].append(us)
        else:
            acc[nm].append(us)
    for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):4d} x {sum(v) / len(v):9.1f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
