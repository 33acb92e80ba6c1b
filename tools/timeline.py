#!/usr/bin/env python3
"""Kernel timeline of a rocprofv3 --kernel-trace run (diagnostic): per dispatch its
queue, start/end relative to the first dispatch, and how long it ran alongside a
kernel of another queue.

  python tools/timeline.py gpurun_out/tl_c5 [--last N]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=40)
    a = ap.parse_args()
    f = sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    ev = []
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")[:48]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", "?")), name))
    ev.sort()
    ev = ev[-a.last:]
    t0 = ev[0][0]
    for s, e, q, n in ev:
        ov = sum(max(0, min(e, e2) - max(s, s2)) for s2, e2, q2, _ in ev if q2 != q)
        print(f"q{q:>3} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  "
              f"beside other queue {ov / 1e3:8.1f}  {n}")


if __name__ == "__main__":
    main()
