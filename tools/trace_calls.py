#!/usr/bin/env python3
"""Cuts a rocprofv3 kernel trace into calls separated by host gaps (> --gap-us idle
on the device) and prints, per call, its device span, the kernels' busy time, how many
kernels ran and the short ones (< --closed-us: gated launches that were closed).

  python tools/trace_calls.py <run_kernel_trace.csv> [--gap-us 500] [--closed-us 15]
"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-us", type=float, default=500)
    ap.add_argument("--closed-us", type=float, default=15)
    ap.add_argument("--detail", action="store_true", help="list every kernel of every call")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and s - last_end > args.gap_us * 1e3 and cur:
            calls.append(cur)
            cur = []
        cur.append((s, e, re.sub(r"\(.*", "", r["Kernel_Name"])[:90], r.get("Grid_Size_X", "?")))
        last_end = e if last_end is None else max(last_end, e)
    if cur:
        calls.append(cur)
    for i, c in enumerate(calls):
        span = (max(x[1] for x in c) - c[0][0]) / 1e3
        busy = sum(x[1] - x[0] for x in c) / 1e3
        short = [(x[1] - x[0]) / 1e3 for x in c if (x[1] - x[0]) / 1e3 < args.closed_us]
        print(f"call {i:3d}: span {span:9.1f} us  busy {busy:9.1f} us  kernels {len(c):3d}  "
              f"short {len(short):3d} ({sum(short):6.1f} us)  first {c[0][2][:40]}")
        if args.detail:
            for s, e, nm, g in c:
                print(f"      +{(s - c[0][0]) / 1e3:8.1f} {(e - s) / 1e3:8.1f} us  grid {g:>9}  {nm}")


if __name__ == "__main__":
    main()
