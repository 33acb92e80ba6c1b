#!/usr/bin/env python3
"""Auto probe against the best single path, per shape and batch, from
tools/archive/gpu_r06sh.sh output directories (tools/probe_chunk.py summaries):
  python tools/auto_regret.py <dir> [<dir of another library, same box> ...]
Each row: the shape, the batch, the fastest of lane / tiled / split (ms), then per
directory auto (device choice) and its cost against that best."""
import glob
import os
import re
import sys


def parse(path):
    if not os.path.exists(path):
        return None
    txt = open(path).read()
    m = re.search(r"^(shape_\S+): n=(\d+)", txt, re.M)
    if not m or "summary" not in txt:
        return None
    rows = {}
    for line in txt.split("summary", 1)[1].splitlines()[1:]:
        mm = re.match(r"\s*(.+?)\s+((?:\S+\s+[\d.]+\s*)+)$", line)
        if not mm:
            continue
        vals = mm.group(2).split()
        rows[mm.group(1).strip()] = {vals[i]: float(vals[i + 1]) for i in range(0, len(vals), 2)}
    return m.group(1), int(m.group(2)), rows, "identical to the lane path: yes" in txt


def main():
    dirs = sys.argv[1:]
    names = sorted({os.path.basename(p) for d in dirs for p in glob.glob(os.path.join(d, "*.txt"))
                    if parse(p)})
    hdr = f"{'shape':<34}{'n':>6} {'batch':<8}{'best':>16}" + "".join(
        f"{'auto ' + os.path.basename(d.rstrip('/')):>22}" for d in dirs)
    print(hdr)
    for nm in names:
        parsed = [parse(os.path.join(d, nm)) for d in dirs]
        if any(p is None for p in parsed):
            continue
        shape, n, rows0, _ = parsed[0]
        for b in rows0.get("lane", {}):
            paths = {p: rows0[k][b] for p, k in (("lane", "lane"), ("tiled", "tiled C=policyM"), ("split", "split"))
                     if k in rows0}
            best = min(paths, key=paths.get)
            line = f"{shape:<34}{n / 1e6:>5.0f}M {b:<8}{best:>7} {paths[best]:8.3f}"
            for _, _, rows, ok in parsed:
                a = rows["auto pct=policy"][b]
                line += f"{a:12.3f} {100 * (a / paths[best] - 1):+7.1f} %{'' if ok else '!'}"
            print(line)
    print("(! = answers differed from the lane path's)")


if __name__ == "__main__":
    main()
