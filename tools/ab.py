#!/usr/bin/env python3
"""Same-box A/B of build-kernel variants (diagnostic, run under gpurun).

  python tools/ab.py --workloads c2,c4 --reps 2 \
      base:NB_LIB=build_ab/libnasp_bloom_base.so  new:  new_intmod:NB_FPMOD=0

Each variant is `label:VAR=value,VAR=value` (library builds are selected with
NB_LIB, kernel knobs with their env variables).  Variants are interleaved per
repetition so box drift hits them alike; every run is one `bench.py` process
(device-resident, no CPU baseline / host path / probe), and the table reports
the HIP-event build time (`roofline.kernel_ms`) per run.  Raw lines go to
gpurun_out/ab_<label>_<workload>_<rep>.json.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--workloads", default="c2,c4")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--timeout", type=int, default=240)
    args = ap.parse_args()
    out_dir = os.path.join(REPO, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    table = {}
    for rep in range(args.reps):
        for wl in args.workloads.split(","):
            for v in args.variants:
                label, _, envs = v.partition(":")
                env = dict(os.environ)
                for kv in filter(None, envs.split(",")):
                    k, _, val = kv.partition("=")
                    env[k] = os.path.join(REPO, val) if k == "NB_LIB" else val
                steps = min(args.steps, 3) if wl in ("c5", "c5r") else args.steps
                # c5r: the per-rank share of an 8-GPU C5 step (bench.py per_rank_at_8)
                cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--workload", wl[:2],
                       "--no-cpu-baseline", "--no-host-path", "--no-probe", "--no-c2",
                       "--steps", str(1 if wl == "c5r" else steps),
                       "--warmup", "1" if wl in ("c5", "c5r") else "3"]
                if wl != "c5r":
                    cmd.append("--no-rank-share")
                r = subprocess.run(cmd, env=env, capture_output=True, text=True,
                                   timeout=args.timeout)
                if r.returncode != 0:
                    print(f"{label} {wl}: rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
                    sys.exit(1)
                line = r.stdout.strip().splitlines()[-1]
                open(os.path.join(out_dir, f"ab_{label}_{wl}_{rep}.json"), "w").write(line + "\n")
                d = json.loads(line)
                ms = d["roofline"].get("kernel_ms", d["ms_per_step"])  # c5: whole step
                if wl == "c5r":
                    ms = d["per_rank_at_8"]["ms"]
                table.setdefault((wl, label), []).append(ms)
                ss = d.get("steady_state", {}).get("last20_mean_ms")
                if ss is not None:
                    table.setdefault((wl, label + "/settled"), []).append(ss)
                print(f"rep {rep} {wl:3s} {label:14s} {ms:.4f} ms  {d['value']:.0f} Mkeys/s "
                      f"frac {d['roofline']['frac']:.4f}" + (f"  settled {ss:.4f} ms" if ss else ""), flush=True)
    print("summary (kernel ms per build, each rep; /settled: bench steady_state last-20 mean):")
    for (wl, label), v in sorted(table.items()):
        print(f"  {wl:3s} {label:14s} " + " ".join(f"{x:.4f}" for x in v) + f"   min {min(v):.4f}")


if __name__ == "__main__":
    main()
