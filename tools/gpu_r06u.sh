#!/bin/bash
# Round 6: E32 tiled at two passes (per-pass bin / tile times); auto's gated calls.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_present_50 -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch present --path tiled --entries 32 --kpts 2 --chunk 50000000 > $O/ab_present_50.txt 2>&1 || { tail -20 $O/ab_present_50.txt; exit 13; }
grep "ms per call" $O/ab_present_50.txt; python3 tools/trace_rounds.py $O/prof_present_50/run_kernel_trace.csv | head -3
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_auto -o run --output-format csv -- python3 tools/probe_auto_trace.py --reps 2 > $O/auto.txt 2>&1 || { tail -20 $O/auto.txt; exit 14; }
python3 tools/trace_calls.py $O/prof_auto/run_kernel_trace.csv > $O/auto_calls.txt; tail -20 $O/auto_calls.txt
python3 - <<'PY'
import csv, re
rows = sorted(csv.DictReader(open("gpurun_out/r06u/prof_auto/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
# the first gated auto call on present keys: kernels with durations and gaps
calls, cur, last = [], [], None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if last is not None and s - last > 500e3 and cur:
        calls.append(cur); cur = []
    cur.append((s, e, re.sub(r"\(.*", "", r["Kernel_Name"])[:70], r["Grid_Size_X"]))
    last = e if last is None else max(last, e)
calls.append(cur)
for c in calls[3:5]:
    print("---")
    for s, e, n, g in c:
        print(f"{(s - c[0][0]) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us grid {g:>9} {n}")
PY
