#!/bin/bash
# Round 6: split p30 one pass vs two -- per-round kernel traces; auto-host's split.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
for ch in 0 50000000; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$ch -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch p30 --path split --entries 0 --chunk $ch > $O/ab_$ch.txt 2>&1 || { tail -20 $O/ab_$ch.txt; exit 13; }
  echo "== chunk $ch"; grep "ms per call" $O/ab_$ch.txt
  python3 tools/trace_rounds.py $O/prof_$ch/run_kernel_trace.csv | head -8
done
