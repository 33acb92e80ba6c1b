#!/bin/bash
# Round 6: one-slot write-out again; E32 tiled in one pass (policy) vs two (chunk 50M).
set -u
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py -k "entry_formats or overflow or c4_full" tests/test_gpu_graph.py > $O/tests.txt 2>&1 || { grep -v "^frame" $O/tests.txt | tail -30; exit 11; }
tail -2 $O/tests.txt
for ch in 0 50000000; do
 for b in present p30; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${b}_$ch -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch $b --path tiled --entries 32 --kpts 2 --chunk $ch > $O/ab_${b}_$ch.txt 2>&1 || { tail -20 $O/ab_${b}_$ch.txt; exit 13; }
  echo "== $b chunk $ch"; grep "ms per call" $O/ab_${b}_$ch.txt
  python3 tools/trace_rounds.py $O/prof_${b}_$ch/run_kernel_trace.csv | head -3
 done
done
