#!/bin/bash
# Round 6: tiled probe per-kernel times (e32 vs e64, one pass vs the 2-pass policy).
set -u
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py -k "entry_formats or overflow" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 11; }
tail -2 $O/tests.txt
for ch in 0 100000000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_present_$ch -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch present --path tiled --chunk $ch > $O/ab_present_$ch.txt 2>&1 || { tail -20 $O/ab_present_$ch.txt; exit 13; }
  grep "ms per call" $O/ab_present_$ch.txt
  python3 tools/trace_rounds.py $O/prof_present_$ch/run_kernel_trace.csv | head -5
done
timeout -k 10 600 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0,100000000,34000000 --entries 32,64 --batches present,absent,p30 --no-lane > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -8 $O/probe_c4.txt
