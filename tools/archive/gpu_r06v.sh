#!/bin/bash
# Round 6: LOOP kernels for gated launches only -- tests, per-kernel traces of the
# ungated tiled path (one pass / two), auto vs host pick.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py tests/test_gpu_graph.py tests/test_gpu_buckets.py > $O/tests.txt 2>&1 || { grep -v "^frame" $O/tests.txt | tail -30; exit 11; }
tail -2 $O/tests.txt
for ch in 0 50000000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_present_$ch -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch present --path tiled --entries 32 --kpts 2 --chunk $ch > $O/ab_present_$ch.txt 2>&1 || { tail -20 $O/ab_present_$ch.txt; exit 13; }
  echo "== chunk $ch"; grep "ms per call" $O/ab_present_$ch.txt; python3 tools/trace_rounds.py $O/prof_present_$ch/run_kernel_trace.csv | head -3
done
timeout -k 10 700 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0,50000000 --split --batches present,absent,p30 --auto-pct policy \
   --variant 'auto-host:auto:NB_PROBE_HOST_PICK=1' --variant auto-g8:auto:NB_PROBE_BIN_GRID=8 > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -9 $O/probe_c4.txt
