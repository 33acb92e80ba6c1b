#!/bin/bash
# Round 6: the E32 bin write-out as a running-maximum scan -- tests, per-kernel trace,
# auto vs host pick.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06y
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py tests/test_gpu_graph.py tests/test_gpu_buckets.py > $O/tests.txt 2>&1 || { grep -v "^frame" $O/tests.txt | tail -30; exit 11; }
tail -2 $O/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_present -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch present --path tiled --entries 32 --kpts 1,2 > $O/ab_present.txt 2>&1 || { tail -20 $O/ab_present.txt; exit 13; }
grep "ms per call" $O/ab_present.txt; python3 tools/trace_rounds.py $O/prof_present/run_kernel_trace.csv | head -5
timeout -k 10 700 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --batches present,absent,p30 --auto-pct policy \
   --variant 'auto-host:auto:NB_PROBE_HOST_PICK=1' > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -7 $O/probe_c4.txt
