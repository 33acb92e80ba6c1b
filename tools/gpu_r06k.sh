#!/bin/bash
# Round 6: E32 one-pass policy vs two passes; auto's gated calls in a kernel trace.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py -k "entry_formats or overflow or c4_full" tests/test_gpu_buckets.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 11; }
tail -2 $O/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_auto -o run --output-format csv -- python3 tools/probe_auto_trace.py > $O/auto.txt 2>&1 || { tail -20 $O/auto.txt; exit 13; }
grep call $O/auto.txt | tail -24
python3 tools/trace_calls.py $O/prof_auto/run_kernel_trace.csv > $O/auto_calls.txt; tail -26 $O/auto_calls.txt
timeout -k 10 600 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0,50000000 --entries 32 --batches present,absent,p30 --no-lane > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -4 $O/probe_c4.txt
