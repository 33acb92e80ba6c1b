#!/bin/bash
# Round 6: one gated and one host-pick auto call on present keys, kernel by kernel.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_auto -o run --output-format csv -- python3 tools/probe_auto_trace.py --reps 2 --batches present,absent > $O/auto.txt 2>&1 || { tail -20 $O/auto.txt; exit 14; }
python3 tools/trace_calls.py $O/prof_auto/run_kernel_trace.csv --detail > $O/auto_calls.txt; cat $O/auto_calls.txt | tail -80
