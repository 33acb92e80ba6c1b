#!/bin/bash
# Round 6: tile32 with the misses' list loads batched; per-round kernel traces.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py -k "entry_formats or overflow or c4_full" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 11; }
tail -3 $O/tests.txt
for b in p30 absent; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$b -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch $b --path split > $O/ab_$b.txt 2>&1 || { tail -20 $O/ab_$b.txt; exit 13; }
  grep "ms per call" $O/ab_$b.txt
  python3 tools/trace_rounds.py $O/prof_$b/run_kernel_trace.csv | head -9
done
timeout -k 10 700 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --entries 32,64 --batches present,absent,p30 --no-lane --auto-pct policy --variant 'auto-host:auto:NB_PROBE_HOST_PICK=1' > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -8 $O/probe_c4.txt
