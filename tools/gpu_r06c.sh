#!/bin/bash
# Round 6: device-gated auto + grid-stride probe bin kernels -- probe / graph / bucket
# tests, then same-box A/Bs on C4's filter.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py tests/test_gpu_graph.py tests/test_gpu_buckets.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 11; }
tail -3 $O/tests.txt
timeout -k 10 600 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --entries 32 --batches present,absent,p30 --auto-pct policy --variant 'auto-host:auto:NB_PROBE_HOST_PICK=1' --variant 'tiled-grid-full:tiled:NB_PROBE_BIN_GRID=1000' --variant 'split-grid-full:split:NB_PROBE_BIN_GRID=1000' > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -9 $O/probe_c4.txt
for b in p30 absent; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$b -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch $b --path split > $O/ab_$b.txt 2>&1 || { tail -20 $O/ab_$b.txt; exit 13; }
  grep "ms per call" $O/ab_$b.txt
done
