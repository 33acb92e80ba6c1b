#!/bin/bash
# Round 6: covering grids skip the bin-block counters, 64 counter classes for capped
# grids -- tests, traces of the ungated tiled path, auto vs host pick.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py tests/test_gpu_graph.py tests/test_gpu_buckets.py > $O/tests.txt 2>&1 || { grep -v "^frame" $O/tests.txt | tail -30; exit 11; }
tail -2 $O/tests.txt
for b in present p30; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${b} -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch $b --path tiled --entries 32 --kpts 2 > $O/ab_${b}.txt 2>&1 || { tail -20 $O/ab_${b}.txt; exit 13; }
  echo "== $b"; grep "ms per call" $O/ab_${b}.txt
  python3 tools/trace_rounds.py $O/prof_${b}/run_kernel_trace.csv | head -3
done
timeout -k 10 700 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --batches present,absent,p30 --auto-pct policy \
   --variant 'auto-host:auto:NB_PROBE_HOST_PICK=1' > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -7 $O/probe_c4.txt
