#!/bin/bash
# Round 6: the graph replay of every auto path after the coherent gate loads (the
# replay that faulted in r06q), then the probe / graph / bucket suites, then traces.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 200 python3 tools/diag_graph_auto.py graph split > $O/diag_graph_split.txt 2>&1 && timeout -k 10 200 python3 tools/diag_graph_auto.py graph > $O/diag_graph.txt 2>&1 || { grep -v "^frame" $O/diag_graph*.txt | tail -20; exit 10; }
cat $O/diag_graph_split.txt | grep -v amdgpu.ids
cat $O/diag_graph.txt | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py tests/test_gpu_graph.py tests/test_gpu_buckets.py > $O/tests.txt 2>&1 || { grep -v "^frame" $O/tests.txt | tail -30; exit 11; }
tail -2 $O/tests.txt
for b in present p30; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$b -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch $b --path tiled --entries 32 --kpts 1,2 > $O/ab_$b.txt 2>&1 || { tail -20 $O/ab_$b.txt; exit 13; }
  echo "== $b"; grep "ms per call" $O/ab_$b.txt
  python3 tools/trace_rounds.py $O/prof_$b/run_kernel_trace.csv | head -5
done
