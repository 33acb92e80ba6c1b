#!/bin/bash
# Quick GPU iteration: a parity subset, then bench lines for c2/c4/c3 and a kernel trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
SEL=${1:-"golden_build or fixed16 or varlen or k_range or chunking or overflow or stride or overwrite or edge_m or c5 or cooperative or deterministic or dropin"}
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "$SEL" > gpurun_out/q_pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/q_pytest.log
tail -3 gpurun_out/q_pytest.log
grep -q "rc=0" gpurun_out/q_pytest.log || exit 1
for w in c2 c4 c3; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-host-path --steps 10 > gpurun_out/q_bench_$w.json 2> gpurun_out/q_bench_$w.err || exit 2
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q_trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-path --steps 10 > /dev/null 2>&1 || exit 3
echo quick ok
