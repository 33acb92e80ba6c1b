#!/bin/bash
# Round evidence, call A: smoke, the full GPU suite, bench lines C2 (with probe /
# host path / CPU baseline), C5, C3 and C4 (with their CPU baselines), Merkle.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/full_gpu.sh || exit 1
timeout -k 10 300 python bench.py --workload c3 --no-host-path --no-probe > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 5
timeout -k 10 300 python bench.py --workload c4 --no-host-path --no-probe > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 5
timeout -k 10 300 python bench.py --workload merkle > gpurun_out/bench_merkle.json 2> gpurun_out/bench_merkle.err || exit 6
echo "round A ok"
