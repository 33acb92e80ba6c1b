#!/bin/bash
# Round-end GPU evidence in one call: smoke, the full GPU suite, the bench lines
# (C2 default with probe / host-path / CPU baseline; C3, C4, C5, Merkle), the C2
# kernel trace + PMC passes, and kernel traces of C5 and Merkle.  Outputs under
# gpurun_out/; copy what is judged into profiles/ afterwards.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/full_gpu.sh || exit 1
timeout -k 10 300 python bench.py --workload c3 --no-host-path --no-probe > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 5
# C4 with its 8-core CPU baseline (8 concurrent reference builds)
timeout -k 10 300 python bench.py --workload c4 --no-host-path --no-probe > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 5
timeout -k 10 300 python bench.py --workload merkle > gpurun_out/bench_merkle.json 2> gpurun_out/bench_merkle.err || exit 6
bash tools/profile_round.sh r01 c2 || exit 7
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_merkle -o run --output-format csv -- python3 bench.py --workload merkle --no-cpu-baseline --steps 5 > /dev/null 2>&1 || exit 8
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 2 --warmup 1 > /dev/null 2>&1 || exit 9
echo "round ok"
