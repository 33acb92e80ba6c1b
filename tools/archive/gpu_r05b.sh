#!/bin/bash
# Round 5: the GPU suite after the variant pruning (counted tiles on every tail),
# the C5 per-rank sub-pass sweep, and the C4 line.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05b_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r05b_pytest_gpu.log; tail -3 gpurun_out/r05b_pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 240 ./tools/ubench_r05 8 prod,s2,s4 > gpurun_out/r05b_ub.txt 2>&1 || { echo "ub rc=$?"; cat gpurun_out/r05b_ub.txt; exit 4; }
cat gpurun_out/r05b_ub.txt
timeout -k 10 400 python -u tools/c5_rank_sweep.py --reps 2 > gpurun_out/r05b_c5_sweep.txt 2>&1 || { echo "sweep rc=$?"; tail -5 gpurun_out/r05b_c5_sweep.txt; exit 2; }
cat gpurun_out/r05b_c5_sweep.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > gpurun_out/r05b_bench_c4.json 2> gpurun_out/r05b_bench_c4.err || { echo "bench rc=$?"; tail -20 gpurun_out/r05b_bench_c4.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/r05b_bench_c4.json'));print(d['value'],d['ms_per_step'],d.get('steady_state',{}).get('last20_mean_ms'))"
