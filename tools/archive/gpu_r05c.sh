#!/bin/bash
# Round 5: same-box A/B of the placement change (one add per index) against the
# HEAD library (build_ab/libnasp_bloom_base.so), then lane vs tiled vs auto probe
# on C5's shape at 20/30/40 % present (the auto threshold per shape).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_counted_tiles.py tests/test_gpu_buckets.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05c_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -20 gpurun_out/r05c_pytest.log; exit 3; }
tail -2 gpurun_out/r05c_pytest.log
timeout -k 10 900 python -u tools/ab.py --workloads c4,c2,c3 --reps 3 base:NB_LIB=build_ab/libnasp_bloom_base.so new: > gpurun_out/r05c_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r05c_ab.txt; exit 1; }
tail -12 gpurun_out/r05c_ab.txt
timeout -k 10 400 python -u tools/probe_chunk.py --workload c5 --reps 2 --chunks 0 --batches present,absent,p20,p30,p40 --auto-pct 30,50 > gpurun_out/r05c_probe_c5.txt 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/r05c_probe_c5.txt; exit 2; }
tail -8 gpurun_out/r05c_probe_c5.txt
