#!/bin/bash
# Round 5: the probe tile kernel reading its shards interleaved (key-order sweep):
# parity, then lane / tiled / split / auto on C4's filter and C5's shape.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_probe.py tests/test_gpu_buckets.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05f_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05f_pytest.log; exit 3; }
tail -2 gpurun_out/r05f_pytest.log
timeout -k 10 600 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --batches present,absent,p10,p20,p30,p40,p50,p70 --auto-pct 30 > gpurun_out/r05f_probe_c4.txt 2>&1 || { echo "probe c4 rc=$?"; tail -20 gpurun_out/r05f_probe_c4.txt; exit 2; }
tail -7 gpurun_out/r05f_probe_c4.txt
timeout -k 10 400 python -u tools/probe_chunk.py --workload c5 --reps 2 --chunks 0 --split --batches present,absent,p10,p20,p30,p40,p50,p70 --auto-pct 30 > gpurun_out/r05f_probe_c5.txt 2>&1 || { echo "probe c5 rc=$?"; tail -20 gpurun_out/r05f_probe_c5.txt; exit 4; }
tail -7 gpurun_out/r05f_probe_c5.txt
