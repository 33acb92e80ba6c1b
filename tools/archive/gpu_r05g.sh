#!/bin/bash
# Round 5: the tiled probe's misses through per-tile lists binned by key block
# (NB_PROBE_MISS=1) against a byte store per miss: parity, then C4 / C5-shape sweeps.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_probe.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05g_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05g_pytest.log; exit 3; }
tail -2 gpurun_out/r05g_pytest.log
timeout -k 10 600 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --miss-ab --batches present,absent,p10,p20,p30,p50,p70 --auto-pct 30 > gpurun_out/r05g_probe_c4.txt 2>&1 || { echo "probe c4 rc=$?"; tail -20 gpurun_out/r05g_probe_c4.txt; exit 2; }
tail -9 gpurun_out/r05g_probe_c4.txt
timeout -k 10 400 python -u tools/probe_chunk.py --workload c5 --reps 2 --chunks 0 --miss-ab --batches present,absent,p10,p20,p30,p50,p70 --auto-pct 30 > gpurun_out/r05g_probe_c5.txt 2>&1 || { echo "probe c5 rc=$?"; tail -20 gpurun_out/r05g_probe_c5.txt; exit 4; }
tail -7 gpurun_out/r05g_probe_c5.txt
