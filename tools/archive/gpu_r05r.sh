#!/bin/bash
# Round 5: the split probe's compacted second round for variable-length keys too:
# parity (probe, graph, bucket tests), then C3's keys and filter across present fractions.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_probe.py tests/test_gpu_graph.py tests/test_gpu_buckets.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05r_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05r_pytest.log; exit 3; }
tail -2 gpurun_out/r05r_pytest.log
timeout -k 10 700 python -u tools/probe_chunk.py --workload c3 --reps 2 --chunks 0 --split --batches present,absent,p10,p20,p30,p40,p50,p60,p70 --auto-pct 30 > gpurun_out/r05r_probe_c3.txt 2>&1 || { echo "probe c3 rc=$?"; tail -20 gpurun_out/r05r_probe_c3.txt; exit 2; }
tail -6 gpurun_out/r05r_probe_c3.txt
