#!/bin/bash
# Round 5: the split probe's first round at four keys per thread (kSplitKPT): parity
# (probe + graph tests), C4's filter across present fractions, and a kernel trace of
# the split vs one-round tiled probe (tools/probe_split_trace.py).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_probe.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05k_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05k_pytest.log; exit 3; }
tail -2 gpurun_out/r05k_pytest.log
timeout -k 10 600 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --batches present,absent,p10,p20,p30,p40,p50,p70 --auto-pct 30 > gpurun_out/r05k_probe_c4.txt 2>&1 || { echo "probe c4 rc=$?"; tail -20 gpurun_out/r05k_probe_c4.txt; exit 2; }
tail -6 gpurun_out/r05k_probe_c4.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_split_k -o run -- python3 tools/probe_split_trace.py > gpurun_out/r05k_split.txt 2>&1 || { echo "trace rc=$?"; tail -20 gpurun_out/r05k_split.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05k_split.txt | tail -8
