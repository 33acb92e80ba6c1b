#!/bin/bash
# Round 5: kernel trace of the split vs one-round tiled probe (tools/probe_split_trace.py).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_split -o run -- python3 tools/probe_split_trace.py > gpurun_out/r05e_split.txt 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r05e_split.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05e_split.txt | tail -8
find gpurun_out/prof_split -name "*kernel_trace.csv" | head -3
