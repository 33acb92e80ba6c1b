#!/bin/bash
# Round-3 development call (run under gpurun): selected GPU tests, then a same-box
# A/B of knob variants.
#   tools/gpu_dev_r03c.sh "<pytest -k>" "<workloads>" <variant>...
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
K=$1; W=$2; shift 2
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "$K" > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
fi
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u tools/ab.py --workloads $W --reps 3 "$@" > gpurun_out/ab.txt 2>&1 || { tail -20 gpurun_out/ab.txt; exit 4; }
  tail -12 gpurun_out/ab.txt
fi
