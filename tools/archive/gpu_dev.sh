#!/bin/bash
# Development GPU call (run under gpurun): GPU suite, phase timings and per-phase
# counters of the bin kernel (tools/ubench_tiled), then an A/B of library builds.
#   tools/gpu_dev.sh "<ab variants>" [workloads]
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
for w in c2 c4 c3; do
  timeout -k 5 200 tools/ubench_tiled $w > gpurun_out/ubt_$w.txt 2>&1 || exit 2
  head -3 gpurun_out/ubt_$w.txt
done
tools/pmc_phase.sh || exit 3
if [ -n "${1:-}" ]; then
  timeout -k 10 600 python -u tools/ab.py --workloads ${2:-c2,c4} --reps 2 $1 > gpurun_out/ab.txt 2>&1 || { tail -20 gpurun_out/ab.txt; exit 4; }
  tail -8 gpurun_out/ab.txt
fi
echo dev ok
