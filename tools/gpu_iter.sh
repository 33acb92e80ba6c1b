#!/bin/bash
# One GPU iteration (run under gpurun): full GPU suite on the in-tree library,
# then a same-box A/B of build variants (tools/ab.py) and a kernel trace of C2/C4.
#   tools/gpu_iter.sh "<ab variants>" [workloads] [reps]
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS=${1:-"base:NB_LIB=build_ab/libnasp_bloom_base.so new:"}
WLS=${2:-c2,c4}
REPS=${3:-2}
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/ab.py --workloads $WLS --reps $REPS $VARIANTS > gpurun_out/ab.txt 2>&1 || { tail -20 gpurun_out/ab.txt; exit 2; }
tail -12 gpurun_out/ab.txt
for w in ${WLS//,/ }; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$w -o run --output-format csv -- python3 bench.py --workload $w --no-cpu-baseline --no-host-path --no-probe --no-c2 --steps 10 --warmup 2 > /dev/null 2> gpurun_out/trace_$w.err || exit 3
done
echo iter ok
