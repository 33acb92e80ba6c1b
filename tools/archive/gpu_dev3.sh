#!/bin/bash
# Round-3 development call (run under gpurun): GPU suite, the probe paths' rates on
# C4, then a same-box A/B of the bin-kernel library variants in build_ab/.
#   tools/gpu_dev3.sh "<ab variants>" [workloads] [pytest -k]
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${3:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "$3" > gpurun_out/pytest_gpu.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
fi
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-path --no-c2 --steps 10 > gpurun_out/bench_probe_c4.json 2> gpurun_out/bench_probe_c4.err || exit 2
python -c "import json; d=json.load(open('gpurun_out/bench_probe_c4.json')); print(d['value'], d['roofline']['kernel_ms']); print(json.dumps(d['probe']))"
if [ -n "${1:-}" ]; then
  timeout -k 10 900 python -u tools/ab.py --workloads ${2:-c4,c2} --reps 2 $1 > gpurun_out/ab.txt 2>&1 || { tail -20 gpurun_out/ab.txt; exit 4; }
  tail -8 gpurun_out/ab.txt
fi
exit $rc
