#!/bin/bash
# Round-3 development call (run under gpurun): the GPU tests touched since the
# last full run, the probe paths' rates, then a same-box A/B of knob variants.
#   tools/gpu_dev_r03b.sh "<pytest -k>" "<ab variants>" [ab workloads]
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "$1" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit 1
for w in c4 c3; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-host-path --no-c2 --steps 10 > gpurun_out/bench_probe_$w.json 2> gpurun_out/bench_probe_$w.err || exit 2
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['roofline']['kernel_ms']); [print(' ', p, d['probe'][p]['present']['ms'], d['probe'][p]['absent']['ms']) for p in ('auto','lane','tiled')]" gpurun_out/bench_probe_$w.json
done
if [ -n "${2:-}" ]; then
  timeout -k 10 900 python -u tools/ab.py --workloads ${3:-c5} --reps 2 $2 > gpurun_out/ab.txt 2>&1 || { tail -20 gpurun_out/ab.txt; exit 4; }
  tail -8 gpurun_out/ab.txt
fi
exit $rc
