#!/bin/bash
# Round-3 call: probe / graph tests and the C4 probe rates (auto / lane / tiled).
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "probe or graph" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for w in c4 c3; do
timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-host-path --no-c2 --steps 10 > gpurun_out/bench_probe_$w.json 2> gpurun_out/bench_probe_$w.err || exit 2
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['roofline']['kernel_ms']); [print(' ', p, d['probe'][p]['present']['ms'], d['probe'][p]['absent']['ms']) for p in ('auto','lane','tiled')]" gpurun_out/bench_probe_$w.json
done
