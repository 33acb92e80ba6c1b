set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-path --no-c2 --steps 10 > gpurun_out/bench_probe_c4.json 2> gpurun_out/bench_probe_c4.err || exit 2
python -c "import json; d=json.load(open('gpurun_out/bench_probe_c4.json')); print(d['value'], d['roofline']['kernel_ms']); print(json.dumps(d['probe']))"
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || exit 3
cat gpurun_out/bench_c5.json
exit $rc
