#!/bin/bash
# Round 5, first GPU call: the persistent / phase-offset bin kernel A/B
# (tools/ubench_r05), then the C4 bench line at HEAD with the driver's flags.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 ./tools/ubench_r05 10 > gpurun_out/r05a_ub.txt 2>&1 || { echo "ubench rc=$?"; cat gpurun_out/r05a_ub.txt; exit 1; }
cat gpurun_out/r05a_ub.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > gpurun_out/r05a_bench_c4.json 2> gpurun_out/r05a_bench_c4.err || { echo "bench rc=$?"; tail -20 gpurun_out/r05a_bench_c4.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/r05a_bench_c4.json'));print(d['value'],d['ms_per_step'],d.get('steady_state',{}))"
