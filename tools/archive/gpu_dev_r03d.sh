#!/bin/bash
# Round-3 development call: probe / graph / two-level tests, C4 probe rates after
# the zero-copy sample, an A/B of the pipelined two-level sub-passes (C5 and its
# per-rank share), and a kernel-trace timeline of one pipelined C5 step.
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "probe or graph or overlap or two_level" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --no-host-path --no-c2 --steps 10 > gpurun_out/bench_probe_c4.json 2> gpurun_out/bench_probe_c4.err || exit 2
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['kernel_ms']); [print(' ', p, d['probe'][p]['present']['ms'], d['probe'][p]['absent']['ms']) for p in ('auto','lane','tiled')]" gpurun_out/bench_probe_c4.json
timeout -k 10 900 python -u tools/ab.py --workloads c5r,c5 --reps 2 base: s2:NB_SUBPASSES=2 ov2s2:NB_OVERLAP=2,NB_SUBPASSES=2 ov2s4:NB_OVERLAP=2,NB_SUBPASSES=4 ov6s2:NB_OVERLAP=6,NB_SUBPASSES=2 > gpurun_out/ab.txt 2>&1 || { tail -20 gpurun_out/ab.txt; exit 4; }
tail -12 gpurun_out/ab.txt
NB_OVERLAP=2 NB_SUBPASSES=2 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_c5 -o run --output-format csv -- python3 bench.py --workload c5 --no-cpu-baseline --no-host-path --no-probe --no-c2 --no-rank-share --steps 1 --warmup 1 > gpurun_out/tl_c5.json 2> gpurun_out/tl_c5.err || exit 3
echo timeline ok
