#!/bin/bash
# Round-4 development call C: per-build times of back-to-back C4 builds after
# different preludes (tools/clock_ramp.py), then the default bench line at HEAD.
set -u
mkdir -p gpurun_out/r04c; export TMPDIR=/tmp
O=gpurun_out/r04c
timeout -k 10 200 python -u tools/clock_ramp.py 80 > $O/clock_ramp.txt 2>&1 || { tail -20 $O/clock_ramp.txt; exit 1; }
head -4 $O/clock_ramp.txt
timeout -k 10 400 python -u bench.py > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 2; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']); print(d.get('c2')); print({p: (d['probe'][p]['present']['ms'], d['probe'][p]['absent']['ms']) for p in ('auto','lane','tiled')}); print(d['cpu_baseline']['value'], d['host_path']['value'], d['host_path'].get('dropin_class',{}).get('value'))" $O/bench_c4.json
