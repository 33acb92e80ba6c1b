#!/bin/bash
# Round-4 development call I: bench stdout holds exactly one JSON line (the RCCL
# banner and other notes go to stderr) for the default line and for C5.
set -u
mkdir -p gpurun_out/r04i; export TMPDIR=/tmp
O=gpurun_out/r04i
timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-path --no-probe --steps 5 --warmup 2 > $O/c4.out 2> $O/c4.err || exit 1
timeout -k 10 200 python bench.py --workload c5 --steps 1 --warmup 1 --no-rank-share > $O/c5.out 2> $O/c5.err || exit 2
for f in c4 c5; do echo "$f: $(wc -l < $O/$f.out) stdout line(s)"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $O/$f.out || exit 3; done
