#!/bin/bash
# Round-4 development call J: bench stdout = one JSON line (default line, C5), then
# C5's per-rank share (one pass of 125M keys) against the number of pipelined
# sub-passes, interleaved A/B.
set -u
mkdir -p gpurun_out/r04j; export TMPDIR=/tmp
O=gpurun_out/r04j
timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-path --no-probe --steps 5 --warmup 2 > $O/c4.out 2> $O/c4.err || exit 1
timeout -k 10 200 python bench.py --workload c5 --steps 1 --warmup 1 --no-rank-share > $O/c5.out 2> $O/c5.err || exit 2
for f in c4 c5; do echo "$f: $(wc -l < $O/$f.out) stdout line(s)"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $O/$f.out || exit 3; done
timeout -k 10 900 python -u tools/ab.py --workloads c5r --reps 3 s2:NB_SUBPASSES=2 s3:NB_SUBPASSES=3 s4:NB_SUBPASSES=4 s1:NB_SUBPASSES=1 > $O/ab_c5r_sub.txt 2>&1 || { tail -20 $O/ab_c5r_sub.txt; exit 4; }
tail -6 $O/ab_c5r_sub.txt
