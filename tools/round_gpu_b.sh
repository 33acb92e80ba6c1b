#!/bin/bash
# Round evidence, call B: kernel traces + PMC passes for C2, C3, C4; C5 trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in c2 c3 c4; do bash tools/profile_round.sh r01 $w || exit 1; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 2 --warmup 1 > /dev/null 2>&1 || exit 9
echo "round B ok"
