#!/bin/bash
# Round 4: C4 phase stops and the bucket-layout A/B in the product configuration
# (tools/ubench_c4 cstops / layout), then a kernel trace of C5's per-rank share.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 ./tools/ubench_c4 cstops > gpurun_out/c4_cstops.txt 2>&1
timeout -k 10 300 ./tools/ubench_c4 layout > gpurun_out/c4_layout.txt 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c5r -o k -- \
    python3 bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --no-host-path --no-probe --no-c2 \
    > gpurun_out/prof_c5r.txt 2>&1
