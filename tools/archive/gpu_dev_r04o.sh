#!/bin/bash
# Round 4: shard-major buckets (NB_BUCKET_GMAJOR) on the other workloads, same box,
# interleaved: C2, C3, C5's per-rank share (one pass) and the whole C5 step.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/ab.py --workloads c2,c3,c5r --reps 3 --timeout 400 \
    base: gm:NB_BUCKET_GMAJOR=1 > gpurun_out/ab_gmajor_other.txt 2>&1
timeout -k 10 900 python -u tools/ab.py --workloads c5 --reps 2 --timeout 400 \
    base: gm:NB_BUCKET_GMAJOR=1 > gpurun_out/ab_gmajor_c5.txt 2>&1
