#!/bin/bash
# Round 4: C5 sub-pass count under shard-major buckets, same box, interleaved:
# the per-rank share (one pass) with 1 / 2 / 3 sub-passes, the whole step by policy / 1 / 3.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/ab.py --workloads c5r --reps 3 --timeout 400 \
    s1:NB_SUBPASSES=1 s2:NB_SUBPASSES=2 s3:NB_SUBPASSES=3 > gpurun_out/ab_c5r_subpasses_gm.txt 2>&1
timeout -k 10 900 python -u tools/ab.py --workloads c5 --reps 2 --timeout 400 \
    policy: s1:NB_SUBPASSES=1 s3:NB_SUBPASSES=3 > gpurun_out/ab_c5_subpasses_gm.txt 2>&1
