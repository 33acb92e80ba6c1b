#!/bin/bash
# Round-4 development call K: the C5 step at N = 1 (8 passes) with 1 vs 2 pipelined
# sub-passes, and the per-rank share under the new policy (1 sub-pass), interleaved.
set -u
mkdir -p gpurun_out/r04k; export TMPDIR=/tmp
O=gpurun_out/r04k
timeout -k 10 1000 python -u tools/ab.py --workloads c5,c5r --reps 2 policy: s1:NB_SUBPASSES=1 s2:NB_SUBPASSES=2 > $O/ab_c5_sub.txt 2>&1 || { tail -20 $O/ab_c5_sub.txt; exit 4; }
tail -8 $O/ab_c5_sub.txt
