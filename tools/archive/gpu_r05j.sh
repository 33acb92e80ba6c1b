#!/bin/bash
# Round 5: C5's per-rank share, two-level (product) against the single-level build
# straight into the fine tiles (NB_TWO_LEVEL=0, no re-bin round trip), VERDICT r04 item 2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/c5_rank_sweep.py --reps 3 --configs "1:6:1,1:6:0" \
    > gpurun_out/r05j_c5_single.txt 2>&1
rc=$?
cat gpurun_out/r05j_c5_single.txt
exit $rc
