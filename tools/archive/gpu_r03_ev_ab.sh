#!/bin/bash
# Round-3 call: the round's evidence at HEAD (smoke, GPU suite, bench lines), then
# a same-box A/B of the wide bin blocks (NB_BIN_WIDE) on C4 and C5.
#   tools/gpu_r03_ev_ab.sh <tag>
set -u
bash tools/round_evidence.sh "$1" || exit $?
timeout -k 10 600 python -u tools/ab.py --workloads c4,c5 --reps 3 base: wide:NB_BIN_WIDE=1 \
  > gpurun_out/ab_wide.txt 2>&1 || { tail -20 gpurun_out/ab_wide.txt; exit 8; }
tail -6 gpurun_out/ab_wide.txt
