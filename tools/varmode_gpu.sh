#!/bin/bash
# A/B of the variable-length key readers (NB_VAR_MODE) on C3, plus a parity check.
set -u
mkdir -p gpurun_out
MODES=${MODES:-"0 2"}  # NB_VAR_MODE values to compare
MODES="$MODES" timeout -k 10 300 python tools/debug_chunk.py > gpurun_out/debug_chunk.txt 2>&1 || exit 1
for mode in $MODES; do
  NB_VAR_MODE=$mode timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --steps 5 > gpurun_out/var_$mode.json 2>&1 || exit 2
done
echo ok
