#!/bin/bash
# Round 4: tiled-probe passes by key range (NB_PROBE_CHUNK): one kernel trace each of
# the policy (2 passes), 33.4M, 25M and 12.5M-key passes on present and absent keys.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 0 33400000 25000000 12500000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pc_$c -o pc -- \
      python3 tools/probe_chunk.py --reps 1 --no-lane --chunks $c --batches present,absent \
      > gpurun_out/prof_pc_$c.txt 2>&1
done
