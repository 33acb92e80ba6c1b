#!/bin/bash
# Round 5: C4's bin kernel with fixed-capacity slot ranges per tile
# against the product's, interleaved after a settle (tools/ubench_slots.hip).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/ubench_slots 10 prod,slotsA,slotsA_stop1,slotsA_stop2 > gpurun_out/r05i_slots.txt 2>&1
rc=$?
cat gpurun_out/r05i_slots.txt
exit $rc
