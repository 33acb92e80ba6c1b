#!/bin/bash
# Round 5: same-box phase stops of the product bin kernel (ubench_c4 cstops) beside the
# slot-range kernel and its phase stops (ubench_slots), for DESIGN §6's comparison.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/ubench_c4 cstops > gpurun_out/r05p_cstops.txt 2>&1 || { tail -20 gpurun_out/r05p_cstops.txt; exit 1; }
cat gpurun_out/r05p_cstops.txt
timeout -k 10 300 ./tools/ubench_slots 10 prod,slotsA,slotsA_stop1,slotsA_stop2 > gpurun_out/r05p_slots.txt 2>&1 || { tail -20 gpurun_out/r05p_slots.txt; exit 2; }
cat gpurun_out/r05p_slots.txt
