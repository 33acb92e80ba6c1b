#!/bin/bash
# Round 5: C4's bin kernel body at three resident blocks per CU (tools/ubench_occ.hip).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/ubench_occ 10 prod,k2n768,k2n640,k2n704,k2n512 > gpurun_out/r05q_occ.txt 2>&1
rc=$?
cat gpurun_out/r05q_occ.txt
exit $rc
