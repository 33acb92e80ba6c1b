#!/bin/bash
# Pipelined vs classic bin kernel: parity subset first, then bench A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "golden_build or fixed16 or k_range or chunking or overflow or stride or overwrite or edge_m or c5 or cooperative or deterministic or dropin" > gpurun_out/pipe_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pipe_pytest.log; tail -3 gpurun_out/pipe_pytest.log
[ $rc -eq 0 ] || exit 1
for w in c2 c4 c3; do
  for mode in 1 0; do
    NB_BIN_MODE=$mode timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-host-path --steps 10 > gpurun_out/pipe_${w}_$mode.json 2> /dev/null || exit 2
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pipe_trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-path --steps 10 > /dev/null 2>&1 || exit 3
echo pipe ok
