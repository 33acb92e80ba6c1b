#!/bin/bash
# Round 6: dynamic bin-block distribution in the gated grid-stride bin kernels; caps.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py tests/test_gpu_graph.py tests/test_gpu_buckets.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 11; }
tail -2 $O/tests.txt
timeout -k 10 700 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --batches present,absent,p30 --no-lane \
   --variant 'auto-g2:auto:NB_PROBE_BIN_GRID=2' --variant 'auto-g4:auto:NB_PROBE_BIN_GRID=4' --variant 'auto-g8:auto:NB_PROBE_BIN_GRID=8' \
   --variant 'auto-host:auto:NB_PROBE_HOST_PICK=1' > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -8 $O/probe_c4.txt
