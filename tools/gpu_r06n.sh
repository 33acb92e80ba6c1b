#!/bin/bash
# Round 6: split path in one pass (policy) vs two; auto gated vs host pick.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py tests/test_gpu_buckets.py tests/test_gpu_graph.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 11; }
tail -2 $O/tests.txt
timeout -k 10 700 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks "" --split --batches present,absent,p30 --no-lane --auto-pct policy \
   --variant 'split-2pass:split:NB_PROBE_CHUNK=50000000' --variant 'auto-host:auto:NB_PROBE_HOST_PICK=1' > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -6 $O/probe_c4.txt
