#!/bin/bash
# Round 4: auto probe threshold (NB_PROBE_TILED_PCT 50 -> 30): probe parity, then the
# lane / tiled / auto paths on batches of 0-100 % present keys, same box, interleaved.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_probe.py tests/test_gpu_graph.py > gpurun_out/pytest_pct.log 2>&1
timeout -k 10 500 python -u tools/probe_chunk.py --reps 2 --chunks 0 --auto-pct 50,30 --batches p20,p30,p40,mixed \
    > gpurun_out/probe_pct.txt 2>&1
