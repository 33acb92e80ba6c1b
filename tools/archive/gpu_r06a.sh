#!/bin/bash
# Round 6: 32-bit probe entries -- probe parity tests, then a same-box A/B of the
# entry formats on C4's filter.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py -k "entry_formats or overflow" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 11; }
tail -3 $O/tests.txt
timeout -k 10 500 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --entries 32,64 --batches present,absent,p30 > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -8 $O/probe_c4.txt
