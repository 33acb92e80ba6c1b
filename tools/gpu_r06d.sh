#!/bin/bash
# Round 6: lane-strided tile32 kernel; bin-grid cap sweep; entry formats.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py -k "entry_formats or overflow or c4_full" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 11; }
tail -3 $O/tests.txt
timeout -k 10 700 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --entries 32,64 --batches present,absent,p30 --no-lane \
  --variant 'tiled-g2:tiled:NB_PROBE_BIN_GRID=2' --variant 'tiled-g4:tiled:NB_PROBE_BIN_GRID=4' --variant 'tiled-g32:tiled:NB_PROBE_BIN_GRID=32' --variant 'tiled-gfull:tiled:NB_PROBE_BIN_GRID=1000' \
  --variant 'split-gfull:split:NB_PROBE_BIN_GRID=1000' > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -12 $O/probe_c4.txt
