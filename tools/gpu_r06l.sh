#!/bin/bash
# Round 6: the gated bin kernels' grid cap (NB_PROBE_BIN_GRID 2 / 4 / 8 per CU) for auto,
# against the host pick.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 700 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks "" --batches present,absent,p30 --no-lane \
   --variant 'auto-g2:auto:NB_PROBE_BIN_GRID=2' --variant 'auto-g4:auto:NB_PROBE_BIN_GRID=4' --variant 'auto-g8:auto:NB_PROBE_BIN_GRID=8' \
   --variant 'auto-g16:auto:NB_PROBE_BIN_GRID=16' --variant 'auto-host:auto:NB_PROBE_HOST_PICK=1' > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 12; }
tail -7 $O/probe_c4.txt
