#!/bin/bash
# Round-4 development call A: C4 phase stops at HEAD (the ceiling section), CU-mask
# placement, the tile / bin kernels on masked CU sets and the chunked bin/tile
# pipeline on disjoint CU sets (tools/ubench_c4.hip); then the per-dispatch clock of
# the bench's bin kernel (GRBM_GUI_ACTIVE with the kernel trace, one PMC pass).
set -u
mkdir -p gpurun_out/r04a; export TMPDIR=/tmp
O=gpurun_out/r04a
timeout -k 10 240 tools/ubench_c4 stops > $O/ubc4_stops.txt 2>&1 || { cat $O/ubc4_stops.txt; exit 1; }
cat $O/ubc4_stops.txt
timeout -k 10 240 tools/ubench_c4 mask > $O/ubc4_mask.txt 2>&1 || { cat $O/ubc4_mask.txt; exit 2; }
cat $O/ubc4_mask.txt
timeout -k 10 300 tools/ubench_c4 pipe > $O/ubc4_pipe.txt 2>&1 || { cat $O/ubc4_pipe.txt; exit 3; }
cat $O/ubc4_pipe.txt
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d $O/grbm -o run --output-format csv -- python3 bench.py --workload c4 --no-cpu-baseline --no-host-path --no-probe --no-c2 --steps 30 --warmup 2 > $O/grbm_bench.json 2> $O/grbm.err || { tail -5 $O/grbm.err; exit 4; }
echo grbm ok
