#!/bin/bash
# Round-4 development call A (second form): the counted-tile parity tests, the
# per-dispatch clock of the bench's bin kernel (GRBM_GUI_ACTIVE with the kernel trace,
# one PMC pass), then the CU-mask placement probe and, if masked streams run, the
# masked tile / bin kernels and the chunked bin/tile pipeline (tools/ubench_c4.hip).
set -u
mkdir -p gpurun_out/r04a; export TMPDIR=/tmp
O=gpurun_out/r04a
timeout -k 10 600 python -u -m pytest tests/test_gpu_counted_tiles.py tests/test_gpu_parity.py -m gpu -x -v --timeout 170 --timeout-method thread -k "counted or c4_full or c3_full or tile_policy or overflow_spill or overwrite_mode or chunking" > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; exit 2; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d $O/grbm -o run --output-format csv -- python3 bench.py --workload c4 --no-cpu-baseline --no-host-path --no-probe --no-c2 --steps 30 --warmup 2 > $O/grbm_bench.json 2> $O/grbm.err || { tail -5 $O/grbm.err; exit 4; }
echo grbm ok
timeout -k 10 120 tools/ubench_c4 mask > $O/ubc4_mask.txt 2>&1; rc=$?
cat $O/ubc4_mask.txt
[ $rc -eq 0 ] || exit 0   # masked streams unusable: nothing more to measure
timeout -k 10 300 tools/ubench_c4 pipe > $O/ubc4_pipe.txt 2>&1; rc=$?
cat $O/ubc4_pipe.txt
exit $rc
