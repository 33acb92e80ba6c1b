#!/bin/bash
# Round-4 development call E: the pipelined bin kernel (NB_BIN_PIPE=1) -- its own
# parity tests (one and several batches per block), C4-shaped parity tests through
# it, then an interleaved A/B against the two-blocks-per-CU bin kernel (bench
# kernel_ms and the settled last-20 mean).
set -u
mkdir -p gpurun_out/r04e; export TMPDIR=/tmp
O=gpurun_out/r04e
timeout -k 10 300 python -u -m pytest tests/test_gpu_bin_pipe.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_pipe_own.log 2>&1
rc=$?; tail -3 $O/pytest_pipe_own.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_pipe_own.log | head -20; exit 1; }
NB_BIN_PIPE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_counted_tiles.py tests/test_gpu_parity.py -m gpu -x -v --timeout 170 --timeout-method thread -k "counted or c4_full or tile_policy or overflow_spill or overwrite_mode or chunking or fixed16_configs or golden_large_m or deterministic" > $O/pytest_pipe.log 2>&1
rc=$?; tail -3 $O/pytest_pipe.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_pipe.log | head -20; exit 2; }
timeout -k 10 600 python -u tools/ab.py --workloads c4 --reps 3 base:NB_BIN_PIPE=0 pipe:NB_BIN_PIPE=1 > $O/ab_pipe.txt 2>&1 || { tail -20 $O/ab_pipe.txt; exit 3; }
cat $O/ab_pipe.txt
