#!/bin/bash
# Round-4 development call G: bin blocks of two sizes (NB_BIN_MIX) -- parity, then an
# interleaved A/B of C4 against the default.
set -u
mkdir -p gpurun_out/r04g; export TMPDIR=/tmp
O=gpurun_out/r04g
timeout -k 10 300 python -u -m pytest tests/test_gpu_bin_pipe.py -m gpu -x -v --timeout 120 --timeout-method thread -k mix > $O/pytest_mix.log 2>&1
rc=$?; tail -3 $O/pytest_mix.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_mix.log | head -20; exit 1; }
NB_BIN_MIX=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 170 --timeout-method thread -k "c4_full" > $O/pytest_mix_c4.log 2>&1
rc=$?; tail -3 $O/pytest_mix_c4.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 600 python -u tools/ab.py --workloads c4 --reps 3 base: mix:NB_BIN_MIX=1 > $O/ab_mix.txt 2>&1 || { tail -20 $O/ab_mix.txt; exit 3; }
cat $O/ab_mix.txt
