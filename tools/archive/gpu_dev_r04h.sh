#!/bin/bash
# Round-4 development call H: after the counted-tile gating fix -- the test that
# faulted (NB_PACK=0 past 4 GiB), the counted-tile and bin-variant tests.
set -u
mkdir -p gpurun_out/r04h; export TMPDIR=/tmp
O=gpurun_out/r04h
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_counted_tiles.py tests/test_gpu_bin_pipe.py -m gpu -x -v --timeout 170 --timeout-method thread -k "past_4gib or counted or pipe or mix or tile_policy" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; exit 1; }
