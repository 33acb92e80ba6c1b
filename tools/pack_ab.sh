set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "tile_policy or spill or c3_full or c4_full or varlen or chunking or k_range or overwrite or golden_large" > gpurun_out/pk.log 2>&1
rc=$?; tail -5 gpurun_out/pk.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_tiles_pk.sh
