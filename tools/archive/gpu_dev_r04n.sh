#!/bin/bash
# Round 4: shard-major buckets (NB_BUCKET_GMAJOR): parity, then same-box A/Bs of the
# C4 build (one and two passes) and of the tiled probe by key-range passes.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_bucket_layout.py > gpurun_out/pytest_gmajor.log 2>&1
timeout -k 10 700 python -u tools/ab.py --workloads c4 --reps 3 \
    base: gm:NB_BUCKET_GMAJOR=1 c50:NB_CHUNK_KEYS=50000000 gm_c50:NB_BUCKET_GMAJOR=1,NB_CHUNK_KEYS=50000000 \
    > gpurun_out/ab_c4_gmajor.txt 2>&1
NB_BUCKET_GMAJOR=1 timeout -k 10 400 python -u tools/probe_chunk.py --reps 2 --no-lane \
    --chunks 0,25000000,16700000 > gpurun_out/probe_chunk_gmajor.txt 2>&1
