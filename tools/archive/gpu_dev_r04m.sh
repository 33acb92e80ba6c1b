#!/bin/bash
# Round 4: C4 build by key-range passes (NB_CHUNK_KEYS), same box, interleaved;
# then kernel traces of the one-pass and two-pass C4 builds.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab.py --workloads c4 --reps 3 \
    base: c50:NB_CHUNK_KEYS=50000000 c34:NB_CHUNK_KEYS=33400000 c25:NB_CHUNK_KEYS=25000000 \
    > gpurun_out/ab_c4_chunks.txt 2>&1
for c in 0 50000000; do
  NB_CHUNK_KEYS=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4ch_$c -o k -- \
      python3 bench.py --no-cpu-baseline --no-host-path --no-probe --no-c2 --no-steady --steps 20 --warmup 5 \
      > gpurun_out/prof_c4ch_$c.txt 2>&1
done
