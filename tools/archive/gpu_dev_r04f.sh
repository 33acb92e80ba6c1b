#!/bin/bash
# Round-4 development call F: C2 (10M keys, 183 power-of-two tiles: the tile kernel
# fills 183 of 256 CUs) against 256 / 512 counted tiles, interleaved A/B.
set -u
mkdir -p gpurun_out/r04f; export TMPDIR=/tmp
O=gpurun_out/r04f
timeout -k 10 600 python -u tools/ab.py --workloads c2 --reps 3 base: t256:NB_TILE_COUNT=256 t512:NB_TILE_COUNT=512 > $O/ab_c2_tiles.txt 2>&1 || { tail -20 $O/ab_c2_tiles.txt; exit 3; }
cat $O/ab_c2_tiles.txt
