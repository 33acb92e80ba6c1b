#!/bin/bash
# A/B sweep of the tile geometry knobs (NB_TILE_BITS, NB_SHARDS) on C2/C3/C4, one box.
set -u
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
run() {  # name workload env...
  local name=$1 w=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-host-path --no-probe --steps 10 \
    > gpurun_out/sweep/$name.json 2> gpurun_out/sweep/$name.err || { echo "$name failed"; return 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['roofline'].get('kernel_ms'), d['ms_per_step'])"
}
run c2_g8 c2 NB_SHARDS=8 && run c2_g16 c2 NB_SHARDS=16 && run c2_g12 c2 NB_SHARDS=12 && run c2_g8b c2 NB_SHARDS=8 && run c2_g16b c2 NB_SHARDS=16 \
&& run c4_g8 c4 NB_SHARDS=8 && run c4_g16 c4 NB_SHARDS=16 && run c4_g8b c4 NB_SHARDS=8 \
&& run c3_g8 c3 NB_SHARDS=8 && run c3_g16 c3 NB_SHARDS=16 \
&& run c5_g8 c5 NB_SHARDS=8 && run c5_g16 c5 NB_SHARDS=16
