#!/bin/bash
# A/B sweep of the tile geometry knobs (NB_TILE_BITS, NB_SHARDS, NB_PACK) on one box.
set -u
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
run() {  # name workload env...
  local name=$1 w=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-host-path --no-probe --steps 10 \
    > gpurun_out/sweep/$name.json 2> gpurun_out/sweep/$name.err || { echo "$name failed"; return 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['roofline'].get('kernel_ms'), d['ms_per_step'])"
}
run c2_ts16 c2 NB_X=0 && run c2_ts17p c2 NB_TILE_BITS=17 && run c2_ts18p c2 NB_TILE_BITS=18 && run c2_ts19p c2 NB_TILE_BITS=19 && run c2_ts16b c2 NB_X=0 \
&& run c4_ts20 c4 NB_X=0 && run c4_ts19p c4 NB_TILE_BITS=19
