#!/bin/bash
# A/B of packed (3 x 21-bit per u64) vs 32-bit bucket entries on C3/C4, one box.
set -u
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
run() {  # name workload env...
  local name=$1 w=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-host-path --no-probe --steps 10 \
    > gpurun_out/sweep/$name.json 2> gpurun_out/sweep/$name.err || { echo "$name failed"; return 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['roofline'].get('kernel_ms'), d['ms_per_step'])"
}
run c4_u32 c4 NB_PACK=0 && run c4_pk c4 NB_PACK=1 && run c4_u32b c4 NB_PACK=0 && run c4_pkb c4 NB_PACK=1 \
&& run c3_u32 c3 NB_PACK=0 && run c3_pk c3 NB_PACK=1 && run c2 c2 NB_PACK=1
