#!/bin/bash
# Packed fine entries in the two-level build: parity subset, then C5 A/B.
set -u
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "two_level or tile_policy or c5 or edge_m or golden_large or spill" > gpurun_out/pk5.log 2>&1
rc=$?; tail -5 gpurun_out/pk5.log; [ $rc -eq 0 ] || exit $rc
run() {  # name workload env...
  local name=$1 w=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-host-path --no-probe --steps 3 --warmup 1 \
    > gpurun_out/sweep/$name.json 2> gpurun_out/sweep/$name.err || { echo "$name failed"; return 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'])"
}
run c5_u32 c5 NB_PACK=0 && run c5_pk c5 NB_PACK=1 && run c5_u32b c5 NB_PACK=0 && run c5_pkb c5 NB_PACK=1
