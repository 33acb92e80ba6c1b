#!/bin/bash
# C2 A/B with repeats: default policy (packed entries, 2^19-bit tiles) vs NB_PACK=0
# (u16 entries at 2^16-bit tiles), after the parity tests that cover the policy.
set -u
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
run() {
  local name=$1 w=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-host-path --no-probe --steps 50 \
    > gpurun_out/sweep/$name.json 2> gpurun_out/sweep/$name.err || { echo "$name failed"; return 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['roofline'].get('kernel_ms'), d['ms_per_step'])"
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tp3.log 2>&1
rc=$?; tail -3 gpurun_out/tp3.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  run c2_pk_$r c2 NB_X=0 && run c2_u16_$r c2 NB_PACK=0 || exit 1
done
