#!/bin/bash
# Baseline measurements at HEAD on one box: bench lines (device-resident only),
# kernel-trace stats and the SQ VALU counters of the build kernels for each
# workload given (default c2 c4).  Output under gpurun_out/base_<tag>/.
set -u
TAG=${1:-r02}
shift || true
WLS=${@:-c2 c4}
OUT=gpurun_out/base_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in $WLS; do
  B="python3 bench.py --workload $w --no-cpu-baseline --no-host-path --no-probe --steps 10 --warmup 2"
  timeout -k 10 300 $B > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$w" -o run --output-format csv -- $B > /dev/null 2> "$OUT/trace_$w.err" || exit 2
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/sq_$w" -o run --output-format csv -- $B > /dev/null 2> "$OUT/sq_$w.err" || exit 3
done
echo "baseline ok"
