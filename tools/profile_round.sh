#!/bin/bash
# Profile bench.py's build kernels on the GPU box (run under gpurun):
#   1. kernel trace + stats (per-kernel durations)
#   2. separate PMC passes: FETCH_SIZE, WRITE_SIZE (TCC slots don't fit both), SQ counters
# Outputs under gpurun_out/prof_<tag>/; tools/pmc_traffic.py turns them into
# profiles/<tag>_pmc_<workload>.json.
set -u
TAG=${1:-r01}
WL=${2:-c2}
OUT=gpurun_out/prof_${TAG}_${WL}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --workload $WL --no-cpu-baseline --no-host-path --no-probe --steps 10 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $B > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/fetch" -o run --output-format csv -- $B > /dev/null 2> "$OUT/fetch.err" || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write" -o run --output-format csv -- $B > /dev/null 2> "$OUT/write.err" || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/sq" -o run --output-format csv -- $B > /dev/null 2> "$OUT/sq.err" || exit 4
echo "profile ok"
