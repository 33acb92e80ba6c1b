#!/bin/bash
# THE recipe for a round's profiles (run under gpurun; one workload per call is
# safest -- each pass re-runs bench.py):
#   tools/profile_round.sh <tag> <workload>      e.g.  tools/profile_round.sh r02 c4
# 1. kernel trace + stats of the device-resident bench (per-kernel durations);
# 2. separate PMC passes (a TCC pass cannot hold both): FETCH_SIZE, then WRITE_SIZE;
# 3. an SQ pass (VALU / LDS instruction counts, busy cycles, GRBM_GUI_ACTIVE clock).
# Outputs under gpurun_out/prof_<tag>_<workload>/; then, in the build container:
#   python tools/pmc_traffic.py <tag> <workload>   -> profiles/<tag>_pmc_<wl>.json (+ kernel stats csv)
#   python tools/sq_summary.py <tag> <wl key> gpurun_out/prof_<tag>_<wl>/sq/run_counter_collection.csv
#                                                -> profiles/<tag>_sq_<wl>.json
# bench.py reads both back (roofline.traffic, roofline.valu_frac) only while their
# kernel_source_sha matches the current kernels.
set -u
TAG=${1:-r02}
WL=${2:-c4}
OUT=gpurun_out/prof_${TAG}_${WL}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --workload $WL --no-cpu-baseline --no-host-path --no-probe --no-c2 --no-rank-share --no-steady --steps 10 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $B > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/fetch" -o run --output-format csv -- $B > /dev/null 2> "$OUT/fetch.err" || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write" -o run --output-format csv -- $B > /dev/null 2> "$OUT/write.err" || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/sq" -o run --output-format csv -- $B > /dev/null 2> "$OUT/sq.err" || exit 4
echo "profile ok $TAG $WL"
