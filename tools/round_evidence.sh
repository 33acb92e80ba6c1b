#!/bin/bash
# Round-end GPU evidence (run under gpurun), part 1: smoke, the full GPU suite and
# the bench lines.  Part 2 is tools/profile_round.sh per workload.
#   tools/round_evidence.sh <tag>
set -u
TAG=${1:-r02}
O=gpurun_out/ev_$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$O/pytest_gpu.log"; tail -2 "$O/pytest_gpu.log"
[ $rc -eq 0 ] || exit 2
# the driver's line (its own flags): C4 (+ C2, probe, host path, 8-core reference baseline)
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_c4.json" 2> "$O/bench_c4.err" || exit 3
timeout -k 10 300 python bench.py --workload c3 --no-host-path > "$O/bench_c3.json" 2> "$O/bench_c3.err" || exit 4
timeout -k 10 300 python bench.py --workload c2 --no-host-path --no-probe > "$O/bench_c2.json" 2> "$O/bench_c2.err" || exit 5
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 > "$O/bench_c5.json" 2> "$O/bench_c5.err" || exit 6
timeout -k 10 300 python bench.py --workload merkle > "$O/bench_merkle.json" 2> "$O/bench_merkle.err" || exit 7
echo "evidence ok $TAG"
