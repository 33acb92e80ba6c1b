#!/bin/bash
# Round 6 close, part 2 (after tools/final_profiles.sh <tag> c4 c2, <tag> c3 c5 and
# tools/profile_probe.sh <tag>, their summaries copied into profiles/): smoke, the GPU
# suite, the bench lines (tools/round_evidence.sh), the N = 2 rehearsals of
# `bench.py --gpus 2` with no external launcher (it starts its two ranks itself;
# NB_BENCH_BACKEND=gloo lets them share the one GPU), and the C4 probe sweep.
set -u
TAG=${1:-r06z}
export TMPDIR=/tmp
bash tools/round_evidence.sh "$TAG" || exit $?
O=gpurun_out/ev_$TAG
for w in c4 c5; do
  NB_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --workload $w --steps 3 --warmup 1 > $O/rehearse_${w}_n2.json 2> $O/rehearse_${w}_n2.err || { tail -20 $O/rehearse_${w}_n2.err; exit 12; }
  tail -c 400 $O/rehearse_${w}_n2.json; echo
done
timeout -k 10 600 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --batches present,absent,p10,p30,p50,p70 --auto-pct policy --variant 'auto-host:auto:NB_PROBE_HOST_PICK=1' > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 13; }
tail -8 $O/probe_c4.txt
echo "final ok $TAG"
