#!/bin/bash
# Round 5 close, part 2 (after tools/final_profiles.sh <tag> c4 c2 c3 c5 and the
# profiles copied into profiles/): smoke, the GPU suite, the bench lines
# (tools/round_evidence.sh) and the N = 2 gloo rehearsals of bench.py at the final
# kernels (two ranks sharing the one GPU; C4 and C5, with their per-rank fields), and
# the probe sweeps.
set -u
TAG=${1:-r05x}
export TMPDIR=/tmp
bash tools/round_evidence.sh "$TAG" || exit $?
O=gpurun_out/ev_$TAG
for w in c4 c5; do
  NB_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2961$([ $w = c4 ] && echo 1 || echo 2) bench.py --gpus 2 --workload $w --steps 3 --warmup 1 > $O/rehearse_${w}_n2.json 2> $O/rehearse_${w}_n2.err || { tail -20 $O/rehearse_${w}_n2.err; exit 12; }
  tail -c 400 $O/rehearse_${w}_n2.json; echo
done
# the probe paths across present fractions (C4's filter, C5's shape, C3's keys), answers checked
timeout -k 10 600 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --batches present,absent,p10,p20,p30,p40,p50,p60,p70 --auto-pct 30 > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 13; }
tail -6 $O/probe_c4.txt
timeout -k 10 400 python -u tools/probe_chunk.py --workload c5 --reps 1 --chunks 0 --split --batches present,absent,p10,p20,p30,p40,p50,p70 --auto-pct 30 > $O/probe_c5.txt 2>&1 || { tail -20 $O/probe_c5.txt; exit 14; }
tail -6 $O/probe_c5.txt
timeout -k 10 700 python -u tools/probe_chunk.py --workload c3 --reps 1 --chunks 0 --split --batches present,absent,p10,p20,p30,p40,p50,p70 --auto-pct 30 > $O/probe_c3.txt 2>&1 || { tail -20 $O/probe_c3.txt; exit 15; }
tail -6 $O/probe_c3.txt
echo "final ok $TAG"
