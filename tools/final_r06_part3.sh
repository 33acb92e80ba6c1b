set -u
export TMPDIR=/tmp
O=gpurun_out/ev_r06z
mkdir -p $O
for w in c4 c5; do
  NB_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --workload $w --steps 3 --warmup 1 > $O/rehearse_${w}_n2.json 2> $O/rehearse_${w}_n2.err || { tail -20 $O/rehearse_${w}_n2.err; exit 12; }
  tail -c 300 $O/rehearse_${w}_n2.json; echo
done
timeout -k 10 600 python -u tools/probe_chunk.py --workload c4 --reps 2 --chunks 0 --split --batches present,absent,p10,p30,p50,p70 --auto-pct policy --variant 'auto-host:auto:NB_PROBE_HOST_PICK=1' > $O/probe_c4.txt 2>&1 || { tail -20 $O/probe_c4.txt; exit 13; }
tail -8 $O/probe_c4.txt
