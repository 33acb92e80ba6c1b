#!/bin/bash
# Round 4 close: the N = 2 gloo rehearsals of bench.py (two ranks sharing the one GPU)
# at the final kernels, C4 and C5, with their per-rank diagnostic fields.
set -u
mkdir -p gpurun_out/r04u; export TMPDIR=/tmp
O=gpurun_out/r04u
for w in c4 c5; do
  NB_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2961$([ $w = c4 ] && echo 1 || echo 2) bench.py --gpus 2 --workload $w --steps 3 --warmup 1 > $O/rehearse_${w}_n2.json 2> $O/rehearse_${w}_n2.err || { tail -20 $O/rehearse_${w}_n2.err; exit 2; }
  tail -c 600 $O/rehearse_${w}_n2.json; echo
done
echo r04u ok
