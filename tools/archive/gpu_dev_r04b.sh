#!/bin/bash
# Round-4 development call B: the new GPU tests (large-k probe LDS fallback, engine
# flush with an injected device failure), C5's profile (kernel trace + FETCH / WRITE
# / SQ passes -> r04_pmc_c5, r04_kernel_stats_c5, r04_sq_c5) and the N = 2 gloo
# rehearsals of bench.py's C4 / C5 lines with the per-rank diagnostics.
set -u
mkdir -p gpurun_out/r04b; export TMPDIR=/tmp
O=gpurun_out/r04b
timeout -k 10 400 python -u -m pytest tests/test_gpu_probe.py tests/test_engine_dropin.py -m gpu -x -v --timeout 170 --timeout-method thread -k "large_k or injected" > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for w in c4 c5; do
  NB_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2951$([ $w = c4 ] && echo 1 || echo 2) bench.py --gpus 2 --workload $w --steps 3 --warmup 1 > $O/rehearse_${w}_n2.json 2> $O/rehearse_${w}_n2.err || { tail -20 $O/rehearse_${w}_n2.err; exit 2; }
  tail -c 1500 $O/rehearse_${w}_n2.json; echo
done
bash tools/profile_round.sh r04 c5 || exit 3
python3 tools/pmc_traffic.py r04 c5 gpurun_out/prof_r04_c5 || exit 4
python3 tools/sq_summary.py r04 c5 gpurun_out/prof_r04_c5/sq/run_counter_collection.csv || exit 5
cp profiles/r04_* $O/
echo r04b ok
