# Round 6 (r06tl): same-box A/B of auto's gated tile kernels looping over the tiles
# (variant since removed; profiles/r06tl_gated_tile_loop_ab.txt).  The two libraries were
# built in this container by __graft_entry__.build() at HEAD and with the variant, copied
# to abtmp/ and picked per run through NB_LIB.
set -e
O=gpurun_out/r06tl
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_probe.py tests/test_gpu_graph.py tests/test_gpu_buckets.py > $O/tests.txt 2>&1
for i in 1 2; do for v in head new; do
NB_LIB=abtmp/libnasp_bloom_$v.so timeout -k 10 200 python -u tools/probe_chunk.py --workload c4 --no-lane --reps 3 --chunks 0 --split --auto-pct policy --variant auto-host:auto:NB_PROBE_HOST_PICK=1 > $O/c4_${v}_$i.txt 2>&1
done; done
for v in head new; do NB_LIB=abtmp/libnasp_bloom_$v.so bash tools/archive/gpu_r06sh.sh $O/sh_$v u3 u4 u5 u7 t2 t3; done
