# Round 6 (r06pl): same-box A/B of the probe's looping bin kernel, HEAD against a variant that
# preloads the next bin block's keys (reverted; profiles/r06pl_loop_bin_sq_and_preload_ab.txt).
# The two libraries were built in this container by __graft_entry__.build() at HEAD and with the
# variant, copied to abtmp/ (since removed), and picked per run through NB_LIB.
set -e
mkdir -p gpurun_out/r06pl
for i in 1 2; do
for v in head pre; do
NB_LIB=abtmp/libnasp_bloom_$v.so timeout -k 10 150 python -u tools/probe_chunk.py --workload c4 --no-lane --reps 3 --chunks 0 --auto-pct policy --variant auto-host:auto:NB_PROBE_HOST_PICK=1 > gpurun_out/r06pl/ab_c4_${v}_$i.txt 2>&1
done; done
for v in head pre; do
NB_LIB=abtmp/libnasp_bloom_$v.so timeout -k 10 150 python -u tools/probe_chunk.py --workload c5 --no-lane --reps 3 --chunks 0 --auto-pct policy --variant auto-host:auto:NB_PROBE_HOST_PICK=1 > gpurun_out/r06pl/ab_c5_${v}.txt 2>&1
done
