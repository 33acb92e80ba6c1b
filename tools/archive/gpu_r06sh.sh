# Round 6 (r06sh): the auto probe on shapes its split thresholds were not fitted to
# (VERDICT r05 weak 7); every path against the lane path's answers, same box.
#   bash tools/archive/gpu_r06sh.sh <outdir> [shape names...]
set -e
O=${1:-gpurun_out/r06sh}; shift || true
mkdir -p $O
run() {  # name m k key_len n
  timeout -k 10 240 python -u tools/probe_chunk.py --workload shape --m $2 --k $3 --key-len $4 --n $5 \
    --reps 2 --chunks 0 --split --batches present,absent,p30 --auto-pct policy \
    --variant auto-host:auto:NB_PROBE_HOST_PICK=1 > $O/$1.txt 2>&1
}
SHAPES="
s1 134217728 3 16 30000000
s2 1073741824 5 8 50000000
s3 536870912 10 64 30000000
s4 3000000000 13 24 50000000
s5 4294967295 4 12 50000000
t2 1073741824 5 16 50000000
t3 2147483648 8 16 50000000
t4 536870912 12 32 30000000
t5 4294967295 16 32 50000000
t6 33554432 4 16 5000000
t7 268435456 6 32 30000000
u1 958505838 3 16 50000000
u2 958505838 4 16 50000000
u3 958505838 7 16 5000000
u4 958505838 7 16 10000000
u5 958505838 7 16 20000000
u6 67108864 4 16 10000000
u7 268435456 7 32 5000000
v1 33554432 4 16 30000000
v2 16777216 7 32 20000000
v3 67108864 7 16 30000000
"
# s*: fixed lengths other than 16 / 32 bytes, and t5 (k = 16 at m = 2^32 - 1) probe on
# the lane kernel only; v1 / v2: filters smaller than the batch (the filled keys repeated)
echo "$SHAPES" | while read name m k kl n; do
  [ -z "$name" ] && continue
  if [ $# -gt 0 ] && ! [[ " $* " == *" $name "* ]]; then continue; fi
  run $name $m $k $kl $n
done
