#!/bin/bash
# Round 4: write-out unroll and placement batching re-checked under shard-major buckets
# (compile-time variants from build_variant.sh), C4 and C3, same box, interleaved.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/ab.py --workloads c4,c3 --reps 2 --timeout 300 \
    base:NB_LIB=build_ab/libnasp_bloom_base.so wo1:NB_LIB=build_ab/libnasp_bloom_wo1.so \
    wo4:NB_LIB=build_ab/libnasp_bloom_wo4.so pb0:NB_LIB=build_ab/libnasp_bloom_pb0.so \
    pb2:NB_LIB=build_ab/libnasp_bloom_pb2.so > gpurun_out/ab_wo_pb_gmajor.txt 2>&1
