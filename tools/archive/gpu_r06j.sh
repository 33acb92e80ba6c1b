#!/bin/bash
# Round 6: per-kernel traces of the one-round tiled probe (E32 kpt 1 / 2, E64) on
# present / p30 keys, product library and the one-block-per-bin-block build.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
for v in gs nogs; do
  if [ $v = nogs ]; then export NB_LIB=nasp-key-value-engine_amd/build/libnasp_bloom_nogs.so; else unset NB_LIB; fi
  for b in present p30; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$b -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch $b --path tiled --entries 32,64 --kpts 1,2 > $O/ab_${v}_$b.txt 2>&1 || { tail -20 $O/ab_${v}_$b.txt; exit 13; }
    echo "== $v $b"; grep "ms per call" $O/ab_${v}_$b.txt
    python3 tools/trace_rounds.py $O/prof_${v}_$b/run_kernel_trace.csv | head -7
  done
done
