#!/bin/bash
# Round 6: probe tile kernels software-pipelined (product) vs not (NB_PROBE_PREFETCH=0
# build), interleaved processes; tests of the product first.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py -k "entry_formats or overflow or c4_full" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 11; }
tail -3 $O/tests.txt
for rep in 0 1; do
  for v in pf nopf; do
    if [ $v = nopf ]; then export NB_LIB=nasp-key-value-engine_amd/build/libnasp_bloom_nopf.so; else unset NB_LIB; fi
    timeout -k 10 400 python -u tools/probe_chunk.py --workload c4 --reps 1 --chunks 0 --split --entries 0 --batches present,absent,p30 --no-lane > $O/probe_${v}_$rep.txt 2>&1 || { tail -20 $O/probe_${v}_$rep.txt; exit 12; }
    echo "== $v rep $rep"; tail -4 $O/probe_${v}_$rep.txt
  done
done
