#!/bin/bash
# Round 6: grid-stride bin kernel with laundered arguments (product) vs one block per
# bin block (NB_PROBE_GRID_STRIDE=0 build, ungated paths only); kpt 1 / 2; auto.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py tests/test_gpu_graph.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 11; }
tail -2 $O/tests.txt
for rep in 0 1; do
  for v in gs nogs; do
    if [ $v = nogs ]; then export NB_LIB=nasp-key-value-engine_amd/build/libnasp_bloom_nogs.so; A=""; else unset NB_LIB; A="--auto-pct policy --variant auto-host:auto:NB_PROBE_HOST_PICK=1"; fi
    timeout -k 10 400 python -u tools/probe_chunk.py --workload c4 --reps 1 --chunks 0 --entries 32 --split --batches present,absent,p30 --no-lane $A \
      --variant 'tiled-kpt1:tiled:NB_PROBE_KPT=1' > $O/probe_${v}_$rep.txt 2>&1 || { tail -20 $O/probe_${v}_$rep.txt; exit 12; }
    echo "== $v rep $rep"; tail -6 $O/probe_${v}_$rep.txt
  done
done
