#!/bin/bash
# Round 6: one-round E32 tiled probe -- 1 vs 2 keys per bin thread, grid-stride bin
# kernel (product) vs one block per bin block (NB_PROBE_GRID_STRIDE=0 build), and auto.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py -k "entry_formats or overflow" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 11; }
tail -2 $O/tests.txt
for rep in 0 1; do
  for v in gs nogs; do
    if [ $v = nogs ]; then export NB_LIB=nasp-key-value-engine_amd/build/libnasp_bloom_nogs.so; else unset NB_LIB; fi
    timeout -k 10 400 python -u tools/probe_chunk.py --workload c4 --reps 1 --chunks 0 --entries 32 --batches present,absent,p30 --no-lane --auto-pct policy \
      --variant 'tiled-kpt1:tiled:NB_PROBE_KPT=1' --variant 'tiled-kpt2:tiled:NB_PROBE_KPT=2' --variant 'auto-host:auto:NB_PROBE_HOST_PICK=1' > $O/probe_${v}_$rep.txt 2>&1 || { tail -20 $O/probe_${v}_$rep.txt; exit 12; }
    echo "== $v rep $rep"; tail -6 $O/probe_${v}_$rep.txt
  done
done
