#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pp
for w in ${WORKLOADS:-c2 c4 c3}; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pp/$w -o run --output-format csv -- tools/ubench_tiled $w pmc > gpurun_out/pp/$w.log 2>&1 || exit 1
done
echo pmc ok
