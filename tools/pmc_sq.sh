#!/bin/bash
# SQ stall breakdown of the build kernels (one PMC pass, kernel trace only).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq_${1:-c2}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU --kernel-trace -d $OUT/a -o run --output-format csv -- python3 bench.py --workload ${1:-c2} --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2> $OUT/a.err || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/b -o run --output-format csv -- python3 bench.py --workload ${1:-c2} --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2> $OUT/b.err || exit 2
echo ok
