#!/bin/bash
# Dynamic instruction counts per bin-kernel phase (C2 shape): the diag build
# (tools/ubench_tiled pmc) dispatches the kernel once per stop point; one PMC pass.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/phase_pmc
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES --kernel-trace -d $OUT -o run --output-format csv -- tools/ubench_tiled pmc > $OUT/log.txt 2>&1 || exit 1
echo ok
