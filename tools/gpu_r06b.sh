#!/bin/bash
# Round 6: per-kernel times of the split probe's entry formats on p30 / absent / present.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
for b in p30 absent present; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$b -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch $b --path split > $O/ab_$b.txt 2>&1 || { tail -20 $O/ab_$b.txt; exit 11; }
  grep "ms per call" $O/ab_$b.txt
done
