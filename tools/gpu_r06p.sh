#!/bin/bash
# Round 6: probe PMC profiles, then a short bench line that reads them back.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
bash tools/profile_probe.sh r06p || exit 11
timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 12; }
python3 -c "
import json; d=json.loads(open('$O/bench_c4.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for p,v in d['probe'].items():
    if p=='note': continue
    print(p, {b: (x['ms'], x['roofline']['frac'], x['roofline']['traffic']) for b,x in v.items()})
"
