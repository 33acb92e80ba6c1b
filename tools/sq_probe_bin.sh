set -u
export TMPDIR=/tmp
O=gpurun_out/r06x
mkdir -p $O
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d $O/sq -o run --output-format csv -- python3 tools/probe_kernel_ab.py --batch present --path tiled --entries 32 --kpts 2 --reps 2 > $O/sq.out 2>&1 || { tail -5 $O/sq.out; exit 3; }
python3 - <<'PY'
import csv
from collections import defaultdict
acc=defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open("gpurun_out/r06x/sq/run_counter_collection.csv")):
    n=r["Kernel_Name"]
    k="probe_bin" if "probe_bin" in n else "tile32" if "tile32" in n else "build_bin" if "bloom_bin_kernel" in n else "build_tile" if "tile_or" in n else None
    if k: acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k,v in acc.items():
    print(k, {c: round(sum(x)/len(x)) for c,x in v.items()})
PY
