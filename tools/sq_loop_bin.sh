set -u
export TMPDIR=/tmp
O=gpurun_out/r06loop
mkdir -p $O
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/sq -o run --output-format csv -- python3 tools/probe_auto_trace.py --reps 2 --batches present > $O/sq.out 2>&1 || { tail -5 $O/sq.out; exit 3; }
python3 - <<'PY'
import csv
from collections import defaultdict
acc=defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open("gpurun_out/r06loop/sq/run_counter_collection.csv")):
    n=r["Kernel_Name"]
    if "probe_bin_loop" in n: k="loop_bin"
    elif "probe_bin_kernel" in n: k="plain_bin"
    else: continue
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k,v in acc.items():
    print(k, {c: [round(x) for x in xs] for c,xs in v.items()})
PY
