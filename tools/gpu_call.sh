set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
for rep in 0 1; do for v in base pserial; do
  if [ $v = base ]; then L=""; else L="$PWD/build_ab/libnasp_bloom_$v.so"; fi
  NB_LIB=$L timeout -k 10 200 python bench.py --workload c4 --no-cpu-baseline --no-host-path --no-c2 --steps 5 > gpurun_out/probe_${v}_$rep.json 2>gpurun_out/probe_${v}_$rep.err || exit 3
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d['probe']; print(sys.argv[2], 'present', p['present']['ms'], 'absent', p['absent']['ms'], p['absent']['positive_rate'])" gpurun_out/probe_${v}_$rep.json $v
done; done
timeout -k 10 900 python -u tools/ab.py --workloads c4,c3,c5 --reps 2 base: ntkeys:NB_LIB=build_ab/libnasp_bloom_ntkeys.so ntld0:NB_LIB=build_ab/libnasp_bloom_ntld0.so > gpurun_out/ab_nt2.txt 2>&1 || { tail -20 gpurun_out/ab_nt2.txt; exit 4; }
tail -10 gpurun_out/ab_nt2.txt
echo done
