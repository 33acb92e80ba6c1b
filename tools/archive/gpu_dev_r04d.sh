set -u
mkdir -p gpurun_out/r04d
timeout -k 10 300 tools/ubench_c4 pipe > gpurun_out/r04d/ubc4_pipe.txt 2>&1; rc=$?
cat gpurun_out/r04d/ubc4_pipe.txt; exit $rc
