#!/bin/bash
# The batch probe's profiles (run under gpurun): per batch kind, a kernel trace and
# separate FETCH_SIZE / WRITE_SIZE passes of tools/probe_pmc.py, then (on the box, so
# a later bench.py in the same call reads it back) tools/pmc_probe.py ->
# profiles/<tag>_pmc_probe_c4.json.
#   tools/profile_probe.sh <tag>
set -u
TAG=${1:-r06}
OUT=gpurun_out/prof_${TAG}_probe
mkdir -p "$OUT"
export TMPDIR=/tmp
for b in present p30 absent; do
  mkdir -p "$OUT/$b"
  P="python3 tools/probe_pmc.py --batch $b --calls 3"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$b/trace" -o run --output-format csv -- $P > "$OUT/$b/trace.out" 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/$b/fetch" -o run --output-format csv -- $P > "$OUT/$b/fetch.out" 2>&1 || exit 2
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/$b/write" -o run --output-format csv -- $P > "$OUT/$b/write.out" 2>&1 || exit 3
done
python3 tools/pmc_probe.py "$TAG" "$OUT" 3 || exit 4
cp profiles/${TAG}_pmc_probe_c4.json "$OUT/"
echo "probe profile ok $TAG"
