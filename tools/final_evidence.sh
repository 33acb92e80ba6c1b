#!/bin/bash
# One GPU call for a round's closing evidence at the current kernels: profiles of
# C4/C2/C3/C5 (tools/profile_round.sh), their summaries written into profiles/ on
# the box (so bench.py reads them back) and copied to gpurun_out/ for the build
# container, then smoke, the GPU suite and the bench lines (tools/round_evidence.sh).
#   tools/final_evidence.sh <tag>
set -u
TAG=${1:-r02e}
for w in c4 c2 c3 c5; do bash tools/profile_round.sh "$TAG" "$w" || exit 1; done
for w in c4 c2 c3 c5; do python3 tools/pmc_traffic.py "$TAG" "$w" "gpurun_out/prof_${TAG}_$w" || exit 2; done
for w in c4 c2 c3 c5; do
  python3 tools/sq_summary.py "$TAG" "$w" "gpurun_out/prof_${TAG}_$w/sq/run_counter_collection.csv" || exit 3
done
mkdir -p "gpurun_out/profiles_$TAG"
cp profiles/${TAG}_* "gpurun_out/profiles_$TAG/"
bash tools/round_evidence.sh "$TAG"
