#!/bin/bash
# A round's closing profiles at the current kernels, one GPU call (part 1 of the
# closing evidence; part 2 is tools/round_evidence.sh): tools/profile_round.sh per
# workload, then the PMC traffic and SQ summaries written into profiles/ on the box
# (so the bench lines of part 2 read them back) and copied to gpurun_out/.
#   tools/final_profiles.sh <tag> [workloads...]
set -u
TAG=${1:-r04f}; shift
WLS=${@:-c4 c2 c3 c5}
for w in $WLS; do bash tools/profile_round.sh "$TAG" "$w" || exit 1; done
for w in $WLS; do
  python3 tools/pmc_traffic.py "$TAG" "$w" "gpurun_out/prof_${TAG}_$w" || exit 2
  python3 tools/sq_summary.py "$TAG" "$w" "gpurun_out/prof_${TAG}_$w/sq/run_counter_collection.csv" || exit 3
done
mkdir -p "gpurun_out/profiles_$TAG"
cp profiles/${TAG}_* "gpurun_out/profiles_$TAG/"
echo "profiles ok $TAG"
