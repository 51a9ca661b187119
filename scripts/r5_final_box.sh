#!/bin/bash
# GPU box (round 5, final measurements): per workload the full bench line (accounting, CPU baseline, timed-batch
# parity; the end-to-end leg for C3) then its rocprofv3 kernel trace + PMC passes (scripts/profile_box.sh).
# Usage: bash scripts/r5_final_box.sh <tag> <workload>...
set -o pipefail
TAG=${1:-r5z}; shift
mkdir -p gpurun_out
for wl in "$@"; do
  bash scripts/r5_box.sh $TAG notests $wl || exit 2
  bash scripts/profile_box.sh ${TAG}_$wl --workload $wl || exit 3
done
echo all-done
