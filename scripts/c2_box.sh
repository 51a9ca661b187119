#!/bin/bash
# GPU box: the C2 line (PodSecurity restricted over 1M Pods, one MI355X) with CPU baseline + prefix parity, then its
# kernel-trace stats and PMC passes. Usage: bash scripts/c2_box.sh <tag>
set -o pipefail
TAG=${1:-c2}
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload c2 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
grep -v "^{" gpurun_out/${TAG}_bench.log | tail -6
bash scripts/profile_box.sh $TAG --workload c2 || exit 2
