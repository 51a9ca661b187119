#!/bin/bash
# GPU box (round 5, second half): the GPU suite; the C5 match lists (KYV_DEBUG_STATS) and bench line; C5 profile.
# Usage: bash scripts/r5b_box.sh <tag>
set -o pipefail
TAG=${1:-r5b}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
KYV_DEBUG_STATS=1 timeout -k 10 400 python -u bench.py --workload c5 --steps 5 --no-e2e --no-cpu-baseline --no-account > gpurun_out/${TAG}_c5_dbg.log 2>&1 || { tail -30 gpurun_out/${TAG}_c5_dbg.log; exit 2; }
grep "match lists" gpurun_out/${TAG}_c5_dbg.log | head -3
bash scripts/r5_box.sh $TAG notests c5 || exit 3
bash scripts/profile_box.sh ${TAG}_c5 --workload c5 || exit 4
echo all-done
