#!/bin/bash
# GPU box (round 5): the match-related GPU tests, then the C4 bench line (accounting, CPU baseline, timed-batch parity)
set -o pipefail
TAG=${1:-c4q}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "c4 or match or exception or accounting or goldens" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
KYV_DEBUG_STATS=1 bash scripts/r5_box.sh $TAG notests c4
grep "match records" gpurun_out/${TAG}_c4_bench.log | head -8
