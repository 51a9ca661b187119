#!/bin/bash
# GPU box (round 5): condition / C5 GPU tests, then the C5 bench line (accounting, CPU baseline, timed-batch parity)
set -o pipefail
TAG=${1:-c5q}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "c5 or condition or pss or accounting or foreach or jmes or exception" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
bash scripts/r5_box.sh $TAG notests c5
