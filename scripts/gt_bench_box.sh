#!/bin/bash
# GPU box: selected GPU tests, then a short default bench (timed line + native gather, no CPU baseline / e2e).
# Usage: bash scripts/gt_bench_box.sh <tag> <pytest -k expression>
set -o pipefail
TAG=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$2" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-account > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 2; }
grep -v "^{" gpurun_out/${TAG}_bench.log | tail -4
