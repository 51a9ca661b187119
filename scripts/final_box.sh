#!/bin/bash
# GPU box: full GPU test suite, the default bench line (with CPU baseline), the admission micro-batching bench.
# Usage: bash scripts/final_box.sh <tag>
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 2; }
grep -v "^{" gpurun_out/${TAG}_bench.log | tail -4
timeout -k 10 200 python -u scripts/bench_admission.py --seconds 6 > gpurun_out/${TAG}_admission.log 2>&1 || { tail -20 gpurun_out/${TAG}_admission.log; exit 3; }
grep admission gpurun_out/${TAG}_admission.log
