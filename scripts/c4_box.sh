#!/bin/bash
# GPU box: C4 rule-slice tests and the C4 bench line (10k policies over 1M mixed resources).
set -o pipefail
TAG=${1:-c4}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "c4" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -4 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-e2e > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 3; }
grep -v "^{" gpurun_out/${TAG}_bench.log | tail -8
