#!/bin/bash
# GPU box: parity tests then a short bench (no CPU baseline). Usage: bash scripts/gpu_check.sh <tag> [bench args]
set -o pipefail
TAG=${1:-chk}; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 2; }
grep -v "^{" gpurun_out/${TAG}_bench.log | tail -5
python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/${TAG}_bench.log') if l.startswith('{')][0]); print('VALUE %.4g evals/s  kernel %.3f ms  frac %.4f' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
