#!/bin/bash
# GPU box: selected GPU parity tests, then the default bench line (no CPU baseline) and its kernel-trace stats.
# Usage: bash scripts/quick_box.sh <tag> "<pytest -k expression or empty>" [bench args...]
set -o pipefail
TAG=${1:-q}; K=${2:-}; shift 2
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e "$@" > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 3; }
grep -v "^{" gpurun_out/${TAG}_bench.log | tail -4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/gpurun_out/prof_$TAG -o run -- python3 $OLDPWD/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e "$@" > $OLDPWD/gpurun_out/${TAG}_trace.log 2>&1 || exit 4
head -6 $OLDPWD/gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -c1-160
