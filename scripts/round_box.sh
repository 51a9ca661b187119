#!/bin/bash
# GPU box: GPU test suite, smoke(), the default bench line (CPU baseline + prefix parity + e2e).
# Usage: bash scripts/round_box.sh <tag> [extra bench args...]
set -o pipefail
TAG=${1:-r}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 2; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 700 python -u bench.py "$@" > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 3; }
grep -v "^{" gpurun_out/${TAG}_bench.log | tail -6
