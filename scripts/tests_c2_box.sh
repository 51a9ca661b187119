#!/bin/bash
# GPU box: the GPU test suite, then the C2 profile (kernel trace + PMC passes).
# Usage: bash scripts/tests_c2_box.sh <tag>
set -o pipefail
TAG=${1:-r}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
bash scripts/profile_box.sh ${TAG}_c2 --workload c2 || exit 2
echo done
