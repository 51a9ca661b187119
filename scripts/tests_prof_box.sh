#!/bin/bash
# GPU box: the GPU test suite, then a profile (kernel trace + PMC passes) of one workload.
# Usage: bash scripts/tests_prof_box.sh <tag> [bench args for the profile...]
set -o pipefail
TAG=${1:-r}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
bash scripts/profile_box.sh ${TAG} "$@" || exit 2
echo done
