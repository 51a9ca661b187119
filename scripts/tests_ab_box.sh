#!/bin/bash
# GPU box: the GPU test suite, then an env A/B of the C3 bench (scripts/env_ab.sh specs as arguments).
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
export KYV_CORPUS_CACHE=/tmp/kc BENCH_ARGS="--no-account --no-gather"
bash scripts/env_ab.sh "$@"
