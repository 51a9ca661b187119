#!/bin/bash
# GPU box (round 6): selected GPU tests, then C5 and C3 quick bench lines (no accounting / CPU baseline)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "c5 or jmes or exclude_all or function or condition" > gpurun_out/r6g_tests.log 2>&1 || { tail -40 gpurun_out/r6g_tests.log; exit 1; }
tail -2 gpurun_out/r6g_tests.log
BENCH_ARGS="--workload c5 --no-account" bash scripts/env_ab.sh "c5:KYV_COLCACHE=4" || exit 2
BENCH_ARGS="--no-account" bash scripts/env_ab.sh "c3:KYV_COLCACHE=4" || exit 3
