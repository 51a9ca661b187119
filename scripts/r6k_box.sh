#!/bin/bash
# GPU box: PodSecurity GPU tests, then the C2 quick line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "pss or c2 or goldens" > gpurun_out/r6k_tests.log 2>&1 || { tail -40 gpurun_out/r6k_tests.log; exit 1; }
tail -2 gpurun_out/r6k_tests.log
BENCH_ARGS="--workload c2 --no-account" bash scripts/env_ab.sh "c2:KYV_COLCACHE=4" || exit 2
