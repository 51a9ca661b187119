#!/bin/bash
# GPU box: PodSecurity GPU tests, then C2 and C5 quick lines (C5 with both waves/EU targets of the precondition PSS kernel)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "pss or c2 or c5 or goldens" > gpurun_out/r6j_tests.log 2>&1 || { tail -40 gpurun_out/r6j_tests.log; exit 1; }
tail -2 gpurun_out/r6j_tests.log
BENCH_ARGS="--workload c2 --no-account" bash scripts/env_ab.sh "c2:KYV_COLCACHE=4" || exit 2
BENCH_ARGS="--workload c5 --no-account" bash scripts/env_ab.sh "c5w6:KYV_PSS_PRE_WPE=6" "c5w4:KYV_PSS_PRE_WPE=4" || exit 3
