#!/bin/bash
# GPU box: PodSecurity parity tests, then C2 bench A/B over the PSS kernel knobs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pss or c2" > gpurun_out/c2ab_tests.log 2>&1 || { tail -40 gpurun_out/c2ab_tests.log; exit 1; }
tail -3 gpurun_out/c2ab_tests.log
BENCH_ARGS="--workload c2" bash scripts/env_ab.sh "w6:X=1" "w4:KYV_PSS_WPE=4" "w8:KYV_PSS_WPE=8" "matchk:KYV_PSS_KERNEL=0" "w6r:X=1"
