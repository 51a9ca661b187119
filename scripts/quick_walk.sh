#!/bin/bash
# GPU box: walk-kernel parity tests (runtime-compiled and interpreted walks vs the oracle) + a 1.25M C3 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "jit or interpreter or walk_goldens or c3_synthetic or quirk or c4_rule_slices or empty" > gpurun_out/qw_tests.log 2>&1 || { tail -40 gpurun_out/qw_tests.log; exit 1; }
tail -3 gpurun_out/qw_tests.log
timeout -k 10 300 python -u bench.py --resources 1250000 --no-cpu-baseline --no-e2e --steps 10 --warmup 2 > gpurun_out/qw_bench.log 2>&1 || { tail -30 gpurun_out/qw_bench.log; exit 3; }
grep -o '"phase_ms": {[^}]*}' gpurun_out/qw_bench.log
