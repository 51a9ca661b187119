#!/bin/bash
# GPU box (round 5): (1) the round-4 source with the loop-carried PodSecurity flags as uint32_t words, checks inlined
# (exp_build/wt4 variant inlu): expected 0 mismatches where the bool version (inl) had 20,613; (2) the current product
# (checks inlined into eval_pss, integer flags): C5 device == host, the PSS / accounting / staging-ring GPU tests.
set -o pipefail
mkdir -p gpurun_out
(cd exp_build/wt4 && KYV_LIB=exp_build/inlu/libkyvgpu.so timeout -k 10 300 python -u scripts/dbg_pss_guard.py) > gpurun_out/r5d_pss4_inlu.log 2>&1 || { tail -20 gpurun_out/r5d_pss4_inlu.log; exit 1; }
cat gpurun_out/r5d_pss4_inlu.log
DBG_JIT=1 timeout -k 10 300 python -u scripts/dbg_pss_guard.py > gpurun_out/r5d_pss_prod.log 2>&1 || { tail -20 gpurun_out/r5d_pss_prod.log; exit 2; }
cat gpurun_out/r5d_pss_prod.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_accounting.py tests/test_gpu_staging.py "tests/test_gpu_parity.py::test_pss_with_preconditions_gpu_equals_cpu" "tests/test_gpu_parity.py::test_c5_oracle_matrix_at_scale" > gpurun_out/r5d_tests.log 2>&1 || { tail -30 gpurun_out/r5d_tests.log; exit 3; }
tail -3 gpurun_out/r5d_tests.log
