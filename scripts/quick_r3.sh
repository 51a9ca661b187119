set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_jmes_foreach.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "jmes or foreach or c3_oracle or c5 or goldens_merged_gpu_jit or condition" > gpurun_out/r3c_tests.log 2>&1 || { tail -40 gpurun_out/r3c_tests.log; exit 1; }
tail -3 gpurun_out/r3c_tests.log
timeout -k 10 300 python -u bench.py --resources 1250000 --no-cpu-baseline --no-e2e > gpurun_out/r3c_bench.log 2>&1 || { tail -30 gpurun_out/r3c_bench.log; exit 3; }
grep -o '"phase_ms": {[^}]*}' gpurun_out/r3c_bench.log
