#!/bin/bash
# GPU box (round 5): C4 parity with the per-class kind folding of match records (default) and with the lanes = records
# kernel (KYV_MATCH_TILE=1); then C4 bench lines: default, folding off (KYV_KIND_FOLD=0), tile kernel on.
# Usage: bash scripts/r5f_box.sh <tag>
set -o pipefail
TAG=${1:-r5f}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread -k "c4" > gpurun_out/${TAG}_c4_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_c4_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_c4_tests.log
export KYV_CORPUS_CACHE=/tmp/kyv_corpus_c4
for cfg in "KYV_KIND_FOLD=1" "KYV_KIND_FOLD=0" "KYV_MATCH_TILE=1"; do
  env $cfg timeout -k 10 400 python -u bench.py --workload c4 --steps 5 --no-e2e --no-cpu-baseline --no-account > gpurun_out/${TAG}_c4_$cfg.log 2>&1 || { tail -30 gpurun_out/${TAG}_c4_$cfg.log; exit 3; }
  grep "^{" gpurun_out/${TAG}_c4_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $cfg', d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d['roofline']['phase_ms'].items()})"
done
KYV_MATCH_TILE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c4_shape or c4_rule_slices" > gpurun_out/${TAG}_c4_tile_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_c4_tile_tests.log; exit 4; }
tail -2 gpurun_out/${TAG}_c4_tile_tests.log
echo all-done
