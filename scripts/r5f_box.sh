#!/bin/bash
# GPU box (round 5): C4 with the lanes = records match kernel (KYV_MATCH_TILE=1) against match_rec_kernel alone, then
# its parity test with the tile kernel on.
# Usage: bash scripts/r5f_box.sh <tag>
set -o pipefail
TAG=${1:-r5f}
mkdir -p gpurun_out
export KYV_CORPUS_CACHE=/tmp/kyv_corpus_c4
for mode in 0 1; do
  KYV_MATCH_TILE=$mode timeout -k 10 400 python -u bench.py --workload c4 --steps 5 --no-e2e --no-cpu-baseline --no-account > gpurun_out/${TAG}_c4_tile$mode.log 2>&1 || { tail -30 gpurun_out/${TAG}_c4_tile$mode.log; exit 3; }
  grep "^{" gpurun_out/${TAG}_c4_tile$mode.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 tile=$mode', d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d['roofline']['phase_ms'].items()})"
done
KYV_MATCH_TILE=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread -k "c4_shape or c4_rule_slices or c4_policycache" > gpurun_out/${TAG}_c4_tile_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_c4_tile_tests.log; exit 4; }
tail -2 gpurun_out/${TAG}_c4_tile_tests.log
echo all-done
