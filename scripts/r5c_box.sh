#!/bin/bash
# GPU box (round 5): the GPU suite, the C5 match lists (KYV_DEBUG_STATS), then C3 with the fused walk's parts as one
# kernel (KYV_FUSED_MERGE=1) against the default split.
# Usage: bash scripts/r5c_box.sh <tag> [notests]
set -o pipefail
TAG=${1:-r5c}
mkdir -p gpurun_out
if [ "$2" != notests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
KYV_DEBUG_STATS=1 timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --no-e2e --no-cpu-baseline --no-account > gpurun_out/${TAG}_c5_dbg.log 2>&1 || { tail -30 gpurun_out/${TAG}_c5_dbg.log; exit 2; }
grep "match lists" gpurun_out/${TAG}_c5_dbg.log | head -3
grep "^{" gpurun_out/${TAG}_c5_dbg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d['roofline']['phase_ms'].items()}, d['cpu_fallback_by_reason'])"
export KYV_CORPUS_CACHE=/tmp/kyv_corpus_c3
for mode in 0 1; do
  KYV_FUSED_MERGE=$mode timeout -k 10 400 python -u bench.py --steps 20 --no-e2e --no-cpu-baseline --no-account > gpurun_out/${TAG}_c3_merge$mode.log 2>&1 || { tail -30 gpurun_out/${TAG}_c3_merge$mode.log; exit 3; }
  grep "^{" gpurun_out/${TAG}_c3_merge$mode.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 merge=$mode', d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d['roofline']['phase_ms'].items()})"
done
echo all-done
