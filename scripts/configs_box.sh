#!/bin/bash
# GPU box: bench lines (with CPU baseline + oracle prefix parity) of the non-headline configs C2, C4, C5.
# Usage: bash scripts/configs_box.sh <tag>
set -o pipefail
TAG=${1:-cfg}
mkdir -p gpurun_out
for w in c2 c5 c4; do
  S=20; [ $w = c4 ] && S=3
  timeout -k 10 400 python -u bench.py --workload $w --steps $S --warmup 1 --no-e2e > gpurun_out/${TAG}_$w.log 2>&1 || { echo "FAIL $w"; tail -20 gpurun_out/${TAG}_$w.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/${TAG}_$w.log') if l.startswith('{')][0]); print('$w', '%.4g evals/s' % d['value'], '%.3f ms/step' % d['ms_per_step'], 'cpu %.4g' % d['cpu_baseline']['value'], 'parity', d['parity_prefix']['status'], d['parity_prefix']['pairs_compared'], 'fb', d['config']['cpu_fallback_pairs_per_step'])"
done
