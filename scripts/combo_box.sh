#!/bin/bash
# GPU box: GPU tests, then C2 new-vs-alt library A/B, then C5 with / without the deny kernel.
# Usage: bash scripts/combo_box.sh <tag> <alt lib>
set -o pipefail
TAG=$1
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
bash scripts/c2_ab_box.sh $2 || exit 2
export KYV_CORPUS_CACHE=/tmp/kc5
for n in d1 d0 d1b; do
  if [ $n = d0 ]; then E="KYV_DENY_KERNEL=0"; else E="KYV_X=0"; fi
  env $E timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-account > gpurun_out/ab/c5_$n.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/ab/c5_$n.log; exit 3; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab/c5_$n.log') if l.startswith('{')][0]); print('c5 %-4s eval %.4f ms value %.4g phases %s' % ('$n', d['roofline']['evaluation_ms'], d['value'], {k: round(x, 4) for k, x in d['roofline']['phase_ms'].items()}))"
done
