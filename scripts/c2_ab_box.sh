#!/bin/bash
# GPU box: C2 timing of the in-tree library against an alternative build (KYV_LIB), alternating, twice each.
# Usage: bash scripts/c2_ab_box.sh <alt lib path>
set -o pipefail
mkdir -p gpurun_out/ab
export KYV_CORPUS_CACHE=/tmp/kc2
for i in 1 2; do
  for n in new old; do
    if [ $n = old ]; then L="KYV_LIB=$1"; else L="KYV_X=0"; fi
    env $L timeout -k 10 200 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-account > gpurun_out/ab/c2_${n}_$i.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/ab/c2_${n}_$i.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/ab/c2_${n}_$i.log') if l.startswith('{')][0]); print('%-4s %d eval %.4f ms phases %s' % ('$n', $i, d['roofline']['evaluation_ms'], {k: round(x, 4) for k, x in d['roofline']['phase_ms'].items()}))"
  done
done
