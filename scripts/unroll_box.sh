#!/bin/bash
# GPU box: C3 condition-kernel loop unrolling A/B (KYV_JC_UNROLL), evaluation phases per variant
set -o pipefail
mkdir -p gpurun_out/ab
for u in 1 2; do
  KYV_JIT_DEFS="-DKYV_JC_UNROLL=_Pragma(\"unroll $u\")" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-account \
    > gpurun_out/ab/u$u.log 2>&1 || { echo "FAIL u$u"; tail -5 gpurun_out/ab/u$u.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab/u$u.log') if l.startswith('{')][0]); print('u$u eval %.3f ms value %.4g phases %s' % (d['roofline']['evaluation_ms'], d['value'], {k: round(x, 3) for k, x in d['roofline']['phase_ms'].items()}))"
done
