#!/bin/bash
# GPU box: C3 A/B of the per-rule View laundering (KYV_RULE_VIEW) in the runtime-compiled kernels
set -o pipefail
mkdir -p gpurun_out/ab
for v in launder plain; do
  if [ $v = plain ]; then export KYV_JIT_DEFS="-DKYV_RULE_VIEW(x)=(x)"; else unset KYV_JIT_DEFS; fi
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-account > gpurun_out/ab/rv_$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/ab/rv_$v.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab/rv_$v.log') if l.startswith('{')][0]); print('$v eval %.3f ms value %.4g phases %s' % (d['roofline']['evaluation_ms'], d['value'], {k: round(x, 3) for k, x in d['roofline']['phase_ms'].items()}))"
done
