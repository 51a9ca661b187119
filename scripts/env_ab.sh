#!/bin/bash
# GPU box: time the in-tree library under environment variants. Usage: bash scripts/env_ab.sh "NAME:VAR=x,VAR2=y" ...
set -o pipefail
mkdir -p gpurun_out/ab
for spec in "$@"; do
  n=${spec%%:*}; vars=${spec#*:}
  env_args=$(echo "$vars" | tr ',' ' ')
  env $env_args timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e $BENCH_ARGS > gpurun_out/ab/$n.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/ab/$n.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab/$n.log') if l.startswith('{')][0]); print('%-14s eval %.3f ms value %.4g fb %d phases %s' % ('$n', d['roofline']['evaluation_ms'], d['value'], d['config'].get('cpu_fallback_pairs_per_step', -1), {k: round(x, 3) for k, x in d['roofline']['phase_ms'].items()}))"
done
