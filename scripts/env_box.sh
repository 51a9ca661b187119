#!/bin/bash
# GPU box: bench under several environment settings. Usage: bash scripts/env_box.sh "VAR=a VAR2=b" "VAR=c" ...
set -o pipefail
mkdir -p gpurun_out/env
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/env/$i.log 2>&1 || { echo "FAIL $E"; tail -5 gpurun_out/env/$i.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/env/$i.log') if l.startswith('{')][0]); print('%-40s kernel %.3f ms  %.4g evals/s' % ('$E', d['roofline']['kernel_ms'], d['value']))"
done
