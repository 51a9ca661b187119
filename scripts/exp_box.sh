#!/bin/bash
# GPU box: time kernel variants (exp_build/<name>/libkyvgpu.so) against the in-tree library.
# Usage: [BARGS="--workload c2"] bash scripts/exp_box.sh name...
set -o pipefail
mkdir -p gpurun_out/exp
for n in base "$@"; do
  if [ "$n" = base ]; then L=""; else L=$PWD/exp_build/$n/libkyvgpu.so; fi
  KYV_LIB=$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e $BARGS > gpurun_out/exp/$n.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/exp/$n.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/exp/$n.log') if l.startswith('{')][0]); print('%-12s kernel %.3f ms  value %.4g  verdicts %s' % ('$n', d['roofline']['kernel_ms'], d['value'], d['verdicts']))"
done
