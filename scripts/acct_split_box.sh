#!/bin/bash
# GPU box: the C3 walk's algorithmic bytes by load kind (kyv_eval.h KYV_ACCT_SEL): one accounted bench per selection
set -o pipefail
mkdir -p gpurun_out/acct_split
for s in 0 1 2 12; do
  KYV_JIT_DEFS="-DKYV_ACCT_SEL=$s" timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-gather \
    > gpurun_out/acct_split/sel$s.log 2>&1 || { echo "FAIL sel$s"; tail -5 gpurun_out/acct_split/sel$s.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/acct_split/sel$s.log') if l.startswith('{')][0]); r=d['roofline']; print('sel $s', r['phase_alg_bytes'], r.get('alg_bytes_by_class'))"
done
