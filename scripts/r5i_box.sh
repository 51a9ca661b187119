#!/bin/bash
# GPU box (round 5, last check): the GPU suite, smoke(), then C5 with the facts table skipped for few records
# (default) and forced (KYV_FACTS_MIN=0).
set -o pipefail
TAG=${1:-r5i}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 2; }
tail -1 gpurun_out/${TAG}_smoke.log
for fm in 64 0; do
  KYV_FACTS_MIN=$fm timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --no-e2e --no-cpu-baseline --no-account > gpurun_out/${TAG}_c5_fm$fm.log 2>&1 || { tail -30 gpurun_out/${TAG}_c5_fm$fm.log; exit 3; }
  grep "^{" gpurun_out/${TAG}_c5_fm$fm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 facts_min=$fm', d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d['roofline']['phase_ms'].items()})"
done
echo all-done
