#!/bin/bash
# GPU box: the GPU test suite, then short benches. Usage: bash scripts/tests_c4_box.sh <tag> [workloads...] (default c4 c2)
set -o pipefail
TAG=$1; shift
WL=${*:-c4 c2}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for w in $WL; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-account > gpurun_out/${TAG}_$w.log 2>&1 || { tail -10 gpurun_out/${TAG}_$w.log; exit 2; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/${TAG}_$w.log') if l.startswith('{')][0]); print('$w', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in d['roofline']['phase_ms'].items()})"
done
