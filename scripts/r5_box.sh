#!/bin/bash
# GPU box (round 5): the GPU test suite, then bench lines of the given workloads (accounting, CPU baseline and
# timed-batch parity on; no end-to-end leg for the non-headline configs).
# Usage: bash scripts/r5_box.sh <tag> [tests|notests] [workload...]
set -o pipefail
TAG=${1:-r5}; shift
MODE=${1:-tests}; shift
mkdir -p gpurun_out
if [ "$MODE" = tests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
for wl in "$@"; do
  extra="--no-e2e"
  [ "$wl" = c3 ] && extra=""
  timeout -k 10 700 python -u bench.py --workload $wl $extra > gpurun_out/${TAG}_${wl}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_${wl}_bench.log; exit 2; }
  grep -v "^{" gpurun_out/${TAG}_${wl}_bench.log | tail -4
  grep "^{" gpurun_out/${TAG}_${wl}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; p=d.get('parity_prefix') or {}; print('$wl', 'value %.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'phase_ms', {k: round(v,3) for k,v in r['phase_ms'].items()}, 'frac %.3f' % r['frac'], 'valid', r['valid'], 'parity', p.get('status'), (p.get('timed_batch') or {}).get('mismatches'))"
done
