#!/bin/bash
# GPU box (round 6, late): the GPU test suite, smoke, then the default C3 bench line
set -o pipefail
TAG=${1:-r6e}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 2; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_c3_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_c3_bench.log; exit 3; }
grep '^{' gpurun_out/${TAG}_c3_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print('value %.4g ms/step %.3f frac %.3f eval %.3f phases %s' % (d['value'], d['ms_per_step'], r['frac'], r['evaluation_ms'], {k: round(x, 3) for k, x in r['phase_ms'].items()}))"
