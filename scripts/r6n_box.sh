#!/bin/bash
# GPU box (round 6, final state after the PodSecurity changes): GPU test suite, smoke, C2 and C5 lines
set -o pipefail
TAG=${1:-r6n}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 2; }
tail -1 gpurun_out/${TAG}_smoke.log
bash scripts/r5_box.sh $TAG notests c2 c5 || exit 3
echo final-done
