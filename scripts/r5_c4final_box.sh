#!/bin/bash
# GPU box (round 5): the final C4 line + profile, then C3 with the condition kernels on the evaluation stream
# (KYV_COND_STREAM=0) against the default concurrent stream.
set -o pipefail
TAG=${1:-r5z}
mkdir -p gpurun_out
bash scripts/r5_final_box.sh $TAG c4 || exit 2
export KYV_CORPUS_CACHE=/tmp/kyv_corpus_c3
for cs in 1 0; do
  KYV_COND_STREAM=$cs timeout -k 10 400 python -u bench.py --steps 20 --no-e2e --no-cpu-baseline --no-account > gpurun_out/${TAG}_c3_cs$cs.log 2>&1 || { tail -30 gpurun_out/${TAG}_c3_cs$cs.log; exit 3; }
  grep "^{" gpurun_out/${TAG}_c3_cs$cs.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 cond_stream=$cs', d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d['roofline']['phase_ms'].items()})"
done
echo all-done
