#!/bin/bash
# GPU box (round 6): optional GPU test subset / whole suite, then C3 environment A/B variants (scripts/env_ab.sh).
# Usage: bash scripts/r6_box.sh <tag> <pytest -k expr | all | none> [NAME:VAR=x,VAR2=y ...]
set -o pipefail
TAG=${1:-r6}; shift
SEL=${1:-none}; shift
mkdir -p gpurun_out
export KYV_CORPUS_CACHE=/tmp/kyv_corpus_$TAG
if [ "$SEL" != none ]; then
  K=""; [ "$SEL" != all ] && K="-k $SEL"
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread $K > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
[ $# -gt 0 ] && { bash scripts/env_ab.sh "$@" || exit 2; }
echo r6-done
