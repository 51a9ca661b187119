#!/bin/bash
# GPU box (round 5 diagnostic): the PodSecurity column checks inlined into eval_pss vs out of line, with and without
# the KYV_PSS_DBG_GUARD loop guards (scripts/dbg_pss_guard.py), product library as the control.
set -o pipefail
mkdir -p gpurun_out
for v in prod inl inlg oolg; do
  if [ $v = prod ]; then L=""; else L="exp_build/$v/libkyvgpu.so"; fi
  KYV_LIB=$L timeout -k 10 240 python -u scripts/dbg_pss_guard.py > gpurun_out/r5a_pss_$v.log 2>&1 || { echo "FAIL $v"; tail -20 gpurun_out/r5a_pss_$v.log; exit 1; }
  cat gpurun_out/r5a_pss_$v.log
done
