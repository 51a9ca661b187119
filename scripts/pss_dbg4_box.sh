#!/bin/bash
# GPU box (round 5 diagnostic): the round-4 source (worktree exp_build/wt4 at e8c1f4d) with the PodSecurity column
# checks inlined into eval_pss, with and without loop guards, vs its product library.
set -o pipefail
mkdir -p gpurun_out
cd exp_build/wt4
for v in prod inl inlg; do
  if [ $v = prod ]; then L=""; else L="exp_build/$v/libkyvgpu.so"; fi
  KYV_LIB=$L DBG_JIT=1 timeout -k 10 300 python -u scripts/dbg_pss_guard.py > ../../gpurun_out/r5b_pss4_$v.log 2>&1 || { echo "FAIL $v"; tail -20 ../../gpurun_out/r5b_pss4_$v.log; exit 1; }
  cat ../../gpurun_out/r5b_pss4_$v.log
done
