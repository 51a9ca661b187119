#!/bin/bash
# GPU box (round 5 diagnostic): round-4 source (exp_build/wt4) with diagnostic hashes of the container-list, port-list,
# port-entry and capability-entry loads folded into mask bits 21..31; inlined (inld) vs out of line (oold).
set -o pipefail
mkdir -p gpurun_out
cd exp_build/wt4
for v in oold inld; do
  KYV_LIB=exp_build/$v/libkyvgpu.so timeout -k 10 300 python -u scripts/dbg_pss_guard.py > ../../gpurun_out/r5c_pss4_$v.log 2>&1 || { echo "FAIL $v"; tail -20 ../../gpurun_out/r5c_pss4_$v.log; exit 1; }
  cat ../../gpurun_out/r5c_pss4_$v.log
done
