#!/bin/bash
# GPU box: per-rule walk kernel times (KYV_JIT_GROUP=1: one kernel per compiled pattern rule) from a rocprofv3 kernel trace.
set -o pipefail
mkdir -p gpurun_out/split
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
KYV_JIT_GROUP=1 KYV_JIT_DEFS="-DKYV_JIT_NOEXTRA -DKYV_JIT_WPE=8" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/split -o run -- python3 $R/bench.py --resources 1250000 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/split/bench.log 2>&1 || { tail -20 $R/gpurun_out/split/bench.log; exit 1; }
echo done
