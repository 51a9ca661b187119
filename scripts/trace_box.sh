#!/bin/bash
# GPU box: kernel-trace stats of a short bench run. Usage: bash scripts/trace_box.sh <tag> [bench args]
set -o pipefail
TAG=${1:-t}; shift
R=$PWD
mkdir -p $R/gpurun_out/trace_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/gpurun_out/trace_$TAG/log.txt 2>&1 || exit 1
cat $R/gpurun_out/trace_$TAG/run_kernel_stats.csv | cut -c1-160
