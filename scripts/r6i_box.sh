#!/bin/bash
# GPU box: C3 quick line, then a kernel trace of C3 (per-kernel times)
set -o pipefail
BENCH_ARGS="--no-account" bash scripts/env_ab.sh "c3:KYV_COLCACHE=4" || exit 1
bash scripts/trace_box2.sh r6i_c3 c3 || exit 2
