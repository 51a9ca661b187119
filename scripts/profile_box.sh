#!/bin/bash
# Run on the GPU box (via gpurun): kernel-trace stats + separate PMC passes of the bench workload.
# Usage: bash scripts/profile_box.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r1}; shift
R=$PWD
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
BARGS="--steps 5 --warmup 1 --no-cpu-baseline $*"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $BARGS > $OUT/bench_trace.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $BARGS > $OUT/pmc_fetch.log 2>&1 || exit 2
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $BARGS > $OUT/pmc_write.log 2>&1 || exit 3
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq -o run -- python3 $R/bench.py $BARGS > $OUT/pmc_sq.log 2>&1 || exit 4
echo done
