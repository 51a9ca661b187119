#!/bin/bash
# GPU box: list counters + SQ instruction-mix passes over the bench (diagnostics). Usage: bash scripts/sq_box.sh <tag>
set -o pipefail
TAG=${1:-sq}
R=$PWD
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
BARGS="--steps 2 --warmup 1 --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o run -- python3 $R/bench.py $BARGS > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d $OUT/p2 -o run -- python3 $R/bench.py $BARGS > $OUT/p2.log 2>&1 || exit 2
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_SENDMSG SQ_INSTS_VMEM SQ_LEVEL_WAVES --output-format csv -d $OUT/p3 -o run -- python3 $R/bench.py $BARGS > $OUT/p3.log 2>&1 || exit 3
echo done
