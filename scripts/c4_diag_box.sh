#!/bin/bash
# GPU box (round 5 diagnostics): C4 timing under generator / kernel knobs, then instruction-mix and wait counters
# of the match kernels (one rocprofv3 --pmc pass each).
set -o pipefail
TAG=${1:-c4d}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export KYV_CORPUS_CACHE=/tmp/kyv_corpus_$TAG
B="--workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-account --no-gather"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -u $R/bench.py $B > $OUT/$n.log 2>&1 || { echo "FAIL $n"; tail -5 $OUT/$n.log; exit 1; }
  grep "^{" $OUT/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n', 'ms/step %.2f' % d['ms_per_step'], {k: round(v,2) for k,v in r['phase_ms'].items()})"
}
run base KYV_X=0
#run notail KYV_TAIL_FACTS=0
run wpe5 KYV_MATCHW_WPE=5

cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LEVEL_WAVES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-account --no-serial --no-gather > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 2; }
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(out + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    if "rocclr" in k or "match" not in k: continue
    print("%-40s %-24s %.4g" % (k[-40:], c, sum(v) / len(v)))
PY
