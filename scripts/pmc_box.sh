#!/bin/bash
# GPU box: one rocprofv3 --pmc pass per argument (quoted counter list) over a short bench run.
# Usage: bash scripts/pmc_box.sh <tag> "CNT1 CNT2 ..." ["CNT3 ..."]
set -o pipefail
TAG=$1; shift
R=$PWD
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-account --no-serial > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(out + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    if "rocclr" in k: continue
    print("%-22s %-28s %.4g" % (k[-22:], c, sum(v) / len(v)))
PY
