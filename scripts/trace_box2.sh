#!/bin/bash
# GPU box: rocprofv3 kernel trace (stats only) of one bench workload. Usage: bash scripts/trace_box2.sh <tag> <workload>
set -o pipefail
TAG=$1; WL=$2
R=$PWD
OUT=$R/gpurun_out/trace_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --workload $WL --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-account --no-serial --no-gather > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$OUT/run_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]: print("%-70s calls %6s avg_us %9.1f total_ms %8.2f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"])/1e3, float(r["TotalDurationNs"])/1e6))
PY
