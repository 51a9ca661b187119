#!/bin/bash
# GPU box: profiles of several workloads back to back. Usage: bash scripts/prof2_box.sh <tag1> <workload1> [<tag2> <workload2> ...]
set -o pipefail
i=1
while [ $# -ge 2 ]; do
  bash scripts/profile_box.sh $1 --workload $2 || exit $i
  shift 2
  i=$((i + 1))
done
echo done
