#!/bin/bash
# GPU box: profiles of two workloads back to back. Usage: bash scripts/prof2_box.sh <tag1> <workload1> <tag2> <workload2>
set -o pipefail
bash scripts/profile_box.sh $1 --workload $2 || exit 1
bash scripts/profile_box.sh $3 --workload $4 || exit 2
echo done
