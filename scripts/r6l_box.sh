#!/bin/bash
# GPU box: final C2 line (accounting, CPU baseline, parity) and its profile
set -o pipefail
bash scripts/r5_box.sh r6l notests c2 || exit 1
bash scripts/profile_box.sh r6l_c2 --workload c2 || exit 2
echo done
