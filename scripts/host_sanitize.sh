#!/bin/bash
# Host AddressSanitizer + UndefinedBehaviorSanitizer run of the C-ABI library (sanitizers on the CPU build).
# Builds exp_build/asan/libkyvgpu.so with the sanitizers on the HOST side only (each -fsanitize behind -Xarch_host for
# the .hip sources, -fno-gpu-sanitize for the host sources; the device code is untouched), then runs the CPU test
# suite against it: the flattener, the ruleset compiler, the host instantiation of the evaluator (backend="cpu": the
# same kyv_eval.h / kyv_pss.h / kyv_cond.h source the kernels run), messages and the C-ABI. Any ASan report or UBSan
# diagnostic aborts the test process (halt_on_error / -fno-sanitize-recover).
#
#   bash scripts/host_sanitize.sh            # build + the CPU suite (minutes)
#   bash scripts/host_sanitize.sh tests/test_flatten.py   # build + the given tests
# CPU only: never run on the GPU box.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
python - <<'PY'
import os, sys
sys.path.insert(0, os.getcwd())
from kyverno_amd import build as B
d = os.path.join(os.getcwd(), "exp_build", "asan")
B.build(verbose=True, lib=os.path.join(d, "libkyvgpu.so"), obj_dir=d,
        host_flags=["-fsanitize=address", "-fsanitize=undefined", "-fno-sanitize-recover=undefined",
                    "-fno-omit-frame-pointer", "-g1"],
        link_flags=["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-shared-libsan"])
PY
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
TESTS=${@:-tests}
export KYV_LIB="$ROOT/exp_build/asan/libkyvgpu.so"
export KYV_CSRC="$ROOT/kyverno_amd/csrc"  # headers of the runtime-compiled kernels
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$RT" python -m pytest -x -q -m "not gpu" -p no:cacheprovider $TESTS
