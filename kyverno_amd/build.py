"""Build libkyvgpu.so (the C-ABI library) in-tree with hipcc for gfx950.

python -m kyverno_amd.build   # or __graft_entry__.build()
"""
import concurrent.futures
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(HERE, "libkyvgpu.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KYV_OFFLOAD_ARCH", "gfx950")

HOST_SRCS = ["pjson.cpp", "compiler.cpp", "batch.cpp", "capi.cpp"]
HIP_SRCS = ["kyv_engine.hip"]
HEADERS = ["kyv_layout.h", "kyv_eval.h", "kyv_pss.h", "kyv_host.h", "pjson.h", "kyv_wave.h"]
COMMON = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-value", "-Wno-unused-function", "-Wno-unused-variable",
          "-Wno-unused-but-set-variable", "-I" + os.path.join(ROOT, "include")]


def _needs(obj, src):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [src] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "kyvgpu.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(src):
    path = os.path.join(CSRC, src)
    obj = os.path.join(OBJ, src + ".o")
    if not _needs(obj, path):
        return obj
    cmd = [HIPCC] + COMMON
    if src.endswith(".hip"):
        cmd += ["--offload-arch=" + ARCH, "-x", "hip"]
    cmd += ["-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s" % (" ".join(cmd), r.stderr[-6000:]))
    return obj


def build(verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    srcs = HOST_SRCS + HIP_SRCS
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs + ["-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed: %s\n%s" % (" ".join(cmd), r.stderr[-4000:]))
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
