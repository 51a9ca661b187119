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

HOST_SRCS = ["pjson.cpp", "compiler.cpp", "batch.cpp", "capi.cpp", "jit.cpp", "pss_msg.cpp", "typed.cpp", "regex.cpp"]
HIP_SRCS = ["kyv_prod_j.hip", "kyv_acct_j.hip", "kyv_prod.hip", "kyv_acct.hip", "kyv_engine.hip"]
HEADERS = ["kyv_layout.h", "kyv_eval.h", "kyv_cond.h", "kyv_pss.h", "kyv_host.h", "pjson.h", "kyv_wave.h", "kyv_walk.h", "kyv_jcond.h", "kyv_kernels.h", "kyv_acct.h", "kyv_fused.h", "k8s_types.h", "kyv_launch.inc"]
COMMON = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-value", "-Wno-unused-function", "-Wno-unused-variable",
          "-Wno-unused-but-set-variable", "-I" + os.path.join(ROOT, "include")]


def _deps(path, seen=None):
    """path and every local header it includes, transitively (#include "..." resolved in csrc/ or include/): a source
    is rebuilt only when something it actually includes changed (the kernels' translation units take minutes)"""
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path, errors="replace") as f:
        for line in f:
            t = line.strip()
            if t.startswith("#include") and '"' in t:
                name = t.split('"')[1]
                for d in (os.path.dirname(path), CSRC, os.path.join(ROOT, "include")):
                    q = os.path.join(d, name)
                    if os.path.exists(q):
                        _deps(q, seen)
                        break
    return seen


def _needs(obj, src):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in _deps(src))


def _compile(src, obj_dir=OBJ, defines=(), host_flags=()):
    path = os.path.join(CSRC, src)
    obj = os.path.join(obj_dir, src + ".o")
    if not _needs(obj, path):
        return obj
    cmd = [HIPCC] + COMMON + ["-D" + d for d in defines]
    if src.endswith(".hip"):
        cmd += ["--offload-arch=" + ARCH, "-x", "hip"]
        for f in host_flags:  # host-side only (sanitizers): never applied to the device code
            cmd += ["-Xarch_host", f]
    else:
        cmd += list(host_flags) + (["-fno-gpu-sanitize"] if host_flags else [])
    cmd += ["-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s" % (" ".join(cmd), r.stderr[-6000:]))
    return obj


def build(verbose=False, lib=LIB, defines=(), obj_dir=OBJ, host_flags=(), link_flags=()):
    """Build the library; `defines`/`lib`/`obj_dir` are for kernel-variant experiments (scripts/build_variants.py),
    `host_flags`/`link_flags` for the host-sanitizer build (scripts/host_sanitize.sh)."""
    os.makedirs(obj_dir, exist_ok=True)
    srcs = HOST_SRCS + HIP_SRCS
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, obj_dir, defines, host_flags), srcs))
    if not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs + list(link_flags) + \
              ["-lpthread", "-L/opt/rocm/lib", "-lhiprtc", "-lrccl", "-ldl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed: %s\n%s" % (" ".join(cmd), r.stderr[-4000:]))
    if verbose:
        print("built", lib)
    return lib


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
