"""Compile a workload's generated kernel source with hipcc (same options as the hipRTC path) and print each kernel's
register / scratch metadata. Experiments only: the environment selects generator knobs (KYV_JC_INLINE, KYV_JIT_ONLY_COND ...).

  python scripts/jit_meta.py [c3|c2|c4|c5] [extra -D defines...]
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kyverno_amd import engine as E  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
rs = E.Ruleset(bench.load_policies(wl))
src = rs.jit_source()[0]
d = tempfile.mkdtemp()
f = os.path.join(d, "k.hip")
open(f, "w").write(src)
co = os.path.join(d, "k.co")
cmd = ["/opt/rocm/lib/llvm/bin/clang++", "-x", "hip", "--offload-arch=gfx950", "--offload-device-only", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "kyverno_amd", "csrc"),
       "-I" + os.path.join(ROOT, "include"), "-DKYV_JIT_WPE=" + os.environ.get("KYV_JIT_WPE", "4"), "-DKYV_JIT_NOEXTRA"] + sys.argv[2:] + [f, "-o", co]
if os.environ.get("JIT_META_ASM"):  # also write the device assembly there
    subprocess.run([c for c in cmd if c not in ("-o", co)][:-1] + ["-S", f, "-o", os.environ["JIT_META_ASM"]], check=True)
r = subprocess.run(cmd, capture_output=True, text=True)
if r.returncode:
    print(r.stderr[-3000:])
    sys.exit(1)
elf = os.path.join(d, "k.elf")
subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                "--input=" + co, "--output=" + elf, "--unbundle"], check=True)
out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", elf], capture_output=True, text=True).stdout
keys = (".name:", "private_segment_fixed_size", ".vgpr_count", ".sgpr_count", "vgpr_spill", "sgpr_spill")
for line in out.splitlines():
    if any(k in line for k in keys):
        print(line.strip())
