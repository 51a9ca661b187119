"""Per-kernel ISA statistics of the evaluation kernels (CPU only: hipcc cross-compiles gfx950 device assembly).

  python scripts/isa_stats.py [filter] [source]   # every kernel of the source (default kyv_prod.hip; kyv_prod_j.hip:
                                                  # the JMESPath instantiations) whose mangled name contains filter

Prints, per kernel: VGPR / SGPR counts, private segment (scratch) bytes, spill counts, scratch instructions, calls
(s_swappc) and their targets. Used to find where a kernel's frame goes through scratch memory (round 5: C5's
match_deny_kernel wrote 0.86 GB of scratch per evaluation)."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "kyverno_amd", "csrc")


def compile_asm(src="kyv_prod.hip", out="/tmp/kyv_isa.s", defines=()):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--offload-device-only", "-S", "-O3", "-std=c++17",
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "-o", out, os.path.join(CSRC, src)] + ["-D" + d for d in defines]
    subprocess.check_call(cmd)
    return out


def stats(asm, filt=""):
    s = open(asm).read()
    rows = []
    for m in re.finditer(r"^(_Z\S+):", s, re.M):
        name = m.group(1)
        if filt not in name or "kernel" not in name:
            continue
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end]
        md = s[end:end + 4000]  # the per-function comment block after .Lfunc_end

        def mdv(key):
            r = re.search(r"; " + key + r":\s+(\d+)", md)
            return int(r.group(1)) if r else -1
        meta = s.find(".name:           " + name + "\n")
        yml = s[meta:meta + 1500] if meta > 0 else ""

        def ymv(key):
            r = re.search(r"\." + key + r":\s+(\d+)", yml)
            return int(r.group(1)) if r else -1
        calls = collections.Counter(re.findall(r"s_add_u32\s+s\d+,\s+s\d+,\s+(\S+)@rel32@lo", body))
        calls.pop(".str", None)
        rows.append((name, mdv("NumVgprs"), mdv("TotalNumSgprs"), mdv("ScratchSize"),
                     ymv("vgpr_spill_count"), ymv("sgpr_spill_count"), body.count("scratch_"), body.count("s_swappc"),
                     dict(calls.most_common(4))))
    return rows


if __name__ == "__main__":
    filt = sys.argv[1] if len(sys.argv) > 1 else ""
    src = sys.argv[2] if len(sys.argv) > 2 else "kyv_prod.hip"
    asm = "/tmp/kyv_isa.s" if os.environ.get("KYV_ISA_REUSE") else compile_asm(src)
    for r in stats(asm, filt):
        print("%s\n   vgpr %d sgpr %d private %d spill v%d s%d scratch-ops %d calls %d %s" % r)
