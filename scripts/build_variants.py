"""Build kernel-variant libraries for timing experiments: exp_build/<name>/libkyvgpu.so with extra -D flags.

  python scripts/build_variants.py name=DEF1,DEF2 [name2=...]

Run one on the GPU box with KYV_LIB=exp_build/<name>/libkyvgpu.so python bench.py ... (experiments only; the
variants skip work, so their verdicts are not valid and they are never the bench or test library).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kyverno_amd import build as B  # noqa: E402

for arg in sys.argv[1:]:
    name, _, defs = arg.partition("=")
    d = os.path.join(ROOT, "exp_build", name)
    B.build(verbose=True, lib=os.path.join(d, "libkyvgpu.so"), defines=[x for x in defs.split(",") if x], obj_dir=d)
