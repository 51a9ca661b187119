"""Diagnostic (round 5): C5 over 30 k Pods on the device vs the host instantiation of the same evaluator, for the
library named by KYV_LIB (kernel-variant builds of scripts/build_variants.py): verdict mismatches, and how many
device PodSecurity masks carry the KYV_PSS_DBG_GUARD bits (30: a sub-array loop iteration beyond its lane's trip
count, 31: an iteration on a lane whose guard condition is false; both: the container loop)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collections import Counter  # noqa: E402
import numpy as np  # noqa: E402
from kyverno_amd import synth, engine as E  # noqa: E402

pods, nsl = synth.pods(30_000, seed=42)
rs = E.Ruleset(synth.c5_policies(50))
b = E.Batch(rs, pods, nsl)
c = E.evaluate(rs, b, backend="cpu")
for jit in ((False, True) if os.environ.get("DBG_JIT") else (False,)):
    g = E.evaluate(rs, b, backend="gpu", jit=jit)
    d = np.nonzero(np.asarray(g.raw) != np.asarray(c.raw))
    pss_rules = [k for k, r in enumerate(rs.rules) if r["kind"] == "podSecurity"]
    bits = Counter()
    xor = Counter()
    for k in pss_rules:
        for r in range(b.n):
            m = g.pss_mask(r, k)
            if m >> 30:
                bits[(k, m >> 30)] += 1
    for k, r in list(zip(*d))[:4000]:
        gm, hm = g.pss_mask(int(r), int(k)), c.pss_mask(int(r), int(k))
        xor[(int(k), hex(gm ^ hm))] += 1
    print("KYV_LIB=%s jit=%s mismatches=%d rules=%s" % (os.environ.get("KYV_LIB"), jit, len(d[0]),
                                                      sorted(set(d[0].tolist()))[:8]))
    print("  guard bits (rule, bits>>30): %s" % dict(bits.most_common(8)))
    print("  mask xor (rule, xor): %s" % dict(xor.most_common(8)))
