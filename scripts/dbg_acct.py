"""Debug: product vs host instantiation on the C5 PodSecurity rule with preconditions (which checks differ)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from kyverno_amd import synth, engine as E
pods, nsl = synth.pods(30_000, seed=42)
rs = E.Ruleset(synth.c5_policies(50))
b = E.Batch(rs, pods, nsl)
p1 = E.evaluate(rs, b, backend="gpu", jit=False)
c = E.evaluate(rs, b, backend="cpu")
d = np.nonzero(p1.raw != c.raw)
print("KYV_PSS_KERNEL", os.environ.get("KYV_PSS_KERNEL"), "differs", len(d[0]), sorted(set(d[0].tolist())))
from collections import Counter
cnt = Counter()
for k, r in list(zip(*d))[:3000]:
    g, h = p1.pss_mask(int(r), int(k)), c.pss_mask(int(r), int(k))
    cnt[(int(k), hex(g), hex(h), hex(g ^ h))] += 1
for x, n in cnt.most_common(12):
    print(x, n)
for k in sorted(set(d[0].tolist()))[:2]:
    r = int(d[1][d[0] == k][0])
    print("rule", k, rs.rules[k]["name"], "res", r, "doc", pods[r] if r < len(pods) else None)
