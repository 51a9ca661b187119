"""Debug: device vs host instantiation of the PodSecurity rules of C5 policy c5-006 (baseline, with preconditions)."""
import sys, os, copy
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from kyverno_amd import synth, engine as E, _lib as K
data, nsl = synth.corpus_ndjson(20000, seed=54, edge=True)
base = [p for p in synth.c5_policies(50) if p['metadata']['name'] == "c5-006"]
nopre = copy.deepcopy(base)
del nopre[0]["spec"]["rules"][0]["preconditions"]
restr = copy.deepcopy(base)
restr[0]["spec"]["rules"][0]["validate"]["podSecurity"]["level"] = "restricted"
for name, pols in (("c5-006", base), ("no-pre", nopre), ("restricted+pre", restr)):
    rs = E.Ruleset(pols)
    b = E.Batch(rs, data, nsl)
    g = E.evaluate(rs, b, backend="gpu", jit=False)
    c = E.evaluate(rs, b, backend="cpu")
    d = np.nonzero(np.asarray(g.status) != np.asarray(c.status))
    print(name, os.environ.get("KYV_PSS_NOCOLS"), "mismatches", len(d[0]))
    for k, r in list(zip(*d))[:2]:
        print("  rule", k, "res", r, "gpu", int(g.status[k, r]), hex(g.pss_mask(int(r), int(k))), "cpu", int(c.status[k, r]), hex(c.pss_mask(int(r), int(k))))
