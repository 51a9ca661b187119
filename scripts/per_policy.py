"""Diagnostics (GPU box): kernel time per policy of the C3 set on one synthetic corpus.

  python scripts/per_policy.py [resources]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kyverno_amd import engine as E  # noqa: E402
from kyverno_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300000
pols = bench.load_policies("c3")
data, nsl = synth.cached_corpus(n, kind="mixed", seed=bench.SEED)
tot = 0.0
for p in pols:
    rs = E.Ruleset([p])
    b = E.Batch(rs, data, nsl)
    E.evaluate(rs, b, backend="gpu", copy_back=False)
    r = E.evaluate(rs, b, backend="gpu", iterations=3, copy_back=False)
    walked = r.counts["pass"] + r.counts["fail"] + r.counts["skip"] + r.counts["error"]
    tot += r.kernel_ms
    print("%-45s rules %2d kinds %-22s kernel %7.3f ms  walked %8d  ns/walked %.3f" % (
        p["metadata"]["name"], len(rs.rules), ",".join(sorted(set(x["kind"] for x in rs.rules))), r.kernel_ms, walked,
        r.kernel_ms * 1e6 / max(1, walked)), flush=True)
print("sum of per-policy kernels %.3f ms" % tot)
