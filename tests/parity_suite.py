"""Parity corpora run through libkyvgpu for a given backend and checked against the oracle (shared by
test_cpu_backend_parity.py and test_gpu_parity.py)."""
import cases
import parity_util as PU


def assert_clean(name, st):
    assert st["nbad"] == 0, "%s: %d mismatches, first: %r" % (name, st["nbad"], st["bad"][:5])


def run_engine_goldens(backend):
    n = 0
    for i, (pols, res) in enumerate(cases.engine_cases()):
        st, _ = PU.compare(pols, res, None, backend=backend)
        assert_clean("engine[%d]" % i, st)
        n += st["compared"]
    return n


def run_cli_goldens(backend):
    n = 0
    for d, pols, res in cases.cli_cases():
        st, _ = PU.compare(pols, res, None, backend=backend)
        assert_clean("cli/" + d, st)
        n += st["compared"]
    return n


def run_walk_goldens(backend):
    pols, res = cases.walk_policy_cases()
    n = 0
    for i in range(len(pols)):
        st, _ = PU.compare([pols[i]], [res[i]], None, backend=backend)
        assert_clean("walk[%d]" % i, st)
        n += st["compared"]
    return n


def run_pss_goldens(backend):
    """pkg/pss/evaluate_test.go: device verdict must equal the oracle's and the reference's `allowed`."""
    n = 0
    for name, pol, pod, allowed in cases.pss_cases():
        st, res = PU.compare([pol], [pod], None, backend=backend)
        assert_clean("pss/" + name, st)
        s = int(res.status[0, 0])
        if s in (PU.K.ST_PASS, PU.K.ST_FAIL):
            assert (s == PU.K.ST_PASS) == allowed, name
        n += st["compared"]
    return n


def run_synthetic(backend, policies, n, seed, kind="mixed", edge=True, jit=None):
    from kyverno_amd import synth
    docs, nsl = (synth.mixed if kind == "mixed" else synth.pods)(n, seed=seed, edge=edge)
    st, res = PU.compare(policies, docs, nsl, backend=backend, jit=jit)
    assert_clean("synthetic/%s/%d" % (kind, seed), st)
    return st, res


def run_merged(backend, groups, name, jit=None):
    """All (policies, resources) groups of a golden corpus as ONE ruleset over ONE batch (policy names prefixed
    per group so they stay distinct): every policy meets every resource, and a runtime-compiled walk kernel is
    compiled once for the whole corpus."""
    import copy
    pols, res = [], []
    for gi, (ps, rs_) in enumerate(groups):
        for p in ps:
            q = copy.deepcopy(p)
            q.setdefault("metadata", {})["name"] = "g%d-%s" % (gi, q.get("metadata", {}).get("name", ""))
            pols.append(q)
        res.extend(rs_)
    st, r = PU.compare(pols, res, None, backend=backend, jit=jit)
    assert_clean(name, st)
    return st, r


def golden_groups():
    """engine + cli + walk golden corpora as (policies, resources) groups"""
    groups = [(p, r) for p, r in cases.engine_cases()]
    groups += [(p, r) for _, p, r in cases.cli_cases()]
    wp, wr = cases.walk_policy_cases()
    groups += [([wp[i]], [wr[i]]) for i in range(len(wp))]
    return groups


def run_c4(backend, npol, nres, seed=11, jit=None):
    """BASELINE configs[3] (C4): generated wildcard-heavy match/exclude policies over mixed resources,
    status parity on every pair against the oracle's verdict matrix."""
    from kyverno_amd import synth
    pols = synth.c4_policies(npol)
    docs, nsl = synth.mixed(nres, seed=seed, edge=True)
    st, res = PU.compare_matrix(pols, docs, nsl, backend=backend, jit=jit)
    assert_clean("c4/%dx%d" % (npol, nres), st)
    assert st["matched"] > 0
    return st, res


def run_condition_goldens(backend):
    """pkg/engine/variables/evaluate_test.go TestEvaluate through the device evaluator: every golden condition
    becomes a deny rule over one Pod (deny true -> fail, false -> pass); the verdict must equal the golden result
    (and the oracle). Map literals are compiled to CPU fallback and are skipped."""
    import json
    from kyverno_amd import _lib as K
    recs = cases.load("conditions.json")
    pols = []
    for i, r in enumerate(recs):
        cond = {"key": json.loads(r["key"]), "operator": r["operator"], "value": json.loads(r["value"])}
        pols.append({"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "cond-%03d" % i, "annotations": {"pod-policies.kyverno.io/autogen-controllers": "none"}},
                     "spec": {"rules": [{"name": "c", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                                         "validate": {"deny": {"conditions": {"all": [cond]}}}}]}})
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "default"},
           "spec": {"containers": [{"name": "c", "image": "nginx"}]}}
    st, res = PU.compare(pols, [pod], None, backend=backend)
    assert_clean("conditions", st)
    n = 0
    for k, rule in enumerate(res.ruleset.rules):
        s = int(res.status[k, 0])
        if s == K.ST_FALLBACK:
            continue
        i = int(res.ruleset.policies[rule["policy"]]["name"].split("-")[1])
        assert s == (K.ST_FAIL if recs[i]["result"] else K.ST_PASS), (recs[i], K.STATUS_NAMES[s])
        n += 1
    return n
