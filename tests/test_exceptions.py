"""PolicyException match blocks compiled as device match programs (compiler.cpp compile_exc_block, RuleDesc.exc,
kyv_eval.h match_exception): after a rule matches, its exception candidates are checked in FindExceptions order
(pkg/engine/policyContext.go:150-169) with CheckMatchesResources semantics (pkg/utils/match/match.go:26-203), and
a pair an exception applies to is a skip with "rule skipped due to policy exception <key>" (validation.go:797-848).
Only the pairs an exception really matches change; every other pair of the rule is still decided on the device.

Pinned by the reference's kuttl fixtures (test/conformance/kuttl/reports/background/exception,
exceptions/allows-rejects-creation: the ConfigMap `emergency` is skipped, `foo` fails) and, at scale, by the oracle's
restatement of hasPolicyExceptions (oracle/oengine.cpp matching_exception)."""
import numpy as np
import pytest

import cases
from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from kyverno_amd import synth
from oracle import oracle as O
from parity_util import _MATRIX_TO_DEVICE

# kuttl fixtures (reports/background/exception/{policy,exception,configmap}.yaml and
# exceptions/allows-rejects-creation/configmap-rejected.yaml), as data
KUTTL_POLICY = {"apiVersion": "kyverno.io/v2beta1", "kind": "ClusterPolicy", "metadata": {"name": "require-labels"},
                "spec": {"validationFailureAction": "Enforce", "background": True, "rules": [{
                    "name": "require-team", "match": {"any": [{"resources": {"kinds": ["ConfigMap"]}}]},
                    "validate": {"message": "The label `team` is required.",
                                 "pattern": {"metadata": {"labels": {"team": "?*"}}}}}]}}
KUTTL_EXCEPTION = {"apiVersion": "kyverno.io/v2alpha1", "kind": "PolicyException", "metadata": {"name": "mynewpolex"},
                   "spec": {"exceptions": [{"policyName": "require-labels", "ruleNames": ["require-team"]}],
                            "match": {"any": [{"resources": {"kinds": ["ConfigMap"], "names": ["emergency"]}}]}}}


def _cm(name):
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name}}


@pytest.mark.parametrize("backend", ["cpu"])
def test_kuttl_background_exception_report(backend):
    """report-assert.yaml: require-labels / require-team -> skip for ConfigMap emergency; configmap-rejected.yaml: foo
    is still denied"""
    rs = E.Ruleset([KUTTL_POLICY], exceptions=[KUTTL_EXCEPTION])
    assert rs.rules[0]["kind"] == "pattern"  # the rule stays on the device
    res = E.evaluate(rs, E.Batch(rs, [_cm("emergency"), _cm("foo")]), backend=backend)
    assert list(res.status[0]) == [K.ST_SKIP, K.ST_FAIL]
    assert res.message(0, 0) == "rule skipped due to policy exception mynewpolex"
    assert res.message(1, 0).startswith("validation error: The label `team` is required.")
    o = O.validate([KUTTL_POLICY], _cm("emergency"), {}, exceptions=[KUTTL_EXCEPTION])
    assert o[0]["rules"][0]["status"] == "skip" and o[0]["rules"][0]["message"] == res.message(0, 0)


def _exc(name, targets, match, ns=None):
    meta = {"name": name}
    if ns:
        meta["namespace"] = ns
    by = {}
    for p, r in targets:
        by.setdefault(p, []).append(r)
    return {"apiVersion": "kyverno.io/v2alpha1", "kind": "PolicyException", "metadata": meta,
            "spec": {"exceptions": [{"policyName": p, "ruleNames": rn} for p, rn in by.items()], "match": match}}


def exception_suite(pols):
    """PolicyExceptions over the device rules of `pols`, each match shape of CheckMatchesResources: names / namespaces
    globs, label and namespace selectors, any vs all, an empty match (applies to everything), a statement with only
    user info (never satisfied without admission info), an empty statement (never matches), a kinds ["*"] statement
    with a namespace selector, a namespaced exception key, and two exceptions on one rule (the first one wins)"""
    rs = E.Ruleset(pols)
    keys = [(rs.policies[r["policy"]]["name"], r["name"]) for r in rs.rules if r["kind"] != "fallback"]
    assert len(keys) >= 8
    t = lambda *i: [keys[j % len(keys)] for j in i]
    return [
        _exc("by-name", t(0, 1), {"any": [{"resources": {"kinds": ["Pod", "Deployment"], "names": ["pod-00000[1-3]*", "*-0000004"]}}]}),
        _exc("by-name-glob", t(0, 2), {"any": [{"resources": {"names": ["*1?"]}}]}),
        _exc("by-ns", t(3), {"any": [{"resources": {"namespaces": ["ns-00*", "ns-09?1"]}}]}, ns="kyverno"),
        _exc("by-selector", t(4, 5), {"any": [{"resources": {"selector": {"matchLabels": {"tier": "data"}}}}]}),
        _exc("by-all", t(6, 0), {"all": [{"resources": {"kinds": ["*"]}},
                                      {"resources": {"selector": {"matchExpressions": [
                                          {"key": "owner", "operator": "Exists"}]}}}]}),
        _exc("everything", t(7), {}),
        _exc("userinfo-only", t(1, 8), {"any": [{"roles": ["admin"]}]}),
        _exc("empty-statement", t(9), {"any": [{"resources": {}}]}),
        _exc("star-nssel", t(10, 2), {"any": [{"resources": {"kinds": ["*"], "namespaceSelector": {
            "matchLabels": {"env": "prod"}}}}]}),
        _exc("annotations", t(11), {"any": [{"resources": {"annotations": {"*": "*"}}}]}),
    ]


def _run(pols, docs, nsl, backend, jit=None):
    exc = exception_suite(pols)
    rs = E.Ruleset(pols, exceptions=exc, background=True)  # the oracle runs background-scan semantics
    b = E.Batch(rs, docs, nsl)
    res = E.evaluate(rs, b, backend=backend, **({"jit": jit} if backend == "gpu" else {}))
    names, m, tx = O.validate_matrix(pols, docs, nsl, threads=8, texts=("skip", "fail"), exceptions=exc)
    row = {nm: i for i, nm in enumerate(names)}
    lut = np.array([_MATRIX_TO_DEVICE[i] for i in range(8)], dtype=np.uint8)
    st = np.asarray(res.status)
    n = {"exc_skip": 0, "compared": 0, "bad": 0, "msg": 0}
    bad = []
    for k, rule in enumerate(rs.rules):
        key = (rs.policies[rule["policy"]]["name"], rule["name"])
        want = lut[m[row[key]]] if key in row else np.zeros(len(docs), np.uint8)
        got = st[k, : len(docs)]
        ok = want == got  # an ND pair must be ND on both sides
        n["compared"] += int(ok.size)
        for ri in np.nonzero(~ok)[0][:3]:
            bad.append((key, int(ri), K.STATUS_NAMES[got[ri]], K.STATUS_NAMES[want[ri]]))
        n["bad"] += int((~ok).sum())
        skips = np.nonzero(got == K.ST_SKIP)[0]
        if len(skips):
            msgs = res.texts(k, "message", (K.ST_SKIP,), res0=0, nres=len(docs))
            for ri in skips.tolist():
                o = tx.get((row[key], ri))
                if msgs[ri] is not None and msgs[ri].startswith(b"rule skipped due to policy exception"):
                    n["exc_skip"] += 1
                    if o is None or msgs[ri] != o[1]:
                        n["msg"] += 1
                        if len(bad) < 20:
                            bad.append(("message", key, ri, msgs[ri], o and o[1]))
    return n, bad, rs, res


def test_userinfo_exception_needs_background_flag():
    """an exception keyed on roles / clusterRoles / subjects depends on the admission request (checkUserInfo,
    pkg/utils/match/match.go:110-150): an admission-capable ruleset hands the rules it names to the CPU engine; a
    background-only ruleset (empty AdmissionInfo) compiles it as never matching"""
    pols = cases.best_practices()
    exc = exception_suite(pols)
    named = {(pn, rn) for e in exc for x in e["spec"]["exceptions"] for rn in x["ruleNames"] for pn in [x["policyName"]]
             if any(f.get("roles") for f in (e["spec"]["match"].get("any") or []))}
    assert named
    adm = E.Ruleset(pols, exceptions=exc)
    bg = E.Ruleset(pols, exceptions=exc, background=True)
    for rs, want_fb in ((adm, True), (bg, False)):
        for r in rs.rules:
            key = (rs.policies[r["policy"]]["name"], r["name"])
            if key in named:
                assert (r["kind"] == "fallback" and r["reason"].startswith("exception: userInfo")) == want_fb, (key, r)


def test_exceptions_cpu_vs_oracle():
    pols = cases.best_practices()
    docs, nsl = synth.mixed(2000, seed=81, edge=True)
    n, bad, rs, _ = _run(pols, docs, nsl, "cpu")
    print(n)
    assert n["bad"] == 0 and n["msg"] == 0, bad
    assert n["exc_skip"] > 300
    assert not any(r["kind"] == "fallback" and r["reason"] == "exception" for r in rs.rules)


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [False, True])
def test_exceptions_gpu_vs_oracle(jit):
    """the device match programs of the exceptions, through the match kernel and (jit) the runtime-compiled
    condition / walk kernels, against the oracle on every pair"""
    pols = cases.best_practices()
    docs, nsl = synth.mixed(20000, seed=82, edge=True)
    n, bad, rs, res = _run(pols, docs, nsl, "gpu", jit=jit)
    print(n)
    assert n["bad"] == 0 and n["msg"] == 0, bad
    assert n["exc_skip"] > 3000
    if jit:
        assert res.jit
