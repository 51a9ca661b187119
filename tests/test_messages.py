"""RuleResponse.Message of pattern pairs the failure records cannot describe: skip pairs (PatternError.Error() of a
conditional / global anchor error), error pairs ("execution error: <err>") and anyPattern results with a path-less
failure ("rule <name>[<i>] failed: <err>"). The library renders them with a host walk of the one pair
(kyv_engine.hip pattern_error_text; pkg/engine/validation.go:618-758, pkg/engine/validate/validate.go:31-247,
pkg/engine/anchor/handlers.go, anchor/error.go); every rendered text is compared with the oracle's."""
import numpy as np
import pytest

import cases
from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from kyverno_amd import synth
from oracle import oracle as O


def anchor_policies():
    """conditional / global / negation / existence anchors, anyPattern, nested arrays, wildcard keys: shapes whose
    skip and error texts nest (conditional anchor inside array inside conditional anchor, multierr joins)"""
    def pol(name, rule):
        rule.setdefault("match", {"any": [{"resources": {"kinds": ["Pod"]}}]})
        return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
                "spec": {"rules": [dict(name="r", **rule)]}}
    return cases.quirk_policies() + [
        pol("cond-nested", {"validate": {"pattern": {"spec": {"(hostNetwork)": False, "containers": [
            {"(name)": "c?", "=(securityContext)": {"(runAsNonRoot)": True, "runAsUser": ">0"}}]}}}}),
        pol("cond-missing", {"validate": {"pattern": {"spec": {"(dnsPolicy)": "ClusterFirst", "containers": [
            {"name": "*"}]}}}}),
        pol("global-num", {"validate": {"pattern": {"spec": {"<(hostPID)": True, "containers": [{"image": "registry/*"}]}}}}),
        pol("cond-array-skip", {"validate": {"pattern": {"spec": {"containers": [
            {"(image)": "nginx*", "resources": {"limits": {"memory": "?*"}}}]}}}}),
        pol("star-missing", {"validate": {"message": "labels required", "pattern": {"metadata": {"labels": {"app": "*"}}}}}),
        pol("keys-missing", {"validate": {"pattern": {"spec": {"containers": [{"(nonexistent)": "x"}]}}}}),
        pol("any-cond", {"validate": {"message": "one of", "anyPattern": [
            {"spec": {"(hostNetwork)": True, "hostPID": True}},
            {"spec": {"containers": [{"(name)": "zz*", "image": "*:v1"}]}},
            {"metadata": {"(labels)": {"tier": "web"}}}]}}),
        pol("struct-mismatch", {"validate": {"pattern": {"spec": {"containers": {"name": "x"}}}}}),
        pol("keys-err", {"validate": {"pattern": {"spec": {"containers": [
            {"^(ports)": [{"containerPort": ">0"}], "image": "*:v9"}]}}}}),
        pol("keys-err-msg", {"validate": {"message": "image tag v9", "pattern": {"spec": {"containers": [
            {"X(livenessProbe)": "null", "image": "*:v9"}]}}}}),
        pol("any-keys-err", {"validate": {"anyPattern": [
            {"spec": {"containers": [{"X(securityContext)": "null", "name": "zz"}]}},
            {"metadata": {"name": "nope-*"}}]}}),
        pol("float-leaf", {"validate": {"pattern": {"spec": {"=(terminationGracePeriodSeconds)": "<=1000000.5",
                                                             "=(priority)": 1500000}}}}),
    ]


def _skip_error_texts(pols, docs, nsl, backend):
    """(status counts of rendered / unrendered skip+error pairs, mismatches) of every skip / error pair and every
    anyPattern FAIL pair against the oracle's messages"""
    rs = E.Ruleset(pols)
    b = E.Batch(rs, docs, nsl)
    res = E.evaluate(rs, b, backend=backend)
    names, m, tx = O.validate_matrix(pols, docs, nsl, threads=8, texts=("skip", "error", "fail"))
    row = {nm: i for i, nm in enumerate(names)}
    st = np.asarray(res.status)
    n = {"skip": 0, "error": 0, "anyfail": 0, "unrendered": 0, "compared": 0, "mismatch": 0}
    bad = []
    for k, rule in enumerate(rs.rules):
        if rule["kind"] not in ("pattern", "anyPattern"):
            continue
        key = (rs.policies[rule["policy"]]["name"], rule["name"])
        for which, s in (("skip", K.ST_SKIP), ("error", K.ST_ERROR), ("anyfail", K.ST_FAIL)):
            if which == "anyfail" and rule["kind"] != "anyPattern":
                continue
            idx = np.nonzero(st[k] == s)[0]
            if not len(idx):
                continue
            msgs = res.texts(k, "message", (s,), res0=0, nres=len(docs))
            for r in idx.tolist():
                n[which] += 1
                o = tx.get((row[key], r))
                if msgs[r] is None:
                    n["unrendered"] += 1
                    continue
                if o is None or o[2]:
                    continue  # no oracle text / unpinned
                n["compared"] += 1
                if msgs[r] != o[1]:
                    n["mismatch"] += 1
                    if len(bad) < 10:
                        bad.append((key, r, msgs[r][:300], o[1][:300]))
    return n, bad


def test_skip_and_error_messages_cpu():
    docs, nsl = synth.mixed(2500, seed=71, edge=True)
    n, bad = _skip_error_texts(anchor_policies(), docs, nsl, "cpu")
    print(n)
    assert n["mismatch"] == 0, bad
    assert n["skip"] > 3000 and n["error"] > 100 and n["anyfail"] > 100
    assert n["unrendered"] == 0
    assert n["compared"] == n["skip"] + n["error"] + n["anyfail"]


@pytest.mark.gpu
def test_skip_and_error_messages_gpu():
    """>= 10k skip pairs (and the error / path-less anyPattern failures) decided on the device, every message equal
    to the oracle's"""
    docs, nsl = synth.mixed(8000, seed=72, edge=True)
    n, bad = _skip_error_texts(anchor_policies(), docs, nsl, "gpu")
    print(n)
    assert n["mismatch"] == 0, bad
    assert n["skip"] >= 10000 and n["unrendered"] == 0
