"""$() references in patterns (variables.substituteReferences, pkg/engine/variables/vars.go:244-346), resolved by
the rule compiler at compile time (kyverno_amd/csrc/compiler.cpp) and restated in the oracle (oracle/orefs.cpp).

Pinned by tests/golden/references.json: the validate_test.go reference walks (substituted first, or walked raw),
vars_test.go Test_*ReferenceSubstitution documents and TestFormAbsolutePath_*. The substituted walks are also run
end to end as policies: the library resolves them (no CPU fallback) and its verdict / failing path equals the
reference's and the oracle's."""
import json
import os

import pytest

from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "references.json")


def _recs(kind):
    with open(GOLD) as f:
        return [r for r in json.load(f) if r["kind"] == kind]


def _walk(entry, resource, pattern):
    import ctypes
    L = O.lib()
    L.oracle_validate_entry.restype = ctypes.c_void_p
    return json.loads(O._take(L.oracle_validate_entry(entry.encode(), resource.encode(), pattern.encode(), 1)))


def test_oracle_form_absolute_path():
    recs = _recs("abs")
    assert len(recs) == 4
    for r in recs:
        assert O.form_absolute_path(r["ref"], r["at"]) == r["want"], r


def test_oracle_substitution_documents():
    recs = _recs("subst")
    assert len(recs) == 2
    for r in recs:
        out = O.substitute_references(r["document"])
        assert out["ok"] and not out["nd"], out
        assert out["doc"] == r["expected"], r["test"]


def test_oracle_reference_walks():
    recs = _recs("walk")
    assert len(recs) == 8
    for r in recs:
        pat = r["pattern"]
        if r["substitute"]:
            out = O.substitute_references(pat)
            assert out["ok"], (r["test"], out)
            pat = out["doc"]
        w = _walk("validateResourceElement", json.dumps(r["resource"]), json.dumps(pat))
        assert w["path"] == (r["path"] or ""), (r["test"], w)
        assert (not w["err"]) == r["err_nil"], (r["test"], w)


def _policy(i, pattern):
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "ref-%d" % i},
            "spec": {"rules": [{"name": "r", "match": {"any": [{"resources": {"kinds": ["Deployment", "Pod"]}}]},
                                "validate": {"message": "m", "pattern": pattern}}]}}


def _end_to_end(backend):
    recs = [r for r in _recs("walk") if r["substitute"]]
    pols = [_policy(i, r["pattern"]) for i, r in enumerate(recs)]
    # the walk tests' resources carry no kind: give them one the policies match (the patterns read neither field)
    docs = [dict({"apiVersion": "v1", "kind": "Pod"}, **r["resource"]) for r in recs]
    rs = E.Ruleset(pols)
    names = {(rs.policies[r["policy"]]["name"], r["name"]): k for k, r in enumerate(rs.rules)}
    assert all(r["kind"] == "pattern" for r in rs.rules if not r["name"].startswith("autogen")), \
        [(r["name"], r["kind"], r.get("reason")) for r in rs.rules]
    res = E.evaluate(rs, E.Batch(rs, docs), backend=backend)
    for i, r in enumerate(recs):
        k = names[("ref-%d" % i, "r")]
        st = int(res.status[k, i])
        want = K.ST_PASS if r["err_nil"] else K.ST_FAIL
        assert st == want, (r["test"], K.STATUS_NAMES[st])
        o = O.validate([pols[i]], json.dumps(docs[i]))[0]["rules"][0]
        assert o["status"] == K.STATUS_NAMES[st], (r["test"], o)
        if st == K.ST_FAIL:
            assert res.path(i, k) == r["path"] == o["path"], (r["test"], res.path(i, k), o["path"])
            assert res.message(i, k) == o["message"], (res.message(i, k), o["message"])


def test_reference_walks_end_to_end_cpu():
    _end_to_end("cpu")


@pytest.mark.gpu
def test_reference_walks_end_to_end_gpu():
    _end_to_end("gpu")


def test_unresolvable_references_fall_back_with_reason():
    """references the reference turns into rule errors or order-dependent results stay on the CPU engine"""
    cases = {
        "unresolved": {"spec": {"a": "$(./../nothing)"}},
        "non-string raw value": {"spec": {"a": "$(./../b)", "b": 5}},
        "several elements": {"spec": {"a": "$(/spec/m)", "m": {"x": "1", "y": "2"}}},
        "empty": {"spec": {"a": "$(<=)"}},
        # the reference path is compared with anchor-free element paths, so an anchored segment never resolves
        "anchored segment": {"metadata": {"labels": {"t": "$(./../../(ann)/o)"}, "(ann)": {"o": "c"}}},
    }
    pols = [_policy(i, p) for i, p in enumerate(cases.values())]
    rs = E.Ruleset(pols)
    for r in rs.rules:
        if r["name"] == "r":
            assert r["kind"] == "fallback" and r["reason"].startswith("references:"), r
    doc = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p"}, "spec": {"a": "1", "b": 5}}
    for i, p in enumerate(pols):
        o = O.validate([p], json.dumps(doc))[0]["rules"][0]
        assert o["status"] == "error" or o.get("nondeterministic"), (list(cases)[i], o)


def test_resolved_reference_kinds():
    """operator prefixes over strings and numbers (fmt %f of the float64), the single key of a one-entry map,
    escaped references, anchored keys on the path -- CPU library vs oracle on pass and fail resources"""
    pats = [
        {"spec": {"replicas": "$(>=./../min)", "min": 2}},
        {"spec": {"replicas": "$(<./../max)", "max": "10"}},
        {"metadata": {"name": "$(/metadata/labels/app)", "labels": {"app": "web"}}},
        {"metadata": {"labels": {"team": "$(./../../annotations/owner)"}, "(annotations)": {"owner": "core"}}},
        {"metadata": {"annotations": {"note": "\\$(LITERAL)"}}},
        {"spec": {"k": "$(/spec/only)", "only": {"solo": 1}}},
        {"metadata": {"name": "?$(./../labels/app)", "labels": {"app": "eb"}}},
    ]
    docs = [
        {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web", "labels": {"app": "web", "team": "core"},
                                                                     "annotations": {"owner": "core", "note": "$(LITERAL)"}},
         "spec": {"replicas": 3, "min": 2, "max": "10", "k": "solo", "only": {"solo": 1}}},
        {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "api", "labels": {"app": "web", "team": "x"},
                                                                     "annotations": {"owner": "core", "note": "other"}},
         "spec": {"replicas": 1, "min": 2, "max": "10", "k": "no", "only": {"solo": 1}}},
    ]
    pols = [_policy(i, p) for i, p in enumerate(pats)]
    rs = E.Ruleset(pols)
    kinds = {rs.policies[r["policy"]]["name"]: (r["kind"], r.get("reason")) for r in rs.rules if r["name"] == "r"}
    res = E.evaluate(rs, E.Batch(rs, docs), backend="cpu")
    names = {(rs.policies[r["policy"]]["name"], r["name"]): k for k, r in enumerate(rs.rules)}
    compared = 0
    for ri, d in enumerate(docs):
        for p in O.validate(pols, json.dumps(d)):
            for rr in p["rules"]:
                if rr["name"] != "r":
                    continue
                k = names[(p["policy"], "r")]
                st = K.STATUS_NAMES[int(res.status[k, ri])]
                if st == "fallback":
                    continue
                assert st == rr["status"], (p["policy"], kinds[p["policy"]], ri, st, rr)
                if st == "fail":
                    assert res.path(ri, k) == rr["path"], (p["policy"], res.path(ri, k), rr["path"])
                compared += 1
    assert all(v[0] == "pattern" for v in kinds.values()), kinds
    assert compared == 2 * len(pats)
