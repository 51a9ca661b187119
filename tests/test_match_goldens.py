"""match / exclude (MatchesResourceDescription, pkg/engine/utils.go:185-289) pinned by the reference's own
pkg/engine/utils_test.go tables (tests/golden/match.json): the oracle must reproduce every case whose rules do not
name roles / clusterRoles / subjects (background semantics: the admission info only matters for those), and the
device's match program (explicit CPU instantiation here; the MI355X in the -m gpu variant) must agree with the
oracle, incl. the OldResource retry of validation.go:600-615."""
import copy
import json

import pytest

from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from oracle import oracle as O


def _userinfo(block):
    if not isinstance(block, dict):
        return False
    if any(block.get(k) for k in ("roles", "clusterRoles", "subjects")):
        return True
    return any(_userinfo(b) for key in ("any", "all") for b in (block.get(key) or []))


def cases(golden):
    for rec in golden("match.json"):
        for rule in O.compute_rules(rec["policy"]):
            if _userinfo(rule.get("match")) or _userinfo(rule.get("exclude")):
                continue
            yield rec, rule


def test_oracle_matches_reference_tables(golden):
    n = 0
    for rec, rule in cases(golden):
        got = O.rule_matches(rule, json.dumps(rec["resource"]))
        assert got == (not rec["errors_expected"]), (rec["test"], rec["description"], rule["name"])
        n += 1
    assert n >= 30


def _device_policy(rec):
    """the golden policy with every rule turned into a validate rule (same match / exclude, empty pattern), autogen
    switched off so that rule names stay the golden's"""
    p = copy.deepcopy(rec["policy"])
    p["kind"] = "ClusterPolicy"
    p.setdefault("metadata", {}).setdefault("annotations", {})["pod-policies.kyverno.io/autogen-controllers"] = "none"
    for r in p["spec"]["rules"]:
        for k in ("mutate", "generate", "validate", "verifyImages"):
            r.pop(k, None)
        r["validate"] = {"pattern": {}}
    return p


def check_device(golden, backend):
    n = 0
    for rec in golden("match.json"):
        p = _device_policy(rec)
        if any(_userinfo(r.get("match")) or _userinfo(r.get("exclude")) for r in p["spec"]["rules"]):
            continue
        rs = E.Ruleset([p])
        b = E.Batch(rs, [rec["resource"]])
        res = E.evaluate(rs, b, backend=backend)
        for k, r in enumerate(rs.rules):
            base = [x for x in p["spec"]["rules"] if x["name"] == r["name"]][0]
            want = O.rule_matches(base, json.dumps(rec["resource"])) or O.rule_matches(base, None)
            got = int(res.status[k, 0]) != K.ST_NONE
            assert got == want, (rec["test"], rec["description"], r["name"], K.STATUS_NAMES[int(res.status[k, 0])])
            n += 1
    assert n >= 30


def test_device_match_program_cpu_instantiation(golden):
    check_device(golden, "cpu")


@pytest.mark.gpu
def test_device_match_program_gpu(golden):
    check_device(golden, "gpu")


# ---------------------------------------------------------------- pkg/utils/match + pkg/utils/kube unit tables
def _one(match_rd, resource, backend):
    """device verdict: does a rule whose match is `match_rd` (a ResourceDescription) select `resource`?"""
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy",
           "metadata": {"name": "u", "annotations": {"pod-policies.kyverno.io/autogen-controllers": "none"}},
           "spec": {"rules": [{"name": "r", "match": {"any": [{"resources": match_rd}]}, "validate": {"pattern": {}}}]}}
    rs = E.Ruleset([pol])
    res = E.evaluate(rs, E.Batch(rs, [resource]), backend=backend)
    dev = int(res.status[0, 0]) != K.ST_NONE
    ora = O.rule_matches(pol["spec"]["rules"][0], json.dumps(resource))
    return dev, ora


def _pod(name="p", labels=None, ann=None, api="v1", kind="Pod"):
    md = {"name": name, "namespace": "d"}
    if labels is not None:
        md["labels"] = labels
    if ann is not None:
        md["annotations"] = ann
    return {"apiVersion": api, "kind": kind, "metadata": md}


def check_units(golden, backend):
    u = golden("match_units.json")
    n = 0
    for c in u["name"]:  # CheckName (name.go:7-9); an empty name in a ResourceDescription is "no constraint"
        assert O.wildcard(c["expected"], c["actual"]) == c["want"], c
        if c["expected"] and c["actual"]:
            dev, ora = _one({"kinds": ["Pod"], "name": c["expected"]}, _pod(c["actual"]), backend)
            assert dev == ora == c["want"], c
            n += 1
    for c in u["annotations"]:  # CheckAnnotations (annotations.go:7-23)
        if not c["expected"]:
            continue
        dev, ora = _one({"kinds": ["Pod"], "annotations": c["expected"]}, _pod(ann=c["actual"]), backend)
        assert dev == ora == c["want"], c
        n += 1
    for c in u["selector"]:  # CheckSelector (labels.go:10-24): an error is no match
        dev, ora = _one({"kinds": ["Pod"], "selector": c["expected"]}, _pod(labels=c["actual"]), backend)
        assert dev == ora == (c["want"] and not c["wantErr"]), c
        n += 1
    for c in u["check_kind"]:  # CheckKind (kind.go:14-38), background scans: no subresource
        if c["subresource"] or c["subresource_map"]:
            continue
        api = c["group"] + "/" + c["version"] if c["group"] else c["version"]
        dev, ora = _one({"kinds": c["kinds"]}, _pod(api=api, kind=c["kind"]), backend)
        assert dev == ora == c["want"], c
        n += 1
    for c in u["gv_matches"]:  # GroupVersionMatches (kube/kind.go:63-75) through a kinds entry "<gv>/Pod"
        dev, ora = _one({"kinds": [c["group_version"] + "/Pod"]}, _pod(api=c["server"]), backend)
        assert dev == ora == c["want"], c
        n += 1
    assert n >= 30


def test_match_unit_tables_cpu_instantiation(golden):
    check_units(golden, "cpu")


@pytest.mark.gpu
def test_match_unit_tables_gpu(golden):
    check_units(golden, "gpu")


def test_get_kind_from_gvk_golden(golden):
    """kube.GetKindFromGVK (kind.go:11-32) as the policy-cache mirror restates it (kyverno_amd/admission.py)"""
    from kyverno_amd import admission as A
    recs = golden("match_units.json")["gvk"]
    assert len(recs) >= 14
    for c in recs:
        assert A.kind_from_gvk(c["gvk"]) == (c["group_version"], c["kind"]), c
