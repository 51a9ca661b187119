"""Policy cache (kyverno_amd/policycache.py) against pkg/policycache/cache_test.go: the validate-type lookups of
Test_Get_Policies, Test_Get_Policies_Ns, Test_Get_Policies_Validate_Failure_Action_Overrides and
Test_Validate_Enforce_Policy (tests/golden/policycache.json), plus set / unset and the subresource map."""
import json
import os

import pytest

from kyverno_amd import policycache as PC

GOLD = os.path.join(os.path.dirname(__file__), "golden", "policycache.json")


def _cases():
    with open(GOLD) as f:
        return json.load(f)


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["test"])
def test_policycache_goldens(case):
    cache = PC.PolicyCache()
    for p in case["policies"]:
        cache.set(PC.policy_key(p), p)
    for c in case["calls"]:
        if c["api"] == "get":
            got = cache.get(c["type"], c["kind"], c["namespace"])
        else:
            got = cache.get_policies(c["type"], c["kind"], c["namespace"])
        assert len(got) == c["expected"], c


def _pol(name, kinds, action="Audit", ns=None, validate=True, overrides=None):
    rule = {"name": "r", "match": {"any": [{"resources": {"kinds": kinds}}]}}
    if validate:
        rule["validate"] = {"pattern": {"metadata": {"labels": {"a": "?*"}}}}
    else:
        rule["mutate"] = {"patchStrategicMerge": {"metadata": {"labels": {"a": "b"}}}}
    md = {"name": name}
    if ns:
        md["namespace"] = ns
    spec = {"validationFailureAction": action, "rules": [rule]}
    if overrides:
        spec["validationFailureActionOverrides"] = overrides
    return {"apiVersion": "kyverno.io/v1", "kind": "Policy" if ns else "ClusterPolicy", "metadata": md, "spec": spec}


def test_set_unset_and_kinds():
    cache = PC.PolicyCache()
    a = _pol("a", ["Pod"], "Enforce")
    b = _pol("b", ["*"], "Enforce")
    c = _pol("c", ["ConfigMap"], "Enforce", ns="team")
    m = _pol("m", ["Pod"], "Enforce", validate=False)
    for p in (a, b, c, m):
        cache.set(PC.policy_key(p), p)
    assert PC.policy_key(c) == "team/c"
    # autogen: a Pod rule is indexed under the pod controllers too
    assert cache.get_policy_keys(PC.VALIDATE_ENFORCE, "Deployment", "") == ["a", "b"]
    assert cache.get_policy_keys(PC.VALIDATE_ENFORCE, "apps/v1/Deployment", "") == ["a", "b"]
    assert cache.get_policy_keys(PC.VALIDATE_ENFORCE, "ConfigMap", "team") == ["b", "team/c"]
    assert cache.get_policy_keys(PC.VALIDATE_ENFORCE, "ConfigMap", "other") == ["b"]
    assert cache.get_policy_keys(PC.VALIDATE_AUDIT, "Pod", "") == []  # mutate-only m is never indexed for validate
    cache.unset("b")
    assert cache.get_policy_keys(PC.VALIDATE_ENFORCE, "ConfigMap", "team") == ["team/c"]
    # a policy flipping to Audit moves between the two sets on re-set (store.go set() deletes from the other)
    a2 = _pol("a", ["Pod"], "Audit")
    cache.set("a", a2)
    assert cache.get_policy_keys(PC.VALIDATE_ENFORCE, "Pod", "") == []
    assert cache.get_policy_keys(PC.VALIDATE_AUDIT, "Pod", "") == ["a"]


def test_subresource_kind_map():
    """the subresourceGVKToKind map overrides computeKind for a gvk (store.go:103-106)"""
    cache = PC.PolicyCache()
    p = _pol("s", ["Pod/exec"], "Enforce")
    cache.set("s", p)
    assert cache.get_policy_keys(PC.VALIDATE_ENFORCE, "Pod", "") == ["s"]
    cache2 = PC.PolicyCache()
    cache2.set("s", p, {"Pod/exec": "PodExecOptions"})
    assert cache2.get_policy_keys(PC.VALIDATE_ENFORCE, "Pod", "") == []
    assert cache2.get_policy_keys(PC.VALIDATE_ENFORCE, "PodExecOptions", "") == ["s"]


def test_overrides_filter():
    """filterPolicies: an Audit policy with an Enforce override for ns-* is indexed as enforce; the enforce lookup
    keeps it for any non-empty namespace (checkValidationFailureActionOverrides only drops it where an override of
    the other action matches), the audit lookup drops it where the Enforce override matches"""
    p = _pol("o", ["Pod"], "Audit", overrides=[{"action": "Enforce", "namespaces": ["ns-*"]}])
    cache = PC.PolicyCache()
    cache.set("o", p)
    assert cache.get_policy_keys(PC.VALIDATE_ENFORCE, "Pod", "ns-1") == ["o"]
    assert cache.get_policy_keys(PC.VALIDATE_ENFORCE, "Pod", "default") == ["o"]
    assert cache.get_policy_keys(PC.VALIDATE_ENFORCE, "Pod", "") == []
    assert cache.get_policy_keys(PC.VALIDATE_AUDIT, "Pod", "default") == ["o"]
    assert cache.get_policy_keys(PC.VALIDATE_AUDIT, "Pod", "ns-1") == []
