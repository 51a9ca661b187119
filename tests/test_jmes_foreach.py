"""JMESPath-subset operands and foreach-deny rules on the explicit CPU instantiation of
the device evaluator, against the oracle (oracle/ojmes.cpp restates go-jmespath + the kyverno fork's missing-key
rule, pinned by the Test_Apply and test/cli/test/foreach goldens), pair by pair with messages, over the chart's
projection / foreach rules and hand-built edge cases (missing and null lists, non-map elements, empty lists,
non-string capabilities, elementScope on strings, NotFound chains, length() of arrays / maps / strings /
projections / missing values)."""
import copy

import cases
import parity_util as PU
from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from kyverno_amd import synth


def _pol(name, validate, pre=None, kinds=("Pod",)):
    rule = {"name": "r", "match": {"any": [{"resources": {"kinds": list(kinds)}}]}, "validate": validate}
    if pre is not None:
        rule["preconditions"] = pre
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy",
            "metadata": {"name": name, "annotations": {"pod-policies.kyverno.io/autogen-controllers": "none"}},
            "spec": {"rules": [rule]}}


def jmes_policies():
    chart = [p for p in cases.chart_restricted()
             if p["metadata"]["name"] in ("disallow-capabilities", "disallow-capabilities-strict", "restrict-volume-types")]
    extra = [
        _pol("images-foreach", {"message": "images must begin with ghcr.io", "foreach": [
            {"list": "request.object.spec.containers[].image",
             "deny": {"conditions": {"all": [{"key": "{{ element }}", "operator": "NotEquals", "value": "ghcr.io*"}]}}}]}),
        _pol("scope-error", {"message": "m", "foreach": [
            {"list": "request.object.spec.containers[].name", "elementScope": True,
             "deny": {"conditions": {"all": [{"key": "{{ element }}", "operator": "Equals", "value": "x"}]}}}]}),
        _pol("pure-element-chain", {"message": "m", "foreach": [
            {"list": "request.object.spec.containers",
             "deny": {"conditions": {"any": [{"key": "{{ element.securityContext.privileged }}", "operator": "Equals",
                                              "value": True}]}}}]}),
        _pol("pre-element", {"foreach": [
            {"list": "request.object.spec.[initContainers, containers][]",
             "preconditions": {"all": [{"key": "{{ element.image || '' }}", "operator": "NotEquals", "value": ""}]},
             "deny": {"conditions": {"all": [{"key": "{{ element.ports[].containerPort || `[]` }}",
                                              "operator": "AnyIn", "value": [22, 23]}]}}}]}),
        _pol("keys-of-labels", {"message": "no x- labels", "deny": {"conditions": {"any": [
            {"key": "{{ request.object.metadata.labels.keys(@) || `[]` }}", "operator": "AnyIn", "value": ["x-*"]}]}}}),
        _pol("op-precondition", {"message": "m", "pattern": {"metadata": {"name": "?*"}}},
             pre={"all": [{"key": "{{ request.operation || 'BACKGROUND' }}", "operator": "Equals", "value": "CREATE"}]}),
        _pol("len-containers", {"message": "at most one container", "deny": {"conditions": {"any": [
            {"key": "{{ length(request.object.spec.containers) }}", "operator": "GreaterThan", "value": 1}]}}}),
        _pol("len-labels-name", {"deny": {"conditions": {"all": [
            {"key": "{{ length(request.object.metadata.labels) }}", "operator": "Equals", "value": 1},
            {"key": "{{length(request.object.metadata.name)}}", "operator": "LessThanOrEquals", "value": 2}]}}}),
        _pol("len-projection", {"deny": {"conditions": {"any": [
            {"key": "{{ length(request.object.spec.containers[].image) }}", "operator": "Equals", "value": 0},
            {"key": "{{ length(request.object.spec.volumes[].keys(@)[]) }}", "operator": "GreaterThanOrEquals",
             "value": 4}]}}}),
        _pol("len-element", {"foreach": [
            {"list": "request.object.spec.containers",
             "deny": {"conditions": {"all": [{"key": "{{ length(element.name) }}", "operator": "LessThan",
                                              "value": 2}]}}}]}),
        _pol("dur-ttl", {"message": "ttl above one hour", "deny": {"conditions": {"any": [
            {"key": "{{ request.object.metadata.annotations.ttl || '0s' }}", "operator": "DurationGreaterThan",
             "value": "1h"},
            {"key": "{{ request.object.metadata.annotations.ttl || `90` }}", "operator": "DurationLessThan",
             "value": 60}]}}}),
        _pol("dur-grace", {"deny": {"conditions": {"all": [
            {"key": "{{ request.object.spec.terminationGracePeriodSeconds }}", "operator": "DurationLessThanOrEquals",
             "value": "30s"},
            {"key": "45s", "operator": "DurationGreaterThanOrEquals", "value": 44.9}]}}}),
        _pol("dur-spelling", {"deny": {"conditions": {"any": [
            {"key": "2h", "operator": "durationGreaterThan", "value": "1h"}]}}}),
        _pol("vol-keys", {"deny": {"conditions": {"all": [
            {"key": "{{ request.object.spec.volumes[].keys(@)[] || '' }}", "operator": "AnyIn",
             "value": ["hostPath", "nfs"]}]}}}),
    ]
    return chart + extra


def edge_pods():
    base = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "d", "labels": {"a": "b"}}}
    specs = [
        None, {}, {"containers": None}, {"containers": []},
        {"containers": [{"name": "c", "image": "ghcr.io/x"}]},
        {"containers": [{"name": "c", "image": "docker.io/x", "securityContext": None}]},
        {"containers": [{"name": "c", "securityContext": {"capabilities": {"add": ["SYS_ADMIN"], "drop": ["ALL"]}}}]},
        {"containers": [{"name": "c", "securityContext": {"capabilities": {"add": [], "drop": []}}}]},
        {"containers": [{"name": "c", "securityContext": {"capabilities": {"add": ["NET_BIND_SERVICE"], "drop": ["ALL"]},
                                                          "privileged": True}}]},
        {"containers": [{"name": "c", "securityContext": {"capabilities": {"add": [5, True], "drop": "ALL"}}}]},
        {"initContainers": [{"name": "i", "image": "a", "ports": [{"containerPort": 22}]}],
         "ephemeralContainers": [{"name": "e", "securityContext": {"capabilities": {"add": ["CHOWN"]}}}],
         "containers": [{"name": "c", "image": "b", "ports": [{"containerPort": 80}]}]},
        {"containers": [{"name": "c"}], "volumes": None},
        {"containers": [{"name": "c"}], "volumes": []},
        {"containers": [{"name": "c"}], "volumes": [{"name": "v", "hostPath": {"path": "/"}}, {"name": "w", "emptyDir": {}}]},
        {"containers": [{"name": "c"}], "volumes": [{"name": "v", "configMap": {}}, "oops"]},
        {"containers": [{"name": "c"}], "volumes": [{"name": "v", "csi": {}}, None]},
        {"containers": "notalist"},
        {"containers": [None, {"name": "c", "image": "ghcr.io/y"}]},
    ]
    out = []
    for i, sp in enumerate(specs):
        d = copy.deepcopy(base)
        d["metadata"]["name"] = "p%d" % i
        if i % 3 == 0:
            d["metadata"]["labels"] = {"x-team": "1"}
        if i == 5:
            d["metadata"]["labels"] = None
        ttl = ("30m", "2h", "3600", "bad", "0", "1.5h", "-5s", None, "1h0m1s", "59")[i % 10]
        if ttl is not None:
            d["metadata"]["annotations"] = {"ttl": ttl}
        if i % 4 == 1:
            d["spec"] = dict(sp or {}, terminationGracePeriodSeconds=(30, 31, 29.5, "30")[(i // 4) % 4])
        if sp is not None and "spec" not in d:
            d["spec"] = sp
        out.append(d)
    return out


def test_jmes_foreach_edge_cases_equal_oracle():
    pols = jmes_policies()
    rs = E.Ruleset(pols)
    kinds = {rs.policies[r["policy"]]["name"]: r["kind"] for r in rs.rules}
    assert kinds["images-foreach"] == "foreach" and kinds["disallow-capabilities-strict"] == "foreach"
    assert kinds["restrict-volume-types"] == "deny" and kinds["keys-of-labels"] == "deny"
    assert all(r["kind"] != "fallback" for r in rs.rules), [(r["name"], r["reason"]) for r in rs.rules]
    assert any(r["uses_operation"] for r in rs.rules)
    st, res = PU.compare(pols, edge_pods(), None, backend="cpu")
    assert st["nbad"] == 0, st["bad"]
    assert st["compared"] > 100 and st["messages"] > 50
    for s in ("pass", "fail", "skip", "error"):
        assert res.counts[s] > 0, (s, res.counts)


def test_jmes_foreach_synthetic_equal_oracle():
    pols = jmes_policies()
    docs, nsl = synth.mixed(3000, seed=91, edge=True)
    st, res = PU.compare(pols, docs, nsl, backend="cpu")
    assert st["nbad"] == 0, st["bad"]
    assert res.counts["fail"] > 100 and res.counts["pass"] > 1000
    assert res.counts["fallback"] < 0.01 * st["pairs"]


import pytest  # noqa: E402


@pytest.mark.gpu
def test_jmes_foreach_edge_cases_gpu():
    st, res = PU.compare(jmes_policies(), edge_pods(), None, backend="gpu")
    assert st["nbad"] == 0, st["bad"]
    assert st["compared"] > 100


@pytest.mark.gpu
def test_jmes_foreach_synthetic_gpu():
    docs, nsl = synth.mixed(3000, seed=92, edge=True)
    st, res = PU.compare(jmes_policies(), docs, nsl, backend="gpu")
    assert st["nbad"] == 0, st["bad"]
    assert res.counts["fail"] > 100


@pytest.mark.gpu
def test_jmes_foreach_edge_cases_gpu_compiled():
    """the runtime-compiled condition kernel (jit.cpp CondGen: path-column reads, streamed foreach lists, LDS operand
    lists) on the same edge cases"""
    st, res = PU.compare(jmes_policies(), edge_pods(), None, backend="gpu", jit=True)
    assert res.jit_cond
    assert st["nbad"] == 0, st["bad"]
    assert st["compared"] > 100


@pytest.mark.gpu
def test_jmes_foreach_synthetic_gpu_compiled():
    docs, nsl = synth.mixed(3000, seed=93, edge=True)
    st, res = PU.compare(jmes_policies(), docs, nsl, backend="gpu", jit=True)
    assert res.jit_cond
    assert st["nbad"] == 0, st["bad"]
    assert res.counts["fail"] > 100
