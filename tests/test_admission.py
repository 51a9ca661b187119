"""Admission micro-batching (kyverno_amd/admission.py): decision helpers pinned by the reference's own webhook tests,
and the batched device path vs a per-request CPU path (the oracle's engine.Validate restatement) on the same requests.
"""
import collections
import copy
import json
import random

import pytest

import cases
from kyverno_amd import admission as A
from kyverno_amd import engine as E
from kyverno_amd import synth
from oracle import oracle as O


def _er(policy, rules, action, resource=("foo", "bar", "baz")):
    return {"policy": policy, "action": action, "resource": resource,
            "rules": [{"name": n, "status": s, "message": m} for n, s, m in rules]}


# pkg/webhooks/utils/block_test.go:12-44 (Test_getAction)
@pytest.mark.parametrize("viol,n,want", [(True, 1, "violation"), (True, 5, "violations"), (False, 1, "error"),
                                         (False, 5, "errors")])
def test_get_action_golden(viol, n, want):
    assert A.get_action(viol, n) == want


# pkg/webhooks/utils/block_test.go:46-189 (TestBlockRequest); RuleStatusWarn has no device counterpart but is
# kept as a status string
@pytest.mark.parametrize("action,status,fp,want", [
    ("Enforce", "fail", "Fail", True), ("Audit", "fail", "Fail", False), ("Audit", "error", "Fail", True),
    ("Audit", "error", "Ignore", False), ("Audit", "warn", "Ignore", False), ("Audit", "warn", "Fail", False)])
def test_block_request_golden(action, status, fp, want):
    er = _er("test", [("rule", status, "m")], action)
    assert A.block_request(er, fp) == want


# pkg/webhooks/utils/block_test.go:191-291 (TestGetBlockedMessages)
def test_get_blocked_messages_golden():
    got, exact = A.get_blocked_messages([_er("test", [("rule-fail", "fail", "message fail")], "Enforce")])
    assert exact and got == "\n\npolicy foo/bar/baz for resource violation: \n\ntest:\n  rule-fail: message fail\n"
    got, _ = A.get_blocked_messages([_er("test", [("rule-error", "error", "message error")], "Enforce")])
    assert got == "\n\npolicy foo/bar/baz for resource error: \n\ntest:\n  rule-error: message error\n"
    got, _ = A.get_blocked_messages([_er("test", [("rule-fail", "fail", "message fail"),
                                                  ("rule-error", "error", "message error")], "Enforce")])
    assert got == ("\n\npolicy foo/bar/baz for resource violation: \n\ntest:\n  rule-error: message error\n"
                   "  rule-fail: message fail\n")


# pkg/webhooks/utils/warning_test.go:12-101 (TestGetWarningMessages)
def test_get_warning_messages_golden():
    assert A.get_warning_messages([]) is None
    assert A.get_warning_messages([_er("test", [], "Audit")]) is None
    assert A.get_warning_messages([_er("test", [("rule", "warn", "message warn")], "Audit")]) == \
        ["policy test.rule: message warn"]
    rules = [("rule-pass", "pass", "message pass"), ("rule-warn", "warn", "message warn"),
             ("rule-fail", "fail", "message fail"), ("rule-error", "error", "message error"),
             ("rule-skip", "skip", "message skip")]
    assert A.get_warning_messages([_er("test", rules, "Audit")]) == [
        "policy test.rule-warn: message warn", "policy test.rule-fail: message fail",
        "policy test.rule-error: message error"]


def test_yaml_scalar_styles():
    """go-yaml v2 emitter restatement: quoting, '' escapes, folding at width 80 (continuation indent 4).
    Only the short plain cases are pinned by a reference test (above); the rest is the published emitter."""
    msg = ("validation error: Using a mutable image tag e.g. 'latest' is not allowed. rule validate-image-tag "
           "failed at path /spec/containers/0/image/")
    body, exact = A.yaml_marshal_failures({"disallow-latest-tag": {"validate-image-tag": msg}})
    assert exact
    assert body == ("disallow-latest-tag:\n  validate-image-tag: 'validation error: Using a mutable image tag e.g. "
                    "''latest''\n    is not allowed. rule validate-image-tag failed at path /spec/containers/0/image/'\n")
    body, _ = A.yaml_marshal_failures({"p": {"r": "true"}})
    assert body == 'p:\n  r: "true"\n'
    assert A._sorted_keys(["rule-10", "rule-9", "rule-a", "rule-"]) == ["rule-", "rule-9", "rule-10", "rule-a"]


def test_policycache_enforce_filter():
    """cache.go checkValidationFailureActionOverrides / engineresponse.go GetValidationFailureAction"""
    p = {"kind": "ClusterPolicy", "metadata": {"name": "x"},
         "spec": {"validationFailureAction": "Audit", "rules": [{"name": "r", "validate": {}}],
                  "validationFailureActionOverrides": [{"action": "Enforce", "namespaces": ["prod-*"]},
                                                       {"action": "Audit", "namespaces": ["prod-dev"]}]}}
    assert A.compute_enforce_policy(p)
    assert A.keep_for_enforce(p, "prod-1") and A.keep_for_enforce(p, "default")
    assert not A.keep_for_enforce(p, "prod-dev") and not A.keep_for_enforce(p, "")
    assert A.response_action(p, "prod-1", {}) == "Enforce"
    assert A.response_action(p, "default", {}) == "Audit"
    q = {"spec": {"validationFailureAction": "Audit", "validationFailureActionOverrides": [
        {"action": "Enforce", "namespaceSelector": {"matchLabels": {"env": "prod"}}}]}}
    assert A.response_action(q, "a", {"env": "prod"}) == "Enforce"
    assert A.response_action(q, "a", {"env": "dev"}) == "Audit"
    assert A.wildcard_match("ns-?0*", "ns-10abc") and not A.wildcard_match("ns-?0*", "ns-1")


# ------------------------------------------------------------------------------------ batched path vs per request
def admission_policies(seed=7):
    """C3's device-covered policies (charts restricted + best practices without the JMESPath/foreach ones), with
    seeded Enforce / Audit / failurePolicy / override variations"""
    pols = cases.best_practices() + cases.chart_restricted()
    rs = E.Ruleset(pols)
    cpu_only = {rs.policies[r["policy"]]["name"] for r in rs.rules if r["kind"] == "fallback"}
    rng = random.Random(seed)
    out = []
    for p in pols:
        if p["metadata"]["name"] in cpu_only:
            continue
        p = copy.deepcopy(p)
        s = p["spec"]
        s["validationFailureAction"] = rng.choice(["Enforce", "enforce", "Audit", "audit"])
        if rng.random() < 0.3:
            s["failurePolicy"] = "Ignore"
        if rng.random() < 0.25:
            s["validationFailureActionOverrides"] = [{"action": "Audit", "namespaces": ["ns-00*"]},
                                                     {"action": "Enforce", "namespaces": ["ns-01*"]}]
        out.append(p)
    return out


def admission_requests(n, seed=11):
    docs, nsl = synth.mixed(n, seed=seed, edge=True)
    rng = random.Random(seed)
    reqs = []
    for i, d in enumerate(docs):
        md = d.get("metadata") if isinstance(d.get("metadata"), dict) else {}
        ns = md.get("namespace") if isinstance(md.get("namespace"), str) else ""
        op = "UPDATE" if rng.random() < 0.2 else "CREATE"
        old = None
        if op == "UPDATE":
            old = copy.deepcopy(d)
            if rng.random() < 0.5 and isinstance(old.get("metadata"), dict):
                old["metadata"]["labels"] = {"changed": "yes"}
            if rng.random() < 0.05 and isinstance(old.get("metadata"), dict):
                old["metadata"]["deletionTimestamp"] = "2024-01-01T00:00:00Z"
        reqs.append({"uid": "u%d" % i, "operation": op, "kind": d.get("kind", ""), "namespace": ns, "object": d,
                     "oldObject": old, "namespace_labels": nsl.get(ns) if ns else None})
    return reqs


def oracle_engine(policy, rq):
    """engine.Validate on the CPU for one policy (test checker: the oracle restatement)"""
    nsl = rq.get("namespace_labels") or {}
    pr = O.validate([policy], json.dumps(rq["object"]), nsl)
    return [{"name": r["name"], "status": r["status"], "message": r["message"]} for p in pr for r in p["rules"]]


def _gvk_kind(gvk):
    """pkg/policycache/store.go computeKind (GetKindFromGVK + SplitSubresource), restated for the test"""
    parts = gvk.split("/")
    ver = lambda x: x == "*" or any(x[i] == "v" and x[i + 1].isdigit() for i in range(len(x) - 1))
    if len(parts) == 2:
        k = parts[1].replace(".", "/", 1) if ver(parts[0]) else parts[0] + "/" + parts[1]
    elif len(parts) == 3:
        k = parts[1] + "/" + parts[2] if ver(parts[0]) else parts[2].replace(".", "/", 1)
    elif len(parts) == 4:
        k = parts[2] + "/" + parts[3]
    else:
        k = gvk.replace(".", "/", 1)
    sp = k.split("/")
    return sp[0] if len(sp) == 2 else k


class PolicyCache:
    """Independent policy cache for the test (pkg/policycache/store.go:96-170, cache.go:38-88): kinds come from the
    oracle's ComputeRules, not from the library."""

    def __init__(self, policies):
        self.entries = []
        for p in policies:
            s = p.get("spec") or {}
            enforce = A.action_enforce(s.get("validationFailureAction", "Audit")) or any(
                A.action_enforce((o or {}).get("action")) for o in s.get("validationFailureActionOverrides") or [])
            kinds = set()
            for r in O.compute_rules(p):
                if r.get("validate"):
                    m = r.get("match") or {}
                    ks = list((m.get("resources") or {}).get("kinds") or [])
                    for b in (m.get("any") or []) + (m.get("all") or []):
                        ks += (b.get("resources") or {}).get("kinds") or []
                    kinds.update(_gvk_kind(k) for k in ks)
            ns = (p.get("metadata") or {}).get("namespace", "") if p.get("kind") == "Policy" else ""
            self.entries.append((p, ns, kinds, enforce))

    def get_enforce(self, kind, ns):
        out = []
        for scope in [""] + ([ns] if ns else []):
            for key in (_gvk_kind(kind), "*"):
                for p, pns, kinds, enf in self.entries:
                    if enf and pns == scope and key in kinds and A.keep_for_enforce(p, ns):
                        out.append(p)
        return out


def per_request_decisions(batcher, reqs):
    """Reference shape: the enforce policies of every request (independent kind-indexed policy cache) through the CPU
    engine, one request at a time"""
    out = []
    cache = PolicyCache(batcher.policies)
    for rq in reqs:
        new, old = rq.get("object") or {}, rq.get("oldObject") or {}
        dts = A._meta(old).get("deletionTimestamp") if new else A._meta(new).get("deletionTimestamp")
        if dts is not None and rq["operation"] == "UPDATE":
            out.append((True, "", None))
            continue
        pols = cache.get_enforce(rq.get("kind", ""), rq.get("namespace") or "")
        if not pols:
            out.append((True, "", None))
            continue
        md = A._meta(new)
        resource = (new.get("kind", ""), md.get("namespace", ""), md.get("name", ""))
        fp, ers = "Ignore", []
        for p in pols:
            if ((p.get("spec") or {}).get("failurePolicy") or "Fail") == "Fail":
                fp = "Fail"
            ers.append({"policy": p["metadata"]["name"], "rules": oracle_engine(p, rq), "resource": resource,
                        "action": A.response_action(p, resource[1], rq.get("namespace_labels"))})
        allowed, msg, warns, _ = A.decide(ers, fp)
        out.append((allowed, msg, warns))
    return out


def check_admission(backend, n, max_batch, pols=None):
    pols = pols or admission_policies()
    reqs = admission_requests(n)
    b = A.AdmissionBatcher(pols, backend=backend, cpu_engine=oracle_engine, max_batch=max_batch)
    got = []
    for i in range(0, len(reqs), max_batch):
        got.extend(b.handle_batch(reqs[i:i + max_batch]))
    want = per_request_decisions(b, reqs)
    bad = [(rq["uid"], g, w) for rq, g, w in zip(reqs, got, want)
           if (g["allowed"], g["message"], g["warnings"]) != w]
    assert not bad, bad[:3]
    blocked = sum(1 for g in got if g["allowed"] is False)
    assert 0 < blocked < len(reqs)
    assert b.stats["device_policies"] > b.stats["cpu_policies"]
    return b, reqs, got


def test_admission_batched_matches_per_request_cpu():
    check_admission("cpu", 300, 128)


def test_admission_threaded_microbatches():
    pols = admission_policies()
    reqs = admission_requests(120, seed=3)
    b = A.AdmissionBatcher(pols, backend="cpu", cpu_engine=oracle_engine, max_batch=32, max_wait_ms=2.0).start()
    try:
        futs = [b.submit(rq) for rq in reqs]
        got = [f.result(timeout=120) for f in futs]
    finally:
        b.stop()
    want = A.AdmissionBatcher(pols, backend="cpu", cpu_engine=oracle_engine).handle_batch(reqs)
    assert [g["uid"] for g in got] == [rq["uid"] for rq in reqs]
    assert [(g["allowed"], g["message"], g["warnings"]) for g in got] == \
        [(w["allowed"], w["message"], w["warnings"]) for w in want]
    assert b.stats["batches"] >= 4


def test_admission_routing_without_cpu_engine():
    """Pairs the device cannot decide leave the decision pending (the Go shim runs engine.Validate for them)"""
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "ui"},
           "spec": {"validationFailureAction": "Enforce", "rules": [{
               "name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}, "subjects": [{"kind": "User", "name": "x"}]}]},
               "validate": {"message": "m", "pattern": {"metadata": {"labels": {"a": "?*"}}}}}]}}
    b = A.AdmissionBatcher([pol], backend="cpu")
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "d"}, "spec": {}}
    out = b.handle_batch([{"uid": "1", "operation": "CREATE", "kind": "Pod", "namespace": "d", "object": pod},
                          {"uid": "2", "operation": "DELETE", "kind": "Pod", "namespace": "d", "object": None,
                           "oldObject": pod}])
    assert out[0]["allowed"] is None and out[0]["cpu_pending"] == ["ui"]
    assert out[1]["allowed"] is None


def test_admission_pss_and_quirks_enforce():
    """PodSecurity and quirk policies under Enforce: device pairs whose message the library cannot render (PSS
    failures, skip / error texts) send the whole policy to the CPU engine instead of failing the batch"""
    pols = []
    for p in [c[1] for c in cases.pss_cases()[:6]] + cases.quirk_policies():
        p = copy.deepcopy(p)
        p["spec"]["validationFailureAction"] = "Enforce"
        pols.append(p)
    check_admission("cpu", 200, 64, pols=pols)


def test_admission_failure_policy_is_kind_indexed():
    """policycache.GetPolicies(ValidateEnforce, kind, ns) decides failurePolicy: a default-Fail policy matching only
    Deployments must not turn a Pod's error under an Ignore policy into a block (validation.go:105-114)"""
    dep_only = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "dep-only"},
                "spec": {"validationFailureAction": "Enforce", "rules": [{
                    "name": "r", "match": {"any": [{"resources": {"kinds": ["apps/v1/Deployment"]}}]},
                    "validate": {"pattern": {"metadata": {"labels": {"a": "?*"}}}}}]}}
    erring = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "erring"},
              "spec": {"validationFailureAction": "Enforce", "failurePolicy": "Ignore", "rules": [{
                  "name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                  "validate": {"anyPattern": {"spec": {"x": "1"}}}}]}}
    b = A.AdmissionBatcher([dep_only, erring], backend="cpu", cpu_engine=oracle_engine)
    assert b.enforce_policies("d", "Pod") == [1]
    assert b.enforce_policies("d", "Deployment") == [0, 1]  # erring's autogen rule covers Deployments
    assert b.enforce_policies("d", "ConfigMap") == []
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "d"}, "spec": {"x": "2"}}
    out = b.handle_batch([{"uid": "1", "operation": "CREATE", "kind": "Pod", "namespace": "d", "object": pod}])
    want = per_request_decisions(b, [{"uid": "1", "operation": "CREATE", "kind": "Pod", "namespace": "d",
                                      "object": pod}])
    assert (out[0]["allowed"], out[0]["message"], out[0]["warnings"]) == want[0]
    assert out[0]["allowed"] is True and out[0]["warnings"]  # the error is a warning, not a block


def test_admission_cancelled_future_does_not_stall():
    pols = admission_policies()
    reqs = admission_requests(40, seed=5)
    b = A.AdmissionBatcher(pols, backend="cpu", cpu_engine=oracle_engine, max_batch=8, max_wait_ms=50.0).start()
    try:
        futs = [b.submit(rq) for rq in reqs]
        for f in futs[::3]:
            f.cancel()
        left = [f for f in futs if not f.cancelled()]
        got = [f.result(timeout=120) for f in left]
        assert len(got) == len(left)
        again = b.submit(reqs[0]).result(timeout=60)  # the batcher thread is still alive
        assert again["uid"] == reqs[0]["uid"]
    finally:
        b.stop()


@pytest.mark.gpu
def test_admission_gpu_matches_per_request_cpu():
    check_admission("gpu", 2000, 512)


def test_wildcard_golden_admission(golden):
    """the override namespace matcher vs pkg/utils/wildcard/match_test.go (52 vectors, go-wildcard v1.0.3)"""
    recs = golden("wildcard.json")
    assert len(recs) >= 50
    for r in recs:
        assert A.wildcard_match(r["pattern"], r["text"]) == r["matched"], r


def test_admission_metrics_only_device_responses():
    """kyverno_policy_results of an admission batch counts exactly the engine responses the device produced: nothing
    for a userInfo policy (its responses come from the CPU engine, recorded by the Go shim), nothing for a policy
    reading request.operation on an UPDATE, nothing for the OldResource row, and one set of responses per device-decided
    (request, policy) pair (pkg/webhooks/utils/metrics.go:25-64)"""
    ui = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "ui"},
          "spec": {"validationFailureAction": "Enforce", "rules": [{
              "name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}, "subjects": [{"kind": "User", "name": "x"}]}]},
              "validate": {"message": "m", "pattern": {"metadata": {"labels": {"a": "?*"}}}}}]}}
    op = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "op"},
          "spec": {"validationFailureAction": "Enforce", "rules": [{
              "name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
              "preconditions": {"all": [{"key": "{{ request.operation }}", "operator": "Equals", "value": "CREATE"}]},
              "validate": {"message": "m", "pattern": {"metadata": {"labels": {"a": "?*"}}}}}]}}
    plain = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "plain"},
             "spec": {"validationFailureAction": "Enforce", "rules": [{
                 "name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                 "validate": {"message": "m", "pattern": {"metadata": {"labels": {"b": "?*"}}}}}]}}
    calls = []

    def engine(p, rq):
        calls.append((p["metadata"]["name"], rq["operation"]))
        return oracle_engine(p, rq)

    b = A.AdmissionBatcher([ui, op, plain], backend="cpu", cpu_engine=engine)
    pod = lambda n, lab: {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": n, "namespace": "d", "labels": lab},
                          "spec": {}}
    reqs = [{"uid": "c", "operation": "CREATE", "kind": "Pod", "namespace": "d", "object": pod("p1", {"a": "1"})},
            {"uid": "u", "operation": "UPDATE", "kind": "Pod", "namespace": "d", "object": pod("p2", {"b": "1"}),
             "oldObject": pod("p2", {})}]
    b.handle_batch(reqs)
    by = collections.Counter()
    for key, n in b.metrics.results.items():
        by[(key[4], key[7])] += n  # (policy name, operation)
    # device responses: "op" for the CREATE, "plain" for both requests; "ui" never; "op" not for the UPDATE
    assert by == {("op", "create"): 1, ("plain", "create"): 1, ("plain", "update"): 1}, by
    assert sorted(calls) == [("op", "UPDATE"), ("ui", "CREATE"), ("ui", "UPDATE")]
