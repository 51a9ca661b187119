"""Admission micro-batching (kyverno_amd/admission.py): decision helpers pinned by the reference's own webhook tests,
and the batched device path vs a per-request CPU path (the oracle's engine.Validate restatement) on the same requests.
"""
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


def per_request_decisions(batcher, reqs):
    """Reference shape: every enforce policy of every request through the CPU engine, one request at a time"""
    out = []
    for rq in reqs:
        new, old = rq.get("object") or {}, rq.get("oldObject") or {}
        dts = A._meta(old).get("deletionTimestamp") if new else A._meta(new).get("deletionTimestamp")
        if dts is not None and rq["operation"] == "UPDATE":
            out.append((True, "", None))
            continue
        pols = batcher.enforce_policies(rq.get("namespace") or "")
        if not pols:
            out.append((True, "", None))
            continue
        md = A._meta(new)
        resource = (new.get("kind", ""), md.get("namespace", ""), md.get("name", ""))
        fp, ers = "Ignore", []
        for pi in pols:
            p = batcher.pol[pi]
            if p["fail_policy"] == "Fail":
                fp = "Fail"
            ers.append({"policy": p["name"], "rules": oracle_engine(p["doc"], rq), "resource": resource,
                        "action": A.response_action(p["doc"], resource[1], rq.get("namespace_labels"))})
        allowed, msg, warns, _ = A.decide(ers, fp)
        out.append((allowed, msg, warns))
    return out


def check_admission(backend, n, max_batch):
    pols = admission_policies()
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


@pytest.mark.gpu
def test_admission_gpu_matches_per_request_cpu():
    check_admission("gpu", 2000, 512)


def test_wildcard_golden_admission(golden):
    """the override namespace matcher vs pkg/utils/wildcard/match_test.go (52 vectors, go-wildcard v1.0.3)"""
    recs = golden("wildcard.json")
    assert len(recs) >= 50
    for r in recs:
        assert A.wildcard_match(r["pattern"], r["text"]) == r["matched"], r
