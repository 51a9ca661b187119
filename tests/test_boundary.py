"""C-ABI additions of round 2 (include/kyvgpu.h), on the explicit CPU instantiation of the evaluator:
PolicyException input (kyv_ruleset_compile_ex), per-pair fallback reasons, the policy cache's kind index
(kyv_ruleset_rule_kinds), and the PodSecurity failure message / PodSecurityChecks (kyv_results_pss_checks),
each against the reference behaviour it replaces."""
import json

import cases
from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from oracle import oracle as O


def _pod_policy(name="p", rule="r", pattern=None, kinds=("Pod",)):
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
            "spec": {"rules": [{"name": rule, "match": {"any": [{"resources": {"kinds": list(kinds)}}]},
                                "validate": {"message": "m", "pattern": pattern or {"metadata": {"labels": {"app": "?*"}}}}}]}}


def _pod(name="x", labels=None, ns="default"):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": ns, "labels": labels or {}},
            "spec": {"containers": [{"name": "c", "image": "nginx"}]}}


def test_policy_exception_candidates():
    """A PolicyException naming (policy, rule) stays a device rule: the pairs its match block applies to are skips
    with the exception's key (hasPolicyExceptions, validation.go:797-848), the others keep their verdicts; autogen
    rules are named separately (the exception lists computed rule names), other policies and rules are unaffected"""
    pols = [_pod_policy("p", "r"), _pod_policy("q", "r")]
    exc = [{"apiVersion": "kyverno.io/v2alpha1", "kind": "PolicyException", "metadata": {"name": "e", "namespace": "ns"},
            "spec": {"exceptions": [{"policyName": "p", "ruleNames": ["r", "autogen-cronjob-r"]},
                                    {"policyName": "nope", "ruleNames": ["r"]}],
                     "match": {"any": [{"resources": {"kinds": ["Pod"], "names": ["b*"]}}]}}}]
    rs = E.Ruleset(pols, exceptions=exc)
    assert all(r["kind"] == "pattern" for r in rs.rules)
    b = E.Batch(rs, [_pod("a", {"app": "x"}), _pod("b"), _pod("bb", {"app": "y"}), _pod("c")])
    res = E.evaluate(rs, b, backend="cpu")
    k = [i for i, r in enumerate(rs.rules) if (rs.policies[r["policy"]]["name"], r["name"]) == ("p", "r")][0]
    q = [i for i, r in enumerate(rs.rules) if (rs.policies[r["policy"]]["name"], r["name"]) == ("q", "r")][0]
    assert list(res.status[k]) == [K.ST_PASS, K.ST_SKIP, K.ST_SKIP, K.ST_FAIL]
    assert res.message(1, k) == "rule skipped due to policy exception ns/e"
    assert list(res.status[q]) == [K.ST_PASS, K.ST_FAIL, K.ST_PASS, K.ST_FAIL]


def test_namespaced_policy_exception_key():
    """policy keys are cache.MetaNamespaceKeyFunc: "<ns>/<name>" for a namespaced Policy; an exception whose match
    has neither any nor all applies to every matched resource (CheckMatchesResources returns no error)"""
    pol = _pod_policy("p", "r")
    pol["kind"] = "Policy"
    pol["metadata"]["namespace"] = "team"
    exc = lambda pn: [{"apiVersion": "kyverno.io/v2alpha1", "kind": "PolicyException", "metadata": {"name": "e"},
                       "spec": {"exceptions": [{"policyName": pn, "ruleNames": ["r"]}], "match": {}}}]
    docs = [_pod("a", ns="team"), _pod("b", {"app": "x"}, ns="team")]
    for pn, want in (("p", [K.ST_FAIL, K.ST_PASS]), ("team/p", [K.ST_SKIP, K.ST_SKIP])):
        rs = E.Ruleset([pol], exceptions=exc(pn))
        assert rs.rules[0]["kind"] == "pattern"
        assert list(E.evaluate(rs, E.Batch(rs, docs), backend="cpu").status[0]) == want


def test_policy_exception_limit_falls_back():
    """more candidates than a skip status can name (27) hand the rule to the CPU engine"""
    pol = _pod_policy("p", "r")
    exc = [{"apiVersion": "kyverno.io/v2alpha1", "kind": "PolicyException", "metadata": {"name": f"e{i}"},
            "spec": {"exceptions": [{"policyName": "p", "ruleNames": ["r"]}],
                     "match": {"any": [{"resources": {"names": [f"n{i}"]}}]}}} for i in range(28)]
    rs = E.Ruleset([pol], exceptions=exc)
    assert rs.rules[0]["kind"] == "fallback" and rs.rules[0]["reason"].startswith("exception")


def test_runtime_fallback_reason_anchor_phrase():
    """a resource string holding an anchor-error phrase: the reference classifies errors by substring
    (anchor/error.go:64-75), so the device hands such pattern pairs to the CPU engine and says why"""
    rs = E.Ruleset([_pod_policy()])
    b = E.Batch(rs, [_pod("a", {"app": "conditional anchor mismatch"}), _pod("b", {"app": "ok"})])
    res = E.evaluate(rs, b, backend="cpu")
    assert res.status[0, 0] == K.ST_FALLBACK and res.status[0, 1] == K.ST_PASS
    assert "anchor-error phrase" in res.fallback_reason(0, 0)
    assert res.fallback_reason(1, 0) == ""


def test_rule_kinds_policy_cache_index():
    """MatchResources.GetKinds of the autogen-expanded rules (policyMap.set, pkg/policycache/store.go:96-138)"""
    rs = E.Ruleset([_pod_policy()])
    kinds = {r["name"]: r["match_kinds"] for r in rs.rules}
    assert kinds["r"] == ["Pod"]
    assert set(kinds["autogen-r"]) == {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet",
                                      "ReplicationController"}
    assert kinds["autogen-cronjob-r"] == ["CronJob"]
    assert all(r["has_validate"] for r in rs.rules)
    # the oracle's ComputeRules agrees on the kinds
    for r in O.compute_rules(_pod_policy()):
        assert kinds[r["name"]] == r["match"]["any"][0]["resources"]["kinds"]


_KUTTL_POLICY = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "podsecurity-subrule-restricted"},
                 "spec": {"background": True, "validationFailureAction": "audit", "rules": [
                     {"name": "restricted", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                      "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}}]}}
_KUTTL_POD = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "badpod01", "namespace": "default"},
              "spec": {"containers": [{"name": "container01", "image": "dummyimagename", "securityContext": {
                  "allowPrivilegeEscalation": False, "runAsNonRoot": True, "seccompProfile": {"type": "RuntimeDefault"}}}]}}


def test_pss_failure_message_kuttl_golden():
    """test/conformance/kuttl/reports/background/test-report-background-mode/report-assert.yaml: the exact
    PodSecurity fail message, rendered by the library from the device's check mask"""
    rs = E.Ruleset([_KUTTL_POLICY])
    b = E.Batch(rs, [_KUTTL_POD])
    res = E.evaluate(rs, b, backend="cpu")
    assert res.status[0, 0] == K.ST_FAIL
    detail = 'ForbiddenDetail:container "container01" must set securityContext.capabilities.drop=["ALL"]'
    line = "({Allowed:false ForbiddenReason:unrestricted capabilities " + detail + "})\n"
    assert res.message(0, 0) == ("Validation rule 'restricted' failed. It violates PodSecurity \"restricted:latest\": "
                                 + line + line)
    chk = res.pss_checks(0, 0)
    assert chk["level"] == "restricted" and chk["version"] == "latest"
    assert [c["id"] for c in chk["checks"]] == ["capabilities_restricted"] * 2
    assert chk["checks"][0]["reason"] == "unrestricted capabilities"


def test_pss_messages_equal_oracle_on_goldens():
    """every evaluate_test.go PodSecurity case without exclusions renders the oracle's message exactly; cases with
    exclusions (Go-map order in the reference) are not rendered (None -> the CPU engine formats them)"""
    n = 0
    for name, pol, pod, allowed in cases.pss_cases():
        for p in (pol, json.loads(json.dumps(pol))):
            p["spec"]["rules"][0]["validate"]["podSecurity"].pop("exclude", None) if p is not pol else None
            rs = E.Ruleset([p])
            b = E.Batch(rs, [pod])
            res = E.evaluate(rs, b, backend="cpu")
            o = O.validate([p], json.dumps(pod))[0]["rules"][0]
            st = K.STATUS_NAMES[int(res.status[0, 0])]
            assert st == o["status"], (name, st, o["status"])
            m = res.message(0, 0)
            has_excl = bool(p["spec"]["rules"][0]["validate"]["podSecurity"].get("exclude"))
            if st == "fail":
                if has_excl:
                    assert m is None
                else:
                    assert m == o["message"], (name, m, o["message"])
                    n += 1
    assert n > 20


def test_template_ids_rolled_back_with_a_fallback_rule():
    """A rule whose compile falls back after it interned path templates (here: an anchor-error phrase in a later
    pattern value) must not leave stale template ids behind: the next rule with the same paths gets its own
    templates and renders the oracle's failing path and message"""
    pat = {"spec": {"containers": [{"image": "!*:latest", "name": "?*"}]}}
    bad = json.loads(json.dumps(pat))
    bad["spec"]["zz"] = "conditional anchor mismatch"  # compiled after the container leaves -> Fallback
    pols = [_pod_policy("a", "r", bad), _pod_policy("b", "r", pat), _pod_policy("c", "r", {"spec": {"other": {"k": "v"}}})]
    rs = E.Ruleset(pols)
    assert rs.rules[0]["kind"] == "fallback"
    pod = _pod("x")
    pod["spec"]["containers"] = [{"name": "c", "image": "nginx"}, {"name": "d", "image": "nginx:latest"}]
    b = E.Batch(rs, [pod])
    res = E.evaluate(rs, b, backend="cpu")
    ora = {(p["policy"], r["name"]): r for p in O.validate(pols, json.dumps(pod)) for r in p["rules"]}
    for k, r in enumerate(rs.rules):
        pol = rs.policies[r["policy"]]["name"]
        if pol == "a":
            continue
        o = ora.get((pol, r["name"]))
        if o is None:  # not matched (autogen rules vs a Pod)
            assert res.status[k, 0] == K.ST_NONE
            continue
        assert K.STATUS_NAMES[int(res.status[k, 0])] == o["status"]
        if o["status"] == "fail":
            assert res.path(0, k) == o["path"]
            assert res.message(0, k) == o["message"]


def test_foreach_list_of_request_operation_falls_back():
    """foreach over `request.operation` (the reference iterates the one-element list ["CREATE"]) is not a list
    program the device runs: compile-time fallback, never a JMESPath program read from a literal's index"""
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "p"},
           "spec": {"rules": [{"name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                               "validate": {"foreach": [{"list": "request.operation", "deny": {"conditions": {"any": [
                                   {"key": "{{ element }}", "operator": "Equals", "value": "CREATE"}]}}}]}}]}}
    rs = E.Ruleset([pol])
    assert rs.rules[0]["kind"] == "fallback" and rs.rules[0]["reason"].startswith("foreach")
