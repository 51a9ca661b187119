"""Pins the oracle (oracle/, the CPU restatement of the reference validate path) against the golden
vectors extracted from the reference's own tests (tests/golden/extract.py). CPU only."""
import copy
import ctypes
import json

import pytest

from oracle import oracle as O


def test_wildcard_golden(golden):
    recs = golden("wildcard.json")
    assert len(recs) == 52
    for r in recs:
        assert O.wildcard(r["pattern"], r["text"]) == r["matched"], r


def test_pattern_leaf_golden(golden):
    L = O.lib()
    L.oracle_leaf.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p]
    recs = golden("pattern_leaf.json")
    assert len(recs) >= 100
    for r in recs:
        got = L.oracle_leaf(r["fn"].encode(), r["value"].encode(), 1 if r.get("value_float") else 0,
                            r["pattern"].encode(), r.get("op", "").encode())
        assert got == int(r["expect"]), r


def _walk(entry, resource, pattern):
    L = O.lib()
    L.oracle_validate_entry.restype = ctypes.c_void_p
    return json.loads(O._take(L.oracle_validate_entry(entry.encode(), resource.encode(), pattern.encode(), 1)))


def test_validate_walk_golden(golden):
    recs = golden("validate_walk.json")
    n = 0
    for r in recs:
        if "status" in r:  # TestConditionalAnchorWithMultiplePatterns / Test_global_anchor
            out = O.match_pattern(r["resource"], r["pattern"])
            st = "pass" if out["ok"] else ("skip" if out["skip"] else ("error" if out["path"] == "" else "fail"))
            if r["status"] in ("pass", "skip"):
                assert st == r["status"], (r["test"], out)
            else:
                # the reference asserts nothing for Fail rows (validate_test.go:1663-1690); some rows are
                # labelled Fail although the code path is a global-anchor skip. Pin only "not pass".
                assert st != "pass", (r["test"], out)
            n += 1
            continue
        out = _walk(r["entry"], r["resource"], r["pattern"])
        if r["path"] is not None:
            assert out["path"] == r["path"], (r["test"], out)
        if r["err_nil"] is not None:
            assert (not out["err"]) == r["err_nil"], (r["test"], out)
        n += 1
    assert n == len(recs)


def test_engine_golden(golden):
    for r in golden("engine.json"):
        out = O.validate(json.loads(r["policy"]), r["resource"])
        rules = out[0]["rules"]
        sts = [x["status"] for x in rules]
        if "unsupported" in sts:
            continue  # variables / JMESPath: routed to the reference CPU engine, not this path
        if r.get("msgs") is not None:
            for i, x in enumerate(rules):
                assert x["message"] == r["msgs"][i], r["test"]
        if r.get("statuses") is not None:
            assert sts == r["statuses"], r["test"]
        if r.get("successful") is not None:
            assert (not any(s in ("fail", "error") for s in sts)) == r["successful"], r["test"]
        e = r.get("expect")
        if e == "failed":
            assert any(s == "fail" for s in sts), r["test"]
        elif e == "skipped":
            assert sts and all(s == "skip" for s in sts), r["test"]
        elif e == "success":
            assert not any(s in ("fail", "error") for s in sts), r["test"]


def test_pss_golden(golden):
    recs = golden("pss.json")
    assert len(recs) == 128
    for r in recs:
        out = O.pss(r["rule"], r["pod"])
        assert out["allowed"] == r["allowed"], r["name"]


def test_pss_kuttl_message():
    # test/conformance/kuttl/reports/background/test-report-background-mode/report-assert.yaml
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "podsecurity-subrule-restricted"},
           "spec": {"background": True, "validationFailureAction": "audit", "rules": [
               {"name": "restricted", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}}]}}
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "badpod01", "namespace": "default"},
           "spec": {"containers": [{"name": "container01", "image": "dummyimagename", "securityContext": {
               "allowPrivilegeEscalation": False, "runAsNonRoot": True, "seccompProfile": {"type": "RuntimeDefault"}}}]}}
    out = O.validate(pol, json.dumps(pod))
    r = out[0]["rules"][0]
    assert r["status"] == "fail"
    detail = 'ForbiddenDetail:container "container01" must set securityContext.capabilities.drop=["ALL"]'
    line = "({Allowed:false ForbiddenReason:unrestricted capabilities " + detail + "})\n"
    assert r["message"] == ("Validation rule 'restricted' failed. It violates PodSecurity \"restricted:latest\": " + line + line)


def cli_cases(golden):
    for d in golden("cli.json"):
        pols = {p["metadata"]["name"]: p for p in d["policies"] if isinstance(p, dict) and p.get("kind") in ("ClusterPolicy", "Policy")}
        for res in d["results"]:
            res = dict(res, result=res.get("result") or res.get("status"))  # newer kyverno-test.yaml: "status"
            if res.get("result") is None:
                continue
            pol = pols.get(res["policy"].split("/")[-1])
            if pol is None or any(r.get("mutate") or r.get("generate") for r in pol["spec"].get("rules", [])):
                continue
            if pol.get("kind") == "Policy" and not pol["metadata"].get("namespace"):
                continue  # `kyverno test` namespacing of a namespace-less Policy is not restated
            cands = [r for r in d["resources"] if isinstance(r, dict) and r.get("metadata", {}).get("name") == res["resource"]
                     and (not res.get("kind") or r.get("kind") == res["kind"])]
            if not cands:
                continue
            r = copy.deepcopy(cands[0])
            if not r["metadata"].get("namespace"):
                r["metadata"]["namespace"] = "default"  # fetch.go:310-312
            yield d["dir"], pol, r, res


def test_cli_golden(golden):
    n = 0
    for dname, pol, resource, res in cli_cases(golden):
        out = O.validate(pol, json.dumps(resource))
        rules = {x["name"]: x for x in out[0]["rules"]}
        rr = rules.get(res["rule"]) or rules.get("autogen-" + res["rule"]) or rules.get("autogen-cronjob-" + res["rule"])
        if rr and rr["status"] in ("unsupported", "panic"):
            continue
        st = rr["status"] if rr else "skip"
        if st == "fail" and pol["metadata"].get("annotations", {}).get("policies.kyverno.io/scored") == "false":
            st = "warn"
        assert st == res["result"], (dname, res)
        n += 1
    assert n >= 20


def test_conditions_golden(golden):
    """pkg/engine/variables/evaluate_test.go TestEvaluate: every (key, operator, value) -> bool case"""
    recs = golden("conditions.json")
    assert len(recs) >= 330
    for r in recs:
        assert O.condition(r["key"], r["operator"], r["value"]) == r["result"], r
