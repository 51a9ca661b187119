"""autogen.ComputeRules (pkg/autogen/autogen.go:280-314, rule.go:73-319) pinned by pkg/autogen/autogen_test.go
(tests/golden/autogen.json): CanAutoGen / GetSupportedControllers decisions, autogen rule-name truncation at 63
characters, the computed rule count of a podSecurity policy; the library's compiled rules (its own autogen in
compiler.cpp) must carry exactly the oracle's computed validate-rule names."""
from kyverno_amd import engine as E
from oracle import oracle as O


def _validate_names(rules):
    return [r["name"] for r in rules if r.get("validate")]


def test_can_autogen_tables(golden):
    recs = golden("autogen.json")["controllers"]
    assert len(recs) >= 30
    for r in recs:
        names = [x["name"] for x in O.compute_rules(r["policy"])]
        generated = any(n.startswith("autogen-") for n in names)
        assert generated == (r["controllers"] != "none"), (r["test"], r["name"], names)
        lib = [x["name"] for x in E.Ruleset([r["policy"]]).rules]
        assert lib == _validate_names(O.compute_rules(r["policy"])), (r["test"], r["name"], lib)


def test_autogen_rule_name_truncation(golden):
    recs = golden("autogen.json")["rule_names"]
    assert len(recs) == 4
    for r in recs:
        pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "p"},
               "spec": {"rules": [{"name": r["rule"], "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                                   "validate": {"pattern": {"metadata": {"name": "?*"}}}}]}}
        want = {"autogen": "autogen-", "autogen-cronjob": "autogen-cronjob-"}[r["prefix"]]
        oracle_names = [x["name"] for x in O.compute_rules(pol)]
        lib_names = [x["name"] for x in E.Ruleset([pol]).rules]
        assert r["expected"] in oracle_names and r["expected"] in lib_names, (r, oracle_names, lib_names)
        assert len(r["expected"]) <= 63 and r["expected"].startswith(want)


def test_pod_security_rule_count(golden):
    for r in golden("autogen.json")["rule_counts"]:
        assert len(O.compute_rules(r["policy"])) == r["rules"]
        assert len(E.Ruleset([r["policy"]]).rules) == r["rules"]
