"""Parity corpora built from the golden fixtures (tests/golden) and the synthetic generator."""
import copy
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def load(name):
    with open(os.path.join(HERE, "golden", name)) as f:
        return json.load(f)


def best_practices():
    return [r["policy"] for r in load("best_practices.json")]


def chart_restricted():
    return [r["policy"] for r in load("chart_restricted.json")]


def engine_cases():
    """(policies, resources) pairs from pkg/engine/validation_test.go."""
    out = []
    for r in load("engine.json"):
        out.append(([json.loads(r["policy"])], [json.loads(r["resource"])]))
    return out


def cli_cases():
    """(policies, resources) per test/cli/test directory (namespace defaulted like fetch.go:310-312)."""
    out = []
    for d in load("cli.json"):
        pols = [p for p in d["policies"] if isinstance(p, dict) and p.get("kind") in ("ClusterPolicy", "Policy")]
        res = []
        for r in d["resources"]:
            if not isinstance(r, dict):
                continue
            r = copy.deepcopy(r)
            md = r.setdefault("metadata", {})
            if isinstance(md, dict) and not md.get("namespace"):
                md["namespace"] = "default"
            res.append(r)
        if pols and res:
            out.append((d["dir"], pols, res))
    return out


def walk_policy_cases():
    """Each pattern of pkg/engine/validate/validate_test.go wrapped in a ClusterPolicy rule (kinds: *)."""
    pols, res = [], []
    for i, r in enumerate(load("validate_walk.json")):
        try:
            pat = json.loads(r["pattern"])
            rsrc = json.loads(r["resource"])
        except ValueError:
            continue
        if not isinstance(rsrc, dict):
            continue
        pols.append({"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "walk-%d" % i},
                     "spec": {"rules": [{"name": "r", "match": {"any": [{"resources": {"kinds": ["*"]}}]},
                                         "validate": {"pattern": pat}}]}})
        res.append(rsrc)
    return pols, res


def pss_cases():
    """pkg/pss/evaluate_test.go rules as podSecurity rules, each paired with its pod."""
    out = []
    for i, r in enumerate(load("pss.json")):
        rule = json.loads(r["rule"])
        pod = json.loads(r["pod"])
        pod.setdefault("kind", "Pod")
        pod.setdefault("apiVersion", "v1")
        pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "pss-%d" % i},
               "spec": {"rules": [{"name": "pss", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                                   "validate": {"podSecurity": rule}}]}}
        out.append((r["name"], pol, pod, r["allowed"]))
    return out


def quirk_policies():
    """Hand-written rules exercising anchors, existence, global/conditional skips, anyPattern skips,
    ranges/quantities/durations and match filters (selectors, namespaces, annotations, exclude)."""
    def pol(name, rules, **meta):
        return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": dict(name=name, **meta),
                "spec": {"validationFailureAction": "audit", "rules": rules}}
    pod_any = {"any": [{"resources": {"kinds": ["Pod"]}}]}
    return [
        pol("cond-image", [{"name": "latest-needs-always", "match": pod_any, "validate": {"pattern": {"spec": {"containers": [
            {"(image)": "*:latest", "imagePullPolicy": "Always"}]}}}}]),
        pol("global-image", [{"name": "g", "match": pod_any, "validate": {"pattern": {"spec": {"containers": [
            {"name": "*", "<(image)": "*:latest", "imagePullPolicy": "!Always"}]}}}}]),
        pol("neg-hostpath", [{"name": "n", "match": pod_any, "validate": {"pattern": {"spec": {"=(volumes)": [{"X(hostPath)": "null"}]}}}}]),
        pol("exist-ports", [{"name": "e", "match": pod_any, "validate": {"pattern": {"spec": {"containers": [
            {"^(ports)": [{"containerPort": ">=80 & <9000"}]}]}}}}]),
        pol("mem-range", [{"name": "m", "match": pod_any, "validate": {"pattern": {"spec": {"containers": [
            {"=(resources)": {"=(limits)": {"=(memory)": "64Mi-1Gi"}}}]}}}}]),
        pol("cpu-notrange", [{"name": "c", "match": pod_any, "validate": {"pattern": {"spec": {"containers": [
            {"=(resources)": {"=(requests)": {"=(cpu)": "200m!-800m"}}}]}}}}]),
        pol("any-owner", [{"name": "a", "match": {"any": [{"resources": {"kinds": ["Pod", "Deployment"]}}]}, "validate": {"anyPattern": [
            {"metadata": {"labels": {"owner": "?*"}}}, {"metadata": {"labels": {"(tier)": "backend", "app": "*"}}}]}}]),
        pol("sel-team", [{"name": "s", "match": {"any": [{"resources": {"kinds": ["Pod"], "selector": {"matchLabels": {"tier": "fr*"}}}}]},
                          "exclude": {"any": [{"resources": {"namespaces": ["ns-00?1", "ns-01*"]}}]},
                          "validate": {"pattern": {"metadata": {"labels": {"app": "app-*"}}}}}]),
        pol("nssel", [{"name": "ns", "match": {"any": [{"resources": {"kinds": ["Pod"], "namespaceSelector": {"matchExpressions": [
            {"key": "env", "operator": "In", "values": ["prod"]}]}}}]}, "validate": {"pattern": {"spec": {"containers": [
                {"securityContext": {"runAsNonRoot": True}}]}}}}]),
        pol("star-kind", [{"name": "sk", "match": {"any": [{"resources": {"kinds": ["*"]}}]},
                           "exclude": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                           "validate": {"pattern": {"metadata": {"name": "?*"}}}}]),
        pol("ann-match", [{"name": "am", "match": {"all": [{"resources": {"kinds": ["Pod"], "annotations": {"example.com/a*": "value-1*"}}}]},
                           "validate": {"pattern": {"spec": {"=(hostNetwork)": False}}}}]),
        pol("user-run", [{"name": "u", "match": pod_any, "validate": {"pattern": {"spec": {"=(securityContext)": {"=(runAsUser)": ">0"},
                          "containers": [{"=(securityContext)": {"=(runAsUser)": ">0"}}]}}}}]),
        pol("exact-num", [{"name": "x", "match": pod_any, "validate": {"pattern": {"spec": {"containers": [
            {"=(ports)": [{"containerPort": 80}]}]}}}}]),
        pol("nil-pat", [{"name": "np", "match": pod_any, "validate": {"pattern": {"spec": {"=(hostPID)": None}}}}]),
        pol("star-field", [{"name": "sf", "match": pod_any, "validate": {"pattern": {"spec": {"containers": [{"resources": {"limits": "*"}}]}}}}]),
        pol("pss-restricted", [{"name": "restricted", "match": pod_any, "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}}]),
        pol("pss-baseline-excl", [{"name": "baseline", "match": pod_any, "validate": {"podSecurity": {"level": "baseline", "version": "v1.24",
            "exclude": [{"controlName": "Host Namespaces"}, {"controlName": "Capabilities", "images": ["registry.example.com/team1*"]}]}}}]),
    ]
