"""foreach validation with patterns: foreach entries whose validator is a pattern / anyPattern
(element-scoped or not, element variables substituted as typed values), nested foreach, preconditions and
elementScope, evaluated by the library (host instantiation here, the MI355X in the -m gpu tests) against the oracle's
restatement of validateForEach / validateElements (pkg/engine/validation.go:242-421), pair by pair.

The reference's own fixture (test/cli/test/foreach/policies.yaml) filters its list with a JMESPath filter expression
(`volumes[?contains(keys(@), 'emptyDir')]`): its two policies are here verbatim (fe-fixture-*), over a corpus whose
containers mount the pods' volumes, plus ==/!= filters and a filter with a projection after it; the fixture's own
resources and verdicts are checked in test_foreach_fixture_* (tests/golden/cli.json)."""
import copy

import numpy as np
import pytest

from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from kyverno_amd import synth
import parity_util as PU


def _pol(name, fe, message="foreach check failed", kinds=("Pod",)):
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
            "spec": {"validationFailureAction": "Audit", "background": True, "rules": [{
                "name": name + "-r", "match": {"any": [{"resources": {"kinds": list(kinds)}}]},
                "validate": {"message": message, "foreach": fe}}]}}


def foreach_pattern_policies():
    C = "request.object.spec.containers"
    return [
        # element-scoped pattern (containers are maps)
        _pol("fe-image", [{"list": C, "pattern": {"image": "!*:latest"}}]),
        _pol("fe-image-init", [{"list": "request.object.spec.initContainers", "pattern": {"image": "registry.example.com/*"}}]),
        # anyPattern per element
        _pol("fe-any", [{"list": C, "anyPattern": [{"securityContext": {"runAsNonRoot": True}},
                                                  {"securityContext": {"allowPrivilegeEscalation": False}}]}]),
        # elements that are strings: not element-scoped, the pattern validates the resource
        _pol("fe-strings", [{"list": C + "[].name", "pattern": {"metadata": {"labels": {"app": "?*"}}}}]),
        # elementScope false + a string element variable (the reference fixture's shape without its filter)
        _pol("fe-var", [{"list": C, "elementScope": False, "pattern": {"spec": {"containers": [
            {"(name)": "{{element.name}}", "image": "registry.example.com/*"}]}}}]),
        # an element variable under a conditional anchor, a bool variable, and one whose key can be missing
        _pol("fe-var-bool", [{"list": C, "elementScope": False, "pattern": {"spec": {"containers": [
            {"(name)": "{{ element.name }}", "=(securityContext)": {"=(runAsNonRoot)": "{{element.securityContext.runAsNonRoot}}"}}]}}}]),
        # nested foreach: the ports of every container (integers are float64 in the element)
        _pol("fe-nested", [{"list": C, "foreach": [{"list": "element.ports", "pattern": {"containerPort": "<8081"}}]}]),
        _pol("fe-nested-deny", [{"list": C, "foreach": [{"list": "element.ports", "deny": {"conditions": {"any": [
            {"key": "{{element.containerPort}}", "operator": "GreaterThan", "value": 8080}]}}}]}]),
        # elementScope true over non-map elements: the addElementToContext error
        _pol("fe-scope-err", [{"list": C + "[].image", "elementScope": True, "pattern": {"x": "y"}}]),
        # per-element preconditions + pattern, and an entry without a validator
        _pol("fe-pre", [{"list": C, "preconditions": {"any": [{"key": "{{element.name}}", "operator": "Equals",
                                                               "value": "c0"}]},
                         "pattern": {"securityContext": {"allowPrivilegeEscalation": False}}},
                        {"list": C}]),
        # elementIndex as a number pattern; entries mixing deny and pattern
        _pol("fe-index", [{"list": C, "pattern": {"=(terminationGracePeriod)": "{{elementIndex}}", "name": "{{elementIndex}}"}},
                          {"list": C, "deny": {"conditions": {"any": [{"key": "{{element.image}}", "operator": "Equals",
                                                                         "value": "nginx:latest"}]}}}]),
        # a controller kind: containers under spec.template.spec, and resources without the list (entry skipped)
        _pol("fe-deploy", [{"list": "request.object.spec.template.spec.containers",
                            "pattern": {"resources": {"limits": {"memory": "?*"}}}}], kinds=("Deployment", "Pod")),
        # filter projections: the reference fixture's two policies (test/cli/test/foreach/policies.yaml) ...
        _pol("fe-fixture-mountpath", [{"list": "request.object.spec.volumes[?contains(keys(@), 'emptyDir')]",
                                       "elementScope": False, "pattern": {"spec": {"containers": [
                                           {"name": "*", "volumeMounts": [{"(name)": "{{element.name}}",
                                                                           "mountPath": "/tmp/*"}]}]}}}],
             message="emptyDir volumes must be mounted under /tmp"),
        _pol("fe-fixture-resources", [{"list": "request.object.spec.volumes[?contains(keys(@), 'emptyDir')]",
                                       "elementScope": False, "pattern": {"spec": {"containers": [
                                           {"volumeMounts": [{"<(name)": "{{element.name}}"}],
                                            "resources": {"requests": {"ephemeral-storage": "?*"},
                                                          "limits": {"ephemeral-storage": "?*"}}}]}}}],
             message="ephemeral-storage requests and limits are required for emptyDir volumes"),
        # ... equality filters on a field chain (string / boolean literals), and a projection after the filter
        _pol("fe-filter-eq", [{"list": "request.object.spec.containers[?name == 'c0']",
                               "pattern": {"securityContext": {"runAsNonRoot": True}}}]),
        _pol("fe-filter-ne", [{"list": "request.object.spec.containers[?securityContext.privileged != `true`].image",
                               "deny": {"conditions": {"any": [{"key": "{{element}}", "operator": "Equals",
                                                                "value": "*:latest"}]}}}]),
        _pol("fe-filter-keys", [{"list": "request.object.spec.volumes[?contains(keys(@), 'hostPath')].hostPath.path",
                                 "deny": {"conditions": {"any": [{"key": "{{element}}", "operator": "Equals",
                                                                  "value": "/var/run/docker.sock"}]}}}]),
    ]


def with_mounts(docs, seed):
    """the corpus with volumeMounts on the pods' containers (mount paths under /tmp or not, some mounts missing),
    ephemeral-storage resources on some containers, and now and then a volume list holding a non-map element (the
    filter's keys() type error: the reference skips the entry)"""
    import random
    rng = random.Random(seed)
    out = copy.deepcopy(docs)
    for d in out:
        spec = d.get("spec")
        if isinstance(spec, dict) and isinstance(spec.get("template"), dict):
            spec = spec["template"].get("spec")
        if not isinstance(spec, dict):
            continue
        vols = spec.get("volumes")
        if not isinstance(vols, list):
            continue
        for c in spec.get("containers") or []:
            if not isinstance(c, dict):
                continue
            mounts = [{"name": v.get("name"), "mountPath": rng.choice(["/tmp/" + str(v.get("name")), "/data", "/tmp"])}
                      for v in vols if isinstance(v, dict) and rng.random() < 0.8]
            if mounts:
                c["volumeMounts"] = mounts
            if rng.random() < 0.5:
                res = c.setdefault("resources", {}) if isinstance(c.get("resources", {}), dict) else {}
                res.setdefault("requests", {})["ephemeral-storage"] = "1Gi"
                if rng.random() < 0.7:
                    res.setdefault("limits", {})["ephemeral-storage"] = "2Gi"
        if rng.random() < 0.02:
            vols.append(rng.choice(["bad-volume", 7, None]))
    return out


@pytest.mark.parametrize("backend", ["cpu"])
def test_foreach_patterns_vs_oracle(backend):
    pols = foreach_pattern_policies()
    rs = E.Ruleset(pols)
    fb = [(r["name"], r["reason"]) for r in rs.rules if r["kind"] == "fallback"]
    assert not fb, fb  # every shape above compiles to the device
    docs, nsl = synth.mixed(3000, seed=71, edge=True)
    docs = with_mounts(docs, 71)
    st, res = PU.compare(pols, docs, nsl, backend=backend)
    assert st["nbad"] == 0, st["bad"]
    assert st["compared"] > 3000
    counts = res.counts
    assert counts["pass"] > 0 and counts["fail"] > 0 and counts["skip"] > 0 and counts["error"] > 0
    # every filter policy decides both ways on this corpus
    status = np.asarray(res.status)
    for k, rule in enumerate(rs.rules):
        if rule["name"].startswith(("fe-fixture", "fe-filter")):
            vals = set((status[k] & 7).tolist())
            assert K.ST_PASS in vals and K.ST_FAIL in vals, (rule["name"], vals)


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [False, True])
def test_foreach_patterns_gpu_vs_oracle(jit):
    """the same corpus through the device: the interpreted match kernel and (jit) the compiled condition kernels"""
    pols = foreach_pattern_policies()
    docs, nsl = synth.mixed(20000, seed=72, edge=True)
    docs = with_mounts(docs, 72)
    st, res = PU.compare(pols, docs, nsl, backend="gpu", jit=jit)
    assert st["nbad"] == 0, st["bad"]
    assert st["compared"] > 20000
    assert res.counts["fallback"] == 0


def nested_policies():
    """foreach nested two and three levels deep (newForEachValidator(..., nesting+1), validation.go:360 -- the
    reference recurses without limit; the device compiles up to FOREACH_MAX_NEST levels below the top), and one four
    levels deep, which stays on the CPU engine"""
    C = "request.object.spec.containers"
    mounts_tmp = {"list": "element.mountPath", "pattern": {"mountPath": "/tmp/*"}}
    vol_deny = {"list": "request.object.spec.volumes", "deny": {"conditions": {"any": [
        {"key": "{{element.name}}", "operator": "AnyIn", "value": ["host*", "vol2"]}]}}}
    return [
        # containers -> their mounts -> the mount path (a string: not element-scoped, the pattern validates the mount)
        _pol("fe-nest2", [{"list": C, "foreach": [{"list": "element.volumeMounts", "foreach": [mounts_tmp]}]}]),
        # ... -> the pod's volumes (a list from the resource root at the third level), deny per volume
        _pol("fe-nest3", [{"list": C, "foreach": [{"list": "element.volumeMounts", "foreach": [
            {"list": "element.mountPath", "foreach": [vol_deny]}]}]}]),
        # mixed entries: a nested level beside a pattern entry, preconditions inside the nesting
        _pol("fe-nest2-mixed", [{"list": C, "pattern": {"name": "?*"}},
                                {"list": C, "foreach": [{"list": "element.volumeMounts",
                                                         "preconditions": {"all": [{"key": "{{element.name}}",
                                                                                    "operator": "NotEquals",
                                                                                    "value": "v0"}]},
                                                         "foreach": [mounts_tmp]}]}]),
        # four levels below the top: beyond the compiled depth (CPU engine)
        _pol("fe-nest4", [{"list": C, "foreach": [{"list": "element.volumeMounts", "foreach": [
            {"list": "element.mountPath", "foreach": [{"list": "request.object.spec.volumes", "foreach": [
                {"list": "element.name", "pattern": {"name": "?*"}}]}]}]}]}]),
    ]


def test_foreach_nesting_vs_oracle():
    pols = nested_policies()
    rs = E.Ruleset(pols)
    fb = {r["name"]: r["reason"] for r in rs.rules if r["kind"] == "fallback"}
    assert fb and all(n.endswith("fe-nest4-r") for n in fb), fb  # (with its autogen rules)
    docs, nsl = synth.mixed(3000, seed=73, edge=True)
    docs = with_mounts(docs, 73)
    st, res = PU.compare(pols, docs, nsl, backend="cpu")
    assert st["nbad"] == 0, st["bad"]
    status = np.asarray(res.status)
    for k, rule in enumerate(rs.rules):
        if not rule["name"].endswith("fe-nest4-r") and rule["name"].startswith("fe-"):
            vals = set((status[k] & 7).tolist())
            assert K.ST_PASS in vals and K.ST_FAIL in vals, (rule["name"], vals)


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [False, True])
def test_foreach_nesting_gpu_vs_oracle(jit):
    pols = nested_policies()
    docs, nsl = synth.mixed(20000, seed=74, edge=True)
    docs = with_mounts(docs, 74)
    st, res = PU.compare(pols, docs, nsl, backend="gpu", jit=jit)
    assert st["nbad"] == 0, st["bad"]
    assert st["compared"] > 20000
