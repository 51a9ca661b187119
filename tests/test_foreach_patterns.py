"""foreach validation with patterns: foreach entries whose validator is a pattern / anyPattern
(element-scoped or not, element variables substituted as typed values), nested foreach, preconditions and
elementScope, evaluated by the library (host instantiation here, the MI355X in the -m gpu tests) against the oracle's
restatement of validateForEach / validateElements (pkg/engine/validation.go:242-421), pair by pair.

The reference's own fixture (test/cli/test/foreach/policies.yaml) additionally filters its list with a JMESPath filter
expression; the same shapes without the filter are here, and the fixture's policies themselves are checked in
test_foreach_fixture_* (tests/golden/cli.json)."""
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
    ]


@pytest.mark.parametrize("backend", ["cpu"])
def test_foreach_patterns_vs_oracle(backend):
    pols = foreach_pattern_policies()
    rs = E.Ruleset(pols)
    fb = [(r["name"], r["reason"]) for r in rs.rules if r["kind"] == "fallback"]
    assert not fb, fb  # every shape above compiles to the device
    docs, nsl = synth.mixed(3000, seed=71, edge=True)
    st, res = PU.compare(pols, docs, nsl, backend=backend)
    assert st["nbad"] == 0, st["bad"]
    assert st["compared"] > 3000
    counts = res.counts
    assert counts["pass"] > 0 and counts["fail"] > 0 and counts["skip"] > 0 and counts["error"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [False, True])
def test_foreach_patterns_gpu_vs_oracle(jit):
    """the same corpus through the device: the interpreted match kernel and (jit) the compiled condition kernels"""
    pols = foreach_pattern_policies()
    docs, nsl = synth.mixed(20000, seed=72, edge=True)
    st, res = PU.compare(pols, docs, nsl, backend="gpu", jit=jit)
    assert st["nbad"] == 0, st["bad"]
    assert st["compared"] > 20000
    assert res.counts["fallback"] == 0
