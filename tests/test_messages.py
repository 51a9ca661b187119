"""Rule messages with variables (RuleResponse.Message).

- pattern rules: buildErrorMessage substitutes the message's variables (validation.go:722-745) -- the reference's own
  fixture test/cli/test/mixed/policy.yaml:21 (`{{ request.object.metadata.namespace }} pods must be managed by
  open-ondemand`) has this shape; rendered on the host from the resource (capi.cpp subst_message);
- anyPattern rules take the message as written (buildAnyPatternErrorMessage, validation.go:747-758);
- PodSecurity responses do not use the message (validation.go:560-566);
- a reference that does not resolve makes buildErrorMessage embed the Go error string: the device leaves that text to
  the reference engine (message None), the oracle marks it unpinned.
Every verdict, path and rendered message against the oracle (host instantiation here, the kernels under -m gpu)."""
import pytest

import parity_util as PU


def _pol(name, rules):
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
            "spec": {"validationFailureAction": "Audit", "background": True, "rules": rules}}


def policies():
    pod = {"any": [{"resources": {"kinds": ["Pod"]}}]}
    return [
        _pol("ondemand", [{  # test/cli/test/mixed/policy.yaml:12-24
            "name": "ondemand-managed_by",
            "match": {"any": [{"resources": {"kinds": ["Pod"], "namespaces": ["user-?*"]}}]},
            "validate": {"message": "{{ request.object.metadata.namespace }} pods must be managed by open-ondemand",
                         "pattern": {"metadata": {"labels": {"app.kubernetes.io/managed-by": "open-ondemand"}}}}}]),
        _pol("whole-var", [{
            "name": "name-message", "match": pod,
            "validate": {"message": "{{request.object.metadata.name}}",
                         "pattern": {"spec": {"containers": [{"image": "!*:latest"}]}}}}]),
        _pol("typed-vars", [{
            "name": "typed", "match": pod,
            "validate": {"message": "replicas {{request.object.spec.priority}} host {{request.object.spec.hostNetwork}} "
                                    "label {{request.object.metadata.labels.tier}}.",
                         "pattern": {"metadata": {"labels": {"tier": "frontend | backend"}}}}}]),
        _pol("missing-var", [{
            "name": "missing", "match": pod,
            "validate": {"message": "owner {{request.object.metadata.labels.owner}} is not allowed",
                         "pattern": {"metadata": {"labels": {"team": "?*"}}}}}]),
        _pol("any-raw", [{
            "name": "any-message", "match": pod,
            "validate": {"message": "pod {{request.object.metadata.name}} needs a tier",
                         "anyPattern": [{"metadata": {"labels": {"tier": "frontend"}}},
                                        {"metadata": {"labels": {"tier": "backend"}}}]}}]),
        _pol("pss-message", [{
            "name": "baseline", "match": pod,
            "validate": {"message": "{{request.object.metadata.name}} violates baseline",
                         "podSecurity": {"level": "baseline", "version": "latest"}}}]),
    ]


def pods(n=240):
    out = []
    for i in range(n):
        labels = {}
        if i % 4 == 0:
            labels["app.kubernetes.io/managed-by"] = "open-ondemand"
        if i % 4:
            labels["tier"] = ["frontend", "backend", "data"][i % 3]
        if i % 5 == 0:
            labels["owner"] = "team-%d" % (i % 7)
        if i % 6 == 0:
            labels["team"] = "t%d" % i
        spec = {"containers": [{"name": "c", "image": "nginx:latest" if i % 2 else "nginx:1.25"}]}
        if i % 7 == 0:  # both typed fields of the "typed" message present
            spec["priority"] = i * 10
            spec["hostNetwork"] = bool(i % 2)
        if i % 11 == 0:
            spec["containers"][0]["securityContext"] = {"privileged": True}
        out.append({"apiVersion": "v1", "kind": "Pod",
                    "metadata": {"name": "pod-%d" % i, "namespace": ["user-%d" % (i % 5), "default", "user-"][i % 3],
                                 "labels": labels},
                    "spec": spec})
    return out


def _check(backend):
    pols, docs = policies(), pods()
    st, res = PU.compare(pols, docs, backend=backend)
    assert st["nbad"] == 0, st["bad"]
    return st, res


def test_variable_messages_cpu_instantiation():
    st, res = _check("cpu")
    assert st["messages"] > 500
    msgs = {}
    import numpy as np
    from kyverno_amd import _lib as K
    fails = np.argwhere(res.status == K.ST_FAIL)
    for k, r in fails:
        m = res.message(int(r), int(k))
        msgs.setdefault(int(k), []).append(m)
    flat = [m for v in msgs.values() for m in v if m]
    # substituted pattern message (the mixed fixture's shape)
    assert any(m.startswith("validation error: user-") and "pods must be managed by open-ondemand. rule "
               "ondemand-managed_by failed at path /metadata/labels/" in m for m in flat), flat[:5]
    # whole-message variable: the resource name, then the trailing '.'
    assert any(m.startswith("validation error: pod-") and ". rule name-message failed at path" in m for m in flat)
    # typed values: a number and a boolean in the substituted text
    assert any(m.startswith("validation error: replicas ") and " host true label " in m for m in flat)
    # anyPattern keeps the raw message
    assert any(m.startswith("validation error: pod {{request.object.metadata.name}} needs a tier.") for m in flat)
    # PodSecurity ignores the message
    assert any(m.startswith("Validation rule 'baseline' failed. It violates PodSecurity") for m in flat)


@pytest.mark.gpu
def test_variable_messages_gpu():
    st, _ = _check("gpu")
    assert st["messages"] > 500
