"""The typed pod decode of podSecurity rules (getSpec, pkg/engine/validation.go:481-532: json.Unmarshal of the
resource into corev1.Pod / appsv1.Deployment / batchv1.CronJob) beyond the fields the checks read: a type error in a
commonly set field -- env[].value / name / valueFrom, command / args items, workingDir, imagePullPolicy,
nodeSelector values, serviceAccountName, restartPolicy, terminationGracePeriodSeconds, activeDeadlineSeconds -- is a
decode error (rule status error), on the device as in the oracle's restatement (oracle/opss.cpp dec_pod,
oracle/otyped.cpp for the whole object). No reference fixture holds such an object (the API server rejects them):
parity unpinned beyond the restatement; keys no Go type declares are ignored on both sides."""
import copy

import pytest

import parity_util as PU
from kyverno_amd import _lib as K

POL = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "psa"},
       "spec": {"rules": [{"name": "restricted", "match": {"any": [{"resources": {"kinds": ["Pod", "Deployment", "CronJob"]}}]},
                           "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}}]}}

GOOD_C = {"name": "c", "image": "nginx", "securityContext": {"allowPrivilegeEscalation": False, "runAsNonRoot": True,
          "capabilities": {"drop": ["ALL"]}, "seccompProfile": {"type": "RuntimeDefault"}}}


def _pod(spec_extra=None, c_extra=None, kind="Pod"):
    c = dict(copy.deepcopy(GOOD_C), **(c_extra or {}))
    spec = dict({"containers": [c]}, **(spec_extra or {}))
    if kind == "Pod":
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "d"}, "spec": spec}
    if kind == "Deployment":
        return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "p", "namespace": "d"},
                "spec": {"template": {"metadata": {}, "spec": spec}}}
    return {"apiVersion": "batch/v1", "kind": "CronJob", "metadata": {"name": "p", "namespace": "d"},
            "spec": {"schedule": "* * * * *", "jobTemplate": {"spec": {"template": {"metadata": {}, "spec": spec}}}}}


def corpus():
    """(resource, expected device status) -- every case also compared with the oracle"""
    out = []
    for kind in ("Pod", "Deployment", "CronJob"):
        out += [
            (_pod(kind=kind), K.ST_PASS),
            (_pod(c_extra={"env": [{"name": "A", "value": 5}]}, kind=kind), K.ST_ERROR),
            (_pod(c_extra={"env": [{"name": 1, "value": "x"}]}, kind=kind), K.ST_ERROR),
            (_pod(c_extra={"env": [{"name": "A", "valueFrom": "x"}]}, kind=kind), K.ST_ERROR),
            (_pod(c_extra={"env": [{"name": "A", "value": None}, None]}, kind=kind), K.ST_PASS),
            (_pod(c_extra={"env": {"A": "b"}}, kind=kind), K.ST_ERROR),
            (_pod(c_extra={"command": ["sh", 1]}, kind=kind), K.ST_ERROR),
            (_pod(c_extra={"args": "x"}, kind=kind), K.ST_ERROR),
            (_pod(c_extra={"args": ["-v", None]}, kind=kind), K.ST_PASS),
            (_pod(c_extra={"workingDir": 3}, kind=kind), K.ST_ERROR),
            (_pod(c_extra={"imagePullPolicy": True}, kind=kind), K.ST_ERROR),
            (_pod(spec_extra={"nodeSelector": ["a"]}, kind=kind), K.ST_ERROR),
            (_pod(spec_extra={"nodeSelector": {"a": 1}}, kind=kind), K.ST_ERROR),
            (_pod(spec_extra={"nodeSelector": {"a": "b", "c": None}}, kind=kind), K.ST_PASS),
            (_pod(spec_extra={"serviceAccountName": 7}, kind=kind), K.ST_ERROR),
            (_pod(spec_extra={"restartPolicy": {}}, kind=kind), K.ST_ERROR),
            (_pod(spec_extra={"terminationGracePeriodSeconds": "30"}, kind=kind), K.ST_ERROR),
            (_pod(spec_extra={"terminationGracePeriodSeconds": 30, "activeDeadlineSeconds": 5}, kind=kind), K.ST_PASS),
            (_pod(spec_extra={"activeDeadlineSeconds": 1.5}, kind=kind), K.ST_ERROR),
            # the whole object is decoded (k8s_types.h, test_typed_decode.py): spec.hostname is a string field
            (_pod(spec_extra={"hostname": 5}, kind=kind), K.ST_ERROR),
            (_pod(spec_extra={"notAField": 5}, kind=kind), K.ST_PASS),  # unknown keys are ignored
        ]
    return out


def _check(backend):
    cases = corpus()
    docs = [d for d, _ in cases]
    st, res = PU.compare([POL], docs, None, backend=backend)
    assert st["nbad"] == 0, st["bad"]
    got = [int(res.status[0, i]) for i in range(len(docs))]
    want = [w for _, w in cases]
    assert got == want, [(i, K.STATUS_NAMES[g], K.STATUS_NAMES[w]) for i, (g, w) in enumerate(zip(got, want)) if g != w]


def test_typed_decode_errors_cpu():
    _check("cpu")


@pytest.mark.gpu
def test_typed_decode_errors_gpu():
    _check("gpu")
