"""Whole-object typed decode of podSecurity rules (pkg/engine/validation.go:481-532 getSpec: a
json.Unmarshal of the whole resource into corev1.Pod, appsv1.Deployment -- every workload kind -- or batchv1.CronJob;
a type error anywhere is the rule's error status, :538-540).

A generated corpus sets ONE wrongly typed value per resource, for every field of the three target types tabled in
kyverno_amd/csrc/k8s_types.h (k8s.io/api v0.26.1 restated: PodSpec, Container, Volume and its sources,
PodSecurityContext, ObjectMeta, status, the Deployment / CronJob / Job specs ...), at the Pod, spec.template and
spec.jobTemplate.spec.template positions; each must be an error on both sides (the library's flattener + device,
the oracle's own decoder, oracle/otyped.cpp). Valid but unusual encodings (numbers as quantities, int-or-string
strings, RFC 3339 offsets and fractions, case-folded keys, unknown keys, nulls) must not be.

Parity unpinned: k8s.io/api and encoding/json are not vendored under /root/reference and no fixture there holds a
wrongly typed pod; the decode rules are restated from the published Go types and the encoding/json documentation."""
import copy
import os
import re

import numpy as np
import pytest

from kyverno_amd import _lib as K
from kyverno_amd import engine as E
import parity_util as PU

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRIM = {"s", "b", "i32", "i64", "q", "ios", "t", "any"}


def load_schema():
    """the k8s_types.h table (data) -> {struct: [(field, type text)]}, embedded bases promoted"""
    text = open(os.path.join(ROOT, "kyverno_amd", "csrc", "k8s_types.h")).read()
    body = text[text.index('R"(') + 3:text.index(')";')]
    decl = {}
    for line in body.strip().splitlines():
        m = re.match(r"(\w+)(?::(\w+))?\{(.*)\}$", line.strip())
        assert m, line
        fields = [tuple(f.split(":", 1)) for f in m.group(3).split()]
        decl[m.group(1)] = (m.group(2), fields)
    out = {}

    def build(n):
        if n not in out:
            base, fs = decl[n]
            out[n] = (build(base) if base else []) + fs
        return out[n]
    for n in decl:
        build(n)
    return out


# one wrong value per type (and a second for some): json.Unmarshal fails on each
WRONG = {"s": [5], "b": ["yes"], "i32": ["1", 2 ** 31], "i64": [1.5], "q": [True, "1.5.5"], "ios": [True],
         "t": ["yesterday", "2023-02-29T00:00:00Z"]}


def wrong_values(t):
    if t in WRONG:
        return WRONG[t]
    if t == "any":
        return []
    if t.startswith("["):
        return ["x"]
    if t.startswith("{"):
        return [7]
    return ["x"]  # a struct


def leaf_paths(S, tname, prefix=(), seen=()):
    """(path, type) for every field reachable from struct tname: struct fields by name, slice elements at index 0"""
    for f, t in S[tname]:
        p = prefix + (f,)
        yield p, t
        inner, q = t, p
        while inner.startswith("["):
            inner, q = inner[1:-1], q + (0,)
            if inner != t:
                yield q, inner
        if inner not in PRIM and not inner.startswith("{") and inner not in seen:
            yield from leaf_paths(S, inner, q, seen + (tname,))


def set_path(doc, path, value):
    cur = doc
    for i, k in enumerate(path):
        last = i == len(path) - 1
        nxt = None if last else path[i + 1]
        if isinstance(k, int):
            if not isinstance(cur, list):
                raise TypeError
            while len(cur) <= k:
                cur.append({} if not isinstance(nxt, int) else [])
            if last:
                cur[k] = value
            else:
                if not isinstance(cur[k], (dict, list)) or (isinstance(nxt, int) != isinstance(cur[k], list)):
                    cur[k] = [] if isinstance(nxt, int) else {}
                cur = cur[k]
        else:
            if last:
                cur[k] = value
            else:
                if not isinstance(cur.get(k), (dict, list)) or (isinstance(nxt, int) != isinstance(cur.get(k), list)):
                    cur[k] = [] if isinstance(nxt, int) else {}
                cur = cur[k]


def pod_spec():
    return {"containers": [{"name": "app", "image": "registry.example.com/app:1.0",
                            "ports": [{"containerPort": 8080, "protocol": "TCP"}],
                            "resources": {"limits": {"cpu": "500m", "memory": "128Mi"}},
                            "securityContext": {"allowPrivilegeEscalation": False, "runAsNonRoot": True}}],
            "volumes": [{"name": "data", "emptyDir": {}}]}


def bases():
    meta = {"name": "x", "namespace": "default", "labels": {"app": "x"}}
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": dict(meta), "spec": pod_spec()}
    dep = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": dict(meta),
           "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "x"}},
                    "template": {"metadata": {"labels": {"app": "x"}}, "spec": pod_spec()}}}
    cj = {"apiVersion": "batch/v1", "kind": "CronJob", "metadata": dict(meta),
          "spec": {"schedule": "*/5 * * * *", "jobTemplate": {"spec": {"template": {"spec": pod_spec()}}}}}
    return {"Pod": pod, "Deployment": dep, "CronJob": cj}


def wrong_corpus():
    S = load_schema()
    docs, where = [], []
    for root, base in bases().items():
        for path, t in leaf_paths(S, root):
            if path[0] in ("kind", "apiVersion"):
                continue  # they decide the rule's match, not only the decode
            for w in wrong_values(t):
                d = copy.deepcopy(base)
                try:
                    set_path(d, path, w)
                except TypeError:
                    continue
                docs.append(d)
                where.append((root, ".".join(map(str, path)), repr(w)))
    return docs, where


def valid_corpus():
    """unusual but valid encodings (no decode error), plus the workload kinds decoded as a Deployment"""
    b = bases()
    out = []

    def pod(mut):
        d = copy.deepcopy(b["Pod"])
        mut(d)
        d["metadata"]["name"] = "v%d" % len(out)
        out.append(d)
    c = lambda d: d["spec"]["containers"][0]
    pod(lambda d: c(d)["resources"].update({"limits": {"cpu": 1, "memory": 1.5e9}, "requests": {"cpu": " 250m "}}))
    pod(lambda d: c(d).update({"livenessProbe": {"httpGet": {"port": "http", "path": "/"}},
                               "readinessProbe": {"tcpSocket": {"port": 8080}}}))
    pod(lambda d: d["metadata"].update({"creationTimestamp": "2024-02-29T3:04:05.123+05:30"}))
    pod(lambda d: d["metadata"].update({"creationTimestamp": None, "deletionTimestamp": "2023-01-02T03:04:05,5Z"}))
    pod(lambda d: d["spec"].update({"HostNetwork": False, "unknownField": {"x": [1, "y"]}}))
    pod(lambda d: d["spec"].update({"securityContext": None, "affinity": None, "os": None}))
    pod(lambda d: d.update({"status": {"phase": "Running", "startTime": "2023-05-06T07:08:09Z",
                                       "containerStatuses": [{"name": "app", "ready": True, "restartCount": 0,
                                                              "state": {"running": {"startedAt": "2023-05-06T07:08:10Z"}}}]}}))
    pod(lambda d: d["metadata"].update({"managedFields": [{"manager": "m", "fieldsV1": {"f:spec": {}}}]}))
    pod(lambda d: d["spec"]["volumes"].append({"name": "q", "emptyDir": {"sizeLimit": 1024}}))
    for kind in ("Job", "DaemonSet", "StatefulSet", "ReplicaSet"):
        d = copy.deepcopy(b["Deployment"])
        d["kind"] = kind
        d["apiVersion"] = "batch/v1" if kind == "Job" else "apps/v1"
        if kind == "Job":
            d["spec"].update({"completions": 3, "backoffLimit": 2})
            d["status"] = {"startTime": "2023-01-01T00:00:00Z", "conditions": [
                {"type": "Complete", "status": "True", "lastProbeTime": "2023-01-01T00:00:00Z"}]}
        if kind == "StatefulSet":
            d["spec"]["volumeClaimTemplates"] = [{"metadata": {"name": "x"}}]
        d["metadata"]["name"] = "v%d" % len(out)
        out.append(d)
    rc = copy.deepcopy(b["Deployment"])
    rc.update({"kind": "ReplicationController", "apiVersion": "v1"})
    rc["spec"]["selector"] = {"app": "x"}  # map[string]string in core/v1: unknown keys of the LabelSelector struct
    rc["metadata"]["name"] = "v%d" % len(out)
    out.append(rc)
    return out


def pss_policy():
    kinds = ["Pod", "Deployment", "CronJob", "Job", "DaemonSet", "StatefulSet", "ReplicaSet", "ReplicationController"]
    return [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "pss-typed"},
             "spec": {"validationFailureAction": "Audit", "background": True, "rules": [{
                 "name": "baseline", "match": {"any": [{"resources": {"kinds": kinds}}]},
                 "validate": {"podSecurity": {"level": "baseline", "version": "latest"}}}]}}]


def _check(backend, jit=None):
    wrong, where = wrong_corpus()
    valid = valid_corpus()
    docs = wrong + valid
    pols = pss_policy()
    st, res = PU.compare(pols, docs, {}, backend=backend, jit=jit)
    assert st["nbad"] == 0, st["bad"]
    status = np.asarray(res.status)[0] & 7
    # verdict columns are in input order
    not_err = [where[i] for i in range(len(wrong)) if status[i] != K.ST_ERROR]
    assert not not_err, not_err[:20]
    errs = [docs[len(wrong) + j]["metadata"]["name"] for j in range(len(valid)) if status[len(wrong) + j] == K.ST_ERROR]
    assert not errs, errs
    return len(wrong)


def test_typed_decode_corpus_cpu():
    n = _check("cpu")
    assert n > 1500  # every field of Pod / Deployment / CronJob, some twice


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [False, True])
def test_typed_decode_corpus_gpu(jit):
    _check("gpu", jit=jit)


def test_review_examples_are_errors():
    """the four examples named in the round-3 review: spec.hostname 5, spec.dnsPolicy [], a container port's protocol
    1, a secret volume's defaultMode "x" """
    b = bases()["Pod"]
    docs = []
    for path, w in [(("spec", "hostname"), 5), (("spec", "dnsPolicy"), []),
                    (("spec", "containers", 0, "ports", 0, "protocol"), 1),
                    (("spec", "volumes", 0, "secret", "defaultMode"), "x")]:
        d = copy.deepcopy(b)
        set_path(d, path, w)
        d["metadata"]["name"] = "e%d" % len(docs)
        docs.append(d)
    st, res = PU.compare(pss_policy(), docs, {}, backend="cpu")
    assert st["nbad"] == 0, st["bad"]
    assert set((np.asarray(res.status)[0] & 7).tolist()) == {K.ST_ERROR}


@pytest.mark.parametrize("backend", ["cpu"])
def test_case_folded_key_goes_back_to_the_caller(backend):
    """encoding/json matches `HostNetwork` to hostNetwork (case-insensitive fallback); the PodSecurity checks read
    exact keys, so such a resource's PodSecurity pairs are handed back (ST_FALLBACK; the oracle: not restated)"""
    d = copy.deepcopy(bases()["Pod"])
    d["spec"]["HostNetwork"] = True
    st, res = PU.compare(pss_policy(), [d], {}, backend=backend)
    assert st["nbad"] == 0, st["bad"]
    assert int(res.status[0, 0]) & 7 == K.ST_FALLBACK
