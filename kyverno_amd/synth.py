"""Seeded synthetic Kubernetes resources (SURVEY.md 8(d) Pod model / mixed-kind model).

Used by tests (parity corpora) and bench.py (workload). Not part of the evaluation path.
`edge=True` mixes in the quirks the reference handles specially (nulls, wrong JSON types, numbers where
strings are expected, float values, empty maps) so parity covers them.
"""
import json
import random

SEED = 0x4B59564E

QTY = ["100m", "0.5", "1", "250m", "64Mi", "256Mi", "1Gi", "1.5Gi", "2G"]
CAPS_ADD = ["NET_BIND_SERVICE", "SYS_ADMIN", "CHOWN", "NET_RAW"]
SYSCTL_OK = ["kernel.shm_rmid_forced", "net.ipv4.ip_local_port_range", "net.ipv4.tcp_syncookies"]
SYSCTL_BAD = ["kernel.msgmax", "net.core.somaxconn"]
VOL_TYPES = ["configMap", "secret", "emptyDir", "persistentVolumeClaim", "projected", "downwardAPI", "csi", "nfs",
             "gitRepo"]


class Gen:
    def __init__(self, seed=SEED, edge=False, namespaces=1000):
        self.r = random.Random(seed)
        self.edge = edge
        self.namespaces = ["ns-%04d" % i for i in range(namespaces)]
        self.repos = ["registry.example.com/team%d/app%d" % (i % 50, i) for i in range(2000)]

    def p(self, x):
        return self.r.random() < x

    def ns_labels(self):
        rr = random.Random(SEED ^ 0x55)
        out = {}
        for ns in self.namespaces:
            n = rr.randint(2, 4)
            lab = {"kubernetes.io/metadata.name": ns, "team": "team-%d" % rr.randint(0, 40)}
            if n > 2:
                lab["env"] = rr.choice(["prod", "dev", "staging"])
            if n > 3:
                lab["tier"] = rr.choice(["frontend", "backend", "data"])
            out[ns] = lab
        return out

    def image(self):
        repo = self.r.choice(self.repos)
        u = self.r.random()
        if u < 0.10:
            return repo + ":latest"
        if u < 0.15:
            return repo
        if u < 0.20:
            return repo + "@sha256:" + "%064x" % self.r.getrandbits(256)
        return repo + ":v%d.%d.%d" % (self.r.randint(0, 3), self.r.randint(0, 20), self.r.randint(0, 9))

    def sec_ctx(self):
        sc = {}
        if self.p(0.02):
            sc["privileged"] = True
        elif self.p(0.05):
            sc["privileged"] = False
        u = self.r.random()
        if u < 0.70:
            sc["allowPrivilegeEscalation"] = False
        elif u < 0.75:
            sc["allowPrivilegeEscalation"] = True
        if self.p(0.60):
            sc["runAsNonRoot"] = True
        elif self.p(0.05):
            sc["runAsNonRoot"] = False
        if self.p(0.03):
            sc["runAsUser"] = 0
        elif self.p(0.3):
            sc["runAsUser"] = self.r.choice([1000, 65534, 1001])
        if self.p(0.2):
            sc["runAsGroup"] = self.r.choice([0, 1000, 3000])
        caps = {}
        if self.p(0.55):
            caps["drop"] = ["ALL"]
        u = self.r.random()
        if u < 0.05:
            caps["add"] = ["NET_BIND_SERVICE"]
        elif u < 0.06:
            caps["add"] = ["SYS_ADMIN"]
        elif u < 0.065:
            caps["add"] = ["CHOWN", "NET_RAW"]
        if caps:
            sc["capabilities"] = caps
        u = self.r.random()
        if u < 0.60:
            sc["seccompProfile"] = {"type": "RuntimeDefault"}
        elif u < 0.65:
            sc["seccompProfile"] = {"type": "Localhost", "localhostProfile": "profiles/audit.json"}
        elif u < 0.67:
            sc["seccompProfile"] = {"type": "Unconfined"}
        if self.p(0.03):
            sc["seLinuxOptions"] = {"type": "spc_t" if self.p(0.33) else "container_t"}
            if self.p(0.1):
                sc["seLinuxOptions"]["user"] = "system_u"
        if self.p(0.005):
            sc["procMount"] = "Unmasked"
        elif self.p(0.01):
            sc["procMount"] = "Default"
        if self.p(0.002):
            sc["windowsOptions"] = {"hostProcess": True}
        if self.edge:
            if self.p(0.004):
                sc["privileged"] = "true"  # wrong JSON type (string)
            if self.p(0.004):
                sc["runAsUser"] = "1000"
            if self.p(0.003):
                sc["runAsUser"] = 1000.0 if self.p(0.5) else 0.5
            if self.p(0.003):
                sc["allowPrivilegeEscalation"] = None
            if self.p(0.002):
                sc["capabilities"] = None
        return sc

    def container(self, i, kind="c"):
        c = {"name": "%s%d" % (kind, i), "image": self.image()}
        if self.p(0.7):
            ports = []
            for j in range(self.r.choice([1, 1, 2, 3])):
                pt = {"containerPort": self.r.choice([80, 443, 8080, 9090, 5432]) + j, "protocol": "TCP"}
                if self.p(0.02):
                    pt["hostPort"] = self.r.choice([80, 8080, 30000])
                elif self.p(0.05):
                    pt["hostPort"] = 0
                ports.append(pt)
            c["ports"] = ports
        if self.p(0.75):
            c["securityContext"] = self.sec_ctx()
        if self.p(0.8):
            res = {}
            if self.p(0.9):
                res["requests"] = {"cpu": self.r.choice(QTY[:4]), "memory": self.r.choice(QTY[4:])}
                if self.p(0.1):
                    del res["requests"]["cpu"]
            if self.p(0.85):
                res["limits"] = {"memory": self.r.choice(QTY[4:])}
                if self.p(0.5):
                    res["limits"]["cpu"] = self.r.choice(QTY[:4])
            if self.edge and self.p(0.01):
                res["limits"] = {"memory": self.r.choice([1073741824, 0.5, "", None])}
            c["resources"] = res
        if self.p(0.3):
            c["imagePullPolicy"] = self.r.choice(["Always", "IfNotPresent", "Never"])
        if self.p(0.2):
            c["env"] = [{"name": "E%d" % k, "value": str(self.r.randint(0, 99))} for k in range(self.r.randint(1, 4))]
        return c

    def pod_spec(self):
        spec = {}
        n = self.r.choices([1, 2, 3, 4], weights=[60, 25, 10, 5])[0]
        spec["containers"] = [self.container(i) for i in range(n)]
        if self.p(0.2):
            spec["initContainers"] = [self.container(0, "init")]
        if self.p(0.01):
            spec["ephemeralContainers"] = [self.container(0, "debug")]
        for f in ("hostNetwork", "hostPID", "hostIPC"):
            if self.p(0.01):
                spec[f] = True
            elif self.p(0.05):
                spec[f] = False
        psc = {}
        if self.p(0.4):
            psc["runAsNonRoot"] = True
        if self.p(0.01):
            psc["runAsUser"] = 0
        if self.p(0.3):
            psc["fsGroup"] = self.r.choice([0, 2000])
        if self.p(0.15):
            psc["runAsGroup"] = self.r.choice([0, 3000])
        if self.p(0.1):
            psc["supplementalGroups"] = [self.r.choice([0, 4000])]
        if self.p(0.3):
            psc["seccompProfile"] = {"type": self.r.choice(["RuntimeDefault", "RuntimeDefault", "Localhost", "Unconfined"])}
        if self.p(0.02):
            psc["sysctls"] = [{"name": self.r.choice(SYSCTL_OK if self.p(0.5) else SYSCTL_BAD), "value": "1"}]
        if self.p(0.01):
            psc["seLinuxOptions"] = {"type": "container_t", "level": "s0:c123,c456"}
        if psc or self.p(0.2):
            spec["securityContext"] = psc
        vols = []
        for k in range(self.r.choice([0, 0, 1, 2, 3])):
            t = self.r.choice(VOL_TYPES)
            v = {"name": "vol%d" % k, t: {} if t not in ("nfs",) else {"server": "nfs.local", "path": "/x"}}
            vols.append(v)
        if self.p(0.03):
            vols.append({"name": "hostvol", "hostPath": {"path": self.r.choice(["/var/run/docker.sock", "/data"])}})
        if vols:
            spec["volumes"] = vols
        if self.p(0.01):
            spec["os"] = {"name": "windows" if self.p(0.3) else "linux"}
        if self.p(0.3):
            spec["serviceAccountName"] = "sa-%d" % self.r.randint(0, 9)
        if self.edge:
            if self.p(0.003):
                spec["hostNetwork"] = "false"
            if self.p(0.003):
                spec["containers"] = []
            if self.p(0.002):
                spec["volumes"] = None
        return spec

    def metadata(self, name, ns, pod=True, ncontainers=1):
        labels = {"app": "app-%d" % self.r.randint(0, 300), "app.kubernetes.io/name": name.split("-")[0],
                  "tier": self.r.choice(["frontend", "backend", "data"])}
        for k in range(self.r.randint(0, 5)):
            labels["label-%d" % k] = "v%d" % self.r.randint(0, 9)
        if self.p(0.3):
            labels["owner"] = "team-%d" % self.r.randint(0, 30)
        md = {"name": name, "namespace": ns, "labels": labels}
        ann = {}
        for k in range(self.r.randint(0, 6)):
            ann["example.com/a%d" % k] = "value-%d" % self.r.randint(0, 999)
        if pod and self.p(0.05):
            ann["container.apparmor.security.beta.kubernetes.io/c0"] = "unconfined" if self.p(0.2) else "runtime/default"
        if pod and self.p(0.01):
            ann["seccomp.security.alpha.kubernetes.io/pod"] = "unconfined" if self.p(0.5) else "runtime/default"
        if ann:
            md["annotations"] = ann
        if self.edge and self.p(0.002):
            md["labels"] = {"app": 7}  # non-string label value (apimachinery GetLabels -> nil)
        return md

    def pod(self, i):
        ns = self.r.choice(self.namespaces)
        name = "pod-%07d" % i
        return {"apiVersion": "v1", "kind": "Pod", "metadata": self.metadata(name, ns), "spec": self.pod_spec()}

    def workload(self, i):
        u = self.r.random() * 100
        if u < 70:
            return self.pod(i)
        ns = self.r.choice(self.namespaces)
        kinds = [(82, "apps/v1", "Deployment"), (86, "apps/v1", "ReplicaSet"), (89, "apps/v1", "StatefulSet"),
                 (91, "apps/v1", "DaemonSet"), (94, "batch/v1", "Job"), (96, "batch/v1", "CronJob"),
                 (97, "v1", "ReplicationController")]
        for thr, av, kind in kinds:
            if u < thr:
                name = "%s-%07d" % (kind.lower(), i)
                tpl = {"metadata": {"labels": {"app": name}}, "spec": self.pod_spec()}
                if self.p(0.05):
                    tpl["metadata"]["annotations"] = {"container.apparmor.security.beta.kubernetes.io/c0": "runtime/default"}
                if kind == "CronJob":
                    spec = {"schedule": "*/5 * * * *", "jobTemplate": {"spec": {"template": tpl}}}
                elif kind == "Job":
                    spec = {"template": tpl, "backoffLimit": 3}
                else:
                    spec = {"replicas": self.r.randint(1, 5), "selector": {"matchLabels": {"app": name}}, "template": tpl}
                return {"apiVersion": av, "kind": kind, "metadata": self.metadata(name, ns, pod=False), "spec": spec}
        k = self.r.choice(["ConfigMap", "Service", "Namespace"])
        name = "%s-%07d" % (k.lower(), i)
        if k == "ConfigMap":
            return {"apiVersion": "v1", "kind": k, "metadata": self.metadata(name, ns, pod=False), "data": {"k": "v"}}
        if k == "Service":
            return {"apiVersion": "v1", "kind": k, "metadata": self.metadata(name, ns, pod=False),
                    "spec": {"type": self.r.choice(["ClusterIP", "LoadBalancer"]), "ports": [{"port": 80}]}}
        return {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": self.r.choice(self.namespaces)}}


def pods(n, seed=SEED, edge=False):
    g = Gen(seed, edge)
    return [g.pod(i) for i in range(n)], g.ns_labels()


def mixed(n, seed=SEED, edge=False):
    g = Gen(seed, edge)
    return [g.workload(i) for i in range(n)], g.ns_labels()


def ndjson(docs):
    return ("\n".join(json.dumps(d, separators=(",", ":")) for d in docs)).encode()


def _chunk(args):
    kind, seed, start, n, edge = args
    g = Gen((seed * 1000003 + start) & 0xFFFFFFFFFFFF, edge)
    make = g.pod if kind == "pods" else g.workload
    return ("\n".join(json.dumps(make(start + i), separators=(",", ":")) for i in range(n)) + "\n").encode()


def corpus_ndjson(n, kind="mixed", seed=SEED, edge=False, workers=None, chunk=20000, start=0):
    """Large seeded corpus as NDJSON bytes, generated in parallel chunks (resource names stay unique:
    the chunk's first index is part of every name). Returns (bytes, namespace labels).
    start: generate resources [start, start + n) of the corpus seeded `seed` (start a multiple of `chunk`): a rank's
    shard of one corpus, byte-identical to that slice of the whole corpus whatever the number of shards."""
    import multiprocessing as mp
    import os
    if start % chunk:
        raise ValueError("corpus shard start must be a multiple of the chunk size")
    jobs = [(kind, seed, s, min(chunk, start + n - s), edge) for s in range(start, start + n, chunk)]
    workers = workers or min(len(jobs), int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1, 16)
    if workers <= 1 or len(jobs) == 1:
        parts = [_chunk(j) for j in jobs]
    else:
        pool = mp.get_context("fork").Pool(workers)
        try:
            parts = pool.map(_chunk, jobs)
        finally:
            pool.close()  # let the workers exit on their own (no SIGTERM under profilers)
            pool.join()
    return b"".join(parts), Gen(seed).ns_labels()


def cached_corpus(n, kind="mixed", seed=SEED, edge=False, cache_dir=None, start=0):
    """corpus_ndjson with an optional on-disk cache (KYV_CORPUS_CACHE): profiler runs reuse the corpus a
    plain run generated, so no worker processes are forked under the profiler."""
    import os
    cache_dir = cache_dir or os.environ.get("KYV_CORPUS_CACHE")
    if not cache_dir:
        return corpus_ndjson(n, kind=kind, seed=seed, edge=edge, start=start)
    base = os.path.join(cache_dir, "corpus_%s_%d_%x_%d_%d" % (kind, n, seed, int(edge), start))
    if os.path.exists(base + ".ndjson") and os.path.exists(base + ".nsl.json"):
        with open(base + ".ndjson", "rb") as f:
            data = f.read()
        with open(base + ".nsl.json") as f:
            return data, json.load(f)
    data, nsl = corpus_ndjson(n, kind=kind, seed=seed, edge=edge, start=start)
    os.makedirs(cache_dir, exist_ok=True)
    with open(base + ".ndjson.tmp", "wb") as f:
        f.write(data)
    os.replace(base + ".ndjson.tmp", base + ".ndjson")
    with open(base + ".nsl.json", "w") as f:
        json.dump(nsl, f)
    return data, nsl


def c4_policies(n=10000, seed=SEED):
    """BASELINE configs[3]: n generated ClusterPolicies, one validate rule each, with
    wildcard-heavy match (kinds incl. group/version and `*`, names, namespaces, matchLabels / matchExpressions
    selectors, annotations, namespaceSelector) and exclude blocks; simple metadata patterns. Kinds naming Pod
    or Deployment get autogen rules, so the compiled rule count is ~2-3x n."""
    r = random.Random(seed ^ 0xC4)
    kinds = [["Pod"], ["Deployment"], ["apps/v1/Deployment"], ["*"], ["ConfigMap"], ["Pod", "Service"],
             ["v1/Pod"], ["apps/*/StatefulSet"], ["Job", "CronJob"], ["Namespace"]]
    names = ["pod-*", "*-00001*", "deployment-??0*", "*", "pod-000?1*", "configmap-*"]
    nss = ["ns-?0*", "ns-00*", "ns-01??", "ns-*1", "team-*"]
    patterns = [{"metadata": {"labels": {"owner": "?*"}}}, {"metadata": {"labels": {"app": "app-*"}}},
                {"metadata": {"name": "!*-x"}}, {"metadata": {"=(annotations)": {"=(example.com/a0)": "value-?*"}}},
                {"metadata": {"labels": {"tier": "frontend | backend"}}}]
    out = []
    for i in range(n):
        res = {"kinds": list(r.choice(kinds))}
        u = r.random()
        if u < 0.3:
            res["names"] = [r.choice(names)] + ([r.choice(names)] if r.random() < 0.3 else [])
        elif u < 0.4:
            res["name"] = r.choice(names)
        if r.random() < 0.4:
            res["namespaces"] = [r.choice(nss)]
        v = r.random()
        if v < 0.25:
            res["selector"] = {"matchLabels": {"tier": r.choice(["fr*", "back?nd", "data", "*"])}}
        elif v < 0.35:
            res["selector"] = {"matchExpressions": [{"key": "app", "operator": r.choice(["In", "NotIn"]),
                                                     "values": ["app-%d" % r.randint(0, 300) for _ in range(3)]},
                                                    {"key": "owner", "operator": r.choice(["Exists", "DoesNotExist"])}]}
        elif v < 0.42:
            res["namespaceSelector"] = {"matchLabels": {"env": r.choice(["prod", "dev"])}}
        if r.random() < 0.15:
            res["annotations"] = {"example.com/a%d" % r.randint(0, 2): "value-%d*" % r.randint(0, 9)}
        match = {"any": [{"resources": res}]}
        if r.random() < 0.2:
            match["any"].append({"resources": {"kinds": ["Service"], "names": ["service-*"]}})
        rule = {"name": "r%05d" % i, "match": match,
                "validate": {"message": "generated rule %d" % i, "pattern": r.choice(patterns)}}
        w = r.random()
        if w < 0.25:
            rule["exclude"] = {"any": [{"resources": {"namespaces": [r.choice(nss)]}}]}
        elif w < 0.35:
            rule["exclude"] = {"any": [{"resources": {"annotations": {"example.com/a1": "value-?0*"}}}]}
        out.append({"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy",
                    "metadata": {"name": "c4-%05d" % i},
                    "spec": {"validationFailureAction": "Audit", "background": True, "rules": [rule]}})
    return out


def c5_policies(n=50, seed=SEED):
    """BASELINE configs[4]: n policies whose rules use preconditions / deny conditions with
    variables. About 60% use only `{{ request.object.<path> }}` operands with the condition operators (the
    device-compilable subset: Equals / NotEquals / In / AnyIn / AllIn / NotIn / AnyNotIn / AllNotIn / numeric,
    old-list and any/all forms, literal ranges, JSON-string lists, quantities, durations, message variables);
    the rest use JMESPath projections, length(), `||` defaults or request.operation (device-compiled too), and
    regex_match / to_upper (round 6: device-compiled as per-string columns of the batch dictionary)."""
    r = random.Random(seed ^ 0xC5)
    pod = {"any": [{"resources": {"kinds": ["Pod"]}}]}
    wl = {"any": [{"resources": {"kinds": ["Deployment", "StatefulSet"]}}]}
    svc = {"any": [{"resources": {"kinds": ["Service"]}}]}
    allk = {"any": [{"resources": {"kinds": ["Pod", "Deployment", "ConfigMap", "Service"]}}]}

    def c(k, op, v):
        return {"key": k, "operator": op, "value": v}

    o = "{{request.object.%s}}"
    gpu = [
        lambda: ("deny", pod, {"any": [c(o % "metadata.labels.tier", "Equals", r.choice(["data", "front*"]))]}, None,
                 "tier not allowed"),
        lambda: ("deny", allk, {"all": [c("{{ request.object.metadata.namespace }}", "AnyIn", ["ns-00*", "ns-01?0"]),
                                        c(o % "metadata.labels.app", "NotEquals", "app-1*")]}, None,
                 "{{request.object.metadata.name}} in {{request.object.metadata.namespace}} is not allowed"),
        lambda: ("pattern", pod, None, {"all": [c(o % "metadata.labels.tier", "In", ["frontend", "backend"])]},
                 "owner label required"),
        lambda: ("deny", wl, [c(o % "spec.replicas", r.choice(["GreaterThan", "LessThanOrEquals"]), r.choice([3, "2", 1.5]))],
                 None, ""),
        lambda: ("deny", pod, {"all": [c("1Gi", "GreaterThanOrEquals", "1024Mi"), c("1h", "GreaterThan", "30m"),
                                       c(o % "metadata.labels.owner", "Equals", "team-1?")]}, None, "owner team-1x"),
        lambda: ("deny", pod, [c(o % "spec.serviceAccountName", "Equals", "sa-" + str(r.randint(0, 9)))], None,
                 "service account {{request.object.spec.serviceAccountName}} is reserved"),
        lambda: ("pss", pod, None, {"any": [c(o % "metadata.namespace", "AnyNotIn", ["ns-000*"])]}, ""),
        lambda: ("deny", pod, {"any": [c(o % "spec.securityContext.supplementalGroups", r.choice(["AnyIn", "AllNotIn"]), [0])]},
                 None, "group 0"),
        lambda: ("deny", wl, {"all": [c(o % "spec.replicas", r.choice(["AnyIn", "AnyNotIn", "AllIn"]), "2-4")]}, None,
                 "replicas range"),
        lambda: ("deny", pod, {"any": [c(o % "metadata.labels.tier", "AnyIn", '["frontend","data"]')]}, None, "tier list"),
        lambda: ("deny", pod, {"any": [c(o % "spec.securityContext.fsGroup", r.choice(["Equals", "NotEquals"]), "2000")]},
                 None, "fsGroup"),
        lambda: ("deny", pod, {"any": [c(o % "spec.hostNetwork", "Equals", True)]}, None, "hostNetwork"),
        lambda: ("deny", allk, {"any": [c(o % "kind", "equals", "ConfigMap"),
                                        c(o % 'metadata.annotations."example.com/a0"', "In", ["value-1*", "value-2"])]},
                 None, "annotated"),
        lambda: ("pattern", pod, None, [c(o % "metadata.namespace", "NotIn", ["ns-0001", "ns-0002"])],
                 "tier label required"),
        lambda: ("deny", svc, {"any": [c(o % "spec.type", "Equals", "LoadBalancer")]}, None, "no load balancers"),
    ]
    cpu = [
        lambda: ("deny", pod, {"any": [c("{{ request.object.spec.containers[].image }}", "AnyIn", ["*:latest"])]}, None,
                 "latest"),
        lambda: ("deny", pod, {"any": [c("{{ length(request.object.spec.containers) }}", "GreaterThan", 2)]}, None, "many"),
        lambda: ("deny", pod, {"any": [c("{{ request.object.metadata.labels.app || '' }}", "Equals", "")]}, None, "app"),
        lambda: ("pattern", pod, None, {"any": [c("{{ request.operation }}", "Equals", "CREATE")]}, "owner"),
        # kyverno's JMESPath functions on one string (round 6: Batch::str_rx / str_upper, evaluated on the device; until
        # round 5 these rules were CPU fallback)
        lambda: ("deny", pod, {"any": [c("{{ regex_match('^team-[0-9]+$', request.object.metadata.labels.owner || '') }}",
                                         "Equals", False)]}, None, "owner format"),
        lambda: ("deny", pod, {"any": [c("{{ to_upper(request.object.metadata.labels.tier || '') }}", "Equals", "DATA")]},
                 None, "tier case"),
    ]
    out = []
    for i in range(n):
        t = (gpu[i % len(gpu)] if r.random() < 0.6 else cpu[i % len(cpu)])()
        kind, match, cond, pre, msg = t
        rule = {"name": "c5-r%03d" % i, "match": match}
        if pre is not None:
            rule["preconditions"] = pre
        if kind == "deny":
            rule["validate"] = {"message": msg, "deny": {"conditions": cond}} if msg else {"deny": {"conditions": cond}}
        elif kind == "pattern":
            rule["validate"] = {"message": msg, "pattern": {"metadata": {"labels": {"owner": "?*"}}}}
        else:
            rule["validate"] = {"podSecurity": {"level": "baseline", "version": "latest"}}
        out.append({"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "c5-%03d" % i},
                    "spec": {"validationFailureAction": "Audit", "background": True, "rules": [rule]}})
    return out
