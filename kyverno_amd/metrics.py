"""Per-batch policy metrics in the reference's namespace (pkg/metrics), from one device evaluation.

The reference records, for every EngineResponse a webhook produces (pkg/webhooks/utils/metrics.go:25-64):
  kyverno_policy_results                      counter, one per rule response (policyresults/policyResults.go:35-79,
                                              metrics.go:174-193)
  kyverno_policy_execution_duration_seconds   histogram of each rule response's ExecutionStats.ProcessingTime
                                              (policyexecutionduration/policyExecutionDuration.go:35-80)
with the labels of metrics.go:178-191. Here a batch of (resource, rule) verdicts is tallied at once: the verdict
matrix is grouped by (rule, resource kind, resource namespace, result) with one bincount per rule, so the cost is
O(pairs) vectorised work instead of one counter update per pair. A rule response's processing time is not measured
per pair on the device; the batch's device time is amortised over its decided pairs (stated in `duration_basis`).

Rule responses follow EngineResponse semantics: ST_NONE pairs have no response; ApplyOne truncates after the first
applied rule (validation.go:176-178); fail on a policy whose rule is unscored is still "fail" here (the report's
warn mapping is a report concern, results.go:117-119). Pairs the CPU engine decides (fallback / panic / nd) are not
tallied: the Go shim records those responses itself.
"""
import numpy as np

from . import _lib as K

RESULT = {K.ST_PASS: "pass", K.ST_FAIL: "fail", K.ST_SKIP: "skip", K.ST_ERROR: "error"}
# OpenTelemetry's default explicit-bucket boundaries (the reference registers the histogram without a view)
DEFAULT_BUCKETS = (0.0, 5.0, 10.0, 25.0, 50.0, 75.0, 100.0, 250.0, 500.0, 750.0, 1000.0, 2500.0, 5000.0, 7500.0, 10000.0)
LABELS = ("policy_validation_mode", "policy_type", "policy_background_mode", "policy_namespace", "policy_name",
          "resource_kind", "resource_namespace", "resource_request_operation", "rule_name", "rule_result", "rule_type",
          "rule_execution_cause")
DURATION_LABELS = ("policy_validation_mode", "policy_type", "policy_background_mode", "policy_namespace", "policy_name",
                   "resource_namespace", "rule_name", "rule_result", "rule_type", "rule_execution_cause")


def policy_infos(doc):
    """metrics.GetPolicyInfos (parsers.go:71-82): name, namespace, type, background mode, validation mode"""
    md = doc.get("metadata") or {}
    spec = doc.get("spec") or {}
    namespaced = doc.get("kind") == "Policy"
    action = str(spec.get("validationFailureAction") or "Audit")
    return {"name": md.get("name", ""), "namespace": md.get("namespace", "") if namespaced else "",
            "type": "namespaced" if namespaced else "cluster",
            "background": "false" if spec.get("background") is False else "true",
            "validation": "enforce" if action.lower() == "enforce" else "audit"}


def responded(status, first, n, apply_one):
    """bool [n, nres] of the pairs of one policy's rules that produce a rule response (ApplyOne truncation). Under
    ApplyOne a pair the CPU engine decides (fallback / panic / nd) ends the device's share of the resource: whether
    the rules after it respond depends on the CPU verdict (engine.Engine.validate stops there too)."""
    sub = np.asarray(status[first:first + n]) & 7
    has = sub != K.ST_NONE
    if not apply_one:
        return has
    out = np.zeros_like(has)
    active = np.ones(sub.shape[1], dtype=bool)
    for i in range(n):
        out[i] = has[i] & active
        cpu = (sub[i] == K.ST_FALLBACK) | (sub[i] == K.ST_PANIC) | (sub[i] == K.ST_ND)
        active &= ~(((sub[i] == K.ST_PASS) | (sub[i] == K.ST_FAIL) | cpu) & out[i])
    return out


def policy_stats(ruleset, status):
    """PolicyResponse.PolicyStats of every (policy, resource) (validation.go:196-208): (applied int32 [policies,
    nres] = pass + fail rule responses, errors int32 [policies, nres] = error rule responses)"""
    nres = np.asarray(status).shape[1]
    applied = np.zeros((len(ruleset.policies), nres), dtype=np.int32)
    errors = np.zeros_like(applied)
    for pi, pm in enumerate(ruleset.policies):
        if not pm["nrules"]:
            continue
        sub = np.asarray(status[pm["first_rule"]:pm["first_rule"] + pm["nrules"]]) & 7
        r = responded(status, pm["first_rule"], pm["nrules"], pm["apply_one"])
        applied[pi] = (r & ((sub == K.ST_PASS) | (sub == K.ST_FAIL))).sum(axis=0)
        errors[pi] = (r & (sub == K.ST_ERROR)).sum(axis=0)
    return applied, errors


class PolicyMetrics:
    """Accumulates kyverno_policy_results / kyverno_policy_execution_duration_seconds over batches."""

    def __init__(self, buckets=DEFAULT_BUCKETS):
        self.results = {}     # label tuple (LABELS) -> count
        self.durations = {}   # label tuple (DURATION_LABELS) -> [bucket counts..., +Inf count, sum]
        self.buckets = tuple(buckets)
        self.duration_basis = "device time of the batch / decided pairs (amortised per rule response)"

    def record(self, ruleset, policy_docs, res, kinds, namespaces, cause="background_scan", operation="",
               seconds=None, mask=None):
        """one evaluated batch: res (engine.Results, verdicts copied back), kinds / namespaces: per resource (batch
        input order) resource kind (None: the row records nothing) and namespace; policy_docs: the policy documents in ruleset.policies order;
        cause: "admission_request" / "background_scan"; operation: "create" / "update" / ... ("" for scans), or one
        per resource; mask: optional bool [policies, nres], only the (policy, resource) pairs whose engine response the
        device produced (an admission batch hands some to the CPU engine, whose responses the Go shim records)"""
        st = np.asarray(res.status)
        nres = st.shape[1]
        include = np.array([k is not None for k in kinds], dtype=bool)  # None: a row with no response of its own
        kinds, namespaces = [k or "" for k in kinds], [n or "" for n in namespaces]
        ops = [operation] * nres if isinstance(operation, str) else [o or "" for o in operation]
        assert len(kinds) == len(namespaces) == len(ops) == nres
        groups, gid = np.unique(np.array([k + "\x00" + n + "\x00" + o for k, n, o in zip(kinds, namespaces, ops)],
                                         dtype=object), return_inverse=True)
        gid = gid.astype(np.int64)
        ng = len(groups)
        decided = sum(int(res.counts.get(K.STATUS_NAMES[s], 0)) for s in RESULT)
        if seconds is None:
            seconds = res.kernel_ms / 1e3
        per = seconds / max(1, decided)
        for pi, pm in enumerate(ruleset.policies):
            info = policy_infos(policy_docs[pi] if pi < len(policy_docs) else {})
            pns = "-" if info["type"] == "cluster" else info["namespace"]
            resp = responded(st, pm["first_rule"], pm["nrules"], pm["apply_one"])
            pmask = include if mask is None else (include & np.asarray(mask[pi], dtype=bool))
            for i in range(pm["nrules"]):
                k = pm["first_rule"] + i
                s = st[k] & 7
                m = resp[i] & np.isin(s, list(RESULT)) & pmask
                if not m.any():
                    continue
                c = np.bincount(gid[m] * 8 + s[m].astype(np.int64), minlength=ng * 8).reshape(ng, 8)
                rname = ruleset.rules[k]["name"]
                for g, sv in zip(*np.nonzero(c)):
                    kind, ns, op = groups[g].split("\x00")
                    n = int(c[g, sv])
                    key = (info["validation"], info["type"], info["background"], pns, info["name"], kind, ns,
                           op, rname, RESULT[int(sv)], "validate", cause)
                    self.results[key] = self.results.get(key, 0) + n
                    dkey = (info["validation"], info["type"], info["background"], pns, info["name"], ns, rname,
                            RESULT[int(sv)], "validate", cause)
                    h = self.durations.setdefault(dkey, [0] * (len(self.buckets) + 1) + [0.0])
                    b = int(np.searchsorted(self.buckets, per, side="left"))  # first boundary >= value (le)
                    h[b] += n
                    h[-1] += per * n

    def collector(self):
        """a prometheus_client collector exposing both families (counter as kyverno_policy_results_total)"""
        from prometheus_client.core import CounterMetricFamily, HistogramMetricFamily
        m = self

        class _C:
            def collect(self):
                c = CounterMetricFamily("kyverno_policy_results", "can be used to track the results associated with "
                                        "the policies applied in the user's cluster", labels=LABELS)
                for key, n in sorted(m.results.items()):
                    c.add_metric(list(key), n)
                yield c
                h = HistogramMetricFamily("kyverno_policy_execution_duration_seconds", "can be used to track the "
                                          "latencies (in seconds) associated with the execution/processing of the "
                                          "individual rules", labels=DURATION_LABELS)
                for key, v in sorted(m.durations.items()):
                    cum, acc = [], 0
                    for i, bnd in enumerate(m.buckets):
                        acc += v[i]
                        cum.append((repr(float(bnd)), acc))
                    acc += v[len(m.buckets)]
                    cum.append(("+Inf", acc))
                    h.add_metric(list(key), cum, v[-1])
                yield h

        return _C()

    def exposition(self):
        """Prometheus text exposition of the two families"""
        from prometheus_client import CollectorRegistry, generate_latest
        reg = CollectorRegistry()
        reg.register(self.collector())
        return generate_latest(reg).decode()
