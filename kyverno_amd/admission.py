"""Admission micro-batching: concurrent AdmissionReviews evaluated in one device batch.

The reference handles one AdmissionRequest at a time (pkg/webhooks/resource/validation/validation.go:72-147):
the enforce policies for the request's kind and namespace come from the policy cache
(pkg/policycache/cache.go:38-88, store.go:70-138), `engine.Validate` runs once per policy, and the request is
blocked when a response fails under an Enforce action or errors under failurePolicy Fail
(pkg/utils/engine/response.go:21-29, pkg/webhooks/utils/block.go:26-67); otherwise the non-pass, non-skip rule
messages become warnings (pkg/webhooks/utils/warning.go:9-20).

Here requests are queued and evaluated together: one `kyv_batch_build` + `kyv_eval` over the new objects (and the
old objects of UPDATE requests) of every queued request, then the per-request decision above is assembled on the
host from the device verdicts. Everything the device subset does not decide for a (request, policy) goes to the
CPU engine for that whole policy (`cpu_engine`, the Go shim's engine.Validate):
  * pairs the device reports as KYV_ST_FALLBACK / PANIC / ND;
  * rules whose match or exclude names roles / clusterRoles / subjects (admission userInfo: the device path has
    background-scan semantics, where the admission info is empty, utils.go:258-262);
  * policies with a condition on request.operation for requests other than CREATE (the device binds it to the
    background scan's "CREATE");
  * UPDATE requests where a rule does not match the new object but matches the old one (the OldResource retry of
    validation.go:600-615 then validates the new object, which the device did not do);
  * DELETE requests (the new object is empty; validateResourceWithRule skips patterns, validation.go:568-579).
The micro-batch knobs (max batch, max wait) trade latency for throughput; `handle_batch` is the synchronous core.
"""
import json
import re
import threading
import time
from concurrent.futures import Future

import numpy as np

from . import _lib as K
from . import engine as E

CPU_STATUSES = (K.ST_FALLBACK, K.ST_PANIC, K.ST_ND)
STATUS_TEXT = {K.ST_PASS: "pass", K.ST_FAIL: "fail", K.ST_SKIP: "skip", K.ST_ERROR: "error"}
AUTOGEN_PREFIXES = ("autogen-cronjob-", "autogen-")


# ----------------------------------------------------------------------------------------------- go-wildcard / labels
def wildcard_match(pattern, s):
    """go-wildcard v1.0.3 Match (pkg/utils/wildcard/match.go:7): '*' any run, '?' exactly one rune"""
    if pattern == "":
        return s == ""
    if pattern == "*":
        return True
    p, t = list(pattern), list(s)
    pi = ti = 0
    star, mark = -1, 0
    while ti < len(t):
        if pi < len(p) and (p[pi] == "?" or p[pi] == t[ti]):
            pi += 1
            ti += 1
        elif pi < len(p) and p[pi] == "*":
            star, mark = pi, ti
            pi += 1
        elif star >= 0:
            pi = star + 1
            mark += 1
            ti = mark
        else:
            return False
    while pi < len(p) and p[pi] == "*":
        pi += 1
    return pi == len(p)


def check_patterns(patterns, s):
    """wildcard.CheckPatterns (pkg/utils/wildcard/utils.go): any pattern matches"""
    return any(wildcard_match(p, s) for p in (patterns or []))


def check_selector(selector, labels):
    """utils.CheckSelector (pkg/utils/match/labels.go:10-24) with apimachinery LabelSelectorAsSelector semantics:
    nil selector -> labels.Nothing() (no match); {} -> Everything; an invalid selector -> error (False, err)."""
    if selector is None:
        return False, None
    labels = labels or {}
    for k, v in (selector.get("matchLabels") or {}).items():
        if labels.get(k) != v:
            return False, None
    for req in selector.get("matchExpressions") or []:
        op, key, vals = req.get("operator"), req.get("key"), req.get("values") or []
        if op == "In":
            if not vals:
                return False, "values: Required value"
            if key not in labels or labels[key] not in vals:
                return False, None
        elif op == "NotIn":
            if not vals:
                return False, "values: Required value"
            if key in labels and labels[key] in vals:
                return False, None
        elif op == "Exists":
            if key not in labels:
                return False, None
        elif op == "DoesNotExist":
            if key in labels:
                return False, None
        else:
            return False, "not a valid selector operator"
    return True, None


# ------------------------------------------------------------------------------------------------------ policy spec
def _spec(p):
    return p.get("spec") or {}


def action_enforce(a):
    """ValidationFailureAction.Enforce (api/kyverno/v1/spec_types.go): "enforce" / "Enforce" """
    return a in ("enforce", "Enforce")


def action_valid(a):
    return a in ("enforce", "Enforce", "audit", "Audit")


def failure_policy(p):
    """Spec.GetFailurePolicy (spec_types.go:221-228): default Fail"""
    return _spec(p).get("failurePolicy") or "Fail"


def has_validate(p):
    return any("validate" in (r or {}) for r in _spec(p).get("rules") or [])


def compute_enforce_policy(p):
    """store.go computeEnforcePolicy"""
    s = _spec(p)
    if action_enforce(s.get("validationFailureAction", "Audit")):
        return True
    return any(action_enforce((o or {}).get("action")) for o in s.get("validationFailureActionOverrides") or [])


def keep_for_enforce(p, ns):
    """cache.go checkValidationFailureActionOverrides(enforce=true, ns, policy)"""
    from .policycache import check_overrides
    return check_overrides(True, ns, p)


def response_action(p, resource_ns, ns_labels):
    """EngineResponse.GetValidationFailureAction (pkg/engine/api/engineresponse.go:106-130)"""
    s = _spec(p)
    for o in s.get("validationFailureActionOverrides") or []:
        a = o.get("action")
        if not action_valid(a):
            continue
        if o.get("namespaces") is None:
            ok, err = check_selector(o.get("namespaceSelector"), ns_labels)
            if err is None and ok:
                return a
        for ns in o.get("namespaces") or []:
            if wildcard_match(ns, resource_ns):
                if o.get("namespaceSelector") is None:
                    return a
                ok, err = check_selector(o.get("namespaceSelector"), ns_labels)
                if err is None and ok:
                    return a
    return s.get("validationFailureAction", "")


def kind_from_gvk(s):
    """kubeutils.GetKindFromGVK (pkg/utils/kube/kind.go:11-32) -> (groupVersion, kind)"""
    parts = s.split("/")
    ver = re.compile(r"v\d((alpha|beta)\d)?")
    fmt = lambda x: x.replace(".", "/", 1)
    if len(parts) == 2:
        if ver.search(parts[0]) or parts[0] == "*":
            return parts[0], fmt(parts[1])
        return "", parts[0] + "/" + parts[1]
    if len(parts) == 3:
        if ver.search(parts[0]) or parts[0] == "*":
            return parts[0], parts[1] + "/" + parts[2]
        return parts[0] + "/" + parts[1], fmt(parts[2])
    if len(parts) == 4:
        return parts[0] + "/" + parts[1], parts[2] + "/" + parts[3]
    return "", fmt(s)


def compute_kind(gvk):
    """policycache computeKind (store.go:70-74): GetKindFromGVK then SplitSubresource"""
    _, k = kind_from_gvk(gvk)
    parts = k.split("/")
    return parts[0] if len(parts) == 2 else k


def _uses_userinfo(block):
    if not isinstance(block, dict):
        return False
    if any(block.get(k) for k in ("roles", "clusterRoles", "subjects")):
        return True
    return any(_uses_userinfo(b) for key in ("any", "all") for b in (block.get(key) or []))


def rule_uses_userinfo(rule):
    return _uses_userinfo(rule.get("match")) or _uses_userinfo(rule.get("exclude"))


# ------------------------------------------------------------------------------------------- messages (go-yaml v2)
def _go_yaml_key_less(a, b):
    """go-yaml v2 keyList.Less (sorter.go): letters after non-letters, digit runs compared as numbers"""
    ar, br = list(a), list(b)
    for i in range(min(len(ar), len(br))):
        if ar[i] == br[i]:
            continue
        al, bl = ar[i].isalpha(), br[i].isalpha()
        if al and bl:
            return ar[i] < br[i]
        if al or bl:
            return bl
        an = bn = 0
        if ar[i] == "0" or br[i] == "0":
            j = i - 1
            while j >= 0 and ar[j].isdigit():
                if ar[j] != "0":
                    an = bn = 1
                    break
                j -= 1
        ai = i
        while ai < len(ar) and ar[ai].isdigit():
            an = an * 10 + ord(ar[ai]) - 48
            ai += 1
        bi = i
        while bi < len(br) and br[bi].isdigit():
            bn = bn * 10 + ord(br[bi]) - 48
            bi += 1
        if an != bn:
            return an < bn
        if ai != bi:
            return ai < bi
        return ar[i] < br[i]
    return len(ar) < len(br)


def _sorted_keys(d):
    import functools
    return sorted(d, key=functools.cmp_to_key(lambda a, b: -1 if _go_yaml_key_less(a, b) else
                                              (1 if _go_yaml_key_less(b, a) else 0)))


_RESOLVES_NON_STR = {"", "~", "null", "Null", "NULL", "true", "True", "TRUE", "false", "False", "FALSE", "y", "Y",
                     "yes", "Yes", "YES", "n", "N", "no", "No", "NO", "on", "On", "ON", "off", "Off", "OFF",
                     ".nan", ".NaN", ".NAN", ".inf", ".Inf", ".INF", "+.inf", "+.Inf", "+.INF", "-.inf", "-.Inf",
                     "-.INF", "<<"}


_YAML_NUM = re.compile(r"[-+]?(0b[01]+|0o?[0-7]+|0x[0-9a-fA-F]+|[0-9]+|(\.[0-9]+|[0-9]+(\.[0-9]*)?)([eE][-+]?[0-9]+)?"
                       r"|\.?[iI]nf(inity)?|\.?[nN]a[nN])")


def _resolves_non_str(s):
    """go-yaml v2 resolve(): would the plain scalar read back as something other than a string (null / bool /
    int via strconv.ParseInt base 0 / float via ParseFloat, '_' removed)?"""
    if s in _RESOLVES_NON_STR:
        return True
    t = s.replace("_", "")
    return bool(t) and t[0] in "+-.0123456789" and _YAML_NUM.fullmatch(t) is not None


_BLOCK_IND_ANYWHERE = re.compile(r":(?:[ \t\r\n]|$)|[ \t\r\n]#")


def _analyze(s):
    """yaml_emitter_analyze_scalar (emitterc.go) for the block context: (block_plain_allowed, special).
    special = a character outside printable ASCII (the emitter's double-quoted / unicode branches)."""
    if s == "":
        return False, False
    special = not (s.isascii() and s.isprintable())
    c0 = s[0]
    f0 = len(s) == 1 or s[1] in " \t\r\n"
    block_ind = (s.startswith("---") or s.startswith("...") or c0 in "#,[]{}&*!|>'\"%@`"
                 or (c0 in "?:-" and f0) or _BLOCK_IND_ANYWHERE.search(s, 1) is not None)
    block_plain = not (s[0] == " " or s[-1] == " " or block_ind)
    return block_plain, special


def _fold(s, column, indent, quoted):
    """write_plain / write_single_quoted line folding (emitterc.go): at a space not preceded by a space and not
    followed by one, break the line when the column is past best_width (80); single-quoted scalars never break
    at their first or last character. s is the already-escaped text; column is where it starts."""
    out, start, line_col = [], 0, column  # line_col: column of s[start]
    n = len(s)
    pos = s.find(" ")
    while pos != -1:
        col = line_col + (pos - start)
        if (col > 80 and (pos == 0 or s[pos - 1] != " ") and (pos + 1 >= n or s[pos + 1] != " ")
                and (not quoted or 0 < pos < n - 1)):
            out.append(s[start:pos])
            out.append("\n" + " " * indent)
            start, line_col = pos + 1, indent
        pos = s.find(" ", pos + 1)
    out.append(s[start:])
    return "".join(out)


def _emit_value(s, column, indent):
    """One block-mapping value as go-yaml v2 writes it (plain / single-quoted, folded at best_width 80).
    Returns (text, exact): exact is False for scalars outside the restated subset (newlines, non-ASCII)."""
    block_plain, special = _analyze(s)
    if special:
        return " " + json.dumps(s), False
    if _resolves_non_str(s):  # encode.go stringv: quoted so it reads back as a string
        return " " + json.dumps(s), True
    if block_plain:
        return " " + _fold(s, column + 1, indent, False), True
    # single-quoted: the quote is column+1; a '' escape is emitted before the folding check of later spaces, so the
    # column bookkeeping on the escaped text is exact (a quote is never a fold point)
    return " '" + _fold(s.replace("'", "''"), column + 2, indent, True) + "'", True


def yaml_marshal_failures(failures):
    """sigs.k8s.io/yaml.Marshal of map[policy]map[rule]message (block.go:64). -> (text, exact)"""
    lines, exact = [], True
    for pol in _sorted_keys(failures):
        lines.append(pol + ":\n")
        for rule in _sorted_keys(failures[pol]):
            head = "  " + rule + ":"
            body, ok = _emit_value(failures[pol][rule], len(head), 4)
            exact = exact and ok
            lines.append(head + body + "\n")
    return "".join(lines), exact


def get_action(has_violations, n):
    """block.go getAction"""
    a = "violation" if has_violations else "error"
    return a + "s" if n > 1 else a


def get_blocked_messages(responses):
    """block.go:38-67 GetBlockedMessages. responses: [{"policy", "rules": [{name, status, message}], "resource"}]
    -> (message, exact)"""
    if not responses:
        return "", True
    failures, has_viol = {}, False
    for er in responses:
        reasons = {}
        for r in er["rules"]:
            if r["status"] != "pass":
                reasons[r["name"]] = r["message"]
                if r["status"] == "fail":
                    has_viol = True
        if reasons:
            failures[er["policy"]] = reasons
    if not failures:
        return "", True
    kind, ns, name = responses[0]["resource"]
    body, exact = yaml_marshal_failures(failures)
    return "\n\npolicy %s/%s/%s for resource %s: \n\n%s" % (kind, ns, name, get_action(has_viol, len(failures)),
                                                             body), exact


def get_warning_messages(responses):
    """warning.go:9-20"""
    out = []
    for er in responses:
        for r in er["rules"]:
            if r["status"] not in ("pass", "skip"):
                out.append("policy %s.%s: %s" % (er["policy"], r["name"], r["message"]))
    return out or None


def block_request(er, fail_policy):
    """pkg/utils/engine/response.go:21-29"""
    sts = {r["status"] for r in er["rules"]}
    if "fail" in sts and action_enforce(er["action"]):
        return True
    return "error" in sts and fail_policy == "Fail"


def decide(responses, fail_policy):
    """HandleValidation's tail (validation.go:136-147): (allowed, message, warnings, exact)"""
    if any(block_request(er, fail_policy) for er in responses):
        msg, exact = get_blocked_messages(responses)
        return False, msg, None, exact
    return True, "", get_warning_messages(responses), True


# ------------------------------------------------------------------------------------------------------- batching
def _dumps1(doc):
    return json.dumps(doc, separators=(",", ":")).encode()


def _meta(obj):
    m = obj.get("metadata") if isinstance(obj, dict) else None
    return m if isinstance(m, dict) else {}


class AdmissionBatcher:
    """Micro-batched validating admission over one compiled policy set.

    requests: dicts {"uid", "operation" (CREATE / UPDATE / DELETE / CONNECT), "kind" (request.Kind.Kind),
    "namespace", "object", "oldObject", "namespace_labels"}; "object_raw" / "oldObject_raw" (the request's JSON bytes,
    AdmissionRequest.Object.Raw) are flattened as they are when present instead of re-serialising the dicts.
    cpu_engine(policy, request) -> list of rule responses [{name, status, message}] (engine.Validate on the CPU,
    the Go shim's job); when None, requests needing it come back with "cpu_pending" set and no decision."""

    def __init__(self, policies, backend="gpu", device=0, cpu_engine=None, max_batch=512, max_wait_ms=1.0):
        self.policies = [p for p in policies if isinstance(p, dict) and p.get("kind") in ("ClusterPolicy", "Policy")]
        self.ruleset = E.Ruleset(self.policies)
        self.backend, self.device, self.cpu_engine = backend, device, cpu_engine
        self.max_batch, self.max_wait = max_batch, max_wait_ms / 1000.0
        by_key = {(_meta(p).get("namespace") or "", _meta(p).get("name")): p for p in self.policies}
        self.pol = []
        for pm in self.ruleset.policies:
            p = by_key.get((pm["namespace"], pm["name"])) or by_key.get(("", pm["name"])) or {}
            base = {(r or {}).get("name"): r for r in _spec(p).get("rules") or []}
            userinfo = False
            for k in range(pm["first_rule"], pm["first_rule"] + pm["nrules"]):
                nm = self.ruleset.rules[k]["name"]
                for pre in AUTOGEN_PREFIXES:
                    if nm.startswith(pre) and nm[len(pre):] in base:
                        nm = nm[len(pre):]
                        break
                userinfo = userinfo or rule_uses_userinfo(base.get(nm) or {})
            uses_op = any(self.ruleset.rules[k]["uses_operation"]
                          for k in range(pm["first_rule"], pm["first_rule"] + pm["nrules"]))
            self.pol.append({"doc": p, "name": pm["name"], "namespace": pm["namespace"], "first": pm["first_rule"],
                             "n": pm["nrules"], "apply_one": pm["apply_one"], "userinfo": userinfo, "uses_op": uses_op,
                             "enforce": has_validate(p) and compute_enforce_policy(p),
                             "fail_policy": failure_policy(p)})
        # the policy cache (pkg/policycache) indexed from the compiled ruleset's autogen rules and their kinds
        from .policycache import PolicyCache, VALIDATE_ENFORCE
        self._vtype = VALIDATE_ENFORCE
        self.cache, self._key_index = PolicyCache(), {}
        for i, pm in enumerate(self.ruleset.policies):
            key = pm["namespace"] + "/" + pm["name"] if pm["namespace"] else pm["name"]
            rules = [(self.ruleset.rules[k]["match_kinds"], self.ruleset.rules[k]["has_validate"])
                     for k in range(pm["first_rule"], pm["first_rule"] + pm["nrules"])]
            self.cache.set(key, self.pol[i]["doc"], rules=rules)
            self._key_index[key] = i
        self.stats = {"requests": 0, "batches": 0, "device_policies": 0, "cpu_policies": 0}
        # kyverno_policy_results / _execution_duration_seconds of the device-decided rule responses of every batch
        # (pkg/webhooks/utils/metrics.go:25-64); the CPU engine's responses are recorded by the Go shim
        from .metrics import PolicyMetrics
        self.metrics = PolicyMetrics()
        self._q, self._cv, self._stop, self._thr = [], threading.Condition(), False, None
        self._enforce_cache = {}

    def enforce_policies(self, ns, kind):
        """policycache.GetPolicies(ValidateEnforce, kind, ns) (cache.go:38-57) as indices into self.pol; a policy
        indexed under both the kind and "*" comes back twice, as the reference's appends return it"""
        return [self._key_index[k] for k in self.cache.get_policy_keys(self._vtype, kind, ns)]

    def _device_rules(self, pi, st, r, res):
        """rule responses of policy pi for batch resource r from the device (ApplyOne truncation as
        validation.go:176-178), or None when any pair needs the CPU engine. Pass messages are not materialised:
        no admission output reads them (block.go:47, warning.go:13)."""
        p = self.pol[pi]
        rules, applied = [], 0
        for k in range(p["first"], p["first"] + p["n"]):
            s = int(st[k, r])
            if s == K.ST_NONE:
                continue
            if s in CPU_STATUSES:
                return None
            msg = None
            if s != K.ST_PASS:
                msg = res.message(r, k)
                if msg is None:  # message not renderable from device verdicts: the CPU engine decides the policy
                    return None
            rules.append({"name": self.ruleset.rules[k]["name"], "status": STATUS_TEXT[s], "message": msg})
            if s in (K.ST_PASS, K.ST_FAIL):
                applied += 1
            if p["apply_one"] and applied > 0:
                break
        return rules

    def handle_batch(self, requests):
        """Evaluate a list of requests in one device batch -> list of decisions (same order)."""
        docs, ns_labels, slots, mkind, mns, mop = [], {}, [], [], [], []
        for rq in requests:
            op = rq.get("operation", "CREATE")
            new, old = rq.get("object") or {}, rq.get("oldObject") or {}
            ns = rq.get("namespace") or ""
            if ns and rq.get("namespace_labels") is not None:
                ns_labels[ns] = rq["namespace_labels"]
            i_new = i_old = None
            if op != "DELETE" and new:
                i_new = len(docs)
                docs.append(rq.get("object_raw") or _dumps1(new))
                mkind.append(new.get("kind", "") if isinstance(new, dict) else "")
                mns.append(_meta(new).get("namespace", ""))
                mop.append(op.lower())
                if op == "UPDATE" and old:
                    i_old = len(docs)
                    docs.append(rq.get("oldObject_raw") or _dumps1(old))
                    mkind.append(None)  # the OldResource retry's row: no response of its own
                    mns.append("")
                    mop.append("")
            slots.append((i_new, i_old))
        st = res = None
        quiet = cpu = None
        if docs:
            batch = E.Batch(self.ruleset, b"\n".join(docs), ns_labels or None)  # NDJSON
            res = E.evaluate(self.ruleset, batch, backend=self.backend, device=self.device)
            st = res.status
            # per policy over the whole batch: "every matched rule passed" (the policy cannot change the decision)
            # and "some pair needs the CPU engine"; only the remaining (request, policy) pairs are assembled rule
            # by rule
            quiet = np.zeros((len(self.pol), len(docs)), dtype=bool)
            cpu = np.zeros((len(self.pol), len(docs)), dtype=bool)
            for pi, p in enumerate(self.pol):
                if not p["enforce"] or p["n"] == 0:
                    quiet[pi] = True
                    continue
                sub = st[p["first"]:p["first"] + p["n"]]
                cpu[pi] = np.isin(sub, CPU_STATUSES).any(axis=0)
                quiet[pi] = ((sub == K.ST_NONE) | (sub == K.ST_PASS)).all(axis=0) & ~cpu[pi]
        out = []
        # (policy, batch row) pairs whose engine response the device produced: only those are recorded as metrics
        # (userInfo / operation policies, OldResource retries, CPU pairs and policies the cache does not select for
        # the request are the CPU engine's responses, recorded by the Go shim, or no response at all)
        rec = np.zeros((len(self.pol), len(docs)), dtype=bool) if docs else None
        for rq, (i_new, i_old) in zip(requests, slots):
            out.append(self._decide(rq, i_new, i_old, st, res, quiet, cpu, rec))
        if docs:
            self.metrics.record(self.ruleset, [p["doc"] for p in self.pol], res, mkind, mns,
                                cause="admission_request", operation=mop, mask=rec)
        self.stats["requests"] += len(requests)
        self.stats["batches"] += 1
        return out

    def _decide(self, rq, i_new, i_old, st, res, quiet, cpu, rec=None):
        op = rq.get("operation", "CREATE")
        new, old = rq.get("object") or {}, rq.get("oldObject") or {}
        ns = rq.get("namespace") or ""
        dts = _meta(old).get("deletionTimestamp") if new else _meta(new).get("deletionTimestamp")
        if dts is not None and op == "UPDATE":
            return {"uid": rq.get("uid"), "allowed": True, "message": "", "warnings": None, "exact": True}
        patched0 = new if new else old
        rkind = rq.get("kind")
        if rkind is None:
            rkind = patched0.get("kind", "") if isinstance(patched0, dict) else ""
        pols = self._enforce_cache.get((ns, rkind))
        if pols is None:
            pols = self._enforce_cache[(ns, rkind)] = self.enforce_policies(ns, rkind)
        if not pols:
            return {"uid": rq.get("uid"), "allowed": True, "message": "", "warnings": None, "exact": True}
        patched = new if new else old
        resource = (patched.get("kind", "") if isinstance(patched, dict) else "", _meta(patched).get("namespace", ""),
                    _meta(patched).get("name", ""))
        nsl = rq.get("namespace_labels")
        responses, pending, fp = [], [], "Ignore"
        for pi in pols:
            p = self.pol[pi]
            if p["fail_policy"] == "Fail":
                fp = "Fail"
            rules = None
            # the device evaluates request.operation as the background scan's "CREATE"
            if i_new is not None and not p["userinfo"] and not (p["uses_op"] and op != "CREATE"):
                old_retry = i_old is not None and any(
                    int(st[k, i_new]) == K.ST_NONE and int(st[k, i_old]) != K.ST_NONE
                    for k in range(p["first"], p["first"] + p["n"]))
                if not old_retry:  # else the OldResource retry would match: the CPU engine validates the new object
                    if quiet[pi, i_new]:
                        self.stats["device_policies"] += 1
                        if rec is not None:
                            rec[pi, i_new] = True
                        continue  # pass / no rule responses: no effect on blocking, messages or warnings
                    if not cpu[pi, i_new]:
                        rules = self._device_rules(pi, st, i_new, res)
                        if rules is not None and rec is not None:
                            rec[pi, i_new] = True
            if rules is None:
                if self.cpu_engine is None:
                    pending.append(p["name"])
                    continue
                rules = self.cpu_engine(p["doc"], rq)
                self.stats["cpu_policies"] += 1
            else:
                self.stats["device_policies"] += 1
            responses.append({"policy": p["name"], "rules": rules, "resource": resource,
                              "action": response_action(p["doc"], resource[1], nsl)})
        if pending:
            return {"uid": rq.get("uid"), "allowed": None, "cpu_pending": pending, "exact": True}
        allowed, msg, warns, exact = decide(responses, fp)
        return {"uid": rq.get("uid"), "allowed": allowed, "message": msg, "warnings": warns, "exact": exact}

    # ------------------------------------------------------------------ threaded micro-batching
    def start(self):
        self._stop = False
        self._thr = threading.Thread(target=self._loop, daemon=True)
        self._thr.start()
        return self

    def stop(self):
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        if self._thr:
            self._thr.join()

    def submit(self, request):
        """queue one request -> Future resolving to its decision"""
        f = Future()
        with self._cv:
            self._q.append((request, f, time.perf_counter()))
            self._cv.notify()
        return f

    def _loop(self):
        while True:
            with self._cv:
                while not self._q and not self._stop:
                    self._cv.wait()
                if self._stop and not self._q:
                    return
                deadline = self._q[0][2] + self.max_wait
                while len(self._q) < self.max_batch and not self._stop:
                    left = deadline - time.perf_counter()
                    if left <= 0:
                        break
                    self._cv.wait(left)
                take, self._q = self._q[:self.max_batch], self._q[self.max_batch:]
            # a future its caller cancelled is dropped here; the others are marked running (no later cancel)
            take = [t for t in take if t[1].set_running_or_notify_cancel()]
            if not take:
                continue
            try:
                outs = self.handle_batch([t[0] for t in take])
            except Exception as e:  # surface device errors to every waiter of the batch
                for _, f, _ in take:
                    _resolve(f, exc=e)
                continue
            for (_, f, _), o in zip(take, outs):
                _resolve(f, result=o)


def _resolve(f, result=None, exc=None):
    """complete one waiter; a future that is already resolved must not take the batcher thread down"""
    try:
        if exc is not None:
            f.set_exception(exc)
        else:
            f.set_result(result)
    except Exception:  # InvalidStateError: resolved elsewhere
        pass


def latency_summary(lat_s):
    a = np.sort(np.asarray(lat_s, dtype=np.float64)) * 1e3
    if a.size == 0:
        return {}
    return {"p50_ms": float(np.percentile(a, 50)), "p99_ms": float(np.percentile(a, 99)), "max_ms": float(a[-1])}
