"""`kyverno apply` result counting over the batched device path (BASELINE configs[0]).

The reference CLI loops policy x resource (cmd/cli/kubectl-kyverno/apply/apply_command.go:388-441), runs
`engine.Validate` per pair through `ApplyPolicyOnResource` (utils/common/common.go:371-564) and tallies every
response with `ProcessValidateEngineResponse` (common.go:712-795):
  * every autogen-computed rule that has a validate block (or image checks) is looked up in the response by name;
  * a rule absent from the response (not matched, or cut by applyRules: One) counts as skip;
  * pass -> pass; fail -> warn when the policy is annotated policies.kyverno.io/scored: "false", or when --audit-warn
    is set and the response's validationFailureAction is Audit, else fail; error -> error; skip -> skip.
The summary line is "pass: %d, fail: %d, warn: %d, error: %d, skip: %d" (apply_command.go:505).

Here one `kyv_eval` decides every (resource, compiled rule) pair; (policy, resource) pairs with a FALLBACK / PANIC /
ND verdict are handed whole to `cpu_engine(policy, resource) -> [{name, status, message}]` (the Go shim's
engine.Validate) and tallied the same way. Resources get the CLI's default namespace first
(convertResourceToUnstructured, fetch.go:310-312: empty metadata.namespace -> "default").

Out of scope (not the validate path): mutate before validate (the reference validates the mutated resource, so
policies with mutate rules go to `cpu_engine` whole), generate / verifyImages counts, variables files.
"""
import copy

from . import _lib as K
from . import admission as A
from . import engine as E

CPU_STATUSES = (K.ST_FALLBACK, K.ST_PANIC, K.ST_ND)
_TEXT = {K.ST_PASS: "pass", K.ST_FAIL: "fail", K.ST_SKIP: "skip", K.ST_ERROR: "error"}


class ResultCounts:
    """common.ResultCounts"""

    def __init__(self):
        self.pass_ = self.fail = self.warn = self.error = self.skip = 0

    def as_dict(self):
        return {"pass": self.pass_, "fail": self.fail, "warn": self.warn, "error": self.error, "skip": self.skip}

    def line(self):
        """apply_command.go:505"""
        return "\npass: %d, fail: %d, warn: %d, error: %d, skip: %d \n" % (self.pass_, self.fail, self.warn,
                                                                           self.error, self.skip)


def _scored_false(policy):
    return ((policy.get("metadata") or {}).get("annotations") or {}).get("policies.kyverno.io/scored") == "false"


def process_validate_response(rule_names, response_rules, policy, rc, audit_warn=False, action=""):
    """ProcessValidateEngineResponse (common.go:712-795) counting: rule_names = the policy's computed rules with a
    validate block, in order; response_rules = [{name, status}] of one engine response"""
    by_name = {r["name"]: r for r in response_rules}
    for name in rule_names:
        r = by_name.get(name)
        if r is None:
            rc.skip += 1
            continue
        st = r["status"]
        if st == "pass":
            rc.pass_ += 1
        elif st == "fail":
            if _scored_false(policy):
                rc.warn += 1
            elif audit_warn and action in ("audit", "Audit"):
                rc.warn += 1
            else:
                rc.fail += 1
        elif st == "error":
            rc.error += 1
        elif st == "warn":
            rc.warn += 1
        elif st == "skip":
            rc.skip += 1


def _with_default_namespace(resources):
    out = []
    for r in resources:
        if isinstance(r, dict) and isinstance(r.get("metadata"), dict) and not r["metadata"].get("namespace"):
            r = copy.deepcopy(r)
            r["metadata"]["namespace"] = "default"
        out.append(r)
    return out


def apply(policies, resources, ns_labels=None, backend="gpu", device=0, audit_warn=False, cpu_engine=None):
    """`kyverno apply` over one batch -> (ResultCounts, pending): pending lists the (policy name, resource index) pairs
    that needed `cpu_engine` when none was given (their rules are not counted)."""
    pols = [p for p in policies if isinstance(p, dict) and p.get("kind") in ("ClusterPolicy", "Policy")]
    docs = _with_default_namespace(resources)
    rs = E.Ruleset(pols)
    batch = E.Batch(rs, docs, ns_labels)
    res = E.evaluate(rs, batch, backend=backend, device=device)
    st = res.status
    rc, pending = ResultCounts(), []
    for pi, pm in enumerate(rs.policies):
        pol = pols[pi]
        ks = range(pm["first_rule"], pm["first_rule"] + pm["nrules"])
        names = [rs.rules[k]["name"] for k in ks]
        has_mutate = any("mutate" in (r or {}) for r in (pol.get("spec") or {}).get("rules") or [])
        for ri, doc in enumerate(docs):
            cpu = has_mutate or any(int(st[k, ri]) in CPU_STATUSES for k in ks)
            action = ""
            if audit_warn:
                md = doc.get("metadata") if isinstance(doc, dict) else None
                ns = md.get("namespace", "") if isinstance(md, dict) else ""
                action = A.response_action(pol, ns, (ns_labels or {}).get(ns))
            if cpu:
                if cpu_engine is None:
                    pending.append((pm["name"], ri))
                    continue
                process_validate_response(names, cpu_engine(pol, doc), pol, rc, audit_warn, action)
                continue
            rules, applied = [], 0
            for k in ks:  # engine response: matched rules in order, applyRules: One (validation.go:176-178)
                s = int(st[k, ri])
                if s == K.ST_NONE:
                    continue
                rules.append({"name": rs.rules[k]["name"], "status": _TEXT[s]})
                applied += s in (K.ST_PASS, K.ST_FAIL)
                if pm["apply_one"] and applied:
                    break
            process_validate_response(names, rules, pol, rc, audit_warn, action)
    return rc, pending
