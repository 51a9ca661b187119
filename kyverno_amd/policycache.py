"""Policy cache: which policies an admission request of a given kind and namespace is validated against.

Restates pkg/policycache for the validate policy types (ValidateEnforce / ValidateAudit, type.go:5-15):
  * store.go:96-138 policyMap.set -- a policy is indexed under the kind of every gvk its autogen-expanded rules
    match (computeKind, store.go:70-74, unless the subresource map names it) when one of those rules has a validate
    block; under ValidateEnforce when computeEnforcePolicy (store.go:76-86) holds, else ValidateAudit;
  * store.go:140-146 unset, store.go:148-171 get (cluster policies for namespace "", a namespaced Policy only for
    its own namespace);
  * cache.go:38-57 GetPolicies (kind then "*", cluster then namespace, ValidateAudit also pulls ValidateEnforce
    policies) and cache.go:60-89 filterPolicies / checkValidationFailureActionOverrides.
The autogen expansion and each rule's kinds come from the compiled ruleset (kyv_ruleset_rule_kinds), so the index
is built from the same ComputeRules the device evaluates. Keys are cache.MetaNamespaceKeyFunc ("ns/name" for a
Policy, "name" for a ClusterPolicy); results keep insertion order where the reference iterates a Go set (the
reference's tests compare lengths only).
"""
import threading

from . import admission as A
from . import engine as E

VALIDATE_ENFORCE = "ValidateEnforce"
VALIDATE_AUDIT = "ValidateAudit"
TYPES = (VALIDATE_ENFORCE, VALIDATE_AUDIT)


def policy_key(policy):
    """cache.MetaNamespaceKeyFunc"""
    md = policy.get("metadata") or {}
    ns = md.get("namespace") or ""
    return ns + "/" + md.get("name", "") if ns else md.get("name", "")


def split_key(key):
    """cache.SplitMetaNamespaceKey -> (namespace, name)"""
    parts = key.split("/")
    if len(parts) == 2:
        return parts[0], parts[1]
    return "", key


def rule_kinds(policy):
    """[(MatchResources.GetKinds, HasValidate)] of autogen.ComputeRules(policy), from the compiler"""
    rs = E.Ruleset([policy])
    return [(r["match_kinds"], r["has_validate"]) for r in rs.rules]


class PolicyCache:
    """policycache.Cache restricted to the validate policy types"""

    def __init__(self):
        self._lock = threading.RLock()
        self.policies = {}
        self.kind_type = {}  # kind -> {type -> {key: None}} (ordered set)

    def set(self, key, policy, subresource_gvk_to_kind=None, rules=None):
        """store.go:96-138; `rules` = rule_kinds(policy) when the caller already compiled it"""
        sub = subresource_gvk_to_kind or {}
        enforce = A.compute_enforce_policy(policy)
        has_val = {}
        for kinds, validate in (rules if rules is not None else rule_kinds(policy)):
            for gvk in kinds:
                kind = sub.get(gvk)
                if kind is None:
                    kind = A.compute_kind(gvk)
                has_val[kind] = has_val.get(kind, False) or bool(validate)
        with self._lock:
            self.policies[key] = policy
            for kind, validate in has_val.items():
                t = self.kind_type.setdefault(kind, {ty: {} for ty in TYPES})
                for ty, on in ((VALIDATE_ENFORCE, validate and enforce), (VALIDATE_AUDIT, validate and not enforce)):
                    if on:
                        t[ty][key] = None
                    else:
                        t[ty].pop(key, None)

    def unset(self, key):
        """store.go:140-146"""
        with self._lock:
            self.policies.pop(key, None)
            for t in self.kind_type.values():
                for s in t.values():
                    s.pop(key, None)

    def get_keys(self, ptype, gvk, namespace):
        """store.go:148-171, as policy keys"""
        kind = A.compute_kind(gvk)
        out = []
        with self._lock:
            for key in (self.kind_type.get(kind) or {}).get(ptype) or {}:
                ns, _ = split_key(key)
                if (ns == "" and namespace == "") or ns == namespace:
                    out.append(key)
        return out

    def get(self, ptype, gvk, namespace):
        return [self.policies[k] for k in self.get_keys(ptype, gvk, namespace)]

    def get_policy_keys(self, ptype, kind, nspace):
        """cache.go:38-57 GetPolicies, as policy keys (duplicates kept, as the reference's appends keep them)"""
        keys = self.get_keys(ptype, kind, "") + self.get_keys(ptype, "*", "")
        if nspace != "":
            keys += self.get_keys(ptype, kind, nspace) + self.get_keys(ptype, "*", nspace)
        if ptype == VALIDATE_AUDIT:
            keys += self.get_keys(VALIDATE_ENFORCE, kind, "") + self.get_keys(VALIDATE_ENFORCE, "*", "")
        if ptype in TYPES:
            enforce = ptype == VALIDATE_ENFORCE
            keys = [k for k in keys if check_overrides(enforce, nspace, self.policies[k])]
        return keys

    def get_policies(self, ptype, kind, nspace):
        return [self.policies[k] for k in self.get_policy_keys(ptype, kind, nspace)]


def check_overrides(enforce, ns, policy):
    """cache.go:73-89 checkValidationFailureActionOverrides"""
    s = policy.get("spec") or {}
    overrides = s.get("validationFailureActionOverrides") or []
    if A.action_enforce(s.get("validationFailureAction", "")) != enforce and (ns == "" or not overrides):
        return False
    for o in overrides:
        if A.action_enforce((o or {}).get("action")) != enforce and A.check_patterns((o or {}).get("namespaces"), ns):
            return False
    return True
