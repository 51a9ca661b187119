// ORACLE — test infrastructure only (see ojson.h header).
//
// Engine-level restatement of the validate path for background-scan semantics (empty admission info,
// no PolicyExceptions, no discovery subresources):
//   pkg/engine/validation.go:39-183 (Validate/validateResource), :276-317 (validator.validate dispatch),
//     :535-566 (validatePodSecurity), :600-615 (matches, incl. the always-taken OldResource retry),
//     :618-702 (validatePatterns), :722-758 (messages)
//   pkg/engine/utils.go:37-289 (match/exclude), pkg/utils/match/*.go, pkg/utils/kube/kind.go
//   pkg/autogen/autogen.go:70-314 + rule.go:73-319 (ComputeRules)
//   k8s.io/apimachinery v0.26.1 labels selectors (LabelSelectorAsSelector / Requirement.Matches) — restated
#include "oengine.h"
#include "orefs.h"
#include "ojmes.h"

#include <algorithm>
#include <set>

#include "goutil.h"
#include "ocond.h"
#include "opss.h"
#include "otyped.h"
#include "ovalidate.h"

namespace orc {
using oj::T;
using oj::Value;
using oj::VP;

static bool isnil(const VP& v) { return !v || v->t == T::Null; }

static std::vector<std::string> str_list(const VP& v) {
  std::vector<std::string> out;
  if (v && v->t == T::Arr)
    for (auto& e : v->a) out.push_back(e && e->t == T::Str ? e->s : "");
  return out;
}

// ---------------- unstructured accessors (apimachinery unstructured helpers) ----------------
static bool nested(const VP& obj, std::initializer_list<const char*> path, VP& out) {
  VP cur = obj;
  for (const char* f : path) {
    if (!cur || cur->t != T::Obj) return false;
    auto it = cur->o.find(f);
    if (it == cur->o.end()) return false;
    cur = it->second;
  }
  out = cur;
  return true;
}
std::string nested_string(const VP& obj, std::initializer_list<const char*> path) {
  VP v;
  if (!nested(obj, path, v) || !v || v->t != T::Str) return "";
  return v->s;
}
// NestedStringMap -> nil on any error (non-map / non-string value)
static bool nested_string_map(const VP& obj, std::initializer_list<const char*> path, std::map<std::string, std::string>& out) {
  VP v;
  out.clear();
  if (!nested(obj, path, v)) return false;
  if (isnil(v)) return false;
  if (v->t != T::Obj) return false;
  for (auto& kv : v->o) {
    if (!kv.second || kv.second->t != T::Str) { out.clear(); return false; }
    out[kv.first] = kv.second->s;
  }
  return true;
}

struct Res {
  bool empty = true;
  std::string kind, name, genName, ns;
  std::string group, version, gvkKind;  // GroupVersionKind()
  bool hasLabels = false, hasAnn = false;
  std::map<std::string, std::string> labels, ann;
};

static Res res_info(const VP& obj) {
  Res r;
  if (!obj) return r;
  r.empty = false;
  r.kind = nested_string(obj, {"kind"});
  r.name = nested_string(obj, {"metadata", "name"});
  r.genName = nested_string(obj, {"metadata", "generateName"});
  r.ns = nested_string(obj, {"metadata", "namespace"});
  r.hasLabels = nested_string_map(obj, {"metadata", "labels"}, r.labels);
  r.hasAnn = nested_string_map(obj, {"metadata", "annotations"}, r.ann);
  std::string av = nested_string(obj, {"apiVersion"});
  size_t slashes = std::count(av.begin(), av.end(), '/');
  if (av.empty() || av == "/") { r.gvkKind = r.kind; }
  else if (slashes == 0) { r.version = av; r.gvkKind = r.kind; }
  else if (slashes == 1) { size_t i = av.find('/'); r.group = av.substr(0, i); r.version = av.substr(i + 1); r.gvkKind = r.kind; }
  else { /* ParseGroupVersion error -> empty GVK */ }
  return r;
}

// ---------------- kinds (pkg/utils/kube/kind.go, pkg/utils/match/kind.go) ----------------
static bool version_regex(const std::string& s) {  // v\d((alpha|beta)\d)? unanchored
  for (size_t i = 0; i + 1 < s.size(); i++) if (s[i] == 'v' && s[i + 1] >= '0' && s[i + 1] <= '9') return true;
  return false;
}
static std::string format_subresource(std::string s) {
  size_t i = s.find('.');
  if (i != std::string::npos) s[i] = '/';
  return s;
}
void get_kind_from_gvk(const std::string& str, std::string& gv, std::string& kind) {
  auto parts = gou::split(str, '/');
  gv.clear();
  if (parts.size() == 2) {
    if (version_regex(parts[0]) || parts[0] == "*") { gv = parts[0]; kind = format_subresource(parts[1]); }
    else kind = parts[0] + "/" + parts[1];
  } else if (parts.size() == 3) {
    if (version_regex(parts[0]) || parts[0] == "*") { gv = parts[0]; kind = parts[1] + "/" + parts[2]; }
    else { gv = parts[0] + "/" + parts[1]; kind = format_subresource(parts[2]); }
  } else if (parts.size() == 4) {
    gv = parts[0] + "/" + parts[1];
    kind = parts[2] + "/" + parts[3];
  } else {
    kind = format_subresource(str);
  }
}
static bool parse_gv(const std::string& s, std::string& g, std::string& v) {
  g.clear(); v.clear();
  if (s.empty() || s == "/") return true;
  size_t n = std::count(s.begin(), s.end(), '/');
  if (n == 0) { v = s; return true; }
  if (n == 1) { size_t i = s.find('/'); g = s.substr(0, i); v = s.substr(i + 1); return true; }
  return false;
}
static bool group_version_matches(const std::string& gv, const std::string& server) {
  if (gv.find('*') != std::string::npos) {
    std::string p = gv;
    if (!p.empty() && p.back() == '*') p.pop_back();
    return server.compare(0, p.size(), p) == 0;
  }
  std::string g1, v1, g2, v2;
  if (parse_gv(gv, g1, v1)) {
    parse_gv(server, g2, v2);
    return g1 == g2 && v1 == v2;
  }
  return false;
}
static bool check_kind(const std::vector<std::string>& kinds, const Res& r) {
  std::string serverGV = r.group.empty() ? r.version : r.group + "/" + r.version;
  for (auto& k : kinds) {
    bool result;
    if (k != "*") {
      std::string gv, kind;
      get_kind_from_gvk(k, gv, kind);
      result = kind == r.gvkKind;
      if (!gv.empty()) result = result && group_version_matches(gv, serverGV);
    } else {
      result = true;
    }
    if (result) return true;
  }
  return false;
}

// ---------------- label selectors (apimachinery) ----------------
static bool qname_char(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }
static bool qualified_name_part(const std::string& n) {  // ([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9], len<=63
  if (n.empty() || n.size() > 63) return false;
  if (!qname_char(n.front()) || !qname_char(n.back())) return false;
  for (char c : n) if (!(qname_char(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}
static bool dns1123_subdomain(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  for (auto& lab : gou::split(s, '.')) {
    if (lab.empty()) return false;
    auto alnum = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!alnum(lab.front()) || !alnum(lab.back())) return false;
    for (char c : lab) if (!(alnum(c) || c == '-')) return false;
  }
  return true;
}
static bool valid_label_key(const std::string& k) {
  auto parts = gou::split(k, '/');
  if (parts.size() == 1) return qualified_name_part(parts[0]);
  if (parts.size() == 2) return !parts[0].empty() && dns1123_subdomain(parts[0]) && qualified_name_part(parts[1]);
  return false;
}
static bool valid_label_value(const std::string& v) { return v.empty() || qualified_name_part(v); }

struct Req { std::string key, op; std::vector<std::string> vals; };

// CheckSelector (pkg/utils/match/labels.go:10-24) incl. wildcards.ReplaceInSelector; returns 0 no match, 1 match,
// -1 error (invalid selector), and flags nondeterminism when several labels can satisfy a wildcard entry.
static int check_selector(const VP& sel, const std::map<std::string, std::string>& labels, bool* nd) {
  if (isnil(sel)) return 0;
  std::vector<Req> reqs;
  VP ml = sel->get("matchLabels");
  std::map<std::string, std::string> result;
  if (ml && ml->t == T::Obj) {
    for (auto& kv : ml->o) {
      std::string k = kv.first, v = kv.second && kv.second->t == T::Str ? kv.second->s : "";
      if (gou::contains_wildcard(k) || gou::contains_wildcard(v)) {
        int n = 0;
        std::string mk, mv;
        for (auto& lv : labels)
          if (gou::wildcard_match(k, lv.first) && gou::wildcard_match(v, lv.second)) {
            if (n == 0) { mk = lv.first; mv = lv.second; }
            n++;
          }
        if (n > 1 && nd) *nd = true;
        if (n == 0) {
          for (auto& c : k) if (c == '*' || c == '?') c = '0';
          for (auto& c : v) if (c == '*' || c == '?') c = '0';
          mk = k; mv = v;
        }
        if (result.count(mk) && nd) *nd = true;
        result[mk] = mv;
      } else {
        if (result.count(k) && nd) *nd = true;
        result[k] = v;
      }
    }
  }
  VP me = sel->get("matchExpressions");
  size_t nexpr = me && me->t == T::Arr ? me->a.size() : 0;
  if (result.empty() && nexpr == 0) return 1;  // Everything
  for (auto& kv : result) reqs.push_back(Req{kv.first, "=", {kv.second}});
  for (size_t i = 0; i < nexpr; i++) {
    VP e = me->a[i];
    std::string op = oj::get_str(e, "operator");
    std::string o;
    if (op == "In") o = "in";
    else if (op == "NotIn") o = "notin";
    else if (op == "Exists") o = "exists";
    else if (op == "DoesNotExist") o = "!";
    else return -1;
    reqs.push_back(Req{oj::get_str(e, "key"), o, str_list(e ? e->get("values") : nullptr)});
  }
  for (auto& r : reqs) {  // NewRequirement validation
    if (!valid_label_key(r.key)) return -1;
    if ((r.op == "in" || r.op == "notin") && r.vals.empty()) return -1;
    if (r.op == "=" && r.vals.size() != 1) return -1;
    if ((r.op == "exists" || r.op == "!") && !r.vals.empty()) return -1;
    for (auto& v : r.vals) if (!valid_label_value(v)) return -1;
  }
  for (auto& r : reqs) {
    auto it = labels.find(r.key);
    bool has = it != labels.end();
    bool inset = has && std::find(r.vals.begin(), r.vals.end(), it->second) != r.vals.end();
    bool ok;
    if (r.op == "=" || r.op == "in") ok = inset;
    else if (r.op == "notin") ok = !has || !inset;
    else if (r.op == "exists") ok = has;
    else ok = !has;
    if (!ok) return 0;
  }
  return 1;
}

// ---------------- match / exclude (pkg/engine/utils.go) ----------------
static bool rd_is_zero(const VP& rd) {
  if (isnil(rd)) return true;
  for (const char* k : {"kinds", "names", "namespaces", "annotations", "selector", "namespaceSelector"})
    if (!isnil(rd->get(k))) return false;
  return oj::get_str(rd, "name").empty();
}
static bool ui_is_zero(const VP& f) {
  if (isnil(f)) return true;
  for (const char* k : {"roles", "clusterRoles", "subjects"})
    if (!isnil(f->get(k))) return false;
  return true;
}

// doesResourceMatchConditionBlock (utils.go:71-160): true when no errors. exc: the checkResourceDescription /
// checkUserInfo form of pkg/utils/match/match.go:110-203 (PolicyException match), whose namespaceSelector is skipped
// for every resource with an empty kind
static bool condition_block(const VP& rd, const VP& ui, const Res& r, const std::map<std::string, std::string>& nsLabels,
                            bool* nd, bool exc = false) {
  bool ok = true;
  std::vector<std::string> kinds = str_list(rd ? rd->get("kinds") : nullptr);
  if (!kinds.empty() && !check_kind(kinds, r)) ok = false;
  std::string rname = r.name.empty() ? r.genName : r.name;
  std::string name = oj::get_str(rd, "name");
  if (!name.empty() && !gou::wildcard_match(name, rname)) ok = false;
  auto names = str_list(rd ? rd->get("names") : nullptr);
  if (!names.empty()) {
    bool any = false;
    for (auto& n : names) if (gou::wildcard_match(n, rname)) { any = true; break; }
    if (!any) ok = false;
  }
  auto nss = str_list(rd ? rd->get("namespaces") : nullptr);
  if (!nss.empty()) {
    std::string rns = r.kind == "Namespace" ? r.name : r.ns;
    bool any = false;
    for (auto& n : nss) if (gou::wildcard_match(n, rns)) { any = true; break; }
    if (!any) ok = false;
  }
  VP ann = rd ? rd->get("annotations") : nullptr;
  if (ann && ann->t == T::Obj && !ann->o.empty()) {
    for (auto& kv : ann->o) {
      std::string v = kv.second && kv.second->t == T::Str ? kv.second->s : "";
      bool m = false;
      for (auto& a : r.ann)
        if (gou::wildcard_match(kv.first, a.first) && gou::wildcard_match(v, a.second)) { m = true; break; }
      if (!m) { ok = false; break; }
    }
  }
  VP sel = rd ? rd->get("selector") : nullptr;
  if (!isnil(sel)) {
    if (check_selector(sel, r.labels, nd) != 1) ok = false;
  }
  VP nsel = rd ? rd->get("namespaceSelector") : nullptr;
  if (!isnil(nsel) && r.kind != "Namespace" &&
      (!r.kind.empty() || (!exc && std::find(kinds.begin(), kinds.end(), "*") != kinds.end()))) {
    if (check_selector(nsel, nsLabels, nd) != 1) ok = false;
  }
  // userInfo with empty admission info: roles / clusterRoles / subjects never satisfied
  if (!isnil(ui)) {
    if (!str_list(ui->get("roles")).empty()) ok = false;
    if (!str_list(ui->get("clusterRoles")).empty()) ok = false;
    VP subj = ui->get("subjects");
    if (subj && subj->t == T::Arr && !subj->a.empty()) ok = false;
  }
  return ok;
}

// matchesResourceDescriptionMatchHelper: errors? (true = matched)
static bool match_helper(const VP& filter_rd, const Res& r, const std::map<std::string, std::string>& nsl, bool* nd) {
  // empty admission info => userInfo cleared
  if (rd_is_zero(filter_rd)) return false;  // "match cannot be empty"
  return condition_block(filter_rd, nullptr, r, nsl, nd);
}
// matchesResourceDescriptionExcludeHelper: true = excluded
static bool exclude_helper(const VP& filter_rd, const VP& ui, const Res& r, const std::map<std::string, std::string>& nsl,
                           bool* nd) {
  if (rd_is_zero(filter_rd) && ui_is_zero(ui)) return false;
  return condition_block(filter_rd, ui, r, nsl, nd);
}

bool matches_resource_description(const VP& rule, const VP& resource, const std::map<std::string, std::string>& nsl,
                                  bool* nd) {  // utils.go:185-256
  Res r = res_info(resource);
  VP match = rule->get("match"), exclude = rule->get("exclude");
  bool failed = false;
  VP any = match ? match->get("any") : nullptr, all = match ? match->get("all") : nullptr;
  if (any && any->t == T::Arr && !any->a.empty()) {
    bool one = false;
    for (auto& f : any->a) if (match_helper(f ? f->get("resources") : nullptr, r, nsl, nd)) { one = true; break; }
    if (!one) failed = true;
  } else if (all && all->t == T::Arr && !all->a.empty()) {
    for (auto& f : all->a) if (!match_helper(f ? f->get("resources") : nullptr, r, nsl, nd)) failed = true;
  } else {
    if (!match_helper(match ? match->get("resources") : nullptr, r, nsl, nd)) failed = true;
  }
  VP eany = exclude ? exclude->get("any") : nullptr, eall = exclude ? exclude->get("all") : nullptr;
  if (eany && eany->t == T::Arr && !eany->a.empty()) {
    for (auto& f : eany->a) if (exclude_helper(f ? f->get("resources") : nullptr, f, r, nsl, nd)) failed = true;
  } else if (eall && eall->t == T::Arr && !eall->a.empty()) {
    bool byAll = true;
    for (auto& f : eall->a) if (!exclude_helper(f ? f->get("resources") : nullptr, f, r, nsl, nd)) { byAll = false; break; }
    if (byAll) failed = true;
  } else if (exclude) {
    if (exclude_helper(exclude->get("resources"), exclude, r, nsl, nd)) failed = true;
  }
  return !failed;
}

// ---------------- PolicyException (validation.go:797-848, pkg/utils/match/match.go:26-108) ----------------
static std::vector<VP> g_exceptions;  // set before a run starts; read-only while it runs
void set_exceptions(const std::vector<VP>& ex) { g_exceptions = ex; }

// CheckMatchesResources with empty admission info: true = no errors (the exception applies)
static bool check_matches_resources(const VP& match, const Res& r, const std::map<std::string, std::string>& nsl, bool* nd) {
  VP any = match ? match->get("any") : nullptr, all = match ? match->get("all") : nullptr;
  auto filter = [&](const VP& f) {  // checkResourceFilter: "statement cannot be empty" when both parts are zero
    VP rd = f ? f->get("resources") : nullptr;
    if (rd_is_zero(rd) && ui_is_zero(f)) return false;
    return condition_block(rd, f, r, nsl, nd, true);
  };
  if (any && any->t == T::Arr && !any->a.empty()) {
    for (auto& f : any->a) if (filter(f)) return true;
    return false;
  }
  if (all && all->t == T::Arr && !all->a.empty()) {
    bool ok = true;
    for (auto& f : all->a) if (!filter(f)) ok = false;
    return ok;
  }
  return true;  // neither any nor all: no errors
}

// matchesException: key (cache.MetaNamespaceKeyFunc) of the first exception (FindExceptions order = input order)
// listing (policy key, rule) whose match applies to the resource, or "" when none does
static std::string matching_exception(const std::string& pkey, const std::string& rule, const VP& resource,
                                      const std::map<std::string, std::string>& nsl, bool* nd) {
  Res r = res_info(resource);
  for (auto& ex : g_exceptions) {
    VP spec = ex ? ex->get("spec") : nullptr;
    VP lst = spec ? spec->get("exceptions") : nullptr;
    if (oj::get_str(ex, "kind") != "PolicyException" || !lst || lst->t != T::Arr) continue;
    bool named = false;
    for (auto& e : lst->a) {  // Exception.Contains (policy_exception_types.go:100-103)
      if (oj::get_str(e, "policyName") != pkey) continue;
      for (auto& rn : str_list(e ? e->get("ruleNames") : nullptr)) if (rn == rule) named = true;
    }
    if (!named) continue;
    if (check_matches_resources(spec->get("match"), r, nsl, nd)) {
      std::string ns = nested_string(ex, {"metadata", "namespace"}), nm = nested_string(ex, {"metadata", "name"});
      return ns.empty() ? nm : ns + "/" + nm;
    }
  }
  return "";
}

// ---------------- autogen (pkg/autogen) ----------------
static bool contains_kind(const std::vector<std::string>& list, const std::string& kind) {
  for (auto& e : list) {
    std::string gv, k;
    get_kind_from_gvk(e, gv, k);
    auto parts = gou::split(k, '/');
    if (parts.size() == 2) k = parts[0];
    if (k == kind) return true;
  }
  return false;
}
static std::vector<std::string> get_kinds(const VP& mr) {  // MatchResources.GetKinds
  std::vector<std::string> out;
  if (isnil(mr)) return out;
  VP rd = mr->get("resources");
  for (auto& k : str_list(rd ? rd->get("kinds") : nullptr)) out.push_back(k);
  for (const char* blk : {"all", "any"}) {
    VP l = mr->get(blk);
    if (l && l->t == T::Arr)
      for (auto& f : l->a) {
        VP frd = f ? f->get("resources") : nullptr;
        for (auto& k : str_list(frd ? frd->get("kinds") : nullptr)) out.push_back(k);
      }
  }
  return out;
}
static bool check_autogen_support(bool& needed, const VP& rd) {
  if (isnil(rd)) return true;
  static const std::set<std::string> podctl = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet",
                                               "ReplicationController", "CronJob", "Pod"};
  auto kinds = str_list(rd->get("kinds"));
  if (!oj::get_str(rd, "name").empty() || !str_list(rd->get("names")).empty() || !isnil(rd->get("selector")) ||
      !isnil(rd->get("annotations")) || (kinds.size() > 1 && contains_kind(kinds, "Pod")))
    return false;
  for (auto& k : kinds) if (podctl.count(k)) needed = true;
  return true;
}
bool has_nonempty(const VP& o, const char* k) {
  VP v = o ? o->get(k) : nullptr;
  if (isnil(v)) return false;
  if (v->t == T::Obj) return !v->o.empty();
  if (v->t == T::Arr) return !v->a.empty();
  if (v->t == T::Str) return !v->s.empty();
  return true;
}
static bool can_autogen(const VP& spec, std::string& controllers) {  // autogen.go:70-136
  bool needed = false;
  VP rules = spec ? spec->get("rules") : nullptr;
  if (rules && rules->t == T::Arr)
    for (auto& rule : rules->a) {
      VP mut = rule->get("mutate");
      if ((mut && !oj::get_str(mut, "patchesJson6902").empty()) || has_nonempty(rule, "generate")) {
        controllers = "none";
        return false;
      }
      VP m = rule->get("match"), e = rule->get("exclude");
      if (!check_autogen_support(needed, m ? m->get("resources") : nullptr) ||
          !check_autogen_support(needed, e ? e->get("resources") : nullptr)) { controllers = ""; return false; }
      for (VP blk : {m, e})
        for (const char* w : {"any", "all"}) {
          VP l = blk ? blk->get(w) : nullptr;
          if (l && l->t == T::Arr)
            for (auto& f : l->a)
              if (!check_autogen_support(needed, f ? f->get("resources") : nullptr)) { controllers = ""; return false; }
        }
    }
  if (!needed) { controllers = ""; return false; }
  controllers = "DaemonSet,Deployment,Job,StatefulSet,ReplicaSet,ReplicationController,CronJob";
  return true;
}

static std::string autogen_name(const std::string& prefix, const std::string& name) {
  std::string n = prefix + "-" + name;
  if (n.size() > 63) n = n.substr(0, 63);
  return n;
}

static VP replace_kinds_in_filters(const VP& filters, const std::string& match, const std::vector<std::string>& kinds) {
  VP out = oj::deep_copy(filters);
  for (auto& f : out->a) {
    VP rd = f ? f->get("resources") : nullptr;
    if (rd && contains_kind(str_list(rd->get("kinds")), match)) {
      auto arr = Value::arr();
      for (auto& k : kinds) arr->a.push_back(Value::str(k));
      rd->o["kinds"] = arr;
    }
  }
  return out;
}

static VP kinds_arr(const std::vector<std::string>& kinds) {
  auto arr = Value::arr();
  for (auto& k : kinds) arr->a.push_back(Value::str(k));
  return arr;
}

static bool validation_nonempty(const VP& v) { return v && v->t == T::Obj && !v->o.empty(); }

// generateRule (rule.go:73-204)
static VP generate_rule(const std::string& name, const VP& rule0, const std::string& tplKey, const std::vector<std::string>& kinds,
                        const std::string& grfKind) {
  if (!rule0) return nullptr;
  VP rule = oj::deep_copy(rule0);
  rule->o["name"] = Value::str(name);
  VP m = rule->get("match");
  if (!m) { m = Value::obj(); rule->o["match"] = m; }
  if (m->get("any") && m->get("any")->t == T::Arr && !m->get("any")->a.empty()) m->o["any"] = replace_kinds_in_filters(m->get("any"), grfKind, kinds);
  else if (m->get("all") && m->get("all")->t == T::Arr && !m->get("all")->a.empty()) m->o["all"] = replace_kinds_in_filters(m->get("all"), grfKind, kinds);
  else {
    VP rd = m->get("resources");
    if (isnil(rd)) { rd = Value::obj(); m->o["resources"] = rd; }
    rd->o["kinds"] = kinds_arr(kinds);
  }
  VP e = rule->get("exclude");
  if (e) {
    if (e->get("any") && e->get("any")->t == T::Arr && !e->get("any")->a.empty()) e->o["any"] = replace_kinds_in_filters(e->get("any"), grfKind, kinds);
    else if (e->get("all") && e->get("all")->t == T::Arr && !e->get("all")->a.empty()) e->o["all"] = replace_kinds_in_filters(e->get("all"), grfKind, kinds);
    else {
      VP rd = e->get("resources");
      if (rd && !str_list(rd->get("kinds")).empty()) rd->o["kinds"] = kinds_arr(kinds);
    }
  }
  VP mut = rule->get("mutate");
  if (mut && (!isnil(mut->get("patchStrategicMerge")) || has_nonempty(mut, "foreach"))) {
    return rule;  // mutation branches keep the validation untouched (not exercised on the validate path)
  }
  VP val = rule->get("validate");
  if (!val) return nullptr;
  std::string msg = oj::get_str(val, "message");
  auto wrap = [&](const VP& p) {
    auto inner = Value::obj();
    inner->o[tplKey] = p;
    auto outer = Value::obj();
    outer->o["spec"] = inner;
    return outer;
  };
  auto nv = Value::obj();
  if (!msg.empty()) nv->o["message"] = Value::str(msg);
  if (!isnil(val->get("pattern"))) {
    nv->o["pattern"] = wrap(val->get("pattern"));
  } else if (!isnil(val->get("deny"))) {
    nv->o["deny"] = val->get("deny");
  } else if (!isnil(val->get("podSecurity"))) {
    auto ps = Value::obj();
    VP ops = val->get("podSecurity");
    if (!oj::get_str(ops, "level").empty()) ps->o["level"] = Value::str(oj::get_str(ops, "level"));
    if (!oj::get_str(ops, "version").empty()) ps->o["version"] = Value::str(oj::get_str(ops, "version"));
    VP ex = ops->get("exclude");
    if (ex && ex->t == T::Arr && !ex->a.empty()) ps->o["exclude"] = ex;
    nv->o["podSecurity"] = ps;
  } else if (!isnil(val->get("anyPattern"))) {
    auto arr = Value::arr();
    VP ap = val->get("anyPattern");
    if (ap->t == T::Arr) for (auto& p : ap->a) arr->a.push_back(wrap(p));
    nv->o["anyPattern"] = arr;
  } else if (has_nonempty(val, "foreach")) {
    nv->o["foreach"] = val->get("foreach");
  } else if (has_nonempty(rule, "verifyImages")) {
    return rule;
  } else {
    return nullptr;
  }
  rule->o["validate"] = nv;
  return rule;
}

static VP generate_rule_for_controllers(const VP& rule, std::string controllers) {  // rule.go:228-279
  std::string name = oj::get_str(rule, "name");
  if (name.compare(0, 8, "autogen-") == 0 || controllers.empty()) return nullptr;
  auto mk = get_kinds(rule->get("match")), ek = get_kinds(rule->get("exclude"));
  if (!contains_kind(mk, "Pod") || (!ek.empty() && !contains_kind(ek, "Pod"))) return nullptr;
  static const std::set<std::string> list = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet", "ReplicationController"};
  if (controllers == "all") controllers = "DaemonSet,Deployment,Job,StatefulSet,ReplicaSet,ReplicationController";
  else if (controllers != "none") {
    std::vector<std::string> v;
    for (auto& c : gou::split(controllers, ',')) if (list.count(c)) v.push_back(c);
    if (!v.empty()) {
      controllers.clear();
      for (size_t i = 0; i < v.size(); i++) { if (i) controllers += ","; controllers += v[i]; }
    }
  }
  return generate_rule(autogen_name("autogen", name), rule, "template", gou::split(controllers, ','), "Pod");
}

static VP generate_cronjob_rule(const VP& rule, const std::string& controllers) {  // rule.go:281-297
  if (controllers.find("CronJob") == std::string::npos && controllers.find("all") == std::string::npos) return nullptr;
  return generate_rule(autogen_name("autogen-cronjob", oj::get_str(rule, "name")), generate_rule_for_controllers(rule, controllers),
                       "jobTemplate", {"CronJob"}, "Job");
}

static std::string replace_all(std::string s, const std::string& from, const std::string& to) {
  size_t p = 0;
  while ((p = s.find(from, p)) != std::string::npos) { s.replace(p, from.size(), to); p += to.size(); }
  return s;
}

static VP convert_rule(const VP& rule, const std::string& kind) {  // autogen.go:238-276
  std::string b = oj::dump(rule);
  VP val = rule->get("validate");
  bool pss = val && !isnil(val->get("podSecurity"));
  if (pss) {
    if (kind == "Pod") b = replace_all(b, "\"restrictedField\":\"spec", "\"restrictedField\":\"spec.template.spec");
    else b = replace_all(b, "\"restrictedField\":\"spec", "\"restrictedField\":\"spec.jobTemplate.spec.template.spec");
    b = replace_all(b, "metadata", "spec.template.metadata");
  } else {
    if (kind == "Pod") b = replace_all(b, "request.object.spec", "request.object.spec.template.spec");
    else b = replace_all(b, "request.object.spec", "request.object.spec.jobTemplate.spec.template.spec");
    b = replace_all(b, "request.object.metadata", "request.object.spec.template.metadata");
  }
  return oj::parse(b, true);
}

std::vector<VP> compute_rules(const VP& policy) {  // autogen.go:280-314
  VP spec = policy->get("spec");
  std::vector<VP> rules;
  VP rl = spec ? spec->get("rules") : nullptr;
  if (rl && rl->t == T::Arr) rules = rl->a;
  std::string desired;
  bool apply = can_autogen(spec, desired);
  if (!apply) desired = "none";
  std::string actual = desired;
  VP ann = nullptr;
  VP meta = policy->get("metadata");
  if (meta) ann = meta->get("annotations");
  VP a = ann ? ann->get("pod-policies.kyverno.io/autogen-controllers") : nullptr;
  if (a && apply) actual = a->t == T::Str ? a->s : "";
  if (actual == "none") return rules;
  std::vector<VP> gen;
  std::string stripped;
  {
    std::vector<std::string> v;
    for (auto& c : gou::split(actual, ',')) if (c != "CronJob") v.push_back(c);
    for (size_t i = 0; i < v.size(); i++) { if (i) stripped += ","; stripped += v[i]; }
  }
  for (auto& r : rules) {
    VP g = generate_rule_for_controllers(r, stripped);
    if (g) gen.push_back(convert_rule(g, "Pod"));
    VP c = generate_cronjob_rule(r, actual);
    if (c) gen.push_back(convert_rule(c, "Cronjob"));
  }
  if (gen.empty()) return rules;
  std::vector<VP> out;
  for (auto& r : rules) if (oj::get_str(r, "name").compare(0, 8, "autogen-") != 0) out.push_back(r);
  for (auto& g : gen) out.push_back(g);
  return out;
}

// ---------------- rule evaluation (validation.go) ----------------
static bool contains_vars(const VP& v) {
  if (!v) return false;
  if (v->t == T::Str) return v->s.find("{{") != std::string::npos || v->s.find("$(") != std::string::npos;
  if (v->t == T::Arr) { for (auto& e : v->a) if (contains_vars(e)) return true; return false; }
  if (v->t == T::Obj) {
    for (auto& kv : v->o) {
      if (kv.first.find("{{") != std::string::npos || kv.first.find("$(") != std::string::npos) return true;
      if (contains_vars(kv.second)) return true;
    }
  }
  return false;
}

static bool contains_braces(const VP& v) {
  if (!v) return false;
  if (v->t == T::Str) return v->s.find("{{") != std::string::npos;
  for (auto& e : v->a) if (contains_braces(e)) return true;
  for (auto& kv : v->o) if (kv.first.find("{{") != std::string::npos || contains_braces(kv.second)) return true;
  return false;
}

// ---------------------------------------------------------------- foreach (validation.go:242-421)
// A pattern string that is exactly one element variable: `{{element}}`, `{{element.<ident>...}}` or `{{elementIndex}}`
// (the innermost element; vars.go:352-431 substitutes a whole-string variable by its typed value) -> its dotted path
// after "element" ("" for the element itself) or "#" for elementIndex
static bool element_var(const std::string& s, std::string* path) {
  if (s.size() < 4 || s.compare(0, 2, "{{") != 0 || s.compare(s.size() - 2, 2, "}}") != 0) return false;
  std::string in = s.substr(2, s.size() - 4);
  if (in.find('{') != std::string::npos || in.find('}') != std::string::npos) return false;
  in = gou::trim_space(in);
  if (in == "elementIndex") { *path = "#"; return true; }
  if (in.compare(0, 7, "element") != 0) return false;
  std::string rest = in.substr(7);
  if (!rest.empty() && rest[0] != '.') return false;
  // identifiers only: [A-Za-z_][A-Za-z0-9_]* separated by dots
  for (size_t i = 0; i < rest.size();) {
    if (rest[i] != '.') return false;
    size_t j = i + 1;
    if (j >= rest.size() || !(isalpha((unsigned char)rest[j]) || rest[j] == '_')) return false;
    while (j < rest.size() && (isalnum((unsigned char)rest[j]) || rest[j] == '_')) j++;
    i = j;
  }
  *path = rest;
  return true;
}

// a foreach pattern / anyPattern whose only variables are whole-string element variables in values
static bool foreach_pattern_ok(const VP& p) {
  if (!p) return true;
  if (p->t == T::Str) {
    if (p->s.find("$(") != std::string::npos) return false;
    if (p->s.find("{{") == std::string::npos) return true;
    std::string path;
    return element_var(p->s, &path);
  }
  if (p->t == T::Arr) { for (auto& e : p->a) if (!foreach_pattern_ok(e)) return false; return true; }
  if (p->t == T::Obj)
    for (auto& kv : p->o) {
      if (kv.first.find("{{") != std::string::npos || kv.first.find("$(") != std::string::npos) return false;
      if (!foreach_pattern_ok(kv.second)) return false;
    }
  return true;
}

// foreach entries the restatement covers: a JMESPath-subset list (over request.object, and over the enclosing
// element inside a nested foreach), per-element preconditions / elementScope, and one of deny conditions, pattern,
// anyPattern (element variables as whole-string values) or a nested foreach (three levels below the top: the
// recursion itself has no limit, deeper rules are just not run on the device); context entries and other
// variables are not restated
static bool foreach_entries_supported(const VP& fe, int depth) {
  if (!fe || fe->t != T::Arr || depth > 3) return false;  // (the device's FOREACH_MAX_NEST: deeper is not exercised)
  for (auto& e : fe->a) {
    if (!e || e->t != T::Obj) return false;
    for (auto& kv : e->o)
      if (kv.first != "list" && kv.first != "deny" && kv.first != "preconditions" && kv.first != "elementScope" &&
          kv.first != "pattern" && kv.first != "anyPattern" && kv.first != "foreach")
        return false;
    VP l = e->get("list");
    if (!l || l->t != T::Str || !jmes_supported(l->s, depth > 0)) return false;
    VP d = e->get("deny");
    if (!isnil(d)) {
      if (d->t != T::Obj || !conditions_supported_element(d->get("conditions"))) return false;
    } else if (!isnil(e->get("pattern")) || !isnil(e->get("anyPattern"))) {
      if (!foreach_pattern_ok(e->get("pattern")) || !foreach_pattern_ok(e->get("anyPattern"))) return false;
      VP ap = e->get("anyPattern");
      if (isnil(e->get("pattern")) && ap->t != T::Arr) return false;
    } else if (has_nonempty(e, "foreach")) {
      if (!foreach_entries_supported(e->get("foreach"), depth + 1)) return false;
    }
    if (!conditions_supported_element(e->get("preconditions"))) return false;
    VP es = e->get("elementScope");
    if (!isnil(es) && es->t != T::Bool) return false;
  }
  return true;
}
static bool foreach_supported(const VP& val) {
  std::string msg = oj::get_str(val, "message");
  if (msg.find("{{") != std::string::npos || msg.find("$(") != std::string::npos) return false;
  return foreach_entries_supported(val->get("foreach"), 0);
}

// Go %T of a decoded JSON element (addElementToContext error text, validation.go:395-397)
static std::string go_type_name(const VP& v) {
  if (isnil(v)) return "<nil>";
  switch (v->t) {
    case T::Bool: return "bool";
    case T::Int: case T::Float: return "float64";
    case T::Str: return "string";
    case T::Arr: return "[]interface {}";
    case T::Obj: return "map[string]interface {}";
    default: return "<nil>";
  }
}

static std::string build_error_message(const std::string& rname, const std::string& msg0, const std::string& err, const std::string& path);

// substitutePatterns (validation.go:760-782) of a foreach pattern: every whole-string element variable replaced by
// its typed value from the JSON context (numbers float64); a key missing on the way is the fork's NotFoundError
static VP subst_element_vars(const VP& p, const VP& el, int64_t idx, std::string* err) {
  if (!p || !err->empty()) return p;
  if (p->t == T::Str) {
    std::string path;
    if (!element_var(p->s, &path)) return p;
    if (path == "#") return Value::flt((double)idx);
    VP cur = json_floats(el);
    size_t i = 0;
    while (i < path.size()) {
      size_t j = path.find('.', i + 1);
      const std::string k = path.substr(i + 1, (j == std::string::npos ? path.size() : j) - i - 1);
      if (!cur || cur->t != T::Obj) { cur = Value::null(); break; }
      if (!cur->has(k)) { *err = "Unknown key \"" + k + "\" in path"; return p; }
      cur = cur->get(k);
      i = j == std::string::npos ? path.size() : j;
    }
    return cur ? cur : Value::null();
  }
  if (p->t == T::Arr) {
    auto o = Value::arr();
    for (auto& e : p->a) o->a.push_back(subst_element_vars(e, el, idx, err));
    return o;
  }
  if (p->t == T::Obj) {
    auto o = Value::obj();
    for (auto& kv : p->o) o->o[kv.first] = subst_element_vars(kv.second, el, idx, err);
    return o;
  }
  return p;
}

// validatePatterns (validation.go:618-702) of a pattern / anyPattern against `target`: the response status and message
static RuleResult pattern_response(const std::string& rname, const std::string& msg, const VP& pattern, const VP& any_pattern,
                                   const VP& target) {
  RuleResult out;
  out.name = rname;
  if (!isnil(pattern)) {
    EvalFlags fl;
    PatternResult pr = match_pattern(target, pattern, fl);
    out.nondeterministic |= fl.nondeterministic;
    if (pr.ok) { out.status = "pass"; out.message = "validation rule '" + rname + "' passed."; return out; }
    if (pr.skip) { out.status = "skip"; out.message = pr.err; return out; }
    if (pr.path.empty()) { out.status = "error"; out.message = build_error_message(rname, msg, pr.err, ""); return out; }
    out.status = "fail";
    out.path = pr.path;
    out.message = build_error_message(rname, msg, pr.err, pr.path);
    return out;
  }
  std::vector<std::string> failed, skipped;
  for (size_t idx = 0; idx < any_pattern->a.size(); idx++) {
    EvalFlags fl;
    PatternResult pr = match_pattern(target, any_pattern->a[idx], fl);
    out.nondeterministic |= fl.nondeterministic;
    if (pr.ok) {
      out.status = "pass";
      out.message = "validation rule '" + rname + "' anyPattern[" + std::to_string(idx) + "] passed.";
      return out;
    }
    std::string pre = "rule " + rname + "[" + std::to_string(idx) + "]";
    if (pr.skip) skipped.push_back(pre + " skipped: " + pr.err);
    else if (pr.path.empty()) failed.push_back(pre + " failed: " + pr.err);
    else failed.push_back(pre + " failed at path " + pr.path);
  }
  if (!skipped.empty() && failed.empty()) {
    out.status = "skip";
    for (size_t i = 0; i < skipped.size(); i++) out.message += (i ? " " : "") + skipped[i];
    return out;
  }
  if (!failed.empty()) {
    std::string s;
    for (size_t i = 0; i < failed.size(); i++) { if (i) s += " "; s += failed[i]; }
    out.status = "fail";
    if (msg.empty()) out.message = "validation error: " + s;
    else if (msg.back() == '.') out.message = "validation error: " + msg + " " + s;
    else out.message = "validation error: " + msg + ". " + s;
    return out;
  }
  out.status = "pass";
  out.message = msg;
  return out;
}

// validateForEach (validation.go:319-341) over the entries `fes` at nesting level `depth`: `el` / `idx` the enclosing
// element (null at the top), `root` what a pattern validates when the element is not element-scoped (the resource at
// the top -- NewResource, integers int64 --, else the enclosing scoped element: PolicyContext.Copy keeps it)
static RuleResult foreach_level(const VP& rule, const VP& fes, const VP& resource, const VP& el, int64_t idx, const VP& root,
                                int depth) {
  VP val = rule->get("validate");
  const std::string msg = oj::get_str(val, "message");
  RuleResult out;
  out.name = oj::get_str(rule, "name");
  int applyCount = 0;
  for (auto& fe : fes->a) {
    VP list;
    try {
      list = jmes_query(fe->get("list")->s, resource, el, idx);  // evaluateList (utils.go:343-355)
    } catch (JmesNotFound&) {
      continue;
    } catch (JmesError&) {
      continue;
    }
    std::vector<VP> elements;
    if (list && list->t == T::Arr) elements = list->a; else elements.push_back(list);
    VP scope = fe->get("elementScope");
    int count = 0;
    // validateElements (validation.go:343-381)
    for (size_t i = 0; i < elements.size(); i++) {
      const VP& e = elements[i];
      if (isnil(e)) continue;
      if (!isnil(scope) && scope->b && e->t != T::Obj) {  // addElementToContext error: ruleError, returned as is
        out.status = "error";
        out.message = "failed to process foreach: cannot use elementScope=true foreach rules for elements that are not "
                      "maps, expected type=map got type=" + go_type_name(e);
        return out;
      }
      const bool scoped = isnil(scope) ? e->t == T::Obj : scope->b;
      const VP target = scoped ? json_floats(e) : root;
      // the element's own validator (validate(), validation.go:276-317): preconditions, then deny / pattern / foreach
      RuleResult r;
      bool have = true;
      CondResult pc = eval_conditions_element(fe->get("preconditions"), resource, e, (int64_t)i);
      if (pc.r == CondOutcome::Unsupported) { out.status = "unsupported"; out.message = "foreach preconditions"; return out; }
      if (pc.r == CondOutcome::Error) {
        r.status = "error";
        r.message = "failed to evaluate preconditions: failed to substitute variables in preconditions: " + pc.err;
        out.message_unpinned |= pc.err_unpinned;
      } else if (pc.r == CondOutcome::False) {
        r.status = "skip";  // "preconditions not met"
      } else if (!isnil(fe->get("deny"))) {
        CondResult c = eval_conditions_element(fe->get("deny")->get("conditions"), resource, e, (int64_t)i);
        if (c.r == CondOutcome::Unsupported) { out.status = "unsupported"; out.message = "foreach deny"; return out; }
        if (c.r == CondOutcome::Error) {
          r.status = "error";
          r.message = "failed to substitute variables in deny conditions: " + c.err;
          out.message_unpinned |= c.err_unpinned;
        } else if (c.r == CondOutcome::True) {
          r.status = "fail";
          r.message = msg.empty() ? "validation error: rule " + out.name + " failed" : msg;
        } else {
          r.status = "pass";
        }
      } else if (!isnil(fe->get("pattern")) || !isnil(fe->get("anyPattern"))) {
        std::string err;
        VP pat = subst_element_vars(fe->get("pattern"), e, (int64_t)i, &err);
        VP ap = subst_element_vars(fe->get("anyPattern"), e, (int64_t)i, &err);
        if (!err.empty()) {
          r.status = "error";
          r.message = "variable substitution failed: " + err;
          out.message_unpinned = true;  // the fork's NotFoundError text is not pinned by a fixture
        } else {
          r = pattern_response(out.name, msg, pat, ap, target);
          out.nondeterministic |= r.nondeterministic;
        }
      } else if (has_nonempty(fe, "foreach")) {
        r = foreach_level(rule, fe->get("foreach"), resource, e, (int64_t)i, target, depth + 1);
        if (r.status == "unsupported") return r;
        out.nondeterministic |= r.nondeterministic;
        out.message_unpinned |= r.message_unpinned;
      } else {
        have = false;  // no validator: "skip rule due to empty result"
      }
      if (!have || r.status == "skip") continue;
      if (r.status == "pass") { count++; continue; }
      if (r.status == "error" && i + 1 < elements.size()) continue;  // an error ends it only on the last element
      out.status = r.status;
      out.message = "validation failure: " + r.message;
      return out;
    }
    applyCount += count;
  }
  if (applyCount == 0) { out.status = "skip"; out.message = "rule skipped"; return out; }
  out.status = "pass";
  out.message = "rule passed";
  return out;
}

static RuleResult validate_foreach(const VP& rule, const VP& resource, RuleResult out) {
  RuleResult r = foreach_level(rule, rule->get("validate")->get("foreach"), resource, nullptr, 0, resource, 0);
  r.name = out.name;
  return r;
}

std::string rule_unsupported_reason(const VP& rule) {
  VP val = rule->get("validate");
  if (has_nonempty(rule, "context")) return "context";
  if (!isnil(rule->get("preconditions")) && !conditions_supported(rule->get("preconditions"))) return "preconditions";
  if (has_nonempty(rule, "verifyImages")) return "verifyImages";
  if (!val) return "";
  if (!isnil(val->get("deny"))) {
    VP d = val->get("deny");
    if (d->t != T::Obj || !conditions_supported(d->get("conditions"))) return "deny";
  }
  // $() references are restated (orefs.cpp); `{{ }}` variables in patterns are not
  if (contains_braces(val->get("pattern")) || contains_braces(val->get("anyPattern"))) return "variables";
  if (isnil(val->get("pattern")) && isnil(val->get("anyPattern")) && isnil(val->get("podSecurity")) && has_nonempty(val, "foreach") &&
      !foreach_supported(val))
    return "foreach";
  if (!isnil(val->get("manifests"))) return "manifests";
  return "";
}

static std::string build_error_message(const std::string& rname, const std::string& msg0, const std::string& err, const std::string& path) {
  if (msg0.empty()) {
    if (!path.empty()) return "validation error: rule " + rname + " failed at path " + path;
    return "validation error: rule " + rname + " execution error: " + err;
  }
  std::string msg = msg0;
  if (msg.empty() || msg.back() != '.') msg += ".";
  if (!path.empty()) return "validation error: " + msg + " rule " + rname + " failed at path " + path;
  return "validation error: " + msg + " rule " + rname + " execution error: " + err;
}

static RuleResult validate_rule_body(const VP& rule, const VP& resource) {
  RuleResult out;
  out.name = oj::get_str(rule, "name");
  std::string why = rule_unsupported_reason(rule);
  if (!why.empty()) { out.status = "unsupported"; out.message = why; return out; }
  VP val = rule->get("validate");
  std::string msg = oj::get_str(val, "message");
  try {
    VP pre = rule->get("preconditions");
    if (!isnil(pre)) {  // checkPreconditions (validation.go:281-288, utils.go:328-341)
      CondResult c = eval_conditions(pre, resource);
      if (c.r == CondOutcome::Unsupported) { out.status = "unsupported"; out.message = "preconditions"; return out; }
      if (c.r == CondOutcome::Error) {
        out.status = "error";
        out.message = "failed to evaluate preconditions: failed to substitute variables in preconditions: " + c.err;
        out.message_unpinned = c.err_unpinned;
        return out;
      }
      if (c.r != CondOutcome::True) { out.status = "skip"; out.message = "preconditions not met"; return out; }
    }
    if (!isnil(val->get("deny"))) {  // validateDeny (validation.go:437-479)
      CondResult c = eval_conditions(val->get("deny")->get("conditions"), resource);
      if (c.r == CondOutcome::Unsupported) { out.status = "unsupported"; out.message = "deny"; return out; }
      if (c.r == CondOutcome::Error) {
        out.status = "error";
        out.message = "failed to substitute variables in deny conditions: " + c.err;
        out.message_unpinned = c.err_unpinned;
        return out;
      }
      if (c.r == CondOutcome::True) {
        out.status = "fail";
        bool unp = false;
        out.message = msg.empty() ? "validation error: rule " + out.name + " failed" : render_message(msg, resource, &unp);
        out.message_unpinned = unp;
        out.deny_message = true;
      } else {
        out.status = "pass";
        out.message = "validation rule '" + out.name + "' passed.";
      }
      return out;
    }
    VP pattern = val->get("pattern"), any_pattern = val->get("anyPattern");
    if (!isnil(pattern) || !isnil(any_pattern)) {  // substitutePatterns (validation.go:294-297, :760-782)
      for (VP* doc : {&pattern, &any_pattern}) {
        if (isnil(*doc) || !has_references(*doc)) continue;
        RefResult rr = substitute_references(*doc);
        out.nondeterministic |= rr.nd;
        if (!rr.ok) {
          out.status = "error";
          out.message = "variable substitution failed: " + rr.err;
          out.message_unpinned = rr.err_unpinned;
          return out;
        }
        *doc = rr.doc;
      }
    }
    if (!isnil(pattern)) {  // validatePatterns single pattern (validation.go:619-641)
      EvalFlags fl;
      PatternResult pr = match_pattern(resource, pattern, fl);
      out.nondeterministic |= fl.nondeterministic;
      if (pr.ok) { out.status = "pass"; out.message = "validation rule '" + out.name + "' passed."; return out; }
      if (pr.skip) { out.status = "skip"; out.message = pr.err; return out; }
      // buildErrorMessage substitutes the message (validation.go:731-745); its substitution-error text embeds the Go
      // error string of the pattern failure and a non-string whole-message value panics: unpinned here
      std::string head = msg;
      if (!msg.empty() && substitute_message(msg, resource, &head) != 0) { head = msg; out.message_unpinned = true; }
      if (pr.path.empty()) { out.status = "error"; out.message = build_error_message(out.name, head, pr.err, ""); return out; }
      out.status = "fail";
      out.path = pr.path;
      out.message = build_error_message(out.name, head, pr.err, pr.path);
      return out;
    }
    if (!isnil(any_pattern)) {  // validation.go:644-701
      VP ap = any_pattern;
      if (ap->t != T::Arr) {
        out.status = "error";
        out.message = "failed to deserialize anyPattern, expected type array: json: cannot unmarshal into []interface {}";
        return out;
      }
      std::vector<std::string> failed, skipped;
      for (size_t idx = 0; idx < ap->a.size(); idx++) {
        EvalFlags fl;
        PatternResult pr = match_pattern(resource, ap->a[idx], fl);
        out.nondeterministic |= fl.nondeterministic;
        if (pr.ok) {
          out.status = "pass";
          out.message = "validation rule '" + out.name + "' anyPattern[" + std::to_string(idx) + "] passed.";
          return out;
        }
        std::string pre = "rule " + out.name + "[" + std::to_string(idx) + "]";
        if (pr.skip) skipped.push_back(pre + " skipped: " + pr.err);
        else if (pr.path.empty()) failed.push_back(pre + " failed: " + pr.err);
        else failed.push_back(pre + " failed at path " + pr.path);
        out.branch_paths.push_back(pr.skip ? "<skip>" : pr.path);
      }
      if (!skipped.empty() && failed.empty()) {
        out.status = "skip";
        std::string s;
        for (size_t i = 0; i < skipped.size(); i++) { if (i) s += " "; s += skipped[i]; }
        out.message = s;
        return out;
      }
      if (!failed.empty()) {
        std::string s;
        for (size_t i = 0; i < failed.size(); i++) { if (i) s += " "; s += failed[i]; }
        out.status = "fail";
        if (msg.empty()) out.message = "validation error: " + s;
        else if (msg.back() == '.') out.message = "validation error: " + msg + " " + s;
        else out.message = "validation error: " + msg + ". " + s;
        return out;
      }
      out.status = "pass";
      out.message = msg;
      return out;
    }
    if (isnil(val->get("pattern")) && isnil(val->get("anyPattern")) && isnil(val->get("podSecurity")) &&
        has_nonempty(val, "foreach"))
      return validate_foreach(rule, resource, out);
    if (!isnil(val->get("podSecurity"))) {  // validatePodSecurity (validation.go:535-566)
      // getSpec (validation.go:481-532): typed decode of the whole object; a non-object on the way to the
      // pod template is a decode error
      std::string kind = nested_string(resource, {"kind"});
      VP meta, spec;
      bool derr = false;
      auto step = [&](const VP& o, const char* k) -> VP {
        if (derr || isnil(o)) return nullptr;
        if (o->t != T::Obj) { derr = true; return nullptr; }
        VP v = o->get(k);
        if (!isnil(v) && v->t != T::Obj) { derr = true; return nullptr; }
        return v;
      };
      static const std::set<std::string> ctl = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet", "ReplicationController"};
      // getSpec's json.Unmarshal of the whole resource (validation.go:481-532) comes before EvaluatePod's version
      // parse: a type error anywhere in the object is the rule's error (otyped.cpp, parity unpinned)
      {
        bool folded = false;
        const std::string terr = typed_decode_error(resource, kind, &folded);
        if (!terr.empty()) {
          out.status = "error";
          out.message = "Error while getting new resource: " + terr;
          out.message_unpinned = true;
          return out;
        }
        if (folded) {  // a case-folded key decodes into its field; the checks below read exact keys
          out.status = "unsupported";
          out.message = "podSecurity: case-folded keys";
          return out;
        }
      }
      VP outerMeta = step(resource, "metadata");
      if (ctl.count(kind)) {
        VP tpl = step(step(resource, "spec"), "template");
        meta = step(tpl, "metadata");
        spec = step(tpl, "spec");
      } else if (kind == "CronJob") {
        VP jt = step(step(resource, "spec"), "jobTemplate");
        meta = step(jt, "metadata");
        spec = step(step(step(jt, "spec"), "template"), "spec");
      } else if (kind == "Pod") {
        meta = outerMeta;
        spec = step(resource, "spec");
      } else {
        out.status = "panic";
        out.message = "nil pod spec";
        return out;
      }
      if (derr) { out.status = "error"; out.message = "Error while getting new resource: json: cannot unmarshal"; out.message_unpinned = true; return out; }
      VP ps = val->get("podSecurity");
      PSSEval ev = pss_evaluate(ps, meta, spec, outerMeta);
      if (!ev.decode_error.empty()) { out.status = "error"; out.message = "Error while getting new resource: " + ev.decode_error; out.message_unpinned = true; return out; }
      if (!ev.ok) { out.status = "error"; out.message = ev.error; out.message_unpinned = true; return out; }
      out.pss_checks = ev.checks;
      out.message_unpinned = ev.order_nondeterministic;
      std::string level = oj::get_str(ps, "level"), version = oj::get_str(ps, "version");
      if (ev.allowed) { out.status = "pass"; out.message = "Validation rule '" + out.name + "' passed."; return out; }
      out.status = "fail";
      out.message = "Validation rule '" + out.name + "' failed. It violates PodSecurity \"" + level + ":" + version + "\": " +
                    format_checks_print(ev.checks);
      return out;
    }
  } catch (RefPanic& p) {
    out.status = "panic";
    out.message = p.what;
    return out;
  }
  out.status = "none";  // "invalid validation rule": no response
  return out;
}

RuleResult validate_rule(const VP& rule, const VP& resource) {
  RuleResult out = validate_rule_body(rule, resource);
  // Variables in validate.message change only the message text (validation.go:469, :731), never the verdict:
  // the verdict stays pinned, the rendered text is left to the JMESPath substitution on the host.
  std::string msg = oj::get_str(rule->get("validate"), "message");
  if (!out.deny_message && (msg.find("{{") != std::string::npos || msg.find("$(") != std::string::npos))
    out.message_unpinned = true;
  return out;
}

static bool rule_has_validate(const VP& rule) {
  VP v = rule->get("validate");
  return v && v->t == T::Obj && !v->o.empty();
}

// Validate (validation.go:39-183) for one policy and one resource
PolicyResult validate_policy(const VP& policy, const VP& resource, const std::map<std::string, std::string>& nsLabels) {
  return validate_policy_rules(policy, compute_rules(policy), resource, nsLabels);
}

// validate_policy with the policy's computed rules (autogen.ComputeRules) prepared by the caller
PolicyResult validate_policy_rules(const VP& policy, const std::vector<VP>& rules, const VP& resource,
                                   const std::map<std::string, std::string>& nsLabels) {
  PolicyResult pr;
  pr.name = nested_string(policy, {"metadata", "name"});
  std::string kind = oj::get_str(policy, "kind");
  if (kind == "Policy") {  // namespaced policy filter (validation.go:124-132)
    std::string pns = nested_string(policy, {"metadata", "namespace"});
    std::string rns = nested_string(resource, {"metadata", "namespace"});
    if (rns != pns || rns.empty()) { pr.namespace_skipped = true; return pr; }
  }
  VP spec = policy->get("spec");
  bool applyOne = oj::get_str(spec, "applyRules") == "One";
  int applied = 0;
  for (auto& rule : rules) {
    if (!rule_has_validate(rule) && !has_nonempty(rule, "verifyImages")) continue;
    bool nd = false;
    bool m = matches_resource_description(rule, resource, nsLabels, &nd);
    if (!m) m = matches_resource_description(rule, nullptr, nsLabels, &nd);  // OldResource retry (validation.go:606)
    if (!m) continue;
    if (!g_exceptions.empty()) {  // hasPolicyExceptions (validation.go:158-161)
      const std::string pns = nested_string(policy, {"metadata", "namespace"});
      const std::string rname = oj::get_str(rule, "name");
      std::string key = matching_exception(pns.empty() ? pr.name : pns + "/" + pr.name, rname, resource, nsLabels, &nd);
      if (!key.empty()) {
        RuleResult rr;
        rr.name = rname;
        rr.status = "skip";
        rr.message = "rule skipped due to policy exception " + key;
        rr.nondeterministic = nd;
        pr.rules.push_back(rr);
        continue;
      }
    }
    RuleResult rr = validate_rule(rule, resource);
    rr.nondeterministic |= nd;
    if (rr.status == "none") continue;
    if (rr.status == "pass" || rr.status == "fail") applied++;
    pr.rules.push_back(rr);
    if (applyOne && applied > 0) break;
    if (rr.status == "unsupported" && applyOne) { pr.truncated_unknown = true; break; }
  }
  return pr;
}

}  // namespace orc
