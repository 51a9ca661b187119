// Policy compiler: ClusterPolicy/Policy JSON -> autogen-expanded rules -> device rule programs.
//
// Reference behaviour restated here (paths relative to /root/reference):
//   pkg/autogen/autogen.go:70-314, rule.go:73-319   ComputeRules (autogen-<rule>, autogen-cronjob-<rule>)
//   pkg/engine/validation.go:276-317                 dispatch order deny > pattern/anyPattern > podSecurity > foreach
//   pkg/engine/anchor/anchor.go:19,37-44             anchor grammar
//   pkg/engine/validate/validate.go:118-161 + utils.go:11-69  map traversal order (compile-time resolved)
//   pkg/engine/pattern/pattern.go, operator/operator.go       string pattern mini-language -> atoms
//   pkg/engine/wildcards/wildcards.go:62-151          metadata wildcard keys -> run-time slots
//   pkg/engine/utils.go:37-289, pkg/utils/match, pkg/utils/kube/kind.go   match/exclude programs
//   pkg/pss/evaluate.go, pkg/pss/utils/mapping.go     PodSecurity descriptors
// Rules needing variables, JMESPath, context, preconditions, deny, foreach or image verification are
// classified RK_FALLBACK (counted, handed back to the reference CPU engine by the caller).
#include <algorithm>
#include <cmath>
#include <list>
#include <map>
#include <set>

#include "kyv_host.h"

namespace kyv {
using pj::T;
using pj::Value;

void seed_dict(Dict& d) {
  const char* fixed[] = {"", "0", "true", "false", "*"};
  for (const char* s : fixed) d.intern(s);
  const char* wk[] = {
#define KYV_WK_STR(id, s) s,
      KYV_WELL_KNOWN(KYV_WK_STR)
#undef KYV_WK_STR
  };
  for (const char* s : wk) d.intern(s);
  const char* vs[] = {
#define KYV_VS_STR(id) #id,
      KYV_VOLUME_SOURCES(KYV_VS_STR)
#undef KYV_VS_STR
  };
  for (const char* s : vs) d.intern(s);
  if (d.strs.size() != SID_SEED_END) throw std::runtime_error("seed dictionary has duplicate entries");
}

Ruleset::~Ruleset() {}

namespace {

bool nil(const Value* v) { return !v || v->t == T::Null; }
std::vector<std::string> strs(const Value* v) {
  std::vector<std::string> out;
  if (v && v->t == T::Arr) for (auto& e : v->a) out.push_back(e.t == T::Str ? e.s : "");
  return out;
}
bool nonempty(const Value* v) {
  if (nil(v)) return false;
  if (v->t == T::Obj) return !v->o.empty();
  if (v->t == T::Arr) return !v->a.empty();
  if (v->t == T::Str) return !v->s.empty();
  return true;
}

// ---------------------------------------------------------------- anchors (anchor.go)
enum class AT { None, Cond, Global, Neg, Add, Eq, Exist };
struct Anc { AT t = AT::None; std::string key; };
Anc parse_anchor(const std::string& raw) {
  Anc a;
  std::string s = pj::go_trim_space(raw);
  if (s.size() < 3 || s.back() != ')') return a;
  size_t p = 0;
  AT t = AT::Cond;
  switch (s[0]) {
    case '+': t = AT::Add; p = 1; break;
    case '<': t = AT::Global; p = 1; break;
    case '=': t = AT::Eq; p = 1; break;
    case 'X': t = AT::Neg; p = 1; break;
    case '^': t = AT::Exist; p = 1; break;
    default: break;
  }
  if (s[p] != '(') return a;
  std::string k = s.substr(p + 1, s.size() - p - 2);
  if (k.empty() || k.find('\n') != std::string::npos) return a;
  a.t = t;
  a.key = k;
  return a;
}
std::string anchor_str(AT t, const std::string& k) {
  const char* m = t == AT::Global ? "<" : t == AT::Neg ? "X" : t == AT::Add ? "+" : t == AT::Eq ? "=" : t == AT::Exist ? "^" : "";
  return std::string(m) + "(" + k + ")";
}
bool has_wild(const std::string& s) { return s.find('*') != std::string::npos || s.find('?') != std::string::npos; }
bool has_magic(const std::string& s) {
  return s.find("negation anchor matched in resource") != std::string::npos ||
         s.find("conditional anchor mismatch") != std::string::npos || s.find("global anchor mismatch") != std::string::npos;
}

// ---------------------------------------------------------------- kinds (pkg/utils/kube/kind.go)
bool version_like(const std::string& s) {
  for (size_t i = 0; i + 1 < s.size(); i++) if (s[i] == 'v' && s[i + 1] >= '0' && s[i + 1] <= '9') return true;
  return false;
}
std::vector<std::string> split(const std::string& s, char c) {
  std::vector<std::string> out;
  size_t st = 0;
  for (size_t i = 0; i <= s.size(); i++)
    if (i == s.size() || s[i] == c) { out.push_back(s.substr(st, i - st)); st = i + 1; }
  return out;
}
std::string sub_dot(std::string s) {
  size_t i = s.find('.');
  if (i != std::string::npos) s[i] = '/';
  return s;
}
void kind_from_gvk(const std::string& str, std::string& gv, std::string& kind) {
  auto p = split(str, '/');
  gv.clear();
  if (p.size() == 2) {
    if (version_like(p[0]) || p[0] == "*") { gv = p[0]; kind = sub_dot(p[1]); } else kind = p[0] + "/" + p[1];
  } else if (p.size() == 3) {
    if (version_like(p[0]) || p[0] == "*") { gv = p[0]; kind = p[1] + "/" + p[2]; }
    else { gv = p[0] + "/" + p[1]; kind = sub_dot(p[2]); }
  } else if (p.size() == 4) {
    gv = p[0] + "/" + p[1];
    kind = p[2] + "/" + p[3];
  } else {
    kind = sub_dot(str);
  }
}
bool contains_kind(const std::vector<std::string>& l, const std::string& kind) {
  for (auto& e : l) {
    std::string gv, k;
    kind_from_gvk(e, gv, k);
    auto parts = split(k, '/');
    if (parts.size() == 2) k = parts[0];
    if (k == kind) return true;
  }
  return false;
}

// ---------------------------------------------------------------- autogen (pkg/autogen)
std::vector<std::string> match_kinds(const Value* mr) {  // MatchResources.GetKinds
  std::vector<std::string> out;
  if (nil(mr)) return out;
  const Value* rd = mr->get("resources");
  for (auto& k : strs(rd ? rd->get("kinds") : nullptr)) out.push_back(k);
  for (const char* b : {"all", "any"}) {
    const Value* l = mr->get(b);
    if (l && l->t == T::Arr)
      for (auto& f : l->a) {
        const Value* frd = f.get("resources");
        for (auto& k : strs(frd ? frd->get("kinds") : nullptr)) out.push_back(k);
      }
  }
  return out;
}
bool autogen_subject_ok(bool& needed, const Value* rd) {  // checkAutogenSupport autogen.go:33-43
  if (nil(rd)) return true;
  static const std::set<std::string> pc = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet",
                                           "ReplicationController", "CronJob", "Pod"};
  auto kinds = strs(rd->get("kinds"));
  if (!rd->str_or("name").empty() || !strs(rd->get("names")).empty() || !nil(rd->get("selector")) ||
      !nil(rd->get("annotations")) || (kinds.size() > 1 && contains_kind(kinds, "Pod")))
    return false;
  for (auto& k : kinds) if (pc.count(k)) needed = true;
  return true;
}
bool can_autogen(const Value* spec) {  // CanAutoGen autogen.go:70-136
  bool needed = false;
  const Value* rules = spec ? spec->get("rules") : nullptr;
  if (rules && rules->t == T::Arr)
    for (auto& r : rules->a) {
      const Value* mut = r.get("mutate");
      if ((mut && !mut->str_or("patchesJson6902").empty()) || nonempty(r.get("generate"))) return false;
      const Value* m = r.get("match");
      const Value* e = r.get("exclude");
      if (!autogen_subject_ok(needed, m ? m->get("resources") : nullptr) ||
          !autogen_subject_ok(needed, e ? e->get("resources") : nullptr))
        return false;
      for (const Value* blk : {m, e})
        for (const char* w : {"any", "all"}) {
          const Value* l = blk ? blk->get(w) : nullptr;
          if (l && l->t == T::Arr)
            for (auto& f : l->a) if (!autogen_subject_ok(needed, f.get("resources"))) return false;
        }
    }
  return needed;
}
Value kinds_value(const std::vector<std::string>& k) {
  Value a = Value::A();
  for (auto& s : k) a.a.push_back(Value::S(s));
  return a;
}
void replace_filter_kinds(Value& filters, const std::string& match, const std::vector<std::string>& kinds) {
  for (auto& f : filters.a) {
    Value* rd = f.getm("resources");
    if (rd && contains_kind(strs(rd->get("kinds")), match)) rd->set("kinds", kinds_value(kinds));
  }
}
bool nonempty_list(const Value* v) { return v && v->t == T::Arr && !v->a.empty(); }

// generateRule (rule.go:73-204); returns false when no rule is generated
bool generate_rule(const std::string& name, const Value& r0, const std::string& tplKey, const std::vector<std::string>& kinds,
                   const std::string& grfKind, Value& out) {
  out = r0;
  out.set("name", Value::S(name));
  Value* m = out.getm("match");
  if (!m) { out.set("match", Value::O()); m = out.getm("match"); }
  if (nonempty_list(m->get("any"))) replace_filter_kinds(*m->getm("any"), grfKind, kinds);
  else if (nonempty_list(m->get("all"))) replace_filter_kinds(*m->getm("all"), grfKind, kinds);
  else {
    Value* rd = m->getm("resources");
    if (!rd || rd->t != T::Obj) { m->set("resources", Value::O()); rd = m->getm("resources"); }
    rd->set("kinds", kinds_value(kinds));
  }
  Value* e = out.getm("exclude");
  if (e && e->t == T::Obj) {
    if (nonempty_list(e->get("any"))) replace_filter_kinds(*e->getm("any"), grfKind, kinds);
    else if (nonempty_list(e->get("all"))) replace_filter_kinds(*e->getm("all"), grfKind, kinds);
    else {
      Value* rd = e->getm("resources");
      if (rd && !strs(rd->get("kinds")).empty()) rd->set("kinds", kinds_value(kinds));
    }
  }
  const Value* mut = out.get("mutate");
  if (mut && (!nil(mut->get("patchStrategicMerge")) || nonempty(mut->get("foreach")))) return true;
  const Value* val = out.get("validate");
  if (!val) return false;
  std::string msg = val->str_or("message");
  auto wrap = [&](const Value& p) {
    Value inner = Value::O();
    inner.set(tplKey, p);
    Value outer = Value::O();
    outer.set("spec", inner);
    return outer;
  };
  Value nv = Value::O();
  if (!msg.empty()) nv.set("message", Value::S(msg));
  if (!nil(val->get("pattern"))) nv.set("pattern", wrap(*val->get("pattern")));
  else if (!nil(val->get("deny"))) nv.set("deny", *val->get("deny"));
  else if (!nil(val->get("podSecurity"))) {
    const Value* ps = val->get("podSecurity");
    Value np = Value::O();
    if (!ps->str_or("level").empty()) np.set("level", Value::S(ps->str_or("level")));
    if (!ps->str_or("version").empty()) np.set("version", Value::S(ps->str_or("version")));
    if (nonempty_list(ps->get("exclude"))) np.set("exclude", *ps->get("exclude"));
    nv.set("podSecurity", np);
  } else if (!nil(val->get("anyPattern"))) {
    Value arr = Value::A();
    const Value* ap = val->get("anyPattern");
    if (ap->t == T::Arr) for (auto& p : ap->a) arr.a.push_back(wrap(p));
    nv.set("anyPattern", arr);
  } else if (nonempty(val->get("foreach"))) {
    nv.set("foreach", *val->get("foreach"));
  } else if (nonempty(out.get("verifyImages"))) {
    return true;
  } else {
    return false;
  }
  out.set("validate", nv);
  return true;
}

std::string autogen_name(const std::string& prefix, const std::string& n) {
  std::string s = prefix + "-" + n;
  return s.size() > 63 ? s.substr(0, 63) : s;
}

bool gen_for_controllers(const Value& r, std::string controllers, Value& out) {  // rule.go:228-279
  std::string name = r.str_or("name");
  if (name.compare(0, 8, "autogen-") == 0 || controllers.empty()) return false;
  auto mk = match_kinds(r.get("match")), ek = match_kinds(r.get("exclude"));
  if (!contains_kind(mk, "Pod") || (!ek.empty() && !contains_kind(ek, "Pod"))) return false;
  static const std::set<std::string> ok = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet", "ReplicationController"};
  if (controllers == "all") controllers = "DaemonSet,Deployment,Job,StatefulSet,ReplicaSet,ReplicationController";
  else if (controllers != "none") {
    std::string v;
    for (auto& c : split(controllers, ','))
      if (ok.count(c)) v += (v.empty() ? "" : ",") + c;
    if (!v.empty()) controllers = v;
  }
  return generate_rule(autogen_name("autogen", name), r, "template", split(controllers, ','), "Pod", out);
}

bool gen_cronjob(const Value& r, const std::string& controllers, Value& out) {  // rule.go:281-297
  if (controllers.find("CronJob") == std::string::npos && controllers.find("all") == std::string::npos) return false;
  Value mid;
  if (!gen_for_controllers(r, controllers, mid)) return false;
  return generate_rule(autogen_name("autogen-cronjob", r.str_or("name")), mid, "jobTemplate", {"CronJob"}, "Job", out);
}

std::string replace_all(std::string s, const std::string& a, const std::string& b) {
  size_t p = 0;
  while ((p = s.find(a, p)) != std::string::npos) { s.replace(p, a.size(), b); p += b.size(); }
  return s;
}

Value convert_rule(const Value& r, bool cronjob) {  // convertRule autogen.go:238-276 (text rewrite on the JSON)
  std::string b = pj::dump(r);
  const Value* val = r.get("validate");
  if (val && !nil(val->get("podSecurity"))) {
    b = replace_all(b, "\"restrictedField\":\"spec", cronjob ? "\"restrictedField\":\"spec.jobTemplate.spec.template.spec"
                                                             : "\"restrictedField\":\"spec.template.spec");
    b = replace_all(b, "metadata", "spec.template.metadata");
  } else {
    b = replace_all(b, "request.object.spec", cronjob ? "request.object.spec.jobTemplate.spec.template.spec" : "request.object.spec.template.spec");
    b = replace_all(b, "request.object.metadata", "request.object.spec.template.metadata");
  }
  return pj::parse(b, true);
}

std::vector<Value> compute_rules(const Value& policy) {  // ComputeRules autogen.go:280-314
  const Value* spec = policy.get("spec");
  std::vector<Value> rules;
  if (spec && spec->get("rules") && spec->get("rules")->t == T::Arr) rules = spec->get("rules")->a;
  bool apply = can_autogen(spec);
  std::string actual = apply ? "DaemonSet,Deployment,Job,StatefulSet,ReplicaSet,ReplicationController,CronJob" : "none";
  const Value* meta = policy.get("metadata");
  const Value* ann = meta ? meta->get("annotations") : nullptr;
  const Value* a = ann ? ann->get("pod-policies.kyverno.io/autogen-controllers") : nullptr;
  if (a && apply) actual = a->t == T::Str ? a->s : "";
  if (actual == "none") return rules;
  std::string stripped;
  for (auto& c : split(actual, ',')) if (c != "CronJob") stripped += (stripped.empty() ? "" : ",") + c;
  std::vector<Value> gen;
  for (auto& r : rules) {
    Value g;
    if (gen_for_controllers(r, stripped, g)) gen.push_back(convert_rule(g, false));
    if (gen_cronjob(r, actual, g)) gen.push_back(convert_rule(g, true));
  }
  if (gen.empty()) return rules;
  std::vector<Value> out;
  for (auto& r : rules) if (r.str_or("name").compare(0, 8, "autogen-") != 0) out.push_back(r);
  for (auto& g : gen) out.push_back(g);
  return out;
}

// ---------------------------------------------------------------- compile state
struct Fallback { std::string why; };

struct Cx {
  Ruleset& rs;
  bool background = false;  // KYV_COMPILE_BACKGROUND: no admission request info ever reaches these rules
  RuleDesc* rd = nullptr;
  std::map<std::string, int> abits;  // raw anchor key -> bit (per pattern)
  int nslots = 0;
  uint32_t nmeta = 0;
  std::vector<MetaSite> sites;
  bool allow_element = false;  // compiling conditions of a foreach entry (`element` is bound)
  // compiling a foreach pattern: a value that is exactly one element variable becomes an L_DYN leaf; dyn: the
  // entry's element variables (kind 0 path / 1 elementIndex, path segments as sids)
  bool dyn_ok = false;
  std::vector<std::vector<uint32_t>> dyn;
  bool uses_op = false;        // some condition read request.operation
  uint32_t tmpl(const std::string& s) {
    auto it = rs.template_ids.find(s);
    if (it != rs.template_ids.end()) return it->second;
    rs.templates.push_back(s);
    const uint32_t id = (uint32_t)rs.templates.size() - 1;
    rs.template_ids.emplace(s, id);
    return id;
  }
  uint32_t sid(const std::string& s) { return rs.dict.intern(s); }
};

std::string idx_ph(int level) { return std::string("\x01") + (char)('0' + level); }
std::string key_ph(int slot) { return std::string("\x02") + (char)('0' + slot); }

// glob classification for compareString atoms
void classify_glob(Cx& c, Atom& a, const std::string& p) {
  a.pat = c.sid(p);
  a.lit = NONE;
  if (p.empty()) { a.glob = G_EMPTY; return; }
  if (!has_wild(p)) { a.glob = G_EXACT; return; }
  bool allstar = true;
  for (char ch : p) if (ch != '*') allstar = false;
  if (allstar) { a.glob = G_ANY; return; }
  if (p == "?*" || p == "*?") { a.glob = G_NONEMPTY; return; }
  auto lit_ok = [](const std::string& s) { return !s.empty() && !has_wild(s); };
  if (p.size() >= 2 && p.back() == '*' && lit_ok(p.substr(0, p.size() - 1))) { a.glob = G_PREFIX; a.lit = c.sid(p.substr(0, p.size() - 1)); return; }
  if (p.size() >= 2 && p[0] == '*' && lit_ok(p.substr(1))) { a.glob = G_SUFFIX; a.lit = c.sid(p.substr(1)); return; }
  if (p.size() >= 3 && p[0] == '*' && p.back() == '*' && lit_ok(p.substr(1, p.size() - 2))) {
    a.glob = G_CONTAINS;
    a.lit = c.sid(p.substr(1, p.size() - 2));
    return;
  }
  a.glob = G_GENERAL;
}

// range regexes (operator.go:30-31): [-|\+]?\d+(?:\.\d+)?[A-Za-z]*
bool range_side(const std::string& s, size_t& i) {
  size_t st = i;
  if (i < s.size() && (s[i] == '-' || s[i] == '|' || s[i] == '+')) i++;
  size_t d = i;
  while (i < s.size() && isdigit((unsigned char)s[i])) i++;
  if (i == d) { i = st; return false; }
  if (i + 1 < s.size() && s[i] == '.' && isdigit((unsigned char)s[i + 1])) { i++; while (i < s.size() && isdigit((unsigned char)s[i])) i++; }
  while (i < s.size() && isalpha((unsigned char)s[i])) i++;
  return true;
}
bool range_split(const std::string& s, const std::string& sep, std::string& l, std::string& r) {
  size_t i = 0;
  if (!range_side(s, i)) return false;
  size_t le = i;
  if (s.compare(i, sep.size(), sep) != 0) return false;
  i += sep.size();
  size_t rs = i;
  if (!range_side(s, i) || i != s.size()) return false;
  l = s.substr(0, le);
  r = s.substr(rs);
  return true;
}

Atom simple_atom(Cx& c, uint8_t op, const std::string& p) {
  Atom a{};
  a.op = op;
  a.sub = NONE;
  int64_t d;
  if (pj::go_parse_duration(p, &d)) { a.flags |= AF_DUR; a.dur = d; }
  int64_t lo, hi;
  int q = pj::go_parse_quantity(p, &lo, &hi);
  if (q == 2) throw Fallback{"pattern quantity beyond int128 nano range"};
  if (q == 1) { a.flags |= AF_QTY; a.qlo = lo; a.qhi = hi; }
  classify_glob(c, a, p);
  return a;
}

// validateStringPattern (pattern.go:175-197) compiled to one atom
uint32_t compile_atom(Cx& c, const std::string& atom) {
  std::string l, r;
  uint8_t op;
  size_t oplen = 0;
  if (atom.size() < 2) op = A_EQ;
  else if (atom.compare(0, 2, ">=") == 0) { op = A_GE; oplen = 2; }
  else if (atom.compare(0, 2, "<=") == 0) { op = A_LE; oplen = 2; }
  else if (atom[0] == '>') { op = A_GT; oplen = 1; }
  else if (atom[0] == '<') { op = A_LT; oplen = 1; }
  else if (atom[0] == '!') { op = A_NE; oplen = 1; }
  else if (range_split(atom, "!-", l, r)) op = A_RANGE_OUT;
  else if (range_split(atom, "-", l, r)) op = A_RANGE_IN;
  else op = A_EQ;
  if (op == A_RANGE_IN || op == A_RANGE_OUT) {
    Atom a{};
    a.op = op;
    a.sub = (uint32_t)c.rs.atoms.size() + 1;
    uint32_t id = (uint32_t)c.rs.atoms.size();
    c.rs.atoms.push_back(a);
    // ">= "+left / "<= "+right  resp. "< "+left / "> "+right, operator stripped + TrimSpace
    c.rs.atoms.push_back(simple_atom(c, op == A_RANGE_IN ? A_GE : A_LT, pj::go_trim_space(" " + l)));
    c.rs.atoms.push_back(simple_atom(c, op == A_RANGE_IN ? A_LE : A_GT, pj::go_trim_space(" " + r)));
    return id;
  }
  uint32_t id = (uint32_t)c.rs.atoms.size();
  c.rs.atoms.push_back(simple_atom(c, op, pj::go_trim_space(atom.substr(oplen))));
  return id;
}

std::string trim_sp(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && s[b] == ' ') b++;
  while (e > b && s[e - 1] == ' ') e--;
  return s.substr(b, e - b);
}

// a foreach pattern value that is exactly one element variable (vars.go:352-431 substitutes it by its typed value):
// `{{element}}`, `{{element.<ident>...}}` -> [0, nseg, sids...], `{{elementIndex}}` -> [1, 0]
bool element_var_desc(Cx& c, const std::string& s, std::vector<uint32_t>* d) {
  if (s.size() < 4 || s.compare(0, 2, "{{") != 0 || s.compare(s.size() - 2, 2, "}}") != 0) return false;
  std::string in = s.substr(2, s.size() - 4);
  if (in.find('{') != std::string::npos || in.find('}') != std::string::npos) return false;
  size_t b = 0, e = in.size();
  while (b < e && isspace((unsigned char)in[b])) b++;
  while (e > b && isspace((unsigned char)in[e - 1])) e--;
  in = in.substr(b, e - b);
  if (in == "elementIndex") { *d = {1u, 0u}; return true; }
  if (in.compare(0, 7, "element") != 0) return false;
  std::vector<uint32_t> segs;
  for (size_t i = 7; i < in.size();) {
    if (in[i] != '.') return false;
    size_t j = i + 1;
    if (j >= in.size() || !(isalpha((unsigned char)in[j]) || in[j] == '_')) return false;
    while (j < in.size() && (isalnum((unsigned char)in[j]) || in[j] == '_')) j++;
    segs.push_back(c.sid(in.substr(i + 1, j - i - 1)));
    i = j;
  }
  *d = {0u, (uint32_t)segs.size()};
  d->insert(d->end(), segs.begin(), segs.end());
  return true;
}

bool keys_have_vars(const Value& p) {
  if (p.t == T::Obj)
    for (auto& kv : p.o)
      if (kv.first.find("{{") != std::string::npos || kv.first.find("$(") != std::string::npos || keys_have_vars(kv.second))
        return true;
  if (p.t == T::Arr) for (auto& e : p.a) if (keys_have_vars(e)) return true;
  return false;
}

uint32_t compile_leaf(Cx& c, const Value& p) {  // pattern.Validate leaf types
  Leaf L{};
  L.exact = NONE;
  switch (p.t) {
    case T::Null: L.type = L_NIL; break;
    case T::Bool: L.type = L_BOOL; L.bval = p.b; break;
    case T::Int:
      L.type = L_FLOAT; L.f = (double)p.i; L.fint = 1; L.fi = p.i;
      break;
    case T::Float: {
      L.type = L_FLOAT;
      L.f = p.f;
      L.fint = p.f == std::trunc(p.f);
      if (!(p.f > -9.223372036854775808e18 && p.f < 9.223372036854775807e18)) L.fi = INT64_MIN;
      else L.fi = (int64_t)p.f;
      break;
    }
    case T::Str: {
      if (c.dyn_ok && (p.s.find("{{") != std::string::npos || p.s.find("$(") != std::string::npos)) {
        std::vector<uint32_t> d;
        if (!element_var_desc(c, p.s, &d)) throw Fallback{"foreach: pattern variables other than whole-string element values"};
        uint32_t slot = 0;
        while (slot < c.dyn.size() && c.dyn[slot] != d) slot++;
        if (slot == c.dyn.size()) c.dyn.push_back(d);
        if (c.dyn.size() > MAX_DYN) throw Fallback{"foreach: more element variables than the device resolves"};
        L.type = L_DYN;
        L.exact = slot;
        break;
      }
      if (has_magic(p.s)) throw Fallback{"pattern text contains an anchor-error phrase"};
      L.type = L_STR;
      L.exact = c.sid(p.s);
      std::vector<uint32_t> groups;
      for (auto& g0 : split(p.s, '|')) {
        std::string g = trim_sp(g0);
        std::vector<uint32_t> atoms;
        for (auto& a0 : split(g, '&')) atoms.push_back(compile_atom(c, trim_sp(a0)));
        // atoms of one group must be consecutive: re-emit as a contiguous block of references
        uint32_t first = (uint32_t)c.rs.atoms.size();
        for (uint32_t id : atoms) {
          Atom a = c.rs.atoms[id];
          c.rs.atoms.push_back(a);
        }
        groups.push_back(first);
        groups.push_back((uint32_t)atoms.size());
      }
      L.groups = (uint32_t)c.rs.pool.size();
      L.ngroups = (uint32_t)groups.size() / 2;
      for (auto g : groups) c.rs.pool.push_back(g);
      break;
    }
    case T::Obj: L.type = L_MAP; break;
    default: L.type = L_ARR; break;
  }
  c.rs.leaves.push_back(L);
  return (uint32_t)c.rs.leaves.size() - 1;
}

uint32_t new_pnode(Cx& c, uint8_t kind, const std::string& path) {
  PNode P{};
  P.kind = kind;
  P.tmpl = c.tmpl(path);
  c.rs.pnodes.push_back(P);
  return (uint32_t)c.rs.pnodes.size() - 1;
}

bool has_nested_anchors(const Value& p) {  // validate/utils.go:11-33
  if (p.t == T::Obj) {
    for (auto& kv : p.o) {
      Anc a = parse_anchor(kv.first);
      if (a.t == AT::Cond || a.t == AT::Exist || a.t == AT::Eq || a.t == AT::Neg || a.t == AT::Global) return true;
    }
    for (auto& kv : p.o) if (has_nested_anchors(kv.second)) return true;
    return false;
  }
  if (p.t == T::Arr) for (auto& e : p.a) if (has_nested_anchors(e)) return true;
  return false;
}

struct Loc {
  int level = 0;     // enclosing array-of-maps nesting (dynamic index slots used)
  bool loop = false; // inside a loop construct (array of maps / existence trial)
  int depth = 0;
};

uint32_t compile_elem(Cx& c, const Value& p, const std::string& path, Loc loc, int wild_slot_base = -1);

// which pattern key selects metadata/labels (getPatternValue, wildcards.go:85-96)
const std::pair<std::string, Value>* pattern_value(const Value& m, const std::string& tag) {
  const std::pair<std::string, Value>* hit = nullptr;
  int n = 0;
  for (auto& kv : m.o) {
    Anc a = parse_anchor(kv.first);
    if (kv.first == tag || (a.t != AT::None && a.key == tag)) { hit = &kv; n++; }
  }
  if (n > 1) throw Fallback{"pattern selects " + tag + " twice (Go map order decides)"};
  return hit;
}

uint32_t compile_map(Cx& c, const Value& p, const std::string& path, Loc loc) {
  for (auto& kv : p.o) if (has_magic(kv.first)) throw Fallback{"pattern key contains an anchor-error phrase"};
  uint32_t id = new_pnode(c, P_MAP, path);
  // ExpandInMetadata site (wildcards.go:62-83)
  int meta_site = -1;
  std::string meta_key;
  int labels_slot0 = -1, ann_slot0 = -1;
  std::string labels_pkey, ann_pkey;
  if (auto mv = pattern_value(p, "metadata")) {
    if (!mv->second.nil()) {
      if (mv->second.t != T::Obj) throw Fallback{"pattern metadata is not a map (reference panics)"};
      MetaSite ms{};
      ms.wild_l = ms.wild_a = (uint32_t)c.rs.pool.size();
      for (int tag = 0; tag < 2; tag++) {
        auto lv = pattern_value(mv->second, tag == 0 ? "labels" : "annotations");
        if (!lv || lv->second.nil()) continue;
        if (lv->second.t != T::Obj) throw Fallback{"pattern labels/annotations is not a map (reference panics)"};
        std::vector<std::pair<std::string, std::string>> wild;
        for (auto& kv : lv->second.o) {
          if (kv.second.t != T::Str) throw Fallback{"non-string metadata pattern value (reference panics)"};
          if (has_wild(kv.first)) {
            Anc a = parse_anchor(kv.first);
            wild.push_back({a.t != AT::None ? a.key : kv.first, a.t != AT::None ? a.key : kv.first});
          }
        }
        if (!wild.empty() && (loc.loop || lv->second.o.size() != 1))
          throw Fallback{"wildcard metadata keys inside a loop or beside other keys (order/collision is run-time)"};
        if (tag == 0) ms.has_labels = 1; else ms.has_ann = 1;
        uint32_t off = (uint32_t)c.rs.pool.size();
        for (auto& w : wild) { c.rs.pool.push_back(c.sid(w.first)); c.rs.pool.push_back(c.sid(w.second)); }
        int slot0 = c.nslots;
        c.nslots += (int)wild.size();
        if (c.nslots > MAX_SLOTS) throw Fallback{"too many metadata wildcard keys"};
        if (tag == 0) { ms.wild_l = off; ms.nwild_l = (uint32_t)wild.size(); ms.slot_l = slot0; labels_slot0 = wild.empty() ? -1 : slot0; labels_pkey = lv->first; }
        else { ms.wild_a = off; ms.nwild_a = (uint32_t)wild.size(); ms.slot_a = slot0; ann_slot0 = wild.empty() ? -1 : slot0; ann_pkey = lv->first; }
      }
      if (ms.has_labels || ms.has_ann) {
        meta_site = (int)c.sites.size();
        c.sites.push_back(ms);
        meta_key = mv->first;
      }
    }
  }
  // entry order: anchors sorted, then getSortedNestedAnchorResource (validate.go:118-161)
  std::vector<std::string> anchors, others;
  for (auto& kv : p.o) {
    Anc a = parse_anchor(kv.first);
    if (a.t == AT::Cond || a.t == AT::Exist || a.t == AT::Eq || a.t == AT::Neg) anchors.push_back(kv.first);
    else others.push_back(kv.first);
  }
  std::sort(anchors.begin(), anchors.end());
  std::sort(others.begin(), others.end());
  std::list<std::string> order;
  for (auto& k : others) {
    if (parse_anchor(k).t == AT::Global || has_nested_anchors(*p.get(k))) order.push_front(k);
    else order.push_back(k);
  }
  std::vector<std::string> keys = anchors;
  for (auto& k : order) keys.push_back(k);
  std::vector<PEntry> ents;
  for (auto& k : keys) {
    const Value& v = *p.get(k);
    PEntry E{};
    E.abit = 0xFF;
    E.child = NONE;
    Anc a = parse_anchor(k);
    std::string lookup = (a.t == AT::None || a.t == AT::Add) ? k : a.key;
    std::string cur = path + lookup + "/";
    if (a.t == AT::Cond || a.t == AT::Exist || a.t == AT::Neg) {
      auto it = c.abits.find(k);
      int bit;
      if (it == c.abits.end()) {
        bit = (int)c.abits.size();
        if (bit >= 64) throw Fallback{"more than 64 distinct anchor keys"};
        c.abits[k] = bit;
      } else bit = it->second;
      E.abit = (uint8_t)bit;
    }
    E.key = c.sid(lookup);
    Loc child = loc;
    child.depth++;
    switch (a.t) {
      case AT::Cond: E.handler = H_CONDITION; break;
      case AT::Global: E.handler = H_GLOBAL; break;
      case AT::Eq: E.handler = H_EQUALITY; break;
      case AT::Neg: E.handler = H_NEGATION; break;
      case AT::Exist: E.handler = H_EXISTENCE; break;
      default: E.handler = (v.t == T::Str && v.s == "*") ? H_STAR : H_DEFAULT; break;
    }
    E.tmpl = c.tmpl(cur);
    if (E.handler == H_EXISTENCE) {
      bool bad = v.t != T::Arr;
      if (!bad) for (auto& e : v.a) if (e.t != T::Obj) bad = true;
      if (bad) E.handler = H_EXIST_BADPAT;
      else {
        Loc tl = child;
        tl.loop = true;
        std::vector<uint32_t> maps;
        for (auto& e : v.a) maps.push_back(compile_elem(c, e, cur + "\x03/", tl));  // trial paths never reported
        E.child = (uint32_t)c.rs.pool.size();
        c.rs.pool.push_back((uint32_t)maps.size());
        for (auto m : maps) c.rs.pool.push_back(m);
      }
    } else if (E.handler != H_NEGATION && E.handler != H_STAR) {
      E.child = compile_elem(c, v, cur, child);
    }
    ents.push_back(E);
  }
  // metadata expansion: wildcard entries of the labels/annotations maps read their key from a slot
  if (meta_site >= 0) {
    c.rs.pnodes[id].flags |= PF_META;
    c.rs.pnodes[id].meta = (uint8_t)meta_site;
    (void)meta_key;
  }
  PNode& P = c.rs.pnodes[id];
  P.first = (uint32_t)c.rs.pentries.size();
  P.n = (uint32_t)ents.size();
  for (auto& e : ents) c.rs.pentries.push_back(e);
  (void)labels_slot0; (void)ann_slot0; (void)labels_pkey; (void)ann_pkey;
  return id;
}

uint32_t compile_elem(Cx& c, const Value& p, const std::string& path, Loc loc, int) {
  if (loc.depth > 64) throw Fallback{"pattern nesting too deep"};
  if (p.t == T::Obj) return compile_map(c, p, path, loc);
  if (p.t == T::Arr) {
    if (p.a.empty()) return new_pnode(c, P_ARR_EMPTY, path);
    const Value& f = p.a[0];
    if (f.t == T::Obj) {
      if (loc.level >= MAX_IDX) throw Fallback{"arrays of maps nested deeper than the index slots"};
      uint32_t id = new_pnode(c, P_ARR_MAPS, path);
      Loc cl = loc;
      cl.level++;
      cl.loop = true;
      cl.depth++;
      uint32_t child = compile_elem(c, f, path + idx_ph(loc.level) + "/", cl);
      c.rs.pnodes[id].first = child;
      c.rs.pnodes[id].level = (uint8_t)loc.level;
      return id;
    }
    if (f.t != T::Arr) {
      uint32_t id = new_pnode(c, P_ARR_SCALAR, path);
      uint32_t leaf = new_pnode(c, P_LEAF, path);
      c.rs.pnodes[leaf].first = compile_leaf(c, f);
      c.rs.pnodes[id].first = leaf;
      return id;
    }
    uint32_t id = new_pnode(c, P_ARR_POS, path);
    std::vector<uint32_t> kids;
    Loc cl = loc;
    cl.depth++;
    for (size_t i = 0; i < p.a.size(); i++) kids.push_back(compile_elem(c, p.a[i], path + std::to_string(i) + "/", cl));
    c.rs.pnodes[id].first = (uint32_t)c.rs.pool.size();
    c.rs.pnodes[id].n = (uint32_t)kids.size();
    for (auto k : kids) c.rs.pool.push_back(k);
    return id;
  }
  uint32_t id = new_pnode(c, P_LEAF, path);
  c.rs.pnodes[id].first = compile_leaf(c, p);
  return id;
}

// mark EF_WILD entries: labels/annotations maps below a metadata site whose keys are wildcards
void mark_wild_entries(Cx& c, uint32_t site_pnode) {
  PNode& P = c.rs.pnodes[site_pnode];
  const MetaSite& ms = c.sites[P.meta];
  for (uint32_t e = 0; e < P.n; e++) {
    PEntry& E = c.rs.pentries[P.first + e];
    const std::string& key = c.rs.dict.strs[E.key];
    if (key != "metadata" || E.child == NONE || c.rs.pnodes[E.child].kind != P_MAP) continue;
    PNode& M = c.rs.pnodes[E.child];
    for (uint32_t f = 0; f < M.n; f++) {
      PEntry& L = c.rs.pentries[M.first + f];
      const std::string& lk = c.rs.dict.strs[L.key];
      int tag = lk == "labels" ? 0 : lk == "annotations" ? 1 : -1;
      if (tag < 0 || L.child == NONE || c.rs.pnodes[L.child].kind != P_MAP) continue;
      PNode& W = c.rs.pnodes[L.child];
      uint32_t wl = tag == 0 ? ms.wild_l : ms.wild_a, nw = tag == 0 ? ms.nwild_l : ms.nwild_a;
      uint32_t slot0 = tag == 0 ? ms.slot_l : ms.slot_a;
      for (uint32_t g = 0; g < W.n; g++) {
        PEntry& X = c.rs.pentries[W.first + g];
        for (uint32_t w = 0; w < nw; w++) {
          if (c.rs.pool[wl + 2 * w + 1] == X.key) {
            X.flags |= EF_WILD;
            X.slot = (uint8_t)(slot0 + w);
            // currentPath uses the expanded key
            std::string t = c.rs.templates[X.tmpl];
            std::string unresolved = c.rs.dict.strs[X.key];
            t = t.substr(0, t.size() - unresolved.size() - 1) + key_ph(slot0 + w) + "/";
            X.tmpl = c.tmpl(t);
            if (X.child != NONE) c.rs.pnodes[X.child].tmpl = X.tmpl;  // metadata values are leaves (strings)
          }
        }
      }
    }
  }
}

uint32_t compile_pattern_root(Cx& c, const Value& p) {
  c.abits.clear();
  uint32_t root = compile_elem(c, p, "/", Loc());
  for (uint32_t i = 0; i < c.rs.pnodes.size(); i++)
    if (i >= root && (c.rs.pnodes[i].flags & PF_META)) mark_wild_entries(c, i);
  return root;
}

// ---------------------------------------------------------------- match programs
bool valid_qname(const std::string& n) {
  if (n.empty() || n.size() > 63) return false;
  auto an = [](char ch) { return isalnum((unsigned char)ch) != 0; };
  if (!an(n.front()) || !an(n.back())) return false;
  for (char ch : n) if (!(an(ch) || ch == '-' || ch == '_' || ch == '.')) return false;
  return true;
}
bool valid_dns_sub(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  for (auto& l : split(s, '.')) {
    if (l.empty()) return false;
    auto ok = [](char ch) { return (ch >= 'a' && ch <= 'z') || (ch >= '0' && ch <= '9'); };
    if (!ok(l.front()) || !ok(l.back())) return false;
    for (char ch : l) if (!(ok(ch) || ch == '-')) return false;
  }
  return true;
}
bool valid_label_key(const std::string& k) {
  auto p = split(k, '/');
  if (p.size() == 1) return valid_qname(p[0]);
  if (p.size() == 2) return !p[0].empty() && valid_dns_sub(p[0]) && valid_qname(p[1]);
  return false;
}
bool valid_label_value(const std::string& v) { return v.empty() || valid_qname(v); }

uint32_t compile_selector(Cx& c, const Value* sel) {
  SelDesc sd{};
  sd.reqs = (uint32_t)c.rs.reqs.size();
  const Value* ml = sel->get("matchLabels");
  size_t nml = ml && ml->t == T::Obj ? ml->o.size() : 0;
  bool anywild = false;
  if (nml) {
    for (auto& kv : ml->o) {
      std::string k = kv.first, v = kv.second.t == T::Str ? kv.second.s : "";
      SelReq r{};
      if (has_wild(k) || has_wild(v)) {
        anywild = true;
        r.op = RQ_WILD;
        r.key = c.sid(k);
        r.vals = c.sid(v);
        std::string k0 = k, v0 = v;
        for (auto& ch : k0) if (ch == '*' || ch == '?') ch = '0';
        for (auto& ch : v0) if (ch == '*' || ch == '?') ch = '0';
        if (valid_label_key(k0) && valid_label_value(v0)) { r.rkey = c.sid(k0); r.rval = c.sid(v0); }
        else { r.rkey = NONE; r.rval = NONE; }
      } else {
        r.op = RQ_EQ;
        r.key = c.sid(k);
        r.vals = (uint32_t)c.rs.pool.size();
        r.nvals = 1;
        c.rs.pool.push_back(c.sid(v));
        if (!valid_label_key(k) || !valid_label_value(v)) sd.invalid = 1;
      }
      c.rs.reqs.push_back(r);
    }
    if (anywild && nml > 1) throw Fallback{"wildcard matchLabels beside other entries (collision decided by Go map order)"};
  }
  const Value* me = sel->get("matchExpressions");
  if (me && me->t == T::Arr)
    for (auto& e : me->a) {
      SelReq r{};
      std::string op = e.str_or("operator");
      if (op == "In") r.op = RQ_IN;
      else if (op == "NotIn") r.op = RQ_NOTIN;
      else if (op == "Exists") r.op = RQ_EXISTS;
      else if (op == "DoesNotExist") r.op = RQ_NOTEXISTS;
      else { sd.invalid = 1; continue; }
      std::string key = e.str_or("key");
      r.key = c.sid(key);
      auto vals = strs(e.get("values"));
      r.vals = (uint32_t)c.rs.pool.size();
      r.nvals = (uint32_t)vals.size();
      for (auto& v : vals) { c.rs.pool.push_back(c.sid(v)); if (!valid_label_value(v)) sd.invalid = 1; }
      if (!valid_label_key(key)) sd.invalid = 1;
      if ((r.op == RQ_IN || r.op == RQ_NOTIN) && vals.empty()) sd.invalid = 1;
      if ((r.op == RQ_EXISTS || r.op == RQ_NOTEXISTS) && !vals.empty()) sd.invalid = 1;
      c.rs.reqs.push_back(r);
    }
  sd.nreqs = (uint32_t)c.rs.reqs.size() - sd.reqs;
  c.rs.sels.push_back(sd);
  return (uint32_t)c.rs.sels.size() - 1;
}

bool rd_zero(const Value* rd) {
  if (nil(rd)) return true;
  for (const char* k : {"kinds", "names", "namespaces", "annotations", "selector", "namespaceSelector"})
    if (!nil(rd->get(k))) return false;
  return rd->str_or("name").empty();
}

uint32_t compile_filter(Cx& c, const Value* f, const Value* rd, bool* empty_may) {
  Filter F{};
  F.name = NONE;
  if (rd_zero(rd)) F.flags |= FF_ZERO_RD;
  if (f && (!nil(f->get("roles")) || !nil(f->get("clusterRoles")) || !nil(f->get("subjects")))) {
    bool any = !strs(f->get("roles")).empty() || !strs(f->get("clusterRoles")).empty() || nonempty_list(f->get("subjects"));
    if (any) F.flags |= FF_USERINFO;
    const Value* subj = f->get("subjects");
    if (subj && subj->t == T::Arr)
      for (auto& s : subj->a) if (s.str_or("name").empty()) throw Fallback{"subject with empty name (mock/user matching)"};
  }
  auto kinds = strs(rd ? rd->get("kinds") : nullptr);
  F.kinds = (uint32_t)c.rs.kinds.size();
  F.nkinds = (uint16_t)kinds.size();
  bool star = false, emptykind = kinds.empty();
  for (auto& k : kinds) {
    KindDesc K{};
    if (k == "*") { K.kind = NONE; star = true; }
    else {
      std::string gv, kind;
      kind_from_gvk(k, gv, kind);
      K.kind = c.sid(kind);
      if (kind.empty()) emptykind = true;
      if (gv.empty()) K.gv_mode = 0;
      else if (gv.find('*') != std::string::npos) {
        K.gv_mode = 2;
        std::string pre = gv;
        if (!pre.empty() && pre.back() == '*') pre.pop_back();
        K.g = c.sid(pre);
      } else {
        size_t sl = std::count(gv.begin(), gv.end(), '/');
        if (gv == "/") { K.gv_mode = 1; K.g = SID_EMPTY; K.v = SID_EMPTY; }
        else if (sl == 0) { K.gv_mode = 1; K.g = SID_EMPTY; K.v = c.sid(gv); }
        else if (sl == 1) { K.gv_mode = 1; K.g = c.sid(gv.substr(0, gv.find('/'))); K.v = c.sid(gv.substr(gv.find('/') + 1)); }
        else K.gv_mode = 3;
      }
    }
    c.rs.kinds.push_back(K);
  }
  if (star) F.flags |= FF_KINDS_STAR;
  if (star || emptykind) *empty_may = true;
  std::string name = rd ? rd->str_or("name") : "";
  if (!name.empty()) F.name = c.sid(name);
  auto names = strs(rd ? rd->get("names") : nullptr);
  F.names = (uint32_t)c.rs.pool.size();
  F.nnames = (uint32_t)names.size();
  for (auto& n : names) c.rs.pool.push_back(c.sid(n));
  auto nss = strs(rd ? rd->get("namespaces") : nullptr);
  F.nss = (uint32_t)c.rs.pool.size();
  F.nnss = (uint32_t)nss.size();
  for (auto& n : nss) c.rs.pool.push_back(c.sid(n));
  const Value* ann = rd ? rd->get("annotations") : nullptr;
  F.ann = (uint32_t)c.rs.pool.size();
  if (ann && ann->t == T::Obj) {
    F.nann = (uint32_t)ann->o.size();
    for (auto& kv : ann->o) { c.rs.pool.push_back(c.sid(kv.first)); c.rs.pool.push_back(c.sid(kv.second.t == T::Str ? kv.second.s : "")); }
  }
  const Value* sel = rd ? rd->get("selector") : nullptr;
  const Value* nsel = rd ? rd->get("namespaceSelector") : nullptr;
  // selector and namespaceSelector occupy two consecutive SelDesc slots
  F.sel = (uint32_t)c.rs.sels.size();
  {
    Value emptysel = Value::O();
    uint32_t a = compile_selector(c, nil(sel) ? &emptysel : sel);
    uint32_t b = compile_selector(c, nil(nsel) ? &emptysel : nsel);
    (void)a; (void)b;
  }
  if (!nil(sel)) F.flags |= FF_HAS_SEL;
  if (!nil(nsel)) F.flags |= FF_HAS_NSSEL;
  c.rs.filters.push_back(F);
  return (uint32_t)c.rs.filters.size() - 1;
}

MatchBlock compile_block(Cx& c, const Value* mr, bool is_match, bool* empty_may) {
  MatchBlock B{};
  if (nil(mr)) { B.mode = is_match ? MM_PLAIN : MM_NONE; if (is_match) { B.filters = (uint32_t)c.rs.filters.size(); compile_filter(c, nullptr, nullptr, empty_may); B.nfilters = 1; } return B; }
  const Value* any = mr->get("any");
  const Value* all = mr->get("all");
  std::vector<std::pair<const Value*, const Value*>> fl;
  if (nonempty_list(any)) { B.mode = MM_ANY; for (auto& f : any->a) fl.push_back({&f, f.get("resources")}); }
  else if (nonempty_list(all)) { B.mode = MM_ALL; for (auto& f : all->a) fl.push_back({&f, f.get("resources")}); }
  else { B.mode = MM_PLAIN; fl.push_back({mr, mr->get("resources")}); }
  // compile filters contiguously
  std::vector<uint32_t> ids;
  bool em = false;
  for (auto& p : fl) ids.push_back(compile_filter(c, p.first, p.second, &em));
  if (is_match && em) *empty_may = true;
  // filters were appended in order; selectors appended inside keep filter indices contiguous
  B.filters = ids.empty() ? (uint32_t)c.rs.filters.size() : ids[0];
  B.nfilters = (uint32_t)ids.size();
  return B;
}

// A PolicyException's spec.match (kyvernov2beta1.MatchResources: any / all only) as (mode, filters, nfilters) for
// match_exception (kyv_eval.h; CheckMatchesResources, pkg/utils/match/match.go:26-76)
void compile_exc_block(Cx& c, const Value* mr, std::vector<uint32_t>& out) {
  const Value* any = mr ? mr->get("any") : nullptr;
  const Value* all = mr ? mr->get("all") : nullptr;
  uint32_t mode = MM_EXC_ALL;
  const Value* lst = nullptr;
  if (nonempty_list(any)) { mode = MM_ANY; lst = any; }
  else if (nonempty_list(all)) { mode = MM_ALL; lst = all; }
  const uint32_t f0 = (uint32_t)c.rs.filters.size();
  bool em = false;
  if (lst)
    for (auto& f : lst->a) {
      // checkUserInfo (pkg/utils/match/match.go:110-150) compares roles / clusterRoles / subjects with the request's
      // AdmissionInfo: empty in a background scan (never satisfied, compiled as FF_USERINFO), unknown to the device
      // for an admission caller -> the rule goes to the CPU engine unless the ruleset is background-only
      if (!c.background)
        for (const char* k : {"roles", "clusterRoles", "subjects"})
          if (nonempty_list(f.get(k))) throw Fallback{"exception: userInfo (roles / clusterRoles / subjects need the admission request)"};
      const uint32_t id = compile_filter(c, &f, f.get("resources"), &em);
      c.rs.filters[id].flags &= (uint16_t)~FF_KINDS_STAR;  // namespaceSelector: kind != "" only (match.go:186)
    }
  out.push_back(mode);
  out.push_back(f0);
  out.push_back(lst ? (uint32_t)lst->a.size() : 0u);
}

// ---------------------------------------------------------------- PodSecurity
uint32_t control_slots(const std::string& control) {  // pkg/pss/utils/mapping.go:45-111 -> check-version slots
  auto S = [](std::initializer_list<int> l) { uint32_t m = 0; for (int s : l) m |= 1u << s; return m; };
  // slot order as kyv_pss.h PssSlot
  if (control == "Capabilities") return S({3, 4, 5});
  if (control == "Seccomp") return S({15, 16, 17, 18});
  if (control == "Privileged Containers") return S({9});
  if (control == "Host Ports") return S({8});
  if (control == "/proc Mount Type") return S({10});
  if (control == "AppArmor") return S({2});
  if (control == "SELinux") return S({14});
  if (control == "Host Namespaces") return S({6});
  if (control == "HostPath Volumes") return S({7});
  if (control == "Sysctls") return S({19});
  if (control == "HostProcess") return S({20});
  if (control == "Privilege Escalation") return S({0, 1});
  if (control == "Running as Non-root") return S({12});
  if (control == "Running as Non-root user") return S({13});
  if (control == "Volume Types") return S({11});
  return 0;
}

bool pss_version_ok(const std::string& v) {  // api.ParseVersion / "latest"
  if (v.empty() || v == "latest") return true;
  if (v.size() < 4 || v.compare(0, 3, "v1.") != 0) return false;
  std::string m = v.substr(3);
  if (m.size() > 1 && m[0] == '0') return false;
  for (char ch : m) if (!isdigit((unsigned char)ch)) return false;
  return !m.empty() && m.size() < 10;
}

uint32_t compile_pss(Cx& c, const Value& ps) {
  PssDesc d{};
  if (ps.str_or("level") == "baseline") d.flags |= PSS_BASELINE;
  if (!pss_version_ok(ps.str_or("version"))) d.flags |= PSS_BAD_VERSION;
  const Value* ex = ps.get("exclude");
  std::vector<uint32_t> recs;
  if (ex && ex->t == T::Arr)
    for (auto& e : ex->a) {
      uint32_t off = (uint32_t)c.rs.pool.size();
      auto imgs = strs(e.get("images"));
      c.rs.pool.push_back(control_slots(e.str_or("controlName")));
      c.rs.pool.push_back((uint32_t)imgs.size());
      for (auto& i : imgs) c.rs.pool.push_back(c.sid(i));
      recs.push_back(off);
    }
  d.excl = (uint32_t)c.rs.pool.size();
  d.nexcl = (uint32_t)recs.size();
  d.cols = NONE;  // path-column table: build_path_trie (TrieBuilder::pss)
  for (auto r : recs) c.rs.pool.push_back(r);
  c.rs.pss.push_back(d);
  return (uint32_t)c.rs.pss.size() - 1;
}

// ---------------------------------------------------------------- conditions (deny / preconditions)
// `{{ request.object(.seg)* }}` with segments that are JMESPath identifiers or quoted identifiers (no escapes):
// the reference subset the device evaluates (vars.go:352-431 with DefaultVariableResolver)
bool object_var(const std::string& s, std::vector<std::string>& segs, std::string* text) {
  if (s.size() < 4 || s.compare(0, 2, "{{") != 0 || s.compare(s.size() - 2, 2, "}}") != 0) return false;
  std::string inner = s.substr(2, s.size() - 4);
  if (inner.find('{') != std::string::npos || inner.find('}') != std::string::npos) return false;
  inner = pj::go_trim_space(inner);
  const std::string pre = "request.object";
  if (inner.compare(0, pre.size(), pre) != 0) return false;
  auto ident = [](char ch, bool first) { return isalpha((unsigned char)ch) || ch == '_' || (!first && isdigit((unsigned char)ch)); };
  size_t i = pre.size();
  if (i < inner.size() && ident(inner[i], false)) return false;
  segs.clear();
  while (i < inner.size()) {
    if (inner[i] != '.' || ++i >= inner.size()) return false;
    if (inner[i] == '"') {
      size_t j = i + 1;
      while (j < inner.size() && inner[j] != '"') { if (inner[j] == '\\') return false; j++; }
      if (j >= inner.size() || j == i + 1) return false;
      segs.push_back(inner.substr(i + 1, j - i - 1));
      i = j + 1;
    } else if (ident(inner[i], true)) {
      size_t j = i;
      while (j < inner.size() && ident(inner[j], false)) j++;
      segs.push_back(inner.substr(i, j - i));
      i = j;
    } else {
      return false;
    }
  }
  if (text) *text = inner;
  return true;
}
bool var_syntax(const std::string& s) { return s.find("{{") != std::string::npos || s.find("$(") != std::string::npos; }

uint32_t emit_cnode(Cx& c, const Value& v);

// ---- JMESPath subset (OK_JMES programs, kyv_layout.h): go-jmespath's Pratt grammar for fields, quoted fields,
// sub-expressions, multi-select lists, flatten projections, keys(@), `||`, raw-string / JSON literals and filter
// projections whose predicate the device evaluates (kyv_layout.h FilterKind), then linearised into root + ops.
// Anything else (other predicates, indexes, other functions, pipes, ...) -> CPU fallback.
struct JNode {
  enum K { Field, Sub, Proj, Flat, Multi, Func, Cur, Ident, Or, Lit, Filter, Cmp, And, Not } k;
  std::string name;
  Value lit;
  std::vector<std::shared_ptr<JNode>> kids;
};
using JP = std::shared_ptr<JNode>;
struct JParser {
  enum Tok { End, Id, Quoted, Dot, LBr, RBr, Flatten, Comma, LPar, RPar, At, OrT, Raw, Json, FilterT, AndT, NotT, Cmp };
  std::vector<std::pair<Tok, std::string>> toks;
  size_t at = 0;
  explicit JParser(const std::string& s) {
    size_t i = 0;
    auto is0 = [](char c) { return isalpha((unsigned char)c) || c == '_'; };
    while (i < s.size()) {
      char c = s[i];
      if (c == ' ' || c == '\t' || c == '\n' || c == '\r') { i++; continue; }
      if (is0(c)) {
        size_t j = i;
        while (j < s.size() && (is0(s[j]) || isdigit((unsigned char)s[j]))) j++;
        toks.push_back({Id, s.substr(i, j - i)});
        i = j;
        continue;
      }
      if (c == '\'') {  // raw string (lexer.go consumeRawStringLiteral): \' is a quote, other backslashes stay
        std::string v;
        size_t j = i + 1;
        for (; j < s.size() && s[j] != '\''; j++) {
          if (s[j] == '\\' && j + 1 < s.size() && s[j + 1] == '\'') { v += '\''; j++; continue; }
          v += s[j];
        }
        if (j >= s.size()) throw Fallback{"JMESPath: unterminated literal"};
        toks.push_back({Raw, v});
        i = j + 1;
        continue;
      }
      if (c == '"' || c == '`') {
        size_t j = i + 1;
        while (j < s.size() && s[j] != c) { if (s[j] == '\\') throw Fallback{"JMESPath: escapes"}; j++; }
        if (j >= s.size()) throw Fallback{"JMESPath: unterminated literal"};
        toks.push_back({c == '"' ? Quoted : Json, s.substr(i + 1, j - i - 1)});
        i = j + 1;
        continue;
      }
      if (c == '[' && i + 1 < s.size() && s[i + 1] == ']') { toks.push_back({Flatten, "[]"}); i += 2; continue; }
      if (c == '|' && i + 1 < s.size() && s[i + 1] == '|') { toks.push_back({OrT, "||"}); i += 2; continue; }
      // go-jmespath lexer.go: "[?", "&&", comparators, "!"
      if (c == '[' && i + 1 < s.size() && s[i + 1] == '?') { toks.push_back({FilterT, "[?"}); i += 2; continue; }
      if (c == '&' && i + 1 < s.size() && s[i + 1] == '&') { toks.push_back({AndT, "&&"}); i += 2; continue; }
      if ((c == '=' || c == '!' || c == '<' || c == '>') && i + 1 < s.size() && s[i + 1] == '=') {
        toks.push_back({Cmp, s.substr(i, 2)}); i += 2; continue;
      }
      if (c == '<' || c == '>') { toks.push_back({Cmp, std::string(1, c)}); i++; continue; }
      if (c == '!') { toks.push_back({NotT, "!"}); i++; continue; }
      Tok t;
      switch (c) {
        case '.': t = Dot; break;
        case '[': t = LBr; break;
        case ']': t = RBr; break;
        case ',': t = Comma; break;
        case '(': t = LPar; break;
        case ')': t = RPar; break;
        case '@': t = At; break;
        default: throw Fallback{"JMESPath: expression outside the device subset"};
      }
      toks.push_back({t, std::string(1, c)});
      i++;
    }
    toks.push_back({End, ""});
  }
  static int bp(Tok t) {  // parser.go bindingPowers
    return t == OrT ? 2 : t == AndT ? 3 : t == Cmp ? 5 : t == Flatten ? 9 : t == FilterT ? 21 : t == Dot ? 40 :
           t == NotT ? 45 : t == LBr ? 55 : t == LPar ? 60 : 0;
  }
  Tok look() const { return toks[at].first; }
  void eat(Tok t) { if (look() != t) throw Fallback{"JMESPath: syntax"}; at++; }
  static JP mk(JNode::K k, std::vector<JP> kids = {}, const std::string& n = "") {
    auto x = std::make_shared<JNode>();
    x->k = k; x->kids = std::move(kids); x->name = n;
    return x;
  }
  JP expr(int b) {
    auto t = toks[at++];
    JP left = nud(t);
    while (b < bp(look())) left = led(toks[at++], left);
    return left;
  }
  JP nud(const std::pair<Tok, std::string>& t) {
    switch (t.first) {
      case Id: return mk(JNode::Field, {}, t.second);
      case Quoted: if (look() == LPar) throw Fallback{"JMESPath: syntax"}; return mk(JNode::Field, {}, t.second);
      case At: return mk(JNode::Cur);
      case Raw: { JP x = mk(JNode::Lit); x->lit = Value::S(t.second); return x; }
      case Json: { JP x = mk(JNode::Lit); x->lit = pj::parse(t.second, true); return x; }
      case Flatten: return mk(JNode::Proj, {mk(JNode::Flat, {mk(JNode::Ident)}), proj_rhs(bp(Flatten))});
      case LBr: return multi();
      case FilterT: return filter(mk(JNode::Ident));
      case NotT: return mk(JNode::Not, {expr(bp(NotT))});
      case LPar: { JP x = expr(0); eat(RPar); return x; }
      default: throw Fallback{"JMESPath: expression outside the device subset"};
    }
  }
  JP filter(JP left) {  // parseFilter: [left, rhs, condition]
    JP cond = expr(0);
    eat(RBr);
    JP rhs = look() == Flatten ? mk(JNode::Ident) : proj_rhs(bp(FilterT));
    return mk(JNode::Filter, {left, rhs, cond});
  }
  JP led(const std::pair<Tok, std::string>& t, JP left) {
    switch (t.first) {
      case Dot: return mk(JNode::Sub, {left, dot_rhs(bp(Dot))});
      case Flatten: return mk(JNode::Proj, {mk(JNode::Flat, {left}), proj_rhs(bp(Flatten))});
      case OrT: return mk(JNode::Or, {left, expr(bp(OrT))});
      case AndT: return mk(JNode::And, {left, expr(bp(AndT))});
      case Cmp: return mk(JNode::Cmp, {left, expr(bp(Cmp))}, t.second);
      case FilterT: return filter(left);
      case LPar: {
        if (left->k != JNode::Field) throw Fallback{"JMESPath: syntax"};
        std::vector<JP> args;
        while (look() != RPar) { args.push_back(expr(0)); if (look() == Comma) eat(Comma); }
        eat(RPar);
        return mk(JNode::Func, args, left->name);
      }
      default: throw Fallback{"JMESPath: expression outside the device subset"};
    }
  }
  JP dot_rhs(int b) {
    if (look() == Id || look() == Quoted) return expr(b);
    if (look() == LBr) { eat(LBr); return multi(); }
    throw Fallback{"JMESPath: expression outside the device subset"};
  }
  JP proj_rhs(int b) {
    if (bp(look()) < 10) return mk(JNode::Ident);
    if (look() == LBr) return expr(b);
    if (look() == Dot) { eat(Dot); return dot_rhs(b); }
    throw Fallback{"JMESPath: syntax"};
  }
  JP multi() {
    std::vector<JP> items;
    for (;;) { items.push_back(expr(0)); if (look() == RBr) break; eat(Comma); }
    eat(RBr);
    return mk(JNode::Multi, items);
  }
};

// linearise: ops of the expression evaluated on the current value; `list` tracks projection (List) mode
void jlin(Cx& c, const JP& n, std::vector<uint32_t>& out, bool& list) {
  switch (n->k) {
    case JNode::Field: out.push_back(JO_FIELD); out.push_back(c.sid(n->name)); return;
    case JNode::Sub:
      jlin(c, n->kids[0], out, list);
      jlin(c, n->kids[1], out, list);
      return;
    case JNode::Multi:
      if (list) throw Fallback{"JMESPath: multi-select inside a projection"};
      out.push_back(JO_MULTI);
      out.push_back((uint32_t)n->kids.size());
      for (auto& k : n->kids) {
        if (k->k != JNode::Field) throw Fallback{"JMESPath: multi-select of non-fields"};
        out.push_back(c.sid(k->name));
      }
      return;
    case JNode::Proj: {
      const JP& f = n->kids[0];
      if (f->k != JNode::Flat || f->kids[0]->k == JNode::Ident) throw Fallback{"JMESPath: projection form"};
      jlin(c, f->kids[0], out, list);
      out.push_back(JO_FLAT);
      list = true;
      const JP& r = n->kids[1];
      if (r->k == JNode::Ident) return;
      if (r->k == JNode::Func) {  // [].keys(@) must be flattened by the next [] (fused below)
        if (r->name != "keys" || r->kids.size() != 1 || r->kids[0]->k != JNode::Cur) throw Fallback{"JMESPath: function"};
        out.push_back(JO_KEYS);
        return;
      }
      jlin(c, r, out, list);
      return;
    }
    case JNode::Func:
      if (n->name != "keys" || n->kids.size() != 1 || n->kids[0]->k != JNode::Cur) throw Fallback{"JMESPath: function"};
      if (list) throw Fallback{"JMESPath: keys() inside a projection"};
      out.push_back(JO_KEYS);
      list = true;
      return;
    default: throw Fallback{"JMESPath: expression outside the device subset"};
  }
}

// the predicate of a filter projection -> JO_FILTER op (kyv_layout.h FilterKind); other predicates -> Fallback
void jfilter(Cx& c, const JP& cond, std::vector<uint32_t>& out) {
  if (cond->k == JNode::Func && cond->name == "contains" && cond->kids.size() == 2) {
    const JP& a = cond->kids[0];
    const JP& b = cond->kids[1];
    if (a->k == JNode::Func && a->name == "keys" && a->kids.size() == 1 && a->kids[0]->k == JNode::Cur &&
        b->k == JNode::Lit && b->lit.is(pj::T::Str)) {
      out.insert(out.end(), {JO_FILTER, FK_HASKEY, c.sid(b->lit.s), 0u});
      return;
    }
    throw Fallback{"JMESPath: filter predicate"};
  }
  if (cond->k == JNode::Cmp && (cond->name == "==" || cond->name == "!=")) {
    JP f = cond->kids[0], l = cond->kids[1];
    if (f->k == JNode::Lit) std::swap(f, l);  // DeepEqual is symmetric
    if (l->k != JNode::Lit || !(l->lit.is(pj::T::Str) || l->lit.is(pj::T::Bool) || l->lit.is(pj::T::Null)))
      throw Fallback{"JMESPath: filter comparison"};
    std::vector<uint32_t> keys;
    std::function<void(const JP&)> chain = [&](const JP& x) {
      if (x->k == JNode::Field) { keys.push_back(c.sid(x->name)); return; }
      if (x->k == JNode::Sub) { chain(x->kids[0]); chain(x->kids[1]); return; }
      if (x->k == JNode::Cur) return;
      throw Fallback{"JMESPath: filter comparison"};
    };
    chain(f);
    out.insert(out.end(), {JO_FILTER, cond->name == "==" ? FK_EQ : FK_NE, emit_cnode(c, l->lit), (uint32_t)keys.size()});
    out.insert(out.end(), keys.begin(), keys.end());
    return;
  }
  throw Fallback{"JMESPath: filter predicate"};
}

// the ops of a chain program before its function: fields, then an optional `|| literal` (kyv_layout.h jmes_chain_form)
static bool jmes_chain_form_ops(const std::vector<uint32_t>& ops) {
  size_t i = 0;
  while (i + 1 < ops.size() && ops[i] == JO_FIELD) i += 2;
  if (i + 1 < ops.size() && ops[i] == JO_OR) i += 2;
  return i == ops.size();
}

// `{{ <expr> }}` -> OK_JMES operand (false: not a single-variable string; throws Fallback outside the subset);
// *uses_op when the expression reads request.operation
bool jmes_var(Cx& c, const std::string& s, bool allow_element, CondOperand* o, std::string* text, bool* uses_op) {
  if (s.size() < 4 || s.compare(0, 2, "{{") != 0 || s.compare(s.size() - 2, 2, "}}") != 0) return false;
  std::string inner = s.substr(2, s.size() - 4);
  if (inner.find('{') != std::string::npos || inner.find('}') != std::string::npos) return false;
  inner = pj::go_trim_space(inner);
  if (text) *text = inner;
  JParser p(inner);
  JP n = p.expr(0);
  if (p.look() != JParser::End) throw Fallback{"JMESPath: syntax"};
  Value orlit;
  bool has_or = false;
  if (n->k == JNode::Or) {
    if (n->kids[1]->k != JNode::Lit) throw Fallback{"JMESPath: || with a non-literal"};
    orlit = n->kids[1]->lit;
    has_or = true;
    n = n->kids[0];
  }
  // length(<path>) (go-jmespath jpfLength): the argument's ops, then JO_LENGTH
  bool has_len = false;
  if (n->k == JNode::Func && n->name == "length") {
    if (has_or) throw Fallback{"JMESPath: length() with ||"};
    if (n->kids.size() != 1) throw Fallback{"JMESPath: function"};
    n = n->kids[0];
    has_len = true;
  }
  // to_upper(<arg>) / regex_match('<pattern>', <arg>) (kyverno pkg/engine/jmespath/functions.go:681-689, 786-799),
  // <arg> a field chain of request.object with an optional `|| <literal>`: the chain's ops, the default, then JO_UPPER /
  // JO_REGEX q, evaluated on the dictionary (Batch::str_upper / str_rx, regex.cpp; kyv_cond.h jmes_chain_cv). A pattern
  // outside the device regex subset leaves the rule on the CPU engine.
  uint32_t post = NONE, post_q = 0;
  if (n->k == JNode::Func && (n->name == "to_upper" || n->name == "regex_match")) {
    if (has_or) throw Fallback{"JMESPath: function result with ||"};
    JP arg;
    if (n->name == "to_upper") {
      if (n->kids.size() != 1) throw Fallback{"JMESPath: function"};
      arg = n->kids[0];
      post = JO_UPPER;
    } else {
      if (n->kids.size() != 2 || n->kids[0]->k != JNode::Lit || !n->kids[0]->lit.is(pj::T::Str))
        throw Fallback{"JMESPath: regex_match pattern"};
      const std::string& re = n->kids[0]->lit.s;
      auto it = std::find(c.rs.rx_src.begin(), c.rs.rx_src.end(), re);
      if (it == c.rs.rx_src.end()) {
        RxDfa d;
        std::string why;
        if (!rx_compile(re, &d, &why)) throw Fallback{"JMESPath: regex_match pattern outside the device subset (" + why + ")"};
        if (c.rs.rx_src.size() >= RX_MAX) throw Fallback{"JMESPath: too many regex_match patterns"};
        c.rs.rx_src.push_back(re);
        c.rs.rxs.push_back(std::move(d));
        post_q = (uint32_t)c.rs.rx_src.size() - 1;
      } else {
        post_q = (uint32_t)(it - c.rs.rx_src.begin());
      }
      arg = n->kids[1];
      post = JO_REGEX;
    }
    if (arg->k == JNode::Or) {
      if (arg->kids[1]->k != JNode::Lit) throw Fallback{"JMESPath: || with a non-literal"};
      orlit = arg->kids[1]->lit;
      has_or = true;
      arg = arg->kids[0];
    }
    n = arg;
  }
  // split the root off the left spine: request.object / request.operation / element
  std::vector<JNode*> spine;
  for (JNode* x = n.get();;) {
    spine.push_back(x);
    if (x->k == JNode::Field) break;
    if (x->k != JNode::Sub && x->k != JNode::Proj && x->k != JNode::Flat && x->k != JNode::Filter)
      throw Fallback{"JMESPath: root"};
    x = x->kids[0].get();
  }
  std::vector<uint32_t> ops;
  bool list = false;
  uint32_t root;
  JP body;
  const std::string r0 = spine.back()->name;
  if (r0 == "element") {
    if (!allow_element) throw Fallback{"JMESPath: element outside foreach"};
    root = JR_ELEMENT;
    if (spine.size() == 1) body = nullptr;
    else { JNode* top = spine[spine.size() - 2]; if (top->k != JNode::Sub) throw Fallback{"JMESPath: root"};
           top->kids[0] = JParser::mk(JNode::Cur); body = n; }
  } else if (r0 == "request") {
    if (spine.size() < 2 || spine[spine.size() - 2]->k != JNode::Sub || spine[spine.size() - 2]->kids[1]->k != JNode::Field)
      throw Fallback{"JMESPath: root"};
    JNode* top = spine[spine.size() - 2];
    const std::string r1 = top->kids[1]->name;
    if (r1 == "operation") {
      if (spine.size() != 2 || has_len) throw Fallback{"JMESPath: request.operation path"};
      root = JR_OPERATION;
      body = nullptr;
      if (uses_op) *uses_op = true;
    } else if (r1 == "object") {
      root = JR_OBJECT;
      if (spine.size() == 2) body = nullptr;
      else { JNode* nx = spine[spine.size() - 3]; nx->kids[0] = JParser::mk(JNode::Cur); body = n; }
    } else {
      throw Fallback{"conditions: variables beyond request.object paths"};
    }
  } else {
    throw Fallback{"conditions: variables beyond request.object paths"};
  }
  // the body's left spine now ends in `@` (Cur): linearise without it
  std::function<void(const JP&)> lin = [&](const JP& x) {
    if (x->k == JNode::Cur) return;
    if (x->k == JNode::Sub && x->kids[0]->k == JNode::Cur) { jlin(c, x->kids[1], ops, list); return; }
    if (x->k == JNode::Sub) { lin(x->kids[0]); jlin(c, x->kids[1], ops, list); return; }
    if (x->k == JNode::Proj) {
      const JP& f = x->kids[0];
      if (f->k != JNode::Flat) throw Fallback{"JMESPath: projection form"};
      lin(f->kids[0]);
      ops.push_back(JO_FLAT);
      list = true;
      const JP& rr = x->kids[1];
      if (rr->k == JNode::Ident) return;
      if (rr->k == JNode::Func) {
        if (rr->name != "keys" || rr->kids.size() != 1 || rr->kids[0]->k != JNode::Cur) throw Fallback{"JMESPath: function"};
        ops.push_back(JO_KEYS);
        return;
      }
      jlin(c, rr, ops, list);
      return;
    }
    if (x->k == JNode::Filter) {
      lin(x->kids[0]);
      if (list) throw Fallback{"JMESPath: filter inside a projection"};
      jfilter(c, x->kids[2], ops);
      list = true;
      const JP& rr = x->kids[1];
      if (rr->k == JNode::Ident) return;
      jlin(c, rr, ops, list);
      return;
    }
    throw Fallback{"JMESPath: expression outside the device subset"};
  };
  if (body) lin(body);
  // fuse projection keys(@) + flatten; keys() left unflattened inside a projection is a list of lists
  std::vector<uint32_t> fused;
  bool pure = !has_or;
  for (size_t i = 0; i < ops.size();) {
    const uint32_t op = ops[i];
    if (op == JO_FIELD) { fused.push_back(op); fused.push_back(ops[i + 1]); i += 2; continue; }
    pure = false;
    if (op == JO_MULTI || op == JO_FILTER) {
      const uint32_t w = jop_width(ops.data() + i);
      fused.insert(fused.end(), ops.begin() + i, ops.begin() + i + w);
      i += w;
      continue;
    }
    if (op == JO_KEYS) {
      bool in_list = false;  // was a FLAT before it?
      for (size_t j = 0; j < fused.size(); j += jop_width(fused.data() + j))
        if (fused[j] == JO_FLAT || fused[j] == JO_FILTER) in_list = true;
      if (in_list) {
        if (i + 1 >= ops.size() || ops[i + 1] != JO_FLAT) throw Fallback{"JMESPath: keys() projection without []"};
        fused.push_back(JO_KEYS_FLAT);
        i += 2;
      } else {
        fused.push_back(JO_KEYS);
        i++;
      }
      continue;
    }
    fused.push_back(op);
    i++;
  }
  // a multi-select list or keys() outside a projection is a plain list: only [] (or the end) may follow
  for (size_t i = 0; i < fused.size();) {
    const uint32_t op = fused[i];
    const size_t w = jop_width(fused.data() + i);
    if ((op == JO_MULTI || op == JO_KEYS) && i + w < fused.size() && fused[i + w] != JO_FLAT)
      throw Fallback{"JMESPath: list outside a projection"};
    i += w;
  }
  if (has_len) {
    fused.push_back(JO_LENGTH);
    pure = false;  // the argument of a function: a missing key is null, not NotFoundError
  }
  if (has_or) {
    Value lit = pj::parse(pj::dump(orlit), false);
    fused.push_back(JO_OR);
    fused.push_back(emit_cnode(c, lit));
  }
  if (post != NONE) {  // the function's argument: a missing key is null, not NotFoundError
    if (root != JR_OBJECT || !jmes_chain_form_ops(fused)) throw Fallback{"JMESPath: function of a projection / element"};
    fused.push_back(post);
    if (post == JO_REGEX) fused.push_back(post_q);
    pure = false;
    if (post == JO_UPPER) c.rs.uses_upper = true;
  }
  // request.operation: the background scan's JSON context holds "CREATE" (scanner.go:97; CLI default common.go:287)
  const uint32_t oplit = root == JR_OPERATION ? emit_cnode(c, Value::S("CREATE")) : NONE;
  if (root == JR_OPERATION) {
    // the value is that literal whatever follows (`|| <default>` never applies to the non-empty "CREATE"): a plain
    // literal operand, so the rule needs no JMESPath evaluation (light match kernel)
    o->kind = OK_LIT;
    o->a = oplit;
    o->nseg = 0;
    return true;
  }
  o->kind = OK_JMES;
  o->a = (uint32_t)c.rs.pool.size();
  c.rs.pool.push_back(root | (pure ? JF_PURE : 0u));
  for (auto w : fused) c.rs.pool.push_back(w);
  o->nseg = (uint16_t)(c.rs.pool.size() - o->a);
  return true;
}
bool var_anywhere(const Value& v) {
  if (v.t == T::Str) return var_syntax(v.s);
  for (auto& e : v.a) if (var_anywhere(e)) return true;
  for (auto& kv : v.o) if (var_syntax(kv.first) || var_anywhere(kv.second)) return true;
  return false;
}
// operator.GetOperatorFromStringPattern(s) == InRange (pkg/engine/operator/operator.go:35-61)
bool in_range_pattern(const std::string& s) {
  if (s.size() < 2) return false;
  if (s[0] == '>' || s[0] == '<' || s[0] == '!') return false;
  std::string l, r;
  if (range_split(s, "!-", l, r)) return false;
  return range_split(s, "-", l, r);
}

// literal JSON value -> cnodes (after the Condition.GetKey round trip: json.Marshal + util/json decode)
uint32_t emit_cnode(Cx& c, const Value& v) {
  Node n{};
  switch (v.t) {
    case T::Null: n.tk = N_NULL; break;
    case T::Bool: n.tk = v.b ? N_TRUE : N_FALSE; n.a = v.b; break;
    case T::Int: n.tk = N_INT; n.a = (uint32_t)(uint64_t)v.i; n.b = (uint32_t)((uint64_t)v.i >> 32);
      n.c = c.sid(std::to_string(v.i)); break;
    case T::Float: {
      uint64_t bits;
      memcpy(&bits, &v.f, 8);
      n.tk = N_FLOAT; n.a = (uint32_t)bits; n.b = (uint32_t)(bits >> 32); n.c = c.sid(pj::go_fmt_g(v.f));
      break;
    }
    case T::Str: n.tk = N_STR; n.a = c.sid(v.s); break;
    case T::Arr: {
      uint32_t at = (uint32_t)c.rs.cnodes.size();
      n.tk = N_ARR; n.a = at + 1; n.b = (uint32_t)v.a.size();
      c.rs.cnodes.push_back(n);
      for (auto& e : v.a) {
        if (e.t == T::Arr || e.t == T::Obj) throw Fallback{"conditions: nested literal"};
        emit_cnode(c, e);
      }
      return at;
    }
    default: throw Fallback{"conditions: map literal"};
  }
  c.rs.cnodes.push_back(n);
  return (uint32_t)c.rs.cnodes.size() - 1;
}

CondOperand compile_operand(Cx& c, const Value* v, CondText& ct, int side, const std::string& path) {
  CondOperand o{};
  o.kind = OK_NIL;
  ct.path[side] = path;
  if (!v || v->t == T::Null) return o;
  if (v->t == T::Str && var_syntax(v->s)) {
    std::vector<std::string> segs;
    if (!object_var(v->s, segs, &ct.var[side])) {
      if (v->s.find("$(") != std::string::npos || !jmes_var(c, v->s, c.allow_element, &o, &ct.var[side], &c.uses_op))
        throw Fallback{"conditions: variables beyond request.object paths"};
      return o;
    }
    o.kind = OK_PATH;
    o.nseg = (uint16_t)segs.size();
    o.a = (uint32_t)c.rs.pool.size();
    for (auto& sg : segs) c.rs.pool.push_back(c.sid(sg));
    ct.segs[side] = segs;
    return o;
  }
  if (var_anywhere(*v)) throw Fallback{"conditions: variables inside a literal"};
  Value lit = pj::parse(pj::dump(*v), false);
  if (lit.t == T::Null) return o;
  o.kind = OK_LIT;
  o.a = emit_cnode(c, lit);
  if (lit.t == T::Str) {
    const std::string& s = lit.s;
    if (in_range_pattern(s)) o.sv |= SV_RANGE;
    try {
      Value j = pj::parse(s, true);
      o.sv |= SV_JSON;
      bool ok = j.t == T::Null || j.t == T::Arr;
      if (j.t == T::Arr) for (auto& e : j.a) if (e.t != T::Str && e.t != T::Null) ok = false;
      if (ok) {
        o.sv |= SV_LIST;
        o.list = (uint32_t)c.rs.pool.size();
        o.nlist = (uint32_t)j.a.size();
        for (auto& e : j.a) c.rs.pool.push_back(c.sid(e.t == T::Str ? e.s : ""));
      }
    } catch (pj::Error&) {
    }
  }
  return o;
}

// operator name -> CondOp (operator.go:27-75: handler chosen case-insensitively; numeric compareByCondition
// matches the exact operator name, so other spellings of the numeric operators are always false)
uint8_t cond_op(const std::string& op) {
  std::string l = op;
  for (auto& ch : l) ch = (char)tolower((unsigned char)ch);
  if (l == "durationgreaterthanorequals" || l == "durationgreaterthan" || l == "durationlessthanorequals" ||
      l == "durationlessthan") {  // DurationOperatorHandler: durationCompareByCondition matches the exact name
    if (op == "DurationGreaterThan") return CO_DGT;
    if (op == "DurationGreaterThanOrEquals") return CO_DGE;
    if (op == "DurationLessThan") return CO_DLT;
    if (op == "DurationLessThanOrEquals") return CO_DLE;
    return CO_FALSE;
  }
  if (l == "equal" || l == "equals") return CO_EQ;
  if (l == "notequal" || l == "notequals") return CO_NE;
  if (l == "in") return CO_IN;
  if (l == "notin") return CO_NOTIN;
  if (l == "anyin") return CO_ANYIN;
  if (l == "allin") return CO_ALLIN;
  if (l == "anynotin") return CO_ANYNOTIN;
  if (l == "allnotin") return CO_ALLNOTIN;
  if (op == "GreaterThan") return CO_GT;
  if (op == "GreaterThanOrEquals") return CO_GE;
  if (op == "LessThan") return CO_LT;
  if (op == "LessThanOrEquals") return CO_LE;
  return CO_FALSE;
}
bool valid_op_exact(const std::string& op) {  // kyvernov1.ConditionOperators (common_types.go:225-244)
  static const char* ops[] = {"Equal", "Equals", "NotEqual", "NotEquals", "In", "AnyIn", "AllIn", "NotIn", "AnyNotIn",
                              "AllNotIn", "GreaterThanOrEquals", "GreaterThan", "LessThanOrEquals", "LessThan",
                              "DurationGreaterThanOrEquals", "DurationGreaterThan", "DurationLessThanOrEquals",
                              "DurationLessThan"};
  for (auto o : ops) if (op == o) return true;
  return false;
}

uint32_t compile_cond(Cx& c, const Value& e, const std::string& path, bool old_list) {
  if (e.t != T::Obj) throw Fallback{"conditions: malformed condition"};
  for (auto& kv : e.o)
    if (kv.first != "key" && kv.first != "operator" && kv.first != "value" && kv.first != "message")
      throw Fallback{"conditions: unknown condition field"};
  const Value* op = e.get("operator");
  if (op && op->t != T::Str && op->t != T::Null) throw Fallback{"conditions: malformed operator"};
  std::string ops = op && op->t == T::Str ? op->s : "";
  if (old_list && !valid_op_exact(ops)) throw Fallback{"conditions: invalid condition operator"};
  Cond cd{};
  cd.op = cond_op(ops);
  cd.leaf = cd.leaf_neg = NONE;
  CondText ct;
  cd.key = compile_operand(c, e.get("key"), ct, 0, path + "/key");
  cd.value = compile_operand(c, e.get("value"), ct, 1, path + "/value");
  if (cd.value.sv & SV_RANGE) {
    const std::string& s = c.rs.dict.strs[c.rs.cnodes[cd.value.a].a];
    cd.leaf = compile_leaf(c, Value::S(s));
    std::string s2 = s;
    size_t i = s2.find('-');
    if (i != std::string::npos) s2.replace(i, 1, "!-");
    cd.leaf_neg = compile_leaf(c, Value::S(s2));
  }
  c.rs.conds.push_back(cd);
  c.rs.cond_text.push_back(ct);
  return (uint32_t)c.rs.conds.size() - 1;
}

// rule.preconditions / validate.deny.conditions -> CondProg (utils/utils.go:52 TransformConditions,
// pkg/utils/api/json.go:30-85); shapes outside the device subset throw Fallback
uint32_t compile_conds(Cx& c, const Value* doc) {
  CondProg p{};
  p.nany = NONE;
  std::vector<Cond> blk;
  auto block = [&](const Value& list, const std::string& base, bool old_list, uint32_t* first, uint32_t* n) {
    std::vector<uint32_t> ids;
    for (size_t i = 0; i < list.a.size(); i++) ids.push_back(compile_cond(c, list.a[i], base + "/" + std::to_string(i), old_list));
    *first = ids.empty() ? (uint32_t)c.rs.conds.size() : ids[0];
    *n = (uint32_t)ids.size();
  };
  if (!doc || doc->t == T::Null) {
    p.all0 = 0; p.nall = 0;
  } else if (doc->t == T::Arr) {
    block(*doc, "", true, &p.all0, &p.nall);
  } else if (doc->t == T::Obj) {
    for (auto& kv : doc->o) if (kv.first != "any" && kv.first != "all") throw Fallback{"conditions: unknown field"};
    const Value* any = doc->get("any");
    const Value* all = doc->get("all");
    if (any && any->t != T::Null) {
      if (any->t != T::Arr) throw Fallback{"conditions: malformed any"};
      block(*any, "/any", false, &p.any0, &p.nany);
    }
    if (all && all->t != T::Null) {
      if (all->t != T::Arr) throw Fallback{"conditions: malformed all"};
      block(*all, "/all", false, &p.all0, &p.nall);
    }
  } else {
    throw Fallback{"conditions: malformed"};
  }
  c.rs.cprogs.push_back(p);
  return (uint32_t)c.rs.cprogs.size() - 1;
}

// validate.foreach (validation.go:319-421): entries with a JMESPath-subset list (over request.object; inside a nested
// foreach also over the enclosing element), optional per-element preconditions / elementScope, and one validator:
// deny conditions, a pattern / anyPattern (element variables as whole-string values, L_DYN), or a nested foreach (one
// level). Context entries and other variables stay on the CPU. Returns the pool offset of [n, entries...].
uint32_t compile_foreach_entries(Cx& c, const Value& fe, int depth, bool* plain_deny) {
  if (fe.t != T::Arr || fe.a.empty()) throw Fallback{"foreach"};
  if (depth > (int)FOREACH_MAX_NEST) throw Fallback{"foreach: nested deeper than the device evaluates"};
  std::vector<ForeachEntry> ents;
  for (auto& e : fe.a) {
    if (e.t != T::Obj) throw Fallback{"foreach"};
    for (auto& kv : e.o)
      if (kv.first != "list" && kv.first != "deny" && kv.first != "preconditions" && kv.first != "elementScope" &&
          kv.first != "pattern" && kv.first != "anyPattern" && kv.first != "foreach")
        throw Fallback{"foreach: " + kv.first};
    const Value* l = e.get("list");
    if (!l || l->t != T::Str) throw Fallback{"foreach"};
    ForeachEntry fx{};
    fx.dyn = NONE;
    fx.body = NONE;
    std::vector<std::string> segs;
    if (object_var("{{" + l->s + "}}", segs, nullptr)) {  // plain request.object chain
      fx.list.kind = OK_PATH;
      fx.list.nseg = (uint16_t)segs.size();
      fx.list.a = (uint32_t)c.rs.pool.size();
      for (auto& sg : segs) c.rs.pool.push_back(c.sid(sg));
    } else {
      const bool ae = c.allow_element;
      c.allow_element = depth > 0;  // a nested list reads the enclosing element
      if (!jmes_var(c, "{{" + l->s + "}}", c.allow_element, &fx.list, nullptr, &c.uses_op)) throw Fallback{"foreach: list"};
      c.allow_element = ae;
      // eval_foreach iterates path and JMESPath lists only; a literal (request.operation: the one-element list
      // ["CREATE"] in the reference) is not a program it can run
      if (fx.list.kind != OK_PATH && fx.list.kind != OK_JMES) throw Fallback{"foreach: list"};
    }
    const Value* es = e.get("elementScope");
    if (es && es->t != T::Null && es->t != T::Bool) throw Fallback{"foreach: elementScope"};
    fx.scope = !es || es->t == T::Null ? 0u : es->b ? 2u : 1u;
    c.allow_element = true;
    const Value* pre = e.get("preconditions");
    fx.pre = pre && pre->t != T::Null ? compile_conds(c, pre) : NONE;
    const Value* d = e.get("deny");
    const Value* pat = e.get("pattern");
    const Value* ap = e.get("anyPattern");
    if (d && d->t != T::Null) {  // validate(): deny wins over pattern / anyPattern and foreach
      if (d->t != T::Obj) throw Fallback{"foreach"};
      fx.kind = FE_DENY;
      fx.deny = compile_conds(c, d->get("conditions"));
      if (depth > 0) *plain_deny = false;
    } else if ((pat && pat->t != T::Null) || (ap && ap->t != T::Null)) {
      *plain_deny = false;
      fx.deny = NONE;
      if ((pat && pat->t != T::Null && keys_have_vars(*pat)) || (ap && ap->t != T::Null && keys_have_vars(*ap)))
        throw Fallback{"foreach: variables in pattern keys"};
      c.dyn_ok = true;
      c.dyn.clear();
      if (pat && pat->t != T::Null) {
        fx.kind = FE_PATTERN;
        fx.body = compile_pattern_root(c, *pat);
      } else {
        if (ap->t != T::Arr) throw Fallback{"foreach: anyPattern is not a list"};
        std::vector<uint32_t> roots;
        for (auto& p : ap->a) roots.push_back(compile_pattern_root(c, p));
        if (roots.size() > MAX_ALTS) throw Fallback{"too many anyPattern alternatives"};
        fx.kind = FE_ANYPATTERN;
        fx.nalts = (uint32_t)roots.size();
        fx.body = (uint32_t)c.rs.pool.size();
        for (auto x : roots) c.rs.pool.push_back(x);
      }
      c.dyn_ok = false;
      if (!c.dyn.empty()) {
        fx.dyn = (uint32_t)c.rs.pool.size();
        c.rs.pool.push_back((uint32_t)c.dyn.size());
        for (auto& dv : c.dyn) c.rs.pool.insert(c.rs.pool.end(), dv.begin(), dv.end());
      }
    } else if (nonempty(e.get("foreach"))) {
      *plain_deny = false;
      fx.deny = NONE;
      fx.kind = FE_NESTED;
      c.allow_element = false;
      fx.body = compile_foreach_entries(c, *e.get("foreach"), depth + 1, plain_deny);
    } else {
      fx.kind = FE_NONE;  // no validator for the element: "skip rule due to empty result"
      fx.deny = NONE;
      *plain_deny = false;
    }
    c.allow_element = false;
    ents.push_back(fx);
  }
  const uint32_t at = (uint32_t)c.rs.pool.size();
  c.rs.pool.push_back((uint32_t)ents.size());
  for (auto& fx : ents) {
    uint32_t w[sizeof(ForeachEntry) / 4];
    memcpy(w, &fx, sizeof fx);
    for (uint32_t x : w) c.rs.pool.push_back(x);
  }
  return at;
}

uint32_t compile_foreach(Cx& c, const Value& fe, const std::string& message, bool* plain_deny) {
  if (var_syntax(message)) throw Fallback{"foreach: message with variables"};
  *plain_deny = true;
  return compile_foreach_entries(c, fe, 0, plain_deny);
}

// deny message with `{{ request.object... }}` references -> parts (false: other variables, escapes, references)
bool compile_message(Cx& c, const std::string& msg, RuleMeta& rm) {
  rm.msg_parts.clear();
  rm.msg_whole_var = false;
  if (!var_syntax(msg)) return true;
  if (msg.find("$(") != std::string::npos || msg.find("\\{{") != std::string::npos) return false;
  std::vector<std::string> segs;
  auto add_var = [&](const std::vector<std::string>& sg) {
    RuleMeta::MsgPart mp;
    mp.var = true;
    for (auto& x : sg) mp.segs.push_back(c.sid(x));
    rm.msg_parts.push_back(mp);
  };
  if (object_var(msg, segs, nullptr)) { rm.msg_whole_var = true; add_var(segs); return true; }
  size_t i = 0;
  while (i < msg.size()) {
    size_t a = msg.find("{{", i);
    if (a == std::string::npos) { rm.msg_parts.push_back({msg.substr(i), {}, false}); break; }
    size_t b = msg.find("}}", a + 2);
    if (b == std::string::npos) return false;
    if (!object_var(msg.substr(a, b + 2 - a), segs, nullptr)) return false;
    if (a > i) rm.msg_parts.push_back({msg.substr(i, a - i), {}, false});
    add_var(segs);
    i = b + 2;
  }
  return true;
}

// ---------------------------------------------------------------- $() references (variables/vars.go:244-346)
// Pattern references resolve against the pattern document itself (substituteReferences runs on the raw pattern /
// anyPattern before variables), so they are resolved here, once, at compile time. Resolved: a reference naming
// exactly one leaf (or the single key of a one-entry map) whose value is a string, or a number / string under an
// operator prefix. Everything the reference turns into a rule error (unresolvable path, nil, a non-string raw value)
// and every order-dependent case (several elements on one path, a renamed key colliding) stays a CPU fallback.
struct RefFail { std::string why; };
Value str_value(const std::string& s) {
  Value v;
  v.t = T::Str;
  v.s = s;
  return v;
}

// end of `.[^ ]*\)` starting at q (the '.'), or npos: the last ')' before the first space after q
size_t ref_tail(const std::string& s, size_t q) {
  if (q >= s.size() || s[q] == '\n') return std::string::npos;
  size_t lim = s.find(' ', q + 1);
  if (lim == std::string::npos) lim = s.size();
  for (size_t e = lim; e-- > q + 1;) if (s[e] == ')') return e;
  return std::string::npos;
}
// RegexReferences `^\$\(.[^\ ]*\)|[^\\]\$\(.[^\ ]*\)` / RegexEscpReferences `\\\$\(.[^\ ]*\)` FindAllString
std::vector<std::string> find_refs(const std::string& s, bool escaped) {
  std::vector<std::string> out;
  size_t p = 0;
  while (p < s.size()) {
    size_t e = std::string::npos;
    if (escaped) {
      if (s[p] == '\\' && s.compare(p + 1, 2, "$(") == 0) e = ref_tail(s, p + 3);
    } else {
      if (p == 0 && s.compare(0, 2, "$(") == 0) e = ref_tail(s, 2);
      if (e == std::string::npos && s[p] != '\\' && s.compare(p + 1, 2, "$(") == 0) e = ref_tail(s, p + 3);
    }
    if (e == std::string::npos) { p++; continue; }
    out.push_back(s.substr(p, e + 1 - p));
    p = e + 1;
  }
  return out;
}
// path.Clean
std::string clean_path(const std::string& p) {
  if (p.empty()) return ".";
  const bool rooted = p[0] == '/';
  std::vector<std::string> st;
  size_t i = 0;
  while (i <= p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    std::string e = p.substr(i, j - i);
    if (!(e.empty() || e == ".")) {
      if (e == "..") {
        if (!st.empty() && st.back() != "..") st.pop_back();
        else if (!rooted) st.push_back("..");
      } else {
        st.push_back(e);
      }
    }
    if (j == p.size()) break;
    i = j + 1;
  }
  std::string out = rooted ? "/" : "";
  for (size_t k = 0; k < st.size(); k++) out += (k ? "/" : "") + st[k];
  return out.empty() ? "." : out;
}
// anchor.RemoveAnchorsFromPath (anchor/utils.go:23-40)
std::string remove_anchors_from_path(const std::string& str) {
  std::vector<std::string> parts;
  size_t st = 0;
  for (size_t i = 0; i <= str.size(); i++)
    if (i == str.size() || str[i] == '/') { parts.push_back(str.substr(st, i - st)); st = i + 1; }
  if (!parts.empty() && parts[0].empty()) parts.erase(parts.begin());
  std::string joined;
  for (auto& p : parts) {
    Anc a = parse_anchor(p);
    const std::string q = a.t != AT::None ? a.key : p;
    if (!q.empty()) joined += joined.empty() ? q : "/" + q;
  }
  std::string out = joined.empty() ? "" : clean_path(joined);
  if (!str.empty() && str[0] == '/') out = "/" + (out == "." ? std::string() : out);
  return out;
}
// the elements getValueFromReference visits (vars.go:560-575 over jsonutils' OnlyForLeafsAndKeys): leaves at their
// own path, map keys at their map's path; keyed by RemoveAnchorsFromPath(path)
void ref_index(const Value& v, const std::string& path, std::map<std::string, std::vector<Value>>* idx) {
  if (v.t == T::Obj) {
    for (auto& kv : v.o) {
      if (kv.first.find('/') != std::string::npos) throw RefFail{"a pattern key contains '/'"};
      (*idx)[remove_anchors_from_path(path)].push_back(str_value(kv.first));
      ref_index(kv.second, path + "/" + kv.first, idx);
    }
  } else if (v.t == T::Arr) {
    for (size_t i = 0; i < v.a.size(); i++) ref_index(v.a[i], path + "/" + std::to_string(i), idx);
  } else {
    (*idx)[remove_anchors_from_path(path)].push_back(v);
  }
}
// operator.GetOperatorFromStringPattern prefix length (operator.go:35-61); -1 for the range operators
int ref_op_len(const std::string& p) {
  if (p.size() < 2) return 0;
  if (p.compare(0, 2, ">=") == 0 || p.compare(0, 2, "<=") == 0) return 2;
  if (p[0] == '>' || p[0] == '<' || p[0] == '!') return 1;
  std::string l, r;
  if (range_split(p, "!-", l, r) || range_split(p, "-", l, r)) return -1;
  return 0;
}
// substituteReferencesIfAny on one string at `path` (vars.go:286-346)
std::string subst_refs(const std::string& in, const std::string& path, const std::map<std::string, std::vector<Value>>& idx) {
  std::string value = in;
  for (std::string v : find_refs(in, false)) {
    const bool initial = v.compare(0, 2, "$(") == 0;
    const std::string old = v;
    if (!initial) v = v.substr(1);
    // resolveReference (vars.go:472-502): strings.Trim(reference, "$()"), operator prefix, absolute path
    size_t a = 0, b = v.size();
    auto trim = [](char c) { return c == '$' || c == '(' || c == ')'; };
    while (a < b && trim(v[a])) a++;
    while (b > a && trim(v[b - 1])) b--;
    std::string p = v.substr(a, b - a);
    const int ol = ref_op_len(p);
    if (ol < 0) throw RefFail{"range operator in a reference"};
    const std::string op = p.substr(0, ol);
    p = p.substr(ol);
    if (p.empty()) throw RefFail{"empty reference (rule error)"};
    const std::string abs = p[0] == '/' ? p : clean_path(path.empty() ? p : path + "/" + p);
    auto it = idx.find(abs);
    if (it == idx.end()) throw RefFail{"unresolved reference (rule error)"};
    if (it->second.size() != 1) throw RefFail{"reference names several elements (map order)"};
    const Value& x = it->second[0];
    std::string val;
    if (op.empty()) {
      if (x.t != T::Str) throw RefFail{"reference to a non-string value (rule error)"};
      val = x.s;
    } else if (x.t == T::Str) {
      val = op + x.s;
    } else if (x.t == T::Float) {
      val = op + pj::go_fmt_f6(x.f);  // fmt "%f" of the float64 the policy JSON decodes to
    } else if (x.t == T::Int) {
      val = op + std::to_string(x.i);
    } else {
      throw RefFail{"operator reference to a non-scalar (rule error)"};
    }
    const std::string repl = (initial ? std::string() : std::string(1, old[0])) + val;
    size_t at = value.find(old);
    if (at != std::string::npos) value.replace(at, old.size(), repl);
  }
  for (const std::string& v : find_refs(value, true)) {  // `\$(...)` -> `$(...)`, every occurrence
    const std::string to = v.substr(1);
    for (size_t at = value.find(v); at != std::string::npos; at = value.find(v, at + to.size())) value.replace(at, v.size(), to);
  }
  return value;
}
Value resolve_refs_rec(const Value& v, const std::string& path, const std::map<std::string, std::vector<Value>>& idx) {
  if (v.t == T::Str) return str_value(subst_refs(v.s, path, idx));
  if (v.t == T::Arr) {
    Value out = v;
    for (size_t i = 0; i < v.a.size(); i++) out.a[i] = resolve_refs_rec(v.a[i], path + "/" + std::to_string(i), idx);
    return out;
  }
  if (v.t == T::Obj) {
    Value out;
    out.t = T::Obj;
    for (auto& kv : v.o) {
      std::string k = subst_refs(kv.first, path, idx);
      Value val = resolve_refs_rec(kv.second, path + "/" + kv.first, idx);
      for (auto& e : out.o) if (e.first == k) throw RefFail{"renamed key collides (map order)"};
      if (k != kv.first) for (auto& e : v.o) if (e.first == k) throw RefFail{"renamed key collides (map order)"};
      out.o.emplace_back(k, std::move(val));
    }
    return out;
  }
  return v;
}
bool has_ref_syntax(const Value& v) {
  if (v.t == T::Str) return v.s.find("$(") != std::string::npos;
  for (auto& e : v.a) if (has_ref_syntax(e)) return true;
  for (auto& kv : v.o) if (kv.first.find("$(") != std::string::npos || has_ref_syntax(kv.second)) return true;
  return false;
}
// the pattern / anyPattern document after substituteReferences, or RefFail
Value resolve_references(const Value& doc) {
  std::map<std::string, std::vector<Value>> idx;
  ref_index(doc, "", &idx);
  return resolve_refs_rec(doc, "", idx);
}

// ---------------------------------------------------------------- rule classification
bool contains_vars(const Value& v) {  // after reference resolution: `{{ }}` variables remain for the CPU engine
  auto hit = [](const std::string& s) { return s.find("{{") != std::string::npos; };
  if (v.t == T::Str) return hit(v.s);
  if (v.t == T::Arr) { for (auto& e : v.a) if (contains_vars(e)) return true; return false; }
  if (v.t == T::Obj) { for (auto& kv : v.o) if (hit(kv.first) || contains_vars(kv.second)) return true; }
  return false;
}

std::string fallback_reason(const Value& r) {  // validator.validate dispatch (validation.go:276-317)
  const Value* val = r.get("validate");
  if (nonempty(r.get("context"))) return "context";
  if (nonempty(r.get("verifyImages"))) return "verifyImages";
  if (!val) return "";
  if (!nil(val->get("deny"))) return val->get("deny")->t == T::Obj ? "" : "deny";
  if ((val->get("pattern") && contains_vars(*val->get("pattern"))) || (val->get("anyPattern") && contains_vars(*val->get("anyPattern"))))
    return "variables";
  if (!nil(val->get("manifests"))) return "manifests";
  return "";
}

}  // namespace

void mark_gate_exact(Ruleset& rs);

Ruleset* compile_ruleset(const char* json, size_t len, std::string* err, const char* exceptions, size_t ex_len,
                         bool background) {
  auto rs = std::make_unique<Ruleset>();
  try {
    seed_dict(rs->dict);
    std::vector<Value> docs = pj::parse_many(json, len, true);
    // PolicyExceptions in input order (the lister order FindExceptions walks, pkg/engine/policyContext.go:150-169):
    // key (cache.MetaNamespaceKeyFunc), the (policy key, rule name) pairs it lists, its match block
    struct Exc { std::string key; std::set<std::pair<std::string, std::string>> names; const Value* match; };
    std::vector<Value> exdocs;
    std::vector<Exc> excs;
    if (exceptions && ex_len) {
      exdocs = pj::parse_many(exceptions, ex_len, true);
      for (auto& ex : exdocs) {
        if (ex.t != T::Obj || ex.str_or("kind") != "PolicyException") continue;
        const Value* spec = ex.get("spec");
        const Value* lst = spec ? spec->get("exceptions") : nullptr;
        if (!lst || lst->t != T::Arr) continue;
        const Value* meta = ex.get("metadata");
        const std::string ns = meta ? meta->str_or("namespace") : "", nm = meta ? meta->str_or("name") : "";
        Exc e{ns.empty() ? nm : ns + "/" + nm, {}, spec->get("match")};
        for (auto& x : lst->a)
          for (auto& rn : strs(x.get("ruleNames"))) e.names.insert({x.str_or("policyName"), rn});
        excs.push_back(std::move(e));
      }
    }
    Cx c{*rs};
    c.background = background;
    for (auto& pol : docs) {
      if (pol.t != T::Obj) continue;
      std::string kind = pol.str_or("kind");
      if (kind != "ClusterPolicy" && kind != "Policy") continue;
      PolicyMeta pm;
      const Value* meta = pol.get("metadata");
      pm.name = meta ? meta->str_or("name") : "";
      pm.ns = meta ? meta->str_or("namespace") : "";
      pm.kind = kind;
      const Value* ann = meta ? meta->get("annotations") : nullptr;
      pm.scored_false = ann && ann->str_or("policies.kyverno.io/scored") == "false";
      const Value* spec = pol.get("spec");
      pm.apply_one = spec && spec->str_or("applyRules") == "One";
      pm.failure_action = spec ? spec->str_or("validationFailureAction", "Audit") : "Audit";
      uint32_t pidx = (uint32_t)rs->policies.size();
      pm.first_rule = (uint32_t)rs->rules.size();
      for (auto& r : compute_rules(pol)) {
        pm.all_rule_names.push_back(r.str_or("name"));
        const Value* val = r.get("validate");
        bool hasValidate = val && val->t == T::Obj && !val->o.empty();
        if (!hasValidate && !nonempty(r.get("verifyImages"))) continue;  // no response (validation.go:144-149)
        RuleDesc rd{};
        rd.pre = NONE;
        rd.exc = NONE;
        RuleMeta rm;
        rm.name = r.str_or("name");
        rm.message = val ? val->str_or("message") : "";
        rm.policy = pidx;
        rm.kinds = match_kinds(r.get("match"));
        rm.has_validate = hasValidate;
        rm.message_vars = rm.message.find("{{") != std::string::npos || rm.message.find("$(") != std::string::npos;
        rd.policy = pidx;
        size_t mark_p = rs->pnodes.size(), mark_e = rs->pentries.size(), mark_l = rs->leaves.size(),
               mark_a = rs->atoms.size(), mark_pool = rs->pool.size(), mark_t = rs->templates.size(),
               mark_cn = rs->cnodes.size(), mark_cd = rs->conds.size(), mark_cp = rs->cprogs.size();
        try {
          bool em = false;
          rd.match = compile_block(c, r.get("match"), true, &em);
          rd.exclude = compile_block(c, r.get("exclude"), false, &em);
          rd.empty_may_match = em;
          // $() references of the pattern / anyPattern, resolved against the document (substitutePatterns)
          Value rr;
          const Value* rp = &r;
          std::string ref_why;
          for (const char* f : {"pattern", "anyPattern"}) {
            const Value* pv = val ? val->get(f) : nullptr;
            if (!pv || !has_ref_syntax(*pv)) continue;
            try {
              Value resolved = resolve_references(*pv);
              if (rp == &r) { rr = r; rp = &rr; }
              rr.getm("validate")->set(f, std::move(resolved));
            } catch (RefFail& e) {
              ref_why = std::string("references: ") + e.why;
            }
          }
          const Value* rval = rp->get("validate");
          std::string why = ref_why.empty() ? fallback_reason(*rp) : ref_why;
          const std::string pkey = pm.ns.empty() ? pm.name : pm.ns + "/" + pm.name;  // cache.MetaNamespaceKeyFunc
          // exception candidates of this rule (PolicyExceptionSpec.Contains), checked after the match on the device
          rd.exc = NONE;
          std::vector<uint32_t> cands;
          for (auto& e : excs) {
            if (!e.names.count({pkey, rm.name})) continue;
            compile_exc_block(c, e.match, cands);
            rm.exc_keys.push_back(e.key);
          }
          if (rm.exc_keys.size() > MAX_EXC) throw Fallback{"exception: more than 27 PolicyExceptions name the rule"};
          if (!rm.exc_keys.empty()) {
            rd.exc = (uint32_t)rs->pool.size();
            rs->pool.push_back((uint32_t)rm.exc_keys.size());
            rs->pool.insert(rs->pool.end(), cands.begin(), cands.end());
          }
          c.nslots = 0;
          c.sites.clear();
          c.uses_op = false;
          c.allow_element = false;
          c.dyn_ok = false;
          c.dyn.clear();
          rd.pre = NONE;
          if (why.empty() && !nil(r.get("preconditions"))) rd.pre = compile_conds(c, r.get("preconditions"));
          if (!why.empty()) {
            rd.kind = RK_FALLBACK;
            rm.reason = why;
          } else if (val && !nil(val->get("deny"))) {  // deny wins over pattern (validation.go:290-292)
            rd.kind = RK_DENY;
            rd.root = compile_conds(c, val->get("deny")->get("conditions"));
            rm.message_vars = !compile_message(c, rm.message, rm);
          } else if (val && !nil(val->get("pattern"))) {
            rd.kind = RK_PATTERN;
            rd.root = compile_pattern_root(c, *rval->get("pattern"));
            // buildErrorMessage substitutes the message's variables (validation.go:722-745): request.object
            // references are rendered on the host from the resource (capi.cpp subst_message)
            rm.message_vars = !compile_message(c, rm.message, rm);
          } else if (val && !nil(val->get("anyPattern"))) {
            const Value* ap = rval->get("anyPattern");
            if (ap->t != T::Arr) {
              rd.kind = RK_ERROR;
              rm.reason = "failed to deserialize anyPattern, expected type array";
            } else {
              std::vector<uint32_t> roots;
              for (auto& p : ap->a) roots.push_back(compile_pattern_root(c, p));
              if (roots.size() > MAX_ALTS) throw Fallback{"too many anyPattern alternatives"};
              rd.kind = RK_ANYPATTERN;
              rd.root = (uint32_t)rs->pool.size();
              rd.nalts = (uint32_t)roots.size();
              for (auto x : roots) rs->pool.push_back(x);
              rm.message_vars = false;  // buildAnyPatternErrorMessage / the pass response take the message as written
                                        // (validation.go:701, 747-758): no substitution
            }
          } else if (val && !nil(val->get("podSecurity"))) {
            rd.kind = RK_PSS;
            rd.root = compile_pss(c, *val->get("podSecurity"));
            rm.pss_level = val->get("podSecurity")->str_or("level");
            rm.pss_version = val->get("podSecurity")->str_or("version");
            rm.message_vars = false;  // the PodSecurity responses do not use the message (validation.go:560-566)
          } else if (val && nonempty(val->get("foreach"))) {
            rd.kind = RK_FOREACH;
            rd.root = compile_foreach(c, *val->get("foreach"), rm.message, &rm.foreach_texts);
          } else {
            continue;  // "invalid validation rule": no response
          }
          if (c.uses_op) rd.flags |= RD_USES_OPERATION;
          rd.meta_sites = (uint32_t)rs->metas.size();
          rd.nmeta = (uint32_t)c.sites.size();
          for (auto& s : c.sites) rs->metas.push_back(s);
          rd.nslots = (uint8_t)c.nslots;
          rd.uses_meta = c.sites.empty() ? 0 : 1;
        } catch (Fallback& f) {
          rs->pnodes.resize(mark_p); rs->pentries.resize(mark_e); rs->leaves.resize(mark_l);
          rs->atoms.resize(mark_a); rs->templates.resize(mark_t);
          // interned templates created by the abandoned rule are gone: drop their ids so that a later rule with the
          // same path string interns it again instead of receiving an id past the end of `templates`
          for (auto it = rs->template_ids.begin(); it != rs->template_ids.end();)
            it = it->second >= mark_t ? rs->template_ids.erase(it) : std::next(it);
          rs->cnodes.resize(mark_cn); rs->conds.resize(mark_cd); rs->cond_text.resize(mark_cd); rs->cprogs.resize(mark_cp);
          (void)mark_pool;
          rd.kind = RK_FALLBACK;
          rd.pre = NONE;
          rd.exc = NONE;
          rm.exc_keys.clear();
          rm.reason = f.why;
          rm.msg_parts.clear();
        }
        rm.kind = rd.kind;
        rs->rules.push_back(rd);
        rs->meta.push_back(rm);
      }
      pm.nrules = (uint32_t)rs->rules.size() - pm.first_rule;
      rs->policies.push_back(pm);
    }
    build_path_trie(*rs);
    mark_gate_exact(*rs);
    assign_glob_masks(*rs);
    return rs.release();
  } catch (std::exception& e) {
    if (err) *err = e.what();
    return nullptr;
  }
}

// ---------------------------------------------------------------- path trie (kyv_layout.h "Path columns")
namespace {
struct TrieBuilder {
  Ruleset& rs;
  std::vector<uint32_t> pn_trie;  // trie node a pnode was compiled against (CONFLICT: reached from two paths)
  static constexpr uint32_t UNSET = NONE, CONFLICT = NONE - 1;
  uint32_t child(uint32_t t, uint32_t key) {
    for (auto& kv : rs.trie[t].kids) if (kv.first == key) return kv.second;
    uint32_t id = (uint32_t)rs.trie.size();
    uint32_t space = rs.trie[t].rowspace;
    rs.trie.emplace_back();
    rs.trie[id].rowspace = space;
    rs.trie[id].col = rs.ncols++;
    rs.col_rowspace.push_back(space);
    rs.trie[t].kids.push_back({key, id});
    return id;
  }
  uint32_t star(uint32_t t) {
    if (rs.trie[t].star != NONE) return rs.trie[t].star;
    uint32_t id = (uint32_t)rs.trie.size();
    rs.trie.emplace_back();
    rs.trie[id].rowspace = rs.nrowspaces++;
    rs.trie[id].col = rs.ncols++;  // self column of the elements
    rs.col_rowspace.push_back(rs.trie[id].rowspace);
    rs.trie[t].star = id;
    rs.trie[t].lencol = rs.ncols++;  // (count, element-0 row) of the arrays at t
    rs.col_rowspace.push_back(rs.trie[t].rowspace);
    return id;
  }
  // t == NONE: the pattern position has no static path (below a wildcard key): lookups binary-search
  void walk(uint32_t pn, uint32_t t, int guard) {
    if (pn == NONE || pn >= rs.pnodes.size() || guard > 4 * MAX_DEPTH) return;
    if (pn_trie[pn] == UNSET) pn_trie[pn] = t;
    else if (pn_trie[pn] != t) pn_trie[pn] = CONFLICT;
    if (pn_trie[pn] == CONFLICT) t = NONE;
    const PNode P = rs.pnodes[pn];
    switch (P.kind) {
      case P_MAP:
        for (uint32_t e = 0; e < P.n; e++) {
          uint32_t ct = (t == NONE || (rs.pentries[P.first + e].flags & EF_WILD)) ? NONE : child(t, rs.pentries[P.first + e].key);
          PEntry& E = rs.pentries[P.first + e];
          E.col = ct == NONE ? NONE : rs.trie[ct].col;
          if (E.col == NONE) rs.pnodes[pn].flags |= PF_NEEDROW;
          if (E.handler == H_STAR || E.handler == H_NEGATION || E.handler == H_EXIST_BADPAT || E.child == NONE) continue;
          if (E.handler == H_EXISTENCE) {
            uint32_t st = ct == NONE ? NONE : star(ct);
            rs.pe_self[P.first + e] = st == NONE ? NONE : rs.trie[st].col;
            rs.pe_len[P.first + e] = st == NONE ? NONE : rs.trie[ct].lencol;
            uint32_t npat = rs.pool[E.child];
            for (uint32_t j = 0; j < npat; j++) walk(rs.pool[E.child + 1 + j], st, guard + 1);
          } else {
            walk(E.child, ct, guard + 1);
          }
        }
        break;
      case P_ARR_MAPS: {
        uint32_t st = t == NONE ? NONE : star(t);
        rs.pn_self[pn] = st == NONE ? NONE : rs.trie[st].col;
        rs.pn_len[pn] = st == NONE ? NONE : rs.trie[t].lencol;
        walk(P.first, st, guard + 1);
        break;
      }
      case P_ARR_SCALAR: {  // element values through the self column
        uint32_t st = t == NONE ? NONE : star(t);
        rs.pn_self[pn] = st == NONE ? NONE : rs.trie[st].col;
        rs.pn_len[pn] = st == NONE ? NONE : rs.trie[t].lencol;
        break;
      }
      case P_ARR_POS: {
        uint32_t st = t == NONE ? NONE : star(t);
        rs.pn_self[pn] = st == NONE ? NONE : rs.trie[st].col;
        rs.pn_len[pn] = st == NONE ? NONE : rs.trie[t].lencol;
        for (uint32_t i = 0; i < P.n; i++) walk(rs.pool[P.first + i], st, guard + 1);
        break;
      }
      default: break;
    }
  }

  // JMESPath-subset condition operands (kyv_layout.h OK_JMES) compiled by jit.cpp's CondGen read their static
  // field / flatten steps from path columns: register those paths. Returns the trie positions the operand's
  // result (or its list's elements) can have and whether the result is a list; NONE = no static position.
  // The transitions are the ones CondGen::jgen / fgen take (a flatten inside a projection keeps non-array
  // elements in place, which have no static position).
  struct Pos { std::vector<uint32_t> t; bool list = false; };
  uint32_t ch(uint32_t t, uint32_t key) { return t == NONE ? NONE : child(t, key); }
  uint32_t st(uint32_t t) { return t == NONE ? NONE : star(t); }
  Pos jmes(const CondOperand& o, const std::vector<uint32_t>& elem) {
    Pos r;
    r.t.push_back(NONE);
    if (o.kind != OK_JMES) return r;
    const uint32_t* p = rs.pool.data() + o.a;
    const uint32_t root = p[0] & 0xFFu;
    if ((p[0] & JF_PURE) || root == JR_OPERATION) return r;
    std::vector<uint32_t> S = root == JR_OBJECT ? std::vector<uint32_t>{0u} : elem;
    if (S.empty()) S.push_back(NONE);
    bool list = false;
    auto uniq = [](std::vector<uint32_t> v) {
      std::sort(v.begin(), v.end());
      v.erase(std::unique(v.begin(), v.end()), v.end());
      return v;
    };
    for (uint32_t q = 1; q < o.nseg;) {
      const uint32_t op = p[q];
      std::vector<uint32_t> N;
      if (op == JO_FIELD) {
        for (uint32_t t : S) N.push_back(ch(t, p[q + 1]));
        q += 2;
      } else if (op == JO_MULTI) {
        const uint32_t m = p[q + 1];
        for (uint32_t t : S) for (uint32_t j = 0; j < m; j++) N.push_back(ch(t, p[q + 2 + j]));
        list = true;
        q += 2 + m;
      } else if (op == JO_FLAT) {
        for (uint32_t t : S) N.push_back(st(t));
        if (list) N.push_back(NONE);
        list = true;
        q++;
      } else if (op == JO_KEYS || op == JO_KEYS_FLAT) {
        N.push_back(NONE);
        list = list || op == JO_KEYS;
        q++;
      } else if (op == JO_FILTER) {  // the kept elements: array elements (compiled kernels do not generate filters)
        for (uint32_t t : S) N.push_back(st(t));
        list = true;
        q += jop_width(p + q);
      } else if (op == JO_LENGTH) {  // a number: no trie position
        S = {NONE};
        list = false;
        break;
      } else {
        break;  // JO_OR ends the program
      }
      S = uniq(N);
    }
    r.t = S;
    r.list = list;
    return r;
  }
  // a plain `{{ request.object.<path> }}` operand: its whole path is one column (cv_operand reads it first)
  void path(CondOperand& o) {
    if (o.kind != OK_PATH) return;
    uint32_t t = 0;
    for (uint32_t s = 0; s < o.nseg && t != NONE; s++) t = ch(t, rs.pool[o.a + s]);
    o.list = (t == NONE || o.nseg == 0) ? 0u : rs.trie[t].col + 1;
  }
  // a chain-form JMESPath operand (kyv_layout.h jmes_chain_form: fields, then `|| lit` and / or one function) whose
  // fields jmes() registered: the column of the field chain (o.list = column + 1), which the light kernels' chain
  // evaluator reads instead of searching the maps field by field (kyv_cond.h jmes_chain_cv)
  void chain(CondOperand& o) {
    if (o.kind != OK_JMES || o.sv || !jmes_chain_form(rs.pool.data() + o.a, o.nseg)) return;
    const uint32_t* p = rs.pool.data() + o.a;
    if (p[0] & JF_PURE) return;  // (pure programs are not registered: jmes())
    uint32_t t = 0, nf = 0;
    for (uint32_t q = 1; q + 1 < o.nseg && p[q] == JO_FIELD && t != NONE; q += 2, nf++) t = ch(t, p[q + 1]);
    o.list = (t == NONE || nf == 0) ? 0u : rs.trie[t].col + 1;
  }
  void prog(uint32_t pr, const std::vector<uint32_t>& elem) {
    if (pr == NONE || pr >= rs.cprogs.size()) return;
    const CondProg& P = rs.cprogs[pr];
    const uint32_t nany = P.nany == NONE ? 0u : P.nany;
    auto one = [&](Cond& c) { jmes(c.key, elem); jmes(c.value, elem); path(c.key); path(c.value); chain(c.key); chain(c.value); };
    for (uint32_t i = 0; i < nany; i++) one(rs.conds[P.any0 + i]);
    for (uint32_t i = 0; i < P.nall; i++) one(rs.conds[P.all0 + i]);
  }
  // PodSecurity rules (kyv_pss.h pss_checks_cols): the fields the checks read, at the pod positions getSpec
  // (validation.go:481-532) takes for the rule's kinds, as path columns; the table goes to the rule's PssDesc
  void pss_rule(const RuleDesc& rd) {
    if (rd.kind != RK_PSS || rd.root >= rs.pss.size()) return;
    bool pos[PSS_NPOS] = {false, false, false};
    bool any = rd.match.mode == MM_NONE || rd.match.nfilters == 0;
    for (uint32_t i = 0; i < rd.match.nfilters && !any; i++) {
      const Filter& f = rs.filters[rd.match.filters + i];
      if (f.nkinds == 0) any = true;
      for (uint32_t j = 0; j < f.nkinds; j++) {
        const uint32_t k = rs.kinds[f.kinds + j].kind;
        if (k == NONE) any = true;
        else if (k == KSID(POD)) pos[0] = true;
        else if (k == KSID(DAEMONSET) || k == KSID(DEPLOYMENT) || k == KSID(JOB) || k == KSID(STATEFULSET) ||
                 k == KSID(REPLICASET) || k == KSID(RC)) pos[1] = true;
        else if (k == KSID(CRONJOB)) pos[2] = true;
      }
    }
    if (any) pos[0] = pos[1] = pos[2] = true;
    std::vector<uint32_t> tab(PSS_NPOS * PC_COUNT, NONE);
    auto col = [&](uint32_t t) { return rs.trie[t].col; };
    for (uint32_t p = 0; p < PSS_NPOS; p++) {
      if (!pos[p]) continue;
      uint32_t* T = tab.data() + p * PC_COUNT;
      uint32_t t = 0;
      if (p == 1) t = child(child(t, KSID(SPEC)), KSID(TEMPLATE));
      if (p == 2) t = child(child(child(child(t, KSID(SPEC)), KSID(JOBTEMPLATE)), KSID(SPEC)), KSID(TEMPLATE));
      const uint32_t meta = child(t, KSID(METADATA)), spec = child(t, KSID(SPEC));
      T[PC_ANN] = col(child(meta, KSID(ANNOTATIONS)));
      const uint32_t psc = child(spec, KSID(SECCTX));
      T[PC_PSC] = col(psc);
      T[PC_PSC_NONROOT] = col(child(psc, KSID(RUNASNONROOT)));
      T[PC_PSC_USER] = col(child(psc, KSID(RUNASUSER)));
      const uint32_t sel = child(psc, KSID(SELINUX));
      T[PC_PSC_SEL] = col(sel);
      T[PC_PSC_SEL_USER] = col(child(sel, KSID(USER)));
      T[PC_PSC_SEL_ROLE] = col(child(sel, KSID(ROLE)));
      T[PC_PSC_SEL_TYPE] = col(child(sel, KSID(TYPE)));
      const uint32_t sec = child(psc, KSID(SECCOMP));
      T[PC_PSC_SEC] = col(sec);
      T[PC_PSC_SEC_TYPE] = col(child(sec, KSID(TYPE)));
      const uint32_t win = child(psc, KSID(WINOPTS));
      T[PC_PSC_WIN] = col(win);
      T[PC_PSC_WIN_HP] = col(child(win, KSID(HOSTPROCESS)));
      T[PC_PSC_SYSCTLS] = col(child(psc, KSID(SYSCTLS)));
      T[PC_OS_NAME] = col(child(child(spec, KSID(OS)), KSID(NAME)));
      T[PC_HOSTNET] = col(child(spec, KSID(HOSTNETWORK)));
      T[PC_HOSTPID] = col(child(spec, KSID(HOSTPID)));
      T[PC_HOSTIPC] = col(child(spec, KSID(HOSTIPC)));
      T[PC_VOLUMES] = col(child(spec, KSID(VOLUMES)));
      const uint32_t lkeys[PSS_NLISTS] = {KSID(INITCONTAINERS), KSID(CONTAINERS), KSID(EPHEMERALCONTAINERS)};
      for (uint32_t l = 0; l < PSS_NLISTS; l++) {
        uint32_t* L = T + PC_LISTS + l * PCL_COUNT;
        const uint32_t lt = child(spec, lkeys[l]), el = star(lt);
        L[PCL_LEN] = rs.trie[lt].lencol;
        L[PCL_SELF] = col(el);
        L[PCL_NAME] = col(child(el, KSID(NAME)));
        const uint32_t sc = child(el, KSID(SECCTX));
        L[PCL_SC] = col(sc);
        L[PCL_PRIV] = col(child(sc, KSID(PRIVILEGED)));
        L[PCL_APE] = col(child(sc, KSID(APE)));
        L[PCL_NONROOT] = col(child(sc, KSID(RUNASNONROOT)));
        L[PCL_USER] = col(child(sc, KSID(RUNASUSER)));
        const uint32_t csel = child(sc, KSID(SELINUX));
        L[PCL_SEL] = col(csel);
        L[PCL_SEL_USER] = col(child(csel, KSID(USER)));
        L[PCL_SEL_ROLE] = col(child(csel, KSID(ROLE)));
        L[PCL_SEL_TYPE] = col(child(csel, KSID(TYPE)));
        const uint32_t csec = child(sc, KSID(SECCOMP));
        L[PCL_SEC] = col(csec);
        L[PCL_SEC_TYPE] = col(child(csec, KSID(TYPE)));
        const uint32_t cwin = child(sc, KSID(WINOPTS));
        L[PCL_WIN] = col(cwin);
        L[PCL_WIN_HP] = col(child(cwin, KSID(HOSTPROCESS)));
        const uint32_t caps = child(sc, KSID(CAPS));
        L[PCL_CAPS] = col(caps);
        const uint32_t add = child(caps, KSID(ADD)), adds = star(add);
        L[PCL_ADD_LEN] = rs.trie[add].lencol;
        L[PCL_ADD_SELF] = col(adds);
        const uint32_t drop = child(caps, KSID(DROP)), drops = star(drop);
        L[PCL_DROP_LEN] = rs.trie[drop].lencol;
        L[PCL_DROP_SELF] = col(drops);
        L[PCL_PROC] = col(child(sc, KSID(PROCMOUNT)));
        const uint32_t ports = child(el, KSID(PORTS)), ps = star(ports);
        L[PCL_PORTS_LEN] = rs.trie[ports].lencol;
        L[PCL_PORT_HOSTPORT] = col(child(ps, KSID(HOSTPORT)));
      }
    }
    PssDesc& pd = rs.pss[rd.root];
    if (pd.cols == NONE) {
      pd.cols = (uint32_t)rs.pool.size();
      rs.pool.insert(rs.pool.end(), tab.begin(), tab.end());
    } else {
      std::copy(tab.begin(), tab.end(), rs.pool.begin() + pd.cols);
    }
  }
  void cond_rule(const RuleDesc& rd) {
    prog(rd.pre, {});
    if (rd.kind == RK_DENY) prog(rd.root, {});
    if (rd.kind != RK_FOREACH) return;
    const uint32_t nent = rs.pool[rd.root];
    for (uint32_t e = 0; e < nent; e++) {
      ForeachEntry fe;
      memcpy(&fe, rs.pool.data() + rd.root + 1 + e * (sizeof(ForeachEntry) / 4), sizeof fe);
      Pos lp = jmes(fe.list, {});
      std::vector<uint32_t> E;
      if (lp.list) E = lp.t;
      else for (uint32_t t : lp.t) E.push_back(st(t));  // a single array's items
      prog(fe.pre, E);
      prog(fe.deny, E);
    }
  }
};
}  // namespace

// RD_GATE_EXACT: the rule's match block is decided by the resource kind alone (every filter is a plain kinds
// list without group/version, no exclude, no empty-OldResource retry), so the batch's per-kind-class rule gate
// (batch.cpp rule_gate) equals MatchesResourceDescription (pkg/engine/utils.go:185-256) for it.
void mark_gate_exact(Ruleset& rs) {
  for (auto& rd : rs.rules) {
    rd.flags &= (uint8_t)~RD_GATE_EXACT;
    if (rd.empty_may_match || rd.exclude.mode != MM_NONE || rd.pre != NONE || rd.exc != NONE) continue;
    const MatchBlock& m = rd.match;
    if (m.mode == MM_NONE || m.nfilters == 0) continue;
    if (m.mode != MM_ANY && m.nfilters != 1) continue;
    bool ok = true;
    for (uint32_t i = 0; i < m.nfilters && ok; i++) {
      const Filter& f = rs.filters[m.filters + i];
      if (f.nkinds == 0 || f.name != NONE || f.nnames || f.nnss || f.nann ||
          (f.flags & (FF_HAS_SEL | FF_HAS_NSSEL | FF_ZERO_RD)))
        ok = false;
      for (uint32_t j = 0; j < f.nkinds && ok; j++) {
        const KindDesc& k = rs.kinds[f.kinds + j];
        if (k.kind != NONE && k.gv_mode != 0) ok = false;
      }
    }
    if (ok) rd.flags |= RD_GATE_EXACT;
  }
}

// Glob masks (kyv_layout.h SF_GIDX_SHIFT): the ruleset's wildcard patterns that would otherwise run a byte loop
// per test -- pattern atoms (prefix / suffix / contains / general), metadata-expansion key globs, then every other
// wildcard literal (match-program names / namespaces / annotations, condition values) -- up to MAX_GMASK of them
void assign_glob_masks(Ruleset& rs) {
  rs.gpats.clear();
  std::vector<uint32_t> idx(rs.dict.strs.size(), 0);
  auto add = [&](uint32_t sid) -> uint8_t {
    if (sid == NONE || sid >= idx.size()) return 0;
    if (!idx[sid]) {
      if (rs.gpats.size() >= MAX_GMASK) return 0;
      rs.gpats.push_back(sid);
      idx[sid] = (uint32_t)rs.gpats.size();
    }
    return (uint8_t)idx[sid];
  };
  for (auto& a : rs.atoms) {
    a.gidx = 0;
    if (a.glob == G_PREFIX || a.glob == G_SUFFIX || a.glob == G_CONTAINS || a.glob == G_GENERAL) a.gidx = add(a.pat);
  }
  for (auto& m : rs.metas) {
    for (uint32_t i = 0; i < m.nwild_l; i++) add(rs.pool[m.wild_l + 2 * i]);
    for (uint32_t i = 0; i < m.nwild_a; i++) add(rs.pool[m.wild_a + 2 * i]);
  }
  for (uint32_t s = 0; s < rs.dict.strs.size(); s++) {
    const std::string& x = rs.dict.strs[s];
    bool globby = x.find_first_of("*?") != std::string::npos;
    for (unsigned char ch : x) if (ch >= 0x80) globby = true;
    if (globby) add(s);
  }
  assign_cond_sets(rs);
}

// Condition-set masks: an AnyIn / AllIn / AnyNotIn / AllNotIn (or In / NotIn with a scalar key) condition with one
// literal side and one JMESPath side asks, per element of the resource-side list, "does wild2(element, e) hold for
// some literal element e" (op_any_all / key_exists, kyv_cond.h; anyin.go:115-180, in.go:52-86). That predicate depends
// on the element's string only, so the device evaluates it once per dictionary string (gmask_kernel, mask bit
// gpats.size() + set index) and the compiled condition kernel streams the list with one mask load per element
// instead of materialising it (jit.cpp CondGen). Only sets whose literal elements all have a fmt.Sprint form are
// used (a literal the device cannot render makes the operator fall back, which the set cannot express).
static uint32_t lit_sprint(const Ruleset& rs, const Node& n) {
  switch (node_type(n)) {
    case N_NULL: return KSID(NIL_STR);
    case N_FALSE: return SID_FALSE;
    case N_TRUE: return SID_TRUE;
    case N_INT: case N_FLOAT: return n.c;
    case N_STR: return n.a;
    default: return NONE;
  }
}
void assign_cond_sets(Ruleset& rs) {
  rs.gsets.clear();
  rs.cond_set.assign(rs.conds.size(), 0);
  std::map<std::vector<uint32_t>, uint32_t> seen;
  for (size_t ci = 0; ci < rs.conds.size(); ci++) {
    const Cond& c = rs.conds[ci];
    const bool anyall = c.op == CO_ANYIN || c.op == CO_ALLIN || c.op == CO_ANYNOTIN || c.op == CO_ALLNOTIN;
    const bool in = c.op == CO_IN || c.op == CO_NOTIN;
    std::vector<uint32_t> set;
    if (anyall && c.key.kind == OK_JMES && c.value.kind == OK_LIT && node_type(rs.cnodes[c.value.a]) == N_ARR) {
      // shape A: resource-side key list, literal value list
      const Node& a = rs.cnodes[c.value.a];
      bool ok = true;
      for (uint32_t j = 0; j < a.b && ok; j++) {
        const uint32_t s = lit_sprint(rs, rs.cnodes[a.a + j]);
        if (s == NONE) ok = false; else set.push_back(s);
      }
      if (!ok) continue;
    } else if ((anyall || in) && c.key.kind == OK_LIT && c.value.kind == OK_JMES) {
      // shape B: literal scalar key, resource-side value list
      const Node& k = rs.cnodes[c.key.a];
      if (node_type(k) != N_STR && node_type(k) != N_INT && node_type(k) != N_FLOAT) continue;
      const uint32_t s = lit_sprint(rs, k);
      if (s == NONE) continue;
      set.push_back(s);
    } else {
      continue;
    }
    std::sort(set.begin(), set.end());
    set.erase(std::unique(set.begin(), set.end()), set.end());
    auto it = seen.find(set);
    if (it == seen.end()) {
      if (rs.gpats.size() + rs.gsets.size() >= MAX_GMASK) continue;
      it = seen.emplace(set, (uint32_t)rs.gsets.size()).first;
      rs.gsets.push_back(set);
    }
    rs.cond_set[ci] = it->second + 1;
  }
}

void build_path_trie(Ruleset& rs) {
  rs.trie.assign(1, Ruleset::TrieNode{});
  rs.ncols = 0;
  rs.nrowspaces = 1;
  rs.col_rowspace.clear();
  for (auto& E : rs.pentries) E.col = NONE;
  for (auto& P : rs.pnodes) P.flags &= (uint8_t)~PF_NEEDROW;
  rs.pn_self.assign(rs.pnodes.size(), NONE);
  rs.pe_self.assign(rs.pentries.size(), NONE);
  rs.pn_len.assign(rs.pnodes.size(), NONE);
  rs.pe_len.assign(rs.pentries.size(), NONE);
  TrieBuilder tb{rs, std::vector<uint32_t>(rs.pnodes.size(), TrieBuilder::UNSET)};
  for (auto& rd : rs.rules) {
    if (rd.kind == RK_PATTERN) tb.walk(rd.root, 0, 0);
    else if (rd.kind == RK_ANYPATTERN)
      for (uint32_t a = 0; a < rd.nalts; a++) tb.walk(rs.pool[rd.root + a], 0, 0);
  }
  for (auto& rd : rs.rules) tb.cond_rule(rd);
  if (!getenv("KYV_PSS_NOCOLS"))
    for (auto& rd : rs.rules) tb.pss_rule(rd);
  // entries of pnodes that conflicted after their first visit assigned columns: clear the whole subtree
  // (a conflicting subtree is walked with t == NONE, which already cleared its entries' columns)
}

}  // namespace kyv
