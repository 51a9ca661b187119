// ORACLE — test infrastructure only (see ojson.h header).
//
// CPU restatement of the reference pattern walk. Each function names the reference function it
// follows (paths relative to /root/reference):
//   pkg/engine/validate/validate.go, pkg/engine/validate/utils.go
//   pkg/engine/anchor/{anchor.go,handlers.go,anchormap.go,error.go,utils.go}
//   pkg/engine/pattern/pattern.go, pkg/engine/operator/operator.go
//   pkg/engine/wildcards/wildcards.go
#include "ovalidate.h"

#include <algorithm>
#include <list>
#include <set>

#include "goutil.h"

namespace orc {
using oj::T;
using oj::VP;
using oj::Value;

static bool isnil(const VP& v) { return !v || v->t == T::Null; }

// Go %T of a decoded value
static std::string go_T(const VP& v) {
  if (isnil(v)) return "<nil>";
  switch (v->t) {
    case T::Bool: return "bool";
    case T::Int: return "int64";
    case T::Float: return "float64";
    case T::Str: return "string";
    case T::Arr: return "[]interface {}";
    case T::Obj: return "map[string]interface {}";
    default: return "<nil>";
  }
}

// ---------------- anchor (pkg/engine/anchor/anchor.go) ----------------
enum class AT { None, Condition, Global, Negation, AddIfNotPresent, Equality, Existence };
struct Anchor {
  AT t = AT::None;
  std::string key;
};

// anchor.Parse: regex ^(?P<modifier>[+<=X^])?\((?P<key>.+)\)$ after strings.TrimSpace (anchor.go:19,37-44)
static Anchor parse_anchor(const std::string& raw) {
  Anchor a;
  std::string s = gou::trim_space(raw);
  if (s.size() < 3) return a;
  size_t p = 0;
  AT t = AT::Condition;
  switch (s[0]) {
    case '+': t = AT::AddIfNotPresent; p = 1; break;
    case '<': t = AT::Global; p = 1; break;
    case '=': t = AT::Equality; p = 1; break;
    case 'X': t = AT::Negation; p = 1; break;
    case '^': t = AT::Existence; p = 1; break;
    default: break;
  }
  if (p >= s.size() || s[p] != '(' || s.back() != ')') return a;
  std::string key = s.substr(p + 1, s.size() - p - 2);
  if (key.empty()) return a;
  if (key.find('\n') != std::string::npos) return a;  // '.' does not match newline
  a.t = t;
  a.key = key;
  return a;
}

static std::string anchor_string(AT t, const std::string& key) {
  if (key.empty()) return "";
  std::string m;
  switch (t) {
    case AT::Global: m = "<"; break;
    case AT::Negation: m = "X"; break;
    case AT::AddIfNotPresent: m = "+"; break;
    case AT::Equality: m = "="; break;
    case AT::Existence: m = "^"; break;
    default: break;
  }
  return m + "(" + key + ")";
}

// ---------------- anchor errors (anchor/error.go) ----------------
static const char* kNegMsg = "negation anchor matched in resource";
static const char* kCondMsg = "conditional anchor mismatch";
static const char* kGlobMsg = "global anchor mismatch";

static bool is_error(const Err& e, int code, const char* msg) {
  if (!e.present) return false;
  if (e.code >= 0) return e.code == code;
  return e.msg.find(msg) != std::string::npos;
}
bool is_conditional_err(const Err& e) { return is_error(e, 0, kCondMsg); }
bool is_global_err(const Err& e) { return is_error(e, 1, kGlobMsg); }
bool is_negation_err(const Err& e) { return is_error(e, 2, kNegMsg); }

// ---------------- AnchorMap (anchor/anchormap.go) ----------------
struct AnchorMap {
  std::map<std::string, bool> m;
  bool keys_are_missing() const {
    for (auto& kv : m) if (!kv.second) return true;
    return false;
  }
  // resourceHasValueForKey (anchor/utils.go:43-60)
  static bool has_value_for_key(const VP& res, const std::string& key) {
    if (!res) return false;
    if (res->t == T::Obj) return res->o.count(key) > 0;
    if (res->t == T::Arr) {
      for (auto& e : res->a) if (has_value_for_key(e, key)) return true;
    }
    return false;
  }
  void check_anchor_in_resource(const VP& pattern, const VP& resource) {
    for (auto& kv : pattern->o) {
      Anchor a = parse_anchor(kv.first);
      if (a.t == AT::Condition || a.t == AT::Existence || a.t == AT::Negation) {
        auto it = m.find(kv.first);
        if (it == m.end()) m[kv.first] = false;
        else if (it->second) continue;
        if (has_value_for_key(resource, a.key)) m[kv.first] = true;
      }
    }
  }
};

// ---------------- operator (operator/operator.go) ----------------
enum class Op { Equal, MoreEqual, LessEqual, NotEqual, More, Less, InRange, NotInRange };

static size_t op_len(Op o) {
  switch (o) {
    case Op::MoreEqual: case Op::LessEqual: case Op::NotInRange: return 2;
    case Op::NotEqual: case Op::More: case Op::Less: case Op::InRange: return 1;
    default: return 0;
  }
}

// one side of the range regexes: [-|\+]?\d+(?:\.\d+)?[A-Za-z]*   (operator.go:30-31)
static bool range_side(const std::string& s, size_t& i) {
  size_t st = i;
  if (i < s.size() && (s[i] == '-' || s[i] == '|' || s[i] == '+')) i++;
  size_t d0 = i;
  while (i < s.size() && s[i] >= '0' && s[i] <= '9') i++;
  if (i == d0) { i = st; return false; }
  if (i + 1 < s.size() && s[i] == '.' && s[i + 1] >= '0' && s[i + 1] <= '9') {
    i++;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') i++;
  }
  while (i < s.size() && ((s[i] >= 'A' && s[i] <= 'Z') || (s[i] >= 'a' && s[i] <= 'z'))) i++;
  return true;
}

static bool range_match(const std::string& s, const std::string& sep, std::string* l, std::string* r) {
  size_t i = 0;
  if (!range_side(s, i)) return false;
  size_t le = i;
  if (s.compare(i, sep.size(), sep) != 0) return false;
  i += sep.size();
  size_t rs = i;
  if (!range_side(s, i)) return false;
  if (i != s.size()) return false;
  if (l) *l = s.substr(0, le);
  if (r) *r = s.substr(rs);
  return true;
}

static Op get_operator(const std::string& p) {
  if (p.size() < 2) return Op::Equal;
  if (p.compare(0, 2, ">=") == 0) return Op::MoreEqual;
  if (p.compare(0, 2, "<=") == 0) return Op::LessEqual;
  if (p[0] == '>') return Op::More;
  if (p[0] == '<') return Op::Less;
  if (p[0] == '!') return Op::NotEqual;
  if (range_match(p, "!-", nullptr, nullptr)) return Op::NotInRange;
  if (range_match(p, "-", nullptr, nullptr)) return Op::InRange;
  return Op::Equal;
}

// ---------------- pattern (pattern/pattern.go) ----------------
static int64_t go_f2i(double p) {
  if (!(p > -9.223372036854775808e18 && p < 9.223372036854775807e18)) return INT64_MIN;
  return (int64_t)p;
}

static bool validate_float_pattern(const VP& v, double p) {  // pattern.go:87-116
  if (isnil(v)) return false;
  switch (v->t) {
    case T::Int: if (p != std::trunc(p)) return false; return go_f2i(p) == v->i;
    case T::Float: return v->f == p;
    case T::Str: { double d; if (!gou::parse_float(v->s, d)) return false; return d == p; }
    default: return false;
  }
}

static bool validate_nil_pattern(const VP& v) {  // pattern.go:118-139
  if (isnil(v)) return true;
  switch (v->t) {
    case T::Float: return v->f == 0.0;
    case T::Int: return v->i == 0;
    case T::Str: return v->s.empty();
    case T::Bool: return !v->b;
    default: return false;
  }
}

// convertNumberToString (pattern.go:303-321)
static bool convert_number_to_string(const VP& v, std::string& out) {
  if (isnil(v)) { out = "0"; return true; }
  switch (v->t) {
    case T::Str: out = v->s; return true;
    case T::Float: out = gou::format_float_f6(v->f); return true;
    case T::Int: out = std::to_string(v->i); return true;
    default: return false;
  }
}

template <class X>
static bool cmp_op(Op op, X c) {  // c = cmp(value, pattern)
  switch (op) {
    case Op::Equal: return c == 0;
    case Op::NotEqual: return c != 0;
    case Op::More: return c > 0;
    case Op::Less: return c < 0;
    case Op::MoreEqual: return c >= 0;
    case Op::LessEqual: return c <= 0;
    default: return false;
  }
}

static bool compare_duration(const VP& v, const std::string& p, Op op) {  // pattern.go:213-237
  int64_t pd, vd;
  std::string vs;
  if (!gou::parse_duration(p, pd)) return false;
  if (!convert_number_to_string(v, vs)) return false;
  if (!gou::parse_duration(vs, vd)) return false;
  int c = vd < pd ? -1 : (vd > pd ? 1 : 0);
  return cmp_op(op, c);
}

static bool compare_quantity(const VP& v, const std::string& p, Op op) {  // pattern.go:239-264
  gou::Quantity pq, vq;
  std::string vs;
  if (!gou::parse_quantity(p, pq)) return false;
  if (!convert_number_to_string(v, vs)) return false;
  if (!gou::parse_quantity(vs, vq)) return false;
  return cmp_op(op, gou::quantity_cmp(vq, pq));
}

static bool compare_string(const VP& v, const std::string& p, Op op) {  // pattern.go:266-301
  if (op != Op::Equal && op != Op::NotEqual) return false;
  std::string sv;
  if (isnil(v)) return false;
  switch (v->t) {
    case T::Float: sv = gou::format_float_E(v->f); break;
    case T::Int: sv = std::to_string(v->i); break;
    case T::Str: sv = v->s; break;
    case T::Bool: sv = v->b ? "true" : "false"; break;
    default: return false;
  }
  bool r = gou::wildcard_match(p, sv);
  return op == Op::NotEqual ? !r : r;
}

static bool validate_string_pattern(const VP& v, const std::string& pattern);

static bool validate_string(const VP& v, const std::string& p, Op op) {  // pattern.go:207-211
  return compare_duration(v, p, op) || compare_quantity(v, p, op) || compare_string(v, p, op);
}

static bool validate_string_pattern(const VP& v, const std::string& pattern) {  // pattern.go:175-197
  Op op = get_operator(pattern);
  if (op == Op::InRange) {
    std::string l, r;
    if (range_match(pattern, "-", &l, &r))
      return validate_string_pattern(v, ">= " + l) && validate_string_pattern(v, "<= " + r);
    return false;
  }
  if (op == Op::NotInRange) {
    std::string l, r;
    if (range_match(pattern, "!-", &l, &r))
      return validate_string_pattern(v, "< " + l) || validate_string_pattern(v, "> " + r);
    return false;
  }
  std::string p = gou::trim_space(pattern.substr(op_len(op)));
  return validate_string(v, p, op);
}

static bool validate_string_patterns(const VP& v, const std::string& pattern) {  // pattern.go:152-173
  if (v && v->t == T::Str && v->s == pattern) return true;
  for (auto& cond0 : gou::split(pattern, '|')) {
    std::string cond = gou::trim_spaces(cond0);
    bool all = true;
    for (auto& c0 : gou::split(cond, '&')) {
      if (!validate_string_pattern(v, gou::trim_spaces(c0))) { all = false; break; }
    }
    if (all) return true;
  }
  return false;
}

bool pattern_validate(const VP& value, const VP& pattern) {  // pattern.go:26-49
  if (isnil(pattern)) return validate_nil_pattern(value);
  switch (pattern->t) {
    case T::Bool: return value && value->t == T::Bool && value->b == pattern->b;
    case T::Int: {  // validateIntPattern (unreachable for JSON-decoded patterns)
      if (isnil(value)) return false;
      if (value->t == T::Int) return value->i == pattern->i;
      if (value->t == T::Float) return value->f == std::trunc(value->f) && go_f2i(value->f) == pattern->i;
      if (value->t == T::Str) { int64_t x; return gou::parse_int64(value->s, x) && x == pattern->i; }
      return false;
    }
    case T::Float: return validate_float_pattern(value, pattern->f);
    case T::Obj: return value && value->t == T::Obj;
    case T::Str: return validate_string_patterns(value, pattern->s);
    default: return false;
  }
}

// ---------------- wildcards (wildcards/wildcards.go) ----------------
struct Ctx {
  EvalFlags* fl;
  AnchorMap ac;
};

// getPatternValue (wildcards.go:85-96): first key == tag or anchor with Key()==tag (Go map order)
static bool get_pattern_value(const std::string& tag, const VP& m, std::string& key, VP& val, EvalFlags* fl) {
  int found = 0;
  for (auto& kv : m->o) {
    Anchor a = parse_anchor(kv.first);
    if (kv.first == tag || (a.t != AT::None && a.key == tag)) {
      if (found == 0) { key = kv.first; val = kv.second; }
      found++;
    }
  }
  if (found > 1 && fl) fl->nondeterministic = true;
  return found > 0;
}

// getValueAsStringMap (wildcards.go:113-132); panics like the reference on type assertions
static bool get_value_as_string_map(const std::string& tag, const VP& data, std::string& pkey,
                                    std::map<std::string, std::string>& out, EvalFlags* fl) {
  if (isnil(data)) return false;
  if (data->t != T::Obj) throw RefPanic{"metadata is not a map"};
  VP val;
  if (!get_pattern_value(tag, data, pkey, val, fl)) return false;
  if (isnil(val)) return false;
  if (val->t != T::Obj) throw RefPanic{tag + " is not a map"};
  for (auto& kv : val->o) {
    if (!kv.second || kv.second->t != T::Str) throw RefPanic{tag + " value is not a string"};
    out[kv.first] = kv.second->s;
  }
  return true;
}

// expandWildcards (wildcards.go:33-49) with matchValue=false, replace=false
static std::string expand_key(const std::string& k, const std::map<std::string, std::string>& res, EvalFlags* fl) {
  std::string first;
  int n = 0;
  for (auto& kv : res) {
    if (gou::wildcard_match(k, kv.first)) {
      if (n == 0) first = kv.first;
      n++;
    }
  }
  if (n > 1 && fl) fl->nondeterministic = true;
  return n ? first : k;
}

// replaceWildcardsInMapKeys (wildcards.go:135-151)
static VP replace_wildcards_in_map_keys(const std::map<std::string, std::string>& pat,
                                        const std::map<std::string, std::string>& res, EvalFlags* fl) {
  auto out = Value::obj();
  std::set<std::string> produced;
  for (auto& kv : pat) {
    std::string nk;
    if (gou::contains_wildcard(kv.first)) {
      Anchor a = parse_anchor(kv.first);
      if (a.t != AT::None) nk = anchor_string(a.t, expand_key(a.key, res, fl));
      else nk = expand_key(kv.first, res, fl);
    } else {
      nk = kv.first;
    }
    if (produced.count(nk) && fl) fl->nondeterministic = true;  // collision: Go map order decides
    produced.insert(nk);
    out->o[nk] = Value::str(kv.second);
  }
  return out;
}

static void expand_in_metadata(const VP& patternMap, const VP& resourceMap, EvalFlags* fl) {  // wildcards.go:62-83
  std::string mkey;
  VP pmeta;
  if (!get_pattern_value("metadata", patternMap, mkey, pmeta, fl) || isnil(pmeta)) return;
  VP rmeta = resourceMap->get("metadata");
  if (isnil(rmeta)) return;
  if (pmeta->t != T::Obj) throw RefPanic{"pattern metadata is not a map"};
  for (const char* tag : {"labels", "annotations"}) {
    std::string pk, rk;
    std::map<std::string, std::string> pdata, rdata;
    if (!get_value_as_string_map(tag, pmeta, pk, pdata, fl)) continue;
    if (!get_value_as_string_map(tag, rmeta, rk, rdata, fl)) continue;
    pmeta->o[pk] = replace_wildcards_in_map_keys(pdata, rdata, fl);
  }
}

// ---------------- validate walk (validate/validate.go) ----------------
struct Ret {
  std::string path;
  Err err;
};

static Ret validate_element(Ctx& c, const VP& res, const VP& pat, const std::string& path);

static bool skip_err(const Err& e) { return is_conditional_err(e) || is_global_err(e); }

// hasNestedAnchors / getAnchorsFromMap (validate/utils.go:11-33,61-69)
static bool has_nested_anchors(const VP& p) {
  if (!p) return false;
  if (p->t == T::Obj) {
    for (auto& kv : p->o) {
      Anchor a = parse_anchor(kv.first);
      if (a.t == AT::Condition || a.t == AT::Existence || a.t == AT::Equality || a.t == AT::Negation || a.t == AT::Global)
        return true;
    }
    for (auto& kv : p->o) if (has_nested_anchors(kv.second)) return true;
    return false;
  }
  if (p->t == T::Arr) {
    for (auto& e : p->a) if (has_nested_anchors(e)) return true;
  }
  return false;
}

static Ret validate_existence_list(Ctx& c, const VP& list, const VP& pmap, const std::string& path) {  // handlers.go:262-275
  for (size_t i = 0; i < list->a.size(); i++) {
    std::string cp = path + std::to_string(i) + "/";
    Ret r = validate_element(c, list->a[i], pmap, cp);
    if (!r.err.present) return Ret();
  }
  return Ret{path, Err::make("existence anchor validation failed at path " + path)};
}

// CreateElementHandler(...).Handle (anchor/handlers.go:31-260)
static Ret handle(Ctx& c, const std::string& element, const VP& pattern, const std::string& path, const VP& resMap) {
  Anchor a = parse_anchor(element);
  switch (a.t) {
    case AT::Condition: {  // handlers.go:160-176
      std::string cp = path + a.key + "/";
      auto it = resMap->o.find(a.key);
      if (it != resMap->o.end()) {
        Ret r = validate_element(c, it->second, pattern, cp);
        if (r.err.present) return Ret{r.path, Err::make(std::string(kCondMsg) + ": " + r.err.msg, 0)};
        return Ret();
      }
      return Ret{cp, Err::make(std::string(kCondMsg) + ": conditional anchor key doesn't exist in the resource", 0)};
    }
    case AT::Global: {  // handlers.go:195-209
      std::string cp = path + a.key + "/";
      auto it = resMap->o.find(a.key);
      if (it != resMap->o.end()) {
        Ret r = validate_element(c, it->second, pattern, cp);
        if (r.err.present) return Ret{r.path, Err::make(std::string(kGlobMsg) + ": " + r.err.msg, 1)};
      }
      return Ret();
    }
    case AT::Existence: {  // handlers.go:228-260
      std::string cp = path + a.key + "/";
      auto it = resMap->o.find(a.key);
      if (it == resMap->o.end()) return Ret();
      const VP& value = it->second;
      if (value && value->t == T::Arr) {
        if (!pattern || pattern->t != T::Arr)
          return Ret{cp, Err::make("invalid pattern type " + go_T(pattern) + ": Pattern has to be of list to compare against resource")};
        Ret last;
        for (auto& pm : pattern->a) {
          if (!pm || pm->t != T::Obj)
            return Ret{cp, Err::make("invalid pattern type " + go_T(pattern) + ": Pattern has to be of type map to compare against items in resource")};
          last = validate_existence_list(c, value, pm, cp);
          if (last.err.present) return last;
        }
        return last;
      }
      return Ret{cp, Err::make("invalid resource type " + go_T(value) + ": Existence ^ () anchor can be used only on list/array type resource")};
    }
    case AT::Equality: {  // handlers.go:96-109
      std::string cp = path + a.key + "/";
      auto it = resMap->o.find(a.key);
      if (it != resMap->o.end()) {
        Ret r = validate_element(c, it->second, pattern, cp);
        if (r.err.present) return r;
      }
      return Ret();
    }
    case AT::Negation: {  // handlers.go:66-77
      std::string cp = path + a.key + "/";
      if (resMap->o.count(a.key)) return Ret{cp, Err::make(std::string(kNegMsg) + ": " + cp + " is not allowed", 2)};
      return Ret();
    }
    default: {  // defaultHandler handlers.go:128-141 (also AddIfNotPresent and non-anchors, raw element)
      std::string cp = path + element + "/";
      VP rv = resMap->get(element);
      bool star = pattern && pattern->t == T::Str && pattern->s == "*";
      if (star && !isnil(rv)) return Ret();
      if (star) return Ret{path, Err::make(path + "/" + element + " not found")};
      Ret r = validate_element(c, rv, pattern, cp);
      if (r.err.present) return r;
      return Ret();
    }
  }
}

// anchor.GetAnchorsResourcesFromMap (anchor/utils.go:9-20): condition / existence / equality / negation keys vs the rest
static void split_anchors(const VP& patMap, std::vector<std::string>* anchors, std::vector<std::string>* resources) {
  for (auto& kv : patMap->o) {
    Anchor a = parse_anchor(kv.first);
    if (a.t == AT::Condition || a.t == AT::Existence || a.t == AT::Equality || a.t == AT::Negation) anchors->push_back(kv.first);
    else resources->push_back(kv.first);
  }
}

static Ret validate_map(Ctx& c, const VP& resMap, const VP& patMap, const std::string& path) {  // validate.go:118-161
  expand_in_metadata(patMap, resMap, c.fl);
  std::vector<std::string> anchors, resources;
  split_anchors(patMap, &anchors, &resources);
  // std::map iteration is already sorted (sort.Strings)
  for (auto& k : anchors) {
    Ret r = handle(c, k, patMap->o[k], path, resMap);
    if (r.err.present) return r;
  }
  // getSortedNestedAnchorResource (validate/utils.go:36-58)
  std::list<std::string> order;
  for (auto& k : resources) {
    if (parse_anchor(k).t == AT::Global || has_nested_anchors(patMap->o[k])) order.push_front(k);
    else order.push_back(k);
  }
  for (auto& k : order) {
    Ret r = handle(c, k, patMap->o[k], path, resMap);
    if (r.err.present) return r;
  }
  return Ret();
}

static Err combine_skips(const std::vector<Err>& errs) {  // multierr.Combine(...) then PatternError (untyped)
  std::string m;
  for (size_t i = 0; i < errs.size(); i++) { if (i) m += "; "; m += errs[i].msg; }
  return Err::make(m, -1);
}

static Ret validate_array_of_maps(Ctx& c, const VP& resArr, const VP& patMap, const std::string& path) {  // validate.go:218-247
  int apply = 0;
  std::vector<Err> skips;
  for (size_t i = 0; i < resArr->a.size(); i++) {
    std::string cp = path + std::to_string(i) + "/";
    Ret r = validate_element(c, resArr->a[i], patMap, cp);
    if (r.err.present) {
      if (skip_err(r.err)) { skips.push_back(r.err); continue; }
      return r;
    }
    apply++;
  }
  if (apply == 0 && !skips.empty()) return Ret{path, combine_skips(skips)};
  return Ret();
}

static bool is_scalar(const VP& p) {
  return isnil(p) || p->t == T::Str || p->t == T::Float || p->t == T::Int || p->t == T::Bool;
}

static Ret validate_array(Ctx& c, const VP& resArr, const VP& patArr, const std::string& path) {  // validate.go:163-214
  if (patArr->a.empty()) return Ret{path, Err::make("pattern Array empty")};
  const VP& first = patArr->a[0];
  if (first && first->t == T::Obj) {
    Ret r = validate_array_of_maps(c, resArr, first, path);
    if (r.err.present) return r;
    return Ret();
  }
  if (is_scalar(first)) {
    Ret r = validate_element(c, resArr, first, path);
    if (r.err.present) return r;
    return Ret();
  }
  if (resArr->a.size() < patArr->a.size())
    return Ret{"", Err::make("validate Array failed, array length mismatch, resource Array len is " + std::to_string(resArr->a.size()) +
                             " and pattern Array len is " + std::to_string(patArr->a.size()))};
  int apply = 0;
  std::vector<Err> skips;
  for (size_t i = 0; i < patArr->a.size(); i++) {
    std::string cp = path + std::to_string(i) + "/";
    Ret r = validate_element(c, resArr->a[i], patArr->a[i], cp);
    if (r.err.present) {
      if (skip_err(r.err)) { skips.push_back(r.err); continue; }
      return r;
    }
    apply++;
  }
  if (apply == 0 && !skips.empty()) return Ret{path, combine_skips(skips)};
  return Ret();
}

static Ret validate_element(Ctx& c, const VP& res, const VP& pat, const std::string& path) {  // validate.go:71-114
  if (pat && pat->t == T::Obj) {
    if (!res || res->t != T::Obj)
      return Ret{path, Err::make("pattern and resource have different structures. Path: " + path + ". Expected " + go_T(pat) + ", found " + go_T(res))};
    c.ac.check_anchor_in_resource(pat, res);
    return validate_map(c, res, pat, path);
  }
  if (pat && pat->t == T::Arr) {
    if (!res || res->t != T::Arr)
      return Ret{path, Err::make("validation rule failed at path " + path + ", resource does not satisfy the expected overlay pattern")};
    return validate_array(c, res, pat, path);
  }
  // elementary values
  auto mismatch = [&]() {
    return Ret{path, Err::make("resource value '" + oj::go_v(res) + "' does not match '" + oj::go_v(pat) + "' at path " + path)};
  };
  if (res && res->t == T::Arr) {
    for (auto& e : res->a)
      if (!pattern_validate(e, pat)) return mismatch();
    return Ret();
  }
  if (!pattern_validate(res, pat)) return mismatch();
  return Ret();
}

PatternResult match_pattern(const VP& resource, const VP& pattern0, EvalFlags& fl) {  // validate.go:31-56
  VP pattern = oj::deep_copy(pattern0);  // the reference validates a freshly decoded pattern per call
  Ctx c;
  c.fl = &fl;
  Ret r = validate_element(c, resource, pattern, "/");
  PatternResult out;
  if (!r.err.present) return out;
  out.ok = false;
  out.err = r.err.msg;
  if (skip_err(r.err)) { out.skip = true; out.path = ""; return out; }
  if (is_negation_err(r.err)) { out.path = r.path; return out; }
  if (c.ac.keys_are_missing()) { out.path = ""; return out; }
  out.path = r.path;
  return out;
}

}  // namespace orc

namespace orc {

// Test hooks: the reference's unexported leaf functions (pattern_test.go) and raw walk entries
// (validate_test.go call validateMap / validateResourceElement directly).
bool leaf_fn(const std::string& fn, const VP& v, const VP& p, const std::string& op) {
  Op o = Op::Equal;
  if (op == "!") o = Op::NotEqual;
  else if (op == ">") o = Op::More;
  else if (op == "<") o = Op::Less;
  else if (op == ">=") o = Op::MoreEqual;
  else if (op == "<=") o = Op::LessEqual;
  std::string ps = p && p->t == T::Str ? p->s : "";
  if (fn == "Validate") return pattern_validate(v, p);
  if (fn == "validateFloatPattern") return validate_float_pattern(v, p->t == T::Float ? p->f : (double)p->i);
  if (fn == "validateNilPattern") return validate_nil_pattern(v);
  if (fn == "validateStringPattern") return validate_string_pattern(v, ps);
  if (fn == "validateStringPatterns") return validate_string_patterns(v, ps);
  if (fn == "validateString") return validate_string(v, ps, o);
  if (fn == "compareString") return compare_string(v, ps, o);
  throw std::runtime_error("unknown leaf fn " + fn);
}

RawWalk validate_entry(const std::string& entry, const VP& res, const VP& pat0, EvalFlags& fl) {
  VP pat = oj::deep_copy(pat0);
  Ctx c;
  c.fl = &fl;
  RawWalk out;
  Ret r;
  if (entry == "validateMap") r = validate_map(c, res, pat, "/");
  else if (entry == "validateArray") r = validate_array(c, res, pat, "/");
  else r = validate_element(c, res, pat, "/");
  out.path = r.path;
  out.err = r.err.present;
  out.msg = r.err.msg;
  return out;
}

}  // namespace orc

namespace orc {
// operator.GetOperatorFromStringPattern(p) == operator.InRange (pkg/engine/operator/operator.go:35-61)
bool is_in_range_pattern(const std::string& p) { return get_operator(p) == Op::InRange; }
}  // namespace orc

namespace orc {
// anchor.RemoveAnchorsFromPath (anchor/utils.go:23-40): split on "/", drop a leading empty part, replace every
// part that parses as an anchor by its key, path.Join (which Cleans), re-root when the input was absolute
std::string remove_anchors_from_path(const std::string& str) {
  std::vector<std::string> parts;
  size_t st = 0;
  for (size_t i = 0; i <= str.size(); i++)
    if (i == str.size() || str[i] == '/') { parts.push_back(str.substr(st, i - st)); st = i + 1; }
  if (!parts.empty() && parts[0].empty()) parts.erase(parts.begin());
  std::string joined;
  for (auto& p : parts) {
    Anchor a = parse_anchor(p);
    std::string q = a.t != AT::None ? a.key : p;
    if (q.empty()) continue;  // path.Join ignores empty elements
    joined += joined.empty() ? q : "/" + q;
  }
  std::string out = joined.empty() ? "" : gou::clean_path(joined);
  if (!str.empty() && str[0] == '/') out = "/" + (out == "." ? std::string() : out);
  return out;
}

static const char* at_name(AT t) {
  switch (t) {
    case AT::Condition: return "Condition";
    case AT::Global: return "Global";
    case AT::Negation: return "Negation";
    case AT::AddIfNotPresent: return "AddIfNotPresent";
    case AT::Equality: return "Equality";
    case AT::Existence: return "Existence";
    default: return "";
  }
}
static AT at_from(const std::string& n) {
  for (AT t : {AT::Condition, AT::Global, AT::Negation, AT::AddIfNotPresent, AT::Equality, AT::Existence})
    if (n == at_name(t)) return t;
  return AT::None;
}

// Probe of the anchor package's helpers for its unit-test tables (tests/golden/anchor.json); JSON text out.
std::string anchor_probe(const std::string& op, const std::string& a, const std::string& b) {
  auto q = [](const std::string& s) { return oj::dump(Value::str(s)); };
  if (op == "parse") {
    Anchor x = parse_anchor(a);
    if (x.t == AT::None) return "null";
    return std::string("{\"type\":") + q(at_name(x.t)) + ",\"key\":" + q(x.key) + "}";
  }
  if (op == "string") return q(anchor_string(at_from(a), b));  // anchor.New(t, key).String(): "" for an empty key
  if (op == "is") {  // a: predicate, b: anchor type ("" = nil anchor)
    AT t = at_from(b);
    bool r = false;
    if (a == "IsCondition") r = t == AT::Condition;
    else if (a == "IsGlobal") r = t == AT::Global;
    else if (a == "IsNegation") r = t == AT::Negation;
    else if (a == "IsAddIfNotPresent") r = t == AT::AddIfNotPresent;
    else if (a == "IsEquality") r = t == AT::Equality;
    else if (a == "IsExistence") r = t == AT::Existence;
    else if (a == "ContainsCondition") r = t == AT::Condition || t == AT::Global;
    return r ? "true" : "false";
  }
  if (op == "err") {  // a: error kind; b: {"code": typed kind or -1, "msg": text} or null
    VP e = oj::parse(b, true);
    Err x = e->t == T::Null ? Err::none() : Err::make(e->o["msg"]->s, (int)e->o["code"]->f);
    bool r = a == "negation" ? is_negation_err(x) : a == "conditional" ? is_conditional_err(x) : is_global_err(x);
    return r ? "true" : "false";
  }
  if (op == "has_value") return AnchorMap::has_value_for_key(oj::parse(a, true), b) ? "true" : "false";
  if (op == "keys_missing") {
    AnchorMap m;
    VP v = oj::parse(a, true);
    for (auto& kv : v->o) m.m[kv.first] = kv.second->t == T::Bool && kv.second->b;
    return m.keys_are_missing() ? "true" : "false";
  }
  if (op == "remove_path") return q(remove_anchors_from_path(a));
  if (op == "split") {
    std::vector<std::string> an, rs;
    split_anchors(oj::parse(a, true), &an, &rs);
    std::string o = "{\"anchors\":[";
    for (size_t i = 0; i < an.size(); i++) o += (i ? "," : "") + q(an[i]);
    o += "],\"resources\":[";
    for (size_t i = 0; i < rs.size(); i++) o += (i ? "," : "") + q(rs[i]);
    return o + "]}";
  }
  throw std::runtime_error("anchor_probe: unknown op " + op);
}
}  // namespace orc
