// ORACLE — test infrastructure only (see ojson.h header). Conditions (deny / preconditions); see ocond.h.
#include "ocond.h"
#include "ojmes.h"

#include <cmath>

#include "goutil.h"
#include "ovalidate.h"

namespace orc {
using oj::T;
using oj::Value;
using oj::VP;

static bool isnil(const VP& v) { return !v || v->t == T::Null; }

VP condition_operand(const VP& v) {  // Condition.GetKey(): json.Marshal -> util/json decode (int64 if integral)
  if (!v) return nullptr;
  if (v->t == T::Null) return nullptr;
  return oj::parse(oj::dump(v), false);
}

// ---------------------------------------------------------------- helpers (operator.go)
static std::string sprint(const VP& v) { return oj::go_v(v); }  // fmt.Sprint

static int64_t wrap_mul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
static int64_t go_f2i(double f) {  // int64(float64): truncation (out-of-range is platform defined; amd64 -> min int64)
  if (std::isnan(f) || f >= 9223372036854775808.0 || f < -9223372036854775808.0) return INT64_MIN;
  return (int64_t)f;
}
static double dur_seconds(int64_t d) {  // time.Duration.Seconds
  int64_t sec = d / 1000000000LL, nsec = d % 1000000000LL;
  return (double)sec + (double)nsec / 1e9;
}

// operator.parseDuration (operator.go:94-138): both sides as durations, or false
static bool parse_duration2(const VP& key, const VP& value, double& ks, double& vs) {
  int64_t kd = 0, vd = 0;
  bool hk = false, hv = false;
  if (key && key->t == T::Str && key->s != "0" && gou::parse_duration(key->s, kd)) hk = true;
  if (value && value->t == T::Str && value->s != "0" && gou::parse_duration(value->s, vd)) hv = true;
  if (!hk && !hv) return false;
  if (!hk) {
    if (key && key->t == T::Int) kd = wrap_mul(key->i, 1000000000LL);
    else if (key && key->t == T::Float) kd = wrap_mul(go_f2i(key->f), 1000000000LL);
    else return false;
  }
  if (!hv) {
    if (value && value->t == T::Int) vd = wrap_mul(value->i, 1000000000LL);
    else if (value && value->t == T::Float) vd = wrap_mul(go_f2i(value->f), 1000000000LL);
    else return false;
  }
  ks = dur_seconds(kd);
  vs = dur_seconds(vd);
  return true;
}

static bool deep_equal(const VP& a, const VP& b) {  // reflect.DeepEqual on decoded JSON
  if (isnil(a) || isnil(b)) return isnil(a) && isnil(b);
  if (a->t != b->t) return false;
  switch (a->t) {
    case T::Bool: return a->b == b->b;
    case T::Int: return a->i == b->i;
    case T::Float: return a->f == b->f;
    case T::Str: return a->s == b->s;
    case T::Arr:
      if (a->a.size() != b->a.size()) return false;
      for (size_t i = 0; i < a->a.size(); i++) if (!deep_equal(a->a[i], b->a[i])) return false;
      return true;
    case T::Obj: {
      if (a->o.size() != b->o.size()) return false;
      for (auto& kv : a->o) {
        auto it = b->o.find(kv.first);
        if (it == b->o.end() || !deep_equal(kv.second, it->second)) return false;
      }
      return true;
    }
    default: return true;
  }
}

// json.Unmarshal(s, &[]string)
static bool unmarshal_strings(const std::string& s, std::vector<std::string>& out) {
  VP v;
  try { v = oj::parse(s, true); } catch (...) { return false; }
  out.clear();
  if (v->t == T::Null) return true;
  if (v->t != T::Arr) return false;
  for (auto& e : v->a) {
    if (isnil(e)) out.push_back("");
    else if (e->t == T::Str) out.push_back(e->s);
    else return false;
  }
  return true;
}
static bool json_valid(const std::string& s) {
  try { oj::parse(s, true); return true; } catch (...) { return false; }
}

// ---------------------------------------------------------------- Equal / NotEqual (equal.go, notequal.go)
static bool eq_int(int64_t k, const VP& v) {
  if (isnil(v)) return false;
  switch (v->t) {
    case T::Int: return v->i == k;
    case T::Float: return v->f == std::trunc(v->f) ? go_f2i(v->f) == k : false;
    case T::Str: { int64_t x; return gou::parse_int64(v->s, x) ? x == k : false; }
    default: return false;
  }
}
static bool eq_float(double k, const VP& v) {
  if (isnil(v)) return false;
  switch (v->t) {
    case T::Int: return k == std::trunc(k) ? go_f2i(k) == v->i : false;
    case T::Float: return v->f == k;
    case T::Str: { double x; return gou::parse_float(v->s, x) ? x == k : false; }
    default: return false;
  }
}
static bool eq_string(const std::string& k, const VP& key, const VP& v) {
  double ks, vs;
  if (parse_duration2(key, v, ks, vs)) return ks == vs;
  gou::Quantity qk;
  if (gou::parse_quantity(k, qk)) {
    if (v && v->t == T::Str) {
      gou::Quantity qv;
      if (!gou::parse_quantity(v->s, qv)) return false;
      return gou::quantity_cmp(qk, qv) == 0;
    }
  }
  if (v && v->t == T::Str) return gou::wildcard_match(v->s, k);
  return false;
}
static bool op_equal(const VP& k, const VP& v) {
  if (isnil(k)) return false;
  switch (k->t) {
    case T::Bool: return v && v->t == T::Bool && v->b == k->b;
    case T::Int: return eq_int(k->i, v);
    case T::Float: return eq_float(k->f, v);
    case T::Str: return eq_string(k->s, k, v);
    case T::Obj: return v && v->t == T::Obj && deep_equal(k, v);
    case T::Arr: return v && v->t == T::Arr && deep_equal(k, v);
    default: return false;
  }
}
static bool ne_int(int64_t k, const VP& v) {
  if (isnil(v)) return true;
  switch (v->t) {
    case T::Int: return v->i != k;
    case T::Float: return v->f == std::trunc(v->f) ? go_f2i(v->f) != k : false;
    case T::Str: { int64_t x; return gou::parse_int64(v->s, x) ? x != k : true; }
    default: return true;
  }
}
static bool ne_float(double k, const VP& v) {
  if (isnil(v)) return true;
  switch (v->t) {
    case T::Int: return k == std::trunc(k) ? go_f2i(k) != v->i : true;
    case T::Float: return v->f != k;
    case T::Str: { double x; return gou::parse_float(v->s, x) ? x != k : true; }
    default: return true;
  }
}
static bool ne_string(const std::string& k, const VP& key, const VP& v) {
  double ks, vs;
  if (parse_duration2(key, v, ks, vs)) return ks != vs;
  gou::Quantity qk;
  if (gou::parse_quantity(k, qk)) {
    if (v && v->t == T::Str) {
      if (v->s.empty()) return !gou::wildcard_match(v->s, k);
      gou::Quantity qv;
      if (!gou::parse_quantity(v->s, qv)) return false;
      return gou::quantity_cmp(qk, qv) != 0;
    }
  }
  if (v && v->t == T::Str) return !gou::wildcard_match(v->s, k);
  return true;
}
static bool op_not_equal(const VP& k, const VP& v) {
  if (isnil(k)) return false;
  switch (k->t) {
    case T::Bool: return !(v && v->t == T::Bool) ? true : v->b != k->b;
    case T::Int: return ne_int(k->i, v);
    case T::Float: return ne_float(k->f, v);
    case T::Str: return ne_string(k->s, k, v);
    case T::Obj: return v && v->t == T::Obj ? !deep_equal(k, v) : true;
    case T::Arr: return v && v->t == T::Arr ? !deep_equal(k, v) : true;
    default: return false;
  }
}

// ---------------------------------------------------------------- In / NotIn (in.go, notin.go)
// keyExistsInArray (in.go:52-86): returns invalidType, sets exists
static bool key_exists_in_array(const std::string& key, const VP& v, bool& exists) {
  exists = false;
  if (isnil(v)) return true;
  if (v->t == T::Arr) {
    for (auto& e : v->a) {
      std::string s = sprint(e);
      if (gou::wildcard_match(s, key) || gou::wildcard_match(key, s)) { exists = true; return false; }
    }
    return false;
  }
  if (v->t == T::Str) {
    if (gou::wildcard_match(v->s, key)) { exists = true; return false; }
    std::vector<std::string> arr;
    if (!unmarshal_strings(v->s, arr)) return true;
    for (auto& s : arr) if (key == s) { exists = true; return false; }
    return false;
  }
  return true;
}
static bool is_in(const std::vector<std::string>& key, const std::vector<std::string>& value) {
  for (auto& k : key) {
    bool f = false;
    for (auto& v : value) if (v == k) { f = true; break; }
    if (!f) return false;
  }
  return true;
}
static bool is_not_in(const std::vector<std::string>& key, const std::vector<std::string>& value) {
  for (auto& k : key) {
    bool f = false;
    for (auto& v : value) if (v == k) { f = true; break; }
    if (!f) return true;
  }
  return false;
}
// setExistsInArray (in.go:104-143)
static bool set_exists_in_array(const std::vector<std::string>& key, const VP& v, bool notIn, bool& out) {
  out = false;
  if (isnil(v)) return true;
  if (v->t == T::Arr) {
    std::vector<std::string> vs;
    for (auto& e : v->a) {
      if (isnil(e) || e->t != T::Str) return true;
      vs.push_back(e->s);
    }
    out = notIn ? is_not_in(key, vs) : is_in(key, vs);
    return false;
  }
  if (v->t == T::Str) {
    if (key.size() == 1 && key[0] == v->s) { out = true; return false; }
    std::vector<std::string> arr;
    if (!unmarshal_strings(v->s, arr)) return true;
    out = notIn ? is_not_in(key, arr) : is_in(key, arr);
    return false;
  }
  return true;
}
static std::vector<std::string> string_elems_or_panic(const VP& k) {  // v.(string) in in.go:37 / notin.go:37
  std::vector<std::string> out;
  for (auto& e : k->a) {
    if (isnil(e) || e->t != T::Str) throw RefPanic{"interface conversion: interface {} is not string"};
    out.push_back(e->s);
  }
  return out;
}
static bool op_in(const VP& k, const VP& v, bool notIn) {
  if (isnil(k)) return false;
  if (k->t == T::Str || k->t == T::Int || k->t == T::Float) {
    std::string ks = k->t == T::Str ? k->s : sprint(k);
    bool exists;
    if (key_exists_in_array(ks, v, exists)) return false;
    return notIn ? !exists : exists;
  }
  if (k->t == T::Arr) {
    auto keys = string_elems_or_panic(k);
    bool out;
    if (set_exists_in_array(keys, v, notIn, out)) return false;
    return out;
  }
  return false;
}

// ---------------------------------------------------------------- AnyIn / AllIn / AnyNotIn / AllNotIn
static bool handle_range(const std::string& key, const std::string& pattern) {  // anyin.go:98-104
  return pattern_validate(Value::str(key), Value::str(pattern));
}
// anyKeyExistsInArray == allKeyExistsInArray (anyin.go:51-96, allin.go:51-96)
static bool any_key_exists(const std::string& key, const VP& v, bool& exists) {
  exists = false;
  if (isnil(v)) return true;
  if (v->t == T::Arr) {
    for (auto& e : v->a) {
      std::string s = sprint(e);
      if (gou::wildcard_match(s, key) || gou::wildcard_match(key, s)) { exists = true; return false; }
    }
    return false;
  }
  if (v->t == T::Str) {
    if (gou::wildcard_match(v->s, key)) { exists = true; return false; }
    if (is_in_range_pattern(v->s)) { exists = handle_range(key, v->s); return false; }
    std::vector<std::string> arr;
    if (json_valid(v->s)) {
      if (!unmarshal_strings(v->s, arr)) return true;
    } else {
      arr.push_back(v->s);
    }
    for (auto& s : arr) if (key == s) { exists = true; return false; }
    return false;
  }
  return true;
}
static bool wild2(const std::string& a, const std::string& b) {
  return gou::wildcard_match(a, b) || gou::wildcard_match(b, a);
}
static size_t count_matched(const std::vector<std::string>& key, const std::vector<std::string>& value) {
  size_t n = 0;
  for (auto& k : key)
    for (auto& v : value)
      if (wild2(k, v)) { n++; break; }
  return n;
}
// anySetExistsInArray (anyin.go:115-180) / allSetExistsInArray (allin.go:115-180)
static bool set_exists_any_all(const std::vector<std::string>& key, const VP& v, bool all, bool neg, bool& out) {
  out = false;
  if (isnil(v)) return true;
  auto decide = [&](const std::vector<std::string>& vals) {
    size_t n = count_matched(key, vals);
    if (!all) return neg ? n < key.size() : n > 0;
    return neg ? n == 0 : n == key.size();
  };
  if (v->t == T::Arr) {
    std::vector<std::string> vs;
    for (auto& e : v->a) vs.push_back(sprint(e));
    out = decide(vs);
    return false;
  }
  if (v->t == T::Str) {
    if (key.size() == 1 && key[0] == v->s) { out = !neg; return false; }
    if (is_in_range_pattern(v->s)) {
      if (!all && neg) {
        std::string s2 = v->s;
        size_t i = s2.find('-');
        if (i != std::string::npos) s2.replace(i, 1, "!-");
        for (auto& k : key) if (handle_range(k, s2)) { out = true; break; }
      } else if (!all) {
        for (auto& k : key) if (handle_range(k, v->s)) { out = true; break; }
      } else if (neg) {
        out = true;
        for (auto& k : key) if (handle_range(k, v->s)) out = false;
      } else {
        size_t c = 0;
        for (auto& k : key) if (handle_range(k, v->s)) c++;
        out = c == key.size();
      }
      return false;
    }
    std::vector<std::string> arr;
    if (json_valid(v->s)) {
      if (!unmarshal_strings(v->s, arr)) return true;
    } else {
      arr.push_back(v->s);
    }
    out = decide(arr);
    return false;
  }
  return true;
}
static bool op_any_all(const VP& k, const VP& v, bool all, bool neg) {
  if (isnil(k)) return false;
  if (k->t == T::Str || k->t == T::Int || k->t == T::Float) {
    std::string ks = k->t == T::Str ? k->s : sprint(k);
    bool exists;
    if (any_key_exists(ks, v, exists)) return false;
    return neg ? !exists : exists;
  }
  if (k->t == T::Arr) {
    std::vector<std::string> keys;
    for (auto& e : k->a) keys.push_back(sprint(e));
    bool out;
    if (set_exists_any_all(keys, v, all, neg, out)) return false;
    return out;
  }
  return false;
}

// ---------------------------------------------------------------- semver (blang/semver v4)
struct SemVer {
  uint64_t maj = 0, min = 0, pat = 0;
  std::vector<std::pair<bool, std::string>> pre;  // (numeric, text)
  std::vector<uint64_t> pren;
};
static bool only(const std::string& s, bool alnum) {
  for (char c : s) {
    bool d = c >= '0' && c <= '9';
    bool a = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '-';
    if (!(d || (alnum && a))) return false;
  }
  return true;
}
static bool parse_u64(const std::string& s, uint64_t& out) {
  if (s.empty()) return false;
  unsigned __int128 v = 0;
  for (char c : s) {
    if (c < '0' || c > '9') return false;
    v = v * 10 + (unsigned)(c - '0');
    if (v > UINT64_MAX) return false;
  }
  out = (uint64_t)v;
  return true;
}
static bool semver_parse(const std::string& s, SemVer& v) {
  if (s.empty()) return false;
  auto parts = std::vector<std::string>();
  size_t a = s.find('.');
  if (a == std::string::npos) return false;
  size_t b = s.find('.', a + 1);
  if (b == std::string::npos) return false;
  parts = {s.substr(0, a), s.substr(a + 1, b - a - 1), s.substr(b + 1)};
  auto num = [&](const std::string& p, uint64_t& o) {
    if (!only(p, false)) return false;
    if (p.size() > 1 && p[0] == '0') return false;
    return parse_u64(p, o);
  };
  if (!num(parts[0], v.maj) || !num(parts[1], v.min)) return false;
  std::string patch = parts[2];
  std::vector<std::string> build, pre;
  size_t bi = patch.find('+');
  if (bi != std::string::npos) { build = gou::split(patch.substr(bi + 1), '.'); patch = patch.substr(0, bi); }
  size_t pi = patch.find('-');
  if (pi != std::string::npos) { pre = gou::split(patch.substr(pi + 1), '.'); patch = patch.substr(0, pi); }
  if (!num(patch, v.pat)) return false;
  for (auto& p : pre) {
    if (p.empty()) return false;
    if (only(p, false)) {
      if (p.size() > 1 && p[0] == '0') return false;
      uint64_t n;
      if (!parse_u64(p, n)) return false;
      v.pre.push_back({true, p});
      v.pren.push_back(n);
    } else {
      if (!only(p, true)) return false;
      v.pre.push_back({false, p});
      v.pren.push_back(0);
    }
  }
  for (auto& x : build) if (x.empty() || !only(x, true)) return false;
  return true;
}
static int semver_cmp(const SemVer& a, const SemVer& b) {
  if (a.maj != b.maj) return a.maj > b.maj ? 1 : -1;
  if (a.min != b.min) return a.min > b.min ? 1 : -1;
  if (a.pat != b.pat) return a.pat > b.pat ? 1 : -1;
  if (a.pre.empty() && b.pre.empty()) return 0;
  if (a.pre.empty()) return 1;
  if (b.pre.empty()) return -1;
  size_t i = 0;
  for (; i < a.pre.size() && i < b.pre.size(); i++) {
    bool an = a.pre[i].first, bn = b.pre[i].first;
    int c;
    if (an && bn) c = a.pren[i] == b.pren[i] ? 0 : (a.pren[i] > b.pren[i] ? 1 : -1);
    else if (an) c = -1;
    else if (bn) c = 1;
    else c = a.pre[i].second == b.pre[i].second ? 0 : (a.pre[i].second > b.pre[i].second ? 1 : -1);
    if (c) return c;
  }
  if (i == a.pre.size() && i == b.pre.size()) return 0;
  return i == a.pre.size() ? -1 : 1;
}
bool semver_ok(const std::string& s) { SemVer v; return semver_parse(s, v); }
bool semver_parse_cmp(const std::string& a, const std::string& b, int* cmp, bool* b_ok) {
  SemVer x, y;
  if (!semver_parse(a, x)) return false;
  *b_ok = semver_parse(b, y);
  if (*b_ok) *cmp = semver_cmp(x, y);
  return true;
}

// ---------------------------------------------------------------- numeric (numeric.go)
static bool cmp_by(double k, double v, const std::string& op) {  // compareByCondition: exact operator names
  if (op == "GreaterThanOrEquals") return k >= v;
  if (op == "GreaterThan") return k > v;
  if (op == "LessThanOrEquals") return k <= v;
  if (op == "LessThan") return k < v;
  return false;
}
static bool num_float(double k, const VP& v, const VP& key, const std::string& op) {
  if (isnil(v)) return false;
  switch (v->t) {
    case T::Int: return cmp_by(k, (double)v->i, op);
    case T::Float: return cmp_by(k, v->f, op);
    case T::Str: {
      double ks, vs;
      if (parse_duration2(key, v, ks, vs)) return cmp_by(ks, vs, op);
      double f;
      if (gou::parse_float(v->s, f)) return cmp_by(k, f, op);
      int64_t i;
      if (gou::parse_int64(v->s, i)) return cmp_by(k, (double)i, op);
      return false;
    }
    default: return false;
  }
}
static bool op_numeric(const VP& k, const VP& v, const std::string& op) {
  if (isnil(k)) return false;
  switch (k->t) {
    case T::Int: return num_float((double)k->i, v, k, op);
    case T::Float: return num_float(k->f, v, k, op);
    case T::Str: {
      double ks, vs;
      if (parse_duration2(k, v, ks, vs)) return cmp_by(ks, vs, op);
      if (v && v->t == T::Str) {
        gou::Quantity qk, qv;
        if (gou::parse_quantity(k->s, qk) && gou::parse_quantity(v->s, qv))
          return cmp_by((double)gou::quantity_cmp(qk, qv), 0, op);
      }
      double f;
      if (gou::parse_float(k->s, f)) return num_float(f, v, Value::flt(f), op);
      int64_t i;
      if (gou::parse_int64(k->s, i)) return num_float((double)i, v, Value::integer(i), op);
      if (semver_ok(k->s)) {
        if (!(v && v->t == T::Str)) return false;
        int c = 0;
        bool ok = false;
        semver_parse_cmp(k->s, v->s, &c, &ok);
        if (!ok) return false;
        return cmp_by((double)c, 0, op);
      }
      return false;
    }
    default: return false;
  }
}

// DurationOperatorHandler (pkg/engine/variables/operator/duration.go:30-150): Evaluate's type switches, then
// durationCompareByCondition on the exact operator name
static bool dur_operand(const VP& x, int64_t& d) {
  if (!x) return false;
  if (x->t == T::Int) { d = wrap_mul(x->i, 1000000000LL); return true; }
  if (x->t == T::Float) { d = wrap_mul(go_f2i(x->f), 1000000000LL); return true; }
  if (x->t == T::Str) return gou::parse_duration(x->s, d);
  return false;
}
static bool op_duration(const VP& key, const VP& value, const std::string& op) {
  int64_t kd, vd;
  if (!dur_operand(key, kd) || !dur_operand(value, vd)) return false;
  if (op == "DurationGreaterThanOrEquals") return kd >= vd;
  if (op == "DurationGreaterThan") return kd > vd;
  if (op == "DurationLessThanOrEquals") return kd <= vd;
  if (op == "DurationLessThan") return kd < vd;
  return false;
}

static std::string lower(std::string s) {
  for (auto& c : s) c = gou::lower(c);
  return s;
}

bool evaluate_condition(const VP& key, const std::string& op, const VP& value) {  // operator.go:27-75
  std::string o = lower(op);
  if (o == "equal" || o == "equals") return op_equal(key, value);
  if (o == "notequal" || o == "notequals") return op_not_equal(key, value);
  if (o == "in") return op_in(key, value, false);
  if (o == "notin") return op_in(key, value, true);
  if (o == "anyin") return op_any_all(key, value, false, false);
  if (o == "allin") return op_any_all(key, value, true, false);
  if (o == "anynotin") return op_any_all(key, value, false, true);
  if (o == "allnotin") return op_any_all(key, value, true, true);
  if (o == "greaterthanorequals" || o == "greaterthan" || o == "lessthanorequals" || o == "lessthan")
    return op_numeric(key, value, op);
  if (o == "durationgreaterthanorequals" || o == "durationgreaterthan" || o == "durationlessthanorequals" ||
      o == "durationlessthan")
    return op_duration(key, value, op);
  return false;  // no handler
}

// ---------------------------------------------------------------- substitution (vars.go, restricted)
static bool is_ident_start(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_'; }
static bool is_ident(char c) { return is_ident_start(c) || (c >= '0' && c <= '9'); }

// `{{ request.object(.seg)* }}` -> path segments; false when the string is not exactly one such variable
static bool parse_object_var(const std::string& s, std::vector<std::string>& segs) {
  if (s.size() < 4 || s.compare(0, 2, "{{") != 0 || s.compare(s.size() - 2, 2, "}}") != 0) return false;
  std::string inner = s.substr(2, s.size() - 4);
  if (inner.find('{') != std::string::npos || inner.find('}') != std::string::npos) return false;
  inner = gou::trim_space(inner);
  const std::string pre = "request.object";
  if (inner.compare(0, pre.size(), pre) != 0) return false;
  size_t i = pre.size();
  segs.clear();
  if (i < inner.size() && is_ident(inner[i])) return false;  // request.objectX
  while (i < inner.size()) {
    if (inner[i] != '.') return false;
    i++;
    if (i >= inner.size()) return false;
    if (inner[i] == '"') {
      size_t j = i + 1;
      while (j < inner.size() && inner[j] != '"') {
        if (inner[j] == '\\') return false;  // escapes: not in the subset
        j++;
      }
      if (j >= inner.size() || j == i + 1) return false;
      segs.push_back(inner.substr(i + 1, j - i - 1));
      i = j + 1;
    } else if (is_ident_start(inner[i])) {
      size_t j = i;
      while (j < inner.size() && is_ident(inner[j])) j++;
      segs.push_back(inner.substr(i, j - i));
      i = j;
    } else {
      return false;
    }
  }
  return true;
}
static bool has_var_syntax(const std::string& s) {
  return s.find("{{") != std::string::npos || s.find("$(") != std::string::npos;
}

// a string that is exactly one `{{ <JMESPath> }}` variable (no nested braces) -> the trimmed expression
static bool single_var(const std::string& s, std::string* expr) {
  if (s.size() < 4 || s.compare(0, 2, "{{") != 0 || s.compare(s.size() - 2, 2, "}}") != 0) return false;
  std::string inner = s.substr(2, s.size() - 4);
  if (inner.find('{') != std::string::npos || inner.find('}') != std::string::npos) return false;
  *expr = gou::trim_space(inner);
  return true;
}

static bool conditions_supported_in(const VP& v, bool allow_element) {
  if (!v) return true;
  if (v->t == T::Str) {
    if (!has_var_syntax(v->s)) return true;
    std::vector<std::string> segs;
    if (parse_object_var(v->s, segs)) return true;
    std::string expr;
    return v->s.find("$(") == std::string::npos && single_var(v->s, &expr) && jmes_supported(expr, allow_element);
  }
  if (v->t == T::Arr) { for (auto& e : v->a) if (!conditions_supported_in(e, allow_element)) return false; return true; }
  if (v->t == T::Obj) {
    for (auto& kv : v->o) {
      if (has_var_syntax(kv.first)) return false;
      if (!conditions_supported_in(kv.second, allow_element)) return false;
    }
  }
  return true;
}

bool conditions_supported(const VP& v) { return conditions_supported_in(v, false); }
bool conditions_supported_element(const VP& v) { return conditions_supported_in(v, true); }

static VP floats(const VP& v) {  // encoding/json decode of the JSON context: every number float64
  if (!v) return Value::null();
  switch (v->t) {
    case T::Int: return Value::flt((double)v->i);
    case T::Arr: { auto o = Value::arr(); for (auto& e : v->a) o->a.push_back(floats(e)); return o; }
    case T::Obj: { auto o = Value::obj(); for (auto& kv : v->o) o->o[kv.first] = floats(kv.second); return o; }
    default: return v;
  }
}
// JMESPath field chain over the JSON context (kyverno/go-jmespath fork): a key missing from a map is
// NotFoundError("Unknown key \"k\" in path"); a field of null / a non-map is null (no error)
static VP resolve(const std::vector<std::string>& segs, const VP& resource, std::string* missing) {
  VP cur = resource;
  for (auto& s : segs) {
    if (isnil(cur) || cur->t != T::Obj) return Value::null();
    if (!cur->has(s)) { *missing = s; return nullptr; }
    cur = cur->get(s);
  }
  return isnil(cur) ? Value::null() : floats(cur);
}
static std::string var_text(const std::string& s) {  // replaceBracesAndTrimSpaces (vars.go:462-467)
  return gou::trim_space(s.substr(2, s.size() - 4));
}
struct SubstErr {
  int n = 0;
  std::string first;
  bool unpinned = false;
};
struct VarCtx { VP resource; VP element; int64_t index; };
// substituteVariablesIfAny over the condition document (vars.go:352-431); data.Path is the JSON pointer of the
// string ("/0/key", "/any/1/value"; '/' in keys escaped as "\/", traverse.go:93)
static VP substitute(const VP& v, const VarCtx& cx, const std::string& path, SubstErr& e) {
  if (!v) return v;
  if (v->t == T::Str) {
    std::vector<std::string> segs;
    if (has_var_syntax(v->s) && parse_object_var(v->s, segs)) {
      std::string missing;
      VP r = resolve(segs, cx.resource, &missing);
      if (!r) {
        if (e.n++ == 0)
          e.first = "failed to resolve " + var_text(v->s) + " at path " + path +
                    ": JMESPath query failed: Unknown key \"" + missing + "\" in path";
        return Value::null();
      }
      return r;
    }
    std::string expr;
    if (has_var_syntax(v->s) && single_var(v->s, &expr)) {  // JMESPath subset (ojmes.h)
      try {
        return jmes_query(expr, cx.resource, cx.element, cx.index);
      } catch (JmesNotFound& nf) {
        if (e.n++ == 0)
          e.first = "failed to resolve " + expr + " at path " + path + ": JMESPath query failed: Unknown key \"" +
                    nf.key + "\" in path";
      } catch (JmesError& je) {
        if (e.n++ == 0) e.first = "failed to resolve " + expr + " at path " + path + ": " + je.msg;
        e.unpinned = true;
      }
      return Value::null();
    }
    return v;
  }
  if (v->t == T::Arr) {
    auto o = Value::arr();
    for (size_t i = 0; i < v->a.size(); i++) o->a.push_back(substitute(v->a[i], cx, path + "/" + std::to_string(i), e));
    return o;
  }
  if (v->t == T::Obj) {
    auto o = Value::obj();
    for (auto& kv : v->o) {
      std::string k;
      for (char c : kv.first) { if (c == '/') k += "\\/"; else k += c; }
      o->o[kv.first] = substitute(kv.second, cx, path + "/" + k, e);
    }
    return o;
  }
  return v;
}

// SubstituteAll of a message's `{{ request.object... }}` references (vars.go): 0 the text in *out; 1 a reference does
// not resolve (NotFoundError); 2 the whole message is one reference whose value is not a string; 3 outside the
// restated subset ($() references, escapes, other variables, nested variables in a value)
int substitute_message(const std::string& msg, const VP& resource, std::string* out) {
  if (!has_var_syntax(msg)) return *out = msg, 0;
  if (msg.find("$(") != std::string::npos || msg.find("\\{{") != std::string::npos) return 3;
  std::vector<std::string> segs;
  if (parse_object_var(msg, segs)) {  // whole message is one variable: the typed value
    std::string missing;
    VP r = resolve(segs, resource, &missing);
    if (!r) return 1;
    if (r->t == T::Str) return *out = r->s, 0;
    return 2;
  }
  std::string o;
  size_t i = 0;
  while (i < msg.size()) {
    size_t a = msg.find("{{", i);
    if (a == std::string::npos) { o += msg.substr(i); break; }
    size_t b = msg.find("}}", a + 2);
    if (b == std::string::npos) return 3;
    std::string var = msg.substr(a, b + 2 - a);
    if (!parse_object_var(var, segs)) return 3;
    std::string missing;
    VP r = resolve(segs, resource, &missing);
    if (!r) return 1;
    o += msg.substr(i, a - i);
    std::string sub = r->t == T::Str ? r->s : oj::dump(r);
    if (sub.find("{{") != std::string::npos) return 3;  // nested variables are re-scanned
    o += sub;
    i = b + 2;
  }
  return *out = o, 0;
}

// getDenyMessage (validation.go:461-479): a substitution error leaves the message as written
std::string render_message(const std::string& msg, const VP& resource, bool* unpinned) {
  *unpinned = false;
  std::string o;
  switch (substitute_message(msg, resource, &o)) {
    case 0: return o;
    case 1: return msg;
    case 2: return "the produced message didn't resolve to a string, check your policy definition.";
    default: *unpinned = true; return msg;
  }
}

static bool valid_op_exact(const std::string& op) {  // kyvernov1.ConditionOperators values (common_types.go:225-244)
  static const char* ops[] = {"Equal", "Equals", "NotEqual", "NotEquals", "In", "AnyIn", "AllIn", "NotIn", "AnyNotIn",
                              "AllNotIn", "GreaterThanOrEquals", "GreaterThan", "LessThanOrEquals", "LessThan",
                              "DurationGreaterThanOrEquals", "DurationGreaterThan", "DurationLessThanOrEquals",
                              "DurationLessThan"};
  for (auto o : ops) if (op == o) return true;
  return false;
}

// one Condition object -> (key, operator, value); false when its shape is outside the subset
static bool condition_fields(const VP& c, VP& key, std::string& op, VP& value) {
  if (isnil(c) || c->t != T::Obj) return false;
  for (auto& kv : c->o)
    if (kv.first != "key" && kv.first != "operator" && kv.first != "value" && kv.first != "message") return false;
  VP o = c->get("operator");
  if (o && o->t != T::Str && o->t != T::Null) return false;
  op = o && o->t == T::Str ? o->s : "";
  key = condition_operand(c->get("key"));
  value = condition_operand(c->get("value"));
  return true;
}

CondResult eval_conditions(const VP& conditions, const VP& resource) {
  return eval_conditions_element(conditions, resource, nullptr, 0);
}

CondResult eval_conditions_element(const VP& conditions, const VP& resource, const VP& element, int64_t index) {
  CondResult r;
  if (!conditions_supported_in(conditions, element != nullptr)) { r.r = CondOutcome::Unsupported; return r; }
  SubstErr se;
  VP doc;
  try {
    doc = substitute(conditions, VarCtx{resource, element, index}, "", se);
  } catch (JmesUnsupported&) {  // a value outside the restatement at run time (to_upper / regex_match subjects)
    r.r = CondOutcome::Unsupported;
    return r;
  }
  if (se.n) { r.r = CondOutcome::Error; r.err = se.first; r.err_unpinned = se.n > 1 || se.unpinned; return r; }
  if (isnil(doc)) { r.r = CondOutcome::True; return r; }  // null -> empty old-style list -> all true
  if (doc->t == T::Arr) {  // []Condition (evaluate.go:72-81), operators checked exactly (json.go:57-72)
    std::vector<std::tuple<VP, std::string, VP>> cs;
    for (auto& c : doc->a) {
      VP k, v;
      std::string op;
      if (!condition_fields(c, k, op, v) || !valid_op_exact(op)) { r.r = CondOutcome::Unsupported; return r; }
      cs.emplace_back(k, op, v);
    }
    for (auto& c : cs)
      if (!evaluate_condition(std::get<0>(c), std::get<1>(c), std::get<2>(c))) { r.r = CondOutcome::False; return r; }
    r.r = CondOutcome::True;
    return r;
  }
  if (doc->t == T::Obj) {  // AnyAllConditions (evaluate.go:42-69)
    for (auto& kv : doc->o) if (kv.first != "any" && kv.first != "all") { r.r = CondOutcome::Unsupported; return r; }
    VP any = doc->get("any"), all = doc->get("all");
    for (auto& blk : {any, all}) {
      if (isnil(blk)) continue;
      if (blk->t != T::Arr) { r.r = CondOutcome::Unsupported; return r; }
      for (auto& c : blk->a) {
        VP k, v;
        std::string op;
        if (!condition_fields(c, k, op, v)) { r.r = CondOutcome::Unsupported; return r; }
      }
    }
    bool anyRes = true, allRes = true;
    if (!isnil(any)) {
      anyRes = false;
      for (auto& c : any->a) {
        VP k, v;
        std::string op;
        condition_fields(c, k, op, v);
        if (evaluate_condition(k, op, v)) { anyRes = true; break; }
      }
    }
    if (!isnil(all))
      for (auto& c : all->a) {
        VP k, v;
        std::string op;
        condition_fields(c, k, op, v);
        if (!evaluate_condition(k, op, v)) { allRes = false; break; }
      }
    r.r = anyRes && allRes ? CondOutcome::True : CondOutcome::False;
    return r;
  }
  r.r = CondOutcome::Unsupported;
  return r;
}

}  // namespace orc
