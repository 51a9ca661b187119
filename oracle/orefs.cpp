// ORACLE — test infrastructure only (see ojson.h header).
//
// $() references in patterns: variables.substituteReferences (pkg/engine/variables/vars.go:244-346) run through
// jsonutils.Traversal with OnlyForLeafsAndKeys (pkg/engine/jsonutils/traverse.go): every map key (at its map's
// path) and every leaf (at its own path, keys escaped "/" -> "\/") is a string the action rewrites. References are
// looked up in the ORIGINAL document (getValueFromReference, vars.go:560-575: the last element visited whose
// anchor-free path equals the absolute reference path).
#include "orefs.h"

#include <regex>

#include "goutil.h"
#include "ovalidate.h"

namespace orc {
using oj::T;
using oj::Value;
using oj::VP;

namespace {

bool isnil(const VP& v) { return !v || v->t == T::Null; }

std::string esc_key(const std::string& k) {
  std::string o;
  for (char c : k) { if (c == '/') o += "\\/"; else o += c; }
  return o;
}

// `.[^\ ]*\)` from position q: '.' is any byte but '\n', then greedy non-space bytes, backtracking to a ')'
long tail_end(const std::string& s, size_t q) {
  if (q >= s.size() || s[q] == '\n') return -1;
  size_t stop = q + 1;
  while (stop < s.size() && s[stop] != ' ') stop++;
  for (size_t e = stop; e > q + 1; e--) if (s[e - 1] == ')') return (long)(e - 1);
  return -1;
}

// regexp.FindAllString of RegexReferences (vars.go:27) or RegexEscpReferences (vars.go:30)
std::vector<std::string> find_all(const std::string& s, bool escp) {
  std::vector<std::string> out;
  for (size_t p = 0; p < s.size();) {
    long e = -1;
    if (escp) {
      if (s[p] == '\\' && s.compare(p + 1, 2, "$(") == 0) e = tail_end(s, p + 3);
    } else {
      if (p == 0 && s.compare(0, 2, "$(") == 0) e = tail_end(s, 2);  // ^\$\(...
      if (e < 0 && s[p] != '\\' && s.compare(p + 1, 2, "$(") == 0) e = tail_end(s, p + 3);  // [^\\]\$\(...
    }
    if (e < 0) { p++; continue; }
    out.push_back(s.substr(p, (size_t)e + 1 - p));
    p = (size_t)e + 1;
  }
  return out;
}

// operator.GetOperatorFromStringPattern (pkg/engine/operator/operator.go:35-61)
std::string operator_prefix(const std::string& p) {
  if (p.size() < 2) return "";
  for (const char* o : {">=", "<=", ">", "<", "!"})
    if (p.compare(0, strlen(o), o) == 0) return o;
  static const std::regex notin(R"(^([-|\+]?\d+(?:\.\d+)?[A-Za-z]*)!-([-|\+]?\d+(?:\.\d+)?[A-Za-z]*)$)");
  static const std::regex in(R"(^([-|\+]?\d+(?:\.\d+)?[A-Za-z]*)-([-|\+]?\d+(?:\.\d+)?[A-Za-z]*)$)");
  if (std::regex_match(p, notin)) return "!-";
  if (std::regex_match(p, in)) return "-";
  return "";
}

}  // namespace

// path.Join(absolutePath, referencePath) unless the reference is absolute (formAbsolutePath, vars.go:552-558)
std::string form_absolute_path(const std::string& ref, const std::string& at) {
  if (!ref.empty() && ref[0] == '/') return ref;
  std::string j;
  for (const std::string& e : {at, ref}) if (!e.empty()) j += j.empty() ? e : "/" + e;
  return j.empty() ? "" : gou::clean_path(j);
}

namespace {

void visit(const VP& v, const std::string& path, const std::string& want, std::vector<VP>* hits) {
  if (!isnil(v) && v->t == T::Obj) {
    for (auto& kv : v->o) {
      if (remove_anchors_from_path(path) == want) hits->push_back(Value::str(kv.first));
      visit(kv.second, path + "/" + esc_key(kv.first), want, hits);
    }
  } else if (!isnil(v) && v->t == T::Arr) {
    for (size_t i = 0; i < v->a.size(); i++) visit(v->a[i], path + "/" + std::to_string(i), want, hits);
  } else {
    if (remove_anchors_from_path(path) == want) hits->push_back(v ? v : Value::null());
  }
}

struct Fail { std::string msg; bool unpinned; };

std::string go_v(const VP& v, bool* unpinned) {  // %v of a decoded JSON scalar
  if (isnil(v)) return "<nil>";
  if (v->t == T::Bool) return v->b ? "true" : "false";
  if (v->t == T::Str) return v->s;
  *unpinned = true;
  return oj::dump(v);
}

// substituteReferencesIfAny on one key or leaf (vars.go:286-346)
std::string subst(const std::string& in, const std::string& path, const VP& doc, RefResult* st) {
  std::string value = in;
  for (std::string v : find_all(in, false)) {
    const bool initial = v.compare(0, 2, "$(") == 0;
    const std::string old = v;
    if (!initial) v = v.substr(1);
    // resolveReference (vars.go:472-502)
    size_t a = 0, b = v.size();
    auto cut = [](char c) { return c == '$' || c == '(' || c == ')'; };
    while (a < b && cut(v[a])) a++;
    while (b > a && cut(v[b - 1])) b--;
    std::string p = v.substr(a, b - a);
    const std::string op = operator_prefix(p);
    p = p.substr(op.size());
    if (p.empty()) throw Fail{"failed to resolve " + v + " at path " + path + ": expected path, found empty reference", false};
    std::vector<VP> hits;
    visit(doc, "", form_absolute_path(p, path), &hits);
    VP found = hits.empty() ? nullptr : hits.back();
    for (auto& h : hits) if (oj::dump(h) != oj::dump(found)) st->nd = true;  // last visited wins: Go map order
    VP res;
    if (op.empty()) {
      res = found;
    } else {
      std::string s;
      if (isnil(found)) {
        bool unp = false;
        throw Fail{"failed to resolve " + v + " at path " + path + ": incorrect expression: operator " + op +
                       " does not match with value " + go_v(found, &unp), unp};
      }
      if (found->t == T::Str) s = found->s;
      else if (found->t == T::Float) s = gou::format_float_f6(found->f);
      else if (found->t == T::Int) s = std::to_string(found->i);
      else {
        bool unp = false;
        std::string shown = go_v(found, &unp);
        throw Fail{"failed to resolve " + v + " at path " + path + ": incorrect expression: operator " + op +
                       " does not match with value " + shown, true};
      }
      res = Value::str(op + s);
    }
    if (isnil(res)) throw Fail{"got nil resolved variable " + v + " at path " + path + ": <nil>", false};
    if (res->t != T::Str) throw Fail{"NotResolvedReferenceErr,reference " + v + " not resolved at path " + path, false};
    const std::string repl = (initial ? std::string() : old.substr(0, 1)) + res->s;
    size_t at = value.find(old);
    if (at != std::string::npos) value.replace(at, old.size(), repl);
  }
  for (const std::string& e : find_all(value, true)) {
    std::string out;
    size_t from = 0;
    for (size_t at = value.find(e); at != std::string::npos; at = value.find(e, from)) {
      out += value.substr(from, at - from) + e.substr(1);
      from = at + e.size();
    }
    value = out + value.substr(from);
  }
  return value;
}

VP walk(const VP& v, const std::string& path, const VP& doc, RefResult* st) {
  if (isnil(v)) return v;
  if (v->t == T::Str) return Value::str(subst(v->s, path, doc, st));
  if (v->t == T::Arr) {
    auto o = std::make_shared<Value>(*v);
    for (size_t i = 0; i < v->a.size(); i++) o->a[i] = walk(v->a[i], path + "/" + std::to_string(i), doc, st);
    return o;
  }
  if (v->t == T::Obj) {
    auto o = std::make_shared<Value>();
    o->t = T::Obj;
    for (auto& kv : v->o) {
      std::string k = subst(kv.first, path, doc, st);
      VP x = walk(kv.second, path + "/" + esc_key(kv.first), doc, st);
      if (k != kv.first && (v->o.count(k) || o->o.count(k))) st->nd = true;  // rename onto another key
      o->o[k] = x;
    }
    return o;
  }
  return v;
}

}  // namespace

bool has_references(const VP& v) {
  if (isnil(v)) return false;
  if (v->t == T::Str) return v->s.find("$(") != std::string::npos;
  for (auto& e : v->a) if (has_references(e)) return true;
  for (auto& kv : v->o) if (kv.first.find("$(") != std::string::npos || has_references(kv.second)) return true;
  return false;
}

RefResult substitute_references(const VP& doc) {
  RefResult r;
  try {
    r.doc = walk(doc, "", doc, &r);
  } catch (Fail& f) {
    r.ok = false;
    r.err = f.msg;
    r.err_unpinned = f.unpinned;
    r.doc = doc;
  }
  return r;
}

}  // namespace orc
