// ORACLE — test infrastructure only (see ojson.h header).
//
// Restatement of the whole-object typed decode validatePodSecurity does (pkg/engine/validation.go:481-532 getSpec:
// encoding/json Unmarshal of the resource into corev1.Pod, appsv1.Deployment for every workload kind, or
// batchv1.CronJob; an error is the rule's error, :538-540), over the parsed resource (oj::Value), against the field
// types of k8s.io/api v0.26.1 tabled in kyverno_amd/csrc/k8s_types.h (data: the same table the flattener reads; the
// decoding rules here are this file's own). Parity unpinned: neither k8s.io/api nor encoding/json is vendored under
// /root/reference, and no fixture there holds a wrongly typed pod.
//
// encoding/json (Go 1.19) rules restated: null leaves any field's zero value; a JSON string / bool / number only
// into a field of that kind, an integer field taking a literal strconv.ParseInt accepts within its bit size; objects
// into structs (an unknown key is skipped; a key matches a field exactly, else case-insensitively, first field in
// order) and into maps; arrays into slices. UnmarshalJSON methods: resource.Quantity (ParseQuantity of the trimmed
// string, or of a number's literal), intstr.IntOrString (a string, else json.Unmarshal into int32), metav1.Time (a
// string, then time.Parse(time.RFC3339)).
#include "otyped.h"

#include <cctype>
#include <functional>
#include <map>
#include <stdexcept>
#include <vector>

#include "../kyverno_amd/csrc/k8s_types.h"
#include "goutil.h"

namespace orc {
using oj::T;
using oj::VP;

namespace {

// a type: primitive name ("s", "b", "i32", "i64", "q", "ios", "t", "any"), "[...]" slice, "{...}" map, or a struct
struct OStruct { std::vector<std::pair<std::string, std::string>> fields; };  // (json name, type text), Go order

std::map<std::string, OStruct> load() {
  std::map<std::string, std::pair<std::string, std::vector<std::pair<std::string, std::string>>>> decl;
  std::vector<std::string> order;
  const std::string s = k8st::kSchema;
  size_t i = 0;
  auto skip = [&] { while (i < s.size() && std::isspace((unsigned char)s[i])) i++; };
  auto word = [&] {
    size_t j = i;
    while (j < s.size() && (std::isalnum((unsigned char)s[j]) || s[j] == '_')) j++;
    std::string w = s.substr(i, j - i);
    i = j;
    return w;
  };
  for (skip(); i < s.size(); skip()) {
    std::string name = word(), base;
    if (s[i] == ':') { i++; base = word(); }
    if (s[i++] != '{') throw std::runtime_error("schema: { expected");
    std::vector<std::pair<std::string, std::string>> fs;
    for (skip(); s[i] != '}'; skip()) {
      std::string f = word();
      if (s[i++] != ':') throw std::runtime_error("schema: : expected");
      int depth = 0;
      size_t j = i;
      while (j < s.size() && (depth > 0 || (s[j] != ' ' && s[j] != '}' && s[j] != '\n'))) {
        if (s[j] == '[' || s[j] == '{') depth++;
        else if (s[j] == ']' || s[j] == '}') depth--;
        j++;
      }
      fs.emplace_back(f, s.substr(i, j - i));
      i = j;
    }
    i++;
    decl[name] = {base, fs};
    order.push_back(name);
  }
  std::map<std::string, OStruct> out;
  std::function<void(const std::string&)> build = [&](const std::string& n) {
    if (out.count(n)) return;
    auto& d = decl.at(n);
    OStruct st;
    if (!d.first.empty()) { build(d.first); st = out.at(d.first); }
    for (auto& f : d.second) st.fields.push_back(f);
    out[n] = st;
  };
  for (auto& n : order) build(n);
  return out;
}

const std::map<std::string, OStruct>& structs() {
  static const std::map<std::string, OStruct> m = load();
  return m;
}

bool is_null(const VP& v) { return !v || v->t == T::Null; }

// time.Parse(time.RFC3339, v): layout "2006-01-02T15:04:05Z07:00" through Go's general parser (format.go Parse):
// stdLongYear 4 digits, stdZeroMonth / stdZeroDay / stdZeroMinute / stdZeroSecond getnum(fixed), stdHour getnum(not
// fixed: one or two digits), a fractional second after the seconds when the value has one, stdISO8601ColonTZ 'Z' or
// sign hh ':' mm (hh <= 24, mm <= 60); no text left; day within the month
bool time_ok(const std::string& v) {
  auto d = [&](size_t k) { return k < v.size() && std::isdigit((unsigned char)v[k]); };
  size_t p = 0;
  if (!(d(0) && d(1) && d(2) && d(3))) return false;
  int year = std::stoi(v.substr(0, 4));
  p = 4;
  auto two = [&](int& x) { if (!d(p) || !d(p + 1)) return false; x = std::stoi(v.substr(p, 2)); p += 2; return true; };
  auto ch = [&](char c) { if (p < v.size() && v[p] == c) { p++; return true; } return false; };
  int mon, day, hh, mi, ss;
  if (!ch('-') || !two(mon)) return false;
  if (mon < 1 || mon > 12) return false;
  if (!ch('-') || !two(day)) return false;
  if (!ch('T')) return false;
  if (!d(p)) return false;
  if (d(p + 1)) { hh = std::stoi(v.substr(p, 2)); p += 2; } else { hh = v[p] - '0'; p++; }
  if (hh >= 24) return false;
  if (!ch(':') || !two(mi) || mi >= 60) return false;
  if (!ch(':') || !two(ss) || ss >= 60) return false;
  if (p + 1 < v.size() && (v[p] == '.' || v[p] == ',') && d(p + 1)) { p += 2; while (d(p)) p++; }
  if (ch('Z')) {
  } else {
    if (v.size() - p < 6 || (v[p] != '+' && v[p] != '-') || v[p + 3] != ':') return false;
    if (!d(p + 1) || !d(p + 2) || !d(p + 4) || !d(p + 5)) return false;
    if (std::stoi(v.substr(p + 1, 2)) > 24 || std::stoi(v.substr(p + 4, 2)) > 60) return false;
    p += 6;
  }
  if (p != v.size()) return false;
  const bool leap = year % 4 == 0 && (year % 100 != 0 || year % 400 == 0);
  const int dim[] = {31, leap ? 29 : 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  return day >= 1 && day <= dim[mon - 1];
}

std::string trim_space(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && std::isspace((unsigned char)s[a])) a++;
  while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
  return s.substr(a, b - a);
}

std::string lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

void check(const VP& v, const std::string& type, const std::string& path, bool* folded) {
  if (is_null(v)) return;
  auto fail = [&](const std::string& why) { throw TypedDecodeError{"json: cannot unmarshal " + why + " into field " + path + " of type " + type}; };
  if (type == "s") { if (v->t != T::Str) fail("non-string"); return; }
  if (type == "b") { if (v->t != T::Bool) fail("non-bool"); return; }
  if (type == "i32" || type == "i64" || type == "ios") {
    if (type == "ios" && v->t == T::Str) return;
    if (v->t != T::Int) fail("non-integer");
    if (type != "i64" && (v->i < INT32_MIN || v->i > INT32_MAX)) fail("out-of-range number");
    return;
  }
  if (type == "q") {
    if (v->t == T::Int || v->t == T::Float) return;
    gou::Quantity q;
    if (v->t != T::Str || !gou::parse_quantity(trim_space(v->s), q)) fail("a non-quantity");
    return;
  }
  if (type == "t") { if (v->t != T::Str || !time_ok(v->s)) fail("a non-RFC3339 value"); return; }
  if (type == "any") return;
  if (type[0] == '[') {
    if (v->t != T::Arr) fail("non-array");
    const std::string et = type.substr(1, type.size() - 2);
    for (size_t i = 0; i < v->a.size(); i++) check(v->a[i], et, path + "[" + std::to_string(i) + "]", folded);
    return;
  }
  if (type[0] == '{') {
    if (v->t != T::Obj) fail("non-object");
    const std::string et = type.substr(1, type.size() - 2);
    for (auto& kv : v->o) check(kv.second, et, path + "." + kv.first, folded);
    return;
  }
  const OStruct& st = structs().at(type);
  if (v->t != T::Obj) fail("non-object");
  for (auto& kv : v->o) {
    const std::pair<std::string, std::string>* f = nullptr;
    for (auto& x : st.fields) if (x.first == kv.first) { f = &x; break; }
    if (!f) {
      const std::string lk = lower(kv.first);
      for (auto& x : st.fields) if (lower(x.first) == lk) { f = &x; *folded = true; break; }
    }
    if (f) check(kv.second, f->second, path + "." + kv.first, folded);
  }
}

}  // namespace

std::string typed_decode_error(const VP& resource, const std::string& kind, bool* folded) {
  bool fold = false;
  std::string root;
  if (kind == "Pod") root = "Pod";
  else if (kind == "DaemonSet" || kind == "Deployment" || kind == "Job" || kind == "StatefulSet" || kind == "ReplicaSet" ||
           kind == "ReplicationController") root = "Deployment";
  else if (kind == "CronJob") root = "CronJob";
  else return "";
  try {
    check(resource, root, root, &fold);
  } catch (TypedDecodeError& e) {
    return e.msg;
  }
  if (folded) *folded = fold;
  return "";
}

}  // namespace orc
