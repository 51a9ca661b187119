// ORACLE — test infrastructure only. Never linked into, imported by, or called from the
// product path (kyverno_amd/, libkyvgpu.so). Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load it, and only as the checker.
//
// Minimal JSON DOM with the decoding semantics the reference relies on:
//  * resources decode like k8s.io/apimachinery unstructured (pkg/utils/kube/unstructured.go:10-17
//    -> utiljson.Unmarshal): integral literals that fit int64 become int64, every other number float64;
//  * policy patterns decode like encoding/json into interface{} (api/kyverno/v1/utils.go:10):
//    every number is float64;
//  * strings: invalid UTF-8 bytes and unpaired UTF-16 surrogates become U+FFFD (encoding/json unquote);
//  * objects keep Go-map semantics: duplicate keys -> last wins; iteration is sorted (std::map),
//    which equals sort.Strings order wherever the reference sorts.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace oj {

enum class T : uint8_t { Null, Bool, Int, Float, Str, Arr, Obj };

struct Value;
using VP = std::shared_ptr<Value>;

struct Value {
  T t = T::Null;
  bool b = false;
  int64_t i = 0;
  double f = 0;
  std::string s;
  std::vector<VP> a;
  std::map<std::string, VP> o;

  static VP null() { return std::make_shared<Value>(); }
  static VP boolean(bool v) { auto p = std::make_shared<Value>(); p->t = T::Bool; p->b = v; return p; }
  static VP integer(int64_t v) { auto p = std::make_shared<Value>(); p->t = T::Int; p->i = v; return p; }
  static VP flt(double v) { auto p = std::make_shared<Value>(); p->t = T::Float; p->f = v; return p; }
  static VP str(const std::string& v) { auto p = std::make_shared<Value>(); p->t = T::Str; p->s = v; return p; }
  static VP arr() { auto p = std::make_shared<Value>(); p->t = T::Arr; return p; }
  static VP obj() { auto p = std::make_shared<Value>(); p->t = T::Obj; return p; }

  bool is_null() const { return t == T::Null; }
  bool is_obj() const { return t == T::Obj; }
  bool is_arr() const { return t == T::Arr; }
  bool is_str() const { return t == T::Str; }
  // lookup; returns nullptr when absent
  VP get(const std::string& k) const {
    if (t != T::Obj) return nullptr;
    auto it = o.find(k);
    return it == o.end() ? nullptr : it->second;
  }
  bool has(const std::string& k) const { return t == T::Obj && o.count(k) > 0; }
};

VP deep_copy(const VP& v);

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// numbers_as_float: encoding/json interface{} decoding (patterns). Otherwise unstructured decoding.
VP parse(const std::string& text, bool numbers_as_float);

// Compact JSON serialisation (Go json.Marshal-compatible for the value kinds used here).
std::string dump(const VP& v);

// Go fmt "%v" rendering of a decoded JSON value (maps print sorted: map[k:v ...]).
std::string go_v(const VP& v);

// helpers
std::string get_str(const VP& obj, const std::string& k);  // "" unless a string
bool truthy_path_str(const VP& obj, std::initializer_list<const char*> path, std::string* out);

}  // namespace oj
