// Product-side JSON reader (policies and resources).  Decoding semantics follow the reference inputs:
// resources decode like apimachinery unstructured (integral literals that fit int64 -> int64, other
// numbers -> float64); policy patterns decode like encoding/json into interface{} (all numbers
// float64); invalid UTF-8 / unpaired surrogates become U+FFFD; duplicate keys keep the last value.
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace pj {

enum class T : uint8_t { Null, Bool, Int, Float, Str, Arr, Obj };

struct Value {
  T t = T::Null;
  bool b = false;
  int64_t i = 0;
  double f = 0;
  std::string s;
  std::vector<Value> a;                           // Arr
  std::vector<std::pair<std::string, Value>> o;   // Obj (unique keys, input order of last occurrence)

  bool is(T x) const { return t == x; }
  bool nil() const { return t == T::Null; }
  const Value* get(const std::string& k) const {
    if (t != T::Obj) return nullptr;
    for (auto& kv : o) if (kv.first == k) return &kv.second;
    return nullptr;
  }
  Value* getm(const std::string& k) {
    if (t != T::Obj) return nullptr;
    for (auto& kv : o) if (kv.first == k) return &kv.second;
    return nullptr;
  }
  void set(const std::string& k, Value v) {
    for (auto& kv : o) if (kv.first == k) { kv.second = std::move(v); return; }
    o.emplace_back(k, std::move(v));
  }
  void erase(const std::string& k) {
    for (size_t n = 0; n < o.size(); n++) if (o[n].first == k) { o.erase(o.begin() + n); return; }
  }
  std::string str_or(const std::string& k, const std::string& d = "") const {
    const Value* v = get(k);
    return v && v->t == T::Str ? v->s : d;
  }
  static Value S(const std::string& s) { Value v; v.t = T::Str; v.s = s; return v; }
  static Value O() { Value v; v.t = T::Obj; return v; }
  static Value A() { Value v; v.t = T::Arr; return v; }
};

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

Value parse(const char* p, size_t n, bool numbers_as_float);
inline Value parse(const std::string& s, bool f) { return parse(s.data(), s.size(), f); }
// parse a JSON array (or newline-delimited JSON objects) into a list of documents
std::vector<Value> parse_many(const char* p, size_t n, bool numbers_as_float);
std::string dump(const Value& v);

// Go-compatible helpers shared by the compiler and the flattener
int utf8_dec(const char* s, size_t n, size_t i, uint32_t* r);
void utf8_put(std::string& out, uint32_t r);
bool go_parse_int64(const std::string& s, int64_t* out);
bool go_parse_float(const std::string& s, double* out);
std::string go_fmt_E(double f);   // strconv.FormatFloat(f,'E',-1,64)
std::string go_fmt_f6(double f);  // fmt %f
std::string go_fmt_g(double f);   // fmt %v
std::string go_fmt_json(double f);
std::string go_trim_space(const std::string& s);
bool go_parse_duration(const std::string& s, int64_t* ns);
// resource.ParseQuantity -> exact value rounded up to 1e-9 (BinarySI capped); returns 0 error, 1 ok (nano
// units in lo/hi int128), 2 ok but out of int128 nano range
int go_parse_quantity(const std::string& s, int64_t* lo, int64_t* hi);
bool go_wildcard(const std::string& pattern, const std::string& s);

}  // namespace pj
