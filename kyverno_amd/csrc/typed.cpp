// Whole-object typed decode of the resources a podSecurity rule reads (pkg/engine/validation.go:481-532 getSpec:
// json.Unmarshal into corev1.Pod / appsv1.Deployment / batchv1.CronJob; an error there is the rule's error status,
// :538-540). Done once per resource by the flattener over its node table (RF_PSS_DEC_ERR), against the field types
// of k8s_types.h, with encoding/json's rules: null is the zero value of any type; a string, bool or number only into
// a field of that kind (integers: a literal strconv.ParseInt accepts, in the field's range); objects into structs
// (unknown keys ignored, keys matched exactly, else ASCII case-insensitively) and maps; arrays into slices; and the
// UnmarshalJSON methods of resource.Quantity (ParseQuantity of the string or number literal, trimmed),
// intstr.IntOrString (a string, else an int32) and metav1.Time (a string that time.Parse(RFC3339) accepts).
#include <cctype>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "k8s_types.h"
#include "kyv_host.h"
#include "pjson.h"

namespace kyv {
namespace {

enum TK : uint8_t { K_S, K_B, K_I32, K_I64, K_Q, K_IOS, K_T, K_ANY, K_SLICE, K_MAP, K_STRUCT };
struct TRef { TK k; uint32_t x; };  // K_SLICE / K_MAP: element type index (Schema::elems); K_STRUCT: struct index
struct Field { std::string name; TRef t; };
struct Struct {
  std::string name, base;
  std::vector<Field> fields;
  std::unordered_map<std::string, uint32_t> folded;  // lower-case field name -> field (first in order)
};
struct Schema {
  std::vector<Struct> structs;
  std::vector<TRef> elems;
  std::unordered_map<std::string, uint32_t> by_name;
  std::vector<std::string> names;                     // distinct field names
  std::vector<std::vector<int32_t>> field_of_name;    // [struct][name] -> field or -1
};

std::string lower(const std::string& s) {
  std::string o = s;
  for (auto& c : o) c = (char)std::tolower((unsigned char)c);
  return o;
}

struct SchemaParser {
  const char* p;
  Schema& S;
  std::vector<std::vector<std::pair<std::string, std::string>>> raw;  // per struct: (field, type text)
  void ws() { while (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r') p++; }
  std::string ident() {
    std::string o;
    while (std::isalnum((unsigned char)*p) || *p == '_') o += *p++;
    if (o.empty()) throw std::runtime_error(std::string("k8s_types: identifier expected at ") + std::string(p, 20));
    return o;
  }
  std::string type_text() {
    std::string o;
    int depth = 0;
    while (*p && (depth > 0 || (*p != ' ' && *p != '}'))) {
      if (*p == '[' || *p == '{') depth++;
      if (*p == ']' || (*p == '}' && depth > 0)) depth--;
      o += *p++;
    }
    return o;
  }
  void run() {
    for (ws(); *p; ws()) {
      Struct st;
      st.name = ident();
      if (*p == ':') { p++; st.base = ident(); }
      if (*p++ != '{') throw std::runtime_error("k8s_types: '{' expected after " + st.name);
      std::vector<std::pair<std::string, std::string>> fs;
      for (ws(); *p != '}'; ws()) {
        std::string f = ident();
        if (*p++ != ':') throw std::runtime_error("k8s_types: ':' expected after " + f);
        fs.emplace_back(f, type_text());
      }
      p++;
      S.by_name[st.name] = (uint32_t)S.structs.size();
      S.structs.push_back(std::move(st));
      raw.push_back(std::move(fs));
    }
    std::vector<int> done(S.structs.size(), 0);
    for (size_t i = 0; i < S.structs.size(); i++) resolve(i, done);
    std::unordered_map<std::string, uint32_t> nid;
    for (auto& st : S.structs)
      for (auto& f : st.fields)
        if (!nid.count(f.name)) { nid[f.name] = (uint32_t)S.names.size(); S.names.push_back(f.name); }
    S.field_of_name.assign(S.structs.size(), std::vector<int32_t>(S.names.size(), -1));
    for (size_t i = 0; i < S.structs.size(); i++) {
      Struct& st = S.structs[i];
      for (size_t j = 0; j < st.fields.size(); j++) {
        S.field_of_name[i][nid[st.fields[j].name]] = (int32_t)j;
        st.folded.emplace(lower(st.fields[j].name), (uint32_t)j);  // emplace keeps the first
      }
    }
  }
  void resolve(size_t i, std::vector<int>& done) {
    if (done[i] == 2) return;
    if (done[i] == 1) throw std::runtime_error("k8s_types: embedding cycle at " + S.structs[i].name);
    done[i] = 1;
    Struct& st = S.structs[i];
    std::vector<Field> fs;
    if (!st.base.empty()) {
      auto it = S.by_name.find(st.base);
      if (it == S.by_name.end()) throw std::runtime_error("k8s_types: unknown base " + st.base);
      resolve(it->second, done);
      fs = S.structs[it->second].fields;
    }
    for (auto& f : raw[i]) {
      const char* q = f.second.c_str();
      fs.push_back(Field{f.first, type(q)});
    }
    S.structs[i].fields = std::move(fs);
    done[i] = 2;
  }
  TRef type(const char*& q) {
    if (*q == '[' || *q == '{') {
      const char close = *q == '[' ? ']' : '}';
      const TK k = *q == '[' ? K_SLICE : K_MAP;
      q++;
      TRef e = type(q);
      if (*q++ != close) throw std::runtime_error("k8s_types: unbalanced type");
      S.elems.push_back(e);
      return TRef{k, (uint32_t)S.elems.size() - 1};
    }
    std::string n;
    while (std::isalnum((unsigned char)*q) || *q == '_') n += *q++;
    static const std::unordered_map<std::string, TK> prim = {{"s", K_S}, {"b", K_B}, {"i32", K_I32}, {"i64", K_I64},
                                                             {"q", K_Q}, {"ios", K_IOS}, {"t", K_T}, {"any", K_ANY}};
    auto pit = prim.find(n);
    if (pit != prim.end()) return TRef{pit->second, 0};
    auto it = S.by_name.find(n);
    if (it == S.by_name.end()) throw std::runtime_error("k8s_types: unknown type " + n);
    return TRef{K_STRUCT, it->second};
  }
};

const Schema& schema() {
  static Schema S;
  static std::once_flag once;
  std::call_once(once, [] { SchemaParser{k8st::kSchema, S, {}}.run(); });
  return S;
}

// time.Parse(time.RFC3339, s) acceptance (Go's general parser for the layout "2006-01-02T15:04:05Z07:00": 4-digit
// year, 2-digit month / day / minute / second, 1- or 2-digit hour, optional ',' or '.' fraction after the seconds,
// then 'Z' or a +hh:mm / -hh:mm offset (hours <= 24, minutes <= 60), nothing after; the day checked against the month)
bool rfc3339_ok(const std::string& v) {
  size_t i = 0;
  const size_t n = v.size();
  auto dig = [&](size_t k) { return k < n && v[k] >= '0' && v[k] <= '9'; };
  auto num2 = [&](int* out) {  // getnum(fixed=true)
    if (!dig(i) || !dig(i + 1)) return false;
    *out = (v[i] - '0') * 10 + (v[i + 1] - '0');
    i += 2;
    return true;
  };
  auto lit = [&](char c) { if (i < n && v[i] == c) { i++; return true; } return false; };
  if (!(dig(0) && dig(1) && dig(2) && dig(3))) return false;
  const int year = (v[0] - '0') * 1000 + (v[1] - '0') * 100 + (v[2] - '0') * 10 + (v[3] - '0');
  i = 4;
  int month, day, hour, minute, second;
  if (!lit('-') || !num2(&month) || month < 1 || month > 12) return false;
  if (!lit('-') || !num2(&day)) return false;
  if (!lit('T')) return false;
  if (!dig(i)) return false;  // stdHour: getnum(fixed=false)
  hour = v[i] - '0';
  i++;
  if (dig(i)) { hour = hour * 10 + (v[i] - '0'); i++; }
  if (hour >= 24) return false;
  if (!lit(':') || !num2(&minute) || minute >= 60) return false;
  if (!lit(':') || !num2(&second) || second >= 60) return false;
  if (i + 1 < n && (v[i] == '.' || v[i] == ',') && dig(i + 1)) {
    i += 2;
    while (dig(i)) i++;
  }
  if (i < n && v[i] == 'Z') {
    i++;
  } else {
    if (n - i < 6 || v[i + 3] != ':' || (v[i] != '+' && v[i] != '-')) return false;
    if (!dig(i + 1) || !dig(i + 2) || !dig(i + 4) || !dig(i + 5)) return false;
    const int hr = (v[i + 1] - '0') * 10 + (v[i + 2] - '0'), mm = (v[i + 4] - '0') * 10 + (v[i + 5] - '0');
    if (hr > 24 || mm > 60) return false;
    i += 6;
  }
  if (i != n) return false;
  static const int mdays[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  int dim = mdays[month - 1];
  if (month == 2 && year % 4 == 0 && (year % 100 != 0 || year % 400 == 0)) dim = 29;
  return day >= 1 && day <= dim;
}

bool quantity_ok(std::string s) {  // Quantity.UnmarshalJSON: ParseQuantity(strings.TrimSpace(...))
  size_t a = 0, b = s.size();
  auto sp = [](char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; };
  while (a < b && sp(s[a])) a++;
  while (b > a && sp(s[b - 1])) b--;
  int64_t lo, hi;
  return pj::go_parse_quantity(s.substr(a, b - a), &lo, &hi) != 0;
}

}  // namespace

TypedDecoder::TypedDecoder(const std::function<uint32_t(const std::string&)>& find_sid) {
  const Schema& S = schema();
  for (uint32_t i = 0; i < S.names.size(); i++) {
    const uint32_t sid = find_sid(S.names[i]);
    if (sid != NONE) name_of_sid.emplace(sid, i);
  }
}

int TypedDecoder::decode(const Node* R, const std::vector<std::string>& strs, int target) const {
  const Schema& S = schema();
  static const char* roots[] = {"Pod", "Deployment", "CronJob"};
  const uint32_t root = S.by_name.at(roots[target]);
  struct Item { uint32_t node; TRef t; };
  std::vector<Item> stack;
  stack.push_back({0u, TRef{K_STRUCT, root}});
  bool folded = false;
  while (!stack.empty()) {
    const Item it = stack.back();
    stack.pop_back();
    const Node& x = R[it.node];
    const uint32_t ty = node_type(x);
    if (ty == N_NULL) continue;  // the zero value, whatever the type
    switch (it.t.k) {
      case K_S: if (ty != N_STR) return DEC_ERR; break;
      case K_B: if (ty != N_TRUE && ty != N_FALSE) return DEC_ERR; break;
      case K_I32: case K_I64: case K_IOS: {
        if (it.t.k == K_IOS && ty == N_STR) break;
        if (ty != N_INT) return DEC_ERR;  // floats, exponents and literals beyond int64 fail strconv.ParseInt
        const int64_t val = (int64_t)((uint64_t)x.a | ((uint64_t)x.b << 32));
        if (it.t.k != K_I64 && (val < INT32_MIN || val > INT32_MAX)) return DEC_ERR;
        break;
      }
      case K_Q:
        if (ty == N_INT || ty == N_FLOAT) break;  // a JSON number literal is a quantity
        if (ty != N_STR || !quantity_ok(strs[x.a])) return DEC_ERR;
        break;
      case K_T: if (ty != N_STR || !rfc3339_ok(strs[x.a])) return DEC_ERR; break;
      case K_ANY: break;
      case K_SLICE:
        if (ty != N_ARR) return DEC_ERR;
        for (uint32_t j = 0; j < x.b; j++) stack.push_back({x.a + j, S.elems[it.t.x]});
        break;
      case K_MAP:
        if (ty != N_MAP) return DEC_ERR;
        for (uint32_t j = 0; j < x.b; j++) stack.push_back({x.a + j, S.elems[it.t.x]});
        break;
      case K_STRUCT: {
        if (ty != N_MAP) return DEC_ERR;
        const Struct& st = S.structs[it.t.x];
        for (uint32_t j = 0; j < x.b; j++) {
          const uint32_t key = node_key(R[x.a + j]);
          int32_t f = -1;
          auto nit = name_of_sid.find(key);
          if (nit != name_of_sid.end()) f = S.field_of_name[it.t.x][nit->second];
          if (f < 0) {  // no exact match: encoding/json's case-insensitive match
            auto fit = st.folded.find(lower(strs[key]));
            if (fit == st.folded.end()) continue;  // unknown field: ignored
            f = (int32_t)fit->second;
            folded = true;
          }
          stack.push_back({x.a + j, st.fields[f].t});
        }
        break;
      }
    }
  }
  return folded ? DEC_FOLD : DEC_OK;
}

}  // namespace kyv
