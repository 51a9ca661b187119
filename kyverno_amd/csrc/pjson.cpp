// Product-side JSON reader and Go-compatible scalar helpers (see pjson.h).
#include "pjson.h"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>

namespace pj {

// ---------------------------------------------------------------- UTF-8
int utf8_dec(const char* s0, size_t n, size_t i, uint32_t* r) {
  const unsigned char* s = (const unsigned char*)s0;
  unsigned b0 = s[i];
  if (b0 < 0x80) { *r = b0; return 1; }
  size_t rem = n - i;
  auto c = [&](size_t k, unsigned lo, unsigned hi) { return k < rem && s[i + k] >= lo && s[i + k] <= hi; };
  if (b0 >= 0xC2 && b0 <= 0xDF && c(1, 0x80, 0xBF)) { *r = ((b0 & 0x1F) << 6) | (s[i + 1] & 0x3F); return 2; }
  if (b0 >= 0xE0 && b0 <= 0xEF && c(1, b0 == 0xE0 ? 0xA0 : 0x80, b0 == 0xED ? 0x9F : 0xBF) && c(2, 0x80, 0xBF)) {
    *r = ((b0 & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
    return 3;
  }
  if (b0 >= 0xF0 && b0 <= 0xF4 && c(1, b0 == 0xF0 ? 0x90 : 0x80, b0 == 0xF4 ? 0x8F : 0xBF) && c(2, 0x80, 0xBF) &&
      c(3, 0x80, 0xBF)) {
    *r = ((b0 & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
    return 4;
  }
  *r = 0xFFFD;
  return 1;
}

void utf8_put(std::string& out, uint32_t r) {
  if (r < 0x80) { out += (char)r; return; }
  if (r < 0x800) { out += (char)(0xC0 | (r >> 6)); out += (char)(0x80 | (r & 0x3F)); return; }
  if (r < 0x10000) { out += (char)(0xE0 | (r >> 12)); out += (char)(0x80 | ((r >> 6) & 0x3F)); out += (char)(0x80 | (r & 0x3F)); return; }
  out += (char)(0xF0 | (r >> 18)); out += (char)(0x80 | ((r >> 12) & 0x3F));
  out += (char)(0x80 | ((r >> 6) & 0x3F)); out += (char)(0x80 | (r & 0x3F));
}

// ---------------------------------------------------------------- parser
namespace {
struct P {
  const char* s;
  size_t n, i = 0;
  bool fl;
  [[noreturn]] void fail(const char* m) { throw Error(std::string("json: ") + m + " at offset " + std::to_string(i)); }
  void ws() { while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++; }
  static int hx(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  bool u4(size_t at, uint32_t* v) {
    if (at + 4 > n) return false;
    uint32_t x = 0;
    for (int k = 0; k < 4; k++) { int h = hx(s[at + k]); if (h < 0) return false; x = x * 16 + h; }
    *v = x;
    return true;
  }
  void str(std::string& out) {
    i++;  // opening quote
    out.clear();
    size_t run = i;
    for (;;) {
      if (i >= n) fail("unterminated string");
      unsigned char c = s[i];
      if (c == '"') { out.append(s + run, i - run); i++; return; }
      if (c == '\\') {
        out.append(s + run, i - run);
        i++;
        if (i >= n) fail("bad escape");
        char e = s[i++];
        switch (e) {
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'n': out += '\n'; break;
          case 'r': out += '\r'; break;
          case 't': out += '\t'; break;
          case 'u': {
            uint32_t r;
            if (!u4(i, &r)) fail("bad \\u escape");
            i += 4;
            if (r >= 0xD800 && r < 0xDC00) {
              uint32_t r2;
              if (i + 6 <= n && s[i] == '\\' && s[i + 1] == 'u' && u4(i + 2, &r2) && r2 >= 0xDC00 && r2 < 0xE000) {
                i += 6;
                r = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00);
              } else {
                r = 0xFFFD;
              }
            } else if (r >= 0xDC00 && r < 0xE000) {
              r = 0xFFFD;
            }
            utf8_put(out, r);
            break;
          }
          default: fail("bad escape");
        }
        run = i;
        continue;
      }
      if (c < 0x20) fail("control character in string");
      if (c < 0x80) { i++; continue; }
      uint32_t r;
      int w = utf8_dec(s, n, i, &r);
      if (r == 0xFFFD && w == 1) {
        out.append(s + run, i - run);
        utf8_put(out, 0xFFFD);
        i++;
        run = i;
        continue;
      }
      i += w;
    }
  }
  void num(Value& v) {
    size_t st = i;
    bool integral = true;
    if (s[i] == '-') i++;
    if (i >= n) fail("bad number");
    if (s[i] == '0') i++;
    else if (s[i] >= '1' && s[i] <= '9') while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    else fail("bad number");
    if (i < n && s[i] == '.') {
      integral = false;
      i++;
      if (i >= n || s[i] < '0' || s[i] > '9') fail("bad fraction");
      while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    }
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
      integral = false;
      i++;
      if (i < n && (s[i] == '+' || s[i] == '-')) i++;
      if (i >= n || s[i] < '0' || s[i] > '9') fail("bad exponent");
      while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    }
    std::string lit(s + st, i - st);
    if (!fl && integral && go_parse_int64(lit, &v.i)) { v.t = T::Int; return; }
    if (!go_parse_float(lit, &v.f)) fail("number out of range");
    v.t = T::Float;
  }
  void val(Value& v, int depth) {
    if (depth > 512) fail("nesting too deep");
    ws();
    if (i >= n) fail("unexpected end of input");
    char c = s[i];
    if (c == '{') {
      i++;
      v.t = T::Obj;
      ws();
      if (i < n && s[i] == '}') { i++; return; }
      std::string k;
      for (;;) {
        ws();
        if (i >= n || s[i] != '"') fail("expected key");
        str(k);
        ws();
        if (i >= n || s[i] != ':') fail("expected ':'");
        i++;
        Value x;
        val(x, depth + 1);
        bool dup = false;
        for (auto& kv : v.o) if (kv.first == k) { kv.second = std::move(x); dup = true; break; }
        if (!dup) v.o.emplace_back(k, std::move(x));
        ws();
        if (i < n && s[i] == ',') { i++; continue; }
        if (i < n && s[i] == '}') { i++; return; }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      i++;
      v.t = T::Arr;
      ws();
      if (i < n && s[i] == ']') { i++; return; }
      for (;;) {
        v.a.emplace_back();
        val(v.a.back(), depth + 1);
        ws();
        if (i < n && s[i] == ',') { i++; continue; }
        if (i < n && s[i] == ']') { i++; return; }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') { v.t = T::Str; str(v.s); return; }
    if (c == 't' && n - i >= 4 && memcmp(s + i, "true", 4) == 0) { i += 4; v.t = T::Bool; v.b = true; return; }
    if (c == 'f' && n - i >= 5 && memcmp(s + i, "false", 5) == 0) { i += 5; v.t = T::Bool; v.b = false; return; }
    if (c == 'n' && n - i >= 4 && memcmp(s + i, "null", 4) == 0) { i += 4; v.t = T::Null; return; }
    if (c == '-' || (c >= '0' && c <= '9')) { num(v); return; }
    fail("unexpected character");
  }
};
}  // namespace

Value parse(const char* p, size_t n, bool f) {
  P ps{p, n, 0, f};
  Value v;
  ps.val(v, 0);
  ps.ws();
  if (ps.i != n) ps.fail("trailing data");
  return v;
}

std::vector<Value> parse_many(const char* p, size_t n, bool f) {
  P ps{p, n, 0, f};
  ps.ws();
  std::vector<Value> out;
  if (ps.i < n && p[ps.i] == '[') {
    Value v;
    ps.val(v, 0);
    ps.ws();
    if (ps.i != n) ps.fail("trailing data");
    out = std::move(v.a);
    return out;
  }
  while (ps.i < n) {  // NDJSON / concatenated documents
    out.emplace_back();
    ps.val(out.back(), 0);
    ps.ws();
  }
  return out;
}

static void dump_str(std::string& o, const std::string& s) {
  o += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      case '<': o += "\\u003c"; break;
      case '>': o += "\\u003e"; break;
      case '&': o += "\\u0026"; break;
      default:
        if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); o += b; }
        else o += (char)c;
    }
  }
  o += '"';
}

static void dump_rec(std::string& o, const Value& v) {
  switch (v.t) {
    case T::Null: o += "null"; break;
    case T::Bool: o += v.b ? "true" : "false"; break;
    case T::Int: o += std::to_string(v.i); break;
    case T::Float: o += go_fmt_json(v.f); break;
    case T::Str: dump_str(o, v.s); break;
    case T::Arr:
      o += '[';
      for (size_t k = 0; k < v.a.size(); k++) { if (k) o += ','; dump_rec(o, v.a[k]); }
      o += ']';
      break;
    case T::Obj: {
      // encoding/json sorts map keys
      std::vector<const std::pair<std::string, Value>*> ks;
      for (auto& kv : v.o) ks.push_back(&kv);
      std::sort(ks.begin(), ks.end(), [](auto* a, auto* b) { return a->first < b->first; });
      o += '{';
      for (size_t k = 0; k < ks.size(); k++) {
        if (k) o += ',';
        dump_str(o, ks[k]->first);
        o += ':';
        dump_rec(o, ks[k]->second);
      }
      o += '}';
      break;
    }
  }
}

std::string dump(const Value& v) {
  std::string o;
  dump_rec(o, v);
  return o;
}

// ---------------------------------------------------------------- numbers
bool go_parse_int64(const std::string& s, int64_t* out) {
  size_t i = 0;
  bool neg = false;
  if (s.empty()) return false;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
  if (i >= s.size()) return false;
  unsigned __int128 v = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (unsigned)(s[i] - '0');
    if (v > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  *out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

static char lc(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }

bool go_parse_float(const std::string& s, double* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool sign = false;
  if (s[0] == '+' || s[0] == '-') { sign = true; i = 1; }
  std::string rest;
  for (size_t k = i; k < s.size(); k++) rest += lc(s[k]);
  if (rest == "inf" || rest == "infinity") { *out = s[0] == '-' ? -INFINITY : INFINITY; return true; }
  if (!sign && rest == "nan") { *out = NAN; return true; }
  bool hex = i + 1 < s.size() && s[i] == '0' && lc(s[i + 1]) == 'x';
  std::string clean = s.substr(0, i);
  if (hex) { clean += "0x"; i += 2; }
  bool digits = false, dot = false, underscore = false;
  for (; i < s.size(); i++) {
    char c = s[i];
    if (c == '_') { underscore = true; continue; }
    if (c == '.') { if (dot) return false; dot = true; clean += c; continue; }
    if ((c >= '0' && c <= '9') || (hex && lc(c) >= 'a' && lc(c) <= 'f')) { digits = true; clean += c; continue; }
    break;
  }
  if (!digits) return false;
  bool exp = false;
  if (i < s.size() && lc(s[i]) == (hex ? 'p' : 'e')) {
    clean += s[i++];
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) clean += s[i++];
    if (i >= s.size() || s[i] < '0' || s[i] > '9') return false;
    while (i < s.size() && ((s[i] >= '0' && s[i] <= '9') || s[i] == '_')) {
      if (s[i] == '_') underscore = true; else clean += s[i];
      i++;
    }
    exp = true;
  }
  if (i != s.size() || (hex && !exp)) return false;
  if (underscore) {  // strconv underscoreOK: '_' only between digits (base prefix counts as a digit)
    size_t k = (s[0] == '+' || s[0] == '-') ? 1 : 0;
    char saw = '^';
    if (hex) { k += 2; saw = '0'; }
    for (; k < s.size(); k++) {
      char c = s[k];
      if ((c >= '0' && c <= '9') || (hex && lc(c) >= 'a' && lc(c) <= 'f')) { saw = '0'; continue; }
      if (c == '_') { if (saw != '0') return false; saw = '_'; continue; }
      if (saw == '_') return false;
      saw = '!';
    }
    if (saw == '_') return false;
  }
  char* end = nullptr;
  double d = strtod(clean.c_str(), &end);
  if (end != clean.c_str() + clean.size() || std::isinf(d)) return false;
  *out = d;
  return true;
}

static void shortest(double f, std::string& digs, int& dp) {
  char buf[64];
  double a = std::fabs(f);
  for (int p = 1; p <= 17; p++) {
    snprintf(buf, sizeof buf, "%.*e", p - 1, a);
    if (strtod(buf, nullptr) == a || p == 17) break;
  }
  char* e = strchr(buf, 'e');
  digs.clear();
  for (char* q = buf; q < e; q++) if (*q != '.') digs += *q;
  while (digs.size() > 1 && digs.back() == '0') digs.pop_back();
  dp = atoi(e + 1) + 1;
}

static std::string exp2(int ex) {
  std::string d = std::to_string(ex < 0 ? -ex : ex);
  if (d.size() < 2) d = "0" + d;
  return std::string(ex < 0 ? "-" : "+") + d;
}

static std::string fixed(const std::string& d, int dp) {
  if (dp <= 0) return "0." + std::string(-dp, '0') + d;
  if ((int)d.size() <= dp) return d + std::string(dp - d.size(), '0');
  return d.substr(0, dp) + "." + d.substr(dp);
}

std::string go_fmt_E(double f) {
  if (std::isnan(f)) return "NaN";
  if (std::isinf(f)) return f > 0 ? "+Inf" : "-Inf";
  std::string sg = std::signbit(f) ? "-" : "";
  if (f == 0) return sg + "0E+00";
  std::string d; int dp;
  shortest(f, d, dp);
  return sg + d.substr(0, 1) + (d.size() > 1 ? "." + d.substr(1) : "") + "E" + exp2(dp - 1);
}

std::string go_fmt_g(double f) {
  if (std::isnan(f)) return "NaN";
  if (std::isinf(f)) return f > 0 ? "+Inf" : "-Inf";
  std::string sg = std::signbit(f) ? "-" : "";
  if (f == 0) return sg + "0";
  std::string d; int dp;
  shortest(f, d, dp);
  int ex = dp - 1;
  if (ex < -4 || ex >= 6) return sg + d.substr(0, 1) + (d.size() > 1 ? "." + d.substr(1) : "") + "e" + exp2(ex);
  return sg + fixed(d, dp);
}

std::string go_fmt_json(double f) {
  if (f == 0) return std::signbit(f) ? "-0" : "0";
  std::string sg = f < 0 ? "-" : "";
  std::string d; int dp;
  shortest(f, d, dp);
  double a = std::fabs(f);
  if (a < 1e-6 || a >= 1e21) {
    int ex = dp - 1;
    return sg + d.substr(0, 1) + (d.size() > 1 ? "." + d.substr(1) : "") + "e" + (ex < 0 ? "-" : "+") + std::to_string(ex < 0 ? -ex : ex);
  }
  return sg + fixed(d, dp);
}

std::string go_fmt_f6(double f) {
  if (std::isnan(f)) return "NaN";
  if (std::isinf(f)) return f > 0 ? "+Inf" : "-Inf";
  char buf[400];
  snprintf(buf, sizeof buf, "%f", f);
  return buf;
}

static bool space_rune(uint32_t r) {
  return r == '\t' || r == '\n' || r == '\v' || r == '\f' || r == '\r' || r == ' ' || r == 0x85 || r == 0xA0 ||
         r == 0x1680 || (r >= 0x2000 && r <= 0x200a) || r == 0x2028 || r == 0x2029 || r == 0x202f || r == 0x205f ||
         r == 0x3000;
}

std::string go_trim_space(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e) {
    uint32_t r;
    int w = utf8_dec(s.data(), s.size(), b, &r);
    if (!space_rune(r)) break;
    b += w;
  }
  while (e > b) {
    size_t k = e - 1;
    while (k > b && ((unsigned char)s[k] & 0xC0) == 0x80 && e - k < 4) k--;
    uint32_t r;
    int w = utf8_dec(s.data(), s.size(), k, &r);
    if (k + (size_t)w != e) { k = e - 1; r = 0xFFFD; }
    if (!space_rune(r)) break;
    e = k;
  }
  return s.substr(b, e - b);
}

bool go_parse_duration(const std::string& orig, int64_t* out) {
  const uint64_t LIM = (uint64_t)1 << 63;
  size_t i = 0;
  bool neg = false;
  if (!orig.empty() && (orig[0] == '-' || orig[0] == '+')) { neg = orig[0] == '-'; i = 1; }
  if (orig.size() - i == 1 && orig[i] == '0') { *out = 0; return true; }
  if (i == orig.size()) return false;
  unsigned __int128 total = 0;
  while (i < orig.size()) {
    char c0 = orig[i];
    if (!(c0 == '.' || (c0 >= '0' && c0 <= '9'))) return false;
    uint64_t v = 0, f = 0;
    double scale = 1;
    size_t st = i;
    while (i < orig.size() && orig[i] >= '0' && orig[i] <= '9') {
      if (v > LIM / 10) return false;
      v = v * 10 + (uint64_t)(orig[i] - '0');
      if (v > LIM) return false;
      i++;
    }
    bool pre = i != st, post = false;
    if (i < orig.size() && orig[i] == '.') {
      i++;
      size_t fs = i;
      bool of = false;
      while (i < orig.size() && orig[i] >= '0' && orig[i] <= '9') {
        if (!of) {
          if (f > (LIM - 1) / 10) of = true;
          else {
            uint64_t y = f * 10 + (uint64_t)(orig[i] - '0');
            if (y > LIM) of = true; else { f = y; scale *= 10; }
          }
        }
        i++;
      }
      post = i != fs;
    }
    if (!pre && !post) return false;
    size_t us = i;
    while (i < orig.size() && orig[i] != '.' && !(orig[i] >= '0' && orig[i] <= '9')) i++;
    if (i == us) return false;
    std::string u = orig.substr(us, i - us);
    uint64_t unit;
    if (u == "ns") unit = 1;
    else if (u == "us" || u == "\xC2\xB5s" || u == "\xCE\xBCs") unit = 1000;
    else if (u == "ms") unit = 1000000;
    else if (u == "s") unit = 1000000000ULL;
    else if (u == "m") unit = 60000000000ULL;
    else if (u == "h") unit = 3600000000000ULL;
    else return false;
    if (v > LIM / unit) return false;
    v *= unit;
    if (f > 0) {
      v += (uint64_t)((double)f * ((double)unit / scale));
      if (v > LIM) return false;
    }
    total += v;
    if (total > LIM) return false;
  }
  if (neg) { *out = (int64_t)(-(__int128)total); return true; }
  if (total > (unsigned __int128)INT64_MAX) return false;
  *out = (int64_t)total;
  return true;
}

// ParseQuantity -> exact value in nano units (int128), rounded up (magnitude) to 1e-9; BinarySI capped.
int go_parse_quantity(const std::string& str, int64_t* lo, int64_t* hi) {
  *lo = 0; *hi = 0;
  if (str.empty()) return 0;
  if (str == "0") return 1;
  size_t pos = 0, end = str.size();
  bool positive = true;
  if (str[0] == '-') { positive = false; pos++; }
  else if (str[0] == '+') pos++;
  std::string num, denom, suf;
  bool done = false;
  while (pos < end && str[pos] == '0') pos++;
  if (pos >= end) { num = "0"; done = true; }
  if (!done) {
    size_t st = pos;
    while (pos < end && str[pos] >= '0' && str[pos] <= '9') pos++;
    num = str.substr(st, pos - st);
    if (pos >= end) done = true;
  }
  if (!done) {
    if (num.empty()) num = "0";
    if (pos < end && str[pos] == '.') {
      pos++;
      size_t st = pos;
      while (pos < end && str[pos] >= '0' && str[pos] <= '9') pos++;
      denom = str.substr(st, pos - st);
      if (pos >= end) done = true;
    }
  }
  if (!done) {
    size_t ss = pos;
    while (pos < end && strchr("eEinumkKMGTP", str[pos])) pos++;
    if (pos < end) {
      if (str[pos] == '-' || str[pos] == '+') pos++;
      while (pos < end && str[pos] >= '0' && str[pos] <= '9') pos++;
      if (pos < end) return 0;  // ErrFormatWrong
    }
    suf = str.substr(ss);
  }
  if (num.empty()) num = "0";
  // suffix
  int64_t ex = 0;
  bool bin = false;
  static const char* ds[] = {"n", "u", "m", "", "k", "M", "G", "T", "P", "E"};
  static const int de[] = {-9, -6, -3, 0, 3, 6, 9, 12, 15, 18};
  static const char* bs[] = {"Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
  bool ok = false;
  for (int k = 0; k < 10 && !ok; k++) if (suf == ds[k]) { ex = de[k]; ok = true; }
  for (int k = 0; k < 6 && !ok; k++) if (suf == bs[k]) { ex = 10 * (k + 1); bin = true; ok = true; }
  if (!ok && suf.size() > 1 && (suf[0] == 'e' || suf[0] == 'E')) {
    int64_t pe;
    if (!go_parse_int64(suf.substr(1), &pe)) return 0;
    ex = (int32_t)pe;
    ok = true;
  }
  if (!ok) return 0;
  // digits D = num+denom (value = D * 10^-len(denom)), nano = D * base^ex * 10^(9-len(denom))
  std::string D = num + denom;
  size_t z = 0;
  while (z + 1 < D.size() && D[z] == '0') z++;
  D = D.substr(z);
  int64_t e10 = 9 - (int64_t)denom.size() + (bin ? 0 : ex);
  using U = unsigned __int128;
  const U MAXM = ~(U)0 >> 1;  // int128 magnitude bound
  bool sticky = false;
  if (e10 < 0) {
    int64_t drop = -e10;
    if ((int64_t)D.size() <= drop) {
      for (char c : D) if (c != '0') sticky = true;
      D = "0";
    } else {
      for (size_t k = D.size() - drop; k < D.size(); k++) if (D[k] != '0') sticky = true;
      D = D.substr(0, D.size() - drop);
    }
    e10 = 0;
  }
  U m = 0;
  for (char c : D) {
    if (m > MAXM / 10) return 2;
    m = m * 10 + (unsigned)(c - '0');
  }
  if (bin) {
    for (int64_t k = 0; k < ex; k++) { if (m > MAXM / 2) return 2; m *= 2; }
  }
  for (int64_t k = 0; k < e10; k++) {
    if (m == 0) break;
    if (m > MAXM / 10) return 2;
    m *= 10;
  }
  if (bin && sticky) {
    // BinarySI with a long fraction: the 2^ex factor was applied after the truncation; redo exactly
    return 2;
  }
  if (sticky) m += 1;
  if (bin) {
    U cap = (U)INT64_MAX * (U)1000000000ULL;
    if (m > cap) m = cap;
  }
  __int128 v = positive ? (__int128)m : -(__int128)m;
  *lo = (int64_t)(uint64_t)((unsigned __int128)v);
  *hi = (int64_t)(v >> 64);
  return 1;
}

bool go_wildcard(const std::string& pat, const std::string& s) {
  if (pat.empty()) return s.empty();
  if (pat == "*") return true;
  std::vector<uint32_t> p, t;
  for (size_t i = 0; i < pat.size();) { uint32_t r; i += utf8_dec(pat.data(), pat.size(), i, &r); p.push_back(r); }
  for (size_t i = 0; i < s.size();) { uint32_t r; i += utf8_dec(s.data(), s.size(), i, &r); t.push_back(r); }
  size_t pi = 0, si = 0, star = (size_t)-1, mark = 0;
  while (si < t.size()) {
    if (pi < p.size() && p[pi] != '*' && (p[pi] == '?' || p[pi] == t[si])) { pi++; si++; }
    else if (pi < p.size() && p[pi] == '*') { star = pi++; mark = si; }
    else if (star != (size_t)-1) { pi = star + 1; si = ++mark; }
    else return false;
  }
  while (pi < p.size() && p[pi] == '*') pi++;
  return pi == p.size();
}

}  // namespace pj
