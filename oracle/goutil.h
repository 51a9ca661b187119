// ORACLE — test infrastructure only (see ojson.h header).
//
// Go-runtime / third-party primitives the reference's validate path relies on, restated from their
// published algorithms (the modules are not present under /root/reference; pinned versions from
// /root/reference/go.mod):
//   * unicode/utf8.DecodeRuneInString (Go 1.19 stdlib)
//   * github.com/IGLOU-EU/go-wildcard v1.0.3 Match  (pkg/utils/wildcard/match.go:7-9)
//   * strconv.ParseInt / ParseFloat / FormatFloat('E'|'g'|'f', -1)  (pkg/engine/pattern/pattern.go:75,106,272,311)
//   * time.ParseDuration (pattern.go:214,218)
//   * k8s.io/apimachinery v0.26.1 resource.ParseQuantity + Quantity.Cmp (pattern.go:240-247)
//   * strconv.Quote (%q in pod-security-admission messages)
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cerrno>
#include <string>
#include <vector>

namespace gou {

inline void append_utf8(std::string& out, uint32_t r) {
  if (r < 0x80) out += (char)r;
  else if (r < 0x800) { out += (char)(0xC0 | (r >> 6)); out += (char)(0x80 | (r & 0x3F)); }
  else if (r < 0x10000) {
    out += (char)(0xE0 | (r >> 12)); out += (char)(0x80 | ((r >> 6) & 0x3F)); out += (char)(0x80 | (r & 0x3F));
  } else {
    out += (char)(0xF0 | (r >> 18)); out += (char)(0x80 | ((r >> 12) & 0x3F));
    out += (char)(0x80 | ((r >> 6) & 0x3F)); out += (char)(0x80 | (r & 0x3F));
  }
}

// utf8.DecodeRuneInString: returns width; invalid -> (0xFFFD, 1)
inline int utf8_decode(const std::string& s, size_t i, uint32_t& r) {
  size_t n = s.size() - i;
  unsigned char b0 = s[i];
  if (b0 < 0x80) { r = b0; return 1; }
  auto cont = [&](size_t k, unsigned lo, unsigned hi) {
    if (k >= n) return false;
    unsigned char c = s[i + k];
    return c >= lo && c <= hi;
  };
  if (b0 >= 0xC2 && b0 <= 0xDF) {
    if (cont(1, 0x80, 0xBF)) { r = ((b0 & 0x1F) << 6) | (s[i + 1] & 0x3F); return 2; }
  } else if (b0 >= 0xE0 && b0 <= 0xEF) {
    unsigned lo = 0x80, hi = 0xBF;
    if (b0 == 0xE0) lo = 0xA0;
    if (b0 == 0xED) hi = 0x9F;
    if (cont(1, lo, hi) && cont(2, 0x80, 0xBF)) {
      r = ((b0 & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
      return 3;
    }
  } else if (b0 >= 0xF0 && b0 <= 0xF4) {
    unsigned lo = 0x80, hi = 0xBF;
    if (b0 == 0xF0) lo = 0x90;
    if (b0 == 0xF4) hi = 0x8F;
    if (cont(1, lo, hi) && cont(2, 0x80, 0xBF) && cont(3, 0x80, 0xBF)) {
      r = ((b0 & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
      return 4;
    }
  }
  r = 0xFFFD;
  return 1;
}

inline std::vector<uint32_t> runes(const std::string& s) {
  std::vector<uint32_t> out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size();) {
    uint32_t r;
    i += utf8_decode(s, i, r);
    out.push_back(r);
  }
  return out;
}

// go-wildcard v1.0.3: "" matches only ""; "*" matches all; '*' any rune run, '?' exactly one rune.
// The backtracking recursion of the library decides plain glob-language membership, which this
// iterative matcher decides too.
inline bool wildcard_match(const std::string& pattern, const std::string& name) {
  if (pattern.empty()) return name.empty();
  if (pattern == "*") return true;
  std::vector<uint32_t> p = runes(pattern), s = runes(name);
  size_t pi = 0, si = 0, star = (size_t)-1, mark = 0;
  while (si < s.size()) {
    if (pi < p.size() && p[pi] != '*' && (p[pi] == '?' || p[pi] == s[si])) { pi++; si++; }
    else if (pi < p.size() && p[pi] == '*') { star = pi++; mark = si; }
    else if (star != (size_t)-1) { pi = star + 1; si = ++mark; }
    else return false;
  }
  while (pi < p.size() && p[pi] == '*') pi++;
  return pi == p.size();
}

inline bool contains_wildcard(const std::string& v) {
  return v.find('*') != std::string::npos || v.find('?') != std::string::npos;
}

// strconv.ParseInt(s, 10, 64)
inline bool parse_int64(const std::string& s, int64_t& out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
  if (i >= s.size()) return false;
  unsigned __int128 v = 0;
  for (; i < s.size(); i++) {
    char c = s[i];
    if (c < '0' || c > '9') return false;
    v = v * 10 + (c - '0');
    if (v > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

inline char lower(char c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

inline bool underscore_ok(std::string s) {
  char saw = '^';
  size_t i = 0;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) s = s.substr(1);
  bool hex = false;
  if (s.size() >= 2 && s[0] == '0' && (lower(s[1]) == 'b' || lower(s[1]) == 'o' || lower(s[1]) == 'x')) {
    i = 2; saw = '0'; hex = lower(s[1]) == 'x';
  }
  for (; i < s.size(); i++) {
    if ((s[i] >= '0' && s[i] <= '9') || (hex && lower(s[i]) >= 'a' && lower(s[i]) <= 'f')) { saw = '0'; continue; }
    if (s[i] == '_') { if (saw != '0') return false; saw = '_'; continue; }
    if (saw == '_') return false;
    saw = '!';
  }
  return saw != '_';
}

// strconv.ParseFloat(s, 64): returns false on syntax error or overflow (ErrRange).
inline bool parse_float(const std::string& s, double& out) {
  if (s.empty()) return false;
  // specials
  {
    size_t i = 0;
    int sign = 1;
    bool hadsign = false;
    if (s[0] == '+' || s[0] == '-') { sign = s[0] == '-' ? -1 : 1; i = 1; hadsign = true; }
    std::string rest;
    for (size_t k = i; k < s.size(); k++) rest += lower(s[k]);
    if (rest == "inf" || rest == "infinity") { out = sign * INFINITY; return true; }
    if (!hadsign && rest == "nan") { out = NAN; return true; }
  }
  size_t i = 0;
  if (s[0] == '+' || s[0] == '-') i = 1;
  bool hex = false;
  if (i + 1 < s.size() && s[i] == '0' && lower(s[i + 1]) == 'x') { hex = true; i += 2; }
  bool sawdigits = false, sawdot = false, sawexp = false, underscores = false;
  std::string clean = s.substr(0, hex ? i : (s[0] == '+' || s[0] == '-') ? 1 : 0);
  for (; i < s.size(); i++) {
    char c = s[i];
    if (c == '_') { underscores = true; continue; }
    if (c == '.') { if (sawdot) return false; sawdot = true; clean += c; continue; }
    if ((c >= '0' && c <= '9') || (hex && lower(c) >= 'a' && lower(c) <= 'f')) { sawdigits = true; clean += c; continue; }
    break;
  }
  if (!sawdigits) return false;
  if (i < s.size() && lower(s[i]) == (hex ? 'p' : 'e')) {
    clean += s[i];
    i++;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) { clean += s[i]; i++; }
    if (i >= s.size() || s[i] < '0' || s[i] > '9') return false;
    while (i < s.size() && ((s[i] >= '0' && s[i] <= '9') || s[i] == '_')) {
      if (s[i] == '_') underscores = true; else clean += s[i];
      i++;
    }
    sawexp = true;
  }
  if (i != s.size()) return false;
  if (hex && !sawexp) return false;
  if (underscores && !underscore_ok(s)) return false;
  errno = 0;
  char* end = nullptr;
  double d = strtod(clean.c_str(), &end);
  if (end != clean.c_str() + clean.size()) return false;
  if (std::isinf(d)) return false;  // overflow -> ErrRange
  out = d;
  return true;
}

// shortest round-trip decimal digits of |f| (f finite, nonzero): digits and decimal exponent such that
// value = 0.d1d2...dn * 10^dp
inline void shortest_digits(double f, std::string& digits, int& dp) {
  char buf[64];
  double a = std::fabs(f);
  for (int p = 1; p <= 17; p++) {
    snprintf(buf, sizeof buf, "%.*e", p - 1, a);
    if (strtod(buf, nullptr) == a || p == 17) {
      // parse "d.ddde[+-]XX"
      digits.clear();
      char* e = strchr(buf, 'e');
      for (char* q = buf; q < e; q++) if (*q != '.') digits += *q;
      int ex = atoi(e + 1);
      while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
      dp = ex + 1;
      return;
    }
  }
}

inline std::string exp_str(int ex, int mindigits = 2) {
  std::string s = ex < 0 ? "-" : "+";
  std::string d = std::to_string(ex < 0 ? -ex : ex);
  while ((int)d.size() < mindigits) d = "0" + d;
  return s + d;
}

// strconv.FormatFloat(f, 'E', -1, 64)
inline std::string format_float_E(double f) {
  if (std::isnan(f)) return "NaN";
  if (std::isinf(f)) return f > 0 ? "+Inf" : "-Inf";
  std::string sign = std::signbit(f) ? "-" : "";
  if (f == 0) return sign + "0E+00";
  std::string d; int dp;
  shortest_digits(f, d, dp);
  std::string m = d.substr(0, 1);
  if (d.size() > 1) m += "." + d.substr(1);
  return sign + m + "E" + exp_str(dp - 1);
}

// %f with shortest digits (used by 'g' and json 'f')
inline std::string fixed_from_digits(const std::string& d, int dp) {
  std::string out;
  if (dp <= 0) {
    out = "0";
    out += ".";
    for (int k = 0; k < -dp; k++) out += '0';
    out += d;
  } else if ((int)d.size() <= dp) {
    out = d;
    for (int k = (int)d.size(); k < dp; k++) out += '0';
  } else {
    out = d.substr(0, dp) + "." + d.substr(dp);
  }
  return out;
}

// strconv.FormatFloat(f, 'g', -1, 64) (== fmt %v of float64)
inline std::string format_float_g(double f) {
  if (std::isnan(f)) return "NaN";
  if (std::isinf(f)) return f > 0 ? "+Inf" : "-Inf";
  std::string sign = std::signbit(f) ? "-" : "";
  if (f == 0) return sign + "0";
  std::string d; int dp;
  shortest_digits(f, d, dp);
  int ex = dp - 1;
  if (ex < -4 || ex >= 21 /*eprec, shortest: max(nd,21)? see below*/) {}
  // strconv: eprec = 6 when shortest; but if eprec > nd && nd >= dp -> eprec = nd happens first and
  // is then overridden by shortest -> 6.  However %v of large integers prints e.g. 1e+06.
  int eprec = 6;
  if (ex < -4 || ex >= eprec) {
    std::string m = d.substr(0, 1);
    if (d.size() > 1) m += "." + d.substr(1);
    return sign + m + "e" + exp_str(ex);
  }
  return sign + fixed_from_digits(d, dp);
}

// encoding/json float64 encoding
inline std::string format_float_json(double f) {
  if (f == 0) return std::signbit(f) ? "-0" : "0";
  std::string sign = f < 0 ? "-" : "";
  double a = std::fabs(f);
  std::string d; int dp;
  shortest_digits(f, d, dp);
  if (a < 1e-6 || a >= 1e21) {
    std::string m = d.substr(0, 1);
    if (d.size() > 1) m += "." + d.substr(1);
    int ex = dp - 1;
    std::string es = ex < 0 ? "-" : "+";
    es += std::to_string(ex < 0 ? -ex : ex);  // json cleans e-09 -> e-9; e+21 stays 2 digits anyway
    return sign + m + "e" + es;
  }
  return sign + fixed_from_digits(d, dp);
}

// fmt "%f"
inline std::string format_float_f6(double f) {
  if (std::isnan(f)) return "NaN";
  if (std::isinf(f)) return f > 0 ? "+Inf" : "-Inf";
  char buf[400];
  snprintf(buf, sizeof buf, "%f", f);
  return buf;
}

// time.ParseDuration
inline bool parse_duration(const std::string& orig, int64_t& out) {
  std::string s = orig;
  unsigned __int128 d = 0;
  bool neg = false;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) { neg = s[0] == '-'; s = s.substr(1); }
  if (s == "0") { out = 0; return true; }
  if (s.empty()) return false;
  const uint64_t LIM = (uint64_t)1 << 63;
  while (!s.empty()) {
    uint64_t v = 0, f = 0;
    double scale = 1;
    if (!(s[0] == '.' || (s[0] >= '0' && s[0] <= '9'))) return false;
    size_t i = 0;
    size_t pl = s.size();
    // leadingInt
    for (; i < s.size(); i++) {
      char c = s[i];
      if (c < '0' || c > '9') break;
      if (v > LIM / 10) return false;
      v = v * 10 + (c - '0');
      if (v > LIM) return false;
    }
    s = s.substr(i);
    bool pre = pl != s.size();
    bool post = false;
    if (!s.empty() && s[0] == '.') {
      s = s.substr(1);
      size_t pl2 = s.size();
      size_t k = 0;
      bool overflow = false;
      for (; k < s.size(); k++) {
        char c = s[k];
        if (c < '0' || c > '9') break;
        if (overflow) continue;
        if (f > (LIM - 1) / 10) { overflow = true; continue; }
        uint64_t y = f * 10 + (c - '0');
        if (y > LIM) { overflow = true; continue; }
        f = y;
        scale *= 10;
      }
      s = s.substr(k);
      post = pl2 != s.size();
    }
    if (!pre && !post) return false;
    size_t u = 0;
    for (; u < s.size(); u++) {
      char c = s[u];
      if (c == '.' || (c >= '0' && c <= '9')) break;
    }
    if (u == 0) return false;
    std::string unit = s.substr(0, u);
    s = s.substr(u);
    uint64_t um;
    if (unit == "ns") um = 1;
    else if (unit == "us" || unit == "\xC2\xB5s" || unit == "\xCE\xBCs") um = 1000ULL;
    else if (unit == "ms") um = 1000000ULL;
    else if (unit == "s") um = 1000000000ULL;
    else if (unit == "m") um = 60ULL * 1000000000ULL;
    else if (unit == "h") um = 3600ULL * 1000000000ULL;
    else return false;
    if (v > LIM / um) return false;
    v *= um;
    if (f > 0) {
      v += (uint64_t)((double)f * ((double)um / scale));
      if (v > LIM) return false;
    }
    d += v;
    if (d > LIM) return false;
  }
  if (neg) { out = (int64_t)(-(__int128)d); return true; }
  if (d > (unsigned __int128)INT64_MAX) return false;
  out = (int64_t)d;
  return true;
}

// ---------------- resource.Quantity (exact decimal) ----------------
struct Dec {
  bool neg = false;
  std::string mag;   // decimal digits, no leading zeros; "" == 0
  int64_t exp = 0;   // value = mag * 10^exp
  void norm() {
    size_t k = 0;
    while (k < mag.size() && mag[k] == '0') k++;
    mag = mag.substr(k);
    while (!mag.empty() && mag.back() == '0') { mag.pop_back(); exp++; }
    if (mag.empty()) { exp = 0; neg = false; }
  }
  bool zero() const { return mag.empty(); }
};

inline int cmp_mag(const Dec& a, const Dec& b) {
  if (a.zero() || b.zero()) return (a.zero() ? 0 : 1) - (b.zero() ? 0 : 1);
  int64_t la = (int64_t)a.mag.size() + a.exp, lb = (int64_t)b.mag.size() + b.exp;
  if (la != lb) return la < lb ? -1 : 1;
  size_t n = std::max(a.mag.size(), b.mag.size());
  for (size_t k = 0; k < n; k++) {
    char ca = k < a.mag.size() ? a.mag[k] : '0';
    char cb = k < b.mag.size() ? b.mag[k] : '0';
    if (ca != cb) return ca < cb ? -1 : 1;
  }
  return 0;
}

inline int dec_cmp(const Dec& a, const Dec& b) {
  int sa = a.zero() ? 0 : (a.neg ? -1 : 1);
  int sb = b.zero() ? 0 : (b.neg ? -1 : 1);
  if (sa != sb) return sa < sb ? -1 : 1;
  if (sa == 0) return 0;
  int m = cmp_mag(a, b);
  return sa > 0 ? m : -m;
}

inline void mag_mul_small(std::string& mag, unsigned m) {
  unsigned carry = 0;
  for (int k = (int)mag.size() - 1; k >= 0; k--) {
    unsigned v = (mag[k] - '0') * m + carry;
    mag[k] = '0' + v % 10;
    carry = v / 10;
  }
  while (carry) { mag.insert(mag.begin(), '0' + carry % 10); carry /= 10; }
}

struct Quantity {
  Dec v;
  bool binary = false;
};

// k8s.io/apimachinery/pkg/api/resource ParseQuantity (v0.26.1)
inline bool parse_quantity(const std::string& str, Quantity& q) {
  q = Quantity();
  if (str.empty()) return false;
  if (str == "0") return true;
  // parseQuantityString
  bool positive = true;
  size_t pos = 0, end = str.size();
  std::string value, num, denom, suf;
  if (pos < end) {
    if (str[0] == '-') { positive = false; pos++; }
    else if (str[0] == '+') pos++;
  }
  bool done = false;
  // strip leading zeros
  for (size_t i = pos;; i++) {
    if (i >= end) { num = "0"; value = num; done = true; break; }
    if (str[i] == '0') pos++;
    else break;
  }
  if (!done) {
    for (size_t i = pos;; i++) {
      if (i >= end) { num = str.substr(pos, end - pos); value = str.substr(0, end); done = true; break; }
      if (!(str[i] >= '0' && str[i] <= '9')) { num = str.substr(pos, i - pos); pos = i; break; }
    }
  }
  if (!done) {
    if (num.empty()) num = "0";
    if (pos < end && str[pos] == '.') {
      pos++;
      for (size_t i = pos;; i++) {
        if (i >= end) { denom = str.substr(pos, end - pos); value = str.substr(0, end); done = true; break; }
        if (!(str[i] >= '0' && str[i] <= '9')) { denom = str.substr(pos, i - pos); pos = i; break; }
      }
    }
  }
  if (!done) {
    value = str.substr(0, pos);
    size_t suffixStart = pos;
    bool sdone = false;
    for (size_t i = pos;; i++) {
      if (i >= end) { suf = str.substr(suffixStart, end - suffixStart); sdone = true; break; }
      if (!strchr("eEinumkKMGTP", str[i])) { pos = i; break; }
    }
    if (!sdone) {
      if (pos < end && (str[pos] == '-' || str[pos] == '+')) pos++;
      for (size_t i = pos;; i++) {
        if (i >= end) { suf = str.substr(suffixStart, end - suffixStart); sdone = true; break; }
        if (!(str[i] >= '0' && str[i] <= '9')) break;
      }
      if (!sdone) return false;  // ErrFormatWrong
    }
  }
  // suffix interpretation
  int base = 10;
  int64_t exponent = 0;
  bool binary = false;
  static const char* decs[] = {"n", "u", "m", "", "k", "M", "G", "T", "P", "E"};
  static const int dece[] = {-9, -6, -3, 0, 3, 6, 9, 12, 15, 18};
  static const char* bins[] = {"Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
  bool ok = false;
  for (int k = 0; k < 10; k++) if (suf == decs[k]) { exponent = dece[k]; ok = true; }
  if (!ok) for (int k = 0; k < 6; k++) if (suf == bins[k]) { base = 2; exponent = 10 * (k + 1); binary = true; ok = true; }
  if (!ok && suf.size() > 1 && (suf[0] == 'E' || suf[0] == 'e')) {
    int64_t pe;
    if (!parse_int64(suf.substr(1), pe)) return false;
    exponent = (int32_t)pe;
    ok = true;
  }
  if (!ok) return false;
  // exact value of `value` string (sign, digits, optional '.', digits)
  Dec d;
  {
    size_t k = 0;
    if (k < value.size() && (value[k] == '+' || value[k] == '-')) k++;
    std::string digits;
    int64_t frac = 0;
    bool dot = false;
    for (; k < value.size(); k++) {
      if (value[k] == '.') { dot = true; continue; }
      digits += value[k];
      if (dot) frac++;
    }
    d.mag = digits;
    d.exp = -frac;
    d.neg = !positive;
  }
  if (base == 10) d.exp += exponent;
  else for (int64_t k = 0; k < exponent; k++) mag_mul_small(d.mag, 2);
  d.norm();
  if (!positive && !d.zero()) d.neg = true;
  // round magnitude up to 1e-9
  if (!d.zero() && d.exp < -9) {
    int64_t drop = -9 - d.exp;
    bool nonzero = false;
    if ((int64_t)d.mag.size() <= drop) {
      d.mag = "1";
      d.exp = -9;
    } else {
      for (size_t k = d.mag.size() - drop; k < d.mag.size(); k++) if (d.mag[k] != '0') nonzero = true;
      d.mag = d.mag.substr(0, d.mag.size() - drop);
      d.exp = -9;
      if (nonzero) {
        int k = (int)d.mag.size() - 1;
        while (k >= 0 && d.mag[k] == '9') { d.mag[k] = '0'; k--; }
        if (k < 0) d.mag.insert(d.mag.begin(), '1'); else d.mag[k]++;
      }
    }
    bool neg = d.neg;
    d.norm();
    d.neg = neg && !d.zero();
  }
  if (binary) {
    Dec cap; cap.mag = "9223372036854775807"; cap.exp = 0;
    if (cmp_mag(d, cap) > 0) { bool neg = d.neg; d = cap; d.neg = neg; }
  }
  q.v = d;
  q.binary = binary;
  return true;
}

inline int quantity_cmp(const Quantity& a, const Quantity& b) { return dec_cmp(a.v, b.v); }

// strconv.Quote
inline std::string go_quote(const std::string& s) {
  std::string out = "\"";
  for (size_t i = 0; i < s.size();) {
    uint32_t r;
    int w = utf8_decode(s, i, r);
    if (r == 0xFFFD && w == 1) {
      char b[8];
      snprintf(b, sizeof b, "\\x%02x", (unsigned char)s[i]);
      out += b;
      i += 1;
      continue;
    }
    i += w;
    switch (r) {
      case '"': out += "\\\""; continue;
      case '\\': out += "\\\\"; continue;
      case '\a': out += "\\a"; continue;
      case '\b': out += "\\b"; continue;
      case '\f': out += "\\f"; continue;
      case '\n': out += "\\n"; continue;
      case '\r': out += "\\r"; continue;
      case '\t': out += "\\t"; continue;
      case '\v': out += "\\v"; continue;
    }
    if (r < 0x20 || r == 0x7F) {
      char b[8];
      snprintf(b, sizeof b, "\\x%02x", r);
      out += b;
    } else {
      append_utf8(out, r);  // printable assumption for non-ASCII
    }
  }
  return out + "\"";
}

// unicode.IsSpace-based strings.TrimSpace
inline bool is_space_rune(uint32_t r) {
  return r == '\t' || r == '\n' || r == '\v' || r == '\f' || r == '\r' || r == ' ' || r == 0x85 || r == 0xA0 ||
         r == 0x1680 || (r >= 0x2000 && r <= 0x200a) || r == 0x2028 || r == 0x2029 || r == 0x202f || r == 0x205f ||
         r == 0x3000;
}

// path.Clean (Go): collapse slashes, drop "." elements, resolve ".." against the preceding element (kept when
// nothing precedes it in a relative path, dropped at the root of an absolute one); "" -> "."
inline std::string clean_path(const std::string& p) {
  if (p.empty()) return ".";
  const bool rooted = p[0] == '/';
  std::vector<std::string> st;
  size_t i = 0;
  while (i <= p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    std::string e = p.substr(i, j - i);
    i = j + 1;
    if (e.empty() || e == ".") { if (j == p.size()) break; continue; }
    if (e == "..") {
      if (!st.empty() && st.back() != "..") st.pop_back();
      else if (!rooted) st.push_back("..");
    } else {
      st.push_back(e);
    }
    if (j == p.size()) break;
  }
  std::string out = rooted ? "/" : "";
  for (size_t k = 0; k < st.size(); k++) out += (k ? "/" : "") + st[k];
  if (out.empty()) return ".";
  return out;
}

inline std::string trim_space(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e) {
    uint32_t r;
    int w = utf8_decode(s, b, r);
    if (!is_space_rune(r)) break;
    b += w;
  }
  while (e > b) {
    // step back one rune
    size_t k = e - 1;
    while (k > b && ((unsigned char)s[k] & 0xC0) == 0x80 && e - k < 4) k--;
    uint32_t r;
    int w = utf8_decode(s, k, r);
    if (k + w != e) { k = e - 1; w = 1; r = 0xFFFD; }
    if (!is_space_rune(r)) break;
    e = k;
  }
  return s.substr(b, e - b);
}

// strings.Trim(s, " ")
inline std::string trim_spaces(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && s[b] == ' ') b++;
  while (e > b && s[e - 1] == ' ') e--;
  return s.substr(b, e - b);
}

inline std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  size_t st = 0;
  for (size_t i = 0; i <= s.size(); i++) {
    if (i == s.size() || s[i] == sep) { out.push_back(s.substr(st, i - st)); st = i + 1; }
  }
  return out;
}

}  // namespace gou
