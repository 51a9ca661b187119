// ORACLE — test infrastructure only (see ojson.h header).
#include "ojson.h"

#include <cmath>
#include <cstdio>
#include <cstring>

#include "goutil.h"

namespace oj {

VP deep_copy(const VP& v) {
  if (!v) return v;
  auto p = std::make_shared<Value>(*v);
  for (auto& e : p->a) e = deep_copy(e);
  for (auto& kv : p->o) kv.second = deep_copy(kv.second);
  return p;
}

namespace {

struct Parser {
  const std::string& s;
  size_t i = 0;
  bool as_float;
  Parser(const std::string& str, bool f) : s(str), as_float(f) {}

  [[noreturn]] void fail(const char* m) { throw ParseError(std::string("json: ") + m + " at " + std::to_string(i)); }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++;
  }
  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  bool hex4(size_t at, uint32_t& out) {
    if (at + 4 > s.size()) return false;
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) {
      int h = hexv(s[at + k]);
      if (h < 0) return false;
      v = v * 16 + h;
    }
    out = v;
    return true;
  }
  std::string str() {
    if (s[i] != '"') fail("expected string");
    i++;
    std::string out;
    while (true) {
      if (i >= s.size()) fail("unterminated string");
      unsigned char c = s[i];
      if (c == '"') { i++; break; }
      if (c == '\\') {
        i++;
        if (i >= s.size()) fail("bad escape");
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
            if (!hex4(i, r)) fail("bad \\u");
            i += 4;
            if (r >= 0xD800 && r < 0xDC00) {
              // possible surrogate pair (encoding/json getu4 + utf16.DecodeRune)
              uint32_t r2;
              if (i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u' && hex4(i + 2, r2) && r2 >= 0xDC00 && r2 < 0xE000) {
                i += 6;
                r = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00);
              } else {
                r = 0xFFFD;
              }
            } else if (r >= 0xDC00 && r < 0xE000) {
              r = 0xFFFD;
            }
            gou::append_utf8(out, r);
            break;
          }
          default: fail("bad escape char");
        }
        continue;
      }
      if (c < 0x20) fail("control char in string");
      if (c < 0x80) { out += (char)c; i++; continue; }
      uint32_t r;
      int w = gou::utf8_decode(s, i, r);
      if (r == 0xFFFD && w == 1) {
        gou::append_utf8(out, 0xFFFD);
      } else {
        out.append(s, i, w);
      }
      i += w;
    }
    return out;
  }
  VP num() {
    size_t st = i;
    if (s[i] == '-') i++;
    if (i >= s.size()) fail("bad number");
    if (s[i] == '0') i++;
    else if (s[i] >= '1' && s[i] <= '9') { while (i < s.size() && isdigit((unsigned char)s[i])) i++; }
    else fail("bad number");
    bool integral = true;
    if (i < s.size() && s[i] == '.') {
      integral = false;
      i++;
      if (i >= s.size() || !isdigit((unsigned char)s[i])) fail("bad fraction");
      while (i < s.size() && isdigit((unsigned char)s[i])) i++;
    }
    if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
      integral = false;
      i++;
      if (i < s.size() && (s[i] == '+' || s[i] == '-')) i++;
      if (i >= s.size() || !isdigit((unsigned char)s[i])) fail("bad exponent");
      while (i < s.size() && isdigit((unsigned char)s[i])) i++;
    }
    std::string lit = s.substr(st, i - st);
    if (!as_float && integral) {
      int64_t v;
      if (gou::parse_int64(lit, v)) return Value::integer(v);
    }
    double d;
    if (!gou::parse_float(lit, d)) fail("number out of range");
    return Value::flt(d);
  }
  VP val(int depth) {
    if (depth > 10000) fail("too deep");
    ws();
    if (i >= s.size()) fail("unexpected end");
    char c = s[i];
    if (c == '{') {
      i++;
      auto o = Value::obj();
      ws();
      if (i < s.size() && s[i] == '}') { i++; return o; }
      while (true) {
        ws();
        if (i >= s.size()) fail("unterminated object");
        std::string k = str();
        ws();
        if (i >= s.size() || s[i] != ':') fail("expected :");
        i++;
        VP v = val(depth + 1);
        o->o[k] = v;  // last wins
        ws();
        if (i < s.size() && s[i] == ',') { i++; continue; }
        if (i < s.size() && s[i] == '}') { i++; break; }
        fail("expected , or }");
      }
      return o;
    }
    if (c == '[') {
      i++;
      auto a = Value::arr();
      ws();
      if (i < s.size() && s[i] == ']') { i++; return a; }
      while (true) {
        a->a.push_back(val(depth + 1));
        ws();
        if (i < s.size() && s[i] == ',') { i++; continue; }
        if (i < s.size() && s[i] == ']') { i++; break; }
        fail("expected , or ]");
      }
      return a;
    }
    if (c == '"') return Value::str(str());
    if (c == 't' && s.compare(i, 4, "true") == 0) { i += 4; return Value::boolean(true); }
    if (c == 'f' && s.compare(i, 5, "false") == 0) { i += 5; return Value::boolean(false); }
    if (c == 'n' && s.compare(i, 4, "null") == 0) { i += 4; return Value::null(); }
    if (c == '-' || (c >= '0' && c <= '9')) return num();
    fail("unexpected char");
  }
};

void dump_str(std::string& out, const std::string& s) {
  out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '<': out += "\\u003c"; break;
      case '>': out += "\\u003e"; break;
      case '&': out += "\\u0026"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          out += b;
        } else {
          out += (char)c;
        }
    }
  }
  out += '"';
}

void dump_rec(std::string& out, const VP& v) {
  if (!v) { out += "null"; return; }
  switch (v->t) {
    case T::Null: out += "null"; break;
    case T::Bool: out += v->b ? "true" : "false"; break;
    case T::Int: out += std::to_string(v->i); break;
    case T::Float: out += gou::format_float_json(v->f); break;
    case T::Str: dump_str(out, v->s); break;
    case T::Arr: {
      out += '[';
      bool first = true;
      for (auto& e : v->a) { if (!first) out += ','; first = false; dump_rec(out, e); }
      out += ']';
      break;
    }
    case T::Obj: {
      out += '{';
      bool first = true;
      for (auto& kv : v->o) {
        if (!first) out += ',';
        first = false;
        dump_str(out, kv.first);
        out += ':';
        dump_rec(out, kv.second);
      }
      out += '}';
      break;
    }
  }
}

void gov_rec(std::string& out, const VP& v) {
  if (!v) { out += "<nil>"; return; }
  switch (v->t) {
    case T::Null: out += "<nil>"; break;
    case T::Bool: out += v->b ? "true" : "false"; break;
    case T::Int: out += std::to_string(v->i); break;
    case T::Float: out += gou::format_float_g(v->f); break;
    case T::Str: out += v->s; break;
    case T::Arr: {
      out += '[';
      bool first = true;
      for (auto& e : v->a) { if (!first) out += ' '; first = false; gov_rec(out, e); }
      out += ']';
      break;
    }
    case T::Obj: {
      out += "map[";
      bool first = true;
      for (auto& kv : v->o) {
        if (!first) out += ' ';
        first = false;
        out += kv.first;
        out += ':';
        gov_rec(out, kv.second);
      }
      out += ']';
      break;
    }
  }
}

}  // namespace

VP parse(const std::string& text, bool numbers_as_float) {
  Parser p(text, numbers_as_float);
  VP v = p.val(0);
  p.ws();
  if (p.i != text.size()) p.fail("trailing data");
  return v;
}

std::string dump(const VP& v) {
  std::string out;
  dump_rec(out, v);
  return out;
}

std::string go_v(const VP& v) {
  std::string out;
  gov_rec(out, v);
  return out;
}

std::string get_str(const VP& obj, const std::string& k) {
  VP v = obj ? obj->get(k) : nullptr;
  if (v && v->t == T::Str) return v->s;
  return "";
}

}  // namespace oj
