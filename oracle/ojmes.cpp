// ORACLE — test infrastructure only (see ojson.h header). JMESPath subset; see ojmes.h.
#include "ojmes.h"

#include <functional>
#include <memory>
#include <regex>
#include <vector>

#include "goutil.h"

namespace orc {
using oj::T;
using oj::Value;
using oj::VP;

namespace {

// ---------------------------------------------------------------- lexer (go-jmespath lexer.go, subset)
enum Tok { tEOF, tIdent, tQuoted, tDot, tLbracket, tRbracket, tFlatten, tComma, tLparen, tRparen, tCurrent, tOr,
           tRaw, tJSON, tFilter, tAnd, tNot, tEQ, tNE, tLT, tLTE, tGT, tGTE, tOther };
struct Token { Tok t; std::string v; };

std::vector<Token> lex(const std::string& s) {
  std::vector<Token> out;
  size_t i = 0;
  auto ident_start = [](char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_'; };
  auto ident = [&](char c) { return ident_start(c) || (c >= '0' && c <= '9'); };
  while (i < s.size()) {
    char c = s[i];
    if (c == ' ' || c == '\t' || c == '\n' || c == '\r') { i++; continue; }
    if (ident_start(c)) {
      size_t j = i;
      while (j < s.size() && ident(s[j])) j++;
      out.push_back({tIdent, s.substr(i, j - i)});
      i = j;
    } else if (c == '"') {
      size_t j = i + 1;
      while (j < s.size() && s[j] != '"') { if (s[j] == '\\') throw JmesUnsupported{"escaped quoted identifier"}; j++; }
      if (j >= s.size()) throw JmesUnsupported{"unterminated quoted identifier"};
      out.push_back({tQuoted, s.substr(i + 1, j - i - 1)});
      i = j + 1;
    } else if (c == '\'') {  // lexer.go consumeRawStringLiteral: \' is a quote, any other backslash is kept
      std::string v;
      size_t j = i + 1;
      for (; j < s.size() && s[j] != '\''; j++) {
        if (s[j] == '\\' && j + 1 < s.size() && s[j + 1] == '\'') { v += '\''; j++; continue; }
        v += s[j];
      }
      if (j >= s.size()) throw JmesUnsupported{"unterminated raw string"};
      out.push_back({tRaw, v});
      i = j + 1;
    } else if (c == '`') {
      size_t j = i + 1;
      while (j < s.size() && s[j] != '`') { if (s[j] == '\\') throw JmesUnsupported{"escaped JSON literal"}; j++; }
      if (j >= s.size()) throw JmesUnsupported{"unterminated JSON literal"};
      out.push_back({tJSON, s.substr(i + 1, j - i - 1)});
      i = j + 1;
    } else if (c == '.') { out.push_back({tDot, "."}); i++; }
    else if (c == '[') {
      if (i + 1 < s.size() && s[i + 1] == ']') { out.push_back({tFlatten, "[]"}); i += 2; }
      else if (i + 1 < s.size() && s[i + 1] == '?') { out.push_back({tFilter, "[?"}); i += 2; }
      else { out.push_back({tLbracket, "["}); i++; }
    } else if (c == ']') { out.push_back({tRbracket, "]"}); i++; }
    else if (c == ',') { out.push_back({tComma, ","}); i++; }
    else if (c == '(') { out.push_back({tLparen, "("}); i++; }
    else if (c == ')') { out.push_back({tRparen, ")"}); i++; }
    else if (c == '@') { out.push_back({tCurrent, "@"}); i++; }
    else if (c == '|' && i + 1 < s.size() && s[i + 1] == '|') { out.push_back({tOr, "||"}); i += 2; }
    else if (c == '&' && i + 1 < s.size() && s[i + 1] == '&') { out.push_back({tAnd, "&&"}); i += 2; }
    else if (c == '=' && i + 1 < s.size() && s[i + 1] == '=') { out.push_back({tEQ, "=="}); i += 2; }
    else if (c == '!') {  // lexer.go matchOrElse('!', '=', tNE, tNot)
      if (i + 1 < s.size() && s[i + 1] == '=') { out.push_back({tNE, "!="}); i += 2; }
      else { out.push_back({tNot, "!"}); i++; }
    } else if (c == '<') {
      if (i + 1 < s.size() && s[i + 1] == '=') { out.push_back({tLTE, "<="}); i += 2; }
      else { out.push_back({tLT, "<"}); i++; }
    } else if (c == '>') {
      if (i + 1 < s.size() && s[i + 1] == '=') { out.push_back({tGTE, ">="}); i += 2; }
      else { out.push_back({tGT, ">"}); i++; }
    }
    else throw JmesUnsupported{std::string("token '") + c + "'"};
  }
  out.push_back({tEOF, ""});
  return out;
}

// ---------------------------------------------------------------- parser (go-jmespath parser.go, subset)
enum NodeKind { NField, NSubexpr, NProjection, NFlatten, NMultiList, NFunction, NCurrent, NIdentity, NOr, NLiteral,
                NFilterProjection, NComparator, NAnd, NNot };
struct Node {
  NodeKind k;
  std::string name;  // NField / NFunction / NComparator (the operator)
  VP lit;            // NLiteral
  std::vector<std::shared_ptr<Node>> kids;
};
using NP = std::shared_ptr<Node>;
NP mk(NodeKind k, std::vector<NP> kids = {}, const std::string& name = "") {
  auto n = std::make_shared<Node>();
  n->k = k;
  n->kids = std::move(kids);
  n->name = name;
  return n;
}

int binding_power(Tok t) {  // parser.go bindingPowers (tokens outside the subset never reach here)
  switch (t) {
    case tOr: return 2;
    case tAnd: return 3;
    case tEQ: case tNE: case tLT: case tLTE: case tGT: case tGTE: return 5;
    case tFlatten: return 9;
    case tFilter: return 21;
    case tDot: return 40;
    case tNot: return 45;
    case tLbracket: return 55;
    case tLparen: return 60;
    default: return 0;
  }
}

struct Parser {
  std::vector<Token> toks;
  size_t at = 0;
  Tok look() const { return toks[at].t; }
  Token next() { return toks[at++]; }
  void match(Tok t) { if (look() != t) throw JmesUnsupported{"syntax"}; at++; }

  NP expr(int bp) {
    NP left = nud(next());
    while (bp < binding_power(look())) left = led(next(), left);
    return left;
  }
  NP nud(const Token& t) {
    switch (t.t) {
      case tIdent: return mk(NField, {}, t.v);
      case tQuoted:
        if (look() == tLparen) throw JmesUnsupported{"quoted identifier as function name"};
        return mk(NField, {}, t.v);
      case tCurrent: return mk(NCurrent);
      case tRaw: { auto n = mk(NLiteral); n->lit = Value::str(t.v); return n; }
      case tJSON: {
        auto n = mk(NLiteral);
        try { n->lit = oj::parse(t.v, true); } catch (...) { throw JmesUnsupported{"JSON literal"}; }
        return n;
      }
      case tFlatten: {  // nud(tFlatten): projection over the flattened current node
        NP left = mk(NFlatten, {mk(NIdentity)});
        return mk(NProjection, {left, projection_rhs(binding_power(tFlatten))});
      }
      case tLbracket:
        return multi_list();
      case tFilter: return filter(mk(NIdentity));
      case tNot: return mk(NNot, {expr(binding_power(tNot))});
      case tLparen: {  // nud(tLparen): a parenthesised expression
        NP x = expr(0);
        match(tRparen);
        return x;
      }
      default: throw JmesUnsupported{"expression start"};
    }
  }
  NP led(const Token& t, NP left) {
    switch (t.t) {
      case tDot: return mk(NSubexpr, {left, dot_rhs(binding_power(tDot))});
      case tFlatten: return mk(NProjection, {mk(NFlatten, {left}), projection_rhs(binding_power(tFlatten))});
      case tOr: return mk(NOr, {left, expr(binding_power(tOr))});
      case tAnd: return mk(NAnd, {left, expr(binding_power(tAnd))});
      case tEQ: case tNE: case tLT: case tLTE: case tGT: case tGTE:
        return mk(NComparator, {left, expr(binding_power(t.t))}, t.v);
      case tFilter: return filter(left);
      case tLparen: {
        if (left->k != NField) throw JmesUnsupported{"function name"};
        std::vector<NP> args;
        while (look() != tRparen) {
          args.push_back(expr(0));
          if (look() == tComma) match(tComma);
        }
        match(tRparen);
        return mk(NFunction, args, left->name);
      }
      default: throw JmesUnsupported{"operator"};
    }
  }
  NP dot_rhs(int bp) {
    Tok l = look();
    if (l == tIdent || l == tQuoted) return expr(bp);
    if (l == tLbracket) { match(tLbracket); return multi_list(); }
    throw JmesUnsupported{"dot rhs"};
  }
  NP projection_rhs(int bp) {
    if (binding_power(look()) < 10) return mk(NIdentity);  // projectionStop
    if (look() == tLbracket || look() == tFilter) return expr(bp);
    if (look() == tDot) { match(tDot); return dot_rhs(bp); }
    throw JmesUnsupported{"projection rhs"};
  }
  NP filter(NP left) {  // parseFilter: children [left, right, condition]
    NP cond = expr(0);
    match(tRbracket);
    NP right = look() == tFlatten ? mk(NIdentity) : projection_rhs(binding_power(tFilter));
    return mk(NFilterProjection, {left, right, cond});
  }
  NP multi_list() {  // '[' already consumed
    std::vector<NP> items;
    for (;;) {
      items.push_back(expr(0));
      if (look() == tRbracket) break;
      match(tComma);
    }
    match(tRbracket);
    return mk(NMultiList, items);
  }
};

NP parse(const std::string& s) {
  Parser p{lex(s), 0};
  NP n = p.expr(0);
  if (p.look() != tEOF) throw JmesUnsupported{"trailing tokens"};
  return n;
}

// ---------------------------------------------------------------- interpreter (go-jmespath interpreter.go)
bool is_false(const VP& v) {  // util.go isFalse
  if (!v || v->t == T::Null) return true;
  switch (v->t) {
    case T::Bool: return !v->b;
    case T::Str: return v->s.empty();
    case T::Arr: return v->a.empty();
    case T::Obj: return v->o.empty();
    default: return false;
  }
}

// reflect.DeepEqual of two decoded JSON values (every number float64 in the JSON context)
bool objs_equal(const VP& a, const VP& b) {
  const bool an = !a || a->t == T::Null, bn = !b || b->t == T::Null;
  if (an || bn) return an && bn;
  auto num = [](const VP& v, double* d) {
    if (v->t == T::Int) { *d = (double)v->i; return true; }
    if (v->t == T::Float) { *d = v->f; return true; }
    return false;
  };
  double x, y;
  if (num(a, &x) || num(b, &y)) return num(a, &x) && num(b, &y) && x == y;
  if (a->t != b->t) return false;
  switch (a->t) {
    case T::Bool: return a->b == b->b;
    case T::Str: return a->s == b->s;
    case T::Arr:
      if (a->a.size() != b->a.size()) return false;
      for (size_t i = 0; i < a->a.size(); i++) if (!objs_equal(a->a[i], b->a[i])) return false;
      return true;
    case T::Obj:
      if (a->o.size() != b->o.size()) return false;
      for (auto& kv : a->o) { if (!b->has(kv.first) || !objs_equal(kv.second, b->get(kv.first))) return false; }
      return true;
    default: return false;
  }
}

VP eval(const NP& n, const VP& value) {
  switch (n->k) {
    case NField:
      if (value && value->t == T::Obj) { VP x = value->get(n->name); return x ? x : Value::null(); }
      return Value::null();
    case NSubexpr: return eval(n->kids[1], eval(n->kids[0], value));
    case NProjection: {
      VP left = eval(n->kids[0], value);
      if (!left || left->t != T::Arr) return Value::null();
      auto out = Value::arr();
      for (auto& e : left->a) {
        VP r = eval(n->kids[1], e);
        if (r && r->t != T::Null) out->a.push_back(r);
      }
      return out;
    }
    case NFlatten: {
      VP left = eval(n->kids[0], value);
      if (!left || left->t != T::Arr) return Value::null();
      auto out = Value::arr();
      for (auto& e : left->a) {
        if (e && e->t == T::Arr) for (auto& x : e->a) out->a.push_back(x);
        else out->a.push_back(e ? e : Value::null());
      }
      return out;
    }
    case NMultiList: {
      if (!value || value->t == T::Null) return Value::null();
      auto out = Value::arr();
      for (auto& k : n->kids) out->a.push_back(eval(k, value));
      return out;
    }
    case NFunction: {
      if (n->name == "length" && n->kids.size() == 1) {  // jpfLength: runes of a string, items of an array / object
        VP arg = eval(n->kids[0], value);
        if (arg && arg->t == T::Str) {
          size_t runes = 0;
          for (unsigned char ch : arg->s) runes += (ch & 0xC0) != 0x80;
          return Value::flt((double)runes);
        }
        if (arg && arg->t == T::Arr) return Value::flt((double)arg->a.size());
        if (arg && arg->t == T::Obj) return Value::flt((double)arg->o.size());
        throw JmesError{"invalid type for: <nil>, expected: []jpType{\"string\", \"array\", \"object\"}"};
      }
      if (n->name == "contains" && n->kids.size() == 2) {  // jpfContains: substring of a string, member of an array
        VP subject = eval(n->kids[0], value), el = eval(n->kids[1], value);
        if (subject && subject->t == T::Str) return Value::boolean(el && el->t == T::Str && subject->s.find(el->s) != std::string::npos);
        if (!subject || subject->t != T::Arr) throw JmesError{"invalid type for: <nil>, expected: []jpType{\"array\", \"string\"}"};
        for (auto& x : subject->a) {  // Go interface ==: same dynamic type and value (scalars here)
          if (!x || !el) { if ((!x || x->t == T::Null) && (!el || el->t == T::Null)) return Value::boolean(true); continue; }
          if (x->t == T::Arr || x->t == T::Obj || el->t == T::Arr || el->t == T::Obj) throw JmesUnsupported{"contains of a container"};
          if (objs_equal(x, el)) return Value::boolean(true);
        }
        return Value::boolean(false);
      }
      if (n->name == "to_upper" && n->kids.size() == 1) {
        // jpfToUpper (kyverno pkg/engine/jmespath/functions.go:681-689): the argument type check (JpString) first, then
        // strings.ToUpper; restated for ASCII strings (Unicode case mapping: outside the restatement)
        VP arg = eval(n->kids[0], value);
        if (!arg || arg->t != T::Str) throw JmesError{"invalid type for: <nil>, expected: []jpType{\"string\"}"};
        std::string u = arg->s;
        for (char& ch : u) {
          if ((unsigned char)ch >= 0x80) throw JmesUnsupported{"to_upper of a non-ASCII string"};
          if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 'a' + 'A');
        }
        return Value::str(u);
      }
      if (n->name == "regex_match" && n->kids.size() == 2) {
        // jpRegexMatch (functions.go:786-799): argument types (JpString, JpString | JpNumber), then
        // regexp.Match(regex, []byte(ifaceToString(src))) -- an unanchored search. The pattern is checked against the
        // restated subset by nodes_ok (rx_restated); subjects outside printable ASCII and numbers (ifaceToString's
        // FormatFloat(f, 'f', -1, 32)) are outside the restatement
        VP re = eval(n->kids[0], value), src = eval(n->kids[1], value);
        if (!re || re->t != T::Str) throw JmesError{"invalid type for: <nil>, expected: []jpType{\"string\"}"};
        if (!src || (src->t != T::Str && src->t != T::Int && src->t != T::Float))
          throw JmesError{"invalid type for: <nil>, expected: []jpType{\"string\", \"number\"}"};
        if (src->t != T::Str) throw JmesUnsupported{"regex_match of a number"};
        for (unsigned char ch : src->s)
          if (ch < 0x20 || ch > 0x7E) throw JmesUnsupported{"regex_match subject outside printable ASCII"};
        return Value::boolean(std::regex_search(src->s, std::regex(re->s, std::regex::ECMAScript)));
      }
      if (n->name != "keys" || n->kids.size() != 1) throw JmesUnsupported{"function " + n->name};
      VP arg = eval(n->kids[0], value);
      if (!arg || arg->t != T::Obj) throw JmesError{"invalid type for: <nil>, expected: []jpType{\"object\"}"};
      auto out = Value::arr();  // Go map iteration order in the reference; sorted here (order-free uses only)
      for (auto& kv : arg->o) out->a.push_back(Value::str(kv.first));
      return out;
    }
    case NCurrent: case NIdentity: return value ? value : Value::null();
    case NOr: {
      VP m = eval(n->kids[0], value);
      return is_false(m) ? eval(n->kids[1], value) : m;
    }
    case NLiteral: return n->lit;
    case NFilterProjection: {  // interpreter.go ASTFilterProjection
      VP left = eval(n->kids[0], value);
      if (!left || left->t != T::Arr) return Value::null();
      auto out = Value::arr();
      for (auto& e : left->a) {
        VP el = e ? e : Value::null();
        if (is_false(eval(n->kids[2], el))) continue;
        VP r = eval(n->kids[1], el);
        if (r && r->t != T::Null) out->a.push_back(r);
      }
      return out;
    }
    case NComparator: {  // interpreter.go ASTComparator: ==/!= by DeepEqual, ordering only for two numbers
      VP l = eval(n->kids[0], value), r = eval(n->kids[1], value);
      if (n->name == "==") return Value::boolean(objs_equal(l, r));
      if (n->name == "!=") return Value::boolean(!objs_equal(l, r));
      auto num = [](const VP& v, double* d) {
        if (v && v->t == T::Int) { *d = (double)v->i; return true; }
        if (v && v->t == T::Float) { *d = v->f; return true; }
        return false;
      };
      double x, y;
      if (!num(l, &x) || !num(r, &y)) return Value::null();
      if (n->name == "<") return Value::boolean(x < y);
      if (n->name == "<=") return Value::boolean(x <= y);
      if (n->name == ">") return Value::boolean(x > y);
      return Value::boolean(x >= y);
    }
    case NAnd: {
      VP l = eval(n->kids[0], value);
      return is_false(l) ? l : eval(n->kids[1], value);
    }
    case NNot: return Value::boolean(is_false(eval(n->kids[0], value)));
  }
  return Value::null();
}

// plain field chain (the fork's NotFoundError applies): field names in order
bool pure_chain(const NP& n, std::vector<std::string>& out) {
  if (n->k == NField) { out.push_back(n->name); return true; }
  if (n->k == NSubexpr) return pure_chain(n->kids[0], out) && pure_chain(n->kids[1], out);
  return false;
}

VP floats(const VP& v) {  // encoding/json decode of the JSON context: every number float64
  if (!v) return Value::null();
  switch (v->t) {
    case T::Int: return Value::flt((double)v->i);
    case T::Arr: { auto o = Value::arr(); for (auto& e : v->a) o->a.push_back(floats(e)); return o; }
    case T::Obj: { auto o = Value::obj(); for (auto& kv : v->o) o->o[kv.first] = floats(kv.second); return o; }
    default: return v;
  }
}

}  // namespace

VP json_floats(const VP& v) { return floats(v); }

// The regex_match patterns the restatement evaluates with std::regex (ECMAScript): a subset of Go's RE2 syntax whose
// matches coincide with RE2's on printable-ASCII subjects -- literal characters, `.`, escaped metacharacters (and '/',
// '-'), \d \D \w \W \s \S, bracket classes (ranges, negation; no POSIX classes, no ']' first), ( ) and (?: ) groups,
// `|`, the quantifiers * + ? {n} {n,} {n,m} (bounds <= 64, one per atom, an optional lazy '?'), '^' only as the first
// and '$' only as the last pattern character (then no '|' outside parentheses). Anything else: JmesUnsupported.
static bool rx_restated(const std::string& re) {
  std::string b = re;
  bool anchored = false;
  if (!b.empty() && b[0] == '^') { b.erase(0, 1); anchored = true; }
  if (!b.empty() && b.back() == '$') {
    size_t bs = 0;
    for (size_t j = b.size() - 1; j > 0 && b[j - 1] == '\\'; j--) bs++;
    if (bs % 2 == 0) { b.pop_back(); anchored = true; }
  }
  const std::string meta = "^$\\.*+?()[]{}|";
  auto esc_ok = [&](char e) { return std::string("dDwWsS").find(e) != std::string::npos || meta.find(e) != std::string::npos ||
                                     e == '/' || e == '-'; };
  int depth = 0;
  bool atom = false, quant = false;  // an atom precedes (a quantifier may follow); the atom is quantified already
  for (size_t i = 0; i < b.size(); i++) {
    const unsigned char c = (unsigned char)b[i];
    if (c < 0x20 || c > 0x7E) return false;
    if (c == '\\') {
      if (i + 1 >= b.size() || !esc_ok(b[i + 1])) return false;
      i++;
      atom = true; quant = false;
    } else if (c == '[') {
      size_t j = i + 1;
      if (j < b.size() && b[j] == '^') j++;
      if (j >= b.size() || b[j] == ']') return false;
      bool closed = false;
      int prev = -1;  // last single character of the class (a range's start)
      for (; j < b.size(); j++) {
        if (b[j] == ']') { closed = true; break; }
        if (b[j] == '[') return false;
        int ch;
        if (b[j] == '\\') {
          if (j + 1 >= b.size() || !esc_ok(b[j + 1])) return false;
          ch = std::string("dDwWsS").find(b[j + 1]) != std::string::npos ? -1 : (unsigned char)b[j + 1];
          j++;
        } else {
          ch = (unsigned char)b[j];
          if (ch < 0x20 || ch > 0x7E) return false;
        }
        if (ch == '-' && prev >= 0 && j + 1 < b.size() && b[j + 1] != ']') {  // range prev-next
          int hi;
          if (b[j + 1] == '\\') {
            if (j + 2 >= b.size() || std::string("dDwWsS").find(b[j + 2]) != std::string::npos || !esc_ok(b[j + 2])) return false;
            hi = (unsigned char)b[j + 2];
            j += 2;
          } else {
            if (b[j + 1] == '[') return false;
            hi = (unsigned char)b[j + 1];
            j++;
          }
          if (hi < prev) return false;
          prev = -1;
          continue;
        }
        prev = ch;
      }
      if (!closed) return false;
      i = j;
      atom = true; quant = false;
    } else if (c == '(') {
      if (i + 1 < b.size() && b[i + 1] == '?') {
        if (i + 2 >= b.size() || b[i + 2] != ':') return false;
        i += 2;
      }
      depth++;
      atom = false; quant = false;
    } else if (c == ')') {
      if (--depth < 0) return false;
      atom = true; quant = false;
    } else if (c == '|') {
      if (depth == 0 && anchored) return false;
      atom = false; quant = false;
    } else if (c == '*' || c == '+' || c == '?' || c == '{') {
      if (!atom || quant) return false;
      if (c == '{') {
        size_t j = i + 1;
        int lo = 0, hi = -2, nd = 0;
        while (j < b.size() && isdigit((unsigned char)b[j]) && nd < 4) { lo = lo * 10 + (b[j++] - '0'); nd++; }
        if (!nd) return false;
        hi = lo;
        if (j < b.size() && b[j] == ',') {
          j++;
          if (j < b.size() && b[j] == '}') hi = -1;
          else {
            int h = 0, hd = 0;
            while (j < b.size() && isdigit((unsigned char)b[j]) && hd < 4) { h = h * 10 + (b[j++] - '0'); hd++; }
            if (!hd) return false;
            hi = h;
          }
        }
        if (j >= b.size() || b[j] != '}' || lo > 64 || hi > 64 || (hi >= 0 && hi < lo)) return false;
        i = j;
      }
      if (i + 1 < b.size() && b[i + 1] == '?') i++;      // lazy
      if (i + 1 < b.size() && b[i + 1] == '+') return false;  // possessive: not RE2
      quant = true;
    } else if (c == '^' || c == '$' || c == ']' || c == '}') {
      return false;
    } else {
      atom = true; quant = false;
    }
  }
  if (depth != 0) return false;
  try {
    std::regex x(re, std::regex::ECMAScript);
  } catch (std::regex_error&) {
    return false;
  }
  return true;
}

// every node within the restated interpreter (functions: keys(@), length(), contains(), to_upper() and regex_match()
// with a raw-string pattern of the restated subset)
static bool nodes_ok(const NP& n) {
  if (n->k == NFunction && n->name == "regex_match") {
    if (n->kids.size() != 2 || n->kids[0]->k != NLiteral || !n->kids[0]->lit || n->kids[0]->lit->t != T::Str ||
        !rx_restated(n->kids[0]->lit->s))
      return false;
  } else if (n->k == NFunction && !(n->name == "length" && n->kids.size() == 1) &&
             !(n->name == "contains" && n->kids.size() == 2) && !(n->name == "to_upper" && n->kids.size() == 1) &&
             (n->name != "keys" || n->kids.size() != 1 || n->kids[0]->k != NCurrent)) {
    return false;
  }
  for (auto& k : n->kids) if (!nodes_ok(k)) return false;
  return true;
}

bool jmes_supported(const std::string& expr, bool allow_element) {
  try {
    NP n = parse(expr);
    if (!nodes_ok(n)) return false;
    // left spine down to the innermost node whose left child is the root field
    const Node* c = n.get();
    if (c->k == NField) return c->name == "element" && allow_element;
    for (;;) {
      if (c->kids.empty()) return false;
      // a function's subject: regex_match's second argument (its first is the pattern literal), else the first
      const Node* l = (c->k == NFunction && c->name == "regex_match" && c->kids.size() == 2) ? c->kids[1].get()
                                                                                          : c->kids[0].get();
      if (l->k == NField) break;
      if (l->k != NSubexpr && l->k != NProjection && l->k != NFlatten && l->k != NOr && l->k != NFilterProjection)
        return false;
      c = l;
    }
    const std::string& root = c->kids[0]->name;
    if (root == "element") return allow_element;
    if (root != "request" || c->k != NSubexpr || c->kids[1]->k != NField) return false;
    return c->kids[1]->name == "object" || c->kids[1]->name == "operation";
  } catch (JmesUnsupported&) {
    return false;
  }
}

VP jmes_query(const std::string& expr, const VP& resource, const VP& element, int64_t index) {
  NP n = parse(expr);
  auto ctx = Value::obj();
  auto req = Value::obj();
  req->o["object"] = floats(resource);
  req->o["operation"] = Value::str("CREATE");  // scanner.go:97 / CLI default (common.go:287)
  ctx->o["request"] = req;
  if (element) {
    ctx->o["element"] = floats(element);
    ctx->o["elementIndex"] = Value::flt((double)index);
  }
  std::vector<std::string> chain;
  if (pure_chain(n, chain)) {  // kyverno/go-jmespath fork: a key missing from a map is NotFoundError
    VP cur = ctx;
    for (auto& k : chain) {
      if (!cur || cur->t != T::Obj) return Value::null();
      if (!cur->has(k)) throw JmesNotFound{k};
      cur = cur->get(k);
    }
    return cur ? cur : Value::null();
  }
  return eval(n, ctx);
}

}  // namespace orc
