// regex_match (kyverno pkg/engine/jmespath/functions.go:786-799: regexp.Match(regex, []byte(src)), Go's RE2 syntax,
// unanchored search) compiled for the per-dictionary-string precompute of the batch (batch.cpp): the pattern, a ruleset
// literal, becomes a DFA over printable ASCII, and every dictionary string gets one bit per regex (Batch::str_rx).
//
// The subset, chosen so that Go regexp and the oracle's std::regex (ECMAScript, oracle/ojmes.cpp) accept exactly the same
// subjects of printable ASCII: literal characters, `.`, escaped metacharacters, \d \D \w \W \s \S, bracket classes with
// ranges and negation (no POSIX [:classes:], no `]` first), groups `( )` and `(?: )`, alternation, the quantifiers
// * + ? {n} {n,} {n,m} (n, m <= 64, a trailing lazy `?` ignored: a boolean search does not depend on it), `^` as the
// first and `$` as the last character of the whole pattern (then no top-level `|`). Anything else -- back-references,
// look-around, flags, \b, \p{..}, octal / hex escapes -- is outside: the rule goes to the CPU engine (compiler.cpp).
// A subject with a byte outside 0x20..0x7E matches nothing here: its pairs are per-pair CPU fallback (bit RX_FB).
#include <bitset>
#include <map>
#include <memory>

#include "kyv_host.h"

namespace kyv {

namespace {

constexpr int kSyms = RX_SYMS;  // printable ASCII 0x20..0x7E
using Set = std::bitset<kSyms>;

struct Ast {
  enum K { SET, CAT, ALT, REP, EMPTY } k;
  Set set;
  int lo = 0, hi = 0;  // REP: hi < 0 unbounded
  std::vector<std::unique_ptr<Ast>> kids;
};
using AP = std::unique_ptr<Ast>;

struct Fail { std::string why; };

Set sym_range(int a, int b) {
  Set s;
  for (int c = a; c <= b; c++)
    if (c >= 0x20 && c <= 0x7E) s.set((size_t)(c - 0x20));
  return s;
}
Set cls_digit() { return sym_range('0', '9'); }
Set cls_word() { return sym_range('0', '9') | sym_range('A', 'Z') | sym_range('a', 'z') | sym_range('_', '_'); }
Set cls_space() { return sym_range(' ', ' '); }  // \s = [\t\n\f\r ] (RE2) / ECMAScript's white space: in printable ASCII, ' '

bool is_meta(char c) { return std::string("^$\\.*+?()[]{}|").find(c) != std::string::npos; }

struct Parser {
  const std::string& s;
  size_t i = 0;
  int depth = 0;
  explicit Parser(const std::string& x) : s(x) {}
  bool at_end() const { return i >= s.size(); }
  char peek() const { return s[i]; }

  AP mk(Ast::K k) { AP a(new Ast()); a->k = k; return a; }
  AP set_node(const Set& st) { AP a = mk(Ast::SET); a->set = st; return a; }

  AP alt() {
    AP first = cat();
    if (at_end() || peek() != '|') return first;
    AP a = mk(Ast::ALT);
    a->kids.push_back(std::move(first));
    while (!at_end() && peek() == '|') {
      i++;
      a->kids.push_back(cat());
    }
    return a;
  }
  AP cat() {
    AP c = mk(Ast::CAT);
    while (!at_end() && peek() != '|' && peek() != ')') c->kids.push_back(repeat());
    if (c->kids.empty()) return mk(Ast::EMPTY);
    return c;
  }
  bool number(int* v) {
    size_t j = i;
    int x = 0;
    while (j < s.size() && isdigit((unsigned char)s[j]) && j - i < 4) x = x * 10 + (s[j++] - '0');
    if (j == i) return false;
    i = j;
    *v = x;
    return true;
  }
  AP repeat() {
    AP a = atom();
    bool quantified = false;
    while (!at_end()) {
      const char c = peek();
      int lo, hi;
      if (c == '*') { lo = 0; hi = -1; i++; }
      else if (c == '+') { lo = 1; hi = -1; i++; }
      else if (c == '?') { lo = 0; hi = 1; i++; }
      else if (c == '{') {
        i++;
        if (!number(&lo)) throw Fail{"'{' not a repetition"};
        hi = lo;
        if (!at_end() && peek() == ',') {
          i++;
          if (!at_end() && peek() == '}') hi = -1;
          else if (!number(&hi)) throw Fail{"bad repetition"};
        }
        if (at_end() || peek() != '}') throw Fail{"bad repetition"};
        i++;
        if (lo > 64 || hi > 64 || (hi >= 0 && hi < lo)) throw Fail{"repetition bounds"};
      } else {
        break;
      }
      if (quantified) throw Fail{"repeated quantifier"};  // RE2: bad repetition operator
      quantified = true;
      if (!at_end() && peek() == '?') i++;  // lazy: the same set of matched subjects
      if (!at_end() && peek() == '+') throw Fail{"possessive quantifier"};
      AP r = mk(Ast::REP);
      r->lo = lo;
      r->hi = hi;
      r->kids.push_back(std::move(a));
      a = std::move(r);
    }
    return a;
  }
  Set escape_class(char e, bool* ok) {
    *ok = true;
    switch (e) {
      case 'd': return cls_digit();
      case 'D': return ~cls_digit();
      case 'w': return cls_word();
      case 'W': return ~cls_word();
      case 's': return cls_space();
      case 'S': return ~cls_space();
      default: *ok = false; return Set();
    }
  }
  AP atom() {
    const char c = peek();
    if (c == '(') {
      i++;
      if (!at_end() && peek() == '?') {
        if (i + 1 < s.size() && s[i + 1] == ':') i += 2;
        else throw Fail{"group flags / look-around"};
      }
      if (++depth > 32) throw Fail{"nesting"};
      AP a = alt();
      depth--;
      if (at_end() || peek() != ')') throw Fail{"missing ')'"};
      i++;
      return a;
    }
    if (c == '[') return bracket();
    if (c == '.') { i++; return set_node(~Set()); }
    if (c == '\\') {
      if (i + 1 >= s.size()) throw Fail{"trailing backslash"};
      const char e = s[i + 1];
      i += 2;
      bool ok;
      Set st = escape_class(e, &ok);
      if (ok) return set_node(st);
      if (is_meta(e) || e == '/' || e == '-') return set_node(sym_range(e, e));
      throw Fail{"escape outside the subset"};
    }
    if (c == '^' || c == '$') throw Fail{"anchor inside the pattern"};
    if (c == '*' || c == '+' || c == '?' || c == '{') throw Fail{"missing argument to repetition"};
    if (c == ')' || c == ']' || c == '}') throw Fail{"unbalanced"};
    if ((unsigned char)c < 0x20 || (unsigned char)c > 0x7E) throw Fail{"non-printable pattern character"};
    i++;
    return set_node(sym_range(c, c));
  }
  AP bracket() {
    i++;  // '['
    bool neg = false;
    if (!at_end() && peek() == '^') { neg = true; i++; }
    if (!at_end() && peek() == ']') throw Fail{"']' first in a class"};
    Set st;
    bool any = false;
    for (;;) {
      if (at_end()) throw Fail{"missing ']'"};
      char c = peek();
      if (c == ']') { i++; break; }
      if (c == '[') throw Fail{"'[' in a class"};
      int lo;
      if (c == '\\') {
        if (i + 1 >= s.size()) throw Fail{"trailing backslash"};
        const char e = s[i + 1];
        i += 2;
        bool ok;
        Set cs = escape_class(e, &ok);
        if (ok) { st |= cs; any = true; continue; }
        if (!(is_meta(e) || e == '/' || e == '-')) throw Fail{"escape outside the subset"};
        lo = (unsigned char)e;
      } else {
        if ((unsigned char)c < 0x20 || (unsigned char)c > 0x7E) throw Fail{"non-printable pattern character"};
        lo = (unsigned char)c;
        i++;
      }
      // a range lo-hi (a '-' before ']' is a literal)
      if (i + 1 < s.size() && peek() == '-' && s[i + 1] != ']') {
        i++;
        int hi;
        char h = peek();
        if (h == '\\') {
          if (i + 1 >= s.size()) throw Fail{"trailing backslash"};
          const char e = s[i + 1];
          if (!(is_meta(e) || e == '/' || e == '-')) throw Fail{"range end outside the subset"};
          hi = (unsigned char)e;
          i += 2;
        } else {
          if (h == '[') throw Fail{"'[' in a class"};
          if ((unsigned char)h < 0x20 || (unsigned char)h > 0x7E) throw Fail{"non-printable pattern character"};
          hi = (unsigned char)h;
          i++;
        }
        if (hi < lo) throw Fail{"bad range"};
        st |= sym_range(lo, hi);
      } else {
        st |= sym_range(lo, lo);
      }
      any = true;
    }
    if (!any) throw Fail{"empty class"};
    return set_node(neg ? ~st : st);
  }
};

// Thompson NFA
struct NState { int type; Set set; int o1, o2; };  // type 0 CHAR(set) -> o1, 1 SPLIT o1 / o2, 2 MATCH, 3 EPS -> o1
struct Nfa {
  std::vector<NState> st;
  int add(int t, const Set& s = Set(), int o1 = -1, int o2 = -1) {
    if (st.size() >= 8192) throw Fail{"pattern too large"};
    st.push_back({t, s, o1, o2});
    return (int)st.size() - 1;
  }
};
struct Frag { int start; std::vector<int*> outs; };

// outs hold indices into st via (state, which) pairs: patched through patch()
struct Builder {
  Nfa n;
  std::vector<std::pair<int, int>> pending;  // unused
  // fragment: entry state and the list of (state, slot) to patch
  struct F { int start; std::vector<std::pair<int, int>> outs; };
  void patch(const F& f, int to) {
    for (auto& o : f.outs) (o.second == 1 ? n.st[(size_t)o.first].o1 : n.st[(size_t)o.first].o2) = to;
  }
  F build(const Ast& a) {
    switch (a.k) {
      case Ast::SET: { int s = n.add(0, a.set); return F{s, {{s, 1}}}; }
      case Ast::EMPTY: { int s = n.add(3); return F{s, {{s, 1}}}; }
      case Ast::CAT: {
        F f = build(*a.kids[0]);
        for (size_t k = 1; k < a.kids.size(); k++) {
          F g = build(*a.kids[k]);
          patch(f, g.start);
          f.outs = g.outs;
        }
        return f;
      }
      case Ast::ALT: {
        F f = build(*a.kids[0]);
        for (size_t k = 1; k < a.kids.size(); k++) {
          F g = build(*a.kids[k]);
          int s = n.add(1, Set(), f.start, g.start);
          F h{s, f.outs};
          h.outs.insert(h.outs.end(), g.outs.begin(), g.outs.end());
          f = h;
        }
        return f;
      }
      case Ast::REP: {
        const Ast& x = *a.kids[0];
        // x{lo}, then x* (unbounded) or (hi - lo) optional copies
        int e0 = n.add(3);
        F f{e0, {{e0, 1}}};
        for (int q = 0; q < a.lo; q++) {
          F g = build(x);
          patch(f, g.start);
          f.outs = g.outs;
        }
        if (a.hi < 0) {
          int sp = n.add(1);
          F g = build(x);
          n.st[(size_t)sp].o1 = g.start;
          patch(g, sp);
          patch(f, sp);
          f.outs = {{sp, 2}};
        } else {
          for (int q = a.lo; q < a.hi; q++) {
            int sp = n.add(1);
            F g = build(x);
            n.st[(size_t)sp].o1 = g.start;
            patch(f, sp);
            f.outs = g.outs;
            f.outs.push_back({sp, 2});
          }
        }
        return f;
      }
    }
    throw Fail{"internal"};
  }
};

void closure(const Nfa& n, std::vector<int>& set) {
  std::vector<char> in(n.st.size(), 0);
  std::vector<int> stack(set.begin(), set.end());
  for (int s : set) in[(size_t)s] = 1;
  while (!stack.empty()) {
    int s = stack.back();
    stack.pop_back();
    const NState& x = n.st[(size_t)s];
    auto push = [&](int t) { if (t >= 0 && !in[(size_t)t]) { in[(size_t)t] = 1; set.push_back(t); stack.push_back(t); } };
    if (x.type == 1) { push(x.o1); push(x.o2); }
    else if (x.type == 3) push(x.o1);
  }
  std::sort(set.begin(), set.end());
}

}  // namespace

bool rx_compile(const std::string& re, RxDfa* out, std::string* why) {
  try {
    std::string body = re;
    bool a0 = false, a1 = false;
    if (!body.empty() && body[0] == '^') { a0 = true; body.erase(0, 1); }
    if (!body.empty() && body.back() == '$') {
      size_t bs = 0;  // an even run of backslashes before it: an anchor, else an escaped '$'
      for (size_t j = body.size() - 1; j > 0 && body[j - 1] == '\\'; j--) bs++;
      if (bs % 2 == 0) { a1 = true; body.pop_back(); }
    }
    Parser p(body);
    AP ast = p.alt();
    if (!p.at_end()) throw Fail{"unbalanced ')'"};
    if ((a0 || a1) && ast->k == Ast::ALT) throw Fail{"anchor with top-level alternation"};
    Builder b;
    Builder::F f = b.build(*ast);
    int m = b.n.add(2);
    b.patch(f, m);
    int start = f.start;
    if (!a0) {  // search: any prefix, then the pattern
      int sp = b.n.add(1, Set(), -1, f.start);
      int any = b.n.add(0, ~Set(), sp);
      b.n.st[(size_t)sp].o1 = any;
      start = sp;
    }
    // subset construction
    std::map<std::vector<int>, uint32_t> ids;
    std::vector<std::vector<int>> sets;
    std::vector<int> s0{start};
    closure(b.n, s0);
    ids[s0] = 0;
    sets.push_back(s0);
    RxDfa d;
    d.end_anchor = a1;
    for (size_t q = 0; q < sets.size(); q++) {
      if (sets.size() > RX_MAX_STATES) throw Fail{"too many DFA states"};
      const std::vector<int> cur = sets[q];
      bool acc = false;
      for (int s : cur) acc = acc || b.n.st[(size_t)s].type == 2;
      d.accept.push_back(acc ? 1 : 0);
      d.next.resize((q + 1) * kSyms);
      for (int c = 0; c < kSyms; c++) {
        std::vector<int> nx;
        for (int s : cur) {
          const NState& x = b.n.st[(size_t)s];
          if (x.type == 0 && x.set.test((size_t)c)) nx.push_back(x.o1);
        }
        std::sort(nx.begin(), nx.end());
        nx.erase(std::unique(nx.begin(), nx.end()), nx.end());
        closure(b.n, nx);
        auto it = ids.find(nx);
        uint32_t id;
        if (it == ids.end()) {
          id = (uint32_t)sets.size();
          ids.emplace(nx, id);
          sets.push_back(nx);
        } else {
          id = it->second;
        }
        d.next[q * kSyms + (size_t)c] = (uint16_t)id;
      }
    }
    if (sets.size() > RX_MAX_STATES) throw Fail{"too many DFA states"};
    d.nstates = (uint32_t)sets.size();
    *out = std::move(d);
    return true;
  } catch (Fail& f) {
    if (why) *why = f.why;
    return false;
  }
}

int rx_match(const RxDfa& d, const uint8_t* s, size_t n) {
  uint32_t st = 0;
  bool hit = !d.end_anchor && d.accept[0];
  for (size_t i = 0; i < n; i++) {
    const uint8_t c = s[i];
    if (c < 0x20 || c > 0x7E) return -1;
    if (hit) continue;  // (the subject is still checked for bytes outside the subset)
    st = d.next[(size_t)st * RX_SYMS + (c - 0x20)];
    if (!d.end_anchor && d.accept[st]) hit = true;
  }
  if (d.end_anchor) hit = d.accept[st] != 0;
  return hit ? 1 : 0;
}

}  // namespace kyv
