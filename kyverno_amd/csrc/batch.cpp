// Flattener: resource JSON -> columnar node tables + interned dictionary (host, multithreaded).
//
// Reference accessors restated for the per-resource header (k8s.io/apimachinery unstructured, used by
// pkg/engine/utils.go:71-160): GetKind/GetName/GetGenerateName/GetNamespace (NestedString -> "" unless a
// string), GetLabels/GetAnnotations (NestedStringMap -> nil unless a map of strings), GroupVersionKind
// (ParseGroupVersion; more than one '/' -> empty GVK).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <chrono>
#include <cstring>
#include <deque>
#include <emmintrin.h>
#include <memory>
#include <string_view>
#include <thread>

#include "kyv_host.h"
#include "kyv_pss.h"

namespace kyv {
using pj::T;
using pj::Value;

Batch::~Batch() {}

namespace {

template <class F>
void parallel_for(size_t n, int T, F&& f) {  // f(k) for k in [0, n) over min(T, n) threads (the caller is one)
  if (n == 0) return;
  size_t t = std::min<size_t>((size_t)std::max(1, T), n);
  if (t <= 1) { for (size_t k = 0; k < n; k++) f(k); return; }
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (;;) {
      size_t k = next.fetch_add(1);
      if (k >= n) break;
      f(k);
    }
  };
  std::vector<std::thread> th;
  for (size_t q = 1; q < t; q++) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
}

bool magic(std::string_view s) {
  if (s.size() < 22 || s.find("anchor") == std::string_view::npos) return false;
  return s.find("negation anchor matched in resource") != std::string_view::npos ||
         s.find("conditional anchor mismatch") != std::string_view::npos ||
         s.find("global anchor mismatch") != std::string_view::npos;
}

bool go_space(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

bool is_anchor_key(std::string_view s, const char* tag) {  // key that anchor.Parse() maps onto tag
  while (!s.empty() && go_space((unsigned char)s.front())) s.remove_prefix(1);
  while (!s.empty() && go_space((unsigned char)s.back())) s.remove_suffix(1);
  if (s.size() < 3 || s.back() != ')') return false;
  size_t p = (s[0] == '+' || s[0] == '<' || s[0] == '=' || s[0] == 'X' || s[0] == '^') ? 1 : 0;
  if (s[p] != '(') return false;
  return s.substr(p + 1, s.size() - p - 2) == tag;
}

inline uint64_t hash_bytes(const char* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)n * 0xff51afd7ed558ccdull);
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    h = (h ^ w) * 0xbf58476d1ce4e5b9ull;
    h ^= h >> 31;
    p += 8;
    n -= 8;
  }
  uint64_t w = 0;
  if (n) memcpy(&w, p, n);  // (an empty string_view may carry a null pointer)
  h = (h ^ w ^ ((uint64_t)n << 56)) * 0x94d049bb133111ebull;
  h ^= h >> 29;
  h *= 0xbf58476d1ce4e5b9ull;
  h ^= h >> 32;
  return h;
}

// Open-addressing string table over views (into the input buffer, the ruleset dictionary or owned storage).
// Ids are dense in insertion order.
struct StrTab {
  std::vector<std::string_view> strs;
  std::vector<uint64_t> hashes;
  std::vector<uint64_t> slots;  // (hash high 32 bits << 32) | (id + 1); 0 = empty
  std::deque<std::string> own;  // unescaped / formatted strings that are not in any input buffer
  uint64_t mask = 0;
  StrTab() { rehash(64); }
  static uint64_t tag(uint64_t h) { return h & 0xFFFFFFFF00000000ull; }
  void rehash(size_t cap) {
    slots.assign(cap, 0);
    mask = cap - 1;
    for (uint32_t id = 0; id < strs.size(); id++) {
      uint64_t p = hashes[id] & mask;
      while (slots[p]) p = (p + 1) & mask;
      slots[p] = tag(hashes[id]) | (id + 1);
    }
  }
  uint32_t find(std::string_view s, uint64_t h) const {
    const uint64_t t = tag(h);
    for (uint64_t p = h & mask;; p = (p + 1) & mask) {
      uint64_t e = slots[p];
      if (!e) return NONE;
      uint32_t id = (uint32_t)e - 1;
      if ((e & 0xFFFFFFFF00000000ull) == t && strs[id] == s) return id;
    }
  }
  // returns the id; *added set when the string was new (its view must then outlive the table)
  uint32_t add(std::string_view s, uint64_t h, bool* added) {
    const uint64_t t = tag(h);
    uint64_t p = h & mask;
    for (;; p = (p + 1) & mask) {
      uint64_t e = slots[p];
      if (!e) break;
      uint32_t id = (uint32_t)e - 1;
      if ((e & 0xFFFFFFFF00000000ull) == t && strs[id] == s) { *added = false; return id; }
    }
    uint32_t id = (uint32_t)strs.size();
    strs.push_back(s);
    hashes.push_back(h);
    slots[p] = t | (id + 1);
    *added = true;
    if ((strs.size() + 1) * 2 > slots.size()) rehash(slots.size() * 2);
    return id;
  }
};

enum : uint8_t { LF_MAGIC = 1, LF_ANCHORISH = 2 };
// chunk-local ids interned first, in this order, by every chunk
enum : uint32_t { L_EMPTY, L_KIND, L_APIVERSION, L_METADATA, L_NAME, L_GENNAME, L_NAMESPACE, L_LABELS, L_ANN, L_SPEC,
                  L_TEMPLATE, L_JOBTEMPLATE, L_FIXED };
const char* const kLocalFixed[L_FIXED] = {"", "kind", "apiVersion", "metadata", "name", "generateName", "namespace",
                                          "labels", "annotations", "spec", "template", "jobTemplate"};

// one worker's share of the documents: nodes, headers and float forms with chunk-local string ids, remapped to
// batch ids after the parallel phase
struct Chunk {
  StrTab tab;
  std::vector<uint8_t> lflags;  // per local id
  std::vector<Node> nodes;
  std::vector<ResHeader> hdr;
  std::vector<FloatAux> faux;
  std::string err;
  Chunk() { for (const char* s : kLocalFixed) local(s); }
  uint32_t local(std::string_view s) { return local(s, hash_bytes(s.data(), s.size())); }
  // direct-mapped front cache of short strings (bytes held inline, so a hit touches one line and no table memory)
  struct Hot { uint64_t h; uint32_t id; uint32_t len; char b[16]; };
  std::vector<Hot> hot = std::vector<Hot>(1024, Hot{0, NONE, 0, {}});
  uint32_t local(std::string_view s, uint64_t h) {
    Hot* e = nullptr;
    if (s.size() <= 16) {
      e = &hot[(h >> 20) & 1023];
      if (e->h == h && e->len == s.size() && e->id != NONE && (s.empty() || memcmp(e->b, s.data(), s.size()) == 0))
        return e->id;
    }
    uint32_t id = intern(s, h);
    if (e) {
      e->h = h;
      e->id = id;
      e->len = (uint32_t)s.size();
      if (!s.empty()) memcpy(e->b, s.data(), s.size());
    }
    return id;
  }
  uint32_t intern(std::string_view s, uint64_t h) {
    bool added;
    uint32_t id = tab.add(s, h, &added);
    if (added) lflags.push_back((magic(s) ? LF_MAGIC : 0) |
                                (is_anchor_key(s, "labels") || is_anchor_key(s, "annotations") ? LF_ANCHORISH : 0));
    return id;
  }
  uint32_t local_owned(std::string&& s) {
    uint64_t h = hash_bytes(s.data(), s.size());
    uint32_t id = tab.find(s, h);
    if (id != NONE) return id;
    tab.own.push_back(std::move(s));
    return local(tab.own.back(), h);
  }
};

// Streaming flattener: one pass over a document's bytes emits its node table directly (children blocks in
// post-order, the root at relative node 0), with the JSON grammar, escapes, UTF-8 repair, number classification
// and duplicate-key rule (last value wins) of the pjson reader the rest of the library uses (pjson.cpp).
struct Flat {
  const char* s;
  size_t n, i = 0;
  Chunk& ch;
  std::vector<Node> out;
  std::vector<Node> pend;  // children of the containers being parsed, innermost last
  std::string tmp;
  bool magicf = false, anchorish = false;
  explicit Flat(Chunk& c) : s(nullptr), n(0), ch(c) {}

  [[noreturn]] void fail(const char* m) { throw pj::Error(std::string("json: ") + m + " at offset " + std::to_string(i)); }
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
  // string at s[i] == '"' -> chunk-local id
  uint32_t str() {
    size_t st = ++i;
    // 16 bytes at a time: stop at '"', '\\', control bytes and non-ASCII bytes (signed compare: >= 0x80 is < 0)
    const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), sp = _mm_set1_epi8(0x20);
    while (i + 16 <= n) {
      __m128i v = _mm_loadu_si128((const __m128i*)(s + i));
      __m128i hit = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, q), _mm_cmpeq_epi8(v, bs)), _mm_cmplt_epi8(v, sp));
      int m = _mm_movemask_epi8(hit);
      if (m) { i += __builtin_ctz(m); break; }
      i += 16;
    }
    for (;;) {
      if (i >= n) fail("unterminated string");
      unsigned char c = s[i];
      if (c == '"') { i++; return ch.local(std::string_view(s + st, i - 1 - st)); }
      if (c == '\\' || c < 0x20 || c >= 0x80) break;
      i++;
    }
    // escapes, control characters or non-ASCII: the pjson string rules (UTF-8 repaired to U+FFFD)
    tmp.assign(s + st, i - st);
    size_t run = i;
    bool changed = false;
    for (;;) {
      if (i >= n) fail("unterminated string");
      unsigned char c = s[i];
      if (c == '"') {
        tmp.append(s + run, i - run);
        i++;
        if (!changed) return ch.local(std::string_view(s + st, i - 1 - st));
        return ch.local_owned(std::move(tmp));
      }
      if (c == '\\') {
        changed = true;
        tmp.append(s + run, i - run);
        i++;
        if (i >= n) fail("bad escape");
        char e = s[i++];
        switch (e) {
          case '"': tmp += '"'; break;
          case '\\': tmp += '\\'; break;
          case '/': tmp += '/'; break;
          case 'b': tmp += '\b'; break;
          case 'f': tmp += '\f'; break;
          case 'n': tmp += '\n'; break;
          case 'r': tmp += '\r'; break;
          case 't': tmp += '\t'; break;
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
            pj::utf8_put(tmp, r);
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
      int w = pj::utf8_dec(s, n, i, &r);
      if (r == 0xFFFD && w == 1) {
        changed = true;
        tmp.append(s + run, i - run);
        pj::utf8_put(tmp, 0xFFFD);
        i++;
        run = i;
        continue;
      }
      i += w;
    }
  }
  void num(Node& nd) {
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
    std::string_view lit(s + st, i - st);
    if (integral) {
      int64_t v;
      bool ok;
      size_t d0 = lit[0] == '-' ? 1 : 0;
      if (lit.size() - d0 <= 18) {  // fits int64 without overflow checks
        int64_t m = 0;
        for (size_t k = d0; k < lit.size(); k++) m = m * 10 + (lit[k] - '0');
        v = d0 ? -m : m;
        ok = true;
      } else {
        ok = pj::go_parse_int64(std::string(lit), &v);
      }
      if (ok) {
        nd.tk = N_INT;
        uint64_t u = (uint64_t)v;
        nd.a = (uint32_t)u;
        nd.b = (uint32_t)(u >> 32);
        nd.c = lit == "-0" ? ch.local(std::string_view("0")) : ch.local(lit);  // strconv.FormatInt form
        return;
      }
    }
    double f;
    if (!pj::go_parse_float(std::string(lit), &f)) fail("number out of range");
    nd.tk = N_FLOAT;
    uint64_t u = __builtin_bit_cast(uint64_t, f);
    nd.a = (uint32_t)u;
    nd.b = (uint32_t)(u >> 32);
    nd.c = (uint32_t)ch.faux.size();
    uint32_t e = ch.local_owned(pj::go_fmt_E(f));
    uint32_t f6 = ch.local_owned(pj::go_fmt_f6(f));
    ch.faux.push_back(FloatAux{e, f6});
  }
  // parse one value; containers append their children block to `out`
  Node val(int depth, bool metadata_map) {
    if (depth > 512) fail("nesting too deep");
    ws();
    if (i >= n) fail("unexpected end of input");
    Node nd{};
    char c = s[i];
    if (c == '{') {
      i++;
      nd.tk = N_MAP;
      size_t base = pend.size();
      std::unique_ptr<std::unordered_map<uint32_t, size_t>> big;
      ws();
      if (i < n && s[i] == '}') {
        i++;
      } else {
        for (;;) {
          ws();
          if (i >= n || s[i] != '"') fail("expected key");
          uint32_t k = str();
          uint8_t kf = ch.lflags[k];
          if (kf & LF_MAGIC) magicf = true;
          if (metadata_map && (kf & LF_ANCHORISH)) anchorish = true;
          ws();
          if (i >= n || s[i] != ':') fail("expected ':'");
          i++;
          Node x = val(depth + 1, k == L_METADATA);
          x.tk |= k << 4;
          size_t at = NONE;  // duplicate key: the later value replaces the earlier one in place
          if (big) {
            auto it = big->find(k);
            if (it != big->end()) at = it->second;
          } else {
            for (size_t q = base; q < pend.size(); q++)
              if (node_key(pend[q]) == k) { at = q; break; }
          }
          if (at != (size_t)NONE) {
            pend[at] = x;
          } else {
            if (big) big->emplace(k, pend.size());
            pend.push_back(x);
            if (!big && pend.size() - base > 32) {
              big = std::make_unique<std::unordered_map<uint32_t, size_t>>();
              for (size_t q = base; q < pend.size(); q++) big->emplace(node_key(pend[q]), q);
            }
          }
          ws();
          if (i < n && s[i] == ',') { i++; continue; }
          if (i < n && s[i] == '}') { i++; break; }
          fail("expected ',' or '}'");
        }
      }
      size_t cnt = pend.size() - base;
      if (cnt > 0xFFFF) magicf = true;  // walk frames count entries in 16 bits
      nd.a = (uint32_t)out.size();
      nd.b = (uint32_t)cnt;
      out.insert(out.end(), pend.begin() + base, pend.end());
      pend.resize(base);
      return nd;
    }
    if (c == '[') {
      i++;
      nd.tk = N_ARR;
      nd.c = NONE;  // path-column row of element 0, set by resolve_path_columns
      size_t base = pend.size();
      ws();
      if (i < n && s[i] == ']') {
        i++;
      } else {
        for (uint32_t k = 0;; k++) {
          Node x = val(depth + 1, false);
          x.tk |= k << 4;
          pend.push_back(x);
          ws();
          if (i < n && s[i] == ',') { i++; continue; }
          if (i < n && s[i] == ']') { i++; break; }
          fail("expected ',' or ']'");
        }
      }
      size_t cnt = pend.size() - base;
      if (cnt > 0xFFFF) magicf = true;  // walk frames count elements in 16 bits
      nd.a = (uint32_t)out.size();
      nd.b = (uint32_t)cnt;
      out.insert(out.end(), pend.begin() + base, pend.end());
      pend.resize(base);
      return nd;
    }
    if (c == '"') {
      nd.tk = N_STR;
      nd.a = str();
      if (ch.lflags[nd.a] & LF_MAGIC) magicf = true;
      return nd;
    }
    if (c == 't' && n - i >= 4 && memcmp(s + i, "true", 4) == 0) { i += 4; nd.tk = N_TRUE; nd.a = 1; return nd; }
    if (c == 'f' && n - i >= 5 && memcmp(s + i, "false", 5) == 0) { i += 5; nd.tk = N_FALSE; return nd; }
    if (c == 'n' && n - i >= 4 && memcmp(s + i, "null", 4) == 0) { i += 4; nd.tk = N_NULL; return nd; }
    if (c == '-' || (c >= '0' && c <= '9')) { num(nd); return nd; }
    fail("unexpected character");
  }

  // one document -> node table + header (unstructured accessors on the final values)
  void doc(const char* p, size_t len) {
    s = p; n = len; i = 0;
    magicf = anchorish = false;
    out.clear();
    out.resize(1);
    Node root = val(0, false);
    ws();
    if (i != n) fail("trailing data");
    out[0] = root;
    ResHeader h{};
    h.root = (uint32_t)ch.nodes.size();
    h.nnodes = (uint32_t)out.size();
    h.labels = h.ann = h.nsl = NONE;
    uint32_t kind = L_EMPTY, av = L_EMPTY, name = L_EMPTY, gen = L_EMPTY, ns = L_EMPTY;
    auto child = [&](uint32_t m, uint32_t key) -> uint32_t {  // relative index of the entry with key, NONE
      if (m == NONE || node_type(out[m]) != N_MAP) return NONE;
      for (uint32_t q = 0; q < out[m].b; q++) if (node_key(out[out[m].a + q]) == key) return out[m].a + q;
      return NONE;
    };
    auto sval = [&](uint32_t x) { return x != NONE && node_type(out[x]) == N_STR ? out[x].a : (uint32_t)L_EMPTY; };
    kind = sval(child(0, L_KIND));
    av = sval(child(0, L_APIVERSION));
    uint32_t meta = child(0, L_METADATA);
    if (meta != NONE && node_type(out[meta]) == N_MAP) {
      name = sval(child(meta, L_NAME));
      gen = sval(child(meta, L_GENNAME));
      ns = sval(child(meta, L_NAMESPACE));
      auto smap = [&](uint32_t x) -> uint32_t {  // NestedStringMap: a map whose values are all strings
        if (x == NONE || node_type(out[x]) != N_MAP) return NONE;
        for (uint32_t q = 0; q < out[x].b; q++) if (node_type(out[out[x].a + q]) != N_STR) return NONE;
        return x;
      };
      h.labels = smap(child(meta, L_LABELS));
      h.ann = smap(child(meta, L_ANN));
    }
    h.kind = kind;
    h.name = name;
    h.gen_name = gen;
    h.ns = ns;
    std::string_view avs = ch.tab.strs[av];
    size_t sl = std::count(avs.begin(), avs.end(), '/');
    std::string_view g, ver;
    bool gvok = true;
    if (avs.empty() || avs == "/") {}
    else if (sl == 0) ver = avs;
    else if (sl == 1) { g = avs.substr(0, avs.find('/')); ver = avs.substr(avs.find('/') + 1); }
    else gvok = false;
    h.gvk_kind = gvok ? kind : (uint32_t)L_EMPTY;
    h.group = ch.local(g);
    h.version = ch.local(ver);
    h.gv = g.empty() ? h.version : av;  // GroupVersion().String(): "group/version" is the apiVersion itself
    h.flags = (magicf ? RF_MAGIC : 0) | (anchorish ? RF_ANCHORISH : 0) | (node_type(root) == N_MAP ? RF_ROOT_MAP : 0);
    // ExpandInMetadata's type assertions for the metadata of the root and of the two pod-template positions
    auto meta_flags = [&](uint32_t m, uint32_t shift) {  // m: the map holding `metadata` (NONE: not a map there)
      if (m == NONE || node_type(out[m]) != N_MAP) return;
      const uint32_t md = child(m, L_METADATA);
      if (md == NONE || node_type(out[md]) == N_NULL) { h.flags |= 1u << shift; return; }
      if (node_type(out[md]) != N_MAP) { h.flags |= 2u << shift; return; }
      auto bad = [&](uint32_t x) {  // present, not null, not a map of strings
        if (x == NONE || node_type(out[x]) == N_NULL) return false;
        if (node_type(out[x]) != N_MAP) return true;
        for (uint32_t q = 0; q < out[x].b; q++) if (node_type(out[out[x].a + q]) != N_STR) return true;
        return false;
      };
      if (bad(child(md, L_LABELS))) h.flags |= 4u << shift;
      if (bad(child(md, L_ANN))) h.flags |= 8u << shift;
    };
    meta_flags(0, RF_META_SHIFT);
    {
      const uint32_t sp = child(0, L_SPEC);
      meta_flags(child(sp, L_TEMPLATE), RF_TMETA1_SHIFT);
      const uint32_t jt = child(sp, L_JOBTEMPLATE);
      meta_flags(child(child(jt, L_SPEC), L_TEMPLATE), RF_TMETA2_SHIFT);
    }
    ch.hdr.push_back(h);
    ch.nodes.insert(ch.nodes.end(), out.begin(), out.end());
  }
};

// split a JSON array / concatenated documents into document byte ranges (serial; any input form)
std::vector<std::pair<size_t, size_t>> split_docs(const char* p, size_t n) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t i = 0;
  while (i < n && isspace((unsigned char)p[i])) i++;
  bool array = i < n && p[i] == '[';
  if (array) i++;
  while (i < n) {
    while (i < n && (isspace((unsigned char)p[i]) || (array && p[i] == ','))) i++;
    if (i >= n || (array && p[i] == ']')) break;
    size_t st = i;
    int depth = 0;
    bool in_str = false;
    for (; i < n; i++) {
      char c = p[i];
      if (in_str) {
        if (c == '\\') i++;
        else if (c == '"') in_str = false;
        continue;
      }
      if (c == '"') in_str = true;
      else if (c == '{' || c == '[') depth++;
      else if (c == '}' || c == ']') {
        depth--;
        if (depth == 0) { i++; break; }
      } else if (depth == 0 && (c == ',' || c == '\n')) break;
    }
    if (i == st) i++;  // a stray separator: a one-byte document that fails to parse
    out.push_back({st, i - st});
  }
  return out;
}

// NDJSON fast path: one document per non-blank line (JSON strings cannot hold a raw newline), found with memchr in
// parallel. Returns false for input that is not line-delimited objects; a line that turns out not to be exactly one
// document fails its parse and the caller re-splits serially.
bool split_lines(const char* p, size_t n, int T, std::vector<std::pair<size_t, size_t>>* docs) {
  size_t i = 0;
  while (i < n && isspace((unsigned char)p[i])) i++;
  if (i >= n || p[i] != '{') return false;
  size_t parts = std::max<size_t>(1, std::min<size_t>((size_t)T * 4, n / (1 << 20) + 1));
  std::vector<std::vector<std::pair<size_t, size_t>>> part(parts);
  // part k owns the lines that start in [n*k/parts, n*(k+1)/parts)
  parallel_for(parts, T, [&](size_t k) {
    size_t lo = n * k / parts, hi = n * (k + 1) / parts;
    size_t a = lo;
    if (lo > 0 && p[lo - 1] != '\n') {  // the line running through lo belongs to an earlier part
      const char* e = (const char*)memchr(p + lo, '\n', n - lo);
      if (!e) return;
      a = (size_t)(e - p) + 1;
    }
    while (a < hi) {
      const char* e = (const char*)memchr(p + a, '\n', n - a);
      size_t b = e ? (size_t)(e - p) : n;
      size_t x = a, y = b;
      while (x < y && isspace((unsigned char)p[x])) x++;
      while (y > x && isspace((unsigned char)p[y - 1])) y--;
      if (y > x) part[k].push_back({x, y - x});
      a = b + 1;
    }
  });
  size_t tot = 0;
  for (auto& v : part) tot += v.size();
  docs->clear();
  docs->reserve(tot);
  for (auto& v : part) docs->insert(docs->end(), v.begin(), v.end());
  return true;
}

}  // namespace

void derive_strings(Batch& b, size_t from, int threads) {
  size_t n = b.dict.strs.size();
  // the PodSecurity checks' fixed prefixes (seeded well-known strings)
  const std::string pfx_aa = b.dict.strs[KSID(APPARMOR_PREFIX)], pfx_lh = b.dict.strs[KSID(LOCALHOST_PREFIX)],
                    pfx_sc = b.dict.strs[KSID(SECCOMP_CONTAINER_PREFIX)];
  std::vector<uint32_t> gidx;  // ruleset glob-mask index + 1 per (seeded) pattern string
  if (b.rs) {
    gidx.assign(std::min(n, b.rs->dict.strs.size()), 0);
    for (size_t g = 0; g < b.rs->gpats.size(); g++) if (b.rs->gpats[g] < gidx.size()) gidx[b.rs->gpats[g]] = (uint32_t)g + 1;
  }
  b.str_flags.resize(n);
  b.str_dur.resize(n);
  b.str_qty.resize(2 * n);
  b.str_f64.resize(n);
  std::atomic<size_t> next{from};
  auto work = [&]() {
    for (;;) {
      size_t s0 = next.fetch_add(4096);
      if (s0 >= n) break;
      size_t s1 = std::min(n, s0 + 4096);
      for (size_t s = s0; s < s1; s++) {
        const std::string& x = b.dict.strs[s];
        uint32_t f = 0;
        bool ascii = true;
        for (unsigned char c : x) if (c >= 0x80) { ascii = false; break; }
        if (ascii) f |= SF_ASCII;
        if (!ascii || x.find_first_of("*?") != std::string::npos) f |= SF_GLOBBY;
        {  // SF_PLAIN (kyv_layout.h): as a pattern string, only the string itself (or a bool's FormatBool) matches it
          const char h = x.empty() ? 0 : x[0];
          const bool plain = ascii && x.find_first_of("|&*?") == std::string::npos &&
                             (x.empty() || (x.front() != ' ' && x.back() != ' ')) &&
                             !(x.size() >= 2 && (h == '<' || h == '>' || h == '!')) &&
                             !((h >= '0' && h <= '9') || h == '+' || h == '-' || h == '.');
          if (plain) f |= SF_PLAIN;
        }
        if (s < gidx.size()) f |= gidx[s] << SF_GIDX_SHIFT;
        if (x.compare(0, pfx_aa.size(), pfx_aa) == 0) f |= SF_PFX_APPARMOR;
        if (x.compare(0, pfx_lh.size(), pfx_lh) == 0) f |= SF_PFX_LOCALHOST;
        if (x.compare(0, pfx_sc.size(), pfx_sc) == 0) f |= SF_PFX_SECCOMP_C;
        // time.ParseDuration and resource.ParseQuantity need a sign, digit or '.' first; strconv.ParseFloat also
        // accepts inf / infinity / nan spellings -- every other string skips the parsers
        const char c0 = x.empty() ? 0 : x[0];
        const bool numish = (c0 >= '0' && c0 <= '9') || c0 == '+' || c0 == '-' || c0 == '.';
        int64_t d;
        if (numish && pj::go_parse_duration(x, &d)) { f |= SF_DUR; b.str_dur[s] = d; } else b.str_dur[s] = 0;
        int64_t lo, hi;
        int q = numish ? pj::go_parse_quantity(x, &lo, &hi) : 0;
        if (q == 1) { f |= SF_QTY; b.str_qty[2 * s] = lo; b.str_qty[2 * s + 1] = hi; }
        else { b.str_qty[2 * s] = 0; b.str_qty[2 * s + 1] = 0; if (q == 2) f |= SF_QTY_BIG; }
        double fv;
        const bool floatish = numish || c0 == 'i' || c0 == 'I' || c0 == 'n' || c0 == 'N';
        if (floatish && pj::go_parse_float(x, &fv)) { f |= SF_FLOAT; b.str_f64[s] = fv; } else b.str_f64[s] = 0;
        {  // strconv.ParseInt(x, 10, 64): optional sign, decimal digits, int64 range
          size_t i0 = (!x.empty() && (x[0] == '+' || x[0] == '-')) ? 1 : 0;
          bool digits = x.size() > i0;
          for (size_t i = i0; i < x.size() && digits; i++) digits = x[i] >= '0' && x[i] <= '9';
          if (digits) {
            unsigned __int128 m = 0;
            bool ovf = false;
            for (size_t i = i0; i < x.size() && !ovf; i++) { m = m * 10 + (unsigned)(x[i] - '0'); ovf = m > ((unsigned __int128)1 << 63); }
            bool neg = i0 && x[0] == '-';
            if (!ovf && (neg || m < ((unsigned __int128)1 << 63))) {
              f |= SF_INT;
              if (m > ((unsigned __int128)1 << 53)) f |= SF_INT_BIG;
            }
          }
          if (!x.empty() && x[0] >= '0' && x[0] <= '9' && std::count(x.begin(), x.end(), '.') >= 2) f |= SF_SEMVERISH;
        }
        // label key / value validity (apimachinery validation.IsQualifiedName / IsValidLabelValue)
        auto qn = [](const std::string& nm) {
          if (nm.empty() || nm.size() > 63) return false;
          auto an = [](char c) { return isalnum((unsigned char)c) != 0; };
          if (!an(nm.front()) || !an(nm.back())) return false;
          for (char c : nm) if (!(an(c) || c == '-' || c == '_' || c == '.')) return false;
          return true;
        };
        auto dns = [](const std::string& z) {
          if (z.empty() || z.size() > 253) return false;
          size_t st = 0;
          for (size_t i = 0; i <= z.size(); i++) {
            if (i == z.size() || z[i] == '.') {
              std::string l = z.substr(st, i - st);
              st = i + 1;
              if (l.empty()) return false;
              auto ok = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
              if (!ok(l.front()) || !ok(l.back())) return false;
              for (char c : l) if (!(ok(c) || c == '-')) return false;
            }
          }
          return true;
        };
        size_t slash = x.find('/');
        bool lkey;
        if (slash == std::string::npos) lkey = qn(x);
        else if (x.find('/', slash + 1) != std::string::npos) lkey = false;
        else lkey = slash > 0 && dns(x.substr(0, slash)) && qn(x.substr(slash + 1));
        if (lkey) f |= SF_LKEY;
        if (x.empty() || qn(x)) f |= SF_LVAL;
        if (magic(x)) f |= SF_MAGIC;
        b.str_flags[s] = f;
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < std::max(1, threads); t++) th.emplace_back(work);
  for (auto& t : th) t.join();
  // heap
  b.str_off.resize(n);
  b.str_len.resize(n);
  size_t off = from ? b.heap.size() : 0;
  if (!from) b.heap.clear();
  size_t total = off;
  for (size_t s = from; s < n; s++) total += b.dict.strs[s].size();
  b.heap.resize(total + 16);
  for (size_t s = from; s < n; s++) {
    const std::string& x = b.dict.strs[s];
    b.str_off[s] = (uint32_t)off;
    b.str_len[s] = (uint32_t)x.size();
    memcpy(b.heap.data() + off, x.data(), x.size());
    off += x.size();
  }
  if (total > 0xFFFFFFFFull) throw std::runtime_error("string heap exceeds 4 GiB per batch");
}

// Kind gate of one compiled rule: the gvk kinds its match block can accept (MatchesResourceDescription
// checks kinds first, utils.go:81-85). `any` when some reachable filter has no kinds or "*", when the empty
// OldResource retry may match, or when the match program fell back.
KindGate rule_gate(const Ruleset& rs, const RuleDesc& rd) {
  KindGate g;
  if (rd.empty_may_match || rd.match.mode == MM_NONE) { g.any = true; return g; }
  const MatchBlock& m = rd.match;
  bool any_filter = false;
  for (uint32_t i = 0; i < m.nfilters; i++) {
    const Filter& f = rs.filters[m.filters + i];
    if (m.mode == MM_ANY && (f.flags & FF_ZERO_RD)) continue;  // never matches in match.any
    if (f.nkinds == 0) {
      if (m.mode == MM_ANY) { g.any = true; return g; }
      continue;  // match.all: another filter may still constrain the kind
    }
    std::vector<uint32_t> ks;
    for (uint32_t j = 0; j < f.nkinds; j++) {
      const KindDesc& k = rs.kinds[f.kinds + j];
      if (k.kind == NONE) { ks.clear(); break; }
      ks.push_back(k.kind);
    }
    if (ks.empty()) {  // "*"
      if (m.mode == MM_ANY) { g.any = true; return g; }
      continue;
    }
    if (m.mode == MM_ANY) {
      g.kinds.insert(g.kinds.end(), ks.begin(), ks.end());
      any_filter = true;
    } else if (!any_filter) {  // all/plain: every filter must accept the kind; the first kinds list bounds it
      g.kinds = ks;
      any_filter = true;
    }
  }
  if (!any_filter && m.mode != MM_ANY) g.any = true;  // no filter constrains kinds
  return g;
}

// Stable sort of the headers by kind class + the per-class rule gate table.
void order_by_kind(Batch& b) {
  const Ruleset& rs = *b.rs;
  size_t n = b.hdr.size(), nr = rs.rules.size();
  std::unordered_map<uint32_t, uint32_t> cls;  // gvk_kind sid -> class
  std::vector<uint32_t> cls_kind;
  std::vector<uint32_t> cls_count;
  for (auto& h : b.hdr) {
    auto it = cls.find(h.gvk_kind);
    if (it == cls.end()) {
      it = cls.emplace(h.gvk_kind, (uint32_t)cls_kind.size()).first;
      cls_kind.push_back(h.gvk_kind);
      cls_count.push_back(0);
    }
    h.kclass = it->second;
    cls_count[it->second]++;
  }
  b.nclass = (uint32_t)cls_kind.size();
  b.gate_words = (uint32_t)((nr + 31) / 32);
  b.gate.assign((size_t)std::max<uint32_t>(b.nclass, 1) * std::max<uint32_t>(b.gate_words, 1), 0);
  for (size_t k = 0; k < nr; k++) {
    KindGate g = rule_gate(rs, rs.rules[k]);
    for (uint32_t c = 0; c < b.nclass; c++) {
      bool on = g.any || std::find(g.kinds.begin(), g.kinds.end(), cls_kind[c]) != g.kinds.end();
      if (on) b.gate[(size_t)c * b.gate_words + k / 32] |= 1u << (k % 32);
    }
  }
  // counting sort by class (stable)
  std::vector<uint32_t> start(b.nclass + 1, 0);
  for (uint32_t c = 0; c < b.nclass; c++) start[c + 1] = start[c] + cls_count[c];
  bulk_vector<ResHeader> sorted(n);
  b.order.resize(n);
  b.inv.resize(n);
  for (size_t i = 0; i < n; i++) {
    ResHeader h = b.hdr[i];
    uint32_t pos = start[h.kclass]++;
    h.orig = (uint32_t)i;
    sorted[pos] = h;
    b.order[pos] = (uint32_t)i;
    b.inv[i] = pos;
  }
  b.hdr.swap(sorted);
}

Batch* build_batch(const Ruleset* rs, const char* json, size_t len, const char* nsl_json, size_t nsl_len, int threads,
                   std::string* err) {
  auto b = std::make_unique<Batch>();
  const bool stats = getenv("KYV_DEBUG_STATS") != nullptr;
  auto t0 = std::chrono::steady_clock::now();
  auto phase = [&](const char* what) {
    if (!stats) return;
    auto t1 = std::chrono::steady_clock::now();
    fprintf(stderr, "[kyvgpu] flatten %-12s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(t1 - t0).count());
    t0 = t1;
  };
  try {
    b->rs = rs;
    b->dict.strs = rs->dict.strs;  // batch strings are appended; the batch needs no reverse map after the build
    const int T0 = std::max(1, threads);
    std::vector<std::pair<size_t, size_t>> docs;
    bool lines = split_lines(json, len, T0, &docs);
    if (!lines) docs = split_docs(json, len);
    phase("split");
    // threads scaled to the work: thread start-up is tens of microseconds, which dominates small (admission)
    // batches when every phase spawns the machine's thread count
    int T = 1;
    std::vector<Chunk> chunks;
    auto parse_all = [&]() {
      T = std::max(1, std::min(T0, (int)(docs.size() / 256) + 1));
      // chunks of at most ~2k documents keep each chunk's string table cache-resident while it is parsed
      size_t nchunks = std::max<size_t>(1, std::min(docs.size(), std::max((size_t)T * 8, docs.size() / 2048)));
      chunks.clear();
      chunks.resize(nchunks);
      parallel_for(nchunks, T, [&](size_t c) {
        Chunk& ch = chunks[c];
        Flat f(ch);
        size_t d0 = docs.size() * c / nchunks, d1 = docs.size() * (c + 1) / nchunks;
        try {
          for (size_t d = d0; d < d1; d++) f.doc(json + docs[d].first, docs[d].second);
        } catch (std::exception& e) {
          ch.err = e.what();
        }
      });
    };
    parse_all();
    bool bad = false;
    for (auto& c : chunks) bad = bad || !c.err.empty();
    if (bad && lines) {  // not one document per line after all: split by the JSON grammar and parse again
      docs = split_docs(json, len);
      parse_all();
    }
    for (auto& c : chunks) if (!c.err.empty()) throw std::runtime_error(c.err);
    const size_t nchunks = chunks.size();
    phase("parse");

    // batch string ids: the ruleset's dictionary keeps its ids; new strings are interned in 256 hash shards in
    // parallel, each shard in chunk order (= first-occurrence order within the shard, independent of T)
    const auto& seed = rs->dict.strs;
    const size_t nseed = seed.size();
    StrTab seedtab;
    {
      size_t cap = 64;
      while (cap < 2 * nseed + 2) cap <<= 1;
      seedtab.rehash(cap);
      bool added;
      for (auto& s : seed) seedtab.add(s, hash_bytes(s.data(), s.size()), &added);
    }
    constexpr uint32_t NSH = 256;
    auto shard_of = [](uint64_t h) { return (uint32_t)(h >> 56); };
    std::vector<std::vector<uint32_t>> remap(nchunks), grp(nchunks), goff(nchunks);
    parallel_for(nchunks, T, [&](size_t c) {
      const StrTab& tab = chunks[c].tab;
      size_t m = tab.strs.size();
      auto& rm = remap[c];
      rm.assign(m, NONE);
      std::vector<uint32_t> off(NSH + 1, 0);
      for (size_t s = 0; s < m; s++) {
        uint32_t id = seedtab.find(tab.strs[s], tab.hashes[s]);
        if (id != NONE) rm[s] = id;
        else off[shard_of(tab.hashes[s]) + 1]++;
      }
      for (uint32_t h = 0; h < NSH; h++) off[h + 1] += off[h];
      std::vector<uint32_t> pos(off.begin(), off.end() - 1);
      grp[c].resize(off[NSH]);
      for (size_t s = 0; s < m; s++)
        if (rm[s] == NONE) grp[c][pos[shard_of(tab.hashes[s])]++] = (uint32_t)s;
      goff[c].swap(off);
    });
    std::vector<StrTab> shard(NSH);
    parallel_for(NSH, T, [&](size_t h) {
      StrTab& t = shard[h];
      size_t want = 0;
      for (size_t c = 0; c < nchunks; c++) want += goff[c][h + 1] - goff[c][h];
      size_t cap = 64;
      while (cap < 2 * want + 2) cap <<= 1;
      t.rehash(cap);
      bool added;
      for (size_t c = 0; c < nchunks; c++) {
        const StrTab& tab = chunks[c].tab;
        for (uint32_t q = goff[c][h]; q < goff[c][h + 1]; q++) {
          uint32_t s = grp[c][q];
          remap[c][s] = 0x80000000u | t.add(tab.strs[s], tab.hashes[s], &added);
        }
      }
    });
    std::vector<size_t> shbase(NSH + 1, nseed);
    for (uint32_t h = 0; h < NSH; h++) shbase[h + 1] = shbase[h] + shard[h].strs.size();
    if (shbase[NSH] > 0x7FFFFFF0ull) throw std::runtime_error("batch dictionary exceeds 2^31 strings; split the batch");
    b->dict.strs.resize(shbase[NSH]);
    parallel_for(NSH, T, [&](size_t h) {
      for (size_t j = 0; j < shard[h].strs.size(); j++) b->dict.strs[shbase[h] + j].assign(shard[h].strs[j]);
    });
    parallel_for(nchunks, T, [&](size_t c) {
      const StrTab& tab = chunks[c].tab;
      for (size_t s = 0; s < remap[c].size(); s++)
        if (remap[c][s] & 0x80000000u)
          remap[c][s] = (uint32_t)(shbase[shard_of(tab.hashes[s])] + (remap[c][s] & 0x7FFFFFFFu));
    });
    std::unordered_map<std::string, uint32_t> extra;  // namespace-label strings the batch does not hold
    auto intern = [&](const std::string& s) -> uint32_t {
      uint64_t h = hash_bytes(s.data(), s.size());
      uint32_t id = seedtab.find(s, h);
      if (id != NONE) return id;
      id = shard[shard_of(h)].find(s, h);
      if (id != NONE) return (uint32_t)(shbase[shard_of(h)] + id);
      auto it = extra.find(s);
      if (it != extra.end()) return it->second;
      id = (uint32_t)b->dict.strs.size();
      b->dict.strs.push_back(s);
      extra.emplace(s, id);
      return id;
    };
    phase("merge-dict");
    // namespace label sets
    std::unordered_map<uint32_t, uint32_t> ns_set;
    b->nsl_off.push_back(0);
    if (nsl_json && nsl_len) {
      Value nsl = pj::parse(nsl_json, nsl_len, false);
      if (nsl.t == T::Obj)
        for (auto& kv : nsl.o) {
          ns_set[intern(kv.first)] = (uint32_t)b->nsl_names.size();
          b->nsl_names.push_back(kv.first);
          if (kv.second.t == T::Obj)
            for (auto& lv : kv.second.o) {
              b->nsl_kv.push_back(intern(lv.first));
              b->nsl_kv.push_back(intern(lv.second.t == T::Str ? lv.second.s : ""));
            }
          b->nsl_off.push_back((uint32_t)b->nsl_kv.size() / 2);
        }
    }
    // concatenate + remap + sort map entries by key id (+ labels / annotations entries found again after the sort)
    size_t total_nodes = 0, total_res = 0, total_faux = 0;
    std::vector<size_t> node_base(nchunks), res_base(nchunks), faux_base(nchunks);
    for (size_t c = 0; c < nchunks; c++) {
      node_base[c] = total_nodes; res_base[c] = total_res; faux_base[c] = total_faux;
      total_nodes += chunks[c].nodes.size();
      total_res += chunks[c].hdr.size();
      total_faux += chunks[c].faux.size();
    }
    if (total_nodes > 0xFFFFFFFFull) throw std::runtime_error("batch exceeds 2^32 nodes; split it");
    b->nodes.resize(total_nodes);
    b->hdr.resize(total_res);
    b->faux.resize(total_faux);
    bool pss_rules = false;
    for (auto& rd : rs->rules) pss_rules = pss_rules || rd.kind == RK_PSS;
    std::unique_ptr<TypedDecoder> typed;
    if (pss_rules)
      typed.reset(new TypedDecoder([&](const std::string& s) -> uint32_t {
        const uint64_t h = hash_bytes(s.data(), s.size());
        uint32_t id = seedtab.find(s, h);
        if (id != NONE) return id;
        id = shard[shard_of(h)].find(s, h);
        return id == NONE ? NONE : (uint32_t)(shbase[shard_of(h)] + id);
      }));
    parallel_for(nchunks, T, [&](size_t c) {
      Chunk& ch = chunks[c];
      const auto& rm = remap[c];
      for (size_t k = 0; k < ch.faux.size(); k++)
        b->faux[faux_base[c] + k] = FloatAux{rm[ch.faux[k].sid_E], rm[ch.faux[k].sid_F]};
      for (size_t r = 0; r < ch.hdr.size(); r++) {
        ResHeader h = ch.hdr[r];
        Node* R = b->nodes.data() + node_base[c] + h.root;
        const Node* src = ch.nodes.data() + h.root;
        for (uint32_t i = 0; i < h.nnodes; i++) {
          Node n = src[i];
          uint32_t t = node_type(n);
          if (t == N_STR) n.a = rm[n.a];
          else if (t == N_INT) n.c = rm[n.c];
          else if (t == N_FLOAT) n.c += (uint32_t)faux_base[c];
          R[i] = n;
        }
        for (uint32_t i = 0; i < h.nnodes; i++) {  // map entries: key ids remapped, then sorted by key
          if (node_type(R[i]) != N_MAP) continue;
          Node* ch0 = R + R[i].a;
          for (uint32_t k = 0; k < R[i].b; k++) ch0[k].tk = (rm[ch0[k].tk >> 4] << 4) | (ch0[k].tk & 0xF);
          const uint32_t m = R[i].b;
          if (m <= 24) {
            for (uint32_t a = 1; a < m; a++) {
              Node x = ch0[a];
              uint32_t z = a;
              for (; z > 0 && (ch0[z - 1].tk >> 4) > (x.tk >> 4); z--) ch0[z] = ch0[z - 1];
              ch0[z] = x;
            }
          } else {
            std::sort(ch0, ch0 + m, [](const Node& x, const Node& y) { return (x.tk >> 4) < (y.tk >> 4); });
          }
        }
        if (h.labels != NONE || h.ann != NONE) {
          auto find = [&](uint32_t m, uint32_t key) -> uint32_t {
            if (m == NONE || node_type(R[m]) != N_MAP) return NONE;
            for (uint32_t i = 0; i < R[m].b; i++) if (node_key(R[R[m].a + i]) == key) return R[m].a + i;
            return NONE;
          };
          uint32_t meta = find(0, KSID(METADATA));
          if (h.labels != NONE) h.labels = find(meta, KSID(LABELS));
          if (h.ann != NONE) h.ann = find(meta, KSID(ANNOTATIONS));
        }
        h.root = (uint32_t)(node_base[c] + h.root);
        h.kind = rm[h.kind]; h.gvk_kind = rm[h.gvk_kind]; h.group = rm[h.group]; h.version = rm[h.version];
        h.gv = rm[h.gv]; h.name = rm[h.name]; h.gen_name = rm[h.gen_name]; h.ns = rm[h.ns];
        if (pss_rules) {  // typed pod decode once per resource (eval_pss skips it on RF_PSS_DONE)
          uint32_t pm, ps;
          const uint8_t st = pss_pod(NodeTab{R}, h.kind, true, &pm, &ps);
          uint32_t f = st == ST_ERROR ? RF_PSS_DEC_ERR : 0u;
          if (!f && st != ST_PANIC) {  // the whole object, as getSpec's json.Unmarshal (typed.cpp)
            const int tgt = h.kind == KSID(POD) ? TypedDecoder::POD
                          : h.kind == KSID(CRONJOB) ? TypedDecoder::CRONJOB : TypedDecoder::DEPLOYMENT;
            const int d = typed->decode(R, b->dict.strs, tgt);
            f = d == TypedDecoder::DEC_ERR ? RF_PSS_DEC_ERR : d == TypedDecoder::DEC_FOLD ? RF_PSS_FOLD : 0u;
          }
          h.flags |= RF_PSS_DONE | f;
        }
        auto it = ns_set.find(h.ns);
        h.nsl = it == ns_set.end() ? NONE : it->second;
        b->hdr[res_base[c] + r] = h;
      }
    });
    phase("remap");
    derive_strings(*b, 0, std::max(1, std::min(T, (int)(b->dict.strs.size() / 8192) + 1)));
    phase("strings");
    order_by_kind(*b);
    phase("kind-order");
    resolve_path_columns(*b, T);
    phase("path-cols");
    // to_upper on the dictionary (round 6, kyverno functions.go:681-689 strings.ToUpper): the upper-case form of every
    // string that can reach a to_upper argument -- the values of the argument's field chain (its path column, filled
    // above) and the ruleset's literals (`|| 'default'`) -- interned, so that a result compares, globs and parses like
    // any other dictionary string (the new strings' derived columns are computed here). Strings with no lowercase
    // letter map to themselves; non-ASCII strings and strings outside that domain to NONE (the pair goes to the CPU
    // engine: a value the column does not hold, e.g. of a resource without path columns).
    if (rs->uses_upper) {
      const size_t n0 = b->dict.strs.size();
      std::vector<uint8_t> want(n0, 0);
      for (size_t s2 = 0; s2 < rs->dict.strs.size() && s2 < n0; s2++) want[s2] = 1;
      bool all = false;
      auto mark_operand = [&](const CondOperand& o) {
        if (o.kind != OK_JMES) return;
        const uint32_t* p = rs->pool.data() + o.a;
        if (!jmes_chain_form(p, o.nseg)) return;
        bool up = false;
        for (uint32_t q = 1; q < o.nseg; q += jop_width(p + q)) up = up || p[q] == JO_UPPER;
        if (!up) return;
        uint32_t t = 0;  // the chain's trie position (request.object = the resource root)
        for (uint32_t q = 1; q + 1 < o.nseg && p[q] == JO_FIELD && t != NONE; q += 2) {
          uint32_t nx = NONE;
          for (const auto& kv : rs->trie[t].kids) if (kv.first == p[q + 1]) nx = kv.second;
          t = nx;
        }
        const uint32_t col = t == NONE ? NONE : rs->trie[t].col;
        if (col == NONE || col >= b->col_off.size()) { all = true; return; }
        const size_t rows = b->rs_rows[rs->col_rowspace[col]];
        const uint64_t* cv = b->colv.data() + b->col_off[col];
        for (size_t r2 = 0; r2 < rows; r2++) {
          const uint32_t lo = (uint32_t)cv[r2];
          if (lo != NONE && (lo >> COL_TYPE_SHIFT) == N_STR && (uint32_t)(cv[r2] >> 32) < n0) want[(uint32_t)(cv[r2] >> 32)] = 1;
        }
      };
      for (const Cond& c : rs->conds) { mark_operand(c.key); mark_operand(c.value); }
      std::vector<uint32_t> up(n0, NONE);
      std::vector<uint8_t> todo(n0, 0);
      const size_t nk = std::max<size_t>(1, std::min<size_t>((size_t)T * 4, n0 / 4096 + 1));
      parallel_for(nk, T, [&](size_t k) {
        for (size_t s2 = n0 * k / nk; s2 < n0 * (k + 1) / nk; s2++) {
          if (!all && !want[s2]) continue;
          const std::string& x = b->dict.strs[s2];
          bool lower = false, ascii = true;
          for (unsigned char ch : x) { ascii = ascii && ch < 0x80; lower = lower || (ch >= 'a' && ch <= 'z'); }
          if (!ascii) continue;
          if (!lower) { up[s2] = (uint32_t)s2; continue; }
          std::string u = x;
          for (char& ch : u) if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 'a' + 'A');
          const uint64_t h = hash_bytes(u.data(), u.size());
          uint32_t id = seedtab.find(u, h);
          if (id == NONE) {
            id = shard[shard_of(h)].find(u, h);
            if (id != NONE) id = (uint32_t)(shbase[shard_of(h)] + id);
          }
          if (id != NONE) up[s2] = id;
          else todo[s2] = 1;
        }
      });
      for (size_t s2 = 0; s2 < n0; s2++)
        if (todo[s2]) {
          std::string u = b->dict.strs[s2];
          for (char& ch : u) if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 'a' + 'A');
          up[s2] = intern(u);
        }
      const size_t n1 = b->dict.strs.size();
      if (n1 > n0) derive_strings(*b, n0, std::max(1, std::min(T, (int)((n1 - n0) / 8192) + 1)));
      b->str_upper.assign(n1, NONE);
      for (size_t s2 = 0; s2 < n1; s2++) b->str_upper[s2] = s2 < n0 ? up[s2] : (uint32_t)s2;
      phase("upper");
    }
    // regex_match on the dictionary (round 6, kyverno functions.go:786-799 regexp.Match): bit q of a string = its match
    // by the ruleset's regex q (regex.cpp DFA, the device subset), RX_FB for a string with a byte outside printable
    // ASCII (its pairs go to the CPU engine)
    if (!rs->rxs.empty()) {
      const size_t ns = b->dict.strs.size();
      b->str_rx.assign(ns, 0);
      const size_t nk = std::max<size_t>(1, std::min<size_t>((size_t)T * 4, ns / 4096 + 1));
      parallel_for(nk, T, [&](size_t k) {
        for (size_t s2 = ns * k / nk; s2 < ns * (k + 1) / nk; s2++) {
          const std::string& x = b->dict.strs[s2];
          uint32_t bits = 0;
          for (size_t q = 0; q < rs->rxs.size(); q++) {
            const int m = rx_match(rs->rxs[q], (const uint8_t*)x.data(), x.size());
            if (m < 0) { bits = RX_FB; break; }
            if (m) bits |= 1u << q;
          }
          b->str_rx[s2] = bits;
        }
      });
      phase("regex");
    }
    if ((!b->str_upper.empty() && b->str_upper.size() != b->dict.strs.size()) ||
        (!b->str_rx.empty() && b->str_rx.size() != b->dict.strs.size()))
      throw std::runtime_error("internal: per-string JMESPath columns do not cover the dictionary");
    return b.release();
  } catch (std::exception& e) {
    if (err) *err = e.what();
    return nullptr;
  }
}

// Path columns (kyv_layout.h): for every resource (in kind-major order, so row space 0 rows are the kernel's
// resource positions) follow the ruleset's path trie through the node table, recording each static lookup's
// result; arrays at "[*]" trie positions get batch-wide element rows. Two passes: count element rows per
// row space per chunk, then fill from the chunk's exclusive prefix.
namespace {
struct Resolver {
  const Ruleset& rs;
  const std::vector<std::vector<std::pair<uint32_t, uint32_t>>>& kids;  // trie kids sorted by key sid
  Node* R;
  uint64_t* colv;            // nullptr in the counting pass
  const uint32_t* col_off;
  uint32_t* next;            // next free row per row space
  uint64_t entry(uint32_t x) const {
    return ((uint64_t)R[x].a << 32) | ((uint64_t)node_type(R[x]) << COL_TYPE_SHIFT) | x;
  }
  static uint32_t find(const Node* R, const Node& m, uint32_t key) {
    uint32_t lo = m.a, hi = m.a + m.b;
    while (lo < hi) {
      uint32_t mid = (lo + hi) >> 1, k = node_key(R[mid]);
      if (k == key) return mid;
      if (k < key) lo = mid + 1; else hi = mid;
    }
    return NONE;
  }
  void go(uint32_t m, uint32_t t, uint32_t row) {
    const Ruleset::TrieNode& T = rs.trie[t];
    const Node mn = R[m];
    if (node_type(mn) == N_MAP) {
      const auto& K = kids[t];
      auto hit = [&](uint32_t x, uint32_t kid) {
        if (colv) colv[(size_t)col_off[rs.trie[kid].col] + row] = entry(x);
        go(x, kid, row);
      };
      if (mn.b <= 2 * K.size() + 4) {  // merge join of two key-sorted lists
        uint32_t a = mn.a, e = mn.a + mn.b;
        size_t j = 0;
        while (a < e && j < K.size()) {
          uint32_t k = node_key(R[a]);
          if (k < K[j].first) a++;
          else if (k > K[j].first) j++;
          else { hit(a, K[j].second); a++; j++; }
        }
      } else {
        for (auto& kv : K) {
          uint32_t x = find(R, mn, kv.first);
          if (x != NONE) hit(x, kv.second);  // columns are NONE-initialised
        }
      }
    } else if (node_type(mn) == N_ARR && T.star != NONE) {
      uint32_t space = rs.trie[T.star].rowspace;
      uint32_t base = next[space];
      next[space] += mn.b;
      if (colv) {
        R[m].c = base;
        colv[(size_t)col_off[T.lencol] + row] = (uint64_t)mn.b | ((uint64_t)base << 32);
        const size_t self = col_off[rs.trie[T.star].col];
        for (uint32_t i = 0; i < mn.b; i++) colv[self + base + i] = entry(mn.a + i);
      }
      for (uint32_t i = 0; i < mn.b; i++) go(mn.a + i, T.star, base + i);
    }
  }
};
}  // namespace

void resolve_path_columns(Batch& b, int threads) {
  const Ruleset& rs = *b.rs;
  size_t n = b.hdr.size();
  uint32_t nsp = rs.nrowspaces;
  b.rs_rows.assign(nsp, 0);
  b.col_off.assign(rs.ncols, 0);
  b.colv.clear();
  if (rs.ncols == 0 || n == 0) return;
  int T = std::max(1, threads);
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> kids(rs.trie.size());
  for (size_t t = 0; t < rs.trie.size(); t++) {
    kids[t] = rs.trie[t].kids;
    std::sort(kids[t].begin(), kids[t].end());
  }
  size_t nch = std::min(n, (size_t)T * 8);
  std::vector<std::vector<uint32_t>> cnt(nch, std::vector<uint32_t>(nsp, 0));
  auto eligible = [&](const ResHeader& h) { return h.nnodes < (1u << COL_TYPE_SHIFT); };
  auto run = [&](bool fill, std::vector<std::vector<uint32_t>>& nexts) {
    std::atomic<size_t> nx{0};
    auto work = [&]() {
      for (;;) {
        size_t c = nx.fetch_add(1);
        if (c >= nch) break;
        size_t r0 = n * c / nch, r1 = n * (c + 1) / nch;
        for (size_t r = r0; r < r1; r++) {
          ResHeader& h = b.hdr[r];
          if (!eligible(h)) continue;
          Resolver rv{rs, kids, b.nodes.data() + h.root, fill ? b.colv.data() : nullptr, b.col_off.data(), nexts[c].data()};
          rv.go(0, 0, (uint32_t)r);
        }
      }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) th.emplace_back(work);
    for (auto& t : th) t.join();
  };
  run(false, cnt);
  std::vector<std::vector<uint32_t>> base(nch, std::vector<uint32_t>(nsp, 0));
  std::vector<uint64_t> tot(nsp, 0);
  for (size_t c = 0; c < nch; c++)
    for (uint32_t s = 1; s < nsp; s++) {
      if (tot[s] + cnt[c][s] > 0xFFFFFFF0ull) throw std::runtime_error("path-column row space exceeds 2^32 rows; split the batch");
      base[c][s] = (uint32_t)tot[s];
      tot[s] += cnt[c][s];
    }
  b.rs_rows[0] = (uint32_t)n;
  for (uint32_t s = 1; s < nsp; s++) b.rs_rows[s] = (uint32_t)tot[s];
  uint64_t total = 0;
  for (uint32_t c = 0; c < rs.ncols; c++) {
    b.col_off[c] = (uint32_t)total;
    total += b.rs_rows[rs.col_rowspace[c]];
    if (total > 0xFFFFFFF0ull) throw std::runtime_error("path columns exceed 2^32 entries; split the batch");
  }
  b.colv.resize(total + 1);  // NONE-initialised in parallel, one slice per worker
  {
    const size_t per = (1u << 20);
    parallel_for((total + per) / per, T, [&](size_t k) {
      size_t lo = k * per, hi = std::min<size_t>(total + 1, lo + per);
      std::fill(b.colv.begin() + lo, b.colv.begin() + hi, (uint64_t)NONE);
    });
  }
  if (getenv("KYV_DEBUG_STATS")) {
    fprintf(stderr, "[kyvgpu] path columns: %u columns, %u row spaces, %llu entries (rows:", rs.ncols, nsp,
            (unsigned long long)total);
    for (uint32_t sp = 0; sp < nsp; sp++) fprintf(stderr, " %u", b.rs_rows[sp]);
    fprintf(stderr, ")\n");
  }
  run(true, base);
  // resources too large for column encoding: pattern pairs fall back (RF_MAGIC), so no column is read
  for (auto& h : b.hdr) if (!eligible(h)) h.flags |= RF_MAGIC;
}

std::string format_path(const Ruleset& rs, const Batch& b, uint32_t tmpl, const uint16_t* idx, const uint32_t* key) {
  if (tmpl == NONE) return "";
  const std::string& t = rs.templates[tmpl];
  std::string out;
  for (size_t i = 0; i < t.size(); i++) {
    if (t[i] == '\x01' && i + 1 < t.size()) { out += std::to_string(idx[t[i + 1] - '0']); i++; continue; }
    if (t[i] == '\x02' && i + 1 < t.size()) {
      uint32_t k = key[t[i + 1] - '0'];
      out += k < b.dict.strs.size() ? b.dict.strs[k] : std::string("?");
      i++;
      continue;
    }
    out += t[i];
  }
  return out;
}

}  // namespace kyv
