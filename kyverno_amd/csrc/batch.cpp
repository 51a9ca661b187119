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
#include <thread>

#include "kyv_host.h"

namespace kyv {
using pj::T;
using pj::Value;

Batch::~Batch() {}

namespace {

bool magic(const std::string& s) {
  return s.find("negation anchor matched in resource") != std::string::npos ||
         s.find("conditional anchor mismatch") != std::string::npos || s.find("global anchor mismatch") != std::string::npos;
}

bool is_anchor_key(const std::string& raw, const char* tag) {  // key that anchor.Parse() maps onto tag
  std::string s = pj::go_trim_space(raw);
  if (s.size() < 3 || s.back() != ')') return false;
  size_t p = (s[0] == '+' || s[0] == '<' || s[0] == '=' || s[0] == 'X' || s[0] == '^') ? 1 : 0;
  if (s[p] != '(') return false;
  return s.substr(p + 1, s.size() - p - 2) == tag;
}

// chunk-local interning, remapped to global ids after the parallel phase
struct Chunk {
  std::vector<std::string> strs;
  std::unordered_map<std::string, uint32_t> ids;
  std::vector<Node> nodes;
  std::vector<ResHeader> hdr;
  std::vector<FloatAux> faux;
  std::vector<uint32_t> ns_names;  // local sid of namespace per resource
  std::string err;
  uint32_t local(const std::string& s) {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    uint32_t id = (uint32_t)strs.size();
    strs.push_back(s);
    ids.emplace(s, id);
    return id;
  }
};

struct Emitter {
  Chunk& ch;
  std::vector<Node> out;
  bool magicflag = false;
  uint32_t put_children_map(const Value& v) {
    uint32_t first = (uint32_t)out.size();
    out.resize(first + v.o.size());
    for (size_t k = 0; k < v.o.size(); k++) {
      if (magic(v.o[k].first)) magicflag = true;
      fill(first + (uint32_t)k, v.o[k].second, (ch.local(v.o[k].first) << 4));
    }
    return first;
  }
  void fill(uint32_t idx, const Value& v, uint32_t keybits) {
    Node n{};
    switch (v.t) {
      case T::Null: n.tk = N_NULL; break;
      case T::Bool: n.tk = v.b ? N_TRUE : N_FALSE; n.a = v.b; break;
      case T::Int: {
        n.tk = N_INT;
        uint64_t u = (uint64_t)v.i;
        n.a = (uint32_t)u;
        n.b = (uint32_t)(u >> 32);
        n.c = ch.local(std::to_string(v.i));
        break;
      }
      case T::Float: {
        n.tk = N_FLOAT;
        uint64_t u = __builtin_bit_cast(uint64_t, v.f);
        n.a = (uint32_t)u;
        n.b = (uint32_t)(u >> 32);
        n.c = (uint32_t)ch.faux.size();
        ch.faux.push_back(FloatAux{ch.local(pj::go_fmt_E(v.f)), ch.local(pj::go_fmt_f6(v.f))});
        break;
      }
      case T::Str:
        n.tk = N_STR;
        n.a = ch.local(v.s);
        if (magic(v.s)) magicflag = true;
        break;
      case T::Obj: {
        n.tk = N_MAP;
        n.b = (uint32_t)v.o.size();
        if (v.o.size() > 0xFFFF) magicflag = true;  // walk frames count entries in 16 bits
        out[idx] = n;  // reserve before recursion (out may grow)
        uint32_t first = put_children_map(v);
        out[idx].a = first;
        out[idx].tk |= keybits;
        return;
      }
      case T::Arr: {
        n.tk = N_ARR;
        n.b = (uint32_t)v.a.size();
        n.c = NONE;  // path-column row of element 0, set by resolve_path_columns
        if (v.a.size() > 0xFFFF) magicflag = true;  // walk frames count elements in 16 bits
        out[idx] = n;
        uint32_t first = (uint32_t)out.size();
        out.resize(first + v.a.size());
        for (size_t k = 0; k < v.a.size(); k++) fill(first + (uint32_t)k, v.a[k], (uint32_t)k << 4);
        out[idx].a = first;
        out[idx].tk |= keybits;
        return;
      }
    }
    n.tk |= keybits;
    out[idx] = n;
  }
};

const Value* nested(const Value& o, std::initializer_list<const char*> path) {
  const Value* cur = &o;
  for (const char* f : path) {
    if (cur->t != T::Obj) return nullptr;
    cur = cur->get(f);
    if (!cur) return nullptr;
  }
  return cur;
}
std::string nested_str(const Value& o, std::initializer_list<const char*> path) {
  const Value* v = nested(o, path);
  return v && v->t == T::Str ? v->s : "";
}

// relative node index of a string map at metadata.<key> (NestedStringMap), NONE otherwise
uint32_t string_map_node(const std::vector<Node>& R, uint32_t meta, uint32_t keysid_local, const Value* v) {
  if (!v || v->t != T::Obj) return NONE;
  for (auto& kv : v->o) if (kv.second.t != T::Str) return NONE;
  const Node& m = R[meta];
  for (uint32_t i = 0; i < m.b; i++)
    if (node_key(R[m.a + i]) == keysid_local) return m.a + i;
  return NONE;
}

void flatten_one(Chunk& ch, const Value& doc) {
  Emitter em{ch};
  em.out.resize(1);
  em.fill(0, doc, 0);
  ResHeader h{};
  h.root = (uint32_t)ch.nodes.size();
  h.nnodes = (uint32_t)em.out.size();
  std::string kind = nested_str(doc, {"kind"});
  h.kind = ch.local(kind);
  std::string av = nested_str(doc, {"apiVersion"});
  size_t sl = std::count(av.begin(), av.end(), '/');
  std::string g, ver;
  bool gvok = true;
  if (av.empty() || av == "/") {}
  else if (sl == 0) ver = av;
  else if (sl == 1) { g = av.substr(0, av.find('/')); ver = av.substr(av.find('/') + 1); }
  else gvok = false;
  h.gvk_kind = ch.local(gvok ? kind : "");
  h.group = ch.local(g);
  h.version = ch.local(ver);
  h.gv = ch.local(g.empty() ? ver : g + "/" + ver);
  h.name = ch.local(nested_str(doc, {"metadata", "name"}));
  h.gen_name = ch.local(nested_str(doc, {"metadata", "generateName"}));
  std::string ns = nested_str(doc, {"metadata", "namespace"});
  h.ns = ch.local(ns);
  h.labels = h.ann = NONE;
  h.nsl = NONE;
  h.flags = em.magicflag ? RF_MAGIC : 0;
  if (doc.t == T::Obj) h.flags |= RF_ROOT_MAP;
  const Value* meta = nested(doc, {"metadata"});
  if (meta && meta->t == T::Obj) {
    uint32_t mnode = NONE;
    const Node& root = em.out[0];
    uint32_t msid = ch.local("metadata");
    for (uint32_t i = 0; i < root.b; i++) if (node_key(em.out[root.a + i]) == msid) mnode = root.a + i;
    if (mnode != NONE) {
      h.labels = string_map_node(em.out, mnode, ch.local("labels"), meta->get("labels"));
      h.ann = string_map_node(em.out, mnode, ch.local("annotations"), meta->get("annotations"));
    }
  }
  // any map key directly under a "metadata" map that anchor.Parse() resolves to labels/annotations
  std::vector<const Value*> stack{&doc};
  while (!stack.empty()) {
    const Value* v = stack.back();
    stack.pop_back();
    if (v->t == T::Obj) {
      for (auto& kv : v->o) {
        if (kv.first == "metadata" && kv.second.t == T::Obj)
          for (auto& m2 : kv.second.o)
            if (is_anchor_key(m2.first, "labels") || is_anchor_key(m2.first, "annotations")) h.flags |= RF_ANCHORISH;
        stack.push_back(&kv.second);
      }
    } else if (v->t == T::Arr) {
      for (auto& e : v->a) stack.push_back(&e);
    }
  }
  ch.hdr.push_back(h);
  ch.ns_names.push_back(h.ns);
  ch.nodes.insert(ch.nodes.end(), em.out.begin(), em.out.end());
}

// split a JSON array / NDJSON buffer into document byte ranges
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
    out.push_back({st, i - st});
  }
  return out;
}

}  // namespace

void derive_strings(Batch& b, size_t from, int threads) {
  size_t n = b.dict.strs.size();
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
        int64_t d;
        if (pj::go_parse_duration(x, &d)) { f |= SF_DUR; b.str_dur[s] = d; } else b.str_dur[s] = 0;
        int64_t lo, hi;
        int q = pj::go_parse_quantity(x, &lo, &hi);
        if (q == 1) { f |= SF_QTY; b.str_qty[2 * s] = lo; b.str_qty[2 * s + 1] = hi; }
        else { b.str_qty[2 * s] = 0; b.str_qty[2 * s + 1] = 0; if (q == 2) f |= SF_QTY_BIG; }
        double fv;
        if (pj::go_parse_float(x, &fv)) { f |= SF_FLOAT; b.str_f64[s] = fv; } else b.str_f64[s] = 0;
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
struct KindGate {
  bool any = false;
  std::vector<uint32_t> kinds;
};

static KindGate rule_gate(const Ruleset& rs, const RuleDesc& rd) {
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
  std::vector<ResHeader> sorted(n);
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
  try {
    b->rs = rs;
    b->dict = rs->dict;
    auto docs = split_docs(json, len);
    // threads scaled to the work: thread start-up is tens of microseconds, which dominates small (admission)
    // batches when every phase spawns the machine's thread count
    int T = std::max(1, std::min(threads, (int)(docs.size() / 256) + 1));
    size_t nchunks = std::min(docs.size(), (size_t)T * 8);
    if (nchunks == 0) nchunks = 1;
    std::vector<Chunk> chunks(nchunks);
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (;;) {
        size_t c = next.fetch_add(1);
        if (c >= nchunks) break;
        size_t d0 = docs.size() * c / nchunks, d1 = docs.size() * (c + 1) / nchunks;
        try {
          for (size_t d = d0; d < d1; d++) {
            Value doc = pj::parse(json + docs[d].first, docs[d].second, false);
            flatten_one(chunks[c], doc);
          }
        } catch (std::exception& e) {
          chunks[c].err = e.what();
        }
      }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) th.emplace_back(work);
    for (auto& t : th) t.join();
    for (auto& c : chunks) if (!c.err.empty()) throw std::runtime_error(c.err);
    size_t seed = b->dict.strs.size();
    // merge dictionaries
    std::vector<std::vector<uint32_t>> remap(nchunks);
    for (size_t c = 0; c < nchunks; c++) {
      remap[c].resize(chunks[c].strs.size());
      for (size_t s = 0; s < chunks[c].strs.size(); s++) remap[c][s] = b->dict.intern(chunks[c].strs[s]);
    }
    // namespace label sets
    std::unordered_map<uint32_t, uint32_t> ns_set;
    if (nsl_json && nsl_len) {
      Value nsl = pj::parse(nsl_json, nsl_len, false);
      b->nsl_off.push_back(0);
      if (nsl.t == T::Obj)
        for (auto& kv : nsl.o) {
          ns_set[b->dict.intern(kv.first)] = (uint32_t)b->nsl_names.size();
          b->nsl_names.push_back(kv.first);
          if (kv.second.t == T::Obj)
            for (auto& lv : kv.second.o) {
              b->nsl_kv.push_back(b->dict.intern(lv.first));
              b->nsl_kv.push_back(b->dict.intern(lv.second.t == T::Str ? lv.second.s : ""));
            }
          b->nsl_off.push_back((uint32_t)b->nsl_kv.size() / 2);
        }
    } else {
      b->nsl_off.push_back(0);
    }
    // concatenate + remap + sort map entries
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
    next = 0;
    auto fix = [&]() {
      for (;;) {
        size_t c = next.fetch_add(1);
        if (c >= nchunks) break;
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
            // key bits hold a local sid for map entries: detect by parent type below; remap all key fields of
            // map children after copying
            if (t == N_STR) n.a = rm[n.a];
            else if (t == N_INT) n.c = rm[n.c];
            else if (t == N_FLOAT) n.c += (uint32_t)faux_base[c];
            R[i] = n;
          }
          for (uint32_t i = 0; i < h.nnodes; i++) {
            if (node_type(R[i]) != N_MAP) continue;
            Node* ch0 = R + R[i].a;
            for (uint32_t k = 0; k < R[i].b; k++) ch0[k].tk = (rm[ch0[k].tk >> 4] << 4) | (ch0[k].tk & 0xF);
            std::sort(ch0, ch0 + R[i].b, [](const Node& x, const Node& y) { return (x.tk >> 4) < (y.tk >> 4); });
          }
          h.root = (uint32_t)(node_base[c] + h.root);
          h.kind = rm[h.kind]; h.gvk_kind = rm[h.gvk_kind]; h.group = rm[h.group]; h.version = rm[h.version];
          h.gv = rm[h.gv]; h.name = rm[h.name]; h.gen_name = rm[h.gen_name]; h.ns = rm[h.ns];
          auto it = ns_set.find(h.ns);
          h.nsl = it == ns_set.end() ? NONE : it->second;
          b->hdr[res_base[c] + r] = h;
        }
      }
    };
    th.clear();
    for (int t = 0; t < T; t++) th.emplace_back(fix);
    for (auto& t : th) t.join();
    // labels/annotations node indices moved when map entries were sorted: recompute from the sorted tables
    for (auto& h : b->hdr) {
      if (h.labels == NONE && h.ann == NONE) continue;
      const Node* R = b->nodes.data() + h.root;
      uint32_t meta = (node_type(R[0]) == N_MAP) ? [&]() {
        for (uint32_t i = 0; i < R[0].b; i++) if (node_key(R[R[0].a + i]) == KSID(METADATA)) return R[0].a + i;
        return NONE;
      }() : NONE;
      auto find = [&](uint32_t key) -> uint32_t {
        if (meta == NONE || node_type(R[meta]) != N_MAP) return NONE;
        for (uint32_t i = 0; i < R[meta].b; i++) if (node_key(R[R[meta].a + i]) == key) return R[meta].a + i;
        return NONE;
      };
      if (h.labels != NONE) h.labels = find(KSID(LABELS));
      if (h.ann != NONE) h.ann = find(KSID(ANNOTATIONS));
    }
    derive_strings(*b, 0, std::max(1, std::min(T, (int)(b->dict.strs.size() / 8192) + 1)));
    order_by_kind(*b);
    resolve_path_columns(*b, T);
    (void)seed;
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
      for (auto& kv : T.kids) {
        uint32_t x = find(R, mn, kv.first);
        if (x == NONE) continue;  // columns are NONE-initialised
        if (colv) colv[(size_t)col_off[rs.trie[kv.second].col] + row] = entry(x);
        go(x, kv.second, row);
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
          Resolver rv{rs, b.nodes.data() + h.root, fill ? b.colv.data() : nullptr, b.col_off.data(), nexts[c].data()};
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
  b.colv.assign(total + 1, (uint64_t)NONE);
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
