// Conditions of validate.deny and rule preconditions for one (resource, rule) pair, __host__ __device__.
//
// Reference (paths relative to /root/reference):
//   pkg/engine/variables/evaluate.go:11-83           Evaluate, any/all blocks, old-style list
//   pkg/engine/variables/operator/*.go               operator handlers (equal, notequal, in, notin, anyin, allin,
//                                                    anynotin, allnotin, numeric)
//   pkg/engine/variables/vars.go:352-431             `{{ request.object... }}` substitution; a key missing from a map
//                                                    is a NotFoundError from the kyverno/go-jmespath fork
//   api/kyverno/v1/common_types.go:185-199           Condition.GetKey/GetValue: the substituted document goes
//                                                    through json.Marshal + apimachinery util/json (integral -> int64)
//
// Values are typed as the operator handlers see them (after that round trip). Where the device cannot
// reproduce the reference bit for bit (fmt.Sprint of a float that is not in the dictionary, a resource-side
// string the handler would JSON-decode, semver operands, quantities beyond int128 nano units, composite
// elements) the pair returns ST_FALLBACK and the CPU engine decides it.
#pragma once
#include "kyv_eval.h"

namespace kyv {

enum CondRes : uint8_t { CR_FALSE = 0, CR_TRUE = 1, CR_FB = 2, CR_PANIC = 3 };
enum CType : uint8_t { CT_NIL = 0, CT_BOOL = 1, CT_INT = 2, CT_FLOAT = 3, CT_STR = 4, CT_ARR = 5, CT_MAP = 6 };

struct CV {
  uint8_t t;       // CType
  uint8_t res;     // 1: resource node table, 0: ruleset literal (cnodes)
  uint8_t b;       // CT_BOOL
  uint8_t pad;     // CT_ARR with vl: log2 of the element stride in vl (0 packed JList; 6 the compiled kernels'
                   // lane-interleaved LDS lists)
  uint32_t sid;    // CT_STR: the string; else fmt.Sprint form (NONE when not in the dictionary)
  uint32_t node;   // CT_ARR / CT_MAP: node index (relative to the resource root / absolute in cnodes)
  uint32_t n;      // CT_ARR: element count
  int64_t i;
  double f;
  const uint32_t* vl;  // CT_ARR produced by a JMESPath projection: element nodes (JMES_KEYBIT: a map key; NONE: null)
};

constexpr double TWO63 = 9223372036854775808.0;

KYV_HD int64_t go_f2i(double f) {  // int64(float64) as amd64 does it (out of range -> min int64)
  if (!(f >= -TWO63 && f < TWO63)) return INT64_MIN;
  return (int64_t)f;
}

KYV_HD CV cv_node(const Node& n, bool res) {
  CV x;
  x.t = CT_NIL; x.res = res ? 1 : 0; x.b = 0; x.pad = 0; x.sid = KSID(NIL_STR); x.node = NONE; x.n = 0; x.i = 0; x.f = 0;
  x.vl = nullptr;
  switch (node_type(n)) {
    case N_NULL: break;
    case N_FALSE: x.t = CT_BOOL; x.sid = SID_FALSE; break;
    case N_TRUE: x.t = CT_BOOL; x.b = 1; x.sid = SID_TRUE; break;
    case N_INT: {
      int64_t i = (int64_t)(((uint64_t)n.b << 32) | n.a);
      x.t = CT_INT; x.i = i; x.sid = n.c;
      if (res) {  // JSON context decode (float64) then the util/json round trip
        double d = (double)i;
        if (d >= TWO63) { x.t = CT_FLOAT; x.f = d; x.sid = NONE; }
        else { x.i = (int64_t)d; if (x.i != i) x.sid = NONE; }
      }
      break;
    }
    case N_FLOAT: {
      double f = __builtin_bit_cast(double, ((uint64_t)n.b << 32) | n.a);
      x.t = CT_FLOAT; x.f = f; x.sid = res ? NONE : n.c;
      if (res && f == __builtin_trunc(f) && f > -1e21 && f < 1e21 && f >= -TWO63 && f < TWO63) {
        x.t = CT_INT; x.i = (int64_t)f;  // integral: json "%f"-style digits decode as int64
      }
      break;
    }
    case N_STR: x.t = CT_STR; x.sid = n.a; break;
    case N_ARR: x.t = CT_ARR; x.node = NONE; x.n = n.b; x.sid = NONE; break;
    case N_MAP: x.t = CT_MAP; x.sid = NONE; break;
    default: break;
  }
  return x;
}

// element j of an array operand
KYV_HD CV cv_elem(const View& v, NodeTab R, const CV& arr, uint32_t j) {
  if (arr.vl) {
    const uint32_t e = arr.vl[(size_t)j << arr.pad];
    if (e == NONE) return cv_node(Node{N_NULL, 0, 0, 0}, true);
    if ((e & (JMES_KEYBIT | JMES_SIDBIT)) == JMES_SIDBIT) {
      CV x = cv_node(Node{N_NULL, 0, 0, 0}, true);
      x.t = CT_STR;
      x.sid = e & ~JMES_SIDBIT;
      return x;
    }
    if (e & JMES_KEYBIT) {
      CV x = cv_node(Node{N_NULL, 0, 0, 0}, true);
      x.t = CT_STR;
      x.sid = node_key(R[e & ~JMES_KEYBIT]);
      return x;
    }
    return cv_node(R[e], true);
  }
  if (arr.res) {
    const Node& a = R[arr.node];
    return cv_node(R[a.a + j], true);
  }
  const Node& a = v.cnodes[arr.node];
  return cv_node(v.cnodes[a.a + j], false);
}

// operand value; returns false on a NotFoundError (*miss = failing segment). `row`: the resource's position in the
// batch; a path whose column resolved (every parent a map holding the next key) is one load, anything else takes
// the key-by-key search (which tells a missing key -- NotFoundError -- from a null or non-map parent)
KYV_HD bool cv_operand(const View& v, NodeTab R, const CondOperand& o, CV* out, uint32_t* miss, uint32_t row = NONE) {
  if (o.kind == OK_LIT) {
    *out = cv_node(v.cnodes[o.a], false);
    if (out->t == CT_ARR) out->node = o.a;
    return true;
  }
  Node nil{N_NULL, 0, 0, 0};
  if (o.kind != OK_PATH) { *out = cv_node(nil, false); return true; }
  if (o.list && row != NONE && v.colv) {
    KYV_ACCT_ADD(0, 8);
    const uint32_t e = (uint32_t)v.colv[(size_t)v.col_off[o.list - 1] + row];
    if (e != NONE) {
      const uint32_t x = e & COL_INDEX_MASK;
      *out = cv_node(R[x], true);
      if (out->t == CT_ARR) out->node = x;
      return true;
    }
  }
  uint32_t cur = 0;  // request.object = the resource root
  for (uint32_t s = 0; s < o.nseg; s++) {
    const Node& n = R[cur];
    if (node_type(n) != N_MAP) { *out = cv_node(nil, true); return true; }  // field of a non-map: null
    uint32_t nx = map_find(R, cur, v.pool[o.a + s]);
    if (nx == NONE) { *miss = s; return false; }
    cur = nx;
  }
  *out = cv_node(R[cur], true);
  if (out->t == CT_ARR) out->node = cur;
  return true;
}


KYV_HD uint32_t sflags(const View& v, uint32_t sid) { return v.str_flags[sid]; }

// ---------------------------------------------------------------- JMESPath subset (OK_JMES, kyv_layout.h)
// go-jmespath interpreter semantics on the resource's node table: field of a non-map -> null; a key missing from
// a map -> null (NotFoundError only for JF_PURE chains); flatten splices arrays and a projection drops null
// results; keys(@) of a non-map is an error the device leaves to the CPU engine; `|| lit` replaces a false-like
// result (null, false, "", empty list / map).
struct JList { uint32_t n; uint32_t e[JMES_MAX_LIST]; };
struct JRes {
  bool lst;        // result is the projection list L
  uint32_t cur;    // single result: node (JMES_KEYBIT: a map key), NONE = null
  uint32_t lit;    // cnode literal result (|| default, request.operation), NONE otherwise
  uint32_t num;    // length() result (a number), NONE otherwise
};
// JS_ERR: a run-time JMESPath error other than NotFound (length() of a null / number / boolean): the substitution
// fails, so the condition program is an error (vars.go:352-431)
// JS_TERR: a function argument type error (keys() of a non-object inside a filter): a foreach list query that errors
// skips its entry (validation.go:322-326); in a condition operand the CPU engine words the error
enum JStat { JS_OK = 0, JS_NOTFOUND = 1, JS_FB = 2, JS_ERR = 3, JS_TERR = 4 };

KYV_HD bool j_false(const View& v, NodeTab R, const JRes& r, const JList& L) {  // util.go isFalse
  if (r.lst) return L.n == 0;
  if (r.lit != NONE) {
    const Node& c = v.cnodes[r.lit];
    switch (node_type(c)) {
      case N_NULL: case N_FALSE: return true;
      case N_STR: return c.a == SID_EMPTY;
      case N_ARR: case N_MAP: return c.b == 0;
      default: return false;
    }
  }
  if (r.cur == NONE) return true;
  if (r.cur & JMES_KEYBIT) return node_key(R[r.cur & ~JMES_KEYBIT]) == SID_EMPTY;
  const Node& n = R[r.cur];
  switch (node_type(n)) {
    case N_NULL: case N_FALSE: return true;
    case N_STR: return n.a == SID_EMPTY;
    case N_ARR: case N_MAP: return n.b == 0;
    default: return false;
  }
}
KYV_HD bool j_map(NodeTab R, uint32_t n) { return n != NONE && !(n & JMES_KEYBIT) && node_type(R[n]) == N_MAP; }
KYV_HD bool j_arr(NodeTab R, uint32_t n) { return n != NONE && !(n & JMES_KEYBIT) && node_type(R[n]) == N_ARR; }
KYV_HD uint32_t j_field(NodeTab R, uint32_t m, uint32_t key, bool* missing) {
  *missing = false;
  if (!j_map(R, m)) return NONE;
  uint32_t x = map_find(R, m, key);
  if (x == NONE) { *missing = true; return NONE; }
  return node_type(R[x]) == N_NULL ? NONE : x;
}

// run an OK_JMES program; `elem` = the foreach element (node / JMES_KEYBIT key) or NONE.
// A flatten starts a projection: its right-hand ops run on every element (null ones included: keys(@) of a null
// element is an error), and the projection's null results are dropped when it ends (next [], ||, or the end).
KYV_HD void j_drop_nulls(JList& L) {
  uint32_t w = 0;
  for (uint32_t j = 0; j < L.n; j++) if (L.e[j] != NONE) L.e[w++] = L.e[j];
  L.n = w;
}
__host__ __device__ inline __attribute__((noinline)) int jmes_run(const View& v, NodeTab R, const CondOperand& o, uint32_t elem, JList& L, JRes* out, uint32_t* miss) {
  const uint32_t* p = v.pool + o.a;
  const uint32_t n = o.nseg, root = p[0] & 0xFFu;
  const bool pure = (p[0] & JF_PURE) != 0;
  JRes r;
  r.lst = false; r.cur = NONE; r.lit = NONE; r.num = NONE;
  L.n = 0;
  bool proj = false;
  uint32_t i = 1, fields = 0;
  if (root == JR_OBJECT) r.cur = 0;
  else if (root == JR_ELEMENT) r.cur = elem;
  else { r.lit = p[1]; i = 2; }
  while (i < n) {
    const uint32_t op = p[i];
    if (op == JO_FIELD) {
      const uint32_t key = p[i + 1];
      i += 2;
      bool missing;
      if (!r.lst) {
        r.cur = j_field(R, r.cur, key, &missing);
        if (missing && pure) { *miss = fields; return JS_NOTFOUND; }
      } else {
        for (uint32_t j = 0; j < L.n; j++) L.e[j] = j_field(R, L.e[j], key, &missing);
      }
      fields++;
    } else if (op == JO_MULTI) {
      const uint32_t m = p[i + 1];
      if (r.cur != NONE) {  // multi-select on null is null
        if (m > JMES_MAX_LIST) return JS_FB;
        bool missing;
        for (uint32_t j = 0; j < m; j++) L.e[j] = j_field(R, r.cur, p[i + 2 + j], &missing);
        L.n = m;
        r.lst = true;
      }
      i += 2 + m;
    } else if (op == JO_FLAT) {
      i++;
      if (!r.lst) {
        if (!j_arr(R, r.cur)) { r.cur = NONE; proj = false; continue; }  // flatten of a non-list: null
        const Node& a = R[r.cur];
        if (a.b > JMES_MAX_LIST) return JS_FB;
        for (uint32_t j = 0; j < a.b; j++) L.e[j] = node_type(R[a.a + j]) == N_NULL ? NONE : a.a + j;
        L.n = a.b;
        r.lst = true;
      } else {
        if (proj) j_drop_nulls(L);
        uint32_t t[JMES_MAX_LIST];
        const uint32_t tn = L.n;
        for (uint32_t j = 0; j < tn; j++) t[j] = L.e[j];
        uint32_t w = 0;
        for (uint32_t j = 0; j < tn; j++) {
          const uint32_t x = t[j];
          if (j_arr(R, x)) {
            const Node& a = R[x];
            for (uint32_t q = 0; q < a.b; q++) {
              if (w >= JMES_MAX_LIST) return JS_FB;
              L.e[w++] = node_type(R[a.a + q]) == N_NULL ? NONE : a.a + q;
            }
          } else {
            if (w >= JMES_MAX_LIST) return JS_FB;
            L.e[w++] = x;
          }
        }
        L.n = w;
      }
      proj = true;
    } else if (op == JO_KEYS) {
      i++;
      if (r.lst || !j_map(R, r.cur)) return JS_FB;  // keys() of a non-object: the reference errors
      const Node& m = R[r.cur];
      if (m.b > JMES_MAX_LIST) return JS_FB;
      for (uint32_t j = 0; j < m.b; j++) L.e[j] = (m.a + j) | JMES_KEYBIT;
      L.n = m.b;
      r.lst = true;
    } else if (op == JO_KEYS_FLAT) {
      i++;
      if (!r.lst) continue;  // the projection's left side was null: so is the result
      uint32_t t[JMES_MAX_LIST];
      const uint32_t tn = L.n;
      for (uint32_t j = 0; j < tn; j++) t[j] = L.e[j];
      uint32_t w = 0;
      for (uint32_t j = 0; j < tn; j++) {
        if (!j_map(R, t[j])) return JS_FB;  // keys() of null / a non-object element: the reference errors
        const Node& m = R[t[j]];
        for (uint32_t q = 0; q < m.b; q++) {
          if (w >= JMES_MAX_LIST) return JS_FB;
          L.e[w++] = (m.a + q) | JMES_KEYBIT;
        }
      }
      L.n = w;
      proj = true;
    } else if (op == JO_LENGTH) {
      // jpfLength (go-jmespath functions.go): rune count of a string, element count of an array / object; other
      // types fail the argument type check
      i++;
      if (proj) { j_drop_nulls(L); proj = false; }
      uint32_t cnt;
      if (r.lst) {
        cnt = L.n;
      } else {
        uint32_t sid = NONE;
        if (r.cur == NONE) return JS_ERR;
        if (r.cur & JMES_KEYBIT) sid = node_key(R[r.cur & ~JMES_KEYBIT]);
        else {
          const Node& x = R[r.cur];
          if (node_type(x) == N_ARR || node_type(x) == N_MAP) cnt = x.b;
          else if (node_type(x) == N_STR) sid = x.a;
          else return JS_ERR;
        }
        if (sid != NONE) {  // ASCII: bytes == runes; other strings go to the CPU engine
          const uint32_t ln = v.str_len[sid];
          const uint8_t* b = sbytes(v, sid);
          for (uint32_t q = 0; q < ln; q++) if (b[q] >= 0x80) return JS_FB;
          cnt = ln;
        }
      }
      r.lst = false; r.cur = NONE; r.num = cnt;
    } else if (op == JO_FILTER) {
      // filter projection (go-jmespath ASTFilterProjection): the elements of a list whose predicate is not false-like;
      // a non-list is null. The ops after it run per kept element (a projection: null results dropped at its end)
      const uint32_t fk = p[i + 1], lit = p[i + 2], nf = p[i + 3];
      const uint32_t* fkeys = p + i + 4;
      i += 4 + nf;
      if (r.lst) return JS_FB;  // a filter inside a projection: not compiled (compiler.cpp jmes_var)
      if (!j_arr(R, r.cur)) { r.cur = NONE; proj = false; continue; }
      const Node& a = R[r.cur];
      uint32_t w = 0;
      for (uint32_t j = 0; j < a.b; j++) {
        const uint32_t e = a.a + j;
        bool keep;
        if (fk == FK_HASKEY) {  // contains(keys(@), 'lit'): keys() of a non-object fails the argument type check
          if (node_type(R[e]) != N_MAP) return JS_TERR;
          keep = map_find(R, e, lit) != NONE;
        } else {  // <fields> ==/!= literal (reflect.DeepEqual): string by id, boolean, null
          uint32_t x = node_type(R[e]) == N_NULL ? NONE : e;
          bool missing;
          for (uint32_t q = 0; q < nf && x != NONE; q++) x = j_field(R, x, fkeys[q], &missing);
          const Node& c = v.cnodes[lit];
          const uint32_t ct = node_type(c);
          bool eq;
          if (x == NONE) eq = ct == N_NULL;
          else {
            const Node& n = R[x];
            const uint32_t nt = node_type(n);
            if (nt == N_INT || nt == N_FLOAT || nt == N_ARR || nt == N_MAP) {
              if (ct == N_STR || ct == N_TRUE || ct == N_FALSE || ct == N_NULL) eq = false;
              else return JS_FB;
            } else {
              eq = nt == ct && (nt != N_STR || n.a == c.a);
            }
          }
          keep = fk == FK_EQ ? eq : !eq;
        }
        if (!keep) continue;
        if (w >= JMES_MAX_LIST) return JS_FB;
        L.e[w++] = node_type(R[e]) == N_NULL ? NONE : e;
      }
      L.n = w;
      r.lst = true;
      proj = true;
    } else if (op == JO_OR) {
      const uint32_t lit = p[i + 1];
      i += 2;
      if (proj) { j_drop_nulls(L); proj = false; }
      if (j_false(v, R, r, L)) { r.lst = false; r.cur = NONE; r.lit = lit; }
    } else {
      return JS_FB;
    }
  }
  if (proj) j_drop_nulls(L);
  *out = r;
  return JS_OK;
}

KYV_HD CV jres_cv(const View& v, NodeTab R, const JRes& r, const JList& L) {
  if (r.num != NONE) {  // float64 count; integral, so the JSON context round trip presents it as an int
    CV x = cv_node(Node{N_NULL, 0, 0, 0}, true);
    x.t = CT_INT; x.i = r.num; x.sid = NONE;
    return x;
  }
  if (r.lit != NONE) {
    CV x = cv_node(v.cnodes[r.lit], false);
    if (x.t == CT_ARR) x.node = r.lit;
    return x;
  }
  if (r.lst) {
    CV x = cv_node(Node{N_NULL, 0, 0, 0}, true);
    x.t = CT_ARR; x.sid = NONE; x.n = L.n; x.vl = L.e;
    return x;
  }
  if (r.cur == NONE) return cv_node(Node{N_NULL, 0, 0, 0}, true);
  if (r.cur & JMES_KEYBIT) {
    CV x = cv_node(Node{N_NULL, 0, 0, 0}, true);
    x.t = CT_STR;
    x.sid = node_key(R[r.cur & ~JMES_KEYBIT]);
    return x;
  }
  CV x = cv_node(R[r.cur], true);
  if (x.t == CT_ARR) x.node = r.cur;
  return x;
}

// A chain-form program (kyv_layout.h jmes_chain_form) -> CV: the field chain as j_field walks it (a missing key is
// NotFound only for a JF_PURE program), `|| literal` when the value is false-like (util.go isFalse), then the function:
//  - length(): jpfLength -- element count of an array / object, rune count of a string (ASCII here; other strings go to
//    the CPU engine), an error for anything else;
//  - to_upper(): jpfToUpper (functions.go:681-689) -- the argument must be a string (else the argument type error), the
//    result is the dictionary string strings.ToUpper(s) (Batch::str_upper; a non-ASCII string goes to the CPU engine);
//  - regex_match(re, x): jpRegexMatch (functions.go:786-799) -- x must be a string or a number (else the type error); a
//    string's result is its precomputed bit (Batch::str_rx, regex.cpp), a number (ifaceToString's float32 formatting)
//    or a string outside printable ASCII goes to the CPU engine
// row: the resource's batch position; with the field chain's path column (o.list = column + 1, compiler.cpp
// TrieBuilder::chain) an entry present there is the node the chain reaches -- one coalesced load instead of a map
// search per field (round 6: C5's regex_match / to_upper rules walked metadata.labels.<key> by binary searches, 8x the
// cost of a path-column rule per pair); an absent entry (missing or null on the way, a non-map parent) takes the walk
KYV_HD int jmes_chain_cv(const View& v, NodeTab R, const CondOperand& o, CV* out, uint32_t* miss, uint32_t row = NONE) {
  const uint32_t* p = v.pool + o.a;
  const uint32_t n = o.nseg;
  const bool pure = (p[0] & JF_PURE) != 0;
  uint32_t cur = 0, fields = 0, i = 1;
  if (o.list && row != NONE && v.colv) {
    KYV_ACCT_ADD(0, 8);
    const uint32_t e = (uint32_t)v.colv[(size_t)v.col_off[o.list - 1] + row];
    if (e != NONE) {
      cur = e & COL_INDEX_MASK;
      for (; i + 1 < n && p[i] == JO_FIELD; i += 2) fields++;
    }
  }
  for (; i + 1 < n && p[i] == JO_FIELD; i += 2) {
    bool missing;
    cur = j_field(R, cur, p[i + 1], &missing);
    if (missing && pure) { *miss = fields; return JS_NOTFOUND; }
    fields++;
  }
  uint32_t lit = NONE;
  if (i + 1 < n && p[i] == JO_OR) {
    JRes r;
    r.lst = false; r.cur = cur; r.lit = NONE; r.num = NONE;
    JList none;
    none.n = 0;
    if (j_false(v, R, r, none)) { lit = p[i + 1]; cur = NONE; }
    i += 2;
  }
  CV x = lit != NONE ? cv_node(v.cnodes[lit], false) : cur == NONE ? cv_node(Node{N_NULL, 0, 0, 0}, true) : cv_node(R[cur], true);
  if (x.t == CT_ARR) x.node = lit != NONE ? lit : cur;
  if (i < n) {
    const uint32_t op = p[i];
    if (op == JO_LENGTH) {
      if (lit != NONE || cur == NONE) return JS_ERR;
      const Node& y = R[cur];
      uint32_t cnt;
      if (node_type(y) == N_ARR || node_type(y) == N_MAP) {
        cnt = y.b;
      } else if (node_type(y) == N_STR) {
        const uint32_t ln = v.str_len[y.a];
        const uint8_t* b = sbytes(v, y.a);
        for (uint32_t q = 0; q < ln; q++) if (b[q] >= 0x80) return JS_FB;  // (other strings: the CPU engine)
        cnt = ln;
      } else {
        return JS_ERR;
      }
      CV c = cv_node(Node{N_NULL, 0, 0, 0}, true);
      c.t = CT_INT; c.i = cnt; c.sid = NONE;  // a float64 count, integral: an int after the JSON context round trip
      x = c;
    } else if (op == JO_UPPER) {
      if (x.t != CT_STR) return JS_ERR;
      const uint32_t u = v.str_upper ? v.str_upper[x.sid] : NONE;
      if (u == NONE) return JS_FB;
      CV c = cv_node(Node{N_NULL, 0, 0, 0}, true);
      c.t = CT_STR; c.sid = u;
      x = c;
    } else if (op == JO_REGEX) {
      if (x.t == CT_INT || x.t == CT_FLOAT) return JS_FB;
      if (x.t != CT_STR) return JS_ERR;
      const uint32_t bits = v.str_rx ? v.str_rx[x.sid] : RX_FB;
      if (bits & RX_FB) return JS_FB;
      x = cv_node(Node{((bits >> p[i + 1]) & 1u) ? (uint32_t)N_TRUE : (uint32_t)N_FALSE, 0, 0, 0}, true);
    }
  }
  *out = x;
  return JS_OK;
}

KYV_HD int operand_cv(const View& v, NodeTab R, const CondOperand& o, uint32_t elem, JList& L, CV* out, uint32_t* miss,
                      uint32_t row = NONE) {
  if (o.kind != OK_JMES) return cv_operand(v, R, o, out, miss, row) ? JS_OK : JS_NOTFOUND;
  if (jmes_chain_form(v.pool + o.a, o.nseg)) return jmes_chain_cv(v, R, o, out, miss, row);
  JRes r;
  const int st = jmes_run(v, R, o, elem, L, &r, miss);
  if (st != JS_OK) return st;
  *out = jres_cv(v, R, r, L);
  return JS_OK;
}


// operator.parseDuration (operator.go:94-138): 1 both durations (seconds), 0 not durations
KYV_HD int dur_side(const View& v, const CV& x, int64_t* d, bool* have) {
  *have = false;
  if (x.t == CT_STR && x.sid != SID_ZERO && (sflags(v, x.sid) & SF_DUR)) { *d = v.str_dur[x.sid]; *have = true; }
  return 0;
}
KYV_HD bool num_secs(const CV& x, int64_t* d) {
  if (x.t == CT_INT) { *d = (int64_t)((uint64_t)x.i * 1000000000ull); return true; }
  if (x.t == CT_FLOAT) { *d = (int64_t)((uint64_t)go_f2i(x.f) * 1000000000ull); return true; }
  return false;
}
KYV_HD double dur_seconds(int64_t d) {  // time.Duration.Seconds
  int64_t sec = d / 1000000000LL, nsec = d % 1000000000LL;
  return (double)sec + (double)nsec / 1e9;
}
KYV_HD bool parse_duration2(const View& v, const CV& k, const CV& x, double* ks, double* vs) {
  int64_t kd = 0, vd = 0;
  bool hk, hv;
  dur_side(v, k, &kd, &hk);
  dur_side(v, x, &vd, &hv);
  if (!hk && !hv) return false;
  if (!hk && !num_secs(k, &kd)) return false;
  if (!hv && !num_secs(x, &vd)) return false;
  *ks = dur_seconds(kd);
  *vs = dur_seconds(vd);
  return true;
}

KYV_HD bool qty_ok(const View& v, uint32_t sid) { return (sflags(v, sid) & (SF_QTY | SF_QTY_BIG)) != 0; }
// Quantity.Cmp; CR_FB when either side is beyond int128 nano units
KYV_HD int qty_cmp(const View& v, uint32_t a, uint32_t b, bool* fb) {
  if ((sflags(v, a) | sflags(v, b)) & SF_QTY_BIG) { *fb = true; return 0; }
  return cmp128(v.str_qty[2 * a + 1], (uint64_t)v.str_qty[2 * a], v.str_qty[2 * b + 1], (uint64_t)v.str_qty[2 * b]);
}
// strconv.ParseInt(s, 10, 64): 1 ok (*out), 0 error, 2 ok but not exact in the dictionary's float column
KYV_HD int parse_int_sid(const View& v, uint32_t sid, int64_t* out) {
  uint32_t f = sflags(v, sid);
  if (!(f & SF_INT)) return 0;
  if (f & SF_INT_BIG) return 2;
  *out = (int64_t)v.str_f64[sid];
  return 1;
}

// ---------------------------------------------------------------- Equal / NotEqual (equal.go, notequal.go)
KYV_HD int deep_equal_arr(const View& v, NodeTab R, const CV& a, const CV& b) {
  if (a.n != b.n) return CR_FALSE;
  for (uint32_t j = 0; j < a.n; j++) {
    CV x = cv_elem(v, R, a, j), y = cv_elem(v, R, b, j);
    if (x.t == CT_ARR || x.t == CT_MAP || y.t == CT_ARR || y.t == CT_MAP) return CR_FB;
    if (x.t != y.t) return CR_FALSE;
    bool eq = true;
    switch (x.t) {
      case CT_BOOL: eq = x.b == y.b; break;
      case CT_INT: eq = x.i == y.i; break;
      case CT_FLOAT: eq = x.f == y.f; break;
      case CT_STR: eq = x.sid == y.sid; break;
      default: break;
    }
    if (!eq) return CR_FALSE;
  }
  return CR_TRUE;
}

KYV_HD int op_equal(const View& v, NodeTab R, const CV& k, const CV& x, bool neg) {
  auto ret = [&](bool b) { return (int)((b != neg) ? CR_TRUE : CR_FALSE); };
  switch (k.t) {
    case CT_BOOL:
      if (x.t != CT_BOOL) return neg ? CR_TRUE : CR_FALSE;
      return ret(x.b == k.b);
    case CT_INT:
      switch (x.t) {
        case CT_INT: return ret(x.i == k.i);
        case CT_FLOAT: return x.f == __builtin_trunc(x.f) ? ret(go_f2i(x.f) == k.i) : CR_FALSE;
        case CT_STR: {
          int64_t y;
          int p = parse_int_sid(v, x.sid, &y);
          if (p == 2) return CR_FB;
          return p ? ret(y == k.i) : (neg ? CR_TRUE : CR_FALSE);
        }
        default: return neg ? CR_TRUE : CR_FALSE;
      }
    case CT_FLOAT:
      switch (x.t) {
        case CT_INT: return k.f == __builtin_trunc(k.f) ? ret(go_f2i(k.f) == x.i) : (neg ? CR_TRUE : CR_FALSE);
        case CT_FLOAT: return ret(x.f == k.f);
        case CT_STR:
          if (sflags(v, x.sid) & SF_FLOAT) return ret(v.str_f64[x.sid] == k.f);
          return neg ? CR_TRUE : CR_FALSE;
        default: return neg ? CR_TRUE : CR_FALSE;
      }
    case CT_STR: {
      double ks, vs;
      if (parse_duration2(v, k, x, &ks, &vs)) return ret(ks == vs);
      if (qty_ok(v, k.sid) && x.t == CT_STR) {
        if (neg && x.sid == SID_EMPTY) return glob_sid(v, x.sid, k.sid) ? CR_FALSE : CR_TRUE;
        if (!qty_ok(v, x.sid)) return CR_FALSE;
        bool fb = false;
        int c = qty_cmp(v, k.sid, x.sid, &fb);
        if (fb) return CR_FB;
        return ret(c == 0);
      }
      if (x.t == CT_STR) return ret(glob_sid(v, x.sid, k.sid));
      return neg ? CR_TRUE : CR_FALSE;
    }
    case CT_ARR:
      if (x.t != CT_ARR) return neg ? CR_TRUE : CR_FALSE;
      {
        int r = deep_equal_arr(v, R, k, x);
        return r == CR_FB ? CR_FB : ret(r == CR_TRUE);
      }
    case CT_MAP:
      if (x.t != CT_MAP) return neg ? CR_TRUE : CR_FALSE;
      return CR_FB;
    default: return CR_FALSE;  // nil key: no handler branch
  }
}

// ---------------------------------------------------------------- In / NotIn (in.go, notin.go)
KYV_HD bool wild2(const View& v, uint32_t a, uint32_t b) { return glob_sid(v, a, b) || glob_sid(v, b, a); }

// fmt.Sprint form of a scalar key / element; NONE -> the device cannot render it
KYV_HD uint32_t sprint_sid(const CV& x) {
  if (x.t == CT_ARR || x.t == CT_MAP) return NONE;
  return x.sid;
}

// key string vs value: keyExistsInArray (in.go:52-86) when in_list; anyKeyExistsInArray (anyin.go:51-96) otherwise.
// returns CR_TRUE/CR_FALSE for exists, CR_FB, or 4 = invalidType
constexpr int CR_INVALID = 4;
KYV_HD int key_exists(const View& v, NodeTab R, uint32_t ks, const CV& x, const Cond& c, bool in_list) {
  if (x.t == CT_ARR) {
    for (uint32_t j = 0; j < x.n; j++) {
      uint32_t es = sprint_sid(cv_elem(v, R, x, j));
      if (es == NONE) return CR_FB;
      if (wild2(v, es, ks)) return CR_TRUE;
    }
    return CR_FALSE;
  }
  if (x.t != CT_STR) return CR_INVALID;
  if (glob_sid(v, x.sid, ks)) return CR_TRUE;
  if (x.res) return CR_FB;  // resource-side string the handler would JSON-decode
  const CondOperand& o = c.value;
  if (!in_list) {
    if (o.sv & SV_RANGE) {
      Val y;
      y.t = N_STR; y.sid = y.wsid = y.nsid = ks; y.i = 0; y.f = 0;
      bool fb = false;
      bool r = leaf_match(v, v.leaves[c.leaf], y, &fb);
      if (fb) return CR_FB;
      return r ? CR_TRUE : CR_FALSE;
    }
    if (!(o.sv & SV_JSON)) return ks == x.sid ? CR_TRUE : CR_FALSE;  // arr = [value]
  }
  if (!(o.sv & SV_LIST)) return CR_INVALID;
  for (uint32_t j = 0; j < o.nlist; j++) if (v.pool[o.list + j] == ks) return CR_TRUE;
  return CR_FALSE;
}

constexpr uint32_t MAX_CKEYS = 16;

// key list: element sids (fmt.Sprint, or v.(string) for In/NotIn which panics on non-strings). key_list checks
// every element in order (CR_PANIC / CR_FB on the first that fails); key_at(i) is element i's sid, recomputed
// where it is used instead of copied into a per-lane array (which would live in scratch memory)
KYV_HD int key_list(const View& v, NodeTab R, const CV& k, bool strict) {
  if (k.n > MAX_CKEYS) return CR_FB;
  for (uint32_t j = 0; j < k.n; j++) {
    CV e = cv_elem(v, R, k, j);
    if (strict && e.t != CT_STR) return CR_PANIC;
    if (sprint_sid(e) == NONE) return CR_FB;
  }
  return CR_TRUE;
}
KYV_HD uint32_t key_at(const View& v, NodeTab R, const CV& k, uint32_t i) { return sprint_sid(cv_elem(v, R, k, i)); }

KYV_HD int op_in(const View& v, NodeTab R, const Cond& c, const CV& k, const CV& x, bool notin) {
  if (k.t == CT_STR || k.t == CT_INT || k.t == CT_FLOAT) {
    uint32_t ks = sprint_sid(k);
    if (ks == NONE) return CR_FB;
    int e = key_exists(v, R, ks, x, c, true);
    if (e == CR_FB) return CR_FB;
    if (e == CR_INVALID) return CR_FALSE;
    return (e == CR_TRUE) != notin ? CR_TRUE : CR_FALSE;
  }
  if (k.t != CT_ARR) return CR_FALSE;
  const uint32_t n = k.n;
  int kr = key_list(v, R, k, true);
  if (kr != CR_TRUE) return kr;
  // setExistsInArray (in.go:104-143). The value side is x itself or the condition's literal list, chosen by a flag:
  // a pointer that may point at the caller's CV forces that CV into scratch memory (round 5: 165 scratch
  // instructions in match_deny_kernel)
  const bool use_arr = x.t == CT_ARR;
  auto found = [&](uint32_t s) {
    if (use_arr) {
      for (uint32_t j = 0; j < x.n; j++) if (cv_elem(v, R, x, j).sid == s) return true;
      return false;
    }
    for (uint32_t j = 0; j < c.value.nlist; j++) if (v.pool[c.value.list + j] == s) return true;
    return false;
  };
  if (use_arr) {
    for (uint32_t j = 0; j < x.n; j++) if (cv_elem(v, R, x, j).t != CT_STR) return CR_FALSE;  // invalidType
  } else if (x.t == CT_STR) {
    if (n == 1 && key_at(v, R, k, 0) == x.sid) return CR_TRUE;
    if (x.res) return CR_FB;
    if (!(c.value.sv & SV_LIST)) return CR_FALSE;
  } else {
    return CR_FALSE;
  }
  bool all_in = true;
  for (uint32_t i = 0; i < n; i++) if (!found(key_at(v, R, k, i))) { all_in = false; break; }
  return (notin ? !all_in : all_in) ? CR_TRUE : CR_FALSE;
}

// ---------------------------------------------------------------- AnyIn / AllIn / AnyNotIn / AllNotIn
KYV_HD int op_any_all(const View& v, NodeTab R, const Cond& c, const CV& k, const CV& x, bool all, bool neg) {
  if (k.t == CT_STR || k.t == CT_INT || k.t == CT_FLOAT) {
    uint32_t ks = sprint_sid(k);
    if (ks == NONE) return CR_FB;
    int e = key_exists(v, R, ks, x, c, false);
    if (e == CR_FB) return CR_FB;
    if (e == CR_INVALID) return CR_FALSE;
    return (e == CR_TRUE) != neg ? CR_TRUE : CR_FALSE;
  }
  if (k.t != CT_ARR) return CR_FALSE;
  const uint32_t n = k.n;
  int kr = key_list(v, R, k, false);
  if (kr != CR_TRUE) return kr;
  // anySetExistsInArray / allSetExistsInArray (anyin.go:115-180, allin.go:115-180)
  uint32_t matched = 0;
  if (x.t == CT_ARR) {
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t ki = key_at(v, R, k, i);
      for (uint32_t j = 0; j < x.n; j++) {
        uint32_t es = sprint_sid(cv_elem(v, R, x, j));
        if (es == NONE) return CR_FB;
        if (wild2(v, ki, es)) { matched++; break; }
      }
    }
  } else if (x.t == CT_STR) {
    if (n == 1 && key_at(v, R, k, 0) == x.sid) return neg ? CR_FALSE : CR_TRUE;
    if (x.res) return CR_FB;
    const CondOperand& o = c.value;
    if (o.sv & SV_RANGE) {
      uint32_t hits = 0;
      for (uint32_t i = 0; i < n; i++) {
        Val y;
        y.t = N_STR; y.sid = y.wsid = y.nsid = key_at(v, R, k, i); y.i = 0; y.f = 0;
        bool fb = false;
        bool r = leaf_match(v, v.leaves[(!all && neg) ? c.leaf_neg : c.leaf], y, &fb);
        if (fb) return CR_FB;
        hits += r ? 1u : 0u;
      }
      if (!all) return hits > 0 ? CR_TRUE : CR_FALSE;       // AnyIn; AnyNotIn (on the "!-" pattern)
      if (neg) return hits == 0 ? CR_TRUE : CR_FALSE;       // AllNotIn
      return hits == n ? CR_TRUE : CR_FALSE;                // AllIn
    }
    if (o.sv & SV_JSON) {
      if (!(o.sv & SV_LIST)) return CR_FALSE;  // invalidType
      for (uint32_t i = 0; i < n; i++) {
        const uint32_t ki = key_at(v, R, k, i);
        for (uint32_t j = 0; j < o.nlist; j++)
          if (wild2(v, ki, v.pool[o.list + j])) { matched++; break; }
      }
    } else {
      for (uint32_t i = 0; i < n; i++) if (wild2(v, key_at(v, R, k, i), x.sid)) matched++;
    }
  } else {
    return CR_FALSE;
  }
  bool r;
  if (!all) r = neg ? matched < n : matched > 0;
  else r = neg ? matched == 0 : matched == n;
  return r ? CR_TRUE : CR_FALSE;
}

// ---------------------------------------------------------------- numeric (numeric.go)
KYV_HD bool cmp_by(uint8_t op, double a, double b) {
  switch (op) {
    case CO_GT: return a > b;
    case CO_GE: return a >= b;
    case CO_LT: return a < b;
    case CO_LE: return a <= b;
    default: return false;
  }
}
KYV_HD int num_float(const View& v, uint8_t op, double kf, const CV& kcv, const CV& x) {
  switch (x.t) {
    case CT_INT: return cmp_by(op, kf, (double)x.i) ? CR_TRUE : CR_FALSE;
    case CT_FLOAT: return cmp_by(op, kf, x.f) ? CR_TRUE : CR_FALSE;
    case CT_STR: {
      double ks, vs;
      if (parse_duration2(v, kcv, x, &ks, &vs)) return cmp_by(op, ks, vs) ? CR_TRUE : CR_FALSE;
      if (sflags(v, x.sid) & SF_FLOAT) return cmp_by(op, kf, v.str_f64[x.sid]) ? CR_TRUE : CR_FALSE;
      return CR_FALSE;  // ParseInt cannot succeed where ParseFloat failed
    }
    default: return CR_FALSE;
  }
}
KYV_HD int op_numeric(const View& v, const CV& k, const CV& x, uint8_t op) {
  switch (k.t) {
    case CT_INT: return num_float(v, op, (double)k.i, k, x);
    case CT_FLOAT: return num_float(v, op, k.f, k, x);
    case CT_STR: {
      double ks, vs;
      if (parse_duration2(v, k, x, &ks, &vs)) return cmp_by(op, ks, vs) ? CR_TRUE : CR_FALSE;
      if (x.t == CT_STR && qty_ok(v, k.sid) && qty_ok(v, x.sid)) {
        bool fb = false;
        int c = qty_cmp(v, k.sid, x.sid, &fb);
        if (fb) return CR_FB;
        return cmp_by(op, (double)c, 0.0) ? CR_TRUE : CR_FALSE;
      }
      if (sflags(v, k.sid) & SF_FLOAT) {
        CV kf = k;
        kf.t = CT_FLOAT;
        kf.f = v.str_f64[k.sid];
        return num_float(v, op, kf.f, kf, x);
      }
      if (sflags(v, k.sid) & SF_SEMVERISH) return CR_FB;  // blang/semver comparison: CPU engine
      return CR_FALSE;
    }
    default: return CR_FALSE;
  }
}

// ---------------------------------------------------------------- Duration* (duration.go:30-150)
// DurationOperatorHandler.Evaluate: an int / float operand is time.Duration(x) seconds (float truncated, the product
// wrapping like Go's), a string one time.ParseDuration'd (failure: false); any other type: false
KYV_HD bool dur_operand(const View& v, const CV& x, int64_t* d) {
  if (x.t == CT_INT || x.t == CT_FLOAT) return num_secs(x, d);
  if (x.t == CT_STR && x.sid != NONE && (sflags(v, x.sid) & SF_DUR)) { *d = v.str_dur[x.sid]; return true; }
  return false;
}
KYV_HD int op_duration(const View& v, const CV& k, const CV& x, uint8_t op) {
  int64_t kd, vd;
  if (!dur_operand(v, k, &kd) || !dur_operand(v, x, &vd)) return CR_FALSE;
  bool r;
  switch (op) {
    case CO_DGT: r = kd > vd; break;
    case CO_DGE: r = kd >= vd; break;
    case CO_DLT: r = kd < vd; break;
    default: r = kd <= vd; break;
  }
  return r ? CR_TRUE : CR_FALSE;
}

KYV_HD int eval_cond(const View& v, NodeTab R, const Cond& c, const CV& k, const CV& x) {
  switch (c.op) {
    case CO_EQ: return op_equal(v, R, k, x, false);
    case CO_NE: return op_equal(v, R, k, x, true);
    case CO_IN: return op_in(v, R, c, k, x, false);
    case CO_NOTIN: return op_in(v, R, c, k, x, true);
    case CO_ANYIN: return op_any_all(v, R, c, k, x, false, false);
    case CO_ALLIN: return op_any_all(v, R, c, k, x, true, false);
    case CO_ANYNOTIN: return op_any_all(v, R, c, k, x, false, true);
    case CO_ALLNOTIN: return op_any_all(v, R, c, k, x, true, true);
    case CO_GT: case CO_GE: case CO_LT: case CO_LE: return op_numeric(v, k, x, c.op);
    case CO_DGT: case CO_DGE: case CO_DLT: case CO_DLE: return op_duration(v, k, x, c.op);
    default: return CR_FALSE;
  }
}

// Whole program: substitution first (every reference of the document, vars.go:352-431: any NotFoundError ->
// error), then any/all evaluation (evaluate.go:42-69). Returns CR_TRUE / CR_FALSE / CR_FB / CR_PANIC, or
// CP_ERROR with *err_cond / *err_side / *err_seg naming the first unresolved reference (for the host message).
// kJ = false instantiates the program without the JMESPath interpreter (no projection lists on the stack): the
// light match kernel evaluates only rules whose programs hold no OK_JMES operand (the host routes the others).
constexpr int CP_ERROR = 5;
// eval_prog_inl: the body, always inlined (the match kernels call it from ONE site each, so the program is inline code
// instead of a call whose frame goes through scratch memory); eval_prog: the same, left to the inliner (foreach)
template <bool kJ = true>
KYV_HD __attribute__((always_inline)) int eval_prog_inl(const View& v, NodeTab R, uint32_t prog, uint32_t* err_cond,
                                                        uint32_t* err_side, uint32_t* err_seg, uint32_t elem = NONE,
                                                        uint32_t row = NONE) {
  const CondProg& p = v.cprogs[prog];
  const uint32_t nany = p.nany == NONE ? 0u : p.nany;
  for (uint32_t blk = 0; blk < 2; blk++) {
    uint32_t c0 = blk ? p.all0 : p.any0, n = blk ? p.nall : nany;
    for (uint32_t i = 0; i < n; i++) {
      const Cond& c = v.conds[c0 + i];
      CV tmp;
      uint32_t miss = 0;
      for (uint32_t side = 0; side < 2; side++) {
        const CondOperand& o = side ? c.value : c.key;
        if (o.kind == OK_PATH && !cv_operand(v, R, o, &tmp, &miss, row)) {
          *err_cond = c0 + i; *err_side = side; *err_seg = miss;
          return CP_ERROR;
        }
        if (o.kind == OK_JMES) {
          if constexpr (!kJ) {
            if (!jmes_chain_form(v.pool + o.a, o.nseg)) return CR_FB;
            const int st = jmes_chain_cv(v, R, o, &tmp, &miss, row);
            if (st == JS_FB) return CR_FB;
            if (st == JS_NOTFOUND) { *err_cond = c0 + i; *err_side = side; *err_seg = miss; return CP_ERROR; }
            if (st == JS_ERR) { *err_cond = c0 + i; *err_side = side; *err_seg = NONE; return CP_ERROR; }
          } else {
            JList L;
            const int st = operand_cv(v, R, o, elem, L, &tmp, &miss, row);
            if (st == JS_FB || st == JS_TERR) return CR_FB;
            if (st == JS_NOTFOUND) { *err_cond = c0 + i; *err_side = side; *err_seg = miss; return CP_ERROR; }
            if (st == JS_ERR) { *err_cond = c0 + i; *err_side = side; *err_seg = NONE; return CP_ERROR; }
          }
        }
      }
    }
  }
  // the any / all evaluation (evaluate.go:42-69) as ONE loop over the conditions, per-lane state instead of two loops
  // around a per-condition callable: the compiler kept that callable out of line (two call sites), and every call saved
  // the caller's registers to scratch memory (C5 round 4: 1.8 GB of scratch writes per evaluation in match_deny_kernel)
  const uint32_t na = p.nany == NONE ? 0u : p.nany;
  uint32_t any = 0;  // (a loop-carried flag: an integer word, kyv_pss.h eval_pss)
  for (uint32_t q = 0; q < na + p.nall; q++) {
    const bool isany = q < na;
    if (!isany && q == na && p.nany != NONE && !any) return CR_FALSE;  // no any-condition held
    if (isany && any) continue;
    const Cond& c = v.conds[isany ? p.any0 + q : p.all0 + (q - na)];
    CV k, x;
    uint32_t miss;
    int r;
    if constexpr (kJ) {
      JList lk, lx;
      operand_cv(v, R, c.key, elem, lk, &k, &miss, row);
      operand_cv(v, R, c.value, elem, lx, &x, &miss, row);
      r = eval_cond(v, R, c, k, x);
    } else {
      if (c.key.kind == OK_JMES) jmes_chain_cv(v, R, c.key, &k, &miss, row);  // (a chain program: checked in the first pass)
      else cv_operand(v, R, c.key, &k, &miss, row);
      if (c.value.kind == OK_JMES) jmes_chain_cv(v, R, c.value, &x, &miss, row);
      else cv_operand(v, R, c.value, &x, &miss, row);
      r = eval_cond(v, R, c, k, x);
    }
    if (r == CR_FB || r == CR_PANIC) return r;
    if (isany) { if (r == CR_TRUE) any = 1; }
    else if (r == CR_FALSE) return CR_FALSE;
  }
  if (p.nany != NONE && !any) return CR_FALSE;
  return CR_TRUE;
}
template <bool kJ = true>
KYV_HD int eval_prog(const View& v, NodeTab R, uint32_t prog, uint32_t* err_cond, uint32_t* err_side, uint32_t* err_seg,
                     uint32_t elem = NONE, uint32_t row = NONE) {
  return eval_prog_inl<kJ>(v, R, prog, err_cond, err_side, err_seg, elem, row);
}

}  // namespace kyv
