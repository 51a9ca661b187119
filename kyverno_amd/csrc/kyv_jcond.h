// Device helpers of the runtime-compiled condition kernel (jit.cpp CondGen): deny / foreach / precondition rules
// whose conditions hold JMESPath-subset operands (kyv_layout.h OK_JMES), generated per ruleset.
//
// Reference semantics are those of the interpreter in kyv_cond.h (jmes_run, eval_prog) and kyv_pss.h
// (eval_foreach): pkg/engine/variables/evaluate.go:11-83, vars.go:352-431, pkg/engine/validation.go:319-421 and the
// kyverno/go-jmespath fork. What the generated code changes is how values are reached, not what they are:
//  - every static field / flatten step of a program is a path-column read (kyv_layout.h "Path columns": the
//    compiler registers the programs' static paths in the path trie next to the patterns'), so a chain like
//    spec.containers[].securityContext.capabilities.drop[] costs one round of independent loads per level
//    instead of a binary search per key;
//  - foreach lists are streamed (nested loops over the list's arrays, no materialised element list);
//  - condition operands that are lists live in LDS, lane-interleaved (element j of lane l at j * 64 + l), so no
//    per-lane scratch memory is touched.
// A value is (node index relative to the resource root or NONE, node type or T_UNK when not loaded, the node's `a`,
// its column row in the row space of its static trie position or NONE).
#pragma once
#include "kyv_wave.h"
#include "kyv_cond.h"
#include "kyv_pss.h"

namespace kyv {

constexpr uint32_t JCAP = 16;  // lane list capacity of an operand (longer -> the pair goes to the CPU engine)

__device__ __forceinline__ uint64_t jc_col(const View& v, uint32_t col, uint32_t row) {
  if (row == NONE) return COL_NONE;
  KYV_ACCT_ADDK(2u, 0, 8);
  const uint32_t off = sld32(v.col_off + col);
  return *(const KYV_AS_GLOBAL uint64_t*)(v.colv + (size_t)off + row);
}
__device__ __forceinline__ uint32_t jc_dec(uint64_t x, uint32_t* t, uint32_t* a) {
  const uint32_t lo = (uint32_t)x;
  *a = (uint32_t)(x >> 32);
  if (lo == NONE) { *t = T_UNK; *a = 0; return NONE; }
  *t = lo >> COL_TYPE_SHIFT;
  return lo & COL_INDEX_MASK;
}
// node type of a value (loads the row when the column did not supply it); NONE reads as null
__device__ __forceinline__ uint32_t jc_type(const Node* R, uint32_t i, uint32_t t) {
  if (i == NONE) return N_NULL;
  return t != T_UNK ? t : (gtk(R + i) & 0xFu);
}
// j_field (kyv_cond.h): field `key` of a value; a non-map, a missing key and a null value all give NONE.
// col: the path column of this lookup at the value's row (NONE: binary search over the map's sorted keys)
__device__ __forceinline__ void jc_field(const View& v, const Node* R, uint32_t i, uint32_t row, uint32_t col, uint32_t key,
                                         uint32_t* oi, uint32_t* ot, uint32_t* oa) {
  *ot = T_UNK;
  *oa = 0;
  if (col != NONE && row != NONE) {
    // the column alone decides: its entry exists iff the value reached along this static path is a map holding
    // `key` (a null or absent parent has no entry), so a chain of fields from one row is one round of independent
    // loads
    uint32_t x = jc_dec(jc_col(v, col, row), ot, oa);
    if (x != NONE && *ot == N_NULL) { x = NONE; *ot = T_UNK; *oa = 0; }
    *oi = x;
    return;
  }
  if (i == NONE) { *oi = NONE; return; }
  const Node m = gnode(R + i);
  if (node_type(m) != N_MAP) { *oi = NONE; return; }
  const uint32_t x = wmap_find(R, m.a, m.b, key);
  if (x == NONE) { *oi = NONE; return; }
  const Node n = gnode(R + x);
  if (node_type(n) == N_NULL) { *oi = NONE; return; }
  *oi = x;
  *ot = node_type(n);
  *oa = n.a;
}
// array view of a value: element count, first element, row of element 0 in the elements' row space (NONE when the
// elements have no rows); false when the value is not an array. lencol: the (count, element-0 row) column of the
// value's trie position, read when the value came through a column
__device__ __forceinline__ bool jc_arr(const View& v, const Node* R, uint32_t i, uint32_t t, uint32_t a, uint32_t row,
                                       uint32_t lencol, uint32_t* cnt, uint32_t* aa, uint32_t* eb) {
  if (i == NONE) return false;
  if (t != T_UNK && t != N_ARR) return false;
  if (t == N_ARR && lencol != NONE && row != NONE) {
    const uint64_t x = jc_col(v, lencol, row);
    if ((uint32_t)x != NONE) { *cnt = (uint32_t)x; *eb = (uint32_t)(x >> 32); *aa = a; return true; }
  }
  const Node n = gnode(R + i);
  if (node_type(n) != N_ARR) return false;
  *cnt = n.b;
  *aa = n.a;
  *eb = n.c;
  return true;
}
// element j of an array: index aa + j, row eb + j; type and `a` from the elements' self column when it exists;
// a null element reads as NONE (the flatten of jmes_run)
__device__ __forceinline__ void jc_elem(const View& v, const Node* R, uint32_t aa, uint32_t eb, uint32_t j, uint32_t self,
                                        uint32_t* oi, uint32_t* ot, uint32_t* oa, uint32_t* orow) {
  *oi = aa + j;
  *ot = T_UNK;
  *oa = 0;
  *orow = eb == NONE ? NONE : eb + j;
  if (self != NONE && *orow != NONE) {
    uint32_t t, a;
    if (jc_dec(jc_col(v, self, *orow), &t, &a) != NONE) { *ot = t; *oa = a; }
  }
  if (jc_type(R, *oi, *ot) == N_NULL) { *oi = NONE; *ot = T_UNK; *oa = 0; }
}
// list entry of a (non-null) value: a string whose type and id came with its column entry goes in by id (the
// operator reads it without loading the node), anything else by node index
__device__ __forceinline__ uint32_t jc_ent(uint32_t i, uint32_t t, uint32_t a) {
  return (t == N_STR && a < JMES_SIDBIT) ? (a | JMES_SIDBIT) : i;
}
// list entry of a map key (keys(@)): the key string by id, read from the entry's node word here, where the loads of
// one map's entries are independent, instead of one dependent node load per element in the operator
__device__ __forceinline__ uint32_t jc_keyent(const Node* R, uint32_t idx) {
  const uint32_t k = gtk(R + idx) >> 4;
  return k < JMES_SIDBIT ? (k | JMES_SIDBIT) : (idx | JMES_KEYBIT);
}
// one list element into the lane's LDS list (lane-interleaved); false when the list is full
__device__ __forceinline__ bool jc_push(uint32_t* L, uint32_t* n, uint32_t e) {
  if (*n >= JCAP) return false;
  L[(size_t)*n << 6] = e;
  (*n)++;
  return true;
}
// util.go isFalse of a single (non-list, non-literal) result
__device__ __forceinline__ bool jc_false1(const Node* R, uint32_t cur) {
  if (cur == NONE) return true;
  if (cur & JMES_KEYBIT) return node_key(gnode(R + (cur & ~JMES_KEYBIT))) == SID_EMPTY;
  const Node n = gnode(R + cur);
  switch (node_type(n)) {
    case N_NULL: case N_FALSE: return true;
    case N_STR: return n.a == SID_EMPTY;
    case N_ARR: case N_MAP: return n.b == 0;
    default: return false;
  }
}
// fmt.Sprint sid of a (non-null) list element as the operators see it (sprint_sid(cv_elem(...)), kyv_cond.h): a
// string whose id came with its column entry directly, anything else from its node (NONE: no device rendering)
__device__ __forceinline__ uint32_t jc_sprint(const Node* R, uint32_t i, uint32_t t, uint32_t a) {
  if (i == NONE) return KSID(NIL_STR);
  if (t == N_STR) return a;
  return sprint_sid(cv_node(gnode(R + i), true));
}
// condition-set test of string s (compiler.cpp assign_cond_sets): wild2(s, e) for some e of the set; one mask load
// when the batch has glob masks (bit = gpats.size() + set index), else the set's literals one by one
__device__ __forceinline__ bool jc_inset(const View& v, uint32_t bit, const uint32_t* set, uint32_t n, uint32_t s) {
  if (v.str_gmask) return (v.str_gmask[(size_t)s * v.gmask_words + bit / 32] >> (bit % 32)) & 1u;
  for (uint32_t j = 0; j < n; j++) if (wild2(v, s, set[j])) return true;
  return false;
}
// operand value of a JMESPath result (jres_cv with the list in LDS)
__device__ __forceinline__ CV jc_cv(const View& v, const Node* R, bool lst, uint32_t cur, uint32_t lit, const uint32_t* L,
                                    uint32_t n) {
  const Node nil{N_NULL, 0, 0, 0};
  if (lit != NONE) {
    CV x = cv_node(v.cnodes[lit], false);
    if (x.t == CT_ARR) x.node = lit;
    return x;
  }
  if (lst) {
    CV x = cv_node(nil, true);
    x.t = CT_ARR; x.sid = NONE; x.n = n; x.vl = L; x.pad = 6;
    return x;
  }
  if (cur == NONE) return cv_node(nil, true);
  if (cur & JMES_KEYBIT) {
    CV x = cv_node(nil, true);
    x.t = CT_STR;
    x.sid = node_key(gnode(R + (cur & ~JMES_KEYBIT)));
    return x;
  }
  CV x = cv_node(gnode(R + cur), true);
  if (x.t == CT_ARR) x.node = cur;
  return x;
}
__device__ __forceinline__ CV jc_lit(const View& v, uint32_t a) {
  CV x = cv_node(v.cnodes[a], false);
  if (x.t == CT_ARR) x.node = a;
  return x;
}

}  // namespace kyv
