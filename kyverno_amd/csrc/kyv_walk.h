// validatePatterns (pkg/engine/validation.go:618-702) over a Walker: the alternative loop of pattern /
// anyPattern rules, their statuses and failing-path records. Shared by the host backend, the interpreted walk
// kernel (kyv_engine.hip) and the runtime-compiled walk kernels (jit.cpp).
#pragma once
#include "kyv_eval.h"

namespace kyv {

// The pattern / anyPattern verdict (validatePatterns, validation.go:618-702) for the lanes with `walk`; every lane
// of a wave calls this for the same rule, so the failing-path records are emitted through `sink` at
// wave-uniform points: one emit per anyPattern alternative (trip count uniform per rule), with `has` set on
// the lanes whose alternative failed.
//
// `Walker::run(v, root, walk, R, hp, row, rd, out)` runs one compiled pattern for the lanes with `walk` set (row: the
// resource's batch position, i.e. its column row, passed explicitly rather than derived from `hp`): the host
// instantiation is the per-lane eval_pattern (HostWalker below), the kernel's is the wave-uniform walker
// (kyv_wave.h).
struct HostWalker {
  Stack stk;
  KYV_HD void run(const View& v, uint32_t root, bool walk, const Node* R, const ResHeader* hp, uint32_t row,
                  const RuleDesc& rd, PatOut& out) {
    (void)row;
    out.status = ST_NONE;
    if (walk) eval_pattern(v, root, NodeTab{R}, *hp, rd, stk, out);
  }
};

// The alternative loop of validatePatterns over a callable that walks alternative `a` (alt(a, walk, po)): shared by
// pair_walk (the alternative's root read from the rule) and the fused compiled walk kernels (jit.cpp), whose
// per-rule code passes its roots as constants
template <class Sink, class AltFn>
KYV_HD uint8_t pair_walk_alts(bool pattern, uint32_t nalts, bool walk, uint32_t r, uint32_t k, Sink& sink, AltFn&& alt) {
  uint8_t st = ST_NONE;
  uint32_t nfail = 0, nskip = 0;
  for (uint32_t a = 0; a < nalts; a++) {
    PatOut po;
    alt(a, walk, po);
    bool rec = false;
    if (walk) {
      switch (po.status) {
        case ST_PASS: st = (uint8_t)(ST_PASS | ((a < 30 ? a : 30) << 3)); walk = false; break;  // alt index for the message
        case ST_SKIP: nskip++; break;
        case ST_FAIL: case ST_ERROR:
          if (pattern && po.status == ST_ERROR) { st = ST_ERROR; walk = false; break; }
          rec = true;
          nfail++;
          break;
        default: st = po.status; walk = false;  // fallback / panic / nondeterministic at this point of the walk
      }
    }
    FailRec fr;
    if (rec) {
      fr.res = r; fr.rule = k; fr.tmpl = po.status == ST_FAIL ? po.tmpl : NONE; fr.alt = (uint16_t)a; fr.nalt = 0;
      for (int i = 0; i < MAX_IDX; i++) fr.idx[i] = (uint16_t)(po.idx >> (16 * i));
      fr.key[0] = po.key0;
      fr.key[1] = po.key1;
    }
    sink.emit(rec, fr);
  }
  if (walk) {
    if (pattern) st = nfail ? ST_FAIL : ST_SKIP;
    else if (nfail) st = ST_FAIL;
    else if (nskip) st = ST_SKIP;
    else st = (uint8_t)(ST_PASS | (31 << 3));  // empty anyPattern list: pass with the rule message (validation.go:701)
  }
  return st;
}

template <class Sink, class Walker>
KYV_HD uint8_t pair_walk(const View& v, const RuleDesc& rd, bool walk, uint32_t r, uint32_t k, const Node* R, Walker& wk,
                         Sink& sink) {
  // address only (walkers read it for metadata expansion); not predicated on `walk`, so a compiled walker's column
  // preload (row r) does not wait for the loads `walk` depends on
  const ResHeader* hp = v.hdr + r;
  const uint32_t nalts = rd.kind == RK_PATTERN ? 1 : rd.nalts;  // uniform across the wave
  const uint32_t row = r < v.nres ? r : NONE;
  return pair_walk_alts(rd.kind == RK_PATTERN, nalts, walk, r, k, sink, [&](uint32_t a, bool w, PatOut& po) {
    wk.run(v, rd.kind == RK_PATTERN ? rd.root : v.pool[rd.root + a], w, R, hp, row, rd, po);
  });
}

}  // namespace kyv
