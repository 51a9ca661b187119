// ORACLE — test infrastructure only (see ojson.h header). C entry points for ctypes (oracle/oracle.py).
// Every function returns a malloc'ed JSON string (free with oracle_free) or an int.
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <cstring>

#include "goutil.h"
#include "ocond.h"
#include "oengine.h"
#include "ojson.h"
#include "opss.h"
#include "orefs.h"
#include "ovalidate.h"

using namespace orc;
using oj::T;
using oj::Value;
using oj::VP;

static char* dup(const std::string& s) {
  char* p = (char*)malloc(s.size() + 1);
  memcpy(p, s.c_str(), s.size() + 1);
  return p;
}

static std::map<std::string, std::string> labels_of(const VP& v) {
  std::map<std::string, std::string> m;
  if (v && v->t == T::Obj)
    for (auto& kv : v->o) m[kv.first] = kv.second && kv.second->t == T::Str ? kv.second->s : "";
  return m;
}

static VP rule_result_json(const RuleResult& r) {
  auto o = Value::obj();
  o->o["name"] = Value::str(r.name);
  o->o["status"] = Value::str(r.status);
  o->o["message"] = Value::str(r.message);
  o->o["path"] = Value::str(r.path);
  o->o["nondeterministic"] = Value::boolean(r.nondeterministic);
  o->o["message_unpinned"] = Value::boolean(r.message_unpinned);
  auto bp = Value::arr();
  for (auto& b : r.branch_paths) bp->a.push_back(Value::str(b));
  o->o["branch_paths"] = bp;
  auto checks = Value::arr();
  for (auto& c : r.pss_checks) {
    auto co = Value::obj();
    co->o["id"] = Value::str(c.id);
    co->o["reason"] = Value::str(c.r.reason);
    co->o["detail"] = Value::str(c.r.detail);
    checks->a.push_back(co);
  }
  o->o["pss_checks"] = checks;
  return o;
}

extern "C" {

void oracle_free(char* p) { free(p); }

int oracle_wildcard(const char* pattern, const char* text) { return gou::wildcard_match(pattern, text) ? 1 : 0; }

// PolicyException documents (a JSON array, or "" for none) that later validate / validate_matrix runs check
int oracle_set_exceptions(const char* json) {
  try {
    std::vector<VP> ex;
    if (json && *json) {
      VP a = oj::parse(json, false);
      if (a && a->t == T::Arr) ex = a->a;
    }
    set_exceptions(ex);
    return 0;
  } catch (...) {
    return -1;
  }
}

// value decoded with unstructured semantics, pattern with interface{} (float) semantics
int oracle_pattern_validate(const char* value_json, const char* pattern_json) {
  try {
    VP v = oj::parse(value_json, false);
    VP p = oj::parse(pattern_json, true);
    return pattern_validate(v, p) ? 1 : 0;
  } catch (...) {
    return -1;
  }
}

// quantity compare: -1/0/1, or -2 when either side fails to parse
int oracle_quantity_cmp(const char* a, const char* b) {
  gou::Quantity qa, qb;
  if (!gou::parse_quantity(a, qa) || !gou::parse_quantity(b, qb)) return -2;
  return gou::quantity_cmp(qa, qb);
}

// duration: returns 1 and sets *ns on success
int oracle_duration(const char* s, long long* ns) {
  int64_t v;
  if (!gou::parse_duration(s, v)) return 0;
  *ns = v;
  return 1;
}

char* oracle_format_float(double f, int kind) {  // 0:'E' 1:'g' 2:%f 3:json
  switch (kind) {
    case 0: return dup(gou::format_float_E(f));
    case 1: return dup(gou::format_float_g(f));
    case 2: return dup(gou::format_float_f6(f));
    default: return dup(gou::format_float_json(f));
  }
}

char* oracle_match_pattern(const char* resource_json, const char* pattern_json) {
  auto o = Value::obj();
  try {
    VP r = oj::parse(resource_json, false);
    VP p = oj::parse(pattern_json, true);
    EvalFlags fl;
    PatternResult pr = match_pattern(r, p, fl);
    o->o["ok"] = Value::boolean(pr.ok);
    o->o["skip"] = Value::boolean(pr.skip);
    o->o["path"] = Value::str(pr.path);
    o->o["err"] = Value::str(pr.err);
    o->o["nondeterministic"] = Value::boolean(fl.nondeterministic);
  } catch (RefPanic& e) {
    o->o["panic"] = Value::str(e.what);
  } catch (std::exception& e) {
    o->o["exception"] = Value::str(e.what());
  }
  return dup(oj::dump(o));
}

char* oracle_pss(const char* rule_json, const char* pod_json) {
  auto o = Value::obj();
  try {
    VP rule = oj::parse(rule_json, true);
    VP pod = oj::parse(pod_json, false);
    PSSEval ev = pss_evaluate(rule, pod->get("metadata"), pod->get("spec"));
    o->o["ok"] = Value::boolean(ev.ok);
    o->o["error"] = Value::str(ev.error + ev.decode_error);
    o->o["allowed"] = Value::boolean(ev.allowed);
    auto checks = Value::arr();
    for (auto& c : ev.checks) {
      auto co = Value::obj();
      co->o["id"] = Value::str(c.id);
      co->o["reason"] = Value::str(c.r.reason);
      co->o["detail"] = Value::str(c.r.detail);
      checks->a.push_back(co);
    }
    o->o["checks"] = checks;
    o->o["message"] = Value::str(format_checks_print(ev.checks));
  } catch (std::exception& e) {
    o->o["exception"] = Value::str(e.what());
  }
  return dup(oj::dump(o));
}

// policy JSON -> computed rules (autogen) as JSON array
char* oracle_compute_rules(const char* policy_json) {
  try {
    VP p = oj::parse(policy_json, true);
    auto arr = Value::arr();
    for (auto& r : compute_rules(p)) arr->a.push_back(r);
    return dup(oj::dump(arr));
  } catch (std::exception& e) {
    return dup(std::string("{\"exception\":") + "\"" + e.what() + "\"}");
  }
}

int oracle_rule_matches(const char* rule_json, const char* resource_json, const char* nslabels_json) {
  try {
    VP rule = oj::parse(rule_json, true);
    VP res = resource_json && *resource_json ? oj::parse(resource_json, false) : nullptr;
    VP nsl = nslabels_json && *nslabels_json ? oj::parse(nslabels_json, false) : nullptr;
    bool nd = false;
    return matches_resource_description(rule, res, labels_of(nsl), &nd) ? 1 : 0;
  } catch (...) {
    return -1;
  }
}

// engine.Validate for a list of policies against one resource:
// -> [{"policy": name, "namespace_skipped": bool, "rules": [...]}]
char* oracle_validate(const char* policies_json, const char* resource_json, const char* nslabels_json) {
  auto out = Value::arr();
  try {
    VP pols = oj::parse(policies_json, true);
    VP res = oj::parse(resource_json, false);
    VP nsl = nslabels_json && *nslabels_json ? oj::parse(nslabels_json, false) : nullptr;
    auto nsLabels = labels_of(nsl);
    std::vector<VP> list;
    if (pols->t == T::Arr) list = pols->a; else list.push_back(pols);
    for (auto& p : list) {
      PolicyResult pr = validate_policy(p, res, nsLabels);
      auto po = Value::obj();
      po->o["policy"] = Value::str(pr.name);
      po->o["namespace_skipped"] = Value::boolean(pr.namespace_skipped);
      auto rules = Value::arr();
      for (auto& r : pr.rules) rules->a.push_back(rule_result_json(r));
      po->o["rules"] = rules;
      out->a.push_back(po);
    }
  } catch (std::exception& e) {
    auto o = Value::obj();
    o->o["exception"] = Value::str(e.what());
    return dup(oj::dump(o));
  }
  return dup(oj::dump(out));
}

// Batch timing entry for the CPU baseline: evaluate every (policy, resource) pair; resources is a JSON
// array. Returns the number of (resource x computed rule) evaluations performed (matched or not).
long long oracle_validate_batch(const char* policies_json, const char* resources_json, const char* nslabels_json, int nthreads,
                                long long* status_counts /* pass fail skip error other */, double* seconds);
}

#include <atomic>
#include <chrono>
#include <thread>

// Batch entry for the CPU baseline (bench.py cpu_baseline leg). Policies' computed rules are prepared once
// (generous to the CPU: engine.Validate recomputes them per call, validation.go:118) and resources are decoded
// before the clock starts. The timed region is the per-(resource, policy) loop of engine.Validate
// (validation.go:120-183): namespaced-policy filter, match incl. OldResource retry, pattern walk / PSS,
// applyRules: One truncation. Returns resources x compiled validate rules (the bench's unit of work).
long long oracle_validate_batch(const char* policies_json, const char* resources_json, const char* nslabels_json, int nthreads,
                                long long* status_counts, double* seconds) {
  VP pols = oj::parse(policies_json, true);
  VP res = oj::parse(resources_json, false);
  VP nsl = nslabels_json && *nslabels_json ? oj::parse(nslabels_json, false) : nullptr;
  std::map<std::string, std::map<std::string, std::string>> nsLabels;  // namespace -> labels
  if (nsl && nsl->t == T::Obj) for (auto& kv : nsl->o) nsLabels[kv.first] = labels_of(kv.second);
  static const std::map<std::string, std::string> kNoLabels;
  struct Pol { VP policy; std::vector<VP> rules; bool namespaced; std::string ns; bool applyOne; };
  std::vector<Pol> plist;
  std::vector<VP> list;
  if (pols->t == T::Arr) list = pols->a; else list.push_back(pols);
  size_t nrules = 0;
  for (auto& p : list) {
    if (!p || p->t != T::Obj) continue;
    std::string kind = oj::get_str(p, "kind");
    if (kind != "ClusterPolicy" && kind != "Policy") continue;
    Pol x{p, {}, kind == "Policy", nested_string(p, {"metadata", "namespace"}),
          oj::get_str(p->get("spec"), "applyRules") == "One"};
    for (auto& r : compute_rules(p)) {
      VP v = r->get("validate");
      if ((v && v->t == T::Obj && !v->o.empty()) || has_nonempty(r, "verifyImages")) x.rules.push_back(r);
    }
    nrules += x.rules.size();
    plist.push_back(std::move(x));
  }
  std::vector<VP>& rs = res->a;
  if (nthreads < 1) nthreads = 1;
  std::atomic<long long> cnt[5];
  for (auto& c : cnt) c = 0;
  std::atomic<size_t> next{0};
  auto t0 = std::chrono::steady_clock::now();
  auto work = [&]() {
    long long local[5] = {0, 0, 0, 0, 0};
    while (true) {
      size_t i = next.fetch_add(64);
      if (i >= rs.size()) break;
      size_t e = std::min(rs.size(), i + 64);
      for (size_t k = i; k < e; k++) {
        const VP& r = rs[k];
        std::string rns = nested_string(r, {"metadata", "namespace"});
        auto it = nsLabels.find(rns);
        const auto& labels = it == nsLabels.end() ? kNoLabels : it->second;
        for (auto& pol : plist) {
          if (pol.namespaced && (rns != pol.ns || rns.empty())) { local[4] += pol.rules.size(); continue; }
          int applied = 0;
          size_t done = 0;
          for (auto& rule : pol.rules) {
            done++;
            bool nd = false;
            bool m = matches_resource_description(rule, r, labels, &nd);
            if (!m) m = matches_resource_description(rule, nullptr, labels, &nd);
            if (!m) { local[4]++; continue; }
            RuleResult rr = validate_rule(rule, r);
            if (rr.status == "pass") local[0]++, applied++;
            else if (rr.status == "fail") local[1]++, applied++;
            else if (rr.status == "skip") local[2]++;
            else if (rr.status == "error") local[3]++;
            else local[4]++;
            if (pol.applyOne && applied > 0) break;
          }
          local[4] += pol.rules.size() - done;
        }
      }
    }
    for (int j = 0; j < 5; j++) cnt[j] += local[j];
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; t++) th.emplace_back(work);
  for (auto& t : th) t.join();
  auto t1 = std::chrono::steady_clock::now();
  if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
  if (status_counts) for (int j = 0; j < 5; j++) status_counts[j] = cnt[j];
  return (long long)rs.size() * (long long)nrules;
}

// Per-pair verdict matrix for parity at sizes where one oracle_validate call per resource is too slow (C4:
// thousands of policies). Same semantics as oracle_validate (validate_policy, autogen computed once per policy
// instead of per call). out[rule * nres + res] for the policies' validate rules in order: 0 not matched / no
// response, 1 pass, 2 fail, 3 skip, 4 error, 5 panic, 6 unsupported (CPU fallback), 7 nondeterministic.
// Returns the rule names as a JSON array [[policy, rule], ...] (free with oracle_free), or null on error.
extern "C" char* oracle_validate_matrix_t(const char* policies_json, const char* resources_json,
                                          const char* nslabels_json, int nthreads, unsigned char* out, long long out_len,
                                          double* seconds);
extern "C" char* oracle_validate_matrix(const char* policies_json, const char* resources_json, const char* nslabels_json,
                                        int nthreads, unsigned char* out, long long out_len) {
  return oracle_validate_matrix_t(policies_json, resources_json, nslabels_json, nthreads, out, out_len, nullptr);
}

// Same, timing the per-(resource, policy) loop only (policies compiled and resources decoded before the clock, as in
// oracle_validate_batch): the bench's CPU baseline, whose verdicts are then compared with the device's.
extern "C" char* oracle_validate_matrix_x(const char* policies_json, const char* resources_json,
                                          const char* nslabels_json, int nthreads, unsigned char* out, long long out_len,
                                          double* seconds, unsigned text_mask, char** texts, long long* texts_len);
extern "C" char* oracle_validate_matrix_t(const char* policies_json, const char* resources_json,
                                          const char* nslabels_json, int nthreads, unsigned char* out, long long out_len,
                                          double* seconds) {
  return oracle_validate_matrix_x(policies_json, resources_json, nslabels_json, nthreads, out, out_len, seconds, 0,
                                  nullptr, nullptr);
}

// Same, also returning the texts of the pairs whose matrix code c has bit c set in text_mask: a malloc'ed buffer
// (*texts, *texts_len bytes; free with oracle_free) of records in (rule, resource) order
//   u64 rule * nres + res | u32 flags (bit 0 message_unpinned) | u32 path length | u32 message length | path | message
// where path = RuleResponse's failing PatternError.Path (single patterns) and message = RuleResponse.Message: the
// parity tests compare the device's failing paths and messages pair by pair at scale.
extern "C" char* oracle_validate_matrix_x(const char* policies_json, const char* resources_json,
                                          const char* nslabels_json, int nthreads, unsigned char* out, long long out_len,
                                          double* seconds, unsigned text_mask, char** texts, long long* texts_len) {
  try {
    VP pols = oj::parse(policies_json, true);
    VP res = oj::parse(resources_json, false);
    VP nsl = nslabels_json && *nslabels_json ? oj::parse(nslabels_json, false) : nullptr;
    std::map<std::string, std::map<std::string, std::string>> nsLabels;
    if (nsl && nsl->t == T::Obj) for (auto& kv : nsl->o) nsLabels[kv.first] = labels_of(kv.second);
    static const std::map<std::string, std::string> kNoLabels;
    std::vector<VP> list;
    if (pols->t == T::Arr) list = pols->a; else list.push_back(pols);
    struct Pol { VP policy; std::vector<VP> rules; size_t first; std::map<std::string, size_t> idx; };
    std::vector<Pol> plist;
    auto names = Value::arr();
    size_t nrules = 0;
    for (auto& p : list) {
      if (!p || p->t != T::Obj) continue;
      std::string kind = oj::get_str(p, "kind");
      if (kind != "ClusterPolicy" && kind != "Policy") continue;
      Pol x{p, compute_rules(p), nrules, {}};
      std::string pname = nested_string(p, {"metadata", "name"});
      for (auto& r : x.rules) {
        VP v = r->get("validate");
        if (!((v && v->t == T::Obj && !v->o.empty()) || has_nonempty(r, "verifyImages"))) continue;
        std::string rn = oj::get_str(r, "name");
        x.idx[rn] = nrules++;
        auto pr = Value::arr();
        pr->a.push_back(Value::str(pname));
        pr->a.push_back(Value::str(rn));
        names->a.push_back(pr);
      }
      plist.push_back(std::move(x));
    }
    if (res->t != T::Arr) return nullptr;
    size_t n = res->a.size();
    if ((long long)(nrules * n) > out_len) return nullptr;
    std::fill(out, out + nrules * n, (unsigned char)0);
    std::atomic<size_t> next{0};
    struct Text { uint64_t at; uint32_t flags; std::string path, msg; };
    std::mutex tmu;
    std::vector<Text> all_texts;
    const bool want_texts = texts && texts_len && text_mask;
    auto t0 = std::chrono::steady_clock::now();
    auto work = [&]() {
      std::vector<Text> mine;
      while (true) {
        size_t i = next.fetch_add(16);
        if (i >= n) break;
        for (size_t k = i; k < std::min(n, i + 16); k++) {
          const VP& r = res->a[k];
          auto it = nsLabels.find(nested_string(r, {"metadata", "namespace"}));
          const auto& labels = it == nsLabels.end() ? kNoLabels : it->second;
          for (auto& pol : plist) {
            PolicyResult pr = validate_policy_rules(pol.policy, pol.rules, r, labels);
            for (auto& rr : pr.rules) {
              auto f = pol.idx.find(rr.name);
              if (f == pol.idx.end()) continue;
              unsigned char c = rr.status == "pass" ? 1 : rr.status == "fail" ? 2 : rr.status == "skip" ? 3
                              : rr.status == "error" ? 4 : rr.status == "panic" ? 5 : 6;
              if (rr.nondeterministic && c != 6) c = 7;
              out[f->second * n + k] = c;
              if (want_texts && ((text_mask >> c) & 1u))
                mine.push_back(Text{(uint64_t)f->second * n + k, rr.message_unpinned ? 1u : 0u, rr.path, rr.message});
            }
          }
        }
      }
      if (want_texts) {
        std::lock_guard<std::mutex> g(tmu);
        for (auto& t : mine) all_texts.push_back(std::move(t));
      }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < std::max(1, nthreads); t++) th.emplace_back(work);
    for (auto& t : th) t.join();
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (want_texts) {
      std::sort(all_texts.begin(), all_texts.end(), [](const Text& a, const Text& b) { return a.at < b.at; });
      size_t total = 0;
      for (auto& t : all_texts) total += 20 + t.path.size() + t.msg.size();
      char* buf = (char*)malloc(std::max<size_t>(1, total));
      size_t at = 0;
      for (auto& t : all_texts) {
        uint32_t pl = (uint32_t)t.path.size(), ml = (uint32_t)t.msg.size();
        memcpy(buf + at, &t.at, 8);
        memcpy(buf + at + 8, &t.flags, 4);
        memcpy(buf + at + 12, &pl, 4);
        memcpy(buf + at + 16, &ml, 4);
        memcpy(buf + at + 20, t.path.data(), pl);
        memcpy(buf + at + 20 + pl, t.msg.data(), ml);
        at += 20 + pl + ml;
      }
      *texts = buf;
      *texts_len = (long long)total;
    }
    return dup(oj::dump(names));
  } catch (std::exception&) {
    return nullptr;
  }
}

// One condition as pkg/engine/variables/evaluate_test.go TestEvaluate drives it: key/value are the raw JSON of
// Condition.RawKey / RawValue (decoded by GetKey/GetValue). Returns 1 true, 0 false, 2 reference panic, -1 bad input.
extern "C" int oracle_condition(const char* key_json, const char* op, const char* value_json) {
  try {
    VP k = key_json && *key_json ? oj::parse(key_json, false) : nullptr;
    VP v = value_json && *value_json ? oj::parse(value_json, false) : nullptr;
    if (k && k->t == T::Null) k = nullptr;
    if (v && v->t == T::Null) v = nullptr;
    return evaluate_condition(k, op, v) ? 1 : 0;
  } catch (RefPanic&) {
    return 2;
  } catch (...) {
    return -1;
  }
}

extern "C" {
int oracle_leaf(const char* fn, const char* value_json, int value_float, const char* pattern_json, const char* op) {
  try {
    VP v = oj::parse(value_json, value_float != 0);
    VP p = oj::parse(pattern_json, true);
    return leaf_fn(fn, v, p, op) ? 1 : 0;
  } catch (...) {
    return -1;
  }
}

char* oracle_validate_entry(const char* entry, const char* resource_json, const char* pattern_json, int resource_float) {
  auto o = Value::obj();
  try {
    VP r = oj::parse(resource_json, resource_float != 0);
    VP p = oj::parse(pattern_json, true);
    EvalFlags fl;
    RawWalk w = validate_entry(entry, r, p, fl);
    o->o["path"] = Value::str(w.path);
    o->o["err"] = Value::boolean(w.err);
    o->o["msg"] = Value::str(w.msg);
  } catch (RefPanic& e) {
    o->o["panic"] = Value::str(e.what);
  } catch (std::exception& e) {
    o->o["exception"] = Value::str(e.what());
  }
  return dup(oj::dump(o));
}

char* oracle_anchor_probe(const char* op, const char* a, const char* b) {
  try {
    return dup(anchor_probe(op, a, b));
  } catch (std::exception& e) {
    return dup(std::string("{\"exception\":") + oj::dump(Value::str(e.what())) + "}");
  }
}

// $() reference helpers (orefs.cpp): op "subst" (a = document JSON) -> {"ok","nd","err","doc"}; op "abs"
// (a = reference path, b = absolute path) -> formAbsolutePath
char* oracle_refs(const char* op, const char* a, const char* b) {
  auto o = Value::obj();
  try {
    if (std::string(op) == "abs") return dup(oj::dump(Value::str(form_absolute_path(a, b))));
    RefResult r = substitute_references(oj::parse(a, true));
    o->o["ok"] = Value::boolean(r.ok);
    o->o["nd"] = Value::boolean(r.nd);
    o->o["err"] = Value::str(r.err);
    o->o["doc"] = r.doc;
  } catch (std::exception& e) {
    o->o["exception"] = Value::str(e.what());
  }
  return dup(oj::dump(o));
}
}
