// C-ABI (include/kyvgpu.h). No exception crosses this boundary.
#include <algorithm>
#include <array>
#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <sched.h>
#include <cstring>

#include "../../include/kyvgpu.h"
#include "kyv_host.h"

namespace kyv {
void eval_gpu(const Ruleset& rs, const Batch& b, int device, int iters, Results* out, double* kernel_ms_avg, bool copy_back,
              int jit_mode, bool account, bool serial);
void eval_cpu(const Ruleset& rs, const Batch& b, int threads, Results* out, bool account);
void free_device_images(Ruleset& rs, Batch* b);
std::string fallback_why(const Ruleset& rs, const Batch& b, uint32_t res, uint32_t rule);
bool pattern_error_text(const Ruleset& rs, const Batch& b, uint32_t res, uint32_t rule, uint32_t root, uint8_t* status,
                        std::string* path, std::string* text);
int64_t export_status(const Batch& b, int device, uint8_t* dst, size_t cap, void* stream);
int64_t export_failures(const Batch& b, int device, int64_t off, int64_t* dst, size_t cap_rows, void* stream);
int64_t copy_status(const Batch& b, int device, size_t res0, size_t n, uint8_t* host_dst, size_t cap);
int64_t export_report_rows(const Batch& b, int device, uint32_t* rows, uint32_t* wide, uint32_t* nwide_dev,
                           size_t cap_rows, size_t cap_wide, void* stream);
const unsigned long long* device_counts(const Batch& b, int device, size_t* nrules, size_t* nres);
bool pss_checks_render(const Ruleset& rs, const Batch& b, uint32_t pos, uint32_t rule, uint32_t mask,
                       std::vector<std::array<std::string, 3>>* out);
double calibrate_fetch(int device, size_t bytes, int mode);
}  // namespace kyv

using namespace kyv;

struct kyv_ruleset { Ruleset* rs; };
struct kyv_batch { Batch* b; };
struct kyv_results {
  Results r;                  // verdicts in the batch's kind-major order
  // input index -> kind-major position, shared with the batch (a per-evaluation copy of 4 B per resource cost
  // ~0.4 ms of host time per call at 1.25 M resources)
  std::shared_ptr<const std::vector<uint32_t>> inv;
  std::multimap<uint64_t, uint32_t> recidx;  // (rule<<32|res) -> record
  std::atomic<bool> indexed{false};
  std::mutex mu;
};

static thread_local std::string g_err;
static int fail(int code, const std::string& m) { g_err = m; return code; }

// worker threads when the caller passes 0: KYV_THREADS, else the CPUs this process may use -- its affinity mask
// bounded by a cgroup v2 CPU quota (cpu.max), as on shared GPU hosts where the machine's CPU count is many times
// the job's share -- divided among the node's ranks (LOCAL_WORLD_SIZE, set by torch.distributed.run: one process
// per GPU shares the same mask) and capped at 64
static int hw_threads(int t) {
  if (t > 0) return t;
  static const int n = []() {
    if (const char* e = getenv("KYV_THREADS")) {
      int v = atoi(e);
      if (v > 0) return v;
    }
    int c = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) c = CPU_COUNT(&set);
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long period = 0;
      if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
        long quota = atol(q);
        if (quota > 0) c = std::min<long>(c, (quota + period - 1) / period);
      }
      fclose(f);
    }
    if (const char* e = getenv("LOCAL_WORLD_SIZE")) {
      const int lw = atoi(e);
      if (lw > 1) c /= lw;
    }
    return std::max(1, std::min(c, 64));
  }();
  return n;
}

extern "C" {

const char* kyv_last_error(void) { return g_err.c_str(); }
const char* kyv_version(void) { return "kyvgpu 0.1 (gfx950)"; }

int kyv_ruleset_compile(const char* json, size_t len, const kyv_compile_opts* opts, kyv_ruleset** out) {
  return kyv_ruleset_compile_ex(json, len, nullptr, 0, opts, out);
}

int kyv_ruleset_compile_ex(const char* json, size_t len, const char* exceptions_json, size_t ex_len,
                           const kyv_compile_opts* opts, kyv_ruleset** out) {
  if (!json || !out) return fail(KYV_EINVAL, "null argument");
  if (opts && opts->abi_version != KYV_ABI_VERSION) return fail(KYV_EINVAL, "ABI version mismatch");
  try {
    std::string err;
    Ruleset* rs = compile_ruleset(json, len, &err, exceptions_json, exceptions_json ? ex_len : 0,
                                  opts && (opts->flags & KYV_COMPILE_BACKGROUND));
    if (!rs) return fail(KYV_EPARSE, err);
    *out = new kyv_ruleset{rs};
    return KYV_OK;
  } catch (std::exception& e) {
    return fail(KYV_EINTERNAL, e.what());
  }
}

void kyv_ruleset_free(kyv_ruleset* rs) {
  if (!rs) return;
  try { free_device_images(*rs->rs, nullptr); } catch (...) {}
  delete rs->rs;
  delete rs;
}

uint32_t kyv_ruleset_num_rules(const kyv_ruleset* rs) { return rs ? (uint32_t)rs->rs->rules.size() : 0; }
uint32_t kyv_ruleset_num_policies(const kyv_ruleset* rs) { return rs ? (uint32_t)rs->rs->policies.size() : 0; }

int kyv_ruleset_rule_info(const kyv_ruleset* rs, uint32_t k, kyv_rule_info* out) {
  if (!rs || !out || k >= rs->rs->rules.size()) return fail(KYV_ERANGE, "rule index out of range");
  const RuleMeta& m = rs->rs->meta[k];
  out->name = m.name.c_str();
  out->policy = m.policy;
  out->kind = m.kind;
  out->reason = m.reason.c_str();
  return KYV_OK;
}

int64_t kyv_ruleset_rule_kinds(const kyv_ruleset* rs, uint32_t k, char* buf, size_t cap, int32_t* has_validate) {
  if (!rs || k >= rs->rs->rules.size()) return fail(KYV_ERANGE, "rule index out of range"), -1;
  const RuleMeta& m = rs->rs->meta[k];
  std::string s;
  for (size_t i = 0; i < m.kinds.size(); i++) s += (i ? "\n" : "") + m.kinds[i];
  if (has_validate) *has_validate = m.has_validate ? 1 : 0;
  if (buf && cap) { size_t n = std::min(cap - 1, s.size()); memcpy(buf, s.data(), n); buf[n] = 0; }
  return (int64_t)s.size();
}

uint32_t kyv_ruleset_rule_flags(const kyv_ruleset* rs, uint32_t k) {
  if (!rs || k >= rs->rs->rules.size()) return 0;
  return (rs->rs->rules[k].flags & RD_USES_OPERATION) ? KYV_RULE_USES_OPERATION : 0u;
}

int64_t kyv_ruleset_jit_source(const kyv_ruleset* rs, char* buf, size_t cap, uint32_t* nrules_jit) {
  if (!rs) return fail(KYV_EINVAL, "null argument"), -1;
  try {
    std::vector<uint8_t> jr;
    std::vector<uint8_t> jc;
    std::string src = jit_source(*rs->rs, &jr, &jc);
    if (nrules_jit) { *nrules_jit = 0; for (size_t k = 0; k < jr.size(); k++) *nrules_jit += (jr[k] || jc[k]) ? 1 : 0; }
    if (buf && cap) { size_t n = std::min(cap - 1, src.size()); memcpy(buf, src.data(), n); buf[n] = 0; }
    return (int64_t)src.size();
  } catch (std::exception& e) {
    fail(KYV_EINTERNAL, e.what());
    return -1;
  }
}

int kyv_ruleset_jit_compile(const kyv_ruleset* rs, double* seconds, size_t* code_bytes) {
  if (!rs) return fail(KYV_EINVAL, "null argument");
  try {
    std::vector<uint8_t> jr;
    std::vector<uint8_t> jc;
    std::vector<char> code = jit_compile(jit_source(*rs->rs, &jr, &jc), seconds);
    if (code_bytes) *code_bytes = code.size();
    return KYV_OK;
  } catch (std::exception& e) {
    return fail(KYV_EINTERNAL, e.what());
  }
}

int kyv_ruleset_jit_compile_ex(const kyv_ruleset* rs, uint32_t flags, double* seconds, size_t* code_bytes) {
  if (!rs) return fail(KYV_EINVAL, "null argument");
  try {
    std::vector<uint8_t> jr;
    std::vector<uint8_t> jc;
    std::vector<char> code = jit_compile(jit_source(*rs->rs, &jr, &jc), seconds, (flags & KYV_JIT_ACCOUNTING) != 0);
    if (code_bytes) *code_bytes = code.size();
    return KYV_OK;
  } catch (std::exception& e) {
    return fail(KYV_EINTERNAL, e.what());
  }
}

int kyv_ruleset_policy_info(const kyv_ruleset* rs, uint32_t p, kyv_policy_info* out) {
  if (!rs || !out || p >= rs->rs->policies.size()) return fail(KYV_ERANGE, "policy index out of range");
  const PolicyMeta& m = rs->rs->policies[p];
  out->name = m.name.c_str();
  out->namespace_ = m.kind == "Policy" ? m.ns.c_str() : "";
  out->first_rule = m.first_rule;
  out->nrules = m.nrules;
  out->apply_one = m.apply_one;
  out->scored_false = m.scored_false;
  return KYV_OK;
}

int kyv_batch_build(const kyv_ruleset* rs, const char* json, size_t len, const char* nsl, size_t nsl_len,
                    const kyv_batch_opts* opts, kyv_batch** out) {
  if (!rs || !json || !out) return fail(KYV_EINVAL, "null argument");
  if (opts && opts->abi_version != KYV_ABI_VERSION) return fail(KYV_EINVAL, "ABI version mismatch");
  try {
    std::string err;
    Batch* b = build_batch(rs->rs, json, len, nsl, nsl_len, hw_threads(opts ? opts->threads : 0), &err);
    if (!b) return fail(KYV_EPARSE, err);
    *out = new kyv_batch{b};
    return KYV_OK;
  } catch (std::exception& e) {
    return fail(KYV_EINTERNAL, e.what());
  }
}

void kyv_batch_free(kyv_batch* b) {
  if (!b) return;
  try { free_device_images(*const_cast<Ruleset*>(b->b->rs), b->b); } catch (...) {}
  delete b->b;
  delete b;
}

uint32_t kyv_batch_num_resources(const kyv_batch* b) { return b ? (uint32_t)b->b->hdr.size() : 0; }

int kyv_batch_stats_get(const kyv_batch* b, kyv_batch_stats* out) {
  if (!b || !out) return fail(KYV_EINVAL, "null argument");
  const Batch& x = *b->b;
  out->resources = x.hdr.size();
  out->nodes = x.nodes.size();
  out->strings = x.dict.strs.size();
  out->heap_bytes = x.heap.size();
  out->device_bytes = x.nodes.size() * sizeof(Node) + x.hdr.size() * sizeof(ResHeader) + x.heap.size() +
                      x.dict.strs.size() * (4 + 4 + 4 + 8 + 16 + 8) + x.faux.size() * sizeof(FloatAux) +
                      x.colv.size() * sizeof(uint64_t) + x.col_off.size() * 4 + x.gate.size() * 4 +
                      (x.str_upper.size() + x.str_rx.size()) * 4;
  return KYV_OK;
}

int kyv_eval(const kyv_ruleset* rs, const kyv_batch* b, const kyv_eval_opts* opts, kyv_results** out) {
  if (!rs || !b || !out) return fail(KYV_EINVAL, "null argument");
  if (b->b->rs != rs->rs) return fail(KYV_EINVAL, "batch was built for a different ruleset");
  if (opts && opts->abi_version != KYV_ABI_VERSION) return fail(KYV_EINVAL, "ABI version mismatch");
  int backend = opts ? opts->backend : KYV_BACKEND_GPU;
  try {
    auto* res = new kyv_results();
    if (backend == KYV_BACKEND_CPU) {
      eval_cpu(*rs->rs, *b->b, hw_threads(opts ? opts->threads : 0), &res->r, opts && (opts->flags & KYV_EVAL_ACCOUNT_BYTES));
    } else {
      int dev = opts ? opts->device : 0;
      int iters = opts && opts->iterations > 0 ? opts->iterations : 1;
      bool copy = !(opts && (opts->flags & KYV_EVAL_NO_COPYBACK));
      double ms = 0;
      int jm = !opts ? JIT_AUTO : (opts->flags & KYV_EVAL_JIT_OFF) ? JIT_OFF : (opts->flags & KYV_EVAL_JIT_ON) ? JIT_ON : JIT_AUTO;
      eval_gpu(*rs->rs, *b->b, dev, iters, &res->r, &ms, copy, jm, opts && (opts->flags & KYV_EVAL_ACCOUNT_BYTES),
               opts && (opts->flags & KYV_EVAL_SERIAL));
    }
    {
      static std::mutex inv_mu;
      std::lock_guard<std::mutex> g(inv_mu);
      if (!b->b->inv_shared) b->b->inv_shared = std::make_shared<const std::vector<uint32_t>>(b->b->inv);
      res->inv = b->b->inv_shared;
    }
    *out = res;
    return KYV_OK;
  } catch (std::exception& e) {
    return fail(backend == KYV_BACKEND_GPU ? KYV_EDEVICE : KYV_EINTERNAL, e.what());
  }
}

void kyv_results_free(kyv_results* r) { delete r; }

int kyv_results_jit(const kyv_results* r) { return r ? r->r.jit_used : 0; }

int kyv_results_status(const kyv_results* r, uint8_t* out, size_t cap) {
  if (!r || !out) return fail(KYV_EINVAL, "null argument");
  if (cap < r->r.status.size()) return fail(KYV_ERANGE, "buffer too small (or verdicts kept on device)");
  const size_t nres = r->r.nres, nrules = r->r.nrules;
  const uint32_t* inv = r->inv->data();
  // kind-major -> input order: a gather of the whole matrix (C3 10 M: 890 MB), split over the worker threads in
  // blocks of resources so each thread streams its slice of every rule row
  const size_t T = std::max<size_t>(1, std::min<size_t>((size_t)hw_threads(0), (nres * nrules) >> 20));
  auto part = [&](size_t t) {
    const size_t i0 = nres * t / T, i1 = nres * (t + 1) / T;
    for (size_t k = 0; k < nrules; k++) {
      const uint8_t* src = r->r.status.data() + k * nres;
      uint8_t* dst = out + k * nres;
      for (size_t i = i0; i < i1; i++) dst[i] = src[inv[i]];
    }
  };
  if (T == 1) {
    part(0);
  } else {
    std::vector<std::thread> th;
    for (size_t t = 1; t < T; t++) th.emplace_back(part, t);
    part(0);
    for (auto& x : th) x.join();
  }
  return KYV_OK;
}

int64_t kyv_batch_export_status(const kyv_batch* b, int device, uint8_t* dst, size_t cap, void* stream) {
  if (!b) return fail(KYV_EINVAL, "null argument"), -1;
  try {
    return export_status(*b->b, device, dst, cap, stream);
  } catch (std::exception& e) {
    return fail(KYV_EINVAL, e.what()), -1;
  }
}

int64_t kyv_batch_copy_status(const kyv_batch* b, int device, uint64_t res0, uint64_t nres, uint8_t* dst, size_t cap) {
  if (!b) return fail(KYV_EINVAL, "null argument"), -1;
  try {
    return copy_status(*b->b, device, (size_t)res0, (size_t)nres, dst, cap);
  } catch (std::exception& e) {
    return fail(KYV_EINVAL, e.what()), -1;
  }
}

int64_t kyv_batch_export_failures(const kyv_batch* b, int device, int64_t res_offset, int64_t* dst, size_t cap_rows,
                                  void* stream) {
  if (!b) return fail(KYV_EINVAL, "null argument"), -1;
  try {
    return export_failures(*b->b, device, res_offset, dst, cap_rows, stream);
  } catch (std::exception& e) {
    return fail(KYV_EINVAL, e.what()), -1;
  }
}

int64_t kyv_results_count(const kyv_results* r, int s) {
  if (!r || s < 0 || s >= NSTATUS) return -1;
  return r->r.counts[s];
}

int kyv_results_rule_counts(const kyv_results* r, int64_t* out, size_t cap) {
  if (!r || !out) return fail(KYV_EINVAL, "null argument");
  if (cap < r->r.rule_counts.size()) return fail(KYV_ERANGE, "buffer too small");
  std::copy(r->r.rule_counts.begin(), r->r.rule_counts.end(), out);
  return KYV_OK;
}

double kyv_results_kernel_ms(const kyv_results* r) { return r ? r->r.kernel_ms : 0; }
double kyv_calibrate_fetch(int device, uint64_t bytes, int mode) {
  try {
    return calibrate_fetch(device, (size_t)bytes, mode);
  } catch (std::exception& e) {
    fail(KYV_EDEVICE, e.what());
    return -1;
  }
}
double kyv_results_batch_ms(const kyv_results* r, int what) {
  if (!r) return 0;
  return what == 0 ? r->r.h2d_ms : what == 1 ? r->r.gmask_ms : 0;
}

int kyv_results_phase_ms(const kyv_results* r, double* out, size_t cap) {
  if (!r || !out) return fail(KYV_EINVAL, "null argument"), -1;
  for (size_t q = 0; q < 5 && q < cap; q++) out[q] = r->r.phase_ms[q];
  return 5;
}

uint64_t kyv_results_alg_bytes(const kyv_results* r) { return r ? r->r.alg_bytes : 0; }

int kyv_results_alg_bytes_class(const kyv_results* r, uint64_t* out, size_t cap) {
  if (!r || !out) return fail(KYV_EINVAL, "null argument");
  for (size_t q = 0; q < 3 && q < cap; q++) out[q] = r->r.alg_bytes_class[q];
  return 3;
}

int kyv_results_alg_bytes_phase(const kyv_results* r, uint64_t* out, size_t cap) {
  if (!r || !out) return fail(KYV_EINVAL, "null argument"), -1;
  for (size_t q = 0; q < 5 && q < cap; q++) out[q] = r->r.alg_bytes_phase[q];
  return 5;
}

static void ensure_index(kyv_results* r) {
  if (r->indexed.load(std::memory_order_acquire)) return;
  std::lock_guard<std::mutex> g(r->mu);
  if (r->indexed.load(std::memory_order_relaxed)) return;
  for (uint32_t i = 0; i < r->r.fails.size(); i++) {
    const FailRec& f = r->r.fails[i];
    r->recidx.emplace(((uint64_t)f.rule << 32) | f.res, i);
  }
  r->indexed.store(true, std::memory_order_release);
}

static int64_t put(const std::string& s, char* buf, size_t cap) {
  if (buf && cap) {
    size_t n = std::min(cap - 1, s.size());
    memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return (int64_t)s.size();
}

// request.object path on the host copy of a resource (kyverno/go-jmespath semantics, kyv_cond.h cv_operand):
// returns false with *miss on a key missing from a map; *node = NONE for null
static bool host_resolve(const Batch& b, uint32_t res, const std::vector<uint32_t>& segs, uint32_t* node, uint32_t* miss) {
  const Node* R = b.nodes.data() + b.hdr[res].root;
  uint32_t cur = 0;
  for (uint32_t s = 0; s < segs.size(); s++) {
    const Node& n = R[cur];
    if (node_type(n) != N_MAP) { *node = NONE; return true; }
    uint32_t hit = NONE;
    for (uint32_t j = n.a; j < n.a + n.b; j++) if (node_key(R[j]) == segs[s]) { hit = j; break; }
    if (hit == NONE) { *miss = s; return false; }
    cur = hit;
  }
  *node = node_type(R[cur]) == N_NULL ? NONE : cur;
  return true;
}

// vars.go:395-399 error text of the first unresolved reference of a condition program
static bool cond_error_text(const Ruleset& rs, const Batch& b, uint32_t res, uint32_t prog, std::string* out) {
  const CondProg& p = rs.cprogs[prog];
  uint32_t nany = p.nany == NONE ? 0 : p.nany;
  for (int blk = 0; blk < 2; blk++) {
    uint32_t c0 = blk ? p.all0 : p.any0, n = blk ? p.nall : nany;
    for (uint32_t i = 0; i < n; i++) {
      const Cond& c = rs.conds[c0 + i];
      const CondText& ct = rs.cond_text[c0 + i];
      for (int side = 0; side < 2; side++) {
        const CondOperand& o = side ? c.value : c.key;
        if (o.kind != OK_PATH) continue;
        std::vector<uint32_t> segs(rs.pool.begin() + o.a, rs.pool.begin() + o.a + o.nseg);
        uint32_t node, miss;
        if (!host_resolve(b, res, segs, &node, &miss)) {
          *out = "failed to resolve " + ct.var[side] + " at path " + ct.path[side] +
                 ": JMESPath query failed: Unknown key \"" + ct.segs[side][miss] + "\" in path";
          return true;
        }
      }
    }
  }
  return false;
}

// SubstituteAll of a rule message's request.object references (vars.go; validation.go:469 getDenyMessage, :731
// buildErrorMessage) for the resource at kind-major position `res`: SM_OK with the text in *o; SM_MISSING when a
// reference does not resolve (a substitution error); SM_NOT_STRING when the whole message is one reference to a
// non-string; SM_UNRENDERABLE when the text needs the reference engine (a map / array value, nested variables)
enum SubstMsg { SM_OK = 0, SM_MISSING = 1, SM_NOT_STRING = 2, SM_UNRENDERABLE = 3 };
static int subst_message(const RuleMeta& m, const Batch& b, uint32_t res, std::string* o) {
  if (m.msg_parts.empty()) return *o = m.message, SM_OK;
  const Node* R = b.nodes.data() + b.hdr[res].root;
  std::string out;
  for (auto& part : m.msg_parts) {
    if (!part.var) { out += part.text; continue; }
    uint32_t node, miss;
    if (!host_resolve(b, res, part.segs, &node, &miss)) return SM_MISSING;
    std::string sub;
    uint32_t t = node == NONE ? N_NULL : node_type(R[node]);
    if (m.msg_whole_var) {
      if (t != N_STR) return SM_NOT_STRING;
      return *o = b.dict.strs[R[node].a], SM_OK;
    }
    switch (t) {
      case N_STR: sub = b.dict.strs[R[node].a]; break;
      case N_NULL: sub = "null"; break;
      case N_TRUE: sub = "true"; break;
      case N_FALSE: sub = "false"; break;
      case N_INT: sub = pj::go_fmt_json((double)(int64_t)(((uint64_t)R[node].b << 32) | R[node].a)); break;
      case N_FLOAT: {
        uint64_t bits = ((uint64_t)R[node].b << 32) | R[node].a;
        double f;
        memcpy(&f, &bits, 8);
        sub = pj::go_fmt_json(f);
        break;
      }
      default: return SM_UNRENDERABLE;  // json.Marshal of a map / array
    }
    if (sub.find("{{") != std::string::npos) return SM_UNRENDERABLE;  // nested variables are substituted again
    out += sub;
  }
  return *o = out, SM_OK;
}

// getDenyMessage (validation.go:461-479): a substitution error leaves the message as written
static bool deny_message(const RuleMeta& m, const Batch& b, uint32_t res, std::string* o) {
  if (m.message.empty()) return *o = "validation error: rule " + m.name + " failed", true;
  switch (subst_message(m, b, res, o)) {
    case SM_OK: return true;
    case SM_MISSING: return *o = m.message, true;
    case SM_NOT_STRING: return *o = "the produced message didn't resolve to a string, check your policy definition.", true;
    default: return false;
  }
}

// buildErrorMessage's message part (validation.go:731-741): the substituted message with a trailing '.'; false when
// the text needs the reference engine (a substitution error embeds the Go error string, a non-string whole-message
// reference panics on the type assertion)
static bool error_message_head(const RuleMeta& m, const Batch& b, uint32_t res, std::string* o) {
  if (subst_message(m, b, res, o) != SM_OK) return false;
  if (o->empty() || o->back() != '.') *o += ".";
  return true;
}

static uint32_t pss_mask_at(const kyv_results* r, const Ruleset& rs, uint32_t pos, uint32_t rule) {
  uint32_t slot = 0;
  for (uint32_t k = 0; k < rule; k++) if (rs.rules[k].kind == RK_PSS) slot++;
  size_t i = (size_t)slot * r->r.nres + pos;
  return i < r->r.pss_fails.size() ? r->r.pss_fails[i] : 0;
}

static std::string json_str(const std::string& s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
    else if (c < 0x20) { char x[8]; snprintf(x, sizeof x, "\\u%04x", c); o += x; }
    else o += (char)c;
  }
  return o + "\"";
}

// Messages built from the pattern walk's error texts (pattern_error_text, kyv_engine.hip): skip (PatternError.Error()),
// error (buildErrorMessage(err, ""): "execution error: <err>") and anyPattern results with a path-less failure
// ("rule <name>[<i>] failed: <err>") -- validation.go:618-702,722-758. The host walk must reach the device's status.
static bool walk_text_message(const Ruleset& rs, const Batch& b, uint32_t res, uint32_t rule, uint8_t st, std::string* o) {
  const RuleMeta& m = rs.meta[rule];
  const RuleDesc& d = rs.rules[rule];
  if (d.kind == RK_PATTERN) {
    uint8_t s2;
    std::string path, text;
    if (!pattern_error_text(rs, b, res, rule, d.root, &s2, &path, &text) || s2 != st) return false;
    if (st == ST_SKIP) return *o = text, true;
    if (st != ST_ERROR) return false;
    if (m.message.empty()) return *o = "validation error: rule " + m.name + " execution error: " + text, true;
    if (m.message_vars) return false;
    std::string mm;
    if (!error_message_head(m, b, res, &mm)) return false;
    return *o = "validation error: " + mm + " rule " + m.name + " execution error: " + text, true;
  }
  if (d.kind != RK_ANYPATTERN) return false;
  std::vector<std::string> failed, skipped;
  for (uint32_t a = 0; a < d.nalts; a++) {
    uint8_t s2;
    std::string path, text;
    if (!pattern_error_text(rs, b, res, rule, rs.pool[d.root + a], &s2, &path, &text)) return false;
    const std::string nm = "rule " + m.name + "[" + std::to_string(a) + "]";
    if (s2 == ST_PASS) return false;  // the device decided the pair otherwise
    if (s2 == ST_SKIP) skipped.push_back(nm + " skipped: " + text);
    else if (path.empty()) failed.push_back(nm + " failed: " + text);
    else failed.push_back(nm + " failed at path " + path);
  }
  auto join = [](const std::vector<std::string>& v) {
    std::string j;
    for (size_t i = 0; i < v.size(); i++) j += (i ? " " : "") + v[i];
    return j;
  };
  if (failed.empty()) {
    if (st != ST_SKIP || skipped.empty()) return false;
    return *o = join(skipped), true;
  }
  if (st != ST_FAIL) return false;
  if (m.message_vars) return false;
  const std::string e = join(failed);
  if (m.message.empty()) return *o = "validation error: " + e, true;
  if (m.message.back() == '.') return *o = "validation error: " + m.message + " " + e, true;
  return *o = "validation error: " + m.message + ". " + e, true;
}

// validation.go:722-758 (buildErrorMessage / buildAnyPatternErrorMessage) and :640/:665 pass messages of the pair at
// kind-major position `res`; false: the text needs the reference engine (Go error strings, variables)
static bool render_message(kyv_results* r, const Ruleset& rs, const Batch& b, uint32_t res, uint32_t rule, std::string* o) {
  uint8_t sb = r->r.status[(size_t)rule * r->r.nres + res];
  uint8_t st = sb & 7, alt = sb >> 3;
  const RuleMeta& m = rs.meta[rule];
  const RuleDesc& d = rs.rules[rule];
  if (st == ST_SKIP && d.exc != NONE && alt >= 1 && alt <= m.exc_keys.size())  // hasPolicyExceptions (validation.go:838-843)
    return *o = "rule skipped due to policy exception " + m.exc_keys[alt - 1], true;
  if (sb >> 3 == (ST_MARK_PRE >> 3) && d.pre != NONE) {  // checkPreconditions outcome (validation.go:281-288)
    if (st == ST_SKIP) return *o = "preconditions not met", true;
    std::string e;
    if (st == ST_ERROR && cond_error_text(rs, b, res, d.pre, &e))
      return *o = "failed to evaluate preconditions: failed to substitute variables in preconditions: " + e, true;
    return false;
  }
  if (d.kind == RK_DENY) {  // validateDeny (validation.go:437-479)
    if (st == ST_PASS) return *o = "validation rule '" + m.name + "' passed.", true;
    if (st == ST_FAIL) return m.message_vars ? false : deny_message(m, b, res, o);
    std::string e;
    if (st == ST_ERROR && cond_error_text(rs, b, res, d.root, &e))
      return *o = "failed to substitute variables in deny conditions: " + e, true;
    return false;
  }
  if (d.kind == RK_FOREACH) {  // validateForEach / validateElements (validation.go:319-381)
    if (st == ST_PASS) return *o = "rule passed", true;
    if (st == ST_SKIP) return *o = "rule skipped", true;
    if (st == ST_FAIL && m.foreach_texts)  // every entry a top-level deny: the one failure text
      return *o = "validation failure: " + (m.message.empty() ? "validation error: rule " + m.name + " failed" : m.message),
             true;
    return false;  // error texts embed Go error strings; pattern / nested failures embed the element's path
  }
  if (m.message_vars && st == ST_FAIL) return false;  // message needs variable substitution (CPU engine)
  if (d.kind == RK_PSS) {
    if (st == ST_PASS) return *o = "Validation rule '" + m.name + "' passed.", true;
    if (st != ST_FAIL) return false;  // decode / version error texts embed Go error strings
    std::vector<std::array<std::string, 3>> checks;
    if (!pss_checks_render(rs, b, res, rule, pss_mask_at(r, rs, res, rule), &checks)) return false;
    // validation.go:561 + pss.FormatChecksPrint (evaluate.go:160-166): fmt "(%+v)\n" of each CheckResult
    std::string msg = "Validation rule '" + m.name + "' failed. It violates PodSecurity \"" + m.pss_level + ":" +
                      m.pss_version + "\": ";
    for (auto& c : checks) msg += "({Allowed:false ForbiddenReason:" + c[1] + " ForbiddenDetail:" + c[2] + "})\n";
    return *o = msg, true;
  }
  if (st == ST_PASS) {
    if (d.kind == RK_ANYPATTERN) {
      if (alt == 31) return *o = m.message, true;
      return *o = "validation rule '" + m.name + "' anyPattern[" + std::to_string(alt) + "] passed.", true;
    }
    return *o = "validation rule '" + m.name + "' passed.", true;
  }
  if (st == ST_SKIP || st == ST_ERROR) return walk_text_message(rs, b, res, rule, st, o);
  if (st != ST_FAIL) return false;
  ensure_index(r);
  auto range = r->recidx.equal_range(((uint64_t)rule << 32) | res);
  std::vector<const FailRec*> recs;
  for (auto it = range.first; it != range.second; ++it) recs.push_back(&r->r.fails[it->second]);
  std::sort(recs.begin(), recs.end(), [](const FailRec* a, const FailRec* b2) { return a->alt < b2->alt; });
  if (recs.empty()) return false;
  if (d.kind == RK_PATTERN) {
    std::string path = format_path(rs, b, recs[0]->tmpl, recs[0]->idx, recs[0]->key);
    if (m.message.empty()) return *o = "validation error: rule " + m.name + " failed at path " + path, true;
    std::string mm;
    if (!error_message_head(m, b, res, &mm)) return false;
    return *o = "validation error: " + mm + " rule " + m.name + " failed at path " + path, true;
  }
  std::string joined;
  for (size_t i = 0; i < recs.size(); i++) {
    if (recs[i]->tmpl == NONE) return walk_text_message(rs, b, res, rule, st, o);  // "failed: <err>"
    if (i) joined += " ";
    joined += "rule " + m.name + "[" + std::to_string(recs[i]->alt) + "] failed at path " +
              format_path(rs, b, recs[i]->tmpl, recs[i]->idx, recs[i]->key);
  }
  if (m.message.empty()) return *o = "validation error: " + joined, true;
  if (m.message.back() == '.') return *o = "validation error: " + m.message + " " + joined, true;
  return *o = "validation error: " + m.message + ". " + joined, true;
}

int64_t kyv_results_message(const kyv_results* cr, const kyv_ruleset* crs, const kyv_batch* cb, uint32_t res, uint32_t rule,
                            char* buf, size_t cap) {
  auto* r = const_cast<kyv_results*>(cr);
  if (!r || !crs || !cb || rule >= r->r.nrules || res >= r->r.nres || r->r.status.empty()) return -1;
  std::string m;
  try {
    if (!render_message(r, *crs->rs, *cb->b, (*r->inv)[res], rule, &m)) return -1;
  } catch (std::exception& e) {
    fail(KYV_EINTERNAL, e.what());
    return -1;
  }
  return put(m, buf, cap);
}

int64_t kyv_results_failures(const kyv_results* r, kyv_failure* out, size_t cap) {
  if (!r) return fail(KYV_EINVAL, "null argument"), -1;
  if (r->r.status.empty() && r->r.nres && r->r.nrules) return fail(KYV_ERANGE, "verdicts kept on the device"), -1;
  const size_t n = r->r.fails.size();
  std::vector<uint32_t> order(r->inv->size());
  for (size_t i = 0; i < r->inv->size(); i++) order[(*r->inv)[i]] = (uint32_t)i;  // kind-major position -> input index
  for (size_t i = 0; i < n && out && i < cap; i++) {
    const FailRec& f = r->r.fails[i];
    kyv_failure& o = out[i];
    o.res = f.res < order.size() ? order[f.res] : f.res;
    o.rule = f.rule;
    o.alt = f.alt;
    o.path_template = f.tmpl;
    for (int j = 0; j < 4; j++) o.idx[j] = f.idx[j];
    o.key[0] = f.key[0];
    o.key[1] = f.key[1];
  }
  return (int64_t)n;
}

// PatternError.Path of a single-pattern FAIL at kind-major position `res` ("" otherwise)
static std::string render_path(kyv_results* r, const Ruleset& rs, const Batch& b, uint32_t res, uint32_t rule) {
  // records exist for every failing alternative walked, also when a later anyPattern alternative passed
  if ((r->r.status[(size_t)rule * r->r.nres + res] & 7) != ST_FAIL || rs.rules[rule].kind != RK_PATTERN) return "";
  ensure_index(r);
  auto it = r->recidx.find(((uint64_t)rule << 32) | res);
  if (it == r->recidx.end()) return "";
  const FailRec& f = r->r.fails[it->second];
  return format_path(rs, b, f.tmpl, f.idx, f.key);
}

int64_t kyv_results_path(const kyv_results* cr, const kyv_ruleset* crs, const kyv_batch* cb, uint32_t res, uint32_t rule,
                         char* buf, size_t cap) {
  auto* r = const_cast<kyv_results*>(cr);
  if (!r || !crs || !cb || rule >= r->r.nrules || res >= r->r.nres || r->r.status.empty()) return -1;
  try {
    return put(render_path(r, *crs->rs, *cb->b, (*r->inv)[res], rule), buf, cap);
  } catch (std::exception& e) {
    fail(KYV_EINTERNAL, e.what());
    return -1;
  }
}

int64_t kyv_results_texts(const kyv_results* cr, const kyv_ruleset* crs, const kyv_batch* cb, uint32_t rule, uint32_t res0,
                          uint32_t nres, uint32_t status_mask, int32_t what, char* buf, size_t cap, int32_t* lens) {
  auto* r = const_cast<kyv_results*>(cr);
  if (!r || !crs || !cb || rule >= r->r.nrules || (what != KYV_TEXT_MESSAGE && what != KYV_TEXT_PATH))
    return fail(KYV_EINVAL, "bad argument"), -1;
  if ((uint64_t)res0 + nres > r->r.nres) return fail(KYV_ERANGE, "resource range out of bounds"), -1;
  if (r->r.status.empty() && r->r.nres) return fail(KYV_ERANGE, "verdicts kept on the device"), -1;
  try {
    const Ruleset& rs = *crs->rs;
    const Batch& b = *cb->b;
    ensure_index(r);
    // rendered per thread over contiguous slices, then packed in resource order
    const int nt = std::max(1, std::min(hw_threads(0), (int)(nres / 4096) + 1));
    std::vector<std::string> part(nt);
    std::vector<int32_t> len(nres);
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
      th.emplace_back([&, t]() {
        const uint32_t lo = (uint32_t)((uint64_t)nres * t / nt), hi = (uint32_t)((uint64_t)nres * (t + 1) / nt);
        std::string one;
        for (uint32_t i = lo; i < hi; i++) {
          const uint32_t pos = (*r->inv)[res0 + i];
          const uint8_t st = r->r.status[(size_t)rule * r->r.nres + pos] & 7;
          if (!((status_mask >> st) & 1u)) { len[i] = -2; continue; }
          bool ok = true;
          if (what == KYV_TEXT_PATH) one = render_path(r, rs, b, pos, rule);
          else ok = render_message(r, rs, b, pos, rule, &one);
          if (!ok || one.size() > (size_t)INT32_MAX) { len[i] = -1; continue; }
          len[i] = (int32_t)one.size();
          part[t] += one;
        }
      });
    for (auto& x : th) x.join();
    size_t total = 0;
    for (auto& p : part) total += p.size();
    if (lens) memcpy(lens, len.data(), (size_t)nres * sizeof(int32_t));
    if (buf && cap >= total) {
      size_t at = 0;
      for (auto& p : part) { memcpy(buf + at, p.data(), p.size()); at += p.size(); }
    }
    return (int64_t)total;
  } catch (std::exception& e) {
    fail(KYV_EINTERNAL, e.what());
    return -1;
  }
}

int64_t kyv_results_fallback_reason(const kyv_results* r, const kyv_ruleset* rs, const kyv_batch* b, uint32_t res,
                                    uint32_t rule, char* buf, size_t cap) {
  if (!r || !rs || !b || rule >= r->r.nrules || res >= r->r.nres) return -1;
  try {
    const uint32_t pos = (*r->inv)[res];
    if (r->r.status.empty()) return fail(KYV_ERANGE, "verdicts kept on the device"), -1;  // status unknown here
    if ((r->r.status[(size_t)rule * r->r.nres + pos] & 7) != ST_FALLBACK) return put("", buf, cap);
    return put(fallback_why(*rs->rs, *b->b, pos, rule), buf, cap);
  } catch (std::exception& e) {
    fail(KYV_EINTERNAL, e.what());
    return -1;
  }
}

int64_t kyv_results_pss_checks(const kyv_results* cr, const kyv_ruleset* crs, const kyv_batch* cb, uint32_t res,
                               uint32_t rule, char* buf, size_t cap) {
  auto* r = const_cast<kyv_results*>(cr);
  if (!r || !crs || !cb || rule >= r->r.nrules || res >= r->r.nres || r->r.status.empty()) return -1;
  const Ruleset& rs = *crs->rs;
  if (rs.rules[rule].kind != RK_PSS) return -1;
  try {
    const uint32_t pos = (*r->inv)[res];
    const uint8_t st = r->r.status[(size_t)rule * r->r.nres + pos] & 7;
    if (st != ST_PASS && st != ST_FAIL) return -1;
    std::vector<std::array<std::string, 3>> checks;
    if (st == ST_FAIL && !pss_checks_render(rs, *cb->b, pos, rule, pss_mask_at(r, rs, pos, rule), &checks)) return -1;
    const RuleMeta& m = rs.meta[rule];
    std::string o = "{\"level\":" + json_str(m.pss_level) + ",\"version\":" + json_str(m.pss_version) + ",\"checks\":[";
    for (size_t i = 0; i < checks.size(); i++)
      o += std::string(i ? "," : "") + "{\"id\":" + json_str(checks[i][0]) + ",\"allowed\":false,\"reason\":" +
           json_str(checks[i][1]) + ",\"detail\":" + json_str(checks[i][2]) + "}";
    return put(o + "]}", buf, cap);
  } catch (std::exception& e) {
    fail(KYV_EINTERNAL, e.what());
    return -1;
  }
}

uint32_t kyv_results_pss_mask(const kyv_results* r, const kyv_ruleset* rs, uint32_t res, uint32_t rule) {
  if (!r || !rs || rule >= r->r.nrules || res >= r->r.nres) return 0;
  res = (*r->inv)[res];
  uint32_t slot = 0;
  for (uint32_t k = 0; k < rule; k++) if (rs->rs->rules[k].kind == RK_PSS) slot++;
  if (rs->rs->rules[rule].kind != RK_PSS) return 0;
  size_t i = (size_t)slot * r->r.nres + res;
  return i < r->r.pss_fails.size() ? r->r.pss_fails[i] : 0;
}

}  // extern "C"

// ---------------------------------------------------------------- multi-GPU report gather over RCCL
// One process per GPU; the communicator is created by the library itself (no framework in the data path): rank 0
// draws the unique id, the caller hands it to the other ranks out of band (bench.py: a gloo broadcast), every rank
// calls kyv_comm_init on its device. kyv_comm_gather_results all-gathers the device-resident results of a batch's
// last GPU evaluation: the packed verdicts (kyv_batch_export_status layout per rank, padded to the largest shard)
// and the failing-path rows (count, then rows padded to the largest count), each into buffers the communicator owns,
// timed with HIP events on its stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

struct kyv_comm {
  ncclComm_t comm = nullptr;
  int device = 0, rank = 0, nranks = 1;
  hipStream_t stream = nullptr;
  uint8_t* status = nullptr;   // [nranks][status_bytes]
  size_t status_cap = 0, status_bytes = 0;
  int64_t* rows = nullptr;     // [nranks][rows_max][8]
  size_t rows_cap = 0, rows_max = 0;
  std::vector<int64_t> row_counts;
  // kyv_comm_gather_report (to one consumer rank): per rank, its packed verdicts and its 16-byte rows at exact sizes
  int mode = 0;                // last gather: 0 none, 1 all-gather (gather_results), 2 to `root` (gather_report)
  int root = 0;
  std::vector<int64_t> seg_status, seg_rows, seg_wide, res_off;  // per rank: sizes, offsets below, resource offset
  std::vector<size_t> at_status, at_rows, at_wide;
  uint32_t* rrows = nullptr;   // root: every rank's rows, uint32 x 4 each; other ranks: their own (send buffer)
  size_t rrows_cap = 0;
  uint32_t* rwide = nullptr;   // side entries of the rows that do not fit 16 bytes
  size_t rwide_cap = 0;
  uint32_t* nwide = nullptr;   // [1] side-entry count (report_rows_kernel)
  unsigned long long* sums = nullptr;  // kyv_comm_reduce_counts: [rules * NSTATUS + 1]
  size_t sums_cap = 0;
  // device buffer of the size / flag exchanges ([nranks + 1][kXK] int64), allocated once in kyv_comm_init so that an
  // exchange never allocates: a rank always reaches the exchange's all-gather once it has called the collective
  int64_t* xbuf = nullptr;
};

namespace {
constexpr int kXK = 8;  // int64 fields per rank one size / flag exchange carries at most
int nccl_fail(ncclResult_t r, const char* what) {
  return fail(KYV_EDEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}
#define KYV_NCCL(x) do { ncclResult_t r_ = (x); if (r_ != ncclSuccess) return nccl_fail(r_, #x); } while (0)
#define KYV_HIPC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return fail(KYV_EDEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); } while (0)
template <class T>
int grow(T** p, size_t* cap, size_t n) {
  if (n <= *cap && *p) return KYV_OK;
  if (*p) KYV_HIPC(hipFree(*p));
  *p = nullptr;
  KYV_HIPC(hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)));
  *cap = n;
  return KYV_OK;
}
}  // namespace

int kyv_comm_unique_id(uint8_t* id, size_t cap) {
  if (!id || cap < sizeof(ncclUniqueId)) return fail(KYV_ERANGE, "unique id buffer too small");
  ncclUniqueId u;
  KYV_NCCL(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof u);
  return KYV_OK;
}

int kyv_comm_init(const uint8_t* id, size_t len, int nranks, int rank, int device, kyv_comm** out) {
  if (!id || !out || len < sizeof(ncclUniqueId) || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(KYV_EINVAL, "bad communicator arguments");
  auto* c = new kyv_comm();
  c->device = device;
  c->rank = rank;
  c->nranks = nranks;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc((void**)&c->xbuf, sizeof(int64_t) * kXK * (nranks + 1));
  if (e != hipSuccess) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return fail(KYV_EDEVICE, std::string("comm stream / exchange buffer: ") + hipGetErrorString(e));
  }
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    (void)hipStreamDestroy(c->stream);
    (void)hipFree(c->xbuf);
    delete c;
    return nccl_fail(r, "ncclCommInitRank");
  }
  *out = c;
  return KYV_OK;
}

void kyv_comm_free(kyv_comm* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->status) (void)hipFree(c->status);
  if (c->rows) (void)hipFree(c->rows);
  if (c->rrows) (void)hipFree(c->rrows);
  if (c->rwide) (void)hipFree(c->rwide);
  if (c->nwide) (void)hipFree(c->nwide);
  if (c->sums) (void)hipFree(c->sums);
  if (c->xbuf) (void)hipFree(c->xbuf);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

namespace {
// One small all-gather of k int64 per rank (sizes and ok flags) -> out[nranks * k], through the communicator's own
// exchange buffer (no allocation). The all-gather is posted whatever happened before it on this rank: the collectives
// of a report gather are only ever entered behind such an exchange, and every rank leaves the exchange with the same
// view of every rank's flags (a failed upload of this rank's entries returns an error here after the collective).
int exchange_sizes(kyv_comm* c, const int64_t* mine, int k, std::vector<int64_t>* out) {
  const int n = c->nranks;
  if (k < 1 || k > kXK) return fail(KYV_EINTERNAL, "size exchange wider than the exchange buffer");
  int64_t* send = c->xbuf + (size_t)kXK * n;
  const hipError_t up = hipMemcpyAsync(send, mine, sizeof(int64_t) * k, hipMemcpyHostToDevice, c->stream);
  KYV_NCCL(ncclAllGather(send, c->xbuf, k, ncclInt64, c->comm, c->stream));
  out->assign((size_t)k * n, 0);
  KYV_HIPC(hipMemcpyAsync(out->data(), c->xbuf, sizeof(int64_t) * k * n, hipMemcpyDeviceToHost, c->stream));
  KYV_HIPC(hipStreamSynchronize(c->stream));
  if (up != hipSuccess) return fail(KYV_EDEVICE, std::string("upload of the exchanged sizes: ") + hipGetErrorString(up));
  return KYV_OK;
}
// every rank's ok flag (field f of k per rank): all ranks return the same error when any is 0
int check_flags(kyv_comm* c, const std::vector<int64_t>& sz, int k, int f, const std::string& why,
                const char* what = "has no exportable results") {
  for (int q = 0; q < c->nranks; q++)
    if (!sz[(size_t)k * q + f])
      return fail(KYV_EDEVICE, "report gather: rank " + std::to_string(q) + " " + what +
                               (q == c->rank && !why.empty() ? ": " + why : std::string()));
  return KYV_OK;
}
// one flag exchange: every rank continues only when every rank's local step (buffers, exports) succeeded
int agree(kyv_comm* c, bool ok, const std::string& why) {
  const int64_t f = ok ? 1 : 0;
  std::vector<int64_t> sz;
  if (int rc = exchange_sizes(c, &f, 1, &sz)) return rc;
  return check_flags(c, sz, 1, 0, why, "could not prepare its buffers");
}
// HIP-event timing of a gather; a failure to create or record an event costs the timing only, never the collective
struct GatherTimer {
  hipEvent_t e[3] = {nullptr, nullptr, nullptr};
  GatherTimer() {
    for (auto& x : e)
      if (hipEventCreate(&x) != hipSuccess) x = nullptr;
  }
  ~GatherTimer() { for (auto x : e) if (x) (void)hipEventDestroy(x); }
  void mark(int i, hipStream_t s) { if (e[i] && hipEventRecord(e[i], s) != hipSuccess) e[i] = nullptr; }
  float ms(int a, int b) const {
    float t = 0;
    return e[a] && e[b] && hipEventElapsedTime(&t, e[a], e[b]) == hipSuccess ? t : 0.f;
  }
};
// the local preparation steps of a gather record their first failure here instead of returning: the rank still joins
// the flag exchange that follows (a rank returning early would leave its peers inside the collective)
struct LocalOk {
  bool ok = true;
  std::string why;
  void hip(hipError_t e, const char* what) {
    if (ok && e != hipSuccess) { ok = false; why = std::string(what) + ": " + hipGetErrorString(e); }
  }
  void rc(int r, const char* what) {
    if (ok && r != KYV_OK) { ok = false; why = std::string(what) + ": " + kyv_last_error(); }
  }
  void ex(const std::exception& e) { if (ok) { ok = false; why = e.what(); } }
};
}  // namespace

int kyv_comm_gather_results(kyv_comm* c, const kyv_batch* b, int64_t res_offset, kyv_gather_stats* st) {
  if (!c || !b || !st) return fail(KYV_EINVAL, "null argument");
  try {
    *st = kyv_gather_stats{};
    const int n = c->nranks;
    c->mode = 0;
    c->row_counts.clear();
    // sizes of every rank (one small all-gather): verdict bytes, failing-path rows and an ok flag. A rank that cannot
    // take part (no resident results, rows over the resident buffer) still joins this exchange with flag 0, and every
    // rank returns the same error: no rank is left waiting in a collective its peers never enter
    LocalOk lk;
    lk.hip(hipSetDevice(c->device), "hipSetDevice");
    int64_t mine[3] = {0, 0, 0};
    if (lk.ok) {
      try {
        mine[0] = export_status(*b->b, c->device, nullptr, 0, c->stream);
        mine[1] = export_failures(*b->b, c->device, res_offset, nullptr, 0, c->stream);
      } catch (std::exception& e) {
        lk.ex(e);
      }
    }
    mine[2] = lk.ok ? 1 : 0;
    std::vector<int64_t> sz;
    if (int rc = exchange_sizes(c, mine, 3, &sz)) return rc;
    if (int rc = check_flags(c, sz, 3, 2, lk.why)) return rc;
    size_t smax = 0, rmax = 0;
    c->row_counts.assign(n, 0);
    for (int q = 0; q < n; q++) {
      smax = std::max<size_t>(smax, (size_t)sz[3 * q]);
      rmax = std::max<size_t>(rmax, (size_t)sz[3 * q + 1]);
      c->row_counts[q] = sz[3 * q + 1];
      st->failure_rows_total += (uint64_t)sz[3 * q + 1];
    }
    // local: the buffers and this rank's send data; then every rank agrees before the all-gathers
    GatherTimer tm;
    lk.rc(grow(&c->status, &c->status_cap, smax * (n + 1)), "verdict buffer");
    lk.rc(grow(&c->rows, &c->rows_cap, rmax * 8 * (n + 1)), "row buffer");
    uint8_t* sendv = lk.ok ? c->status + smax * n : nullptr;  // this rank's packed verdicts, all-gathered into [0, n * smax)
    int64_t* sendr = lk.ok ? c->rows + rmax * 8 * n : nullptr;
    tm.mark(0, c->stream);
    if (lk.ok) {
      try {
        if (smax) export_status(*b->b, c->device, sendv, smax, c->stream);
        if (rmax) export_failures(*b->b, c->device, res_offset, sendr, rmax, c->stream);
      } catch (std::exception& e) {
        lk.ex(e);
      }
    }
    if (int rc = agree(c, lk.ok, lk.why)) return rc;
    c->status_bytes = smax;
    c->rows_max = rmax;
    // only collectives from here on
    if (smax) KYV_NCCL(ncclAllGather(sendv, c->status, smax, ncclUint8, c->comm, c->stream));
    tm.mark(1, c->stream);
    if (rmax) KYV_NCCL(ncclAllGather(sendr, c->rows, rmax * 8, ncclInt64, c->comm, c->stream));
    tm.mark(2, c->stream);
    KYV_HIPC(hipStreamSynchronize(c->stream));
    st->status_ms = tm.ms(0, 1);
    st->failures_ms = tm.ms(1, 2);
    st->status_bytes_per_rank = smax;
    st->failure_rows_per_rank_max = rmax;
    c->mode = 1;
    return KYV_OK;
  } catch (std::exception& e) {
    return fail(KYV_EINVAL, e.what());
  }
}

int64_t kyv_comm_gathered_status(const kyv_comm* c, int rank, uint8_t* host_dst, size_t cap) {
  if (!c || rank < 0 || rank >= c->nranks) return fail(KYV_EINVAL, "bad rank"), -1;
  if (c->mode == 2) {  // gather_report: exact segments, on the root only
    if (c->rank != c->root) return fail(KYV_EINVAL, "the report was gathered to another rank"), -1;
    const size_t nb = (size_t)c->seg_status[rank];
    if (!host_dst) return (int64_t)nb;
    if (cap < nb) return fail(KYV_ERANGE, "buffer too small"), -1;
    if (nb && (hipSetDevice(c->device) != hipSuccess ||
               hipMemcpy(host_dst, c->status + c->at_status[rank], nb, hipMemcpyDeviceToHost) != hipSuccess))
      return fail(KYV_EDEVICE, "copy of the gathered verdicts failed"), -1;
    return (int64_t)nb;
  }
  if (!host_dst) return (int64_t)c->status_bytes;
  if (cap < c->status_bytes) return fail(KYV_ERANGE, "buffer too small"), -1;
  if (hipSetDevice(c->device) != hipSuccess ||
      hipMemcpy(host_dst, c->status + c->status_bytes * rank, c->status_bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return fail(KYV_EDEVICE, "copy of the gathered verdicts failed"), -1;
  return (int64_t)c->status_bytes;
}

int64_t kyv_comm_gathered_failures(const kyv_comm* c, int rank, int64_t* host_dst, size_t cap_rows) {
  if (!c || rank < 0 || rank >= c->nranks) return fail(KYV_EINVAL, "bad rank"), -1;
  if (c->mode == 2) {  // gather_report: the 16-byte rows (and side entries) expanded to the 8 x int64 row form
    if (c->rank != c->root) return fail(KYV_EINVAL, "the report was gathered to another rank"), -1;
    const size_t nr = (size_t)c->seg_rows[rank], nw = (size_t)c->seg_wide[rank];
    if (!host_dst) return (int64_t)nr;
    if (cap_rows < nr) return fail(KYV_ERANGE, "buffer too small"), -1;
    std::vector<uint32_t> rw(nr * 4), wd(nw * 4);
    if (hipSetDevice(c->device) != hipSuccess ||
        (nr && hipMemcpy(rw.data(), c->rrows + c->at_rows[rank] * 4, nr * 16, hipMemcpyDeviceToHost) != hipSuccess) ||
        (nw && hipMemcpy(wd.data(), c->rwide + c->at_wide[rank] * 4, nw * 16, hipMemcpyDeviceToHost) != hipSuccess))
      return fail(KYV_EDEVICE, "copy of the gathered rows failed"), -1;
    for (size_t i = 0; i < nr; i++) {
      const uint32_t* r = &rw[i * 4];
      int64_t* o = host_dst + i * 8;
      o[0] = (int64_t)r[0] + c->res_off[rank];
      o[3] = r[2];
      if (r[1] & 0x80000000u) {
        if (r[3] >= nw) return fail(KYV_EINTERNAL, "report row side entry out of range"), -1;
        const uint32_t* w = &wd[(size_t)r[3] * 4];
        o[1] = w[0];
        o[2] = w[1];
        o[4] = w[2] & 0xFFFF; o[5] = w[2] >> 16; o[6] = w[3] & 0xFFFF; o[7] = w[3] >> 16;
      } else {
        o[1] = r[1] & 0xFFFFFF;
        o[2] = r[1] >> 24;
        for (int q = 0; q < 4; q++) {
          const uint32_t x = (r[3] >> (8 * q)) & 255u;
          o[4 + q] = x == 255u ? 0xFFFF : x;
        }
      }
    }
    return (int64_t)nr;
  }
  if ((size_t)rank >= c->row_counts.size()) return 0;  // no gather yet (or the last one failed before its counts)
  const size_t nr = (size_t)c->row_counts[rank];
  if (!host_dst) return (int64_t)nr;
  if (cap_rows < nr) return fail(KYV_ERANGE, "buffer too small"), -1;
  if (nr && (hipSetDevice(c->device) != hipSuccess ||
             hipMemcpy(host_dst, c->rows + c->rows_max * 8 * rank, nr * 8 * sizeof(int64_t), hipMemcpyDeviceToHost) != hipSuccess))
    return fail(KYV_EDEVICE, "copy of the gathered rows failed"), -1;
  return (int64_t)nr;
}

// Report assembly to ONE consumer rank (the report controller's process; pkg/controllers/report builds the
// PolicyReports in one place): every rank's packed verdicts and its failing-path rows as 16-byte records (plus 16-byte
// side entries for the rare rows that do not fit) go to `root` with grouped point-to-point sends at their exact sizes
// -- no padding and no copy on the ranks that do not consume them. Bytes on the wire per rank: its packed verdicts
// (2 bits per pair) + 16 B per failing-path row; the root receives the sum over the other ranks.
int kyv_comm_gather_report(kyv_comm* c, const kyv_batch* b, int64_t res_offset, int root, kyv_gather_stats* st) {
  if (!c || !b || !st) return fail(KYV_EINVAL, "null argument");
  if (root < 0 || root >= c->nranks) return fail(KYV_EINVAL, "bad root rank");  // the same on every rank
  try {
    *st = kyv_gather_stats{};
    c->mode = 0;
    const int n = c->nranks;
    const bool me_root = c->rank == root;
    // Local steps before the size exchange (each failure joins the exchange with flag 0): the device, this rank's
    // sizes, and its rows packed now into temporaries (the side-entry count is part of the exchange); the senders send
    // from them, the root moves its own into its receive segments
    LocalOk lk;
    lk.hip(hipSetDevice(c->device), "hipSetDevice");
    if (lk.ok && !c->nwide) lk.hip(hipMalloc((void**)&c->nwide, 4), "side-entry counter");
    int64_t mine[5] = {0, 0, 0, 0, res_offset};
    if (lk.ok) {
      try {
        mine[0] = export_status(*b->b, c->device, nullptr, 0, c->stream);
        mine[1] = export_report_rows(*b->b, c->device, nullptr, nullptr, nullptr, 0, 0, c->stream);
      } catch (std::exception& e) {
        lk.ex(e);
      }
    }
    const size_t own_rows = lk.ok ? (size_t)std::max<int64_t>(mine[1], 0) : 0;
    uint32_t *packed = nullptr, *pwide = nullptr;
    struct Free { void* p; ~Free() { if (p) (void)hipFree(p); } } fp{nullptr}, fw{nullptr};
    if (own_rows) {
      lk.hip(hipMalloc((void**)&packed, own_rows * 16), "row buffer");
      if (lk.ok) fp.p = packed;
      if (lk.ok) lk.hip(hipMalloc((void**)&pwide, own_rows * 16), "side-entry buffer");
      if (lk.ok) fw.p = pwide;
      if (lk.ok) {
        try {
          export_report_rows(*b->b, c->device, packed, pwide, c->nwide, own_rows, own_rows, c->stream);
          uint32_t nw = 0;
          lk.hip(hipMemcpyAsync(&nw, c->nwide, 4, hipMemcpyDeviceToHost, c->stream), "side-entry count");
          if (lk.ok) lk.hip(hipStreamSynchronize(c->stream), "row export");
          mine[2] = nw;
        } catch (std::exception& e) {
          lk.ex(e);
        }
      }
    }
    mine[3] = lk.ok ? 1 : 0;
    std::vector<int64_t> sz;
    if (int rc = exchange_sizes(c, mine, 5, &sz)) return rc;
    if (int rc = check_flags(c, sz, 5, 3, lk.why)) return rc;
    // receive layout on the root: every rank's segment at exact offsets (the same on every rank: from the exchange)
    c->root = root;
    c->seg_status.assign(n, 0);
    c->seg_rows.assign(n, 0);
    c->seg_wide.assign(n, 0);
    c->res_off.assign(n, 0);
    c->at_status.assign(n, 0);
    c->at_rows.assign(n, 0);
    c->at_wide.assign(n, 0);
    size_t ts = 0, tr = 0, tw = 0;
    for (int q = 0; q < n; q++) {
      c->seg_status[q] = sz[5 * q];
      c->seg_rows[q] = sz[5 * q + 1];
      c->seg_wide[q] = sz[5 * q + 2];
      c->res_off[q] = sz[5 * q + 4];
      c->at_status[q] = ts;
      c->at_rows[q] = tr;
      c->at_wide[q] = tw;
      ts += (size_t)sz[5 * q];
      tr += (size_t)sz[5 * q + 1];
      tw += (size_t)sz[5 * q + 2];
      st->failure_rows_total += (uint64_t)sz[5 * q + 1];
    }
    const size_t my_s = (size_t)mine[0], my_w = (size_t)mine[2];
    // Local steps after the size exchange: the buffers (the root holds every segment; a sender only its own verdicts,
    // its rows are sent from `packed`), this rank's packed verdicts exported into place and the root's own rows moved
    // into its segments -- then one flag exchange, and from there only the grouped sends / receives
    GatherTimer tm;
    lk.rc(grow(&c->status, &c->status_cap, me_root ? ts : my_s), "verdict buffer");
    if (me_root) {
      lk.rc(grow(&c->rrows, &c->rrows_cap, tr * 4), "row receive buffer");
      lk.rc(grow(&c->rwide, &c->rwide_cap, tw * 4), "side-entry receive buffer");
    }
    uint8_t* my_status = lk.ok ? c->status + (me_root ? c->at_status[root] : 0) : nullptr;
    tm.mark(0, c->stream);
    if (lk.ok && my_s) {
      try {
        export_status(*b->b, c->device, my_status, my_s, c->stream);
      } catch (std::exception& e) {
        lk.ex(e);
      }
    }
    if (lk.ok && me_root && own_rows)
      lk.hip(hipMemcpyAsync(c->rrows + c->at_rows[root] * 4, packed, own_rows * 16, hipMemcpyDeviceToDevice, c->stream),
             "root's own rows");
    if (lk.ok && me_root && my_w)
      lk.hip(hipMemcpyAsync(c->rwide + c->at_wide[root] * 4, pwide, my_w * 16, hipMemcpyDeviceToDevice, c->stream),
             "root's own side entries");
    if (int rc = agree(c, lk.ok, lk.why)) return rc;
    KYV_NCCL(ncclGroupStart());
    if (me_root) {
      for (int q = 0; q < n; q++)
        if (q != root && c->seg_status[q])
          KYV_NCCL(ncclRecv(c->status + c->at_status[q], (size_t)c->seg_status[q], ncclUint8, q, c->comm, c->stream));
    } else if (my_s) {
      KYV_NCCL(ncclSend(my_status, my_s, ncclUint8, root, c->comm, c->stream));
    }
    KYV_NCCL(ncclGroupEnd());
    tm.mark(1, c->stream);
    KYV_NCCL(ncclGroupStart());
    if (me_root) {
      for (int q = 0; q < n; q++) {
        if (q == root) continue;
        if (c->seg_rows[q])
          KYV_NCCL(ncclRecv(c->rrows + c->at_rows[q] * 4, (size_t)c->seg_rows[q] * 4, ncclUint32, q, c->comm, c->stream));
        if (c->seg_wide[q])
          KYV_NCCL(ncclRecv(c->rwide + c->at_wide[q] * 4, (size_t)c->seg_wide[q] * 4, ncclUint32, q, c->comm, c->stream));
      }
    } else {
      if (own_rows) KYV_NCCL(ncclSend(packed, own_rows * 4, ncclUint32, root, c->comm, c->stream));
      if (my_w) KYV_NCCL(ncclSend(pwide, my_w * 4, ncclUint32, root, c->comm, c->stream));
    }
    KYV_NCCL(ncclGroupEnd());
    tm.mark(2, c->stream);
    KYV_HIPC(hipStreamSynchronize(c->stream));
    st->status_ms = tm.ms(0, 1);
    st->failures_ms = tm.ms(1, 2);
    st->status_bytes_per_rank = my_s;
    st->failure_rows_per_rank_max = 0;
    for (int q = 0; q < n; q++) st->failure_rows_per_rank_max = std::max<uint64_t>(st->failure_rows_per_rank_max, (uint64_t)c->seg_rows[q]);
    c->mode = 2;
    return KYV_OK;
  } catch (std::exception& e) {
    return fail(KYV_EINVAL, e.what());
  }
}

// Cluster-wide per-rule verdict tallies (the summary all-reduce of a sharded background scan, the
// PolicyReport summary counts of pkg/controllers/report): the device-resident [rules][KYV_NSTATUS] tallies of the
// batch's last evaluation summed over ranks with one ncclAllReduce; the none column (not tallied on the device) is
// derived from the summed resource count. host_out [rules * KYV_NSTATUS] int64; returns the entry count (host_out
// NULL: only the count), -1 on error. Every rank must call it (a collective); a rank without results joins with zeros
// and every rank then returns an error.
int64_t kyv_comm_reduce_counts(kyv_comm* c, const kyv_batch* b, int64_t* host_out, size_t cap) {
  if (!c || !b) return fail(KYV_EINVAL, "null argument"), -1;
  try {
    LocalOk lk;
    lk.hip(hipSetDevice(c->device), "hipSetDevice");
    size_t nrules = 0, nres = 0;
    const unsigned long long* cnt = nullptr;
    if (lk.ok) {
      try {
        cnt = device_counts(*b->b, c->device, &nrules, &nres);
      } catch (std::exception& e) {
        lk.ex(e);
      }
    }
    const size_t ne = nrules * NSTATUS;
    // size query (no collective): never an error, so that a caller sizing its buffer always goes on to make the
    // collective call; a rank without results answers 0 and fails below together with its peers
    if (!host_out) return cnt ? (int64_t)ne : 0;
    // local steps first (every rank must reduce the same element count, into a buffer large enough): their outcome
    // is the ok flag of the size exchange
    if (lk.ok && !cnt) { lk.ok = false; lk.why = "no device-resident verdict tallies"; }
    if (lk.ok && cap < ne) { lk.ok = false; lk.why = "buffer too small"; }
    lk.rc(grow(&c->sums, &c->sums_cap, ne + 1), "tally buffer");
    const unsigned long long nr = nres;
    if (lk.ok && ne) lk.hip(hipMemcpyAsync(c->sums, cnt, ne * 8, hipMemcpyDeviceToDevice, c->stream), "tally copy");
    if (lk.ok) lk.hip(hipMemcpyAsync(c->sums + ne, &nr, 8, hipMemcpyHostToDevice, c->stream), "resource count copy");
    int64_t mine[2] = {(int64_t)ne, lk.ok ? 1 : 0};
    std::vector<int64_t> sz;
    if (exchange_sizes(c, mine, 2, &sz)) return -1;
    if (check_flags(c, sz, 2, 1, lk.why, "cannot reduce its tallies")) return -1;
    for (int q = 0; q < c->nranks; q++)
      if (sz[2 * q] != (int64_t)ne) return fail(KYV_EINVAL, "ranks evaluated different rulesets"), -1;
    ncclResult_t r = ncclAllReduce(c->sums, c->sums, ne + 1, ncclUint64, ncclSum, c->comm, c->stream);
    if (r != ncclSuccess) return nccl_fail(r, "ncclAllReduce"), -1;
    std::vector<unsigned long long> h(ne + 1);
    if (hipMemcpyAsync(h.data(), c->sums, (ne + 1) * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      return fail(KYV_EDEVICE, "copy of the reduced tallies failed"), -1;
    for (size_t k = 0; k < nrules; k++) {
      unsigned long long counted = 0;
      for (int s = 1; s < NSTATUS; s++) {
        host_out[k * NSTATUS + s] = (int64_t)h[k * NSTATUS + s];
        counted += h[k * NSTATUS + s];
      }
      host_out[k * NSTATUS + ST_NONE] = (int64_t)(h[ne] - counted);
    }
    return (int64_t)ne;
  } catch (std::exception& e) {
    return fail(KYV_EINTERNAL, e.what()), -1;
  }
}
