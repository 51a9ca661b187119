// HIP execution of the batched validate path on MI355X (gfx950).
//
// Two phases per evaluation (match_eval -> pattern_eval with compaction):
//   match_kernel  one lane per resource, rule loop uniform across the wave: kind gate, match/exclude, dispatch;
//                 final verdicts for every pair that needs no pattern walk (incl. PodSecurity), and per-rule
//                 work lists of the pairs that do (wave ballot + one atomic per wave and rule);
//   walk_kernel   persistent grid-stride over 64-pair chunks of ONE rule each: the wave-uniform pattern walker
//                 (kyv_wave.h) with no idle lanes from gated / non-matching pairs.
// Verdicts are written rule-major (coalesced bytes); failing-path records are staged per walk chunk and compacted
// without atomics (compact_*_kernel); verdict totals are one histogram pass over the status bytes.
// the label-selector check inlined into the statically compiled kernels: as an out-of-line call its callee-saved
// registers went through scratch for every (resource, rule) pair with a selector (C4 round 4: 220 GB of scratch
// writes per evaluation in match_walk_kernel; inlined: 86 VGPRs, no scratch)
#define KYV_SEL_INLINE 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <map>
#include <chrono>
#include <cmath>
#include <functional>
#include <cstdlib>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "kyv_acct.h"
#include "kyv_host.h"
#define KYV_NO_KERNELS 1  // the evaluation kernels are compiled in kyv_prod.hip / kyv_acct.hip (kyv_launch.inc)
#include "kyv_kernels.h"

namespace kyv {

#define HIP_OK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x); \
  } while (0)

// ---------------------------------------------------------------- pinned staging
// Host arrays live in pageable memory (the flattener's vectors). A pageable hipMemcpy moves them through the runtime's
// own small staging buffers one chunk at a time; here they go through a per-process ring of pinned buffers instead:
// chunk i is copied into its pinned slot by several host threads while chunks i-1, i-2 are in flight on the DMA
// engine (hipMemcpyAsync), and a slot is reused only after its transfer's event has completed. The same ring serves
// device-to-host copies of verdicts (DMA into the slot, then a parallel copy out).
struct Staging {
  static constexpr int NSLOT = 3;
  static constexpr size_t CHUNK = (size_t)64 << 20;
  std::mutex mu;
  void* buf[NSLOT] = {nullptr, nullptr, nullptr};
  hipEvent_t ev[NSLOT] = {nullptr, nullptr, nullptr};
  // The ring's DMAs run on its own stream (round 6): a slot event is only ever recorded on this stream, never on a
  // caller's stream that may be destroyed before the slot is reused (HIP then failed the next hipEventSynchronize of
  // the slot with "operation not permitted on an event last recorded in a capturing stream": a batch upload right
  // after an evaluation whose stream was gone). `pre` orders the ring after the caller's stream, `join` the caller's
  // stream after the ring.
  hipStream_t st = nullptr;
  hipEvent_t pre = nullptr, join = nullptr;
  int dev = -1;
  bool ok = false;
  bool init(int device) {
    if (ok && dev == device) return true;
    release();
    dev = device;
    for (int i = 0; i < NSLOT; i++) {
      if (hipHostMalloc(&buf[i], CHUNK, hipHostMallocDefault) != hipSuccess) { release(); return false; }
      if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) { release(); return false; }
    }
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&pre, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&join, hipEventDisableTiming) != hipSuccess) {
      release();
      return false;
    }
    ok = true;
    return true;
  }
  // the ring's stream starts after everything queued on `caller` so far
  hipError_t after(hipStream_t caller) {
    hipError_t e = hipEventRecord(pre, caller);
    return e == hipSuccess ? hipStreamWaitEvent(st, pre, 0) : e;
  }
  // `caller` continues after everything queued on the ring's stream so far
  hipError_t before(hipStream_t caller) {
    hipError_t e = hipEventRecord(join, st);
    return e == hipSuccess ? hipStreamWaitEvent(caller, join, 0) : e;
  }
  void release() {
    for (int i = 0; i < NSLOT; i++) {
      if (ev[i]) (void)hipEventSynchronize(ev[i]);  // no transfer still reads or writes the slot
      if (buf[i]) (void)hipHostFree(buf[i]);
      if (ev[i]) (void)hipEventDestroy(ev[i]);
      buf[i] = nullptr;
      ev[i] = nullptr;
    }
    if (st) { (void)hipStreamSynchronize(st); (void)hipStreamDestroy(st); }
    if (pre) (void)hipEventDestroy(pre);
    if (join) (void)hipEventDestroy(join);
    st = nullptr;
    pre = join = nullptr;
    ok = false;
  }
};
static Staging g_staging;
static bool staging_off() {
  static const bool off = getenv("KYV_PINNED") && atoi(getenv("KYV_PINNED")) == 0;
  return off;
}
// memcpy of n bytes with up to 8 threads (pageable source pages are touched once by the copy)
static void par_memcpy(void* dst, const void* src, size_t n) {
  const size_t per = (size_t)8 << 20;
  const size_t nt = std::min<size_t>(8, (n + per - 1) / per);
  if (nt <= 1) { memcpy(dst, src, n); return; }
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; t++)
    th.emplace_back([=] {
      const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
      memcpy((uint8_t*)dst + lo, (const uint8_t*)src + lo, hi - lo);
    });
  for (auto& x : th) x.join();
}
// host -> device through the pinned ring on `stream` (pageable hipMemcpy when the ring is off or unavailable). Returns
// with up to NSLOT transfers still reading their slots: every later user of a slot (the next upload, a copy-back on
// any thread: staged_d2h) first waits on the slot's event, under the ring's lock
static hipError_t staged_h2d(uint8_t* dev, const void* src, size_t n, hipStream_t stream) {
  if (!n) return hipSuccess;
  int device = 0;
  hipError_t e = hipGetDevice(&device);
  if (e != hipSuccess) return e;
  std::unique_lock<std::mutex> lk(g_staging.mu);
  if (staging_off() || !g_staging.init(device)) return hipMemcpy(dev, src, n, hipMemcpyHostToDevice);
  static int slot = 0;
  if ((e = g_staging.after(stream)) != hipSuccess) return e;
  const hipStream_t rs = g_staging.st;
  for (size_t off = 0; off < n; off += Staging::CHUNK) {
    const size_t m = std::min(Staging::CHUNK, n - off);
    if ((e = hipEventSynchronize(g_staging.ev[slot])) != hipSuccess) return e;  // the slot's last transfer is done
    par_memcpy(g_staging.buf[slot], (const uint8_t*)src + off, m);
    if ((e = hipMemcpyAsync(dev + off, g_staging.buf[slot], m, hipMemcpyHostToDevice, rs)) != hipSuccess) return e;
    if ((e = hipEventRecord(g_staging.ev[slot], rs)) != hipSuccess) return e;
    slot = (slot + 1) % Staging::NSLOT;
  }
  return g_staging.before(stream);
}
// device -> host through the pinned ring: chunk i's DMA overlaps the copy-out of chunk i-1
static hipError_t staged_d2h(void* dst, const uint8_t* dev, size_t n, hipStream_t stream) {
  if (!n) return hipSuccess;
  int device = 0;
  hipError_t e = hipGetDevice(&device);
  if (e != hipSuccess) return e;
  std::unique_lock<std::mutex> lk(g_staging.mu);
  if (staging_off() || !g_staging.init(device)) return hipMemcpy(dst, dev, n, hipMemcpyDeviceToHost);
  const size_t nch = (n + Staging::CHUNK - 1) / Staging::CHUNK;
  auto issue = [&](size_t c) -> hipError_t {
    const int sl = (int)(c % Staging::NSLOT);
    const size_t off = c * Staging::CHUNK, m = std::min(Staging::CHUNK, n - off);
    // the slot's previous transfer may still be in flight: an upload (staged_h2d returns with its last DMAs still
    // reading their slots) from this or another host thread; the DMA into the slot waits for it
    hipError_t r = hipEventSynchronize(g_staging.ev[sl]);
    if (r != hipSuccess) return r;
    r = hipMemcpyAsync(g_staging.buf[sl], dev + off, m, hipMemcpyDeviceToHost, g_staging.st);
    return r == hipSuccess ? hipEventRecord(g_staging.ev[sl], g_staging.st) : r;
  };
  if ((e = g_staging.after(stream)) != hipSuccess) return e;
  for (size_t c = 0; c < nch && c < (size_t)Staging::NSLOT - 1; c++)
    if ((e = issue(c)) != hipSuccess) return e;
  for (size_t c = 0; c < nch; c++) {
    const int sl = (int)(c % Staging::NSLOT);
    if ((e = hipEventSynchronize(g_staging.ev[sl])) != hipSuccess) return e;
    if (c + Staging::NSLOT - 1 < nch && (e = issue(c + Staging::NSLOT - 1)) != hipSuccess) return e;
    const size_t off = c * Staging::CHUNK, m = std::min(Staging::CHUNK, n - off);
    par_memcpy((uint8_t*)dst + off, g_staging.buf[sl], m);
  }
  return g_staging.before(stream);
}

// ---------------------------------------------------------------- device images
// Device-buffer layout of host arrays: offsets are assigned first (256-byte aligned, 16 zero bytes of slack after
// each array), then the buffer is zeroed on the device and every array goes up through the pinned ring
struct Packer {
  struct Part { size_t off; const void* src; size_t bytes; };
  std::vector<Part> parts;
  size_t size = 0;
  template <class V>
  size_t add(const V& v) {
    size_t off = (size + 255) & ~(size_t)255;
    size_t bytes = v.size() * sizeof(*v.data());
    parts.push_back({off, v.data(), bytes});
    size = off + bytes + 16;
    return off;
  }
  hipError_t copy_to(uint8_t* dev) const {
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(dev, 0, size, s);
    for (auto& q : parts)
      if (e == hipSuccess && q.bytes) e = staged_h2d(dev + q.off, q.src, q.bytes, s);
    hipError_t e2 = hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    return e != hipSuccess ? e : e2;
  }
};

struct DevRuleset {
  int device = -1;
  uint8_t* base = nullptr;
  size_t bytes = 0;
  size_t o_rules, o_filters, o_kinds, o_sels, o_reqs, o_pn, o_pe, o_leaves, o_atoms, o_metas, o_pss, o_pool, o_cnodes, o_conds, o_cprogs,
      o_gpats, o_gsets;
  hipModule_t jmod = nullptr;     // runtime-compiled walk kernels (jit.cpp) loaded on this device
  std::vector<hipFunction_t> jfns;  // kyv_jit_walk_<g> per rule group
  std::vector<hipFunction_t> ffns;  // kyv_jit_fused_<g> per rule group, or null (the group has no fused rule)
  std::vector<std::vector<hipFunction_t>> fparts, afparts;  // its further parts kyv_jit_fused_<g>p<1..> (KYV_FUSED_SPLIT)
  std::vector<hipFunction_t> fmfns, afmfns;  // kyv_jit_fusedm_<g>: the parts as one kernel (KYV_FUSED_MERGE), or null
  std::vector<hipFunction_t> jconds;  // [rule] kyv_jit_cond_<k> (compiled deny / foreach rule k) or null
  // compiled condition rules in kernel groups (jit_cond_groups): [group] kyv_jit_condg_<first rule>, its members,
  // the accounting build's kernel; [rule] its group or -1
  std::vector<hipFunction_t> jcg, ajcg;
  hipFunction_t jshapes = nullptr, ajshapes = nullptr;  // kyv_jit_shapes (pattern-shape tables) and its accounting build
  std::vector<std::vector<uint32_t>> jcg_members;
  std::vector<int32_t> jc_group;
  bool jloaded = false;
  // the byte-accounting build of the same kernels (KYV_ACCT), loaded only by an accounting evaluation
  hipModule_t amod = nullptr;
  std::vector<hipFunction_t> afns, aconds, affns;
  unsigned long long* acnt = nullptr;  // its counters (kyv_acct_bytes)
  bool aloaded = false;
};

// ---------------------------------------------------------------- per-batch device memory
// Batches come and go at serving rates (admission micro-batches of 1-4096 resources): hipMalloc / hipFree and
// stream creation per batch cost milliseconds (hipFree synchronises the device). Per-batch buffers therefore come
// from a caching pool per device (power-of-two size classes up to 256 MiB, exact above), and streams / events from
// a per-device free list. Buffers are returned only after the evaluation that used them has completed (every
// kyv_eval synchronises its stream before returning).
static std::mutex g_pool_mu;
struct PoolSlot { int dev; size_t cls; };
static std::vector<std::pair<PoolSlot, void*>> g_pool_free;   // cached buffers
static std::vector<std::pair<void*, PoolSlot>> g_pool_live;   // handed out
static constexpr size_t POOL_MAX_CACHED = 64;
static size_t pool_class(size_t n) {
  n = std::max<size_t>(n, 256);
  if (n > ((size_t)256 << 20)) return (n + ((size_t)1 << 20) - 1) & ~(((size_t)1 << 20) - 1);
  size_t c = 256;
  while (c < n) c <<= 1;
  return c;
}
static bool pool_off() {
  static const bool off = getenv("KYV_NO_POOL") && atoi(getenv("KYV_NO_POOL")) != 0;
  return off;
}
template <class T>
static hipError_t dmalloc(T** p, size_t n) {
  if (pool_off()) return hipMalloc((void**)p, std::max<size_t>(n, 1));
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const size_t cls = pool_class(n);
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    for (size_t i = 0; i < g_pool_free.size(); i++)
      if (g_pool_free[i].first.dev == dev && g_pool_free[i].first.cls == cls) {
        void* q = g_pool_free[i].second;
        g_pool_free.erase(g_pool_free.begin() + i);
        g_pool_live.push_back({q, PoolSlot{dev, cls}});
        *p = (T*)q;
        return hipSuccess;
      }
  }
  void* q = nullptr;
  e = hipMalloc(&q, cls);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(g_pool_mu);
  g_pool_live.push_back({q, PoolSlot{dev, cls}});
  *p = (T*)q;
  return hipSuccess;
}
static void dfree(void* q) {
  if (!q) return;
  std::lock_guard<std::mutex> g(g_pool_mu);
  for (size_t i = 0; i < g_pool_live.size(); i++)
    if (g_pool_live[i].first == q) {
      PoolSlot s = g_pool_live[i].second;
      g_pool_live.erase(g_pool_live.begin() + i);
      if (g_pool_free.size() < POOL_MAX_CACHED && s.cls <= ((size_t)256 << 20)) {
        g_pool_free.push_back({s, q});
      } else {
        int cur = 0;
        hipGetDevice(&cur);
        hipSetDevice(s.dev);
        hipFree(q);
        hipSetDevice(cur);
      }
      return;
    }
  hipFree(q);  // not from the pool
}
struct StreamSet { int dev; hipStream_t s; hipEvent_t e0, e1; };
static std::vector<StreamSet> g_streams_free;
static void stream_get(hipStream_t* s, hipEvent_t* e0, hipEvent_t* e1) {
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    for (size_t i = 0; i < g_streams_free.size(); i++)
      if (g_streams_free[i].dev == dev) {
        *s = g_streams_free[i].s; *e0 = g_streams_free[i].e0; *e1 = g_streams_free[i].e1;
        g_streams_free.erase(g_streams_free.begin() + i);
        return;
      }
  }
  HIP_OK(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
  HIP_OK(hipEventCreate(e0));
  HIP_OK(hipEventCreate(e1));
}
static void stream_put(int dev, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  if (!s) return;
  std::lock_guard<std::mutex> g(g_pool_mu);
  g_streams_free.push_back(StreamSet{dev, s, e0, e1});
}

// rules the light match kernel cannot evaluate: foreach, or a precondition / deny program with a JMESPath operand
static bool prog_jmes(const Ruleset& rs, uint32_t prog) {
  if (prog == NONE) return false;
  const CondProg& p = rs.cprogs[prog];
  // (length(<field chain>) runs in the light kernels too: kyv_cond.h jmes_len_cv)
  auto heavy = [&](const CondOperand& o) {
    return o.kind == OK_JMES && !jmes_chain_form(rs.pool.data() + o.a, o.nseg);
  };
  auto blk = [&](uint32_t c0, uint32_t n) {
    for (uint32_t i = 0; i < n; i++)
      if (heavy(rs.conds[c0 + i].key) || heavy(rs.conds[c0 + i].value)) return true;
    return false;
  };
  return blk(p.any0, p.nany == NONE ? 0u : p.nany) || blk(p.all0, p.nall);
}
static bool rule_needs_jmes(const Ruleset& rs, const RuleDesc& rd) {
  if (rd.kind == RK_FOREACH) return true;
  if (prog_jmes(rs, rd.pre)) return true;
  return rd.kind == RK_DENY && prog_jmes(rs, rd.root);
}

// One rule slice of an evaluation. Work lists, failing-path staging and compaction buffers are sized per (rule,
// resource) pair, so a ruleset whose buffers would not fit (C4: 10k+ rules x 1M resources) is evaluated as
// consecutive slices of its rule range [k0, k1) reusing one set of those buffers; verdict bytes, PSS masks and
// counters stay global. A ruleset that fits (C3) is one slice.
struct SliceSched {
  uint32_t k0 = 0, k1 = 0;
  size_t stage_tot = 0;          // staging slots (records) of the slice
  uint32_t* rbase = nullptr;     // [k1 - k0] first staging slot of each rule (slice-local)
  uint32_t* mrules = nullptr;    // rules of the slice the match phase evaluates (direct-walk rules excluded):
  uint32_t nmw = 0;              // leading rules of mrules on match_walk_generic_kernel (pattern rules: match only)
  uint32_t nmr = 0;              // pattern rules on match_rec_kernel, as staged match records (kyv_kernels.h MRec)
  MRec* mrec = nullptr;          // [nmr]
  uint32_t* mcls = nullptr;      // their kind index (MRecIndex): [nclass + 1] offsets into mcrec
  MRec* mcrec = nullptr;         // the records again, class by class
  uint32_t nclass = 0;
  uint8_t* tails = nullptr;      // lane tail facts of the records (TailTab): TailCfg, then the TailProgs
  uint32_t nmd = 0;              // then deny rules without JMESPath on match_deny_kernel
  uint32_t nmp = 0;              // then pattern rules with preconditions without JMESPath on match_pre_kernel
  uint32_t nmpj = 0;             // then those with JMESPath preconditions (no compiled kernel) on match_pre_kernel<.., true>
  uint32_t nm = 0, nmj = 0, nmc = 0;  // then [0, nm) light, [nm, nm + nmj) with JMESPath operands / foreach on the
                                 // interpreted match_kernel<true>, then nmc of those in the compiled kyv_jit_cond
  std::vector<uint32_t> ml, mj;  // host copies: light rules, JMESPath / foreach rules
  std::vector<uint3> pw;         // PodSecurity rules on pss_kernel: (rule, first match wave, waves)
  std::vector<uint3> cw;         // compiled condition rules: (rule, first match wave, waves) of its kernel's launch
  std::vector<uint32_t> cwm;     // [i] 0: cw[i] is a per-rule kernel; else the member mask of group cw[i].x
  uint2* sched = nullptr;        // chunk schedules of the two walk kernels (ChunkMap slots)
  std::vector<ChunkMap> cm;      // [0] interpreted walk kernel, [1 + g] runtime-compiled group g
  std::vector<uint8_t> fg;       // [g]: the slice has rules of group g on its fused kernel (kyv_jit_fused_<g>)
  std::vector<uint32_t> grid;
  hipEvent_t evs = nullptr;      // slice start (before its resets): phase 0 of every slice, not only the first
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // after match, condition, walk, compaction (phase timing)
  hipEvent_t cev[2] = {nullptr, nullptr};  // the slice's condition kernels on the condition stream (start, end)
  int jit_state = -1;            // what the schedules were laid out for (0 interpreter only, 1 with the jit kernel)
};

struct DeviceResults {
  uint8_t* status = nullptr;
  uint32_t* pss_fails = nullptr;
  uint32_t* pss_slot = nullptr;
  FailRec* recs = nullptr;       // compacted records of the current slice
  uint32_t* nrecs = nullptr;       // [3]: last slice's records, their offset, the evaluation's total (compact_top_kernel)
  bool recs_resident = false;       // the last evaluation's failing-path records are all in recs (a rule-sliced
                                    // evaluation with copy-back gathers them slice by slice into host_recs instead)
  std::vector<FailRec> host_recs;   // that host copy (export_failures serves it)
  FailRec* hrecs_dev = nullptr;     // its upload for an export (every slice's records: may exceed max_recs)
  size_t hrecs_cap = 0;
  FailRec* stage = nullptr;      // per-chunk staging of failing-path records (DevOut), sized for the largest slice
  uint16_t* rcnt = nullptr;
  uint32_t* tsum = nullptr;      // compaction tile sums / offsets
  uint32_t* tseg = nullptr;      // their segment totals / offsets (compact_scan_kernel)
  unsigned long long* counts = nullptr;
  size_t max_recs = 0;             // staging slots of the largest slice (d.stage)
  size_t recs_cap = 0;             // records d.recs holds (>= max_recs; grown between slices when a rule-sliced
                                   // evaluation's appended records could outgrow it)
  uint32_t npss = 0;
  size_t nres = 0, nrules = 0;
  size_t max_slice_rules = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  // the compiled condition kernels run on a second stream, concurrently with the walk (they write other rules'
  // verdict rows and read nothing the match / walk phases produce); joined before the verdict histogram
  hipStream_t cstream = nullptr;
  hipEvent_t cfork = nullptr, cjoin = nullptr;
  // the second and later runtime-compiled walk groups run on a third stream beside the first (independent rules:
  // own chunk schedules, verdict rows and staging slots), joined before the slice's compaction
  hipStream_t wstream = nullptr;
  hipEvent_t wfork = nullptr, wjoin = nullptr;
  View* view = nullptr;  // device copy of the View the kernel reads
  // pattern-shape tables (kyv_jit_shapes, round 5): [shape][res] verdict bytes and records, the per-class shape gate
  uint8_t* shape_st = nullptr;
  FailRec* shape_rec = nullptr;
  uint32_t* shape_gate = nullptr;
  uint32_t nshapes = 0, shape_words = 0;
  int shape_state = -1;  // what the shape gate was laid out for (0: no shapes, 1: the compiled kernels' shapes)
  // per-evaluation resource facts of the match records (facts_kernel): the ruleset-wide tail configuration, the table
  TailCfg* tcfg = nullptr;
  ResFacts* facts = nullptr;
  bool facts_on = false;
  WorkLists wl{};                // walk work lists (kyv_wave.h), slice-local rule index
  std::vector<SliceSched> slices;
  int cus = 256;
};

static void free_dev_results(DeviceResults& d, int dev) {
  dfree(d.view); dfree(d.status); dfree(d.pss_fails); dfree(d.pss_slot); dfree(d.recs); dfree(d.nrecs); dfree(d.counts);
  dfree(d.hrecs_dev);
  dfree(d.stage); dfree(d.rcnt); dfree(d.tsum); dfree(d.tseg);
  dfree(d.shape_st); dfree(d.shape_rec); dfree(d.shape_gate); dfree(d.tcfg); dfree(d.facts);
  dfree(d.wl.items); dfree(d.wl.cnt);
  for (auto& sl : d.slices) {
    dfree(sl.rbase); dfree(sl.mrules); dfree(sl.mrec); dfree(sl.mcls); dfree(sl.mcrec); dfree(sl.tails); dfree(sl.sched);
    if (sl.evs) hipEventDestroy(sl.evs);
    for (auto e : sl.ev) if (e) hipEventDestroy(e);
    for (auto e : sl.cev) if (e) hipEventDestroy(e);
  }
  stream_put(dev, d.stream, d.e0, d.e1);
  stream_put(dev, d.cstream, d.cfork, d.cjoin);
  stream_put(dev, d.wstream, d.wfork, d.wjoin);
  d = DeviceResults();
}

struct DevBatch {
  int device = -1;
  DeviceResults* out = nullptr;  // result buffers + stream, resident across evaluations
  uint8_t* base = nullptr;
  size_t bytes = 0;
  size_t o_nodes, o_hdr, o_faux, o_soff, o_slen, o_sflags, o_sdur, o_sqty, o_sf64, o_heap, o_nsloff, o_nslkv, o_gate,
      o_colv, o_coloff, o_pe, o_supper = SIZE_MAX, o_srx = SIZE_MAX;
  uint32_t* gmask = nullptr;   // [string][words] glob-mask bits, computed on the device once per batch
  uint32_t gmask_words = 0;
  uint32_t* inv = nullptr;     // input index -> kind-major position, and its inverse: uploaded by the first export
  uint32_t* order = nullptr;   // of device-resident results (export_status / export_failures)
  double upload_ms = 0;
  double gmask_ms = 0;  // glob-mask kernel of this batch (once per batch and device), HIP events
};

static DevRuleset* upload_ruleset(const Ruleset& rs, int device) {
  HIP_OK(hipSetDevice(device));
  auto* d = new DevRuleset();
  d->device = device;
  Packer p;
  d->o_rules = p.add(rs.rules);
  d->o_filters = p.add(rs.filters);
  d->o_kinds = p.add(rs.kinds);
  d->o_sels = p.add(rs.sels);
  d->o_reqs = p.add(rs.reqs);
  d->o_pn = p.add(rs.pnodes);
  d->o_pe = p.add(rs.pentries);
  d->o_leaves = p.add(rs.leaves);
  d->o_atoms = p.add(rs.atoms);
  d->o_metas = p.add(rs.metas);
  d->o_pss = p.add(rs.pss);
  d->o_pool = p.add(rs.pool);
  d->o_cnodes = p.add(rs.cnodes);
  d->o_conds = p.add(rs.conds);
  d->o_cprogs = p.add(rs.cprogs);
  d->o_gpats = p.add(rs.gpats);
  // condition sets for gmask_kernel: [nsets + 1] offsets into the sids that follow
  std::vector<uint32_t> gs(rs.gsets.size() + 1, 0);
  for (size_t q = 0; q < rs.gsets.size(); q++) gs[q + 1] = gs[q] + (uint32_t)rs.gsets[q].size();
  for (auto& st : rs.gsets) gs.insert(gs.end(), st.begin(), st.end());
  d->o_gsets = p.add(gs);
  d->bytes = p.size;
  HIP_OK(hipMalloc(&d->base, d->bytes));
  HIP_OK(p.copy_to(d->base));
  return d;
}

static DevBatch* upload_batch(const Batch& b, int device) {
  HIP_OK(hipSetDevice(device));
  auto t0 = std::chrono::steady_clock::now();
  auto* d = new DevBatch();
  d->device = device;
  Packer p;
  d->o_nodes = p.add(b.nodes);
  d->o_hdr = p.add(b.hdr);
  d->o_faux = p.add(b.faux);
  d->o_soff = p.add(b.str_off);
  d->o_slen = p.add(b.str_len);
  d->o_sflags = p.add(b.str_flags);
  d->o_sdur = p.add(b.str_dur);
  d->o_sqty = p.add(b.str_qty);
  d->o_sf64 = p.add(b.str_f64);
  d->o_heap = p.add(b.heap);
  d->o_nsloff = p.add(b.nsl_off);
  d->o_nslkv = p.add(b.nsl_kv);
  d->o_gate = p.add(b.gate);
  d->o_supper = b.str_upper.empty() ? SIZE_MAX : p.add(b.str_upper);
  d->o_srx = b.str_rx.empty() ? SIZE_MAX : p.add(b.str_rx);
  d->o_colv = p.add(b.colv);
  d->o_coloff = p.add(b.col_off);
  // batch-specialised copy of the pattern entries: `col` holds the column's absolute offset into colv, so the
  // walker reads a lookup's column without first reading the batch's column offset table
  std::vector<PEntry> pe = b.rs->pentries;
  for (auto& E : pe) if (E.col != NONE) E.col = b.col_off[E.col];
  d->o_pe = p.add(pe);
  d->bytes = p.size;
  HIP_OK(dmalloc(&d->base, d->bytes));
  HIP_OK(p.copy_to(d->base));
  d->upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return d;
}

static View make_view(const Ruleset& rs, const Batch& b, const uint8_t* rbase, const DevRuleset* dr, const uint8_t* bbase,
                      const DevBatch* db) {
  View v{};
  if (db) {
    v.nodes = (const Node*)(bbase + db->o_nodes);
    v.hdr = (const ResHeader*)(bbase + db->o_hdr);
    v.faux = (const FloatAux*)(bbase + db->o_faux);
    v.str_off = (const uint32_t*)(bbase + db->o_soff);
    v.str_len = (const uint32_t*)(bbase + db->o_slen);
    v.str_flags = (const uint32_t*)(bbase + db->o_sflags);
    v.str_dur = (const int64_t*)(bbase + db->o_sdur);
    v.str_qty = (const int64_t*)(bbase + db->o_sqty);
    v.str_f64 = (const double*)(bbase + db->o_sf64);
    v.heap = bbase + db->o_heap;
    v.nsl_off = (const uint32_t*)(bbase + db->o_nsloff);
    v.nsl_kv = (const uint32_t*)(bbase + db->o_nslkv);
    v.gate = (const uint32_t*)(bbase + db->o_gate);
    v.colv = (const uint64_t*)(bbase + db->o_colv);
    v.col_off = (const uint32_t*)(bbase + db->o_coloff);
    v.str_upper = db->o_supper == SIZE_MAX ? nullptr : (const uint32_t*)(bbase + db->o_supper);
    v.str_rx = db->o_srx == SIZE_MAX ? nullptr : (const uint32_t*)(bbase + db->o_srx);
    v.str_gmask = db->gmask;
    v.gmask_words = db->gmask_words;
  } else {
    v.str_gmask = nullptr;
    v.gmask_words = 0;
    v.nodes = b.nodes.data(); v.hdr = b.hdr.data(); v.faux = b.faux.data();
    v.str_off = b.str_off.data(); v.str_len = b.str_len.data(); v.str_flags = b.str_flags.data();
    v.str_dur = b.str_dur.data(); v.str_qty = b.str_qty.data(); v.str_f64 = b.str_f64.data();
    v.heap = b.heap.data(); v.nsl_off = b.nsl_off.data(); v.nsl_kv = b.nsl_kv.data();
    v.gate = b.gate.data();
    v.str_upper = b.str_upper.empty() ? nullptr : b.str_upper.data();
    v.str_rx = b.str_rx.empty() ? nullptr : b.str_rx.data();
    v.colv = b.colv.data();
    v.col_off = b.col_off.data();
  }
  v.gate_words = b.gate_words;
  v.nres = (uint32_t)b.hdr.size();
  v.nrules = (uint32_t)rs.rules.size();
  if (dr) {
    v.rules = (const RuleDesc*)(rbase + dr->o_rules);
    v.filters = (const Filter*)(rbase + dr->o_filters);
    v.kinds = (const KindDesc*)(rbase + dr->o_kinds);
    v.sels = (const SelDesc*)(rbase + dr->o_sels);
    v.reqs = (const SelReq*)(rbase + dr->o_reqs);
    v.pn = (const PNode*)(rbase + dr->o_pn);
    v.pe = (const PEntry*)(rbase + dr->o_pe);
    v.leaves = (const Leaf*)(rbase + dr->o_leaves);
    v.atoms = (const Atom*)(rbase + dr->o_atoms);
    v.metas = (const MetaSite*)(rbase + dr->o_metas);
    v.pss = (const PssDesc*)(rbase + dr->o_pss);
    v.pool = (const uint32_t*)(rbase + dr->o_pool);
    v.cnodes = (const Node*)(rbase + dr->o_cnodes);
    v.conds = (const Cond*)(rbase + dr->o_conds);
    v.cprogs = (const CondProg*)(rbase + dr->o_cprogs);
  } else {
    v.rules = rs.rules.data(); v.filters = rs.filters.data(); v.kinds = rs.kinds.data(); v.sels = rs.sels.data();
    v.reqs = rs.reqs.data(); v.pn = rs.pnodes.data(); v.pe = rs.pentries.data(); v.leaves = rs.leaves.data();
    v.atoms = rs.atoms.data(); v.metas = rs.metas.data(); v.pss = rs.pss.data(); v.pool = rs.pool.data();
    v.cnodes = rs.cnodes.data(); v.conds = rs.conds.data(); v.cprogs = rs.cprogs.data();
  }
  if (db) v.pe = (const PEntry*)(bbase + db->o_pe);  // device: entries with absolute column offsets
  return v;
}

// ---------------------------------------------------------------- kernels
// match_kernel, match_rec_kernel, pss_kernel, walk_kernel: kyv_kernels.h

// Gather the staged failing-path records of every walk chunk into one dense list, without atomics:
//   compact_sum_kernel   one wave per 64 consecutive chunks: the tile's record total;
//   compact_scan_kernel  exclusive prefix over the tiles, per segment of SCAN_SEG tiles, and the segment totals;
//   compact_top_kernel   exclusive prefix of the segment totals and the grand total;
//   compact_copy_kernel  one wave per tile: wave prefix of the chunks' counts, then the wave copies each
//                        non-empty chunk's records cooperatively (lane i moves record i).
__device__ __forceinline__ const FailRec* chunk_stage(const FailRec* stage, const uint32_t* rbase, const RuleDesc* rules,
                                                      uint32_t nwaves, size_t c) {
  // c: slice-local chunk (rule k - k0, wave w); `rules` and `rbase` are offset to the slice
  const uint32_t k = (uint32_t)(c / nwaves), w = (uint32_t)(c % nwaves);
  const uint32_t alts = rules[k].kind == RK_PATTERN ? 1u : min(rules[k].nalts, (uint32_t)MAX_ALTS);
  return stage + rbase[k] + (size_t)w * WAVE * alts;
}
__global__ void __launch_bounds__(WAVE) compact_sum_kernel(const uint16_t* __restrict__ rcnt, size_t total,
                                                           uint32_t* __restrict__ tsum) {
  const size_t c = (size_t)blockIdx.x * WAVE + threadIdx.x;
  uint32_t n = c < total ? rcnt[c] : 0u;
  for (int off = WAVE / 2; off > 0; off >>= 1) n += __shfl_xor(n, off);
  if (threadIdx.x == 0) tsum[blockIdx.x] = n;
}
// exclusive prefix over `n` values in place, one workgroup: rounds of 8192 consecutive values (each thread scans 8,
// wave inclusive scans of the thread totals, a scan of the 16 wave totals, carry across rounds); returns the total
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t* __restrict__ x0, uint32_t n) {
  __shared__ uint32_t wsum[16];
  constexpr uint32_t PER = 8;
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1), w = t / WAVE;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < n; base += 1024 * PER) {
    const uint32_t i0 = base + t * PER;
    uint32_t x[PER], tot = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) { x[q] = i0 + q < n ? x0[i0 + q] : 0u; tot += x[q]; }
    uint32_t v = tot;
    for (int off = 1; off < WAVE; off <<= 1) {
      const uint32_t y = __shfl_up(v, off);
      if ((int)lane >= off) v += y;
    }
    if (lane == WAVE - 1) wsum[w] = v;
    __syncthreads();
    if (w == 0) {
      uint32_t s2 = lane < 16 ? wsum[lane] : 0u;
      for (int off = 1; off < 16; off <<= 1) {
        const uint32_t y = __shfl_up(s2, off);
        if ((int)lane >= off) s2 += y;
      }
      if (lane < 16) wsum[lane] = s2;
    }
    __syncthreads();
    uint32_t run = carry + (w ? wsum[w - 1] : 0u) + v - tot;  // exclusive offset of this thread's first value
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) {
      if (i0 + q < n) x0[i0 + q] = run;
      run += x[q];
    }
    carry += wsum[15];
    __syncthreads();
  }
  return carry;
}
// tile prefix, two levels (round 5: one workgroup over every tile took 0.39 ms per C4 slice): each workgroup scans one
// segment of SCAN_SEG tiles in place and leaves the segment total; compact_top_kernel scans the segment totals and
// writes the grand total; the copy adds its segment's offset
constexpr uint32_t SCAN_SEG = 8192;
__global__ void __launch_bounds__(1024) compact_scan_kernel(uint32_t* __restrict__ tsum, uint32_t ntiles,
                                                            uint32_t* __restrict__ seg) {
  const uint32_t base = blockIdx.x * SCAN_SEG;
  const uint32_t n = ntiles - base < SCAN_SEG ? ntiles - base : SCAN_SEG;
  const uint32_t tot = block_exclusive_scan(tsum + base, n);
  if (threadIdx.x == 0) seg[blockIdx.x] = tot;
}
// nout[0]: the slice's record count; nout[1]: where its records start in the output (0, or with `accumulate` the
// records of the evaluation's earlier slices: a rule-sliced evaluation keeps every slice's records resident, one
// dense list); nout[2]: the running total
__global__ void __launch_bounds__(1024) compact_top_kernel(uint32_t* __restrict__ seg, uint32_t nseg,
                                                           uint32_t* __restrict__ nout, uint32_t accumulate) {
  const uint32_t tot = block_exclusive_scan(seg, nseg);
  if (threadIdx.x == 0) {
    const uint32_t b = accumulate ? nout[2] : 0u;
    nout[0] = tot;
    nout[1] = b;
    nout[2] = b + tot;
  }
}
// one wave per tile of 64 chunks: every lane copies records i = lane, lane + 64, ... of the tile (the chunk of record
// i found by a binary search over the wave's inclusive prefix of the chunk counts), so all loads are independent
__global__ void __launch_bounds__(WAVE) compact_copy_kernel(const FailRec* __restrict__ stage, const uint32_t* __restrict__ rbase,
                                                            const uint16_t* __restrict__ rcnt, const RuleDesc* __restrict__ rules,
                                                            uint32_t nwaves, size_t total, const uint32_t* __restrict__ tbase,
                                                            const uint32_t* __restrict__ seg, FailRec* __restrict__ out,
                                                            size_t max_out, uint32_t k0, const uint32_t* __restrict__ nout) {
  const uint32_t lane = threadIdx.x;
  const size_t c = (size_t)blockIdx.x * WAVE + lane;
  const uint32_t n = c < total ? rcnt[c] : 0u;
  uint32_t pre = n;  // inclusive wave prefix
  for (int off = 1; off < WAVE; off <<= 1) {
    uint32_t y = __shfl_up(pre, off);
    if ((int)lane >= off) pre += y;
  }
  const uint32_t T = __shfl(pre, WAVE - 1);
  if (T == 0) return;
  // the prefix and each chunk's staging address in LDS: the per-record search below runs with part of the wave
  // masked off (cross-lane reads from inactive lanes are undefined), and a record then needs no rule / rbase loads
  __shared__ uint32_t spre[WAVE];
  __shared__ const FailRec* ssrc[WAVE];
  __shared__ uint32_t skw[WAVE];  // (global rule, match wave, wide): what a 16-byte StageRec leaves implicit
  __shared__ uint32_t sw[WAVE];
  spre[lane] = pre;
  ssrc[lane] = n ? chunk_stage(stage, rbase, rules, nwaves, c) : nullptr;
  if (n) {
    const uint32_t k = (uint32_t)(c / nwaves);
    skw[lane] = (k + k0) | (rules[k].uses_meta ? 0x80000000u : 0u);
    sw[lane] = (uint32_t)(c % nwaves);
  }
  __syncthreads();
  const size_t base = (size_t)nout[1] + tbase[blockIdx.x] + seg[blockIdx.x / SCAN_SEG];
  // one record per lane: whole FailRecs of wide chunks copied, StageRecs expanded; stores of consecutive lanes are
  // consecutive 32-byte records
  for (uint32_t i = lane; i < T; i += WAVE) {
    uint32_t lo = 0, hi = WAVE - 1;  // smallest j with pre[j] > i
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (spre[mid] > i) hi = mid; else lo = mid + 1;
    }
    const uint32_t j = lo;
    const uint32_t first = j ? spre[j - 1] : 0u;
    if (base + i >= max_out) continue;
    uint4* dst = reinterpret_cast<uint4*>(out + base + i);
    const uint32_t kw = skw[j];
    if (kw & 0x80000000u) {
      const uint4* src = reinterpret_cast<const uint4*>(ssrc[j] + (i - first));
      dst[0] = src[0];
      dst[1] = src[1];
    } else {
      const uint4 s = reinterpret_cast<const uint4*>(ssrc[j])[i - first];  // StageRec
      FailRec f;
      f.res = sw[j] * WAVE + (s.y & (WAVE - 1));
      f.rule = kw;
      f.tmpl = s.x;
      f.alt = (uint16_t)(s.y >> 8);
      f.nalt = 0;
      f.idx[0] = (uint16_t)s.z; f.idx[1] = (uint16_t)(s.z >> 16);
      f.idx[2] = (uint16_t)s.w; f.idx[3] = (uint16_t)(s.w >> 16);
      f.key[0] = NONE;
      f.key[1] = NONE;
      const uint4* fp = reinterpret_cast<const uint4*>(&f);
      dst[0] = fp[0];
      dst[1] = fp[1];
    }
  }
}

// Verdict totals: one histogram pass over the [rule][res] status bytes after both phases (the verdict bytes are
// complete there: ST_NONE preset, every decided pair written once). Statuses are 0..7, so a 32-bit word holds four
// 3-bit values and the bytes equal to s are the zero bytes of word ^ (s * 0x01010101). Per thread u32 tallies,
// block reduction in LDS, one atomic per block and status (a few hundred blocks: no hot-address queue).
constexpr int HIST_BLOCK = 256;
__device__ __forceinline__ uint32_t bytes_eq(uint32_t w, uint32_t s) {
  const uint32_t x = w ^ (s * 0x01010101u);
  return 4u - (uint32_t)__popc((x | (x >> 1) | (x >> 2)) & 0x01010101u);
}
__global__ void __launch_bounds__(HIST_BLOCK) status_hist_kernel(const uint8_t* __restrict__ status, size_t nres,
                                                                 unsigned long long* __restrict__ counts) {
  // blockIdx.y = rule: its verdict row is status[k * nres, (k + 1) * nres); per-rule totals feed the report
  // summaries (CalculateSummary, pkg/utils/report/results.go:38-54), their sum the evaluation's verdict counts
  __shared__ uint32_t part[HIST_BLOCK / WAVE][NSTATUS];
  uint32_t c[NSTATUS] = {0};
  const uint8_t* row = status + (size_t)blockIdx.y * nres;
  size_t head = (16 - ((size_t)row & 15)) & 15;
  if (head > nres) head = nres;
  const size_t nv = (nres - head) / 16, tail0 = head + nv * 16, stride = (size_t)gridDim.x * HIST_BLOCK;
  const kyv_u32x4* s4 = (const kyv_u32x4*)(row + head);
  for (size_t i = (size_t)blockIdx.x * HIST_BLOCK + threadIdx.x; i < nv; i += stride) {
    const kyv_u32x4 q = __builtin_nontemporal_load(s4 + i);
#pragma unroll
    for (uint32_t s = 1; s < NSTATUS; s++) c[s] += bytes_eq(q.x, s) + bytes_eq(q.y, s) + bytes_eq(q.z, s) + bytes_eq(q.w, s);
  }
  if (blockIdx.x == 0 && threadIdx.x < head + (nres - tail0)) {  // unaligned head / tail bytes (< 32)
    const size_t at = threadIdx.x < head ? threadIdx.x : tail0 + (threadIdx.x - head);
    const uint32_t b = row[at] & 7u;
#pragma unroll
    for (uint32_t s = 1; s < NSTATUS; s++) c[s] += b == s;
  }
#pragma unroll
  for (uint32_t s = 1; s < NSTATUS; s++) {
    uint32_t x = c[s];
    for (int off = WAVE / 2; off > 0; off >>= 1) x += __shfl_xor(x, off);
    c[s] = x;
  }
  const uint32_t lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
  if (lane == 0)
    for (uint32_t s = 1; s < NSTATUS; s++) part[wv][s] = c[s];
  __syncthreads();
  if (threadIdx.x > 0 && threadIdx.x < NSTATUS) {
    uint32_t t = 0;
    for (int j = 0; j < HIST_BLOCK / WAVE; j++) t += part[j][threadIdx.x];
    if (t) atomicAdd(&counts[(size_t)blockIdx.y * NSTATUS + threadIdx.x], (unsigned long long)t);
  }
}

// wildcard.Match(pattern g, string s) for every dictionary string (one thread each) and masked pattern; then the
// FETCH_SIZE calibration (bench.py KYV_CALIB=1, scripts/pmc_summary.py): streaming reads of a known byte count at W
// bytes per lane (coalesced, grid-stride), and a gather of 16-byte rows (every row once, in a scrambled order) -- the
// guide leaves these access widths uncalibrated (MI355X_MICROARCH.md, HBM), and the walk's reads are 8-byte column
// entries, 16-byte node rows and 4-byte fields
template <int W>
__global__ void __launch_bounds__(256) calib_read_kernel(const uint8_t* __restrict__ p, size_t n, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x * W;
  for (size_t off = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * W; off + W <= n; off += stride) {
    if constexpr (W == 4) {
      acc ^= *(const uint32_t*)(p + off);
    } else if constexpr (W == 8) {
      const uint2 x = *(const uint2*)(p + off);
      acc ^= x.x ^ x.y;
    } else {
      const uint4 x = *(const uint4*)(p + off);
      acc ^= x.x ^ x.y ^ x.z ^ x.w;
    }
  }
  if (acc == 0x9E3779B9u) out[0] = acc;  // (keeps the loads)
}
__global__ void __launch_bounds__(256) calib_gather_kernel(const uint4* __restrict__ rows, size_t nrows,
                                                           uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrows; i += stride) {
    const size_t j = (i * 0x9E3779B97F4A7C15ull) & (nrows - 1);  // odd multiplier mod 2^k: a permutation of the rows
    const uint4 x = rows[j];
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

// condition sets (compiler.cpp assign_cond_sets): bit ng + q = wild2(s, e) for some literal e of set q (kyv_cond.h wild2,
// both match directions)
__global__ void __launch_bounds__(256) gmask_kernel(const View* __restrict__ vp, const uint32_t* __restrict__ gpats,
                                                    uint32_t ng, const uint32_t* __restrict__ gsets, uint32_t nsets,
                                                    uint32_t nstr, uint32_t words, uint32_t* __restrict__ out) {
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  if (s >= nstr) return;
  const View& v = *vp;
  for (uint32_t w = 0; w < words; w++) {
    uint32_t bits = 0;
    for (uint32_t b = 32 * w; b < ng + nsets && b < 32 * w + 32; b++) {
      bool hit = false;
      if (b < ng) {
        hit = glob_sid_raw(v, gpats[b], s);
      } else {
        const uint32_t q = b - ng;
        for (uint32_t i = gsets[q]; i < gsets[q + 1] && !hit; i++) {
          const uint32_t e = gsets[nsets + 1 + i];
          hit = glob_sid_raw(v, e, s) || glob_sid_raw(v, s, e);
        }
      }
      if (hit) bits |= 1u << (b - 32 * w);
    }
    out[(size_t)s * words + w] = bits;
  }
}

// ---------------------------------------------------------------- host entry
// Frames the walk of one pattern node can push (eval_pattern): a map frame stays while its entries are
// walked, array frames while their elements are, an existence frame while its candidates are.
int pattern_depth(const Ruleset& rs, uint32_t pn, int guard) {
  if (pn == NONE || guard > MAX_DEPTH) return MAX_DEPTH + 1;
  const PNode& P = rs.pnodes[pn];
  int d = 0;
  switch (P.kind) {
    case P_MAP:
      for (uint32_t e = 0; e < P.n; e++) {
        const PEntry& E = rs.pentries[P.first + e];
        if (E.handler == H_STAR || E.handler == H_NEGATION || E.child == NONE) continue;
        if (E.handler == H_EXISTENCE || E.handler == H_EXIST_BADPAT) {
          uint32_t npat = rs.pool[E.child];
          for (uint32_t j = 0; j < npat; j++) d = std::max(d, 1 + pattern_depth(rs, rs.pool[E.child + 1 + j], guard + 2));
        } else {
          d = std::max(d, pattern_depth(rs, E.child, guard + 1));
        }
      }
      return 1 + d;
    case P_ARR_MAPS: return 1 + pattern_depth(rs, P.first, guard + 1);
    case P_ARR_POS:
      for (uint32_t i = 0; i < P.n; i++) d = std::max(d, pattern_depth(rs, rs.pool[P.first + i], guard + 1));
      return 1 + d;
    default: return 0;
  }
}

// LDS frames per lane: the deepest compiled pattern (clamped; deeper walks end in ST_FALLBACK at run time)
static int ruleset_depth(const Ruleset& rs) {
  int d = 1;
  for (auto& rd : rs.rules) {
    if (rd.kind == RK_PATTERN) d = std::max(d, pattern_depth(rs, rd.root, 0));
    else if (rd.kind == RK_ANYPATTERN)
      for (uint32_t a = 0; a < rd.nalts; a++) d = std::max(d, pattern_depth(rs, rs.pool[rd.root + a], 0));
  }
  return std::min(d, (int)MAX_DEPTH);
}


// GPU evaluation of every (resource, rule) pair. Device images, result buffers and the stream stay resident
// per batch; `copy_back` false keeps the verdicts on the device (bench mode).
// Compile (once per ruleset) and load (once per device) the ruleset's walk kernel; false if unavailable.
static std::mutex g_jit_mu;
static void mrs_clear_shapes(Ruleset& rs) {  // no shape kernel: every pattern rule walks
  std::fill(rs.jit_shape.begin(), rs.jit_shape.end(), (uint16_t)0);
  rs.jit_nshapes = 0;
}
static bool ensure_jit(Ruleset& rs, DevRuleset* dr) {
  if (dr->jloaded) return true;
  std::lock_guard<std::mutex> lk(g_jit_mu);
  if (!rs.jit_tried) {
    rs.jit_tried = true;
    try {
      std::string src = jit_source(rs, &rs.jit_rules, &rs.jit_cond, &rs.jit_shape);
      rs.jit_nshapes = 0;
      for (auto x : rs.jit_shape) rs.jit_nshapes = std::max<uint32_t>(rs.jit_nshapes, x);
      bool any = false;
      for (auto x : rs.jit_rules) any |= x != 0;
      for (auto x : rs.jit_cond) any |= x != 0;
      if (any) rs.jit_code = jit_compile(src, &rs.jit_compile_s);
    } catch (std::exception& e) {
      rs.jit_error = e.what();
      rs.jit_code.clear();
      fprintf(stderr, "[kyvgpu] runtime-compiled walk kernel unavailable, using the interpreted one: %s\n", e.what());
    }
  }
  if (rs.jit_code.empty()) return false;
  HIP_OK(hipModuleLoadData(&dr->jmod, rs.jit_code.data()));
  uint32_t ng = 0;
  for (auto x : rs.jit_rules) ng = std::max<uint32_t>(ng, x);
  dr->jfns.resize(ng);
  dr->ffns.assign(ng, nullptr);
  for (uint32_t g = 0; g < ng; g++) {
    HIP_OK(hipModuleGetFunction(&dr->jfns[g], dr->jmod, ("kyv_jit_walk_" + std::to_string(g)).c_str()));
    if (hipModuleGetFunction(&dr->ffns[g], dr->jmod, ("kyv_jit_fused_" + std::to_string(g)).c_str()) != hipSuccess)
      dr->ffns[g] = nullptr;
    dr->fparts.resize(ng);
    for (int p = 1; dr->ffns[g]; p++) {
      hipFunction_t f = nullptr;
      if (hipModuleGetFunction(&f, dr->jmod, ("kyv_jit_fused_" + std::to_string(g) + "p" + std::to_string(p)).c_str()) != hipSuccess)
        break;
      dr->fparts[g].push_back(f);
    }
    dr->fmfns.resize(ng, nullptr);
    if (hipModuleGetFunction(&dr->fmfns[g], dr->jmod, ("kyv_jit_fusedm_" + std::to_string(g)).c_str()) != hipSuccess)
      dr->fmfns[g] = nullptr;
  }
  (void)hipGetLastError();
  dr->jshapes = nullptr;
  if (rs.jit_nshapes && hipModuleGetFunction(&dr->jshapes, dr->jmod, "kyv_jit_shapes") != hipSuccess) {
    dr->jshapes = nullptr;
    mrs_clear_shapes(rs);
  }
  (void)hipGetLastError();
  dr->jconds.assign(rs.rules.size(), nullptr);
  dr->jc_group.assign(rs.rules.size(), -1);
  dr->jcg.clear();
  dr->jcg_members.clear();
  {
    std::vector<uint32_t> crules;
    for (size_t k = 0; k < rs.jit_cond.size(); k++) if (rs.jit_cond[k] == 1) crules.push_back((uint32_t)k);
    for (auto& grp : jit_cond_groups(rs, crules)) {
      hipFunction_t f = nullptr;
      if (hipModuleGetFunction(&f, dr->jmod, ("kyv_jit_condg_" + std::to_string(grp[0])).c_str()) != hipSuccess) continue;
      for (uint32_t k : grp) dr->jc_group[k] = (int32_t)dr->jcg.size();
      dr->jcg.push_back(f);
      dr->jcg_members.push_back(grp);
    }
    (void)hipGetLastError();
  }
  for (size_t k = 0; k < rs.jit_cond.size(); k++)
    if (rs.jit_cond[k] == 1 && dr->jc_group[k] < 0)
      HIP_OK(hipModuleGetFunction(&dr->jconds[k], dr->jmod, ("kyv_jit_cond_" + std::to_string(k)).c_str()));
  dr->jloaded = true;
  return true;
}

// The accounting build of the loaded kernels (same generated source, -DKYV_ACCT): compiled (or taken from the code-object
// cache) and loaded on first use; false when the product kernels are not the compiled ones
static bool ensure_jit_acct(Ruleset& rs, DevRuleset* dr) {
  if (dr->aloaded) return true;
  if (!ensure_jit(rs, dr)) return false;
  std::lock_guard<std::mutex> lk(g_jit_mu);
  if (rs.jit_code_acct.empty()) {
    std::vector<uint8_t> jr, jc;
    rs.jit_code_acct = jit_compile(jit_source(rs, &jr, &jc), nullptr, true);
  }
  HIP_OK(hipModuleLoadData(&dr->amod, rs.jit_code_acct.data()));
  dr->afns.resize(dr->jfns.size());
  dr->affns.assign(dr->jfns.size(), nullptr);
  for (size_t g = 0; g < dr->jfns.size(); g++) {
    HIP_OK(hipModuleGetFunction(&dr->afns[g], dr->amod, ("kyv_jit_walk_" + std::to_string(g)).c_str()));
    if (dr->ffns[g]) HIP_OK(hipModuleGetFunction(&dr->affns[g], dr->amod, ("kyv_jit_fused_" + std::to_string(g)).c_str()));
    dr->afparts.resize(dr->jfns.size());
    dr->afparts[g].assign(g < dr->fparts.size() ? dr->fparts[g].size() : 0, nullptr);
    for (size_t p = 0; p < dr->afparts[g].size(); p++)
      HIP_OK(hipModuleGetFunction(&dr->afparts[g][p], dr->amod,
                                  ("kyv_jit_fused_" + std::to_string(g) + "p" + std::to_string(p + 1)).c_str()));
    dr->afmfns.resize(dr->jfns.size(), nullptr);
    if (g < dr->fmfns.size() && dr->fmfns[g])
      HIP_OK(hipModuleGetFunction(&dr->afmfns[g], dr->amod, ("kyv_jit_fusedm_" + std::to_string(g)).c_str()));
  }
  dr->aconds.assign(dr->jconds.size(), nullptr);
  for (size_t k = 0; k < dr->jconds.size(); k++)
    if (dr->jconds[k]) HIP_OK(hipModuleGetFunction(&dr->aconds[k], dr->amod, ("kyv_jit_cond_" + std::to_string(k)).c_str()));
  dr->ajshapes = nullptr;
  if (dr->jshapes) HIP_OK(hipModuleGetFunction(&dr->ajshapes, dr->amod, "kyv_jit_shapes"));
  dr->ajcg.assign(dr->jcg.size(), nullptr);
  for (size_t g = 0; g < dr->jcg.size(); g++)
    HIP_OK(hipModuleGetFunction(&dr->ajcg[g], dr->amod, ("kyv_jit_condg_" + std::to_string(dr->jcg_members[g][0])).c_str()));
  hipDeviceptr_t p = nullptr;
  size_t bytes = 0;
  HIP_OK(hipModuleGetGlobal(&p, &bytes, dr->amod, "kyv_acct_bytes"));
  dr->acnt = (unsigned long long*)p;
  dr->aloaded = true;
  return true;
}

// Walk-buffer bytes one rule costs per resource: its work-list slot (8 B), failing-path staging and compacted
// records (32 B each per anyPattern alternative), plus per-chunk counters.
static size_t rule_slice_bytes(const RuleDesc& rd) {
  const size_t alts = rd.kind == RK_PATTERN ? 1 : rd.kind == RK_ANYPATTERN ? std::min<uint32_t>(rd.nalts, MAX_ALTS) : 0;
  return sizeof(uint2) + 2 * alts * sizeof(FailRec) + 1;
}

// Budget for the per-slice buffers: KYV_SLICE_MB, else half of the free device memory, at most 128 GiB (288 GB of
// HBM3E: C3 at 10 M resources is one slice, 56 GB; each further slice re-reads the headers and kind gates of every
// match wave in the fused walk -- C3 walk 8.11 ms in two slices, 7.92 in one, r4 A/B)
static size_t slice_budget() {
  if (const char* e = getenv("KYV_SLICE_MB")) return (size_t)std::max(1, atoi(e)) << 20;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr == 0) fr = (size_t)64 << 30;
  return std::min<size_t>(fr / 2, (size_t)128 << 30);
}

// Lay out the chunk schedules of one slice's walk kernels (see ChunkMap): runs of match waves with equal gated rule
// sets, wave-major within a run, whole waves placed on one XCD.
// The staged match record of match_walk rule q (kyv_kernels.h MRec): MR_FAST when its match block fits the record
// (compiled, no PolicyException candidates, at most MREC_F filters, 4 kinds, 2 names and 2 namespaces per filter,
// every wildcard pattern with a glob-mask bit); else match_walk_generic_kernel runs pair_match for it
static void build_mrec(const Ruleset& rs, uint32_t q, const std::vector<uint32_t>& gidx, bool masks_on, bool on, MRec& R) {
  memset(&R, 0, sizeof R);
  const RuleDesc& rd = rs.rules[q];
  R.k = q;
  R.kind = rd.kind;
  R.flags = rd.flags;
  bool fast = on && rd.match.mode != MM_NONE && rd.exc == NONE && rd.match.nfilters + rd.exclude.nfilters <= MREC_F;
  bool uses = false;
  auto pat = [&](uint32_t sid) -> uint32_t {  // glob_sid's classification (kyv_eval.h), by the string's content
    if (sid >= rs.dict.strs.size()) { fast = false; return 0; }
    const std::string& x = rs.dict.strs[sid];
    bool globby = x.find_first_of("*?") != std::string::npos;
    for (unsigned char ch : x) if (ch >= 0x80) globby = true;
    if (!globby) {
      if (sid & PAT_MASK) fast = false;
      return sid;
    }
    uses = true;
    const uint32_t g = gidx[sid];
    if (!g || g > 0xFFu || !masks_on) { fast = false; return 0; }
    return PAT_MASK | g;
  };
  auto fill = [&](uint32_t fi, MRecFilter& F) {
    const Filter& f = rs.filters[fi];
    F.idx = fi;
    if (f.nkinds > 4 || f.nnames > 2 || f.nnss > 2) { fast = false; return; }
    uint32_t b = (uint32_t)f.flags | ((uint32_t)f.nkinds << 16) | (f.nnames << 19) | ((f.name != NONE ? 1u : 0u) << 21) |
                 (f.nnss << 22);
    for (uint32_t i = 0; i < f.nkinds; i++) {
      const KindDesc& kd = rs.kinds[f.kinds + i];
      F.kinds[i] = kd.kind;
      if (kd.kind != NONE && kd.gv_mode != 0) b |= 1u << (24 + i);
    }
    if (f.name != NONE) F.pats[0] = pat(f.name);
    for (uint32_t i = 0; i < f.nnames; i++) F.pats[1 + i] = pat(rs.pool[f.names + i]);
    for (uint32_t i = 0; i < f.nnss; i++) F.pats[3 + i] = pat(rs.pool[f.nss + i]);
    if (f.nann || (f.flags & (FF_HAS_SEL | FF_HAS_NSSEL))) b |= 1u << 28;
    F.bits = b;
  };
  if (fast) {
    for (uint32_t i = 0; i < rd.match.nfilters; i++) fill(rd.match.filters + i, R.f[i]);
    for (uint32_t i = 0; i < rd.exclude.nfilters; i++) fill(rd.exclude.filters + i, R.f[rd.match.nfilters + i]);
  }
  R.bits = (fast ? MR_FAST : 0u) | (uses ? MR_MASKS : 0u) | (rd.empty_may_match ? MR_EMPTY : 0u) | ((uint32_t)rd.match.mode << 8) |
           ((uint32_t)rd.exclude.mode << 16) | (fast ? (rd.match.nfilters << 24) | (rd.exclude.nfilters << 28) : 0u);
}

// glob-mask index + 1 of every dictionary string that is a ruleset wildcard pattern (0: none)
static std::vector<uint32_t> glob_index(const Ruleset& rs) {
  std::vector<uint32_t> gidx(rs.dict.strs.size(), 0);
  for (size_t g = 0; g < rs.gpats.size(); g++) if (rs.gpats[g] < gidx.size()) gidx[rs.gpats[g]] = (uint32_t)g + 1;
  return gidx;
}
static bool mrec_masks_on() { static const bool on = !getenv("KYV_NO_GMASK"); return on; }
static bool mrec_recs_on() { static const bool on = !getenv("KYV_MREC") || atoi(getenv("KYV_MREC")) != 0; return on; }
static bool mrec_kernel_on() {
  static const bool on = !getenv("KYV_MATCHW_KERNEL") || atoi(getenv("KYV_MATCHW_KERNEL")) != 0;
  return on;
}
// 1 + the pattern shape whose tables decide rule q's matched pairs in match_rec_kernel (0: the rule walks): a shape
// rule of the compiled kernels (jit.cpp jit_shape_eligible) whose match block fits a staged record
static uint32_t served_shape(const Ruleset& rs, uint32_t q, const std::vector<uint32_t>& gidx, bool jit) {
  if (!jit || !mrec_kernel_on() || q >= rs.jit_shape.size() || !rs.jit_shape[q]) return 0;
  const RuleDesc& rd = rs.rules[q];
  if (rd.pre != NONE || rd.kind != RK_PATTERN || (rd.flags & RD_GATE_EXACT) || rule_needs_jmes(rs, rd)) return 0;
  MRec R;
  build_mrec(rs, q, gidx, mrec_masks_on(), mrec_recs_on(), R);
  return (R.bits & MR_FAST) ? rs.jit_shape[q] : 0u;
}

// A kind-class copy of a match record (round 5): every resource of the class has the same GVK kind, so a filter's
// kinds test (condition_block's checkKind, kyv_eval.h) is a constant of the copy unless a kind of the filter carries a
// group / version refinement. A filter whose kinds accept the class loses the test (no kinds: every kind); one whose
// kinds can never accept it is removed when that cannot change the outcome -- a match filter of an ANY block or an
// exclude filter of an ANY / plain block (it never contributes, and a filter rejected on its kinds raises no
// nondeterminism); an ALL exclude block with such a filter can never exclude and is dropped whole. The empty-OldResource
// retry evaluated on the device (MR_EMPTY without a constant outcome) compares kinds against the empty resource: such
// records keep their filters.
static void fold_kinds(MRec& R, uint32_t ck, size_t* nfold, size_t* ndrop) {
  if ((R.bits & MR_EMPTY) && !(R.bits & MR_ECONST)) return;
  const uint32_t mm = (R.bits >> 8) & 0xFFu, em = (R.bits >> 16) & 0xFFu;
  uint32_t nmf = (R.bits >> 24) & 0xFu, nef = R.bits >> 28;
  MRecFilter out[MREC_F];
  uint32_t no = 0, omf = 0, oef = 0;
  bool drop_excl = false;
  bool excl_tail = false;  // an exclude filter ahead of this one has a tail (selector / annotations: it can raise ND)
  for (uint32_t j = 0; j < nmf + nef; j++) {
    MRecFilter F = R.f[j];
    const bool ism = j < nmf;
    const uint32_t nk = (F.bits >> 16) & 7u;
    int acc = -1;  // 1: the kinds accept the class, 0: they never do, -1: it depends on the resource (group / version)
    if (nk && !(F.bits & FF_ZERO_RD)) {
      bool yes = false, dep = false;
      for (uint32_t i = 0; i < nk && i < 4; i++) {
        const uint32_t kd = F.kinds[i];
        if (kd == NONE) { yes = true; continue; }
        const uint32_t sid = (F.bits & MRF_KPACK) ? (kd & 0xFFFFFFu) : kd;
        const bool gv = (F.bits >> (24 + i)) & 1u;
        if (sid == ck) { if (gv) dep = true; else yes = true; }
      }
      acc = yes ? 1 : dep ? -1 : 0;
    }
    if (acc == 1) {
      F.bits &= ~((7u << 16) | (0xFu << 24) | MRF_KPACK);  // no kinds: the test passes (group / version bits cleared)
      (*nfold)++;
    } else if (acc == 0) {
      if (ism && mm == MM_ANY) { (*ndrop)++; continue; }
      if (!ism && (em == MM_ANY || em == MM_PLAIN)) { (*ndrop)++; continue; }
      // exclude ALL: the reference evaluates the filters ahead of this one while they all exclude, and their
      // nondeterminism counts (match_fast / match_rule_rec), so the block goes only when none of them has a tail
      if (!ism && em == MM_ALL && !excl_tail) drop_excl = true;
    }
    if (!ism && ((F.bits >> 28) & 1u)) excl_tail = true;
    out[no++] = F;
    if (ism) omf++; else oef++;
  }
  if (drop_excl) {  // an ALL exclude block with a filter that never excludes: never excluded
    no = omf;
    oef = 0;
    (*ndrop)++;
  }
  for (uint32_t j = 0; j < MREC_F; j++) R.f[j] = j < no ? out[j] : MRecFilter{};
  R.bits = (R.bits & 0x00FFFFFFu) | (omf << 24) | (oef << 28);
}

// The shape tables of a batch: per kind class the shapes some served rule's kind gate admits (kyv_jit_shapes computes
// only those), and the [shape][res] verdict / record buffers
static void setup_shapes(const Ruleset& rs, const Batch& b, DeviceResults& d, bool jit) {
  d.shape_state = (int)jit;
  d.nshapes = 0;
  if (!jit || !rs.jit_nshapes || !b.gate_words) return;
  const std::vector<uint32_t> gidx = glob_index(rs);
  const uint32_t S = rs.jit_nshapes, words = (S + 31) / 32, gw = b.gate_words;
  const size_t nclass = b.gate.size() / gw;
  std::vector<uint32_t> sg(std::max<size_t>(1, nclass * words), 0);
  bool any = false;
  for (uint32_t k = 0; k < rs.rules.size(); k++) {
    const uint32_t sh = served_shape(rs, k, gidx, jit);
    if (!sh) continue;
    for (size_t c = 0; c < nclass; c++)
      if ((b.gate[c * gw + (k >> 5)] >> (k & 31)) & 1u) { sg[c * words + (sh - 1) / 32] |= 1u << ((sh - 1) % 32); any = true; }
  }
  if (!any) return;
  dfree(d.shape_gate);
  d.shape_gate = nullptr;
  HIP_OK(dmalloc(&d.shape_gate, sg.size() * 4));
  HIP_OK(hipMemcpy(d.shape_gate, sg.data(), sg.size() * 4, hipMemcpyHostToDevice));
  if (!d.shape_st) {
    HIP_OK(dmalloc(&d.shape_st, std::max<size_t>(1, (size_t)S * d.nres)));
    HIP_OK(dmalloc(&d.shape_rec, std::max<size_t>(1, (size_t)S * d.nres) * sizeof(FailRec)));
  }
  d.nshapes = S;
  d.shape_words = words;
}

// Lane tail facts of a slice's match records (kyv_kernels.h TailCfg): the most used exact selector keys become label
// slots (namespace-selector keys namespace slots), distinct wildcard requirements and annotation pairs become atoms,
// each table filled by frequency of use; a tail filter all of whose parts are covered gets a TailProg (MRecFilter.pad
// = 1 + its index) and is decided from the lane's facts, the others run cb_tail
static void build_tails(const Ruleset& rs, const std::vector<MRec>& all, std::vector<MRec>& recs,
                        const std::vector<uint32_t>& gidx, bool onemask, TailCfg& cfg, std::vector<TailProg>& progs) {
  memset(&cfg, 0, sizeof cfg);
  progs.clear();
  using Wild = std::array<uint32_t, 4>;
  std::map<uint32_t, size_t> keyf, nskeyf;
  std::map<Wild, size_t> wildf;
  std::map<std::pair<uint32_t, uint32_t>, size_t> annf;
  auto tails = [&](auto&& fn) {
    for (auto& R : recs) {
      const uint32_t nf = ((R.bits >> 24) & 0xFu) + (R.bits >> 28);
      for (uint32_t j = 0; j < nf && j < MREC_F; j++)
        if ((R.f[j].bits >> 28) & 1u) fn(R.f[j]);
    }
  };
  auto tails_all = [&](auto&& fn) {  // the ruleset's record filters (every slice): the configuration is ruleset-wide
    for (const auto& R : all) {
      const uint32_t nf = ((R.bits >> 24) & 0xFu) + (R.bits >> 28);
      for (uint32_t j = 0; j < nf && j < MREC_F; j++)
        if ((R.f[j].bits >> 28) & 1u) fn(R.f[j]);
    }
  };
  auto wild_of = [](const SelReq& r) { return Wild{r.key, r.vals, r.rkey, r.rval}; };
  tails_all([&](const MRecFilter& F) {
    const Filter& f = rs.filters[F.idx];
    for (uint32_t q = 0; q < f.nann; q++) annf[{rs.pool[f.ann + 2 * q], rs.pool[f.ann + 2 * q + 1]}]++;
    if (f.flags & FF_HAS_SEL) {
      const SelDesc& sd = rs.sels[f.sel];
      if (!sd.invalid)
        for (uint32_t q = 0; q < sd.nreqs; q++) {
          const SelReq& r = rs.reqs[sd.reqs + q];
          if (r.op == RQ_WILD) wildf[wild_of(r)]++; else keyf[r.key]++;
        }
    }
    if (f.flags & FF_HAS_NSSEL) {
      const SelDesc& sd = rs.sels[f.sel + 1];
      if (!sd.invalid)
        for (uint32_t q = 0; q < sd.nreqs; q++)
          if (rs.reqs[sd.reqs + q].op != RQ_WILD) nskeyf[rs.reqs[sd.reqs + q].key]++;
    }
  });
  auto top = [](auto& freq, size_t cap) {  // the `cap` most used, ties by value (deterministic)
    std::vector<std::pair<size_t, typename std::decay_t<decltype(freq)>::key_type>> v;
    for (auto& x : freq) v.push_back({x.second, x.first});
    std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first != b.first ? a.first > b.first : a.second < b.second; });
    std::map<typename std::decay_t<decltype(freq)>::key_type, uint32_t> out;
    for (size_t i = 0; i < v.size() && i < cap; i++) out[v[i].second] = (uint32_t)out.size();
    return out;
  };
  const auto slots = top(keyf, TF_SLOTS), nsslots = top(nskeyf, TF_NSSLOTS);
  const auto wilds = top(wildf, TF_WILD);
  const auto anns = top(annf, TF_ANN);
  cfg.nslot = (uint32_t)slots.size();
  cfg.nnsslot = (uint32_t)nsslots.size();
  cfg.nwild = (uint32_t)wilds.size();
  cfg.nann = (uint32_t)anns.size();
  for (auto& x : slots) cfg.slot[x.second] = x.first;
  for (auto& x : nsslots) cfg.nsslot[x.second] = x.first;
  for (auto& x : wilds) {
    cfg.wkey[x.second] = x.first[0]; cfg.wval[x.second] = x.first[1];
    cfg.wrkey[x.second] = x.first[2]; cfg.wrval[x.second] = x.first[3];
  }
  for (auto& x : anns) { cfg.akey[x.second] = x.first.first; cfg.aval[x.second] = x.first.second; }
  // test codes of the atom patterns (kyv_kernels.h TailCode): glob_sid's classification by content, as build_mrec
  auto code = [&](uint32_t sid) -> uint32_t {
    if (sid >= rs.dict.strs.size()) return 0u;
    const std::string& x = rs.dict.strs[sid];
    bool globby = x.find_first_of("*?") != std::string::npos;
    for (unsigned char ch : x) if (ch >= 0x80) globby = true;
    if (!globby) return TC_EXACT;
    const uint32_t g = gidx[sid];
    return (g && g - 1 < 32 && onemask) ? (TC_MASK | (g - 1)) : 0u;
  };
  for (uint32_t a = 0; a < cfg.nwild; a++) { cfg.wkc[a] = code(cfg.wkey[a]); cfg.wvc[a] = code(cfg.wval[a]); }
  for (uint32_t a = 0; a < cfg.nann; a++) { cfg.akc[a] = code(cfg.akey[a]); cfg.avc[a] = code(cfg.aval[a]); }
  cfg.onemask = onemask ? 1u : 0u;
  // kinds with a group / version refinement: atoms (mode, g, v); the record kind becomes sid | (atom + 1) << 24 and
  // its group / version bit stays set (filt_fast reads the atom, cb_rec / kinds_match the filter)
  std::map<std::array<uint32_t, 3>, uint32_t> gvs;
  for (const auto& R : all) {  // the refinement atoms, in ruleset order
    const uint32_t nf = ((R.bits >> 24) & 0xFu) + (R.bits >> 28);
    for (uint32_t j = 0; j < nf && j < MREC_F; j++) {
      const MRecFilter& F = R.f[j];
      const Filter& f = rs.filters[F.idx];
      const uint32_t nk = (F.bits >> 16) & 7u;
      for (uint32_t i = 0; i < nk; i++) {
        if (!((F.bits >> (24 + i)) & 1u)) continue;
        const KindDesc& kd = rs.kinds[f.kinds + i];
        const std::array<uint32_t, 3> key{kd.gv_mode, kd.g, kd.v};
        if (gvs.count(key) || gvs.size() >= TF_GV) continue;
        const uint32_t a = (uint32_t)gvs.size();
        gvs.emplace(key, a);
        cfg.gvmode[a] = kd.gv_mode; cfg.gvg[a] = kd.g; cfg.gvv[a] = kd.v;
      }
    }
  }
  for (auto& R : recs) {
    const uint32_t nf = ((R.bits >> 24) & 0xFu) + (R.bits >> 28);
    for (uint32_t j = 0; j < nf && j < MREC_F; j++) {
      MRecFilter& F = R.f[j];
      const Filter& f = rs.filters[F.idx];
      const uint32_t nk = (F.bits >> 16) & 7u;
      if (!((F.bits >> 24) & 0xFu)) continue;
      bool ok = true;  // every kind sid fits 24 bits and every refinement gets an atom: the filter's kinds are packed
      std::array<uint32_t, 4> atom{0, 0, 0, 0};
      for (uint32_t i = 0; i < nk && ok; i++) {
        const KindDesc& kd = rs.kinds[f.kinds + i];
        if (kd.kind != NONE && kd.kind >= (1u << 24)) ok = false;
        if (!((F.bits >> (24 + i)) & 1u) || !ok) continue;
        const std::array<uint32_t, 3> key{kd.gv_mode, kd.g, kd.v};
        auto it = gvs.find(key);
        if (it == gvs.end()) { ok = false; continue; }
        atom[i] = it->second + 1;
      }
      if (!ok) continue;
      for (uint32_t i = 0; i < nk; i++)
        if (F.kinds[i] != NONE) F.kinds[i] |= atom[i] << 24;
      F.bits |= MRF_KPACK;
    }
  }
  cfg.ngv = (uint32_t)gvs.size();
  std::map<std::string, uint32_t> seen;  // program bytes -> its index
  tails([&](MRecFilter& F) {
    const Filter& f = rs.filters[F.idx];
    F.pad = 0;
    uint32_t ann = 0;
    for (uint32_t q = 0; q < f.nann; q++) {
      auto it = anns.find({rs.pool[f.ann + 2 * q], rs.pool[f.ann + 2 * q + 1]});
      if (it == anns.end()) return;
      ann |= 1u << it->second;
    }
    // a selector as a program: every requirement in a slot / atom, at most TP_REQ of them with TP_VALS values each
    auto cover = [&](uint32_t si, bool ns, SelProg& sp) {
      memset(&sp, 0, sizeof sp);
      const SelDesc& sd = rs.sels[si];
      if (sd.invalid) { sp.n = NONE; return true; }
      if (sd.nreqs > TP_REQ) return false;
      sp.n = sd.nreqs;
      for (uint32_t q = 0; q < sd.nreqs; q++) {
        const SelReq& r = rs.reqs[sd.reqs + q];
        uint32_t m;
        if (r.op == RQ_WILD) {
          if (ns) return false;
          auto it = wilds.find(wild_of(r));
          if (it == wilds.end()) return false;
          m = it->second;
        } else {
          auto& sl = ns ? nsslots : slots;
          auto it = sl.find(r.key);
          if (it == sl.end() || r.nvals > TP_VALS) return false;
          m = it->second;
          for (uint32_t k = 0; k < r.nvals; k++) sp.vals[q][k] = rs.pool[r.vals + k];
        }
        sp.req[q] = r.op | (m << 8) | ((r.op == RQ_WILD ? 0u : r.nvals) << 16);
      }
      return true;
    };
    TailProg tp;
    memset(&tp, 0, sizeof tp);
    tp.ann = ann;
    if ((f.flags & FF_HAS_SEL) && !cover(f.sel, false, tp.sel)) return;
    if ((f.flags & FF_HAS_NSSEL) && !cover(f.sel + 1, true, tp.nssel)) return;
    std::string key((const char*)&tp, sizeof tp);
    auto it = seen.find(key);
    if (it == seen.end()) {
      it = seen.emplace(key, (uint32_t)progs.size()).first;
      progs.push_back(tp);
    }
    F.pad = it->second + 1;
  });
}

static void layout_schedule(const Ruleset& rs, const Batch& b, const DevRuleset* dr, DeviceResults& d, SliceSched& sl,
                            bool jit) {
  // rules of this slice whose matched pairs the shape tables decide in the match phase: no walk chunks for them
  const std::vector<uint32_t> gidx = glob_index(rs);
  std::vector<uint32_t> by_shape(sl.k1 - sl.k0, 0);
  for (uint32_t k = sl.k0; k < sl.k1; k++) by_shape[k - sl.k0] = served_shape(rs, k, gidx, jit);
  const size_t nres = d.nres;
  const uint32_t WIN = getenv("KYV_WIN") ? (uint32_t)std::max(1, atoi(getenv("KYV_WIN"))) : 0xFFFFu;
  const uint32_t nw = d.wl.nwaves, gw = b.gate_words;
  std::vector<std::pair<uint32_t, std::vector<uint32_t>>> runs;  // (first wave, gate words)
  std::vector<uint8_t> uniform(nw, 0);  // every resource of the wave has one kind class (SLOT_UNIFORM)
  for (uint32_t w = 0; w < nw; w++) {
    std::vector<uint32_t> g(gw, 0);
    const size_t r0 = (size_t)w * WAVE, r1 = std::min(nres, (size_t)(w + 1) * WAVE);
    bool one = true;
    for (size_t r = r0; r < r1; r++) {
      one = one && b.hdr[r].kclass == b.hdr[r0].kclass;
      for (uint32_t i = 0; i < gw; i++) g[i] |= b.gate[(size_t)b.hdr[r].kclass * gw + i];
    }
    uniform[w] = one && !getenv("KYV_NO_UNIFORM");
    if (runs.empty() || runs.back().second != g) runs.push_back({w, std::move(g)});
  }
  const uint32_t ncls = 1 + (jit ? (uint32_t)dr->jfns.size() : 0u);  // 0: interpreter, 1 + g: compiled group g
  sl.fg.assign(jit ? dr->jfns.size() : 0, 0);
  if (jit)
    for (uint32_t k = sl.k0; k < sl.k1; k++)
      if (rs.jit_rules[k] && jit_rule_fused(rs, k) && dr->ffns[rs.jit_rules[k] - 1]) sl.fg[rs.jit_rules[k] - 1] = 1;
      else if (k < rs.jit_cond.size() && rs.jit_cond[k] >= 2 && dr->ffns[rs.jit_cond[k] - 2])
        sl.fg[rs.jit_cond[k] - 2] = 1;  // a condition rule folded into that group's fused walk (jit.cpp)
  std::vector<std::vector<uint2>> slots(ncls);
  for (size_t ri = 0; ri < runs.size(); ri++) {
    const uint32_t wb = runs[ri].first, we = ri + 1 < runs.size() ? runs[ri + 1].first : nw;
    std::vector<std::vector<uint32_t>> ks(ncls);
    for (uint32_t k = sl.k0; k < sl.k1; k++) {
      if (rs.rules[k].kind != RK_PATTERN && rs.rules[k].kind != RK_ANYPATTERN) continue;
      if (jit && rs.jit_rules[k] && jit_rule_fused(rs, k)) continue;  // its group's fused kernel walks it
      if (by_shape[k - sl.k0]) continue;  // decided in the match phase from its shape's tables
      if (!((runs[ri].second[k / 32] >> (k % 32)) & 1u)) continue;
      ks[jit ? rs.jit_rules[k] : 0].push_back(k);
    }
    for (uint32_t cls = 0; cls < ncls; cls++)
      for (size_t i = 0; i < ks[cls].size(); i += WIN) {
        const size_t n = std::min<size_t>(WIN, ks[cls].size() - i);
        for (uint32_t w = wb; w < we; w++)
          for (size_t t = i; t < i + n; t++) {
            const uint32_t k = ks[cls][t];
            const bool u = uniform[w] && (rs.rules[k].flags & RD_GATE_EXACT);
            slots[cls].push_back(make_uint2(k, w | (u ? SLOT_UNIFORM : 0u)));
          }
      }
  }
  size_t tot = 0;
  sl.grid.assign(ncls, 0);
  const bool xcd = !getenv("KYV_XCD") || atoi(getenv("KYV_XCD")) != 0;
  for (uint32_t cls = 0; cls < ncls; cls++) {
    if (slots[cls].size() > 0xFFFFFFF0ull) throw std::runtime_error("walk schedule exceeds 2^32 chunks; split the batch");
    // walk grid: up to 1024 one-wave workgroups per CU, grid-stride beyond that. Measured on C3 (kernel ms):
    // 16/CU 3.03, 64/CU 2.95, 128/CU 2.88, 256/CU 2.78, 512/CU 2.70, 1024/CU 2.66, 2048/CU 2.74, one per chunk 2.75
    // (more resident-or-queued waves hide the walk's dependent-load latency; KYV_GRID overrides)
    static const size_t gmul = getenv("KYV_GRID") ? (size_t)std::max(1, atoi(getenv("KYV_GRID"))) : 1024;
    sl.grid[cls] = (uint32_t)std::min<size_t>(slots[cls].size(), (size_t)d.cus * gmul);
    tot += slots[cls].size();
    // XCD-aware placement: workgroups are dealt round-robin over the 8 XCDs (block b and b + 8 share one L2),
    // and the grid-stride loop hands position p to block p % G. The chunks of one match wave (the same 64
    // resources under its rules) are kept on ONE XCD, so its L2 serves the resources' rows to every rule; whole
    // waves go to the XCD with the least work so far (balance), in schedule order.
    const size_t T = slots[cls].size(), G = sl.grid[cls];
    if (xcd && G >= 8 && T > G) {
      std::vector<std::vector<uint32_t>> pos(8);
      for (size_t q = 0; q < T; q++) pos[(q % G) % 8].push_back((uint32_t)q);
      std::vector<uint2> outv(T);
      size_t fill[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (size_t i = 0; i < T;) {
        size_t j = i;
        while (j < T && (slots[cls][j].y & ~SLOT_UNIFORM) == (slots[cls][i].y & ~SLOT_UNIFORM)) j++;  // one wave's chunks
        int best = -1;
        double br = 2.0;
        for (int x = 0; x < 8; x++) {
          if (fill[x] >= pos[x].size()) continue;
          double r = (double)fill[x] / (double)pos[x].size();
          if (r < br) { br = r; best = x; }
        }
        for (size_t t = i; t < j; t++) {
          int x = best;
          if (fill[x] >= pos[x].size())  // XCD full: next XCD with room
            for (int y = 0; y < 8; y++) if (fill[y] < pos[y].size()) { x = y; break; }
          outv[pos[x][fill[x]++]] = slots[cls][t];
        }
        i = j;
      }
      slots[cls].swap(outv);
    }
  }
  // match-phase rule list: light rules, then the JMESPath / foreach rules the interpreted match_kernel<true> runs,
  // then those the compiled kyv_jit_cond runs
  {
    // PodSecurity rules without preconditions: pss_kernel over the waves of their kind gate (KYV_PSS_KERNEL=0: the
    // match kernel)
    static const bool pss_k = !getenv("KYV_PSS_KERNEL") || atoi(getenv("KYV_PSS_KERNEL")) != 0;
    const bool mw_k = mrec_kernel_on();
    std::vector<uint32_t> mr, cj, mw;
    sl.pw.clear();
    for (uint32_t q : sl.ml) {
      const RuleDesc& rd = rs.rules[q];
      if (mw_k && rd.pre == NONE && (rd.kind == RK_PATTERN || rd.kind == RK_ANYPATTERN || rd.kind == RK_FALLBACK)) {
        mw.push_back(q);  // match_rec_kernel (or the generic kernel)
        continue;
      }
      // (a rule with preconditions too, when they need no JMESPath: evaluated inline, pss_kernel<.., kPre>)
      if (!pss_k || rd.kind != RK_PSS || (rd.pre != NONE && prog_jmes(rs, rd.pre))) { mr.push_back(q); continue; }
      uint32_t lo = nw, hi = 0;
      for (size_t ri = 0; ri < runs.size(); ri++) {
        if (!((runs[ri].second[q / 32] >> (q % 32)) & 1u)) continue;
        lo = std::min(lo, runs[ri].first);
        hi = std::max(hi, ri + 1 < runs.size() ? runs[ri + 1].first : nw);
      }
      if (lo < hi) sl.pw.push_back(make_uint3(q, lo, hi - lo));
    }
    // plain deny rules: match_deny_kernel (KYV_DENY_KERNEL=0: the light match kernel)
    static const bool deny_k = !getenv("KYV_DENY_KERNEL") || atoi(getenv("KYV_DENY_KERNEL")) != 0;
    std::vector<uint32_t> md;
    if (deny_k) {
      std::vector<uint32_t> rest;
      for (uint32_t q : mr) (rs.rules[q].kind == RK_DENY ? md : rest).push_back(q);
      mr.swap(rest);
    }
    // light pattern rules with preconditions: match_pre_kernel (KYV_PRE_KERNEL=0: the light match kernel)
    static const bool pre_k = !getenv("KYV_PRE_KERNEL") || atoi(getenv("KYV_PRE_KERNEL")) != 0;
    std::vector<uint32_t> mp, mpj;
    if (pre_k) {
      std::vector<uint32_t> rest;
      for (uint32_t q : mr) {
        const RuleDesc& rd = rs.rules[q];
        ((rd.kind == RK_PATTERN || rd.kind == RK_ANYPATTERN) && rd.pre != NONE ? mp : rest).push_back(q);
      }
      mr.swap(rest);
    }
    const size_t nlight = mr.size();
    // KYV_JC_ONLY=k1,k2,...: timing experiments only (the compiled condition kernel runs just those rules; the
    // other condition rules' verdicts are left unset)
    std::vector<uint32_t> only;
    if (const char* e = getenv("KYV_JC_ONLY")) for (const char* p = e; *p;) { only.push_back((uint32_t)strtoul(p, (char**)&p, 10)); if (*p) p++; }
    sl.cw.clear();
    sl.cwm.clear();
    // the match waves holding resources of a rule's kind gate: one range in the kind-major batch (waves inside it
    // whose resources the gate excludes exit after one ballot)
    auto gate_range = [&](uint32_t q, uint32_t& lo, uint32_t& hi) {
      for (size_t ri = 0; ri < runs.size(); ri++) {
        if (!((runs[ri].second[q / 32] >> (q % 32)) & 1u)) continue;
        lo = std::min(lo, runs[ri].first);
        hi = std::max(hi, ri + 1 < runs.size() ? runs[ri + 1].first : nw);
      }
    };
    std::vector<uint32_t> gmask(dr->jcg.size(), 0), glo(dr->jcg.size(), nw), ghi(dr->jcg.size(), 0);
    for (uint32_t q : sl.mj) {
      const int32_t grp = jit && q < dr->jc_group.size() ? dr->jc_group[q] : -1;
      if (jit && q < rs.jit_cond.size() && rs.jit_cond[q] >= 2 && dr->ffns[rs.jit_cond[q] - 2]) {
        if (only.empty() || std::find(only.begin(), only.end(), q) != only.end()) cj.push_back(q);
        continue;  // folded into the fused walk of its group (sl.fg)
      }
      if (jit && (grp >= 0 || (q < dr->jconds.size() && dr->jconds[q]))) {
        if (!only.empty() && std::find(only.begin(), only.end(), q) == only.end()) continue;
        cj.push_back(q);
        if (grp >= 0) {  // its group's kernel, with the members of this slice
          const auto& mem = dr->jcg_members[grp];
          gmask[grp] |= 1u << (std::find(mem.begin(), mem.end(), q) - mem.begin());
          gate_range(q, glo[grp], ghi[grp]);
          continue;
        }
        uint32_t lo = nw, hi = 0;
        gate_range(q, lo, hi);
        if (lo < hi) { sl.cw.push_back(make_uint3(q, lo, hi - lo)); sl.cwm.push_back(0); }
      } else if (pre_k && (rs.rules[q].kind == RK_PATTERN || rs.rules[q].kind == RK_ANYPATTERN) && rs.rules[q].pre != NONE) {
        mpj.push_back(q);  // a pattern rule with JMESPath preconditions: match_pre_kernel<JMESPath>
      } else {
        mr.push_back(q);
      }
    }
    for (size_t g = 0; g < gmask.size(); g++)
      if (gmask[g] && glo[g] < ghi[g]) { sl.cw.push_back(make_uint3((uint32_t)g, glo[g], ghi[g] - glo[g])); sl.cwm.push_back(gmask[g]); }
    sl.nm = (uint32_t)nlight;
    sl.nmj = (uint32_t)(mr.size() - nlight);
    sl.nmc = (uint32_t)cj.size();
    mr.insert(mr.end(), cj.begin(), cj.end());
    dfree(sl.mrec);
    sl.mrec = nullptr;
    {  // match_walk rules whose match block fits a staged record go to match_rec_kernel, the rest stay in mrules
      std::vector<MRec> recs;
      std::vector<uint32_t> gen;
      for (uint32_t q : mw) {
        MRec R;
        build_mrec(rs, q, gidx, mrec_masks_on(), mrec_recs_on(), R);
        if (R.bits & MR_FAST) {
          // 1 + its shape: decided from the shape tables; bit 23: the rule stages whole records (metadata keys)
          R.kind |= (by_shape[q - sl.k0] << 8) | (by_shape[q - sl.k0] && rs.rules[q].uses_meta ? 1u << 23 : 0u);
          recs.push_back(R);
        } else {
          gen.push_back(q);
        }
      }
      mw.swap(gen);
      sl.nmr = (uint32_t)recs.size();
      {  // lane tail facts: one device block [TailCfg][TailProg...]
        TailCfg cfg;
        std::vector<TailProg> progs;
        static const bool tails_on = !getenv("KYV_TAIL_FACTS") || atoi(getenv("KYV_TAIL_FACTS")) != 0;
        if (tails_on) {
          // every record rule of the ruleset (all slices): the tail configuration is ruleset-wide, so one facts table
          // per evaluation serves every slice (facts_kernel)
          std::vector<MRec> all;
          for (uint32_t q = 0; q < rs.rules.size(); q++) {
            const RuleDesc& rd = rs.rules[q];
            if (!(mw_k && rd.pre == NONE && (rd.kind == RK_PATTERN || rd.kind == RK_ANYPATTERN || rd.kind == RK_FALLBACK))) continue;
            if ((rd.kind == RK_PATTERN || rd.kind == RK_ANYPATTERN) && (rd.flags & RD_GATE_EXACT)) continue;  // direct walk
            if (rule_needs_jmes(rs, rd)) continue;
            MRec R;
            build_mrec(rs, q, gidx, mrec_masks_on(), mrec_recs_on(), R);
            if (R.bits & MR_FAST) all.push_back(R);
          }
          const bool onemask = mrec_masks_on() && rs.gpats.size() + rs.gsets.size() <= 32;
          build_tails(rs, all, recs, gidx, onemask, cfg, progs);
        }
        else memset(&cfg, 0, sizeof cfg);
        const size_t bytes = sizeof(TailCfg) + std::max<size_t>(1, progs.size()) * sizeof(TailProg);
        dfree(sl.tails);
        sl.tails = nullptr;
        HIP_OK(dmalloc(&sl.tails, bytes));
        HIP_OK(hipMemcpy(sl.tails, &cfg, sizeof cfg, hipMemcpyHostToDevice));
        if (!d.tcfg) HIP_OK(dmalloc(&d.tcfg, sizeof(TailCfg)));
        HIP_OK(hipMemcpy(d.tcfg, &cfg, sizeof cfg, hipMemcpyHostToDevice));  // (ruleset-wide: equal for every slice)
        d.facts_on = tails_on;
        if (!progs.empty()) HIP_OK(hipMemcpy(sl.tails + sizeof(TailCfg), progs.data(), progs.size() * sizeof(TailProg), hipMemcpyHostToDevice));
        // the branch-free path (MR_FASTEVAL: no group / version kinds, every tail covered) and the empty-OldResource
        // retry as a constant of the rule (MR_ECONST: no filter reaches a namespace selector for a kind-less
        // resource), evaluated here with the host instantiation of match_rule against the batch dictionary
        const View hv = make_view(rs, b, nullptr, nullptr, nullptr, nullptr);
        for (auto& R : recs) {
          const uint32_t nf = ((R.bits >> 24) & 0xFu) + (R.bits >> 28);
          bool fast = true, nsstar = false;
          for (uint32_t j = 0; j < nf && j < MREC_F; j++) {
            const MRecFilter& F = R.f[j];
            if (((F.bits >> 24) & 0xFu) && !(F.bits & MRF_KPACK)) fast = false;  // a group / version kind without its atom
            if (((F.bits >> 28) & 1u) && !F.pad) fast = false;
            if ((F.bits & FF_HAS_NSSEL) && (F.bits & FF_KINDS_STAR)) nsstar = true;
          }
          if (fast) R.bits |= MR_FASTEVAL;
          if ((R.bits & MR_EMPTY) && !nsstar) {
            bool nd = false;
            const bool em = match_rule(hv, rs.rules[R.k], ResView{NodeTab{nullptr}, nullptr},
                                       LabelSet{NodeTab{nullptr}, 0, nullptr, 0}, &nd);
            R.bits |= MR_ECONST | (em ? MR_EMATCH : 0u) | (nd ? MR_END : 0u);
          }
        }
        if (getenv("KYV_DEBUG_STATS")) {
          size_t nf = 0, ne = 0, nec = 0, nsh = 0;
          for (auto& R : recs) {
            nf += (R.bits & MR_FASTEVAL) != 0;
            ne += (R.bits & MR_EMPTY) != 0;
            nec += (R.bits & MR_ECONST) != 0;
            nsh += (R.kind >> 8) != 0;
          }
          fprintf(stderr, "[kyvgpu] slice [%u, %u): %zu match records, %zu branch-free, %zu empty retry (%zu constant), "
                  "%zu shape rules; tail facts: %u slots, %u ns slots, %u wildcard, %u annotation, %u group/version atoms, "
                  "%zu covered tails\n", sl.k0, sl.k1, recs.size(), nf, ne, nec, nsh, cfg.nslot, cfg.nnsslot, cfg.nwild,
                  cfg.nann, cfg.ngv, progs.size());
        }
      }
      // the kind index: per kind class of the batch, copies of the records whose rule's kind gate admits it, one
      // contiguous run per class (a uniform wave streams its class's run: no index load in front of each record)
      const uint32_t gw = b.gate_words;
      sl.nclass = gw ? (uint32_t)(b.gate.size() / gw) : 0u;
      std::vector<uint32_t> off(sl.nclass + 1, 0);
      std::vector<MRec> crecs;
      // a class is one GVK kind (order_by_kind): its kind sid, from the first resource of the class
      std::vector<uint32_t> ckind(sl.nclass, NONE);
      for (const ResHeader& h : b.hdr)
        if (h.kclass < sl.nclass && ckind[h.kclass] == NONE) ckind[h.kclass] = h.gvk_kind;
      static const bool kfold = !getenv("KYV_KIND_FOLD") || atoi(getenv("KYV_KIND_FOLD")) != 0;
      size_t nfold = 0, ndrop = 0;
      for (uint32_t c = 0; c < sl.nclass; c++) {
        for (uint32_t q = 0; q < sl.nmr; q++) {
          const uint32_t k = recs[q].k;
          if (!((b.gate[(size_t)c * gw + (k >> 5)] >> (k & 31)) & 1u)) continue;
          MRec R = recs[q];
          if (kfold && ckind[c] != NONE) fold_kinds(R, ckind[c], &nfold, &ndrop);
          crecs.push_back(R);
        }
        off[c + 1] = (uint32_t)crecs.size();
      }
      if (getenv("KYV_DEBUG_STATS"))
        fprintf(stderr, "[kyvgpu] slice [%u, %u): %zu class-record copies, kind checks folded in %zu filters, %zu "
                "filters that cannot accept their class removed\n", sl.k0, sl.k1, crecs.size(), nfold, ndrop);
      dfree(sl.mcls);
      sl.mcls = nullptr;
      HIP_OK(dmalloc(&sl.mcls, off.size() * 4));
      HIP_OK(hipMemcpy(sl.mcls, off.data(), off.size() * 4, hipMemcpyHostToDevice));
      dfree(sl.mcrec);
      sl.mcrec = nullptr;
      HIP_OK(dmalloc(&sl.mcrec, std::max<size_t>(1, crecs.size()) * sizeof(MRec)));
      if (!crecs.empty()) HIP_OK(hipMemcpy(sl.mcrec, crecs.data(), crecs.size() * sizeof(MRec), hipMemcpyHostToDevice));
      recs.resize(std::max<size_t>(1, recs.size()));
      HIP_OK(dmalloc(&sl.mrec, recs.size() * sizeof(MRec)));
      HIP_OK(hipMemcpy(sl.mrec, recs.data(), recs.size() * sizeof(MRec), hipMemcpyHostToDevice));
    }
    sl.nmw = (uint32_t)mw.size();  // device list: [generic][deny][pre][pre JMESPath][light][JMESPath][compiled]
    sl.nmd = (uint32_t)md.size();
    sl.nmp = (uint32_t)mp.size();
    sl.nmpj = (uint32_t)mpj.size();
    mr.insert(mr.begin(), mpj.begin(), mpj.end());
    mr.insert(mr.begin(), mp.begin(), mp.end());
    mr.insert(mr.begin(), md.begin(), md.end());
    mr.insert(mr.begin(), mw.begin(), mw.end());
    if (getenv("KYV_DEBUG_STATS")) {
      fprintf(stderr, "[kyvgpu] slice [%u, %u) match lists: %u generic/records, %u deny, %u pre, %u pre-JMESPath, %u light, "
              "%u JMESPath (interpreted:", sl.k0, sl.k1, sl.nmw, sl.nmd, sl.nmp, sl.nmpj, sl.nm, sl.nmj);
      for (uint32_t i = 0; i < sl.nmj; i++) {
        const RuleDesc& rd = rs.rules[mr[sl.nmw + sl.nmd + sl.nmp + sl.nmpj + sl.nm + i]];
        fprintf(stderr, " %u/k%u%s", mr[sl.nmw + sl.nmd + sl.nmp + sl.nmpj + sl.nm + i], (unsigned)rd.kind,
                rd.pre != NONE ? "p" : "");
      }
      fprintf(stderr, "), %u compiled, %zu pss-kernel\n", sl.nmc, sl.pw.size());
    }
    dfree(sl.mrules);
    sl.mrules = nullptr;
    HIP_OK(dmalloc(&sl.mrules, std::max<size_t>(1, mr.size()) * 4));
    if (!mr.empty()) HIP_OK(hipMemcpy(sl.mrules, mr.data(), mr.size() * 4, hipMemcpyHostToDevice));
  }
  dfree(sl.sched);
  sl.sched = nullptr;
  HIP_OK(dmalloc(&sl.sched, std::max<size_t>(1, tot) * sizeof(uint2)));
  sl.cm.assign(ncls, ChunkMap{nullptr, 0});
  size_t at = 0;
  for (uint32_t cls = 0; cls < ncls; cls++) {
    if (!slots[cls].empty())
      HIP_OK(hipMemcpy(sl.sched + at, slots[cls].data(), slots[cls].size() * sizeof(uint2), hipMemcpyHostToDevice));
    sl.cm[cls] = ChunkMap{sl.sched + at, (uint32_t)slots[cls].size()};
    at += slots[cls].size();
  }
  sl.jit_state = (int)jit;
}

// accumulate one slice's phase times (ms) from its events; `start`: the evaluation's start event for the first slice
// (the verdict resets count to the match phase), the slice's own start event for the others
static void slice_phases(const SliceSched& sl, hipEvent_t start, double* phase) {
  float t = 0;
  if (start && hipEventElapsedTime(&t, start, sl.ev[0]) == hipSuccess) phase[0] += t;
  for (int q = 0; q < 3; q++)
    if (hipEventElapsedTime(&t, sl.ev[q], sl.ev[q + 1]) == hipSuccess) phase[q + 1] += t;
}

void eval_gpu(const Ruleset& rs, const Batch& b, int device, int iters, Results* out, double* kernel_ms_avg, bool copy_back,
              int jit_mode, bool account, bool serial) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) throw std::runtime_error("no HIP device available (GPU backend requested)");
  if (device < 0 || device >= ndev) throw std::runtime_error("device index out of range");
  HIP_OK(hipSetDevice(device));
  Ruleset& mrs = const_cast<Ruleset&>(rs);
  Batch& mb = const_cast<Batch&>(b);
  if ((int)mrs.dev.size() <= device) mrs.dev.resize(device + 1, nullptr);
  if ((int)mb.dev.size() <= device) mb.dev.resize(device + 1, nullptr);
  if (!mrs.dev[device]) mrs.dev[device] = upload_ruleset(rs, device);
  if (!mb.dev[device]) mb.dev[device] = upload_batch(b, device);
  DevRuleset* dr = (DevRuleset*)mrs.dev[device];
  DevBatch* db = (DevBatch*)mb.dev[device];
  if (!db->gmask && rs.gpats.size() + rs.gsets.size() > 0 && !b.str_len.empty() && !getenv("KYV_NO_GMASK")) {
    // glob masks of this batch's dictionary against the ruleset's wildcard patterns (once per batch and device,
    // like the path columns on the host: derived per-string data, not per-evaluation work)
    const size_t nstr = b.str_len.size();
    db->gmask_words = (uint32_t)((rs.gpats.size() + rs.gsets.size() + 31) / 32);
    HIP_OK(dmalloc(&db->gmask, nstr * db->gmask_words * 4));
    View tv = make_view(rs, b, dr->base, dr, db->base, db);
    View* dv = nullptr;
    HIP_OK(dmalloc(&dv, sizeof(View)));
    HIP_OK(hipMemcpy(dv, &tv, sizeof(View), hipMemcpyHostToDevice));
    const uint32_t* gp = (const uint32_t*)(dr->base + dr->o_gpats);
    const uint32_t* gs = (const uint32_t*)(dr->base + dr->o_gsets);
    hipEvent_t g0, g1;
    HIP_OK(hipEventCreate(&g0));
    HIP_OK(hipEventCreate(&g1));
    HIP_OK(hipEventRecord(g0, 0));
    hipLaunchKernelGGL(gmask_kernel, dim3((unsigned)((nstr + 255) / 256)), dim3(256), 0, 0, (const View*)dv, gp,
                       (uint32_t)rs.gpats.size(), gs, (uint32_t)rs.gsets.size(), (uint32_t)nstr, db->gmask_words, db->gmask);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(g1, 0));
    HIP_OK(hipDeviceSynchronize());
    float gms = 0;
    HIP_OK(hipEventElapsedTime(&gms, g0, g1));
    db->gmask_ms = gms;
    (void)hipEventDestroy(g0);
    (void)hipEventDestroy(g1);
    dfree(dv);
  }
  View v = make_view(rs, b, dr->base, dr, db->base, db);
  size_t nres = b.hdr.size(), nrules = rs.rules.size();
  if (!db->out) {
    auto* dd = new DeviceResults();
    DeviceResults& d = *dd;
    d.nres = nres;
    d.nrules = nrules;
    std::vector<uint32_t> pss_slot(nrules, NONE);
    for (size_t k = 0; k < nrules; k++) if (rs.rules[k].kind == RK_PSS) pss_slot[k] = d.npss++;
    HIP_OK(dmalloc(&d.status, std::max<size_t>(1, nres * nrules)));
    HIP_OK(dmalloc(&d.pss_fails, std::max<size_t>(4, (size_t)d.npss * nres * 4)));
    HIP_OK(dmalloc(&d.pss_slot, std::max<size_t>(4, nrules * 4)));
    HIP_OK(dmalloc(&d.nrecs, 16));
    HIP_OK(dmalloc(&d.counts, std::max<size_t>(1, nrules) * NSTATUS * 8));
    HIP_OK(hipMemcpy(d.pss_slot, pss_slot.data(), nrules * 4, hipMemcpyHostToDevice));
    stream_get(&d.stream, &d.e0, &d.e1);
    HIP_OK(dmalloc(&d.view, sizeof(View)));
    HIP_OK(hipMemcpy(d.view, &v, sizeof(View), hipMemcpyHostToDevice));
    d.wl.nwaves = (uint32_t)((nres + WAVE - 1) / WAVE);
    const size_t nwv = d.wl.nwaves;
    // rule slices: consecutive rules while their walk buffers fit the budget (and every slice-local index fits 32 bits)
    const size_t budget = slice_budget();
    for (size_t k = 0; k < nrules || (nrules == 0 && d.slices.empty());) {
      SliceSched sl;
      sl.k0 = (uint32_t)k;
      size_t bytes = 0, stage = 0;
      while (k < nrules) {
        const RuleDesc& rd = rs.rules[k];
        const size_t cost = rule_slice_bytes(rd) * nwv * WAVE + nwv * 2;
        const size_t alts = rd.kind == RK_PATTERN ? 1 : rd.kind == RK_ANYPATTERN ? std::min<uint32_t>(rd.nalts, MAX_ALTS) : 0;
        const size_t st2 = stage + alts * nwv * WAVE;
        const size_t nk = k + 1 - sl.k0;
        if (k > sl.k0 && (bytes + cost > budget || st2 > 0xFFFFFFF0ull || nk * nwv > 0xFFFFFFF0ull)) break;
        if (st2 > 0xFFFFFFF0ull) throw std::runtime_error("batch too large for one rule's failure-record staging");
        bytes += cost;
        stage = st2;
        k++;
      }
      sl.k1 = (uint32_t)k;
      sl.stage_tot = stage;
      std::vector<uint32_t> rb(std::max<size_t>(sl.k1 - sl.k0, 1), 0);
      size_t tot = 0;
      std::vector<uint32_t> ml, mj;
      for (uint32_t q = sl.k0; q < sl.k1; q++) {
        const RuleDesc& rd = rs.rules[q];
        rb[q - sl.k0] = (uint32_t)tot;
        tot += (rd.kind == RK_PATTERN ? 1 : rd.kind == RK_ANYPATTERN ? std::min<uint32_t>(rd.nalts, MAX_ALTS) : 0) * nwv * WAVE;
        const bool direct = (rd.kind == RK_PATTERN || rd.kind == RK_ANYPATTERN) && (rd.flags & RD_GATE_EXACT);
        if (!direct) (rule_needs_jmes(rs, rd) ? mj : ml).push_back(q);
      }
      sl.ml = ml;  // device list laid out by layout_schedule (depends on the compiled kernels)
      sl.mj = mj;
      HIP_OK(dmalloc(&sl.rbase, rb.size() * 4));
      HIP_OK(hipMemcpy(sl.rbase, rb.data(), rb.size() * 4, hipMemcpyHostToDevice));
      d.max_slice_rules = std::max<size_t>(d.max_slice_rules, sl.k1 - sl.k0);
      d.max_recs = std::max<size_t>(d.max_recs, std::max<size_t>(sl.stage_tot, 1));
      d.slices.push_back(std::move(sl));
      if (nrules == 0) break;
    }
    const size_t msr = std::max<size_t>(d.max_slice_rules, 1);
    HIP_OK(dmalloc(&d.stage, d.max_recs * sizeof(FailRec)));
    HIP_OK(dmalloc(&d.recs, d.max_recs * sizeof(FailRec)));
    d.recs_cap = d.max_recs;
    HIP_OK(dmalloc(&d.rcnt, std::max<size_t>(msr * nwv, 1) * 2));
    HIP_OK(dmalloc(&d.tsum, std::max<size_t>((msr * nwv + WAVE - 1) / WAVE, 1) * 4));
    HIP_OK(dmalloc(&d.tseg, std::max<size_t>((msr * nwv + WAVE - 1) / WAVE / SCAN_SEG + 1, 1) * 4));
    // walk work lists: one 64-slot list per (slice rule, match wave)
    HIP_OK(dmalloc(&d.wl.items, std::max<size_t>(1, msr * nwv * WAVE) * sizeof(uint2)));
    HIP_OK(dmalloc(&d.wl.cnt, std::max<size_t>(4, msr * nwv + 4)));
    // persistent grid: enough waves to fill the chip several times over, never more than the chunks
    // CU count per device, queried once (hipGetDeviceProperties costs milliseconds per call)
    static std::mutex cu_mu;
    static std::vector<int> cu_count;
    int cus = 0;
    {
      std::lock_guard<std::mutex> g(cu_mu);
      if ((int)cu_count.size() <= device) cu_count.resize(device + 1, 0);
      if (!cu_count[device]) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c <= 0) c = 256;
        cu_count[device] = c;
      }
      cus = cu_count[device];
    }
    d.cus = cus;
    db->out = dd;
  }
  DeviceResults& d = *db->out;
  hipStream_t stream = d.stream;
  const bool use_jit = jit_mode == JIT_ON || (jit_mode == JIT_AUTO && nres >= JIT_AUTO_MIN_RESOURCES);
  const bool jit = use_jit && ensure_jit(mrs, dr);
  for (auto& sl : d.slices)
    if (sl.jit_state != (int)jit) layout_schedule(rs, b, dr, d, sl, jit);
  if (d.shape_state != (int)jit) setup_shapes(rs, b, d, jit && dr->jshapes);
  const bool multi = d.slices.size() > 1;
  int depth = ruleset_depth(rs);
  size_t lds = (size_t)depth * (sizeof(UFrame) + BLOCK * sizeof(LaneFrame));
  dim3 grid((unsigned)((nres + BLOCK - 1) / BLOCK));
  double total_ms = 0;
  double phase[5] = {0, 0, 0, 0, 0};
  for (auto& sl : d.slices) {
    if (!sl.evs) HIP_OK(hipEventCreate(&sl.evs));
    for (auto& e : sl.ev) if (!e) HIP_OK(hipEventCreate(&e));
    for (auto& e : sl.cev) if (!e) HIP_OK(hipEventCreate(&e));
  }
  int n = std::max(1, iters);
  std::vector<FailRec> host_recs;
  // Byte accounting (KYV_EVAL_ACCOUNT_BYTES on the GPU backend): one evaluation with the KYV_ACCT build of every
  // kernel (kyv_acct.hip; the runtime-compiled kernels with -DKYV_ACCT), phases serialised on the evaluation stream and
  // the device counters read after each phase, so each phase's algorithmic bytes are what its kernels
  // loaded and stored. Verdicts are those of the product kernels (same source).
  const bool acct = account;
  uint64_t aphase[5] = {0, 0, 0, 0, 0};
  uint64_t aclass[3] = {0, 0, 0};
  unsigned long long *acnt_lib = nullptr, *acnt_lib_j = nullptr;
  bool ajit = false;
  std::vector<unsigned long long> ahost(3 * KYV_ACCT_SLOTS);
  auto acct_take = [&]() -> std::array<uint64_t, 3> {  // counters since the last call, by class; then zeroed
    std::array<uint64_t, 3> c{0, 0, 0};
    HIP_OK(hipStreamSynchronize(stream));
    for (unsigned long long* dc : {acnt_lib, acnt_lib_j, ajit ? dr->acnt : nullptr}) {
      if (!dc) continue;
      // on the evaluation stream (a non-blocking stream: null-stream copies / memsets would not order with its
      // kernels, and a counter reset could land after the next phase's first adds)
      HIP_OK(hipMemcpyAsync(ahost.data(), dc, ahost.size() * 8, hipMemcpyDeviceToHost, stream));
      HIP_OK(hipMemsetAsync(dc, 0, ahost.size() * 8, stream));
      HIP_OK(hipStreamSynchronize(stream));
      for (int q = 0; q < 3; q++)
        for (uint32_t i = 0; i < KYV_ACCT_SLOTS; i++) c[q] += ahost[q * KYV_ACCT_SLOTS + i];
    }
    for (int q = 0; q < 3; q++) aclass[q] += c[q];
    return c;
  };
  if (acct) {
    n = 1;
    acnt_lib = kyvacct::counters();
    acnt_lib_j = kyvacct::counters_j();
    ajit = jit && ensure_jit_acct(mrs, dr);
    if (jit && !ajit) throw std::runtime_error("accounting build of the runtime-compiled kernels unavailable");
    acct_take();
  }
  // concurrent condition stream (KYV_COND_STREAM=1; default: the evaluation stream). The fused walk kernels take every
  // wave slot, so the condition kernels found nothing to overlap: C3 10M evaluation 10.88 (second stream) vs 10.82 ms
  // (round 6; round 5: 11.24 vs 11.19)
  static const bool cond_conc = getenv("KYV_COND_STREAM") && atoi(getenv("KYV_COND_STREAM")) != 0;
  bool conc = false;
  for (auto& sl : d.slices) conc = conc || !sl.cw.empty();
  conc = conc && cond_conc && !acct && !serial;
  if (conc && !d.cstream) stream_get(&d.cstream, &d.cfork, &d.cjoin);
  // off by default: measured 13.43 (one stream) vs 13.53 ms (groups overlapped) on C3 10M
  static const bool walk_conc = getenv("KYV_WALK_STREAM") && atoi(getenv("KYV_WALK_STREAM")) != 0;
  bool wconc = false;
  for (auto& sl : d.slices) wconc = wconc || sl.cm.size() > 2;
  wconc = wconc && walk_conc && !acct;
  if (wconc && !d.wstream) stream_get(&d.wstream, &d.wfork, &d.wjoin);
  for (int it = 0; it < n; it++) {
    const bool collect = copy_back && out && it == n - 1;
    const double sum_before = phase[0] + phase[1] + phase[2] + phase[3];
    bool joined = false;
    host_recs.clear();
    d.host_recs.clear();
    d.recs_resident = !(multi && collect);
    HIP_OK(hipEventRecord(d.e0, stream));  // the resets are part of the evaluation
    HIP_OK(hipMemsetAsync(d.counts, 0, std::max<size_t>(1, nrules) * NSTATUS * 8, stream));
    HIP_OK(hipMemsetAsync(d.nrecs, 0, 16, stream));  // also when no slice runs (no rules / no resources)
    // rule slices append to one resident record list, except when copy-back gathers each slice's records on the host
    // (then each slice starts at 0: the buffer holds one slice's worst case)
    const uint32_t accumulate = multi && !collect ? 1u : 0u;
    size_t appended = 0;  // upper bound of the records the slices have appended so far (accumulate)
    HIP_OK(hipMemsetAsync(d.status, ST_NONE, nres * nrules, stream));
    if (d.npss) HIP_OK(hipMemsetAsync(d.pss_fails, 0, (size_t)d.npss * nres * 4, stream));
    if (acct) aphase[0] += (uint64_t)nres * nrules + (uint64_t)d.npss * nres * 4;  // verdict / PSS-mask resets
    // pattern-shape tables (round 5): every shape walked once per resource its users admit, before the match phase
    // that reads them (counted in the match phase: it replaces the walk of the shape rules' matched pairs)
    if (d.nshapes && nres) {
      const View* vp = d.view;
      ShapeOut so{d.shape_st, d.shape_rec, d.shape_gate, d.shape_words, d.wl.nwaves};
      void* args[] = {(void*)&vp, (void*)&so};
      const uint32_t sgrid = (uint32_t)std::min<size_t>(d.wl.nwaves, (size_t)d.cus * 32);
      HIP_OK(hipModuleLaunchKernel(acct ? dr->ajshapes : dr->jshapes, sgrid, 1, 1, BLOCK, 1, 1, 0, stream, args, nullptr));
    }
    bool any_rec = false;
    for (auto& sl : d.slices) any_rec = any_rec || sl.nmr;
    const bool use_facts = any_rec && d.facts_on && d.tcfg && nres;
    if (use_facts) {  // the match records' resource facts, once per evaluation (read by every slice)
      if (!d.facts) HIP_OK(dmalloc(&d.facts, nres * sizeof(ResFacts)));
      const dim3 fg((unsigned)((nres + 255) / 256));
      const bool mw1 = v.gmask_words <= 1;
      (acct ? kyvacct::facts : kyvprod::facts)(mw1, fg.x, stream, d.view, d.tcfg, d.facts);
    }
    for (auto& sl : d.slices) {
      if (!nres || sl.k1 == sl.k0) continue;
      const size_t nsr = sl.k1 - sl.k0;
      DevOut o{d.status, d.pss_fails, d.pss_slot, d.stage, sl.rbase, d.rcnt, sl.k0, sl.k1};
      HIP_OK(hipEventRecord(sl.evs, stream));
      HIP_OK(hipMemsetAsync(d.rcnt, 0, std::max<size_t>(nsr * (size_t)d.wl.nwaves, 1) * 2, stream));
      // match_rec_kernel and the generic kernel: 4 waves/SIMD by default (114 / 86 VGPRs, no scratch); KYV_MATCHW_WPE 5 / 6 / 8
      static const int mwpe = getenv("KYV_MATCHW_WPE") ? atoi(getenv("KYV_MATCHW_WPE")) : 4;
      if (sl.nmr) {
        const bool mw1 = v.gmask_words <= 1;
        const MRecIndex ix{sl.mcls, sl.mcrec};
        const ShapeTab sh{d.shape_st, d.shape_rec, d.wl.nwaves, d.nshapes};
        const TailTab tt{(const TailCfg*)sl.tails, (const TailProg*)(sl.tails + sizeof(TailCfg))};
        const ResFacts* fp = use_facts ? d.facts : nullptr;
        (acct ? kyvacct::match_rec : kyvprod::match_rec)(mwpe, mw1, grid.x, stream, d.view, &o, &d.wl, sl.mrec, sl.nmr,
                                                         &ix, &sh, &tt, fp);
      }
      if (sl.nmw) {
        (acct ? kyvacct::match_walk_generic : kyvprod::match_walk_generic)(mwpe, grid.x, stream, d.view, &o, &d.wl,
                                                                           sl.mrules, sl.nmw);
      }
      if (sl.nmd) {
        (acct ? kyvacct::match_deny : kyvprod::match_deny)(grid.x, stream, d.view, &o, sl.mrules + sl.nmw, sl.nmd);
      }
      if (sl.nmp) {
        (acct ? kyvacct::match_pre : kyvprod::match_pre)(grid.x, stream, d.view, &o, &d.wl, sl.mrules + sl.nmw + sl.nmd,
                                                         sl.nmp);
      }
      if (sl.nmpj) {
        (acct ? kyvacct::match_pre_j : kyvprod::match_pre_j)(grid.x, stream, d.view, &o, &d.wl,
                                                             sl.mrules + sl.nmw + sl.nmd + sl.nmp, sl.nmpj);
      }
      const uint32_t ml0 = sl.nmw + sl.nmd + sl.nmp + sl.nmpj;
      if (sl.nm) {
        (acct ? kyvacct::match : kyvprod::match)(grid.x, stream, d.view, &o, &d.wl, sl.mrules + ml0, sl.nm);
      }
      if (sl.nmj) {
        (acct ? kyvacct::match_j : kyvprod::match_j)(grid.x, stream, d.view, &o, &d.wl, sl.mrules + ml0 + sl.nm, sl.nmj);
      }
      {
        // C2 (round 3, map walk inlined): 4 0.586, 6 0.587, 8 0.514 ms; round 4: the column-only kernel with the
        // containers spread over the wave's lanes needs 41 VGPRs, no scratch at 8
        static const int pwpe = getenv("KYV_PSS_WPE") ? atoi(getenv("KYV_PSS_WPE")) : 8;
        for (const uint3& c : sl.pw) {
          const bool ex = (rs.rules[c.x].flags & RD_GATE_EXACT) && rs.rules[c.x].match.mode != MM_NONE;
          const bool pre = rs.rules[c.x].pre != NONE;
          // rules with preconditions: KYV_PSS_PRE_WPE (6 by default; at 6 the condition code spills 223 VGPRs)
          static const int ppwpe = getenv("KYV_PSS_PRE_WPE") ? atoi(getenv("KYV_PSS_PRE_WPE")) : 6;
          (acct ? kyvacct::pss : kyvprod::pss)(ex, pre, pre ? ppwpe : pwpe, c.z, stream, d.view, &o, c.x, c.y);
          // the pairs it marked ST_PSS_MAP (exclusions, no path columns): the map walk
          (acct ? kyvacct::pss_map : kyvprod::pss_map)(c.z, stream, d.view, &o, c.x, c.y);
        }
      }
      HIP_OK(hipGetLastError());
      HIP_OK(hipEventRecord(sl.ev[0], stream));
      if (acct) { const auto c = acct_take(); aphase[0] += c[0] + c[1]; }
      // compiled condition rules: one kernel each over the waves of its kind gate
      // (the View goes by pointer: a by-value View would be copied to scratch memory, since the kernels take its
      // address for out-of-line helpers; measured 40 % slower)
      hipStream_t cs = stream;
      if (conc && !sl.cw.empty()) {  // fork: after the resets and the match phase on the evaluation stream
        HIP_OK(hipEventRecord(d.cfork, stream));
        HIP_OK(hipStreamWaitEvent(d.cstream, d.cfork, 0));
        HIP_OK(hipEventRecord(sl.cev[0], d.cstream));
        cs = d.cstream;
      }
      for (size_t i = 0; i < sl.cw.size(); i++) {
        const uint3 c = sl.cw[i];
        const View* vp = d.view;
        uint32_t w0 = c.y, mask = sl.cwm[i];
        void* args[] = {(void*)&vp, (void*)&o, (void*)&w0, (void*)&mask};
        hipFunction_t f = mask ? (acct ? dr->ajcg[c.x] : dr->jcg[c.x]) : (acct ? dr->aconds[c.x] : dr->jconds[c.x]);
        HIP_OK(hipModuleLaunchKernel(f, c.z, 1, 1, BLOCK, 1, 1, 0, cs, args, nullptr));
      }
      if (acct) { const auto c = acct_take(); aphase[1] += c[0] + c[1]; }
      if (cs != stream) {
        HIP_OK(hipEventRecord(sl.cev[1], d.cstream));
        HIP_OK(hipEventRecord(d.cjoin, d.cstream));
        joined = true;
      }
      HIP_OK(hipEventRecord(sl.ev[1], stream));
      if (sl.grid[0]) {
        (acct ? kyvacct::walk : kyvprod::walk)(sl.grid[0], lds, stream, d.view, &o, &d.wl, &sl.cm[0], depth);
        HIP_OK(hipGetLastError());
      }
      bool wforked = false;
      if (wconc)  // fork after the match phase (the work lists), before the first group is queued
        for (size_t cls = 2; cls < sl.cm.size() && !wforked; cls++)
          if (sl.grid[cls]) {
            HIP_OK(hipEventRecord(d.wfork, stream));
            HIP_OK(hipStreamWaitEvent(d.wstream, d.wfork, 0));
            wforked = true;
          }
      for (size_t cls = 1; cls < sl.cm.size(); cls++) {
        if (!sl.grid[cls]) continue;
        const View* vp = d.view;
        WorkLists wl = d.wl;
        ChunkMap cmj = sl.cm[cls];
        void* args[] = {(void*)&vp, (void*)&o, (void*)&wl, (void*)&cmj};
        const hipStream_t ws = (wforked && cls >= 2) ? d.wstream : stream;
        HIP_OK(hipModuleLaunchKernel(acct ? dr->afns[cls - 1] : dr->jfns[cls - 1], sl.grid[cls], 1, 1, BLOCK, 1, 1, 0, ws,
                                     args, nullptr));
      }
      // fused groups: one workgroup per match wave, every direct rule of the group walked back to back (kyv_fused.h)
      for (size_t g = 0; g < sl.fg.size(); g++) {
        if (!sl.fg[g]) continue;
        const View* vp = d.view;
        uint32_t nw = d.wl.nwaves;
        void* args[] = {(void*)&vp, (void*)&o, (void*)&nw};
        if (g < dr->fmfns.size() && dr->fmfns[g]) {  // the parts as one kernel (KYV_FUSED_MERGE)
          HIP_OK(hipModuleLaunchKernel(acct ? dr->afmfns[g] : dr->fmfns[g], nw, 1, 1, BLOCK, 1, 1, 0, stream, args, nullptr));
          continue;
        }
        HIP_OK(hipModuleLaunchKernel(acct ? dr->affns[g] : dr->ffns[g], nw, 1, 1, BLOCK, 1, 1, 0, stream, args, nullptr));
        if (g < dr->fparts.size())
          for (size_t p = 0; p < dr->fparts[g].size(); p++)
            HIP_OK(hipModuleLaunchKernel(acct ? dr->afparts[g][p] : dr->fparts[g][p], nw, 1, 1, BLOCK, 1, 1, 0, stream,
                                         args, nullptr));
      }
      uint64_t staged = 0;
      if (acct) { const auto c = acct_take(); aphase[2] += c[0] + c[1] + c[2]; staged = c[2]; }
      if (wforked) {  // the compaction reads every walk group's staged records
        HIP_OK(hipEventRecord(d.wjoin, d.wstream));
        HIP_OK(hipStreamWaitEvent(stream, d.wjoin, 0));
      }
      HIP_OK(hipEventRecord(sl.ev[2], stream));
      const size_t nchunks = nsr * (size_t)d.wl.nwaves;
      const uint32_t ntiles = (uint32_t)((nchunks + WAVE - 1) / WAVE);
      const RuleDesc* drules = (const RuleDesc*)(dr->base + dr->o_rules) + sl.k0;
      hipLaunchKernelGGL(compact_sum_kernel, dim3(ntiles), dim3(WAVE), 0, stream, d.rcnt, nchunks, d.tsum);
      const uint32_t nseg = (ntiles + SCAN_SEG - 1) / SCAN_SEG;
      hipLaunchKernelGGL(compact_scan_kernel, dim3(std::max<uint32_t>(nseg, 1)), dim3(1024), 0, stream, d.tsum, ntiles, d.tseg);
      hipLaunchKernelGGL(compact_top_kernel, dim3(1), dim3(1024), 0, stream, d.tseg, std::max<uint32_t>(nseg, 1), d.nrecs,
                         accumulate);
      if (accumulate) {
        // a rule-sliced evaluation appends every slice's records to one resident list. The host keeps an upper bound of
        // the records appended so far (a slice stages at most d.max_recs); only when that bound could outgrow the
        // list does it read the exact running total compact_top_kernel just computed and, if needed, grow the list
        // in place (earlier slices' records copied over) before this slice's copy -- never a second evaluation
        if (appended + d.max_recs > d.recs_cap) {
          uint32_t c3[3] = {0, 0, 0};
          HIP_OK(hipMemcpyAsync(c3, d.nrecs, 12, hipMemcpyDeviceToHost, stream));
          HIP_OK(hipStreamSynchronize(stream));
          if (c3[2] > d.recs_cap) {
            const size_t left = (size_t)(&d.slices.back() - &sl);  // slices still to come
            const size_t cap = (size_t)c3[2] + std::min<size_t>(left * d.max_recs, (size_t)c3[2] / 4 + 1024);
            FailRec* nr = nullptr;
            HIP_OK(dmalloc(&nr, cap * sizeof(FailRec)));
            if (c3[1]) HIP_OK(hipMemcpyAsync(nr, d.recs, (size_t)c3[1] * sizeof(FailRec), hipMemcpyDeviceToDevice, stream));
            HIP_OK(hipStreamSynchronize(stream));
            dfree(d.recs);
            d.recs = nr;
            d.recs_cap = cap;
            if (getenv("KYV_DEBUG_STATS"))
              fprintf(stderr, "[kyvgpu] resident failure records grown to %zu before slice [%u, %u)\n", cap, sl.k0, sl.k1);
          }
          appended = c3[2];
        } else {
          appended += d.max_recs;
        }
      }
      hipLaunchKernelGGL(compact_copy_kernel, dim3(ntiles), dim3(WAVE), 0, stream, d.stage, sl.rbase, d.rcnt, drules,
                         d.wl.nwaves, nchunks, d.tsum, d.tseg, d.recs, d.recs_cap, sl.k0, (const uint32_t*)d.nrecs);
      HIP_OK(hipGetLastError());
      HIP_OK(hipEventRecord(sl.ev[3], stream));
      if (acct) {  // compaction: chunk counts (read twice), tile sums, the staged records read, the dense records written
        uint32_t nr = 0;
        HIP_OK(hipMemcpyAsync(&nr, d.nrecs, 4, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        aphase[3] += 4ull * nchunks + 12ull * ntiles + staged + (uint64_t)nr * sizeof(FailRec);
      }
      // (no host synchronisation between slices: every slice has its own events, read after the evaluation)
      if (collect && multi) {  // gather this slice's records before the next slice reuses the buffers (offset 0)
        uint32_t nr = 0;
        HIP_OK(hipMemcpyAsync(&nr, d.nrecs, 4, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        if (nr > d.max_recs) throw std::runtime_error("failure record buffer overflow");
        const size_t at = host_recs.size();
        host_recs.resize(at + nr);
        if (nr) HIP_OK(hipMemcpy(host_recs.data() + at, d.recs, (size_t)nr * sizeof(FailRec), hipMemcpyDeviceToHost));
      }
    }
    // histogram blocks per CU: 8 (2.620 ms per evaluation) vs 2 (2.64 ms): more blocks stream the status bytes faster
    static const size_t hmul = getenv("KYV_HIST") ? (size_t)std::max(1, atoi(getenv("KYV_HIST"))) : 8;
    const uint32_t hgrid = (uint32_t)std::max<size_t>(
        1, std::min<size_t>(((size_t)d.cus * hmul + nrules - 1) / std::max<size_t>(1, nrules), (nres / 16 + HIST_BLOCK - 1) / HIST_BLOCK));
    if (joined) HIP_OK(hipStreamWaitEvent(stream, d.cjoin, 0));  // the histogram reads every verdict row
    if (nrules && nres) hipLaunchKernelGGL(status_hist_kernel, dim3(hgrid, (uint32_t)nrules), dim3(HIST_BLOCK), 0, stream, d.status, nres, d.counts);
    HIP_OK(hipGetLastError());
    if (acct) aphase[4] += (uint64_t)nres * nrules;  // the histogram reads every verdict byte
    HIP_OK(hipEventRecord(d.e1, stream));
    HIP_OK(hipEventSynchronize(d.e1));
    if (accumulate) {  // grown between slices above when needed: the list always holds every appended record
      uint32_t c[3] = {0, 0, 0};
      HIP_OK(hipMemcpy(c, d.nrecs, 12, hipMemcpyDeviceToHost));
      if (c[2] > d.recs_cap) throw std::runtime_error("failure record buffer overflow");
    }
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, d.e0, d.e1));
    total_ms += ms;
    if (nres)
      for (auto& sl : d.slices)
        if (sl.k1 > sl.k0) slice_phases(sl, &sl == &d.slices.front() ? d.e0 : sl.evs, phase);
    const double sum_after = phase[0] + phase[1] + phase[2] + phase[3];
    phase[4] += std::max(0.0, ms - (sum_after - sum_before));  // the rest: verdict histogram
    if (joined)  // the condition kernels' own span on their stream (overlapping the walk), per slice
      for (auto& sl : d.slices) {
        float cms = 0;
        if (!sl.cw.empty() && hipEventElapsedTime(&cms, sl.cev[0], sl.cev[1]) == hipSuccess) phase[1] += cms;
      }
  }
#ifdef KYV_EXP_STEPS
  {
    unsigned long long steps = 0;
    HIP_OK(hipMemcpyFromSymbol(&steps, HIP_SYMBOL(kyv_exp_steps), 8));
    fprintf(stderr, "[exp] walker loop iterations (wave-level, all launches so far): %llu\n", steps);
  }
#endif
  if (kernel_ms_avg) *kernel_ms_avg = total_ms / n;
  if (out) {
    out->nres = (uint32_t)nres;
    out->nrules = (uint32_t)nrules;
    out->kernel_ms = total_ms / n;
    for (int q = 0; q < 5; q++) out->phase_ms[q] = phase[q] / n;
    bool cond = false;
    for (auto& sl : d.slices) cond |= sl.nmc != 0;
    out->jit_used = (jit ? 1 : 0) | (jit && cond ? 2 : 0) | (jit && d.nshapes ? 4 : 0);
    out->h2d_ms = db->upload_ms;
    out->gmask_ms = db->gmask_ms;
    if (acct) {
      out->alg_bytes = 0;
      for (int q = 0; q < 5; q++) { out->alg_bytes_phase[q] = aphase[q]; out->alg_bytes += aphase[q]; }
      for (int q = 0; q < 3; q++) out->alg_bytes_class[q] = aclass[q];
    }
    std::vector<unsigned long long> rc(nrules * NSTATUS);
    if (nrules) HIP_OK(hipMemcpy(rc.data(), d.counts, rc.size() * 8, hipMemcpyDeviceToHost));
    // ST_NONE pairs are not tallied on the device
    out->rule_counts.assign(nrules * NSTATUS, 0);
    for (int s = 0; s < NSTATUS; s++) out->counts[s] = 0;
    for (size_t k = 0; k < nrules; k++) {
      int64_t counted = 0;
      for (int s = 1; s < NSTATUS; s++) {
        out->rule_counts[k * NSTATUS + s] = (int64_t)rc[k * NSTATUS + s];
        counted += (int64_t)rc[k * NSTATUS + s];
        out->counts[s] += (int64_t)rc[k * NSTATUS + s];
      }
      out->rule_counts[k * NSTATUS + ST_NONE] = (int64_t)nres - counted;
      out->counts[ST_NONE] += (int64_t)nres - counted;
    }
    if (copy_back) {
      auto t0 = std::chrono::steady_clock::now();
      out->status.resize(nres * nrules);
      HIP_OK(staged_d2h(out->status.data(), d.status, nres * nrules, d.stream));
      out->pss_fails.resize((size_t)d.npss * nres);
      if (d.npss) HIP_OK(hipMemcpy(out->pss_fails.data(), d.pss_fails, out->pss_fails.size() * 4, hipMemcpyDeviceToHost));
      if (multi) {
        d.host_recs = host_recs;  // export_failures serves the rows of this evaluation from the host copy
        out->fails.swap(host_recs);
      } else {
        uint32_t nr = 0;
        HIP_OK(hipMemcpy(&nr, d.nrecs, 4, hipMemcpyDeviceToHost));
        if (nr > d.max_recs) throw std::runtime_error("failure record buffer overflow");
        out->fails.resize(nr);
        if (nr) HIP_OK(hipMemcpy(out->fails.data(), d.recs, (size_t)nr * sizeof(FailRec), hipMemcpyDeviceToHost));
      }
      out->d2h_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
  }
}

struct HostSink {
  std::vector<FailRec>* out;
  uint32_t emitted;
  void emit(bool has, const FailRec& f) {
    if (has) { out->push_back(f); emitted++; }
  }
};

// Explicit CPU backend (development / message formatting only; never selected implicitly).
// With `account` set it also sums the algorithmic bytes of SURVEY §8(d) per pair: the header fields the
// match program reads (16 B), every distinct node-table row the pair touches (16 B each), the verdict byte,
// the PSS fail mask (4 B) and any failing-path records (32 B each). Dictionary columns are excluded.
void eval_cpu(const Ruleset& rs, const Batch& b, int threads, Results* out, bool account) {
  View v = make_view(rs, b, nullptr, nullptr, nullptr, nullptr);
  size_t nres = b.hdr.size(), nrules = rs.rules.size();
  out->nres = (uint32_t)nres;
  out->nrules = (uint32_t)nrules;
  out->status.assign(nres * nrules, ST_NONE);
  std::vector<uint32_t> pss_slot(nrules, NONE);
  uint32_t npss = 0;
  for (size_t k = 0; k < nrules; k++) if (rs.rules[k].kind == RK_PSS) pss_slot[k] = npss++;
  out->pss_fails.assign((size_t)npss * nres, 0);
  int T = std::max(1, threads);
  std::vector<std::vector<FailRec>> recs(T);
  std::vector<std::array<uint64_t, 5>> bytes(T, std::array<uint64_t, 5>{0, 0, 0, 0, 0});
  // device phase that decides each rule's pairs (kyv_results_phase_ms order): pattern walks 2, condition rules with
  // JMESPath operands / foreach 1 (the compiled condition kernel), the rest 0 (match kernel)
  std::vector<uint8_t> rphase(nrules, 0);
  for (size_t k = 0; k < nrules; k++) {
    const RuleDesc& rd = rs.rules[k];
    rphase[k] = (rd.kind == RK_PATTERN || rd.kind == RK_ANYPATTERN) ? 2 : rule_needs_jmes(rs, rd) ? 1 : 0;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t]() {
      Frame frames[MAX_DEPTH];
      HostWalker wk{Stack{frames, 1, MAX_DEPTH}};
      HostSink sink{&recs[t], 0};
      std::vector<uint8_t> seen;
      TouchAcct acct{nullptr, 0, 0};
      for (size_t r = t; r < nres; r += T)
        for (size_t k = 0; k < nrules; k++) {
          uint32_t pf;
          sink.emitted = 0;
          if (account) {
            uint32_t nn = b.hdr[r].nnodes;
            seen.assign(nn, 0);
            acct = TouchAcct{seen.data(), nn, 0};
            g_touch = &acct;
          }
          const uint32_t* gate = v.gate + (size_t)v.hdr[r].kclass * v.gate_words;
          const bool gated = ((gate[k >> 5] >> (k & 31)) & 1u) != 0;
          uint8_t st = eval_pair(v, gated, (uint32_t)r, (uint32_t)k, wk, &pf, sink);
          if (account) {
            g_touch = nullptr;
            auto& by = bytes[t];
            by[4] += 1;  // the verdict histogram reads every status byte
            if (!gated) {
              by[0] += 1;  // kind-gated pair: only the verdict reset writes it (no header or row is read)
            } else {
              by[rphase[k]] += 16 + 16 * acct.rows + 1 + (pss_slot[k] != NONE ? 4 : 0) +
                               (uint64_t)sink.emitted * sizeof(FailRec);
              by[3] += 2 * (uint64_t)sink.emitted * sizeof(FailRec);  // compaction reads + writes each record
            }
          }
          out->status[k * nres + r] = st;
          if (pss_slot[k] != NONE) out->pss_fails[(size_t)pss_slot[k] * nres + r] = pf;
        }
    });
  for (auto& x : th) x.join();
  out->fails.clear();
  for (auto& v2 : recs) out->fails.insert(out->fails.end(), v2.begin(), v2.end());
  for (int s = 0; s < NSTATUS; s++) out->counts[s] = 0;
  out->rule_counts.assign(nrules * NSTATUS, 0);
  for (size_t k = 0; k < nrules; k++)
    for (size_t r = 0; r < nres; r++) out->rule_counts[k * NSTATUS + (out->status[k * nres + r] & 7)]++;
  for (size_t k = 0; k < nrules; k++)
    for (int s = 0; s < NSTATUS; s++) out->counts[s] += out->rule_counts[k * NSTATUS + s];
  out->alg_bytes = 0;
  for (int q = 0; q < 5; q++) out->alg_bytes_phase[q] = 0;
  for (auto& x : bytes)
    for (int q = 0; q < 5; q++) { out->alg_bytes += x[q]; out->alg_bytes_phase[q] += x[q]; }
}

// Reason a pair came back ST_FALLBACK (kyv_results_fallback_reason): the rule's compile-time reason, else the host
// instantiation re-decides the one pair and reports the site that handed it over (KYV_WHY in kyv_eval.h / kyv_pss.h).
std::string fallback_why(const Ruleset& rs, const Batch& b, uint32_t res, uint32_t rule) {
  if (rule >= rs.rules.size() || res >= b.hdr.size()) return "";
  if (rs.rules[rule].kind == RK_FALLBACK) return rs.meta[rule].reason;
  View v = make_view(rs, b, nullptr, nullptr, nullptr, nullptr);
  Frame frames[MAX_DEPTH];
  HostWalker wk{Stack{frames, 1, MAX_DEPTH}};
  std::vector<FailRec> sink_recs;
  HostSink sink{&sink_recs, 0};
  const uint32_t* gate = v.gate + (size_t)v.hdr[res].kclass * v.gate_words;
  uint32_t pf = 0;
  g_fb_why = FBW_NONE;
  const uint8_t st = eval_pair(v, ((gate[rule >> 5] >> (rule & 31)) & 1u) != 0, res, rule, wk, &pf, sink);
  if ((st & 7) != ST_FALLBACK) return "";
  switch (g_fb_why) {
    case FBW_MATCH: return "match block outside the device subset";
    case FBW_PHRASE: return "resource string contains an anchor-error phrase (error classified by substring)";
    case FBW_COND: return "condition operand outside the device subset";
    case FBW_DEPTH: return "pattern walk deeper than the device frame stack";
    case FBW_VALUE: return "value outside the device subset (quantity beyond int128 nano units)";
    case FBW_META: return "anchor-like key under metadata (wildcard expansion)";
    default: return "pattern walk outside the device subset";
  }
}

// ---------------------------------------------------------------- pattern error texts (host)
// The error text of a pattern walk, for the RuleResponse.Message of pairs whose text the failure records cannot give:
// skip pairs (PatternError.Error() of a conditional / global anchor error), error pairs ("execution error: <err>") and
// anyPattern alternatives that failed without a path ("failed: <err>"). The one pair is walked again on the host along
// the compiled pattern program, in the order and with the handler semantics of eval_pattern, and with the error
// strings of the reference:
//   pkg/engine/validate/validate.go:31-56 (MatchPattern), :71-114 (validateResourceElement), :118-161 (validateMap),
//   :163-247 (validateArray / validateArrayOfMaps, multierr.Combine of the skip errors);
//   pkg/engine/anchor/handlers.go:31-275 (handler texts), anchor/error.go:12-90 (prefixes, typed vs substring checks).
// Values print as Go's fmt %v / %T of the unstructured decode (maps with sorted keys, float64 as strconv 'g' -1).
namespace {

// strconv.FormatFloat(f, 'g', -1, 64) (fmt %v of a float64): the shortest digits that round-trip, in %e form when
// the decimal exponent is < -4 or >= 6 (strconv/ftoa.go: eprec = 6 for the shortest precision), else %f form
std::string go_float_g(double f) {
  if (f != f) return "NaN";
  if (f == __builtin_inf()) return "+Inf";
  if (f == -__builtin_inf()) return "-Inf";
  char buf[64];
  std::string mant;
  int exp10 = 0;
  const bool neg = std::signbit(f);
  const double a = std::fabs(f);
  if (a == 0) {
    mant = "0";
  } else {
    for (int prec = 1; prec <= 17; prec++) {
      snprintf(buf, sizeof buf, "%.*e", prec - 1, a);
      if (strtod(buf, nullptr) == a) break;
    }
    const char* e = strchr(buf, 'e');
    exp10 = atoi(e + 1);
    for (const char* q = buf; q < e; q++) if (*q != '.') mant += *q;
    while (mant.size() > 1 && mant.back() == '0') mant.pop_back();
  }
  std::string out = neg ? "-" : "";
  const int nd = (int)mant.size(), dp = exp10 + 1;
  if (exp10 < -4 || exp10 >= 6) {
    out += mant[0];
    if (nd > 1) out += "." + mant.substr(1);
    char eb[16];
    snprintf(eb, sizeof eb, "e%c%02d", exp10 < 0 ? '-' : '+', exp10 < 0 ? -exp10 : exp10);
    return out + eb;
  }
  if (dp <= 0) return out + "0." + std::string(-dp, '0') + mant;
  if (dp >= nd) return out + mant + std::string(dp - nd, '0');
  return out + mant.substr(0, dp) + "." + mant.substr(dp);
}

struct TextWalk {
  const Ruleset& rs;
  const View& v;
  NodeTab R;
  const ResHeader& h;
  const RuleDesc& rd;
  uint64_t seen = 0, found = 0;
  Keys keys{NONE, NONE};
  bool bad = false;  // a case whose text needs the reference engine
  struct Err {
    bool err = false;
    uint8_t code = EC_NONE;  // typed anchor error (anchor/error.go) or EC_NONE: untyped, classified by substring
    std::string text;
  };
  std::string str(uint32_t sid) const { return std::string((const char*)v.heap + v.str_off[sid], v.str_len[sid]); }
  std::string gtype(uint32_t rn) const {  // fmt %T
    if (rn == NONE) return "<nil>";
    switch (node_type(R[rn])) {
      case N_MAP: return "map[string]interface {}";
      case N_ARR: return "[]interface {}";
      case N_STR: return "string";
      case N_INT: return "int64";
      case N_FLOAT: return "float64";
      case N_TRUE: case N_FALSE: return "bool";
      default: return "<nil>";
    }
  }
  std::string gval(uint32_t rn, int depth = 0) {  // fmt %v
    if (rn == NONE || depth > 64) return "<nil>";
    const Node& n = R[rn];
    switch (node_type(n)) {
      case N_NULL: return "<nil>";
      case N_TRUE: return "true";
      case N_FALSE: return "false";
      case N_INT: return std::to_string((int64_t)(((uint64_t)n.b << 32) | n.a));
      case N_FLOAT: return go_float_g(__builtin_bit_cast(double, ((uint64_t)n.b << 32) | n.a));
      case N_STR: return str(n.a);
      case N_ARR: {
        std::string o = "[";
        for (uint32_t i = 0; i < n.b; i++) o += (i ? " " : "") + gval(n.a + i, depth + 1);
        return o + "]";
      }
      case N_MAP: {
        std::vector<std::pair<std::string, uint32_t>> kv;
        for (uint32_t i = 0; i < n.b; i++) kv.push_back({str(node_key(R[n.a + i])), n.a + i});
        std::sort(kv.begin(), kv.end());
        std::string o = "map[";
        for (size_t i = 0; i < kv.size(); i++) o += (i ? " " : "") + kv[i].first + ":" + gval(kv[i].second, depth + 1);
        return o + "]";
      }
      default: return "<nil>";
    }
  }
  std::string pval(const Leaf& L) {  // %v of a pattern scalar (pattern numbers are float64 after the JSON decode)
    switch (L.type) {
      case L_NIL: return "<nil>";
      case L_BOOL: return L.bval ? "true" : "false";
      case L_FLOAT: return go_float_g(L.f);
      case L_STR: return str(L.exact);
      default: bad = true; return "";
    }
  }
  static bool has(const std::string& t, const char* p) { return t.find(p) != std::string::npos; }
  static bool is_skip(const Err& e) {
    if (e.code != EC_NONE) return e.code == EC_COND || e.code == EC_GLOBAL;
    return has(e.text, "conditional anchor mismatch") || has(e.text, "global anchor mismatch");
  }
  static bool is_neg(const Err& e) {
    return e.code != EC_NONE ? e.code == EC_NEG : has(e.text, "negation anchor matched in resource");
  }
  static Err mk(uint8_t code, std::string t) { Err e; e.err = true; e.code = code; e.text = std::move(t); return e; }
  bool leaf_ok(const Leaf& L, uint32_t rn) {
    bool fb = false;
    const bool ok = leaf_match(v, L, value_of(v, R, rn), &fb);
    if (fb) bad = true;
    return ok;
  }
  Err leaf(const Leaf& L, uint32_t rn, const std::string& path, std::string* rp) {  // validate.go:92-107
    bool ok = true;
    if (rn != NONE && node_type(R[rn]) == N_ARR) {
      for (uint32_t i = 0; i < R[rn].b && ok; i++) ok = leaf_ok(L, R[rn].a + i);
    } else {
      ok = leaf_ok(L, rn);
    }
    if (ok) return Err{};
    *rp = path;
    return mk(EC_NONE, "resource value '" + gval(rn) + "' does not match '" + pval(L) + "' at path " + path);
  }
  // validateArray / validateArrayOfMaps element loop: skip errors collected, anything else returned
  Err elems(uint32_t rn, uint32_t n, const std::function<uint32_t(uint32_t)>& pat, const std::string& path, std::string* rp) {
    std::vector<std::string> skips;
    uint32_t applied = 0;
    for (uint32_t i = 0; i < n && !bad; i++) {
      std::string p;
      Err e = elem(R[rn].a + i, pat(i), path + std::to_string(i) + "/", &p);
      if (!e.err) { applied++; continue; }
      if (is_skip(e)) { skips.push_back(e.text); continue; }
      *rp = p;
      return e;
    }
    if (applied == 0 && !skips.empty()) {  // PatternError{multierr.Combine(skips...)}: untyped
      std::string t;
      for (size_t i = 0; i < skips.size(); i++) t += (i ? "; " : "") + skips[i];
      *rp = path;
      return mk(EC_NONE, t);
    }
    return Err{};
  }
  Err elem(uint32_t rn, uint32_t pn, const std::string& path, std::string* rp) {
    if (bad || pn >= rs.pnodes.size() || path.size() > 4096) { bad = true; return Err{}; }
    const PNode& P = rs.pnodes[pn];
    const uint32_t rt = rn == NONE ? 0xFF : node_type(R[rn]);
    switch (P.kind) {
      case P_MAP:
        if (rt != N_MAP) {
          *rp = path;
          return mk(EC_NONE, "pattern and resource have different structures. Path: " + path +
                                 ". Expected map[string]interface {}, found " + gtype(rn));
        }
        return map(rn, P, path, rp);
      case P_LEAF: return leaf(rs.leaves[P.first], rn, path, rp);
      default: break;
    }
    if (rt != N_ARR) {
      *rp = path;
      return mk(EC_NONE, "validation rule failed at path " + path + ", resource does not satisfy the expected overlay pattern");
    }
    const uint32_t cnt = R[rn].b;
    switch (P.kind) {
      case P_ARR_EMPTY: *rp = path; return mk(EC_NONE, "pattern Array empty");
      case P_ARR_SCALAR: return leaf(rs.leaves[rs.pnodes[P.first].first], rn, path, rp);
      case P_ARR_MAPS: return elems(rn, cnt, [&](uint32_t) { return P.first; }, path, rp);
      case P_ARR_POS:
        if (cnt < P.n) {
          *rp = "";
          return mk(EC_NONE, "validate Array failed, array length mismatch, resource Array len is " + std::to_string(cnt) +
                                 " and pattern Array len is " + std::to_string(P.n));
        }
        return elems(rn, P.n, [&](uint32_t i) { return rs.pool[P.first + i]; }, path, rp);
      default: bad = true; return Err{};
    }
  }
  Err map(uint32_t rn, const PNode& P, const std::string& path, std::string* rp) {
    // AnchorMap.CheckAnchorInResource before this level's metadata expansion, as eval_pattern does
    for (uint32_t e = 0; e < P.n; e++) {
      const PEntry& E = rs.pentries[P.first + e];
      if (E.abit == 0xFF) continue;
      const uint64_t b1 = 1ull << E.abit;
      seen |= b1;
      const uint32_t key = (E.flags & EF_WILD) ? keys.get(E.slot) : E.key;
      if (!(found & b1) && map_find(R, rn, key) != NONE) found |= b1;
    }
    if (P.flags & PF_META) {
      if (expand_meta(v, rs.metas[rd.meta_sites + P.meta], R, rn, h, keys) != ST_NONE) { bad = true; return Err{}; }
    }
    for (uint32_t e = 0; e < P.n && !bad; e++) {
      const PEntry& E = rs.pentries[P.first + e];
      const uint32_t key = (E.flags & EF_WILD) ? keys.get(E.slot) : E.key;
      if (key == NONE) { bad = true; return Err{}; }
      const uint32_t c = map_find(R, rn, key);
      const std::string cur = path + str(key) + "/";
      std::string p;
      switch (E.handler) {
        case H_NEGATION:  // handlers.go:66-77
          if (c != NONE) { *rp = cur; return mk(EC_NEG, "negation anchor matched in resource: " + cur + " is not allowed"); }
          break;
        case H_EQUALITY: {  // handlers.go:96-109
          if (c == NONE) break;
          Err x = elem(c, E.child, cur, &p);
          if (x.err) { *rp = p; return x; }
          break;
        }
        case H_GLOBAL: {  // handlers.go:195-209
          if (c == NONE) break;
          Err x = elem(c, E.child, cur, &p);
          if (x.err) { *rp = p; return mk(EC_GLOBAL, "global anchor mismatch: " + x.text); }
          break;
        }
        case H_CONDITION: {  // handlers.go:160-176
          if (c == NONE) { *rp = cur; return mk(EC_COND, "conditional anchor mismatch: conditional anchor key doesn't exist in the resource"); }
          Err x = elem(c, E.child, cur, &p);
          if (x.err) { *rp = p; return mk(EC_COND, "conditional anchor mismatch: " + x.text); }
          break;
        }
        case H_STAR:  // handlers.go:128-141: "*" needs a non-nil value; the error returns the parent path
          if (c != NONE && node_type(R[c]) != N_NULL) break;
          *rp = path;
          return mk(EC_NONE, path + "/" + str(key) + " not found");
        case H_EXISTENCE: case H_EXIST_BADPAT: {  // handlers.go:228-275
          if (c == NONE) break;
          if (node_type(R[c]) != N_ARR) {
            *rp = cur;
            return mk(EC_NONE, "invalid resource type " + gtype(c) + ": Existence ^ () anchor can be used only on list/array type resource");
          }
          if (E.handler == H_EXIST_BADPAT) { bad = true; return Err{}; }  // the text names the pattern's Go type
          for (uint32_t j = 0; j < rs.pool[E.child]; j++) {
            bool hit = false;
            for (uint32_t i = 0; i < R[c].b && !hit && !bad; i++) {
              std::string q;
              hit = !elem(R[c].a + i, rs.pool[E.child + 1 + j], cur + std::to_string(i) + "/", &q).err;
            }
            if (!hit) { *rp = cur; return mk(EC_NONE, "existence anchor validation failed at path " + cur); }
          }
          break;
        }
        default: {  // H_DEFAULT: resourceMap[k] (absent -> nil)
          Err x = elem(c, E.child, cur, &p);
          if (x.err) { *rp = p; return x; }
        }
      }
    }
    return Err{};
  }
};

}  // namespace

// MatchPattern of one compiled pattern root for resource `res` (kind-major position): the status the reference
// derives (validate.go:31-56) and, for a non-nil PatternError, its Path and Error() text. false: a case whose text the
// host does not render (the reference engine decides the message).
bool pattern_error_text(const Ruleset& rs, const Batch& b, uint32_t res, uint32_t rule, uint32_t root, uint8_t* status,
                        std::string* path, std::string* text) {
  if (rule >= rs.rules.size() || res >= b.hdr.size()) return false;
  View v = make_view(rs, b, nullptr, nullptr, nullptr, nullptr);
  const ResHeader& h = b.hdr[res];
  TextWalk w{rs, v, NodeTab{b.nodes.data() + h.root}, h, rs.rules[rule]};
  std::string p;
  TextWalk::Err e = w.elem(0, root, "/", &p);
  if (w.bad) return false;
  text->clear();
  path->clear();
  if (!e.err) { *status = ST_PASS; return true; }
  *text = e.text;
  if (TextWalk::is_skip(e)) { *status = ST_SKIP; return true; }
  if (TextWalk::is_neg(e)) { *status = ST_FAIL; *path = p; return true; }
  if (w.seen & ~w.found) { *status = ST_ERROR; return true; }  // AnchorMap.KeysAreMissing
  *path = p;
  *status = p.empty() ? ST_ERROR : ST_FAIL;
  return true;
}

// ---------------------------------------------------------------- device-resident result export
// The multi-GPU collectives of scan.py (gather_verdicts / gather_failures) all-gather straight from the
// verdicts and failing-path records a batch's last evaluation left on its device: these kernels write the wire form
// into a caller-owned device buffer (a torch tensor) on the caller's stream, in input order, so no host copy is made.

// verdicts two per byte (low nibble: even resource), rule-major rows of ceil(nres / 2) bytes
__global__ void __launch_bounds__(256) pack_status_kernel(const uint8_t* __restrict__ status,
                                                          const uint32_t* __restrict__ inv, size_t nres, size_t half,
                                                          size_t total, uint8_t* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const size_t k = i / half, j = i - k * half;
  const uint8_t* row = status + k * nres;
  const uint8_t a = row[inv[2 * j]] & 7u;
  const uint8_t b = 2 * j + 1 < nres ? (uint8_t)(row[inv[2 * j + 1]] & 7u) : (uint8_t)0;
  dst[i] = (uint8_t)(a | (b << 4));
}

// failing-path records as int64 rows (global resource index, rule, alternative, path template, idx0..3)
__global__ void __launch_bounds__(256) failure_rows_kernel(const FailRec* __restrict__ recs, uint32_t n,
                                                           const uint32_t* __restrict__ order, long long off,
                                                           long long* __restrict__ dst) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const FailRec f = recs[i];
  long long* o = dst + (size_t)i * 8;
  o[0] = (long long)order[f.res] + off;
  o[1] = f.rule;
  o[2] = f.alt;
  o[3] = f.tmpl;  // NONE (no path) as the host rows carry it
  for (int q = 0; q < MAX_IDX; q++) o[4 + q] = f.idx[q];
}

static DevBatch* resident(const Batch& b, int device) {
  if (device < 0 || device >= (int)b.dev.size() || !b.dev[device] || !((DevBatch*)b.dev[device])->out)
    throw std::runtime_error("no device-resident results for this batch on that device (evaluate with the GPU backend first)");
  DevBatch* db = (DevBatch*)b.dev[device];
  HIP_OK(hipSetDevice(device));
  if (!db->inv) {
    const size_t n = b.inv.size();
    std::vector<uint32_t> order(n);
    for (size_t i = 0; i < n; i++) order[b.inv[i]] = (uint32_t)i;
    HIP_OK(dmalloc(&db->inv, std::max<size_t>(4, n * 4)));
    HIP_OK(dmalloc(&db->order, std::max<size_t>(4, n * 4)));
    if (n) {
      HIP_OK(hipMemcpy(db->inv, b.inv.data(), n * 4, hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(db->order, order.data(), n * 4, hipMemcpyHostToDevice));
    }
  }
  return db;
}

int64_t export_status(const Batch& b, int device, uint8_t* dst, size_t cap, void* stream) {
  DevBatch* db = resident(b, device);
  const DeviceResults& d = *db->out;
  const size_t half = (d.nres + 1) / 2, total = half * d.nrules;
  if (!dst) return (int64_t)total;
  if (cap < total) throw std::runtime_error("export buffer too small");
  if (total) {
    hipLaunchKernelGGL(pack_status_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)d.status, (const uint32_t*)db->inv, d.nres, half, total, dst);
    HIP_OK(hipGetLastError());
  }
  return (int64_t)total;
}

// verdict bytes of input-order resources [res0, res0 + n) of every rule, rule-major, gathered on the device from the
// resident (kind-major) rows
__global__ void __launch_bounds__(256) status_rows_kernel(const uint8_t* __restrict__ status, const uint32_t* __restrict__ inv,
                                                          size_t nres, size_t res0, size_t n, size_t total,
                                                          uint8_t* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const size_t k = i / n, j = i - k * n;
  dst[i] = status[k * nres + inv[res0 + j]] & 7u;
}

int64_t copy_status(const Batch& b, int device, size_t res0, size_t n, uint8_t* host_dst, size_t cap) {
  DevBatch* db = resident(b, device);
  const DeviceResults& d = *db->out;
  if (res0 > d.nres) throw std::runtime_error("resource range out of bounds");
  n = std::min(n, d.nres - res0);
  const size_t total = n * d.nrules;
  if (!host_dst) return (int64_t)total;
  if (cap < total) throw std::runtime_error("status buffer too small");
  if (total) {
    uint8_t* tmp = nullptr;
    HIP_OK(dmalloc(&tmp, total));
    hipLaunchKernelGGL(status_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, d.stream,
                       (const uint8_t*)d.status, (const uint32_t*)db->inv, d.nres, res0, n, total, tmp);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(host_dst, tmp, total, hipMemcpyDeviceToHost, d.stream));
    HIP_OK(hipStreamSynchronize(d.stream));
    dfree(tmp);
  }
  return (int64_t)total;
}

// The last evaluation's failing-path records: device-resident (one dense list, every rule slice appended), or for a
// rule-sliced evaluation with copy-back the host copy its slices were gathered into (uploaded for the export)
static const FailRec* failure_records(const Batch& b, int device, uint32_t* n, void* stream) {
  DevBatch* db = resident(b, device);
  DeviceResults& d = *db->out;
  if (!d.recs_resident) {
    if (d.host_recs.size() > 0xFFFFFFFFull) throw std::runtime_error("too many failing-path records for one export");
    *n = (uint32_t)d.host_recs.size();
    if (*n > d.hrecs_cap) {
      dfree(d.hrecs_dev);
      d.hrecs_dev = nullptr;
      d.hrecs_cap = 0;
      HIP_OK(dmalloc(&d.hrecs_dev, (size_t)*n * sizeof(FailRec)));
      d.hrecs_cap = *n;
    }
    if (*n) HIP_OK(hipMemcpyAsync(d.hrecs_dev, d.host_recs.data(), (size_t)*n * sizeof(FailRec), hipMemcpyHostToDevice,
                                  (hipStream_t)stream));
    return (const FailRec*)d.hrecs_dev;
  }
  uint32_t c[3] = {0, 0, 0};
  HIP_OK(hipMemcpy(c, d.nrecs, 12, hipMemcpyDeviceToHost));
  if (c[2] > d.recs_cap)
    throw std::runtime_error("the evaluation's failing-path records exceed the resident record buffer (" +
                             std::to_string(c[2]) + " > " + std::to_string(d.recs_cap) +
                             "): evaluate with copy-back to gather them slice by slice");
  *n = c[2];
  return (const FailRec*)d.recs;
}

int64_t export_failures(const Batch& b, int device, int64_t off, int64_t* dst, size_t cap_rows, void* stream) {
  DevBatch* db = resident(b, device);
  uint32_t nr = 0;
  if (!dst) {  // the count only (no upload of a host copy)
    const DeviceResults& d = *db->out;
    if (!d.recs_resident) return (int64_t)d.host_recs.size();
    failure_records(b, device, &nr, stream);
    return nr;
  }
  const FailRec* recs = failure_records(b, device, &nr, stream);
  if (cap_rows < nr) throw std::runtime_error("export buffer too small");
  if (nr) {
    hipLaunchKernelGGL(failure_rows_kernel, dim3((nr + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       recs, nr, (const uint32_t*)db->order, (long long)off, (long long*)dst);
    HIP_OK(hipGetLastError());
  }
  return nr;
}

// The same rows packed to 16 bytes for the report gather to one consumer rank (kyv_comm_gather_report): per record
// uint32 {input-order resource index on this rank, rule | alternative << 24, path template, four 8-bit path indices};
// a record whose rule, alternative or indices do not fit (rule >= 2^24, alternative >= 128, an index >= 255 other
// than the 0xFFFF "unused" value) sets bit 31 of word 1 and carries the index of a 16-byte side entry {rule,
// alternative, indices as 16-bit values} in word 3 instead (the side list's order is not deterministic; the index
// ties each entry to its row)
__global__ void __launch_bounds__(256) report_rows_kernel(const FailRec* __restrict__ recs, uint32_t n,
                                                          const uint32_t* __restrict__ order, uint4* __restrict__ rows,
                                                          uint4* __restrict__ wide, uint32_t* __restrict__ nwide,
                                                          uint32_t cap_wide) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const FailRec f = recs[i];
  bool fit = f.rule < (1u << 24) && f.alt < 128;
  uint32_t packed = 0;
  for (int q = 0; q < MAX_IDX; q++) {
    const uint32_t x = f.idx[q];
    fit = fit && (x < 255 || x == 0xFFFF);
    packed |= (x == 0xFFFF ? 255u : (x & 255u)) << (8 * q);
  }
  uint4 r;
  r.x = order[f.res];
  r.z = f.tmpl;
  if (fit) {
    r.y = f.rule | ((uint32_t)f.alt << 24);
    r.w = packed;
  } else {
    const uint32_t j = atomicAdd(nwide, 1u);
    r.y = 0x80000000u;
    r.w = j;
    if (j < cap_wide)
      wide[j] = make_uint4(f.rule, f.alt, (uint32_t)f.idx[0] | ((uint32_t)f.idx[1] << 16),
                           (uint32_t)f.idx[2] | ((uint32_t)f.idx[3] << 16));
  }
  rows[i] = r;
}

int64_t export_report_rows(const Batch& b, int device, uint32_t* rows, uint32_t* wide, uint32_t* nwide_dev,
                           size_t cap_rows, size_t cap_wide, void* stream) {
  DevBatch* db = resident(b, device);
  uint32_t nr = 0;
  const FailRec* recs = failure_records(b, device, &nr, stream);
  if (!rows) return nr;
  if (cap_rows < nr) throw std::runtime_error("export buffer too small");
  HIP_OK(hipMemsetAsync(nwide_dev, 0, 4, (hipStream_t)stream));
  if (nr) {
    hipLaunchKernelGGL(report_rows_kernel, dim3((nr + 255) / 256), dim3(256), 0, (hipStream_t)stream, recs, nr,
                       (const uint32_t*)db->order, (uint4*)rows, (uint4*)wide, nwide_dev, (uint32_t)cap_wide);
    HIP_OK(hipGetLastError());
  }
  return nr;
}

// the per-rule verdict tallies of the last evaluation, device-resident ([rules][NSTATUS] uint64, ST_NONE not
// tallied: the caller derives it from the resource count)
const unsigned long long* device_counts(const Batch& b, int device, size_t* nrules, size_t* nres) {
  DevBatch* db = resident(b, device);
  *nrules = db->out->nrules;
  *nres = db->out->nres;
  return (const unsigned long long*)db->out->counts;
}

void free_device_images(Ruleset& rs, Batch* b) {
  if (b) {
    for (auto* p : b->dev)
      if (p) {
        DevBatch* d = (DevBatch*)p;
        hipSetDevice(d->device);
        dfree(d->base);
        dfree(d->gmask);
        dfree(d->inv);
        dfree(d->order);
        if (d->out) { free_dev_results(*d->out, d->device); delete d->out; }
        delete d;
      }
    b->dev.clear();
  } else {
    for (auto* p : rs.dev)
      if (p) {
        DevRuleset* d = (DevRuleset*)p;
        hipSetDevice(d->device);
        hipFree(d->base);
        if (d->jmod) hipModuleUnload(d->jmod);
        delete d;
      }
    rs.dev.clear();
  }
}

// one calibration launch (see calib_read_kernel): mode 4 / 8 / 16 = coalesced reads of that many bytes per lane, 116 =
// gather of 16-byte rows; bytes rounded down to a power of two for the gather. Returns the launch's device time (ms)
double calibrate_fetch(int device, size_t bytes, int mode) {
  HIP_OK(hipSetDevice(device));
  if (mode == 116) { size_t b = 16; while (b * 2 <= bytes) b *= 2; bytes = b; }
  uint8_t* p = nullptr;
  uint32_t* out = nullptr;
  HIP_OK(hipMalloc(&p, bytes));
  HIP_OK(hipMalloc(&out, 4));
  struct Free { void* a; void* b; ~Free() { (void)hipFree(a); (void)hipFree(b); } } fr{p, out};
  HIP_OK(hipMemset(p, 1, bytes));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  const unsigned grid = 256 * 32;
  HIP_OK(hipEventRecord(e0, nullptr));
  switch (mode) {
    case 4: hipLaunchKernelGGL(calib_read_kernel<4>, dim3(grid), dim3(256), 0, nullptr, p, bytes, out); break;
    case 8: hipLaunchKernelGGL(calib_read_kernel<8>, dim3(grid), dim3(256), 0, nullptr, p, bytes, out); break;
    case 16: hipLaunchKernelGGL(calib_read_kernel<16>, dim3(grid), dim3(256), 0, nullptr, p, bytes, out); break;
    case 116: hipLaunchKernelGGL(calib_gather_kernel, dim3(grid), dim3(256), 0, nullptr, (const uint4*)p, bytes / 16, out); break;
    default: throw std::runtime_error("calibrate_fetch: mode 4, 8, 16 or 116");
  }
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(e1, nullptr));
  HIP_OK(hipEventSynchronize(e1));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms;
}

}  // namespace kyv
