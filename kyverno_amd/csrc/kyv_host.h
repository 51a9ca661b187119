// Host-side objects behind the C-ABI handles (kyv_ruleset / kyv_batch / kyv_results).
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "kyv_layout.h"
#include "pjson.h"

namespace kyv {

// String dictionary: seeded with the fixed/well-known ids, then the ruleset literals; every batch copies
// the ruleset dictionary and appends its own strings.
// vector storage without value-initialisation: the flattener's large tables are written once, in parallel, so
// zero-filling them first (serially) would only add page-fault and memset time
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U> struct rebind { using other = NoInitAlloc<U>; };
  NoInitAlloc() = default;
  template <class U> NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  template <class U> void construct(U* p) noexcept { ::new ((void*)p) U; }
  template <class U, class... A> void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};
template <class T> using bulk_vector = std::vector<T, NoInitAlloc<T>>;

struct Dict {
  std::vector<std::string> strs;
  std::unordered_map<std::string, uint32_t> ids;
  uint32_t intern(const std::string& s) {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    uint32_t id = (uint32_t)strs.size();
    strs.push_back(s);
    ids.emplace(s, id);
    return id;
  }
  uint32_t find(const std::string& s) const {
    auto it = ids.find(s);
    return it == ids.end() ? NONE : it->second;
  }
};
void seed_dict(Dict& d);  // fixed + well-known + volume sources, in enum order

struct RuleMeta {
  std::string name;
  std::string message;        // validate.message
  uint32_t policy = 0;
  uint8_t kind = RK_NONE;
  std::string reason;         // RK_FALLBACK / RK_PANIC / RK_ERROR reason
  bool message_vars = false;  // message needs variable substitution (CPU)
  bool foreach_texts = true;  // foreach rule whose entries are all top-level deny: fail texts rendered by the library
  std::string pss_level, pss_version;
  // deny failure message (getDenyMessage, validation.go:466-479): literal text and `{{ request.object... }}`
  // references (key sids); msg_whole_var: the message is exactly one reference
  struct MsgPart { std::string text; std::vector<uint32_t> segs; bool var = false; };
  std::vector<MsgPart> msg_parts;
  bool msg_whole_var = false;
  // MatchResources.GetKinds of the (autogen-expanded) rule and Rule.HasValidate: the policy cache's kind index
  // (pkg/policycache/store.go:96-138)
  std::vector<std::string> kinds;
  bool has_validate = false;
  // keys (cache.MetaNamespaceKeyFunc) of the PolicyExceptions naming the rule, in candidate order (RuleDesc.exc)
  std::vector<std::string> exc_keys;
};

// host-side text of a condition's references, for error messages (vars.go:395-399)
struct CondText {
  std::string var[2];   // key / value: variable text (replaceBracesAndTrimSpaces)
  std::string path[2];  // JSON pointer of the operand in the conditions document (data.Path)
  std::vector<std::string> segs[2];
};

struct PolicyMeta {
  std::string name, ns, kind;
  bool apply_one = false;
  bool scored_false = false;       // policies.kyverno.io/scored: "false" -> fail reported as warn
  std::string failure_action;
  uint32_t first_rule = 0, nrules = 0;  // computed rules (incl. non-validate ones, kind RK_NONE)
  std::vector<std::string> all_rule_names;  // every computed rule name in order (CLI "rule absent -> skip")
};

// regex_match pattern as a DFA over printable ASCII (regex.cpp): next[state * RX_SYMS + (c - 0x20)], state 0 the start
struct RxDfa {
  uint32_t nstates = 0;
  std::vector<uint16_t> next;
  std::vector<uint8_t> accept;
  bool end_anchor = false;  // '$': accept only at the end of the subject (else as soon as an accepting state is reached)
};
// compile a regex_match pattern (false + *why outside the device subset, regex.cpp)
bool rx_compile(const std::string& re, RxDfa* out, std::string* why);
// regexp.Match of the compiled pattern on a subject: 1 / 0, -1 when the subject has a byte outside printable ASCII
int rx_match(const RxDfa& d, const uint8_t* s, size_t n);

struct Ruleset {
  Dict dict;                    // seed dictionary (fixed ids + literals)
  std::vector<RuleDesc> rules;
  std::vector<RuleMeta> meta;
  std::vector<PolicyMeta> policies;
  std::vector<Filter> filters;
  std::vector<KindDesc> kinds;
  std::vector<SelDesc> sels;
  std::vector<SelReq> reqs;
  std::vector<PNode> pnodes;
  std::vector<PEntry> pentries;
  std::vector<Leaf> leaves;
  std::vector<Atom> atoms;
  std::vector<MetaSite> metas;
  std::vector<PssDesc> pss;
  std::vector<uint32_t> pool;
  std::vector<Node> cnodes;     // condition literals
  std::vector<Cond> conds;
  std::vector<CondProg> cprogs;
  std::vector<CondText> cond_text;
  std::vector<std::string> templates;  // path templates: '\x01'+slot = array index, '\x02'+slot = resolved key
  std::unordered_map<std::string, uint32_t> template_ids;  // interned: identical patterns share template ids
  // path trie over every static lookup of every compiled pattern (kyv_layout.h "Path columns")
  struct TrieNode {
    uint32_t col = NONE;        // column id (key edges; "[*]" nodes: the elements' self column)
    uint32_t rowspace = 0;      // row space the column / this node's lookups live in
    uint32_t star = NONE;       // "[*]" child (opens row space trie[star].rowspace)
    uint32_t lencol = NONE;     // with a "[*]" child: column (this node's row space) of the array's (count, row of
                                // element 0) as (low, high) words
    std::vector<std::pair<uint32_t, uint32_t>> kids;  // (key sid, child trie node)
  };
  std::vector<TrieNode> trie;   // trie[0] = resource root
  std::vector<uint32_t> gpats;  // wildcard patterns with a per-string glob mask (index g: mask bit g, SF_GIDX_SHIFT)
  // condition-set masks (compiler.cpp assign_cond_sets): set q's bit (gpats.size() + q) of string s = wild2(s, e) for
  // some literal sid e of the set; cond_set[ci] = set index + 1 of condition ci, 0 none
  std::vector<std::vector<uint32_t>> gsets;
  std::vector<uint32_t> cond_set;
  // round 6: JMESPath functions on the dictionary -- regex_match patterns (JO_REGEX q = rxs[q]) and whether some
  // program applies to_upper (JO_UPPER): the batch then computes Batch::str_rx / str_upper once per string
  std::vector<std::string> rx_src;
  std::vector<RxDfa> rxs;
  bool uses_upper = false;
  uint32_t ncols = 0, nrowspaces = 1;
  std::vector<uint32_t> col_rowspace;
  std::vector<uint32_t> pn_self;  // array pnode -> self column of its elements (NONE: none)
  std::vector<uint32_t> pe_self;  // existence entry -> self column of the candidate elements
  std::vector<uint32_t> pn_len;   // array pnode -> its length column (TrieNode::lencol) or NONE
  std::vector<uint32_t> pe_len;   // existence entry -> length column of the candidate array
  // runtime-compiled walk kernel (jit.cpp): generated once per ruleset, compiled on first use
  bool jit_tried = false;
  std::vector<uint8_t> jit_rules;   // rule k is walked by the compiled kernel
  std::vector<uint8_t> jit_cond;    // rule k (deny / foreach with JMESPath operands) runs in the compiled kyv_jit_cond (1), or folded into fused group g's walk (2 + g)
  std::vector<uint16_t> jit_shape;  // 1 + the pattern shape of rule k in kyv_jit_shapes (0: none; jit.cpp)
  uint32_t jit_nshapes = 0;
  std::vector<char> jit_code;       // gfx950 code object
  std::vector<char> jit_code_acct;  // the same source compiled with -DKYV_ACCT (byte-accounting evaluation only)
  std::string jit_error;
  double jit_compile_s = 0;
  // device copies (one per device, lazily uploaded)
  std::vector<void*> dev;
  ~Ruleset();
};

// whole-object typed decode of getSpec (validation.go:481-532; typed.cpp, types in k8s_types.h), per batch: the
// schema's field names resolved to the batch dictionary once
struct TypedDecoder {
  enum Target { POD = 0, DEPLOYMENT = 1, CRONJOB = 2 };
  explicit TypedDecoder(const std::function<uint32_t(const std::string&)>& find_sid);
  // json.Unmarshal of the resource (node table R, dictionary strs) into the target type: DEC_OK, DEC_ERR, or DEC_FOLD
  // (it succeeds, some key matching its field only case-insensitively)
  enum Outcome { DEC_OK = 0, DEC_ERR = 1, DEC_FOLD = 2 };
  int decode(const Node* R, const std::vector<std::string>& strs, int target) const;
  std::unordered_map<uint32_t, uint32_t> name_of_sid;  // dictionary id -> schema field name index
};

struct Batch {
  const Ruleset* rs = nullptr;
  Dict dict;                      // ruleset dict + batch strings
  bulk_vector<Node> nodes;
  bulk_vector<ResHeader> hdr;
  std::vector<FloatAux> faux;
  std::vector<uint32_t> str_off, str_len, str_flags;
  std::vector<uint32_t> str_upper, str_rx;  // JMESPath functions on the dictionary (empty: the ruleset uses none)
  std::vector<int64_t> str_dur, str_qty;
  std::vector<double> str_f64;
  std::vector<uint8_t> heap;
  std::vector<uint32_t> nsl_off, nsl_kv;
  std::vector<std::string> nsl_names;  // namespace name per set id
  // kind-major order: headers are sorted by kind class so that a wave's lanes share kind (and so mostly share
  // the rules that can match them); verdicts are produced in this order and un-permuted at the C ABI
  std::vector<uint32_t> order;    // sorted position -> input index
  std::vector<uint32_t> inv;      // input index -> sorted position
  std::shared_ptr<const std::vector<uint32_t>> inv_shared;  // immutable copy handed to results (capi.cpp)
  std::vector<uint32_t> gate;     // [kclass][gate_words] bit k: rule k can match a resource of this class
  uint32_t gate_words = 0, nclass = 0;
  // path columns (kyv_layout.h): colv[col_off[c] + row]
  bulk_vector<uint64_t> colv;
  std::vector<uint32_t> col_off, rs_rows;
  std::vector<void*> dev;
  ~Batch();
};

struct FailPath {  // decoded path record
  uint32_t res, rule, alt;
  uint32_t tmpl;
  uint16_t idx[MAX_IDX];
  uint32_t key[2];
};

struct Results {
  uint32_t nres = 0, nrules = 0;
  std::vector<uint8_t> status;      // [rule][res]
  std::vector<uint32_t> pss_fails;  // [rule][res] for PSS rules (empty otherwise)
  std::vector<FailRec> fails;
  int64_t counts[NSTATUS] = {0};
  std::vector<int64_t> rule_counts;  // [rule][status] (report summaries)
  double kernel_ms = 0, h2d_ms = 0, d2h_ms = 0;
  double gmask_ms = 0;  // per-batch device work outside the evaluation: the glob-mask kernel (h2d_ms: the image upload)
  // GPU evaluation split by phase (HIP events on the evaluation stream, averaged over the timed launches):
  // [0] verdict resets + match_kernel(s), [1] compiled condition kernel, [2] pattern walk kernels,
  // [3] failing-path compaction, [4] verdict histogram
  double phase_ms[5] = {0, 0, 0, 0, 0};
  uint64_t alg_bytes = 0;           // CPU backend with KYV_EVAL_ACCOUNT_BYTES
  uint64_t alg_bytes_phase[5] = {0, 0, 0, 0, 0};  // the same split by the device phase that moves them (phase_ms)
  uint64_t alg_bytes_class[3] = {0, 0, 0};  // GPU accounting: counted reads, writes, staged records (kernel counters)
  int jit_used = 0;                 // bit 0: the runtime-compiled walk kernels ran; bit 1: the compiled condition kernel ran
};

// compiler / flattener entry points
// exceptions: PolicyException documents (kyverno.io/v2alpha1) or null; a rule named by an exception
// (PolicyException.Contains, api/kyverno/v2alpha1/policy_exception_types.go:101) carries the exceptions' match
// blocks as device match programs (RuleDesc.exc): a matched pair an exception applies to is a skip
// background: the ruleset serves background scans only (empty AdmissionInfo, KYV_COMPILE_BACKGROUND)
Ruleset* compile_ruleset(const char* json, size_t len, std::string* err, const char* exceptions = nullptr,
                         size_t ex_len = 0, bool background = false);
Batch* build_batch(const Ruleset* rs, const char* json, size_t len, const char* nsl_json, size_t nsl_len, int threads,
                   std::string* err);
void derive_strings(Batch& b, size_t from, int threads);
void build_path_trie(Ruleset& rs);
void assign_glob_masks(Ruleset& rs);
void assign_cond_sets(Ruleset& rs);
std::string jit_source(const Ruleset& rs, std::vector<uint8_t>* jit_rules, std::vector<uint8_t>* jit_cond = nullptr,
                       std::vector<uint16_t>* jit_shape = nullptr);
// pattern rules the shape tables can decide (kyv_jit_shapes): a covered RK_PATTERN rule without metadata expansion,
// preconditions or a fused walk (its match program runs in the match phase)
bool jit_shape_eligible(const Ruleset& rs, uint32_t k);
constexpr uint32_t JIT_MAX_SHAPES = 64;
std::vector<char> jit_compile(const std::string& src, double* seconds, bool acct = false);
// rule k is walked by its group's fused kernel (kyv_jit_fused_<g>) rather than the per-chunk schedule (jit.cpp)
bool jit_rule_fused(const Ruleset& rs, uint32_t k);
// the compiled condition rules (jit_cond) in kernel groups: rules with the same kind gate share one kernel
// (kyv_jit_condg_<first rule>, jit.cpp), at most 8 per group, in rule order
std::vector<std::vector<uint32_t>> jit_cond_groups(const Ruleset& rs, const std::vector<uint32_t>& crules);
// kind gate of a rule (batch.cpp): the gvk kinds its match block can accept, or any
struct KindGate {
  bool any = false;
  std::vector<uint32_t> kinds;
};
KindGate rule_gate(const Ruleset& rs, const RuleDesc& rd);
enum JitMode { JIT_AUTO = 0, JIT_OFF = 1, JIT_ON = 2 };
constexpr size_t JIT_AUTO_MIN_RESOURCES = 65536;  // smaller batches are not worth a compile
void resolve_path_columns(Batch& b, int threads);
std::string format_path(const Ruleset& rs, const Batch& b, uint32_t tmpl, const uint16_t* idx, const uint32_t* key);

}  // namespace kyv
