/*
 * kyvgpu — C ABI of the MI355X batched Kyverno validate evaluator (libkyvgpu.so).
 *
 * Drop-in boundary for the reference's validate hot path. Each entry point names the reference
 * interface it replaces (paths relative to the reference repository):
 *
 *   kyv_ruleset_compile  replaces the per-call policy preparation inside engine.Validate:
 *                        autogen.ComputeRules (pkg/autogen/autogen.go:280), rule.DeepCopy + GetPattern
 *                        JSON decode (pkg/engine/validation.go:225-240, api/kyverno/v1/common_types.go:423),
 *                        anchor/operator parsing (pkg/engine/anchor/anchor.go:37, operator/operator.go:35).
 *                        Done once per policy set instead of once per (policy, resource).
 *   kyv_batch_build      replaces the per-resource PolicyContext/JSON-context setup of the background
 *                        scanner and CLI (pkg/controllers/report/utils/scanner.go:87-100,
 *                        cmd/cli/kubectl-kyverno/utils/common/common.go:434-462): N resources at once,
 *                        flattened into device node tables.
 *   kyv_eval             replaces the loop  for policy { for rule { matches(); validate() } }  of
 *                        engine.Validate (pkg/engine/validation.go:39-183) for every (resource, rule)
 *                        pair of the batch: match/exclude (pkg/engine/utils.go:185-256), pattern /
 *                        anyPattern (validation.go:618-702 -> pkg/engine/validate/validate.go:31) and
 *                        podSecurity (validation.go:535-566 -> pkg/pss/evaluate.go:83).
 *   kyv_results_*        the per-rule part of engineapi.RuleResponse (pkg/engine/api/ruleresponse.go:23):
 *                        status, message, failing path; plus the summary counters used by
 *                        pkg/utils/report/results.go:38 (CalculateSummary).
 *
 * deny, preconditions and foreach-deny run on the device when every variable is a `{{ request.object... }}`,
 * `{{ request.operation }}` or `{{ element... }}` expression of the JMESPath subset the compiler restates
 * (fields, multi-select lists, flatten projections, keys(@), `||` literals; pkg/engine/variables/evaluate.go:21,
 * operator/*.go, validation.go:319-421). Rules that need the reference CPU engine (other JMESPath functions,
 * context entries, foreach patterns, exceptions, image verification) are classified at compile time; their pairs
 * report KYV_ST_FALLBACK and the caller runs engine.Validate for them.
 *
 * Threading: a kyv_ruleset is immutable after compile and may be shared; batches and results are per
 * call. No C++ exception crosses this ABI; failures return a non-zero code and kyv_last_error()
 * (thread-local) describes them.
 */
#ifndef KYVGPU_H
#define KYVGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KYV_ABI_VERSION 1u

typedef struct kyv_ruleset kyv_ruleset;
typedef struct kyv_batch kyv_batch;
typedef struct kyv_results kyv_results;

/* return codes */
enum { KYV_OK = 0, KYV_EINVAL = 1, KYV_EPARSE = 2, KYV_EDEVICE = 3, KYV_EINTERNAL = 4, KYV_ERANGE = 5 };

/* per (resource, rule) verdicts; KYV_ST_NONE = rule not applicable (no RuleResponse) */
enum {
  KYV_ST_NONE = 0,
  KYV_ST_PASS = 1,
  KYV_ST_FAIL = 2,
  KYV_ST_SKIP = 3,
  KYV_ST_ERROR = 4,
  KYV_ST_FALLBACK = 5,   /* rule needs the reference CPU engine */
  KYV_ST_PANIC = 6,      /* the reference would panic on this input */
  KYV_ST_ND = 7,         /* the reference result depends on Go map iteration order */
  KYV_NSTATUS = 8        /* number of verdict values (per-rule tally tables) */
};

/* rule kinds */
enum { KYV_RULE_PATTERN = 1, KYV_RULE_ANYPATTERN = 2, KYV_RULE_PSS = 3, KYV_RULE_FALLBACK = 4, KYV_RULE_PANIC = 5,
       KYV_RULE_ERROR = 6, KYV_RULE_DENY = 7, KYV_RULE_FOREACH = 8 };
/* rule flags (kyv_ruleset_rule_flags) */
enum { KYV_RULE_USES_OPERATION = 1u };  /* a condition reads request.operation, evaluated as the background scan's
                                           "CREATE" (scanner.go:97); admission callers route other operations to
                                           engine.Validate */

enum { KYV_BACKEND_GPU = 0, KYV_BACKEND_CPU = 1 };
enum { KYV_EVAL_NO_COPYBACK = 1u, KYV_EVAL_ACCOUNT_BYTES = 2u,
       /* GPU backend: pattern walks run in a kernel generated and compiled (hipRTC, gfx950) for this ruleset
          on first use; default = on for batches of >= 65536 resources, else the interpreted walk kernel */
       KYV_EVAL_JIT_OFF = 4u, KYV_EVAL_JIT_ON = 8u,
       /* GPU backend: every phase on the evaluation stream (no concurrent condition stream), so the per-phase times
          (kyv_results_phase_ms) are each phase's own kernels, not spans under overlap */
       KYV_EVAL_SERIAL = 16u };

/* compile flags (kyv_compile_opts.flags) */
enum { KYV_COMPILE_BACKGROUND = 1u };  /* the ruleset serves background scans only (empty AdmissionInfo, scanner.go:60-110):
                                          PolicyException match blocks with roles / clusterRoles / subjects are compiled
                                          as never matching (checkUserInfo); without the flag such exceptions send the
                                          rules they name to the CPU engine (reason "exception: userInfo ...") */

typedef struct {
  uint32_t abi_version;
  uint32_t flags;
} kyv_compile_opts;

typedef struct {
  uint32_t abi_version;
  int32_t threads;       /* flattener threads (<=0: hardware concurrency) */
} kyv_batch_opts;

typedef struct {
  uint32_t abi_version;
  int32_t backend;       /* KYV_BACKEND_GPU (default). KYV_BACKEND_CPU only when explicitly requested. */
  int32_t device;        /* HIP device ordinal */
  int32_t iterations;    /* timed kernel launches (>=1); results are those of the last launch */
  int32_t threads;       /* CPU backend threads */
  uint32_t flags;        /* KYV_EVAL_NO_COPYBACK: keep verdicts on the device (timing);
                            KYV_EVAL_ACCOUNT_BYTES: algorithmic bytes; on the GPU backend one
                            evaluation with the byte-accounting build of the same kernels (their loads and stores
                            counted on the device, phases serialised), on the CPU backend the host instantiation's
                            per-pair touch count */
} kyv_eval_opts;

typedef struct {
  const char* name;      /* rule name (autogen names included) */
  uint32_t policy;       /* policy index */
  int32_t kind;          /* KYV_RULE_* */
  const char* reason;    /* fallback / error reason, "" otherwise */
} kyv_rule_info;

typedef struct {
  const char* name;
  const char* namespace_;   /* "" for ClusterPolicy */
  uint32_t first_rule;      /* compiled validate rules [first_rule, first_rule + nrules) */
  uint32_t nrules;
  int32_t apply_one;        /* spec.applyRules == One */
  int32_t scored_false;     /* policies.kyverno.io/scored: "false" (fail -> warn in reports) */
} kyv_policy_info;

typedef struct {
  uint64_t resources, nodes, strings, heap_bytes, device_bytes;
} kyv_batch_stats;

/* one compacted failing-path record (a failing pattern, or one failing anyPattern alternative) */
typedef struct {
  uint32_t res;            /* resource index in the caller's input order */
  uint32_t rule;
  uint32_t alt;            /* anyPattern alternative (0 for single patterns) */
  uint32_t path_template;  /* ruleset path template (0xFFFFFFFF: no path) */
  uint16_t idx[4];         /* array indices substituted into the template */
  uint32_t key[2];         /* batch-local string ids of resolved metadata keys (0xFFFFFFFF: none) */
} kyv_failure;

/* ---- ruleset: replaces per-call ComputeRules + pattern decoding ---- */
int kyv_ruleset_compile(const char* policies_json, size_t len, const kyv_compile_opts* opts, kyv_ruleset** out);
/* same, with the cluster's PolicyExceptions (kyverno.io/v2alpha1 documents, JSON array / NDJSON): replaces the
 * per-rule lister scan of PolicyContext.FindExceptions (pkg/engine/policyContext.go:150-169). The match blocks of the
 * exceptions naming a rule (PolicyException.Contains, api/kyverno/v2alpha1/policy_exception_types.go:101) are
 * compiled as device match programs checked after the rule's match, in input order (CheckMatchesResources,
 * pkg/utils/match/match.go:26-203): a pair the first applicable exception covers is KYV_ST_SKIP and its message is
 * "rule skipped due to policy exception <namespace/name>" (hasPolicyExceptions, pkg/engine/validation.go:797-848);
 * the rule's other pairs are evaluated as usual. A rule named by more than 27 exceptions reports KYV_ST_FALLBACK with
 * reason "exception: ...". exceptions_json may be NULL. */
int kyv_ruleset_compile_ex(const char* policies_json, size_t len, const char* exceptions_json, size_t ex_len,
                           const kyv_compile_opts* opts, kyv_ruleset** out);
void kyv_ruleset_free(kyv_ruleset* rs);
uint32_t kyv_ruleset_num_rules(const kyv_ruleset* rs);
uint32_t kyv_ruleset_num_policies(const kyv_ruleset* rs);
int kyv_ruleset_rule_info(const kyv_ruleset* rs, uint32_t rule, kyv_rule_info* out);
int kyv_ruleset_policy_info(const kyv_ruleset* rs, uint32_t policy, kyv_policy_info* out);
/* MatchResources.GetKinds() of compiled rule `rule` ('\n'-separated, autogen applied) and Rule.HasValidate(): the
 * policy cache's kind index (policyMap.set, pkg/policycache/store.go:96-138); returns the full length or -1 */
int64_t kyv_ruleset_rule_kinds(const kyv_ruleset* rs, uint32_t rule, char* buf, size_t cap, int32_t* has_validate);
uint32_t kyv_ruleset_rule_flags(const kyv_ruleset* rs, uint32_t rule);
/* runtime-compiled walk kernel of a ruleset (diagnostics; kyv_eval compiles it on first use by itself):
   the generated HIP source (returns its full length; rules it covers in *nrules_jit) and a hipRTC compile for
   gfx950 that needs no GPU (seconds, code-object bytes) */
int64_t kyv_ruleset_jit_source(const kyv_ruleset* rs, char* buf, size_t cap, uint32_t* nrules_jit);
int kyv_ruleset_jit_compile(const kyv_ruleset* rs, double* seconds, size_t* code_bytes);
/* the same with flags: KYV_JIT_ACCOUNTING compiles the byte-accounting build (-DKYV_ACCT) that an accounting
   evaluation (KYV_EVAL_ACCOUNT_BYTES on the GPU backend) loads; both land in the code-object cache */
enum { KYV_JIT_ACCOUNTING = 1u };
int kyv_ruleset_jit_compile_ex(const kyv_ruleset* rs, uint32_t flags, double* seconds, size_t* code_bytes);

/* ---- batch: resources (JSON array or NDJSON) + namespace labels ({"ns": {"k": "v"}}) ---- */
int kyv_batch_build(const kyv_ruleset* rs, const char* resources_json, size_t len, const char* ns_labels_json,
                    size_t ns_len, const kyv_batch_opts* opts, kyv_batch** out);
void kyv_batch_free(kyv_batch* b);
uint32_t kyv_batch_num_resources(const kyv_batch* b);
int kyv_batch_stats_get(const kyv_batch* b, kyv_batch_stats* out);

/* ---- evaluation: engine.Validate over every (resource, rule) pair ---- */
int kyv_eval(const kyv_ruleset* rs, const kyv_batch* b, const kyv_eval_opts* opts, kyv_results** out);
void kyv_results_free(kyv_results* r);
/* verdict bytes, rule-major: out[rule * nres + res]; low 3 bits = KYV_ST_*, high 5 bits = anyPattern
 * alternative that passed (31 = none) */
int kyv_results_status(const kyv_results* r, uint8_t* out, size_t cap);
int64_t kyv_results_count(const kyv_results* r, int status);
/* per-rule verdict totals, out[rule * 8 + status] (KYV_ST_*), for report summaries: replaces the per-result tally of
 * CalculateSummary (pkg/utils/report/results.go:38-54) over a background-scan batch; returns KYV_OK */
int kyv_results_rule_counts(const kyv_results* r, int64_t* out, size_t cap);
double kyv_results_kernel_ms(const kyv_results* r);
/* per-batch device work outside the evaluation (paid once per batch and device, before its first evaluation):
 * what = 0 the batch image upload (host -> HBM, ms), 1 the glob-mask kernel over the batch dictionary (ms) */
double kyv_results_batch_ms(const kyv_results* r, int what);
/* GPU evaluation time split by phase (HIP events on the evaluation stream, ms averaged over the launches):
 * out[0] verdict resets + match kernels, [1] compiled condition kernel, [2] pattern walk kernels (the dominant kernel
 * of a pattern ruleset), [3] failing-path compaction, [4] verdict histogram; returns the number of phases (5) */
int kyv_results_phase_ms(const kyv_results* r, double* out, size_t cap);
/* bit 0: the runtime-compiled walk kernels evaluated this result's pattern rules (else the interpreter); bit 1: the
 * runtime-compiled condition kernel evaluated its deny / foreach rules with JMESPath operands; bit 2: pattern-shape
 * tables (each distinct compiled pattern walked once per resource) decided the matched pairs of record rules */
int kyv_results_jit(const kyv_results* r);
/* with KYV_EVAL_ACCOUNT_BYTES: algorithmic bytes of the evaluation (GPU: counted by the accounting build of the
 * kernels -- node rows, path-column entries, header fields, work lists read; verdicts, PSS masks, failing-path records,
 * work lists written; CPU: header fields, distinct node rows, verdict, PSS mask, failure records per pair); 0 otherwise */
uint64_t kyv_results_alg_bytes(const kyv_results* r);
/* the same bytes split by the device phase that moves them (kyv_results_phase_ms order); a kind-gated pair counts
 * only its verdict-reset byte (phase 0) and its histogram read (phase 4); returns 5 */
int kyv_results_alg_bytes_phase(const kyv_results* r, uint64_t* out, size_t cap);
/* GPU accounting evaluation: the counted bytes by class -- out[0] resource-data reads, [1] result / work-list writes,
 * [2] staged failing-path records; returns 3 */
int kyv_results_alg_bytes_class(const kyv_results* r, uint64_t* out, size_t cap);
/* RuleResponse.Message for one pair; returns the full length (may exceed cap), -1 if unavailable */
int64_t kyv_results_message(const kyv_results* r, const kyv_ruleset* rs, const kyv_batch* b, uint32_t res,
                            uint32_t rule, char* buf, size_t cap);
/* the compacted failing-path records of the evaluation (PatternError.Path of every failing pattern / anyPattern
 * alternative, validate.go:15-56): returns their number (copies min(count, cap)); -1 when verdicts stayed on the
 * device */
int64_t kyv_results_failures(const kyv_results* r, kyv_failure* out, size_t cap);
/* ---- device-resident results (multi-GPU assembly; replaces the per-rank report hand-off of the
 * reports controller, pkg/controllers/report/background/controller.go:250-361): the verdicts / failing-path records
 * the batch's last GPU evaluation left on `device`, written into caller-owned DEVICE memory on `stream` (a
 * hipStream_t; NULL = the null stream) for an all-gather over RCCL, in input order.
 * kyv_batch_export_status: two 3-bit verdicts per byte (low nibble = even resource), rule-major rows of
 *   ceil(nres / 2) bytes; returns the byte count (dst NULL: only the count), -1 on error.
 * kyv_batch_export_failures: int64 rows (resource index + res_offset, rule, anyPattern alternative, path template,
 *   idx[4]) of every failing-path record; returns the row count (dst NULL: only the count), -1 on error. A
 *   rule-sliced evaluation appends every slice's records to one resident list (error when they exceed its buffer);
 *   one evaluated with copy-back gathered them slice by slice on the host, and they are uploaded from there. */
int64_t kyv_batch_export_status(const kyv_batch* b, int device, uint8_t* dst, size_t cap, void* stream);
/* the verdict bytes (KYV_ST_*, marks cleared) of input-order resources [res0, res0 + nres) of every rule, rule-major
 * [rules][nres], from the batch's last GPU evaluation on `device` into HOST memory (a parity check of that very
 * evaluation, no re-run); returns the byte count (dst NULL: only the count), -1 on error */
int64_t kyv_batch_copy_status(const kyv_batch* b, int device, uint64_t res0, uint64_t nres, uint8_t* dst, size_t cap);
int64_t kyv_batch_export_failures(const kyv_batch* b, int device, int64_t res_offset, int64_t* dst, size_t cap_rows,
                                  void* stream);
/* ---- multi-GPU report gather (one process per GPU). The library creates its own RCCL communicator:
 * rank 0 calls kyv_comm_unique_id and hands the bytes to the other ranks out of band (a TCP store, a file), then
 * every rank calls kyv_comm_init on its device. kyv_comm_gather_results all-gathers the device-resident results of
 * the batch's last GPU evaluation on that device -- packed verdicts (kyv_batch_export_status layout, padded to the
 * largest shard) and failing-path rows (kyv_batch_export_failures rows + res_offset, padded to the largest count) --
 * into buffers the communicator owns, timed with HIP events on its stream. Replaces the per-controller report
 * assembly of pkg/controllers/report (one process there; one rank per GPU here). */
typedef struct kyv_comm kyv_comm;
typedef struct {
  double status_ms, failures_ms;       /* export + transfer, HIP-event time on the communicator's stream */
  uint64_t status_bytes_per_rank;      /* padded verdict bytes per rank */
  uint64_t failure_rows_per_rank_max;  /* padded rows per rank */
  uint64_t failure_rows_total;
} kyv_gather_stats;
int kyv_comm_unique_id(uint8_t* id, size_t cap);  /* writes the 128-byte id (cap >= 128) */
int kyv_comm_init(const uint8_t* id, size_t len, int nranks, int rank, int device, kyv_comm** out);
void kyv_comm_free(kyv_comm* c);
int kyv_comm_gather_results(kyv_comm* c, const kyv_batch* b, int64_t res_offset, kyv_gather_stats* st);
/* rank q's segment of the last gather, to host memory: its packed verdicts (bytes) / its failing-path rows (rows of
   8 int64); dst NULL: only the size */
int64_t kyv_comm_gathered_status(const kyv_comm* c, int rank, uint8_t* host_dst, size_t cap);
int64_t kyv_comm_gathered_failures(const kyv_comm* c, int rank, int64_t* host_dst, size_t cap_rows);
/* report assembly to ONE consumer rank (the process that writes the PolicyReports): every rank's packed verdicts and
 * its failing-path rows as 16-byte records go to `root` with grouped point-to-point sends at exact sizes (no padding,
 * nothing copied to the other ranks). Afterwards kyv_comm_gathered_status / kyv_comm_gathered_failures on the root
 * return rank q's segment (rows expanded to the 8 x int64 form, res_offset of rank q added); on other ranks they fail.
 * A rule-sliced evaluation's rows are resident too (every slice appended). Every rank reports its sizes and an ok flag
 * first: when any rank has no exportable results, every rank returns the same error (no rank left in a collective).
 * Replaces the report controller's per-process assembly (pkg/controllers/report/utils/scanner.go:60-110 callers). */
int kyv_comm_gather_report(kyv_comm* c, const kyv_batch* b, int64_t res_offset, int root, kyv_gather_stats* st);
/* cluster-wide per-rule verdict tallies of the batch's last evaluation: one ncclAllReduce of the device-resident
 * [rules][KYV_NSTATUS] tallies (none derived from the summed resource count) -- the PolicyReport summary counts of a
 * sharded background scan. host_out [rules * KYV_NSTATUS]; returns the entry count (host_out NULL: only
 * the count), -1 on error. A collective: every rank calls it. */
int64_t kyv_comm_reduce_counts(kyv_comm* c, const kyv_batch* b, int64_t* host_out, size_t cap);

/* failing path of a single-pattern FAIL ("" otherwise); returns the full length */
int64_t kyv_results_path(const kyv_results* r, const kyv_ruleset* rs, const kyv_batch* b, uint32_t res, uint32_t rule,
                         char* buf, size_t cap);
/* the same texts for many pairs at once (report rows of a batch: EngineResponseToReportResults,
 * pkg/utils/report/results.go:84-124, takes RuleResponse.Message of every matched pair): what = KYV_TEXT_MESSAGE
 * (RuleResponse.Message, as kyv_results_message) or KYV_TEXT_PATH (PatternError.Path, as kyv_results_path) of rule
 * `rule` for resources [res0, res0 + nres) in input order. lens[i] (nres entries, may be NULL) = byte length of
 * resource res0+i's text, -1 when it is not renderable (the caller runs engine.Validate for that pair), -2 when its
 * status is not in status_mask (bit s = KYV_ST_s). The renderable texts are packed back to back into buf in resource
 * order when cap >= the total. Returns the total length, -1 on bad arguments / verdicts kept on the device. */
enum { KYV_TEXT_MESSAGE = 0, KYV_TEXT_PATH = 1 };
int64_t kyv_results_texts(const kyv_results* r, const kyv_ruleset* rs, const kyv_batch* b, uint32_t rule, uint32_t res0,
                          uint32_t nres, uint32_t status_mask, int32_t what, char* buf, size_t cap, int32_t* lens);
/* why a KYV_ST_FALLBACK pair needs the reference engine ("" for other statuses): the rule's compile-time reason
 * ("context", "foreach", "exception", "variables", ...) or the run-time site (value / walk outside the device subset);
 * returns the full length, -1 on bad arguments */
int64_t kyv_results_fallback_reason(const kyv_results* r, const kyv_ruleset* rs, const kyv_batch* b, uint32_t res,
                                    uint32_t rule, char* buf, size_t cap);
/* PodSecurity rules: RuleResponse.PodSecurityChecks (pkg/engine/api/ruleresponse.go:13, validation.go:550-564) of a
 * pass / fail pair as JSON {"level","version","checks":[{"id","allowed","reason","detail"}]} in DefaultChecks()
 * order (every failing check version, pkg/pss/evaluate.go:16-37); -1 when not renderable (rules with exclusions:
 * the reference's order is Go map order) -- the caller then runs engine.Validate for the pair */
int64_t kyv_results_pss_checks(const kyv_results* r, const kyv_ruleset* rs, const kyv_batch* b, uint32_t res,
                               uint32_t rule, char* buf, size_t cap);
/* PodSecurity rules: failing (check, version) slot mask after exclusions */
uint32_t kyv_results_pss_mask(const kyv_results* r, const kyv_ruleset* rs, uint32_t res, uint32_t rule);

/* measurement only (not a reference interface): one streaming-read launch of `bytes` on `device` -- mode 4 / 8 / 16
 * bytes per lane coalesced, 116 a gather of 16-byte rows -- whose known byte count calibrates rocprofv3's FETCH_SIZE
 * for the access widths the evaluation kernels use (bench.py KYV_CALIB=1, scripts/pmc_summary.py). Returns device ms,
 * -1 on error. */
double kyv_calibrate_fetch(int device, uint64_t bytes, int mode);

const char* kyv_last_error(void);
const char* kyv_version(void);

#ifdef __cplusplus
}
#endif
#endif /* KYVGPU_H */
