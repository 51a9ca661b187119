"""Host-side mirror of the reference validate interface over libkyvgpu.so.

Reference surface mirrored (paths relative to the reference repository):
  engine.Validate(ctx, loader, PolicyContext, cfg) -> *EngineResponse   pkg/engine/validation.go:39
  EngineResponse / PolicyResponse / RuleResponse                         pkg/engine/api/*.go
  background scan per resource x policy                                  pkg/controllers/report/utils/scanner.go:60
  CLI apply counters (pass/fail/warn/error/skip)                         cmd/cli/kubectl-kyverno/utils/common/common.go:712-795

`Engine(policies)` compiles once (autogen + rule programs); `engine.validate_batch(resources)` evaluates
every (resource, rule) pair on the MI355X and returns per-resource EngineResponses in reference shape.
Rules the device path does not cover come back with status "fallback" (the Go shim runs engine.Validate
for exactly those pairs).
"""
import ctypes
import json

import numpy as np

from . import _lib as K


def _dumps(x):
    if isinstance(x, (bytes, bytearray)):
        return bytes(x)
    if isinstance(x, str):
        return x.encode()
    return json.dumps(x, separators=(",", ":")).encode()


class Ruleset:
    def __init__(self, policies, exceptions=None, background=False):
        """policies: list of ClusterPolicy/Policy dicts (or JSON text); exceptions: PolicyException documents (their
        match blocks run on the device after each named rule's match); background: the ruleset serves background
        scans only (KYV_COMPILE_BACKGROUND: exceptions keyed on roles / subjects never match instead of sending their
        rules to the CPU engine)."""
        L = K.lib()
        data = _dumps(policies if not isinstance(policies, dict) else [policies])
        ex = _dumps(exceptions) if exceptions else None
        h = ctypes.c_void_p()
        opts = K.CompileOpts(K.KYV_ABI_VERSION, 1 if background else 0)
        K.check(L.kyv_ruleset_compile_ex(data, len(data), ex, len(ex) if ex else 0, ctypes.byref(opts), ctypes.byref(h)))
        self.h = h
        self.rules = []
        for k in range(L.kyv_ruleset_num_rules(h)):
            ri = K.RuleInfo()
            K.check(L.kyv_ruleset_rule_info(h, k, ctypes.byref(ri)))
            kb = ctypes.create_string_buffer(4096)
            hv = ctypes.c_int32(0)
            n = L.kyv_ruleset_rule_kinds(h, k, kb, len(kb), ctypes.byref(hv))
            if n >= len(kb):
                kb = ctypes.create_string_buffer(n + 1)
                L.kyv_ruleset_rule_kinds(h, k, kb, len(kb), ctypes.byref(hv))
            kinds = kb.value.decode().split("\n") if n > 0 else []
            self.rules.append({"name": ri.name.decode(), "policy": ri.policy, "kind": K.RULE_KINDS.get(ri.kind, "?"),
                               "reason": ri.reason.decode(), "match_kinds": kinds, "has_validate": bool(hv.value),
                               "uses_operation": bool(L.kyv_ruleset_rule_flags(h, k) & K.RULE_USES_OPERATION)})
        self.policies = []
        for p in range(L.kyv_ruleset_num_policies(h)):
            pi = K.PolicyInfo()
            K.check(L.kyv_ruleset_policy_info(h, p, ctypes.byref(pi)))
            self.policies.append({"name": pi.name.decode(), "namespace": pi.namespace_.decode(), "first_rule": pi.first_rule,
                                  "nrules": pi.nrules, "apply_one": bool(pi.apply_one), "scored_false": bool(pi.scored_false)})

    def jit_source(self):
        """(generated HIP source of the ruleset's walk kernel, number of rules it covers)"""
        L = K.lib()
        n = ctypes.c_uint32()
        size = L.kyv_ruleset_jit_source(self.h, None, 0, ctypes.byref(n))
        buf = ctypes.create_string_buffer(size + 1)
        L.kyv_ruleset_jit_source(self.h, buf, size + 1, ctypes.byref(n))
        return buf.value.decode(), n.value

    def jit_compile(self, accounting=False):
        """hipRTC-compile the walk kernel for gfx950 (no GPU needed) -> (seconds, code-object bytes); accounting=True
        compiles its byte-accounting build (what evaluate(..., account_bytes=True) loads on the GPU)"""
        secs, size = ctypes.c_double(), ctypes.c_size_t()
        K.check(K.lib().kyv_ruleset_jit_compile_ex(self.h, 1 if accounting else 0, ctypes.byref(secs), ctypes.byref(size)))
        return secs.value, size.value

    def __del__(self):
        if getattr(self, "h", None):
            K.lib().kyv_ruleset_free(self.h)
            self.h = None


class Batch:
    def __init__(self, ruleset, resources, ns_labels=None, threads=0):
        """resources: list of dicts, or JSON array / NDJSON bytes."""
        L = K.lib()
        data = _dumps(resources)
        nsl = _dumps(ns_labels) if ns_labels else b""
        h = ctypes.c_void_p()
        opts = K.BatchOpts(K.KYV_ABI_VERSION, threads)
        K.check(L.kyv_batch_build(ruleset.h, data, len(data), nsl, len(nsl), ctypes.byref(opts), ctypes.byref(h)))
        self.h = h
        self.ruleset = ruleset
        self.n = L.kyv_batch_num_resources(h)

    def resident_status(self, device=0, res0=0, nres=None):
        """uint8 [rules, nres] KYV_ST_* verdicts of input-order resources [res0, res0 + nres) as the batch's last GPU
        evaluation left them on `device` (kyv_batch_copy_status: no re-evaluation)"""
        L = K.lib()
        nres = self.n - res0 if nres is None else nres
        total = L.kyv_batch_copy_status(self.h, device, res0, nres, None, 0)
        if total < 0:
            raise K.KyvError(L.kyv_last_error().decode(errors="replace"))
        out = np.empty(max(1, total), dtype=np.uint8)
        if L.kyv_batch_copy_status(self.h, device, res0, nres, out.ctypes.data, out.size) < 0:
            raise K.KyvError(L.kyv_last_error().decode(errors="replace"))
        nr = len(self.ruleset.rules)
        return out[:total].reshape(nr, total // max(1, nr))

    def stats(self):
        s = K.BatchStats()
        K.check(K.lib().kyv_batch_stats_get(self.h, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in K.BatchStats._fields_}

    def __del__(self):
        if getattr(self, "h", None):
            K.lib().kyv_batch_free(self.h)
            self.h = None


class Results:
    def __init__(self, ruleset, batch, h, copied):
        self.ruleset, self.batch, self.h = ruleset, batch, h
        L = K.lib()
        self.counts = {K.STATUS_NAMES[s]: L.kyv_results_count(h, s) for s in range(8)}
        self.kernel_ms = L.kyv_results_kernel_ms(h)
        # per-batch device work before the batch's first evaluation: image upload and glob-mask kernel (ms)
        self.upload_ms = L.kyv_results_batch_ms(h, 0)
        self.gmask_ms = L.kyv_results_batch_ms(h, 1)
        ph = (ctypes.c_double * 5)()
        L.kyv_results_phase_ms(h, ph, 5)
        # match (incl. verdict resets), cond (compiled condition kernel), walk, compact, hist -- ms per launch
        self.phase_ms = dict(zip(("match", "cond", "walk", "compact", "hist"), list(ph)))
        self.alg_bytes = L.kyv_results_alg_bytes(h)
        ab = (ctypes.c_uint64 * 5)()
        L.kyv_results_alg_bytes_phase(h, ab, 5)
        self.alg_bytes_phase = dict(zip(("match", "cond", "walk", "compact", "hist"), list(ab)))
        ac = (ctypes.c_uint64 * 3)()
        L.kyv_results_alg_bytes_class(h, ac, 3)
        self.alg_bytes_class = dict(zip(("reads", "writes", "staged_records"), list(ac)))
        ju = L.kyv_results_jit(h)
        self.jit = bool(ju & 1)          # runtime-compiled walk kernels ran
        self.jit_cond = bool(ju & 2)     # runtime-compiled condition kernel (deny / foreach rules) ran
        self.jit_shapes = bool(ju & 4)   # pattern-shape tables (kyv_jit_shapes) decided matched pairs
        rc = np.zeros(len(ruleset.rules) * 8, dtype=np.int64)
        if rc.size:
            K.check(L.kyv_results_rule_counts(h, rc.ctypes.data, rc.size))
        self.rule_counts = rc.reshape(len(ruleset.rules), 8)  # [rule][status] verdict totals
        self.raw = self._status = None
        if copied:
            nr, nres = len(ruleset.rules), batch.n
            buf = np.empty(nr * nres, dtype=np.uint8)
            K.check(L.kyv_results_status(h, buf.ctypes.data, buf.size))
            self.raw = buf.reshape(nr, nres)  # status bytes in input order (low 3 bits: KYV_ST_*, high bits: marks)

    @property
    def status(self):
        """uint8 [rule, resource] KYV_ST_* verdicts (None when they stayed on the device)"""
        if self._status is None and self.raw is not None:
            self._status = self.raw & 7
        return self._status

    def message(self, res, rule):
        L = K.lib()
        buf = ctypes.create_string_buffer(4096)
        n = L.kyv_results_message(self.h, self.ruleset.h, self.batch.h, res, rule, buf, len(buf))
        if n < 0:
            return None
        if n >= len(buf):
            buf = ctypes.create_string_buffer(n + 1)
            L.kyv_results_message(self.h, self.ruleset.h, self.batch.h, res, rule, buf, len(buf))
        return buf.value.decode(errors="replace")

    def path(self, res, rule):
        buf = ctypes.create_string_buffer(4096)
        K.lib().kyv_results_path(self.h, self.ruleset.h, self.batch.h, res, rule, buf, len(buf))
        return buf.value.decode(errors="replace")

    def texts(self, rule, what="message", statuses=(K.ST_FAIL,), res0=0, nres=None):
        """RuleResponse.Message (what="message") or PatternError.Path (what="path") of rule `rule` for resources
        [res0, res0 + nres) whose status is in `statuses`, rendered in one library call: list of bytes, None for a
        pair whose text needs the CPU engine, and False for a pair whose status is not in `statuses`"""
        L = K.lib()
        nres = self.batch.n - res0 if nres is None else nres
        mask = 0
        for s in statuses:
            mask |= 1 << s
        w = {"message": K.TEXT_MESSAGE, "path": K.TEXT_PATH}[what]
        lens = np.zeros(max(1, nres), dtype=np.int32)
        total = L.kyv_results_texts(self.h, self.ruleset.h, self.batch.h, rule, res0, nres, mask, w, None, 0,
                                    lens.ctypes.data)
        if total < 0:
            raise K.KyvError(L.kyv_last_error().decode(errors="replace"))
        buf = np.zeros(max(1, total), dtype=np.uint8)
        L.kyv_results_texts(self.h, self.ruleset.h, self.batch.h, rule, res0, nres, mask, w, buf.ctypes.data, total,
                            lens.ctypes.data)
        raw = buf.tobytes()
        out, at = [], 0
        for n in lens[:nres].tolist():
            if n >= 0:
                out.append(raw[at:at + n])
                at += n
            else:
                out.append(None if n == -1 else False)
        return out

    def failures(self):
        """compacted failing-path records as a structured numpy array (res in input order, rule, alt,
        path_template, idx[4], key[2])"""
        L = K.lib()
        n = L.kyv_results_failures(self.h, None, 0)
        if n < 0:
            raise K.KyvError(L.kyv_last_error().decode(errors="replace"))
        dt = np.dtype([("res", "<u4"), ("rule", "<u4"), ("alt", "<u4"), ("path_template", "<u4"), ("idx", "<u2", 4),
                       ("key", "<u4", 2)])
        assert dt.itemsize == ctypes.sizeof(K.Failure)
        out = np.zeros(n, dtype=dt)
        if n:
            L.kyv_results_failures(self.h, out.ctypes.data, n)
        return out

    def fallback_reason(self, res, rule):
        """why pair (res, rule) is KYV_ST_FALLBACK ("" otherwise)"""
        buf = ctypes.create_string_buffer(512)
        n = K.lib().kyv_results_fallback_reason(self.h, self.ruleset.h, self.batch.h, res, rule, buf, len(buf))
        if n < 0:
            raise K.KyvError(K.lib().kyv_last_error().decode(errors="replace"))
        return buf.value.decode(errors="replace")

    def pss_checks(self, res, rule):
        """RuleResponse.PodSecurityChecks of a podSecurity pair (dict), or None when not renderable"""
        L = K.lib()
        buf = ctypes.create_string_buffer(8192)
        n = L.kyv_results_pss_checks(self.h, self.ruleset.h, self.batch.h, res, rule, buf, len(buf))
        if n < 0:
            return None
        if n >= len(buf):
            buf = ctypes.create_string_buffer(n + 1)
            L.kyv_results_pss_checks(self.h, self.ruleset.h, self.batch.h, res, rule, buf, len(buf))
        return json.loads(buf.value.decode())

    def pss_mask(self, res, rule):
        return K.lib().kyv_results_pss_mask(self.h, self.ruleset.h, res, rule)

    def __del__(self):
        if getattr(self, "h", None):
            K.lib().kyv_results_free(self.h)
            self.h = None


def evaluate(ruleset, batch, backend="gpu", device=0, iterations=1, threads=0, copy_back=True, account_bytes=False,
             jit=None, serial=False):
    """Evaluate every (resource, rule) pair. backend="gpu" is the product path; "cpu" must be explicit.
    jit: None = library default (runtime-compiled walk kernel for batches >= 65536 resources), True / False force."""
    L = K.lib()
    flags = (0 if copy_back else K.EVAL_NO_COPYBACK) | (K.EVAL_ACCOUNT_BYTES if account_bytes else 0) | \
        (K.EVAL_SERIAL if serial else 0)
    if jit is not None:
        flags |= K.EVAL_JIT_ON if jit else K.EVAL_JIT_OFF
    opts = K.EvalOpts(K.KYV_ABI_VERSION, K.BACKEND_GPU if backend == "gpu" else K.BACKEND_CPU, device, iterations,
                      threads, flags)
    h = ctypes.c_void_p()
    K.check(L.kyv_eval(ruleset.h, batch.h, ctypes.byref(opts), ctypes.byref(h)))
    return Results(ruleset, batch, h, copy_back)


class Engine:
    """engine.Validate over batches: compile once, evaluate many resources per call."""

    def __init__(self, policies, backend="gpu", device=0):
        self.ruleset = Ruleset(policies)
        self.backend, self.device = backend, device

    def validate_batch(self, resources, ns_labels=None):
        """-> list (per resource) of list (per policy) of EngineResponse-like dicts (validation.go:39)."""
        batch = Batch(self.ruleset, resources, ns_labels)
        res = evaluate(self.ruleset, batch, backend=self.backend, device=self.device)
        out = []
        for r in range(batch.n):
            per_policy = []
            for pi, pol in enumerate(self.ruleset.policies):
                rules = []
                applied = errors = 0
                for k in range(pol["first_rule"], pol["first_rule"] + pol["nrules"]):
                    st = int(res.status[k, r])
                    if st == K.ST_NONE:
                        continue
                    name = K.STATUS_NAMES[st]
                    rules.append({"name": self.ruleset.rules[k]["name"], "status": name, "message": res.message(r, k)})
                    if st in (K.ST_PASS, K.ST_FAIL):
                        applied += 1
                    elif st == K.ST_ERROR:
                        errors += 1
                    if pol["apply_one"] and applied > 0:  # validation.go:176-178
                        break
                    if pol["apply_one"] and st == K.ST_FALLBACK:
                        break  # truncation depends on the CPU engine's verdict for this rule
                # PolicyResponse.PolicyStats (validation.go:196-208; pkg/engine/api/stats.go:16-23): the device's
                # share (rules the CPU engine decides add theirs in the Go shim)
                per_policy.append({"policy": pol["name"], "rules": rules,
                                   "stats": {"rulesAppliedCount": applied, "rulesErrorCount": errors}})
            out.append(per_policy)
        return out, res, batch
