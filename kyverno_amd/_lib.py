"""ctypes binding of libkyvgpu.so (include/kyvgpu.h). This is the same binding a cgo shim declares."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# KYV_LIB overrides the library path (kernel-variant experiments built by scripts/build_variants.py only)
LIB_PATH = os.environ.get("KYV_LIB") or os.path.join(HERE, "libkyvgpu.so")

KYV_ABI_VERSION = 1
BACKEND_GPU, BACKEND_CPU = 0, 1
EVAL_NO_COPYBACK = 1
EVAL_ACCOUNT_BYTES = 2
EVAL_JIT_OFF = 4
EVAL_JIT_ON = 8
EVAL_SERIAL = 16

ST_NONE, ST_PASS, ST_FAIL, ST_SKIP, ST_ERROR, ST_FALLBACK, ST_PANIC, ST_ND = range(8)
STATUS_NAMES = ["none", "pass", "fail", "skip", "error", "fallback", "panic", "nondeterministic"]
RULE_KINDS = {1: "pattern", 2: "anyPattern", 3: "podSecurity", 4: "fallback", 5: "panic", 6: "error", 7: "deny",
              8: "foreach"}
RULE_USES_OPERATION = 1
TEXT_MESSAGE, TEXT_PATH = 0, 1


class CompileOpts(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class BatchOpts(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("threads", ctypes.c_int32)]


class EvalOpts(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("backend", ctypes.c_int32), ("device", ctypes.c_int32),
                ("iterations", ctypes.c_int32), ("threads", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class RuleInfo(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("policy", ctypes.c_uint32), ("kind", ctypes.c_int32), ("reason", ctypes.c_char_p)]


class PolicyInfo(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("namespace_", ctypes.c_char_p), ("first_rule", ctypes.c_uint32),
                ("nrules", ctypes.c_uint32), ("apply_one", ctypes.c_int32), ("scored_false", ctypes.c_int32)]


class Failure(ctypes.Structure):
    _fields_ = [("res", ctypes.c_uint32), ("rule", ctypes.c_uint32), ("alt", ctypes.c_uint32),
                ("path_template", ctypes.c_uint32), ("idx", ctypes.c_uint16 * 4), ("key", ctypes.c_uint32 * 2)]


class BatchStats(ctypes.Structure):
    _fields_ = [("resources", ctypes.c_uint64), ("nodes", ctypes.c_uint64), ("strings", ctypes.c_uint64),
                ("heap_bytes", ctypes.c_uint64), ("device_bytes", ctypes.c_uint64)]


EXPORTS = [
    "kyv_ruleset_compile", "kyv_ruleset_free", "kyv_ruleset_num_rules", "kyv_ruleset_num_policies",
    "kyv_ruleset_rule_info", "kyv_ruleset_policy_info", "kyv_batch_build", "kyv_batch_free",
    "kyv_batch_num_resources", "kyv_batch_stats_get", "kyv_eval", "kyv_results_free", "kyv_results_status",
    "kyv_results_count", "kyv_results_kernel_ms", "kyv_results_alg_bytes", "kyv_results_message", "kyv_results_path",
    "kyv_results_pss_mask", "kyv_last_error", "kyv_version", "kyv_results_jit", "kyv_ruleset_jit_source",
    "kyv_ruleset_jit_compile", "kyv_ruleset_jit_compile_ex", "kyv_results_rule_counts", "kyv_ruleset_compile_ex", "kyv_ruleset_rule_kinds",
    "kyv_results_fallback_reason", "kyv_results_pss_checks", "kyv_results_failures", "kyv_ruleset_rule_flags",
    "kyv_results_texts", "kyv_results_phase_ms", "kyv_results_alg_bytes_phase", "kyv_results_alg_bytes_class", "kyv_batch_export_status", "kyv_batch_copy_status",
    "kyv_batch_export_failures", "kyv_comm_unique_id", "kyv_comm_init", "kyv_comm_free", "kyv_comm_gather_results",
    "kyv_comm_gathered_status", "kyv_comm_gathered_failures", "kyv_comm_gather_report", "kyv_comm_reduce_counts", "kyv_results_batch_ms",
    "kyv_calibrate_fetch",
]


class GatherStats(ctypes.Structure):
    _fields_ = [("status_ms", ctypes.c_double), ("failures_ms", ctypes.c_double),
                ("status_bytes_per_rank", ctypes.c_uint64), ("failure_rows_per_rank_max", ctypes.c_uint64),
                ("failure_rows_total", ctypes.c_uint64)]

_lib = None


def lib():
    """Load the in-tree HIP library; fails loudly if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libkyvgpu.so not built: run `python -m kyverno_amd.build` (or __graft_entry__.build())")
    # One HIP runtime per process. torch bundles its own (older) libamdhip64; whichever is loaded first serves
    # both. Default: this library's /opt/rocm runtime (the C3 evaluation measured 2.96 ms on it vs 3.48 ms on
    # torch's). A process that also needs torch on the GPU (RCCL collectives through torch.distributed) must load
    # torch first, else torch finds no GPUs (ProcessGroupNCCL: "no GPUs found"): set KYV_TORCH_FIRST=1 or import
    # torch before kyverno_amd.
    if os.environ.get("KYV_TORCH_FIRST", "0") != "0":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u32, i32, i64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int64
    L.kyv_ruleset_compile.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(CompileOpts), ctypes.POINTER(vp)]
    L.kyv_ruleset_compile_ex.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.POINTER(CompileOpts),
                                         ctypes.POINTER(vp)]
    L.kyv_ruleset_rule_kinds.argtypes = [vp, u32, ctypes.c_char_p, sz, ctypes.POINTER(i32)]
    L.kyv_ruleset_rule_kinds.restype = i64
    L.kyv_results_fallback_reason.argtypes = [vp, vp, vp, u32, u32, ctypes.c_char_p, sz]
    L.kyv_results_fallback_reason.restype = i64
    L.kyv_results_pss_checks.argtypes = [vp, vp, vp, u32, u32, ctypes.c_char_p, sz]
    L.kyv_results_pss_checks.restype = i64
    L.kyv_results_failures.argtypes = [vp, vp, sz]
    L.kyv_results_failures.restype = i64
    L.kyv_batch_export_status.argtypes = [vp, ctypes.c_int, vp, sz, vp]
    L.kyv_batch_export_status.restype = i64
    L.kyv_batch_copy_status.argtypes = [vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, vp, sz]
    L.kyv_batch_copy_status.restype = i64
    L.kyv_batch_export_failures.argtypes = [vp, ctypes.c_int, i64, vp, sz, vp]
    L.kyv_batch_export_failures.restype = i64
    L.kyv_comm_unique_id.argtypes = [vp, sz]
    L.kyv_comm_init.argtypes = [vp, sz, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
    L.kyv_comm_free.argtypes = [vp]
    L.kyv_comm_free.restype = None
    L.kyv_comm_gather_results.argtypes = [vp, vp, i64, ctypes.POINTER(GatherStats)]
    L.kyv_comm_gathered_status.argtypes = [vp, ctypes.c_int, vp, sz]
    L.kyv_comm_gathered_status.restype = i64
    L.kyv_comm_gathered_failures.argtypes = [vp, ctypes.c_int, vp, sz]
    L.kyv_comm_gathered_failures.restype = i64
    L.kyv_comm_gather_report.argtypes = [vp, vp, i64, ctypes.c_int, ctypes.POINTER(GatherStats)]
    L.kyv_comm_reduce_counts.argtypes = [vp, vp, vp, sz]
    L.kyv_comm_reduce_counts.restype = i64
    L.kyv_results_batch_ms.argtypes = [vp, ctypes.c_int]
    L.kyv_results_batch_ms.restype = ctypes.c_double
    L.kyv_ruleset_rule_flags.argtypes = [vp, u32]
    L.kyv_ruleset_rule_flags.restype = u32
    L.kyv_ruleset_free.argtypes = [vp]
    L.kyv_ruleset_num_rules.argtypes = [vp]
    L.kyv_ruleset_num_rules.restype = u32
    L.kyv_ruleset_num_policies.argtypes = [vp]
    L.kyv_ruleset_num_policies.restype = u32
    L.kyv_ruleset_rule_info.argtypes = [vp, u32, ctypes.POINTER(RuleInfo)]
    L.kyv_ruleset_policy_info.argtypes = [vp, u32, ctypes.POINTER(PolicyInfo)]
    L.kyv_batch_build.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.POINTER(BatchOpts), ctypes.POINTER(vp)]
    L.kyv_batch_free.argtypes = [vp]
    L.kyv_batch_num_resources.argtypes = [vp]
    L.kyv_batch_num_resources.restype = u32
    L.kyv_batch_stats_get.argtypes = [vp, ctypes.POINTER(BatchStats)]
    L.kyv_eval.argtypes = [vp, vp, ctypes.POINTER(EvalOpts), ctypes.POINTER(vp)]
    L.kyv_results_free.argtypes = [vp]
    L.kyv_results_status.argtypes = [vp, ctypes.c_void_p, sz]
    L.kyv_results_rule_counts.argtypes = [vp, vp, ctypes.c_size_t]
    L.kyv_results_rule_counts.restype = i32
    L.kyv_results_count.argtypes = [vp, i32]
    L.kyv_results_count.restype = i64
    L.kyv_results_kernel_ms.argtypes = [vp]
    L.kyv_results_kernel_ms.restype = ctypes.c_double
    L.kyv_calibrate_fetch.argtypes = [i32, ctypes.c_uint64, i32]
    L.kyv_calibrate_fetch.restype = ctypes.c_double
    L.kyv_results_alg_bytes.argtypes = [vp]
    L.kyv_results_alg_bytes.restype = ctypes.c_uint64
    L.kyv_results_message.argtypes = [vp, vp, vp, u32, u32, ctypes.c_char_p, sz]
    L.kyv_results_message.restype = i64
    L.kyv_results_path.argtypes = [vp, vp, vp, u32, u32, ctypes.c_char_p, sz]
    L.kyv_results_path.restype = i64
    L.kyv_results_alg_bytes_phase.argtypes = [vp, ctypes.c_void_p, sz]
    L.kyv_results_alg_bytes_phase.restype = i32
    L.kyv_results_alg_bytes_class.argtypes = [vp, ctypes.c_void_p, sz]
    L.kyv_results_alg_bytes_class.restype = i32
    L.kyv_results_phase_ms.argtypes = [vp, ctypes.c_void_p, sz]
    L.kyv_results_phase_ms.restype = i32
    L.kyv_results_texts.argtypes = [vp, vp, vp, u32, u32, u32, u32, i32, ctypes.c_void_p, sz, ctypes.c_void_p]
    L.kyv_results_texts.restype = i64
    L.kyv_results_pss_mask.argtypes = [vp, vp, u32, u32]
    L.kyv_results_pss_mask.restype = u32
    L.kyv_results_jit.argtypes = [vp]
    L.kyv_results_jit.restype = i32
    L.kyv_ruleset_jit_source.argtypes = [vp, ctypes.c_char_p, sz, ctypes.POINTER(u32)]
    L.kyv_ruleset_jit_source.restype = i64
    L.kyv_ruleset_jit_compile.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(sz)]
    L.kyv_ruleset_jit_compile_ex.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(sz)]
    L.kyv_last_error.restype = ctypes.c_char_p
    L.kyv_version.restype = ctypes.c_char_p
    _lib = L
    return L


class KyvError(RuntimeError):
    """A libkyvgpu call returned an error status (message from kyv_last_error)."""


def check(rc):
    if rc != 0:
        raise KyvError("kyvgpu error %d: %s" % (rc, lib().kyv_last_error().decode(errors="replace")))
