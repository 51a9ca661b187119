"""C-ABI boundary (include/kyvgpu.h): the library loads, exports every declared symbol, reports errors
through return codes + kyv_last_error, and never falls back to the CPU when the GPU backend is asked for."""
import ctypes
import os
import re

import pytest

from kyverno_amd import _lib as K
from kyverno_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "kyvgpu.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kyv_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    syms = declared_symbols()
    assert len(syms) >= 20
    lib = ctypes.CDLL(K.LIB_PATH)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(K.EXPORTS) == syms


def test_version_and_errors():
    L = K.lib()
    assert L.kyv_version().decode().startswith("kyvgpu")
    h = ctypes.c_void_p()
    opts = K.CompileOpts(K.KYV_ABI_VERSION, 0)
    rc = L.kyv_ruleset_compile(b"{not json", 9, ctypes.byref(opts), ctypes.byref(h))
    assert rc != 0
    assert L.kyv_last_error().decode()
    with pytest.raises(K.KyvError):
        E.Ruleset(b"[1,")


def test_abi_version_checked():
    L = K.lib()
    h = ctypes.c_void_p()
    opts = K.CompileOpts(K.KYV_ABI_VERSION + 100, 0)
    assert L.kyv_ruleset_compile(b"[]", 2, ctypes.byref(opts), ctypes.byref(h)) != 0


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="host has a GPU")
def test_gpu_backend_fails_loudly_without_device():
    rs = E.Ruleset([{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "p"},
                     "spec": {"rules": [{"name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                                         "validate": {"pattern": {"metadata": {"name": "?*"}}}}]}}])
    b = E.Batch(rs, [{"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "x"}}])
    with pytest.raises(K.KyvError, match="no HIP device"):
        E.evaluate(rs, b, backend="gpu")


def test_batch_for_other_ruleset_rejected():
    p = [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "p"},
          "spec": {"rules": [{"name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                              "validate": {"pattern": {"metadata": {"name": "?*"}}}}]}}]
    a, b = E.Ruleset(p), E.Ruleset(p)
    batch = E.Batch(a, [{"kind": "Pod", "metadata": {"name": "x"}}])
    with pytest.raises(K.KyvError):
        E.evaluate(b, batch, backend="cpu")


def test_jit_walk_kernel_compiles_for_gfx950(monkeypatch):
    """The runtime-compiled walk kernel of a ruleset: generated source covers the pattern rules and hipRTC
    compiles it for gfx950 without a GPU (the GPU tests then check its verdicts against the oracle)."""
    import cases
    monkeypatch.setenv("KYV_JIT_CACHE", "0")  # compile for real; keep the in-tree code-object cache untouched
    from kyverno_amd import engine as E
    rs = E.Ruleset(cases.best_practices() + cases.quirk_policies())
    src, n = rs.jit_source()
    npat = sum(1 for r in rs.rules if r["kind"] in ("pattern", "anyPattern"))
    assert n > 0 and n <= npat
    assert "kyv_jit_walk" in src
    secs, size = rs.jit_compile()
    assert size > 1000


def test_jit_shapes_deduplicated_and_compile(monkeypatch):
    """C4's 10,000 generated policies (10,440 pattern rules) use a handful of pattern shapes: the generator emits one
    walk function tree per shape (a root -> shape table dispatches the rest), so the whole ruleset is covered and
    hipRTC compiles it in seconds; the chart's JMESPath / foreach rules get the compiled condition kernel."""
    import re
    monkeypatch.setenv("KYV_JIT_CACHE", "0")
    from kyverno_amd import engine as E, synth
    rs = E.Ruleset(synth.c4_policies(10000))
    src, n = rs.jit_source()
    npat = sum(1 for r in rs.rules if r["kind"] in ("pattern", "anyPattern"))
    assert npat > 10000 and n == npat
    assert len(re.findall(r"void root\d+\(", src)) <= 32
    assert "kyv_shape0" in src
    secs, size = rs.jit_compile()
    assert size > 1000
    import cases
    rs3 = E.Ruleset(cases.chart_restricted())
    src3, _ = rs3.jit_source()
    assert "kyv_jit_cond" in src3 and src3.count("uint8_t jr") >= 12
