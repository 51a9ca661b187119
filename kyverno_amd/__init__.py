"""kyverno_amd — MI355X batched evaluator for Kyverno's validate hot path (engine.Validate).

The product is the C-ABI library libkyvgpu.so (include/kyvgpu.h) built from kyverno_amd/csrc
(host compiler/flattener in C++, evaluation kernels in HIP for gfx950). This package is the thin
Python host mirror of the reference interface used by tests and bench.py.
"""
from ._lib import STATUS_NAMES, lib  # noqa: F401
from .engine import Batch, Engine, Results, Ruleset, evaluate  # noqa: F401
