"""The byte-accounting build of the kernels (KYV_ACCT; bench.py's roofline bytes) runs the product's
kernel source with counters added: on the MI355X its verdicts must equal the product kernels' byte for byte, and its
per-phase counts must be consistent with what the evaluation provably moves (one verdict-reset byte and one histogram
read per pair, at least one header read per decided pair, one status write per decided pair)."""
import numpy as np
import pytest

import cases
from kyverno_amd import engine as E
from kyverno_amd import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("jit", [False, True])
def test_accounting_build_same_verdicts_c3(jit):
    data, nsl = synth.corpus_ndjson(70_000, seed=41, edge=True)
    rs = E.Ruleset(cases.best_practices() + cases.chart_restricted())
    b = E.Batch(rs, data, nsl)
    prod = E.evaluate(rs, b, backend="gpu", jit=jit)
    acct = E.evaluate(rs, b, backend="gpu", jit=jit, account_bytes=True)
    assert np.array_equal(prod.raw, acct.raw)
    assert prod.counts == acct.counts
    assert bool(acct.jit) == jit
    pairs = len(rs.rules) * b.n
    ph = acct.alg_bytes_phase
    assert acct.alg_bytes == sum(ph.values())
    assert ph["hist"] == pairs  # the histogram reads every verdict byte once
    assert ph["match"] >= pairs  # the verdict reset writes every byte
    decided = pairs - acct.counts["none"]
    cl = acct.alg_bytes_class
    assert cl["writes"] >= decided  # one status byte per decided pair at least
    assert cl["reads"] >= 4 * b.n  # a header word per resource at least
    assert ph["walk"] > 0 and cl["staged_records"] > 0
    assert ph["compact"] >= cl["staged_records"]
    # a second accounting run counts the same bytes (deterministic kernels, counters reset per phase)
    again = E.evaluate(rs, b, backend="gpu", jit=jit, account_bytes=True)
    assert again.alg_bytes_phase == ph


def test_accounting_build_same_verdicts_c2_c5():
    pods, nsl = synth.pods(30_000, seed=42)
    pol = [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "psa"},
            "spec": {"rules": [{"name": "restricted", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                                "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}}]}}]
    for pols in (pol, synth.c5_policies(50)):
        rs = E.Ruleset(pols)
        b = E.Batch(rs, pods, nsl)
        prod = E.evaluate(rs, b, backend="gpu", jit=True)
        acct = E.evaluate(rs, b, backend="gpu", jit=True, account_bytes=True)
        assert np.array_equal(prod.raw, acct.raw)
        assert acct.alg_bytes > len(rs.rules) * b.n
