"""The explicit CPU instantiation of the shared __host__ __device__ evaluator vs the oracle.

This checks the compiler, flattener and evaluator logic without a GPU; the GPU kernel runs the same
evaluator (tests/test_gpu_parity.py repeats these corpora on the device)."""
import cases
import parity_suite as S


def test_engine_goldens():
    assert S.run_engine_goldens("cpu") > 0


def test_cli_goldens():
    assert S.run_cli_goldens("cpu") > 0


def test_walk_goldens():
    assert S.run_walk_goldens("cpu") > 0


def test_pss_goldens():
    assert S.run_pss_goldens("cpu") > 0


def test_c3_synthetic_edge():
    st, _ = S.run_synthetic("cpu", cases.best_practices() + cases.chart_restricted(), 400, seed=21)
    assert st["compared"] > 5000


def test_quirk_policies():
    st, _ = S.run_synthetic("cpu", cases.quirk_policies(), 400, seed=22)
    assert st["compared"] > 2000


def test_goldens_merged_cpu():
    """the merged golden corpus (every golden policy x every golden resource) on the host instantiation"""
    st, _ = S.run_merged("cpu", S.golden_groups(), "goldens-merged/cpu")
    assert st["compared"] > 1000


def test_c4_policycache_stress_cpu():
    """configs[3] shape at reduced size: 1,000 generated wildcard-heavy policies x 300 mixed resources"""
    st, _ = S.run_c4("cpu", 1000, 300)
    assert st["compared"] > 300000


def test_condition_goldens_cpu():
    assert S.run_condition_goldens("cpu") >= 300


def test_c5_conditions_cpu():
    """configs[4]: deny / preconditions with request.object variables, length() included, on the device; since round 6
    the regex_match / to_upper rules too (per-string columns of the dictionary): no rule is handed to the CPU engine"""
    from kyverno_amd import synth
    from kyverno_amd import engine as E
    pols = synth.c5_policies(50)
    st, _ = S.run_synthetic("cpu", pols, 500, seed=12)
    assert st["compared"] > 5000
    rs = E.Ruleset(pols)
    fb = [r for r in rs.rules if r["kind"] == "fallback"]
    assert not fb, fb[:3]
