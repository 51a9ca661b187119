"""Per-batch metrics and PolicyResponse stats (kyverno_amd/metrics.py) against a pair-by-pair restatement of the
reference's recording over the oracle's verdicts: one kyverno_policy_results increment per rule response with the
labels of pkg/metrics/metrics.go:178-191 (policyresults/policyResults.go:35-79), and RulesAppliedCount /
RulesErrorCount per EngineResponse (validation.go:196-208)."""
import collections

import numpy as np

import cases
from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from kyverno_amd import metrics as M
from kyverno_amd import synth
from oracle import oracle as O
from parity_util import _MATRIX_TO_DEVICE

RES = {K.ST_PASS: "pass", K.ST_FAIL: "fail", K.ST_SKIP: "skip", K.ST_ERROR: "error"}


def _setup(n=600, seed=61):
    pols = cases.best_practices() + cases.quirk_policies()
    multi = {pm["name"] for pm in E.Ruleset(pols).policies if pm["nrules"] > 1}
    i = next(i for i, p in enumerate(pols) if p["metadata"]["name"] in multi)  # Enforce + applyRules: One
    pols[i] = dict(pols[i], spec=dict(pols[i]["spec"], validationFailureAction="Enforce", applyRules="One"))
    docs, nsl = synth.mixed(n, seed=seed, edge=True)
    docs = [d for d in docs if isinstance(d, dict)]
    rs = E.Ruleset(pols)
    res = E.evaluate(rs, E.Batch(rs, docs, nsl), backend="cpu")
    by = {(p.get("metadata") or {}).get("name"): p for p in pols}
    docs_by_policy = [by[pm["name"]] for pm in rs.policies]
    return pols, docs, nsl, rs, res, docs_by_policy


def _oracle_status(pols, docs, nsl, rs):
    names, m = O.validate_matrix(pols, docs, nsl, threads=8)
    row = {nm: i for i, nm in enumerate(names)}
    lut = np.array([_MATRIX_TO_DEVICE[i] for i in range(8)], dtype=np.uint8)
    out = np.zeros((len(rs.rules), len(docs)), dtype=np.uint8)
    for k, r in enumerate(rs.rules):
        key = (rs.policies[r["policy"]]["name"], r["name"])
        if key in row:
            out[k] = lut[m[row[key]]]
    return out


def test_policy_results_metric_matches_per_response_recording():
    pols, docs, nsl, rs, res, pdocs = _setup()
    st = np.asarray(res.status) & 7
    assert np.array_equal(st, _oracle_status(pols, docs, nsl, rs))  # the verdicts the metrics are built from
    pm = M.PolicyMetrics()
    kinds = [d.get("kind", "") for d in docs]
    nss = [(d.get("metadata") or {}).get("namespace", "") for d in docs]
    pm.record(rs, pdocs, res, kinds, nss, cause="admission_request", operation="create", seconds=0.01)
    # restatement: walk every EngineResponse (resource x policy), one increment per rule response
    want = collections.Counter()
    for r in range(len(docs)):
        for pi, p in enumerate(rs.policies):
            info = M.policy_infos(pdocs[pi])
            applied = 0
            for k in range(p["first_rule"], p["first_rule"] + p["nrules"]):
                s = int(st[k, r])
                if s == K.ST_NONE:
                    continue
                if s in RES:
                    want[(info["validation"], info["type"], info["background"], "-", info["name"], kinds[r], nss[r],
                          "create", rs.rules[k]["name"], RES[s], "validate", "admission_request")] += 1
                if s in (K.ST_PASS, K.ST_FAIL):
                    applied += 1
                if p["apply_one"] and applied > 0:
                    break
    assert dict(want) == pm.results
    assert sum(want.values()) > 1000 and any(k[0] == "enforce" for k in want)
    text = pm.exposition()
    assert "kyverno_policy_results_total{" in text
    assert "kyverno_policy_execution_duration_seconds_bucket{" in text
    tot = sum(v[-2] + sum(v[:-2]) for v in pm.durations.values())
    assert tot == sum(want.values())


def test_policy_response_stats():
    pols, docs, nsl, rs, res, _ = _setup(300, seed=62)
    applied, errors = M.policy_stats(rs, res.status)
    out, _, _ = E.Engine(pols, backend="cpu").validate_batch(docs, nsl)
    for r, per_policy in enumerate(out):
        for pi, pr in enumerate(per_policy):
            a = sum(1 for x in pr["rules"] if x["status"] in ("pass", "fail"))
            e = sum(1 for x in pr["rules"] if x["status"] == "error")
            assert (applied[pi, r], errors[pi, r]) == (a, e)
            assert pr["stats"] == {"rulesAppliedCount": a, "rulesErrorCount": e}
    assert applied.sum() > 500


def test_apply_one_stops_at_cpu_pair():
    """applyRules: One -- after a pair the CPU engine decides, whether later rules respond depends on its verdict: the
    device records none of them (as engine.Engine.validate stops there)"""
    st = np.array([[K.ST_NONE, K.ST_FALLBACK, K.ST_PASS, K.ST_ND],
                   [K.ST_FAIL, K.ST_PASS, K.ST_PASS, K.ST_SKIP],
                   [K.ST_PASS, K.ST_SKIP, K.ST_FAIL, K.ST_FAIL]], dtype=np.uint8)
    r = M.responded(st, 0, 3, True)
    want = np.array([[False, True, True, True],
                     [True, False, False, False],
                     [False, False, False, False]])
    assert np.array_equal(r, want)
    assert np.array_equal(M.responded(st, 0, 3, False), st != K.ST_NONE)
