"""Property tests (Hypothesis): random patterns (anchors, operators, wildcards, ranges, quantities, durations,
arrays of maps, scalar arrays) over random resources, evaluated by the library's host instantiation of the device
evaluator and by the oracle. Status, failing path and message must agree on every pair both decide (the device's
CPU-fallback / nondeterministic pairs and the oracle's unsupported ones are skipped). SURVEY §4 step 4."""
import json

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from oracle import oracle as O

KEYS = ["a", "b", "c", "name", "image", "ports"]
ANCHORED = ["(a)", "(b)", "X(c)", "=(a)", "^(b)", "<(c)", "+(a)", "(name)", "X(image)", "^(ports)"]
LEAF_PATTERNS = ["*", "?*", "a*", "*b", "!a", "a | b", ">1", "<=5", ">=2", "<3", "1-5", "!1-3", "1Gi", ">1Gi",
                 "<=512Mi", "10s", "<5m", ">=1h", "!*", "?", "", "null", "true", "a?c", "!b | a", "0.5-2.5"]
VALUES = ["a", "ab", "abc", "b", "1", "5", "1Gi", "2Gi", "10s", "1m", "", "true", "a-b", "512Mi", "x*"]

scalar_res = st.one_of(st.sampled_from(VALUES), st.integers(-3, 8), st.sampled_from([0.5, 1.5, 2.0, -1.25]),
                       st.booleans(), st.none())
scalar_pat = st.one_of(st.sampled_from(LEAF_PATTERNS), st.integers(-1, 6), st.sampled_from([1.5, 2.0]),
                       st.booleans(), st.none())


def res_value(depth):
    if depth <= 0:
        return scalar_res
    return st.one_of(
        scalar_res,
        st.dictionaries(st.sampled_from(KEYS), res_value(depth - 1), max_size=4),
        st.lists(res_value(depth - 1), max_size=3),
    )


def pat_value(depth):
    if depth <= 0:
        return scalar_pat
    return st.one_of(
        scalar_pat,
        st.dictionaries(st.sampled_from(KEYS + ANCHORED), pat_value(depth - 1), min_size=1, max_size=3),
        st.lists(st.dictionaries(st.sampled_from(KEYS + ANCHORED), pat_value(depth - 2 if depth > 1 else 0),
                                 min_size=1, max_size=2), min_size=1, max_size=1),
        st.lists(scalar_pat, min_size=1, max_size=2),
    )


def _pod(i, spec):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p%d" % i, "namespace": "d"}, "spec": spec}


def _policies(pats, any_pats):
    out = []
    for i, p in enumerate(pats):
        out.append({"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "pat-%d" % i},
                    "spec": {"rules": [{"name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                                        "validate": {"message": "m%d" % i, "pattern": {"spec": p}}}]}})
    for i, alts in enumerate(any_pats):
        out.append({"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "any-%d" % i},
                    "spec": {"rules": [{"name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                                        "validate": {"anyPattern": [{"spec": a} for a in alts]}}]}})
    return out


ORACLE = {"pass": K.ST_PASS, "fail": K.ST_FAIL, "skip": K.ST_SKIP, "error": K.ST_ERROR, "panic": K.ST_PANIC}


def _compare(pols, docs):
    rs = E.Ruleset(pols)
    res = E.evaluate(rs, E.Batch(rs, docs), backend="cpu")
    idx = {(rs.policies[r["policy"]]["name"], r["name"]): k for k, r in enumerate(rs.rules)}
    n = 0
    for ri, d in enumerate(docs):
        for p in O.validate(pols, json.dumps(d)):
            for rr in p["rules"]:
                k = idx.get((p["policy"], rr["name"]))
                if k is None:
                    continue
                s = int(res.status[k, ri])
                if s in (K.ST_FALLBACK, K.ST_ND) or rr["status"] not in ORACLE or rr.get("nondeterministic"):
                    continue
                ctx = (p["policy"], json.dumps(pols[[q["metadata"]["name"] for q in pols].index(p["policy"])]["spec"]
                                               ["rules"][0]["validate"]), json.dumps(d["spec"]))
                assert s == ORACLE[rr["status"]], ctx + (K.STATUS_NAMES[s], rr)
                if s == K.ST_FAIL and rs.rules[k]["kind"] == "pattern":
                    assert res.path(ri, k) == rr["path"], ctx + (res.path(ri, k), rr["path"])
                m = res.message(ri, k)
                if m is not None and not rr.get("message_unpinned"):
                    assert m == rr["message"], ctx + (m, rr["message"])
                n += 1
    return n


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(pats=st.lists(pat_value(3), min_size=1, max_size=4),
       any_pats=st.lists(st.lists(pat_value(2), min_size=1, max_size=3), max_size=2),
       specs=st.lists(res_value(3), min_size=1, max_size=6))
def test_random_patterns_match_oracle(pats, any_pats, specs):
    pols = _policies(pats, any_pats)
    docs = [_pod(i, s) for i, s in enumerate(specs)]
    _compare(pols, docs)


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(pats=st.lists(pat_value(2), min_size=1, max_size=3),
       specs=st.lists(st.dictionaries(st.sampled_from(KEYS), res_value(2), max_size=5), min_size=1, max_size=6))
def test_random_map_resources_match_oracle(pats, specs):
    """resources whose spec is always a map (the common case), so map-level anchors are exercised more"""
    pols = _policies(pats, [])
    docs = [_pod(i, s) for i, s in enumerate(specs)]
    _compare(pols, docs)
