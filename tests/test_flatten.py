"""The streaming flattener (kyverno_amd/csrc/batch.cpp) on raw JSON bytes: escapes, surrogates, invalid UTF-8,
duplicate keys (the later value wins, also in maps past the hashed-duplicate threshold), number classification
(-0, exponents, int64 overflow), apiVersion forms, anchor-error phrases and anchor-like metadata keys, and the
input framings the C ABI accepts (NDJSON with blank lines / CRLF, a JSON array, pretty-printed concatenated
documents that defeat the line splitter). Every framing must give the same verdict matrix, and that matrix must
equal the oracle's on each document's own bytes (the oracle parses with its own JSON reader)."""
import json

import numpy as np

from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from oracle import oracle as O

ORACLE = {"pass": K.ST_PASS, "fail": K.ST_FAIL, "skip": K.ST_SKIP, "error": K.ST_ERROR, "panic": K.ST_PANIC}


def _pol(name, pattern=None, kinds=("Pod", "Deployment"), deny=None):
    rule = {"name": "r", "match": {"any": [{"resources": {"kinds": list(kinds)}}]}}
    rule["validate"] = {"message": "m", "pattern": pattern} if pattern is not None else {"message": "m", "deny": deny}
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
            "spec": {"validationFailureAction": "Audit", "rules": [rule]}}


POLICIES = [
    _pol("label-app", {"metadata": {"labels": {"app": "?*"}}}),
    _pol("replicas", {"spec": {"replicas": ">1"}}),
    _pol("name-a", {"metadata": {"name": "*A*"}}),
    _pol("deny-zero", deny={"conditions": {"any": [{"key": "{{ request.object.spec.replicas }}", "operator": "Equals",
                                                     "value": 0}]}}),
    _pol("image", {"spec": {"containers": [{"image": "!*:latest"}]}}),
    _pol("any-kind-ns", {"metadata": {"namespace": "?*"}}, kinds=("*",)),
]

_BIG_LABELS = ",".join('"k%d":"v%d"' % (i, i) for i in range(40))

DOCS = [
    b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"dup","namespace":"d","labels":{"app":"x"},'
    b'"labels":{"app2":"y"}},"spec":{"containers":[{"image":"a:1"}]}}',
    b'{"kind":"Pod","apiVersion":"v1","metadata":{"name":"nested","labels":{"app":{"app":"z"}},"labels":{"app":"w"}}}',
    b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"c\\u0041\\n","namespace":"d","labels":{"app":"\\ud83d\\ude00"}},'
    b'"spec":{"containers":[{"image":"x\\/y:latest"}]}}',
    b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"lone\\ud800A","labels":{"app":"\\udc00"}}}',
    b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"bad\xffA\xc3","labels":{"app":"\xe2\x82"}}}',
    b'{"apiVersion":"apps/v1","kind":"Deployment","metadata":{"name":"negzero","namespace":"d"},"spec":{"replicas":-0}}',
    b'{"apiVersion":"apps/v1","kind":"Deployment","metadata":{"name":"exp","namespace":"d"},"spec":{"replicas":1e3}}',
    b'{"apiVersion":"apps/v1","kind":"Deployment","metadata":{"name":"frac","namespace":"d"},"spec":{"replicas":1.5}}',
    b'{"apiVersion":"apps/v1","kind":"Deployment","metadata":{"name":"i64max"},"spec":{"replicas":9223372036854775807}}',
    b'{"apiVersion":"apps/v1","kind":"Deployment","metadata":{"name":"i64ovf"},"spec":{"replicas":9223372036854775808}}',
    b'{"apiVersion":"apps/v1","kind":"Deployment","metadata":{"name":"huge"},"spec":{"replicas":-123456789012345678901}}',
    b'{"apiVersion":"apps/v1","kind":"Deployment","metadata":{"name":"zero"},"spec":{"replicas":0}}',
    b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"big","labels":{' + _BIG_LABELS.encode() +
    b',"app":"first","k5":"again","app":""}}}',
    b'{"apiVersion":"/v1","kind":"Pod","metadata":{"name":"slashv1","labels":{"app":"q"}}}',
    b'{"apiVersion":"a/b/c","kind":"Pod","metadata":{"name":"threeparts","labels":{"app":"q"}}}',
    b'{"apiVersion":"","kind":"Pod","metadata":{"name":"noav","labels":{"app":"q"}}}',
    b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"magic","labels":{"app":"conditional anchor mismatch"}}}',
    b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"anchorish","(labels)":{"app":"q"}}}',
    b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"ws" , "labels" : { "app" : "spaced" } } , "spec" : { } }',
    b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"emptyobj","labels":{}},"spec":{"containers":[]}}',
    b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"nullish","labels":null,"namespace":7},"spec":null}',
    b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"' + b"L" * 300 + b'A","labels":{"app":"' + b"v" * 70 + b'"}}}',
]


def _pretty(doc):
    return json.dumps(json.loads(doc.decode("utf-8", "replace")), indent=2).encode()


def _framings():
    nd = b"\n".join(DOCS)
    yield "ndjson", nd
    yield "ndjson-crlf-blank", b"\r\n\n  \r\n".join(DOCS) + b"\r\n"
    yield "array", b"[" + b",\n".join(DOCS) + b"]"
    yield "concatenated", b"".join(DOCS)


def _oracle_matrix(rs):
    want = np.full((len(rs.rules), len(DOCS)), K.ST_NONE, dtype=np.uint8)
    idx = {(rs.policies[r["policy"]]["name"], r["name"]): k for k, r in enumerate(rs.rules)}
    for ri, d in enumerate(DOCS):
        for p in O.validate(POLICIES, d):
            for rr in p["rules"]:
                st = rr["status"]
                want[idx[(p["policy"], rr["name"])], ri] = ORACLE.get(st, K.ST_FALLBACK)
    return want


def test_framings_agree_and_match_oracle():
    rs = E.Ruleset(POLICIES)
    want = _oracle_matrix(rs)
    mats = {}
    for name, data in _framings():
        b = E.Batch(rs, data)
        assert b.n == len(DOCS), name
        mats[name] = E.evaluate(rs, b, backend="cpu").status.copy()
    base = mats["ndjson"]
    for name, m in mats.items():
        assert np.array_equal(m, base), name
    dev = base.copy()
    # device FALLBACK pairs are the CPU engine's; compare everything else
    mask = (dev != K.ST_FALLBACK) & (want != K.ST_FALLBACK)
    bad = [(rs.rules[k]["name"], rs.policies[rs.rules[k]["policy"]]["name"], DOCS[r][:80], int(dev[k, r]), int(want[k, r]))
           for k, r in zip(*np.nonzero(mask & (dev != want)))]
    assert not bad, bad
    assert mask.sum() > 60


def test_pretty_printed_documents_split_by_grammar():
    """multi-line documents are not one per line: the line splitter's parse fails and the batch is re-split by the
    JSON grammar, giving the same verdicts as the compact form"""
    rs = E.Ruleset(POLICIES)
    docs = [d for d in DOCS if b"\xff" not in d and b"\xe2\x82" not in d and b"\\ud800" not in d and b"\\udc00" not in d]
    compact = E.evaluate(rs, E.Batch(rs, b"\n".join(docs)), backend="cpu").status
    pretty = E.evaluate(rs, E.Batch(rs, b"\n".join(_pretty(d) for d in docs)), backend="cpu").status
    assert np.array_equal(compact, pretty)


def test_malformed_input_errors():
    rs = E.Ruleset(POLICIES)
    for bad in (b'{"a":1}\n{"b":', b'{"a":1},', b'{"a":tru}', b'{"a":"\x01"}', b'{"a":01}'):
        try:
            E.Batch(rs, bad)
        except K.KyvError as e:
            assert "json" in str(e)
        else:
            raise AssertionError("accepted %r" % bad)
