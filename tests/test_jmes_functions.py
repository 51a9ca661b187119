"""JMESPath functions on the dictionary (round 6): kyverno's to_upper() and regex_match()
(pkg/engine/jmespath/functions.go:681-689, 786-799) compiled as per-string columns of the batch -- strings.ToUpper
interned per dictionary string (Batch::str_upper), regexp.Match as one bit per ruleset regex (Batch::str_rx, a DFA
over printable ASCII: kyverno_amd/csrc/regex.cpp) -- and evaluated by the light kernels' chain evaluator
(kyv_cond.h jmes_chain_cv). Checked pair by pair against the oracle's restatement (oracle/ojmes.cpp: std::regex
ECMAScript on the same syntax subset, checked independently there) on the explicit CPU instantiation of the device
evaluator; the GPU path runs the same corpus in tests/test_gpu_parity.py.

The reference's own vectors: functions_test.go's to_upper cases (Test_ToUpper: 'abc' -> 'ABC', '123', 'a#%&123Bc')
and regex_match's ('12.*' against 123 / '12.*' against abs(foo)). Numbers as regex_match subjects are outside the
restatement (ifaceToString formats a float64 as float32 text) and go to the CPU engine on both sides; patterns outside
the syntax subset leave the whole rule on the CPU engine (rule-level fallback on both sides). parity unpinned beyond
those vectors and the restatement."""
import json

import parity_util as PU
from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from kyverno_amd import synth


def _pol(name, cond, pre=None, kinds=("Pod",)):
    rule = {"name": "r", "match": {"any": [{"resources": {"kinds": list(kinds)}}]},
            "validate": {"message": "m", "deny": {"conditions": cond}}}
    if pre is not None:
        rule["preconditions"] = pre
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy",
            "metadata": {"name": name, "annotations": {"pod-policies.kyverno.io/autogen-controllers": "none"}},
            "spec": {"rules": [rule]}}


def _c(k, op, v):
    return {"key": k, "operator": op, "value": v}


REGEXES = [
    "^team-[0-9]+$", "app-(1|2)[a-z]*", "\\d\\d\\d?", "^[^x]+$", "a.b", "(?:fr|ba)ont", "value-1?$", "^$", "",
    "[a-c][^0-9][^0-9]", "tier|owner", "^ns-00[0-9][0-9]$", "registry\\.example\\.com/team1?", "(ab)+c*", "xx?y?$",
    "[\\w-]+:latest$", "\\s", "^\\S+$", "[-a]", "1+?",
]
# outside the device subset (rule-level CPU fallback on both sides): flags, \b, look-ahead, a repeated quantifier,
# POSIX classes, hex escapes, an unbalanced group; and counted repetitions {n,m}, whose braces the compiler does not
# take inside a `{{ }}` variable
OUTSIDE = ["(?i)team", "a\\bb", "(?=x)", "a**", "[[:alpha:]]", "\\x41", "(a", "a{2,1}", "\\d{2,3}"]


def function_policies():
    o = "request.object.%s"
    pols = []
    for i, rx in enumerate(REGEXES + OUTSIDE):
        lit = rx.replace("'", "\\'")
        pols.append(_pol("rx-%02d" % i, {"any": [_c("{{ regex_match('%s', %s || '') }}" % (lit, o % "metadata.labels.owner"),
                                                  "Equals", False)]}))
    pols += [
        _pol("rx-name", {"all": [_c("{{ regex_match('%s', %s) }}" % (REGEXES[1], o % "metadata.name"), "Equals", True)]}),
        _pol("rx-ns", {"any": [_c("{{ regex_match('%s', %s) }}" % (REGEXES[11], o % "metadata.namespace"), "Equals", True),
                               _c("{{ regex_match('%s', %s || 'team-1') }}" % (REGEXES[0], o % "metadata.labels.tier"),
                                  "NotEquals", True)]}),
        # a missing key without a default: the argument is null -> the argument type error (rule error)
        _pol("rx-null", {"any": [_c("{{ regex_match('a', %s) }}" % (o % "metadata.labels.nope"), "Equals", True)]}),
        # a number (replicas) as the subject: outside the restatement on both sides
        _pol("rx-number", {"any": [_c("{{ regex_match('^[0-9]$', %s) }}" % (o % "spec.replicas"), "Equals", True)]},
             kinds=("Deployment",)),
        _pol("up-tier", {"any": [_c("{{ to_upper(%s || '') }}" % (o % "metadata.labels.tier"), "Equals", "DATA")]}),
        _pol("up-tier-in", {"any": [_c("{{ to_upper(%s || 'none') }}" % (o % "metadata.labels.tier"), "In",
                                       ["FRONTEND", "NONE"])]}),
        _pol("up-wild", {"all": [_c("{{ to_upper(%s) }}" % (o % "metadata.name"), "Equals", "POD-1*")]}),
        _pol("up-ns", {"any": [_c("{{ to_upper(%s) }}" % (o % "metadata.namespace"), "AnyIn", ["NS-00*"])]}),
        _pol("up-null", {"any": [_c("{{ to_upper(%s) }}" % (o % "metadata.labels.nope"), "Equals", "X")]}),
        _pol("up-num", {"any": [_c("{{ to_upper(%s) }}" % (o % "spec.replicas"), "Equals", "3")]}, kinds=("Deployment",)),
        _pol("up-pre", {"any": [_c("{{ request.object.metadata.name }}", "Equals", "*")]},
             pre={"all": [_c("{{ to_upper(%s || '') }}" % (o % "metadata.labels.app"), "NotEquals", "APP-1*")]}),
        # functions beside a projection operand: the interpreted / compiled condition kernels take the rule
        _pol("up-mixed", {"all": [_c("{{ request.object.spec.containers[].name }}", "AnyIn", ["*"]),
                                  _c("{{ to_upper(%s || '') }}" % (o % "metadata.labels.owner"), "NotEquals", "")]}),
    ]
    return pols


def _edge_docs():
    base = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "e", "namespace": "ns-0001"},
            "spec": {"containers": [{"name": "c", "image": "nginx:latest"}]}}
    out = []
    for i, owner in enumerate(["team-12", "Team-1", "team-", "tëam-1", "team\t1", "abc", "", "12", "xyz", "a-b",
                               "registry.example.com/team1x", "ABABc", "app-1abc", "value-1", "frant"]):
        d = json.loads(json.dumps(base))
        d["metadata"]["name"] = "edge-%d" % i
        d["metadata"]["labels"] = {"owner": owner, "tier": ["data", "Data", "frontend", "DATA", "dätä", ""][i % 6]}
        out.append(d)
    d = json.loads(json.dumps(base))
    d["metadata"]["labels"] = {"owner": 12, "tier": True}  # non-string values: type error / number subject
    out.append(d)
    return out


def test_function_rules_compile_on_device():
    """every rule compiles to the device except the patterns outside the regex subset (rule-level CPU fallback)"""
    rs = E.Ruleset(function_policies())
    kinds = {rs.policies[r["policy"]]["name"]: r["kind"] for r in rs.rules}
    outside = {"rx-%02d" % i for i in range(len(REGEXES), len(REGEXES) + len(OUTSIDE))}
    assert {n for n, k in kinds.items() if k == "fallback"} == outside, kinds


def test_function_rules_match_oracle_cpu():
    docs, nsl = synth.mixed(4000, seed=71, edge=True)
    docs = _edge_docs() + docs
    st, res = PU.compare_matrix(function_policies(), docs, nsl, backend="cpu", texts=False)
    assert st["nbad"] == 0, st["bad"]
    status = res.status
    # both outcomes of the function rules occur, and the per-pair CPU fallbacks are the non-ASCII / number subjects only
    assert (status == K.ST_FAIL).sum() > 1000 and (status == K.ST_PASS).sum() > 1000
    assert (status == K.ST_ERROR).sum() > 0


def test_reference_function_vectors():
    """functions_test.go: to_upper('abc') == 'ABC', to_upper('123') == '123', to_upper('a#%&123Bc') == 'A#%&123BC';
    regex_match('12.*', '123') is true -- through conditions on a resource holding the arguments"""
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "default",
                                                          "labels": {"a": "abc", "b": "123", "c": "a#%&123Bc"}},
           "spec": {"containers": [{"name": "c", "image": "x"}]}}
    o = "request.object.metadata.labels.%s"
    pols = [_pol("up-a", {"all": [_c("{{ to_upper(%s) }}" % (o % "a"), "Equals", "ABC")]}),
            _pol("up-b", {"all": [_c("{{ to_upper(%s) }}" % (o % "b"), "Equals", "123")]}),
            _pol("up-c", {"all": [_c("{{ to_upper(%s) }}" % (o % "c"), "Equals", "A#%&123BC")]}),
            _pol("rx-b", {"all": [_c("{{ regex_match('12.*', %s) }}" % (o % "b"), "Equals", True)]})]
    rs = E.Ruleset(pols)
    b = E.Batch(rs, [pod], None)
    r = E.evaluate(rs, b, backend="cpu")
    # deny conditions that hold: every rule fails (the function returned the reference's value)
    assert [int(x) for x in r.status[:, 0]] == [K.ST_FAIL] * 4
    _, m, *_ = __import__("oracle.oracle", fromlist=["x"]).validate_matrix(pols, [pod], None, threads=1)
    assert [int(x) for x in m[:, 0]] == [2] * 4
