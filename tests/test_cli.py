"""`kyverno apply` counting (kyverno_amd/cli.py) on BASELINE configs[0]: the two best-practices
policies over 1,000 synthetic Pods; the device verdicts tallied as ProcessValidateEngineResponse does must equal
the same tally over the oracle's engine.Validate responses, pair by pair."""
import json

import pytest

import cases
from kyverno_amd import cli
from kyverno_amd import synth
from oracle import oracle as O

C1 = ("disallow-latest-tag", "require-pod-requests-limits")


def _oracle_engine(policy, resource):
    out = O.validate([policy], json.dumps(resource))
    return [{"name": r["name"], "status": r["status"], "message": r["message"]} for p in out for r in p["rules"]]


def _c1():
    pols = [p for p in cases.best_practices() if p["metadata"]["name"] in C1]
    docs, _ = synth.pods(1000, seed=21, edge=False)
    for d in docs[::7]:
        d["metadata"].pop("namespace", None)  # file resources without a namespace: CLI default "default"
    return pols, docs


def _reference_counts(pols, docs, audit_warn=False):
    rc = cli.ResultCounts()
    for p in pols:
        names = [r["name"] for r in O.compute_rules(p) if r.get("validate")]
        for d in cli._with_default_namespace(docs):
            cli.process_validate_response(names, _oracle_engine(p, d), p, rc, audit_warn,
                                          (p.get("spec") or {}).get("validationFailureAction", ""))
    return rc


def _check(backend):
    pols, docs = _c1()
    calls = []

    def recording_engine(policy, resource):  # must never run: every C1 pair is decided by the library
        calls.append((policy["metadata"]["name"], (resource.get("metadata") or {}).get("name")))
        return _oracle_engine(policy, resource)

    got, pending = cli.apply(pols, docs, backend=backend, cpu_engine=recording_engine)
    assert not pending
    assert calls == [], "C1 pairs handed to the CPU engine: %r" % calls[:5]
    want = _reference_counts(pols, docs)
    assert got.as_dict() == want.as_dict()
    d = got.as_dict()
    assert d["pass"] > 0 and d["fail"] > 0 and d["skip"] > 0  # autogen rules never match Pods -> skip
    assert got.line().startswith("\npass: %d, fail: %d" % (d["pass"], d["fail"]))
    return got


def test_cli_apply_c1_counts_cpu_instantiation():
    _check("cpu")


def test_cli_counts_scored_false_and_audit_warn():
    pols, docs = _c1()
    pols = [json.loads(json.dumps(p)) for p in pols]
    pols[0]["metadata"].setdefault("annotations", {})["policies.kyverno.io/scored"] = "false"
    for p in pols:
        p["spec"]["validationFailureAction"] = "Audit"
    got, _ = cli.apply(pols, docs[:200], backend="cpu", audit_warn=True, cpu_engine=_oracle_engine)
    want = _reference_counts(pols, docs[:200], audit_warn=True)
    assert got.as_dict() == want.as_dict() and got.fail == 0 and got.warn > 0


def test_cli_pending_without_cpu_engine():
    pols = [p for p in cases.best_practices() if p["metadata"]["name"] == "select-secrets"]  # variables: CPU engine
    docs, _ = synth.pods(20, seed=3)
    rc, pending = cli.apply(pols, docs, backend="cpu")
    assert pending


@pytest.mark.gpu
def test_cli_apply_c1_counts_gpu():
    _check("gpu")


def test_cli_apply_report_summaries_golden(golden):
    """cmd/cli/kubectl-kyverno/apply/apply_command_test.go Test_Apply: the report summary of every local-file case
    (incl. test/cli/apply, whose drop-all-capabilities policy runs a foreach over
    `request.object.spec.[ephemeralContainers, initContainers, containers][]` with an `element... || ''` deny) from
    the oracle's responses and from the library's verdicts (explicit CPU instantiation, CPU engine for the rest)"""
    recs = golden("cli_apply.json")
    assert len(recs) >= 6
    for r in recs:
        pols, docs = r["policies"], r["resources"]
        want = r["summary"]
        ref = cli.ResultCounts()
        for p in pols:
            names = [x["name"] for x in O.compute_rules(p) if x.get("validate")]
            for d in cli._with_default_namespace(docs):
                cli.process_validate_response(names, _oracle_engine(p, d), p, ref, r["audit_warn"],
                                              (p.get("spec") or {}).get("validationFailureAction", ""))
        assert ref.as_dict() == want, (r["policy_files"], ref.as_dict(), want)
        got, pending = cli.apply(pols, docs, backend="cpu", audit_warn=r["audit_warn"], cpu_engine=_oracle_engine)
        assert not pending
        assert got.as_dict() == want, (r["policy_files"], got.as_dict(), want)
