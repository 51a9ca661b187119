"""Batched background scan (kyverno_amd/scan.py): per-policy report summaries from the device's per-rule verdict
totals against summaries built from the oracle's per-resource engine.Validate results the way the reference
builds them (EngineResponseToReportResults + CalculateSummary, pkg/utils/report/results.go:38-124); and the
multi-rank path: shard summaries summed with one all-reduce (gloo here, RCCL on the GPU box)."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

import cases
from kyverno_amd import scan as S
from kyverno_amd import synth
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def policy_set():
    pols = cases.best_practices() + cases.chart_restricted() + synth.c5_policies(20) + cases.quirk_policies()
    nbp = len(cases.best_practices())
    for i in range(nbp):  # best-practices policies unscored: their failures are reported as warn
        pols[i] = json.loads(json.dumps(pols[i]))
        pols[i].setdefault("metadata", {}).setdefault("annotations", {})["policies.kyverno.io/scored"] = "false"
    one = json.loads(json.dumps(cases.chart_restricted()[0]))
    one["metadata"]["name"] += "-one"
    one["spec"]["applyRules"] = "One"
    return pols + [one]


def oracle_summary(policies, docs, nsl):
    out = {}
    pols = [p for p in policies if (p.get("spec") or {}).get("background", True) is not False]
    for d in docs:
        ns = (d.get("metadata") or {}).get("namespace") if isinstance(d.get("metadata"), dict) else None
        for pr, pol in zip(O.validate(pols, json.dumps(d), (nsl or {}).get(ns) or {}), pols):
            scored = ((pol.get("metadata") or {}).get("annotations") or {}).get("policies.kyverno.io/scored") != "false"
            s = out.setdefault(S.policy_key(pol), dict.fromkeys(S.SUMMARY_FIELDS, 0))
            for rr in pr["rules"]:
                st = rr["status"]
                if st in ("unsupported", "panic") or rr.get("nondeterministic"):
                    s["cpu_fallback"] += 1
                elif st == "fail" and not scored:
                    s["warn"] += 1
                else:
                    s[st] += 1
    return out


def test_scan_summary_matches_oracle():
    pols = policy_set()
    docs, nsl = synth.mixed(400, seed=41, edge=True)
    rep = S.BackgroundScan(pols, backend="cpu").scan(docs, nsl)
    got, want = rep.summary(), oracle_summary(pols, docs, nsl)
    assert set(got) == set(want)
    bad = {k: (got[k], want[k]) for k in got if got[k] != want[k]}
    assert not bad, list(bad.items())[:3]
    assert sum(v["pass"] + v["fail"] + v["warn"] for v in got.values()) > 1000
    assert any(v["warn"] for v in got.values()) and any(v["cpu_fallback"] for v in got.values())
    # rows of one resource agree with the summary's counting rules
    rows = [r for i in range(len(docs)) for r in rep.results(i)]
    assert sum(1 for r in rows if r.get("cpu_fallback")) == sum(v["cpu_fallback"] for v in got.values())
    assert sum(1 for r in rows if r.get("result") == "warn") == sum(v["warn"] for v in got.values())
    assert len(rep.fallback_pairs()) >= sum(v["cpu_fallback"] for v in got.values())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from kyverno_amd import scan as S2
    from kyverno_amd import synth as syn
    import test_scan as T
    dist.init_process_group("gloo", rank=rank, world_size=world)
    docs, nsl = syn.mixed(300, seed=43, edge=True)
    shard = docs[rank::world]
    sc = S2.BackgroundScan(T.policy_set(), backend="cpu")
    mat = sc.scan(shard, nsl).summary_matrix()
    tot = S2.reduce_summary(mat)
    q.put((rank, tot.tolist()))
    dist.destroy_process_group()


def test_two_rank_summary_allreduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(i, 2, port, q)) for i in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    docs, nsl = synth.mixed(300, seed=43, edge=True)
    full = S.BackgroundScan(policy_set(), backend="cpu").scan(docs, nsl).summary_matrix()
    assert out[0][1] == out[1][1] == full.tolist()


_KUTTL_DIR = "test/conformance/kuttl/reports/background/test-report-background-mode"


def test_pss_report_row_kuttl_golden():
    """The PolicyReport row of the kuttl background-scan fixture (_KUTTL_DIR/report-assert.yaml: category, message,
    policy, result, rule, scored, severity, source) with the properties results.go:102-116 adds for the failed
    PodSecurity checks: standard / version of the rule, controls = the failing check IDs sorted and joined (one per
    failing check version, as PodSecurityChecks lists them)."""
    import test_boundary as TB
    pol = json.loads(json.dumps(TB._KUTTL_POLICY))
    pol["metadata"]["annotations"] = {"policies.kyverno.io/category": "Pod Security",
                                      "policies.kyverno.io/severity": "medium"}  # _KUTTL_DIR/policy.yaml
    rep = S.BackgroundScan([pol], backend="cpu").scan([TB._KUTTL_POD])
    rows = rep.results(0)
    assert len(rows) == 1
    row = rows[0]
    line = ("({Allowed:false ForbiddenReason:unrestricted capabilities ForbiddenDetail:container \"container01\" must "
            "set securityContext.capabilities.drop=[\"ALL\"]})\n")
    want = {"category": "Pod Security", "policy": "podsecurity-subrule-restricted", "result": "fail",
            "rule": "restricted", "scored": True, "severity": "medium", "source": "kyverno",
            "message": "Validation rule 'restricted' failed. It violates PodSecurity \"restricted:latest\": " + line + line}
    assert {k: row[k] for k in want} == want
    assert row["properties"] == {"standard": "restricted", "version": "latest",
                                 "controls": "capabilities_restricted,capabilities_restricted"}
    assert rep.summary()["podsecurity-subrule-restricted"]["fail"] == 1


def test_pss_report_properties_match_oracle_checks():
    """report-row properties of every failing podSecurity pair of a synthetic corpus equal the ones built from the
    oracle's PodSecurityChecks (results.go:102-116 restated on the oracle's rule responses)"""
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "psa"},
           "spec": {"rules": [{"name": "restricted", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                               "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}}]}}
    docs, nsl = synth.mixed(600, seed=47, edge=True)
    rep = S.BackgroundScan([pol], backend="cpu").scan(docs, nsl)
    n = 0
    for i, d in enumerate(docs):
        for row in rep.results(i):
            if row["result"] != "fail":
                continue
            ns = (d.get("metadata") or {}).get("namespace") if isinstance(d.get("metadata"), dict) else None
            o = O.validate([pol], json.dumps(d), (nsl or {}).get(ns) or {})[0]["rules"][0]
            checks = o.get("pss_checks")  # the oracle lists the failing checks
            if checks is None or row["properties"] is None:
                continue
            controls = sorted(c["id"] for c in checks)
            assert row["properties"] == {"standard": "restricted", "version": "latest", "controls": ",".join(controls)}
            n += 1
    assert n > 50
