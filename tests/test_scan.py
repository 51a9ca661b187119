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
