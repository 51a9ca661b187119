"""GPU parity: the HIP kernel (through the C-ABI) against the oracle, bit-exact verdicts, failing paths and
messages, on the reference's golden corpora and on seeded synthetic corpora; plus size-independent checks at
full batch sizes (GPU == explicit CPU instantiation of the same evaluator, count conservation, determinism)."""
import numpy as np
import pytest

import cases
import parity_suite as S
from kyverno_amd import _lib as K
from kyverno_amd import engine as E
from kyverno_amd import synth

pytestmark = pytest.mark.gpu


def test_engine_goldens_gpu():
    assert S.run_engine_goldens("gpu") > 0


def test_cli_goldens_gpu():
    assert S.run_cli_goldens("gpu") > 0


def test_walk_goldens_gpu():
    assert S.run_walk_goldens("gpu") > 0


def test_pss_goldens_gpu():
    assert S.run_pss_goldens("gpu") > 0


def test_c3_synthetic_gpu():
    st, res = S.run_synthetic("gpu", cases.best_practices() + cases.chart_restricted(), 3000, seed=31)
    assert st["compared"] > 50000
    assert res.kernel_ms > 0


def test_c2_pss_pods_gpu():
    pol = [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "psa"},
            "spec": {"rules": [{"name": "restricted", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                                "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}}]}}]
    st, _ = S.run_synthetic("gpu", pol, 4000, seed=32, kind="pods")
    assert st["compared"] >= 4000


def test_quirk_policies_gpu():
    st, _ = S.run_synthetic("gpu", cases.quirk_policies(), 3000, seed=33)
    assert st["compared"] > 10000


def test_gpu_equals_cpu_instantiation_at_scale():
    """200k mixed resources x C3 rules: identical verdict bytes, PSS masks and failing paths."""
    data, nsl = synth.corpus_ndjson(200_000, seed=34, edge=True)
    rs = E.Ruleset(cases.best_practices() + cases.chart_restricted())
    b = E.Batch(rs, data, nsl)
    g = E.evaluate(rs, b, backend="gpu")
    c = E.evaluate(rs, b, backend="cpu")
    assert np.array_equal(g.raw, c.raw)
    assert g.counts == c.counts
    assert sum(g.counts.values()) == len(rs.rules) * b.n
    rng = np.random.default_rng(0)
    fail = np.argwhere(g.status == K.ST_FAIL)
    for k, r in fail[rng.choice(len(fail), size=min(2000, len(fail)), replace=False)]:
        assert g.path(int(r), int(k)) == c.path(int(r), int(k))
        assert g.message(int(r), int(k)) == c.message(int(r), int(k))
        if rs.rules[k]["kind"] == "pss":
            assert g.pss_mask(int(r), int(k)) == c.pss_mask(int(r), int(k))


def _oracle_threads():
    import os
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)))


def test_c3_oracle_matrix_at_scale_jit():
    """configs[2] at scale through the production path (runtime-compiled walk, chosen automatically at this size):
    every verdict of 200k mixed resources x the C3 rules against the oracle's verdict matrix, and the failing path
    (single patterns) and RuleResponse.Message of every one of the ~1M FAIL pairs against the oracle's texts"""
    import parity_util as PU
    data, nsl = synth.corpus_ndjson(200_000, seed=52, edge=True)
    st, res = PU.compare_matrix(cases.best_practices() + cases.chart_restricted(), data, nsl, backend="gpu",
                                threads=_oracle_threads())
    assert res.jit
    assert st["nbad"] == 0, st["bad"]
    assert st["compared"] >= 200_000 * 80 and st["matched"] > 1_000_000
    t = st["texts"]
    print("C3 200k text parity:", {k: v for k, v in t.items() if k != "bad"})
    assert t["fail_pairs"] > 500_000 and t["paths_compared"] > 200_000
    assert t["messages_compared"] == t["fail_pairs"]


def test_c2_oracle_matrix_at_scale():
    """configs[1] at scale: podSecurity restricted/latest over 200k pods, every verdict against the oracle"""
    import parity_util as PU
    pol = [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "psa"},
            "spec": {"rules": [{"name": "restricted", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                                "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}}]}}]
    data, nsl = synth.corpus_ndjson(200_000, kind="pods", seed=53, edge=True)
    st, res = PU.compare_matrix(pol, data, nsl, backend="gpu", threads=_oracle_threads())
    assert st["nbad"] == 0, st["bad"]
    assert st["matched"] >= 200_000
    assert res.counts["fail"] > 0 and res.counts["pass"] > 0


def test_c5_oracle_matrix_at_scale():
    """configs[4] at scale: 50 precondition / deny policies over 200k mixed resources, every verdict against the
    oracle (CPU-fallback pairs must be exactly the oracle's unsupported ones)"""
    import parity_util as PU
    import json
    data, nsl = synth.corpus_ndjson(200_000, seed=54, edge=True)
    pols = synth.c5_policies(50)
    st, res = PU.compare_matrix(pols, data, nsl, backend="gpu", threads=_oracle_threads())
    assert st["nbad"] == 0, st["bad"]
    assert st["matched"] > 1_000_000
    # length() / || / projections and (round 6) regex_match / to_upper on the dictionary compile to the device: no
    # rule is CPU fallback, and the function rules decide pairs on the device
    fb = [r["name"] for r in res.ruleset.rules if r["kind"] == "fallback"]
    assert not fb, fb
    fn = [k for k, r in enumerate(res.ruleset.rules)
          if any(f in json.dumps(pols[r["policy"]]) for f in ("regex_match", "to_upper"))]
    assert fn
    st_fn = np.asarray(res.status)[fn] & 7
    assert ((st_fn == K.ST_PASS) | (st_fn == K.ST_FAIL)).sum() > 100_000


def test_repeat_launches_deterministic():
    data, nsl = synth.corpus_ndjson(50_000, seed=35)
    rs = E.Ruleset(cases.best_practices() + cases.chart_restricted())
    b = E.Batch(rs, data, nsl)
    a = E.evaluate(rs, b, backend="gpu")
    z = E.evaluate(rs, b, backend="gpu", iterations=3)
    assert np.array_equal(a.raw, z.raw)
    assert a.counts == z.counts
    nc = E.evaluate(rs, b, backend="gpu", copy_back=False)
    assert nc.counts == a.counts


def test_empty_and_tiny_batches_gpu():
    rs = E.Ruleset(cases.best_practices())
    for docs in ([], [{}], [{"kind": "Pod"}], [{"apiVersion": "v1", "kind": "Pod", "metadata": None, "spec": []}]):
        b = E.Batch(rs, docs)
        g = E.evaluate(rs, b, backend="gpu")
        c = E.evaluate(rs, b, backend="cpu")
        assert b.n == len(docs)
        if b.n:
            assert np.array_equal(g.raw, c.raw)


def test_c3_synthetic_gpu_jit():
    """Runtime-compiled walk kernel (forced on a small batch) against the oracle: bit-exact verdicts, paths,
    messages on the C3 corpus with edge cases."""
    st, res = S.run_synthetic("gpu", cases.best_practices() + cases.chart_restricted(), 3000, seed=41, jit=True)
    assert res.jit
    assert st["compared"] > 50000


def test_goldens_merged_gpu_jit():
    """Every engine / CLI / validate-walk golden policy against every golden resource, with the pattern walk in
    the runtime-compiled kernel (forced), bit-exact against the oracle."""
    st, res = S.run_merged("gpu", S.golden_groups(), "goldens-merged/jit", jit=True)
    assert res.jit
    assert st["compared"] > 1000


def test_goldens_merged_gpu_interpreter():
    st, res = S.run_merged("gpu", S.golden_groups(), "goldens-merged/interp", jit=False)
    assert not res.jit
    assert st["compared"] > 1000


def test_c4_policycache_stress_gpu():
    """configs[3]: the full 10,000 generated policies (match/exclude stress) over 2,000 mixed resources,
    every pair's status against the oracle's verdict matrix"""
    st, res = S.run_c4("gpu", 10000, 2000)
    assert st["rules"] >= 10000 and st["compared"] > 2e7


def test_c4_rule_slices_gpu(monkeypatch):
    """Rulesets whose walk buffers exceed the slice budget are evaluated in consecutive rule slices (kyv_engine.hip
    SliceSched); a tiny budget forces ~40 slices here: every pair's status, and every failing path / message of a
    sample, must equal the oracle and the single-slice evaluation"""
    import parity_util as PU
    monkeypatch.setenv("KYV_SLICE_MB", "16")
    pols = synth.c4_policies(10000)
    docs, nsl = synth.mixed(3000, seed=61, edge=True)
    st, res = PU.compare_matrix(pols, docs, nsl, backend="gpu", threads=_oracle_threads())
    assert st["nbad"] == 0, st["bad"]
    monkeypatch.delenv("KYV_SLICE_MB")
    rs = E.Ruleset(pols)
    b = E.Batch(rs, docs, nsl)
    one = E.evaluate(rs, b, backend="gpu")
    assert np.array_equal(one.raw, res.raw)
    fail = np.argwhere(one.status == K.ST_FAIL)
    rng = np.random.default_rng(1)
    for k, r in fail[rng.choice(len(fail), size=min(300, len(fail)), replace=False)]:
        assert one.path(int(r), int(k)) == res.path(int(r), int(k))
        assert one.message(int(r), int(k)) == res.message(int(r), int(k))


def test_c4_shape_tables_jit_gpu(monkeypatch):
    """configs[3] through the compiled kernels at a size the oracle checks in full: the 10,000 generated policies
    over 3,000 mixed resources with the kind-indexed match records and the pattern-shape tables (every distinct
    compiled pattern walked once per resource, matched pairs decided in the match phase): every pair's status and every
    FAIL pair's path and message against the oracle; then the same with ~40 rule slices (KYV_SLICE_MB=16), which must
    equal the one-slice evaluation byte for byte"""
    import parity_util as PU
    pols = synth.c4_policies(10000)
    docs, nsl = synth.mixed(3000, seed=63, edge=True)
    st, res = PU.compare_matrix(pols, docs, nsl, backend="gpu", jit=True, threads=_oracle_threads())
    assert st["nbad"] == 0, st["bad"]
    assert res.jit and res.jit_shapes
    assert st["matched"] > 100_000
    monkeypatch.setenv("KYV_SLICE_MB", "16")
    rs = E.Ruleset(pols)
    b = E.Batch(rs, docs, nsl)
    sl = E.evaluate(rs, b, backend="gpu", jit=True)
    assert sl.jit_shapes
    assert np.array_equal(sl.raw, res.raw)
    fail = np.argwhere(sl.status == K.ST_FAIL)
    rng = np.random.default_rng(2)
    for k, r in fail[rng.choice(len(fail), size=min(300, len(fail)), replace=False)]:
        assert sl.path(int(r), int(k)) == res.path(int(r), int(k))


def test_c4_at_scale_gpu():
    """configs[3] at scale: 10,000 generated policies (~10.4k compiled rules) over 100k mixed resources on one
    MI355X (buffers beyond the slice budget -> rule slices); the oracle (0.9 M pairs/s on C4) checks a spread
    sample of 1,500 resources of the batch, every rule"""
    import parity_util as PU
    pols = synth.c4_policies(10000)
    docs, nsl = synth.mixed(100_000, seed=62, edge=True)
    rs = E.Ruleset(pols)
    b = E.Batch(rs, docs, nsl)
    res = E.evaluate(rs, b, backend="gpu")
    assert res.jit  # the production walk at this size (timed by bench --workload c4)
    assert sum(res.counts.values()) == len(rs.rules) * b.n
    idx = np.linspace(0, b.n - 1, 1500).astype(int)
    st = PU.compare_status_sample(rs, res, pols, docs, nsl, idx, threads=_oracle_threads())
    assert st["nbad"] == 0, st["bad"]
    assert st["matched"] > 100_000
    assert st["texts"]["paths_compared"] > 1000


def test_condition_goldens_gpu():
    assert S.run_condition_goldens("gpu") >= 300


def test_c5_conditions_gpu():
    st, _ = S.run_synthetic("gpu", synth.c5_policies(50), 4000, seed=34)
    assert st["compared"] > 40000


_SCAN_RCCL = r"""
import os, sys
import numpy as np
import torch  # loaded before libkyvgpu: torch and the library share one HIP runtime (kyverno_amd/_lib.py)
import torch.distributed as dist
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tests")]
from kyverno_amd import scan as SC, synth
import test_scan as TS
pols = TS.policy_set()
docs, nsl = synth.mixed(20001, seed=44, edge=True)
g = SC.BackgroundScan(pols, backend="gpu").scan(docs, nsl)
c = SC.BackgroundScan(pols, backend="cpu").scan(docs, nsl)
st = g.res.status
for k in range(st.shape[0]):
    assert np.array_equal(np.bincount(st[k], minlength=8), g.res.rule_counts[k]), k
assert np.array_equal(g.summary_matrix(), c.summary_matrix())
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29531")
dist.init_process_group("nccl", rank=0, world_size=1)
try:
    tot = SC.reduce_summary(g.summary_matrix(), device=torch.device("cuda", 0))
finally:
    dist.destroy_process_group()
assert np.array_equal(tot, g.summary_matrix())
print("scan-rccl ok")
"""


def test_scan_summary_gpu_and_rccl():
    """batched background scan on the device: per-rule verdict totals (unaligned rule rows: 20,001 resources) equal
    the verdict bytes, the per-policy summary equals the host instantiation's, and the summary all-reduce runs over
    RCCL (single-rank "nccl" group). Runs in a fresh interpreter that loads torch before the library (one HIP
    runtime per process; this test process already loaded libkyvgpu on its own runtime)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, KYV_TORCH_FIRST="1")
    r = subprocess.run([sys.executable, "-c", _SCAN_RCCL], cwd=root, env=env, capture_output=True, text=True,
                       timeout=200)
    assert r.returncode == 0 and "scan-rccl ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


@pytest.mark.parametrize("jit", [False, True])
def test_pss_with_preconditions_gpu_equals_cpu(jit):
    """PodSecurity rules behind preconditions run eval_pss out of line from the match kernel (its column checks
    inlined there), the others pss_kernel: the round-3 wrong-mask case (C5 policy c5-006, baseline + preconditions)
    and its restricted / precondition-free variants, device verdict bytes and PSS masks == the host instantiation"""
    import copy
    data, nsl = synth.corpus_ndjson(20000, seed=54, edge=True)
    base = [p for p in synth.c5_policies(50) if p["metadata"]["name"] == "c5-006"]
    assert base and base[0]["spec"]["rules"][0].get("preconditions")
    nopre = copy.deepcopy(base)
    del nopre[0]["spec"]["rules"][0]["preconditions"]
    restr = copy.deepcopy(base)
    restr[0]["spec"]["rules"][0]["validate"]["podSecurity"]["level"] = "restricted"
    for pols in (base, nopre, restr, base + nopre + restr):
        rs = E.Ruleset(pols)
        b = E.Batch(rs, data, nsl)
        g = E.evaluate(rs, b, backend="gpu", jit=jit)
        c = E.evaluate(rs, b, backend="cpu")
        assert np.array_equal(g.raw, c.raw)
        nfail = 0
        for k, r in enumerate(rs.rules):
            if r["kind"] != "podSecurity":
                continue
            fails = np.nonzero(np.asarray(g.status[k]) == K.ST_FAIL)[0]
            nfail += len(fails)
            for i in fails[:: max(1, len(fails) // 200)].tolist():
                assert g.pss_mask(i, k) == c.pss_mask(i, k), (r["name"], i)
        assert nfail > 0


def _pss_excl_policies():
    """PodSecurity rules whose exclusions send pairs to pss_map_kernel (eval_pss's map walk over exclusion sub-pods):
    the exclusion shapes of pkg/pss/evaluate_test.go (control-only, and control + images matching init, regular and
    ephemeral containers) on baseline and restricted, pinned and latest versions (pkg/pss/evaluate.go:16-60,83-108)"""
    def pol(name, level, version, excl, kinds=("Pod",)):
        return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
                "spec": {"rules": [{"name": name, "match": {"any": [{"resources": {"kinds": list(kinds)}}]},
                                    "validate": {"podSecurity": {"level": level, "version": version, "exclude": excl}}}]}}
    team1 = ["registry.example.com/team1*"]
    return [
        pol("bl-caps-img", "baseline", "latest", [{"controlName": "Capabilities", "images": team1}]),
        pol("bl-ctl", "baseline", "v1.24", [{"controlName": "Host Namespaces"}, {"controlName": "HostPath Volumes"},
                                            {"controlName": "Host Ports", "images": ["*:latest"]}]),
        pol("bl-mixed", "baseline", "latest", [{"controlName": "Privileged Containers", "images": ["*"]},
                                               {"controlName": "SELinux", "images": ["registry.example.com/team2?/*"]},
                                               {"controlName": "Seccomp"}, {"controlName": "AppArmor"},
                                               {"controlName": "/proc Mount Type", "images": team1}]),
        pol("rs-img", "restricted", "latest", [{"controlName": "Running as Non-root", "images": team1},
                                               {"controlName": "Privilege Escalation", "images": ["*:1.*"]},
                                               {"controlName": "Capabilities", "images": ["registry.example.com/team3*"]}]),
        pol("rs-ctl", "restricted", "v1.24", [{"controlName": "Volume Types"}, {"controlName": "Running as Non-root user"},
                                              {"controlName": "Seccomp", "images": ["*"]}]),
        pol("rs-wl", "restricted", "latest", [{"controlName": "Running as Non-root user", "images": team1},
                                              {"controlName": "Privilege Escalation"}],
            kinds=("Pod", "Deployment", "StatefulSet", "Job", "CronJob")),
    ]


# kyv_pss.h PssSlot order (pss_msg.cpp kSlots): the check id of each bit of a PodSecurity failure mask
_PSS_SLOT_IDS = ["allowPrivilegeEscalation", "allowPrivilegeEscalation", "appArmorProfile", "capabilities_baseline",
                 "capabilities_restricted", "capabilities_restricted", "hostNamespaces", "hostPathVolumes", "hostPorts",
                 "privileged", "procMount", "restrictedVolumes", "runAsNonRoot", "runAsUser", "seLinuxOptions",
                 "seccompProfile_baseline", "seccompProfile_baseline", "seccompProfile_restricted",
                 "seccompProfile_restricted", "sysctls", "windowsHostProcess"]


def test_pss_map_kernel_exclusions_at_scale_gpu():
    """pss_map_kernel at scale (round-6 item: the map-form checks, pss_checks, use integer flag words like the column
    form): 200k pods x six PodSecurity rules with exclusions against the oracle's verdict matrix; every FAIL pair's
    check mask against the host instantiation of the same evaluator, and a sample of 20k FAIL pairs' failed-check sets
    against the oracle's EvaluatePod (exclusion rules have no rendered message: exemptKyvernoExclusion orders its
    checks by Go map iteration, evaluate.go:39-60)"""
    import json
    import parity_util as PU
    from oracle import oracle as O
    pols = _pss_excl_policies()
    data, nsl = synth.corpus_ndjson(200_000, kind="pods", seed=61, edge=True)
    st, res = PU.compare_matrix(pols, data, nsl, backend="gpu", threads=_oracle_threads(), texts=False)
    assert st["nbad"] == 0, st["bad"]
    assert st["matched"] >= 6 * 200_000
    assert res.counts["fail"] > 100_000 and res.counts["pass"] > 0
    rs = E.Ruleset(pols)
    b = E.Batch(rs, data, nsl)
    g = E.evaluate(rs, b, backend="gpu")
    c = E.evaluate(rs, b, backend="cpu")
    assert np.array_equal(g.raw, c.raw)
    lines = [x for x in data.split(b"\n") if x.strip()]
    rng = np.random.default_rng(6)
    nmask, noracle = 0, 0
    for k, r in enumerate(rs.rules):
        assert r["kind"] == "podSecurity"
        pname = rs.policies[r["policy"]]["name"]
        psr = [p for p in pols if p["metadata"]["name"] == pname][0]["spec"]["rules"][0]["validate"]["podSecurity"]
        fails = np.nonzero(np.asarray(g.status[k]) == K.ST_FAIL)[0]
        for i in fails.tolist():
            assert g.pss_mask(i, k) == c.pss_mask(i, k), (r["name"], i)
        nmask += len(fails)
        for i in rng.choice(fails, size=min(len(fails), 4000), replace=False).tolist() if len(fails) else []:
            m = g.pss_mask(i, k)
            got = {_PSS_SLOT_IDS[s] for s in range(len(_PSS_SLOT_IDS)) if (m >> s) & 1}
            want = {x["id"] for x in O.pss(psr, json.loads(lines[i]))["checks"]}
            assert got == want, (r["name"], i, sorted(got), sorted(want))
            noracle += 1
    assert nmask > 100_000 and noracle >= 20_000


def test_exclude_all_nondeterminism_in_kind_folded_records_gpu():
    """An exclude.all block whose later filter can never accept the wave's kind: the match records folded per kind
    class (kyv_engine.hip fold_kinds) keep the block when a filter ahead of it has a selector, so the nondeterminism
    that filter raises (a wildcard selector key matching a valid and an invalid label: Go map order decides,
    pkg/utils/wildcards/wildcards.go:13-50) is the reference's in single-kind waves too. The mirrored order (the
    never-accepting filter first) still drops the block."""
    def pol(name, excl):
        return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy",
                "metadata": {"name": name, "annotations": {"pod-policies.kyverno.io/autogen-controllers": "none"}},
                "spec": {"rules": [{"name": "r", "match": {"any": [{"resources": {"kinds": ["Pod", "Deployment"]}}]},
                                    "exclude": {"all": excl},
                                    "validate": {"message": "m", "pattern": {"metadata": {"name": "?*"}}}}]}}
    sel = {"matchLabels": {"app-*": "x*"}}
    pols = [pol("nd-excl-all", [{"resources": {"kinds": ["Pod"], "selector": sel}}, {"resources": {"kinds": ["Deployment"]}}]),
            pol("nd-excl-all2", [{"resources": {"kinds": ["Deployment"]}}, {"resources": {"kinds": ["Pod"], "selector": sel}}])]
    docs = []
    for i in range(256):  # pods only: every wave is one kind class (folded records)
        labels = [{"app-a": "x1", "app-b": "x!!"}, {"app-a": "x1"}, {"app-a": "y", "app-b": "x2"}, {}][i % 4]
        docs.append({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p%d" % i, "namespace": "default", "labels": labels},
                     "spec": {"containers": [{"name": "c", "image": "x"}]}})
    import parity_util as PU
    st, res = PU.compare(pols, docs, {}, backend="gpu")
    assert st["nbad"] == 0, st["bad"]
    assert st["nd"] == 64, st
