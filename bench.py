"""Throughput bench for the validate hot path: resource x rule evaluations per second on MI355X.

Workload (BASELINE.json configs[2] at weak scaling, SURVEY.md §8(d) "C3"): the charts/kyverno-policies
restricted set + the test/best_practices validate policies (select-secrets excluded, as §8(d) does: it reads
variables), autogen applied (every compiled rule counts: 89), over a seeded synthetic mixed-kind corpus, 1.25M
resources per GPU (10M at 8 GPUs). One "step" = one evaluation of every (resource, compiled rule) pair of the rank's
shard with the batch resident in HBM.

  python bench.py [--gpus N --steps K --warmup W] [--workload c3|c2|c4|c5] [--resources R]

--gpus N > 1 without an external launcher: this script starts N rank processes itself (before any GPU call) and
exits with the worst rank's code; under torch.distributed.run it is one rank. Every rank evaluates its own shard
(no data-path collective; the barrier and the max-over-ranks timing use a gloo group) -> "scaling": "weak".
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "resource×rule evals/sec (background scan, PSS+best-practices) at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); ~6300 GB/s measured streaming copy
SEED = 0x4B59564E
CPU_STATUSES = ("fallback", "panic", "nondeterministic")  # pairs the device hands to the CPU engine


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def load_policies(workload):
    gdir = os.path.join(ROOT, "tests", "golden")
    if workload == "c2":
        return [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "psa"},
                 "spec": {"background": True, "validationFailureAction": "Audit",
                          "rules": [{"name": "restricted", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                                     "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}}]}}]
    if workload == "c4":
        from kyverno_amd import synth
        return synth.c4_policies(10000)
    if workload == "c5":
        from kyverno_amd import synth
        return synth.c5_policies(50)
    out = []
    for f in ("chart_restricted.json", "best_practices.json"):
        with open(os.path.join(gdir, f)) as fh:
            out += [r["policy"] for r in json.load(fh)
                    if r["policy"]["metadata"]["name"] != "select-secrets"]  # variables
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """--gpus N without a launcher: start N rank processes (no GPU call has happened in this parent) and exit with
    the worst rank's code; rank 0 prints the JSON line."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    sys.exit(rc)


def dist_setup(gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (gpus, world))
    pg = None
    if world > 1:
        import torch.distributed as dist  # host-side group only: barrier + max-over-ranks timing
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pg = dist
    return rank, world, local, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


def all_max(pg, x):
    if pg is None:
        return x
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def all_sum(pg, x):
    if pg is None:
        return x
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return float(t.item())


# oracle matrix code -> device status (oracle/ocapi.cpp oracle_validate_matrix; kyvgpu.h KYV_ST_*)
_MATRIX_TO_DEVICE = (0, 1, 2, 3, 4, 6, 5, 7)


def cpu_baseline_and_parity(policies, rs, data, nsl, target_s=10.0, cap=400000, device=0):
    """CPU baseline: the oracle (CPU restatement of engine.Validate, oracle/) over a bounded prefix of this rank's
    corpus, growing until one timed pass takes >= target_s; then the device evaluates the same prefix (its own
    batch) and every (resource, rule) verdict is compared with the oracle's."""
    import numpy as np
    from oracle import oracle as O
    from kyverno_amd import engine as E
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)))
    lines = data.split(b"\n", cap)[:cap]
    want = 512
    while True:
        sample = b"[" + b",".join(lines[:want]) + b"]"
        names, m, secs = O.validate_matrix(policies, sample, nsl, threads=threads, nres=want, timed=True)
        if secs >= target_s or want >= len(lines):
            break
        want = min(len(lines), int(want * min(16.0, max(2.0, 1.2 * target_s / max(secs, 1e-3)))))
    npairs = len(names) * want
    cpu = {"value": npairs / secs, "unit": "resource×rule evals/sec", "cores": threads, "kind": "port",
           "sample": "%d resources x %d compiled rules (first resources of the rank-0 corpus), %.1f s, oracle/ "
                     "tree-walk restatement of engine.Validate, %d threads" % (want, len(names), secs, threads)}
    # parity on the same prefix: device verdict matrix vs the oracle's, pair by pair
    b = E.Batch(rs, b"\n".join(lines[:want]), nsl)
    res = E.evaluate(rs, b, backend="gpu", device=device)
    row = {nm: i for i, nm in enumerate(names)}
    lut = np.array(_MATRIX_TO_DEVICE, dtype=np.uint8)
    st = np.asarray(res.status)
    compared = mism = nd = 0
    first = None
    for k, rule in enumerate(rs.rules):
        key = (rs.policies[rule["policy"]]["name"], rule["name"])
        exp = lut[m[row[key]]] if key in row else np.zeros(want, np.uint8)
        got = st[k]
        ndm = (exp == 7) | (got == 7)
        nd += int(ndm.sum())
        bad = np.nonzero((exp != got) & ~ndm)[0]
        compared += want - int(ndm.sum())
        mism += len(bad)
        if len(bad) and first is None:
            first = {"rule": list(key), "resource": int(bad[0]), "device": int(got[bad[0]]), "oracle": int(exp[bad[0]])}
    parity = {"status": "ok" if mism == 0 else "mismatch", "resources": want, "pairs_compared": compared,
              "mismatches": mism, "nondeterministic_pairs": nd, "first_mismatch": first,
              "jit": bool(res.jit)}
    return cpu, parity


def pmc_traffic(config):
    """HBM-side bytes per launch of the dominant kernel from the newest committed PMC summary
    (profiles/pmc_latest.json, written by scripts/pmc_summary.py from separate rocprofv3 --pmc passes of this
    same command), used only when it was measured on the same workload configuration; else None."""
    f = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(f):
        return None, None
    with open(f) as fh:
        s = json.load(fh)
    bc = s.get("bench_config") or {}
    keys = ("workload", "resources_per_gpu", "compiled_rules")
    if any(bc.get(k) != config.get(k) for k in keys):
        return None, s.get("tag")
    return s.get("traffic_bytes"), s.get("tag")


def fallback_by_reason(rs, res):
    """CPU-handed pairs per reason: the rule's compile-time reason, or "run-time" for pairs of device rules"""
    out = {}
    for k, r in enumerate(rs.rules):
        n = int(sum(res.rule_counts[k][s] for s in (5, 6, 7)))
        if n:
            why = r["reason"] if r["kind"] == "fallback" else "run-time (value / walk outside the device subset)"
            out[why] = out.get(why, 0) + n
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=["c3", "c2", "c4", "c5"])
    ap.add_argument("--resources", type=int, default=0, help="resources per GPU (default 1.25M c3 / 1M c2 / c4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (flatten + H2D + eval + D2H) leg")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(args.gpus)

    from kyverno_amd import engine as E
    from kyverno_amd import synth

    rank, world, local, pg = dist_setup(args.gpus)
    nper = args.resources or (1_250_000 if args.workload == "c3" else 1_000_000)
    kind = "pods" if args.workload in ("c2", "c5") else "mixed"
    policies = load_policies(args.workload)

    t0 = time.time()
    data, nsl = synth.cached_corpus(nper, kind=kind, seed=SEED + rank)
    t_gen = time.time() - t0
    log("rank %d: generated %d resources (%.1f MB) in %.1f s" % (rank, nper, len(data) / 1e6, t_gen))
    t0 = time.time()
    rs = E.Ruleset(policies)
    t_compile = time.time() - t0
    nrules = len(rs.rules)
    t0 = time.time()
    batch = E.Batch(rs, data, nsl)
    t_flat = time.time() - t0
    log("rank %d: flattened %d resources into %d node rows in %.1f s" % (rank, batch.n, batch.stats()["nodes"], t_flat))
    pairs = nrules * batch.n

    # algorithmic bytes per eval: CPU accounting over a sample of this shard
    sample_n = min(batch.n, 20000)
    sb = E.Batch(rs, b"\n".join(data.split(b"\n", sample_n)[:sample_n]), nsl)
    acct = E.evaluate(rs, sb, backend="cpu", account_bytes=True)
    bytes_per_eval = acct.alg_bytes / max(1, nrules * sb.n)
    del sb, acct
    log("rank %d: %.1f algorithmic bytes per eval (CPU accounting over %d resources)" % (rank, bytes_per_eval, sample_n))

    # warmup (first call uploads the batch, loads / compiles the walk kernel, allocates the resident buffers)
    t0 = time.time()
    first = E.evaluate(rs, batch, backend="gpu", device=local, copy_back=False)
    t_upload = time.time() - t0
    counts = first.counts
    fb_reasons = fallback_by_reason(rs, first)
    log("rank %d: first GPU evaluation (incl. upload) %.2f s, kernel %.2f ms" % (rank, t_upload, first.kernel_ms))
    del first
    for _ in range(max(0, args.warmup - 1)):
        E.evaluate(rs, batch, backend="gpu", device=local, copy_back=False)

    barrier(pg)
    t0 = time.perf_counter()
    kms = 0.0
    for _ in range(args.steps):
        r = E.evaluate(rs, batch, backend="gpu", device=local, copy_back=False)
        kms += r.kernel_ms
    barrier(pg)
    dt = time.perf_counter() - t0
    dt_max = all_max(pg, dt)
    kernel_ms = kms / max(1, args.steps)
    kernel_ms_max = all_max(pg, kernel_ms)
    # pairs the device decided: every (resource, compiled rule) pair except those it hands to the CPU engine
    # (FALLBACK / PANIC / ND: rules or pairs outside the GPU subset, counted separately, not in `value`)
    cpu_pairs = int(sum(counts.get(s, 0) for s in CPU_STATUSES))
    dev_pairs = pairs - cpu_pairs
    total_pairs = all_sum(pg, dev_pairs)
    total_fb = all_sum(pg, cpu_pairs)

    # end to end on this rank: JSON -> flatten -> H2D -> evaluate -> D2H of every verdict (walk kernel already loaded)
    e2e = None
    if not args.no_e2e:
        t0 = time.time()
        b2 = E.Batch(rs, data, nsl)
        t1 = time.time()
        r2 = E.evaluate(rs, b2, backend="gpu", device=local, copy_back=True)
        t2 = time.time()
        e2e = {"pairs_per_s": (pairs - int(sum(r2.counts.get(s, 0) for s in CPU_STATUSES))) / (t2 - t0),
               "seconds": t2 - t0, "flatten_s": t1 - t0, "upload_eval_copyback_s": t2 - t1,
               "flatten_resources_per_s": b2.n / max(t1 - t0, 1e-9),
               "flatten_threads": os.cpu_count()}
        del r2, b2

    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline_and_parity(policies, rs, data, nsl, device=local)
        log("rank 0: parity on the cpu_baseline prefix: %s (%d pairs, %d mismatches)" %
            (parity["status"], parity["pairs_compared"], parity["mismatches"]))

    if rank == 0:
        alg_bytes_launch = bytes_per_eval * dev_pairs
        achieved = alg_bytes_launch / (kernel_ms / 1e3) / 1e9
        wl = {"c3": "C3: charts/kyverno-policies restricted + test/best_practices validate policies (select-secrets "
                    "excluded, SURVEY §8(d); %d compiled rules) over %d mixed resources per GPU",
              "c2": "C2: podSecurity restricted/latest (%d compiled rules) over %d pods per GPU",
              "c4": "C4: 10,000 generated policies, wildcard match/exclude stress (%d compiled rules) over %d mixed "
                    "resources per GPU",
              "c5": "C5: 50 generated precondition / deny policies with variables (%d compiled rules) over %d pods "
                    "per GPU"}[args.workload] % (nrules, batch.n)
        config = {"workload": wl, "resources_per_gpu": batch.n, "compiled_rules": nrules,
                  "pairs_per_step": int(total_pairs), "cpu_fallback_pairs_per_step": int(total_fb),
                  "parallelism": "shard%d" % world}
        traffic, pmc_tag = pmc_traffic(config)
        line = {
            "metric": METRIC,
            "value": total_pairs * args.steps / dt_max,
            "unit": "resource×rule evals/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max * 1e3 / max(1, args.steps),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded generator kyverno_amd/synth.py, SURVEY §8(d) model; seed 0x4b59564e + rank)",
            "config": config,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "counter_frac": (traffic / (kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                         "traffic_source": "profiles/%s_summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, bytes "
                                           "per launch)" % pmc_tag if traffic else None,
                         "bytes_per_eval": bytes_per_eval,
                         "achieved_basis": "bytes_per_eval x device-decided pairs (CPU-handed pairs excluded) / "
                                           "evaluation time (HIP events)",
                         "kernel": "one evaluation: match_kernel + walk kernels (kyv_jit_walk) + record compaction",
                         "kernel_ms": kernel_ms,
                         "kernel_ms_max_rank": kernel_ms_max},
            "cpu_baseline": cpu,
            "parity_prefix": parity,
            "verdicts": {k: v for k, v in counts.items()},
            "cpu_fallback_by_reason": fb_reasons,
            "host": {"generate_s": t_gen, "compile_s": t_compile, "flatten_s": t_flat,
                     "flatten_resources_per_s": batch.n / max(t_flat, 1e-9),
                     "first_eval_incl_upload_s": t_upload, "batch_device_bytes": batch.stats()["device_bytes"],
                     "e2e": e2e},
        }
        print(json.dumps(line), flush=True)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
