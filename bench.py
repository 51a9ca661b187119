"""Throughput bench for the validate hot path: resource x rule evaluations per second on MI355X.

Workload (BASELINE.json configs[2] at weak scaling, SURVEY.md §8(d) "C3"): the charts/kyverno-policies
restricted set + test/best_practices validate policies (autogen applied: every compiled rule counts) over a
seeded synthetic mixed-kind corpus, 1.25M resources per GPU (10M at 8 GPUs). One "step" = one evaluation
of every (resource, compiled rule) pair of the rank's shard with the batch resident in HBM (one kernel launch).

  python bench.py [--gpus N --steps K --warmup W] [--workload c3|c2] [--resources R]

For N>1 the driver launches one process per GPU (torch.distributed.run); every rank evaluates its own shard
(no data-path collective; the barrier and the max-over-ranks timing use a gloo group) -> "scaling": "weak".
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "resource×rule evals/sec (background scan, PSS+best-practices) at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); ~6300 GB/s measured streaming copy
SEED = 0x4B59564E


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def load_policies(workload):
    gdir = os.path.join(ROOT, "tests", "golden")
    if workload == "c2":
        return [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "psa"},
                 "spec": {"background": True, "validationFailureAction": "Audit",
                          "rules": [{"name": "restricted", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                                     "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}}]}}]
    out = []
    for f in ("chart_restricted.json", "best_practices.json"):
        with open(os.path.join(gdir, f)) as fh:
            out += [r["policy"] for r in json.load(fh)]
    return out


def dist_setup(gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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


def cpu_baseline(policies, data, nsl, nrules, target_s=10.0):
    """Oracle (CPU restatement of engine.Validate) on a bounded prefix of this rank's corpus: the prefix grows
    until one timed pass takes >= target_s (or the prefix cap is reached)."""
    from oracle import oracle as O
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)))
    lines = data.split(b"\n", 400000)[:400000]
    want = 512
    while True:
        sample = b"[" + b",".join(lines[:want]) + b"]"
        n, _, secs = O.validate_batch(policies, sample, nsl, threads)
        if secs >= target_s or want >= len(lines):
            break
        want = min(len(lines), int(want * min(16.0, max(2.0, 1.2 * target_s / max(secs, 1e-3)))))
    return {"value": n / secs, "unit": "resource×rule evals/sec", "cores": threads, "kind": "port",
            "sample": "%d resources x %d compiled rules (first resources of the rank-0 corpus), %.1f s, oracle/ "
                      "tree-walk restatement of engine.Validate, %d threads" % (want, nrules, secs, threads)}


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=["c3", "c2"])
    ap.add_argument("--resources", type=int, default=0, help="resources per GPU (default 1.25M c3 / 1M c2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    from kyverno_amd import engine as E
    from kyverno_amd import synth

    rank, world, local, pg = dist_setup(args.gpus)
    nper = args.resources or (1_250_000 if args.workload == "c3" else 1_000_000)
    kind = "mixed" if args.workload == "c3" else "pods"
    policies = load_policies(args.workload)

    t0 = time.time()
    data, nsl = synth.cached_corpus(nper, kind=kind, seed=SEED + rank)
    t_gen = time.time() - t0
    log("rank %d: generated %d resources (%.1f MB) in %.1f s" % (rank, nper, len(data) / 1e6, t_gen))
    rs = E.Ruleset(policies)
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

    # warmup (first call uploads the batch and allocates the resident result buffers)
    t0 = time.time()
    first = E.evaluate(rs, batch, backend="gpu", device=local, copy_back=False)
    t_upload = time.time() - t0
    counts = first.counts
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
    # (ST_FALLBACK: rules / pairs outside the GPU subset, counted separately, not in `value`)
    fb_pairs = int(counts.get("fallback", 0))
    total_pairs = all_sum(pg, pairs - fb_pairs)
    total_fb = all_sum(pg, fb_pairs)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(policies, data, nsl, nrules)

    if rank == 0:
        alg_bytes_launch = bytes_per_eval * pairs
        achieved = alg_bytes_launch / (kernel_ms / 1e3) / 1e9
        config = {"workload": "C3: charts/kyverno-policies restricted + test/best_practices (%d compiled rules) "
                              "over %d mixed resources per GPU" % (nrules, batch.n) if args.workload == "c3" else
                              "C2: podSecurity restricted/latest (%d compiled rules) over %d pods per GPU" %
                              (nrules, batch.n),
                  "resources_per_gpu": batch.n, "compiled_rules": nrules, "pairs_per_step": int(total_pairs),
                  "cpu_fallback_pairs_per_step": int(total_fb),
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
                         "traffic_source": "profiles/%s_summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, bytes "
                                           "per launch)" % pmc_tag if traffic else None,
                         "bytes_per_eval": bytes_per_eval,
                         "kernel": "one evaluation: match_kernel + walk kernels (kyv_jit_walk) + record compaction",
                         "kernel_ms": kernel_ms,
                         "kernel_ms_max_rank": kernel_ms_max},
            "cpu_baseline": cpu,
            "verdicts": {k: v for k, v in counts.items()},
            "host": {"generate_s": t_gen, "flatten_s": t_flat, "flatten_resources_per_s": batch.n / max(t_flat, 1e-9),
                     "first_eval_incl_upload_s": t_upload, "batch_device_bytes": batch.stats()["device_bytes"]},
        }
        print(json.dumps(line), flush=True)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
