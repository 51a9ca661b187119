"""Throughput bench for the validate hot path: resource x rule evaluations per second on MI355X.

Workload (BASELINE.json configs[2], SURVEY.md §8(d) "C3"): the charts/kyverno-policies restricted set + the
test/best_practices validate policies (select-secrets excluded, as §8(d) does: it reads variables), autogen applied
(every compiled rule counts: 89), over ONE seeded synthetic mixed-kind corpus of 10M resources -- the configuration
the metric is quoted on. With N GPUs each rank evaluates a contiguous 10M/N shard of that same corpus (strong
scaling; the corpus bytes do not depend on N). One "step" = one evaluation of every (resource, compiled rule) pair of
the rank's shard with the batch resident in HBM.

  python bench.py [--gpus N --steps K --warmup W] [--workload c3|c2|c4|c5] [--resources TOTAL]

--gpus N > 1 without an external launcher: this script starts N rank processes itself (before any GPU call) and
exits with the worst rank's code; under torch.distributed.run it is one rank. Every rank evaluates its own shard
(no data-path collective; the barrier and the max-over-ranks timing use a gloo group).
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


def all_gather_obj(pg, obj):
    if pg is None:
        return [obj]
    out = [None] * pg.get_world_size()
    pg.all_gather_object(out, obj)
    return out


def time_gathers(batch, local, rank, world):
    """Report assembly over the device-resident results of the last timed evaluation: RCCL
    all-gather of every rank's packed verdicts (scan.gather_verdicts_device) and count-then-gather of its failing-path
    rows (scan.gather_failures_device; a rule-sliced shard keeps no resident rows and reports so), each timed on its
    own after a warm-up call, max over ranks. At world size 1 the same calls run over a one-rank RCCL group."""
    import torch
    import torch.distributed as dist
    from kyverno_amd import scan
    from kyverno_amd import _lib as K
    torch.cuda.set_device(local)
    dev = "cuda:%d" % local
    if not dist.is_initialized():  # N = 1: a one-rank group, so the same RCCL path runs
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(dev))
        g, own = None, True
    else:
        g, own = dist.new_group(backend="nccl"), False
    out = {"backend": "nccl (RCCL)", "world": world}
    try:
        def timed(fn):
            fn()  # warm-up (communicator setup)
            torch.cuda.synchronize()
            dist.barrier(group=g)
            t0 = time.perf_counter()
            r = fn()
            torch.cuda.synchronize()
            dist.barrier(group=g)
            return r, time.perf_counter() - t0
        full, tv = timed(lambda: scan.gather_verdicts_device(batch, group=g, device=dev, tensor=True)[0])
        out["verdicts_ms"] = tv * 1e3
        out["verdict_matrix"] = list(full.shape)
        out["verdict_wire_bytes"] = int(full.shape[0]) * ((int(full.shape[1]) + 1) // 2)
        del full
        try:
            rows, tf = timed(lambda: scan.gather_failures_device(batch, 0, group=g, device=dev, tensor=True))
            out["failures_ms"] = tf * 1e3
            out["failure_rows"] = int(rows.shape[0])
            del rows
        except K.KyvError as e:
            out["failures"] = "not resident: %s" % str(e)[:160]
        torch.cuda.empty_cache()
    finally:
        if own:
            dist.destroy_process_group()
    return out


def native_gathers(batch, local, rank, world, pg, res_offset, own_counts=None):
    """Report assembly over the device-resident results of the last timed evaluation with the
    library's own RCCL communicator (kyv_comm_*; no torch in the process): every rank's packed verdicts and its
    failing-path rows (16 B each) sent to rank 0, the report's consumer (kyv_comm_gather_report), and the per-rule
    verdict tallies all-reduced (kyv_comm_reduce_counts); each timed after a warm-up, max over ranks. Checked: the
    root's copy of every rank's verdicts has the checksum its owner computed, every rank's row count arrived, and the
    reduced tallies equal the sum of the ranks' own."""
    import zlib
    import numpy as np
    from kyverno_amd import scan
    uid = scan.Comm.unique_id() if rank == 0 else None
    if pg is not None:
        box = [uid]
        pg.broadcast_object_list(box, src=0)
        uid = box[0]
    comm = scan.Comm(uid, world, rank, local)
    try:
        comm.gather_report(batch, res_offset, root=0)  # warm-up: communicator setup, buffers
        barrier(pg)
        t0 = time.perf_counter()
        st = comm.gather_report(batch, res_offset, root=0)
        wall = time.perf_counter() - t0
        barrier(pg)
        t1 = time.perf_counter()
        tot = comm.reduce_counts(batch)
        reduce_ms = (time.perf_counter() - t1) * 1e3
        own = scan.pack_status(batch.resident_status(device=local))
        mine = None if own_counts is None else np.asarray(own_counts)
        owners = all_gather_obj(pg, (rank, zlib.crc32(own.tobytes()), int(own.size),
                                     None if mine is None else mine.tolist()))
        seen_ok = True
        if rank == 0:
            seen_ok = all(zlib.crc32(comm.status_of(q)[:n].tobytes()) == c for q, c, n, _ in owners)
        sum_ok = None
        if all(m is not None for *_, m in owners):
            sum_ok = bool(np.array_equal(tot, np.sum([np.asarray(m) for *_, m in owners], axis=0)))
        rows_seen = int(st["failure_rows_total"])
    finally:
        comm.close()
    return {"backend": "RCCL (kyv_comm, library-owned communicator): verdicts + 16-B failing-path rows to rank 0, "
                       "tallies all-reduced", "world": world,
            "verdicts_ms": st["status_ms"], "failures_ms": st["failures_ms"], "wall_ms": wall * 1e3,
            "reduce_counts_ms": reduce_ms,
            "verdict_wire_bytes_per_rank": st["status_bytes_per_rank"], "failure_rows_total": rows_seen,
            "failure_row_wire_bytes": 16 * rows_seen,
            "failure_rows_per_rank_max": st["failure_rows_per_rank_max"], "segments_ok": bool(seen_ok),
            "rows_complete": st["failures_ms"] >= 0, "counts_sum_ok": sum_ok}


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


def host_cpus():
    """The host CPUs this job may use, and what the machine has: nproc (os.cpu_count), the affinity mask, a cgroup v2
    CPU quota, the CPU model, and the job's CPU share (OMP_NUM_THREADS, set by the GPU pool to the per-GPU share of
    the host; else affinity bounded by the quota)."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = -(-int(q) // int(per))
    except (OSError, ValueError):
        pass
    info["cgroup_quota"] = quota
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    info["model"] = model
    usable = info["affinity"] or 1
    if quota:
        usable = min(usable, quota)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    info["share"] = omp if omp > 0 else usable
    info["share_source"] = "OMP_NUM_THREADS (the pool's per-GPU CPU share)" if omp > 0 else \
        "affinity mask bounded by the cgroup quota"
    return info


def _lut():
    import numpy as np
    return np.array(_MATRIX_TO_DEVICE, dtype=np.uint8)


def compare_verdicts(rs, names, m, st, n):
    """device verdict rows st [rules, >= n] (input order) vs the oracle matrix m over the same n resources; a pair is
    excluded only when BOTH sides say ND (a one-sided ND is a mismatch)"""
    import numpy as np
    row = {nm: i for i, nm in enumerate(names)}
    lut = _lut()
    compared = mism = nd = 0
    first = None
    for k, rule in enumerate(rs.rules):
        key = (rs.policies[rule["policy"]]["name"], rule["name"])
        exp = lut[m[row[key]]] if key in row else np.zeros(n, np.uint8)
        got = np.asarray(st[k, :n]) & 7
        ndm = (exp == 7) & (got == 7)
        nd += int(ndm.sum())
        bad = np.nonzero(exp != got)[0]
        compared += n - int(ndm.sum())
        mism += len(bad)
        if len(bad) and first is None:
            first = {"rule": list(key), "resource": int(bad[0]), "device": int(got[bad[0]]), "oracle": int(exp[bad[0]])}
    return {"resources": n, "pairs_compared": compared, "mismatches": mism, "nondeterministic_pairs_both": nd,
            "first_mismatch": first}


def timed_prefix_status(batch, device, cap):
    """the timed evaluation's OWN verdicts for the first `cap` input-order resources of the batch (resident on the
    device after the last timed step: kind-major order and every rule slice included), copied back for parity"""
    return batch.resident_status(device=device, res0=0, nres=min(cap, batch.n))


def cpu_baseline_and_parity(policies, rs, data, nsl, jit, timed_status, target_s=10.0, cap=400000, device=0):
    """CPU baseline: the oracle (CPU restatement of engine.Validate, oracle/) over a bounded prefix of this rank's
    corpus on the job's whole CPU share, growing until one timed pass takes >= target_s, plus a single-thread pass
    over a smaller prefix. Parity, two legs over the same prefix:
      timed_batch  the verdicts the timed evaluation itself left on the device (timed_status: first resources of the
                   timed batch in input order -- its kind-major layout and rule slices included) vs the oracle's;
      texts        the failing path and RuleResponse.Message of every FAIL pair, from a device evaluation of the
                   prefix as its own batch (the walk kernel the timed region ran: jit), whose verdicts are also
                   compared pair by pair."""
    from oracle import oracle as O
    from kyverno_amd import engine as E
    hc = host_cpus()
    threads = max(1, hc["share"])
    lines = [x for x in data.split(b"\n", cap)[:cap] if x.strip()]
    want = min(512, len(lines))
    while True:
        sample = b"[" + b",".join(lines[:want]) + b"]"
        names, m, secs, tx = O.validate_matrix(policies, sample, nsl, threads=threads, nres=want, timed=True,
                                               texts=("fail",))
        if secs >= target_s or want >= len(lines):
            break
        want = min(len(lines), int(want * min(16.0, max(2.0, 1.2 * target_s / max(secs, 1e-3)))))
    npairs = len(names) * want
    # single thread, ~target_s / 3 of CPU work
    one_n = max(256, min(want, int(want * (target_s / 3) / max(secs * threads, 1e-3))))
    _, _, one_secs = O.validate_matrix(policies, b"[" + b",".join(lines[:one_n]) + b"]", nsl, threads=1, nres=one_n,
                                       timed=True)
    single = len(names) * one_n / one_secs
    cpu = {"value": npairs / secs, "unit": "resource×rule evals/sec", "cores": threads, "kind": "port",
           "sample": "%d resources x %d compiled rules (first resources of the rank-0 shard), %.1f s, oracle/ "
                     "tree-walk restatement of engine.Validate (C++, std::thread), %d threads = the job's CPU share"
                     % (want, len(names), secs, threads),
           "single_thread": single, "single_thread_sample": "%d resources, %.1f s" % (one_n, one_secs),
           "scaling_vs_single": (npairs / secs) / single,
           "nproc": hc["nproc"], "affinity_cpus": hc["affinity"], "cgroup_cpu_quota": hc["cgroup_quota"],
           "model": hc["model"], "threads_source": hc["share_source"],
           "reference_go_engine": "unavailable offline (no Go toolchain or module cache; SURVEY §8(c)/(d))"}
    # leg 1: the timed batch's own verdicts
    nt = min(want, timed_status.shape[1]) if timed_status is not None else 0
    timed = compare_verdicts(rs, names, m, timed_status, nt) if nt else None
    # leg 2: the prefix as its own batch, pair by pair, then every FAIL pair's texts
    b = E.Batch(rs, b"\n".join(lines[:want]), nsl)
    res = E.evaluate(rs, b, backend="gpu", device=device, jit=jit)
    sep = compare_verdicts(rs, names, m, res.status, want)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import parity_util as PU
    ts = PU.compare_fail_texts(rs, res, names, tx, want)
    ok = sep["mismatches"] == 0 and ts["nbad"] == 0 and (timed is None or timed["mismatches"] == 0)
    parity = {"status": "ok" if ok else "mismatch", "resources": want,
              "timed_batch": timed, "timed_batch_note": "verdicts of the last timed evaluation, read back from the "
                                                        "device (kyv_batch_export_status), first %d resources" % nt,
              "pairs_compared": sep["pairs_compared"], "mismatches": sep["mismatches"],
              "nondeterministic_pairs_both": sep["nondeterministic_pairs_both"], "first_mismatch": sep["first_mismatch"],
              "jit": bool(res.jit), "timed_jit": bool(jit),
              "fail_pairs": ts["fail_pairs"], "paths_compared": ts["paths_compared"],
              "path_mismatches": ts["path_mismatches"], "messages_compared": ts["messages_compared"],
              "message_mismatches": ts["message_mismatches"], "messages_unrenderable": ts["messages_unrenderable"],
              "first_text_mismatch": [str(x)[:300] for x in ts["bad"][:1]]}
    return cpu, parity


def shard_parity(policies, rs, data, nsl, timed_status, cap=100000):
    """ranks > 0 of a multi-GPU run: the timed evaluation's own verdicts on this rank's shard prefix vs the oracle"""
    from oracle import oracle as O
    threads = max(1, host_cpus()["share"])
    lines = [x for x in data.split(b"\n", cap)[:cap] if x.strip()]
    n = min(len(lines), timed_status.shape[1])
    names, m, secs = O.validate_matrix(policies, b"[" + b",".join(lines[:n]) + b"]", nsl, threads=threads, nres=n,
                                       timed=True)
    out = compare_verdicts(rs, names, m, timed_status, n)
    out["status"] = "ok" if out["mismatches"] == 0 else "mismatch"
    out["oracle_s"] = secs
    return out


# device phase -> kernel-name prefixes of that phase in a rocprofv3 kernel trace
PHASE_KERNELS = {"match": ("kyv::match_kernel", "kyv::match_walk_kernel", "kyv::match_walk_generic", "kyv::match_rec_kernel", "kyv::match_pre_kernel", "kyv::facts_kernel", "kyv::pss_kernel", "kyv::pss_map_kernel", "kyv::match_deny_kernel"), "cond": ("kyv_jit_cond",), "walk": ("kyv_jit_walk", "kyv_jit_fused", "kyv_jit_shapes", "kyv::walk_kernel"),
                 "compact": ("kyv::compact",), "hist": ("kyv::status_hist",)}


def largest_kernel(s, pre):
    """The phase's longest kernel per evaluation in a PMC summary: its name, launches and time per evaluation and its
    own memory-side bytes (TCC_EA FETCH_SIZE + WRITE_SIZE) and counter roofline fraction (bytes / its time / peak)."""
    kern = s.get("kernels") or {}
    nev = s.get("evaluations") or sum(k["calls"] for kn, k in kern.items() if "status_hist" in kn) or 1
    best = None
    for kn, k in kern.items():
        n = kn[5:] if kn.startswith("void ") else kn
        if not n.startswith(pre):
            continue
        ns = k["avg_ns"] * k["calls"] / nev
        if best is None or ns > best[1]:
            best = (kn, ns, k["calls"] / nev)
    if best is None:
        return None
    c = (s.get("counters_avg_per_launch") or {}).get(best[0]) or {}
    b = (c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024 * best[2]
    return {"name": best[0], "launches_per_eval": best[2], "ms_per_eval": best[1] / 1e6, "counter_bytes_per_eval": b,
            "counter_frac": b / (best[1] / 1e9) / 1e9 / HBM_PEAK_GBS if best[1] > 0 else None}


def pmc_traffic(config, phase):
    """Memory-side bytes per launch of the dominant kernel (phase) from the newest committed PMC summary
    (profiles/pmc_latest_<workload>.json, else profiles/pmc_latest.json; written by scripts/pmc_summary.py from separate rocprofv3 --pmc passes of this same
    command), used only when it was measured on the same workload configuration; else None. Returns
    (summary, tag) with summary = {traffic raw, traffic with the guide's x2 read correction, kernel ns}, all per
    evaluation (every launch of the phase's kernels in one evaluation)."""
    f = os.path.join(ROOT, "profiles", "pmc_latest_%s.json" % str(config.get("workload", "")).split(":")[0].strip().lower())
    if not os.path.exists(f):
        f = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(f):
        return None, None
    with open(f) as fh:
        s = json.load(fh)
    bc = s.get("bench_config") or {}
    keys = ("workload", "resources_per_gpu", "compiled_rules")
    if any(bc.get(k) != config.get(k) for k in keys):
        return None, s.get("tag")
    pre = PHASE_KERNELS[phase]
    ph = (s.get("phases") or {}).get(phase)
    if ph:  # scripts/pmc_summary.py: per-evaluation totals of the phase's kernels
        return {"raw": ph["traffic_bytes"], "x2read": 2 * ph["fetch_bytes"] + ph["write_bytes"], "fetch": ph["fetch_bytes"],
                "write": ph["write_bytes"], "avg_ns": ph["ns"], "wait_frac": ph.get("wait_frac"),
                "l2_hit": ph.get("l2_hit_rate"), "largest": largest_kernel(s, pre)}, s.get("tag")
    fetch = write = ns = 0.0
    found = False
    kern = s.get("kernels") or {}
    # launches per evaluation: the verdict histogram runs once per evaluation; a phase's kernels may run once per rule
    # slice (the 10M-resource batch is evaluated in rule slices) and several kernels make up one phase (walk groups)
    nev = sum(k["calls"] for kn, k in kern.items() if "status_hist" in kn) or 1
    per_eval = {kn: k["calls"] / nev for kn, k in kern.items()}
    for kn, c in (s.get("counters_avg_per_launch") or {}).items():
        n = kn[5:] if kn.startswith("void ") else kn
        if n.startswith(pre):
            found = True
            f = per_eval.get(kn, 1.0)
            fetch += c.get("FETCH_SIZE", 0.0) * 1024 * f
            write += c.get("WRITE_SIZE", 0.0) * 1024 * f
    for kn, k in kern.items():
        n = kn[5:] if kn.startswith("void ") else kn
        if n.startswith(pre):
            ns += k["avg_ns"] * per_eval[kn]
    if not found:
        return None, s.get("tag")
    return {"raw": fetch + write, "x2read": 2 * fetch + write, "fetch": fetch, "write": write, "avg_ns": ns,
            "wait_frac": s.get("dominant_wait_frac"), "l2_hit": s.get("dominant_l2_hit_rate"),
            "largest": largest_kernel(s, pre)}, s.get("tag")


def _split_ndjson(data, parts):
    """NDJSON bytes -> `parts` chunks cut at line boundaries"""
    out, at, step = [], 0, max(1, len(data) // max(1, parts))
    while at < len(data):
        cut = data.find(b"\n", min(len(data) - 1, at + step))
        cut = len(data) if cut < 0 else cut + 1
        out.append(data[at:cut])
        at = cut
    return out


def end_to_end(E, rs, data, nsl, nrules, device, chunk=1_250_000):
    """JSON in -> verdicts out on this rank, two ways: serial (flatten the whole shard, then upload + evaluate +
    copy every verdict back) and pipelined (the shard in chunks of `chunk` resources: chunk i+1 is flattened on a
    host thread -- the flattener's own worker threads, GIL released in the library call -- while chunk i is uploaded,
    evaluated and copied back). The pipelined rate is the one reported (the caller being replaced scans resources
    one at a time: pkg/controllers/report/utils/scanner.go:60-110)."""
    from concurrent.futures import ThreadPoolExecutor
    t0 = time.time()
    b2 = E.Batch(rs, data, nsl)
    t1 = time.time()
    r2 = E.evaluate(rs, b2, backend="gpu", device=device, copy_back=True)
    t2 = time.time()
    n = b2.n
    serial_dec = nrules * n - int(sum(r2.counts.get(s, 0) for s in CPU_STATUSES))
    del r2, b2
    parts = _split_ndjson(data, max(1, (n + chunk - 1) // chunk))
    decided = 0
    wait = 0.0
    t3 = time.time()
    with ThreadPoolExecutor(max_workers=1) as ex:
        fut = ex.submit(E.Batch, rs, parts[0], nsl)
        for i in range(len(parts)):
            tw = time.time()
            b = fut.result()
            wait += time.time() - tw
            if i + 1 < len(parts):
                fut = ex.submit(E.Batch, rs, parts[i + 1], nsl)
            r = E.evaluate(rs, b, backend="gpu", device=device, copy_back=True)
            decided += nrules * b.n - int(sum(r.counts.get(s, 0) for s in CPU_STATUSES))
            del r, b
    t4 = time.time()
    pipe, serial = decided / (t4 - t3), serial_dec / (t2 - t0)
    # the faster of the two is the rate this rank delivers (on a CPU share of 16 threads the flattener is the bound
    # either way, and the overlapped chunk flatten competes with the verdict copy-back for the same threads)
    return {"pairs_per_s": max(pipe, serial), "mode": "pipelined" if pipe >= serial else "serial",
            "pipelined_pairs_per_s": pipe, "seconds": t4 - t3, "chunks": len(parts),
            "chunk_resources": chunk, "flatten_wait_s": wait,
            "serial_pairs_per_s": serial, "serial_seconds": t2 - t0, "flatten_s": t1 - t0,
            "upload_eval_copyback_s": t2 - t1, "flatten_resources_per_s": n / max(t1 - t0, 1e-9),
            "flatten_threads": host_cpus()["share"]}


def fallback_by_reason(rs, res):
    """CPU-handed pairs per reason: the rule's compile-time reason, or "run-time" for pairs of device rules"""
    out = {}
    for k, r in enumerate(rs.rules):
        n = int(sum(res.rule_counts[k][s] for s in (5, 6, 7)))
        if n:
            why = r["reason"] if r["kind"] == "fallback" else "run-time (value / walk outside the device subset)"
            out[why] = out.get(why, 0) + n
    return out


def shard(total, rank, world, chunk=20000):
    """contiguous shard [lo, hi) of rank `rank`: boundaries on corpus-chunk multiples (synth.corpus_ndjson)"""
    cut = lambda r: min(total, (total * r // world) // chunk * chunk) if r < world else total
    return cut(rank), cut(rank + 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=["c3", "c2", "c4", "c5"])
    ap.add_argument("--resources", type=int, default=0,
                    help="total resources over all GPUs (default 10M c3, 1M c2 / c4 / c5)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (flatten + H2D + eval + D2H) leg")
    ap.add_argument("--no-account", action="store_true",
                    help="profiling runs: skip the byte-accounting evaluation (its kernels share the product's names)")
    ap.add_argument("--no-serial", action="store_true", help="profiling runs: skip the serialised phase-time evaluations")
    ap.add_argument("--gather", action="store_true",
                    help="time the RCCL all-gather of the resident results (loads torch first: KYV_TORCH_FIRST)")
    ap.add_argument("--no-gather", action="store_true", help="skip the report-assembly gather after the timed region")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(args.gpus)

    if args.gather:  # torch.distributed's RCCL needs torch's HIP runtime loaded before the library's (_lib.py)
        os.environ["KYV_TORCH_FIRST"] = "1"
    from kyverno_amd import engine as E
    from kyverno_amd import synth

    rank, world, local, pg = dist_setup(args.gpus)
    total = args.resources or (10_000_000 if args.workload == "c3" else 1_000_000)
    lo, hi = shard(total, rank, world)
    kind = "pods" if args.workload in ("c2", "c5") else "mixed"
    policies = load_policies(args.workload)

    t0 = time.time()
    data, nsl = synth.cached_corpus(hi - lo, kind=kind, seed=SEED, start=lo)
    t_gen = time.time() - t0
    log("rank %d: generated resources [%d, %d) of %d (%.1f MB) in %.1f s" % (rank, lo, hi, total, len(data) / 1e6, t_gen))
    t0 = time.time()
    rs = E.Ruleset(policies)
    t_compile = time.time() - t0
    nrules = len(rs.rules)
    t0 = time.time()
    batch = E.Batch(rs, data, nsl)
    t_flat = time.time() - t0
    log("rank %d: flattened %d resources into %d node rows in %.1f s" % (rank, batch.n, batch.stats()["nodes"], t_flat))
    pairs = nrules * batch.n

    # warmup (first call uploads the batch, loads / compiles the walk kernel, allocates the resident buffers)
    t0 = time.time()
    first = E.evaluate(rs, batch, backend="gpu", device=local, copy_back=False)
    t_upload = time.time() - t0
    counts = first.counts
    timed_jit = bool(first.jit)
    fb_reasons = fallback_by_reason(rs, first)
    batch_dev = {"upload_ms": first.upload_ms, "gmask_kernel_ms": first.gmask_ms,
                 "note": "per-batch device work before the batch's first evaluation (outside `value`): the batch "
                         "image upload through the pinned ring and the glob-mask kernel over its dictionary"}
    log("rank %d: first GPU evaluation (incl. upload) %.2f s, kernel %.2f ms" % (rank, t_upload, first.kernel_ms))
    del first
    for _ in range(max(0, args.warmup - 1)):
        E.evaluate(rs, batch, backend="gpu", device=local, copy_back=False)
    # algorithmic bytes per launch, counted by the kernels themselves: one evaluation of this whole shard
    # with the byte-accounting build of the same kernels (KYV_ACCT: every per-resource load and result store adds its
    # bytes to device counters), phases serialised so each phase's bytes are its own; outside the timed region
    t0 = time.time()
    if args.no_account:
        phase_bytes, alg_class, bytes_per_eval, acct_counts_ok = dict.fromkeys(PHASE_KERNELS, 0), {}, 0.0, None
    else:
        acct = E.evaluate(rs, batch, backend="gpu", device=local, copy_back=False, account_bytes=True, jit=timed_jit)
        phase_bytes = dict(acct.alg_bytes_phase)
        alg_class = dict(acct.alg_bytes_class)
        bytes_per_eval = acct.alg_bytes / max(1, pairs)
        acct_counts_ok = acct.counts == counts  # the accounting build decides every pair as the product build does
        del acct
    log("rank %d: %.1f algorithmic bytes per eval (device-counted over the shard, %.1f s): %s" % (
        rank, bytes_per_eval, time.time() - t0, phase_bytes))

    barrier(pg)
    t0 = time.perf_counter()
    kms = 0.0
    phase = dict.fromkeys(PHASE_KERNELS, 0.0)
    for _ in range(args.steps):
        r = E.evaluate(rs, batch, backend="gpu", device=local, copy_back=False)
        kms += r.kernel_ms
        for k in phase:
            phase[k] += r.phase_ms[k]
    barrier(pg)
    dt = time.perf_counter() - t0
    dt_max = all_max(pg, dt)
    # the timed evaluation's own verdicts for this rank's shard prefix (parity below), read back before any other
    # evaluation (serialised, accounting) replaces the resident results
    prefix_status = None
    if not args.no_cpu_baseline:
        prefix_status = timed_prefix_status(batch, local, 400000 if rank == 0 else 100000)
    kernel_ms = kms / max(1, args.steps)
    kernel_ms_max = all_max(pg, kernel_ms)
    phase_span = {k: v / max(1, args.steps) for k, v in phase.items()}
    # per-phase kernel times for the roofline: evaluations with every phase on one stream (in the timed evaluations
    # the compiled condition kernels run beside the walk, so their phase times are overlapping spans)
    nser = 0 if args.no_serial else max(3, min(10, args.steps))
    phase = dict.fromkeys(PHASE_KERNELS, 0.0)
    ser_ms = 0.0
    for _ in range(nser):
        r = E.evaluate(rs, batch, backend="gpu", device=local, copy_back=False, serial=True)
        ser_ms += r.kernel_ms
        for k in phase:
            phase[k] += r.phase_ms[k] / nser
    ser_ms /= max(1, nser)
    if not nser:
        phase = dict(phase_span)
    # pairs the device decided: every (resource, compiled rule) pair except those it hands to the CPU engine
    # (FALLBACK / PANIC / ND: rules or pairs outside the GPU subset, counted separately, not in `value`)
    cpu_pairs = int(sum(counts.get(s, 0) for s in CPU_STATUSES))
    dev_pairs = pairs - cpu_pairs
    total_pairs = all_sum(pg, dev_pairs)
    total_fb = all_sum(pg, cpu_pairs)

    # report assembly of a multi-GPU scan: RCCL all-gather of every rank's verdicts and failing-path
    # rows straight from the device-resident results of the last timed evaluation, timed after the evaluation
    gathers = None
    if args.gather:  # torch.distributed's RCCL (scan.gather_*_device)
        gathers = time_gathers(batch, local, rank, world)
        log("rank %d: device-resident gathers %s" % (rank, gathers))
    elif not args.no_gather:  # the library's own RCCL communicator
        try:
            gathers = native_gathers(batch, local, rank, world, pg, lo, own_counts=r.rule_counts)
        except Exception as e:  # reported, never fatal for the timed line
            gathers = {"error": str(e)[:300]}
        log("rank %d: device-resident gathers %s" % (rank, gathers))

    # FETCH_SIZE calibration for the profiling runs (scripts/profile_box.sh sets KYV_CALIB=1): launches of known byte
    # counts at the access widths the evaluation kernels use, read back by scripts/pmc_summary.py
    if os.environ.get("KYV_CALIB") == "1" and rank == 0:
        from kyverno_amd import _lib as KL
        for mode in (4, 8, 16, 116):
            ms = KL.lib().kyv_calibrate_fetch(local, 1 << 30, mode)
            log("calibration launch: mode %d, 1 GiB in %.3f ms" % (mode, ms))

    # end to end on this rank: JSON -> flatten -> H2D -> evaluate -> D2H of every verdict (walk kernel already loaded)
    e2e = None
    if not args.no_e2e:
        e2e = end_to_end(E, rs, data, nsl, pairs // max(1, batch.n), local)
        log("rank %d: end to end %.3g pairs/s pipelined over %d chunks (%.2f s; serial %.2f s: flatten %.2f s + "
            "upload / evaluate / copy back %.2f s)" % (rank, e2e["pipelined_pairs_per_s"], e2e["chunks"], e2e["seconds"],
                                                       e2e["serial_seconds"], e2e["flatten_s"],
                                                       e2e["upload_eval_copyback_s"]))

    cpu = parity = None
    rank_parity = None
    if not args.no_cpu_baseline:
        if rank == 0:  # cpu_baseline on rank 0; its prefix is also rank 0's parity sample
            cpu, parity = cpu_baseline_and_parity(policies, rs, data, nsl, timed_jit, prefix_status, device=local)
            log("rank 0: parity on the cpu_baseline prefix: %s (timed batch: %s; %d pairs, %d mismatches; %d FAIL "
                "pairs: %d path / %d message mismatches)" % (
                    parity["status"], parity["timed_batch"], parity["pairs_compared"], parity["mismatches"],
                    parity["fail_pairs"], parity["path_mismatches"], parity["message_mismatches"]))
            mine = {"rank": 0, "status": parity["status"], "timed_batch": parity["timed_batch"]}
        else:  # every other rank checks its own shard prefix of the timed evaluation
            mine = dict(shard_parity(policies, rs, data, nsl, prefix_status), rank=rank)
        rank_parity = all_gather_obj(pg, mine)
        if parity is not None and world > 1:
            parity["ranks"] = rank_parity
            if any(p.get("status") != "ok" for p in rank_parity):
                parity["status"] = "mismatch"
    gather_ranks = all_gather_obj(pg, gathers) if gathers is not None else None

    if rank == 0:
        # dominant kernel: the device phase with the longest time per evaluation, among all five
        dom = max(PHASE_KERNELS, key=lambda k: phase[k])
        dom_ms = phase[dom]
        achieved = phase_bytes[dom] / (dom_ms / 1e3) / 1e9 if dom_ms > 0 else 0.0
        phase_frac = {k: (phase_bytes[k] / (phase[k] / 1e3) / 1e9 / HBM_PEAK_GBS if phase[k] > 0 else 0.0)
                      for k in PHASE_KERNELS}
        eval_frac = sum(phase_bytes.values()) / max(kernel_ms / 1e3, 1e-12) / 1e9 / HBM_PEAK_GBS
        over = {k: f for k, f in phase_frac.items() if f > 1.0}
        if eval_frac > 1.0:
            over["evaluation"] = eval_frac
        wl = {"c3": "C3: charts/kyverno-policies restricted + test/best_practices validate policies (select-secrets "
                    "excluded, SURVEY §8(d); %d compiled rules) over %d mixed resources (%d per GPU)",
              "c2": "C2: podSecurity restricted/latest (%d compiled rules) over %d pods (%d per GPU)",
              "c4": "C4: 10,000 generated policies, wildcard match/exclude stress (%d compiled rules) over %d mixed "
                    "resources (%d per GPU)",
              "c5": "C5: 50 generated precondition / deny policies with variables (%d compiled rules) over %d pods "
                    "(%d per GPU)"}[args.workload] % (nrules, total, batch.n)
        config = {"workload": wl, "resources_total": total, "resources_per_gpu": batch.n, "compiled_rules": nrules,
                  "pairs_per_step": int(total_pairs), "cpu_fallback_pairs_per_step": int(total_fb),
                  "parallelism": "shard%d" % world}
        tr, pmc_tag = pmc_traffic(config, dom)
        line = {
            "metric": METRIC,
            "value": total_pairs * args.steps / dt_max,
            "unit": "resource×rule evals/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max * 1e3 / max(1, args.steps),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded generator kyverno_amd/synth.py, SURVEY §8(d) model; one corpus, seed 0x4b59564e, "
                    "sharded contiguously across ranks)",
            "config": config,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": tr["raw"] if tr else None,
                         "traffic_x2read": tr["x2read"] if tr else None,
                         "counter_frac": (tr["raw"] / (dom_ms / 1e3) / 1e9 / HBM_PEAK_GBS) if tr else None,
                         "traffic_source": "profiles/%s_summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of the "
                                           "%s kernels, bytes per evaluation: every launch of them)" % (pmc_tag, dom)
                                           if tr else None,
                         "profiled_kernel_ms": tr["avg_ns"] / 1e6 if tr else None,
                         "profiled_wait_frac": tr.get("wait_frac") if tr else None,
                         "profiled_l2_hit_rate": tr.get("l2_hit") if tr else None,
                         "largest_kernel": tr.get("largest") if tr else None,
                         "kernel": {"walk": "the pattern-walk phase: kyv_jit_fused_<group>[p<part>] (runtime-compiled "
                                            "fused walks, one kernel per rule group and part), kyv_jit_shapes (shape "
                                            "tables), kyv_jit_walk_<k> (per-chunk walks); frac is the phase's (all its "
                                            "kernels' bytes / their summed time), largest_kernel the longest one's own",
                                    "cond": "kyv_jit_condg_<rule> / kyv_jit_cond_<rule> (runtime-compiled deny / foreach "
                                            "conditions)",
                                    "match": "kyv::match_rec_kernel / match_deny_kernel / match_pre_kernel / match_kernel "
                                             "/ pss_kernel (match / exclude, podSecurity, plain conditions)",
                                    "compact": "kyv::compact_* (failing-path record compaction)",
                                    "hist": "kyv::status_hist_kernel (verdict totals)"}[dom],
                         "kernel_ms": dom_ms,
                         "alg_bytes_per_launch": phase_bytes[dom],
                         "achieved_basis": "algorithmic bytes per launch counted by the kernels themselves: one "
                                           "evaluation of the whole shard with the KYV_ACCT build of the same kernel "
                                           "source (kyv_acct.hip, the runtime-compiled kernels with -DKYV_ACCT), "
                                           "every load of resource data (16-B node rows, 8-B path-column entries, "
                                           "header fields, work lists) and every result store (verdict bytes, PSS "
                                           "masks, staged and compacted failing-path records, work lists) counted, "
                                           "phases serialised; dictionary columns and rule programs excluded (SURVEY "
                                           "§8(d)); / the kernel's time (HIP events on the evaluation stream)",
                         "valid": not over,
                         "frac_over_1": over or None,
                         "phase_frac": phase_frac,
                         "alg_bytes_by_class": alg_class,
                         "accounting_verdicts_match": acct_counts_ok,
                         "overlap": "timed evaluations run the compiled condition kernels on a second HIP stream "
                                    "concurrently with the walk (phase_ms_span: spans under that overlap); kernel_ms / "
                                    "phase_ms come from %d serialised evaluations (KYV_EVAL_SERIAL: %.3f ms each), "
                                    "evaluation_frac is the timed (overlapped) evaluation's figure" % (nser, ser_ms),
                         "phase_ms": phase,
                         "phase_ms_span": phase_span,
                         "serial_evaluation_ms": ser_ms,
                         "phase_alg_bytes": phase_bytes,
                         "evaluation_ms": kernel_ms,
                         "evaluation_ms_max_rank": kernel_ms_max,
                         "evaluation_frac": eval_frac,
                         "bytes_per_eval": bytes_per_eval},
            "cpu_baseline": cpu,
            "parity_prefix": parity,
            "verdicts": {k: v for k, v in counts.items()},
            "cpu_fallback_by_reason": fb_reasons,
            "report_gather": None if not gather_ranks else {
                "verdicts_ms_max_rank": max(g.get("verdicts_ms", 0.0) for g in gather_ranks),
                "failures_ms_max_rank": max(g.get("failures_ms", 0.0) for g in gather_ranks),
                "ranks": gather_ranks,
                "ok": all(g.get("own_segment_ok", True) and g.get("segments_ok", True) and "error" not in g
                          and g.get("rows_complete", True) and g.get("counts_sum_ok") is not False
                          and g.get("failures_ms", 0.0) >= 0 for g in gather_ranks),
                "note": "timed after the evaluation, outside `value`: the packed verdicts and 16-B failing-path rows "
                        "of every rank sent to rank 0 from the device-resident results (kyv_comm_gather_report), the "
                        "per-rule tallies all-reduced (kyv_comm_reduce_counts); --gather: torch.distributed's RCCL "
                        "all-gathers, kyverno_amd/scan.py"},
            "host": {"generate_s": t_gen, "compile_s": t_compile, "flatten_s": t_flat,
                     "flatten_resources_per_s": batch.n / max(t_flat, 1e-9),
                     "first_eval_incl_upload_s": t_upload, "batch_device_bytes": batch.stats()["device_bytes"],
                     "per_batch_device_ms": batch_dev,
                     "e2e": e2e},
        }
        print(json.dumps(line), flush=True)
        if over:  # algorithmic bytes above what HBM can move in the measured time: the accounting is wrong
            log("roofline INVALID: frac > 1 for %s" % over)
            sys.exit(3)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
