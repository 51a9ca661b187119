"""Admission micro-batching latency / throughput on one GPU.

Workload: C3's device-covered policies (charts/kyverno-policies restricted + test/best_practices, without the four
JMESPath / foreach policies the device hands to the CPU engine), every policy set to Enforce, over seeded synthetic
CREATE / UPDATE AdmissionRequests of the mixed-kind model (kyverno_amd/synth.py).

Two measurements:
  sweep    handle_batch() over fixed batch sizes: per-batch latency (host flatten + upload + device evaluation +
           decision assembly) and requests/s;
  threaded C client threads, each submitting one request at a time through the micro-batcher (max_batch, max_wait)
           and waiting for its decision: end-to-end latency percentiles and requests/s.
Prints one JSON line. Usage: python scripts/bench_admission.py [--backend gpu] [--seconds 5]
"""
import argparse
import copy
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import cases  # noqa: E402
from kyverno_amd import admission as A  # noqa: E402
from kyverno_amd import engine as E  # noqa: E402
from kyverno_amd import synth  # noqa: E402


def policies():
    pols = cases.best_practices() + cases.chart_restricted()
    rs = E.Ruleset(pols)
    cpu_only = {rs.policies[r["policy"]]["name"] for r in rs.rules if r["kind"] == "fallback"}
    out = []
    for p in pols:
        if p["metadata"]["name"] in cpu_only:
            continue
        p = copy.deepcopy(p)
        p["spec"]["validationFailureAction"] = "Enforce"
        out.append(p)
    return out, sorted(cpu_only)


def requests(n, seed=0x4b59564e):
    docs, nsl = synth.mixed(n, seed=seed)
    out = []
    for i, d in enumerate(docs):
        md = d.get("metadata") if isinstance(d.get("metadata"), dict) else {}
        ns = md.get("namespace") if isinstance(md.get("namespace"), str) else ""
        out.append({"uid": str(i), "operation": "CREATE", "kind": d.get("kind", ""), "namespace": ns, "object": d,
                    "object_raw": json.dumps(d, separators=(",", ":")).encode(),  # AdmissionRequest.Object.Raw
                    "namespace_labels": nsl.get(ns) if ns else None})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gpu")
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--sizes", default="1,16,128,1024,4096")
    ap.add_argument("--clients", type=int, default=256)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--max-wait-ms", type=float, default=1.0)
    a = ap.parse_args()
    pols, excluded = policies()
    sizes = [int(s) for s in a.sizes.split(",")]
    reqs = requests(max(sizes) * 2)
    b = A.AdmissionBatcher(pols, backend=a.backend, max_batch=a.max_batch, max_wait_ms=a.max_wait_ms)
    b.handle_batch(reqs[:64])  # warm-up: device context, ruleset upload
    sweep = []
    for bs in sizes:
        lat, done, t0, i = [], 0, time.perf_counter(), 0
        while time.perf_counter() - t0 < a.seconds / len(sizes) or not lat:
            chunk = reqs[i:i + bs] if i + bs <= len(reqs) else reqs[:bs]
            i = (i + bs) % max(1, len(reqs) - bs)
            s = time.perf_counter()
            out = b.handle_batch(chunk)
            lat.append(time.perf_counter() - s)
            done += len(out)
        el = time.perf_counter() - t0
        row = {"batch": bs, "requests_per_s": done / el, "batches": len(lat)}
        row.update(A.latency_summary(lat))
        sweep.append(row)
        print("[admission] batch %5d: %9.0f req/s  p50 %.2f ms  p99 %.2f ms" % (bs, row["requests_per_s"],
                                                                             row["p50_ms"], row["p99_ms"]),
              file=sys.stderr, flush=True)
    sample = reqs[:1000]
    blocked = sum(1 for d in b.handle_batch(sample) if d["allowed"] is False) / len(sample)

    # threaded closed loop through the micro-batcher
    b.start()
    lat, lock, stop = [], threading.Lock(), time.perf_counter() + a.seconds

    def client(c):
        j = c
        mine = []
        while time.perf_counter() < stop:
            s = time.perf_counter()
            b.submit(reqs[j % len(reqs)]).result()
            mine.append(time.perf_counter() - s)
            j += a.clients
        with lock:
            lat.extend(mine)

    b0 = b.stats["batches"]
    t0 = time.perf_counter()
    ths = [threading.Thread(target=client, args=(c,)) for c in range(a.clients)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    el = time.perf_counter() - t0
    b.stop()
    nb = b.stats["batches"] - b0
    threaded = {"clients": a.clients, "max_batch": a.max_batch, "max_wait_ms": a.max_wait_ms,
                "requests_per_s": len(lat) / el, "mean_batch": len(lat) / max(1, nb)}
    threaded.update(A.latency_summary(lat))
    print("[admission] threaded %d clients: %.0f req/s, mean batch %.1f, p50 %.2f ms p99 %.2f ms" % (
        a.clients, threaded["requests_per_s"], threaded["mean_batch"], threaded["p50_ms"], threaded["p99_ms"]),
        file=sys.stderr, flush=True)
    print(json.dumps({"metric": "admission requests/s (micro-batched validate, Enforce)", "backend": a.backend,
                      "policies": len(pols), "compiled_rules": len(b.ruleset.rules), "excluded_cpu_policies": excluded,
                      "blocked_fraction": blocked, "sweep": sweep, "threaded": threaded,
                      "data": "synthetic mixed-kind CREATE requests (kyverno_amd/synth.py)"}))


if __name__ == "__main__":
    main()
