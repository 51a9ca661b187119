"""Summarise one profiling run of scripts/profile_box.sh (gpurun_out/prof_<tag>/) into profiles/.

  python scripts/pmc_summary.py <tag>

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats), profiles/<tag>_pmc.csv (per-dispatch
counters of the dominant kernel, one row per PMC pass and dispatch) and profiles/<tag>_summary.json (averages
per launch). bench.py reads profiles/pmc_latest_<workload>.json (a copy of the newest summary of that workload) for roofline.traffic.

Units: rocprofv3 FETCH_SIZE / WRITE_SIZE are KiB per dispatch. MI355X_MICROARCH.md (HBM section) notes that on
gfx950 FETCH_SIZE reports half the bytes of a wide 16-B/lane coalesced stream; this kernel's reads are 16-B
node-row gathers (one row per lane, rows of different resources), an access width the guide leaves uncalibrated,
so traffic is reported both raw (bench.py's roofline.traffic) and with the x2 read correction (upper estimate).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EVAL = ("kyv", "kyv_jit_walk")  # kernels of one evaluation: kyv::match_kernel, walk kernels, compaction


def is_eval(name):
    n = name[5:] if name.startswith("void ") else name  # templates: "void kyv::match_kernel<true>(...)"
    if n.startswith("kyv::gmask_kernel"):  # once per batch (glob masks of the dictionary), not per evaluation
        return False
    if n.startswith("kyv::calib_"):  # FETCH_SIZE calibration launches (bench.py KYV_CALIB=1), reported apart
        return False
    return n.startswith("kyv::") or n.startswith("kyv_jit")


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, tag + "_kernel_stats.csv"))
    stats = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))) if is_eval(r["Name"])]
    per_kernel = {r["Name"].split("(")[0]: {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])} for r in stats}
    counters = {}  # kernel -> counter -> values
    calib = {}     # calibration kernel -> FETCH_SIZE bytes per launch (each launch reads exactly 1 GiB)
    rows_out = []
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not p.startswith("pmc_") or not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            kname = r["Kernel_Name"][5:] if r["Kernel_Name"].startswith("void ") else r["Kernel_Name"]
            if kname.startswith("kyv::calib_"):
                calib.setdefault(kname.split("(")[0], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            if not is_eval(r["Kernel_Name"]):
                continue
            kn = r["Kernel_Name"].split("(")[0]
            counters.setdefault(kn, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            rows_out.append({"pass": p, "dispatch": r["Dispatch_Id"], "kernel": kn, "counter": r["Counter_Name"],
                             "value": r["Counter_Value"], "grid": r["Grid_Size"], "wg": r["Workgroup_Size"],
                             "lds": r["LDS_Block_Size"], "vgpr": r["VGPR_Count"], "sgpr": r["SGPR_Count"],
                             "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
    with open(os.path.join(dst, tag + "_pmc.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows_out[0].keys()) if rows_out else ["pass"])
        w.writeheader()
        w.writerows(rows_out)
    avg = {kn: {c: sum(v) / len(v) for c, v in cs.items()} for kn, cs in counters.items()}
    # launches per evaluation: the verdict histogram runs once per evaluation; the other kernels once per rule slice
    # (10M-resource batches run in two slices) or once per compiled rule (condition kernels)
    nev = sum(k["calls"] for kn, k in per_kernel.items() if "status_hist" in kn) or 1
    fac = {kn: k["calls"] / nev for kn, k in per_kernel.items()}
    fetch = sum(a.get("FETCH_SIZE", 0.0) * fac.get(kn, 1.0) for kn, a in avg.items()) * 1024
    write = sum(a.get("WRITE_SIZE", 0.0) * fac.get(kn, 1.0) for kn, a in avg.items()) * 1024
    eval_ns = sum(k["avg_ns"] * fac[kn] for kn, k in per_kernel.items())
    # per device phase (bench.py PHASE_KERNELS): time, memory-side bytes, stall fraction and L2 hit rate per evaluation
    phases = {"match": ("kyv::match_kernel", "kyv::match_walk_kernel", "kyv::match_walk_generic", "kyv::match_rec_kernel", "kyv::match_pre_kernel", "kyv::facts_kernel", "kyv::pss_kernel", "kyv::pss_map_kernel", "kyv::match_deny_kernel"), "cond": ("kyv_jit_cond",), "walk": ("kyv_jit_walk", "kyv_jit_fused", "kyv_jit_shapes", "kyv::walk_kernel"),
              "compact": ("kyv::compact",), "hist": ("kyv::status_hist",)}
    ph = {}
    for name, pre in phases.items():
        ks = [kn for kn in per_kernel if (kn[5:] if kn.startswith("void ") else kn).startswith(pre)]
        if not ks:
            continue
        t = sum(per_kernel[kn]["avg_ns"] * fac[kn] for kn in ks)
        acc = {}
        for kn in ks:
            for c, x in avg.get(kn, {}).items():
                acc[c] = acc.get(c, 0.0) + x * fac[kn]
        e = {"ns": t, "kernels": len(ks), "fetch_bytes": acc.get("FETCH_SIZE", 0.0) * 1024,
             "write_bytes": acc.get("WRITE_SIZE", 0.0) * 1024}
        e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
        e["traffic_GBs"] = e["traffic_bytes"] / max(t, 1.0)
        if acc.get("SQ_WAVE_CYCLES"):
            e["wait_frac"] = acc.get("SQ_WAIT_ANY", 0.0) / acc["SQ_WAVE_CYCLES"]
        rq = {c: x for c, x in acc.items() if c.startswith("TCC_EA0_RDREQ")}
        if rq:
            e["read_requests"] = rq
        if "TCC_HIT_sum" in acc:
            e["l2_hit_rate"] = acc["TCC_HIT_sum"] / max(1.0, acc["TCC_HIT_sum"] + acc.get("TCC_MISS_sum", 0.0))
        ph[name] = e
    dom_phase = max(("match", "cond", "walk"), key=lambda k: ph.get(k, {}).get("ns", 0.0))
    dom = max(per_kernel.items(), key=lambda kv: kv[1]["avg_ns"] * fac[kv[0]])[0] if per_kernel else None
    out = {
        "tag": tag,
        "kernels": per_kernel,
        "launches_per_evaluation": fac,
        "evaluations": nev,
        "eval_avg_ns": eval_ns,
        "eval_note": "sum of the evaluation's kernel durations; kernels on the concurrent condition stream overlap "
                     "the walk, so this exceeds the evaluation's wall time (bench roofline.evaluation_ms)",
        "dominant_kernel": dom,
        "dominant_phase": dom_phase,
        "phases": ph,
        "counters_avg_per_launch": avg,
        "fetch_bytes_raw": fetch,
        "write_bytes_raw": write,
        "traffic_bytes": fetch + write,
        "traffic_bytes_x2read": 2 * fetch + write,
        "traffic_note": "memory-side bytes of one evaluation (every launch of its kernels) from TCC_EA (FETCH_SIZE + "
                        "WRITE_SIZE, KiB x 1024); traffic_bytes_x2read applies the guide's x2 wide-stream read correction",
    }
    if calib:  # known bytes / counted bytes per access width (bench.py KYV_CALIB=1: 1 GiB per launch)
        out["fetch_calibration"] = {}
        for k, cs in calib.items():
            c = {n: sum(v) / len(v) for n, v in cs.items()}
            e = {"bytes": float(1 << 30), "counters": c}
            if "FETCH_SIZE" in c:
                e["fetch_size_bytes"] = c["FETCH_SIZE"] * 1024
                e["factor"] = float(1 << 30) / max(1.0, c["FETCH_SIZE"] * 1024)
            out["fetch_calibration"][k] = e
        out["fetch_calibration_note"] = ("factor = true bytes / FETCH_SIZE bytes of a launch that reads a known 1 GiB: "
                                         "calib_read_kernel<W> coalesced W bytes per lane, calib_gather_kernel 16-byte "
                                         "rows in scrambled order")
    if dom_phase in ph:
        out["dominant_l2_hit_rate"] = ph[dom_phase].get("l2_hit_rate")
        out["dominant_wait_frac"] = ph[dom_phase].get("wait_frac")
    log = os.path.join(src, "bench_trace.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                b = json.loads(line)
                out["bench_config"] = b.get("config")
                out["bench_value"] = b.get("value")
    js = json.dumps(out, indent=1, sort_keys=True)
    open(os.path.join(dst, tag + "_summary.json"), "w").write(js + "\n")
    # one "latest" per workload (bench.py reads the one of the workload it runs), so profiling C4 / C5 does not
    # displace the headline workload's summary
    wl = ((out.get("bench_config") or {}).get("workload") or "").split(":")[0].strip().lower()
    open(os.path.join(dst, "pmc_latest_%s.json" % wl if wl else "pmc_latest.json"), "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r1")
