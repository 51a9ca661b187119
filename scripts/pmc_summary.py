"""Summarise one profiling run of scripts/profile_box.sh (gpurun_out/prof_<tag>/) into profiles/.

  python scripts/pmc_summary.py <tag>

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats), profiles/<tag>_pmc.csv (per-dispatch
counters of the dominant kernel, one row per PMC pass and dispatch) and profiles/<tag>_summary.json (averages
per launch). bench.py reads profiles/pmc_latest.json (a copy of the newest summary) for roofline.traffic.

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
KERNEL = "eval_kernel"


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, tag + "_kernel_stats.csv"))
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    krow = [r for r in stats if KERNEL in r["Name"]][0]
    counters = {}
    rows_out = []
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not p.startswith("pmc_") or not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            counters.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            rows_out.append({"pass": p, "dispatch": r["Dispatch_Id"], "counter": r["Counter_Name"],
                             "value": r["Counter_Value"], "grid": r["Grid_Size"], "wg": r["Workgroup_Size"],
                             "lds": r["LDS_Block_Size"], "vgpr": r["VGPR_Count"], "sgpr": r["SGPR_Count"],
                             "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
    with open(os.path.join(dst, tag + "_pmc.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows_out[0].keys()) if rows_out else ["pass"])
        w.writeheader()
        w.writerows(rows_out)
    avg = {k: sum(v) / len(v) for k, v in counters.items()}
    fetch = avg.get("FETCH_SIZE", 0.0) * 1024
    write = avg.get("WRITE_SIZE", 0.0) * 1024
    out = {
        "tag": tag,
        "kernel": krow["Name"],
        "launches": int(krow["Calls"]),
        "avg_ns": float(krow["AverageNs"]),
        "counters_avg_per_launch": avg,
        "fetch_bytes_raw": fetch,
        "write_bytes_raw": write,
        "traffic_bytes_raw": fetch + write,
        "traffic_bytes": fetch + write,
        "traffic_bytes_x2read": 2 * fetch + write,
        "traffic_note": "memory-side bytes per launch from TCC_EA (FETCH_SIZE + WRITE_SIZE, KiB x 1024); "
                        "traffic_bytes_x2read applies the guide's x2 wide-stream read correction (upper estimate)",
    }
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        out["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if "SQ_WAVE_CYCLES" in avg:
        out["wait_frac"] = avg.get("SQ_WAIT_ANY", 0) / avg["SQ_WAVE_CYCLES"]
        out["active_frac"] = avg.get("SQ_ACTIVE_INST_ANY", 0) / avg["SQ_WAVE_CYCLES"]
        if "GRBM_GUI_ACTIVE" in avg:
            out["clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / (out["avg_ns"])
    log = os.path.join(src, "bench_trace.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                b = json.loads(line)
                out["bench_config"] = b.get("config")
                out["bench_value"] = b.get("value")
    js = json.dumps(out, indent=1, sort_keys=True)
    open(os.path.join(dst, tag + "_summary.json"), "w").write(js + "\n")
    open(os.path.join(dst, "pmc_latest.json"), "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r1")
