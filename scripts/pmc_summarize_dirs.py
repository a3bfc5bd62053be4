"""Summarise an r3_prof.sh run (gpurun_out/<tag>/<workload>/ traces, gpurun_out/<tag>/pmc_<workload>_<counter>/ PMC
passes) into profiles/<tag>/: each workload's kernel-trace stats CSV and bench line, and per PMC workload a JSON with
every query-path kernel's per-launch counters (FETCH_SIZE / WRITE_SIZE in bytes, SQ_LDS_BANK_CONFLICT in cycles) and
HBM bytes = fetch_correction x FETCH_SIZE + WRITE_SIZE (the correction measured on config 5's register-direct stream,
profiles/pmc_adanalytics.json; the guide's x2 for 16-B/lane streams otherwise).
Usage: python scripts/pmc_summarize_dirs.py <tag>
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATH_KERNELS = ("query_kernel", "part_scan", "part_reduce", "invexp", "rawpred", "hash_", "leafbits", "gdict")
BYTE_COUNTERS = ("FETCH_SIZE", "WRITE_SIZE")


def _path_kernel(name):
    return any(k in name for k in PATH_KERNELS)


def _short(name):
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(DevParams")[0]


def _bench_line(log):
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def _counters(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"].startswith(counter) and _path_kernel(r["Kernel_Name"]):
            v = float(r["Counter_Value"])
            per[_short(r["Kernel_Name"])].append(v * 1024.0 if counter in BYTE_COUNTERS else v)
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def main():
    tag = sys.argv[1]
    src, dst = os.path.join(ROOT, "gpurun_out", tag), os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    factor = 2.0
    cal = os.path.join(ROOT, "profiles", "pmc_adanalytics.json")
    if os.path.exists(cal):
        factor = json.load(open(cal)).get("fetch_correction", 2.0)
    bench = {}
    for wl in sorted(os.listdir(src)):
        stats = os.path.join(src, wl, "run_kernel_stats.csv")
        if wl.startswith("pmc_") or not os.path.exists(stats):
            continue
        shutil.copy(stats, os.path.join(dst, f"kernel_stats_{wl}.csv"))
        b = _bench_line(os.path.join(src, f"{wl}.log"))
        if b:
            bench[wl] = b
    with open(os.path.join(dst, "bench_lines.json"), "w") as f:
        json.dump(bench, f, indent=1)
    pmc_wls = sorted({d[4:].rsplit("_", 2)[0] if d.endswith(("FETCH_SIZE", "WRITE_SIZE")) else d[4:].rsplit("_", 4)[0]
                      for d in os.listdir(src) if d.startswith("pmc_") and os.path.isdir(os.path.join(src, d))})
    for wl in pmc_wls:
        out = {"workload": wl, "tag": tag, "fetch_correction": factor, "kernels": {}}
        for c in ("FETCH_SIZE", "WRITE_SIZE", "SQ_LDS_BANK_CONFLICT"):
            p = os.path.join(src, f"pmc_{wl}_{c}", "run_counter_collection.csv")
            if not os.path.exists(p):
                continue
            avg, n = _counters(p, c)
            for k, v in avg.items():
                out["kernels"].setdefault(k, {})[c] = v
                out["kernels"][k][f"{c}_launches"] = n[k]
        stats = os.path.join(src, wl, "run_kernel_stats.csv")
        if os.path.exists(stats):
            for r in csv.DictReader(open(stats)):
                k = _short(r["Name"])
                if k in out["kernels"]:
                    out["kernels"][k]["rocprof_avg_ns"] = float(r["AverageNs"])
        total = 0.0
        for k, v in out["kernels"].items():
            if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
                v["hbm_bytes_per_launch"] = factor * v["FETCH_SIZE"] + v["WRITE_SIZE"]
                total += v["hbm_bytes_per_launch"]
        out["hbm_bytes_per_query"] = total
        if wl in bench:
            out["algorithmic_bytes_per_launch"] = bench[wl]["roofline"]["algorithmic_bytes_per_launch"]
            out["bench_kernel_ms_avg"] = bench[wl]["roofline"]["kernel_ms_avg"]
        with open(os.path.join(dst, f"pmc_{wl}.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(wl, json.dumps(out))


if __name__ == "__main__":
    main()
