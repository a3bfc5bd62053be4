"""Summarise a profile_round.sh run into profiles/<tag>/ and profiles/pmc_<workload>.json.

HBM bytes per query_kernel launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB counters; FETCH_SIZE doubled per the
gfx950 correction in MI355X_MICROARCH.md "HBM": wide coalesced streaming reads are tallied at half their bytes).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, kernel="query_kernel"):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    vals = [float(r["Counter_Value"]) * 1024.0 for r in rows]
    return sum(vals) / len(vals), len(vals)


def main():
    tag, wl = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "adanalytics"
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"kernel_stats_{wl}.csv"))
    fetch, n1 = per_launch(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"))
    write, n2 = per_launch(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"))
    avg_ns = None
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        if "query_kernel" in r["Name"]:
            avg_ns = float(r["AverageNs"])
    out = {"workload": wl, "tag": tag, "kernel": "query_kernel",
           "fetch_size_bytes_raw": fetch, "write_size_bytes": write, "launches": [n1, n2],
           "hbm_bytes_per_launch": 2 * fetch + write,
           "rocprof_avg_kernel_ns": avg_ns,
           "note": "2 x FETCH_SIZE + WRITE_SIZE per launch; the x2 gfx950 correction is calibrated for 16-B/lane "
                   "streaming reads (the LDS-DMA tile stream); the sparse sector gathers are narrower loads, so "
                   "the true HBM bytes lie between FETCH_SIZE + (dense stream bytes) and this figure"}
    with open(os.path.join(ROOT, "profiles", f"pmc_{wl}.json"), "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.join(dst, f"pmc_{wl}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
