"""Summarise a profile_round.sh run into profiles/<tag>/ and profiles/pmc_<workload>.json.

HBM bytes per query-kernel launch = c x FETCH_SIZE + WRITE_SIZE (KiB counters).  MI355X_MICROARCH.md "HBM": FETCH_SIZE
reads exactly half the bytes of a 16-B/lane streaming read (c = 2 there) and other access widths are uncalibrated --
"calibrate on a known byte count in your own access pattern".  The register-direct stream loads 4 B per lane, so
`c` is measured: the FETCH_SIZE of config 5's filter stream alone (workload adanalytics_count, pmc_cal pass) against
its known byte count (the kernel's own dense-byte count, bench.py bytes_breakdown.dense_stream).  Usage:
  python scripts/pmc_summarize.py <tag> [workload]
"""
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("query_kernel", "query_kernel_direct", "query_kernel_rdirect")


def _is_query_kernel(name: str) -> bool:
    return "query_kernel" in name


def per_launch(path):
    rows = [r for r in csv.DictReader(open(path)) if _is_query_kernel(r["Kernel_Name"])]
    vals = [float(r["Counter_Value"]) * 1024.0 for r in rows]
    return sum(vals) / len(vals), len(vals)


def bench_json(log):
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def main():
    tag, wl = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "adanalytics"
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"kernel_stats_{wl}.csv"))
    fetch, n1 = per_launch(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"))
    write, n2 = per_launch(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"))
    avg_ns, kname = None, None
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        if _is_query_kernel(r["Name"]):
            avg_ns, kname = float(r["AverageNs"]), r["Name"]
    factor, cal = 2.0, None
    cal_csv = os.path.join(src, "pmc_cal", "run_counter_collection.csv")
    if os.path.exists(cal_csv):
        cal_fetch, _ = per_launch(cal_csv)
        b = bench_json(os.path.join(src, "pmc_cal.log"))
        known = b["roofline"]["bytes_breakdown"]["dense_stream"] if b else None
        if known:
            factor = known / cal_fetch
            cal = {"workload": "adanalytics_count", "known_stream_bytes": known, "fetch_size_bytes_raw": cal_fetch,
                   "factor": factor}
    try:
        commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                                text=True).stdout.strip() or "unknown"
    except OSError:
        commit = "unknown"
    out = {"workload": wl, "tag": tag, "kernel": kname, "commit": commit,
           "fetch_size_bytes_raw": fetch, "write_size_bytes": write, "launches": [n1, n2],
           "fetch_correction": factor, "calibration": cal,
           "hbm_bytes_per_launch": factor * fetch + write,
           "rocprof_avg_kernel_ns": avg_ns,
           "note": "fetch_correction x FETCH_SIZE + WRITE_SIZE per launch; the correction is measured on the "
                   "workload's filter stream alone (known bytes) when a calibration pass exists, else the guide's x2 "
                   "for 16-B/lane streams; the sparse sector gathers are other widths, so their share carries the "
                   "stream's factor"}
    with open(os.path.join(ROOT, "profiles", f"pmc_{wl}.json"), "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.join(dst, f"pmc_{wl}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
