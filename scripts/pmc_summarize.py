"""Summarise a scripts/pmc.sh run (its gpurun_out/<tag>_<workload>) into profiles/<tag>/ and profiles/pmc_<workload>.json.

HBM bytes per query-kernel launch = c x FETCH_SIZE + WRITE_SIZE (KiB counters).  MI355X_MICROARCH.md "HBM": FETCH_SIZE
reads exactly half the bytes of a 16-B/lane streaming read (c = 2 there) and other access widths are uncalibrated --
"calibrate on a known byte count in your own access pattern".  The register-direct stream loads 4 B per lane, so
`c` is measured: the FETCH_SIZE of config 5's filter stream alone (workload adanalytics_count, pmc_cal pass) against
its known byte count (the kernel's own dense-byte count, bench.py bytes_breakdown.dense_stream).  Usage:
  python scripts/pmc_summarize.py <tag> [workload]
"""
import csv
import re
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the kernels inside the query's timed region (pgpu_runtime.cpp: HIP events ev0..ev1): leaf bitmaps, the query kernel
# or the partitioned group-by's phases (its sampling and planning passes included), the exact filter statistic's
TIMED = ("rawpred_kernel", "mvpred_kernel", "invexp_kernel", "rkey_ctab_kernel", "progbits_kernel", "query_kernel", "part_scan_kernel",
         "part_plan_kernel", "part_reduce_kernel", "andfsm_tile_kernel", "andfsm_segment_kernel", "leafbits_kernel")


def _base(name: str) -> str:
    """The kernel's own identifier in a demangled name ("void (anonymous namespace)::part_scan_kernel<false>(DevParams)"
    -> "part_scan_kernel")."""
    for m in re.finditer(r"([A-Za-z_][A-Za-z0-9_]*)(?:<[^()]*>)?\(", name):
        if m.group(1) not in ("anonymous", "void"):
            return m.group(1)
    return name


def _is_timed(name: str) -> bool:
    b = _base(name)
    return b in TIMED or b.startswith("query_kernel")


def _is_main(name: str) -> bool:
    """One launch per query: the query kernel, or phase 1 proper of the partitioned group-by."""
    b = _base(name)
    return b.startswith("query_kernel") or (b == "part_scan_kernel" and "<false" in name)


def per_launch(path):
    """(counter bytes per query over the timed kernels, queries)."""
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["Counter_Value"]) * 1024.0 for r in rows if _is_timed(r["Kernel_Name"]))
    # a kernel's counter rows: one per dispatch (per-dispatch aggregation of the counter)
    queries = len({r.get("Dispatch_Id", i) for i, r in enumerate(rows) if _is_main(r["Kernel_Name"])})
    return total / max(1, queries), queries


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
    avg_ns, kname, calls, per_kernel = 0.0, None, 0, {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        if _is_timed(r["Name"]):
            per_kernel[_base(r["Name"]) + ("<false>" if "<false" in r["Name"] else "<true>" if "<true" in r["Name"] else "")] = {
                "calls": int(r["Calls"]), "total_ns": float(r["TotalDurationNs"]), "avg_ns": float(r["AverageNs"])}
            avg_ns += float(r["TotalDurationNs"])
        if _is_main(r["Name"]):
            kname, calls = r["Name"], calls + int(r["Calls"])
    avg_ns = avg_ns / max(1, calls)
    factor, cal = 2.0, None
    cal_csv = os.path.join(src, "pmc_cal", "run_counter_collection.csv")
    if os.path.exists(cal_csv):
        cal_fetch, _ = per_launch(cal_csv)
        full = os.path.join(src, "pmc_cal.json")  # bench.py --full-out: the full records (the stdout line is compact)
        if os.path.exists(full):
            rl = json.load(open(full))["headline"]["roofline"]
        else:
            b = bench_json(os.path.join(src, "pmc_cal.log"))
            rl = b["roofline"] if b else {}
        # the filter stream's known bytes: the kernel's read model (the byte model's full first-leaf stream)
        known = (rl.get("bytes_read_breakdown") or {}).get("dense_stream") or \
            (rl.get("bytes_breakdown") or {}).get("forward_full")
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
           "rocprof_avg_kernel_ns": avg_ns, "rocprof_kernels": per_kernel,
           "note": "fetch_correction x FETCH_SIZE + WRITE_SIZE per query over the kernels of its timed region (TIMED); the correction is measured on the "
                   "workload's filter stream alone (known bytes) when a calibration pass exists, else the guide's x2 "
                   "for 16-B/lane streams; the sparse sector gathers are other widths, so their share carries the "
                   "stream's factor"}
    with open(os.path.join(ROOT, "profiles", f"pmc_{wl}.json"), "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.join(dst, f"pmc_{wl}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))
    for extra in ("pmc_lds", "pmc_sq"):  # optional SQ counter passes, copied beside the summary
        d = os.path.join(src, extra)
        if os.path.isdir(d):
            rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
            keep = [r for r in rows if _is_timed(r["Kernel_Name"])]  # the query's kernels only
            if keep:
                with open(os.path.join(dst, f"{extra}_{wl}.csv"), "w", newline="") as o:
                    wr = csv.DictWriter(o, fieldnames=list(keep[0].keys()))
                    wr.writeheader()
                    wr.writerows(keep)


if __name__ == "__main__":
    main()
