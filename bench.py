"""Benchmark: rows/s of the filtered GROUP BY SUM segment query path on MI355X (BASELINE.json metric).

One step = one query over every segment this GPU owns (30 x 2^25-doc segments = 1B rows per GPU by default,
weak scaling: config 5 "AdAnalytics ... 8B rows sharded across 8xMI355X" at N=8), including the per-query plan
packing, the query kernel, the RCCL all-reduce of the partial group-by tables (N>1) and rank 0's compaction to
host results.  Segments are generated in HBM before timing (synthetic data, seeded; see pinot_amd/synth.py).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload adanalytics|range_in|groupby1m|bitmap5|...]
  torchrun --nproc-per-node N bench.py --gpus N ...       (one process per GPU, RCCL over xGMI)

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (query_kernel: algorithmic bytes per
launch / its HIP-event time) and the CPU baseline (oracle/pinot_cpu.c, Pinot's per-segment operators restated,
timed on a bounded sample on this host).  The default N=1 run also measures BASELINE.json configs 2-4 and the
SURVEY.md 8(d) variants (Zipf keys, inverted-indexed accountId) into a `workloads` sub-object, each with its own
ms/step, roofline and CPU baseline.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="adanalytics")
    ap.add_argument("--segments", type=int, default=0,
                    help="segments per GPU (0 = the workload's BASELINE size: 30, or 60 for groupby1m = 2B rows)")
    ap.add_argument("--docs", type=int, default=1 << 25, help="docs per segment")
    ap.add_argument("--cpu-sample-segments", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="repeat the CPU sample until this much time")
    ap.add_argument("--inflight", type=int, default=3,
                    help="queries in flight at N=1 (the host plans query i+1 while the GPU runs query i)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = Pinot default min(#seg, min(10, nproc/2))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the small GPU-vs-oracle check of this workload")
    ap.add_argument("--no-secondary", dest="secondary", action="store_false",
                    help="measure the headline workload only (default N=1 run: also configs 2-4 and variants)")
    ap.add_argument("--node", action="store_true",
                    help="drive --gpus devices from this one process through libpinotgpu's node combine "
                         "(pgpu_node_query_topk, RCCL inside the library: the one-JVM server's shape) instead of one "
                         "process per GPU")
    ap.add_argument("--full-out", default=os.environ.get("PGPU_BENCH_FULL", os.path.join("gpurun_out", "bench_full.json")),
                    help="file for the full per-workload records (the stdout line carries a compact summary)")
    return ap.parse_args(argv)


def available_cores() -> int:
    """CPU cores this process may use: its affinity set, capped by OMP_NUM_THREADS when the box sets a share."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else max(1, n)


def measure(ex, q, segs, steps, warmup, inflight, world, barrier):
    """Time `steps` whole queries (plan, launch, reduce, finish) with up to `inflight` in flight at N = 1;
    returns (ms_per_step over the max of ranks, average HIP-event kernel ms, last result).  The warmup runs the
    same pipeline for max(warmup, inflight) queries, so every workspace the timed region uses has been sized."""
    import torch
    import torch.distributed as dist

    def run(n):
        pending, kernel_ms, result, submitted = [], [], None, 0
        for _ in range(n):
            while submitted < n and len(pending) < max(1, inflight):
                pending.append(ex.submit(q, segs))
                submitted += 1
            result = ex.collect(pending.pop(0))
            kernel_ms.append(ex.last_stats.kernel_ms)
        return result, kernel_ms

    run(max(warmup, inflight if world == 1 else 1))
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    result, kernel_ms = run(steps)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed * 1000.0 / steps, sum(kernel_ms) / len(kernel_ms), result


def algorithmic_bytes(ex, pm, q, segs_by_dev, w, ids_by_dev, num_docs):
    """SURVEY.md 8(d) algorithmic bytes of the workload (tools/bytemodel.py: from the segments' dict ids and the
    reference's filter tree, the same figure whatever strategy the kernels pick), plus `bytes_read_model`: what this
    build's kernels read by their own stats pass (streamed tiles + 32-B sectors of their gathers + dictionaries +
    bitmaps + output), which moves with the strategy."""
    import torch

    from tools.bytemodel import output_bytes, workload_bytes

    segs = segs_by_dev[0]
    pm.collect_stats = True
    r = ex.execute(q, segs)
    st = ex.last_stats
    pm.collect_stats = False
    all_segs = [s for ss in segs_by_dev for s in ss]
    ngroups = len(r.group_rows or []) if r is not None else 1  # ranks != 0 return no rows
    dict_bytes = 0
    for c in sorted(set(a.column for a in q.aggregations if a.column)):
        width = {0: 4, 1: 8, 2: 4, 3: 8}.get(segs[0].column(c).data_type, 4)
        full = sum(s.column(c).cardinality * width for s in all_segs)
        dict_bytes += min(full, 32 * st.num_docs_scanned)
    out_bytes = output_bytes(ngroups, len(q.aggregations))
    bitmap_bytes = inverted_bytes_read(q, all_segs)
    read = st.dense_bytes + st.sparse_sector_bytes + dict_bytes + bitmap_bytes + out_bytes
    read_parts = {"dense_stream": st.dense_bytes, "sparse_sectors": st.sparse_sector_bytes,
                  "dictionaries": dict_bytes, "inverted_bitmaps": bitmap_bytes, "output": out_bytes}
    algo, parts, matched = 0, {}, 0
    here = torch.cuda.current_device()
    for ss, ids in zip(segs_by_dev, ids_by_dev):  # (node mode: every device's segments, on that device)
        dev = ss[0].ctx.device if len(segs_by_dev) > 1 else here
        torch.cuda.set_device(dev)
        a, pp, m = workload_bytes(w, q, ss, num_docs, ids, torch.device("cuda", dev), ngroups=ngroups)
        algo, matched = algo + a, matched + m
        for k, v in pp.items():
            parts[k] = parts.get(k, 0) + v
    torch.cuda.set_device(here)
    if matched != st.num_docs_scanned:  # the model regenerates the ids: it must see the docs the GPU matched
        raise RuntimeError(f"byte model matched {matched} docs, the GPU {st.num_docs_scanned}")
    return algo, st, parts, read, read_parts


def resident_bytes(ctx, segs, rows):
    """HBM held by the workload's segments on this GPU (pgpu_segment_device_bytes_ex): the reference's own indexes
    and the derived copies the table's policy builds (Workload.sliced_columns / value_planes_columns)."""
    kinds = {}
    for s in segs:
        for k, v in s.device_bytes_by_kind().items():
            kinds[k] = kinds.get(k, 0) + v
    derived = kinds["sliced"] + kinds["value_planes"]
    used, budget = ctx.derived_bytes()
    return {"resident_bytes_per_gpu": kinds["total"], "bytes_per_row": kinds["total"] / rows,
            "forward_index_bytes_per_row": kinds["forward"] / rows, "derived_bytes_per_row": derived / rows,
            "by_kind": kinds, "derived_budget_bytes": budget, "context_derived_bytes": used}


# pgpu_query_stats.kernel_variant -> the query kernel the runtime chose (and the kernels timed beside it)
KERNEL_NAMES = {0: "query_kernel (ring)", 1: "query_kernel_direct", 2: "query_kernel_rdirect", 3: "query_kernel_rstream",
                4: "query_kernel_rprog + invexp_kernel", 5: "query_kernel_rkey + rkey_ctab_kernel",
                6: "query_kernel_cand", 7: "part_scan_kernel + part_reduce_kernel",
                8: "query_kernel_rfsm + andfsm_segment_kernel"}


class NodeExecutor:
    """bench.py's executor interface (submit / collect / execute / last_stats) over pinot_amd.node.GpuNode: one
    process drives every device of the node and the partial tables merge over RCCL inside libpinotgpu
    (pgpu_node_submit / pgpu_node_collect: several node queries in flight, like the per-GPU path's)."""

    def __init__(self, node, segs_by_device):
        self.node = node
        self.segs_by_device = segs_by_device
        self.last_stats = None

    def execute(self, q, _segs=None):
        res = self.node.execute(q, self.segs_by_device)
        self.last_stats = res.stats
        return res

    def submit(self, q, _segs=None):
        return self.node.submit(q, self.segs_by_device)

    def collect(self, pending):
        res = self.node.collect(pending)
        self.last_stats = res.stats
        return res


class _Planners:
    """pm.collect_stats fanned out to every device's plan maker (node mode)."""

    def __init__(self, planners):
        object.__setattr__(self, "_pms", planners)

    def __setattr__(self, name, value):
        for pm in self._pms:
            setattr(pm, name, value)


def kernel_label(ex, opts) -> str:
    variant = getattr(ex.last_stats, "kernel_variant", -1)
    name = KERNEL_NAMES.get(variant, "query_kernel")
    if opts.get("exact_filter_stats") and variant != 8:
        name += " + andfsm_tile_kernel + andfsm_segment_kernel (or leafbits_kernel)"
    return name


def run_workload(name, ctx, args, world, rank, steps, warmup, segments, cpu_seconds, log, barrier, node=None):
    """Generate the workload's segments in HBM, measure it, time the CPU baseline beside it; returns the full
    record of one result (the compact line is built from it by compact_record).  `node` (a GpuNode) drives its
    devices from this process; the segments are then sharded over the node's devices as over ranks."""
    import torch
    from pinot_amd.combine import DistributedExecutor
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.query import parse_sql
    from pinot_amd.synth import WORKLOADS, build_segments_gpu

    w = WORKLOADS[name]
    nseg = segments or w.segments
    ndev = len(node.contexts) if node is not None else 1
    shards = list(range(ndev)) if node is not None else [rank]
    t0 = time.time()
    segs_by_dev, ids_by_dev = [], []
    for i, shard in enumerate(shards):
        dctx = node.contexts[i] if node is not None else ctx
        if node is not None:
            torch.cuda.set_device(dctx.device)
        ids = list(range(shard * nseg, (shard + 1) * nseg))
        segs_by_dev.append(build_segments_gpu(dctx, w, ids, args.docs))
        ids_by_dev.append(ids)
        torch.cuda.synchronize()
    if node is not None:
        torch.cuda.set_device(node.contexts[0].device)
    segs, seg_ids = segs_by_dev[0], ids_by_dev[0]
    gen_s = time.time() - t0
    log(f"{name}: generated {ndev} x {len(segs)} segments x {args.docs} docs in {gen_s:.1f}s")
    hbm = resident_bytes(ctx, segs, nseg * args.docs)
    log(f"{name}: resident {hbm['resident_bytes_per_gpu'] / 1e9:.2f} GB per GPU, {hbm['bytes_per_row']:.2f} B/row "
        f"({hbm['forward_index_bytes_per_row']:.2f} forward index, {hbm['derived_bytes_per_row']:.2f} derived)")
    opts = dict(w.options)
    q = parse_sql(w.sql)
    if node is not None:
        for pm_ in node.planners:
            for k, v in plan_options(opts).items():
                setattr(pm_, k, v)
        pm = _Planners(node.planners)
        ex = NodeExecutor(node, segs_by_dev)
    else:
        pm = GpuPlanMaker(ctx, **plan_options(opts))
        ex = DistributedExecutor(pm)
    try:
        algo_bytes, st, breakdown, read_bytes, read_breakdown = algorithmic_bytes(ex, pm, q, segs_by_dev, w,
                                                                                  ids_by_dev, args.docs)
        log(f"{name}: stats pass: {st.num_docs_scanned} matched, {algo_bytes / 1e9:.3f} GB algorithmic, "
            f"{read_bytes / 1e9:.3f} GB read by the kernels, {st.kernel_ms:.3f} ms")
        ms_per_step, avg_kernel_ms, result = measure(ex, q, segs, steps, warmup, args.inflight, world, barrier)
        rows_per_gpu = nseg * args.docs
        # per GPU: this rank's (or, in node mode, the average device's) algorithmic bytes over the span of the
        # kernels of one query on its stream (the slowest device's in node mode)
        achieved = algo_bytes / ndev / (avg_kernel_ms * 1e-3) / 1e9
        log(f"{name}: timed: {ms_per_step:.3f} ms/step, kernels {avg_kernel_ms:.3f} ms, {achieved:.0f} GB/s per GPU")
        cpu = check = None
        if rank == 0 and not args.no_cpu_baseline:
            cpu, check = cpu_baseline(ctx, w, q, opts, args, cpu_seconds, segs)
        traffic, traffic_src = _pmc_traffic(name)
        return {
            "value": rows_per_gpu * world * ndev / (ms_per_step * 1e-3),
            "ms_per_step": ms_per_step,
            "steps": steps,
            "n_gpus": world * ndev,
            "config": {"workload": name, "description": w.description, "query": w.sql,
                       "segments_per_gpu": nseg, "docs_per_segment": args.docs, "rows_per_gpu": rows_per_gpu,
                       "total_rows": rows_per_gpu * world * ndev,
                       "queries_in_flight": max(1, args.inflight),
                       "parallelism": (f"segments sharded over {ndev} GPU(s) of one process; partial tables merged "
                                       "over RCCL inside libpinotgpu (pgpu_node_query_topk)") if node is not None else
                                      (f"segments sharded over {world} GPU(s), one process each; partial tables "
                                       "merged over RCCL (torch.distributed)")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kernel_label(ex, opts),
                         "algorithmic_bytes_per_launch": algo_bytes / ndev,
                         "kernel_ms_avg": avg_kernel_ms,
                         "kernel_ms_definition": "HIP events on the query stream around every kernel that reads "
                                                 "the segments (leaf bitmaps, query kernel, group-by phases, "
                                                 "filter-statistic kernels)",
                         "bytes_breakdown": breakdown,
                         "bytes_definition": "SURVEY 8(d) workload bytes (tools/bytemodel.py), strategy-independent",
                         "bytes_read_model": read_bytes, "bytes_read_breakdown": read_breakdown},
            "cpu_baseline": cpu,
            "result": {"matched_docs_per_gpu": st.num_docs_scanned // ndev,
                       "groups": (len(result.group_rows) if result and result.group_rows is not None else None),
                       "rows": [list(r) for r in (result.rows[:3] if result else [])]},
            "parity_check": check,
            "hbm": hbm,
            "setup_s": round(gen_s, 1),
        }
    finally:
        for ss in segs_by_dev:
            for s in ss:
                s.release()


# Secondary workloads measured after the headline in the default run (BASELINE.json configs 2-4 and the SURVEY 8(d)
# variants): (name, steps, warmup, segments per GPU or 0 = the workload's own, CPU sample seconds)
SECONDARY = [("range_in", 10, 2, 0, 3.0), ("groupby1m", 5, 1, 0, 3.0), ("bitmap5", 10, 2, 0, 3.0),
             ("groupby1m_zipf", 5, 1, 0, 3.0), ("adanalytics_inv", 10, 2, 0, 3.0), ("adanalytics_exact", 10, 2, 0, 2.0),
             ("adanalytics_8b", 5, 1, 0, 2.0)]


METRIC = "rows/sec for filtered GROUP BY SUM at 1/8 GPUs + achieved HBM GB/s vs peak"
ROOFLINE_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_source", "kernel", "kernel_ms_avg",
                 "algorithmic_bytes_per_launch")
LINE_LIMIT = 6000  # the driver keeps the last 8000 characters of stdout: the line must fit well inside them


def compact_cpu(cpu):
    if not cpu:
        return None
    out = {k: cpu[k] for k in ("value", "unit", "cores", "kind") if k in cpu}
    out["sample"] = cpu.get("sample_short", "")
    if cpu.get("all_cores"):
        out["all_cores"] = {"value": cpu["all_cores"]["value"], "cores": cpu["all_cores"]["cores"]}
    return out


def compact_workload(rec):
    """name -> {ms_per_step, kernel_ms, frac, traffic_ratio, parity_ok, cpu_rows_s} of one secondary workload."""
    if "error" in rec:
        return {"error": rec["error"][:160]}
    rl = rec["roofline"]
    algo = rl.get("algorithmic_bytes_per_launch") or 0
    chk = rec.get("parity_check")
    return {"ms_per_step": round(rec["ms_per_step"], 4), "kernel_ms": round(rl["kernel_ms_avg"], 4),
            "frac": round(rl["frac"], 4),
            "traffic_ratio": round(rl["traffic"] / algo, 3) if rl.get("traffic") and algo else None,
            "parity_ok": None if chk is None else bool(chk.get("ok")),
            "cpu_rows_s": (rec.get("cpu_baseline") or {}).get("value")}


def compact_line(head, workloads, args, n_gpus):
    """The ONE stdout JSON line: the headline with roofline and cpu_baseline, the secondary workloads as a compact
    map; the full records go to --full-out."""
    chk = head.get("parity_check")
    cfg = head["config"]
    line = {
        "metric": METRIC,
        "value": head["value"],
        "unit": "rows/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (seeded dict ids generated in HBM)",
        "config": {"workload": cfg["workload"], "segments_per_gpu": cfg["segments_per_gpu"],
                   "docs_per_segment": cfg["docs_per_segment"], "total_rows": cfg["total_rows"],
                   "queries_in_flight": cfg["queries_in_flight"],
                   "parallelism": ("node" if args.node else "dp") + str(n_gpus)},
        "roofline": {k: head["roofline"].get(k) for k in ROOFLINE_KEYS},
        "cpu_baseline": compact_cpu(head.get("cpu_baseline")),
        "parity_ok": None if chk is None else bool(chk.get("ok")),
        "matched_docs_per_gpu": head["result"]["matched_docs_per_gpu"],
        "full_records": args.full_out,
    }
    if workloads:
        line["workloads"] = {k: compact_workload(v) for k, v in workloads.items()}
    return line


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` started without a launcher: one child process per GPU with the torch.distributed
    environment a launcher would set (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), started
    before this process touches the GPU (device_count() does not initialise it); rank 0 prints the line.  Returns
    the worst child exit status; fewer than N visible devices is an error."""
    import subprocess
    import torch

    have = torch.cuda.device_count()
    if have < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but {have} GPU(s) are visible", file=sys.stderr, flush=True)
        return 2
    port = free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        for p in procs:
            rc = max(rc, p.wait())
            if rc:
                break
    finally:
        for p in procs:  # a failed rank leaves the others blocked in a collective: stop exactly our children
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
    return rc


def main(argv=None):
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not args.node:
        return spawn_ranks(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    log = (lambda *a: print(f"[bench rank {rank}]", *a, file=sys.stderr, flush=True))
    if world > 1 and args.gpus != world:
        log(f"--gpus {args.gpus} but WORLD_SIZE={world}: measuring {world} ranks")
    local %= max(1, torch.cuda.device_count())  # > 1 rank per GPU only in the gloo rehearsal
    if world > 1:
        torch.cuda.set_device(local)
        # PGPU_DIST_BACKEND=gloo rehearses the multi-rank path on one GPU (RCCL needs one GPU per rank)
        backend = os.environ.get("PGPU_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()  # the ranks the process group actually formed
    torch.cuda.set_device(local)

    from pinot_amd.segment import GpuContext

    node = None
    if args.node:
        if world > 1:
            raise SystemExit("--node drives every GPU from one process: start it without a launcher")
        from pinot_amd.node import GpuNode
        have = torch.cuda.device_count()
        if have < args.gpus:
            log(f"--gpus {args.gpus} but {have} GPU(s) are visible")
            return 2
        node = GpuNode(list(range(args.gpus)))
        ctx = node.contexts[0]
    else:
        ctx = GpuContext(local)

    def barrier():
        if world > 1:
            dist.barrier()

    head = run_workload(args.workload, ctx, args, world, rank, args.steps, args.warmup, args.segments,
                        args.cpu_seconds, log, barrier, node=node)
    workloads = {}
    if args.secondary and world == 1 and node is None and args.workload == "adanalytics":
        for name, steps, warmup, nseg, cpu_s in SECONDARY:
            try:
                workloads[name] = run_workload(name, ctx, args, world, rank, steps, warmup, nseg, cpu_s, log, barrier)
            except Exception as e:  # a secondary workload never hides the headline line
                log(f"{name}: failed: {e!r}")
                workloads[name] = {"error": repr(e)}
    if rank == 0:
        full = {"headline": head, "workloads": workloads}
        try:
            os.makedirs(os.path.dirname(os.path.abspath(args.full_out)), exist_ok=True)
            with open(args.full_out, "w") as f:
                json.dump(full, f, default=float, indent=1)
        except OSError as e:
            log(f"full records not written: {e!r}")
        line = compact_line(head, workloads, args, head["n_gpus"])
        text = json.dumps(line, default=float, separators=(",", ":"))
        if len(text) > LINE_LIMIT:  # never let the line outgrow the driver's stdout tail
            line.pop("workloads", None)
            text = json.dumps(line, default=float, separators=(",", ":"))
        print(text, flush=True)
    if node is not None:
        node.close()
    else:
        ctx.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


def _pmc_traffic(workload):
    """HBM bytes per launch measured by rocprofv3 PMC (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) from the
    committed measurement of this workload under profiles/, and where / at which commit it was measured (so a
    figure that predates a kernel change is visibly stale).  (None, None) when there is none."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if os.path.exists(p):
        try:
            with open(p) as f:
                d = json.load(f)
            return d.get("hbm_bytes_per_launch"), f"profiles/pmc_{workload}.json @ {d.get('commit', 'unknown')}"
        except Exception:
            return None, None
    return None, None


def inverted_bytes_read(q, segs):
    """Serialized bytes of every inverted-index bitmap the planned INV leaves read: per
    segment, the bitmaps of the matching (or, for exclusive predicates, non-matching) dict ids."""
    import numpy as np
    from pinot_amd.plan import SegmentFilterPlanner

    total = 0
    for s in segs:
        stack = [SegmentFilterPlanner(s).build(q.filter)] if q.filter is not None else []
        while stack:
            op = stack.pop()
            stack.extend(op.children)
            if op.kind != "INV":
                continue
            ev = op.evaluator
            ids = ev.non_matching_dict_ids() if ev.is_exclusive else ev.matching_dict_ids()
            inv = s.column(op.column).inverted
            offs = np.frombuffer(inv, dtype=">i4", count=s.column(op.column).cardinality + 1).astype(np.int64)
            total += int(sum(offs[i + 1] - offs[i] for i in ids))
    return total


# Looser variants of the bench queries (same plan shapes) so the parity sample matches rows, not only zero.
PARITY_VARIANTS = {"adanalytics": ("accountId IN (123456789)", "accountId < 123456789"),
                   "adanalytics_8b": ("accountId IN (123456789)", "accountId < 123456789"),
                   "adanalytics_exact": ("accountId IN (123456789)", "accountId < 123456789")}


def plan_options(opts):
    """GpuPlanMaker settings of a workload: numGroupsLimit and the server's ORDER BY trim (config 4 runs with
    minServerGroupTrimSize = -1, SURVEY.md 8(d): every group comes back, so the result is exact)."""
    return {"num_groups_limit": opts.get("num_groups_limit", 100_000),
            "min_server_group_trim_size": opts.get("min_server_group_trim_size", 5000),
            "exact_filter_stats": opts.get("exact_filter_stats", False)}


def parity_check(ctx, w, q, opts):
    """GPU vs oracle on 2 small segments of the workload: the bench query and a looser variant of it
    (called from the CPU leg only).  With the server trim off the GPU returns every group, compared as a set
    with the oracle's; with it on, the final ORDER BY / LIMIT rows must be equal and every returned group must
    be one of the oracle's groups with the same values (the trim keeps a subset of the table)."""
    from oracle import engine
    from oracle.segment_writer import pack_fixed_bit
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.query import parse_sql
    from pinot_amd.segment import GpuSegment
    from pinot_amd.synth import build_segment_cpu

    n = 1 << 19
    segs = [build_segment_cpu(w, s, n, pack_fixed_bit) for s in range(2)]
    gs = [GpuSegment(ctx, s) for s in segs]
    queries = [q]
    if w.name in PARITY_VARIANTS:
        a, b = PARITY_VARIANTS[w.name]
        queries.append(parse_sql(w.sql.replace(a, b)))
    po = plan_options(opts)
    out = {"docs": 2 * n, "matched": [], "groups": [], "ok": True,
           "compared": "all groups" if po["min_server_group_trim_size"] <= 0 else "ORDER BY/LIMIT rows + group subset"}
    try:
        for qq in queries:
            res = GpuPlanMaker(ctx, **po).execute(qq, gs)
            ref = engine.execute(qq, segs, num_groups_limit=po["num_groups_limit"],
                                 iterator_stats=po["exact_filter_stats"])
            if qq.group_by:
                got, exp = res.group_rows, ref.group_rows
                if po["min_server_group_trim_size"] <= 0:
                    ok = sorted(got) == sorted(exp)
                else:
                    ok = set(got) <= set(exp) and list(res.rows) == list(ref.rows)
                out["groups"].append(len(got))
            else:
                ok = list(res.aggregation_result) == list(ref.aggregation_result)
            ok = ok and res.stats.num_docs_scanned == ref.num_docs_scanned
            if po["exact_filter_stats"]:  # the reference's numEntriesScannedInFilter (iterator replay)
                ok = ok and res.stats.num_entries_scanned_in_filter == ref.num_entries_scanned_in_filter
            out["matched"].append(ref.num_docs_scanned)
            out["ok"] = bool(out["ok"] and ok)
        return out
    finally:
        for g in gs:
            g.release()


def cpu_baseline(ctx, w, q, opts, args, seconds, gpu_segs):
    """The CPU leg: (1) Pinot's per-segment operators restated in C (oracle/pinot_cpu.c) timed on this host,
    the sample's segments queried repeatedly until ~`seconds` of wall time, at Pinot's default task count and
    with every available core; (2) the GPU-vs-oracle parity check (parity_check) on small segments, and (3) at full
    size: the GPU over the same full-size segments the C port just timed, compared with the C port's results."""
    check = None if args.no_check else parity_check(ctx, w, q, opts)
    cpu, last = c_baseline(w, q, args, seconds)
    if check is not None:
        full = full_size_check(ctx, w, q, opts, args, gpu_segs, last)
        check["full_size"] = bool(full.get("ok"))
        check["full_size_detail"] = full
        check["ok"] = bool(check["ok"] and full.get("ok"))
    return cpu, check


def full_size_check(ctx, w, q, opts, args, gpu_segs, cport):
    """The GPU over the first `cpu_sample_segments` full-size segments of this rank (the ones the C port timed:
    same generator, same seeds), against the C port's matched docs, per-key counts and sums (double
    accumulators, exact for these integer inputs < 2^53): integers bit-exact, every group compared."""
    import numpy as np

    from pinot_amd.plan import GpuPlanMaker

    nseg = min(args.cpu_sample_segments, len(gpu_segs))
    matched, counts, sums = cport
    res = GpuPlanMaker(ctx, **plan_options(opts)).execute(q, gpu_segs[:nseg])
    out = {"segments": nseg, "docs": nseg * args.docs, "matched": int(matched),
           "gpu_matched": int(res.stats.num_docs_scanned)}
    ok = res.stats.num_docs_scanned == matched
    aggs = q.aggregations

    def expect(a, ai, key):
        cnt = int(counts[key])
        if a.function == "COUNT":
            return cnt
        v = float(sums[ai][key])
        return v / cnt if a.function == "AVG" else v

    if not q.group_by:
        exp = [expect(a, ai, 0) for ai, a in enumerate(aggs)] if matched else None
        got = list(res.aggregation_result)
        ok = ok and (exp is None or all(float(g) == float(e) for g, e in zip(got, exp)))
        out["compared"] = "aggregation values"
    else:
        values = {c.name: c.values() for c in w.columns}
        gvals = values[q.group_by[0]]
        live = np.flatnonzero(counts)
        rows = {tuple(r[:1]): r[1:] for r in res.group_rows}
        ok = ok and len(rows) == len(live) and len(q.group_by) == 1
        bad = 0
        for key in live.tolist():
            r = rows.get((int(gvals[key]),))
            if r is None or any(float(g) != float(expect(a, ai, key)) for ai, (a, g) in enumerate(zip(aggs, r))):
                bad += 1
        ok = ok and bad == 0
        out.update({"groups": int(len(live)), "gpu_groups": len(rows), "mismatched_groups": bad,
                    "compared": "every group"})
    out["ok"] = bool(ok)
    return out


def c_baseline(w, q, args, seconds):
    """the C port at Pinot's default parallelism (one task per segment, min(#segments,
    min(10, nproc/2)) threads, CombineOperatorUtils.getNumTasksForQuery) over `cpu_sample_segments` segments, then
    with every core this process may use over as many segments as cores (one task per segment, so the sample
    must hold at least that many for every core to work)."""
    from oracle.cpu import CpuBaseline, synth_segment

    nproc = os.cpu_count() or 1
    cores = available_cores()
    nseg = args.cpu_sample_segments
    segs = [synth_segment(w, s, args.docs) for s in range(max(nseg, cores))]
    threads = args.cpu_threads or max(1, min(nseg, min(10, nproc // 2)))
    cb = CpuBaseline(q, segs[:nseg])
    filt = ("doc-id set algebra of AndDocIdSet / OrDocIdSet over Roaring / sorted / scan leaves" if cb.q.num_nodes
            else "AndDocIdIterator over SVScanDocIdIterators")

    last = []

    def timed(c, th, n, budget):
        total, runs = 0.0, 0
        while runs == 0 or total < budget:
            dt, matched, counts, sums, _ = c.run(th)
            total += dt
            runs += 1
        last[:] = [matched, counts, sums]
        return runs * n * args.docs / total, runs, total

    value, runs, total = timed(cb, threads, nseg, seconds)
    first = list(last)
    all_cb = cb if len(segs) == nseg else CpuBaseline(q, segs)
    all_value, all_runs, all_total = timed(all_cb, cores, len(segs), max(1.0, seconds / 2))
    skew = "" if all(c.dist == "uniform" for c in w.columns) else ", Zipf keys from the same CDF as the GPU's"
    return ({"value": value, "unit": "rows/s", "cores": threads, "kind": "port",
             "sample_short": f"{runs} run(s) x {nseg} seg x {args.docs} docs, oracle/pinot_cpu.c, {threads} threads "
                             f"(Pinot default), nproc={nproc}",
            "sample": f"{runs} run(s) over {nseg} segment(s) x {args.docs} docs of the same workload{skew}, "
                      f"oracle/pinot_cpu.c ({filt}, 10k-doc blocks, double SUM), "
                      f"{threads} thread(s) = Pinot default min(#segments, min(10, nproc/2)), nproc={nproc}",
            "seconds": total,
            "all_cores": {"value": all_value, "cores": cores, "available_cores": cores, "segments": len(segs),
                          "runs": all_runs, "seconds": all_total}}, first)


if __name__ == "__main__":
    sys.exit(main())
