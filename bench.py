"""Benchmark: rows/s of the filtered GROUP BY SUM segment query path on MI355X (BASELINE.json metric).

One step = one query over every segment this GPU owns (30 x 2^25-doc segments = 1B rows per GPU by default,
weak scaling: config 5 "AdAnalytics ... 8B rows sharded across 8xMI355X" at N=8), including the per-query plan
packing, the query kernel, the RCCL all-reduce of the partial group-by tables (N>1) and rank 0's compaction to
host results.  Segments are generated in HBM before timing (synthetic data, seeded; see pinot_amd/synth.py).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload adanalytics|range_in|groupby1m]
  torchrun --nproc-per-node N bench.py --gpus N ...       (one process per GPU, RCCL over xGMI)

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (query_kernel: algorithmic bytes per
launch / its HIP-event time) and the CPU baseline (oracle/pinot_cpu.c, Pinot's per-segment operators restated,
timed on a bounded sample on this host).
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


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
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
    return ap.parse_args()


def main():
    args = parse_args()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local %= max(1, torch.cuda.device_count())  # > 1 rank per GPU only in the gloo rehearsal
    if world > 1:
        torch.cuda.set_device(local)
        # PGPU_DIST_BACKEND=gloo rehearses the multi-rank path on one GPU (RCCL needs one GPU per rank)
        backend = os.environ.get("PGPU_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)

    from pinot_amd.combine import DistributedExecutor
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.query import parse_sql
    from pinot_amd.segment import GpuContext
    from pinot_amd.synth import WORKLOADS, build_segments_gpu

    w = WORKLOADS[args.workload]
    if args.segments <= 0:
        args.segments = w.segments
    log = (lambda *a: print(f"[bench rank {rank}]", *a, file=sys.stderr, flush=True))
    ctx = GpuContext(local)
    seg_ids = list(range(rank * args.segments, (rank + 1) * args.segments))
    t0 = time.time()
    segs = build_segments_gpu(ctx, w, seg_ids, args.docs)
    torch.cuda.synchronize()
    gen_s = time.time() - t0
    log(f"generated {len(segs)} segments x {args.docs} docs in {gen_s:.1f}s")
    opts = dict(w.options)
    q = parse_sql(w.sql)
    pm = GpuPlanMaker(ctx, num_groups_limit=opts.get("num_groups_limit", 100_000))
    ex = DistributedExecutor(pm)

    def barrier():
        if world > 1:
            dist.barrier()

    # algorithmic bytes of one launch (stats pass: dense tile bytes + touched 32-B sectors of sparse reads)
    pm.collect_stats = True
    r_stats = ex.execute(q, segs)
    st = ex.last_stats
    pm.collect_stats = False
    # forward-index bytes (dense tiles + 32-B sectors of sparse reads, exact from the kernel's
    # stats) + dictionary bytes read once per segment per query (bounded by one 32-B sector per matched doc
    # when few docs match) + output bytes
    dict_bytes = 0
    for c in sorted(set(a.column for a in q.aggregations if a.column)):
        width = {0: 4, 1: 8, 2: 4, 3: 8}.get(segs[0].column(c).data_type, 4)
        full = sum(s.column(c).cardinality * width for s in segs)
        dict_bytes += min(full, 32 * st.num_docs_scanned)
    ngroups = len(r_stats.group_rows or []) if r_stats is not None else 1  # ranks != 0 return no rows
    out_bytes = 8 * max(1, ngroups) * (1 + len(q.aggregations))
    bitmap_bytes = inverted_bytes_read(q, segs)
    algo_bytes = st.dense_bytes + st.sparse_sector_bytes + dict_bytes + bitmap_bytes + out_bytes

    log(f"stats pass: {st.num_docs_scanned} matched, {algo_bytes / 1e9:.3f} GB algorithmic, {st.kernel_ms:.3f} ms")
    for _ in range(args.warmup):
        ex.execute(q, segs)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    kernel_ms = []
    t_start = time.perf_counter()
    result = None
    # every step plans, launches, reduces (N > 1: RCCL all-reduce of the partial tables) and finishes one whole
    # query; up to `inflight` are queued at once, so the host side of query i overlaps the GPU running query i+1
    pending = []
    submitted = 0
    for _ in range(args.steps):
        while submitted < args.steps and len(pending) < max(1, args.inflight):
            pending.append(ex.submit(q, segs))
            submitted += 1
        result = ex.collect(pending.pop(0))
        kernel_ms.append(ex.last_stats.kernel_ms)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1000.0 / args.steps
    rows_per_gpu = args.segments * args.docs
    total_rows = rows_per_gpu * world
    value = total_rows / (elapsed / args.steps)

    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    achieved = algo_bytes / (avg_kernel_ms * 1e-3) / 1e9

    # small parity check of the same workload against the oracle (2 x 2^18-doc segments)
    log(f"timed: {ms_per_step:.3f} ms/step, kernel {avg_kernel_ms:.3f} ms, {achieved:.0f} GB/s")
    # the CPU leg (the only one that touches oracle/): Pinot's operators restated on the CPU, timed on this host,
    # and a GPU-vs-CPU check of the same workload on small segments
    check = cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu, check = cpu_baseline(ctx, w, q, opts, args)

    if rank == 0:
        traffic = _pmc_traffic(args.workload)
        line = {
            "metric": "rows/sec for filtered GROUP BY SUM at 1/8 GPUs + achieved HBM GB/s vs peak",
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded dict ids generated in HBM; dictionaries per BASELINE.md section 3)",
            "config": {"workload": args.workload, "description": w.description, "query": w.sql,
                       "segments_per_gpu": args.segments, "docs_per_segment": args.docs,
                       "rows_per_gpu": rows_per_gpu, "total_rows": total_rows,
                       "queries_in_flight": max(1, args.inflight),
                       "parallelism": f"segments sharded over {world} GPU(s); partial tables all-reduced over RCCL"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "query_kernel", "algorithmic_bytes_per_launch": algo_bytes,
                         "kernel_ms_avg": avg_kernel_ms,
                         "bytes_breakdown": {"dense_stream": st.dense_bytes, "sparse_sectors": st.sparse_sector_bytes,
                                             "dictionaries": dict_bytes, "inverted_bitmaps": bitmap_bytes,
                                             "output": out_bytes}},
            "cpu_baseline": cpu,
            "result": {"matched_docs_per_gpu": st.num_docs_scanned, "groups": (len(result.group_rows)
                       if result and result.group_rows is not None else None),
                       "rows": [list(r) for r in (result.rows[:3] if result else [])]},
            "parity_check": check,
            "setup_s": round(gen_s, 1),
        }
        print(json.dumps(line, default=float), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def _pmc_traffic(workload):
    """HBM bytes per launch measured by rocprofv3 PMC (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), when a
    committed measurement for this workload exists under profiles/."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if os.path.exists(p):
        try:
            with open(p) as f:
                return json.load(f).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


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
PARITY_VARIANTS = {"adanalytics": ("accountId IN (123456789)", "accountId < 123456789")}


def parity_check(ctx, w, q, opts):
    """GPU vs oracle on 2 small segments of the workload: the bench query and a looser variant of it
    (called from the CPU leg only)."""
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
    out = {"docs": 2 * n, "matched": [], "ok": True}
    try:
        for qq in queries:
            res = GpuPlanMaker(ctx, num_groups_limit=opts.get("num_groups_limit", 100_000)).execute(qq, gs)
            ref = engine.execute(qq, segs, num_groups_limit=opts.get("num_groups_limit", 100_000))
            if qq.group_by:
                ok = sorted(res.group_rows) == sorted(ref.group_rows)
            else:
                ok = list(res.aggregation_result) == list(ref.aggregation_result)
            ok = ok and res.stats.num_docs_scanned == ref.num_docs_scanned
            out["matched"].append(ref.num_docs_scanned)
            out["ok"] = bool(out["ok"] and ok)
        return out
    finally:
        for g in gs:
            g.release()


def cpu_baseline(ctx, w, q, opts, args):
    """The CPU leg: (1) Pinot's per-segment operators restated in C (oracle/pinot_cpu.c) timed on this host,
    the sample's segments queried repeatedly until ~args.cpu_seconds of wall time with Pinot's default task
    count; filters the C port does not cover (OR / NOT / index leaves) time the numpy restatement
    (oracle/engine.py) instead; (2) the GPU-vs-oracle parity check (parity_check)."""
    check = None if args.no_check else parity_check(ctx, w, q, opts)
    from oracle import cpu as ocpu

    try:
        ocpu._leaves(q.filter)
    except ValueError:
        return engine_baseline(w, q, opts, args), check
    return c_baseline(w, q, args), check


def engine_baseline(w, q, opts, args):
    from oracle import engine
    from oracle.segment_writer import pack_fixed_bit
    from pinot_amd.synth import build_segment_cpu

    nseg, n = 2, 1 << 21
    segs = [build_segment_cpu(w, s, n, pack_fixed_bit) for s in range(nseg)]
    total, runs = 0.0, 0
    while runs == 0 or total < args.cpu_seconds:
        t = time.perf_counter()
        engine.execute(q, segs, num_groups_limit=opts.get("num_groups_limit", 100_000))
        total += time.perf_counter() - t
        runs += 1
    return {"value": runs * nseg * n / total, "unit": "rows/s", "cores": 1, "kind": "port",
            "sample": f"{runs} run(s) over {nseg} segment(s) x {n} docs of the same workload, oracle/engine.py "
                      f"(numpy restatement of the filter operator tree incl. bitmap / sorted-index leaves; the C "
                      f"port covers AND-of-scan filters only), 1 thread",
            "seconds": total}


def c_baseline(w, q, args):
    from oracle.cpu import CpuBaseline, synth_segment

    nseg = args.cpu_sample_segments
    segs = [synth_segment(w, s, args.docs) for s in range(nseg)]
    nproc = os.cpu_count() or 1
    threads = args.cpu_threads or max(1, min(nseg, min(10, nproc // 2)))
    cb = CpuBaseline(q, segs)
    total, runs = 0.0, 0
    while runs == 0 or total < args.cpu_seconds:
        dt, matched, _, _, _ = cb.run(threads)
        total += dt
        runs += 1
    return {"value": runs * nseg * args.docs / total, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"{runs} run(s) over {nseg} segment(s) x {args.docs} docs of the same workload, "
                      f"oracle/pinot_cpu.c (AndDocIdIterator over SVScanDocIdIterators, 10k-doc blocks, double SUM), "
                      f"{threads} thread(s) = Pinot default min(#segments, min(10, nproc/2)), nproc={nproc}",
            "seconds": total}


if __name__ == "__main__":
    main()
