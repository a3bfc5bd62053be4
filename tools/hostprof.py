"""Host-side cost of one query, by phase (GPU box): filter_expr, build_desc, table layout, the submit call, the
collect call and the finish -- each timed over many repetitions of a bench workload's query on small segments.

    python tools/hostprof.py [workload] [segments] [docs] [reps]
"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from pinot_amd import _lib
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.query import parse_sql
    from pinot_amd.segment import GpuContext
    from pinot_amd.synth import WORKLOADS, build_segments_gpu

    name = sys.argv[1] if len(sys.argv) > 1 else "adanalytics_inv"
    nseg = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    docs = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2000
    ctx = GpuContext(0)
    w = WORKLOADS[name]
    segs = build_segments_gpu(ctx, w, list(range(nseg)), docs)
    torch.cuda.synchronize()
    q = parse_sql(w.sql)
    pm = GpuPlanMaker(ctx)
    for _ in range(20):
        pm.collect(pm.submit(q, segs))
    t = {k: 0.0 for k in ("filter_expr", "build_desc", "layout", "trim_order", "submit_call", "matched", "collect",
                          "total")}
    for _ in range(reps):
        t0 = time.perf_counter()
        expr = pm.filter_expr(q, segs)
        t1 = time.perf_counter()
        desc, keep, globals_ = pm.build_desc(q, segs, plan_filters=expr is None)
        t2 = time.perf_counter()
        L = pm.layout(desc)
        t3 = time.perf_counter()
        order = pm.trim_order(q, globals_)
        t4 = time.perf_counter()
        h = C.c_void_p()
        _lib.check(ctx._lib.pgpu_query_submit_ordered(
            ctx.handle, C.byref(desc), expr[0] if expr is not None else None, expr[1] if expr is not None else 0,
            C.byref(order) if order is not None else None, C.byref(h)))
        t5 = time.perf_counter()
        import numpy as np
        from pinot_amd.plan import PendingQuery
        pq = PendingQuery(pm, q, len(segs), h, L, globals_)
        pq.order = order
        pq.matched = np.zeros(max(1, len(segs)), dtype=np.uint8)
        _lib.check(ctx._lib.pgpu_query_matched_segments(h, pq.matched.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                        len(segs)))
        t6 = time.perf_counter()
        pm.collect(pq)
        t7 = time.perf_counter()
        for k, a, b in (("filter_expr", t0, t1), ("build_desc", t1, t2), ("layout", t2, t3), ("trim_order", t3, t4),
                        ("submit_call", t4, t5), ("matched", t5, t6), ("collect", t6, t7), ("total", t0, t7)):
            t[k] += b - a
    print(f"{name}: {nseg} segments x {docs} docs, {reps} queries, us per query:")
    for k, v in t.items():
        print(f"  {k:12s} {1e6 * v / reps:8.1f}")
    for s in segs:
        s.release()


if __name__ == "__main__":
    main()
