"""cProfile of GpuPlanMaker.submit (host planning + pgpu_query_submit) at pipeline depth 3."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import ctypes as C
    import torch
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.query import parse_sql
    from pinot_amd.segment import GpuContext
    from pinot_amd.synth import WORKLOADS, build_segments_gpu
    wl = sys.argv[1] if len(sys.argv) > 1 else "adanalytics"
    w = WORKLOADS[wl]
    ctx = GpuContext(0)
    segs = build_segments_gpu(ctx, w, list(range(30)), 1 << 25)
    q = parse_sql(w.sql)
    pm = GpuPlanMaker(ctx, num_groups_limit=w.options.get("num_groups_limit", 100_000))
    for _ in range(5):
        pm.execute(q, segs)
    torch.cuda.synchronize()
    desc, keep, g = pm.build_desc(q, segs)
    n = 50
    a = time.perf_counter()
    for _ in range(n):
        h = C.c_void_p()
        ctx._lib.pgpu_query_submit(ctx.handle, C.byref(desc), C.byref(h))
        ctx._lib.pgpu_query_release(h)
    print(f"C submit+release (synchronous) {1e3*(time.perf_counter()-a)/n:.3f} ms", flush=True)
    a = time.perf_counter()
    for _ in range(n):
        pm.layout(desc)
    print(f"layout {1e3*(time.perf_counter()-a)/n:.3f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        pm.build_desc(q, segs)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    ctx.close()


if __name__ == "__main__":
    main()
