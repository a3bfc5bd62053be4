"""Host-side overhead profile of one query step (cProfile over repeated DistributedExecutor.execute calls)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pinot_amd.combine import DistributedExecutor
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.query import parse_sql
    from pinot_amd.segment import GpuContext
    from pinot_amd.synth import WORKLOADS, build_segments_gpu
    wl = sys.argv[1] if len(sys.argv) > 1 else "adanalytics"
    nseg = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    w = WORKLOADS[wl]
    ctx = GpuContext(0)
    segs = build_segments_gpu(ctx, w, list(range(nseg)), 1 << 25)
    q = parse_sql(w.sql)
    pm = GpuPlanMaker(ctx, num_groups_limit=w.options.get("num_groups_limit", 100_000))
    ex = DistributedExecutor(pm)
    for _ in range(3):
        ex.execute(q, segs)
    torch.cuda.synchronize()
    t = time.perf_counter()
    ks = []
    for _ in range(20):
        ex.execute(q, segs)
        ks.append(ex.last_stats.kernel_ms)
    dt = (time.perf_counter() - t) / 20
    print(f"{wl}: {dt*1e3:.3f} ms/step, kernel {sum(ks)/len(ks):.3f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        ex.execute(q, segs)
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
    ctx.close()


if __name__ == "__main__":
    main()
