"""Host/GPU overlap of the async query path: per-step time at several pipeline depths, and the time spent
inside submit() and collect()."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
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
    steps = 40
    for depth in (1, 2, 3, 4):
        pend, sub, col, ks = [], [], [], []
        submitted = 0
        t0 = time.perf_counter()
        for _ in range(steps):
            while submitted < steps and len(pend) < depth:
                a = time.perf_counter()
                pend.append(pm.submit(q, segs))
                sub.append(time.perf_counter() - a)
                submitted += 1
            a = time.perf_counter()
            r = pm.collect(pend.pop(0))
            col.append(time.perf_counter() - a)
            ks.append(r.stats.kernel_ms)
        dt = (time.perf_counter() - t0) / steps
        print(f"{wl} depth {depth}: {dt*1e3:.3f} ms/step  submit {1e3*sum(sub)/len(sub):.3f}  "
              f"collect {1e3*sum(col)/len(col):.3f}  kernel {sum(ks)/len(ks):.3f}", flush=True)
    # planning only (no launch)
    a = time.perf_counter()
    for _ in range(steps):
        desc, keep, g = pm.build_desc(q, segs)
    print(f"build_desc {1e3*(time.perf_counter()-a)/steps:.3f} ms", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
