"""Kernel-time breakdown: run SQL variants over one synthetic workload's segments and print kernel ms + GB/s."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.query import parse_sql
    from pinot_amd.segment import GpuContext
    from pinot_amd.synth import WORKLOADS, build_segments_gpu
    wl = sys.argv[1]
    nseg = int(sys.argv[2])
    sqls = sys.argv[3:]
    w = WORKLOADS[wl]
    ctx = GpuContext(0)
    segs = build_segments_gpu(ctx, w, list(range(nseg)), 1 << 25)
    pm = GpuPlanMaker(ctx, num_groups_limit=w.options.get("num_groups_limit", 100_000))
    rows = nseg * (1 << 25)
    for sql in sqls:
        q = parse_sql(sql)
        for _ in range(2):
            pm.execute(q, segs)
        ks = []
        for _ in range(5):
            r = pm.execute(q, segs)
            ks.append(r.stats.kernel_ms)
        k = sorted(ks)[len(ks) // 2]
        print(f"{k:8.3f} ms  {rows / max(k, 1e-9) / 1e6:8.1f} Grows/s  matched {r.stats.num_docs_scanned:>11}  | {sql}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
