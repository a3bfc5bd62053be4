"""cProfile of the pipelined query loop (submit / collect at depth 3) on the GPU box."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
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

    def loop(steps, depth=3):
        pend, sub = [], 0
        for _ in range(steps):
            while sub < steps and len(pend) < depth:
                pend.append(pm.submit(q, segs))
                sub += 1
            pm.collect(pend.pop(0))

    loop(20)
    t = time.perf_counter()
    loop(200)
    print(f"{wl}: {(time.perf_counter() - t) / 200 * 1e3:.3f} ms/step", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    loop(200)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    ctx.close()


if __name__ == "__main__":
    main()
