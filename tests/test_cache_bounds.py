"""Host / HBM caches of per-segment derived state are bounded by the resident segments.

GpuContext's remap tables, GpuPlanMaker's global group dictionaries and DistributedExecutor's cached agreements
are keyed by segment uids; releasing a segment (GpuSegment.release -> GpuContext.segment_released) evicts every
entry naming it.  A server whose pruning yields a different segment set per query (ServerQueryExecutorV1Impl:
segments selected per query) therefore holds state only for the segments still loaded.
"""
import ctypes as C
import itertools

import numpy as np
import pytest

from pinot_amd.segment import DeviceBuffer, GpuContext


class _HostCtx(GpuContext):
    """A GpuContext without a device: remap tables are accounted, not uploaded."""

    def __init__(self):
        super().__init__(0, _handle=C.c_void_p(1))  # not owned: close() never calls pgpu_shutdown

    def _upload_remap(self, table):
        return DeviceBuffer(self, None, 4 * len(table))


_uid = itertools.count(10_000_000)


class _Seg:
    def __init__(self, ctx, rng):
        self.ctx, self.uid = ctx, next(_uid)
        self.dictionaries = {"k": np.unique(rng.integers(0, 1000, 50)).astype(np.int32)}

    def group_view(self, name):
        return name

    def release(self):
        self.ctx.segment_released(self.uid)


def test_plan_maker_and_remaps_return_to_baseline():
    from pinot_amd.plan import GpuPlanMaker
    ctx = _HostCtx()
    pm = GpuPlanMaker(ctx)
    rng = np.random.default_rng(1)
    keep = [_Seg(ctx, rng) for _ in range(3)]
    pm.global_dictionary("k", keep)
    base = (len(pm._global_dicts), len(ctx._remap_cache), ctx.remap_bytes())
    for _ in range(500):
        segs = [_Seg(ctx, rng) for _ in range(3)] + keep[:1]
        pm.global_dictionary("k", segs)
        for s in segs[:3]:
            s.release()
    assert (len(pm._global_dicts), len(ctx._remap_cache), ctx.remap_bytes()) == base
    for s in keep:
        s.release()
    assert len(pm._global_dicts) == 0 and len(ctx._remap_cache) == 0 and ctx.remap_bytes() == 0


def test_executor_agreements_evicted():
    from pinot_amd.combine import DistributedExecutor
    from pinot_amd.plan import GpuPlanMaker
    import torch
    ctx = _HostCtx()
    ex = DistributedExecutor(GpuPlanMaker(ctx), device=torch.device("cpu"))
    rng = np.random.default_rng(2)
    for _ in range(500):
        segs = [_Seg(ctx, rng) for _ in range(2)]
        key = tuple(s.uid for s in segs)
        ex._docs[key] = (1, tuple(segs))
        ex._globals[(("k",), key)] = ([], tuple(segs))
        ex._split[((("SUM", "m"),), ("k",), key)] = (0, tuple(segs))
        for s in segs:
            s.release()
    assert not ex._docs and not ex._globals and not ex._split


@pytest.mark.gpu
def test_gpu_segment_release_frees_caches(gpu_ctx):
    """500 distinct segment sets queried with GROUP BY (global dictionaries + remap tables) and released: the
    plan maker's cache, the remap tables' HBM and the segments' HBM return to their baseline."""
    from oracle.segment_writer import build_segment
    from pinot_amd._lib import PGPU_INT
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.query import parse_sql
    from pinot_amd.segment import GpuSegment

    pm = GpuPlanMaker(gpu_ctx)
    q = parse_sql("SELECT k, COUNT(*), SUM(m) FROM t GROUP BY k")
    rng = np.random.default_rng(3)
    datas = [build_segment(f"c{i}", {"k": (PGPU_INT, rng.integers(0, 40 + i, 3000).astype(np.int32)),
                                     "m": (PGPU_INT, rng.integers(0, 100, 3000).astype(np.int32))})
             for i in range(8)]
    base = (len(pm._global_dicts), gpu_ctx.remap_bytes())
    released = set()
    for it in range(500):
        segs = [GpuSegment(gpu_ctx, datas[(it + j) % 8]) for j in range(3)]
        res = pm.execute(q, segs)
        assert res.stats.num_docs_scanned == 9000
        assert sum(s.device_bytes() for s in segs) > 0
        for s in segs:
            released.add(s.uid)
            s.release()
    assert (len(pm._global_dicts), gpu_ctx.remap_bytes()) == base
    assert not any(k[0] in released for k in gpu_ctx._remap_cache)
