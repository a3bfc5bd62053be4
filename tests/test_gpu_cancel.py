"""Query deadline and cancellation (MI355X only).

The reference's combine stops polling for results blocks at the query's end time and answers
EXECUTION_TIMEOUT_ERROR (core/operator/combine/BaseCombineOperator.java:194-203), cancelling the segment tasks.
Here pgpu_query_desc.deadline_ms / pgpu_query_cancel set the query's cancel word, every kernel polls it per range
of tiles and stops early, and collect returns PGPU_E_TIMEOUT / PGPU_E_CANCELLED.  Checked per kernel family
(partitioned group-by phases 1 + 2, self-loading waves, the loader / consumer ring): the stopped query's kernel
time falls well below the full run's, and the context then answers the same query exactly as before."""
import ctypes as C

import pytest

from pinot_amd import _lib
from pinot_amd.plan import GpuPlanMaker
from pinot_amd.query import parse_sql

pytestmark = pytest.mark.gpu

# (workload, segments, docs per segment): large enough that a full run takes milliseconds
CASES = [("groupby1m", 24, 1 << 25), ("adanalytics", 32, 1 << 24), ("range_in", 32, 1 << 24)]


def _segments(gpu_ctx, wl, nseg, n):
    from pinot_amd.synth import WORKLOADS, build_segments_gpu
    w = WORKLOADS[wl]
    return w, build_segments_gpu(gpu_ctx, w, list(range(nseg)), n)


def _collect_raw(pm, pending):
    """pgpu_query_collect at the C ABI: (status, stats) without raising."""
    L = pending.layout
    cap = int(min(L.num_keys, 1 << 22))
    keys = (C.c_int64 * max(cap, 1))()
    cells = (C.c_int64 * (max(cap, 1) * L.num_sections))()
    n = C.c_uint64()
    st = _lib.QueryStats()
    h, pending.handle = pending.handle, None
    rc = pm.ctx._lib.pgpu_query_collect(h, keys, cells, cap, C.byref(n), C.byref(st))
    return rc, st


@pytest.mark.parametrize("wl,nseg,n", CASES, ids=[c[0] for c in CASES])
def test_cancel_stops_kernels_and_context_stays_usable(gpu_ctx, wl, nseg, n):
    w, gs = _segments(gpu_ctx, wl, nseg, n)
    try:
        opts = dict(num_groups_limit=w.options.get("num_groups_limit", 100_000))
        pm = GpuPlanMaker(gpu_ctx, **opts)
        q = parse_sql(w.sql)
        full = pm.collect(pm.submit(q, gs))
        # cancelled right after submit: the kernels see the word at their first poll
        pending = pm.submit(q, gs)
        pending.cancel()
        rc, st = _collect_raw(pm, pending)
        assert rc == _lib.PGPU_E_CANCELLED
        assert "cancel" in _lib.last_error()
        assert st.kernel_ms < 0.5 * full.stats.kernel_ms, (st.kernel_ms, full.stats.kernel_ms)
        # the Python surface raises
        pending = pm.submit(q, gs)
        pending.cancel()
        with pytest.raises(_lib.QueryCancelledError):
            pm.collect(pending)
        # the context answers the query exactly as before
        again = pm.collect(pm.submit(q, gs))
        assert again.group_rows == full.group_rows if q.group_by else again.aggregation_result == full.aggregation_result
        assert again.stats.num_docs_scanned == full.stats.num_docs_scanned
    finally:
        for g in gs:
            g.release()


@pytest.mark.parametrize("wl,nseg,n", CASES[:2], ids=[c[0] for c in CASES[:2]])
def test_deadline_times_out(gpu_ctx, wl, nseg, n):
    w, gs = _segments(gpu_ctx, wl, nseg, n)
    try:
        opts = dict(num_groups_limit=w.options.get("num_groups_limit", 100_000))
        q = parse_sql(w.sql)
        full = GpuPlanMaker(gpu_ctx, **opts).execute(q, gs)
        # a deadline already passed at submit: the kernels skip their work, collect reports the timeout
        with pytest.raises(_lib.QueryTimeoutError):
            GpuPlanMaker(gpu_ctx, timeout_ms=-1, **opts).execute(q, gs)
        pm = GpuPlanMaker(gpu_ctx, timeout_ms=-1, **opts)
        rc, st = _collect_raw(pm, pm.submit(q, gs))
        assert rc == _lib.PGPU_E_TIMEOUT
        assert st.kernel_ms < 0.5 * full.stats.kernel_ms
        # a generous deadline changes nothing
        ok = GpuPlanMaker(gpu_ctx, timeout_ms=60_000, **opts).execute(q, gs)
        assert ok.group_rows == full.group_rows if q.group_by else ok.aggregation_result == full.aggregation_result
    finally:
        for g in gs:
            g.release()
