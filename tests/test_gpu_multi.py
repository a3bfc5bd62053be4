"""The multi-GPU entry points on one MI355X: pgpu_query_launch / pgpu_query_launch_expr into caller memory +
pgpu_table_compact (the one-process-per-GPU combine, pinot_amd/combine.py), and the node-level RCCL combine inside
the library (pgpu_node_*, pinot_amd/node.py) over a one-device clique.  GPU vs oracle."""
import ctypes as C

import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import build_segment
from pinot_amd import _lib
from pinot_amd._lib import PGPU_DOUBLE, PGPU_INT, PGPU_KEYS_HASH, PGPU_LONG, PGPU_Q_HASH, PGPU_STRING, QueryStats
from pinot_amd.plan import ExecutionStats, GpuPlanMaker, GroupTable, finish, key_words_out
from pinot_amd.query import parse_sql
from pinot_amd.segment import GpuSegment
from tests.helpers import check_groups, close, rows_close

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _segments(seed, nseg=3, n=80_000):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(nseg):
        cols = {"g": (PGPU_STRING, [f"k{x}" for x in rng.integers(0, 40, n)]),
                "h": (PGPU_INT, rng.integers(0, 500, n).astype(np.int32) * (i + 1)),
                "x": (PGPU_INT, rng.integers(0, 100, n).astype(np.int32)),
                "m": (PGPU_INT, rng.integers(-1000, 100_000, n).astype(np.int32)),
                "big": (PGPU_LONG, rng.integers(9 * 10 ** 15, 10 ** 16, n).astype(np.int64)),
                "d": (PGPU_DOUBLE, np.round(rng.normal(10.0, 3.0, n), 3))}
        out.append(build_segment(f"mg{seed}_{i}", cols))
    return out


QUERIES = [
    "SELECT g, SUM(m), MIN(d), MAX(m), AVG(d), COUNT(*) FROM t WHERE x < 60 GROUP BY g ORDER BY SUM(m) DESC LIMIT 10",
    "SELECT COUNT(*), SUM(m), MIN(d), MAX(m), AVG(m), SUM(big) FROM t WHERE x BETWEEN 30 AND 44",
    "SELECT g, h, COUNT(*), SUM(big) FROM t WHERE x < 90 GROUP BY g, h ORDER BY SUM(big) DESC, h LIMIT 15",
]


def _check(res, ref):
    assert res.stats.num_docs_scanned == ref.num_docs_scanned
    assert res.stats.num_total_docs == ref.num_total_docs
    if res.query.group_by:
        check_groups(res, ref, 1e-9)
        assert rows_close([list(r) for r in res.rows], [list(r) for r in ref.rows], 1e-9)
    else:
        assert all(close(a, b, 1e-9) for a, b in zip(res.aggregation_result, ref.aggregation_result))


@pytest.mark.parametrize("flags", [0, PGPU_Q_HASH], ids=["layout_auto", "hash"])
@pytest.mark.parametrize("expr", [False, True], ids=["programs", "expr"])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_launch_into_caller_table_and_compact(gpu_ctx, qi, expr, flags):
    """What DistributedExecutor does per rank: launch into a torch-owned table, wait, compact, finish."""
    segs = _segments(100 + qi)
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        q = parse_sql(QUERIES[qi])
        pm = GpuPlanMaker(gpu_ctx, query_flags=flags)
        ex = pm.filter_expr(q, gs) if expr else None
        assert (ex is not None) == expr
        desc, keep, globals_ = pm.build_desc(q, gs, plan_filters=not expr, reduce_docs=8 * 10 ** 6)
        L = pm.layout(desc)
        nbytes = _lib.table_bytes(L)
        table = torch.empty(nbytes // 8, dtype=torch.int64, device="cuda")
        lib = gpu_ctx._lib
        h = C.c_void_p()
        if expr:
            _lib.check(lib.pgpu_query_launch_expr(gpu_ctx.handle, C.byref(desc), ex[0], ex[1], None,
                                                  C.c_void_p(table.data_ptr()), nbytes, C.byref(h)))
        else:
            _lib.check(lib.pgpu_query_launch(gpu_ctx.handle, C.byref(desc), None, C.c_void_p(table.data_ptr()),
                                             nbytes, C.byref(h)))
        st = QueryStats()
        try:
            _lib.check(lib.pgpu_query_wait(h, C.byref(st)))
        finally:
            lib.pgpu_query_release(h)
        kw = key_words_out(L)
        cap = int(L.num_keys)
        keys = np.empty(cap * kw, dtype=np.int64)
        cells = np.empty((cap, L.num_sections), dtype=np.int64)
        n = C.c_uint64()
        _lib.check(lib.pgpu_table_compact(gpu_ctx.handle, C.byref(L), C.c_void_p(table.data_ptr()), None,
                                          keys.ctypes.data_as(C.POINTER(C.c_int64)),
                                          cells.ctypes.data_as(C.POINTER(C.c_int64)), cap, C.byref(n)))
        k = keys[: n.value * kw].reshape(-1, kw) if kw > 1 else keys[: n.value]
        stats = ExecutionStats(num_docs_scanned=st.num_docs_scanned, num_total_docs=st.num_total_docs)
        res = finish(q, GroupTable.sorted(k, cells[: n.value], L), [g[0] for g in globals_], stats)
        if "big" in QUERIES[qi]:
            assert any(L.agg_sum_parts[i] == 3 for i in range(len(q.aggregations)))  # reduce_docs x 1e16
        if flags and q.group_by:
            assert L.key_kind == PGPU_KEYS_HASH
        _check(res, engine.execute(q, segs))
    finally:
        for g in gs:
            g.release()


@pytest.mark.parametrize("flags", [0, PGPU_Q_HASH], ids=["layout_auto", "hash"])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_node_combine_one_device(qi, flags):
    """pgpu_node_* over a one-GPU RCCL clique: launch, grouped ncclReduce (dense) or key merge (hash), compact."""
    from pinot_amd.node import GpuNode
    segs = _segments(200 + qi)
    with GpuNode([0], query_flags=flags) as node:
        gs = [GpuSegment(node.contexts[0], s) for s in segs]
        try:
            q = parse_sql(QUERIES[qi])
            res = node.execute(q, [gs])
            _check(res, engine.execute(q, segs))
        finally:
            for g in gs:
                g.release()


@pytest.mark.parametrize("scatter", [False, True], ids=["reduce", "reduce_scatter"])
@pytest.mark.parametrize("flags", [0, PGPU_Q_HASH], ids=["dense", "hash"])
def test_node_topk_one_device(monkeypatch, scatter, flags):
    """pgpu_node_query_topk: the node's ORDER BY ... LIMIT trim after the merge -- the dense reduce-scatter path
    (forced onto a small table with PGPU_NODE_SCATTER_MIN=0: slice copy + per-slice trim with key_base) and the hash
    ownership merge (rows routed to their owner, merged in a fresh hash table by node_merge_kernel, trimmed)."""
    from pinot_amd.node import GpuNode
    if scatter:
        monkeypatch.setenv("PGPU_NODE_SCATTER_MIN", "0")
    segs = _segments(300)
    sql = "SELECT g, h, SUM(m), COUNT(*), MAX(m) FROM t GROUP BY g, h ORDER BY SUM(m) DESC LIMIT 7"
    with GpuNode([0], query_flags=flags, min_server_group_trim_size=20) as node:
        gs = [GpuSegment(node.contexts[0], s) for s in segs]
        try:
            q = parse_sql(sql)
            res = node.execute(q, [gs])
            ref = engine.execute(q, segs)
            assert [r[2] for r in res.rows] == [r[2] for r in ref.rows]
            assert rows_close([list(r) for r in res.rows], [list(r) for r in ref.rows])
            assert len(res.group_rows) < len(ref.group_rows)  # the trim cut
        finally:
            for g in gs:
                g.release()


@pytest.mark.parametrize("rccl", [False, True], ids=["direct", "rccl"])
def test_node_queries_in_flight(monkeypatch, rccl):
    """pgpu_node_submit / pgpu_node_collect: three node queries in flight (each in its own table set, merged on the
    merge streams), collected in order -- the same results as one at a time and as the oracle; with
    PGPU_NODE_FORCE_RCCL=1 the one-device clique still reduces through ncclReduce."""
    from pinot_amd.node import GpuNode
    if rccl:
        monkeypatch.setenv("PGPU_NODE_FORCE_RCCL", "1")
    segs = _segments(400)
    with GpuNode([0]) as node:
        gs = [GpuSegment(node.contexts[0], s) for s in segs]
        try:
            qs = [parse_sql(sql) for sql in QUERIES]
            pending = [node.submit(q, [gs]) for q in qs]
            got = [node.collect(p) for p in pending]
            for q, res in zip(qs, got):
                _check(res, engine.execute(q, segs))
            again = [node.execute(q, [gs]) for q in qs]
            for a, b in zip(got, again):
                assert a.rows == b.rows
        finally:
            for g in gs:
                g.release()
