"""Multi-GPU combine logic on the CPU: world_size-2 ``gloo`` process groups.

The GPU path leaves one dense partial table per rank (layout: include/pinot_gpu.h, pgpu_table_layout) and merges
them with one collective per reduction op (pinot_amd/combine.py: reduce_sections), after the group columns' global
dictionaries were unified across ranks (union_dictionaries).  These tests run that exact host code over gloo, with
the per-rank partial tables computed in numpy from each rank's rows (standing in for the query kernel), and check
the merged, finished result against the oracle run over ALL ranks' segments — the reference's single-server
combine (AggregationOnlyCombineOperator.java:47-57, GroupByOrderByCombineOperator.java:127-248).
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from pinot_amd._lib import (PGPU_DOUBLE, PGPU_INT, PGPU_RED_MAX_I64, PGPU_RED_MIN_I64, PGPU_RED_SUM_F64,  # noqa: E402
                            PGPU_RED_SUM_I64, PGPU_STRING, TableLayout)

WORLD = 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(fn, *args):
    port = _free_port()
    mp.spawn(_entry, args=(fn, port, args), nprocs=WORLD, join=True)


def _entry(rank, fn, port, args):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        fn(rank, *args)
    finally:
        dist.destroy_process_group()


def _layout(num_keys, ops, agg_sections=(), agg_types=()):
    L = TableLayout()
    L.num_keys = num_keys
    L.num_sections = len(ops)
    for i, o in enumerate(ops):
        L.section_op[i] = o
    for i, (s, t) in enumerate(zip(agg_sections, agg_types)):
        L.agg_section[i] = s
        L.agg_value_type[i] = t
    return L


def minmax_key(v: float, vtype: int) -> int:
    """Order-preserving int64 key of a MIN/MAX value (inverse of pgpu_decode_minmax_key)."""
    if vtype in (0, 1):
        return int(v)
    b = int(np.float64(v).view(np.int64))
    return b if b >= 0 else b ^ 0x7FFFFFFFFFFFFFFF


# ---- reduce_sections: every op, contiguous and interleaved sections ------------------------------------------
def _reduce_worker(rank):
    from pinot_amd.combine import reduce_sections
    G = 37
    ops = [PGPU_RED_SUM_I64, PGPU_RED_MIN_I64, PGPU_RED_SUM_F64, PGPU_RED_MAX_I64, PGPU_RED_SUM_I64,
           PGPU_RED_SUM_F64]
    L = _layout(G, ops)
    tables = []
    for r in range(WORLD):
        rng = np.random.default_rng(100 + r)
        t = np.empty((len(ops), G), dtype=np.int64)
        for s, op in enumerate(ops):
            if op == PGPU_RED_SUM_F64:
                t[s] = rng.normal(size=G).view(np.int64)
            else:
                t[s] = rng.integers(-2**40, 2**40, size=G)
        tables.append(t)
    mine = torch.from_numpy(tables[rank].reshape(-1).copy())
    reduce_sections(mine, L)
    got = mine.numpy().reshape(len(ops), G)
    for s, op in enumerate(ops):
        col = np.stack([t[s] for t in tables])
        if op == PGPU_RED_SUM_I64:
            exp = col.sum(axis=0)
        elif op == PGPU_RED_MIN_I64:
            exp = col.min(axis=0)
        elif op == PGPU_RED_MAX_I64:
            exp = col.max(axis=0)
        else:
            exp = col.view(np.float64).sum(axis=0).view(np.int64)
        if op == PGPU_RED_SUM_F64:
            np.testing.assert_allclose(got[s].view(np.float64), exp.view(np.float64), rtol=1e-12)
        else:
            np.testing.assert_array_equal(got[s], exp)


def test_reduce_sections_gloo():
    _spawn(_reduce_worker)


# ---- union_dictionaries ---------------------------------------------------------------------------------------
def _union_worker(rank):
    from pinot_amd.combine import union_dictionaries
    ints = [np.array([1, 5, 9], dtype=np.int32), np.array([2, 5, 11, 12], dtype=np.int32)][rank]
    np.testing.assert_array_equal(union_dictionaries(ints), [1, 2, 5, 9, 11, 12])
    strs = [["a", "null", "zz"], ["b", "null"]][rank]
    assert union_dictionaries(strs) == ["a", "b", "null", "zz"]
    empty_side = [np.array([], dtype=np.int64), np.array([3, 4], dtype=np.int64)][rank]
    np.testing.assert_array_equal(union_dictionaries(empty_side), [3, 4])


def test_union_dictionaries_gloo():
    _spawn(_union_worker)


# ---- end to end: per-rank partial tables -> reduce -> finish == oracle over all segments ----------------------
SQL_GB = ("SELECT g, SUM(m), MIN(m), MAX(d), AVG(d), COUNT(*) FROM t WHERE x < 60 "
          "GROUP BY g ORDER BY SUM(m) DESC LIMIT 7")
SQL_AGG = "SELECT COUNT(*), SUM(m), MIN(d), MAX(m), AVG(m) FROM t WHERE x >= 30 AND x < 45"


def _rank_rows(rank, n=3000):
    rng = np.random.default_rng(7 + rank)
    # rank-dependent group dictionaries, so the global dictionary is a real union
    names = [f"g{i:02d}" for i in range(rank * 5, rank * 5 + 20)]
    return {"g": (PGPU_STRING, [names[i] for i in rng.integers(0, len(names), n)]),
            "x": (PGPU_INT, rng.integers(0, 100, n).astype(np.int32)),
            "m": (PGPU_INT, rng.integers(-1000, 100000, n).astype(np.int32)),
            "d": (PGPU_DOUBLE, np.round(rng.normal(50.0, 20.0, n), 3))}


def _partial_table(query, rows, glob, L):
    """What the query kernel leaves in HBM for this rank's rows (include/pinot_gpu.h table layout)."""
    from pinot_amd.query import UNBOUNDED
    x = rows["x"][1]
    mask = np.ones(len(x), dtype=bool)
    def leaves(f):  # conjunctions of range predicates on x (filtered-aggregation passes nest one AND)
        return [f] if f.type == "PREDICATE" else [x for c in f.children for x in leaves(c)]

    preds = leaves(query.filter) if query.filter is not None else []
    for p in preds:
        pr = p.predicate
        lo = -np.inf if pr.lower == UNBOUNDED else float(pr.lower)
        hi = np.inf if pr.upper == UNBOUNDED else float(pr.upper)
        v = x.astype(np.float64)
        mask &= (v > lo) | ((v == lo) & pr.lower_inclusive)
        mask &= (v < hi) | ((v == hi) & pr.upper_inclusive)
    G = int(L.num_keys)
    if query.group_by:
        pos = {v: i for i, v in enumerate(glob)}
        keys = np.array([pos[v] for v in rows["g"][1]], dtype=np.int64)
    else:
        keys = np.zeros(len(x), dtype=np.int64)
    keys = keys[mask]
    t = np.zeros((L.num_sections, G), dtype=np.int64)
    np.add.at(t[0], keys, 1)
    for ai, a in enumerate(query.aggregations):
        s = L.agg_section[ai]
        if s == 0:
            continue
        vt = L.agg_value_type[ai]
        vals = np.asarray(rows[a.column][1])[mask]
        op = L.section_op[s]
        if op == PGPU_RED_SUM_I64:
            np.add.at(t[s], keys, vals.astype(np.int64))
        elif op == PGPU_RED_SUM_F64:
            acc = np.zeros(G, dtype=np.float64)
            np.add.at(acc, keys, vals.astype(np.float64))
            t[s] = acc.view(np.int64)
        else:
            fill = np.iinfo(np.int64).max if op == PGPU_RED_MIN_I64 else np.iinfo(np.int64).min
            t[s] = fill
            kv = np.array([minmax_key(v, vt) for v in vals.tolist()], dtype=np.int64)
            (np.minimum if op == PGPU_RED_MIN_I64 else np.maximum).at(t[s], keys, kv)
    return t


def _layout_for(query, G):
    types = {"m": PGPU_INT, "d": PGPU_DOUBLE}
    ops, secs, vts = [PGPU_RED_SUM_I64], [], []
    for a in query.aggregations:
        if a.function == "COUNT":
            secs.append(0)
            vts.append(-1)
            continue
        vt = types[a.column]
        op = {"MIN": PGPU_RED_MIN_I64, "MAX": PGPU_RED_MAX_I64}.get(
            a.function, PGPU_RED_SUM_I64 if vt == PGPU_INT else PGPU_RED_SUM_F64)
        secs.append(len(ops))
        vts.append(vt)
        ops.append(op)
    return _layout(G, ops, secs, vts)


def _e2e_worker(rank, sql):
    from oracle import engine
    from oracle.segment_writer import build_segment
    from pinot_amd.combine import reduce_sections, union_dictionaries
    from pinot_amd.plan import ExecutionStats, GroupTable, finish
    from pinot_amd.query import parse_sql
    from tests.helpers import close

    q = parse_sql(sql)
    rows = _rank_rows(rank)
    glob = None
    if q.group_by:
        glob = union_dictionaries(sorted(set(rows["g"][1])))
    L = _layout_for(q, len(glob) if glob is not None else 1)
    t = torch.from_numpy(_partial_table(q, rows, glob, L).reshape(-1).copy())
    local_docs = int(t[: int(L.num_keys)].sum())
    reduce_sections(t, L)
    counts = torch.tensor([local_docs], dtype=torch.int64)
    dist.all_reduce(counts)  # numDocsScanned, as DistributedExecutor reduces it
    assert int(counts[0]) == int(t[: int(L.num_keys)].sum())
    if rank != 0:
        return
    cells = t.numpy().reshape(L.num_sections, int(L.num_keys)).T
    keys = np.flatnonzero(cells[:, 0] > 0) if q.group_by else np.array([0])
    gt = GroupTable(keys.astype(np.int64), np.ascontiguousarray(cells[keys]), L)
    res = finish(q, gt, [glob] if q.group_by else [], ExecutionStats(num_docs_scanned=int(counts[0])))
    segs = [build_segment(f"seg{r}", _rank_rows(r)) for r in range(WORLD)]
    ref = engine.execute(q, segs)
    assert res.stats.num_docs_scanned == ref.num_docs_scanned
    if q.group_by:
        got = sorted(res.group_rows)
        exp = sorted(ref.group_rows)
        assert len(got) == len(exp)
        for a, b in zip(got, exp):
            assert a[0] == b[0]
            assert all(close(u, v) for u, v in zip(a[1:], b[1:])), (a, b)
        assert [r[0] for r in res.rows] == [r[0] for r in ref.rows]
    else:
        assert all(close(u, v) for u, v in zip(res.aggregation_result, ref.aggregation_result))


@pytest.mark.parametrize("sql", [SQL_GB, SQL_AGG], ids=["groupby", "aggregation"])
def test_partial_tables_merge_like_reference_combine(sql):
    _spawn(_e2e_worker, sql)


SQL_FILTERED = ("SELECT SUM(m) FILTER(WHERE x < 40), COUNT(*) FILTER(WHERE x >= 70), MAX(d), SUM(d) "
                "FROM t WHERE x > 10")


def _filtered_worker(rank, sql):
    """Filtered aggregations across ranks: every pass (FILTER clauses, then the main filter) is reduced like the
    unfiltered combine, then merged as FilteredAggregationOperator does -- DistributedExecutor.execute's shape."""
    from oracle import engine
    from oracle.segment_writer import build_segment
    from pinot_amd.combine import reduce_sections
    from pinot_amd.plan import ExecutionStats, GroupTable, finish, merge_filtered
    from pinot_amd.query import parse_sql, split_filtered_aggregations
    from tests.helpers import close

    q = parse_sql(sql)
    rows = _rank_rows(rank)
    parts = split_filtered_aggregations(q)
    results = []
    for sq, _ in parts:
        L = _layout_for(sq, 1)
        t = torch.from_numpy(_partial_table(sq, rows, None, L).reshape(-1).copy())
        reduce_sections(t, L)
        cells = t.numpy().reshape(L.num_sections, 1).T
        gt = GroupTable(np.array([0], dtype=np.int64), np.ascontiguousarray(cells), L)
        results.append(finish(sq, gt, [], ExecutionStats(num_docs_scanned=int(cells[0, 0]), num_total_docs=3000 * WORLD)))
    res = merge_filtered(q, parts, results)
    if rank != 0:
        return
    segs = [build_segment(f"seg{r}", _rank_rows(r)) for r in range(WORLD)]
    ref = engine.execute(q, segs)
    assert all(close(u, v) for u, v in zip(res.aggregation_result, ref.aggregation_result)), \
        (res.aggregation_result, ref.aggregation_result)
    assert res.stats.num_docs_scanned == ref.num_docs_scanned
    assert res.stats.num_total_docs == ref.num_total_docs


def test_filtered_aggregations_merge_across_ranks():
    _spawn(_filtered_worker, SQL_FILTERED)
