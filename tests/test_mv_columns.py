"""Multi-value columns: the FixedBitMVForwardIndexWriter format, the loader, applyMV filter
semantics, the *MV aggregation functions and their numEntriesScannedInFilter, GPU against the oracle.

Parity note: the reference's multi-value query tests read test_data-mv.avro, which the reference tree does not hold
(only test_data-sv.avro), so no reference known-answer vector pins these semantics; the oracle restates them from
MVScanDocIdIterator.java:56-100, BaseDictionaryBasedPredicateEvaluator.java:133-149 and the *MVAggregationFunctions,
and the format from FixedBitMVForwardIndexWriter.java:73-159 (hand-computed bytes below).
"""
import math
import os

import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import (build_segment, mv_docs_per_chunk, read_mv_forward, write_mv_forward,
                                   write_segment_dir)
from pinot_amd._lib import PGPU_DOUBLE, PGPU_FLOAT, PGPU_INT, PGPU_LONG, UnsupportedPlanError
from pinot_amd.query import parse_sql

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _brute_mask(rows, p_any, exclusive=False):
    return np.array([all(p_any(v) for v in r) if exclusive else any(p_any(v) for v in r) for r in rows])


# ---- format ------------------------------------------------------------------------------------------------------
def test_mv_forward_bytes_by_hand():
    # rows [1], [2, 3], [0, 0, 1] with 2-bit ids: numValues 6, numDocs 3 -> 6 / 3 = 2 values per doc on average,
    # ceil(2048 / 2.0) = 1024 rows per chunk -> one chunk offset (0); bitmap bits at 0, 1, 3 -> 0b11010000;
    # ids 01 10 11 00 00 01 -> 0b01101100 0b00010000
    data = write_mv_forward([np.array([1]), np.array([2, 3]), np.array([0, 0, 1])], 2)
    assert data == bytes([0, 0, 0, 0, 0b11010000, 0b01101100, 0b00010000])
    off, ids = read_mv_forward(data, 3, 6, 2)
    assert off.tolist() == [0, 1, 3, 6] and ids.tolist() == [1, 2, 3, 0, 0, 1]


@pytest.mark.parametrize("n,maxlen,bits", [(1, 1, 1), (5000, 3, 7), (20000, 1, 12), (3001, 40, 20)])
def test_mv_forward_round_trip(n, maxlen, bits):
    rng = np.random.default_rng(n)
    rows = [rng.integers(0, 1 << bits, rng.integers(1, maxlen + 1)) for _ in range(n)]
    nv = sum(len(r) for r in rows)
    data = write_mv_forward(rows, bits)
    per = mv_docs_per_chunk(n, nv)
    nchunks = (n + per - 1) // per
    assert len(data) == 4 * nchunks + (nv + 7) // 8 + (nv * bits + 7) // 8
    off, ids = read_mv_forward(data, n, nv, bits)
    assert np.array_equal(np.diff(off), [len(r) for r in rows])
    assert np.array_equal(ids, np.concatenate(rows))
    # the chunk header: value index of every chunk's first row (FixedBitMVForwardIndexWriter.updateHeader)
    assert np.frombuffer(data[:4 * nchunks], dtype=">i4").tolist() == off[:-1][::per].tolist()


def test_docs_per_chunk_uses_integer_average():
    # (float) (numValues / numDocs): 5 values over 3 docs average 1, not 1.67 -> 2048 rows per chunk
    assert mv_docs_per_chunk(3, 5) == 2048
    assert mv_docs_per_chunk(10, 30) == 683   # ceil(2048 / 3)
    assert mv_docs_per_chunk(4, 4 * 4096) == 1


def test_empty_rows_are_rejected():
    with pytest.raises(ValueError):
        write_mv_forward([np.array([1]), np.array([], dtype=np.int64)], 2)


def _segment(seed=0, n=6000, inverted=("tags",), name="mv"):
    rng = np.random.default_rng(seed)
    cols = {
        "tags": (PGPU_INT, [rng.integers(0, 40, rng.integers(1, 6)) * 7 for _ in range(n)]),
        "lv": (PGPU_LONG, [rng.integers(-(1 << 40), 1 << 40, rng.integers(1, 4)) for _ in range(n)]),
        "fv": (PGPU_FLOAT, [rng.random(rng.integers(1, 4)).astype(np.float32) * 100 for _ in range(n)]),
        "dv": (PGPU_DOUBLE, [rng.normal(size=rng.integers(1, 3)) for _ in range(n)]),
        "g": (PGPU_INT, rng.integers(0, 6, n)),
        "s": (PGPU_INT, rng.integers(0, 100, n)),
    }
    return build_segment(name, cols, inverted=list(inverted), mv=["tags", "lv", "fv", "dv"], sorted_columns=[])


def _rows(seg, col):
    ds = engine.DecodedSegment(seg)
    off, ids = ds.mv(col)
    d = ds.dictionary(col)
    return [d[ids[off[i]:off[i + 1]]] for i in range(seg.num_docs)]


# ---- oracle semantics ----------------------------------------------------------------------------------------------
def test_oracle_applymv_semantics():
    seg = _segment()
    rows = _rows(seg, "tags")
    cases = [("tags = 21", lambda v: v == 21, False), ("tags IN (0, 70, 273)", lambda v: v in (0, 70, 273), False),
             ("tags <> 21", lambda v: v != 21, True), ("tags NOT IN (0, 70)", lambda v: v not in (0, 70), True),
             ("tags BETWEEN 50 AND 100", lambda v: 50 <= v <= 100, False)]
    for f, pred, excl in cases:
        want = _brute_mask(rows, pred, excl)
        for inv in ((), ("tags",)):
            s = _segment(inverted=inv)
            r = engine.execute(parse_sql(f"SELECT COUNT(*) FROM t WHERE {f}"), [s], iterator_stats=True)
            assert r.aggregation_result[0] == int(want.sum()), (f, inv)
            # a lone scan reads every row's values; a bitmap leaf reads none
            lone_scan = not inv or "BETWEEN" in f
            assert r.num_entries_scanned_in_filter == (sum(len(x) for x in rows) if lone_scan else 0), (f, inv)


def test_oracle_mv_aggregations_brute_force():
    seg = _segment(1)
    tags, lv, fv = _rows(seg, "tags"), _rows(seg, "lv"), _rows(seg, "fv")
    m = np.array([int(x) >= 20 for x in np.frombuffer(seg.column("s").dictionary, dtype=">i4")[
        engine.DecodedSegment(seg).ids("s")]])
    r = engine.execute(parse_sql("SELECT COUNTMV(tags), SUMMV(tags), MINMV(lv), MAXMV(lv), AVGMV(fv), COUNT(*) "
                                 "FROM t WHERE s >= 20"), [seg])
    sel = np.flatnonzero(m)
    vals_t = np.concatenate([tags[i] for i in sel])
    vals_l = np.concatenate([lv[i] for i in sel])
    vals_f = np.concatenate([fv[i].astype(np.float64) for i in sel])
    assert r.aggregation_result[0] == len(vals_t)
    assert r.aggregation_result[1] == float(vals_t.sum())
    assert r.aggregation_result[2] == float(vals_l.min()) and r.aggregation_result[3] == float(vals_l.max())
    assert r.aggregation_result[4] == pytest.approx(vals_f.sum() / len(vals_f), rel=1e-12)
    assert r.aggregation_result[5] == len(sel)


MV_GROUP_QUERIES = [
    "SELECT tags, COUNT(*), SUM(s), MAX(s), MIN(s) FROM t WHERE s < 60 GROUP BY tags",
    "SELECT g, tags, COUNT(*), SUMMV(lv), AVG(s) FROM t GROUP BY g, tags",
    "SELECT tags, g, COUNT(*), MAXMV(fv), COUNTMV(lv) FROM t WHERE tags IN (7, 14, 21) OR s > 90 GROUP BY tags, g",
    "SELECT tags, lv, COUNT(*), SUM(s) FROM t WHERE g = 2 GROUP BY tags, lv",
    "SELECT tags, COUNT(*), SUMMV(tags) FROM t WHERE tags <> 0 GROUP BY tags ORDER BY COUNT(*) DESC LIMIT 5",
]


def _brute_mv_groups(seg, sql):
    """Plain loops over the rows: each matched doc adds to every element of the cartesian product of its group
    columns' values (duplicates kept) -- DictionaryBasedGroupKeyGenerator's multi-value keys."""
    q = parse_sql(sql)
    ds = engine.DecodedSegment(seg)
    # the filter's doc set from the oracle's (separately pinned) filter path; the expansion below is brute force
    where = " WHERE " + sql.split(" WHERE ")[1].split(" GROUP BY")[0] if " WHERE " in sql else ""
    mask = np.zeros(seg.num_docs, bool)
    mask[engine.execute_segment(parse_sql("SELECT COUNT(*) FROM t" + where), seg).matched] = True
    def vals(col, d):
        c = seg.column(col)
        if c.is_mv:
            off, ids = ds.mv(col)
            return list(ds.dictionary(col)[ids[off[d]:off[d + 1]]])
        return [ds.dictionary(col)[ds.ids(col)[d]]]
    groups = {}
    for d in np.flatnonzero(mask):
        keys = [()]
        for col in q.group_by:
            keys = [k + (v.item(),) for k in keys for v in vals(col, d)]
        for k in keys:
            acc = groups.setdefault(k, [])
            acc.append(d)
    out = {}
    for k, docs in groups.items():
        row = []
        for a in q.aggregations:
            if a.function == "COUNT":
                row.append(len(docs))
                continue
            vs = [x for d in docs for x in vals(a.column, d)]
            f = a.function.replace("MV", "") if a.function.endswith("MV") else a.function
            if a.function == "COUNTMV":
                row.append(len(vs))
            elif f == "SUM":
                row.append(float(np.sum(np.asarray(vs, dtype=np.float64))))
            elif f == "MIN":
                row.append(float(min(vs)))
            elif f == "MAX":
                row.append(float(max(vs)))
            else:
                row.append(float(np.sum(np.asarray(vs, dtype=np.float64))) / len(vs))
        out[k] = row
    return out


@pytest.mark.parametrize("sql", MV_GROUP_QUERIES[:4])
def test_oracle_mv_group_by_brute_force(sql):
    seg = _segment(2, n=700)
    want = _brute_mv_groups(seg, sql)
    got = {r[:len(parse_sql(sql).group_by)]: r[len(parse_sql(sql).group_by):]
           for r in engine.execute(parse_sql(sql), [seg]).group_rows}
    assert got.keys() == want.keys()
    for k in got:
        assert all(_close(a, b) for a, b in zip(got[k], want[k])), (k, got[k], want[k])


def test_oracle_mv_group_by_limit_keeps_first_seen():
    """Map-based holder with numGroupsLimit: only the first keys in (doc, value) order get group ids."""
    seg = _segment(4, n=300)
    q = parse_sql("SELECT tags, g, COUNT(*) FROM t GROUP BY tags, g")
    full = engine.execute(q, [seg], num_groups_limit=10**9, max_init_group_holder_capacity=10).group_rows
    lim = engine.execute(q, [seg], num_groups_limit=17, max_init_group_holder_capacity=10).group_rows
    ds = engine.DecodedSegment(seg)
    off, ids = ds.mv("tags")
    first = []
    for d in range(seg.num_docs):
        for v in ids[off[d]:off[d + 1]]:
            k = (int(ds.dictionary("tags")[v]), int(ds.dictionary("g")[ds.ids("g")[d]]))
            if k not in first:
                first.append(k)
    assert sorted(r[:2] for r in lim) == sorted(first[:17])
    fd = {r[:2]: r[2] for r in full}
    assert all(fd[r[:2]] == r[2] for r in lim)


def test_oracle_rejects_sv_functions_on_mv_and_back():
    seg = _segment(2, n=500)
    with pytest.raises(ValueError):
        engine.execute(parse_sql("SELECT SUM(tags) FROM t"), [seg])
    with pytest.raises(ValueError):
        engine.execute(parse_sql("SELECT SUMMV(s) FROM t"), [seg])


def test_loader_reads_mv_columns(tmp_path):
    from pinot_amd.loader import load_segment
    seg = _segment(3, n=3000)
    for version in ("v1", "v3"):
        d = write_segment_dir(seg, str(tmp_path / version), version=version)
        got = load_segment(os.path.dirname(d) if version == "v3" else d)
        for c in ("tags", "lv", "fv", "dv"):
            a, b = got.column(c), seg.column(c)
            assert a.is_mv and (a.mv_forward, a.num_values, a.dictionary, a.inverted) == \
                (b.mv_forward, b.num_values, b.dictionary, b.inverted)
            assert a.max_values == b.max_values
        q = parse_sql("SELECT g, COUNTMV(tags), SUMMV(dv) FROM t WHERE tags IN (7, 14) GROUP BY g")
        assert engine.execute(q, [got]).group_rows == engine.execute(q, [seg]).group_rows


def test_lowering_shapes():
    from pinot_amd.mv import lower
    q = parse_sql("SELECT g, AVGMV(fv), COUNT(*), MINMV(tags) FROM t GROUP BY g ORDER BY AVGMV(fv) DESC LIMIT 3")
    low, parts = lower(q)
    assert [(a.function, a.column) for a in low.aggregations] == [
        ("SUM", "fv$mvsum"), ("SUM", "fv$mvlen"), ("COUNT", None), ("MIN", "tags$mvmin")]
    assert parts == [[0, 1], [2], [3]] and low.order_by == [] and low.group_by == ["g"]


# ---- GPU --------------------------------------------------------------------------------------------------------------
QUERIES = [
    "SELECT COUNT(*), COUNTMV(tags), SUMMV(tags), MINMV(tags), MAXMV(tags), AVGMV(tags) FROM t WHERE tags = 21",
    "SELECT COUNT(*), SUMMV(lv), MINMV(lv), MAXMV(lv), AVGMV(lv) FROM t WHERE tags <> 21",
    "SELECT COUNT(*), SUMMV(fv), MINMV(fv), MAXMV(fv), AVGMV(dv) FROM t WHERE tags NOT IN (0, 70, 140)",
    "SELECT COUNTMV(fv), SUMMV(dv) FROM t WHERE fv BETWEEN 10 AND 20",
    "SELECT COUNT(*), COUNTMV(lv) FROM t WHERE fv > 90 AND s < 50",
    "SELECT COUNT(*), MAXMV(dv) FROM t WHERE (tags IN (7, 14) OR lv > 0) AND NOT (g = 3)",
    "SELECT g, COUNT(*), COUNTMV(tags), SUMMV(lv), AVGMV(fv), MINMV(dv) FROM t WHERE fv < 50 GROUP BY g",
    "SELECT g, AVGMV(tags), COUNT(*) FROM t GROUP BY g ORDER BY AVGMV(tags) DESC LIMIT 3",
    "SELECT MINMV(tags), MAXMV(lv), COUNT(*) FROM t",
    "SELECT COUNT(*), SUM(s) FROM t WHERE tags IN (7, 14, 21) AND dv < 0",
    "SELECT COUNTMV(tags) FILTER(WHERE g = 1), SUMMV(lv), COUNT(*) FROM t WHERE s > 10",
]


def _close(a, b):
    if isinstance(a, tuple):
        return all(_close(x, y) for x, y in zip(a, b))
    if isinstance(a, float) or isinstance(b, float):
        if math.isinf(a) or math.isinf(b):
            return a == b
        return a == pytest.approx(b, rel=1e-9, abs=1e-9)
    return a == b


@pytest.mark.gpu
@pytest.mark.parametrize("sql", QUERIES)
@pytest.mark.parametrize("inverted", [(), ("tags",)])
def test_gpu_mv_queries_match_oracle(gpu_ctx, sql, inverted):
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    segs = [_segment(10 + k, n=[6000, 4097, 2048][k], inverted=inverted, name=f"mv{k}") for k in range(3)]
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        q = parse_sql(sql)
        for exact in (False, True):
            res = GpuPlanMaker(gpu_ctx, exact_filter_stats=exact).execute(q, gs)
            ref = engine.execute(q, segs, iterator_stats=True)
            assert len(res.rows) == len(ref.rows)
            for a, b in zip(res.rows, ref.rows):
                assert _close(tuple(a), tuple(b)), (sql, a, b)
            assert res.stats.num_docs_scanned == ref.num_docs_scanned
            if exact or res.stats.filter_stats_exact:
                assert res.stats.num_entries_scanned_in_filter == ref.num_entries_scanned_in_filter, (sql, exact)
    finally:
        for g in gs:
            g.release()


@pytest.mark.gpu
def test_gpu_lone_mv_scan_counts_every_value(gpu_ctx):
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    seg = _segment(20, n=5000, inverted=())
    g = GpuSegment(gpu_ctx, seg)
    try:
        q = parse_sql("SELECT COUNT(*) FROM t WHERE lv > 0")
        res = GpuPlanMaker(gpu_ctx).execute(q, [g])
        assert res.stats.filter_stats_exact
        assert res.stats.num_entries_scanned_in_filter == seg.column("lv").num_values
    finally:
        g.release()


@pytest.mark.gpu
def test_gpu_mv_unsupported_shapes(gpu_ctx):
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    g = GpuSegment(gpu_ctx, _segment(21, n=1000))
    try:
        pm = GpuPlanMaker(gpu_ctx)
        for sql in ("SELECT SUM(tags) FROM t", "SELECT COUNTMV(s) FROM t"):
            with pytest.raises(UnsupportedPlanError):
                pm.execute(parse_sql(sql), [g])
    finally:
        g.release()


@pytest.mark.gpu
def test_gpu_loaded_mv_segment(gpu_ctx, tmp_path):
    from pinot_amd.loader import load_segment
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    seg = _segment(22, n=7000)
    d = write_segment_dir(seg, str(tmp_path / "s"), version="v3")
    loaded = load_segment(os.path.dirname(d))
    g = GpuSegment(gpu_ctx, loaded)
    try:
        q = parse_sql("SELECT g, COUNTMV(tags), SUMMV(lv), MAXMV(fv) FROM t WHERE tags IN (7, 35) GROUP BY g")
        res = GpuPlanMaker(gpu_ctx).execute(q, [g])
        ref = engine.execute(q, [seg])
        assert sorted(res.group_rows) == sorted(ref.group_rows)
    finally:
        g.release()


@pytest.mark.gpu
@pytest.mark.parametrize("sql", MV_GROUP_QUERIES)
@pytest.mark.parametrize("inverted", [(), ("tags",)])
def test_gpu_mv_group_by_matches_oracle(gpu_ctx, sql, inverted):
    """GROUP BY on multi-value columns (one key per value, cartesian product over several): GPU vs oracle over
    three segments whose dictionaries differ (global dictionary + remap tables), every group compared."""
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    from tests.helpers import check_groups
    segs = [_segment(30 + k, n=[6000, 4097, 2048][k], inverted=inverted, name=f"mvg{k}") for k in range(3)]
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        q = parse_sql(sql)
        res = GpuPlanMaker(gpu_ctx).execute(q, gs)
        ref = engine.execute(q, segs)
        check_groups(res, ref, 1e-9)
        got = {r[:len(q.group_by)]: r for r in res.group_rows}
        for r in ref.group_rows:
            if r[:len(q.group_by)] in got:
                assert _close(tuple(got[r[:len(q.group_by)]]), tuple(r)), (sql, r)
        assert res.stats.num_docs_scanned == ref.num_docs_scanned
        assert res.stats.num_entries_scanned_post_filter == ref.num_entries_scanned_post_filter
        if q.order_by:
            assert [tuple(r) for r in res.rows] == [tuple(r) for r in ref.rows] or \
                all(_close(tuple(a), tuple(b)) for a, b in zip(res.rows, ref.rows))
    finally:
        for g in gs:
            g.release()


@pytest.mark.gpu
@pytest.mark.parametrize("sql,limit", [("SELECT tags, g, COUNT(*), SUM(s) FROM t GROUP BY tags, g", 17),
                                       ("SELECT tags, COUNT(*), MAX(s) FROM t WHERE s < 80 GROUP BY tags", 23),
                                       ("SELECT g, tags, COUNT(*) FROM t GROUP BY g, tags", 100)])
def test_gpu_mv_group_by_first_seen_limit(gpu_ctx, sql, limit):
    """numGroupsLimit on multi-value group keys: the GPU keeps the first `limit` keys in the order
    processMultiValue gives them ids ((doc, expansion) order, DictionaryBasedGroupKeyGenerator.java:186-199), the
    limit's doc cut by its own key expansion (GpuPlanMaker.first_seen_groups, pgpu_segment_mv_row)."""
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    from tests.helpers import check_groups
    segs = [_segment(40 + k, n=[300, 450][k], name=f"mvl{k}") for k in range(2)]
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        q = parse_sql(sql)
        res = GpuPlanMaker(gpu_ctx, num_groups_limit=limit, max_init_group_holder_capacity=10).execute(q, gs)
    finally:
        for g in gs:
            g.release()
    ref = engine.execute(q, segs, num_groups_limit=limit, max_init_group_holder_capacity=10)
    full = engine.execute(q, segs, num_groups_limit=10 ** 9)
    assert len(ref.group_rows) < len(full.group_rows)  # the limit really cuts
    check_groups(res, ref, 1e-9)
    assert sorted(r[:len(q.group_by)] for r in res.group_rows) == sorted(r[:len(q.group_by)] for r in ref.group_rows)
    assert res.stats.num_groups_limit_reached and ref.num_groups_limit_reached
