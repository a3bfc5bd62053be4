"""FLOAT / DOUBLE SUM and AVG over values of wide dynamic range, MI355X only.

north_star: "double SUM/AVG within 1e-9 relative".  The reference adds each group's values as doubles in doc order
(SumAggregationFunction.java:95-111, AvgAggregationFunction.java:58-190).  The GPU sums them in fixed point: the
window (exponent, 21-bit part count) is chosen from the column's own values (pgpu_fixed_sum_layout), so each value is
exact or rounded by at most 2^-41 of itself, and a column whose range needs more than PGPU_MAX_FIXED_PARTS parts
keeps a float64 section.  Each group is checked against the oracle at 1e-9 relative and against the exactly
rounded sum (math.fsum), for groups whose magnitudes differ by up to 1e15 inside one column, through the dense and
hash holders, aggregation-only filters that select only the small rows, the GPU ORDER BY trim, and the one-device
node combine."""
import math

import numpy as np
import pytest

from oracle import engine
from oracle.engine import DecodedSegment
from oracle.segment_writer import build_segment
from pinot_amd import _lib
from pinot_amd._lib import PGPU_DOUBLE, PGPU_FLOAT, PGPU_INT
from pinot_amd.plan import GpuPlanMaker
from pinot_amd.query import parse_sql
from pinot_amd.segment import GpuSegment
from tests.helpers import check_groups, close, fixed_sum_layout

pytestmark = pytest.mark.gpu

REL = 1e-9  # north_star's tolerance for double SUM / AVG

# (small magnitude, large magnitude) of the even / odd groups
RANGES = {
    "milli_tera": (1e-3, 1e12),     # 5 parts, fixed point
    "tiny_unit": (1e-20, 1.0),      # 6 parts, fixed point
    "extreme": (1e-200, 1e200),     # beyond 6 parts: float64 section
}


def _segments(kind, vtype=PGPU_DOUBLE, nseg=3, n=40_000, groups=64, seed=5):
    lo, hi = RANGES[kind]
    rng = np.random.default_rng(seed)
    out = []
    for i in range(nseg):
        a = rng.integers(0, groups, n)
        mag = np.where(a % 2 == 0, lo, hi)
        d = mag * rng.uniform(1.0, 2.0, n) * rng.choice([1.0, 1.0, 1.0, -1.0], n)  # mostly positive, random mantissas
        if vtype == PGPU_FLOAT:
            d = d.astype(np.float32)
        out.append(build_segment(f"fx_{kind}_{i}", {"a": (PGPU_INT, a), "d": (vtype, d)}, sorted_columns=()))
    return out


def _exact_by_group(segs, pred=None):
    vals = {}
    for s in segs:
        ds = DecodedSegment(s)
        a, d = np.asarray(ds.values("a")), np.asarray(ds.values("d"), dtype=np.float64)
        keep = np.ones(len(a), bool) if pred is None else pred(a)
        for k in np.unique(a[keep]):
            vals.setdefault(int(k), []).append(d[keep & (a == k)])
    return {k: np.concatenate(v) for k, v in vals.items()}


def _run(ctx, segs, sql, **kw):
    gs = [GpuSegment(ctx, s) for s in segs]
    try:
        return GpuPlanMaker(ctx, **kw).execute(parse_sql(sql), gs)
    finally:
        for g in gs:
            g.release()


def _layout(ctx, segs, sql, **kw):
    gs = [GpuSegment(ctx, s) for s in segs]
    try:
        pm = GpuPlanMaker(ctx, **kw)
        desc, keep, _ = pm.build_desc(parse_sql(sql), gs)
        return pm.layout(desc)
    finally:
        for g in gs:
            g.release()


@pytest.mark.parametrize("vtype", [PGPU_DOUBLE, PGPU_FLOAT], ids=["double", "float"])
@pytest.mark.parametrize("kind", list(RANGES))
@pytest.mark.parametrize("flags", ["dense", "hash"])
def test_group_sums_wide_range(gpu_ctx, kind, flags, vtype):
    if vtype == PGPU_FLOAT and kind == "extreme":
        pytest.skip("1e+-200 is not a float")
    segs = _segments(kind, vtype)
    sql = "SELECT a, SUM(d), AVG(d), COUNT(*) FROM t GROUP BY a ORDER BY a LIMIT 100"
    qf = _lib.PGPU_Q_HASH if flags == "hash" else 0
    L = _layout(gpu_ctx, segs, sql, query_flags=qf)
    e, parts = fixed_sum_layout(np.concatenate([np.asarray(DecodedSegment(s).values("d"), np.float64) for s in segs]))
    if e == _lib.PGPU_SUM_EXP_F64:
        assert L.section_op[L.agg_section[0]] == _lib.PGPU_RED_SUM_F64 and kind == "extreme"
    else:
        assert (L.agg_sum_exp[0], L.agg_sum_parts[0]) == (e, parts), (L.agg_sum_exp[0], L.agg_sum_parts[0], e, parts)
        assert parts >= 5 or vtype == PGPU_FLOAT
    res = _run(gpu_ctx, segs, sql, query_flags=qf)
    ref = engine.execute(parse_sql(sql), segs)
    check_groups(res, ref, REL)
    exact = _exact_by_group(segs)
    assert len(res.rows) == len(exact)
    for r in res.rows:
        v = exact[r[0]]
        s = math.fsum(v)
        assert close(r[1], s, REL), (kind, r[0], r[1], s)
        assert close(r[2], s / len(v), REL), (kind, r[0], r[2], s / len(v))
        if e != _lib.PGPU_SUM_EXP_F64:  # fixed point: within 2^-41 of sum|v| of the exact sum
            assert abs(r[1] - s) <= 2.0 ** -41 * float(np.abs(v).sum()) + abs(s) * 2.0 ** -52
    if e != _lib.PGPU_SUM_EXP_F64:  # deterministic: integer adds
        again = _run(gpu_ctx, segs, sql, query_flags=qf)
        assert again.rows == res.rows


@pytest.mark.parametrize("kind", ["milli_tera", "tiny_unit"])
def test_filtered_sum_of_small_rows(gpu_ctx, kind):
    """The advisor's case: a filter that keeps only the small-magnitude rows of a wide-range column."""
    segs = _segments(kind)
    sql = "SELECT SUM(d), AVG(d), COUNT(*) FROM t WHERE a IN (0, 2, 4, 6)"
    res = _run(gpu_ctx, segs, sql)
    ref = engine.execute(parse_sql(sql), segs)
    v = np.concatenate(list(_exact_by_group(segs, lambda a: np.isin(a, [0, 2, 4, 6])).values()))
    s = math.fsum(v)
    assert s != 0 and abs(s) < 1e2  # the small rows only: ~1e-3 each
    assert close(res.aggregation_result[0], s, REL), (res.aggregation_result[0], s)
    assert close(res.aggregation_result[1], s / len(v), REL)
    assert all(close(x, y, REL) for x, y in zip(res.aggregation_result, ref.aggregation_result))


@pytest.mark.parametrize("order", ["SUM(d) ASC", "SUM(d) DESC", "AVG(d) ASC"])
def test_topk_over_wide_range_sums(gpu_ctx, order):
    """The GPU ORDER BY trim keys fixed-point sums of 5 parts (pgpu_parts_to_double): the same groups, in the same
    order, as the untrimmed table, and the oracle's order values."""
    segs = _segments("milli_tera", nseg=2, n=60_000, groups=12_000)
    sql = f"SELECT a, SUM(d), AVG(d), COUNT(*) FROM t GROUP BY a ORDER BY {order}, a LIMIT 20"
    trimmed = _run(gpu_ctx, segs, sql)
    full = _run(gpu_ctx, segs, sql, gpu_topk=False)
    assert len(trimmed.group_rows) < len(full.group_rows)
    assert [list(r) for r in trimmed.rows] == [list(r) for r in full.rows]
    ref = engine.execute(parse_sql(sql), segs)
    col = 1 if order.startswith("SUM") else 2
    assert all(close(x[col], y[col], REL) for x, y in zip(trimmed.rows, ref.rows))


@pytest.mark.parametrize("flags", [0, _lib.PGPU_Q_HASH], ids=["dense", "hash"])
def test_node_combine_wide_range(flags):
    """pgpu_node_query over a one-device clique: the agreed layout (pgpu_sum_layout_agree) and the merge."""
    from pinot_amd.node import GpuNode
    segs = _segments("milli_tera", nseg=2)
    sql = "SELECT a, SUM(d), AVG(d), COUNT(*) FROM t GROUP BY a ORDER BY a LIMIT 100"
    with GpuNode([0], query_flags=flags) as node:
        gs = [GpuSegment(node.contexts[0], s) for s in segs]
        try:
            res = node.execute(parse_sql(sql), [gs])
        finally:
            for g in gs:
                g.release()
    ref = engine.execute(parse_sql(sql), segs)
    check_groups(res, ref, REL)
    exact = _exact_by_group(segs)
    for r in res.rows:
        assert close(r[1], math.fsum(exact[r[0]]), REL)
