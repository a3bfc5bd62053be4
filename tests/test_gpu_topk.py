"""GPU ORDER BY ... LIMIT trim (pgpu_query_collect_topk / pgpu_table_topk), MI355X only.

The server's IndexedTable hands the broker only its top max(5 * limit, 5000) groups by the first ORDER BY
expression (GroupByUtils.java:24-41, IndexedTable.finish, TableResizer).  Here the GPU ranks the groups by that
expression's final value and returns the best k with every tie at the k-th kept, so the final ORDER BY ... LIMIT
equals the one over the full table: checked against the untrimmed GPU path (same tie order, exactly) and against
the oracle (values of the ORDER BY expression, whatever the tie order)."""
import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import build_segment
from pinot_amd import _lib
from pinot_amd._lib import PGPU_DOUBLE, PGPU_INT, PGPU_LONG
from pinot_amd.plan import GpuPlanMaker
from pinot_amd.query import parse_sql
from pinot_amd.segment import GpuSegment
from tests.helpers import close, rows_close

pytestmark = pytest.mark.gpu


def _segments(seed, nseg=3, n=60000, big=False):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(nseg):
        cols = {"a": (PGPU_INT, rng.integers(0, 160, n) * 7),
                "b": (PGPU_INT, rng.integers(0, 90, n)),
                "m": (PGPU_INT, rng.integers(-500, 5000, n)),
                "d": (PGPU_DOUBLE, np.round(rng.normal(0, 100, n), 2)),
                "l": (PGPU_LONG, rng.integers(1 << 60, 1 << 62, n) if big else rng.integers(-10**9, 10**9, n)),
                "c": (PGPU_INT, rng.integers(0, 3, n))}
        out.append(build_segment(f"s{i}", cols, sorted_columns=()))
    return out


ORDERS = [
    "SUM(m) DESC", "SUM(m) ASC", "SUM(d) DESC", "MIN(d) ASC", "MAX(m) DESC", "AVG(d) DESC", "AVG(m) ASC",
    "COUNT(*) DESC", "a DESC", "b ASC", "SUM(l) DESC",
]


def _sql(order, limit):
    return (f"SELECT a, b, SUM(m), SUM(d), MIN(d), MAX(m), AVG(d), AVG(m), COUNT(*), SUM(l) FROM t "
            f"WHERE c <> 1 GROUP BY a, b ORDER BY {order} LIMIT {limit}")


def _run(gpu_ctx, segs, sql, **kw):
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        return GpuPlanMaker(gpu_ctx, **kw).execute(parse_sql(sql), gs)
    finally:
        for g in gs:
            g.release()


def _order_column(q, res_rows):
    names = [s if isinstance(s, str) else s.result_name for s in q.select]
    ob = q.order_by[0].expression
    return [r[names.index(ob)] for r in res_rows]


@pytest.mark.parametrize("order", ORDERS)
@pytest.mark.parametrize("limit", [10, 1500])
@pytest.mark.parametrize("flags", ["dense", "hash"])
def test_topk_equals_full_ordering(gpu_ctx, order, limit, flags):
    segs = _segments(7, big=order == "SUM(l) DESC")
    sql = _sql(order, limit)
    qf = _lib.PGPU_Q_HASH if flags == "hash" else 0
    trimmed = _run(gpu_ctx, segs, sql, query_flags=qf)
    full = _run(gpu_ctx, segs, sql, query_flags=qf, gpu_topk=False)
    assert len(trimmed.group_rows) <= len(full.group_rows)
    assert len(full.group_rows) > max(5 * limit, 5000)  # the trim really cut
    assert len(trimmed.group_rows) >= max(5 * limit, 5000)
    # same groups in the same order (ties broken by ascending key on both paths), double sums included: they are
    # fixed-point integer sums on the GPU (pgpu_table_layout.agg_sum_exp), the same whatever order atomics land in
    q = parse_sql(sql)
    assert [r[:2] for r in trimmed.rows] == [r[:2] for r in full.rows]
    assert [list(r) for r in trimmed.rows] == [list(r) for r in full.rows]
    ref = engine.execute(q, segs)
    a, b = _order_column(q, trimmed.rows), _order_column(q, ref.rows)
    assert len(a) == len(b) and all(close(x, y) for x, y in zip(a, b)), (a[:5], b[:5])


def test_topk_ties_all_kept(gpu_ctx):
    """ORDER BY COUNT(*) over groups whose counts mostly tie: every group tied with the k-th comes back."""
    rng = np.random.default_rng(3)
    n = 20000
    cols = {"a": (PGPU_INT, np.arange(n) % 10000), "m": (PGPU_INT, rng.integers(0, 9, n))}
    segs = [build_segment("t", cols, sorted_columns=())]
    sql = "SELECT a, COUNT(*), SUM(m) FROM t GROUP BY a ORDER BY COUNT(*) DESC LIMIT 3"
    trimmed = _run(gpu_ctx, segs, sql)
    full = _run(gpu_ctx, segs, sql, gpu_topk=False)
    assert len(trimmed.group_rows) == 10000  # all 10,000 groups tie at count 2
    assert [r[:2] for r in trimmed.rows] == [r[:2] for r in full.rows]


def test_topk_partitioned_group_by(gpu_ctx):
    """The partitioned group-by's table (>= 65,536 keys) trimmed on the GPU."""
    rng = np.random.default_rng(5)
    n = 400000
    cols = {"k": (PGPU_INT, rng.integers(0, 150000, n)), "m": (PGPU_INT, rng.integers(0, 1 << 16, n))}
    segs = [build_segment("p", cols, sorted_columns=())]
    sql = "SELECT k, SUM(m), MAX(m), COUNT(*) FROM t GROUP BY k ORDER BY SUM(m) DESC LIMIT 100"
    trimmed = _run(gpu_ctx, segs, sql, num_groups_limit=1_000_000)
    full = _run(gpu_ctx, segs, sql, num_groups_limit=1_000_000, gpu_topk=False)
    assert [r[0] for r in trimmed.rows] == [r[0] for r in full.rows] and len(trimmed.group_rows) < len(full.group_rows)
    ref = engine.execute(parse_sql(sql), segs, num_groups_limit=1_000_000)
    assert [r[1] for r in trimmed.rows] == [r[1] for r in ref.rows]


@pytest.mark.parametrize("flags", ["dense", "hash"])
def test_double_sum_deterministic(gpu_ctx, flags):
    """SUM / AVG of a DOUBLE column are bit-identical run to run (fixed-point part sums, no float atomics) and
    within north_star's 1e-9 relative of the exactly rounded sum of each group's values (here within 2^-41 of
    sum|v|: every value exact or rounded by at most 2^-41 of itself, pgpu_fixed_sum_layout)."""
    rng = np.random.default_rng(11)
    n = 200000
    segs = []
    for i in range(2):
        cols = {"a": (PGPU_INT, rng.integers(0, 50, n)),
                "d": (PGPU_DOUBLE, rng.normal(0, 1e6, n) * rng.choice([1e-9, 1.0, 1e3], n))}
        segs.append(build_segment(f"det{i}", cols, sorted_columns=()))
    sql = "SELECT a, SUM(d), AVG(d), COUNT(*) FROM t GROUP BY a ORDER BY SUM(d) DESC LIMIT 50"
    qf = _lib.PGPU_Q_HASH if flags == "hash" else 0
    runs = [_run(gpu_ctx, segs, sql, query_flags=qf).rows for _ in range(3)]
    assert runs[0] == runs[1] == runs[2]
    import math
    from oracle.engine import DecodedSegment
    vals = {}
    for s in segs:
        ds = DecodedSegment(s)
        a, d = np.asarray(ds.values("a")), np.asarray(ds.values("d"), dtype=np.float64)
        for k in np.unique(a):
            vals.setdefault(int(k), []).append(d[a == k])
    for r in runs[0]:
        v = np.concatenate(vals[r[0]])
        exact = math.fsum(v)  # the exactly rounded sum
        assert close(r[1], exact, 1e-9), (r[0], r[1], exact)
        assert close(r[2], exact / len(v), 1e-9)
        assert abs(r[1] - exact) <= 2.0 ** -41 * float(np.abs(v).sum()) + abs(exact) * 2.0 ** -52
