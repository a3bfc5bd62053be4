"""numSegmentsMatched and numGroupsLimitReached on the GPU against the oracle (MI355X only).

The reference counts a segment as matched when its operator's numDocsScanned > 0
(CombineOperatorUtils.setExecutionStatistics, CombineOperatorUtils.java:64-67) and flags numGroupsLimitReached
when a segment's group-by executor holds numGroups >= numGroupsLimit (AggregationGroupByOrderByOperator.java:111).
"""
import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import build_segment
from pinot_amd._lib import PGPU_INT
from pinot_amd.datatable import DataTable, reduce_data_tables, server_data_table
from pinot_amd.plan import GpuPlanMaker
from pinot_amd.query import parse_sql
from pinot_amd.segment import GpuSegment

pytestmark = pytest.mark.gpu


def _segments():
    """Segment 0 matches `x < 10 AND y < 10` (y independent of x); segment 1 has y = 99 - x, so the same filter
    keeps no doc although neither leaf folds away; segment 2's x lies above every literal (RANGE folds to EMPTY)."""
    rng = np.random.default_rng(4)
    n = 50_000
    out = []
    for i in range(3):
        x = rng.integers(0, 100, n)
        y = rng.integers(0, 100, n) if i == 0 else 99 - x
        if i == 2:
            x = x + 1000
        out.append(build_segment(f"m{i}", {"x": (PGPU_INT, x.astype(np.int32)), "y": (PGPU_INT, y.astype(np.int32)),
                                          "k": (PGPU_INT, rng.integers(0, 70_000, n).astype(np.int32)),
                                          "m": (PGPU_INT, rng.integers(0, 1000, n).astype(np.int32))},
                                 sorted_columns=()))
    return out


QUERIES = [
    "SELECT COUNT(*) FROM t WHERE x < 10 AND y < 10",
    "SELECT COUNT(*), SUM(m) FROM t WHERE x < 10 AND y < 10",
    "SELECT x, SUM(m) FROM t WHERE x < 10 AND y < 10 GROUP BY x ORDER BY SUM(m) DESC LIMIT 5",
    "SELECT k, COUNT(*) FROM t WHERE x < 10 AND y < 10 GROUP BY k ORDER BY COUNT(*) DESC, k LIMIT 5",
    "SELECT COUNT(*), SUM(m) FROM t WHERE x < 50",
    "SELECT COUNT(*), MAX(m) FROM t",
    "SELECT COUNT(*) FROM t WHERE x < 10 AND y < 10 OR m = 7",
]


@pytest.mark.parametrize("sql", QUERIES)
def test_num_segments_matched(gpu_ctx, sql):
    segs = _segments()
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        q = parse_sql(sql)
        res = GpuPlanMaker(gpu_ctx).execute(q, gs)
    finally:
        for g in gs:
            g.release()
    ref = engine.execute(q, segs)
    assert res.stats.num_docs_scanned == ref.num_docs_scanned
    assert res.stats.num_segments_matched == ref.num_segments_matched
    assert res.stats.segment_matched is None or list(res.stats.segment_matched) == [int(b) for b in ref.segment_matched]
    types = [PGPU_INT] * len(q.group_by)
    dt = DataTable.from_bytes(server_data_table(q, res, types).to_bytes())
    assert dt.metadata["numSegmentsMatched"] == str(ref.num_segments_matched)
    assert reduce_data_tables(q, [dt]).num_segments_matched == ref.num_segments_matched


def test_num_segments_matched_filtered_aggregations(gpu_ctx):
    """FILTER clauses run one pass each; a segment matched by any pass counts once."""
    segs = _segments()
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        q = parse_sql("SELECT COUNT(*) FILTER(WHERE x < 10 AND y < 10), SUM(m) FILTER(WHERE x >= 1000) FROM t")
        res = GpuPlanMaker(gpu_ctx).execute(q, gs)
    finally:
        for g in gs:
            g.release()
    ref = engine.execute(q, segs)
    assert res.aggregation_result == ref.aggregation_result
    assert res.stats.num_segments_matched == ref.num_segments_matched


@pytest.mark.parametrize("limit,reached", [(20_000, True), (20_001, False), (19_999, True)])
def test_num_groups_limit_reached_at_the_limit(gpu_ctx, limit, reached):
    """A segment with exactly 20,000 distinct keys: numGroups >= numGroupsLimit flags the query at a limit of
    20,000 with nothing dropped; one more and it is not flagged; one less and the first-seen cut applies."""
    rng = np.random.default_rng(9)
    n, card = 60_000, 20_000
    k = np.concatenate([np.arange(card), rng.integers(0, card, n - card)])
    rng.shuffle(k)
    seg = build_segment("lim", {"k": (PGPU_INT, (k * 3).astype(np.int32)),
                                "m": (PGPU_INT, rng.integers(0, 100, n).astype(np.int32))}, sorted_columns=())
    g = GpuSegment(gpu_ctx, seg)
    q = parse_sql("SELECT k, SUM(m), COUNT(*) FROM t GROUP BY k ORDER BY SUM(m) DESC, k LIMIT 10")
    try:
        res = GpuPlanMaker(gpu_ctx, num_groups_limit=limit).execute(q, [g])
    finally:
        g.release()
    ref = engine.execute(q, [seg], num_groups_limit=limit)
    assert ref.num_groups_limit_reached == reached
    assert res.stats.num_groups_limit_reached == reached
    assert res.rows == ref.rows


def test_derived_copies_follow_the_residency_policy(gpu_ctx):
    """pgpu_segment_set_derived / the context budget: the copies seal builds, the bytes reported by kind, and the
    same results with or without them (PhysicalColumnIndexContainer.java:80,151-156 -- only named indexes load)."""
    import numpy as np
    from oracle import engine
    from oracle.segment_writer import build_segment
    from pinot_amd import _lib
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.query import parse_sql
    from pinot_amd.segment import GpuSegment
    from tests.helpers import close
    rng = np.random.default_rng(17)
    n = 300_000
    data = build_segment("res", {"f": (_lib.PGPU_INT, rng.integers(0, 1000, n).astype(np.int32)),
                                 "g": (_lib.PGPU_INT, rng.integers(0, 50, n).astype(np.int32)),
                                 "m": (_lib.PGPU_INT, rng.integers(0, 1 << 16, n).astype(np.int32))},
                         sorted_columns=())
    sqls = ["SELECT COUNT(*), SUM(m), MAX(m) FROM t WHERE f BETWEEN 100 AND 700 AND g IN (3, 7, 11)",
            "SELECT g, SUM(m) FROM t WHERE f < 500 GROUP BY g ORDER BY g LIMIT 100"]
    used0, budget0 = gpu_ctx.derived_bytes()
    assert budget0 > 0
    variants = {"all": None, "none": {"f": 0, "g": 0, "m": 0},
                "policy": {"f": _lib.PGPU_DERIVE_SLICED, "g": _lib.PGPU_DERIVE_SLICED, "m": _lib.PGPU_DERIVE_VALUE_PLANES}}
    for name, derived in variants.items():
        seg = GpuSegment(gpu_ctx, data, derived=derived)
        try:
            b = seg.device_bytes_by_kind()
            assert b["total"] == seg.device_bytes() == sum(v for k, v in b.items() if k != "total")
            if name == "none":
                assert b["sliced"] == 0 and b["value_planes"] == 0
            elif name == "all":
                assert b["sliced"] == b["forward"] and b["value_planes"] > 0
            else:
                assert 0 < b["sliced"] < b["forward"] and b["value_planes"] > 0
            assert gpu_ctx.derived_bytes()[0] == used0 + b["sliced"] + b["value_planes"]
            for sql in sqls:
                q = parse_sql(sql)
                res = GpuPlanMaker(gpu_ctx).execute(q, [seg])
                ref = engine.execute(q, [data])
                if res.aggregation_result is not None:
                    assert all(close(x, y) for x, y in zip(res.aggregation_result, ref.aggregation_result))
                else:
                    assert res.rows == ref.rows
        finally:
            seg.release()
        assert gpu_ctx.derived_bytes()[0] == used0
    # a zero budget: no derived copy at all, whatever the flags say
    gpu_ctx.set_derived_budget(0)
    try:
        seg = GpuSegment(gpu_ctx, data)
        try:
            b = seg.device_bytes_by_kind()
            assert b["sliced"] == 0 and b["value_planes"] == 0
        finally:
            seg.release()
    finally:
        gpu_ctx.set_derived_budget(budget0)


def test_executor_config_applies_the_residency_policy(gpu_ctx):
    """GpuExecutorConfig is where a server applies its keys: upload() passes the table's derived-copy columns to
    seal, apply_budget() the byte budget (a budget of 0 builds no derived copy), plan_maker() the query options."""
    import numpy as np
    from oracle import engine
    from oracle.segment_writer import build_segment
    from pinot_amd import _lib
    from pinot_amd.config import GpuExecutorConfig
    from pinot_amd.query import parse_sql
    from tests.helpers import close
    rng = np.random.default_rng(23)
    n = 200_000
    data = build_segment("cfg", {"f": (_lib.PGPU_INT, rng.integers(0, 1000, n).astype(np.int32)),
                                 "m": (_lib.PGPU_INT, rng.integers(0, 1 << 16, n).astype(np.int32))},
                         sorted_columns=())
    cfg = GpuExecutorConfig.from_properties({"pinot.server.query.executor.gpu.sliced.columns": "f",
                                             "pinot.server.query.executor.gpu.value.planes.columns": "m"})
    seg = cfg.upload(gpu_ctx, data)
    try:
        b = seg.device_bytes_by_kind()
        assert 0 < b["sliced"] < b["forward"] and b["value_planes"] > 0
        q = parse_sql("SELECT COUNT(*), SUM(m) FROM t WHERE f < 300")
        res = cfg.plan_maker(gpu_ctx).execute(q, [seg])
        assert all(close(x, y) for x, y in zip(res.aggregation_result, engine.execute(q, [data]).aggregation_result))
    finally:
        seg.release()
    _, budget = gpu_ctx.derived_bytes()
    zero = GpuExecutorConfig.from_properties({"pinot.server.query.executor.gpu.derived.budget.bytes": "0"})
    try:
        zero.apply_budget(gpu_ctx)
        seg = zero.upload(gpu_ctx, data)
        try:
            b = seg.device_bytes_by_kind()
            assert b["sliced"] == 0 and b["value_planes"] == 0
        finally:
            seg.release()
    finally:
        gpu_ctx.set_derived_budget(budget)
