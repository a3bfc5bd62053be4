"""Non-scan aggregation plan (AggregationPlanNode.buildNonFilteredAggOperator, core/plan/AggregationPlanNode.java
:171-195; NonScanBasedAggregationOperator.java:85-101,253-256): a filter that folds to match-all with only COUNT /
MIN / MAX is answered from metadata and dictionaries, per segment, with statistics (numTotalDocs, 0, 0,
numTotalDocs).  Values must equal the scan plan's; the choice is per segment, so one query can mix both."""
import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import build_segment
from pinot_amd._lib import PGPU_DOUBLE, PGPU_INT
from pinot_amd.query import parse_sql
from tests.helpers import close, sv_segment


def _two_segments():
    rng = np.random.default_rng(11)
    a = {"x": (PGPU_INT, rng.integers(0, 100, 5000).astype(np.int32)),
         "d": (PGPU_DOUBLE, np.round(rng.normal(0, 10, 5000), 2))}
    b = {"x": (PGPU_INT, rng.integers(50, 150, 7000).astype(np.int32)),
         "d": (PGPU_DOUBLE, np.round(rng.normal(5, 10, 7000), 2))}
    return [build_segment("a", a), build_segment("b", b)]


NON_SCAN = "SELECT COUNT(*), MIN(x), MAX(d) FROM t"
# x in [0, 120): every dict id of segment a matches (folds to match-all there), segment b is scanned
MIXED = "SELECT COUNT(*), MIN(d), MAX(x) FROM t WHERE x >= 0 AND x < 120"
SCAN_EQUIV = "SELECT COUNT(*), MIN(x), MAX(d), SUM(x) FROM t"  # SUM forces the scan plan


def test_non_scan_oracle_stats_and_values():
    segs = _two_segments()
    r = engine.execute(parse_sql(NON_SCAN), segs)
    assert (r.num_docs_scanned, r.num_entries_scanned_in_filter, r.num_entries_scanned_post_filter,
            r.num_total_docs) == (12000, 0, 0, 12000)
    s = engine.execute(parse_sql(SCAN_EQUIV), segs)
    assert r.aggregation_result == s.aggregation_result[:3]
    assert s.num_entries_scanned_post_filter == 12000 * 2  # distinct projected columns x, d


def test_non_scan_oracle_mixed_segments():
    segs = _two_segments()
    r = engine.execute(parse_sql(MIXED), segs)
    x_b = segs[1]
    rb = engine.execute(parse_sql(MIXED), [x_b])
    assert rb.num_entries_scanned_post_filter > 0  # segment b is scanned
    assert r.num_entries_scanned_post_filter == rb.num_entries_scanned_post_filter  # segment a adds nothing
    assert r.num_docs_scanned == 5000 + rb.num_docs_scanned


@pytest.mark.gpu
@pytest.mark.parametrize("sql", [NON_SCAN, MIXED, SCAN_EQUIV, "SELECT COUNT(*) FROM t", "SELECT MAX(x) FROM t "
                                 "WHERE x >= 0"])
def test_non_scan_gpu_vs_oracle(gpu_ctx, sql):
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    segs = _two_segments()
    g = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        q = parse_sql(sql)
        res = GpuPlanMaker(gpu_ctx).execute(q, g)
        ref = engine.execute(q, segs)
        assert all(close(u, v) for u, v in zip(res.aggregation_result, ref.aggregation_result))
        assert (res.stats.num_docs_scanned, res.stats.num_entries_scanned_post_filter, res.stats.num_total_docs) == \
            (ref.num_docs_scanned, ref.num_entries_scanned_post_filter, ref.num_total_docs)
    finally:
        for s in g:
            s.release()


@pytest.mark.gpu
def test_non_scan_kat_segment_gpu(gpu_ctx):
    """BaseSingleValueQueriesTest segment: the dictionary answer equals the scanned MIN / MAX."""
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    seg = sv_segment()
    g = GpuSegment(gpu_ctx, seg)
    try:
        pm = GpuPlanMaker(gpu_ctx)
        a = pm.execute(parse_sql("SELECT COUNT(*), MIN(column1), MAX(column3) FROM testTable"), [g, g])
        b = pm.execute(parse_sql("SELECT COUNT(*), MIN(column1), MAX(column3), SUM(column1) FROM testTable"), [g, g])
        assert a.aggregation_result == b.aggregation_result[:3]
        assert a.stats.num_entries_scanned_post_filter == 0 and a.stats.num_docs_scanned == 2 * seg.num_docs
    finally:
        g.release()


@pytest.mark.gpu
def test_non_scan_distributed_executor_single_gpu(gpu_ctx):
    from pinot_amd.combine import DistributedExecutor
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    segs = _two_segments()
    g = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        q = parse_sql(MIXED)
        res = DistributedExecutor(GpuPlanMaker(gpu_ctx)).execute(q, g)
        ref = engine.execute(q, segs)
        assert all(close(u, v) for u, v in zip(res.aggregation_result, ref.aggregation_result))
        assert res.stats.num_entries_scanned_post_filter == ref.num_entries_scanned_post_filter
    finally:
        for s in g:
            s.release()
