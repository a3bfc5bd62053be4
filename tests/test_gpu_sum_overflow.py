"""Integer SUM / AVG beyond int64 and beyond 2^53 (MI355X only).

The reference adds values as doubles in doc order and never wraps (SumAggregationFunction.java:55-92).  The GPU sums
integers exactly: one int64 cell while max|value| x docs < 2^62, else three exact sums of 21-bit parts
(include/pinot_gpu.h, agg_sum_parts), joined on the host and rounded once.  Compared with the oracle's doc-order
double sum within 1e-9 relative (north_star's tolerance for double SUM / AVG)."""
import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import build_segment
from pinot_amd._lib import PGPU_INT, PGPU_LONG, PGPU_Q_SUM_SPLIT
from pinot_amd.plan import GpuPlanMaker
from pinot_amd.query import parse_sql
from pinot_amd.segment import GpuSegment
from tests.helpers import check_groups, close, rows_close

pytestmark = pytest.mark.gpu


def _segments(rng, n, nseg, lo, hi, card=4000):
    segs = []
    for i in range(nseg):
        base = np.sort(rng.choice(np.arange(lo, hi, (hi - lo) // (card * 4), dtype=np.int64), card, replace=False))
        v = base[rng.integers(0, card, n)]
        g = rng.integers(0, 7, n).astype(np.int32)
        f = rng.integers(0, 100, n).astype(np.int32)
        segs.append(build_segment(f"ovf{i}", {"v": (PGPU_LONG, v), "g": (PGPU_INT, g), "f": (PGPU_INT, f)}))
    return segs


def _check(gpu_ctx, sql, segs, flags=0):
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        q = parse_sql(sql)
        res = GpuPlanMaker(gpu_ctx, query_flags=flags).execute(q, gs)
        ref = engine.execute(q, segs)
        if q.group_by:
            check_groups(res, ref, 1e-9)
        else:
            for a, b in zip(res.aggregation_result, ref.aggregation_result):
                assert close(a, b, 1e-9), (res.aggregation_result, ref.aggregation_result)
        assert res.stats.num_docs_scanned == ref.num_docs_scanned
        return res
    finally:
        for g in gs:
            g.release()


QUERIES = [
    "SELECT COUNT(*), SUM(v), AVG(v), MIN(v), MAX(v) FROM t",
    "SELECT COUNT(*), SUM(v), AVG(v) FROM t WHERE f < 3",          # sparse: candidate queue + gathers
    "SELECT COUNT(*), SUM(v) FROM t WHERE f BETWEEN 10 AND 80",     # dense: staged tiles
    "SELECT g, SUM(v), AVG(v), MAX(v), COUNT(*) FROM t GROUP BY g",
    "SELECT g, SUM(v), COUNT(*) FROM t WHERE f < 50 GROUP BY g ORDER BY SUM(v) DESC LIMIT 3",
]


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_long_sum_beyond_int64(gpu_ctx, qi):
    """|SUM| > 2^63: epoch-micros-like values (~1e13) over 3 x 2^20 docs sum to ~3e19."""
    rng = np.random.default_rng(11 + qi)
    segs = _segments(rng, 1 << 20, 3, 9_000_000_000_000, 11_000_000_000_000)
    res = _check(gpu_ctx, QUERIES[qi], segs)
    if qi == 0:
        assert res.aggregation_result[1] > 2.0 ** 63


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_long_sum_between_2p53_and_2p63(gpu_ctx, qi):
    """2^53 < |SUM| < 2^63 with a bound below 2^62: one exact int64 cell, rounded once to double."""
    rng = np.random.default_rng(21 + qi)
    segs = _segments(rng, 1 << 19, 2, -3_000_000_000_000, 900_000_000_000)
    res = _check(gpu_ctx, QUERIES[qi], segs)
    if qi == 0:
        assert 2.0 ** 53 < abs(res.aggregation_result[1]) < 2.0 ** 63


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_forced_split_small_values(gpu_ctx, qi):
    """PGPU_Q_SUM_SPLIT on small signed values: the part sections rebuild sums exactly (negative values included)."""
    rng = np.random.default_rng(31 + qi)
    segs = _segments(rng, 200_003, 2, -5_000_000, 5_000_000)
    _check(gpu_ctx, QUERIES[qi], segs, flags=PGPU_Q_SUM_SPLIT)


def test_split_layout_is_reported(gpu_ctx):
    rng = np.random.default_rng(5)
    segs = _segments(rng, 4096, 1, 9_000_000_000_000, 11_000_000_000_000)
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        pm = GpuPlanMaker(gpu_ctx)
        q = parse_sql("SELECT SUM(v), MIN(v), SUM(f) FROM t")
        desc, keep, _ = pm.build_desc(q, gs)
        L = pm.layout(desc)
        assert [L.agg_sum_parts[i] for i in range(3)] == [1, 1, 1]  # 1e13 x 4096 docs < 2^62
        desc, keep, _ = pm.build_desc(q, gs, reduce_docs=1 << 20)
        L = pm.layout(desc)
        assert [L.agg_sum_parts[i] for i in range(3)] == [3, 1, 1]
        assert L.num_sections == 1 + 3 + 1 + 1
    finally:
        for g in gs:
            g.release()
