"""Register-direct kernel with the prefix pre-filter (DevSeg::pfx_*, plan_prefix in pgpu_runtime.cpp): config 5's
shape -- a selective bit-sliced RANGE leaf streamed in registers AND a residual EQ / IN / RANGE scan leaf on a wide
column gathered per candidate -- where the residual column's top PGPU_PFX_PLANES bit planes are streamed too and
candidates outside the matching prefixes are never gathered.  Doc sets, aggregates and the GPU's own
numEntriesScannedInFilter (every candidate still counts as one residual entry) against the oracle; the stats pass
shows the prefix planes were streamed (dense bytes = (fast-leaf bits + 3) per doc).
"""
import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import build_segment
from pinot_amd._lib import PGPU_INT
from pinot_amd.query import parse_sql
from tests.helpers import check_groups, close

N = 400_000


def _segments(seed, nseg=3):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(nseg):
        n = N - 1000 * i
        cols = {"day": (PGPU_INT, 17500 + rng.integers(0, 1024, n)),           # 10-bit fast leaf
                "acct": (PGPU_INT, rng.integers(0, 1 << 20, n) * 3),             # ~20-bit residual column
                "clicks": (PGPU_INT, rng.integers(0, 5000, n))}
        out.append(build_segment(f"p{i}", cols, sorted_columns=()))
    return out


def _queries(segs):
    d = np.frombuffer(segs[0].column("acct").dictionary, dtype=">i4")
    v1, v2, v3 = int(d[100]), int(d[len(d) // 2]), int(d[-7])
    return [
        f"SELECT day, SUM(clicks), COUNT(*) FROM t WHERE day BETWEEN 17849 AND 17856 AND acct IN ({v1}) GROUP BY day",
        f"SELECT COUNT(*), SUM(clicks) FROM t WHERE day BETWEEN 17600 AND 17615 AND acct IN ({v1}, {v2}, {v3})",
        f"SELECT COUNT(*), MAX(clicks) FROM t WHERE day BETWEEN 17700 AND 17720 AND acct BETWEEN {v2} AND {v2 + 30000}",
        f"SELECT day, COUNT(*) FROM t WHERE day < 17520 AND acct = {v3} GROUP BY day",
    ]


@pytest.mark.gpu
@pytest.mark.parametrize("qi", range(4))
def test_gpu_prefix_prefilter_vs_oracle(gpu_ctx, qi):
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    segs = _segments(11 + qi)
    q = parse_sql(_queries(segs)[qi])
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        res = GpuPlanMaker(gpu_ctx, collect_stats=True).execute(q, gs)
        exact = GpuPlanMaker(gpu_ctx, exact_filter_stats=True).execute(q, gs)
    finally:
        for g in gs:
            g.release()
    ref = engine.execute(q, segs, iterator_stats=True)
    for r in (res, exact):
        if q.group_by:
            check_groups(r, ref)
        else:
            assert all(close(a, b) for a, b in zip(r.aggregation_result, ref.aggregation_result))
        assert r.stats.num_docs_scanned == ref.num_docs_scanned
    # the reference's numEntriesScannedInFilter (its AND iterators leap-frog) from the exact-statistics replay, which
    # reads the leaves' own match bitmaps: untouched by the prefix pre-filter
    assert exact.stats.filter_stats_exact
    assert exact.stats.num_entries_scanned_in_filter == ref.num_entries_scanned_in_filter
    # the stats pass streamed the fast leaf's 10 planes and the residual column's 3 prefix planes over every segment
    # the filter does not fold to EMPTY (a literal absent from its dictionary)
    scanned = [s for s in segs if _has_all_literals(s, q)]
    assert res.stats.dense_bytes == pytest.approx(sum(s.num_docs for s in scanned) * (10 + 3) / 8, rel=0.02)


def _has_all_literals(seg, q):
    d = set(np.frombuffer(seg.column("acct").dictionary, dtype=">i4").tolist())
    for p in _leaves(q.filter):
        if p.column == "acct" and p.type in ("IN", "EQ") and not any(int(v) in d for v in p.values):
            return False
    return True


def _leaves(f):
    if f.type in ("AND", "OR", "NOT"):
        for c in f.children:
            yield from _leaves(c)
    else:
        yield f.predicate
