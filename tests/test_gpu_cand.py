"""Candidate iteration from a sparse leading inverted leaf (query_kernel_cand), MI355X only.

AndDocIdSet.iterator walks the index child's bitmap and applies the scan children to those docs only
(AndDocIdSet.java:87-140, SVScanDocIdIterator.applyAnd :79-94).  When every segment's dense program is one inclusive
inverted leaf holding few docs, the GPU launches over that leaf's Roaring containers instead of the segment's tiles.
Each case runs the same query with the path (kernel_variant PGPU_KV_CAND) and without it (PGPU_NO_CAND=1, the tile
sweep over the expanded bitmap), both against the oracle: results, numDocsScanned, numSegmentsMatched and the
reference's numEntriesScannedInFilter where the GPU reports it as exact -- for every container kind (array, bitmap,
run), aggregation-only / dense / hash group-by modes, and segments the leaf does not touch."""
import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import build_segment, inverted_index_bytes
from pinot_amd import _lib
from pinot_amd.plan import GpuPlanMaker
from pinot_amd.query import parse_sql
from pinot_amd.segment import GpuSegment
from tests.helpers import check_groups, close

pytestmark = pytest.mark.gpu


def _segments(seed=11, nseg=3, n=200_003, force=None, bitmap=False, card=40_000):
    """`a`: 40,000 ids (~5 docs each per segment, inverted); `d`, `e`: scan columns; `g`: group key; `m`, `x`:
    metrics.  `force` rewrites a's inverted index with one container kind (array or run: the portable format takes
    a container of <= 4,096 values for an array, so bitmap containers come from `bitmap`: 5,000 docs of id 77 spread
    over the second container key of the last segment)."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(nseg):
        a = rng.integers(0, card, n)
        if i == 1:  # long runs of one id (run containers in the portable format) in the second segment
            a[50_000:50_600] = 77  # (sparse enough that the scan children stay per-candidate residuals)
            a[120_000:120_500] = 1234
        if bitmap and i == nseg - 1:
            a[65_536 + rng.choice(65_536, 5_000, replace=False)] = 77
        cols = {"a": (_lib.PGPU_INT, a), "d": (_lib.PGPU_INT, rng.integers(0, 100, n)),
                "e": (_lib.PGPU_INT, rng.integers(0, 3, n)), "g": (_lib.PGPU_INT, rng.integers(0, 50, n)),
                "m": (_lib.PGPU_INT, rng.integers(-1000, 100_000, n)),
                "x": (_lib.PGPU_DOUBLE, rng.normal(0, 1e3, n))}
        seg = build_segment(f"cand{i}", cols, inverted=["a"], sorted_columns=[])
        if force is not None:
            col = seg.column("a")
            col.inverted = inverted_index_bytes(engine.DecodedSegment(seg).ids("a"), col.cardinality, True, force)
        out.append(seg)
    return out


QUERIES = [
    "SELECT COUNT(*), SUM(m), MIN(m), MAX(x) FROM t WHERE a IN (5, 77, 1234, 39999) AND d BETWEEN 10 AND 60",
    "SELECT g, SUM(m), COUNT(*), AVG(x) FROM t WHERE a IN (77, 1234) AND d > 3 GROUP BY g",
    "SELECT COUNT(*), SUM(x) FROM t WHERE a = 77",
    "SELECT g, MAX(m), MIN(m) FROM t WHERE a IN (1, 2, 3, 77) AND (d < 5 OR e = 2) AND NOT (g = 7) "
    "GROUP BY g ORDER BY MAX(m) DESC LIMIT 10",
    "SELECT e, d, COUNT(*), SUM(m) FROM t WHERE a IN (77, 500) AND e <> 1 GROUP BY e, d",
    "SELECT COUNT(*) FROM t WHERE a = 2000000 AND d > 5",  # literal absent: EMPTY in every segment
]


def _run(ctx, segs, sql, **kw):
    gs = [GpuSegment(ctx, s) for s in segs]
    try:
        return GpuPlanMaker(ctx, **kw).execute(parse_sql(sql), gs)
    finally:
        for g in gs:
            g.release()


def _check(res, ref):
    if res.aggregation_result is not None:
        assert all(close(a, b, 1e-9) for a, b in zip(res.aggregation_result, ref.aggregation_result)), \
            (res.aggregation_result, ref.aggregation_result)
    else:
        check_groups(res, ref, 1e-9)
    assert res.stats.num_docs_scanned == ref.num_docs_scanned
    assert res.stats.num_total_docs == ref.num_total_docs
    assert res.stats.num_segments_matched == ref.num_segments_matched
    if res.stats.filter_stats_exact:
        assert res.stats.num_entries_scanned_in_filter == ref.num_entries_scanned_in_filter


@pytest.mark.parametrize("force", [None, "array", "run"])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_cand_vs_oracle(gpu_ctx, monkeypatch, qi, force):
    segs = _segments(force=force)
    sql = QUERIES[qi]
    ref = engine.execute(parse_sql(sql), segs, iterator_stats=True)
    res = _run(gpu_ctx, segs, sql)
    if qi != len(QUERIES) - 1:  # (all segments EMPTY: no kernel work at all)
        assert res.stats.kernel_variant == _lib.PGPU_KV_CAND, res.stats.kernel_variant
    _check(res, ref)
    monkeypatch.setenv("PGPU_NO_CAND", "1")
    sweep = _run(gpu_ctx, segs, sql)
    assert sweep.stats.kernel_variant != _lib.PGPU_KV_CAND
    _check(sweep, ref)
    assert res.stats.num_entries_scanned_in_filter == sweep.stats.num_entries_scanned_in_filter


@pytest.mark.parametrize("sql", ["SELECT COUNT(*), SUM(x), MAX(m) FROM t WHERE a = 77",
                                 "SELECT g, COUNT(*), MIN(x) FROM t WHERE a IN (5, 77) GROUP BY g"])
def test_cand_bitmap_container(gpu_ctx, sql):
    """A bitmap container (5,000 docs of one id under one key) read through the wave's LDS image."""
    segs = _segments(seed=13, bitmap=True)
    res = _run(gpu_ctx, segs, sql)
    assert res.stats.kernel_variant == _lib.PGPU_KV_CAND
    _check(res, engine.execute(parse_sql(sql), segs, iterator_stats=True))


@pytest.mark.parametrize("qi", [1, 4])
def test_cand_hash_groupby(gpu_ctx, qi):
    """The hash group-key holder (PGPU_Q_HASH) behind the candidate kernel."""
    segs = _segments(seed=3)
    sql = QUERIES[qi]
    res = _run(gpu_ctx, segs, sql, query_flags=_lib.PGPU_Q_HASH)
    assert res.stats.kernel_variant == _lib.PGPU_KV_CAND
    _check(res, engine.execute(parse_sql(sql), segs, iterator_stats=True))


def test_cand_exact_filter_stats(gpu_ctx):
    """With the reference's numEntriesScannedInFilter requested the leaf is still expanded for the replay, and the
    count equals the oracle's iterator figure."""
    segs = _segments(seed=5, nseg=2)
    sql = QUERIES[0]
    res = _run(gpu_ctx, segs, sql, exact_filter_stats=True)
    ref = engine.execute(parse_sql(sql), segs, iterator_stats=True)
    assert res.stats.kernel_variant == _lib.PGPU_KV_CAND
    assert res.stats.filter_stats_exact
    _check(res, ref)


def test_cand_density_threshold(gpu_ctx, monkeypatch):
    """A leaf above the density bound (3 of 40 ids, ~7.5 % of the docs) takes the tile sweep; raising the bound to 1
    takes the candidate kernel for it, with the same results.  (A long IN list whose containers outnumber the
    segment's tiles keeps the sweep whatever the bound.)"""
    segs = _segments(seed=9, nseg=2, card=40)
    sql = "SELECT g, COUNT(*), SUM(m) FROM t WHERE a IN (0, 1, 2) GROUP BY g"
    ref = engine.execute(parse_sql(sql), segs, iterator_stats=True)
    dense = _run(gpu_ctx, segs, sql)
    assert dense.stats.kernel_variant != _lib.PGPU_KV_CAND
    _check(dense, ref)
    monkeypatch.setenv("PGPU_CAND_DENSITY", "1.0")
    forced = _run(gpu_ctx, segs, sql)
    assert forced.stats.kernel_variant == _lib.PGPU_KV_CAND
    _check(forced, ref)
    many = _segments(seed=9, nseg=1)
    sql = f"SELECT COUNT(*), SUM(m) FROM t WHERE a IN ({', '.join(map(str, range(0, 6000, 3)))})"
    res = _run(gpu_ctx, many, sql)
    assert res.stats.kernel_variant != _lib.PGPU_KV_CAND
    _check(res, engine.execute(parse_sql(sql), many, iterator_stats=True))


def test_cand_adanalytics_inv(gpu_ctx):
    """The bench's accountId-inverted config 5 variant on small segments: the candidate kernel, oracle parity."""
    from oracle.segment_writer import pack_fixed_bit
    from pinot_amd.synth import WORKLOADS, build_segment_cpu
    w = WORKLOADS["adanalytics_inv"]
    segs = [build_segment_cpu(w, s, 1 << 18, pack_fixed_bit) for s in range(3)]
    res = _run(gpu_ctx, segs, w.sql)
    assert res.stats.kernel_variant == _lib.PGPU_KV_CAND
    _check(res, engine.execute(parse_sql(w.sql), segs, iterator_stats=True))


def _sorted_segments(seed=17, nseg=2, n=200_003):
    """`s` sorted (SortedIndexBasedFilterOperator leaves: doc ranges), ~40 docs per value."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(nseg):
        cols = {"s": (_lib.PGPU_INT, np.sort(rng.integers(0, 5_000, n))), "d": (_lib.PGPU_INT, rng.integers(0, 100, n)),
                "e": (_lib.PGPU_INT, rng.integers(0, 3, n)), "g": (_lib.PGPU_INT, rng.integers(0, 50, n)),
                "m": (_lib.PGPU_INT, rng.integers(-1000, 100_000, n))}
        out.append(build_segment(f"sorted{i}", cols, sorted_columns=["s"]))
    return out


def test_cand_sorted_leading_leaf(gpu_ctx, monkeypatch):
    """A sorted leading leaf: its doc ranges, split at 65,536-doc keys (one range crosses doc 65,536), are the units."""
    segs = _sorted_segments()
    sv = np.asarray(engine.DecodedSegment(segs[0]).values("s"))
    lo, hi = int(sv[65_500]), int(sv[65_600])
    for sql in (f"SELECT COUNT(*), SUM(m) FROM t WHERE s BETWEEN {lo} AND {hi} AND d < 50",
                "SELECT g, COUNT(*), MAX(m) FROM t WHERE s IN (17, 2500, 4999) AND e <> 1 GROUP BY g",
                "SELECT COUNT(*), MIN(m) FROM t WHERE s = 3000"):
        ref = engine.execute(parse_sql(sql), segs, iterator_stats=True)
        res = _run(gpu_ctx, segs, sql)
        assert res.stats.kernel_variant == _lib.PGPU_KV_CAND, (sql, res.stats.kernel_variant)
        _check(res, ref)
        monkeypatch.setenv("PGPU_NO_CAND", "1")
        _check(_run(gpu_ctx, segs, sql), ref)
        monkeypatch.delenv("PGPU_NO_CAND")


@pytest.mark.parametrize("sql", ["SELECT COUNT(*), SUM(m), MAX(x) FROM t WHERE a IN (77, 88)",
                                 "SELECT g, COUNT(*), SUM(m) FROM t WHERE a IN (77, 88) GROUP BY g",
                                 "SELECT COUNT(*), SUM(m) FROM t WHERE a = 88",
                                 "SELECT COUNT(*), SUM(m), MAX(x) FROM t WHERE a IN (77, 88) AND d < 90"])
def test_cand_chunk_above_queue_capacity(gpu_ctx, monkeypatch, sql):
    """More than a candidate queue's 1,024 entries inside one 2,048-doc piece of a container: a run of 2,000 docs
    of id 77 (1,760 of them in the tile at doc 10,240) and a bitmap container of id 88 whose first 2,048 docs hold
    1,900 set bits.  The image is enumerated in queue-sized halves; results equal the oracle's and the tile sweep's."""
    segs = []
    rng = np.random.default_rng(21)
    for i in range(2):
        n = 200_003
        a = rng.integers(0, 40_000, n)
        a[10_000:12_000] = 77
        a[65_536:65_536 + 1_900] = 88
        a[65_536 + 2_048 + rng.choice(60_000, 4_000, replace=False)] = 88
        cols = {"a": (_lib.PGPU_INT, a), "d": (_lib.PGPU_INT, rng.integers(0, 100, n)),
                "g": (_lib.PGPU_INT, rng.integers(0, 50, n)), "m": (_lib.PGPU_INT, rng.integers(-1000, 100_000, n)),
                "x": (_lib.PGPU_DOUBLE, rng.normal(0, 1e3, n))}
        segs.append(build_segment(f"bigchunk{i}", cols, inverted=["a"], sorted_columns=[]))
    ref = engine.execute(parse_sql(sql), segs, iterator_stats=True)
    res = _run(gpu_ctx, segs, sql)
    # (with a d residual the clustered runs make d's sectors dense, and SUM(m) alone is answered from value planes
    # by the container-keyed kernel: either may take another kernel; the others must take this one)
    if " AND d " not in sql and "MAX(x)" in sql or "GROUP BY" in sql:
        assert res.stats.kernel_variant == _lib.PGPU_KV_CAND
    _check(res, ref)
    monkeypatch.setenv("PGPU_NO_CAND", "1")
    _check(_run(gpu_ctx, segs, sql), ref)
