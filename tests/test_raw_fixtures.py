"""The raw forward-index reader pinned on the reference's own files.

`tests/golden/fixedByteSVRDoubles.v1` (version 1, SNAPPY, 10,009 docs), `fixedByteCompressed.v2` (version 2,
SNAPPY, 2,000 docs) and `fixedByteRaw.v2` (version 2, PASS_THROUGH, 2,000 docs) are data files of the reference's
test resources (pinot-core/src/test/resources/data/), written by the Java FixedByteChunkSVForwardIndexWriter and
snappy-java.  Their analytic answer is value(doc i) = i + startValue
(FixedByteChunkSVForwardIndexTest.java:259-291: startValue 0 for v1, 100.2356 for both v2 files).

CPU: the oracle's restatement (oracle/rawfwd.py) decodes each file to exactly those doubles.  GPU (`-m gpu`): each
file is uploaded unchanged through pgpu_segment_add_raw_forward_index (DOUBLE, decoded by pgpu_rawfwd.cpp) and
queried through the C ABI: COUNT / MIN / MAX and the matched doc counts of raw-scan RANGE / EQ / IN leaves are
compared bit-exactly with the analytic values; SUM / AVG within north_star's 1e-9 relative (the GPU's fp64 SUM adds
in a parallel order; the values themselves are pinned exactly by MIN / MAX and the EQ leaves).
"""
import os

import numpy as np
import pytest

from oracle import engine, rawfwd
from oracle.segment_writer import build_segment
from pinot_amd._lib import PGPU_DOUBLE, PGPU_INT
from pinot_amd.query import parse_sql

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
# (file, numDocs, startValue, version, ChunkCompressionType ordinal) -- FixedByteChunkSVForwardIndexTest.java:262-276
FIXTURES = [("fixedByteSVRDoubles.v1", 10009, 0.0, 1, rawfwd.SNAPPY),
            ("fixedByteCompressed.v2", 2000, 100.2356, 2, rawfwd.SNAPPY),
            ("fixedByteRaw.v2", 2000, 100.2356, 2, rawfwd.PASS_THROUGH)]


def _bytes(name: str) -> bytes:
    with open(os.path.join(GOLDEN, name), "rb") as f:
        return f.read()


def _expected(n: int, start: float) -> np.ndarray:
    # Java's `i + startValue`: int widened to double, one IEEE addition -- the same as numpy's float64 add
    return np.arange(n, dtype=np.float64) + start


def _segment(name: str, n: int, start: float):
    """A segment whose raw DOUBLE column `v` is the reference's file byte for byte, next to a dictionary-encoded
    INT column `d` (doc % 7) to group by."""
    seg = build_segment("fixture", {"v": (PGPU_DOUBLE, _expected(n, start)),
                                    "d": (PGPU_INT, (np.arange(n) % 7).astype(np.int32))},
                        raw=("v",), sorted_columns=())
    seg.columns["v"].raw_forward = _bytes(name)
    return seg


@pytest.mark.parametrize("name,n,start,version,codec", FIXTURES)
def test_oracle_decodes_reference_file(name, n, start, version, codec):
    b = _bytes(name)
    hdr = np.frombuffer(b[:4], dtype=">i4")
    assert hdr[0] == version
    if version > 1:  # version 2+: the compression type's ordinal sits in the header (BaseChunkSVForwardIndexReader)
        assert np.frombuffer(b[20:24], dtype=">i4")[0] == codec
    v = rawfwd.read_raw_forward(b, PGPU_DOUBLE, n)
    assert v.dtype == np.float64 and len(v) == n
    assert np.array_equal(v.view(np.int64), _expected(n, start).view(np.int64))  # bit-exact


def _queries(n, start):
    lo, hi = start + n // 5, start + (3 * n) // 4 + 0.5
    eq = [start + 17, start + n - 1]
    return [
        ("SELECT COUNT(*), SUM(v), MIN(v), MAX(v), AVG(v) FROM t", np.ones(n, bool)),
        (f"SELECT COUNT(*), SUM(v), MIN(v), MAX(v) FROM t WHERE v BETWEEN {lo!r} AND {hi!r}", None),
        (f"SELECT COUNT(*), MIN(v), MAX(v) FROM t WHERE v = {eq[0]!r} OR v IN ({eq[1]!r}, -1.5)", None),
        (f"SELECT d, COUNT(*), SUM(v), MAX(v) FROM t WHERE v > {lo!r} GROUP BY d", None),
    ]


@pytest.mark.parametrize("name,n,start,version,codec", FIXTURES)
def test_oracle_queries_reference_file(name, n, start, version, codec):
    seg = _segment(name, n, start)
    vals = _expected(n, start)
    for sql, _ in _queries(n, start):
        ref = engine.execute(parse_sql(sql), [seg])
        _check_analytic(sql, ref.aggregation_result, ref.group_rows, ref.num_docs_scanned, vals, n, start)


def _analytic_mask(sql: str, vals: np.ndarray, n: int, start: float) -> np.ndarray:
    lo, hi = start + n // 5, start + (3 * n) // 4 + 0.5
    if "BETWEEN" in sql:
        return (vals >= lo) & (vals <= hi)
    if "v = " in sql:
        return (vals == start + 17) | (vals == start + n - 1) | (vals == -1.5)
    if "v > " in sql:
        return vals > lo
    return np.ones(n, bool)


def _check_analytic(sql, agg, group_rows, matched, vals, n, start):
    m = _analytic_mask(sql, vals, n, start)
    assert matched == int(m.sum()), sql
    sel = vals[m]
    if group_rows is None:
        names = [s.strip().split("(")[0] for s in sql.split("FROM")[0][len("SELECT "):].split(",")]
        exp = {"COUNT": len(sel), "SUM": float(sel.sum()), "MIN": float(sel.min()), "MAX": float(sel.max()),
               "AVG": float(sel.mean())}
        for fn, got in zip(names, agg):
            if fn in ("SUM", "AVG"):
                assert got == pytest.approx(exp[fn], rel=1e-9), (sql, fn)
            else:
                assert got == exp[fn], (sql, fn)  # COUNT, MIN, MAX: bit-exact
        return
    d = np.arange(n) % 7
    got = {r[0]: r[1:] for r in group_rows}
    assert sorted(got) == sorted(set(d[m].tolist())), sql
    for g, (cnt, s, mx) in got.items():
        gv = vals[m & (d == g)]
        assert cnt == len(gv) and mx == float(gv.max()), (sql, g)
        assert s == pytest.approx(float(gv.sum()), rel=1e-9), (sql, g)


@pytest.mark.gpu
@pytest.mark.parametrize("name,n,start,version,codec", FIXTURES)
def test_gpu_queries_reference_file(gpu_ctx, name, n, start, version, codec):
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment

    seg = _segment(name, n, start)
    vals = _expected(n, start)
    g = GpuSegment(gpu_ctx, seg)
    try:
        for sql, _ in _queries(n, start):
            res = GpuPlanMaker(gpu_ctx).execute(parse_sql(sql), [g])
            _check_analytic(sql, res.aggregation_result, res.group_rows, res.stats.num_docs_scanned, vals, n, start)
            ref = engine.execute(parse_sql(sql), [seg], iterator_stats=True)
            assert res.stats.num_entries_scanned_in_filter == ref.num_entries_scanned_in_filter, sql
    finally:
        g.release()
