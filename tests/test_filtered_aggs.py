"""Filtered aggregations, ``AGG(col) FILTER(WHERE ...)``.

Model: FilteredAggregationsTest (pinot-core/src/test/java/org/apache/pinot/queries/FilteredAggregationsTest.java),
whose assertion is that each filtered query returns the same rows as an equivalent non-filtered one, over two
30,000-row segments with INT_COL = NO_INDEX_COL = row index (:113-127) and an inverted index on INT_COL (:96-99).
Pairs from testSimpleQueries (:161-200) and testFilterVsCase (:203-290); CASE WHEN forms are restated as the
equivalent AND filter (exact here: INT_COL >= 0, so ``ELSE 0`` adds nothing to a SUM) and functions our SQL subset
does not parse (STARTSWITH, %, ABS, LN, MOD) are left out.  BOOLEAN_COL is stored as INT (0 / 1) like Pinot's
BOOLEAN stored type."""
import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import build_segment
from pinot_amd._lib import PGPU_INT
from pinot_amd.query import SqlError, parse_sql, split_filtered_aggregations
from tests.helpers import close

N = 30_000
PAIRS = [
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 9999) FROM MyTable WHERE INT_COL < 1000000",
     "SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 9999 AND INT_COL < 1000000"),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL < 3) FROM MyTable WHERE INT_COL > 1",
     "SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 1 AND INT_COL < 3"),
    ("SELECT COUNT(*) FILTER(WHERE INT_COL = 4) FROM MyTable",
     "SELECT COUNT(*) FROM MyTable WHERE INT_COL = 4"),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 8000) FROM MyTable",
     "SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 8000"),
    ("SELECT SUM(INT_COL) FILTER(WHERE NO_INDEX_COL <= 1) FROM MyTable WHERE INT_COL > 1",
     "SELECT SUM(INT_COL) FROM MyTable WHERE NO_INDEX_COL <= 1 AND INT_COL > 1"),
    ("SELECT AVG(INT_COL) FILTER(WHERE NO_INDEX_COL > -1) FROM MyTable",
     "SELECT AVG(INT_COL) FROM MyTable"),
    ("SELECT MIN(INT_COL) FILTER(WHERE NO_INDEX_COL > 29990), MAX(INT_COL) FILTER(WHERE INT_COL > 29990) FROM MyTable",
     "SELECT MIN(INT_COL), MAX(INT_COL) FROM MyTable WHERE INT_COL > 29990"),
    ("SELECT SUM(INT_COL) FILTER(WHERE BOOLEAN_COL = 1) FROM MyTable",
     "SELECT SUM(INT_COL) FROM MyTable WHERE BOOLEAN_COL = 1"),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 1234 AND INT_COL < 22000) FROM MyTable",
     "SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 1234 AND INT_COL < 22000"),
    ("SELECT MAX(INT_COL) FILTER(WHERE INT_COL < 100) FROM MyTable",
     "SELECT MAX(INT_COL) FROM MyTable WHERE INT_COL < 100"),
    ("SELECT MIN(NO_INDEX_COL) FILTER(WHERE INT_COL < 100) FROM MyTable",
     "SELECT MIN(NO_INDEX_COL) FROM MyTable WHERE INT_COL < 100"),
]
# mixed filtered / non-filtered and several FILTER clauses: expected values per aggregation from the
# non-filtered equivalents (one query each)
MIXED = [
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 3), SUM(INT_COL) FILTER(WHERE INT_COL < 4) FROM MyTable "
     "WHERE INT_COL > 2",
     ["SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 2 AND INT_COL > 3",
      "SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 2 AND INT_COL < 4"]),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 12345), SUM(INT_COL) FILTER(WHERE INT_COL < 59999), "
     "MIN(INT_COL) FILTER(WHERE INT_COL > 5000) FROM MyTable WHERE INT_COL > 1000",
     ["SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 1000 AND INT_COL > 12345",
      "SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL > 1000 AND INT_COL < 59999",
      "SELECT MIN(INT_COL) FROM MyTable WHERE INT_COL > 1000 AND INT_COL > 5000"]),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 12345), SUM(NO_INDEX_COL) FILTER(WHERE INT_COL < 59999), "
     "MIN(INT_COL) FILTER(WHERE INT_COL > 5000) FROM MyTable WHERE INT_COL < 28000 AND NO_INDEX_COL > 3000",
     ["SELECT SUM(INT_COL) FROM MyTable WHERE INT_COL < 28000 AND NO_INDEX_COL > 3000 AND INT_COL > 12345",
      "SELECT SUM(NO_INDEX_COL) FROM MyTable WHERE INT_COL < 28000 AND NO_INDEX_COL > 3000 AND INT_COL < 59999",
      "SELECT MIN(INT_COL) FROM MyTable WHERE INT_COL < 28000 AND NO_INDEX_COL > 3000 AND INT_COL > 5000"]),
    ("SELECT SUM(INT_COL) FILTER(WHERE INT_COL > 123 AND INT_COL < 25000), "
     "MAX(INT_COL) FILTER(WHERE INT_COL > 123 AND INT_COL < 25000), COUNT(*), SUM(NO_INDEX_COL) "
     "FROM MyTable WHERE NO_INDEX_COL > 5 AND NO_INDEX_COL < 29999",
     ["SELECT SUM(INT_COL) FROM MyTable WHERE NO_INDEX_COL > 5 AND NO_INDEX_COL < 29999 AND INT_COL > 123 "
      "AND INT_COL < 25000",
      "SELECT MAX(INT_COL) FROM MyTable WHERE NO_INDEX_COL > 5 AND NO_INDEX_COL < 29999 AND INT_COL > 123 "
      "AND INT_COL < 25000",
      "SELECT COUNT(*) FROM MyTable WHERE NO_INDEX_COL > 5 AND NO_INDEX_COL < 29999",
      "SELECT SUM(NO_INDEX_COL) FROM MyTable WHERE NO_INDEX_COL > 5 AND NO_INDEX_COL < 29999"]),
    ("SELECT COUNT(*) FILTER(WHERE INT_COL = 123456) FROM MyTable",  # empty filter pass
     ["SELECT COUNT(*) FROM MyTable WHERE INT_COL = 123456"]),
]


def _segments():
    segs = []
    for k, name in enumerate(("firstTestSegment", "secondTestSegment")):
        i = np.arange(N, dtype=np.int32)
        rng = np.random.default_rng(7 + k)
        cols = {"INT_COL": (PGPU_INT, i), "NO_INDEX_COL": (PGPU_INT, i.copy()),
                "STATIC_INT_COL": (PGPU_INT, np.full(N, 10, dtype=np.int32)),
                "BOOLEAN_COL": (PGPU_INT, rng.integers(0, 2, N).astype(np.int32))}
        # the reference's creator would mark INT_COL / NO_INDEX_COL sorted (values ascend); stored unsorted here so
        # the passes exercise the scan and inverted-index leaves (sorted leaves are covered by the KAT tests)
        segs.append(build_segment(name, cols, inverted=["INT_COL"], sorted_columns=()))
    return segs


def _vals(r):
    return list(r.aggregation_result)


def _same_values(a, b):
    assert len(a) == len(b) and all(close(x, y) for x, y in zip(a, b)), (a, b)


def _expected_docs_scanned(sql, segs):
    """numDocsScanned of FilteredAggregationOperator: Σ over every pass (each FILTER clause, then the main one)."""
    return sum(engine.execute(sq, segs).num_docs_scanned for sq, _ in split_filtered_aggregations(parse_sql(sql)))


# ---- parser / planner --------------------------------------------------------------------------------------------
def test_parse_filter_clause():
    q = parse_sql("SELECT SUM(a) FILTER(WHERE b > 3 AND c IN (1, 'x''y')), SUM(a), COUNT(*) FROM t WHERE d = 1")
    a0, a1, a2 = q.aggregations
    assert a0.filter_key == "b > 3 AND c IN ( 1 , 'x''y' )"
    assert a1.filter_key is None and a2.filter_key is None
    assert a0 != a1 and a0.result_name.startswith("sum(a) FILTER(WHERE")
    assert q.has_filtered_aggregations and set(q.columns) == {"a", "b", "c", "d"}
    parts = split_filtered_aggregations(q)
    assert [idx for _, idx in parts] == [[0], [1, 2]]
    assert parts[0][0].filter.type == "AND" and len(parts[0][0].filter.children) == 2
    assert parts[1][0].filter is q.filter


def test_filtered_group_by_rejected():
    with pytest.raises(SqlError):
        parse_sql("SELECT b, SUM(a) FILTER(WHERE c > 1) FROM t GROUP BY b")


def test_main_pass_always_runs():
    q = parse_sql("SELECT SUM(a) FILTER(WHERE b > 1) FROM t WHERE c < 5")
    parts = split_filtered_aggregations(q)
    assert len(parts) == 2 and parts[1][1] == [] and parts[1][0].aggregations[0].function == "COUNT"


# ---- oracle: the reference test's equivalences -------------------------------------------------------------------
@pytest.fixture(scope="module")
def segs():
    return _segments()


@pytest.mark.parametrize("pair", PAIRS, ids=[p[0][7:60] for p in PAIRS])
def test_filtered_equals_nonfiltered_oracle(segs, pair):
    f, nf = pair
    rf, rnf = engine.execute(parse_sql(f), segs), engine.execute(parse_sql(nf), segs)
    _same_values(_vals(rf), _vals(rnf))
    assert rf.num_total_docs == rnf.num_total_docs == 2 * N


@pytest.mark.parametrize("case", MIXED, ids=[c[0][7:60] for c in MIXED])
def test_mixed_filtered_oracle(segs, case):
    sql, singles = case
    got = _vals(engine.execute(parse_sql(sql), segs))
    want = [engine.execute(parse_sql(s), segs).aggregation_result[0] for s in singles]
    _same_values(got, want)


# ---- GPU ---------------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def gsegs(gpu_ctx, segs):
    from pinot_amd.segment import GpuSegment
    g = [GpuSegment(gpu_ctx, s) for s in segs]
    yield g
    for s in g:
        s.release()


@pytest.mark.gpu
@pytest.mark.parametrize("sql", [p[0] for p in PAIRS] + [c[0] for c in MIXED], ids=lambda s: s[7:60])
def test_filtered_aggregations_gpu_vs_oracle(gpu_ctx, segs, gsegs, sql):
    from pinot_amd.plan import GpuPlanMaker
    q = parse_sql(sql)
    res = GpuPlanMaker(gpu_ctx).execute(q, gsegs)
    ref = engine.execute(q, segs)
    _same_values(_vals(res), _vals(ref))
    assert res.stats.num_docs_scanned == ref.num_docs_scanned == _expected_docs_scanned(sql, segs)
    assert res.stats.num_total_docs == 2 * N


@pytest.mark.gpu
def test_filtered_submit_rejected(gpu_ctx, gsegs):
    from pinot_amd._lib import UnsupportedPlanError
    from pinot_amd.plan import GpuPlanMaker
    with pytest.raises(UnsupportedPlanError):
        GpuPlanMaker(gpu_ctx).submit(parse_sql(PAIRS[0][0]), gsegs)


@pytest.mark.gpu
def test_filtered_aggregations_distributed_executor_gpu(gpu_ctx, segs, gsegs):
    """DistributedExecutor (world size 1 here; the N-rank merge is covered by test_combine_gloo)."""
    from pinot_amd.combine import DistributedExecutor
    from pinot_amd.plan import GpuPlanMaker
    sql = MIXED[3][0]
    res = DistributedExecutor(GpuPlanMaker(gpu_ctx)).execute(parse_sql(sql), gsegs)
    ref = engine.execute(parse_sql(sql), segs)
    _same_values(_vals(res), _vals(ref))
    assert res.stats.num_docs_scanned == ref.num_docs_scanned
