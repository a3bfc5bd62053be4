"""Raw (no-dictionary) metric columns and range indexes.

CPU tests pin the oracle's raw-column restatement: the FixedByteChunkSVForwardIndexWriter format with every codec
(oracle/rawfwd.py), and query results over raw columns equal to the same data dictionary-encoded.  GPU tests
(`-m gpu`) run raw-column aggregations and raw / range-index filter leaves through the C ABI against the oracle,
all four execution statistics included.  Reference: BaseChunkSVForwardIndexReader.java:56-157,
FilterOperatorUtils.java:42-81, RangeIndexBasedFilterOperator.java:52-290, RangePredicateEvaluatorFactory.java:62-110.
"""
import numpy as np
import pytest

from oracle import engine, rawfwd
from oracle.segment_writer import build_segment
from pinot_amd._lib import PGPU_DOUBLE, PGPU_FLOAT, PGPU_INT, PGPU_LONG
from pinot_amd.query import parse_sql
from tests.helpers import check_groups, close, rows_close

CODECS = [(rawfwd.PASS_THROUGH, 2), (rawfwd.SNAPPY, 2), (rawfwd.LZ4, 3), (rawfwd.LZ4_LENGTH_PREFIXED, 4),
          (rawfwd.ZSTANDARD, 3)]


def _data(rng, n):
    return {
        "d": (PGPU_INT, rng.integers(0, 50, n)),
        "k": (PGPU_INT, rng.integers(0, 20, n) * 3),
        "ri": (PGPU_INT, rng.integers(-300, 300, n)),
        "rl": (PGPU_LONG, rng.integers(-10**12, 10**12, n)),
        "rf": (PGPU_FLOAT, np.round(rng.random(n), 3).astype(np.float32)),
        "rd": (PGPU_DOUBLE, rng.normal(0, 1, n)),
    }


RAW = ("ri", "rl", "rf", "rd")
QUERIES = [
    "SELECT COUNT(*), SUM(ri), MIN(rl), MAX(rf), AVG(rd) FROM t WHERE ri BETWEEN -100 AND 200",
    "SELECT SUM(rl), COUNT(*), MAX(rd) FROM t WHERE d IN (1, 2, 3, 17) AND rl > 5000",
    "SELECT k, SUM(rd), MAX(ri), MIN(rf), COUNT(*) FROM t WHERE rf < 0.5 OR d = 7 GROUP BY k",
    "SELECT COUNT(*), SUM(ri) FROM t WHERE ri <> 3 AND NOT rd BETWEEN 0.1 AND 0.9",
    "SELECT COUNT(*), SUM(rf), MIN(rd) FROM t WHERE ri IN (1, 5, 9, -3, 250) OR rf = 0.25",
    "SELECT k, COUNT(*), SUM(rl) FROM t WHERE ri > 10 AND ri < 100 AND d NOT IN (4, 5) GROUP BY k",
    "SELECT SUM(rd), MIN(ri), MAX(rl) FROM t",
    "SELECT MIN(ri), MAX(rd), COUNT(*) FROM t",
    "SELECT COUNT(*), MAX(rd) FROM t WHERE rf >= 0.1 AND rf <= 0.2 AND d BETWEEN 5 AND 30",
]


def _segments(seed, n_list, raw=RAW, codec=(0, 2), range_index=(), range_version=2):
    rng = np.random.default_rng(seed)
    segs, dense = [], []
    for i, n in enumerate(n_list):
        cols = _data(rng, n)
        segs.append(build_segment(f"s{i}", cols, raw=raw, raw_codec=codec[0], raw_version=codec[1],
                                  range_index=range_index, range_index_version=range_version, sorted_columns=()))
        dense.append(build_segment(f"s{i}", cols, sorted_columns=()))
    return segs, dense


# ---- CPU: format and oracle ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("dt,dtype", [(PGPU_INT, np.int32), (PGPU_LONG, np.int64), (PGPU_FLOAT, np.float32),
                                      (PGPU_DOUBLE, np.float64)])
@pytest.mark.parametrize("codec,version", CODECS)
def test_raw_forward_round_trip(dt, dtype, codec, version):
    rng = np.random.default_rng(dt * 7 + codec)
    for n in (0, 1, 999, 1000, 1001, 4097):
        v = rng.integers(-1000, 1000, n).astype(dtype)
        b = rawfwd.write_raw_forward(v, dt, codec, version)
        assert np.array_equal(rawfwd.read_raw_forward(b, dt, n), v)
        hdr = np.frombuffer(b[:28], dtype=">i4")
        assert hdr[0] == version and hdr[5] == codec and hdr[6] == 28
        assert hdr[2] == (1024 if version == 4 else 1000)  # normalizeDocsPerChunk: a power of two from version 4


@pytest.mark.parametrize("data", [b"", b"a", bytes(range(256)) * 40, bytes(5000), b"abcabcabcabcabcab" * 300])
def test_block_codecs_round_trip(data):
    assert rawfwd.snappy_decompress(rawfwd.snappy_compress(data)) == data
    assert rawfwd.lz4_decompress(rawfwd.lz4_compress(data)) == data


@pytest.mark.parametrize("sql", QUERIES)
def test_oracle_raw_equals_dictionary_encoded(sql):
    """A raw column holds the same values as its dictionary-encoded twin: results and docs scanned agree (the range
    index is absent here, so raw leaves are scans like the dictionary ones)."""
    segs, dense = _segments(3, [3000, 4500])
    q = parse_sql(sql)
    a, b = engine.execute(q, segs), engine.execute(q, dense)
    assert a.num_docs_scanned == b.num_docs_scanned and a.num_total_docs == b.num_total_docs
    if q.group_by:
        assert rows_close(sorted(a.group_rows), sorted(b.group_rows))
    else:
        assert all(close(x, y) for x, y in zip(a.aggregation_result, b.aggregation_result))


def test_oracle_range_index_semantics():
    """RangeIndexBasedFilterOperator on a raw column uses the evaluator's bounds inclusively and scans nothing; on a
    dictionary column it is the exact dict-id range (0 entries as well)."""
    segs, _ = _segments(5, [5000], range_index=("ri", "d"))
    plain, _ = _segments(5, [5000])
    ri = engine.execute(parse_sql("SELECT COUNT(*) FROM t WHERE ri > 10 AND ri < 100"), segs, iterator_stats=True)
    sc = engine.execute(parse_sql("SELECT COUNT(*) FROM t WHERE ri >= 10 AND ri <= 100"), plain, iterator_stats=True)
    assert ri.aggregation_result == sc.aggregation_result
    assert ri.num_entries_scanned_in_filter == 0 and sc.num_entries_scanned_in_filter > 0
    d1 = engine.execute(parse_sql("SELECT COUNT(*) FROM t WHERE d BETWEEN 5 AND 20"), segs, iterator_stats=True)
    d2 = engine.execute(parse_sql("SELECT COUNT(*) FROM t WHERE d BETWEEN 5 AND 20"), plain, iterator_stats=True)
    assert d1.aggregation_result == d2.aggregation_result and d1.num_entries_scanned_in_filter == 0


def test_oracle_raw_literal_parsing():
    segs, _ = _segments(6, [100])
    with pytest.raises(ValueError):
        engine.execute(parse_sql("SELECT COUNT(*) FROM t WHERE ri > 1.5"), segs)
    r = engine.execute(parse_sql("SELECT COUNT(*) FROM t WHERE rd > 1"), segs)  # parseDouble("1")
    assert r.aggregation_result[0] >= 0


# ---- GPU ----------------------------------------------------------------------------------------------------------
def _gpu_vs_oracle(gpu_ctx, segs, sql, exact=True, **opts):
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    q = parse_sql(sql)
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        res = GpuPlanMaker(gpu_ctx, exact_filter_stats=exact, **opts).execute(q, gs)
    finally:
        for g in gs:
            g.release()
    ref = engine.execute(q, segs, iterator_stats=True)
    if q.group_by:
        check_groups(res, ref)
    else:
        for a, b in zip(res.aggregation_result, ref.aggregation_result):
            assert close(a, b), (res.aggregation_result, ref.aggregation_result)
    assert res.stats.num_docs_scanned == ref.num_docs_scanned
    assert res.stats.num_entries_scanned_post_filter == ref.num_entries_scanned_post_filter
    assert res.stats.num_total_docs == ref.num_total_docs
    if exact:
        assert res.stats.filter_stats_exact
        assert res.stats.num_entries_scanned_in_filter == ref.num_entries_scanned_in_filter
    return res, ref


@pytest.mark.gpu
@pytest.mark.parametrize("codec", CODECS, ids=[f"{rawfwd.maybe_codec_name(c)}-v{v}" for c, v in CODECS])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_gpu_raw_columns_vs_oracle(gpu_ctx, codec, qi):
    segs, _ = _segments(11 + qi, [5000, 70000, 2049], codec=codec)
    _gpu_vs_oracle(gpu_ctx, segs, QUERIES[qi])


@pytest.mark.gpu
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_gpu_range_index_vs_oracle(gpu_ctx, qi):
    segs, _ = _segments(31 + qi, [40000, 3000], range_index=("ri", "rf", "rd", "d"))
    _gpu_vs_oracle(gpu_ctx, segs, QUERIES[qi])


@pytest.mark.gpu
@pytest.mark.parametrize("qi", [0, 2, 5])
def test_gpu_raw_own_filter_count(gpu_ctx, qi):
    """Without the exact-statistics pass the GPU's own count is reported; results still match."""
    segs, _ = _segments(41 + qi, [30000], range_index=("ri",))
    _gpu_vs_oracle(gpu_ctx, segs, QUERIES[qi], exact=False)


@pytest.mark.gpu
def test_gpu_legacy_range_index_not_exact(gpu_ctx):
    """A version-1 (legacy) range index scans its partial matches in the reference: the GPU answers the same docs and
    flags its filter count as not the reference's."""
    segs, _ = _segments(51, [20000], range_index=("ri",), range_version=1)
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    q = parse_sql("SELECT COUNT(*), SUM(rl) FROM t WHERE ri BETWEEN 0 AND 50")
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        res = GpuPlanMaker(gpu_ctx).execute(q, gs)
    finally:
        for g in gs:
            g.release()
    ref = engine.execute(q, segs)
    assert res.aggregation_result[0] == ref.aggregation_result[0] and close(res.aggregation_result[1],
                                                                            ref.aggregation_result[1])
    assert not res.stats.filter_stats_exact


@pytest.mark.gpu
@pytest.mark.parametrize("flags", ["partition", "hash", "default"])
def test_gpu_raw_aggregation_group_modes(gpu_ctx, flags):
    """Raw aggregation columns under every group-by table strategy (LDS / HBM / partitioned / hash)."""
    from pinot_amd import _lib
    qf = {"partition": _lib.PGPU_Q_PARTITION, "hash": _lib.PGPU_Q_HASH, "default": 0}[flags]
    segs, _ = _segments(61, [60000, 9000])
    _gpu_vs_oracle(gpu_ctx, segs, "SELECT k, SUM(ri), MIN(rf), MAX(rf), COUNT(*) FROM t WHERE d < 40 GROUP BY k",
                   query_flags=qf)
    _gpu_vs_oracle(gpu_ctx, segs, "SELECT d, k, SUM(ri), COUNT(*) FROM t GROUP BY d, k", query_flags=qf)


GROUP_RAW = [
    "SELECT ri, COUNT(*), SUM(rd) FROM t GROUP BY ri",
    "SELECT rf, COUNT(*), MAX(ri), SUM(ri) FROM t WHERE d < 25 GROUP BY rf",
    "SELECT rl, SUM(rl), MIN(rd) FROM t WHERE ri BETWEEN -50 AND 50 GROUP BY rl",
    "SELECT k, ri, COUNT(*), SUM(rf) FROM t WHERE rd > 0 GROUP BY k, ri",
    "SELECT ri, d, COUNT(*) FROM t GROUP BY ri, d ORDER BY COUNT(*) DESC, ri, d LIMIT 20",
]


@pytest.mark.parametrize("sql", GROUP_RAW)
def test_oracle_group_by_raw_equals_dictionary_encoded(sql):
    """NoDictionary*GroupKeyGenerator keys by value: the same groups as the dictionary-encoded twin below the
    numGroupsLimit (at it, the no-dictionary generators cap every key space -- test_oracle_group_by_raw_limit)."""
    segs, dense = _segments(73, [3000, 2500])
    q = parse_sql(sql)
    a, b = engine.execute(q, segs), engine.execute(q, dense)
    c = engine.execute(q, segs[:1] + dense[1:])  # the column raw in one segment, dictionary-encoded in the other
    assert a.num_docs_scanned == b.num_docs_scanned == c.num_docs_scanned
    assert rows_close(sorted(a.group_rows), sorted(b.group_rows))
    assert rows_close(sorted(c.group_rows), sorted(b.group_rows))


def test_oracle_group_by_raw_float_keys():
    """FLOAT / DOUBLE group keys are Float.floatToIntBits / Double.doubleToLongBits: -0.0 and 0.0 are two groups,
    every NaN one (fastutil Float2IntOpenHashMap / Double2IntOpenHashMap)."""
    n = 12
    vals = np.array([0.0, -0.0, 1.5, np.nan, -0.0, np.float32(np.nan), 1.5, 0.0, -2.0, np.nan, 3.0, 0.0],
                    dtype=np.float32)
    vals[5] = np.frombuffer(np.uint32(0x7FC00001).tobytes(), dtype=np.float32)[0]  # a second NaN pattern
    cols = {"d": (PGPU_INT, np.arange(n) % 3), "rf": (PGPU_FLOAT, vals)}
    seg = build_segment("f", cols, raw=("rf",), sorted_columns=())
    r = engine.execute_segment(parse_sql("SELECT rf, COUNT(*) FROM t GROUP BY rf"), seg)
    got = {}
    for k, v in r.groups.items():
        got[np.float32(k[0]).tobytes() if not np.isnan(k[0]) else b"nan"] = v[0]
    assert got[np.float32(0.0).tobytes()] == 3 and got[np.float32(-0.0).tobytes()] == 2
    assert got[b"nan"] == 3 and got[np.float32(1.5).tobytes()] == 2 and len(got) == 6


def test_oracle_group_by_raw_limit():
    """A raw group column caps the segment's groups at numGroupsLimit, first seen in doc order, whatever the key
    space (NoDictionarySingleColumnGroupKeyGenerator.java:199-235) -- a dictionary column of the same cardinality
    below maxInitialResultHolderCapacity would not."""
    n = 500
    cols = {"ri": (PGPU_INT, (np.arange(n) * 7919) % 97), "d": (PGPU_INT, np.arange(n) % 5)}
    raw = build_segment("r", cols, raw=("ri",), sorted_columns=())
    dense = build_segment("r", cols, sorted_columns=())
    q = parse_sql("SELECT ri, COUNT(*) FROM t GROUP BY ri")
    a = engine.execute_segment(q, raw, num_groups_limit=10, max_init_group_holder_capacity=10_000)
    b = engine.execute_segment(q, dense, num_groups_limit=10, max_init_group_holder_capacity=10_000)
    first = list(dict.fromkeys(((np.arange(n) * 7919) % 97).tolist()))[:10]
    assert sorted(k[0] for k in a.groups) == sorted(first)
    assert len(b.groups) == 97


@pytest.mark.gpu
@pytest.mark.parametrize("qi", range(len(GROUP_RAW)))
@pytest.mark.parametrize("flags", ["default", "hash", "partition"])
def test_gpu_group_by_raw_vs_oracle(gpu_ctx, qi, flags):
    """GROUP BY on raw columns through their on-the-fly group dictionaries (pgpu_segment_add_group_dictionary), one
    segment holding the column dictionary-encoded beside raw ones."""
    from pinot_amd import _lib
    qf = {"partition": _lib.PGPU_Q_PARTITION, "hash": _lib.PGPU_Q_HASH, "default": 0}[flags]
    segs, dense = _segments(75 + qi, [5000, 70000, 2049])
    _gpu_vs_oracle(gpu_ctx, segs[:2] + dense[2:], GROUP_RAW[qi], query_flags=qf)


@pytest.mark.gpu
def test_gpu_group_by_raw_float_keys_and_limit(gpu_ctx):
    """-0.0 / 0.0 apart and NaNs as one group on the GPU too; a segment meeting more raw keys than numGroupsLimit keeps
    its first-seen keys, as the reference truncates it."""
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    rng = np.random.default_rng(77)
    n = 9000
    vals = rng.choice(np.array([0.0, -0.0, 1.5, np.nan, -2.25, 7.0], dtype=np.float64), n)
    cols = {"d": (PGPU_INT, rng.integers(0, 9, n)), "rd": (PGPU_DOUBLE, vals), "ri": (PGPU_INT, rng.integers(0, 500, n))}
    seg = build_segment("f", cols, raw=("rd", "ri"), sorted_columns=())
    gs = [GpuSegment(gpu_ctx, seg)]
    try:
        q = parse_sql("SELECT rd, COUNT(*), SUM(d) FROM t GROUP BY rd")
        res = GpuPlanMaker(gpu_ctx).execute(q, gs)
        ref = engine.execute_segment(q, seg)
        got = {np.float64(r[0]).tobytes() if not np.isnan(r[0]) else b"nan": tuple(r[1:]) for r in res.group_rows}
        exp = {np.float64(k[0]).tobytes() if not np.isnan(k[0]) else b"nan": (v[0], v[1]) for k, v in ref.groups.items()}
        assert len(got) == 6 and got == exp
        # ~500 raw keys past a limit of 100: the first-seen 100 (NoDictionarySingleColumnGroupKeyGenerator caps its
        # map at numGroupsLimit), through GpuPlanMaker.first_seen_groups
        q = parse_sql("SELECT ri, COUNT(*) FROM t GROUP BY ri")
        res = GpuPlanMaker(gpu_ctx, num_groups_limit=100).execute(q, gs)
        ref = engine.execute(q, [seg], num_groups_limit=100)
        assert len(res.group_rows) == len(ref.group_rows) == 100
        assert sorted(res.group_rows) == sorted(ref.group_rows)
    finally:
        for g in gs:
            g.release()


@pytest.mark.gpu
def test_gpu_raw_long_sum_overflow_bound(gpu_ctx):
    """LONG raw values near 2^62: the integer SUM bound switches to the exact three-part sections."""
    n = 20000
    rng = np.random.default_rng(81)
    cols = {"d": (PGPU_INT, rng.integers(0, 4, n)),
            "rl": (PGPU_LONG, rng.integers(1 << 61, (1 << 62), n))}
    seg = build_segment("big", cols, raw=("rl",), sorted_columns=())
    res, ref = _gpu_vs_oracle(gpu_ctx, [seg], "SELECT SUM(rl), COUNT(*) FROM t WHERE d <> 2")
    assert abs(res.aggregation_result[0]) > 2.0 ** 63


@pytest.mark.parametrize("version", ["v1", "v3"])
def test_loader_raw_and_range_index_round_trip(tmp_path, version):
    """On-disk segments with raw columns and range indexes: `<col>.sv.raw.fwd` / forward_index entries, the
    `.bitmap.range` / range_index entries and the metadata min / max come back byte for byte."""
    from oracle.segment_writer import write_segment_dir
    from pinot_amd.loader import load_segment
    segs, _ = _segments(91, [3000], codec=(rawfwd.LZ4, 3), range_index=("ri", "d"))
    root = write_segment_dir(segs[0], str(tmp_path / "seg"), version=version)
    got = load_segment(root)
    for name, c in segs[0].columns.items():
        g = got.column(name)
        assert g.is_raw == c.is_raw
        assert g.raw_forward == c.raw_forward and g.range_index == c.range_index
        if c.is_raw:
            assert (g.min_value, g.max_value) == (float(c.min_value), float(c.max_value))
    q = parse_sql(QUERIES[2])
    a, b = engine.execute(q, [got], iterator_stats=True), engine.execute(q, segs, iterator_stats=True)
    assert sorted(a.group_rows) == sorted(b.group_rows)
    assert a.num_entries_scanned_in_filter == b.num_entries_scanned_in_filter
