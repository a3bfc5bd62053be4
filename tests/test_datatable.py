"""The server's DataTable (version 3) and the broker reduce (pinot_amd/datatable.py).

CPU: the byte layout restated independently here from DataTableImplV3.toBytes / DataTableBuilder / DataSchema.toBytes
(core/common/datatable/DataTableImplV3.java:180-290, DataTableBuilder.java:96-296, DataTableUtils.java:59-93,
pinot-common DataSchema.java:152-177) for small tables; java.util.HashMap iteration order (String.hashCode pinned
on its published values); round trips; and the broker reduce of several servers' DataTables against the oracle's
whole-query result.  GPU: GPU results per "server" -> DataTables -> broker reduce == the oracle's answer.  The
reference's own DataTable tests (DataTableSerDeTest) round-trip random tables and hold no golden bytes: parity of the
byte layout rests on the restatement below.
"""
import math
import struct

import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import build_segment
from pinot_amd._lib import PGPU_DOUBLE, PGPU_INT, PGPU_LONG
from pinot_amd.datatable import (DataSchema, DataTable, java_hashmap_order, java_string_hash, reduce_data_tables,
                                 server_data_table)
from pinot_amd.query import parse_sql
from tests.helpers import close


def test_java_string_hash_published_values():
    assert java_string_hash("") == 0
    assert java_string_hash("hello") == 99162322
    assert java_string_hash("Aa") == java_string_hash("BB") == 2112
    assert java_string_hash("polygenelubricants") == -2147483648  # the classic Integer.MIN_VALUE hashCode


def test_java_hashmap_order():
    # small Integer keys sit in bucket = value (capacity 16), whatever the insertion order
    assert java_hashmap_order([5, 3, 17, 1], lambda i: i) == [17, 1, 3, 5]  # 17 -> bucket 1, inserted before 1
    # a resize (13 keys > 12) doubles the table: 17 and 1 land in different buckets
    keys = list(range(13)) + [17]
    assert java_hashmap_order(keys, lambda i: i) == list(range(13)) + [17]


def _expected_bytes(rows, names, types, metadata_order, metadata):
    """DataTableImplV3.toBytes restated field by field for INT / LONG / DOUBLE / OBJECT(AvgPair) columns."""
    fixed, var = b"", b""
    for r in rows:
        for t, v in zip(types, r):
            if t == "INT":
                fixed += struct.pack(">i", v)
            elif t == "LONG":
                fixed += struct.pack(">q", v)
            elif t == "DOUBLE":
                fixed += struct.pack(">d", v)
            else:
                fixed += struct.pack(">ii", len(var), 16)
                var += struct.pack(">idq", 4, v[0], v[1])
    exc = struct.pack(">i", 0)
    dmap = struct.pack(">i", 0)
    schema = struct.pack(">i", len(names)) + b"".join(struct.pack(">i", len(s)) + s.encode() for s in names + types)
    hdr = struct.pack(">iii", 3, len(rows), len(names))
    off = 52
    for sec in (exc, dmap, schema, fixed, var):
        hdr += struct.pack(">ii", off, len(sec))
        off += len(sec)
    ordinals = {"numDocsScanned": (2, ">q"), "totalDocs": (10, ">q"), "numSegmentsProcessed": (6, ">i")}
    md = struct.pack(">i", len(metadata_order))
    for k in metadata_order:
        o, f = ordinals[k]
        md += struct.pack(">i", o) + struct.pack(f, int(metadata[k]))
    return hdr + exc + dmap + schema + fixed + var + struct.pack(">i", len(md)) + md


def test_byte_layout_group_table():
    names, types = ["k", "count(*)", "sum(m)", "avg(x)"], ["INT", "LONG", "DOUBLE", "OBJECT"]
    rows = [(3, 7, 2.5, (10.0, 4)), (-1, 1, -0.0, (1.5, 1))]
    md = {"numDocsScanned": "8", "totalDocs": "100", "numSegmentsProcessed": "2"}
    t = DataTable(DataSchema(names, types), rows, md)
    order = java_hashmap_order(list(md), java_string_hash)
    assert t.to_bytes() == _expected_bytes(rows, names, types, order, md)
    u = DataTable.from_bytes(t.to_bytes())
    assert u.rows == rows and u.metadata == md and u.schema == t.schema


def test_string_columns_and_exceptions_round_trip():
    t = DataTable(DataSchema(["s", "n", "f"], ["STRING", "LONG", "FLOAT"]),
                  [("a", 1, 0.5), ("b", 2, -1.25), ("a", 3, 2.0)],
                  {"numDocsScanned": "3", "numGroupsLimitReached": "true"}, {200: "boom", 150: "x"})
    b = t.to_bytes()
    u = DataTable.from_bytes(b)
    assert u.rows == t.rows and u.metadata == t.metadata and u.exceptions == t.exceptions
    # STRING cells are per-column dictionary ids in first-seen order: "a" -> 0, "b" -> 1
    fixed_start, fixed_len = struct.unpack_from(">ii", b, 12 + 8 * 3)
    ids = [struct.unpack_from(">i", b, fixed_start + r * 20)[0] for r in range(3)]
    assert ids == [0, 1, 0] and fixed_len == 3 * 20  # STRING 4 + LONG 8 + FLOAT 8 (DataTableUtils)


def test_empty_metadata_only_table():
    t = DataTable(None, [], {"numDocsScanned": "0", "totalDocs": "5"})
    u = DataTable.from_bytes(t.to_bytes())
    assert u.schema is None and u.rows == [] and u.metadata == t.metadata


class _Res:
    """A server's combined result as server_data_table reads it (QueryResult surface)."""

    def __init__(self, o):
        from pinot_amd.plan import ExecutionStats
        self.intermediate = o.intermediate
        self.stats = ExecutionStats(num_docs_scanned=o.num_docs_scanned,
                                    num_entries_scanned_in_filter=o.num_entries_scanned_in_filter,
                                    num_entries_scanned_post_filter=o.num_entries_scanned_post_filter,
                                    num_total_docs=o.num_total_docs, num_segments_processed=1,
                                    num_segments_matched=o.num_segments_matched)


def _segments(seed, sizes):
    rng = np.random.default_rng(seed)
    out = []
    for i, n in enumerate(sizes):
        cols = {"k": (PGPU_INT, rng.integers(0, 40, n) * 2), "d": (PGPU_LONG, rng.integers(0, 5, n)),
                "m": (PGPU_INT, rng.integers(-500, 500, n)), "x": (PGPU_DOUBLE, rng.normal(0, 1, n))}
        out.append(build_segment(f"s{i}", cols, sorted_columns=()))
    return out


QUERIES = [
    "SELECT k, COUNT(*), SUM(m), AVG(x), MIN(m), MAX(x) FROM t WHERE d <> 2 GROUP BY k ORDER BY SUM(m) DESC LIMIT 7",
    "SELECT d, k, COUNT(*), AVG(m) FROM t GROUP BY d, k ORDER BY d, k LIMIT 50",
    "SELECT COUNT(*), SUM(x), AVG(m), MIN(x), MAX(m) FROM t WHERE k < 30",
]


def _rows_match(a, b):
    assert len(a) == len(b)
    for r, s in zip(a, b):
        assert len(r) == len(s) and all(close(x, y) for x, y in zip(r, s)), (r, s)


@pytest.mark.parametrize("sql", QUERIES)
def test_broker_reduce_of_server_tables_equals_oracle(sql):
    """Three servers' results through their DataTable bytes and the broker reduce == the whole query on the oracle."""
    q = parse_sql(sql)
    segs = _segments(5, [3000, 2000, 4000, 1500, 2500, 800])
    servers = [segs[0:2], segs[2:4], segs[4:6]]
    tables = []
    for ss in servers:
        o = engine.execute(q, ss)
        types = [PGPU_INT if g == "k" else PGPU_LONG for g in q.group_by]
        tables.append(DataTable.from_bytes(server_data_table(q, _Res(o), types).to_bytes()))
    got = reduce_data_tables(q, tables)
    ref = engine.execute(q, segs)
    _rows_match(got.rows, ref.rows)
    assert got.num_docs_scanned == ref.num_docs_scanned and got.total_docs == ref.num_total_docs
    assert got.num_segments_matched == ref.num_segments_matched


def test_num_segments_matched_counts_segments_with_docs():
    """CombineOperatorUtils.setExecutionStatistics (:64-67): numSegmentsMatched counts the segments whose operator
    scanned a doc -- one server whose first segment matches and whose second does not reports 1."""
    segs = _segments(5, [3000, 2000])
    q = parse_sql("SELECT COUNT(*) FROM t WHERE k < 30 AND m > 499")  # m < 500: nothing, unless the seed says so
    o = engine.execute(q, segs)
    q2 = parse_sql("SELECT COUNT(*) FROM t WHERE k < 30")
    o2 = engine.execute(q2, segs[:1])
    assert o.num_segments_matched == sum(o.segment_matched) == 0
    assert o2.num_segments_matched == 1
    mixed = engine.execute(parse_sql("SELECT COUNT(*) FROM t WHERE m > 490"), segs)
    assert mixed.num_segments_matched == sum(mixed.segment_matched)
    dt = DataTable.from_bytes(server_data_table(q2, _Res(o2)).to_bytes())
    assert dt.metadata["numSegmentsMatched"] == "1"
    assert reduce_data_tables(q2, [dt, DataTable.from_bytes(server_data_table(q, _Res(o)).to_bytes())]
                              ).num_segments_matched == 1


# ---- GPU -----------------------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("sql", QUERIES)
def test_gpu_servers_through_datatables(gpu_ctx, sql):
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    q = parse_sql(sql)
    segs = _segments(9, [30000, 20000, 45000, 5000])
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        tables = []
        for part in (gs[:2], gs[2:]):
            r = GpuPlanMaker(gpu_ctx).execute(q, part)
            types = [p.column(g).data_type for g in q.group_by for p in part[:1]]
            tables.append(DataTable.from_bytes(server_data_table(q, r, types).to_bytes()))
        got = reduce_data_tables(q, tables)
    finally:
        for g in gs:
            g.release()
    ref = engine.execute(q, segs)
    _rows_match(got.rows, ref.rows)
    assert got.num_docs_scanned == ref.num_docs_scanned
    assert got.num_segments_matched == ref.num_segments_matched
    assert not any(isinstance(v, float) and math.isnan(v) for r in got.rows for v in r)
