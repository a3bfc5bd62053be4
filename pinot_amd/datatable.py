"""The server's result block as a DataTable (version 3) and the broker's reduce of DataTables.

Server side: ``IntermediateResultsBlock.getDataTable`` (core/operator/blocks/IntermediateResultsBlock.java:290-432)
turns the combined result into a DataTable -- for GROUP BY one row per group of the trimmed IndexedTable (group
values, then every aggregation's intermediate result; the schema of AggregationGroupByOrderByOperator.java:70-93),
for aggregation-only one row of intermediate results (:382-414) -- and attaches the execution statistics as
metadata (:416-432).  ``DataTableImplV3.toBytes`` (core/common/datatable/DataTableImplV3.java:180-290) lays it out:

    int version (3), numRows, numColumns, then (start, length) of: exceptions, dictionary map, data schema,
    fixed-size data, variable-size data; the five sections; int metadata length; the metadata.

Rows are fixed-size (DataTableUtils.computeColumnOffsets: INT 4, LONG 8, FLOAT 8 (sic), DOUBLE 8, STRING 4 = a
per-column dictionary id, everything else 8 = (offset, length) into the variable-size section); an OBJECT cell's
variable bytes are int ObjectType value + ObjectSerDeUtils bytes (AvgPair: double sum, long count).  Metadata keys
are written by MetadataKey ordinal with INT / LONG values in binary and STRING values as UTF-8 (DataTable.java:94-114).
Java HashMaps are written in their iteration order, which is restated here (String.hashCode, bucket order), so the
bytes match the reference's byte for byte.

Broker side: ``GroupByDataTableReducer`` / ``AggregationDataTableReducer`` (core/query/reduce/GroupByDataTableReducer
.java:85-223) merge the servers' intermediate results per group (AggregationFunction.merge), extract the final
results, apply ORDER BY and LIMIT, and sum the servers' statistics.
"""
from __future__ import annotations

import math
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from .query import QueryContext

VERSION_3 = 3
HEADER_SIZE = 4 * 13

# DataSchema.ColumnDataType (pinot-common/.../DataSchema.java:241-260): written by name
INT, LONG, FLOAT, DOUBLE, STRING, OBJECT = "INT", "LONG", "FLOAT", "DOUBLE", "STRING", "OBJECT"
_FIXED = {INT: 4, LONG: 8, FLOAT: 8, DOUBLE: 8, STRING: 4}

# DataTable.MetadataKey (pinot-common/.../DataTable.java:94-114): (name, value type) in ordinal order
METADATA_KEYS = [("unknown", "S"), ("table", "S"), ("numDocsScanned", "L"), ("numEntriesScannedInFilter", "L"),
                 ("numEntriesScannedPostFilter", "L"), ("numSegmentsQueried", "I"), ("numSegmentsProcessed", "I"),
                 ("numSegmentsMatched", "I"), ("numConsumingSegmentsProcessed", "I"),
                 ("minConsumingFreshnessTimeMs", "L"), ("totalDocs", "L"), ("numGroupsLimitReached", "S"),
                 ("timeUsedMs", "L"), ("traceInfo", "S"), ("requestId", "L"), ("numResizes", "I"),
                 ("resizeTimeMs", "L"), ("threadCpuTimeNs", "L"), ("systemActivitiesCpuTimeNs", "L"),
                 ("responseSerializationCpuTimeNs", "L")]
_KEY_ORDINAL = {name: i for i, (name, _) in enumerate(METADATA_KEYS)}

OBJECT_TYPE_AVG_PAIR = 4  # ObjectSerDeUtils.ObjectType.AvgPair


# ---- Java HashMap iteration order -----------------------------------------------------------------------------------
def java_string_hash(s: str) -> int:
    """String.hashCode over UTF-16 code units, as a signed 32-bit int."""
    h = 0
    for u in struct.unpack(f">{len(s.encode('utf-16-be')) // 2}H", s.encode("utf-16-be")):
        h = (31 * h + u) & 0xFFFFFFFF
    return h - (1 << 32) if h & 0x80000000 else h


def java_hashmap_order(keys: Sequence, hash_of) -> list:
    """Iteration order of a java.util.HashMap holding `keys` inserted in the given order (default capacity 16,
    load factor 0.75, resized by doubling): bucket (h ^ h >>> 16) & (n - 1) ascending, insertion order inside a
    bucket (a resize splits every bucket's list preserving order).  Tree bins (8+ collisions in one bucket) are not
    modelled."""
    n = 16
    while len(keys) > n * 0.75:
        n *= 2
    buckets: Dict[int, list] = {}
    for k in keys:
        h = hash_of(k) & 0xFFFFFFFF
        buckets.setdefault((h ^ (h >> 16)) & (n - 1), []).append(k)
    return [k for b in sorted(buckets) for k in buckets[b]]


def _int_hash(i: int) -> int:
    return i


# ---- DataSchema / DataTable ----------------------------------------------------------------------------------------
@dataclass
class DataSchema:
    column_names: List[str]
    column_types: List[str]

    def to_bytes(self) -> bytes:
        """DataSchema.toBytes (pinot-common/.../DataSchema.java:152-177)."""
        out = [struct.pack(">i", len(self.column_names))]
        for s in list(self.column_names) + list(self.column_types):
            b = s.encode("utf-8")
            out.append(struct.pack(">i", len(b)) + b)
        return b"".join(out)

    @staticmethod
    def from_bytes(b: bytes, pos: int = 0) -> Tuple["DataSchema", int]:
        (n,), pos = struct.unpack_from(">i", b, pos), pos + 4
        strs = []
        for _ in range(2 * n):
            (ln,) = struct.unpack_from(">i", b, pos)
            strs.append(b[pos + 4: pos + 4 + ln].decode("utf-8"))
            pos += 4 + ln
        return DataSchema(strs[:n], strs[n:]), pos


@dataclass
class DataTable:
    """A DataTable's content: schema, rows of Python values (OBJECT AvgPair cells as (sum, count)), metadata
    (MetadataKey name -> string value, inserted in the order the server puts them) and exceptions."""

    schema: Optional[DataSchema]
    rows: List[tuple] = field(default_factory=list)
    metadata: Dict[str, str] = field(default_factory=dict)
    exceptions: Dict[int, str] = field(default_factory=dict)

    def to_bytes(self) -> bytes:
        """DataTableBuilder + DataTableImplV3.toBytes."""
        fixed, var = bytearray(), bytearray()
        dictionaries: Dict[str, Dict[str, int]] = {}
        dict_order: List[str] = []
        if self.schema is not None:
            names, types = self.schema.column_names, self.schema.column_types
            for row in self.rows:
                for name, t, v in zip(names, types, row):
                    if t == INT:
                        fixed += struct.pack(">i", int(v))
                    elif t == LONG:
                        fixed += struct.pack(">q", int(v))
                    elif t == FLOAT:  # setColumn(float) writes 4 bytes into the column's 8
                        fixed += struct.pack(">f", float(v)) + bytes(4)
                    elif t == DOUBLE:
                        fixed += struct.pack(">d", float(v))
                    elif t == STRING:
                        d = dictionaries.get(name)
                        if d is None:
                            d = dictionaries[name] = {}
                            dict_order.append(name)
                        fixed += struct.pack(">i", d.setdefault(v, len(d)))
                    elif t == OBJECT:  # AvgPair: (offset, length) | type, double sum, long count
                        payload = struct.pack(">dq", float(v[0]), int(v[1]))
                        fixed += struct.pack(">ii", len(var), len(payload))
                        var += struct.pack(">i", OBJECT_TYPE_AVG_PAIR) + payload
                    else:
                        raise ValueError(f"column type {t} is not produced on this path")
        exc = bytearray(struct.pack(">i", len(self.exceptions)))
        for code in java_hashmap_order(list(self.exceptions), _int_hash):
            m = self.exceptions[code].encode("utf-8")
            exc += struct.pack(">ii", code, len(m)) + m
        dmap = None
        if self.schema is not None:  # DataTableBuilder always hands its (maybe empty) reverse dictionary map over
            dmap = bytearray(struct.pack(">i", len(dictionaries)))
            for col in java_hashmap_order(dict_order, java_string_hash):
                cb = col.encode("utf-8")
                rev = {i: s for s, i in dictionaries[col].items()}
                dmap += struct.pack(">i", len(cb)) + cb + struct.pack(">i", len(rev))
                for i in java_hashmap_order(list(rev), _int_hash):
                    vb = str(rev[i]).encode("utf-8")
                    dmap += struct.pack(">ii", i, len(vb)) + vb
        schema = self.schema.to_bytes() if self.schema is not None else None
        sections = [bytes(exc), bytes(dmap) if dmap is not None else None, schema,
                    bytes(fixed) if self.schema is not None else None, bytes(var) if self.schema is not None else None]
        ncols = len(self.schema.column_names) if self.schema is not None else 0
        head = [struct.pack(">iii", VERSION_3, len(self.rows) if self.schema is not None else 0, ncols)]
        off = HEADER_SIZE
        for s in sections:
            head.append(struct.pack(">ii", off, len(s) if s is not None else 0))
            if s is not None:
                off += len(s)
        md = bytearray(struct.pack(">i", len(self.metadata)))
        for k in java_hashmap_order(list(self.metadata), java_string_hash):
            ordinal = _KEY_ORDINAL.get(k)
            if ordinal is None:
                continue
            v, kind = self.metadata[k], METADATA_KEYS[ordinal][1]
            md += struct.pack(">i", ordinal)
            if kind == "I":
                md += struct.pack(">i", int(v))
            elif kind == "L":
                md += struct.pack(">q", int(v))
            else:
                vb = v.encode("utf-8")
                md += struct.pack(">i", len(vb)) + vb
        return b"".join(head) + b"".join(s for s in sections if s is not None) + struct.pack(">i", len(md)) + bytes(md)

    @staticmethod
    def from_bytes(b: bytes) -> "DataTable":
        """DataTableImplV3(ByteBuffer) (DataTableImplV3.java:60-140); the version int first
        (DataTableFactory.getDataTable)."""
        version, nrows, ncols = struct.unpack_from(">iii", b, 0)
        if version != VERSION_3:
            raise ValueError(f"DataTable version {version}")
        secs = [struct.unpack_from(">ii", b, 12 + 8 * i) for i in range(5)]
        exceptions: Dict[int, str] = {}
        if secs[0][1]:
            pos = secs[0][0]
            (n,), pos = struct.unpack_from(">i", b, pos), pos + 4
            for _ in range(n):
                code, ln = struct.unpack_from(">ii", b, pos)
                exceptions[code] = b[pos + 8: pos + 8 + ln].decode("utf-8")
                pos += 8 + ln
        dicts: Dict[str, Dict[int, str]] = {}
        if secs[1][1]:
            pos = secs[1][0]
            (n,), pos = struct.unpack_from(">i", b, pos), pos + 4
            for _ in range(n):
                (ln,) = struct.unpack_from(">i", b, pos)
                col = b[pos + 4: pos + 4 + ln].decode("utf-8")
                pos += 4 + ln
                (m,), pos = struct.unpack_from(">i", b, pos), pos + 4
                d = dicts[col] = {}
                for _ in range(m):
                    i, ln = struct.unpack_from(">ii", b, pos)
                    d[i] = b[pos + 8: pos + 8 + ln].decode("utf-8")
                    pos += 8 + ln
        schema = DataSchema.from_bytes(b, secs[2][0])[0] if secs[2][1] else None
        rows: List[tuple] = []
        if schema is not None and secs[3][1]:
            widths = [_FIXED.get(t, 8) for t in schema.column_types]
            rsize = sum(widths)
            fixed = b[secs[3][0]: secs[3][0] + secs[3][1]]
            var = b[secs[4][0]: secs[4][0] + secs[4][1]]
            for r in range(nrows):
                pos = r * rsize
                row = []
                for name, t, w in zip(schema.column_names, schema.column_types, widths):
                    if t == INT:
                        row.append(struct.unpack_from(">i", fixed, pos)[0])
                    elif t == LONG:
                        row.append(struct.unpack_from(">q", fixed, pos)[0])
                    elif t == FLOAT:
                        row.append(struct.unpack_from(">f", fixed, pos)[0])
                    elif t == DOUBLE:
                        row.append(struct.unpack_from(">d", fixed, pos)[0])
                    elif t == STRING:
                        row.append(dicts[name][struct.unpack_from(">i", fixed, pos)[0]])
                    elif t == OBJECT:
                        off, ln = struct.unpack_from(">ii", fixed, pos)
                        (otype,) = struct.unpack_from(">i", var, off)
                        if otype != OBJECT_TYPE_AVG_PAIR:
                            raise ValueError(f"object type {otype}")
                        row.append(struct.unpack_from(">dq", var, off + 4))
                    else:
                        raise ValueError(f"column type {t}")
                    pos += w
                rows.append(tuple(row))
        pos = secs[4][0] + secs[4][1]  # the variable-size section's start is the end of the sections, also when empty
        metadata: Dict[str, str] = {}
        (mlen,) = struct.unpack_from(">i", b, pos)
        if mlen:
            pos += 4
            (n,), pos = struct.unpack_from(">i", b, pos), pos + 4
            for _ in range(n):
                (ordinal,), pos = struct.unpack_from(">i", b, pos), pos + 4
                # MetadataKey.getByOrdinal clamps to the last key, as the reference does (DataTable.java:128-130;
                # its "null" branch at DataTableImplV3.java:351-355 is unreachable)
                name, kind = METADATA_KEYS[min(ordinal, len(METADATA_KEYS) - 1)]
                if kind == "I":
                    metadata[name] = str(struct.unpack_from(">i", b, pos)[0])
                    pos += 4
                elif kind == "L":
                    metadata[name] = str(struct.unpack_from(">q", b, pos)[0])
                    pos += 8
                else:
                    (ln,) = struct.unpack_from(">i", b, pos)
                    metadata[name] = b[pos + 4: pos + 4 + ln].decode("utf-8")
                    pos += 4 + ln
        return DataTable(schema, rows, metadata, exceptions)


# ---- server: the result block -------------------------------------------------------------------------------------
_STORED = {0: INT, 1: LONG, 2: FLOAT, 3: DOUBLE, 4: STRING}  # PGPU_INT .. PGPU_STRING


_TYPE_NAME = {"COUNT": "count", "SUM": "sum", "MIN": "min", "MAX": "max", "AVG": "avg", "COUNTMV": "countMV",
              "SUMMV": "sumMV", "MINMV": "minMV", "MAXMV": "maxMV", "AVGMV": "avgMV"}  # AggregationFunctionType names


def _agg_column(a, result_name: bool) -> Tuple[str, str]:
    """(column name, intermediate result type) of an aggregation: getResultColumnName ("sum(m)", "count(*)") in a
    group-by schema, getColumnName ("sum_m", "count_star") in an aggregation-only one
    (BaseSingleInputAggregationFunction.java:42-49, CountAggregationFunction.java:36-56); LONG for COUNT / COUNTMV,
    OBJECT (AvgPair) for AVG / AVGMV, DOUBLE otherwise (getIntermediateResultColumnType)."""
    fn = a.function
    t = _TYPE_NAME[fn]
    if fn == "COUNT":
        name = "count(*)" if result_name else "count_star"
    else:
        name = f"{t.lower()}({a.column})" if result_name else f"{t}_{a.column}"
    return name, {"COUNT": LONG, "COUNTMV": LONG, "AVG": OBJECT, "AVGMV": OBJECT}.get(fn, DOUBLE)


def server_data_table(query: QueryContext, result, group_types: Sequence[int] = ()) -> DataTable:
    """IntermediateResultsBlock.getDataTable of a combined result (QueryResult): the group rows the server's
    IndexedTable returns (group values + intermediate results) or the one aggregation row, with the statistics
    attachMetadataToDataTable puts (numResizes / resizeTimeMs 0: the GPU table never resizes).  `group_types`: the
    group columns' stored types (PGPU_INT ...)."""
    aggs = [_agg_column(a, bool(query.group_by)) for a in query.aggregations]
    if query.group_by:
        schema = DataSchema(list(query.group_by) + [n for n, _ in aggs],
                            [_STORED[t] for t in group_types] + [t for _, t in aggs])
        rows = [tuple(k) + tuple(v) for k, v in result.intermediate.items()]
    else:
        schema = DataSchema([n for n, _ in aggs], [t for _, t in aggs])
        rows = [tuple(result.intermediate[()])]
    st = result.stats
    md = {"numDocsScanned": str(st.num_docs_scanned),
          "numEntriesScannedInFilter": str(st.num_entries_scanned_in_filter),
          "numEntriesScannedPostFilter": str(st.num_entries_scanned_post_filter),
          "numSegmentsProcessed": str(st.num_segments_processed),
          "numSegmentsMatched": str(st.num_segments_matched),
          "numResizes": "0", "resizeTimeMs": "0", "totalDocs": str(st.num_total_docs)}
    if getattr(st, "num_groups_limit_reached", False):  # DataTable.MetadataKey.NUM_GROUPS_LIMIT_REACHED
        md["numGroupsLimitReached"] = "true"
    return DataTable(schema, rows, md)


# ---- broker: reduce ------------------------------------------------------------------------------------------------
def _group_key(v):
    """A group value as the broker's Key compares it (Float.equals / Double.equals: by bits, one NaN)."""
    if isinstance(v, float):
        return ("f", "nan" if math.isnan(v) else struct.pack(">d", v))
    return ("v", v)


def _merge(fn: str, a, b):
    """AggregationFunction.merge of two intermediate results."""
    if fn in ("COUNT", "SUM", "COUNTMV", "SUMMV"):
        return a + b
    if fn in ("MIN", "MINMV"):
        return min(a, b)
    if fn in ("MAX", "MAXMV"):
        return max(a, b)
    return (a[0] + b[0], a[1] + b[1])  # AVG / AVGMV: AvgPair


def _final(fn: str, v):
    """AggregationFunction.extractFinalResult."""
    if fn in ("AVG", "AVGMV"):
        return -math.inf if v[1] == 0 else v[0] / v[1]
    if fn in ("COUNT", "COUNTMV"):
        return int(v)
    return float(v)


@dataclass
class BrokerResult:
    rows: List[tuple]                   # SELECT order, after ORDER BY / LIMIT
    num_docs_scanned: int = 0
    num_entries_scanned_in_filter: int = 0
    num_entries_scanned_post_filter: int = 0
    num_segments_processed: int = 0
    num_segments_matched: int = 0
    total_docs: int = 0
    num_groups_limit_reached: bool = False
    exceptions: Dict[int, str] = field(default_factory=dict)


def reduce_data_tables(query: QueryContext, tables: Sequence[DataTable]) -> BrokerResult:
    """GroupByDataTableReducer / AggregationDataTableReducer over the servers' DataTables."""
    from .plan import order_and_limit, to_select_order
    res = BrokerResult(rows=[])
    for t in tables:
        md = t.metadata
        res.num_docs_scanned += int(md.get("numDocsScanned", 0))
        res.num_entries_scanned_in_filter += int(md.get("numEntriesScannedInFilter", 0))
        res.num_entries_scanned_post_filter += int(md.get("numEntriesScannedPostFilter", 0))
        res.num_segments_processed += int(md.get("numSegmentsProcessed", 0))
        res.num_segments_matched += int(md.get("numSegmentsMatched", 0))
        res.total_docs += int(md.get("totalDocs", 0))
        res.num_groups_limit_reached |= md.get("numGroupsLimitReached") == "true"
        res.exceptions.update(t.exceptions)
    fns = [a.function for a in query.aggregations]
    ng = len(query.group_by)
    merged: Dict[tuple, list] = {}
    values: Dict[tuple, tuple] = {}
    for t in tables:
        if t.schema is None:
            continue
        for row in t.rows:
            k = tuple(_group_key(v) for v in row[:ng])
            inter = list(row[ng:])
            cur = merged.get(k)
            if cur is None:
                merged[k] = inter
                values[k] = tuple(row[:ng])
            else:
                merged[k] = [_merge(fn, x, y) for fn, x, y in zip(fns, cur, inter)]
    if not ng:
        inter = merged.get((), None)
        if inter is None:  # no server had a row: the functions' empty results
            inter = [{"COUNT": 0, "COUNTMV": 0, "MIN": math.inf, "MINMV": math.inf, "MAX": -math.inf,
                      "MAXMV": -math.inf, "AVG": (0.0, 0), "AVGMV": (0.0, 0)}.get(fn, 0.0) for fn in fns]
        res.rows = [to_select_order(query, tuple(_final(fn, v) for fn, v in zip(fns, inter)))]
        return res
    finals = [values[k] + tuple(_final(fn, v) for fn, v in zip(fns, merged[k])) for k in merged]
    res.rows = [to_select_order(query, r) for r in order_and_limit(query, finals)]
    return res
