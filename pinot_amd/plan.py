"""GpuPlanMaker: the host side of the drop-in boundary for aggregation / group-by queries.

Mirrors the reference's per-segment planning and hands the whole query to libpinotgpu in one call per GPU:

* filter tree -> physical operator tree, exactly as ``FilterPlanNode.constructPhysicalOperator``
  (core/plan/FilterPlanNode.java:192-313) and ``FilterOperatorUtils`` (leaf choice sorted > inverted > scan,
  empty/match-all folding, stable AND re-ordering by priority; core/operator/filter/FilterOperatorUtils.java:42-221);
  the tree is then emitted as the flat prefix program of ``pgpu_filter_node``;
* predicates -> dict-id ranges / sets per segment (``predicate.py``; SortedIndexBasedFilterOperator doc ranges,
  core/operator/filter/SortedIndexBasedFilterOperator.java:60-135; BitmapBasedFilterOperator matching /
  non-matching ids + flip, BitmapBasedFilterOperator.java:66-110);
* group-by columns -> a global dictionary (sorted union of the segment dictionaries) and per-segment remap
  tables, so that per-segment dict-id keys (DictionaryBasedGroupKeyGenerator raw keys, :275-322) merge across
  segments in HBM instead of in ``GroupByOrderByCombineOperator``'s IndexedTable (:127-248);
* results -> final aggregation values (``AggregationFunction.extractFinalResult``) and the execution statistics
  (CombineOperatorUtils.setExecutionStatistics, core/operator/combine/CombineOperatorUtils.java:55-82).

Group-count semantics: a segment whose map-based holder meets more than ``numGroupsLimit`` distinct keys keeps
only the first-seen ones in the reference (DictionaryBasedGroupKeyGenerator.java:137-164, :991-1016).  The library
counts the distinct keys of every segment whose key space could exceed the limit (hash group-by, include/
pinot_gpu.h) and fails only a query where one really does, with PGPU_E_UNSUPPORTED (``UnsupportedPlanError``):
the server keeps its CPU plan for it.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import time
import hashlib
import math
from fractions import Fraction
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import (ExprNode, Literal, PGPU_AGG_AVG, PGPU_AGG_COUNT, PGPU_AGG_MAX, PGPU_AGG_MIN, PGPU_AGG_SUM, PGPU_DOUBLE,
                   PGPU_FLOAT, PGPU_INT, PGPU_LONG, PGPU_RED_MAX_I64, PGPU_RED_MIN_I64, PGPU_RED_SUM_F64,
                   PGPU_RED_SUM_I64, PGPU_STRING, Agg, FilterNode, QueryDesc, QueryStats, SegmentPlan, TableLayout,
                   UnsupportedPlanError)
from .predicate import (DictPredicateEvaluator, RawPredicateEvaluator, SortedDictionary, get_predicate_evaluator,
                        get_raw_predicate_evaluator)
from .query import MV_AGGS, UNBOUNDED, AggregationSpec, FilterContext, QueryContext, split_filtered_aggregations
from .segment import DOCID_COLUMN, GpuContext, GpuSegment

AGG_FN = {"COUNT": PGPU_AGG_COUNT, "SUM": PGPU_AGG_SUM, "MIN": PGPU_AGG_MIN, "MAX": PGPU_AGG_MAX,
          "AVG": PGPU_AGG_AVG}
DEFAULT_NUM_GROUPS_LIMIT = 100_000          # InstancePlanMakerImplV2.java:73-74
DEFAULT_MAX_INIT_GROUP_HOLDER_CAPACITY = 10_000


# ---- physical filter operators (host-side tree) ---------------------------------------------------------------
@dataclass
class FilterOp:
    kind: str                                 # EMPTY, ALL, SCAN, INV, SORTED, RANGE_INDEX, RAW_SCAN, AND, OR, NOT
    children: List["FilterOp"] = field(default_factory=list)
    column: Optional[str] = None
    evaluator: Optional[DictPredicateEvaluator] = None
    raw: Optional[RawPredicateEvaluator] = None   # RAW_SCAN / RANGE_INDEX over a raw (no-dictionary) column
    doc_ranges: Optional[List[Tuple[int, int]]] = None
    negate: bool = False

    def priority(self) -> int:
        """FilterOperatorUtils.reorderAndFilterChildOperators#getPriority (single-value columns)."""
        if self.kind == "SORTED":
            return 0
        if self.kind == "INV":
            return 1
        if self.kind == "RANGE_INDEX":
            return 2
        if self.kind == "AND":
            return 3
        if self.kind == "OR":
            return 4
        if self.kind == "NOT":
            return self.children[0].priority()
        return 5  # SCAN / RAW_SCAN


EMPTY = FilterOp("EMPTY")
ALL = FilterOp("ALL")


class SegmentFilterPlanner:
    """FilterPlanNode + FilterOperatorUtils for one segment."""

    def __init__(self, seg: GpuSegment):
        self.seg = seg

    def dictionary(self, column: str) -> SortedDictionary:
        return self.seg.sorted_dictionary(column)

    def build(self, f: Optional[FilterContext]) -> FilterOp:
        return ALL if f is None else self._construct(f)

    def _construct(self, f: FilterContext) -> FilterOp:
        if f.type == "AND":
            kids = []
            for ch in f.children:
                op = self._construct(ch)
                if op.kind == "EMPTY":
                    return EMPTY
                if op.kind != "ALL":
                    kids.append(op)
            if not kids:
                return ALL
            if len(kids) == 1:
                return kids[0]
            kids.sort(key=lambda o: o.priority())  # stable, like List.sort with a Comparator
            return FilterOp("AND", kids)
        if f.type == "OR":
            kids = []
            for ch in f.children:
                op = self._construct(ch)
                if op.kind == "ALL":
                    return ALL
                if op.kind != "EMPTY":
                    kids.append(op)
            if not kids:
                return EMPTY
            if len(kids) == 1:
                return kids[0]
            return FilterOp("OR", kids)
        if f.type == "NOT":
            child = self._construct(f.children[0])
            if child.kind == "ALL":
                return EMPTY
            if child.kind == "EMPTY":
                return ALL
            return FilterOp("NOT", [child])
        return self._leaf(f.predicate)

    def _leaf(self, p) -> FilterOp:
        col = self.seg.column(p.column)
        if col.is_raw:
            # FilterOperatorUtils.getLeafFilterOperator (:42-81) without a dictionary: no always-true / -false
            # folding, no sorted or inverted index; RANGE over a range index, else a raw-value scan
            rv = get_raw_predicate_evaluator(p, col.data_type)
            kind = "RANGE_INDEX" if p.type == "RANGE" and col.range_index is not None else "RAW_SCAN"
            return FilterOp(kind, column=p.column, raw=rv)
        ev = get_predicate_evaluator(p, self.dictionary(p.column))
        if ev.always_false:
            return EMPTY
        if ev.always_true:
            return ALL
        if col.is_mv:
            # multi-value: BitmapBasedFilterOperator with an inverted index (non-RANGE), else MVScanDocIdIterator
            return FilterOp("INV" if p.type != "RANGE" and col.inverted is not None else "SCAN", column=p.column,
                            evaluator=ev)
        if col.is_sorted:
            return FilterOp("SORTED", column=p.column, evaluator=ev,
                            doc_ranges=self._sorted_ranges(self.seg.sorted_pairs(p.column), ev))
        if p.type == "RANGE" and col.range_index is not None:
            return FilterOp("RANGE_INDEX", column=p.column, evaluator=ev)
        if p.type != "RANGE" and col.inverted is not None:
            return FilterOp("INV", column=p.column, evaluator=ev)
        return FilterOp("SCAN", column=p.column, evaluator=ev)

    @staticmethod
    def _sorted_ranges(pairs: np.ndarray, ev: DictPredicateEvaluator) -> List[Tuple[int, int]]:
        if ev.kind == "RANGE":
            return [(int(pairs[ev.start, 0]), int(pairs[ev.end - 1, 1]))]
        ids = sorted(ev.ids)  # matching (inclusive) or non-matching (exclusive) ids
        ranges: List[Tuple[int, int]] = []
        for i in ids:
            s, e = int(pairs[i, 0]), int(pairs[i, 1])
            if ranges and s == ranges[-1][1] + 1:
                ranges[-1] = (ranges[-1][0], e)
            else:
                ranges.append((s, e))
        return ranges  # exclusive predicates complement these in the kernel (negate)


# numpy images of the C structs (include/pinot_gpu.h; sizes checked against ctypes below), so a whole query's
# per-segment programs are packed into a few buffers instead of thousands of ctypes objects
NODE_DTYPE = np.dtype({"names": ["op", "column", "pred", "negate", "lo", "hi", "ids", "num_ids", "reserved",
                                 "values"],
                       "formats": ["<i4"] * 6 + ["<u8", "<i4", "<i4", "<u8"],
                       "offsets": [0, 4, 8, 12, 16, 20, 24, 32, 36, 40], "itemsize": 48})
PLAN_DTYPE = np.dtype({"names": ["segment", "column_map", "filter", "num_filter_nodes", "reserved", "group_remap"],
                       "formats": ["<u8", "<u8", "<u8", "<i4", "<i4", "<u8"],
                       "offsets": [0, 8, 16, 24, 28, 32], "itemsize": 40})
assert NODE_DTYPE.itemsize == C.sizeof(FilterNode) and PLAN_DTYPE.itemsize == C.sizeof(SegmentPlan)


def raw_node_values(rv: RawPredicateEvaluator) -> Tuple[int, int, int, List[int]]:
    """(pred, lo flag, hi flag, 8-byte values as int64 bit patterns) of a raw-value leaf (include/pinot_gpu.h
    PGPU_F_RAW_SCAN): int64 for INT / LONG columns, IEEE doubles for FLOAT / DOUBLE."""
    def word(v) -> int:
        if rv.is_floating:
            return int(np.array([v], dtype=np.float64).view(np.int64)[0])
        return int(v)
    if rv.kind == "RANGE":
        return (_lib.PGPU_PRED_RANGE, int(rv.lower_inclusive), int(rv.upper_inclusive),
                [word(rv.lower), word(rv.upper)])
    return _lib.PGPU_PRED_SET, 0, 0, [word(v) for v in rv.values]


def emit_program(op: FilterOp, col_index: Dict[str, int], nodes: list, ids: list, vals: list) -> None:
    """Append the prefix-order program of pgpu_filter_node as tuples (op, column, pred, negate, lo, hi, ids
    offset, num_ids, values offset) to `nodes`; id lists go to the shared pool `ids` (offsets in int32 units),
    raw-value leaves' values to `vals` (int64 bit patterns, offsets in 8-byte units)."""
    F = _lib

    def pool(v: Sequence[int]) -> int:
        off = len(ids)
        ids.extend(v)
        return off

    def vpool(v: Sequence[int]) -> int:
        off = len(vals)
        vals.extend(v)
        return off

    def rec(o: FilterOp):
        k = o.kind
        if k == "EMPTY" or k == "ALL":
            nodes.append((F.PGPU_F_EMPTY if k == "EMPTY" else F.PGPU_F_MATCH_ALL, 0, 0, 0, 0, 0, 0, 0))
        elif (k == "RAW_SCAN" or k == "RANGE_INDEX") and o.raw is not None:
            rv = o.raw
            pred, lo, hi, words = raw_node_values(rv)
            nodes.append((F.PGPU_F_RAW_SCAN if k == "RAW_SCAN" else F.PGPU_F_RANGE_INDEX, col_index[o.column], pred,
                          1 if rv.is_exclusive else 0, lo, hi, 0, len(words) if pred == F.PGPU_PRED_SET else 0,
                          vpool(words)))
        elif k == "RANGE_INDEX":  # dictionary column: the dict-id range of the range index's exact answer
            ev = o.evaluator
            nodes.append((F.PGPU_F_RANGE_INDEX, col_index[o.column], F.PGPU_PRED_RANGE, 0, ev.start, ev.end, 0, 0))
        elif k == "SCAN":
            ev = o.evaluator
            neg = 1 if ev.is_exclusive else 0
            if ev.kind == "RANGE":
                nodes.append((F.PGPU_F_SCAN, col_index[o.column], F.PGPU_PRED_RANGE, neg, ev.start, ev.end, 0, 0))
            else:
                sid = sorted(ev.ids)
                if sid and sid[-1] - sid[0] + 1 == len(sid):
                    nodes.append((F.PGPU_F_SCAN, col_index[o.column], F.PGPU_PRED_RANGE, neg, sid[0], sid[-1] + 1,
                                  0, 0))
                else:
                    nodes.append((F.PGPU_F_SCAN, col_index[o.column], F.PGPU_PRED_SET, neg, 0, 0, pool(sid),
                                  len(sid)))
        elif k == "INV":
            ev = o.evaluator
            sid = ev.non_matching_dict_ids() if ev.is_exclusive else ev.matching_dict_ids()
            nodes.append((F.PGPU_F_INVERTED, col_index[o.column], 0, 1 if ev.is_exclusive else 0, 0, 0,
                          pool(sid), len(sid)))
        elif k == "SORTED":
            flat = [v for r in o.doc_ranges for v in r]
            neg = 1 if o.evaluator.is_exclusive and o.evaluator.kind == "SET" else 0
            nodes.append((F.PGPU_F_SORTED, col_index[o.column], 0, neg, 0, 0, pool(flat), len(o.doc_ranges)))
        elif k == "AND" or k == "OR":
            b, ce, e = ((F.PGPU_F_AND_BEGIN, F.PGPU_F_AND_CHILD_END, F.PGPU_F_AND_END) if k == "AND"
                        else (F.PGPU_F_OR_BEGIN, F.PGPU_F_OR_CHILD_END, F.PGPU_F_OR_END))
            nodes.append((b, 0, 0, 0, 0, 0, 0, 0))
            for ch in o.children:
                rec(ch)
                nodes.append((ce, 0, 0, 0, 0, 0, 0, 0))
            nodes.append((e, 0, 0, 0, 0, 0, 0, 0))
        elif k == "NOT":
            nodes.append((F.PGPU_F_NOT, 0, 0, 0, 0, 0, 0, 0))
            rec(o.children[0])
        else:
            raise ValueError(k)

    rec(op)


def check_group_columns(query: QueryContext, segments: Sequence[GpuSegment]) -> None:
    """Aggregation functions must match their columns' arity (*MV functions on multi-value columns only).  GROUP BY
    on a raw (no-dictionary) column reads its on-the-fly group dictionary (GpuSegment.group_view)."""
    for a in query.aggregations:
        if a.column is None or not segments:
            continue
        mv = segments[0].column(a.column).is_mv
        if mv != (a.function in MV_AGGS):
            raise UnsupportedPlanError(_lib.PGPU_E_UNSUPPORTED, f"{a.function} on {'a multi' if mv else 'a single'}"
                                                                f"-value column {a.column!r}")


# ---- results ---------------------------------------------------------------------------------------------------
@dataclass
class ExecutionStats:
    num_docs_scanned: int = 0
    num_entries_scanned_in_filter: int = 0   # the reference's count when filter_stats_exact, else the GPU's own
    num_entries_scanned_post_filter: int = 0
    num_total_docs: int = 0
    num_segments_processed: int = 0
    kernel_ms: float = 0.0
    filter_stats_exact: bool = True          # num_entries_scanned_in_filter is the reference's figure
    sparse_sector_bytes: int = 0
    dense_bytes: int = 0
    num_groups_limit_reached: bool = False   # some segment met >= numGroupsLimit distinct group keys
    num_segments_matched: int = 0            # segments with numDocsScanned > 0 (CombineOperatorUtils.java:64-67)
    segment_matched: Optional[np.ndarray] = None  # per segment of the launch (uint8), for unions over passes
    kernel_variant: int = -1                 # PGPU_KV_* of the launch (diagnostic; -1: not a single GPU launch)


def key_words_out(L: TableLayout) -> int:
    """int64 words per compacted group key (pgpu_table_compact): 2 for two-word hash keys, else 1."""
    return 2 if L.key_kind == _lib.PGPU_KEYS_HASH and L.key_words == 2 else 1


@dataclass
class GroupTable:
    """Compacted partial table: global keys + cells (section 0 = count, then one section per non-COUNT agg)."""

    keys: np.ndarray          # int64 [n] (mixed-radix key) or [n, 2] (two key words, layout.key_split)
    cells: np.ndarray         # int64 [n, nsec]
    layout: TableLayout

    @staticmethod
    def sorted(keys: np.ndarray, cells: np.ndarray, layout: TableLayout) -> "GroupTable":
        """Rows in ascending key order (hash tables compact in slot order; dense ones already are)."""
        if layout.key_kind == _lib.PGPU_KEYS_HASH and len(keys):
            order = np.lexsort((keys[:, 0], keys[:, 1])) if keys.ndim == 2 else np.argsort(keys, kind="stable")
            keys, cells = keys[order], cells[order]
        return GroupTable(keys, cells, layout)


class QueryResult:
    """Final result of one query.  For group-by, ``group_rows`` (every group) and ``intermediate`` are
    materialised from the vectorised columns on first access; ``rows`` (after ORDER BY / LIMIT) always is."""

    def __init__(self, query: QueryContext, stats: Optional[ExecutionStats] = None):
        self.query = query
        self.stats = stats if stats is not None else ExecutionStats()
        self.aggregation_result: Optional[List] = None   # aggregation-only: final values in aggregation order
        self.rows: Optional[List[tuple]] = None           # SELECT-ordered rows after ORDER BY / LIMIT
        self._columns: Optional["GroupColumns"] = None
        self._group_rows: Optional[List[tuple]] = None
        self._intermediate: Optional[dict] = None

    @property
    def group_rows(self) -> Optional[List[tuple]]:
        """group-by: (group values..., final agg values...) for every group, ascending by global key."""
        if self._group_rows is None and self._columns is not None:
            self._group_rows = self._columns.rows()
        return self._group_rows

    @property
    def intermediate(self) -> Optional[dict]:
        """group values -> intermediate values (AVG as (sum, count))."""
        if self._intermediate is None and self._columns is not None:
            self._intermediate = self._columns.intermediate()
        return self._intermediate


def join_parts(row_cells, sec: int, parts: int, exp: Optional[int] = None):
    """Exact SUM of a cell split into 21-bit-part sections (pgpu_table_layout.agg_sum_parts > 1):
    sum_k c[sec+k] * 2^(21k), as a Python int (rounded once, on conversion to double).  A fixed-point floating SUM
    (exp = its agg_sum_exp, see sum_exp_of) is that integer times 2^exp, rounded once to a double -- +-infinity past
    DBL_MAX, as the reference's double adds overflow."""
    if parts <= 1:
        return int(row_cells[sec])
    b = _lib.PGPU_PART_BITS
    total = sum(int(row_cells[sec + k]) << (b * k) for k in range(parts))
    if exp is None:
        return total
    if total == 0 or exp == _lib.PGPU_SUM_EXP_ZERO:
        return 0.0
    try:
        return math.ldexp(float(total), exp)
    except OverflowError:
        return math.inf if total > 0 else -math.inf


def sum_exp_of(L: TableLayout, ai: int) -> Optional[int]:
    """The fixed-point exponent of aggregation ai's split SUM, or None for an integer (or float64) sum: fixed point is
    a FLOAT / DOUBLE SUM carried in part sections, whatever its exponent (0 is a valid one)."""
    if L.agg_value_type[ai] in (PGPU_FLOAT, PGPU_DOUBLE) and L.agg_sum_parts[ai] > 1:
        return L.agg_sum_exp[ai]
    return None


def fixed_window(top: int, bottom: int) -> Tuple[int, int]:
    """(exp, parts) of the fixed-point window covering [2^bottom, 2^top) in 21-bit parts (at least 3), as
    pgpu_sum_layout_agree chooses it; parts > PGPU_MAX_FIXED_PARTS means every launch keeps a float64 section."""
    b = _lib.PGPU_PART_BITS
    p = max(3, -(-(top - bottom) // b))
    return top - b * p, min(p, _lib.PGPU_MAX_FIXED_PARTS + 1)


def final_value(fn: str, cell_count: int, cell: Optional[int], op: int, vtype: int):
    """AggregationFunction.extractFinalResult on a merged cell (an exact Python int for integer sums)."""
    if fn == "COUNT":
        return int(cell_count)
    if fn == "SUM":
        return float(cell) if op == PGPU_RED_SUM_I64 else float(np.int64(cell).view(np.float64))
    if fn in ("MIN", "MAX"):
        if cell_count == 0:
            return math.inf if fn == "MIN" else -math.inf
        return _lib.decode_minmax_key(int(cell), vtype)
    if fn == "AVG":
        if cell_count == 0:
            return -math.inf  # AvgAggregationFunction DEFAULT_FINAL_RESULT
        s = float(cell) if op == PGPU_RED_SUM_I64 else float(np.int64(cell).view(np.float64))
        return s / cell_count
    raise ValueError(fn)


def intermediate_value(fn: str, cell_count: int, cell, op: int, vtype: int):
    if fn == "AVG":
        s = float(cell) if op == PGPU_RED_SUM_I64 else float(np.int64(cell).view(np.float64))
        return (s, int(cell_count))
    return final_value(fn, cell_count, cell, op, vtype)


def order_and_limit(query: QueryContext, rows: List[tuple]) -> List[tuple]:
    """Broker-side ORDER BY / LIMIT over final rows (GroupByDataTableReducer, IndexedTable.finish)."""
    names = list(query.group_by) + [a.result_name for a in query.aggregations]
    if query.order_by:
        for ob in reversed(query.order_by):
            idx = names.index(ob.expression)
            rows = sorted(rows, key=lambda r, i=idx: r[i], reverse=not ob.ascending)
    return rows[: query.limit]


DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE = 5000  # GroupByUtils.DEFAULT_MIN_NUM_GROUPS


def table_capacity(limit: int, min_trim: int = DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE) -> int:
    """GroupByUtils.getTableCapacity(limit, minNumGroups) (core/util/GroupByUtils.java:24-41): the IndexedTable's
    trim size; GroupByOrderByCombineOperator.java:80-95 disables the trim for a non-positive minimum."""
    return max(5 * limit, min_trim) if min_trim > 0 else (1 << 62)


def topk_spec(query: QueryContext, cards: Sequence[int], k: int, key_base: int = 0) -> Optional[_lib.TopK]:
    """pgpu_topk for the query's first ORDER BY expression (include/pinot_gpu.h): the groups the server's
    IndexedTable.finish would hand the broker, ties at the k-th kept.  None when there is nothing to trim by."""
    if not query.group_by or not query.order_by or k <= 0:
        return None
    ob = query.order_by[0]
    names = list(query.group_by) + [a.result_name for a in query.aggregations]
    i = names.index(ob.expression)
    ng = len(query.group_by)
    t = _lib.TopK()
    t.k, t.key_base, t.descending = int(k), int(key_base), 0 if ob.ascending else 1
    if i < ng:
        carr = (C.c_int32 * ng)(*[int(c) for c in cards])  # global cardinality per group column
        t.source, t.group_index, t.num_group_columns = _lib.PGPU_TOPK_GROUP, i, ng
        t.group_cardinalities = C.cast(carr, C.POINTER(C.c_int32))
        t._keep = carr  # the cardinalities live as long as the spec
    else:
        t.source, t.agg_index = _lib.PGPU_TOPK_AGG, i - ng
        t.agg_fn = AGG_FN[query.aggregations[i - ng].function]
    return t


def to_select_order(query: QueryContext, row: tuple) -> tuple:
    names = list(query.group_by) + [a.result_name for a in query.aggregations]
    out = []
    for s in query.select:
        key = s if isinstance(s, str) else s.result_name
        out.append(row[names.index(key)])
    return tuple(out)


def order_key(v: np.ndarray) -> np.ndarray:
    """Sort / equality key of dictionary values: the values themselves, or for FLOAT / DOUBLE their bits as an
    order-preserving int64 (Float.compare order: -0.0 before 0.0, one NaN last) -- the identity of a map key in the
    reference's no-dictionary group-key generators (floatToIntBits / doubleToLongBits)."""
    v = np.asarray(v)
    if v.dtype.kind != "f":
        return v
    if v.dtype == np.float32:
        b = np.where(np.isnan(v), np.int32(0x7FC00000), v.view(np.int32)).astype(np.int64)
        return np.where(b >= 0, b, b ^ np.int64(0x7FFFFFFF))
    b = np.where(np.isnan(v), np.int64(0x7FF8000000000000), v.view(np.int64))
    return np.where(b >= 0, b, b ^ np.int64(0x7FFFFFFFFFFFFFFF))


def union_sorted(parts: Sequence[np.ndarray]) -> np.ndarray:
    """Sorted union of numeric dictionaries; FLOAT / DOUBLE values distinct by bits (order_key)."""
    allv = np.concatenate([np.asarray(p) for p in parts]) if len(parts) else np.zeros(0)
    if allv.dtype.kind != "f":
        return np.unique(allv)
    _, idx = np.unique(order_key(allv), return_index=True)
    return allv[idx]


def dictionary_digest(glob) -> str:
    """Content digest of a global dictionary: remap tables are cached per (segment, column, digest), so two
    different global dictionaries of the same length never share one."""
    h = hashlib.blake2b(digest_size=16)
    if isinstance(glob, list):
        for v in glob:
            b = str(v).encode("utf-8")
            h.update(len(b).to_bytes(4, "little"))
            h.update(b)
    else:
        a = np.ascontiguousarray(glob)
        h.update(str(a.dtype).encode())
        h.update(a.tobytes())
    return h.hexdigest()


# ---- plan maker ------------------------------------------------------------------------------------------------
class GpuPlanMaker:
    """PlanMaker for the GPU path (core/plan/maker/PlanMaker.java:36-59): one launch per query per GPU."""

    def __init__(self, ctx: GpuContext, num_groups_limit: int = DEFAULT_NUM_GROUPS_LIMIT,
                 max_init_group_holder_capacity: int = DEFAULT_MAX_INIT_GROUP_HOLDER_CAPACITY,
                 collect_stats: bool = False, query_flags: int = 0, host_planning: bool = False,
                 exact_filter_stats: bool = False, timeout_ms: Optional[int] = None, gpu_topk: bool = True,
                 min_server_group_trim_size: int = DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE):
        self.ctx = ctx
        # pinot.server.query.executor.min.server.group.trim.size (InstancePlanMakerImplV2.java:80-84): the minimum
        # of the server's ORDER BY trim; <= 0 disables it (every group comes back)
        self.min_server_group_trim_size = min_server_group_trim_size
        # gpu_topk: a GROUP BY ... ORDER BY ... LIMIT query brings back only the groups the server's IndexedTable
        # keeps (table_capacity(limit), ties kept), selected on the GPU (pgpu_query_collect_topk)
        self.gpu_topk = gpu_topk
        # timeout_ms: the query's budget from submit (QueryOptions timeoutMs -> QueryContext.getEndTimeMs); past it
        # the query is cancelled and collect raises QueryTimeoutError (EXECUTION_TIMEOUT_ERROR)
        self.timeout_ms = timeout_ms
        # exact_filter_stats: numEntriesScannedInFilter as the reference's iterators count it, also where they
        # leap-frog (PGPU_Q_EXACT_FILTER_STATS: one more pass over every filter leaf, replayed on the host)
        self.exact_filter_stats = exact_filter_stats
        # host_planning: plan every segment's filter in Python (SegmentFilterPlanner) even when the library could
        # (numeric columns: pgpu_query_submit_expr plans all segments in C++ from the literals)
        self.host_planning = host_planning
        self.query_flags = query_flags   # extra PGPU_Q_* flags (strategy overrides for tests / tuning)
        self.num_groups_limit = num_groups_limit
        self.max_init_group_holder_capacity = max_init_group_holder_capacity
        self.collect_stats = collect_stats
        self._global_dicts: Dict[tuple, tuple] = {}
        self._col_kinds: Dict[tuple, tuple] = {}  # segment uids -> (raw columns, raw or range-indexed columns)
        self._desc_static: Dict[tuple, tuple] = {}  # (segment uids, columns, views) -> (column maps, handles)
        # prepared submissions: the same query object over the same segments with the same options re-submitted
        # (a dashboard's repeated query) reuses its filter program, descriptor and trim -- only the deadline is
        # restamped.  Dropped whenever a global dictionary or a segment it names changes.
        self._prepared: Dict[tuple, tuple] = {}
        if hasattr(ctx, "add_listener"):
            ctx.add_listener(self)  # segment_released: forget global dictionaries naming a released segment

    def segment_released(self, uid: int) -> None:
        self._prepared.clear()
        for k in [k for k in self._global_dicts if uid in k[1]]:
            self._evict_global(k)
        for k in [k for k in self._col_kinds if uid in k[:-1]]:
            del self._col_kinds[k]
        for k in [k for k in self._desc_static if uid in k[0]]:
            del self._desc_static[k]

    def column_kinds(self, segments: Sequence[GpuSegment]) -> tuple:
        """(columns raw in some segment, columns raw or range-indexed in some segment) of a segment set: fixed once
        the segments are sealed, so computed once per set instead of per query and predicate."""
        key = tuple(s.uid for s in segments) + (sum(len(s.derived) for s in segments),)  # (columns derived later)
        hit = self._col_kinds.get(key)
        if hit is None:
            raw, host = set(), set()
            for s in segments:
                for name in set(s.data.columns) | set(s.derived):
                    c = s.column(name)
                    if c.is_raw:
                        raw.add(name)
                    if c.is_raw or c.range_index is not None:
                        host.add(name)
            if len(self._col_kinds) >= 64:
                self._col_kinds.clear()
            hit = self._col_kinds[key] = (frozenset(raw), frozenset(host))
        return hit

    def _evict_global(self, key: tuple) -> None:
        self._prepared.clear()  # (prepared descriptors may name its remap buffers)
        entry = self._global_dicts.pop(key)
        for rk in entry[3]:
            self.ctx.unref_remap(rk)

    # -- global group dictionaries --
    def global_dictionary(self, column: str, segments: Sequence[GpuSegment]):
        """Global dictionary of a group column (sorted union of the segments' dictionaries -- a raw column's
        on-the-fly group dictionaries -- unless a wider one was installed by set_global_dictionary) and per-segment
        remap buffers (None = identity)."""
        key = (column, tuple(s.uid for s in segments))
        hit = self._global_dicts.get(key)
        if hit is not None:
            return hit[:2]
        dicts = [s.dictionaries[s.group_view(column)] for s in segments]
        first = dicts[0]
        if isinstance(first, list):
            glob = sorted(set().union(*[set(d) for d in dicts]))
        elif len(dicts) == 1:
            glob = np.asarray(first)
        else:
            glob = union_sorted(dicts)
        return self.set_global_dictionary(column, segments, glob)

    def set_global_dictionary(self, column: str, segments: Sequence[GpuSegment], glob):
        key = (column, tuple(s.uid for s in segments))
        remaps = []
        rkeys = []
        digest = dictionary_digest(glob)
        if isinstance(glob, list):
            pos = {v: i for i, v in enumerate(glob)}
        for s in segments:
            d = s.dictionaries[s.group_view(column)]
            if not isinstance(glob, list):
                d = np.asarray(d, dtype=glob.dtype)  # exact widening (FLOAT -> DOUBLE keeps -0.0 and NaN)
            if len(d) == len(glob) and (list(d) == list(glob) if isinstance(d, list) else
                                        np.array_equal(order_key(d), order_key(glob))):
                remaps.append(None)
                continue
            if isinstance(glob, list):
                t = np.array([pos[v] for v in d], dtype=np.int32)
            else:
                t = np.searchsorted(order_key(glob), order_key(d)).astype(np.int32)
            remaps.append(self.ctx.remap((s.uid, column, digest), t))
            rkeys.append((s.uid, column, digest))
        if key in self._global_dicts:
            self._evict_global(key)  # replaced (a wider dictionary installed): its remap references go
        # the entry holds the segments themselves, so their uids stay theirs while it is cached
        self._global_dicts[key] = (glob, remaps, tuple(segments), rkeys)
        return glob, remaps

    def filter_expr(self, query: QueryContext, segments: Sequence[GpuSegment]):
        """The query's filter as a pgpu_expr_node program (planned per segment inside the library), or None when
        it must be planned here: STRING columns, literals that are not numbers, or host_planning."""
        f = query.filter
        if f is None or self.host_planning or not segments:
            return None
        col_index = {c: i for i, c in enumerate(query.columns)}
        seg0 = segments[0]
        host_cols = self.column_kinds(segments)[1]
        nodes: list = []
        lits: list = []

        def lit(v: str):
            try:
                i = int(v)
                return (i, float(i), 1) if -(1 << 63) <= i < (1 << 63) else None
            except ValueError:
                pass
            try:
                fr = Fraction(v)
            except (ValueError, ZeroDivisionError):
                return None
            if fr.denominator == 1:
                i = int(fr)
                return (i, float(fr), 1) if -(1 << 63) <= i < (1 << 63) else None
            return (0, float(fr), 0)

        def rec(fc) -> bool:
            if fc.type in ("AND", "OR"):
                nodes.append([_lib.PGPU_X_AND if fc.type == "AND" else _lib.PGPU_X_OR, len(fc.children)])
                return all(rec(ch) for ch in fc.children)
            if fc.type == "NOT":
                nodes.append([_lib.PGPU_X_NOT, 1])
                return rec(fc.children[0])
            p = fc.predicate
            if seg0.column(p.column).data_type == PGPU_STRING:
                return False
            if p.column in host_cols:
                return False  # raw-value leaves / range-index leaves: planned per segment here
            kind = {"EQ": _lib.PGPU_P_EQ, "NOT_EQ": _lib.PGPU_P_NOT_EQ, "IN": _lib.PGPU_P_IN,
                    "NOT_IN": _lib.PGPU_P_NOT_IN, "RANGE": _lib.PGPU_P_RANGE}[p.type]
            if p.type == "RANGE":
                vals = [p.lower if p.lower != UNBOUNDED else "0", p.upper if p.upper != UNBOUNDED else "0"]
            else:
                vals = list(p.values)
            parsed = [lit(v) for v in vals]
            if any(x is None for x in parsed):
                return False
            nodes.append([_lib.PGPU_X_PRED, 0, col_index[p.column], kind, int(p.lower == UNBOUNDED),
                          int(p.upper == UNBOUNDED), int(p.lower_inclusive), int(p.upper_inclusive), len(parsed),
                          len(lits)])
            lits.extend(parsed)
            return True

        if not rec(f):
            return None
        la = (Literal * max(1, len(lits)))(*[Literal(i, d, ig, 0) for i, d, ig in lits])
        arr = (ExprNode * len(nodes))()
        for k, nd in enumerate(nodes):
            e = arr[k]
            e.op, e.num_children = nd[0], nd[1]
            if nd[0] == _lib.PGPU_X_PRED:
                (e.column, e.pred, e.lower_unbounded, e.upper_unbounded, e.lower_inclusive, e.upper_inclusive,
                 e.num_values) = nd[2:9]
                e.values = C.cast(C.byref(la, nd[9] * C.sizeof(Literal)), C.POINTER(Literal))
        return arr, len(nodes), la

    def build_desc(self, query: QueryContext, segments: Sequence[GpuSegment], plan_filters: bool = True,
                   extra_flags: int = 0, reduce_docs: int = 0,
                   sum_layout: Optional[Tuple[Sequence[int], Sequence[int]]] = None):
        """Build the pgpu_query_desc.  Returns (desc, keep, globals_): `keep` owns every buffer the descriptor
        points to (one node array, one id pool, one column-map array, one remap-handle array, one plan array).
        plan_filters=False leaves the per-segment filter programs empty (the library plans them from
        filter_expr); sum_layout = (exps, parts) per aggregation is the floating SUMs' fixed-point layout that callers
        combining tables across ranks agree on (fixed_window; pgpu_query_desc.sum_exp / sum_parts)."""
        columns = list(query.columns)
        col_index = {c: i for i, c in enumerate(columns)}
        nseg = len(segments)
        check_group_columns(query, segments)
        globals_ = [self.global_dictionary(g, segments) for g in query.group_by]
        # a group column that is raw (no-dictionary) in some segment is read through its on-the-fly group dictionary
        # there (GpuSegment.group_view): one more descriptor column per such group column, mapped per segment, so
        # that filters and aggregations on the same column keep reading its values
        group_col = {}
        views: Dict[int, str] = {}
        no_dict = False
        raw_cols = self.column_kinds(segments)[0] if segments else frozenset()
        for g in query.group_by:
            if g in raw_cols:
                no_dict = True
                views[len(columns)] = g
                group_col[g] = len(columns)
                columns.append(f"{g}$group")
            else:
                group_col[g] = col_index[g]
        nodes: list = []
        ids: list = []
        vals: list = []
        flt = query.filter if plan_filters else None
        # the column maps and segment handles are fixed for a segment set and column list: built once, shared
        # read-only by every descriptor that names them
        skey = (tuple(s.uid for s in segments), tuple(columns), tuple(sorted(views.items())))
        static = self._desc_static.get(skey)
        if static is None:
            cmaps = [[slots[seg.group_view(views[i])] if i in views else slots[c] for i, c in enumerate(columns)]
                     if columns else [0] for seg, slots in ((seg, seg.slots) for seg in segments)]
            cmap = np.array(cmaps, dtype=np.int32).reshape(nseg, max(1, len(columns)))
            handles = np.array([seg.handle.value for seg in segments], dtype=np.uint64)
            if len(self._desc_static) >= 64:
                self._desc_static.clear()
            static = self._desc_static[skey] = (cmap, handles)
        cmap, handles = static
        if flt is not None:
            starts = []
            for seg in segments:
                starts.append(len(nodes))
                op = SegmentFilterPlanner(seg).build(flt)
                if op.kind != "ALL":
                    emit_program(op, col_index, nodes, ids, vals)
            starts.append(len(nodes))
        else:
            starts = [0] * (nseg + 1)
        pool = np.array(ids if ids else [0], dtype=np.int32)
        vpool = np.array(vals if vals else [0], dtype=np.int64)
        narr = np.zeros(max(1, len(nodes)), dtype=NODE_DTYPE)
        if nodes:
            t = np.array([nd if len(nd) == 9 else nd + (-1,) for nd in nodes], dtype=np.int64)
            for j, name in enumerate(("op", "column", "pred", "negate", "lo", "hi")):
                narr[name] = t[:, j]
            narr["ids"] = pool.ctypes.data + 4 * t[:, 6]
            narr["num_ids"] = t[:, 7]
            narr["values"] = np.where(t[:, 8] >= 0, vpool.ctypes.data + 8 * np.maximum(t[:, 8], 0), 0).astype(np.uint64)
        ng = len(query.group_by)
        remap = np.zeros((nseg, max(1, ng)), dtype=np.uint64)
        for g, (_, rms) in enumerate(globals_):
            remap[:, g] = [(rm.handle.value or 0) if rm is not None else 0 for rm in rms]
        plans = np.zeros(nseg, dtype=PLAN_DTYPE)
        plans["segment"] = handles
        plans["column_map"] = cmap.ctypes.data + cmap.strides[0] * np.arange(nseg, dtype=np.uint64)
        st = np.array(starts, dtype=np.int64)
        plans["filter"] = narr.ctypes.data + NODE_DTYPE.itemsize * st[:-1].astype(np.uint64)
        plans["num_filter_nodes"] = st[1:] - st[:-1]
        if ng:
            plans["group_remap"] = remap.ctypes.data + remap.strides[0] * np.arange(nseg, dtype=np.uint64)
        aggs = (Agg * len(query.aggregations))(
            *[Agg(AGG_FN[a.function], -1 if a.column is None else col_index[a.column]) for a in query.aggregations])
        gcols = (C.c_int32 * max(1, ng))(*[group_col[g] for g in query.group_by])
        gcards = (C.c_int32 * max(1, ng))(*[len(g[0]) for g in globals_])
        na = max(1, len(query.aggregations))
        sexp = (C.c_int32 * na)(*sum_layout[0]) if sum_layout is not None else None
        sparts = (C.c_int32 * na)(*sum_layout[1]) if sum_layout is not None else None
        keep = [cmap, pool, vpool, narr, remap, plans, aggs, gcols, gcards, sexp, sparts]
        desc = QueryDesc(num_columns=len(columns), num_segments=nseg,
                         segments=C.cast(C.c_void_p(plans.ctypes.data), C.POINTER(SegmentPlan)),
                         num_aggs=len(query.aggregations), num_group_columns=ng, aggs=aggs,
                         group_columns=gcols, group_cardinalities=gcards,
                         flags=(_lib.PGPU_Q_STATS if self.collect_stats else 0) | self.query_flags | extra_flags |
                         (_lib.PGPU_Q_EXACT_FILTER_STATS if self.exact_filter_stats else 0),
                         reduce_docs=reduce_docs, num_groups_limit=self.num_groups_limit,
                         # NoDictionary*GroupKeyGenerator caps every key space at numGroupsLimit: with a raw group
                         # column no segment is array-based (a segment meeting more keys goes back to the CPU)
                         array_based_threshold=0 if no_dict else self.max_init_group_holder_capacity,
                         deadline_ms=0 if self.timeout_ms is None else int(time.time() * 1000) + int(self.timeout_ms),
                         sum_exp=C.cast(sexp, C.POINTER(C.c_int32)) if sexp is not None else None,
                         sum_parts=C.cast(sparts, C.POINTER(C.c_int32)) if sparts is not None else None)
        return desc, keep, globals_

    def layout(self, desc: QueryDesc) -> TableLayout:
        L = TableLayout()
        _lib.check(self.ctx._lib.pgpu_table_layout_of(C.byref(desc), C.byref(L)))
        return L

    def submit(self, query: QueryContext, segments: Sequence[GpuSegment]) -> "PendingQuery":
        """Plan the query and enqueue it on the GPU without waiting (pgpu_query_submit).  Several queries may be
        in flight: the host plans the next one while the GPU runs this one.  *MV aggregations run lowered onto
        the multi-value columns' row columns (pinot_amd/mv.py) and are raised back in collect()."""
        if has_mv_aggregations(query):
            check_group_columns(query, segments)
            low, parts = mv_lower(query)
            pq = self.submit(low, segments)
            pq.mv = (query, parts)
            return pq
        if query.has_filtered_aggregations:
            raise _lib.UnsupportedPlanError(_lib.PGPU_E_UNSUPPORTED,
                                            "filtered aggregations run one pass per FILTER clause: use execute()")
        pkey = (id(query), tuple(s.uid for s in segments), self.collect_stats, self.exact_filter_stats,
                self.query_flags, self.num_groups_limit, self.max_init_group_holder_capacity, self.host_planning,
                self.gpu_topk, self.min_server_group_trim_size)
        hit = self._prepared.get(pkey)
        if hit is not None and hit[0] is query:
            _, expr, desc, keep, globals_, L, order = hit
            desc.deadline_ms = 0 if self.timeout_ms is None else int(time.time() * 1000) + int(self.timeout_ms)
        else:
            expr = self.filter_expr(query, segments)
            desc, keep, globals_ = self.build_desc(query, segments, plan_filters=expr is None)
            L = self.layout(desc)
            # the server trim is known now: big tables are ranked and compacted behind the kernels (collect only
            # copies)
            order = self.trim_order(query, globals_)
            if len(self._prepared) >= 32:
                self._prepared.clear()
            self._prepared[pkey] = (query, expr, desc, keep, globals_, L, order)
        h = C.c_void_p()
        _lib.check(self.ctx._lib.pgpu_query_submit_ordered(
            self.ctx.handle, C.byref(desc), expr[0] if expr is not None else None, expr[1] if expr is not None else 0,
            C.byref(order) if order is not None else None, C.byref(h)))
        pq = PendingQuery(self, query, len(segments), h, L, globals_)
        pq.order = order
        pq.matched = np.zeros(max(1, len(segments)), dtype=np.uint8)
        _lib.check(self.ctx._lib.pgpu_query_matched_segments(h, pq.matched.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                             len(segments)))
        return pq

    def trim_order(self, query: QueryContext, globals_) -> Optional[_lib.TopK]:
        """The IndexedTable trim of GROUP BY ... ORDER BY ... LIMIT (table_capacity(limit), ties kept) as a
        pgpu_topk, or None when every group comes back (no ORDER BY, trim disabled, or gpu_topk off)."""
        if not (self.gpu_topk and self.min_server_group_trim_size > 0):
            return None
        return topk_spec(query, [len(g[0]) for g in globals_],
                         table_capacity(query.limit, self.min_server_group_trim_size))

    def collect(self, pending: "PendingQuery") -> QueryResult:
        """Wait for a submitted query and finish it (pgpu_query_collect + ORDER BY / LIMIT on the host)."""
        if pending.mv is not None:
            query, parts = pending.mv
            pending.mv = None
            return mv_raise(query, parts, self.collect(pending))
        L = pending.layout
        cap = int(min(L.num_keys, 1 << 26))
        kw = key_words_out(L)
        keys = np.empty(max(cap, 1) * kw, dtype=np.int64)
        cells = np.empty((max(cap, 1), L.num_sections), dtype=np.int64)
        n = C.c_uint64()
        st = QueryStats()
        h, pending.handle = pending.handle, None
        query = pending.query
        order = pending.order
        _lib.check(self.ctx._lib.pgpu_query_collect_topk(h, C.byref(order) if order is not None else None,
                                                         keys.ctypes.data_as(C.POINTER(C.c_int64)),
                                                         cells.ctypes.data_as(C.POINTER(C.c_int64)), cap, C.byref(n),
                                                         C.byref(st)))
        table = GroupTable.sorted(keys[: n.value * kw].reshape(-1, kw) if kw > 1 else keys[: n.value],
                                  cells[: n.value], L)
        stats = ExecutionStats(num_docs_scanned=st.num_docs_scanned,
                               num_entries_scanned_in_filter=st.num_entries_scanned_in_filter,
                               num_entries_scanned_post_filter=st.num_docs_scanned * len(query.projected_columns),
                               num_total_docs=st.num_total_docs, num_segments_processed=pending.num_segments,
                               kernel_ms=st.kernel_ms, sparse_sector_bytes=st.sparse_sector_bytes,
                               dense_bytes=st.dense_bytes, filter_stats_exact=bool(st.filter_stats_exact),
                               num_groups_limit_reached=bool(st.num_groups_limit_reached),
                               num_segments_matched=st.num_segments_matched,
                               segment_matched=pending.matched[:pending.num_segments].copy(),
                               kernel_variant=st.kernel_variant)
        return finish(query, table, [g[0] for g in pending.globals_], stats)

    def execute(self, query: QueryContext, segments: Sequence[GpuSegment]) -> QueryResult:
        if query.has_filtered_aggregations:
            parts = split_filtered_aggregations(query)
            pending = [self.submit(sq, segments) for sq, _ in parts]  # all in flight, then collected in order
            return merge_filtered(query, parts, [self._collect_or_first_seen(pq, sq, segments)
                                                 for pq, (sq, _) in zip(pending, parts)])
        non_scan = self.non_scan_segments(query, segments)
        if any(non_scan):
            rest = [s for s, ns in zip(segments, non_scan) if not ns]
            res = self.collect(self.submit(query, rest)) if rest else None
            return merge_non_scan(query, res, [s for s, ns in zip(segments, non_scan) if ns])
        try:
            return self.collect(self.submit(query, segments))
        except _lib.GroupsLimitError:
            return self.first_seen_groups(query, segments)

    def _collect_or_first_seen(self, pending, query: QueryContext, segments: Sequence[GpuSegment]) -> QueryResult:
        """collect(), answering a numGroupsLimit overflow by the first-seen path (a filtered aggregation's part)."""
        try:
            return self.collect(pending)
        except _lib.GroupsLimitError:
            return self.first_seen_groups(query, segments)

    def first_seen_groups(self, query: QueryContext, segments: Sequence[GpuSegment]) -> QueryResult:
        """A segment met more distinct group keys than numGroupsLimit (PGPU_E_GROUPS_LIMIT).  The reference's
        map-based holders give group ids in doc order and drop every key past the limit, with its docs
        (DictionaryBasedGroupKeyGenerator.java:384-463, IntGroupIdMap.getGroupId :991-1016; NoDictionary*
        GroupKeyGenerator likewise).  Segments whose key space cannot exceed the limit run together as usual; each
        other segment runs alone with no limit plus MIN over its doc-id column (GpuSegment.docid_view), i.e. every
        group's first doc, and keeps the num_groups_limit groups of smallest first doc.  The partial results merge
        as the combine merges segment results (AggregationFunction.merge)."""
        from .datatable import _merge
        limit = self.num_groups_limit
        no_dict = any(s.column(g).is_raw for s in segments for g in query.group_by)
        thr = 0 if no_dict else self.max_init_group_holder_capacity

        def key_space(s):
            P = 1
            for g in query.group_by:
                P *= max(1, s.column(s.group_view(g)).cardinality)
            return P

        capped = [key_space(s) > max(0, thr) and key_space(s) > limit for s in segments]
        free = [s for s, c in zip(segments, capped) if not c]
        parts = []
        st = ExecutionStats()
        if free:
            r = self.execute(query, free)
            parts.append((r.intermediate, r.stats))
        sub = GpuPlanMaker(self.ctx, num_groups_limit=0, max_init_group_holder_capacity=self.max_init_group_holder_capacity,
                           collect_stats=self.collect_stats, query_flags=self.query_flags,
                           host_planning=self.host_planning, exact_filter_stats=self.exact_filter_stats,
                           timeout_ms=self.timeout_ms, gpu_topk=False, min_server_group_trim_size=-1)
        probe = dataclasses.replace(query, aggregations=list(query.aggregations) + [AggregationSpec("MIN", DOCID_COLUMN)])
        for s, c in zip(segments, capped):
            if not c:
                continue
            s.docid_view()
            r = sub.execute(probe, [s])
            items = list(r.intermediate.items())
            if len(items) >= limit:  # numGroups >= numGroupsLimit (AggregationGroupByOrderByOperator.java:111)
                st.num_groups_limit_reached = True
                items = sorted(items, key=lambda kv: kv[1][-1])
                if len(items) > limit and any(s.column(g).is_mv for g in query.group_by):
                    items = first_seen_multi_value(query, s, items, limit)
                else:
                    items = items[:limit]
            parts.append(({k: v[:-1] for k, v in items}, r.stats))
        fns = [a.function for a in query.aggregations]
        merged: Dict[tuple, list] = {}
        for inter, rs in parts:
            for k, v in inter.items():
                cur = merged.get(k)
                merged[k] = list(v) if cur is None else [_merge(fn, x, y) for fn, x, y in zip(fns, cur, v)]
            for f in ("num_docs_scanned", "num_entries_scanned_in_filter", "num_total_docs", "num_segments_processed",
                      "num_segments_matched", "kernel_ms", "sparse_sector_bytes", "dense_bytes"):
                setattr(st, f, getattr(st, f) + getattr(rs, f))
            st.filter_stats_exact = st.filter_stats_exact and rs.filter_stats_exact
            st.num_groups_limit_reached = st.num_groups_limit_reached or rs.num_groups_limit_reached
        st.num_entries_scanned_post_filter = st.num_docs_scanned * len(query.projected_columns)
        return result_from_intermediate(query, merged, st)

    def non_scan_segments(self, query: QueryContext, segments: Sequence[GpuSegment]) -> List[bool]:
        """Per segment, AggregationPlanNode.buildNonFilteredAggOperator's choice (core/plan/AggregationPlanNode.java
        :171-195): a filter that folds to match-all plus only COUNT / MIN / MAX is answered from segment metadata
        and the dictionary, with no scan (NonScanBasedAggregationOperator)."""
        q = query
        if q.group_by or q.has_filtered_aggregations or any(a.function not in ("COUNT", "MIN", "MAX", "MINMV", "MAXMV")
                                                            for a in q.aggregations):
            return [False] * len(segments)
        return [s.num_docs > 0 and SegmentFilterPlanner(s).build(q.filter).kind == "ALL" and
                all(s.min_max(a.column) is not None for a in q.aggregations if a.function != "COUNT")
                for s in segments]


@dataclass
class PendingQuery:
    """A submitted, not yet collected query (owns the libpinotgpu query handle)."""
    maker: "GpuPlanMaker"
    query: QueryContext
    num_segments: int
    handle: C.c_void_p
    layout: TableLayout
    globals_: list
    mv: Optional[tuple] = None  # (original query, lowered aggregation indexes) when *MV aggregations were lowered
    matched: Optional[np.ndarray] = None  # per-segment matched flags, filled by the wait (pgpu_query_matched_segments)
    order: Optional[object] = None  # the pgpu_topk given at submit (collect passes the same one)

    def cancel(self) -> None:
        """Stop the query (pgpu_query_cancel): its kernels skip their remaining tiles and collect raises
        QueryCancelledError."""
        if self.handle is not None and self.handle.value:
            _lib.check(self.maker.ctx._lib.pgpu_query_cancel(self.handle))

    def __del__(self):
        if self.handle is not None and self.handle.value:
            self.maker.ctx._lib.pgpu_query_release(self.handle)
            self.handle = None


def first_seen_multi_value(query: QueryContext, seg: GpuSegment, items: List[tuple], limit: int) -> List[tuple]:
    """The first `limit` group keys in the order the reference's holders give them ids when a group column is
    multi-value.  `items` = (group values, intermediate values + [first doc]) sorted by first doc.  Every doc expands
    into one key per element of the cartesian product of its group columns' values, column 0 outermost
    (DictionaryBasedGroupKeyGenerator.getIntRawKeys, :472-544), and processMultiValue (:186-199) gives each new key
    the next id until the limit: the keys first met before the doc where the limit is reached are all kept, and that
    doc's new keys are kept in its own expansion order (single-value columns are constant within a doc, so only the
    multi-value columns' value order matters)."""
    import itertools
    d_cut = items[limit - 1][1][-1]
    before = [kv for kv in items if kv[1][-1] < d_cut]
    tie = {kv[0]: kv for kv in items if kv[1][-1] == d_cut}
    need = limit - len(before)
    mv_pos = [i for i, g in enumerate(query.group_by) if seg.column(g).is_mv]
    per_col = []
    for i in mv_pos:
        g = query.group_by[i]
        d = seg.dictionaries[g]
        per_col.append([d[int(x)].item() if hasattr(d[int(x)], "item") else d[int(x)] for x in seg.mv_row(g, d_cut)])
    rank = {}
    for combo in itertools.product(*per_col):
        rank.setdefault(tuple(combo), len(rank))
    new = sorted(tie.values(), key=lambda kv: rank.get(tuple(kv[0][i] for i in mv_pos), len(rank)))
    return before + new[:need]


def result_from_intermediate(query: QueryContext, merged: Dict[tuple, list], st: ExecutionStats) -> QueryResult:
    """A GROUP BY result from merged intermediate values per group key (the first-seen paths)."""
    from .datatable import _final
    fns = [a.function for a in query.aggregations]
    ng = len(query.group_by)
    finals = [k + tuple(_final(fn, x) for fn, x in zip(fns, v)) for k, v in merged.items()]
    res = QueryResult(query=query, stats=st)
    res._intermediate = merged
    res._group_rows = sorted(finals, key=lambda r: r[:ng])  # ascending keys: ORDER BY ties as the one-launch path
    res.rows = [to_select_order(query, r) for r in order_and_limit(query, res._group_rows)]
    return res


def finish(query: QueryContext, table: GroupTable, global_dicts: Sequence, stats: ExecutionStats) -> QueryResult:
    """Decode a (merged) partial table into final results."""
    L = table.layout
    res = QueryResult(query=query, stats=stats)
    aggs = query.aggregations

    def values_of(row_cells):
        cnt = int(row_cells[0])
        fin, inter = [], []
        for ai, a in enumerate(aggs):
            sec = L.agg_section[ai]
            cell = join_parts(row_cells, sec, L.agg_sum_parts[ai], sum_exp_of(L, ai)) if sec > 0 else None
            op = L.section_op[sec]
            vt = L.agg_value_type[ai]
            fin.append(final_value(a.function, cnt, cell, op, vt))
            inter.append(intermediate_value(a.function, cnt, cell, op, vt))
        return fin, inter

    if not query.group_by:
        if len(table.keys):
            row = table.cells[0]
        else:
            row = np.zeros(L.num_sections, dtype=np.int64)
            for s in range(L.num_sections):
                op = L.section_op[s]
                row[s] = np.iinfo(np.int64).max if op == PGPU_RED_MIN_I64 else (
                    np.iinfo(np.int64).min if op == PGPU_RED_MAX_I64 else 0)
        fin, inter = values_of(row)
        res.aggregation_result = fin
        res._intermediate = {(): inter}
        res.rows = [tuple(fin)]
        return res
    cols = GroupColumns(query, table, global_dicts)
    res._columns = cols
    res.rows = [to_select_order(query, r) for r in cols.rows(cols.order_and_limit())]
    return res


def merge_non_scan(query: QueryContext, scanned: Optional[QueryResult], segments: Sequence[GpuSegment]) -> QueryResult:
    """Merge the scanned segments' result with the non-scan segments' metadata answers
    (NonScanBasedAggregationOperator.java:85-101: COUNT = total docs, MIN / MAX = dictionary min / max as double;
    statistics (numTotalDocs, 0, 0, numTotalDocs) per segment, :253-256)."""
    res = QueryResult(query=query, stats=ExecutionStats() if scanned is None else scanned.stats)
    vals = []
    for ai, a in enumerate(query.aggregations):
        v = {"COUNT": 0, "MIN": math.inf, "MAX": -math.inf, "MINMV": math.inf, "MAXMV": -math.inf}[a.function] \
            if scanned is None else scanned.aggregation_result[ai]
        for s in segments:
            if a.function == "COUNT":
                v += s.num_docs
            else:  # MIN / MAX and MINMV / MAXMV: the dictionary's ends (DICTIONARY_BASED_FUNCTIONS)
                lo, hi = s.min_max(a.column)
                v = min(v, lo) if a.function in ("MIN", "MINMV") else max(v, hi)
        vals.append(v)
    st = res.stats
    st.segment_matched = None  # the launch's per-segment flags no longer line up with the caller's segments
    for s in segments:
        st.num_docs_scanned += s.num_docs
        st.num_total_docs += s.num_docs
        st.num_segments_processed += 1
        st.num_segments_matched += int(s.num_docs > 0)  # numDocsScanned = numTotalDocs
    res.aggregation_result = vals
    res._intermediate = {(): list(vals)}
    res.rows = [to_select_order(query, tuple(vals))]
    return res


def merge_filtered(query: QueryContext, parts, results: Sequence[QueryResult]) -> QueryResult:
    """FilteredAggregationOperator.getNextBlock (core/operator/query/FilteredAggregationOperator.java:62-95):
    results placed back in aggregation order; docs scanned and entries scanned summed over every filter pass
    (the main pass included); numTotalDocs once."""
    res = QueryResult(query=query, stats=ExecutionStats())
    fin: List = [None] * len(query.aggregations)
    inter: List = [None] * len(query.aggregations)
    st = res.stats
    for (_, idx), r in zip(parts, results):
        for j, i in enumerate(idx):
            fin[i] = r.aggregation_result[j]
            inter[i] = r.intermediate[()][j]
        for f in ("num_docs_scanned", "num_entries_scanned_in_filter", "num_entries_scanned_post_filter",
                  "kernel_ms", "sparse_sector_bytes", "dense_bytes"):
            setattr(st, f, getattr(st, f) + getattr(r.stats, f))
        st.filter_stats_exact = st.filter_stats_exact and r.stats.filter_stats_exact
    st.num_total_docs = results[-1].stats.num_total_docs
    st.num_segments_processed = results[-1].stats.num_segments_processed
    # one operator per segment sums its passes' numDocsScanned: a segment matched when any pass matched in it
    flags = [r.stats.segment_matched for r in results]
    if all(f is not None and len(f) == len(flags[0]) for f in flags):
        st.segment_matched = np.bitwise_or.reduce(np.stack(flags), axis=0)
        st.num_segments_matched = int(np.count_nonzero(st.segment_matched))
    else:
        st.num_segments_matched = max(r.stats.num_segments_matched for r in results)
    res.aggregation_result = fin
    res._intermediate = {(): inter}
    res.rows = [to_select_order(query, tuple(fin))]
    return res


class GroupColumns:
    """A compacted group table decoded column-wise (numpy): group values per group column and final values per
    aggregation, so that ORDER BY / LIMIT over a million groups costs a sort, not a Python loop per group.
    Columns are decoded lazily: the ORDER BY keys over every group, everything else only for the rows asked for
    (``rows(idx)``) -- the broker reduce of a trim-free million-group table touches the rest of it once."""

    def __init__(self, query: QueryContext, table: GroupTable, global_dicts: Sequence):
        self.query = query
        self.table = table
        self.global_dicts = global_dicts
        L = table.layout
        keys = np.asarray(table.keys, dtype=np.int64)
        self._words = [keys[:, 0], keys[:, 1]] if keys.ndim == 2 else [keys]
        self._split = L.key_split if keys.ndim == 2 else len(global_dicts)
        self.count = table.cells[:, 0] if len(table.keys) else np.zeros(0, dtype=np.int64)
        self._gid_cache: Dict[int, np.ndarray] = {}
        self._final_cache: Dict[int, tuple] = {}

    def __len__(self):
        return len(self.count)

    # -- group columns --
    def _gids(self, gi: int, idx: Optional[np.ndarray]) -> np.ndarray:
        """Global dictionary ids of group column gi (mixed-radix digit of its key word)."""
        word = 0 if gi < self._split else 1
        first = 0 if word == 0 else self._split
        last = self._split if word == 0 else len(self.global_dicts)
        k = self._words[word] if idx is None else self._words[word][idx]
        if last - first == 1:
            return k  # the word is this column's id
        stride = 1
        for j in range(first, gi):
            stride *= len(self.global_dicts[j])
        return (k // stride) % len(self.global_dicts[gi])

    def value(self, gi: int, idx: Optional[np.ndarray] = None) -> np.ndarray:
        g = self.global_dicts[gi]
        arr = np.asarray(g, dtype=object) if isinstance(g, list) else np.asarray(g)
        return arr[self._gids(gi, idx)]

    @property
    def values(self) -> List[np.ndarray]:
        return [self.value(gi) for gi in range(len(self.global_dicts))]

    # -- aggregations --
    def final(self, ai: int, idx: Optional[np.ndarray] = None):
        """(final values, sums or None) of aggregation ai over every row, or over rows idx."""
        if idx is None and ai in self._final_cache:
            return self._final_cache[ai]
        L = self.table.layout
        a = self.query.aggregations[ai]
        sec = L.agg_section[ai]
        op = L.section_op[sec]
        vt = L.agg_value_type[ai]
        cells = self.table.cells if idx is None else self.table.cells[idx]
        cnt = cells[:, 0]
        cell = cells[:, sec] if sec > 0 else None
        fn = a.function
        s = None
        if fn == "COUNT":
            f = cnt.astype(np.int64)
        elif fn in ("SUM", "AVG") and L.agg_sum_parts[ai] > 1:
            # split sum: join the parts exactly (Python ints), round once to double (fixed point: times 2^exp)
            e, parts = sum_exp_of(L, ai), L.agg_sum_parts[ai]
            s = np.array([float(join_parts(r, sec, parts, e)) for r in cells], dtype=np.float64)
            f = s if fn == "SUM" else s / cnt
        elif fn in ("SUM", "AVG"):
            s = cell.astype(np.float64) if op == PGPU_RED_SUM_I64 else cell.view(np.float64)
            f = s if fn == "SUM" else s / cnt  # compacted groups have count > 0
        else:  # MIN / MAX: order-preserving keys (pgpu_decode_minmax_key)
            if vt in (PGPU_INT, PGPU_LONG):
                f = cell.astype(np.float64)
            else:
                f = np.where(cell >= 0, cell, cell ^ np.int64(0x7FFFFFFFFFFFFFFF)).view(np.float64)
        if idx is None:
            self._final_cache[ai] = (f, s)
        return f, s

    @property
    def finals(self) -> List[np.ndarray]:
        return [self.final(ai)[0] for ai in range(len(self.query.aggregations))]

    def _column(self, name: str, idx: Optional[np.ndarray] = None) -> np.ndarray:
        ng = len(self.query.group_by)
        names = list(self.query.group_by) + [a.result_name for a in self.query.aggregations]
        i = names.index(name)
        return self.value(i, idx) if i < ng else self.final(i - ng, idx)[0]

    def order_and_limit(self, limit: Optional[int] = None) -> np.ndarray:
        """Row indexes after ORDER BY / LIMIT: stable sort by each ORDER BY expression (GroupByDataTableReducer,
        IndexedTable.finish), ties kept in ascending global-key order like ``order_and_limit``.  `limit`
        overrides the query's (a combine keeping its top max(5 * limit, 5000) candidates)."""
        q = self.query
        n = len(self)
        lim = q.limit if limit is None else limit
        if not q.order_by:
            return np.arange(min(n, lim))

        def key_of(ob, idx=None):
            c = self._column(ob.expression, idx)
            if c.dtype.kind in "iuf":
                kk = c.astype(np.float64) if c.dtype.kind == "f" else c.astype(np.int64)
            else:
                kk = np.unique(c, return_inverse=True)[1].astype(np.int64)
            return kk if ob.ascending else -kk

        first = key_of(q.order_by[0])
        if n > 4 * lim > 0:
            # only rows whose primary key is at least as good as the limit-th one can be in the result
            kth = np.partition(first, lim - 1)[lim - 1]
            cand = np.flatnonzero(first <= kth)
            keys = [first[cand]] + [key_of(ob, cand) for ob in q.order_by[1:]]
            return cand[np.lexsort(keys[::-1])][: lim]
        keys = [first] + [key_of(ob) for ob in q.order_by[1:]]
        return np.lexsort(keys[::-1])[: lim]

    def rows(self, idx: Optional[np.ndarray] = None) -> List[tuple]:
        parts = [self.value(gi, idx).tolist() for gi in range(len(self.global_dicts))]
        for ai, a in enumerate(self.query.aggregations):
            f = self.final(ai, idx)[0]
            parts.append([int(x) for x in f.tolist()] if a.function == "COUNT" else f.tolist())
        return [tuple(r) for r in zip(*parts)] if parts else []

    def intermediate(self) -> dict:
        out = {}
        gv = [v.tolist() for v in self.values]
        cnt = self.count.tolist()
        cols = []
        for ai, a in enumerate(self.query.aggregations):
            f, s = self.final(ai)
            if a.function == "AVG":
                cols.append([(x, c) for x, c in zip(s.tolist(), cnt)])
            elif a.function == "COUNT":
                cols.append([int(x) for x in f.tolist()])
            else:
                cols.append(f.tolist())
        for i in range(len(cnt)):
            out[tuple(g[i] for g in gv)] = [c[i] for c in cols]
        return out


def has_mv_aggregations(query: QueryContext) -> bool:
    return any(a.function in MV_AGGS for a in query.aggregations)


def mv_lower(query: QueryContext):
    from .mv import lower
    return lower(query)


def mv_raise(query: QueryContext, parts, low_res):
    from .mv import raise_result
    return raise_result(query, parts, low_res)
