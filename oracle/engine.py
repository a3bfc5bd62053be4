"""Per-segment query execution and combine, restated on the CPU (test infrastructure; see oracle/__init__.py).

Independent of pinot_amd's planner and SQL front end: queries are parsed by oracle/sql.py (engine.execute takes
SQL text; pinot_amd QueryContexts are read through the same attribute names), predicates are evaluated on decoded
VALUES with SQL comparison semantics (not on dict ids), the physical filter tree is rebuilt here from
FilterOperatorUtils' rules, and the iterator model below reproduces numEntriesScannedInFilter.  The segments are
the reference-format bytes in pinot_amd.segment.SegmentData containers, of which only the byte fields are read.

References (abbreviations as in SURVEY.md):
  FilterPlanNode.constructPhysicalOperator ................ core/plan/FilterPlanNode.java:192-313
  FilterOperatorUtils (leaf choice, AND/OR folding, order) . core/operator/filter/FilterOperatorUtils.java:42-221
  AndDocIdSet.iterator / OrDocIdSet.iterator .............. core/operator/docidsets/AndDocIdSet.java:60-146,
                                                             OrDocIdSet.java:58-110, NotDocIdSet.java:34-37
  SVScanDocIdIterator.next/advance/applyAnd ............... core/operator/dociditerators/SVScanDocIdIterator.java:57-94
  AndDocIdIterator / OrDocIdIterator / NotDocIdIterator ... core/operator/dociditerators/*.java
  Sum/Count/Min/Max/AvgAggregationFunction ................ core/query/aggregation/function/*.java
  multi-value: MVScanDocIdIterator (entries += row length) . core/operator/dociditerators/MVScanDocIdIterator.java:56-100
               BaseDictionaryBasedPredicateEvaluator.applyMV core/operator/filter/predicate/
                 (any value for inclusive, every value for exclusive)   BaseDictionaryBasedPredicateEvaluator.java:133-149
               Count/Sum/Min/Max/AvgMVAggregationFunction . core/query/aggregation/function/*MVAggregationFunction.java
  DictionaryBasedGroupKeyGenerator (holders, limit) ........ core/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:100-1016
  AggregationOperator / AggregationGroupByOrderByOperator stats core/operator/query/AggregationOperator.java:58-87
  combine + broker reduce (merge, ORDER BY, LIMIT) ........ core/operator/combine/*.java, core/data/table/IndexedTable.java:103-156
"""
from __future__ import annotations

import bisect
import math
import struct
from dataclasses import dataclass, field
from fractions import Fraction
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from pinot_amd._lib import PGPU_DOUBLE, PGPU_FLOAT, PGPU_INT, PGPU_LONG, PGPU_STRING
from pinot_amd.segment import SegmentData

from .sql import UNBOUNDED, Pred as Predicate, parse as parse_sql, split_filtered

FilterContext = QueryContext = object  # duck-typed: oracle.sql structures or pinot_amd.query ones

from .rawfwd import read_raw_forward
from .segment_writer import NATIVE, read_inverted_bitmap, read_mv_forward, unpack_fixed_bit

MV_FUNCTIONS = {"COUNTMV": "COUNT", "SUMMV": "SUM", "MINMV": "MIN", "MAXMV": "MAX", "AVGMV": "AVG"}

EOF = -(2 ** 31)  # Constants.EOF = Integer.MIN_VALUE


# ---- decoded segment ------------------------------------------------------------------------------------------
_BIG_DICTS: Dict[int, tuple] = {}  # id(bytes) -> (the bytes, decoded values): the last decoded >= 16M-entry dictionary


class DecodedSegment:
    """Dict ids / values of a SegmentData decoded from its reference-format bytes."""

    def __init__(self, seg: SegmentData):
        self.seg = seg
        self.name = seg.name
        self.num_docs = seg.num_docs
        self._ids: Dict[str, np.ndarray] = {}
        self._dict: Dict[str, object] = {}

    def dictionary(self, col: str):
        d = self._dict.get(col)
        if d is None:
            c = self.seg.column(col)
            if c.data_type == PGPU_STRING:
                d = list(c.dictionary)
            else:
                hit = _BIG_DICTS.get(id(c.dictionary))
                if hit is not None and hit[0] is c.dictionary:
                    d = hit[1]
                else:
                    be = {PGPU_INT: ">i4", PGPU_LONG: ">i8", PGPU_FLOAT: ">f4", PGPU_DOUBLE: ">f8"}[c.data_type]
                    d = np.frombuffer(c.dictionary, dtype=be).astype(NATIVE[c.data_type])
                    if len(d) >= (1 << 24):  # decoded once for every segment / query sharing the same bytes
                        _BIG_DICTS.clear()
                        _BIG_DICTS[id(c.dictionary)] = (c.dictionary, d)
            self._dict[col] = d
        return d

    def ids(self, col: str) -> np.ndarray:
        a = self._ids.get(col)
        if a is None:
            c = self.seg.column(col)
            if c.sorted_index is not None:
                pairs = np.frombuffer(c.sorted_index, dtype=">i4").reshape(-1, 2)
                a = np.repeat(np.arange(len(pairs)), pairs[:, 1] - pairs[:, 0] + 1)
            else:
                bits = 1 if c.cardinality - 1 <= 1 else int(c.cardinality - 1).bit_length()
                a = unpack_fixed_bit(c.forward, bits, self.num_docs)
            assert len(a) == self.num_docs
            self._ids[col] = a
        return a

    def mv(self, col: str):
        """(offsets[num_docs + 1], dict ids of every value) of a multi-value column."""
        a = self._ids.get(("mv", col))
        if a is None:
            c = self.seg.column(col)
            a = read_mv_forward(c.mv_forward, self.num_docs, c.num_values, _bits(c.cardinality))
            self._ids[("mv", col)] = a
        return a

    def raw_values(self, col: str) -> np.ndarray:
        """A raw (no-dictionary) column's values by doc id (FixedByteChunkSVForwardIndexReader)."""
        a = self._ids.get(("raw", col))
        if a is None:
            c = self.seg.column(col)
            a = read_raw_forward(c.raw_forward, c.data_type, self.num_docs)
            self._ids[("raw", col)] = a
        return a

    def values(self, col: str):
        if self.seg.column(col).raw_forward is not None:
            return self.raw_values(col)
        d = self.dictionary(col)
        ids = self.ids(col)
        if isinstance(d, list):
            return [d[i] for i in ids]
        return d[ids]


# ---- predicates on values (SQL semantics) -----------------------------------------------------------------------
def _bits(cardinality: int) -> int:
    """PinotDataBitSet.getNumBitsPerValue(cardinality - 1)."""
    return 1 if cardinality - 1 <= 1 else int(cardinality - 1).bit_length()


def _lit(v: str, dt: int):
    if dt == PGPU_STRING:
        return v
    if dt in (PGPU_INT, PGPU_LONG):
        return Fraction(v)
    if dt == PGPU_FLOAT:
        return float(np.float32(float(v)))
    return float(v)


def _padder(pad_char: str, width: int):
    """BaseImmutableDictionary.padString (seglocal/segment/index/readers/BaseImmutableDictionary.java:272-285):
    segments written with a non-zero padding character (legacy '%') compare padded values."""
    if pad_char == "\0" or width <= 0:
        return None
    pb = pad_char.encode("utf-8")[:1]

    def pad(v: str) -> str:
        b = v.encode("utf-8")
        return (b + pb * (width - len(b))).decode("utf-8") if len(b) < width else v
    return pad


def _truth_on_dictionary(d, dt: int, p: Predicate, pad=None) -> np.ndarray:
    """Predicate truth per dictionary value, with SQL comparison semantics on the value (on padded values and
    literals for legacy-padded STRING dictionaries, `pad`)."""
    if dt == PGPU_STRING:
        vals = list(d)
        if pad is not None:
            vals = [pad(v) for v in vals]
            p = Predicate(p.type, p.column, tuple(pad(x) for x in p.values),
                          lower=p.lower if p.lower == UNBOUNDED else pad(p.lower),
                          upper=p.upper if p.upper == UNBOUNDED else pad(p.upper),
                          lower_inclusive=p.lower_inclusive, upper_inclusive=p.upper_inclusive)

        def ok(v):
            if p.type == "EQ":
                return v == p.values[0]
            if p.type == "NOT_EQ":
                return v != p.values[0]
            if p.type == "IN":
                return v in p.values
            if p.type == "NOT_IN":
                return v not in p.values
            r = True
            if p.lower != UNBOUNDED:
                r &= v >= p.lower if p.lower_inclusive else v > p.lower
            if p.upper != UNBOUNDED:
                r &= v <= p.upper if p.upper_inclusive else v < p.upper
            return r

        return np.fromiter((ok(v) for v in vals), dtype=bool, count=len(vals))
    v = np.asarray(d)
    if dt in (PGPU_INT, PGPU_LONG):
        # An integer dictionary is strictly ascending (BaseImmutableDictionary; SegmentDictionaryCreator sorts and
        # dedups), so each comparison with an integer threshold holds on one prefix or suffix of it: found by
        # binary search (insertionIndexOf), the same truth per value as comparing every entry, without a pass
        # over dictionaries of up to 2^30 values.
        n = len(v)
        tmin, tmax = (-(1 << 31), (1 << 31) - 1) if v.dtype.itemsize == 4 else (-(1 << 63), (1 << 63) - 1)

        def count_lt(x: int) -> int:  # entries < x, for any Python int
            if x <= tmin:
                return 0
            if x > tmax:
                return n
            return int(np.searchsorted(v, np.array(x, dtype=v.dtype), side="left"))  # no whole-array cast

        def prefix(k: int) -> np.ndarray:
            m = np.zeros(n, dtype=bool)
            m[:k] = True
            return m

        def eq(lit):
            f = Fraction(lit)
            m = np.zeros(n, dtype=bool)
            if f.denominator == 1:
                i = count_lt(int(f))
                if i < n and int(v[i]) == int(f):
                    m[i] = True
            return m

        def ge(lit, inclusive):  # v >= lit  /  v > lit
            f = Fraction(lit)
            return ~prefix(count_lt(math.ceil(f) if inclusive else math.floor(f) + 1))

        def le(lit, inclusive):  # v <= lit  /  v < lit
            f = Fraction(lit)
            return prefix(count_lt(math.floor(f) + 1 if inclusive else math.ceil(f)))
    else:
        v = v.astype(np.float64)
        cast = (lambda x: float(np.float32(float(x)))) if dt == PGPU_FLOAT else float

        def eq(lit):
            return v == cast(lit)

        def ge(lit, inclusive):
            return v >= cast(lit) if inclusive else v > cast(lit)

        def le(lit, inclusive):
            return v <= cast(lit) if inclusive else v < cast(lit)
    if p.type == "EQ":
        return eq(p.values[0])
    if p.type == "NOT_EQ":
        return ~eq(p.values[0])
    if p.type in ("IN", "NOT_IN"):
        m = np.zeros(len(v), dtype=bool)
        for x in p.values:
            m |= eq(x)
        return m if p.type == "IN" else ~m
    m = np.ones(len(v), dtype=bool)
    if p.lower != UNBOUNDED:
        m &= ge(p.lower, p.lower_inclusive)
    if p.upper != UNBOUNDED:
        m &= le(p.upper, p.upper_inclusive)
    return m


# ---- raw-value predicates (no dictionary) --------------------------------------------------------------------------
_IRANGE = {PGPU_INT: (-(1 << 31), (1 << 31) - 1), PGPU_LONG: (-(1 << 63), (1 << 63) - 1)}


def _raw_literal(v: str, dt: int):
    """Integer.parseInt / Long.parseLong / Float.parseFloat / Double.parseDouble of a literal (ValueError where the
    reference throws NumberFormatException)."""
    if dt in (PGPU_INT, PGPU_LONG):
        body = v[1:] if v[:1] in "+-" else v
        if not (body.isascii() and body.isdigit()):
            raise ValueError(f"NumberFormatException: {v!r}")
        x = int(v)
        if not _IRANGE[dt][0] <= x <= _IRANGE[dt][1]:
            raise ValueError(f"NumberFormatException: {v!r}")
        return x
    t = v.strip()
    core = t.lstrip("+-")
    if core in ("NaN", "Infinity"):
        x = float(t.replace("Infinity", "inf"))
    else:
        if not core or any(ch.isalpha() and ch not in "eEfFdD" for ch in core):
            raise ValueError(f"NumberFormatException: {v!r}")
        x = float(t.rstrip("fFdD"))
    return float(np.float32(x)) if dt == PGPU_FLOAT else x


def _fp_ordinal_key(a: np.ndarray) -> np.ndarray:
    """FPOrdering.ordinalOf order (segment-local/utils/FPOrdering.java): NaN and -inf lowest, -0 == 0."""
    a = np.asarray(a, dtype=np.float64)
    return np.where(np.isnan(a), -np.inf, a) + 0.0  # + 0.0 turns -0.0 into 0.0


def raw_predicate_mask(ds: DecodedSegment, p: Predicate, range_index: bool) -> np.ndarray:
    """Per doc: the raw-value evaluator's applySV (RangePredicateEvaluatorFactory.java:62-110 + the Int/Long/Float/
    DoubleRawValueBasedRangePredicateEvaluator classes; Equals / NotEquals / In / NotIn raw evaluators with
    fastutil sets: float members equal by their bits).  range_index: RangeIndexBasedFilterOperator's evaluation --
    the evaluator's bounds inclusive whatever the flags (RangeIndexBasedFilterOperator.java:165-290), floats
    compared by FPOrdering ordinals."""
    c = ds.seg.column(p.column)
    dt = c.data_type
    v = ds.raw_values(p.column)
    fp = dt in (PGPU_FLOAT, PGPU_DOUBLE)
    if p.type == "RANGE":
        lu, uu = p.lower == UNBOUNDED, p.upper == UNBOUNDED
        ext = _IRANGE[dt] if not fp else (-math.inf, math.inf)
        lo = ext[0] if lu else _raw_literal(p.lower, dt)
        hi = ext[1] if uu else _raw_literal(p.upper, dt)
        li = lu or p.lower_inclusive or range_index
        hi_i = uu or p.upper_inclusive or range_index
        x = v.astype(np.float64) if fp else v.astype(np.int64)
        if fp and range_index:
            x = _fp_ordinal_key(x)
            lo, hi = float(_fp_ordinal_key(np.array([lo]))[0]), float(_fp_ordinal_key(np.array([hi]))[0])
        m = (x >= lo) if li else (x > lo)
        m &= (x <= hi) if hi_i else (x < hi)
        return m
    lits = [_raw_literal(x, dt) for x in p.values]
    if fp:
        bits = v.astype(np.float64).view(np.int64)
        want = np.array(lits, dtype=np.float64).view(np.int64)
        m = np.isin(bits, want)
    else:
        m = np.isin(v.astype(np.int64), np.array(lits, dtype=np.int64))
    return ~m if p.type in ("NOT_EQ", "NOT_IN") else m


def predicate_mask(ds: DecodedSegment, p: Predicate) -> np.ndarray:
    """Boolean per doc: does the doc's value satisfy the predicate (truth per dictionary value, gathered by the
    doc's dict id — value semantics, since the dictionary holds the values)."""
    c = ds.seg.column(p.column)
    pad = _padder(c.pad_char, c.entry_width) if c.data_type == PGPU_STRING else None
    truth = _truth_on_dictionary(ds.dictionary(p.column), c.data_type, p, pad)
    if c.mv_forward is not None:
        # applyMV: an inclusive predicate matches a row holding any matching value, an exclusive one a row whose
        # every value passes (no excluded value) -- rows are never empty
        off, ids = ds.mv(p.column)
        t = truth[ids].astype(np.int8)
        red = np.minimum.reduceat(t, off[:-1]) if p.is_exclusive else np.maximum.reduceat(t, off[:-1])
        return red.astype(bool)
    return truth[ds.ids(p.column)]


# ---- physical operator tree (restated FilterOperatorUtils) ------------------------------------------------------
@dataclass
class POp:
    kind: str                 # EMPTY ALL SCAN RAW_SCAN BITMAP SORTED RANGE_INDEX AND OR NOT
    children: List["POp"] = field(default_factory=list)
    mask: Optional[np.ndarray] = None   # leaf doc set
    weights: Optional[np.ndarray] = None  # multi-value scan: entries read per doc (row lengths)

    def priority(self) -> int:
        return {"SORTED": 0, "BITMAP": 1, "RANGE_INDEX": 2, "AND": 3, "OR": 4, "SCAN": 5,
                "RAW_SCAN": 5}.get(self.kind) if self.kind != "NOT" \
            else self.children[0].priority()


def build_physical(ds: DecodedSegment, f: Optional[FilterContext]) -> POp:
    if f is None:
        return POp("ALL")
    if f.type in ("AND", "OR"):
        kids = []
        for ch in f.children:
            op = build_physical(ds, ch)
            if f.type == "AND":
                if op.kind == "EMPTY":
                    return POp("EMPTY")
                if op.kind != "ALL":
                    kids.append(op)
            else:
                if op.kind == "ALL":
                    return POp("ALL")
                if op.kind != "EMPTY":
                    kids.append(op)
        if not kids:
            return POp("ALL" if f.type == "AND" else "EMPTY")
        if len(kids) == 1:
            return kids[0]
        if f.type == "AND":
            kids = sorted(kids, key=lambda o: o.priority())
        return POp(f.type, kids)
    if f.type == "NOT":
        ch = build_physical(ds, f.children[0])
        if ch.kind == "ALL":
            return POp("EMPTY")
        if ch.kind == "EMPTY":
            return POp("ALL")
        return POp("NOT", [ch])
    p = f.predicate
    col = ds.seg.column(p.column)
    if col.raw_forward is not None:
        # no dictionary: no always-true / -false folding, no sorted / inverted index (FilterOperatorUtils.java:42-81)
        ri = p.type == "RANGE" and col.range_index is not None
        return POp("RANGE_INDEX" if ri else "RAW_SCAN", mask=raw_predicate_mask(ds, p, ri))
    m = predicate_mask(ds, p)
    # alwaysTrue / alwaysFalse are decided on the dictionary (every dict value matches / none does)
    d = ds.dictionary(p.column)
    pad = _padder(col.pad_char, col.entry_width) if col.data_type == PGPU_STRING else None
    truth_card = int(np.count_nonzero(_truth_on_dictionary(d, col.data_type, p, pad)))
    if truth_card == 0:
        return POp("EMPTY")
    if truth_card == len(d):
        return POp("ALL")
    if col.sorted_index is not None:
        return POp("SORTED", mask=m)
    if p.type == "RANGE" and col.range_index is not None:  # exact dict-id range of the range index
        return POp("RANGE_INDEX", mask=m)
    if p.type != "RANGE" and col.inverted is not None:
        # the inverted index is read through its own bytes: checks the Roaring writer too
        inv_mask = np.zeros(ds.num_docs, dtype=bool)
        if col.mv_forward is not None:  # getMatchingDictIds / getNonMatchingDictIds of the dictionary
            tr = _truth_on_dictionary(d, col.data_type, p, pad)
            matching = np.flatnonzero(~tr if p.is_exclusive else tr)
        else:
            ids = ds.ids(p.column)
            matching = np.unique(ids[m]) if not p.is_exclusive else np.unique(ids[~m])
        for i in matching:
            inv_mask[read_inverted_bitmap(col.inverted, col.cardinality, int(i))] = True
        if p.is_exclusive:
            inv_mask = ~inv_mask
        assert np.array_equal(inv_mask, m), "inverted index disagrees with forward index"
        return POp("BITMAP", mask=m)
    if col.mv_forward is not None:
        return POp("SCAN", mask=m, weights=np.diff(ds.mv(p.column)[0]))
    return POp("SCAN", mask=m)


def eval_mask(op: POp, n: int) -> np.ndarray:
    if op.kind == "ALL":
        return np.ones(n, dtype=bool)
    if op.kind == "EMPTY":
        return np.zeros(n, dtype=bool)
    if op.mask is not None:
        return op.mask
    if op.kind == "AND":
        m = np.ones(n, dtype=bool)
        for c in op.children:
            m &= eval_mask(c, n)
        return m
    if op.kind == "OR":
        m = np.zeros(n, dtype=bool)
        for c in op.children:
            m |= eval_mask(c, n)
        return m
    return ~eval_mask(op.children[0], n)


# ---- iterator model (numEntriesScannedInFilter) ------------------------------------------------------------------
class _Scan:
    kind = "scan"

    def __init__(self, mask: np.ndarray, counter: list, weights: Optional[np.ndarray] = None):
        self.n = len(mask)
        self.hits = np.flatnonzero(mask)
        self.mask = mask
        self.nxt = 0
        self.counter = counter
        self.weights = weights  # MVScanDocIdIterator: a doc read costs its row length
        self.cum = None if weights is None else np.concatenate([[0], np.cumsum(weights)])

    def _read(self, a: int, b: int) -> None:
        """docs [a, b) read."""
        self.counter[0] += (b - a) if self.cum is None else int(self.cum[b] - self.cum[a])

    def next(self):
        if self.nxt >= self.n:
            return EOF
        i = bisect.bisect_left(self.hits, self.nxt)
        if i < len(self.hits):
            d = int(self.hits[i])
            self._read(self.nxt, d + 1)
            self.nxt = d + 1
            return d
        self._read(self.nxt, self.n)
        self.nxt = self.n
        return EOF

    def advance(self, t):
        self.nxt = t
        return self.next()

    def apply_and(self, docs: np.ndarray) -> np.ndarray:
        self.counter[0] += len(docs) if self.weights is None else int(self.weights[docs].sum())
        return docs[self.mask[docs]]


class _Docs:
    """BitmapDocIdIterator / RangelessBitmapDocIdIterator / SortedDocIdIterator over a doc array."""

    def __init__(self, docs: np.ndarray, kind: str):
        self.docs = docs
        self.i = 0
        self.kind = kind  # "bitmap" or "sorted"

    def next(self):
        if self.i < len(self.docs):
            self.i += 1
            return int(self.docs[self.i - 1])
        return EOF

    def advance(self, t):
        self.i = bisect.bisect_left(self.docs, t, self.i)
        return self.next()


class _And:
    kind = "other"

    def __init__(self, its):
        self.its = its
        self.nxt = 0

    def next(self):
        mx, mi, i = self.nxt, -1, 0
        while i < len(self.its):
            if i == mi:
                i += 1
                continue
            d = self.its[i].advance(mx)
            if d == EOF:
                return EOF
            if d == mx:
                i += 1
            else:
                mx, mi, i = d, i, 0
        self.nxt = mx + 1
        return mx

    def advance(self, t):
        self.nxt = t
        return self.next()


class _Or:
    kind = "other"

    def __init__(self, its):
        self.its = list(its)
        self.nd = [-1] * len(its)
        self.k = len(its)
        self.prev = -1

    def _drop(self):
        i = 0
        while i < self.k:
            if self.nd[i] == EOF:
                self.k -= 1
                self.its[i] = self.its[self.k]
                self.nd[i] = self.nd[self.k]
            else:
                i += 1

    def next(self):
        best, ex = None, False
        for i in range(self.k):
            d = self.nd[i]
            if d == self.prev:
                d = self.its[i].next()
                self.nd[i] = d
                if d == EOF:
                    ex = True
                    continue
            best = d if best is None else min(best, d)
        if ex:
            self._drop()
        if best is None:
            return EOF
        self.prev = best
        return best

    def advance(self, t):
        best, ex = None, False
        for i in range(self.k):
            d = self.nd[i]
            if d < t:
                d = self.its[i].advance(t)
                self.nd[i] = d
                if d == EOF:
                    ex = True
                    continue
            best = d if best is None else min(best, d)
        if ex:
            self._drop()
        if best is None:
            return EOF
        self.prev = best
        return best


class _Not:
    kind = "other"

    def __init__(self, child, n):
        self.child = child
        self.n = n
        self.nxt = 0
        d = child.next()
        self.nnm = n if d == EOF else d

    def next(self):
        while self.nxt == self.nnm:
            self.nxt += 1
            d = self.child.next()
            self.nnm = self.n if d == EOF else d
        if self.nxt >= self.n:
            return EOF
        self.nxt += 1
        return self.nxt - 1

    def advance(self, t):
        self.nxt = t
        if t > self.nnm:
            d = self.child.advance(t)
            self.nnm = self.n if d == EOF else d
        return self.next()


def make_iterator(op: POp, n: int, counter: list):
    """FilterBlockDocIdSet.iterator() of the physical operator `op`."""
    if op.kind in ("SCAN", "RAW_SCAN"):
        return _Scan(op.mask, counter, op.weights)
    if op.kind in ("BITMAP", "RANGE_INDEX"):  # RangeIndexBasedFilterOperator: a BitmapDocIdSet
        return _Docs(np.flatnonzero(op.mask), "bitmap")
    if op.kind == "SORTED":
        return _Docs(np.flatnonzero(op.mask), "sorted")
    if op.kind == "ALL":
        return _Docs(np.arange(n), "other")
    if op.kind == "EMPTY":
        return _Docs(np.zeros(0, np.int64), "other")
    if op.kind == "NOT":
        return _Not(make_iterator(op.children[0], n, counter), n)
    its = [make_iterator(c, n, counter) for c in op.children]
    idx = [i for i in its if getattr(i, "kind", "") in ("sorted", "bitmap")]
    scans = [i for i in its if getattr(i, "kind", "") == "scan"]
    rest = [i for i in its if i not in idx and i not in scans]
    if op.kind == "AND":
        if (idx and scans) or len(idx) > 1:
            docs = None
            for it in idx:
                docs = it.docs if docs is None else np.intersect1d(docs, it.docs, assume_unique=True)
            for s in scans:
                docs = s.apply_and(docs)
            merged = _Docs(docs, "bitmap")  # RangelessBitmapDocIdIterator is bitmap-based
            return merged if not rest else _And([merged] + rest)
        return _And(its)
    # OR
    if len(idx) > 1:
        docs = np.unique(np.concatenate([i.docs for i in idx]))
        merged = _Docs(docs, "bitmap")
        rest = [i for i in its if i not in idx]
        return merged if not rest else _Or([merged] + rest)
    return _Or(its)


def entries_scanned_in_filter(op: POp, n: int) -> Tuple[int, np.ndarray]:
    """Drain the iterator like DocIdSetOperator; returns (numEntriesScannedInFilter, matched doc ids)."""
    counter = [0]
    it = make_iterator(op, n, counter)
    out = []
    while True:
        d = it.next()
        if d == EOF:
            break
        out.append(d)
    return counter[0], np.asarray(out, dtype=np.int64)


# ---- aggregation -------------------------------------------------------------------------------------------------
def _as_float_values(ds: DecodedSegment, col: str, docs: np.ndarray, fn: str = "") -> np.ndarray:
    c = ds.seg.column(col)
    if (c.mv_forward is not None) != (fn in MV_FUNCTIONS):
        raise ValueError(f"{fn} on {'a multi' if c.mv_forward is not None else 'a single'}-value column {col}")
    if c.mv_forward is not None:
        # the docs' values in doc order, each row's in its stored order (getDictIdMV then the dictionary)
        off, ids = ds.mv(col)
        if len(docs) == 0:
            sel = np.zeros(0, dtype=np.int64)
        else:
            lens = off[docs + 1] - off[docs]
            sel = np.repeat(off[docs] - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
        return ds.dictionary(col)[ids[sel]]
    if c.raw_forward is not None:
        return ds.raw_values(col)[docs]
    d = ds.dictionary(col)
    if isinstance(d, list):
        raise ValueError(f"non-numeric column {col}")
    return d[ds.ids(col)[docs]]


def _sum_reference(vals: np.ndarray) -> float:
    """`sum += values[i]` in doc order starting from 0.0 (SumAggregationFunction.aggregate)."""
    if vals.size == 0:
        return 0.0
    if vals.dtype.kind in "iu":
        exact = int(vals.astype(np.int64).sum(dtype=np.int64)) if vals.size < (1 << 31) else int(sum(map(int, vals)))
        if abs(exact) < (1 << 53) and float(np.abs(vals).max()) * vals.size < 2.0 ** 53:
            return float(exact)  # every partial sum is an exact double
    return float(np.cumsum(vals.astype(np.float64))[-1])


def aggregate(fn: str, vals: Optional[np.ndarray], count: int):
    """Intermediate result of one aggregation over the matching docs of one segment (the *MV functions over the
    docs' values: COUNTMV counts values, AVGMV divides by the value count)."""
    if fn in MV_FUNCTIONS:
        return aggregate(MV_FUNCTIONS[fn], vals, len(vals))
    if fn == "COUNT":
        return count
    if fn == "SUM":
        return _sum_reference(vals)
    if fn == "MIN":
        return float(vals.astype(np.float64).min()) if count else math.inf
    if fn == "MAX":
        return float(vals.astype(np.float64).max()) if count else -math.inf
    if fn == "AVG":
        return (_sum_reference(vals), count)
    raise ValueError(fn)


def merge(fn: str, a, b):
    """AggregationFunction.merge."""
    fn = MV_FUNCTIONS.get(fn, fn)
    if fn in ("COUNT", "SUM"):
        return a + b
    if fn == "MIN":
        return min(a, b)
    if fn == "MAX":
        return max(a, b)
    return (a[0] + b[0], a[1] + b[1])


def final(fn: str, v):
    """AggregationFunction.extractFinalResult."""
    fn = MV_FUNCTIONS.get(fn, fn)
    if fn == "AVG":
        return -math.inf if v[1] == 0 else v[0] / v[1]
    if fn == "COUNT":
        return int(v)
    return float(v)


def fits_non_scan(query: QueryContext, num_docs: int, seg: Optional[SegmentData] = None) -> bool:
    """AggregationPlanNode.isFitForNonScanBasedPlan (core/plan/AggregationPlanNode.java:234-262) for the functions
    this path serves: aggregation-only, no FILTER clauses, only COUNT / MIN / MAX (dictionary-encoded columns).
    Empty segments are left to the scan plan (their dictionaries hold no min / max)."""
    if (query.group_by or query.has_filtered_aggregations or num_docs <= 0
            or any(a.function not in ("COUNT", "MIN", "MAX", "MINMV", "MAXMV") for a in query.aggregations)):
        return False
    # raw columns: MIN / MAX come from the column metadata's min / max values, when it has them (METADATA_BASED_FUNCTIONS)
    return seg is None or all(seg.column(a.column).raw_forward is None or
                              (seg.column(a.column).min_value is not None and seg.column(a.column).max_value is not None)
                              for a in query.aggregations if a.function != "COUNT")


@dataclass
class SegmentResult:
    aggregation: Optional[list] = None               # intermediate values (aggregation only)
    groups: Optional[Dict[tuple, list]] = None       # group values -> intermediate values
    num_docs_scanned: int = 0
    num_entries_scanned_in_filter: int = 0
    num_entries_scanned_post_filter: int = 0
    num_total_docs: int = 0
    matched: Optional[np.ndarray] = None
    num_groups: int = 0                              # GroupByExecutor.getNumGroups (group-by only)


def execute_segment(query: QueryContext, seg: SegmentData, num_groups_limit: int = 100_000,
                    max_init_group_holder_capacity: int = 10_000, iterator_stats: bool = False) -> SegmentResult:
    ds = seg if isinstance(seg, DecodedSegment) else DecodedSegment(seg)
    n = ds.num_docs
    op = build_physical(ds, query.filter)
    if op.kind == "ALL" and fits_non_scan(query, n, ds.seg):
        # NonScanBasedAggregationOperator (core/operator/query/NonScanBasedAggregationOperator.java:85-101,253-256):
        # COUNT from metadata, MIN / MAX from the dictionary's first / last value; stats (total, 0, 0, total)
        agg = []
        for a in query.aggregations:
            if a.function == "COUNT":
                agg.append(n)
            elif ds.seg.column(a.column).raw_forward is not None:
                c = ds.seg.column(a.column)
                agg.append(float(c.min_value if a.function == "MIN" else c.max_value))
            else:
                d = ds.dictionary(a.column)
                agg.append(float(d[0] if a.function in ("MIN", "MINMV") else d[-1]))
        return SegmentResult(aggregation=agg, num_docs_scanned=n, num_total_docs=n)
    mask = eval_mask(op, n)
    docs = np.flatnonzero(mask)
    res = SegmentResult(num_docs_scanned=len(docs), num_total_docs=n, matched=docs)
    if iterator_stats:
        res.num_entries_scanned_in_filter, it_docs = entries_scanned_in_filter(op, n)
        assert np.array_equal(it_docs, docs), "iterator model disagrees with the mask algebra"
    res.num_entries_scanned_post_filter = len(docs) * len(query.projected_columns)
    if not query.group_by:
        res.aggregation = [aggregate(a.function, None if a.column is None else
                                     _as_float_values(ds, a.column, docs, a.function), len(docs))
                           for a in query.aggregations]
        return res
    if any(ds.seg.column(g).mv_forward is not None for g in query.group_by):
        res.groups = _group_multi_value(query, ds, docs, num_groups_limit, max_init_group_holder_capacity)
        res.num_groups = len(res.groups)
        return res
    # group keys: the tuple of dict ids (raw key = sum_j dictId_j * prod_{k<j} card_k when it fits a long); a raw
    # (no-dictionary) group column keys by value (_raw_group_ids)
    gsrc = [_raw_group_ids(ds, g) if ds.seg.column(g).raw_forward is not None else (ds.ids(g), ds.dictionary(g))
            for g in query.group_by]
    cards = [len(d) for _, d in gsrc]
    prod = 1
    for c in cards:
        prod *= c
    # NoDictionarySingleColumnGroupKeyGenerator / NoDictionaryMultiColumnGroupKeyGenerator (any raw group column):
    # a value -> id map capped at numGroupsLimit whatever the key space (:199-235 / :295-330)
    no_dict = any(ds.seg.column(g).raw_forward is not None for g in query.group_by)
    idmat = np.stack([ids[docs].astype(np.int64) for ids, _ in gsrc], axis=1) if len(docs) else \
        np.zeros((0, len(cards)), dtype=np.int64)
    uniq, first, inv = (np.unique(idmat, axis=0, return_index=True, return_inverse=True) if len(docs)
                        else (np.zeros((0, len(cards)), np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64)))
    inv = np.asarray(inv).reshape(-1)
    keep_groups = np.ones(len(uniq), dtype=bool)
    if (no_dict or prod > max_init_group_holder_capacity) and len(uniq) > num_groups_limit:
        # map-based holder: only the first `limit` distinct keys (in doc order) get group ids
        keep_groups[:] = False
        keep_groups[np.argsort(first, kind="stable")[:num_groups_limit]] = True
    # the holder's key count: every distinct key (array-based) or at most the limit (map-based)
    res.num_groups = int(np.count_nonzero(keep_groups))
    order = np.argsort(inv, kind="stable")  # stable: docs stay in doc order inside each group
    inv_s, docs_s = inv[order], docs[order]
    bounds = np.flatnonzero(np.diff(inv_s)) + 1
    groups: Dict[tuple, list] = {}
    dicts = [d for _, d in gsrc]
    for part_docs, part_g in zip(np.split(docs_s, bounds), np.split(inv_s, bounds)):
        if part_docs.size == 0 or not keep_groups[part_g[0]]:
            continue
        vals = []
        for j, d in enumerate(dicts):
            v = d[int(uniq[part_g[0], j])]
            v = v.item() if hasattr(v, "item") else v
            vals.append(JavaFloatKey(v) if isinstance(v, float) else v)
        groups[tuple(vals)] = [aggregate(a.function, None if a.column is None else
                                         _as_float_values(ds, a.column, part_docs, a.function), len(part_docs))
                               for a in query.aggregations]
    res.groups = groups
    return res


def float_bits_key(v: np.ndarray) -> np.ndarray:
    """Java's map key of FLOAT / DOUBLE values -- Float.floatToIntBits / Double.doubleToLongBits (one NaN; -0.0 and
    0.0 apart) -- as an order-preserving int64 (Float.compare order)."""
    if v.dtype == np.float32:
        b = v.view(np.int32).astype(np.int64)
        b = np.where(np.isnan(v), np.int64(0x7FC00000), b)
        return np.where(b >= 0, b, b ^ np.int64(0x7FFFFFFF))
    b = v.view(np.int64)
    b = np.where(np.isnan(v), np.int64(0x7FF8000000000000), b)
    return np.where(b >= 0, b, b ^ np.int64(0x7FFFFFFFFFFFFFFF))


class JavaFloatKey(float):
    """A FLOAT / DOUBLE group value compared as the broker's group keys are (Float.equals / Double.equals: by
    floatToIntBits / doubleToLongBits, so -0.0 != 0.0 and NaN == NaN), so that Python dicts keep -0.0 and 0.0 as two
    groups and merge NaNs.  Hashes agree with plain floats' (NaN: one constant)."""

    def _bits(self):
        return b"nan" if math.isnan(self) else struct.pack(">d", self)

    def __eq__(self, other):
        return isinstance(other, float) and JavaFloatKey._bits(self) == JavaFloatKey._bits(other)

    def __ne__(self, other):
        return not self.__eq__(other)

    def __hash__(self):
        return 0x7FF8 if math.isnan(self) else hash(float(self))


def _raw_group_ids(ds: DecodedSegment, col: str):
    """Per doc an id of its value among the segment's distinct values of a raw column, and those values ascending:
    the keys of NoDictionary*GroupKeyGenerator's value -> id maps (Int2Int / Long2Int / Float2Int / Double2Int
    OpenHashMap: INT / LONG by value, FLOAT / DOUBLE by floatToIntBits / doubleToLongBits)."""
    v = ds.raw_values(col)
    keys = float_bits_key(v) if v.dtype.kind == "f" else v.astype(np.int64)
    uniq, first, inv = np.unique(keys, return_index=True, return_inverse=True)
    return np.asarray(inv).reshape(-1), v[first]


def _group_multi_value(query: QueryContext, ds: DecodedSegment, docs: np.ndarray, num_groups_limit: int,
                       max_init_group_holder_capacity: int) -> Dict[tuple, list]:
    """GROUP BY with multi-value group columns: every matched doc contributes to one group per element of the
    cartesian product of its group columns' values (duplicates within a row kept), in the order
    DictionaryBasedGroupKeyGenerator.getIntRawKeys builds them (columns from last to first, a multi-value column's
    values outermost: DictionaryBasedGroupKeyGenerator.java:472-544); the holders' processMultiValue
    (:325-336, :417-431, :616-630) assign group ids first-seen in that order, and each aggregation's
    aggregateGroupByMV adds the doc's value(s) once per key (e.g. SumAggregationFunction.java:105-114)."""
    cols = list(query.group_by)
    src = []
    for g in cols:
        if ds.seg.column(g).mv_forward is not None:
            off, ids = ds.mv(g)
            src.append((off, ids))
        else:
            src.append(ds.ids(g))
    exp_docs: List[int] = []
    exp_keys: List[tuple] = []
    for d in docs.tolist():
        keys: List[tuple] = [()]
        for j in range(len(cols) - 1, -1, -1):
            s = src[j]
            if isinstance(s, tuple):
                vals = s[1][s[0][d]:s[0][d + 1]].tolist()
                keys = [(v,) + k for v in vals for k in keys]
            else:
                v = int(s[d])
                keys = [(v,) + k for k in keys]
        for k in keys:
            exp_docs.append(d)
            exp_keys.append(k)
    prod = 1
    for g in cols:
        prod *= ds.seg.column(g).cardinality
    order: Dict[tuple, List[int]] = {}
    for d, k in zip(exp_docs, exp_keys):
        lst = order.get(k)
        if lst is None:
            if prod > max_init_group_holder_capacity and len(order) >= num_groups_limit:
                continue  # map-based holder full: new keys get no group id (INVALID_ID)
            lst = order[k] = []
        lst.append(d)
    dicts = [ds.dictionary(g) for g in cols]
    groups: Dict[tuple, list] = {}
    for k, dl in order.items():
        vals = []
        for j, dct in enumerate(dicts):
            v = dct[k[j]]
            vals.append(v.item() if hasattr(v, "item") else v)
        part = np.asarray(dl, dtype=np.int64)
        groups[tuple(vals)] = [aggregate(a.function, None if a.column is None else
                                         _as_float_values(ds, a.column, part, a.function), len(part))
                               for a in query.aggregations]
    return groups


@dataclass
class OracleResult:
    aggregation_result: Optional[list] = None
    group_rows: Optional[List[tuple]] = None
    rows: Optional[List[tuple]] = None
    intermediate: Optional[dict] = None
    num_docs_scanned: int = 0
    num_entries_scanned_in_filter: int = 0
    num_entries_scanned_post_filter: int = 0
    num_total_docs: int = 0
    num_segments_matched: int = 0                    # CombineOperatorUtils.java:64-67: numDocsScanned > 0
    num_groups_limit_reached: bool = False           # AggregationGroupByOrderByOperator.java:111 (any segment)
    segment_matched: Optional[List[bool]] = None     # per segment, for the union over filtered-aggregation passes


def execute(query, segments: Sequence[SegmentData], num_groups_limit: int = 100_000,
            max_init_group_holder_capacity: int = 10_000, iterator_stats: bool = False) -> OracleResult:
    """All segments of one server + the broker reduce (no group trimming).  `query`: SQL text (parsed by
    oracle/sql.py) or a parsed query."""
    if isinstance(query, str):
        query = parse_sql(query)
    if query.has_filtered_aggregations:
        return _execute_filtered(query, segments, num_groups_limit, max_init_group_holder_capacity, iterator_stats)
    fns = [a.function for a in query.aggregations]
    out = OracleResult()
    decoded: Dict[int, DecodedSegment] = {}
    agg = None
    groups: Dict[tuple, list] = {}
    out.segment_matched = []
    for s in segments:
        ds = decoded.setdefault(id(s), DecodedSegment(s))
        r = execute_segment(query, ds, num_groups_limit, max_init_group_holder_capacity, iterator_stats)
        out.segment_matched.append(r.num_docs_scanned > 0)
        out.num_segments_matched += int(r.num_docs_scanned > 0)
        if query.group_by and num_groups_limit > 0 and r.num_groups >= num_groups_limit:
            out.num_groups_limit_reached = True
        out.num_docs_scanned += r.num_docs_scanned
        out.num_entries_scanned_in_filter += r.num_entries_scanned_in_filter
        out.num_entries_scanned_post_filter += r.num_entries_scanned_post_filter
        out.num_total_docs += r.num_total_docs
        if r.aggregation is not None:
            agg = r.aggregation if agg is None else [merge(f, a, b) for f, a, b in zip(fns, agg, r.aggregation)]
        else:
            for k, v in r.groups.items():
                groups[k] = v if k not in groups else [merge(f, a, b) for f, a, b in zip(fns, groups[k], v)]
    if not query.group_by:
        out.intermediate = {(): agg}
        out.aggregation_result = [final(f, v) for f, v in zip(fns, agg)]
        out.rows = [tuple(out.aggregation_result)]
        return out
    out.intermediate = groups
    rows = [k + tuple(final(f, v) for f, v in zip(fns, vs)) for k, vs in groups.items()]
    out.group_rows = rows
    names = list(query.group_by) + [a.result_name for a in query.aggregations]
    ordered = rows
    for ob in reversed(query.order_by):
        i = names.index(ob.expression)
        ordered = sorted(ordered, key=lambda r, i=i: r[i], reverse=not ob.ascending)
    ordered = ordered[: query.limit]
    sel = []
    for r in ordered:
        sel.append(tuple(r[names.index(s if isinstance(s, str) else s.result_name)] for s in query.select))
    out.rows = sel
    return out


def _split_filtered(query):
    from .sql import Agg, Query
    if isinstance(query, Query):
        return split_filtered(query)
    # a pinot_amd QueryContext: its passes restated with the oracle's own structures
    q = Query(query.table, list(query.select), [Agg(a.function, a.column, a.filter_key) for a in query.aggregations],
              query.filter, list(query.group_by), list(query.order_by), query.limit, dict(query.agg_filters))
    return split_filtered(q)


def _execute_filtered(query: QueryContext, segments, num_groups_limit, max_init, iterator_stats) -> OracleResult:
    """FilteredAggregationOperator (core/operator/query/FilteredAggregationOperator.java:62-95) over the passes of
    AggregationPlanNode.buildFilterOperatorInternal (:102-145): one per FILTER clause (main AND clause), then the
    main filter; per-segment sums equal the sums over all segments, so the passes run server-wide."""
    out = OracleResult()
    n = len(query.aggregations)
    fin, inter = [None] * n, [None] * n
    out.segment_matched = [False] * len(segments)
    for sq, idx in _split_filtered(query):
        r = execute(sq, segments, num_groups_limit, max_init, iterator_stats)
        # one FilteredAggregationOperator per segment sums its passes' numDocsScanned
        out.segment_matched = [a or b for a, b in zip(out.segment_matched, r.segment_matched)]
        for j, i in enumerate(idx):
            fin[i] = r.aggregation_result[j]
            inter[i] = r.intermediate[()][j]
        out.num_docs_scanned += r.num_docs_scanned
        out.num_entries_scanned_in_filter += r.num_entries_scanned_in_filter
        out.num_entries_scanned_post_filter += r.num_entries_scanned_post_filter
        out.num_total_docs = r.num_total_docs
    out.num_segments_matched = sum(out.segment_matched)
    out.aggregation_result = fin
    out.intermediate = {(): inter}
    out.rows = [tuple(fin[query.aggregations.index(s)] for s in query.select)]
    return out
