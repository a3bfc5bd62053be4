"""Dictionary-based predicate evaluation on the host (what the GPU receives are dict-id ranges and sets).

Restates, for sorted immutable dictionaries:
  * ``BaseImmutableDictionary.binarySearch`` / ``insertionIndexOf`` / ``indexOf``
    (seglocal/segment/index/readers/BaseImmutableDictionary.java:125-270, IntDictionary.java:33-34, ...)
  * ``EqualsPredicateEvaluatorFactory.DictionaryBasedEqPredicateEvaluator``        (:85-113)
  * ``NotEqualsPredicateEvaluatorFactory.DictionaryBasedNeqPredicateEvaluator``    (:85-130)
  * ``InPredicateEvaluatorFactory.DictionaryBasedInPredicateEvaluator``            (:142-182)
  * ``NotInPredicateEvaluatorFactory.DictionaryBasedNotInPredicateEvaluator``      (:142-200)
  * ``RangePredicateEvaluatorFactory.SortedDictionaryBasedRangePredicateEvaluator`` (:114-198)
all under core/operator/filter/predicate/.  Literal parsing follows the stored type: integral literals for
INT/LONG columns (a fractional literal is compared numerically, the NumericalFilterOptimizer outcome),
doubles for FLOAT/DOUBLE, strings compared by code point for STRING.
"""
from __future__ import annotations

import bisect
import functools
from dataclasses import dataclass
from fractions import Fraction
from typing import List, Sequence, Union

import numpy as np

from ._lib import PGPU_DOUBLE, PGPU_FLOAT, PGPU_INT, PGPU_LONG, PGPU_STRING
from .query import UNBOUNDED, Predicate


@functools.lru_cache(maxsize=65536)
def _key(value: str, data_type: int):
    """Literal parsed as the column's stored type (memoised: the same literal is looked up in every segment)."""
    if data_type == PGPU_STRING:
        return value
    if data_type in (PGPU_INT, PGPU_LONG):
        try:
            return int(value)  # plain integral literal
        except ValueError:
            f = Fraction(value)
            return int(f) if f.denominator == 1 else f
    if data_type == PGPU_FLOAT:
        return float(np.float32(float(value)))
    return float(value)


class SortedDictionary:
    """Sorted dictionary values with the reference's binary-search contract (numpy searchsorted for numeric
    dictionaries, bisect for strings).

    STRING dictionaries of segments written with a non-zero padding character (the legacy '%') are searched on
    padded values with the literal padded the same way, as BaseImmutableDictionary.binarySearch / padString do
    (seglocal/segment/index/readers/BaseImmutableDictionary.java:211-285); with '\\0' padding the unpadded values
    are compared directly."""

    def __init__(self, values: Union[np.ndarray, Sequence[str]], data_type: int, pad_char: str = "\0",
                 entry_width: int = 0):
        self.data_type = data_type
        self._pad = None
        if data_type == PGPU_STRING:
            self.values = list(values)
            if pad_char != "\0" and entry_width > 0:
                self._pad = (pad_char.encode("utf-8")[:1], entry_width)
                self._search = [self._padded(v) for v in self.values]
        elif data_type in (PGPU_INT, PGPU_LONG):
            self.values = np.asarray(values, dtype=np.int64)
        else:
            self.values = np.asarray(values, dtype=np.float64)
        self._n = len(self.values)

    def __len__(self) -> int:
        return self._n

    def _padded(self, v: str) -> str:
        pad, width = self._pad
        b = v.encode("utf-8")
        return (b + pad * (width - len(b))).decode("utf-8") if len(b) < width else v

    def insertion_index_of(self, literal: str) -> int:
        """>= 0: index of an exact match; < 0: -(insertion point + 1)."""
        k = _key(literal, self.data_type)
        if self.data_type == PGPU_STRING:
            vals = self.values
            if self._pad is not None:
                vals, k = self._search, self._padded(k)
            i = bisect.bisect_left(vals, k)
            found = i < self._n and vals[i] == k
        elif isinstance(k, Fraction):  # fractional literal on an integer dictionary: never equal
            i = int(self.values.searchsorted(float(k), side="left"))
            found = False
        else:
            i = int(self.values.searchsorted(k, side="left"))
            found = i < self._n and self.values[i] == k
        return i if found else -(i + 1)

    def index_of(self, literal: str) -> int:
        i = self.insertion_index_of(literal)
        return i if i >= 0 else -1


@dataclass
class DictPredicateEvaluator:
    """Result of predicate evaluation against one segment's dictionary."""

    predicate: Predicate
    cardinality: int
    kind: str                    # "RANGE" or "SET"
    start: int = 0               # RANGE [start, end)
    end: int = 0
    ids: Sequence[int] = ()      # SET: matching ids (inclusive predicates) or non-matching ids (exclusive)
    always_true: bool = False
    always_false: bool = False

    @property
    def is_exclusive(self) -> bool:
        return self.predicate.is_exclusive

    def matching_dict_ids(self) -> List[int]:
        if self.kind == "RANGE":
            return list(range(self.start, self.end))
        if not self.is_exclusive:
            return sorted(self.ids)
        bad = set(self.ids)
        return [i for i in range(self.cardinality) if i not in bad]

    def non_matching_dict_ids(self) -> List[int]:
        if self.kind == "SET" and self.is_exclusive:
            return sorted(self.ids)
        good = set(self.matching_dict_ids())
        return [i for i in range(self.cardinality) if i not in good]


def get_predicate_evaluator(p: Predicate, dictionary: SortedDictionary) -> DictPredicateEvaluator:
    """PredicateEvaluatorProvider.getPredicateEvaluator for dictionary-encoded columns
    (core/operator/filter/predicate/PredicateEvaluatorProvider.java:38-89)."""
    card = len(dictionary)
    if p.type == "EQ":
        i = dictionary.index_of(p.values[0])
        if i < 0:
            return DictPredicateEvaluator(p, card, "SET", ids=(), always_false=True)
        return DictPredicateEvaluator(p, card, "SET", ids=(i,), always_true=card == 1)
    if p.type == "NOT_EQ":
        i = dictionary.index_of(p.values[0])
        if i < 0:
            return DictPredicateEvaluator(p, card, "SET", ids=(), always_true=True)
        return DictPredicateEvaluator(p, card, "SET", ids=(i,), always_false=card == 1)
    if p.type == "IN":
        ids = sorted({i for i in (dictionary.index_of(v) for v in p.values) if i >= 0})
        return DictPredicateEvaluator(p, card, "SET", ids=tuple(ids), always_false=len(ids) == 0,
                                      always_true=len(ids) == card)
    if p.type == "NOT_IN":
        ids = sorted({i for i in (dictionary.index_of(v) for v in p.values) if i >= 0})
        return DictPredicateEvaluator(p, card, "SET", ids=tuple(ids), always_true=len(ids) == 0,
                                      always_false=len(ids) == card)
    if p.type == "RANGE":
        if p.lower == UNBOUNDED:
            start = 0
        else:
            ins = dictionary.insertion_index_of(p.lower)
            start = -(ins + 1) if ins < 0 else (ins if p.lower_inclusive else ins + 1)
        if p.upper == UNBOUNDED:
            end = card
        else:
            ins = dictionary.insertion_index_of(p.upper)
            end = -(ins + 1) if ins < 0 else (ins + 1 if p.upper_inclusive else ins)
        n = end - start
        return DictPredicateEvaluator(p, card, "RANGE", start=start, end=end, always_false=n <= 0,
                                      always_true=n == card)
    raise ValueError(f"unsupported predicate type {p.type}")


# ---- raw (no-dictionary) columns --------------------------------------------------------------------------------
_INT_RANGE = {PGPU_INT: (-(1 << 31), (1 << 31) - 1), PGPU_LONG: (-(1 << 63), (1 << 63) - 1)}


def _java_parse_integral(value: str, data_type: int) -> int:
    """Integer.parseInt / Long.parseLong: optional sign, decimal digits only, in range (NumberFormatException
    otherwise, which fails the query in the reference)."""
    s = value
    body = s[1:] if s[:1] in "+-" else s
    if not body or not body.isascii() or not body.isdigit():
        raise ValueError(f"NumberFormatException: For input string: \"{value}\"")
    v = int(s)
    lo, hi = _INT_RANGE[data_type]
    if not lo <= v <= hi:
        raise ValueError(f"NumberFormatException: For input string: \"{value}\"")
    return v


def _java_parse_floating(value: str, data_type: int) -> float:
    """Float.parseFloat / Double.parseDouble (surrounding whitespace trimmed; NaN / Infinity spelled as Java does)."""
    s = value.strip()
    t = s[1:] if s[:1] in "+-" else s
    if t in ("NaN", "Infinity"):
        v = float(s.replace("Infinity", "inf"))
    elif any(ch.isalpha() and ch not in "eEdDfF" for ch in t) or not t:
        raise ValueError(f"NumberFormatException: For input string: \"{value}\"")
    else:
        v = float(t.rstrip("dDfF")) * (-1.0 if s[:1] == "-" else 1.0)
    return float(np.float32(v)) if data_type == PGPU_FLOAT else v


def parse_raw_literal(value: str, data_type: int):
    """The literal as the raw-value evaluators parse it for the column's stored type."""
    if data_type in (PGPU_INT, PGPU_LONG):
        return _java_parse_integral(value, data_type)
    if data_type in (PGPU_FLOAT, PGPU_DOUBLE):
        return _java_parse_floating(value, data_type)
    raise ValueError(f"raw-value predicates on stored type {data_type} are not on this path")


@dataclass
class RawPredicateEvaluator:
    """PredicateEvaluatorProvider's raw-value branch (core/operator/filter/predicate/PredicateEvaluatorProvider.java
    :38-89) for INT / LONG / FLOAT / DOUBLE columns:
      * RangePredicateEvaluatorFactory.newRawValueBasedEvaluator (:62-110): an unbounded side is the type's extreme,
        inclusive (Integer.MIN_VALUE / Long.MAX_VALUE / Float.NEGATIVE_INFINITY ...);
      * EqualsPredicateEvaluatorFactory / NotEqualsPredicateEvaluatorFactory raw evaluators: one parsed value;
      * InPredicateEvaluatorFactory / NotInPredicateEvaluatorFactory raw evaluators: a set of parsed values.
    A raw evaluator is never always-true / always-false (there is no dictionary to decide it on)."""

    predicate: Predicate
    data_type: int
    kind: str                       # "RANGE" or "SET"
    lower: Union[int, float] = 0    # RANGE bounds (with inclusive flags)
    upper: Union[int, float] = 0
    lower_inclusive: bool = True
    upper_inclusive: bool = True
    values: Sequence = ()           # SET members (EQ: one)

    @property
    def is_exclusive(self) -> bool:
        return self.predicate.is_exclusive

    @property
    def is_floating(self) -> bool:
        return self.data_type in (PGPU_FLOAT, PGPU_DOUBLE)


def get_raw_predicate_evaluator(p: Predicate, data_type: int) -> RawPredicateEvaluator:
    if p.type == "RANGE":
        lu, uu = p.lower == UNBOUNDED, p.upper == UNBOUNDED
        if data_type in (PGPU_INT, PGPU_LONG):
            lo_ext, hi_ext = _INT_RANGE[data_type]
        else:
            lo_ext, hi_ext = float("-inf"), float("inf")
        lo = lo_ext if lu else parse_raw_literal(p.lower, data_type)
        hi = hi_ext if uu else parse_raw_literal(p.upper, data_type)
        return RawPredicateEvaluator(p, data_type, "RANGE", lower=lo, upper=hi,
                                     lower_inclusive=lu or p.lower_inclusive, upper_inclusive=uu or p.upper_inclusive)
    if p.type in ("EQ", "NOT_EQ", "IN", "NOT_IN"):
        vals = tuple(parse_raw_literal(v, data_type) for v in p.values)
        return RawPredicateEvaluator(p, data_type, "SET", values=vals)
    raise ValueError(f"unsupported predicate type {p.type}")
