"""The oracle's own SQL front end (test infrastructure; see oracle/__init__.py), independent of pinot_amd.query so that
a parser bug is not shared by the two sides of a parity test.

It restates what the reference's query compilation yields for the aggregation / group-by subset the tests use
(CalciteSqlParser -> PinotQuery -> QueryContext, pinot-common/.../sql/parsers/CalciteSqlParser.java and
core/query/request/context/utils/QueryContextConverterUtils.java):

* comparison forms -> predicates (core/.../request/context/predicate/*Predicate.java): ``=`` EQ, ``<>`` / ``!=``
  NOT_EQ, ``IN`` / ``NOT IN``, ``BETWEEN`` (inclusive RANGE), ``< <= > >=`` (half-bounded RANGE, the other side
  RangePredicate.UNBOUNDED "*"); ``NOT BETWEEN`` is NOT over the RANGE;
* nested AND / OR flattened (core/query/optimizer/filter/FlattenAndOrFilterOptimizer.java);
* ``AGG(col) FILTER(WHERE ...)`` filtered aggregations (QueryContext._filteredAggregations), their passes split as
  AggregationPlanNode.buildFilterOperatorInternal does (:102-145);
* result column names ``fn(col)`` lower-cased function (AggregationFunction.getResultColumnName).

The structures are duck-compatible with what oracle/engine.py reads (type / children / predicate, function / column,
...), and engine.execute accepts SQL text directly.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

UNBOUNDED = "*"
AGG_FUNCTIONS = ("COUNT", "SUM", "MIN", "MAX", "AVG", "COUNTMV", "SUMMV", "MINMV", "MAXMV", "AVGMV")


@dataclass(frozen=True)
class Pred:
    type: str
    column: str
    values: Tuple[str, ...] = ()
    lower: str = UNBOUNDED
    upper: str = UNBOUNDED
    lower_inclusive: bool = False
    upper_inclusive: bool = False

    @property
    def is_exclusive(self) -> bool:
        return self.type in ("NOT_EQ", "NOT_IN")


@dataclass
class Filt:
    type: str  # AND OR NOT PREDICATE
    children: List["Filt"] = field(default_factory=list)
    predicate: Optional[Pred] = None


@dataclass(frozen=True)
class Agg:
    function: str
    column: Optional[str]
    filter_key: Optional[str] = None

    @property
    def result_name(self) -> str:
        base = "%s(%s)" % (self.function.lower(), self.column or "*")
        return base if self.filter_key is None else "%s FILTER(WHERE %s)" % (base, self.filter_key)


@dataclass(frozen=True)
class Order:
    expression: str
    ascending: bool = True


@dataclass
class Query:
    table: str
    select: list
    aggregations: List[Agg]
    filter: Optional[Filt] = None
    group_by: List[str] = field(default_factory=list)
    order_by: List[Order] = field(default_factory=list)
    limit: int = 10
    agg_filters: dict = field(default_factory=dict)

    @property
    def has_filtered_aggregations(self) -> bool:
        return any(a.filter_key is not None for a in self.aggregations)

    @property
    def projected_columns(self) -> List[str]:
        seen: List[str] = []
        for c in [a.column for a in self.aggregations] + self.group_by:
            if c is not None and c not in seen:
                seen.append(c)
        return seen


_LEX = re.compile(r"""
    (?P<ws>\s+)
  | (?P<str>'(?:''|[^'])*')
  | (?P<num>\d+(?:\.\d*)?(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?)
  | (?P<cmp><=|>=|<>|!=|=|<|>)
  | (?P<punct>[(),*;-])
  | (?P<name>[A-Za-z_$][\w.$]*)
""", re.X)


def _lex(sql: str) -> List[Tuple[str, str]]:
    out, pos = [], 0
    while pos < len(sql):
        m = _LEX.match(sql, pos)
        if m is None:
            raise ValueError("bad character at %r" % sql[pos:pos + 10])
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws" or (kind == "punct" and m.group() == ";"):
            continue
        text = m.group()
        if kind == "str":
            text = text[1:-1].replace("''", "'")
        out.append((kind, text))
    out.append(("end", ""))
    return out


class _P:
    def __init__(self, sql: str):
        self.t = _lex(sql)
        self.k = 0
        self.filters: dict = {}

    def cur(self, off: int = 0):
        return self.t[min(self.k + off, len(self.t) - 1)]

    def take(self):
        tok = self.t[self.k]
        self.k += 1
        return tok

    def word(self, w: str) -> bool:
        kind, text = self.cur()
        if kind == "name" and text.upper() == w:
            self.k += 1
            return True
        return False

    def need_word(self, w: str):
        if not self.word(w):
            raise ValueError("expected %s, found %r" % (w, self.cur()[1]))

    def punct(self, c: str) -> bool:
        if self.cur() == ("punct", c):
            self.k += 1
            return True
        return False

    def need(self, c: str):
        if not self.punct(c):
            raise ValueError("expected %r, found %r" % (c, self.cur()[1]))

    def name(self) -> str:
        kind, text = self.take()
        if kind != "name":
            raise ValueError("expected a name, found %r" % text)
        return text

    def value(self) -> str:
        neg = self.punct("-")
        kind, text = self.take()
        if kind == "num":
            return "-" + text if neg else text
        if kind == "str" and not neg:
            return text
        raise ValueError("expected a literal, found %r" % text)

    # ---- expressions ----
    def item(self):
        kind, text = self.cur()
        if kind == "name" and text.upper() in AGG_FUNCTIONS and self.cur(1) == ("punct", "("):
            fn = text.upper()
            self.k += 2
            col = None if self.punct("*") else self.name()
            self.need(")")
            if col is None and fn != "COUNT":
                raise ValueError("%s(*)" % fn)
            key = None
            if self.word("FILTER"):
                self.need("(")
                self.need_word("WHERE")
                start = self.k
                f = self.disj()
                # the clause's text, token by token (literals re-quoted), names the filtered aggregation
                key = " ".join(("'%s'" % v.replace("'", "''")) if kd == "str" else v
                               for kd, v in self.t[start:self.k])
                self.need(")")
                self.filters[key] = f
            return Agg(fn, None if fn == "COUNT" else col, key)
        return self.name()

    def disj(self) -> Filt:
        parts = [self.conj()]
        while self.word("OR"):
            parts.append(self.conj())
        return _merge("OR", parts)

    def conj(self) -> Filt:
        parts = [self.neg()]
        while self.word("AND"):
            parts.append(self.neg())
        return _merge("AND", parts)

    def neg(self) -> Filt:
        if self.word("NOT"):
            return Filt("NOT", [self.neg()])
        if self.punct("("):
            f = self.disj()
            self.need(")")
            return f
        return self.leaf()

    def leaf(self) -> Filt:
        col = self.name()
        if self.word("NOT"):
            if self.word("IN"):
                return Filt("PREDICATE", predicate=Pred("NOT_IN", col, self.value_list()))
            self.need_word("BETWEEN")
            return Filt("NOT", [self.between(col)])
        if self.word("IN"):
            return Filt("PREDICATE", predicate=Pred("IN", col, self.value_list()))
        if self.word("BETWEEN"):
            return self.between(col)
        kind, op = self.take()
        if kind != "cmp":
            raise ValueError("expected a comparison after %s" % col)
        v = self.value()
        if op == "=":
            p = Pred("EQ", col, (v,))
        elif op in ("<>", "!="):
            p = Pred("NOT_EQ", col, (v,))
        elif op in ("<", "<="):
            p = Pred("RANGE", col, upper=v, upper_inclusive=op == "<=")
        else:
            p = Pred("RANGE", col, lower=v, lower_inclusive=op == ">=")
        return Filt("PREDICATE", predicate=p)

    def between(self, col: str) -> Filt:
        lo = self.value()
        self.need_word("AND")
        hi = self.value()
        return Filt("PREDICATE", predicate=Pred("RANGE", col, lower=lo, upper=hi, lower_inclusive=True,
                                                upper_inclusive=True))

    def value_list(self) -> Tuple[str, ...]:
        self.need("(")
        vals = [self.value()]
        while self.punct(","):
            vals.append(self.value())
        self.need(")")
        return tuple(vals)


def _merge(kind: str, parts: List[Filt]) -> Filt:
    if len(parts) == 1:
        return parts[0]
    kids: List[Filt] = []
    for p in parts:
        kids.extend(p.children if p.type == kind else [p])
    return Filt(kind, kids)


def parse(sql: str) -> Query:
    p = _P(sql)
    p.need_word("SELECT")
    select = [p.item()]
    while p.punct(","):
        select.append(p.item())
    p.need_word("FROM")
    table = p.name()
    filt = p.disj() if p.word("WHERE") else None
    group_by: List[str] = []
    if p.word("GROUP"):
        p.need_word("BY")
        group_by = [p.name()]
        while p.punct(","):
            group_by.append(p.name())
    order_by: List[Order] = []
    if p.word("ORDER"):
        p.need_word("BY")
        while True:
            it = p.item()
            name = it.result_name if isinstance(it, Agg) else it
            asc = not p.word("DESC")
            if asc:
                p.word("ASC")
            order_by.append(Order(name, asc))
            if not p.punct(","):
                break
    limit = int(p.value()) if p.word("LIMIT") else 10
    if p.cur()[0] != "end":
        raise ValueError("trailing input at %r" % p.cur()[1])
    aggs = [s for s in select if isinstance(s, Agg)]
    return Query(table, select, aggs, filt, group_by, order_by, limit, dict(p.filters))


def split_filtered(q: Query) -> List[Tuple[Query, List[int]]]:
    """One pass per distinct FILTER clause (main filter AND the clause), then the main pass with the plain
    aggregations (COUNT(*) when there are none: its matched docs still count in numDocsScanned)."""
    by_key: dict = {}
    plain: List[int] = []
    for i, a in enumerate(q.aggregations):
        (plain if a.filter_key is None else by_key.setdefault(a.filter_key, [])).append(i)

    def one(f, idx):
        aggs = [Agg(q.aggregations[i].function, q.aggregations[i].column) for i in idx] or [Agg("COUNT", None)]
        return Query(q.table, list(aggs), aggs, f, limit=q.limit)

    passes = [(one(q.agg_filters[k] if q.filter is None else Filt("AND", [q.filter, q.agg_filters[k]]), idx), idx)
              for k, idx in by_key.items()]
    passes.append((one(q.filter, plain), plain))
    return passes
