"""QueryContext for the aggregation / group-by shapes this path serves, plus a small SQL front end.

Mirrors the parts of ``core/query/request/context/QueryContext.java`` the path consumes: the filter tree
(``FilterContext`` AND/OR/NOT/PREDICATE, ``Predicate`` EQ/NOT_EQ/IN/NOT_IN/RANGE), the aggregation functions, the
group-by expressions, ORDER BY and LIMIT, and the query options / instance settings that change results
(``numGroupsLimit``, ``maxInitialResultHolderCapacity``; core/plan/maker/InstancePlanMakerImplV2.java:66-88).
The SQL subset is the one the reference's query tests and the BASELINE configs use, so the parity tests read
like ``qtest/*QueriesTest.java``.  AND/OR children are flattened like FlattenAndOrFilterOptimizer
(core/query/optimizer/filter/FlattenAndOrFilterOptimizer.java).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

UNBOUNDED = "*"  # RangePredicate.UNBOUNDED


@dataclass(frozen=True)
class Predicate:
    type: str            # EQ, NOT_EQ, IN, NOT_IN, RANGE
    column: str
    values: Tuple[str, ...] = ()
    lower: str = UNBOUNDED
    upper: str = UNBOUNDED
    lower_inclusive: bool = False
    upper_inclusive: bool = False

    @property
    def is_exclusive(self) -> bool:
        """Predicate.Type.isExclusive: NOT_EQ and NOT_IN."""
        return self.type in ("NOT_EQ", "NOT_IN")


@dataclass
class FilterContext:
    type: str                                  # AND, OR, NOT, PREDICATE
    children: List["FilterContext"] = field(default_factory=list)
    predicate: Optional[Predicate] = None

    @staticmethod
    def leaf(p: Predicate) -> "FilterContext":
        return FilterContext("PREDICATE", predicate=p)


@dataclass(frozen=True)
class AggregationSpec:
    function: str        # COUNT, SUM, MIN, MAX, AVG; COUNTMV, SUMMV, MINMV, MAXMV, AVGMV (multi-value columns)
    column: Optional[str]  # None for COUNT(*)
    filter_key: Optional[str] = None  # FILTER(WHERE ...) clause text; its FilterContext is QueryContext.agg_filters

    @property
    def result_name(self) -> str:
        name = f"{self.function.lower()}({self.column if self.column else '*'})"
        return name if self.filter_key is None else f"{name} FILTER(WHERE {self.filter_key})"


@dataclass(frozen=True)
class OrderByExpr:
    expression: str      # column name or aggregation result name
    ascending: bool = True


@dataclass
class QueryContext:
    table: str
    select: List[object]                       # str column or AggregationSpec, in SELECT order
    aggregations: List[AggregationSpec]
    filter: Optional[FilterContext] = None
    group_by: List[str] = field(default_factory=list)
    order_by: List[OrderByExpr] = field(default_factory=list)
    limit: int = 10
    options: dict = field(default_factory=dict)
    agg_filters: dict = field(default_factory=dict)  # filter_key -> FilterContext (QueryContext._filteredAggregations)

    @property
    def has_filtered_aggregations(self) -> bool:
        """QueryContext.isHasFilteredAggregations (core/query/request/context/QueryContext.java)."""
        return any(a.filter_key is not None for a in self.aggregations)

    @property
    def columns(self) -> List[str]:
        """Distinct columns referenced (filter, aggregations, group-by), in first-reference order."""
        out: List[str] = []

        def add(c):
            if c and c not in out:
                out.append(c)

        def walk(f):
            if f is None:
                return
            if f.type == "PREDICATE":
                add(f.predicate.column)
            for ch in f.children:
                walk(ch)

        walk(self.filter)
        for f in self.agg_filters.values():
            walk(f)
        for a in self.aggregations:
            add(a.column)
        for g in self.group_by:
            add(g)
        return out

    @property
    def projected_columns(self) -> List[str]:
        """Columns the projection reads after the filter (TransformOperator.getNumColumnsProjected)."""
        out: List[str] = []
        for c in [a.column for a in self.aggregations] + list(self.group_by):
            if c and c not in out:
                out.append(c)
        return out


# ---- SQL front end -------------------------------------------------------------------------------------------
_TOKEN = re.compile(r"\s*(?:(?P<num>-?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?)|(?P<str>'(?:[^']|'')*')|"
                    r"(?P<op><>|!=|<=|>=|=|<|>|\(|\)|,|\*)|(?P<id>[A-Za-z_][A-Za-z0-9_.$]*))")
_AGGS = {"COUNT", "SUM", "MIN", "MAX", "AVG", "COUNTMV", "SUMMV", "MINMV", "MAXMV", "AVGMV"}
MV_AGGS = {"COUNTMV": "COUNT", "SUMMV": "SUM", "MINMV": "MIN", "MAXMV": "MAX", "AVGMV": "AVG"}


class SqlError(ValueError):
    pass


class _Parser:
    def __init__(self, sql: str):
        self.toks: List[Tuple[str, str]] = []
        pos = 0
        sql = sql.strip().rstrip(";")
        while pos < len(sql):
            m = _TOKEN.match(sql, pos)
            if not m or m.end() == pos:
                if sql[pos:].strip() == "":
                    break
                raise SqlError(f"cannot tokenize at: {sql[pos:pos + 20]!r}")
            kind = m.lastgroup
            val = m.group(kind)
            if kind == "str":
                val = val[1:-1].replace("''", "'")
            self.toks.append((kind, val))
            pos = m.end()
        self.i = 0
        self.agg_filters: dict = {}

    def peek(self, k=0):
        j = self.i + k
        return self.toks[j] if j < len(self.toks) else ("eof", "")

    def kw(self, word: str) -> bool:
        t = self.peek()
        if t[0] == "id" and t[1].upper() == word:
            self.i += 1
            return True
        return False

    def expect_kw(self, word: str):
        if not self.kw(word):
            raise SqlError(f"expected {word} at {self.peek()}")

    def op(self, o: str) -> bool:
        t = self.peek()
        if t[0] == "op" and t[1] == o:
            self.i += 1
            return True
        return False

    def expect_op(self, o: str):
        if not self.op(o):
            raise SqlError(f"expected {o!r} at {self.peek()}")

    def ident(self) -> str:
        t = self.peek()
        if t[0] != "id":
            raise SqlError(f"expected identifier at {t}")
        self.i += 1
        return t[1]

    def literal(self) -> str:
        t = self.peek()
        if t[0] in ("num", "str"):
            self.i += 1
            return t[1]
        raise SqlError(f"expected literal at {t}")

    # select item: agg(col|*) | column
    def select_item(self):
        t, t2 = self.peek(), self.peek(1)
        if t[0] == "id" and t[1].upper() in _AGGS and t2 == ("op", "("):
            fn = t[1].upper()
            self.i += 2
            if self.op("*"):
                col = None
            else:
                col = self.ident()
            self.expect_op(")")
            if fn != "COUNT" and col is None:
                raise SqlError(f"{fn}(*) is not supported")
            key = None
            if self.kw("FILTER"):  # AGG(col) FILTER(WHERE <filter>)
                self.expect_op("(")
                self.expect_kw("WHERE")
                start = self.i
                f = self.bool_expr()
                key = " ".join(v if k != "str" else "'" + v.replace("'", "''") + "'"
                               for k, v in self.toks[start:self.i])
                self.expect_op(")")
                self.agg_filters[key] = f
            return AggregationSpec(fn, None if fn == "COUNT" else col, key)
        return self.ident()

    def order_item(self) -> OrderByExpr:
        item = self.select_item()
        name = item.result_name if isinstance(item, AggregationSpec) else item
        asc = True
        if self.kw("DESC"):
            asc = False
        else:
            self.kw("ASC")
        return OrderByExpr(name, asc)

    def bool_expr(self) -> FilterContext:
        left = self.and_expr()
        parts = [left]
        while self.kw("OR"):
            parts.append(self.and_expr())
        return _flatten("OR", parts)

    def and_expr(self) -> FilterContext:
        parts = [self.not_expr()]
        while self.kw("AND"):
            parts.append(self.not_expr())
        return _flatten("AND", parts)

    def not_expr(self) -> FilterContext:
        if self.kw("NOT"):
            return FilterContext("NOT", [self.not_expr()])
        if self.op("("):
            f = self.bool_expr()
            self.expect_op(")")
            return f
        return self.predicate()

    def predicate(self) -> FilterContext:
        col = self.ident()
        negate = self.kw("NOT")
        if self.kw("BETWEEN"):
            lo = self.literal()
            self.expect_kw("AND")
            hi = self.literal()
            leaf = FilterContext.leaf(Predicate("RANGE", col, lower=lo, upper=hi, lower_inclusive=True,
                                                upper_inclusive=True))
            return FilterContext("NOT", [leaf]) if negate else leaf
        if self.kw("IN"):
            self.expect_op("(")
            vals = [self.literal()]
            while self.op(","):
                vals.append(self.literal())
            self.expect_op(")")
            return FilterContext.leaf(Predicate("NOT_IN" if negate else "IN", col, tuple(vals)))
        if negate:
            raise SqlError("NOT must be followed by BETWEEN or IN here")
        t = self.peek()
        if t[0] != "op":
            raise SqlError(f"expected comparison at {t}")
        self.i += 1
        v = self.literal()
        o = t[1]
        if o == "=":
            p = Predicate("EQ", col, (v,))
        elif o in ("<>", "!="):
            p = Predicate("NOT_EQ", col, (v,))
        elif o == "<":
            p = Predicate("RANGE", col, upper=v, upper_inclusive=False)
        elif o == "<=":
            p = Predicate("RANGE", col, upper=v, upper_inclusive=True)
        elif o == ">":
            p = Predicate("RANGE", col, lower=v, lower_inclusive=False)
        elif o == ">=":
            p = Predicate("RANGE", col, lower=v, lower_inclusive=True)
        else:
            raise SqlError(f"unsupported operator {o}")
        return FilterContext.leaf(p)


def _flatten(kind: str, parts: List[FilterContext]) -> FilterContext:
    if len(parts) == 1:
        return parts[0]
    out: List[FilterContext] = []
    for p in parts:
        if p.type == kind:
            out.extend(p.children)
        else:
            out.append(p)
    return FilterContext(kind, out)


def parse_sql(sql: str, **options) -> QueryContext:
    """Parse the supported SQL subset into a QueryContext.

    ``SELECT <aggs / group columns> FROM t [WHERE ...] [GROUP BY ...] [ORDER BY ...] [LIMIT n]``.
    Keyword options mirror the instance / query options that change results: ``num_groups_limit`` (default
    100,000, InstancePlanMakerImplV2.java:73-74) and ``max_init_group_holder_capacity`` (10,000).
    """
    p = _Parser(sql)
    p.expect_kw("SELECT")
    select = [p.select_item()]
    while p.op(","):
        select.append(p.select_item())
    p.expect_kw("FROM")
    table = p.ident()
    filt = None
    group_by: List[str] = []
    order_by: List[OrderByExpr] = []
    limit = 10
    if p.kw("WHERE"):
        filt = p.bool_expr()
    if p.kw("GROUP"):
        p.expect_kw("BY")
        group_by.append(p.ident())
        while p.op(","):
            group_by.append(p.ident())
    if p.kw("ORDER"):
        p.expect_kw("BY")
        order_by.append(p.order_item())
        while p.op(","):
            order_by.append(p.order_item())
    if p.kw("LIMIT"):
        limit = int(p.literal())
    if p.peek()[0] != "eof":
        raise SqlError(f"unexpected trailing tokens at {p.peek()}")
    aggs = [s for s in select if isinstance(s, AggregationSpec)]
    if not aggs:
        raise SqlError("only aggregation queries are served by this path")
    for s in select:
        if isinstance(s, str) and s not in group_by:
            raise SqlError(f"column {s} must appear in GROUP BY")
    if p.agg_filters and group_by:
        # filtered aggregations are planned by AggregationPlanNode only (AggregationPlanNode.java:81-145)
        raise SqlError("FILTER(WHERE ...) aggregations are supported for aggregation-only queries")
    return QueryContext(table=table, select=select, aggregations=aggs, filter=filt, group_by=group_by,
                        order_by=order_by, limit=limit, options=dict(options), agg_filters=dict(p.agg_filters))


def split_filtered_aggregations(q: QueryContext) -> List[Tuple[QueryContext, List[int]]]:
    """One sub-query per distinct FILTER clause (WHERE = main AND clause, the CombinedFilterOperator), then the
    main-filter query holding the non-filtered aggregations -- always run, even when it holds none, since its
    matched docs count in numDocsScanned (AggregationPlanNode.buildFilterOperatorInternal :102-145,
    FilteredAggregationOperator.getNextBlock :62-95).  Returns (sub-query, indices into q.aggregations)."""
    groups: dict = {}
    plain: List[int] = []
    for i, a in enumerate(q.aggregations):
        if a.filter_key is None:
            plain.append(i)
        else:
            groups.setdefault(a.filter_key, []).append(i)

    def sub(filt, idx):
        aggs = [AggregationSpec(q.aggregations[i].function, q.aggregations[i].column) for i in idx]
        if not aggs:
            aggs = [AggregationSpec("COUNT", None)]
        return QueryContext(table=q.table, select=list(aggs), aggregations=aggs, filter=filt, limit=q.limit,
                            options=dict(q.options))

    out = []
    for key, idx in groups.items():
        f = q.agg_filters[key]
        out.append((sub(f if q.filter is None else FilterContext("AND", [q.filter, f]), idx), idx))
    out.append((sub(q.filter, plain), plain))
    return out
