"""The oracle's SQL front end (oracle/sql.py) against the product's (pinot_amd/query.py): written independently,
they must agree on every query the test suite and the bench workloads run, and the oracle executes SQL text with
its own parse.  CPU only."""
import ast
import glob
import os

import pytest

from oracle import sql as osql
from pinot_amd.query import parse_sql
from pinot_amd.synth import WORKLOADS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _corpus():
    """Every string literal starting with SELECT in the test files, plus the bench workloads' queries."""
    out = {w.sql for w in WORKLOADS.values()}
    for path in glob.glob(os.path.join(ROOT, "tests", "*.py")):
        tree = ast.parse(open(path).read())
        for node in ast.walk(tree):
            if isinstance(node, ast.Constant) and isinstance(node.value, str) and \
                    node.value.lstrip().upper().startswith("SELECT ") and "{" not in node.value:
                out.add(node.value)
    return sorted(out)


def _canon_filter(f):
    if f is None:
        return None
    if f.type == "PREDICATE":
        p = f.predicate
        return ("P", p.type, p.column, tuple(p.values), p.lower, p.upper, bool(p.lower_inclusive),
                bool(p.upper_inclusive))
    return (f.type, tuple(_canon_filter(c) for c in f.children))


def _canon(q):
    aggs = tuple((a.function, a.column, a.result_name.split(" FILTER")[0]) for a in q.aggregations)
    filt_aggs = tuple(sorted(_canon_filter(f) for f in q.agg_filters.values())) if q.agg_filters else ()
    return (q.table, aggs, _canon_filter(q.filter), tuple(q.group_by),
            tuple((o.expression.split(" FILTER")[0], o.ascending) for o in q.order_by), q.limit, filt_aggs,
            tuple(a.filter_key is not None for a in q.aggregations),
            tuple(s if isinstance(s, str) else s.result_name.split(" FILTER")[0] for s in q.select))


CORPUS = _corpus()


def test_corpus_is_substantial():
    assert len(CORPUS) > 60


@pytest.mark.parametrize("sql", CORPUS)
def test_parsers_agree(sql):
    try:
        prod = parse_sql(sql)
    except ValueError:
        pytest.skip("outside the product's subset (its tests expect the error)")
    assert _canon(osql.parse(sql)) == _canon(prod)


@pytest.mark.parametrize("sql,err", [("SELECT SUM(*) FROM t", ValueError), ("SELECT COUNT(*) FROM t WHERE", ValueError),
                                     ("SELECT COUNT(*) FROM t WHERE a ~ 3", ValueError),
                                     ("SELECT COUNT(*) FROM t LIMIT x", ValueError)])
def test_oracle_parser_errors(sql, err):
    with pytest.raises(err):
        osql.parse(sql)


def test_oracle_parser_forms():
    q = osql.parse("select a, sum(m) from t where (x >= -5 and y not between 1 and 2) or z not in ('a''b', 'c') "
                   "group by a order by sum(m) desc, a limit 7;")
    assert q.filter.type == "OR"
    and_, nin = q.filter.children
    assert and_.children[0].predicate == osql.Pred("RANGE", "x", lower="-5", lower_inclusive=True)
    assert and_.children[1].type == "NOT" and and_.children[1].children[0].predicate.upper == "2"
    assert nin.predicate == osql.Pred("NOT_IN", "z", ("a'b", "c"))
    assert [(o.expression, o.ascending) for o in q.order_by] == [("sum(m)", False), ("a", True)]
    assert q.limit == 7 and q.group_by == ["a"]
    # nested ANDs flatten (FlattenAndOrFilterOptimizer)
    f = osql.parse("SELECT COUNT(*) FROM t WHERE a = 1 AND (b = 2 AND (c = 3 AND d = 4))").filter
    assert f.type == "AND" and len(f.children) == 4


def test_engine_runs_sql_text_with_its_own_parser():
    import numpy as np
    from oracle import engine
    from oracle.segment_writer import build_segment
    from pinot_amd._lib import PGPU_INT
    rng = np.random.default_rng(0)
    seg = build_segment("s", {"a": (PGPU_INT, rng.integers(0, 5, 1000)), "m": (PGPU_INT, rng.integers(0, 9, 1000))})
    sql = "SELECT a, SUM(m), COUNT(*) FROM t WHERE m > 2 GROUP BY a ORDER BY SUM(m) DESC LIMIT 3"
    r1 = engine.execute(sql, [seg])
    r2 = engine.execute(parse_sql(sql), [seg])
    assert r1.rows == r2.rows and r1.group_rows == r2.group_rows
    sql = "SELECT SUM(m) FILTER(WHERE a = 1), COUNT(*) FROM t WHERE m > 2"
    assert engine.execute(sql, [seg]).rows == engine.execute(parse_sql(sql), [seg]).rows
