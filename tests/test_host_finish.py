"""Host-side finish of a group table (pinot_amd/plan.py GroupColumns): vectorised ORDER BY / LIMIT must give
exactly the rows of the per-row stable sorts in ``order_and_limit`` (GroupByDataTableReducer / IndexedTable.finish
order; ties stay in ascending global-key order), including heavy ties and string group values."""
import numpy as np
import pytest

from pinot_amd._lib import (PGPU_DOUBLE, PGPU_INT, PGPU_RED_MAX_I64, PGPU_RED_MIN_I64, PGPU_RED_SUM_F64,
                            PGPU_RED_SUM_I64, TableLayout)
from pinot_amd.plan import GroupColumns, GroupTable, order_and_limit, to_select_order
from pinot_amd.query import parse_sql

QUERIES = [
    "SELECT k, SUM(m), MAX(m), COUNT(*) FROM t GROUP BY k ORDER BY SUM(m) DESC LIMIT 100",
    "SELECT k, SUM(m), MAX(m), COUNT(*) FROM t GROUP BY k ORDER BY COUNT(*) ASC, MAX(m) DESC LIMIT 50",
    "SELECT k, SUM(m), MAX(m), COUNT(*) FROM t GROUP BY k ORDER BY k DESC LIMIT 10",
    "SELECT k, SUM(m), MAX(m), COUNT(*) FROM t GROUP BY k LIMIT 10",
    "SELECT k, AVG(d), MIN(d), COUNT(*) FROM t GROUP BY k ORDER BY AVG(d) ASC, k ASC LIMIT 25",
    "SELECT k, AVG(d), MIN(d), COUNT(*) FROM t GROUP BY k ORDER BY MIN(d) DESC LIMIT 100000",
]


def _table(q, G, rng, strings):
    L = TableLayout()
    L.num_keys = G
    ops = [PGPU_RED_SUM_I64]
    for i, a in enumerate(q.aggregations):
        if a.function == "COUNT":
            L.agg_section[i], L.agg_value_type[i] = 0, -1
            continue
        vt = PGPU_INT if a.column == "m" else PGPU_DOUBLE
        op = {"MIN": PGPU_RED_MIN_I64, "MAX": PGPU_RED_MAX_I64}.get(
            a.function, PGPU_RED_SUM_I64 if vt == PGPU_INT else PGPU_RED_SUM_F64)
        L.agg_section[i], L.agg_value_type[i] = len(ops), vt
        ops.append(op)
    L.num_sections = len(ops)
    for s, o in enumerate(ops):
        L.section_op[s] = o
    n = G // 2
    keys = np.sort(rng.choice(G, n, replace=False)).astype(np.int64)
    cells = np.empty((n, len(ops)), dtype=np.int64)
    cells[:, 0] = rng.integers(1, 20, n)
    for s, o in enumerate(ops[1:], 1):
        if o == PGPU_RED_SUM_F64:
            cells[:, s] = (rng.integers(-50, 50, n) * 0.5).view(np.int64)
        elif o in (PGPU_RED_MIN_I64, PGPU_RED_MAX_I64) and L.agg_value_type[[i for i in range(len(q.aggregations))
                                                                            if L.agg_section[i] == s][0]] == PGPU_DOUBLE:
            v = rng.integers(-40, 40, n) * 0.25
            b = v.view(np.int64)
            cells[:, s] = np.where(b >= 0, b, b ^ np.int64(0x7FFFFFFFFFFFFFFF))
        else:
            cells[:, s] = rng.integers(0, 100, n)
    glob = sorted(f"k{i:06d}" for i in range(G)) if strings else np.arange(G, dtype=np.int32) * 3
    return GroupTable(keys, cells, L), glob


@pytest.mark.parametrize("strings", [False, True], ids=["int_keys", "string_keys"])
@pytest.mark.parametrize("sql", QUERIES)
def test_vectorised_order_by_matches_row_sort(sql, strings):
    q = parse_sql(sql)
    rng = np.random.default_rng(len(sql))
    table, glob = _table(q, 1 << 14, rng, strings)
    gc = GroupColumns(q, table, [glob])
    got = [to_select_order(q, r) for r in gc.rows(gc.order_and_limit())]
    ref = [to_select_order(q, r) for r in order_and_limit(q, gc.rows())]
    assert got == ref
    assert len(gc.rows()) == len(table.keys)
