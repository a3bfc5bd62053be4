"""The *MV aggregation functions on the GPU path: lowered to single-value aggregations over a multi-value column's
per-row reductions, and raised back.

CountMV / SumMV / MinMV / MaxMV / AvgMVAggregationFunction (core/query/aggregation/function/*MVAggregationFunction.java)
aggregate every value of every matched row.  Each row's values reduce first (GpuSegment keeps them as raw columns
``<column>$mvlen|sum|min|max``, built once at upload by pgpu_segment_add_mv_row_columns), so over the matched rows

    COUNTMV(c) = SUM(c$mvlen)      SUMMV(c) = SUM(c$mvsum)      MINMV(c) = MIN(c$mvmin)      MAXMV(c) = MAX(c$mvmax)
    AVGMV(c)   = SUM(c$mvsum) / SUM(c$mvlen)   (intermediate (sum, count) like AvgPair)

The lowered query keeps the filter, GROUP BY and FILTER clauses, drops ORDER BY / LIMIT (applied to the raised
rows, since AVGMV's order is not one lowered column) and returns every group.
"""
from __future__ import annotations

import math
from dataclasses import replace
from typing import List, Optional, Tuple

from .query import MV_AGGS, AggregationSpec, QueryContext
from .segment import mv_row_column

UNLIMITED = 1 << 62


def has_mv_aggregations(query: QueryContext) -> bool:
    return any(a.function in MV_AGGS for a in query.aggregations)


def lower(query: QueryContext) -> Tuple[QueryContext, List[List[int]]]:
    """(lowered query, for each original aggregation the indexes of its lowered aggregations)."""
    aggs: List[AggregationSpec] = []
    parts: List[List[int]] = []

    def add(fn: str, col: Optional[str], key) -> int:
        aggs.append(AggregationSpec(fn, col, key))
        return len(aggs) - 1

    for a in query.aggregations:
        k = a.filter_key
        if a.function == "COUNTMV":
            parts.append([add("SUM", mv_row_column(a.column, "len"), k)])
        elif a.function == "SUMMV":
            parts.append([add("SUM", mv_row_column(a.column, "sum"), k)])
        elif a.function == "MINMV":
            parts.append([add("MIN", mv_row_column(a.column, "min"), k)])
        elif a.function == "MAXMV":
            parts.append([add("MAX", mv_row_column(a.column, "max"), k)])
        elif a.function == "AVGMV":
            parts.append([add("SUM", mv_row_column(a.column, "sum"), k), add("SUM", mv_row_column(a.column, "len"), k)])
        else:
            parts.append([add(a.function, a.column, k)])
    low = replace(query, select=list(query.group_by) + aggs, aggregations=aggs, order_by=[], limit=UNLIMITED)
    return low, parts


def lowered_columns(query: QueryContext) -> List[str]:
    return lower(query)[0].projected_columns


def _raise_values(query: QueryContext, parts: List[List[int]], fin: list, inter: list):
    """Final and intermediate values of the original aggregations from the lowered ones."""
    out_f, out_i = [], []
    for a, idx in zip(query.aggregations, parts):
        if a.function == "COUNTMV":
            v = int(round(fin[idx[0]]))
            out_f.append(v)
            out_i.append(v)
        elif a.function == "AVGMV":
            s, n = float(fin[idx[0]]), int(round(fin[idx[1]]))
            out_f.append(-math.inf if n == 0 else s / n)  # AvgMVAggregationFunction DEFAULT_FINAL_RESULT
            out_i.append((s, n))
        else:
            out_f.append(fin[idx[0]])
            out_i.append(inter[idx[0]])
    return out_f, out_i


def raise_result(query: QueryContext, parts: List[List[int]], low_res):
    """The original query's QueryResult from the lowered query's."""
    from .plan import QueryResult, order_and_limit, to_select_order

    res = QueryResult(query=query, stats=low_res.stats)
    # numEntriesScannedPostFilter = scanned docs x the ORIGINAL query's projected columns (the row columns the
    # lowered query reads stand in for their multi-value column: AggregationGroupByOrderByOperator.java:97-137)
    low_cols = len(lowered_columns(query))
    if low_cols:
        st = res.stats
        st.num_entries_scanned_post_filter = st.num_entries_scanned_post_filter // low_cols * len(query.projected_columns)
    if not query.group_by:
        fin, inter = _raise_values(query, parts, low_res.aggregation_result, low_res.intermediate[()])
        res.aggregation_result = fin
        res._intermediate = {(): inter}
        res.rows = [to_select_order(query, tuple(fin))]
        return res
    ng = len(query.group_by)
    inter_map = low_res.intermediate
    rows, inter_out = [], {}
    for r in low_res.group_rows:
        key = tuple(r[:ng])
        fin, inter = _raise_values(query, parts, list(r[ng:]), inter_map[key])
        rows.append(key + tuple(fin))
        inter_out[key] = inter
    res._group_rows = rows
    res._intermediate = inter_out
    res.rows = [to_select_order(query, r) for r in order_and_limit(query, sorted(rows, key=lambda r: r[:ng]))]
    return res
