"""Shared test fixtures: segments built by the oracle's writers from the committed golden data."""
from __future__ import annotations

import json
import math
import os

import numpy as np

from pinot_amd._lib import PGPU_INT, PGPU_STRING

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def sv_columns():
    d = np.load(os.path.join(GOLDEN, "test_data_sv.npz"))
    out = {}
    for c in d.files:
        a = d[c]
        out[c] = (PGPU_STRING, a.tolist()) if a.dtype.kind == "U" else (PGPU_INT, a)
    return out


def sv_segment():
    """BaseSingleValueQueriesTest's segment: 30000 rows, 11 columns, no inverted index loaded."""
    from oracle.segment_writer import build_segment
    return build_segment("testTable_126164076_167572854", sv_columns())


def simple_data_segments():
    """QueryExecutorTest.java:84-103: two segments of simpleData200001.avro (dim0, dim1, met; default segment
    generator config, no sorted / inverted index configured -- dim0 is generated in sorted order by the creator
    only when the data is sorted, so the columns are plain fixed-bit here)."""
    from oracle.segment_writer import build_segment
    d = np.load(os.path.join(GOLDEN, "simple_data_200001.npz"))
    cols = {c: (PGPU_INT, d[c]) for c in ("dim0", "dim1", "met")}
    return [build_segment(f"testTable_{k}", cols, sorted_columns=()) for k in range(2)]


def fast_count_segment():
    """FastFilteredCountTest.java:104-134: 1000 rows; class/sorted with inverted indexes, sorted column sorted."""
    from oracle.segment_writer import build_segment
    n = 1000
    i = np.arange(n, dtype=np.int32)
    cols = {"sorted": (PGPU_INT, i), "class": (PGPU_INT, i % 8), "intRangeCol": (PGPU_INT, n - i)}
    return build_segment("testSegment", cols, inverted=["class", "sorted"])


def baseball_segment():
    """baseballStats QuickStart table: inverted index on playerID, teamID (offline table config)."""
    from oracle.segment_writer import build_segment
    d = np.load(os.path.join(GOLDEN, "baseball.npz"))
    cols = {"playerID": (PGPU_STRING, d["playerID"].tolist()), "yearID": (PGPU_INT, d["yearID"]),
            "teamID": (PGPU_STRING, d["teamID"].tolist()), "playerName": (PGPU_STRING, d["playerName"].tolist()),
            "runs": (PGPU_INT, d["runs"])}
    return build_segment("baseballStats_OFFLINE_0", cols, inverted=["playerID", "teamID"])


def close(a, b, rel=1e-9):
    if isinstance(a, (int, np.integer)) and isinstance(b, (int, np.integer)):
        return int(a) == int(b)
    a, b = float(a), float(b)
    if math.isinf(a) or math.isinf(b):
        return a == b
    return a == b or abs(a - b) <= rel * max(abs(a), abs(b))


def rows_close(r1, r2, rel=1e-9):
    if len(r1) != len(r2):
        return False
    for x, y in zip(r1, r2):
        if len(x) != len(y):
            return False
        for a, b in zip(x, y):
            if isinstance(a, str) or isinstance(b, str):
                if a != b:
                    return False
            elif not close(a, b, rel):
                return False
    return True


def trims(query, ngroups: int) -> bool:
    """Whether a GROUP BY ... ORDER BY ... LIMIT result holds only the server's trimmed groups (IndexedTable.finish
    keeps max(5 * limit, 5000) of them, GroupByUtils.getTableCapacity): the GPU path returns those."""
    return bool(query.group_by and query.order_by) and ngroups > max(5 * query.limit, 5000)


def check_groups(res, ref, rel=1e-9):
    """GPU group rows against the oracle's.  All groups when the query keeps them all; under the ORDER BY ... LIMIT
    trim, the GPU's groups are a subset of the oracle's with equal values, at least the trim size, and the final
    rows carry the oracle's ORDER BY values in order."""
    q = res.query
    n = len(q.group_by)
    g = {r[:n]: r for r in res.group_rows}
    o = {r[:n]: r for r in ref.group_rows}
    if trims(q, len(o)):
        assert set(g) <= set(o) and len(g) >= max(5 * q.limit, 5000), (len(g), len(o))
        names = [s if isinstance(s, str) else s.result_name for s in q.select]
        i = names.index(q.order_by[0].expression)
        a, b = [r[i] for r in res.rows], [r[i] for r in ref.rows]
        assert len(a) == len(b) and all(close(x, y, rel) for x, y in zip(a, b)), (a[:5], b[:5])
    else:
        assert set(g) == set(o), (len(g), len(o))
    for k in g:
        assert rows_close([g[k]], [o[k]], rel), (k, g[k], o[k])


# ---- fixed-point floating SUM restated (include/pinot_gpu.h, pgpu_fixed_sum_layout / the kernels' fixed_part) ----
def fixed_sum_layout(values):
    """(exp, parts) pgpu_fixed_sum_layout picks for these FLOAT / DOUBLE values (as doubles)."""
    from pinot_amd import _lib
    v = np.asarray(values, dtype=np.float64)
    if not np.all(np.isfinite(v)):
        return _lib.PGPU_SUM_EXP_F64, 1
    nz = np.abs(v[v != 0])
    if len(nz) == 0:
        return _lib.PGPU_SUM_EXP_ZERO, 3
    top = math.frexp(float(nz.max()))[1] + 1  # ilogb(max) + 2
    min_exp = math.frexp(float(nz.min()))[1] - 1
    min_lsb = min(_lsb_exp(float(x)) for x in np.unique(nz))
    need = max(min_lsb, min_exp - _lib.PGPU_FIXED_TOL_BITS)
    parts = max(3, -(-(top - need) // _lib.PGPU_PART_BITS))
    if parts > _lib.PGPU_MAX_FIXED_PARTS:
        return _lib.PGPU_SUM_EXP_F64, 1
    return top - _lib.PGPU_PART_BITS * parts, parts


def _lsb_exp(x: float) -> int:
    m, e = math.frexp(abs(x))
    M = int(m * (1 << 53))  # exact: x = M * 2^(e - 53)
    return e - 53 + ((M & -M).bit_length() - 1)


def fixed_digits(x: float, exp: int, parts: int):
    """The part sections' shares of x: sign(x) * 21-bit digits of rint(|x| * 2^-exp) (half to even)."""
    from fractions import Fraction
    from pinot_amd import _lib
    if x == 0:
        return [0] * parts
    i = round(Fraction(abs(x)) / Fraction(2) ** exp)
    b, m = _lib.PGPU_PART_BITS, (1 << _lib.PGPU_PART_BITS) - 1
    sg = -1 if x < 0 else 1
    return [sg * ((i >> (b * k)) & m) for k in range(parts)]
