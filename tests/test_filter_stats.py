"""numEntriesScannedInFilter: libpinotgpu's host replay of the reference's iterators (pgpu_filter_entries_scanned,
pinot_amd/csrc/pgpu_iterstats.cpp) against the oracle's iterator model (oracle/engine.py), which is pinned on the
InnerSegment KAT (84,134).  CPU only: the replay runs over host bitmaps."""
import ctypes as C

import numpy as np
import pytest

from oracle import engine
from pinot_amd import _lib
from tests.helpers import load_kat, sv_segment


def _program(op):
    """The oracle's physical tree as a prefix-order pgpu_filter_node program (+ leaf masks in leaf order)."""
    nodes, leaves = [], []

    def rec(o):
        k = o.kind
        if k in ("SCAN", "BITMAP", "SORTED"):
            nodes.append({"SCAN": _lib.PGPU_F_SCAN, "BITMAP": _lib.PGPU_F_INVERTED, "SORTED": _lib.PGPU_F_SORTED}[k])
            leaves.append(o.mask)
        elif k in ("ALL", "EMPTY"):
            nodes.append(_lib.PGPU_F_MATCH_ALL if k == "ALL" else _lib.PGPU_F_EMPTY)
        elif k == "NOT":
            nodes.append(_lib.PGPU_F_NOT)
            rec(o.children[0])
        else:
            a = k == "AND"
            nodes.append(_lib.PGPU_F_AND_BEGIN if a else _lib.PGPU_F_OR_BEGIN)
            for ch in o.children:
                rec(ch)
                nodes.append(_lib.PGPU_F_AND_CHILD_END if a else _lib.PGPU_F_OR_CHILD_END)
            nodes.append(_lib.PGPU_F_AND_END if a else _lib.PGPU_F_OR_END)

    rec(op)
    return nodes, leaves


def _replay(op, n):
    lib = _lib.load()
    nodes, leaves = _program(op)
    arr = (_lib.FilterNode * max(1, len(nodes)))()
    for i, o in enumerate(nodes):
        arr[i].op = o
    words = []
    for m in leaves:
        padded = np.zeros((n + 63) // 64 * 64, dtype=bool)
        padded[:n] = m
        words.append(np.packbits(padded.reshape(-1, 8)[:, ::-1]).view("<u4").copy())
    ptrs = (C.POINTER(C.c_uint32) * max(1, len(words)))(*[w.ctypes.data_as(C.POINTER(C.c_uint32)) for w in words])
    out = C.c_int64()
    _lib.check(lib.pgpu_filter_entries_scanned(arr, len(nodes), ptrs, len(words), n, C.byref(out)))
    return out.value


def test_kat_filter_replays_to_84134():
    K = load_kat()
    from pinot_amd.query import parse_sql
    seg = sv_segment()
    ds = engine.DecodedSegment(seg)
    op = engine.build_physical(ds, parse_sql("SELECT COUNT(*) FROM t" + K["filter"]).filter)
    assert _replay(op, ds.num_docs) == 84134 == engine.entries_scanned_in_filter(op, ds.num_docs)[0]


def _random_tree(rng, n, depth=0):
    r = rng.random()
    if depth >= 3 or r < 0.45:
        kind = rng.choice(["SCAN", "SCAN", "BITMAP", "SORTED"])
        dens = rng.choice([0.001, 0.05, 0.3, 0.7, 0.97])
        if kind == "SORTED":
            m = np.zeros(n, dtype=bool)
            for _ in range(rng.integers(1, 4)):
                a = rng.integers(0, n)
                m[a: a + rng.integers(1, max(2, n // 4))] = True
        else:
            m = rng.random(n) < dens
        return engine.POp(kind, mask=m)
    if r < 0.55:
        return engine.POp("NOT", [_random_tree(rng, n, depth + 1)])
    kids = [_random_tree(rng, n, depth + 1) for _ in range(rng.integers(2, 4))]
    if r < 0.8:
        return engine.POp("AND", sorted(kids, key=lambda o: o.priority()))
    return engine.POp("OR", kids)


@pytest.mark.parametrize("seed", range(40))
def test_random_trees_match_the_oracle(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.choice([1, 63, 64, 65, 2048, 5000, 20_011]))
    op = _random_tree(rng, n)
    exp, docs = engine.entries_scanned_in_filter(op, n)
    assert _replay(op, n) == exp
