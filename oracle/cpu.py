"""ctypes driver of oracle/pinot_cpu.c — the timed CPU baseline (test infrastructure; see oracle/__init__.py).

Supports the bench shapes: a filter that is one scan predicate or an AND of scan predicates over fixed-bit
columns, COUNT/SUM/MIN/MAX/AVG, and a dense dictionary group-by.  Predicates are turned into truth bitsets over
each segment's dictionary by the oracle's own value-semantics evaluator (oracle/engine.py).
"""
from __future__ import annotations

import ctypes as C
import os
import time
from typing import List, Sequence

import numpy as np

from pinot_amd.query import QueryContext
from pinot_amd.segment import SegmentData

from .engine import DecodedSegment, _truth_on_dictionary

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpinot_cpu.so")
FN = {"COUNT": 0, "SUM": 1, "MIN": 2, "MAX": 3, "AVG": 1}


class Column(C.Structure):
    _fields_ = [("fwd", C.c_void_p), ("bits", C.c_int32), ("card", C.c_int32), ("dict", C.c_void_p)]


class Segment(C.Structure):
    _fields_ = [("num_docs", C.c_int32), ("num_columns", C.c_int32), ("cols", C.POINTER(Column))]


class Query(C.Structure):
    _fields_ = [("num_leaves", C.c_int32), ("leaf_col", C.POINTER(C.c_int32)),
                ("leaf_truth", C.POINTER(C.c_void_p)), ("num_aggs", C.c_int32), ("agg_fn", C.POINTER(C.c_int32)),
                ("agg_col", C.POINTER(C.c_int32)), ("num_group_cols", C.c_int32),
                ("group_col", C.POINTER(C.c_int32)), ("num_keys", C.c_int64)]


def _lib():
    if not os.path.exists(LIB):
        raise ImportError(f"{LIB} missing: run __graft_entry__.build()")
    lib = C.CDLL(LIB)
    lib.pc_execute.restype = C.c_int64
    lib.pc_execute.argtypes = [C.POINTER(Segment), C.c_int32, C.POINTER(Query), C.c_int32, C.c_void_p, C.c_void_p,
                               C.POINTER(C.c_int64)]
    return lib


def _leaves(f):
    if f is None:
        return []
    if f.type == "PREDICATE":
        return [f.predicate]
    if f.type == "AND" and all(c.type == "PREDICATE" for c in f.children):
        return [c.predicate for c in f.children]
    raise ValueError("cpu baseline supports AND-of-predicates filters only")


class CpuBaseline:
    """Prepared segments + query; `run(threads)` executes and returns (seconds, matched, counts, sums)."""

    def __init__(self, query: QueryContext, segments: Sequence[SegmentData]):
        self.lib = _lib()
        self.query = query
        self.keep: List = []
        cols = query.columns
        idx = {c: i for i, c in enumerate(cols)}
        segs = (Segment * len(segments))()
        preds = _leaves(query.filter)
        self.truths = []
        for si, s in enumerate(segments):
            ds = DecodedSegment(s)
            carr = (Column * len(cols))()
            for ci, c in enumerate(cols):
                col = s.column(c)
                if col.forward is None:
                    raise ValueError("cpu baseline needs fixed-bit columns")
                fwd = np.frombuffer(col.forward + b"\0" * 16, dtype=np.uint8).copy()
                dvals = np.asarray(ds.dictionary(c), dtype=np.float64).copy()
                self.keep += [fwd, dvals]
                carr[ci] = Column(fwd.ctypes.data, col.bits_per_value, col.cardinality, dvals.ctypes.data)
            self.keep.append(carr)
            segs[si] = Segment(s.num_docs, len(cols), carr)
            tr = []
            for p in preds:
                t = _truth_on_dictionary(ds.dictionary(p.column), s.column(p.column).data_type, p)
                bits = np.packbits(t, bitorder="little")
                bits = np.concatenate([bits, np.zeros(8, np.uint8)])
                self.keep.append(bits)
                tr.append(bits)
            self.truths.append(tr)
        for t in self.truths[1:]:
            if not all(np.array_equal(a, b) for a, b in zip(t, self.truths[0])):
                raise ValueError("cpu baseline expects segments that share their filter dictionaries")
        self.segs = segs
        # one query struct per segment is not needed: truths are per segment -> run segment by segment sets
        self.preds = preds
        self.cols = cols
        self.idx = idx
        cards = [segments[0].column(g).cardinality for g in query.group_by]
        self.num_keys = int(np.prod(cards)) if cards else 1
        self.segments = segments

    def _query_for(self, si: int) -> Query:
        q = self.query
        lc = (C.c_int32 * max(1, len(self.preds)))(*[self.idx[p.column] for p in self.preds])
        lt = (C.c_void_p * max(1, len(self.preds)))(*[t.ctypes.data for t in self.truths[si]])
        fn = (C.c_int32 * len(q.aggregations))(*[FN[a.function] for a in q.aggregations])
        ac = (C.c_int32 * len(q.aggregations))(*[self.idx[a.column] if a.column else 0 for a in q.aggregations])
        gc = (C.c_int32 * max(1, len(q.group_by)))(*[self.idx[g] for g in q.group_by])
        self.keep += [lc, lt, fn, ac, gc]
        return Query(len(self.preds), lc, lt, len(q.aggregations), fn, ac, len(q.group_by), gc, self.num_keys)

    def run(self, threads: int):
        """Execute over all segments with `threads` workers (one segment per task)."""
        nagg = len(self.query.aggregations)
        sums = np.zeros(nagg * self.num_keys, dtype=np.float64)
        counts = np.zeros(self.num_keys, dtype=np.int64)
        scanned = C.c_int64()
        q = self._query_for(0)
        t0 = time.perf_counter()
        matched = self.lib.pc_execute(self.segs, len(self.segments), C.byref(q), threads, sums.ctypes.data,
                                      counts.ctypes.data, C.byref(scanned))
        dt = time.perf_counter() - t0
        return dt, int(matched), counts, sums.reshape(nagg, self.num_keys), int(scanned.value)


def synth_segment(w, segment: int, num_docs: int) -> SegmentData:
    """C twin of pinot_amd.synth.build_segment_cpu (uniform columns only): same bytes, ~100x faster."""
    from pinot_amd._lib import PGPU_INT
    from pinot_amd.segment import ColumnIndexes
    from pinot_amd.synth import column_seed

    lib = C.CDLL(LIB)
    lib.pc_synth_fixed_bit.restype = None
    lib.pc_synth_fixed_bit.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_uint32, C.c_uint64]
    seg = SegmentData(f"{w.name}_{segment}", num_docs)
    for c in w.columns:
        if c.dist != "uniform":
            raise ValueError("C generator covers uniform columns")
        bits = 1 if c.cardinality - 1 <= 1 else int(c.cardinality - 1).bit_length()
        n = (num_docs * bits + 7) // 8
        buf = C.create_string_buffer(n + 8)
        lib.pc_synth_fixed_bit(buf, num_docs, bits, c.cardinality, column_seed(w.seed, segment, c.name))
        seg.columns[c.name] = ColumnIndexes(c.name, PGPU_INT, c.cardinality,
                                            dictionary=c.values().astype(">i4").tobytes(), forward=buf.raw[:n])
    return seg
