"""One process, several GPUs: the node-level combine inside libpinotgpu (pgpu_node_*, include/pinot_gpu.h).

The shape of a Pinot server that keeps one JVM for all GPUs of a node: segments are uploaded through each device's
context, a query is planned per device (the same aggregations, group columns and node-global group dictionaries on
every device) and ``pgpu_node_query`` launches every device and merges the partial tables with RCCL over xGMI
inside the library -- the combine the reference runs on the host (AggregationOnlyCombineOperator.java:47-57,
GroupByOrderByCombineOperator.java:127-248).  (``combine.DistributedExecutor`` is the one-process-per-GPU form.)
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import QueryDesc, QueryStats, TableLayout
from .plan import (ExecutionStats, GpuPlanMaker, GroupTable, QueryResult, check_group_columns, finish,
                   has_mv_aggregations, key_words_out, mv_lower, mv_raise, table_capacity, topk_spec, union_sorted)
from .query import QueryContext
from .segment import GpuContext, GpuSegment


def union_dictionary(column: str, segments: Sequence[GpuSegment]):
    """Sorted union of the segments' dictionaries of one group column (host data only)."""
    dicts = [s.dictionaries[s.group_view(column)] for s in segments]
    if isinstance(dicts[0], list):
        return sorted(set().union(*[set(d) for d in dicts]))
    return union_sorted(dicts)


class GpuNode:
    """pgpu_node: contexts for `devices` and one RCCL clique over them."""

    def __init__(self, devices: Sequence[int], **plan_options):
        self._lib = _lib.load()
        arr = (C.c_int32 * len(devices))(*devices)
        h = C.c_void_p()
        _lib.check(self._lib.pgpu_node_init(arr, len(devices), C.byref(h)))
        self.handle = h
        self.contexts: List[GpuContext] = []
        for i, d in enumerate(devices):
            ch = C.c_void_p()
            _lib.check(self._lib.pgpu_node_context(h, i, C.byref(ch)))
            self.contexts.append(GpuContext(d, _handle=ch))
        self.planners = [GpuPlanMaker(c, **plan_options) for c in self.contexts]
        self._globs = {}  # (group columns, segment uids) -> node-global group dictionaries (set on every planner)

    def close(self) -> None:
        if self.handle:
            for c in self.contexts:
                c.close()
            self._lib.pgpu_node_shutdown(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def execute(self, query: QueryContext, segments_by_device: Sequence[Sequence[GpuSegment]]) -> QueryResult:
        """One query over every device's segments, merged inside the library."""
        if has_mv_aggregations(query):  # *MV aggregations over row columns (pinot_amd/mv.py)
            check_group_columns(query, [s for segs in segments_by_device for s in segs])
            low, parts = mv_lower(query)
            return mv_raise(query, parts, self.execute(low, segments_by_device))
        return self.collect(self.submit(query, segments_by_device))

    def submit(self, query: QueryContext, segments_by_device: Sequence[Sequence[GpuSegment]]) -> "_NodePending":
        """Plan the query for every device and launch them (pgpu_node_submit); several may be in flight, collected
        in submission order."""
        if len(segments_by_device) != len(self.contexts):
            raise ValueError("one segment list per device")
        everything = [s for segs in segments_by_device for s in segs]
        check_group_columns(query, everything)
        if has_mv_aggregations(query):
            raise ValueError("*MV aggregations: use execute()")
        gkey = (tuple(query.group_by), tuple(s.uid for s in everything))
        globs = self._globs.get(gkey)
        if globs is None:  # node-global group dictionaries, set on every device (cached for the segment set)
            globs = [union_dictionary(g, everything) for g in query.group_by]
            for pm, segs in zip(self.planners, segments_by_device):
                for g, glob in zip(query.group_by, globs):
                    pm.set_global_dictionary(g, segs, glob)
            if len(self._globs) >= 16:  # (bounded: the oldest segment set's entry goes)
                self._globs.pop(next(iter(self._globs)))
            self._globs[gkey] = globs
        # numeric filters go to the library as expression programs (planned per segment in C++, as the
        # one-process-per-GPU path's pgpu_query_launch_expr does); otherwise every segment's tree is planned here
        exprs = [pm.filter_expr(query, segs) for pm, segs in zip(self.planners, segments_by_device)]
        use_expr = all(e is not None for e in exprs)
        keep, descs = [], []
        for pm, segs in zip(self.planners, segments_by_device):
            desc, k, _ = pm.build_desc(query, segs, plan_filters=not use_expr)
            keep.append((desc, k))
            descs.append(desc)
        arr = (C.POINTER(QueryDesc) * len(descs))(*[C.pointer(d) for d in descs])
        L0 = self.planners[0].layout(descs[0])
        h = C.c_void_p()
        if use_expr:
            earr = (C.POINTER(_lib.ExprNode) * len(exprs))(*[C.cast(e[0], C.POINTER(_lib.ExprNode)) for e in exprs])
            narr = (C.c_int32 * len(exprs))(*[int(e[1]) for e in exprs])
            keep.append((exprs, earr, narr))
            _lib.check(self._lib.pgpu_node_submit_expr(self.handle, arr, earr, narr, C.byref(h)))
        else:
            _lib.check(self._lib.pgpu_node_submit(self.handle, arr, C.byref(h)))
        return _NodePending(query, globs, keep, arr, L0, h, len(everything), segments_by_device)

    def collect(self, p: "_NodePending", min_cap: int = 0) -> QueryResult:
        """Wait for a submitted node query, merge and compact / trim it (pgpu_node_collect), finish on the host."""
        query, globs, L0 = p.query, p.globs, p.layout
        # the server's ORDER BY ... LIMIT trim (IndexedTable.finish): every device keeps its best rows of the
        # groups it owns after the merge
        pm0 = self.planners[0]
        order = None
        if pm0.gpu_topk and pm0.min_server_group_trim_size > 0:
            order = topk_spec(query, [len(g) for g in globs], table_capacity(query.limit, pm0.min_server_group_trim_size))
        # result rows: a dense table's G keys (merged onto one key space); a hash table's keys are disjoint per
        # owner device, at most every device's capacity; the ORDER BY trim keeps k per trimming device plus ties
        ndev = len(self.contexts)
        cap = int(L0.num_keys) * (ndev if L0.key_kind == _lib.PGPU_KEYS_HASH else 1)
        if order is not None:
            cap = min(cap, 2 * ndev * int(order.k))
        cap = max(cap, 1, min_cap)
        n = C.c_uint64()
        st = QueryStats()
        L = TableLayout()
        keys = np.empty(cap * 2, dtype=np.int64)  # two key words at most
        cells = np.empty((cap, _lib.PGPU_MAX_SECTIONS), dtype=np.int64)  # the agreed layout's sections fit
        h, p.handle = p.handle, None
        rc = self._lib.pgpu_node_collect(h, C.byref(order) if order is not None else None,
                                         keys.ctypes.data_as(C.POINTER(C.c_int64)),
                                         cells.ctypes.data_as(C.POINTER(C.c_int64)), cap, C.byref(n), C.byref(st),
                                         C.byref(L))
        if rc != _lib.PGPU_OK and n.value > cap and not min_cap:  # (a tie-heavy trim past the estimate: again, with room)
            return self.collect(self.submit(query, p.segments_by_device), min_cap=int(n.value))
        _lib.check(rc)
        kw = key_words_out(L)
        ng = n.value
        k = keys[: ng * kw].reshape(ng, kw) if kw > 1 else keys[:ng]
        c = cells.reshape(-1)[: ng * L.num_sections].reshape(ng, L.num_sections)
        stats = ExecutionStats(num_docs_scanned=st.num_docs_scanned,
                               num_entries_scanned_in_filter=st.num_entries_scanned_in_filter,
                               num_entries_scanned_post_filter=st.num_docs_scanned * len(query.projected_columns),
                               num_total_docs=st.num_total_docs, num_segments_processed=p.num_segments,
                               num_segments_matched=st.num_segments_matched,
                               num_groups_limit_reached=bool(st.num_groups_limit_reached),
                               kernel_ms=st.kernel_ms, sparse_sector_bytes=st.sparse_sector_bytes,
                               dense_bytes=st.dense_bytes, filter_stats_exact=bool(st.filter_stats_exact),
                               kernel_variant=st.kernel_variant)
        return finish(query, GroupTable.sorted(k, c, L), globs, stats)


class _NodePending:
    """A submitted node query: its descriptors (kept alive until collect) and the handle."""

    def __init__(self, query, globs, keep, arr, layout, handle, num_segments, segments_by_device):
        self.query, self.globs, self.keep, self.arr, self.layout = query, globs, keep, arr, layout
        self.handle, self.num_segments, self.segments_by_device = handle, num_segments, segments_by_device
