"""Multi-GPU combine: one process per GPU, partial tables merged with RCCL over xGMI.

Replaces the host-side merge of the reference — ``AggregationOnlyCombineOperator.mergeResultsBlocks``
(core/operator/combine/AggregationOnlyCombineOperator.java:47-57) and the ``GroupByOrderByCombineOperator``
IndexedTable upserts (core/operator/combine/GroupByOrderByCombineOperator.java:127-248) — for segments sharded over
the GPUs of one node (north_star).  Each rank runs ONE query launch over its own segments and leaves
a dense partial table in HBM (layout: include/pinot_gpu.h, pgpu_table_layout).  Sections are reduced with one
collective per reduction op (int64 SUM for counts and integer sums, float64 SUM for double sums, int64 MIN/MAX of
order-preserving keys), then rank 0 compacts the non-empty keys and finishes ORDER BY / LIMIT.  Doc-id sets never
leave their GPU; the only exchange is the table (G x sections x 8 bytes).

Group keys must mean the same thing on every rank: each group column's global dictionary is the sorted union of
every rank's segment dictionaries (``union_dictionaries``, one all_gather_object per query shape, cached).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (PGPU_RED_MAX_I64, PGPU_RED_MIN_I64, PGPU_RED_SUM_F64, PGPU_RED_SUM_I64, QueryStats,
                   TableLayout)
from .plan import ExecutionStats, GpuPlanMaker, GroupTable, QueryResult, finish, merge_filtered
from .query import QueryContext, split_filtered_aggregations
from .segment import GpuSegment


def section_ops(layout: TableLayout) -> List[int]:
    return [layout.section_op[s] for s in range(layout.num_sections)]


def reduce_sections(table, layout: TableLayout, group=None) -> None:
    """In-place all-reduce of a dense partial table (torch int64 tensor [nsec * G], CPU/gloo or GPU/RCCL)."""
    import torch.distributed as dist
    G = int(layout.num_keys)
    ops = section_ops(layout)
    view = table.view(len(ops), G)
    # one collective per op over the (possibly non-contiguous) sections that share it
    for op in (PGPU_RED_SUM_I64, PGPU_RED_SUM_F64, PGPU_RED_MIN_I64, PGPU_RED_MAX_I64):
        idx = [s for s, o in enumerate(ops) if o == op]
        if not idx:
            continue
        rop = {PGPU_RED_SUM_I64: dist.ReduceOp.SUM, PGPU_RED_SUM_F64: dist.ReduceOp.SUM,
               PGPU_RED_MIN_I64: dist.ReduceOp.MIN, PGPU_RED_MAX_I64: dist.ReduceOp.MAX}[op]
        contiguous = idx == list(range(idx[0], idx[-1] + 1))
        buf = view[idx[0]: idx[-1] + 1] if contiguous else view[idx].contiguous()
        t = buf.view(-1)
        if op == PGPU_RED_SUM_F64:
            t = t.view(__import__("torch").float64)
        dist.all_reduce(t, op=rop, group=group)
        if not contiguous:
            view[idx] = buf


def union_dictionaries(local: Sequence, group=None):
    """Sorted union of every rank's dictionary values for one group column."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts: List = [None] * world
    dist.all_gather_object(parts, list(local) if isinstance(local, list) else np.asarray(local).tolist(), group=group)
    if any(isinstance(v, str) for p in parts for v in p[:1]):
        return sorted(set().union(*[set(p) for p in parts]))
    return np.unique(np.concatenate([np.asarray(p) for p in parts]))


class DistributedExecutor:
    """Executes a query over this rank's GPU segments and merges every rank's partial table (rank 0 finishes)."""

    def __init__(self, plan_maker: GpuPlanMaker, group=None):
        import torch
        import torch.distributed as dist
        self.pm = plan_maker
        self.group = group
        self.dist = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if self.dist else 0
        self.world = dist.get_world_size(group) if self.dist else 1
        self.device = torch.device("cuda", plan_maker.ctx.device)
        self._globals: Dict[tuple, tuple] = {}
        self._tables: Dict[int, object] = {}
        self._cap_keys = None
        self.last_stats = None

    def _global_dicts(self, query: QueryContext, segments: Sequence[GpuSegment]):
        key = (tuple(query.group_by), tuple(id(s) for s in segments))
        hit = self._globals.get(key)
        if hit is None:
            hit = []
            for g in query.group_by:
                local, _ = self.pm.global_dictionary(g, segments)
                glob = union_dictionaries(local, self.group) if self.world > 1 else local
                hit.append(glob)
            # per-segment remap against the node-global dictionary
            for g, glob in zip(query.group_by, hit):
                self.pm.set_global_dictionary(g, segments, glob)
            self._globals[key] = hit
        return hit

    def submit(self, query: QueryContext, segments: Sequence[GpuSegment]):
        """Plan and launch this rank's part of the query without waiting (several may be in flight: the host
        plans and reduces query i while the GPU runs query i+1)."""
        if self.world == 1:
            return self.pm.submit(query, segments)
        import torch
        if query.group_by:
            self._global_dicts(query, segments)
        expr = self.pm.filter_expr(query, segments)
        desc, keep, globals_ = self.pm.build_desc(query, segments, plan_filters=expr is None)
        L = self.pm.layout(desc)
        n = int(L.num_sections * L.num_keys)
        pool = self._tables.setdefault(n, [])
        table = pool.pop() if pool else torch.empty(n, dtype=torch.int64, device=self.device)
        # libpinotgpu runs on its own HIP stream: the table memory is shared through the process's GPU address
        # space and ordered by explicit synchronisation (a pooled table's last reduce finished in collect)
        qh = C.c_void_p()
        lib = self.pm.ctx._lib
        if expr is None:
            _lib.check(lib.pgpu_query_launch(self.pm.ctx.handle, C.byref(desc), None,
                                             C.c_void_p(table.data_ptr()), 8 * n, C.byref(qh)))
        else:
            _lib.check(lib.pgpu_query_launch_expr(self.pm.ctx.handle, C.byref(desc), expr[0], expr[1], None,
                                                  C.c_void_p(table.data_ptr()), 8 * n, C.byref(qh)))
        return _DistPending(query, len(segments), L, table, qh, globals_)

    def collect(self, pending) -> Optional[QueryResult]:
        """Wait for this rank's launch, all-reduce the partial table over RCCL; rank 0 compacts and finishes."""
        if self.world == 1:
            res = self.pm.collect(pending)
            self.last_stats = res.stats
            return res
        import torch
        import torch.distributed as dist
        lib = self.pm.ctx._lib
        st = QueryStats()
        qh, pending.handle = pending.handle, None
        try:
            _lib.check(lib.pgpu_query_wait(qh, C.byref(st)))
        finally:
            lib.pgpu_query_release(qh)
        self.last_stats = st
        L, table, query = pending.layout, pending.table, pending.query
        reduce_sections(table, L, self.group)
        counts = torch.tensor([st.num_docs_scanned, st.num_total_docs], dtype=torch.int64, device=self.device)
        dist.all_reduce(counts, group=self.group)
        docs_scanned, total_docs = (int(x) for x in counts.tolist())
        torch.cuda.current_stream(self.device).synchronize()
        try:
            if self.rank != 0:
                return None
            cap = int(L.num_keys)
            keys = np.empty(max(cap, 1), dtype=np.int64)
            cells = np.empty((max(cap, 1), L.num_sections), dtype=np.int64)
            ng = C.c_uint64()
            _lib.check(lib.pgpu_table_compact(self.pm.ctx.handle, C.byref(L), C.c_void_p(table.data_ptr()),
                                              None, keys.ctypes.data_as(C.POINTER(C.c_int64)),
                                              cells.ctypes.data_as(C.POINTER(C.c_int64)), cap, C.byref(ng)))
            gt = GroupTable(keys[: ng.value], cells[: ng.value], L)
            stats = ExecutionStats(num_docs_scanned=docs_scanned,
                                   num_entries_scanned_in_filter=st.num_entries_scanned_in_filter,
                                   num_entries_scanned_post_filter=docs_scanned * len(query.projected_columns),
                                   num_total_docs=total_docs, num_segments_processed=pending.num_segments * self.world,
                                   kernel_ms=st.kernel_ms, sparse_sector_bytes=st.sparse_sector_bytes,
                                   dense_bytes=st.dense_bytes)
            return finish(query, gt, [g[0] for g in pending.globals_], stats)
        finally:
            self._tables.setdefault(int(table.numel()), []).append(table)

    def execute(self, query: QueryContext, segments: Sequence[GpuSegment]) -> Optional[QueryResult]:
        if self.world == 1:  # single GPU: the plan maker's own plan choice (filtered passes, non-scan segments)
            res = self.pm.execute(query, segments)
            self.last_stats = res.stats
            return res
        if query.has_filtered_aggregations:
            # one reduced pass per FILTER clause plus the main pass (FilteredAggregationOperator), merged on rank 0
            parts = split_filtered_aggregations(query)
            pending = [self.submit(sq, segments) for sq, _ in parts]
            results = [self.collect(pq) for pq in pending]
            return None if results[0] is None else merge_filtered(query, parts, results)
        return self.collect(self.submit(query, segments))


class _DistPending:
    """A launched, not yet collected multi-GPU query of this rank."""

    def __init__(self, query, num_segments, layout, table, handle, globals_):
        self.query, self.num_segments, self.layout = query, num_segments, layout
        self.table, self.handle, self.globals_ = table, handle, globals_

    def __del__(self):
        if self.handle is not None and getattr(self.handle, "value", None):
            try:
                from . import _lib as L
                L.load().pgpu_query_release(self.handle)
            except Exception:
                pass
            self.handle = None
