"""Multi-GPU combine: one process per GPU, partial tables merged with RCCL over xGMI.

Replaces the host-side merge of the reference — ``AggregationOnlyCombineOperator.mergeResultsBlocks``
(core/operator/combine/AggregationOnlyCombineOperator.java:47-57) and the ``GroupByOrderByCombineOperator``
IndexedTable upserts (core/operator/combine/GroupByOrderByCombineOperator.java:127-248) — for segments sharded over
the GPUs of one node (north_star).  Each rank runs ONE query launch over its own segments and leaves
a dense partial table in HBM (layout: include/pinot_gpu.h, pgpu_table_layout).  Then:

* small tables (aggregation only, or < 1 MiB): one ``all_reduce`` per reduction op (int64 SUM for counts and
  integer sums, float64 SUM for double sums, int64 MIN / MAX of order-preserving keys); rank 0 compacts the
  non-empty keys and finishes ORDER BY / LIMIT;
* large group-by tables: one ``reduce_scatter`` per section, so each rank owns the FINAL cells of 1/world of the
  key space; each rank compacts its slice and keeps its top ``max(5 * limit, 5000)`` rows by the ORDER BY
  expressions (GroupByUtils.getTableCapacity, core/util/GroupByUtils.java:24-41 — exact here, because every kept
  row's values are already merged over all ranks); rank 0 gathers the candidates and finishes.

Doc-id sets never leave their GPU.  Segments that the reference answers without a scan
(NonScanBasedAggregationOperator: match-all filter, only COUNT / MIN / MAX) are folded into the rank's G = 1 table
from metadata and dictionaries, with the reference's statistics (numTotalDocs, 0, 0, numTotalDocs).

Every decision that shapes a collective (global group dictionaries, the split-SUM table layout) is agreed by all
ranks before the collective runs, so no rank can skip or reorder one.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (PGPU_DOUBLE, PGPU_FLOAT, PGPU_INT, PGPU_LONG, PGPU_RED_MAX_I64, PGPU_RED_MIN_I64,
                   PGPU_RED_SUM_F64, PGPU_RED_SUM_I64, PGPU_STRING, QueryStats, TableLayout)
from .plan import (fixed_window, ExecutionStats, GpuPlanMaker, GroupColumns, GroupTable, QueryResult, check_group_columns, finish,
                   has_mv_aggregations, key_words_out, merge_filtered, mv_lower, mv_raise, table_capacity,
                   topk_spec, union_sorted)
from .query import QueryContext, split_filtered_aggregations
from .segment import GpuSegment

INT64_MAX = np.iinfo(np.int64).max
INT64_MIN = np.iinfo(np.int64).min


def section_ops(layout: TableLayout) -> List[int]:
    return [layout.section_op[s] for s in range(layout.num_sections)]


def section_identity(op: int) -> int:
    return INT64_MAX if op == PGPU_RED_MIN_I64 else (INT64_MIN if op == PGPU_RED_MAX_I64 else 0)


def _dist_op(op: int):
    import torch.distributed as dist
    return {PGPU_RED_SUM_I64: dist.ReduceOp.SUM, PGPU_RED_SUM_F64: dist.ReduceOp.SUM,
            PGPU_RED_MIN_I64: dist.ReduceOp.MIN, PGPU_RED_MAX_I64: dist.ReduceOp.MAX}[op]


def reduce_sections(table, layout: TableLayout, group=None) -> None:
    """In-place all-reduce of a dense partial table (torch int64 tensor [nsec * G], CPU/gloo or GPU/RCCL)."""
    import torch
    import torch.distributed as dist
    G = int(layout.num_keys)
    ops = section_ops(layout)
    view = table.view(len(ops), G)
    # one collective per op over the (possibly non-contiguous) sections that share it
    for op in (PGPU_RED_SUM_I64, PGPU_RED_SUM_F64, PGPU_RED_MIN_I64, PGPU_RED_MAX_I64):
        idx = [s for s, o in enumerate(ops) if o == op]
        if not idx:
            continue
        contiguous = idx == list(range(idx[0], idx[-1] + 1))
        buf = view[idx[0]: idx[-1] + 1] if contiguous else view[idx].contiguous()
        t = buf.view(-1)
        if op == PGPU_RED_SUM_F64:
            t = t.view(torch.float64)
        dist.all_reduce(t, op=_dist_op(op), group=group)
        if not contiguous:
            view[idx] = buf


def reduce_scatter_sections(table, layout: TableLayout, world: int, rank: int, group=None):
    """Reduce-scatter a dense partial table: returns (chunk [nsec, K] int64 tensor, first key) where this rank's
    K = ceil(G / world) keys hold cells reduced over every rank.  One collective per section."""
    import torch
    import torch.distributed as dist
    G = int(layout.num_keys)
    ops = section_ops(layout)
    K = (G + world - 1) // world
    view = table.view(len(ops), G)
    out = torch.empty((len(ops), K), dtype=torch.int64, device=table.device)
    native = hasattr(dist, "reduce_scatter_tensor") and dist.get_backend(group) != "gloo"
    pad = None  # one padded staging row for all sections, only when G does not split evenly (or under gloo)
    for s, op in enumerate(ops):
        if native and K * world == G:
            src = view[s]  # a contiguous row of the table: reduced in place of a copy
        else:
            if pad is None:
                pad = torch.empty((K * world,), dtype=torch.int64, device=table.device)
            pad[G:].fill_(section_identity(op))
            pad[:G].copy_(view[s])
            src = pad
        dst = out[s]
        if op == PGPU_RED_SUM_F64:
            src, dst = src.view(torch.float64), out[s].view(torch.float64)
        if native:
            dist.reduce_scatter_tensor(dst, src, op=_dist_op(op), group=group)
        else:  # gloo has no reduce_scatter: all_reduce, keep this rank's slice
            dist.all_reduce(src, op=_dist_op(op), group=group)
            dst.copy_(src[rank * K:(rank + 1) * K])
    return out, rank * K


def _encode_dictionary(local) -> np.ndarray:
    """A group dictionary as bytes for a tensor collective: int64 / float64 values, or length-prefixed UTF-8."""
    if isinstance(local, list):
        parts = []
        for v in local:
            b = v.encode("utf-8")
            parts.append(len(b).to_bytes(4, "little") + b)
        return np.frombuffer(b"".join(parts), dtype=np.uint8)
    a = np.asarray(local)
    a = a.astype(np.float64) if a.dtype.kind == "f" else a.astype(np.int64)
    return a.view(np.uint8)


def _decode_dictionary(raw: np.ndarray, kind: str):
    if kind == "s":
        out, b, i = [], raw.tobytes(), 0
        while i < len(b):
            n = int.from_bytes(b[i:i + 4], "little")
            out.append(b[i + 4:i + 4 + n].decode("utf-8"))
            i += 4 + n
        return out
    return raw.view(np.float64 if kind == "f" else np.int64)


def union_dictionaries(local: Sequence, group=None, device=None):
    """Sorted union of every rank's dictionary values for one group column, exchanged as byte tensors (sizes,
    then one all_gather of padded payloads)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = device if device is not None else torch.device("cpu")
    kind = "s" if isinstance(local, list) else ("f" if np.asarray(local).dtype.kind == "f" else "i")
    raw = _encode_dictionary(local)
    n = torch.tensor([len(raw)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    pad = max(1, max(sizes))
    mine = torch.zeros(pad, dtype=torch.uint8, device=dev)
    if len(raw):
        mine[: len(raw)] = torch.from_numpy(raw.copy()).to(dev)
    bufs = [torch.zeros(pad, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(bufs, mine, group=group)
    parts = [_decode_dictionary(b[:sz].cpu().numpy(), kind) for b, sz in zip(bufs, sizes)]
    if kind == "s":
        return sorted(set().union(*[set(p) for p in parts]))
    vals = union_sorted(parts)
    if kind == "i":
        return vals.astype(np.int64)
    return vals


def key_owners(keys: np.ndarray, world: int) -> np.ndarray:
    """Rank owning each group key (rows of key words) in the hash-table merge: the key words chained with the
    golden-ratio multiplier, two murmur3 fmix64 steps, modulo world -- the same routing as the node-level combine
    (pgpu_key_owner, pgpu_internal.h pgpu_key_owner_of)."""
    k2 = np.asarray(keys).reshape(len(keys), -1).astype(np.uint64)
    with np.errstate(over="ignore"):
        h = k2[:, 0].copy()
        for w in range(1, k2.shape[1]):
            h = h * np.uint64(0x9E3779B97F4A7C15) + k2[:, w]
        h ^= h >> np.uint64(33)
        h *= np.uint64(0xff51afd7ed558ccd)
        h ^= h >> np.uint64(33)
    return (h % np.uint64(world)).astype(np.int64)


def slice_of(num_keys: int, world: int, rank: int):
    """(first, count) of the keys rank owns after reduce_scatter_sections (pgpu_slice_of)."""
    K = (num_keys + world - 1) // world
    first = min(num_keys, K * rank)
    return first, min(K, num_keys - first)


def minmax_key(value: float, vtype: int) -> int:
    """Order-preserving int64 key of a MIN / MAX value (the inverse of pgpu_decode_minmax_key)."""
    if vtype in (PGPU_INT, PGPU_LONG):
        return int(value)
    b = int(np.float64(value).view(np.int64))
    return b if b >= 0 else b ^ 0x7FFFFFFFFFFFFFFF


def merge_rows(keys: np.ndarray, cells: np.ndarray, L: TableLayout):
    """Rows with equal keys merged section by section (AggregationFunction.merge on the cells): count and
    integer sums add, float sums add as doubles, MIN / MAX keys take the min / max."""
    if len(keys) == 0:
        return keys.reshape(0, keys.shape[1] if keys.ndim == 2 else 1), cells
    k2 = keys.reshape(len(keys), -1)
    uniq, inv = np.unique(k2, axis=0, return_inverse=True)
    inv = np.asarray(inv).reshape(-1)
    out = np.empty((len(uniq), cells.shape[1]), dtype=np.int64)
    for s, op in enumerate(section_ops(L)):
        col = cells[:, s]
        if op == PGPU_RED_SUM_F64:
            acc = np.zeros(len(uniq), dtype=np.float64)
            np.add.at(acc, inv, col.view(np.float64))
            out[:, s] = acc.view(np.int64)
        elif op == PGPU_RED_SUM_I64:
            acc = np.zeros(len(uniq), dtype=np.int64)
            np.add.at(acc, inv, col)
            out[:, s] = acc
        else:
            acc = np.full(len(uniq), section_identity(op), dtype=np.int64)
            (np.minimum if op == PGPU_RED_MIN_I64 else np.maximum).at(acc, inv, col)
            out[:, s] = acc
    return uniq, out


STAT_FIELDS = ("num_docs_scanned", "num_entries_scanned_in_filter", "num_entries_scanned_post_filter",
               "num_total_docs", "num_segments_processed", "num_segments_matched", "sparse_sector_bytes",
               "dense_bytes")

# local wait outcomes agreed by every rank before any collective touches the tables (collect)
_WAIT_OK, _WAIT_GROUPS_LIMIT, _WAIT_FAILED = 0, 1, 2


def _uids_of(key) -> tuple:
    """The segment uids inside a cache key: the key itself (_docs) or its last element (_globals, _split)."""
    if not key:
        return ()
    return key if isinstance(key[0], int) else key[-1]


class DistributedExecutor:
    """Executes a query over this rank's GPU segments and merges every rank's partial table (rank 0 finishes).

    The local kernel step (``_prepare_local`` / ``_wait_local`` / ``_compact``) goes through libpinotgpu; the
    collectives, agreements and finishing are backend-independent (the gloo tests drive them with a numpy
    table producer)."""

    SCATTER_MIN_BYTES = 1 << 20  # group-by tables from 1 MiB up are reduce-scattered
    TOPK_MIN = 5000              # per-rank candidates: max(5 * limit, 5000) (GroupByUtils.java:24-41)

    def __init__(self, plan_maker: Optional[GpuPlanMaker], group=None, device=None):
        import torch
        import torch.distributed as dist
        self.pm = plan_maker
        self.group = group
        self.dist = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if self.dist else 0
        self.world = dist.get_world_size(group) if self.dist else 1
        # the control plane -- cache agreements, wait outcomes, statistics, layout votes: a few int64s per query --
        # runs over a gloo (host) group of the same ranks, so those collectives neither wait for a CU behind the
        # next in-flight query kernel nor synchronise a device stream; the tables themselves go over RCCL
        self.ctrl, self.ctrl_device = group, None
        if self.dist and self.world > 1:
            if dist.get_backend(group) == "gloo":
                self.ctrl_device = torch.device("cpu")
            elif not os.environ.get("PGPU_CONTROL_ON_DEVICE"):
                ranks = None if group is None else dist.get_process_group_ranks(group)
                self.ctrl = dist.new_group(ranks=ranks, backend="gloo")
                self.ctrl_device = torch.device("cpu")
        if device is None:
            device = torch.device("cuda", plan_maker.ctx.device)
        self.device = device
        self._globals: Dict[tuple, tuple] = {}
        self._docs: Dict[tuple, tuple] = {}
        self._split: Dict[tuple, tuple] = {}
        self._tables: Dict[int, list] = {}
        self.last_stats = None
        ctx = getattr(plan_maker, "ctx", None)
        if hasattr(ctx, "add_listener"):
            ctx.add_listener(self)

    def segment_released(self, uid: int) -> None:
        """Forget the agreements naming a released segment (every rank then agrees on a miss: the hit / miss
        decisions stay collective, _agree)."""
        for cache in (self._globals, self._docs, self._split):
            for k in [k for k in cache if uid in _uids_of(k)]:
                del cache[k]

    # ---- collective helpers ------------------------------------------------------------------------------------
    def _allreduce_i64(self, vals: Sequence[int], op: str = "sum") -> List[int]:
        import torch
        import torch.distributed as dist
        dev = self.ctrl_device if self.ctrl_device is not None else self.device
        t = torch.tensor([int(v) for v in vals], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                               "min": dist.ReduceOp.MIN}[op], group=self.ctrl)
        return [int(x) for x in t.cpu().tolist()]

    def _agree(self, flag: bool) -> bool:
        """True on every rank iff it is true on every rank (cache hits must be collective decisions)."""
        return self._allreduce_i64([1 if flag else 0], "min")[0] == 1

    def _agree_hits(self, query: QueryContext, segments: Sequence[GpuSegment]) -> Tuple[bool, bool, bool]:
        """The three agreement caches' hits (global dictionaries, docs, table layout) decided together in ONE
        collective: a query whose agreements are all cached pays one small all-reduce before its launch."""
        mine = [query.group_by == [] or self._globals.get(self._globals_key(query, segments)) is not None,
                self._docs.get(self._seg_key(segments)) is not None,
                self._split.get(self._split_key(query, segments)) is not None]
        got = self._allreduce_i64([int(bool(x)) for x in mine], "min")
        return tuple(bool(x) for x in got)

    @staticmethod
    def _seg_key(segments: Sequence[GpuSegment]) -> tuple:
        return tuple(s.uid for s in segments)

    def _globals_key(self, query, segments):
        return (tuple(query.group_by), self._seg_key(segments))

    def _split_key(self, query, segments):
        return (tuple((a.function, a.column) for a in query.aggregations), tuple(query.group_by),
                self._seg_key(segments))

    def _global_dicts(self, query: QueryContext, segments: Sequence[GpuSegment], agreed: Optional[bool] = None):
        key = self._globals_key(query, segments)
        hit = self._globals.get(key)
        if not (self._agree(hit is not None) if agreed is None else agreed):
            hit = None
        if hit is None:
            check_group_columns(query, segments)
            dicts = []
            for g in query.group_by:
                local, _ = self.pm.global_dictionary(g, segments)
                dicts.append(union_dictionaries(local, self.group, self.device) if self.world > 1 else local)
            for g, glob in zip(query.group_by, dicts):
                self.pm.set_global_dictionary(g, segments, glob)
            hit = (dicts, tuple(segments))
            self._globals[key] = hit
        return hit[0]

    def _reduce_docs(self, segments: Sequence[GpuSegment], agreed: Optional[bool] = None) -> int:
        """Docs over all ranks (the bound of integer SUM cells after the reduce)."""
        key = self._seg_key(segments)
        hit = self._docs.get(key)
        if not (self._agree(hit is not None) if agreed is None else agreed):
            hit = None
        if hit is None:
            hit = (self._allreduce_i64([sum(s.num_docs for s in segments)])[0], tuple(segments))
            self._docs[key] = hit
        return hit[0]

    def _layout_flags(self, query: QueryContext, segments: Sequence[GpuSegment], reduce_docs: int,
                      agreed: Optional[bool] = None):
        """(flags, sum_layout) that give every rank the same table layout: PGPU_Q_SUM_SPLIT when any rank's
        integer-SUM bound needs the split sections, PGPU_Q_HASH when any rank's key space takes the hash group-by,
        and per aggregation the fixed-point window of a floating SUM spanning every rank's own (pgpu_sum_layout_agree
        over the ranks: the highest top, the finest exponent; PGPU_SUM_EXP_F64 anywhere makes every rank keep
        float64 sections)."""
        key = self._split_key(query, segments)
        hit = self._split.get(key)
        if not (self._agree(hit is not None) if agreed is None else agreed):
            hit = None
        if hit is None:
            L = self._local_layout(query, segments, 0, reduce_docs)
            na = len(query.aggregations)
            split = any(L.agg_sum_parts[i] == 3 and L.agg_value_type[i] in (_lib.PGPU_INT, _lib.PGPU_LONG)
                        for i in range(na))
            hashed = L.key_kind == _lib.PGPU_KEYS_HASH
            none = -(1 << 40)
            per = []
            for i in range(na):
                e, p = L.agg_sum_exp[i], L.agg_sum_parts[i]
                fp = L.agg_value_type[i] in (_lib.PGPU_FLOAT, _lib.PGPU_DOUBLE)
                f64 = fp and e == _lib.PGPU_SUM_EXP_F64
                live = fp and p > 1 and e not in (_lib.PGPU_SUM_EXP_F64, _lib.PGPU_SUM_EXP_ZERO)
                per += [int(f64), e + _lib.PGPU_PART_BITS * p if live else none, -e if live else none]
            red = self._allreduce_i64([int(split), int(hashed)] + per, "max")
            s_any, h_any = red[0], red[1]
            exps, parts = [], []
            for i in range(na):
                f64, top, negb = red[2 + 3 * i: 5 + 3 * i]
                if f64:
                    exps.append(_lib.PGPU_SUM_EXP_F64)
                    parts.append(1)
                elif top == none:
                    exps.append(_lib.PGPU_SUM_EXP_ZERO if L.agg_value_type[i] in (_lib.PGPU_FLOAT, _lib.PGPU_DOUBLE)
                                else 0)
                    parts.append(3 if L.agg_value_type[i] in (_lib.PGPU_FLOAT, _lib.PGPU_DOUBLE) else 0)
                else:
                    e, p = fixed_window(top, -negb)
                    exps.append(e)
                    parts.append(p)
            hit = (((_lib.PGPU_Q_SUM_SPLIT if s_any else 0) | (_lib.PGPU_Q_HASH if h_any else 0),
                    (tuple(exps), tuple(parts))), tuple(segments))
            self._split[key] = hit
        return hit[0]

    # ---- local kernel step (libpinotgpu) -------------------------------------------------------------------------
    def _local_layout(self, query, segments, flags, reduce_docs, sum_layout=None) -> TableLayout:
        return self._prepare_local(query, segments, flags, reduce_docs, sum_layout)[0]

    def _alloc_table(self, n: int):
        import torch
        pool = self._tables.setdefault(n, [])
        return pool.pop() if pool else torch.empty(n, dtype=torch.int64, device=self.device)

    def _prepare_local(self, query, segments, flags, reduce_docs, sum_layout=None):
        """(table layout, launch(table) -> handle) for this rank's scanned segments."""
        expr = self.pm.filter_expr(query, segments)
        desc, keep, _ = self.pm.build_desc(query, segments, plan_filters=expr is None, extra_flags=flags,
                                           reduce_docs=reduce_docs, sum_layout=sum_layout)
        L = self.pm.layout(desc)

        def launch(table):
            # libpinotgpu runs on its own HIP stream: the table memory is shared through the process's GPU address
            # space and ordered by explicit synchronisation (pgpu_query_wait before any collective touches it)
            _ = keep
            qh = C.c_void_p()
            lib = self.pm.ctx._lib
            n = int(table.numel())
            if expr is None:
                _lib.check(lib.pgpu_query_launch(self.pm.ctx.handle, C.byref(desc), None,
                                                 C.c_void_p(table.data_ptr()), 8 * n, C.byref(qh)))
            else:
                _lib.check(lib.pgpu_query_launch_expr(self.pm.ctx.handle, C.byref(desc), expr[0], expr[1], None,
                                                      C.c_void_p(table.data_ptr()), 8 * n, C.byref(qh)))
            return qh
        return L, launch

    def _wait_local(self, handle) -> dict:
        lib = self.pm.ctx._lib
        st = QueryStats()
        try:
            _lib.check(lib.pgpu_query_wait(handle, C.byref(st)))
        finally:
            lib.pgpu_query_release(handle)
        return {"num_docs_scanned": st.num_docs_scanned, "num_entries_scanned_in_filter":
                st.num_entries_scanned_in_filter, "num_total_docs": st.num_total_docs,
                "num_segments_matched": st.num_segments_matched,
                "num_groups_limit_reached": st.num_groups_limit_reached,
                "sparse_sector_bytes": st.sparse_sector_bytes, "dense_bytes": st.dense_bytes,
                "kernel_ms": st.kernel_ms, "filter_stats_exact": st.filter_stats_exact}

    def _compact(self, L: TableLayout, table, order=None):
        """Non-empty rows of a device table (pgpu_table_compact), or only the best ones by `order` selected on the
        GPU (pgpu_table_topk)."""
        cap = int(L.num_keys)
        kw = key_words_out(L)
        keys = np.empty(max(cap, 1) * kw, dtype=np.int64)
        cells = np.empty((max(cap, 1), L.num_sections), dtype=np.int64)
        ng = C.c_uint64()
        kp, cp = keys.ctypes.data_as(C.POINTER(C.c_int64)), cells.ctypes.data_as(C.POINTER(C.c_int64))
        if order is not None:
            _lib.check(self.pm.ctx._lib.pgpu_table_topk(self.pm.ctx.handle, C.byref(L), C.c_void_p(table.data_ptr()),
                                                        None, C.byref(order), kp, cp, cap, C.byref(ng)))
        else:
            _lib.check(self.pm.ctx._lib.pgpu_table_compact(self.pm.ctx.handle, C.byref(L),
                                                           C.c_void_p(table.data_ptr()), None, kp, cp, cap,
                                                           C.byref(ng)))
        n = ng.value
        return (keys[: n * kw].reshape(n, kw) if kw > 1 else keys[:n]), cells[:n]

    def _sync_device(self):
        import torch
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    # ---- query ---------------------------------------------------------------------------------------------------
    def submit(self, query: QueryContext, segments: Sequence[GpuSegment]):
        """Plan and launch this rank's part of the query without waiting (several may be in flight: the host
        plans and reduces query i while the GPU runs query i+1)."""
        if self.world == 1:
            return self.pm.submit(query, segments)
        import torch
        if not segments:
            raise ValueError("every rank needs at least one segment")
        hit_g, hit_d, hit_s = self._agree_hits(query, segments)
        globals_ = self._global_dicts(query, segments, hit_g) if query.group_by else []
        reduce_docs = self._reduce_docs(segments, hit_d)
        flags, sum_layout = self._layout_flags(query, segments, reduce_docs, hit_s)
        non_scan = self.pm.non_scan_segments(query, segments)
        scan = [s for s, ns in zip(segments, non_scan) if not ns]
        # the layout is the same on every rank: group cardinalities are global, the split-SUM choice and the
        # fixed-point exponents agreed
        L, launch = self._prepare_local(query, scan if scan else segments, flags, reduce_docs, sum_layout)
        n = _lib.table_bytes(L) // 8 if L.key_kind == _lib.PGPU_KEYS_HASH else int(L.num_sections * L.num_keys)
        table = self._alloc_table(n)
        handle = None
        if scan:
            handle = launch(table)
        else:  # every local segment is answered from metadata: start from the identity table
            ops = section_ops(L)
            table.view(len(ops), -1).copy_(torch.tensor([[section_identity(o)] for o in ops], dtype=torch.int64)
                                           .expand(len(ops), int(L.num_keys)))
        return _DistPending(query, L, table, handle, globals_,
                            [s for s, ns in zip(segments, non_scan) if ns], len(segments), segments)

    def _fold_non_scan(self, p: "_DistPending", stats: dict) -> None:
        """NonScanBasedAggregationOperator answers (NonScanBasedAggregationOperator.java:85-101,253-256) folded
        into this rank's G = 1 table: COUNT = docs, MIN / MAX = the dictionary's first / last value."""
        if not p.non_scan:
            return
        L, query = p.layout, p.query
        view = p.table.view(L.num_sections, int(L.num_keys))
        cnt = sum(s.num_docs for s in p.non_scan)
        view[0, 0] += cnt
        for ai, a in enumerate(query.aggregations):
            if a.function not in ("MIN", "MAX"):
                continue
            sec, vt = L.agg_section[ai], L.agg_value_type[ai]
            for s in p.non_scan:
                lo, hi = s.min_max(a.column)
                k = minmax_key(lo if a.function == "MIN" else hi, vt)
                cur = int(view[sec, 0].item())
                view[sec, 0] = min(cur, k) if a.function == "MIN" else max(cur, k)
        stats["num_docs_scanned"] += cnt
        stats["num_total_docs"] += cnt
        stats["num_segments_matched"] += sum(1 for s in p.non_scan if s.num_docs > 0)

    def collect(self, pending) -> Optional[QueryResult]:
        """Wait for this rank's launch, merge the partial tables over the collectives; rank 0 finishes."""
        if self.world == 1:
            res = self.pm.collect(pending)
            self.last_stats = res.stats
            return res
        p = pending
        stats = {"num_docs_scanned": 0, "num_entries_scanned_in_filter": 0, "num_total_docs": 0,
                 "num_segments_matched": 0, "num_groups_limit_reached": 0,
                 "sparse_sector_bytes": 0, "dense_bytes": 0, "kernel_ms": 0.0}
        # the local wait may fail on some ranks only (a segment past numGroupsLimit, a deadline): every rank learns
        # the worst outcome before the next collective, so no rank is left waiting in one
        status, err = _WAIT_OK, None
        if p.handle is not None:
            h, p.handle = p.handle, None
            try:
                stats.update(self._wait_local(h))
            except _lib.GroupsLimitError as e:
                status, err = _WAIT_GROUPS_LIMIT, e
            except _lib.PinotGpuError as e:
                status, err = _WAIT_FAILED, e
        if status == _WAIT_OK:
            self._fold_non_scan(p, stats)
        query, L, table = p.query, p.layout, p.table
        scan_docs = stats["num_docs_scanned"] - sum(s.num_docs for s in p.non_scan)
        local = [stats["num_docs_scanned"], stats["num_entries_scanned_in_filter"],
                 scan_docs * len(query.projected_columns), stats["num_total_docs"], p.num_segments,
                 stats["num_segments_matched"], stats["sparse_sector_bytes"], stats["dense_bytes"],
                 int(bool(stats["num_groups_limit_reached"])), 0 if stats.get("filter_stats_exact", 1) else 1]
        # the ranks' wait outcomes ride in the same all-reduce as the statistics (counts of ranks per outcome)
        red = self._allreduce_i64([int(status == _WAIT_GROUPS_LIMIT), int(status == _WAIT_FAILED)] + local)
        worst = _WAIT_FAILED if red[1] else (_WAIT_GROUPS_LIMIT if red[0] else _WAIT_OK)
        if worst != _WAIT_OK:
            self._tables.setdefault(int(p.table.numel()), []).append(p.table)
            if worst == _WAIT_FAILED:
                raise err if status == _WAIT_FAILED else _lib.PinotGpuError(
                    _lib.PGPU_E_INVALID, "the query failed on another rank")
            return self._collect_first_seen(p)
        sums = red[2:]
        tot = dict(zip(STAT_FIELDS, sums))
        st = ExecutionStats(kernel_ms=stats["kernel_ms"], filter_stats_exact=sums[-1] == 0,  # this rank's kernel
                            num_groups_limit_reached=sums[-2] > 0, **tot)
        self.last_stats = st
        try:
            big = query.group_by and 8 * int(table.numel()) >= self.SCATTER_MIN_BYTES
            if L.key_kind == _lib.PGPU_KEYS_HASH:
                keys, cells = self._hash_merge_topk(p)
            elif big:
                keys, cells = self._scatter_topk(p)
            else:
                reduce_sections(table, L, self.group)
                self._sync_device()
                if self.rank != 0:
                    return None
                keys, cells = self._compact(L, table)
            if self.rank != 0:
                return None
            if keys.ndim == 1:
                order = np.argsort(keys, kind="stable")
                keys, cells = keys[order], cells[order]
            return finish(query, GroupTable.sorted(keys, cells, L), p.globals_, st)
        finally:
            self._tables.setdefault(int(table.numel()), []).append(table)

    def _collect_first_seen(self, p: "_DistPending") -> Optional[QueryResult]:
        """Some rank's segment met more distinct group keys than numGroupsLimit: every rank answers its own
        segments by the first-seen path (GpuPlanMaker.first_seen_groups: the reference's map-based holders keep
        the first `limit` keys of each segment), and rank 0 merges the ranks' intermediate groups per aggregation
        function (GroupByOrderByCombineOperator's per-key merge) and finishes.  The rare path, so the exchange is
        one object all-gather rather than the table collectives."""
        import torch.distributed as dist

        from .datatable import _merge
        from .plan import result_from_intermediate
        # a failure on one rank must not leave the others waiting in the collective: every rank sends its outcome
        # (an error travels as its message) and all of them raise together
        try:
            r = self.pm.first_seen_groups(p.query, p.segments)
            mine = (r.intermediate, {f: getattr(r.stats, f) for f in STAT_FIELDS},
                    bool(r.stats.num_groups_limit_reached), bool(r.stats.filter_stats_exact), r.stats.kernel_ms, None)
        except Exception as exc:  # noqa: BLE001 -- re-raised below on every rank
            r, mine = None, (None, None, False, False, 0.0, f"rank {self.rank}: {type(exc).__name__}: {exc}")
        failed = self._allreduce_i64([0 if mine[5] is None else 1], "max")[0]
        if failed:
            msg = [None] * self.world
            dist.all_gather_object(msg, mine[5], group=self.group)
            raise _lib.PinotGpuError(_lib.PGPU_E_INVALID, "first-seen group path failed: " +
                                     "; ".join(m for m in msg if m))
        # only rank 0 merges: gather the ranks' groups there
        every = [None] * self.world if self.rank == 0 else None
        dist.gather_object(mine, every, dst=dist.get_global_rank(self.group, 0) if self.group is not None else 0,
                           group=self.group)
        stat_vec = self._allreduce_i64([getattr(r.stats, f) for f in STAT_FIELDS] +
                                       [int(bool(r.stats.num_groups_limit_reached)),
                                        0 if r.stats.filter_stats_exact else 1])
        tot = dict(zip(STAT_FIELDS, stat_vec[:len(STAT_FIELDS)]))
        st = ExecutionStats(kernel_ms=r.stats.kernel_ms, num_groups_limit_reached=stat_vec[-2] > 0,
                            filter_stats_exact=stat_vec[-1] == 0, **tot)
        self.last_stats = st
        if self.rank != 0:
            return None
        fns = [a.function for a in p.query.aggregations]
        merged: Dict[tuple, list] = {}
        for inter, *_ in every:
            for k, v in inter.items():
                cur = merged.get(k)
                merged[k] = list(v) if cur is None else [_merge(fn, x, y) for fn, x, y in zip(fns, cur, v)]
        return result_from_intermediate(p.query, merged, st)

    def _trim_cap(self, query) -> int:
        """GroupByUtils.getTableCapacity(limit, min.server.group.trim.size) of the plan maker (TOPK_MIN without
        one); a non-positive minimum disables the trim (GroupByOrderByCombineOperator.java:80-95)."""
        m = getattr(self.pm, "min_server_group_trim_size", self.TOPK_MIN)
        return table_capacity(query.limit, m)

    def _trim(self, query, L, keys, cells, globals_):
        """This rank's candidate rows: its top max(5 * limit, TOPK_MIN) by the ORDER BY expressions (the rows'
        values are final here), or that many smallest keys without ORDER BY."""
        cap = self._trim_cap(query)
        if len(keys) <= cap:
            return keys, cells
        t = GroupTable.sorted(keys, cells, L)
        idx = np.sort(GroupColumns(query, t, globals_).order_and_limit(limit=cap)) if query.order_by else \
            np.arange(cap)
        return t.keys[idx], t.cells[idx]

    def _gather_rows(self, keys, cells, L):
        """All ranks' candidate rows (key words + cells) gathered on every rank (padded tensors)."""
        import torch
        import torch.distributed as dist
        kw = 1 if keys.ndim == 1 else keys.shape[1]
        n = len(keys)
        width = kw + L.num_sections
        pad = max(1, self._allreduce_i64([n], "max")[0])
        mine = torch.zeros((pad, width), dtype=torch.int64)
        if n:
            mine[:n, :kw] = torch.from_numpy(np.ascontiguousarray(keys.reshape(n, kw), dtype=np.int64))
            mine[:n, kw:] = torch.from_numpy(np.ascontiguousarray(cells))
        counts = [torch.zeros(1, dtype=torch.int64, device=self.device) for _ in range(self.world)]
        dist.all_gather(counts, torch.tensor([n], dtype=torch.int64, device=self.device), group=self.group)
        bufs = [torch.zeros((pad, width), dtype=torch.int64, device=self.device) for _ in range(self.world)]
        dist.all_gather(bufs, mine.to(self.device), group=self.group)
        rows = np.concatenate([b[: int(c.item())].cpu().numpy() for b, c in zip(bufs, counts)])
        k = rows[:, 0].copy() if kw == 1 else np.ascontiguousarray(rows[:, :kw])
        return k, np.ascontiguousarray(rows[:, kw:])

    def _hash_merge_topk(self, p: "_DistPending"):
        """Hash tables (slots differ per rank): compact locally, route every row to the rank owning its key
        (hash of the key words), merge the partial rows by key there (the IndexedTable upsert of
        GroupByOrderByCombineOperator.java:169-190), keep each rank's top-K, gather the candidates."""
        import torch
        import torch.distributed as dist
        L, query = p.layout, p.query
        keys, cells = self._compact(L, p.table)
        kw = 1 if keys.ndim == 1 else keys.shape[1]
        n = len(keys)
        dest = key_owners(keys.reshape(n, kw), self.world)
        order = np.argsort(dest, kind="stable")
        width = kw + L.num_sections
        rows = np.concatenate([keys.reshape(n, kw), cells], axis=1)[order] if n else np.zeros((0, width), np.int64)
        send = np.bincount(dest, minlength=self.world).astype(np.int64)
        send_t = torch.from_numpy(send).to(self.device)
        recv_t = torch.empty(self.world, dtype=torch.int64, device=self.device)
        dist.all_to_all_single(recv_t, send_t, group=self.group)
        recv = recv_t.cpu().numpy()
        out = torch.empty((int(recv.sum()), width), dtype=torch.int64, device=self.device)
        dist.all_to_all_single(out, torch.from_numpy(np.ascontiguousarray(rows)).to(self.device),
                               [int(x) for x in recv], [int(x) for x in send], group=self.group)
        got = out.cpu().numpy()
        mk, mc = merge_rows(got[:, :kw], got[:, kw:], L)
        mk, mc = self._trim(query, L, mk[:, 0] if kw == 1 else mk, mc, p.globals_)
        return self._gather_rows(mk, mc, L)

    def _scatter_topk(self, p: "_DistPending"):
        """Large group-by table: reduce-scatter, per-rank compaction and top-K, gather of the candidates."""
        import torch
        import torch.distributed as dist
        L, query = p.layout, p.query
        chunk, key0 = reduce_scatter_sections(p.table, L, self.world, self.rank, self.group)
        self._sync_device()
        CL = TableLayout()
        C.memmove(C.byref(CL), C.byref(L), C.sizeof(TableLayout))
        CL.num_keys = int(chunk.shape[1])
        # this rank's top max(5 * limit, 5000) of its key slice, selected on the GPU (ORDER BY), else on the host
        cap = self._trim_cap(query)
        order = topk_spec(query, [len(g) for g in p.globals_], cap, key_base=key0) if cap < (1 << 62) else None
        keys, cells = self._compact(CL, chunk.reshape(-1).contiguous(), order)
        keys, cells = self._trim(query, L, keys + key0, cells, p.globals_)
        return self._gather_rows(keys, cells, L)

    def execute(self, query: QueryContext, segments: Sequence[GpuSegment]) -> Optional[QueryResult]:
        if self.world == 1:  # single GPU: the plan maker's own plan choice (filtered passes, non-scan segments)
            res = self.pm.execute(query, segments)
            self.last_stats = res.stats
            return res
        if has_mv_aggregations(query):
            # *MV aggregations over the multi-value columns' row columns (pinot_amd/mv.py), raised on rank 0
            check_group_columns(query, segments)
            low, mv_parts = mv_lower(query)
            res = self.execute(low, segments)
            return None if res is None else mv_raise(query, mv_parts, res)
        if query.has_filtered_aggregations:
            # one reduced pass per FILTER clause plus the main pass (FilteredAggregationOperator), merged on rank 0
            parts = split_filtered_aggregations(query)
            pending = [self.submit(sq, segments) for sq, _ in parts]
            results = [self.collect(pq) for pq in pending]
            return None if results[0] is None else merge_filtered(query, parts, results)
        return self.collect(self.submit(query, segments))


class _DistPending:
    """A launched, not yet collected multi-GPU query of this rank."""

    def __init__(self, query, layout, table, handle, globals_, non_scan, num_segments, segments=()):
        self.query, self.layout, self.table, self.handle = query, layout, table, handle
        self.globals_, self.non_scan, self.num_segments = globals_, non_scan, num_segments
        self.segments = list(segments)

    def __del__(self):
        if self.handle is not None and getattr(self.handle, "value", None):
            try:
                _lib.load().pgpu_query_release(self.handle)
            except Exception:
                pass
            self.handle = None
