"""DistributedExecutor on the CPU: world_size-2 ``gloo`` groups driving the real multi-GPU combine code.

Only the local kernel step is replaced: ``_prepare_local`` / ``_wait_local`` / ``_compact`` produce each rank's
dense partial table in numpy from the oracle's filter evaluation (the table the query kernel leaves in HBM,
include/pinot_gpu.h).  Everything else is the production path: group dictionaries unioned over tensor collectives,
cache hits agreed by all ranks, the split-SUM layout agreed by all ranks, non-scan segments folded into the table,
statistics summed over ranks (CombineOperatorUtils.setExecutionStatistics), all-reduce for small tables and
reduce-scatter + per-rank top-K + gather for large ones.  Results are checked against the oracle over every rank's
segments (the reference's single-server combine: AggregationOnlyCombineOperator.java:47-57,
GroupByOrderByCombineOperator.java:127-248).
"""
from __future__ import annotations

import datetime
import math
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from pinot_amd._lib import (PGPU_DOUBLE, PGPU_FLOAT, PGPU_INT, PGPU_LONG, PGPU_MAX_FIXED_PARTS,  # noqa: E402
                            PGPU_PART_BITS, PGPU_Q_SUM_SPLIT, PGPU_SUM_EXP_F64, PGPU_RED_MAX_I64, PGPU_RED_MIN_I64, PGPU_RED_SUM_F64,
                            PGPU_RED_SUM_I64, PGPU_STRING, TableLayout)

from tests.helpers import fixed_digits, fixed_sum_layout  # noqa: E402

WORLD = 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, fn, port, args, world=2):
    global WORLD
    WORLD = world  # (the spawned process's own module copy: the helpers below read it)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # a collective that one rank skips must fail the test, not hang it
    dist.init_process_group("gloo", rank=rank, world_size=WORLD, timeout=datetime.timedelta(seconds=60))
    try:
        fn(rank, *args)
    finally:
        dist.destroy_process_group()


def _spawn(fn, *args, world=2):
    mp.spawn(_entry, args=(fn, _free_port(), args, world), nprocs=world, join=True)


# ---- a host-only stand-in for GpuSegment / GpuPlanMaker ----------------------------------------------------------
class HostSegment:
    """SegmentData with the GpuSegment surface the planner uses (no device)."""
    _next = [10_000]

    def __init__(self, data):
        from pinot_amd.segment import GpuSegment
        self.data, self.name, self.num_docs = data, data.name, data.num_docs
        HostSegment._next[0] += 1
        self.uid = HostSegment._next[0]
        self.slots = {c: i for i, c in enumerate(data.columns)}
        self.dictionaries = {c: data.columns[c].dictionary_values() for c in data.columns}
        self._gs = GpuSegment

    def column(self, name):
        return self.data.column(name)

    def group_view(self, name):
        return name  # dictionary-encoded columns only (no device to build an on-the-fly group dictionary)

    def sorted_dictionary(self, name):
        return self._gs.sorted_dictionary(self, name)

    def sorted_pairs(self, name):
        return self._gs.sorted_pairs(self, name)

    def min_max(self, name):
        return self._gs.min_max(self, name)


def _plan_maker():
    from pinot_amd.plan import GpuPlanMaker

    class HostPlanMaker(GpuPlanMaker):
        def set_global_dictionary(self, column, segments, glob):  # no remap buffers without a device
            self._global_dicts[(column, tuple(s.uid for s in segments))] = (glob, [None] * len(segments),
                                                                             tuple(segments))
            return glob, [None] * len(segments)

    return HostPlanMaker(ctx=None)


def _layout(query, segments, flags, reduce_docs, globs, sum_layout=None):
    """pgpu_table_layout_of restated (include/pinot_gpu.h), floating SUMs in fixed point (helpers.fixed_sum_layout;
    an agreed sum_layout = (exps, parts) taken verbatim)."""
    L = TableLayout()
    G = 1
    for g in query.group_by:
        G *= len(globs[g])
    L.num_keys = G
    ops = [PGPU_RED_SUM_I64]
    docs = max(sum(s.num_docs for s in segments), reduce_docs)
    for i, a in enumerate(query.aggregations):
        if a.function == "COUNT":
            L.agg_section[i], L.agg_value_type[i] = 0, -1
            continue
        vt = segments[0].column(a.column).data_type
        op = {"MIN": PGPU_RED_MIN_I64, "MAX": PGPU_RED_MAX_I64}.get(a.function, PGPU_RED_SUM_I64)
        parts = 1
        L.agg_sum_exp[i] = 0
        if op == PGPU_RED_SUM_I64 and vt not in (PGPU_INT, PGPU_LONG):
            vals = np.concatenate([np.asarray(s.dictionaries[a.column], dtype=np.float64) for s in segments])
            e, parts = fixed_sum_layout(vals)
            if sum_layout is not None:
                e, parts = sum_layout[0][i], sum_layout[1][i]
            if e == PGPU_SUM_EXP_F64 or parts > PGPU_MAX_FIXED_PARTS:
                op, e, parts = PGPU_RED_SUM_F64, PGPU_SUM_EXP_F64, 1
            L.agg_sum_exp[i] = e
        elif op == PGPU_RED_SUM_I64:
            mx = max(float(np.abs(s.dictionaries[a.column].astype(np.float64)).max()) for s in segments)
            parts = 3 if (flags & PGPU_Q_SUM_SPLIT) or mx * docs >= 2.0 ** 62 else 1
        L.agg_section[i], L.agg_value_type[i], L.agg_sum_parts[i] = len(ops), vt, parts
        ops += [op] * parts
    L.num_sections = len(ops)
    for k, o in enumerate(ops):
        L.section_op[k] = o
    return L


def _numpy_executor(pm):
    from oracle import engine
    from pinot_amd._lib import PGPU_KEYS_HASH, PGPU_Q_HASH
    from pinot_amd.combine import DistributedExecutor, minmax_key, section_identity

    class NumpyExecutor(DistributedExecutor):
        """The local kernel step in numpy: the table pgpu_query_launch leaves in HBM (dense cells indexed by the
        mixed-radix key, or -- PGPU_Q_HASH -- slots whose key words follow the sections)."""

        def _prepare_local(self, query, segments, flags, reduce_docs, sum_layout=None):
            flags |= self.pm.query_flags
            globs = self._globals_of(query, segments)
            L = _layout(query, segments, flags, reduce_docs, globs, sum_layout)
            ops = [L.section_op[k] for k in range(L.num_sections)]
            st = {"num_docs_scanned": 0, "num_entries_scanned_in_filter": 0, "num_total_docs": 0,
                  "num_segments_matched": 0, "sparse_sector_bytes": 0, "dense_bytes": 0, "kernel_ms": 0.0}
            per_seg = []
            for s in segments:
                ds = engine.DecodedSegment(s.data)
                op = engine.build_physical(ds, query.filter)
                docs = np.flatnonzero(engine.eval_mask(op, s.num_docs))
                st["num_docs_scanned"] += len(docs)
                st["num_segments_matched"] += int(len(docs) > 0)
                st["num_total_docs"] += s.num_docs
                st["num_entries_scanned_in_filter"] += engine.entries_scanned_in_filter(op, s.num_docs)[0]
                key = np.zeros(len(docs), dtype=np.int64)
                stride = 1
                for g in query.group_by:
                    glob = globs[g]
                    vals = ds.values(g)
                    if isinstance(glob, list):
                        pos = {v: i for i, v in enumerate(glob)}
                        gid = np.array([pos[vals[d]] for d in docs], dtype=np.int64)
                    else:
                        gid = np.searchsorted(glob, np.asarray(vals)[docs])
                    key += gid * stride
                    stride *= len(glob)
                per_seg.append((ds, docs, key))
            hashed = bool(query.group_by) and bool(flags & PGPU_Q_HASH)
            if hashed:  # slots: the distinct keys, in a table of a power-of-two slot count
                uniq = np.unique(np.concatenate([k for _, _, k in per_seg]))
                slots = 64
                while slots < 2 * len(uniq):
                    slots *= 2
                L.key_kind, L.key_words, L.num_keys = PGPU_KEYS_HASH, 1, slots
            G = int(L.num_keys)
            t = np.array([[section_identity(o)] * G for o in ops] + ([[-1] * G] if hashed else []), dtype=np.int64)
            if hashed:
                t[len(ops), : len(uniq)] = uniq
            for ds, docs, key in per_seg:
                cell = np.searchsorted(uniq, key) if hashed else key
                np.add.at(t[0], cell, 1)
                for i, a in enumerate(query.aggregations):
                    sec = L.agg_section[i]
                    if sec == 0:
                        continue
                    v = np.asarray(ds.values(a.column))[docs]
                    o = L.section_op[sec]
                    if o == PGPU_RED_SUM_I64:
                        if L.agg_value_type[i] not in (PGPU_INT, PGPU_LONG):  # fixed point: signed digits of |I|
                            P = L.agg_sum_parts[i]
                            digits = np.array([fixed_digits(float(x), L.agg_sum_exp[i], P) for x in v],
                                              dtype=np.int64).reshape(len(v), P)
                            for k in range(P):
                                np.add.at(t[sec + k], cell, digits[:, k])
                            continue
                        v = v.astype(np.int64)
                        if L.agg_sum_parts[i] == 3:
                            m = (1 << PGPU_PART_BITS) - 1
                            for k, part in enumerate((v & m, (v >> PGPU_PART_BITS) & m, v >> (2 * PGPU_PART_BITS))):
                                np.add.at(t[sec + k], cell, part)
                        else:
                            np.add.at(t[sec], cell, v)
                    elif o == PGPU_RED_SUM_F64:
                        np.add.at(t[sec].view(np.float64), cell, v.astype(np.float64))
                    else:
                        kv = np.array([minmax_key(float(x), L.agg_value_type[i]) for x in v], dtype=np.int64)
                        (np.minimum if o == PGPU_RED_MIN_I64 else np.maximum).at(t[sec], cell, kv)

            def launch(table):
                table.copy_(torch.from_numpy(t.reshape(-1)))
                return dict(st)
            return L, launch

        def _globals_of(self, query, segments):
            return {g: self.pm.global_dictionary(g, segments)[0] for g in query.group_by}

        def _wait_local(self, handle):
            return handle

        def _compact(self, L, table, order=None):  # every row: the host trim (_trim) then does the top-k
            rows = L.num_sections + (1 if L.key_kind == PGPU_KEYS_HASH else 0)
            t = table.cpu().numpy()[: rows * int(L.num_keys)].reshape(rows, int(L.num_keys))
            live = np.flatnonzero(t[0] > 0)
            keys = t[L.num_sections, live] if L.key_kind == PGPU_KEYS_HASH else live
            return keys.astype(np.int64), np.ascontiguousarray(t[: L.num_sections, live].T)

    return NumpyExecutor(pm, device=torch.device("cpu"))


def _rank_segments(rank, nseg=2, n=2500):
    from oracle.segment_writer import build_segment
    segs = []
    for k in range(nseg):
        rng = np.random.default_rng(100 * rank + k)
        names = [f"g{i:02d}" for i in range(rank * 5, rank * 5 + 20)]
        cols = {"g": (PGPU_STRING, [names[i] for i in rng.integers(0, len(names), n)]),
                "h": (PGPU_INT, (rng.integers(0, 300, n) * (rank + 1)).astype(np.int32)),
                "x": (PGPU_INT, rng.integers(0, 100, n).astype(np.int32)),
                "m": (PGPU_INT, rng.integers(-1000, 100000, n).astype(np.int32)),
                "big": (PGPU_LONG, rng.integers(9 * 10 ** 15, 10 ** 16, n).astype(np.int64)),
                "d": (PGPU_DOUBLE, np.round(rng.normal(50.0, 20.0, n), 3)),
                # rank-dependent magnitude: the ranks' fixed-point exponents differ until they agree on the max
                "e": (PGPU_DOUBLE, rng.normal(0.0, 10.0 ** (4 * rank), n))}
        segs.append(build_segment(f"r{rank}s{k}", cols))
    return segs


def _all_segments():
    return [s for r in range(WORLD) for s in _rank_segments(r)]


def _check(res, ref, q):
    from tests.helpers import close, rows_close
    assert res.stats.num_docs_scanned == ref.num_docs_scanned
    assert res.stats.num_entries_scanned_post_filter == ref.num_entries_scanned_post_filter
    assert res.stats.num_total_docs == ref.num_total_docs
    assert res.stats.num_segments_matched == ref.num_segments_matched
    if q.group_by:
        assert rows_close([list(r) for r in res.rows], [list(r) for r in ref.rows], 1e-9), (res.rows, ref.rows)
    else:
        assert all(close(a, b, 1e-9) for a, b in zip(res.aggregation_result, ref.aggregation_result)), \
            (res.aggregation_result, ref.aggregation_result)


QUERIES = [
    "SELECT g, SUM(m), MIN(m), MAX(d), AVG(d), COUNT(*) FROM t WHERE x < 60 GROUP BY g ORDER BY SUM(m) DESC LIMIT 7",
    "SELECT COUNT(*), SUM(m), MIN(d), MAX(m), AVG(m) FROM t WHERE x >= 30 AND x < 45",
    "SELECT g, h, COUNT(*), SUM(m) FROM t WHERE x < 90 GROUP BY g, h ORDER BY SUM(m) DESC, h LIMIT 15",
    "SELECT SUM(big), AVG(big), COUNT(*) FROM t WHERE x < 70",     # bound >= 2^62: split layout on every rank
    "SELECT COUNT(*), MIN(m), MAX(d) FROM t",                      # every segment answered without a scan
    "SELECT h, SUM(big), COUNT(*) FROM t GROUP BY h ORDER BY h LIMIT 20",
    "SELECT g, SUM(e), AVG(e), COUNT(*) FROM t GROUP BY g ORDER BY SUM(e) DESC LIMIT 9",  # agreed sum_exp
]


def _query_worker(rank, qi, scatter):
    from oracle import engine
    from pinot_amd.query import parse_sql
    q = parse_sql(QUERIES[qi])
    segs = [HostSegment(s) for s in _rank_segments(rank)]
    ex = _numpy_executor(_plan_maker())
    if scatter:
        ex.SCATTER_MIN_BYTES = 0  # every group-by table takes the reduce-scatter + top-K path
        ex.TOPK_MIN = 40          # and per-rank candidates are trimmed to max(5 * limit, 40) rows
    for rep in range(2):
        if rep == 1 and rank == 1:
            # a cache hit on rank 0 and a miss on rank 1 must still run the same collectives on both
            ex._globals.clear()
            ex._docs.clear()
            ex._split.clear()
            ex.pm._global_dicts.clear()
        res = ex.execute(q, segs)
        if rank == 0:
            ref = engine.execute(q, _all_segments())
            _check(res, ref, q)
            if qi == 4:  # NonScanBasedAggregationOperator statistics: (total, 0, 0, total) per segment
                assert res.stats.num_entries_scanned_post_filter == 0
        else:
            assert res is None
        st = ex.last_stats
        assert st is not None and st.num_total_docs == sum(s.num_docs for s in _all_segments())
        assert st.num_segments_processed == 2 * WORLD


@pytest.mark.parametrize("scatter", [False, True], ids=["allreduce", "scatter_topk"])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_distributed_executor_vs_oracle(qi, scatter):
    if scatter and "GROUP BY" not in QUERIES[qi]:
        pytest.skip("aggregation-only tables are always all-reduced")
    _spawn(_query_worker, qi, scatter)


@pytest.mark.parametrize("qi", [0, 2, 6])
def test_distributed_executor_three_ranks(qi):
    """World size 3: the reduce-scatter slices of ceil(G / 3) keys are uneven (the last rank's is short or empty),
    each rank trims its own slice, rank 0 gathers the candidates."""
    _spawn(_query_worker, qi, True, world=3)


def _split_agree_worker(rank):
    """Only rank 1 holds large values: the split-SUM layout must still be chosen on both ranks."""
    from oracle import engine
    from oracle.segment_writer import build_segment
    from pinot_amd.query import parse_sql
    rng = np.random.default_rng(5 + rank)
    n = 3000
    hi = 10 ** 16 if rank == 1 else 1000
    mk = lambda r, k: build_segment(f"a{r}{k}", {  # noqa: E731
        "v": (PGPU_LONG, np.random.default_rng(50 * r + k).integers(0, 10 ** 16 if r == 1 else 1000, n)
              .astype(np.int64)),
        "x": (PGPU_INT, np.random.default_rng(70 * r + k).integers(0, 10, n).astype(np.int32))})
    segs = [HostSegment(mk(rank, k)) for k in range(2)]
    ex = _numpy_executor(_plan_maker())
    q = parse_sql("SELECT SUM(v), COUNT(*) FROM t WHERE x < 7")
    assert hi  # rank-dependent magnitude
    res = ex.execute(q, segs)
    if rank == 0:
        allsegs = [mk(r, k) for r in range(WORLD) for k in range(2)]
        _check(res, engine.execute(q, allsegs), q)


def test_split_layout_agreed_across_ranks():
    _spawn(_split_agree_worker)


def _union_worker(rank):
    from pinot_amd.combine import union_dictionaries
    ints = [np.array([1, 5, 9], dtype=np.int32), np.array([2, 5, 11, 12], dtype=np.int32)][rank]
    np.testing.assert_array_equal(union_dictionaries(ints), [1, 2, 5, 9, 11, 12])
    strs = [["a", "null", "zz", "é"], ["b", "null"]][rank]
    assert union_dictionaries(strs) == ["a", "b", "null", "zz", "é"]
    dbl = [np.array([-0.5, 2.25]), np.array([], dtype=np.float64)][rank]
    np.testing.assert_array_equal(union_dictionaries(dbl), [-0.5, 2.25])
    empty = [[], ["q"]][rank]
    assert union_dictionaries(empty) == ["q"]


def test_union_dictionaries_tensor_collectives():
    _spawn(_union_worker)


def _hash_worker(rank, qi, force_on):
    """Hash tables merged across ranks by key ownership (all_to_all) and top-K; `force_on` = the ranks whose own
    flags ask for the hash layout -- the layout must still be the same on every rank."""
    from oracle import engine
    from pinot_amd._lib import PGPU_Q_HASH
    from pinot_amd.query import parse_sql
    q = parse_sql(QUERIES[qi])
    segs = [HostSegment(s) for s in _rank_segments(rank)]
    pm = _plan_maker()
    if rank in force_on:
        pm.query_flags = PGPU_Q_HASH
    ex = _numpy_executor(pm)
    ex.TOPK_MIN = 40
    res = ex.execute(q, segs)
    if rank == 0:
        _check(res, engine.execute(q, _all_segments()), q)


@pytest.mark.parametrize("force_on", [(0, 1), (1,)], ids=["all_ranks", "one_rank"])
@pytest.mark.parametrize("qi", [0, 2, 5])
def test_hash_tables_merge_by_key_ownership(qi, force_on):
    _spawn(_hash_worker, qi, force_on)


def test_hash_tables_merge_three_ranks():
    """World size 3: hash rows routed to three key owners (all_to_all with uneven splits)."""
    _spawn(_hash_worker, 2, (0, 1, 2), world=3)


LIMIT_SQL = "SELECT g, h, COUNT(*), SUM(m) FROM t WHERE x < 90 GROUP BY g, h ORDER BY SUM(m) DESC, g, h LIMIT 15"


def _limit_worker(rank, mode):
    """One rank's wait fails (numGroupsLimit passed by one of its segments, or a deadline), the other's succeeds:
    both must leave the collect together -- the first-seen path on every rank and rank 0 merging (`limit`), or the
    error on every rank (`timeout`) -- and the executor must stay usable for the next query."""
    from oracle import engine
    from pinot_amd import _lib
    from pinot_amd.plan import ExecutionStats, QueryResult
    from pinot_amd.query import parse_sql
    limit, thr = 300, 100  # map-based holders (key space 20 x 300 > 100) that really pass 300 keys per segment
    q = parse_sql(LIMIT_SQL)
    segs = [HostSegment(s) for s in _rank_segments(rank)]
    pm = _plan_maker()
    pm.num_groups_limit, pm.max_init_group_holder_capacity = limit, thr

    def first_seen(query, segments):  # GpuPlanMaker.first_seen_groups restated by the oracle (no device here)
        ref = engine.execute(query, [s.data for s in segments], num_groups_limit=limit,
                             max_init_group_holder_capacity=thr)
        st = ExecutionStats(num_docs_scanned=ref.num_docs_scanned, num_total_docs=ref.num_total_docs,
                            num_entries_scanned_post_filter=ref.num_entries_scanned_post_filter,
                            num_segments_processed=len(segments), num_segments_matched=ref.num_segments_matched,
                            num_groups_limit_reached=ref.num_groups_limit_reached)
        r = QueryResult(query=query, stats=st)
        r._intermediate = ref.intermediate
        return r

    pm.first_seen_groups = first_seen
    ex = _numpy_executor(pm)
    plain_wait = ex._wait_local

    def failing_wait(handle):
        if rank == 1:
            cls = _lib.GroupsLimitError if mode == "limit" else _lib.QueryTimeoutError
            raise cls(_lib.PGPU_E_GROUPS_LIMIT if mode == "limit" else _lib.PGPU_E_TIMEOUT, "rank 1 only")
        return plain_wait(handle)

    ex._wait_local = failing_wait
    if mode == "limit":
        res = ex.execute(q, segs)
        if rank == 0:
            ref = engine.execute(q, _all_segments(), num_groups_limit=limit, max_init_group_holder_capacity=thr)
            full = engine.execute(q, _all_segments(), num_groups_limit=10 ** 9)
            assert len(ref.group_rows) < len(full.group_rows)  # the limit really truncates
            assert res.rows == ref.rows
            assert res.stats.num_docs_scanned == ref.num_docs_scanned
            assert res.stats.num_groups_limit_reached and ref.num_groups_limit_reached
            assert res.stats.num_segments_matched == ref.num_segments_matched == 2 * WORLD
        else:
            assert res is None
    else:
        with pytest.raises(_lib.PinotGpuError):
            ex.execute(q, segs)
    # the collectives are still in step: the next query runs normally on both ranks
    ex._wait_local = plain_wait
    q2 = parse_sql("SELECT COUNT(*), SUM(m) FROM t WHERE x < 50")
    res = ex.execute(q2, segs)
    if rank == 0:
        _check(res, engine.execute(q2, _all_segments()), q2)


@pytest.mark.parametrize("mode", ["limit", "timeout"])
def test_failure_on_one_rank_agreed(mode):
    _spawn(_limit_worker, mode)
