"""Hash group-by (include/pinot_gpu.h PGPU_KEYS_HASH) and the group-key holder limits, GPU vs oracle (MI355X only).

The reference picks a holder per segment from its cardinality product (DictionaryBasedGroupKeyGenerator.java:
100-170): array (<= max.init.group.holder.capacity), IntMap (<= 2^31), LongMap (<= 2^63), ArrayMap (beyond);
map holders stop at num.groups.limit distinct keys, keeping the first-seen ones.  The GPU keys any space by hash
slots and counts the distinct keys of every segment that could pass the limit; a segment that really does keeps its
first-seen keys (GpuPlanMaker.first_seen_groups: MIN over the doc-id column per group, then the limit smallest)."""
import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import build_segment
from pinot_amd._lib import PGPU_DOUBLE, PGPU_INT, PGPU_KEYS_DENSE, PGPU_KEYS_HASH, PGPU_LONG, PGPU_Q_HASH, \
    PGPU_STRING, GroupsLimitError, UnsupportedPlanError
from pinot_amd.plan import GpuPlanMaker
from pinot_amd.query import parse_sql
from pinot_amd.segment import GpuSegment
from tests.helpers import check_groups, rows_close

pytestmark = pytest.mark.gpu


def _run(gpu_ctx, sql, segs, **kw):
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        pm = GpuPlanMaker(gpu_ctx, **kw)
        q = parse_sql(sql)
        desc, keep, _ = pm.build_desc(q, gs)
        layout = pm.layout(desc)
        return pm.execute(q, gs), layout
    finally:
        for g in gs:
            g.release()


def _same(res, ref):
    check_groups(res, ref, 1e-9)
    if res.query.order_by:  # without ORDER BY the LIMIT keeps arbitrary groups (in the reference too)
        assert rows_close([list(r) for r in res.rows], [list(r) for r in ref.rows], 1e-9)
    assert res.stats.num_docs_scanned == ref.num_docs_scanned


def _sparse_pairs(rng, n, name, card_a=1000, card_b=1000, groups=1000):
    """Two group columns of 1000 values each (key space 10^6) whose docs use only ~`groups` (a, b) pairs."""
    pa = rng.integers(0, card_a, groups)
    pb = rng.integers(0, card_b, groups)
    pick = rng.integers(0, groups, n)
    a = (np.concatenate([np.arange(card_a), pa[pick]]) * 7).astype(np.int32)[: max(n, card_a)]
    b = (np.concatenate([np.arange(card_b), pb[pick]]) * 3 + 1).astype(np.int32)[: max(n, card_b)]
    m = rng.integers(-500, 100_000, len(a)).astype(np.int32)
    f = rng.integers(0, 100, len(a)).astype(np.int32)
    return build_segment(name, {"a": (PGPU_INT, a), "b": (PGPU_INT, b), "m": (PGPU_INT, m), "f": (PGPU_INT, f)})


@pytest.mark.parametrize("sql", [
    "SELECT a, b, COUNT(*), SUM(m), MAX(m) FROM t GROUP BY a, b ORDER BY SUM(m) DESC LIMIT 25",
    "SELECT a, b, AVG(m), MIN(m) FROM t WHERE f < 40 GROUP BY a, b ORDER BY a, b LIMIT 40",
])
def test_sparse_key_space_runs_on_gpu(gpu_ctx, sql):
    """10^6-key space, ~1000 real groups per segment: hash slots, not a 10^6-cell dense table."""
    rng = np.random.default_rng(3)
    segs = [_sparse_pairs(rng, 200_000, f"sp{i}") for i in range(3)]
    res, layout = _run(gpu_ctx, sql, segs)
    # slots sized by the holders' bound (3 segments x numGroupsLimit 100,000), not by the 10^6 key space
    assert layout.key_kind == PGPU_KEYS_HASH and layout.num_keys == 1 << 20
    _same(res, engine.execute(parse_sql(sql), segs))
    res, layout = _run(gpu_ctx, sql, segs, num_groups_limit=20_000)
    assert layout.key_kind == PGPU_KEYS_HASH and layout.num_keys == 1 << 17
    _same(res, engine.execute(parse_sql(sql), segs, num_groups_limit=20_000))


def _random(rng, n, name, cards):
    cols = {}
    for c, card in cards.items():
        base = np.sort(rng.choice(np.arange(card * 4, dtype=np.int64), size=card, replace=False))
        cols[c] = (PGPU_INT, base[rng.integers(0, card, n)].astype(np.int32))
    cols["s"] = (PGPU_STRING, [f"v{x}" for x in rng.integers(0, 50, n)])
    cols["m"] = (PGPU_LONG, rng.integers(-10 ** 9, 10 ** 12, n).astype(np.int64))
    cols["d"] = (PGPU_DOUBLE, np.round(rng.normal(0, 100, n), 4))
    return build_segment(name, cols)


FORCED = [
    "SELECT x, COUNT(*), SUM(m), MIN(d), MAX(m), AVG(d) FROM t GROUP BY x",
    "SELECT x, y, s, COUNT(*), SUM(m) FROM t WHERE z < 300 GROUP BY x, y, s ORDER BY SUM(m) DESC LIMIT 50",
    "SELECT s, z, SUM(d), COUNT(*) FROM t WHERE x > 20 AND y <> 3 GROUP BY s, z",
    "SELECT y, COUNT(*) FROM t WHERE s IN ('v1', 'v7', 'v19') GROUP BY y",
]


@pytest.mark.parametrize("qi", range(len(FORCED)))
def test_forced_hash_vs_oracle(gpu_ctx, qi):
    """PGPU_Q_HASH on key spaces the dense table would serve: identical results through the slot path."""
    rng = np.random.default_rng(60 + qi)
    segs = [_random(rng, n, f"h{i}", {"x": 37, "y": 9, "z": 900}) for i, n in enumerate([150_001, 4097, 64_000])]
    res, layout = _run(gpu_ctx, FORCED[qi], segs, query_flags=PGPU_Q_HASH)
    assert layout.key_kind == PGPU_KEYS_HASH
    _same(res, engine.execute(parse_sql(FORCED[qi]), segs))


def test_long_map_and_array_map_key_spaces(gpu_ctx):
    """Key spaces above 2^31 (one key word) and above 2^63 (two key words, ArrayMapBasedHolder)."""
    rng = np.random.default_rng(17)
    n = 60_000
    cards = {"c1": 60_000, "c2": 50_000, "c3": 40_000, "c4": 30_000, "c5": 70}
    segs = [_random(rng, n, f"w{i}", cards) for i in range(2)]
    for sql, words in [("SELECT c1, c2, COUNT(*), SUM(m) FROM t GROUP BY c1, c2 ORDER BY SUM(m) DESC LIMIT 30", 1),
                       ("SELECT c1, c2, c3, c4, c5, COUNT(*), MAX(d) FROM t WHERE c5 < 150 "
                        "GROUP BY c1, c2, c3, c4, c5 ORDER BY MAX(d) DESC LIMIT 30", 2)]:
        res, layout = _run(gpu_ctx, sql, segs, num_groups_limit=1_000_000)
        assert layout.key_kind == PGPU_KEYS_HASH and layout.key_words == words
        _same(res, engine.execute(parse_sql(sql), segs, num_groups_limit=1_000_000))


def test_group_limit_counts_actual_keys(gpu_ctx):
    """Key space above numGroupsLimit, but fewer real groups: served on the GPU (exact, like the reference);
    a segment that really meets more than the limit declines the query."""
    rng = np.random.default_rng(23)
    small = [_sparse_pairs(rng, 100_000, f"g{i}", groups=800) for i in range(2)]
    sql = "SELECT a, b, SUM(m), COUNT(*) FROM t GROUP BY a, b ORDER BY SUM(m) DESC LIMIT 10"
    res, layout = _run(gpu_ctx, sql, small, num_groups_limit=5_000)
    assert layout.key_kind == PGPU_KEYS_HASH
    _same(res, engine.execute(parse_sql(sql), small, num_groups_limit=5_000))
    # ~1800 distinct pairs per segment (1000 seed pairs + 800): above a limit of 1,500.  The launch reports it
    # (PGPU_E_GROUPS_LIMIT, a GroupsLimitError to submit / collect callers); execute() keeps every such segment's
    # first-seen 1,500 keys like the reference's holders (GpuPlanMaker.first_seen_groups)
    big = small + [_sparse_pairs(rng, 100_000, "g9", groups=800)]
    gs = [GpuSegment(gpu_ctx, s) for s in big]
    try:
        pm = GpuPlanMaker(gpu_ctx, num_groups_limit=1_500)
        with pytest.raises(GroupsLimitError, match="numGroupsLimit"):
            pm.collect(pm.submit(parse_sql(sql), gs))
        res = pm.execute(parse_sql(sql), gs)
    finally:
        for g in gs:
            g.release()
    ref = engine.execute(parse_sql(sql), big, num_groups_limit=1_500)
    assert len(res.group_rows) == len(ref.group_rows) < 3 * 1_800
    _same(res, ref)
    assert res.stats.num_entries_scanned_post_filter == ref.num_entries_scanned_post_filter


@pytest.mark.parametrize("sql,limit", [
    # one group column of 30,000 values (IntMapBasedHolder), filtered: docs of dropped keys are not aggregated
    ("SELECT k, COUNT(*), SUM(m), MIN(m), AVG(m) FROM t WHERE f < 70 GROUP BY k ORDER BY COUNT(*) DESC, k LIMIT 20",
     2_000),
    # two columns, ordered by MAX (ties broken by the keys: the reference leaves tie order to its table)
    ("SELECT k, f, MAX(m), COUNT(*) FROM t GROUP BY k, f ORDER BY MAX(m) DESC, k, f LIMIT 15", 7_000),
    # a raw (no-dictionary) group column: NoDictionarySingleColumnGroupKeyGenerator caps at the limit too
    ("SELECT r, COUNT(*), SUM(m) FROM t GROUP BY r ORDER BY SUM(m) DESC, r LIMIT 10", 3_000),
])
def test_first_seen_truncation_at_num_groups_limit(gpu_ctx, sql, limit):
    """Segments beyond numGroupsLimit keep their first-seen keys (smallest first doc), the others all of theirs;
    the merged result equals the reference's (oracle: DictionaryBasedGroupKeyGenerator's first-seen group ids)."""
    rng = np.random.default_rng(31)
    segs = []
    for i, (n, card) in enumerate([(40_000, 30_000), (25_000, 30_000), (8_000, 500)]):
        k = np.concatenate([np.arange(card), rng.integers(0, card, n - card if n > card else 0)])[:n]
        rng.shuffle(k)
        cols = {"k": (PGPU_INT, (k * 5 + 2).astype(np.int32)), "f": (PGPU_INT, rng.integers(0, 100, n)),
                "m": (PGPU_INT, rng.integers(-1000, 50_000, n)), "r": (PGPU_LONG, rng.integers(0, 9_000, n) * 11)}
        segs.append(build_segment(f"fs{i}", cols, sorted_columns=(), raw=("r",)))
    q = parse_sql(sql)
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    try:
        res = GpuPlanMaker(gpu_ctx, num_groups_limit=limit).execute(q, gs)
    finally:
        for g in gs:
            g.release()
    ref = engine.execute(q, segs, num_groups_limit=limit)
    full = engine.execute(q, segs, num_groups_limit=10 ** 9)
    assert len(ref.group_rows) < len(full.group_rows)  # the limit really truncates
    _same(res, ref)
    assert res.stats.num_groups_limit_reached
    assert res.stats.num_entries_scanned_post_filter == ref.num_entries_scanned_post_filter


def test_dense_layout_kept_for_dense_key_spaces(gpu_ctx):
    rng = np.random.default_rng(8)
    segs = [_random(rng, 100_000, "dd", {"x": 37, "y": 9, "z": 900})]
    res, layout = _run(gpu_ctx, "SELECT x, y, COUNT(*) FROM t GROUP BY x, y", segs)
    assert layout.key_kind == PGPU_KEYS_DENSE and layout.num_keys == 37 * 9
