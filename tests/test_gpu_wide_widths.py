"""Query-path bit widths 22..31 against the oracle (FixedBitIntReader.java:52-117, PinotDataBitSet.java:59-165).

The widest columns of the other GPU tests hold 21 bits.  Here a column `w` gets a dictionary of 2^(b-1) + 1 INT
values, so that PinotDataBitSet.getNumBitsPerValue(cardinality - 1) = b, while the segments keep few docs: the
dict ids are packed directly (FixedBitSVForwardIndexWriter layout, oracle/segment_writer.pack_fixed_bit) instead
of being derived from a value column, with the extreme ids (0, 2^(b-1) - 1, 2^(b-1), card - 1) always present.
The queries put `w` through every consumer of the unpacker: a RANGE / IN / NOT IN filter leaf (bit-sliced or
staged scan), sparse candidate gathers (SUM / MIN / MAX of w under a selective filter), the ring kernel's dense
decode (an unfiltered GROUP BY over every doc) and the hash group-by with `w` as the key.  Doc counts, counts,
integer sums and MIN / MAX are bit-exact (integer data), and so is numEntriesScannedInFilter where the GPU
reports the reference's figure.
"""
import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import bits_per_value, dictionary_bytes, pack_fixed_bit
from pinot_amd._lib import PGPU_INT
from pinot_amd.plan import GpuPlanMaker
from pinot_amd.query import parse_sql
from pinot_amd.segment import ColumnIndexes, GpuSegment, SegmentData
from tests.helpers import check_groups, close

pytestmark = pytest.mark.gpu

WIDTHS = [22, 24, 27, 31]


def _dict_values(card: int) -> np.ndarray:
    step = 2 if 2 * card + 1 < (1 << 31) else 1
    return np.arange(card, dtype=np.int64).astype(np.int32) * step + (1 if step == 2 else 0)


def _segment(name: str, rng, n: int, bits: int, wdict_be: bytes):
    card = (1 << (bits - 1)) + 1
    assert bits_per_value(card) == bits
    ids = rng.integers(0, card, n, dtype=np.int64)
    edge = np.array([0, (1 << (bits - 1)) - 1, 1 << (bits - 1), card - 1, card - 2, 1], dtype=np.int64)
    pos = rng.choice(n, size=4 * len(edge), replace=False)
    ids[pos] = np.resize(edge, len(pos))
    seg = SegmentData(name, n)
    seg.columns["w"] = ColumnIndexes("w", PGPU_INT, card, dictionary=wdict_be, forward=pack_fixed_bit(ids, bits))
    k = rng.integers(0, 10, n)
    seg.columns["k"] = ColumnIndexes("k", PGPU_INT, 10, dictionary=dictionary_bytes(np.arange(10) * 5, PGPU_INT),
                                     forward=pack_fixed_bit(k, bits_per_value(10)))
    m = rng.integers(0, 4096, n)
    seg.columns["m"] = ColumnIndexes("m", PGPU_INT, 4096,
                                     dictionary=dictionary_bytes(np.arange(4096) * 7 - 9000, PGPU_INT),
                                     forward=pack_fixed_bit(m, bits_per_value(4096)))
    return seg


@pytest.fixture(scope="module", params=WIDTHS, ids=lambda b: f"{b}bit")
def wide(request, gpu_ctx):
    bits = request.param
    card = (1 << (bits - 1)) + 1
    vals = _dict_values(card)
    be = dictionary_bytes(vals, PGPU_INT)
    rng = np.random.default_rng(bits)
    segs = [_segment(f"w{bits}_{i}", rng, n, bits, be) for i, n in enumerate([60_001, 4097])]
    del be
    gs = [GpuSegment(gpu_ctx, s) for s in segs]
    yield bits, vals, segs, gs
    for g in gs:
        g.release()


def _queries(vals: np.ndarray):
    card = len(vals)
    v = lambda i: int(vals[i])  # noqa: E731
    q1, q3 = card // 4, (3 * card) // 4
    half = 1 << (card - 1).bit_length() - 1
    return [
        f"SELECT COUNT(*), SUM(m) FROM t WHERE w BETWEEN {v(q1)} AND {v(q3)}",
        f"SELECT COUNT(*), SUM(m), MAX(m) FROM t WHERE w >= {v(half)}",
        f"SELECT COUNT(*), SUM(w), MIN(w), MAX(w) FROM t WHERE w IN ({v(0)}, {v(card - 1)}, {v(half - 1)}, "
        f"{v(half)}, {v(1)})",
        f"SELECT COUNT(*), SUM(w), MIN(w), MAX(w) FROM t WHERE k = 15 AND w < {v(q1)}",
        f"SELECT COUNT(*), SUM(m) FROM t WHERE w NOT IN ({v(0)}, {v(card - 1)}) AND k <> 20",
        f"SELECT COUNT(*), SUM(w) FROM t WHERE w > {v(q3)} OR k IN (5, 35) OR m < 0",
        "SELECT k, COUNT(*), SUM(w), MIN(w), MAX(w) FROM t GROUP BY k",
        f"SELECT k, SUM(w), MAX(w) FROM t WHERE w BETWEEN {v(q1)} AND {v(card - 1)} GROUP BY k",
    ]


@pytest.mark.parametrize("qi", range(8))
def test_wide_width_queries_vs_oracle(gpu_ctx, wide, qi):
    bits, vals, segs, gs = wide
    q = parse_sql(_queries(vals)[qi])
    res = GpuPlanMaker(gpu_ctx).execute(q, gs)
    ref = engine.execute(q, segs, iterator_stats=True)
    if res.aggregation_result is not None:
        assert len(res.aggregation_result) == len(ref.aggregation_result)
        for a, b in zip(res.aggregation_result, ref.aggregation_result):
            assert a == b, (bits, qi, res.aggregation_result, ref.aggregation_result)  # integer data: exact
    else:
        check_groups(res, ref, 0.0)
    assert res.stats.num_docs_scanned == ref.num_docs_scanned
    assert res.stats.num_entries_scanned_post_filter == ref.num_entries_scanned_post_filter
    if res.stats.filter_stats_exact:
        assert res.stats.num_entries_scanned_in_filter == ref.num_entries_scanned_in_filter


def test_wide_width_group_by_wide_key(gpu_ctx, wide):
    """GROUP BY the wide column itself (a key space of 2^(b-1) + 1: the hash group-by's one-word keys) on one
    segment, so the global dictionary is the segment's own."""
    bits, vals, segs, gs = wide
    q = parse_sql("SELECT w, COUNT(*), SUM(m) FROM t WHERE k = 25 GROUP BY w")
    res = GpuPlanMaker(gpu_ctx, num_groups_limit=1_000_000).execute(q, gs[:1])
    ref = engine.execute(q, segs[:1], num_groups_limit=1_000_000)
    check_groups(res, ref, 0.0)
    assert res.stats.num_docs_scanned == ref.num_docs_scanned
    assert close(len(res.group_rows), len(ref.group_rows), 0.0)
