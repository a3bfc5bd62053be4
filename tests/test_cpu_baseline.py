"""The timed CPU baseline (oracle/pinot_cpu.c through oracle/cpu.py) against the oracle engine: the same doc sets,
aggregations and numEntriesScannedInFilter on the bench workloads and on random filter trees over scan, inverted
(Roaring) and sorted leaves.  CPU only."""
import os

import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import build_segment, pack_fixed_bit
from pinot_amd._lib import PGPU_INT
from pinot_amd.query import parse_sql
from pinot_amd.synth import WORKLOADS, build_segment_cpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "libpinot_cpu.so")),
                                reason="oracle/libpinot_cpu.so not built")


def _check(q, segs, check_scanned=True):
    from oracle.cpu import CpuBaseline

    cb = CpuBaseline(q, segs)
    _, matched, counts, sums, scanned = cb.run(2)
    ref = engine.execute(q, segs, num_groups_limit=10 ** 9, iterator_stats=True)
    assert matched == ref.num_docs_scanned
    if check_scanned:
        assert scanned == ref.num_entries_scanned_in_filter
    if not q.group_by:
        for i, a in enumerate(q.aggregations):
            want = ref.intermediate[()][i]
            if a.function == "COUNT":
                assert counts[0] == want
            elif a.function == "AVG":
                assert sums[i][0] == pytest.approx(float(want[0]), rel=1e-12)
            elif matched:
                assert sums[i][0] == pytest.approx(float(want), rel=1e-12)
    return cb, matched


@pytest.mark.parametrize("name", ["bitmap5", "range_in", "adanalytics_inv"])
def test_workloads_match_oracle(name):
    w = WORKLOADS[name]
    from oracle.cpu import synth_segment

    segs = [synth_segment(w, s, 1 << 16) for s in range(2)]
    # the C twin writes the same bytes as the host builder
    ref_seg = build_segment_cpu(w, 1, 1 << 16, pack_fixed_bit)
    for c in w.columns:
        a, b = segs[1].column(c.name), ref_seg.column(c.name)
        assert (a.forward, a.inverted, a.sorted_index) == (b.forward, b.inverted, b.sorted_index)
    q = parse_sql(w.sql)
    cb, _ = _check(q, segs, check_scanned=True)
    kinds = {"bitmap5": "OR", "range_in": None, "adanalytics_inv": "AND"}[name]
    assert (cb.q.num_nodes > 0) == (kinds is not None)


def test_bitmap5_loose_variant_matches_rows():
    w = WORKLOADS["bitmap5"]
    from oracle.cpu import synth_segment

    segs = [synth_segment(w, s, 1 << 16) for s in range(2)]
    q = parse_sql("SELECT COUNT(*), SUM(m1), MIN(m2), MAX(m2) FROM bitmap5 "
                  "WHERE (a = 10 OR b IN (30, 70)) AND NOT (c = 50 AND d <> 90) AND e BETWEEN 640 AND 1910")
    _, matched = _check(q, segs)
    assert matched > 1000


def _random_filter(rng, depth=0):
    cols = {"s": 50, "inv": 40, "srt": 30}
    if depth >= 2 or rng.random() < 0.35:
        c = rng.choice(list(cols))
        v = int(rng.integers(0, cols[c]))
        kind = rng.integers(0, 4)
        if kind == 0:
            return f"{c} = {v}"
        if kind == 1:
            return f"{c} <> {v}"
        if kind == 2:
            return f"{c} IN ({v}, {(v + 7) % cols[c]}, {(v + 3) % cols[c]})"
        return f"{c} BETWEEN {v} AND {v + int(rng.integers(0, 20))}"
    op = rng.choice(["AND", "OR", "NOT"])
    if op == "NOT":
        return f"NOT ({_random_filter(rng, depth + 1)})"
    kids = [_random_filter(rng, depth + 1) for _ in range(int(rng.integers(2, 4)))]
    return "(" + f" {op} ".join(kids) + ")"


@pytest.mark.parametrize("seed", range(12))
def test_random_trees_match_oracle(seed):
    rng = np.random.default_rng(seed)
    n = 70_000 + seed * 977  # ragged: more than one 64K Roaring container, partial last word
    cols = {"s": (PGPU_INT, rng.integers(0, 50, n)),
            "inv": (PGPU_INT, rng.integers(0, 40, n)),
            "srt": (PGPU_INT, np.sort(rng.integers(0, 30, n))),
            "m": (PGPU_INT, rng.integers(0, 1000, n) * 3)}
    seg = build_segment(f"t{seed}", cols, inverted=["inv"], sorted_columns=["srt"], allow_runs=bool(seed % 2))
    f = _random_filter(rng)
    q = parse_sql(f"SELECT COUNT(*), SUM(m), MAX(m) FROM t WHERE {f}")
    # nested AND-of-scans inside an OR / NOT leap-frog in the reference; the C port scans them with applyAnd, so
    # only the doc set and the aggregates are compared there
    _check(q, [seg], check_scanned=False)


def test_group_by_tree():
    rng = np.random.default_rng(5)
    n = 50_000
    cols = {"g": (PGPU_INT, rng.integers(0, 7, n)),
            "inv": (PGPU_INT, rng.integers(0, 20, n)),
            "m": (PGPU_INT, rng.integers(0, 100, n))}
    seg = build_segment("g", cols, inverted=["inv"], sorted_columns=[])
    q = parse_sql("SELECT g, COUNT(*), SUM(m) FROM t WHERE inv IN (1, 2, 3) OR m < 10 GROUP BY g")
    from oracle.cpu import CpuBaseline

    _, matched, counts, sums, _ = CpuBaseline(q, [seg]).run(1)
    ref = engine.execute(q, [seg])
    got = {(int(k),): (int(counts[k]), float(sums[1][k])) for k in range(7) if counts[k]}
    want = {r[:1]: (r[1], r[2]) for r in ref.group_rows}
    assert got.keys() == want.keys()
    for k in got:
        assert got[k][0] == want[k][0] and got[k][1] == pytest.approx(want[k][1])


def test_zipf_generator_and_group_by_match_oracle():
    """The C generator's Zipf(1.1) keys (the CDF search of synth.hip's synth_id) write the host builder's bytes,
    and the C port's GROUP BY over them matches the oracle (config 4's skewed variant, timed by bench.py)."""
    w = WORKLOADS["groupby1m_zipf"]
    from oracle.cpu import CpuBaseline, synth_segment

    segs = [synth_segment(w, s, 1 << 16) for s in range(2)]
    ref_seg = build_segment_cpu(w, 1, 1 << 16, pack_fixed_bit)
    for c in w.columns:
        assert segs[1].column(c.name).forward == ref_seg.column(c.name).forward
    q = parse_sql("SELECT k, SUM(m), COUNT(*) FROM synth WHERE m < 500000 GROUP BY k")
    _, matched, counts, sums, _ = CpuBaseline(q, segs).run(2)
    ref = engine.execute(q, segs, num_groups_limit=10 ** 9)
    assert matched == ref.num_docs_scanned
    keys = w.columns[0].values()
    got = {(int(keys[k]),): (int(counts[k]), float(sums[0][k])) for k in np.flatnonzero(counts)}
    want = {r[:1]: (r[2], r[1]) for r in ref.group_rows}
    assert got.keys() == want.keys()
    for k in got:
        assert got[k][0] == want[k][0] and got[k][1] == pytest.approx(want[k][1], rel=1e-12)
