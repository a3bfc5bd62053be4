"""tools/bytemodel.py: bench.py's workload byte model on CPU.

The model regenerates the synthetic dict ids with torch and walks the reference's filter tree; its matched-doc
count must equal the oracle's on the same segments, and its bytes must follow the 8(d) definition: the first AND
child streamed whole, later children and the aggregated columns as 32-B sectors of the surviving docs."""
import numpy as np
import pytest
import torch

from oracle import engine
from oracle.segment_writer import pack_fixed_bit
from pinot_amd.predicate import SortedDictionary
from pinot_amd.query import parse_sql
from pinot_amd.synth import WORKLOADS, build_segment_cpu, dict_ids_cpu, zipf_cdf
from tools.bytemodel import dict_ids_torch, sector_bytes, workload_bytes


class HostSegment:
    """The planner's view of a segment (column / sorted_dictionary / sorted_pairs) over host SegmentData."""

    def __init__(self, data):
        self.data, self.num_docs = data, data.num_docs

    def column(self, name):
        return self.data.column(name)

    def sorted_dictionary(self, name):
        c = self.column(name)
        return SortedDictionary(c.dictionary_values(), c.data_type, pad_char=c.pad_char, entry_width=c.entry_width)

    def sorted_pairs(self, name):
        return np.frombuffer(self.column(name).sorted_index, dtype=">i4").reshape(-1, 2).astype(np.int64)


@pytest.mark.parametrize("card,zipf", [(1024, False), (1 << 20, False), (1 << 20, True), (16, False)])
def test_ids_match_numpy_restatement(card, zipf):
    cdf = zipf_cdf(card, 1.1) if zipf else None
    for seed in (5, 0xFFFFFFFFFFFFFFFD, 1234567890123):
        a = dict_ids_cpu(seed, 50_000, card, cdf=cdf, doc0=12345)
        b = dict_ids_torch(seed, 50_000, card, "cpu", cdf=cdf, doc0=12345).numpy()
        assert np.array_equal(a, b)


def test_sector_bytes_counts_straddling_values():
    m = torch.zeros(1000, dtype=torch.bool)
    m[[0, 13, 14, 500]] = True       # 20-bit values: sectors 0, 1 (docs 13 and 14 share it), 39
    assert sector_bytes(m, 20) == 3 * 32
    m = torch.zeros(1000, dtype=torch.bool)
    m[12] = True                     # bits 240..259: straddles sectors 0 and 1
    assert sector_bytes(m, 20) == 2 * 32
    assert sector_bytes(torch.zeros(10, dtype=torch.bool), 16) == 0


# a looser config-5 filter so that the accountId leaf keeps docs at this size
CASES = [("adanalytics", None), ("adanalytics", ("accountId IN (123456789)", "accountId < 123456789")),
         ("range_in", None), ("groupby1m", None), ("bitmap5", None)]


@pytest.mark.parametrize("name,variant", CASES)
def test_model_matches_oracle(name, variant):
    w = WORKLOADS[name]
    n = 1 << 16
    sql = w.sql if variant is None else w.sql.replace(*variant)
    q = parse_sql(sql)
    datas = [build_segment_cpu(w, s, n, pack_fixed_bit) for s in range(2)]
    total, parts, matched = workload_bytes(w, q, [HostSegment(d) for d in datas], n, [0, 1], "cpu", ngroups=3)
    ref = engine.execute(sql, datas)
    assert matched == ref.num_docs_scanned
    assert total == sum(parts.values())
    assert parts["output"] == 8 * 3 * (1 + len(q.aggregations))
    if name == "groupby1m":  # no filter: both columns streamed whole
        assert parts["forward_full"] == 2 * (n * 20 // 8 + n * 16 // 8) and parts["forward_sectors"] == 0
    if name.startswith("adanalytics"):  # the day column (10-bit, first AND child) streamed whole, the rest sectors
        assert parts["forward_full"] == 2 * n * 10 // 8
        assert 0 < parts["forward_sectors"] < 2 * n * 20 // 8
    if name == "bitmap5":  # index-only filter: bitmaps + sorted pairs, metrics as sectors
        assert parts["forward_full"] == 0 and parts["inverted_bitmaps"] > 0 and parts["sorted_pairs"] > 0
