"""Synthetic segment sets for the BASELINE workloads (bench.py and the GPU tests).

Dictionary values are generated on the host (small); forward indexes are generated directly in HBM by
libpinotgpu_synth.so and uploaded with ``pgpu_segment_add_forward_index(..., PGPU_MEM_DEVICE)``.  Every dict id is a
counter-based hash of (seed, doc) that ``dict_ids_cpu`` restates in numpy, so any generated segment can be rebuilt
bit-identically on the CPU (parity tests, CPU baseline).

Workloads (one GPU's shard, weak scaling: rank r owns global segments r*S .. r*S+S-1):
  adanalytics  config 5  daysSinceEpoch 10-bit, accountId 20-bit, clicks / impressions 16-bit metric dicts
  range_in     config 2  r 16-bit, i 4-bit, m 16-bit metric
  groupby1m    config 4  k 20-bit (1,048,576 keys), m 16-bit metric
  bitmap5      config 3  a/b/c/d inverted-indexed (card 4 / 16 / 64 / 256: bitmap, borderline, array, array
                         containers), e sorted (card 256: doc ranges), m1 / m2 16-bit metrics
"""
from __future__ import annotations

import ctypes as C
import os
import dataclasses
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

from ._lib import PGPU_INT, SYNTH_LIB_PATH
from .segment import ColumnIndexes, GpuContext, GpuSegment, SegmentData, num_bits_per_value

M64 = (1 << 64) - 1


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15))
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def dict_ids_cpu(seed: int, num_docs: int, card: int, doc0: int = 0, cdf: Optional[np.ndarray] = None) -> np.ndarray:
    """numpy restatement of synth.hip's synth_id for docs [doc0, doc0 + num_docs)."""
    with np.errstate(over="ignore"):
        docs = np.arange(doc0, doc0 + num_docs, dtype=np.uint64)
        u = (splitmix64_np(np.uint64(seed) ^ (docs * np.uint64(0xD1B54A32D192ED03))) >> np.uint64(32))
    if cdf is None:
        return ((u * np.uint64(card)) >> np.uint64(32)).astype(np.int32)
    return np.searchsorted(cdf.astype(np.uint64), u, side="right").astype(np.int32)


def column_seed(base: int, segment: int, column: str) -> int:
    h = base
    for ch in column.encode():
        h = splitmix64((h * 131 + ch) & M64)
    return splitmix64((h ^ (segment * 0x9E3779B97F4A7C15)) & M64)


def zipf_cdf(card: int, s: float) -> np.ndarray:
    """uint32 CDF table (scaled to 2^32) of a Zipf(s) distribution over ranks 0..card-1."""
    w = 1.0 / np.power(np.arange(1, card + 1, dtype=np.float64), s)
    c = np.cumsum(w)
    c /= c[-1]
    t = np.minimum(np.floor(c * 4294967296.0), 4294967295.0).astype(np.uint64)
    t[-1] = 4294967295
    return t.astype(np.uint32)


# ---- dictionaries -------------------------------------------------------------------------------------------
def sorted_distinct_in(card: int, limit: int, seed: int) -> np.ndarray:
    """`card` sorted distinct INT values spread uniformly over [0, limit): stride buckets + hashed offset."""
    step = limit // card
    k = np.arange(card, dtype=np.uint64)
    off = (splitmix64_np(np.uint64(seed) ^ k) % np.uint64(max(step, 1))).astype(np.int64)
    return (np.arange(card, dtype=np.int64) * step + off).astype(np.int32)


@dataclass
class SynthColumn:
    name: str
    cardinality: int
    values: Callable[[], np.ndarray]   # sorted INT dictionary
    dist: str = "uniform"
    zipf_s: float = 1.1
    index: str = "fwd"      # "fwd" forward index only, "inv" + bitmap inverted index, "sorted" sorted column


@dataclass
class Workload:
    name: str
    table: str
    columns: List[SynthColumn]
    sql: str
    options: Dict
    seed: int
    description: str
    segments: int = 30      # segments per GPU in bench.py (2^25 docs each): BASELINE.json configs' row counts
    # the table's GPU IndexLoadingConfig (pinot.server.query.executor.gpu.sliced.columns / .value.planes.columns):
    # its scan-filter columns get a bit-sliced copy, its dense metric columns value planes; None = every column
    sliced_columns: Optional[Tuple[str, ...]] = None
    value_planes_columns: Optional[Tuple[str, ...]] = None

    def derived_flags(self) -> Dict[str, int]:
        """Column -> PGPU_DERIVE_* flags of the copies seal builds (GpuSegment(derived=...))."""
        from ._lib import PGPU_DERIVE_SLICED, PGPU_DERIVE_VALUE_PLANES
        return {c.name: (PGPU_DERIVE_SLICED if self.sliced_columns is None or c.name in self.sliced_columns else 0) |
                        (PGPU_DERIVE_VALUE_PLANES if self.value_planes_columns is None or
                         c.name in self.value_planes_columns else 0)
                for c in self.columns}


def _days():
    return np.arange(17500, 17500 + 1024, dtype=np.int32)


def _accounts():
    k = np.arange(1 << 20, dtype=np.int64)
    return (123456789 + (k - (1 << 19)) * 61).astype(np.int32)  # contains 123456789 at k = 2^19


WORKLOADS: Dict[str, Workload] = {
    "adanalytics": Workload(
        "adanalytics", "adAnalytics",
        [SynthColumn("daysSinceEpoch", 1024, _days),
         SynthColumn("accountId", 1 << 20, _accounts),
         SynthColumn("clicks", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 11)),
         SynthColumn("impressions", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 12))],
        "SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics "
        "WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) "
        "GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100",
        {}, 5, "config 5: AdAnalytics filtered GROUP BY SUM (README example query)",
        sliced_columns=("daysSinceEpoch", "accountId"), value_planes_columns=()),
    "range_in": Workload(
        "range_in", "synth",
        [SynthColumn("r", 1 << 16, lambda: (np.arange(1 << 16, dtype=np.int32) * 7 + 3)),
         SynthColumn("i", 16, lambda: np.arange(16, dtype=np.int32) * 100),
         SynthColumn("m", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 13))],
        "SELECT COUNT(*), SUM(m) FROM synth WHERE r BETWEEN 114691 AND 344060 AND i IN (100, 500, 900)",
        {}, 1, "config 2: COUNT(*)+SUM(metric) WHERE range AND IN",
        sliced_columns=("r", "i"), value_planes_columns=("m",)),
    "groupby1m": Workload(
        "groupby1m", "synth",
        [SynthColumn("k", 1 << 20, lambda: np.arange(1 << 20, dtype=np.int32) * 3),
         SynthColumn("m", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 14))],
        "SELECT k, SUM(m), MAX(m), COUNT(*) FROM synth GROUP BY k ORDER BY SUM(m) DESC LIMIT 100",
        {"num_groups_limit": 2_000_000, "min_server_group_trim_size": -1}, 4, "config 4: 1M-key GROUP BY SUM/MAX/COUNT",
        segments=60, sliced_columns=(), value_planes_columns=()),
    "bitmap5": Workload(
        "bitmap5", "bitmap5",
        [SynthColumn("a", 4, lambda: np.arange(4, dtype=np.int32) * 10, index="inv"),
         SynthColumn("b", 16, lambda: np.arange(16, dtype=np.int32) * 10, index="inv"),
         SynthColumn("c", 64, lambda: np.arange(64, dtype=np.int32) * 10, index="inv"),
         SynthColumn("d", 256, lambda: np.arange(256, dtype=np.int32) * 10, index="inv"),
         SynthColumn("e", 256, lambda: np.arange(256, dtype=np.int32) * 10, index="sorted"),
         SynthColumn("m1", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 15)),
         SynthColumn("m2", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 16))],
        "SELECT SUM(m1), SUM(m2) FROM bitmap5 "
        "WHERE (a = 10 AND b IN (30, 70)) OR (c = 50 AND d <> 90 AND e BETWEEN 640 AND 1910)",
        {}, 3, "config 3: inverted-index (Roaring) AND/OR/NOT filter + sorted range, SUM on 2 metric columns",
        sliced_columns=(), value_planes_columns=("m1", "m2")),
    # SURVEY.md 8(d) variants: config 4 with Zipf(1.1)-skewed keys, config 5 with accountId inverted-indexed
    "groupby1m_zipf": Workload(
        "groupby1m_zipf", "synth",
        [SynthColumn("k", 1 << 20, lambda: np.arange(1 << 20, dtype=np.int32) * 3, dist="zipf", zipf_s=1.1),
         SynthColumn("m", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 14))],
        "SELECT k, SUM(m), MAX(m), COUNT(*) FROM synth GROUP BY k ORDER BY SUM(m) DESC LIMIT 100",
        {"num_groups_limit": 2_000_000, "min_server_group_trim_size": -1}, 4, "config 4, Zipf(1.1) keys: 1M-key GROUP BY SUM/MAX/COUNT",
        segments=60, sliced_columns=(), value_planes_columns=()),
    # PMC calibration (not a bench line): config 5's filter stream alone, a known byte count for FETCH_SIZE
    "adanalytics_count": Workload(
        "adanalytics_count", "adAnalytics",
        [SynthColumn("daysSinceEpoch", 1024, _days),
         SynthColumn("accountId", 1 << 20, _accounts),
         SynthColumn("clicks", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 11)),
         SynthColumn("impressions", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 12))],
        "SELECT COUNT(*) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856",
        {}, 5, "config 5's filter stream alone (FETCH_SIZE calibration of the register-direct stream)",
        sliced_columns=("daysSinceEpoch", "accountId"), value_planes_columns=()),
    # config 5 with the reference's numEntriesScannedInFilter (PGPU_Q_EXACT_FILTER_STATS: one more pass over every
    # filter leaf and the host iterator replay): the cost of pinot.server.query.executor.gpu.exact.filter.stats
    "adanalytics_exact": Workload(
        "adanalytics_exact", "adAnalytics",
        [SynthColumn("daysSinceEpoch", 1024, _days),
         SynthColumn("accountId", 1 << 20, _accounts),
         SynthColumn("clicks", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 11)),
         SynthColumn("impressions", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 12))],
        "SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics "
        "WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) "
        "GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100",
        {"exact_filter_stats": True}, 5, "config 5 with the reference's exact numEntriesScannedInFilter",
        sliced_columns=("daysSinceEpoch", "accountId"), value_planes_columns=()),
    "adanalytics_inv": Workload(
        "adanalytics_inv", "adAnalytics",
        [SynthColumn("daysSinceEpoch", 1024, _days),
         SynthColumn("accountId", 1 << 20, _accounts, index="inv"),
         SynthColumn("clicks", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 11)),
         SynthColumn("impressions", 1 << 16, lambda: sorted_distinct_in(1 << 16, 1 << 20, 12))],
        "SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics "
        "WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) "
        "GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100",
        {}, 5, "config 5, accountId inverted-indexed: the IN leaf is a Roaring bitmap",
        sliced_columns=("daysSinceEpoch",), value_planes_columns=()),
}
# config 5 at its literal size on ONE GPU: 8B rows (240 segments of 2^25 docs) -- HBM residency bounded by the
# table's derived-copy policy (forward indexes 62 bits/row + the two filter columns' bit-sliced copies 30 bits/row)
WORKLOADS["adanalytics_8b"] = dataclasses.replace(
    WORKLOADS["adanalytics"], name="adanalytics_8b", segments=240,
    description="config 5 at 8B rows on one GPU (240 x 2^25 docs): HBM residency under the derived-copy policy")


def sorted_index_bytes(num_docs: int, card: int) -> bytes:
    """Sorted column with dict id floor(doc * card / num_docs): (start, end inclusive) big-endian int32 pairs
    (SortedIndexReaderImpl layout)."""
    v = np.arange(card + 1, dtype=np.int64)
    starts = (v * num_docs + card - 1) // card
    pairs = np.stack([starts[:-1], starts[1:] - 1], axis=1).astype(">i4")
    return pairs.tobytes()


class SynthLib:
    def __init__(self, path: str = SYNTH_LIB_PATH):
        if not os.path.exists(path):
            raise ImportError(f"{path} is missing: run __graft_entry__.build()")
        self.lib = C.CDLL(path)
        self.lib.synth_fixed_bit.restype = C.c_int
        self.lib.synth_fixed_bit.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_uint64, C.c_void_p,
                                             C.c_void_p]
        self.lib.synth_alloc.restype = C.c_void_p
        self.lib.synth_alloc.argtypes = [C.c_uint64]
        self.lib.synth_free.argtypes = [C.c_void_p]
        self.lib.synth_sync.restype = C.c_int
        self.lib.synth_copy_to_host.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        self.lib.synth_copy_to_host.restype = C.c_int
        self.lib.synth_inverted_index.restype = C.c_int
        self.lib.synth_inverted_index.argtypes = [C.c_char_p, C.c_int64, C.c_int32, C.c_int32,
                                                  C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_uint64)]
        self.lib.synth_host_free.argtypes = [C.c_void_p]

    def inverted(self, fwd: bytes, num_docs: int, bits: int, card: int) -> bytes:
        """BitmapInvertedIndexWriter file of the dict ids in a fixed-bit forward index (host C builder)."""
        buf = bytes(fwd) + b"\0" * 8  # the reader takes 5 bytes per value
        out = C.POINTER(C.c_uint8)()
        n = C.c_uint64()
        rc = self.lib.synth_inverted_index(buf, num_docs, bits, card, C.byref(out), C.byref(n))
        if rc != 0:
            raise RuntimeError(f"synth_inverted_index failed ({rc})")
        try:
            return C.string_at(out, n.value)
        finally:
            self.lib.synth_host_free(out)

    def alloc(self, nbytes: int) -> int:
        p = self.lib.synth_alloc(nbytes)
        if not p:
            raise MemoryError(f"synth_alloc({nbytes}) failed")
        return p

    def generate(self, dev_out: int, num_docs: int, bits: int, card: int, seed: int, dev_cdf=None) -> None:
        rc = self.lib.synth_fixed_bit(dev_out, num_docs, bits, card, seed, dev_cdf, None)
        if rc != 0 or self.lib.synth_sync() != 0:
            raise RuntimeError(f"synth_fixed_bit failed ({rc})")

    def to_host(self, dev: int, nbytes: int) -> bytes:
        buf = C.create_string_buffer(nbytes)
        if self.lib.synth_copy_to_host(buf, dev, nbytes) != 0:
            raise RuntimeError("synth_copy_to_host failed")
        return buf.raw


def forward_index_bytes(num_docs: int, bits: int) -> int:
    return (num_docs * bits + 7) // 8


def build_segment_cpu(w: Workload, segment: int, num_docs: int, pack: Callable) -> SegmentData:
    """Host-side twin of build_segment_gpu: `pack(ids, bits) -> bytes` is the caller's fixed-bit writer."""
    seg = SegmentData(f"{w.name}_{segment}", num_docs)
    sl = None
    for c in w.columns:
        vals = c.values()
        d = vals.astype(">i4").tobytes()
        if c.index == "sorted":
            seg.columns[c.name] = ColumnIndexes(c.name, PGPU_INT, c.cardinality, dictionary=d,
                                                sorted_index=sorted_index_bytes(num_docs, c.cardinality))
            continue
        cdf = zipf_cdf(c.cardinality, c.zipf_s) if c.dist == "zipf" else None
        ids = dict_ids_cpu(column_seed(w.seed, segment, c.name), num_docs, c.cardinality, cdf=cdf)
        bits = num_bits_per_value(c.cardinality - 1)
        fwd = pack(ids, bits)
        inv = None
        if c.index == "inv":
            sl = sl or SynthLib()
            inv = sl.inverted(fwd, num_docs, bits, c.cardinality)
        seg.columns[c.name] = ColumnIndexes(c.name, PGPU_INT, c.cardinality, dictionary=d, forward=fwd, inverted=inv)
    return seg


def build_segments_gpu(ctx: GpuContext, w: Workload, segment_ids: List[int], num_docs: int) -> List[GpuSegment]:
    """Generate the forward indexes in HBM and upload them as PGPU_MEM_DEVICE sources (D2D copies inside the
    same HIP runtime as libpinotgpu; no host round trip)."""
    sl = SynthLib()
    dicts = {c.name: c.values().astype(">i4").tobytes() for c in w.columns}
    max_bytes = max(forward_index_bytes(num_docs, num_bits_per_value(c.cardinality - 1)) for c in w.columns)
    scratch = sl.alloc(((max_bytes + 64) // 4) * 4)
    cdfs = {}
    out = []
    try:
        for c in w.columns:
            if c.dist == "zipf":
                table = zipf_cdf(c.cardinality, c.zipf_s)
                p = sl.alloc(table.nbytes)
                _h2d(sl, p, table)
                cdfs[c.name] = p
        for s in segment_ids:
            gs = GpuSegment.begin(ctx, f"{w.name}_{s}", num_docs, len(w.columns), derived=w.derived_flags())
            for c in w.columns:
                if c.index == "sorted":
                    gs.add_column(ColumnIndexes(c.name, PGPU_INT, c.cardinality, dictionary=dicts[c.name],
                                                sorted_index=sorted_index_bytes(num_docs, c.cardinality)))
                    continue
                bits = num_bits_per_value(c.cardinality - 1)
                nbytes = forward_index_bytes(num_docs, bits)
                sl.generate(scratch, num_docs, bits, c.cardinality, column_seed(w.seed, s, c.name), cdfs.get(c.name))
                inv = None
                if c.index == "inv":
                    inv = sl.inverted(sl.to_host(scratch, nbytes), num_docs, bits, c.cardinality)
                gs.add_column(ColumnIndexes(c.name, PGPU_INT, c.cardinality, dictionary=dicts[c.name],
                                            forward_device=scratch, forward_device_bytes=nbytes, inverted=inv))
                gs.data.columns[c.name].forward_device = None  # the scratch buffer is reused by the next column
            gs.seal()
            out.append(gs)
    finally:
        sl.lib.synth_free(scratch)
        for p in cdfs.values():
            sl.lib.synth_free(p)
    return out


def _h2d(sl: SynthLib, dev: int, arr: np.ndarray) -> None:
    lib = sl.lib
    lib.synth_copy_from_host.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    lib.synth_copy_from_host.restype = C.c_int
    a = np.ascontiguousarray(arr)
    if lib.synth_copy_from_host(dev, a.ctypes.data, a.nbytes) != 0:
        raise RuntimeError("synth_copy_from_host failed")
