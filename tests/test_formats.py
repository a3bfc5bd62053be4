"""Reference on-disk formats: the oracle's writers against real reference segment bytes and round trips (CPU)."""
import os
import re
import struct

import numpy as np
import pytest

from oracle.segment_writer import (bits_per_value, inverted_index_bytes, pack_fixed_bit, read_int,
                                   read_inverted_bitmap, roaring_deserialize, roaring_serialize,
                                   sorted_index_bytes, unpack_fixed_bit)
from tests.helpers import GOLDEN

PAD = np.load(os.path.join(GOLDEN, "padding_segments.npz"))


def _meta(name):
    text = PAD[f"{name}/metadata.properties"].tobytes().decode()
    return dict(re.findall(r"^(\S+)\s*=\s*(.*)$", text, flags=re.M))


@pytest.mark.parametrize("name", ["paddingNull", "paddingOld", "paddingPercent"])
def test_padding_segment_forward_index_bytes(name):
    """Real 5-doc segments written by the reference: decode every column's fixed-bit forward index with the
    restated reader and re-encode it with the restated writer — bytes must be identical."""
    meta = _meta(name)
    for col in ("age", "name", "percent", "outgoingName1"):
        fwd = PAD[f"{name}/{col}.sv.unsorted.fwd"].tobytes()
        card = int(meta[f"column.{col}.cardinality"])
        bits = int(meta[f"column.{col}.bitsPerElement"])
        assert bits == bits_per_value(card)
        ids = unpack_fixed_bit(fwd, bits, 5)
        assert ids.max() < card
        assert [read_int(fwd, i, bits) for i in range(5)] == ids.tolist()
        assert pack_fixed_bit(ids, bits) == fwd[: (5 * bits + 7) // 8]


def test_padding_segment_int_dictionary():
    d = np.frombuffer(PAD["paddingNull/age.dict"].tobytes(), dtype=">i4")
    assert d.tolist() == [617, 824, 837, 1209, 1228]       # sorted, big-endian
    ids = unpack_fixed_bit(PAD["paddingNull/age.sv.unsorted.fwd"].tobytes(), 3, 5)
    assert ids.tolist() == [4, 2, 3, 0, 1]


@pytest.mark.parametrize("bits", [1, 2, 3, 4, 7, 8, 10, 13, 16, 17, 20, 24, 31, 32])
def test_fixed_bit_round_trip(bits):
    rng = np.random.default_rng(bits)
    n = 10_007
    hi = 1 << bits
    v = rng.integers(0, hi, size=n, dtype=np.uint64).astype(np.uint32)
    data = pack_fixed_bit(v, bits)
    assert len(data) == (n * bits + 7) // 8
    assert np.array_equal(unpack_fixed_bit(data, bits, n), v.astype(np.int64))
    for i in (0, 1, n // 2, n - 2, n - 1):
        assert read_int(data, i, bits) == v[i]


@pytest.mark.parametrize("docs", [
    [], [0], [65535, 65536], list(range(0, 5000)), list(range(3, 200_000, 7)), list(range(10, 70_000)),
    [0, 1, 2, 100_000, 100_001, 1 << 20],
])
@pytest.mark.parametrize("force", [None, "array", "run"])
def test_roaring_round_trip(docs, force):
    if force == "array":
        # an array container holds at most 4096 values
        counts = np.bincount(np.asarray(docs, dtype=np.int64) >> 16) if docs else []
        if len(counts) and max(counts) > 4096:
            pytest.skip("array container limit")
    data = roaring_serialize(docs, force=force)
    assert roaring_deserialize(data).tolist() == sorted(set(docs))


def test_roaring_container_choice():
    """Default writer: dense chunks -> bitmap, sparse -> array, long runs -> run (cookie 12347)."""
    dense = np.arange(0, 65536, 2)
    assert struct.unpack_from("<I", roaring_serialize(dense))[0] == 12346  # bitmap, no runs
    run = np.arange(0, 60_000)
    cookie = struct.unpack_from("<I", roaring_serialize(run))[0]
    assert cookie & 0xFFFF == 12347


def test_inverted_index_file_and_sorted_index():
    rng = np.random.default_rng(7)
    ids = rng.integers(0, 17, size=150_000)
    inv = inverted_index_bytes(ids, 17)
    offs = np.frombuffer(inv, dtype=">i4", count=18)
    assert offs[0] == 4 * 18 and offs[-1] == len(inv)
    for d in range(17):
        assert np.array_equal(read_inverted_bitmap(inv, 17, d), np.flatnonzero(ids == d))
    s = np.sort(ids)
    pairs = np.frombuffer(sorted_index_bytes(s, 17), dtype=">i4").reshape(-1, 2)
    for d in range(17):
        assert pairs[d, 0] == np.searchsorted(s, d) and pairs[d, 1] == np.searchsorted(s, d, side="right") - 1


@pytest.mark.parametrize("card,n,layout", [(4, 70_000, "uniform"), (16, 200_003, "uniform"), (64, 150_001, "uniform"),
                                           (256, 131_072, "uniform"), (3, 5, "uniform"), (256, 300_000, "sorted"),
                                           (16, 140_000, "blocks")])
def test_synth_inverted_index_matches_oracle(card, n, layout):
    """The bench's inverted-index builder (synth.hip, C++) writes the oracle's bytes exactly: offsets header,
    cookies 12346 / 12347, array / bitmap / run containers chosen as RoaringBitmapWriter + runOptimize."""
    from pinot_amd.synth import SynthLib
    rng = np.random.default_rng(card * 7 + n)
    if layout == "sorted":
        ids = np.sort(rng.integers(0, card, n))
    elif layout == "blocks":
        ids = np.repeat(rng.integers(0, card, n // 700 + 1), 700)[:n]
    else:
        ids = rng.integers(0, card, n)
    bits = bits_per_value(card)
    fwd = pack_fixed_bit(ids, bits)
    assert SynthLib().inverted(fwd, n, bits, card) == inverted_index_bytes(ids, card)
