"""Reference on-disk formats, restated in numpy (test infrastructure; see oracle/__init__.py).

* dictionary        SegmentDictionaryCreator: sorted unique values, big-endian fixed width
                    (seglocal/segment/creator/impl/SegmentDictionaryCreator.java:92-156)
* fixed-bit fwd     FixedBitSVForwardIndexWriter + PinotDataBitSet.writeInt: value i at bits [i*b, (i+1)*b) of a
                    MSB-first big-endian stream, ceil(N*b/8) bytes
                    (seglocal/io/writer/impl/FixedBitSVForwardIndexWriter.java:39-47,
                     seglocal/io/util/PinotDataBitSet.java:59-165)
* sorted index      2 big-endian int32 (start, end inclusive) per dict id
                    (seglocal/segment/index/readers/sorted/SortedIndexReaderImpl.java:37-121)
* Roaring bitmap    RoaringBitmap 0.9.26 portable serialization (third-party, pom.xml:412-415, not vendored):
                    cookie 12346 / 12347, (key, card-1) pairs, offsets, array / bitmap / run containers; run
                    containers are chosen as RoaringBitmapWriter's default runOptimize does (run when its
                    2 + 4*runs bytes are smaller than the array / bitmap form)
* inverted index    BitmapInvertedIndexWriter: (card+1) big-endian int32 absolute offsets, then the bitmaps
                    (seglocal/segment/creator/impl/inv/BitmapInvertedIndexWriter.java:35-124)
* MV forward index  FixedBitMVForwardIndexWriter: big-endian int32 chunk offsets (value index of each chunk's first
                    row; ceil(2048 / (numValues / numDocs)) rows per chunk), a row-start bitmap over the value
                    index (PinotDataBitSet.setBit, MSB-first), then the values' dict ids fixed-bit
                    (seglocal/io/writer/impl/FixedBitMVForwardIndexWriter.java:73-159,
                     seglocal/segment/index/readers/forward/FixedBitMVForwardIndexReader.java:58-140)
"""
from __future__ import annotations

import struct
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

from pinot_amd._lib import PGPU_DOUBLE, PGPU_FLOAT, PGPU_INT, PGPU_LONG, PGPU_STRING
from pinot_amd.segment import ColumnIndexes, SegmentData

_BE = {PGPU_INT: ">i4", PGPU_LONG: ">i8", PGPU_FLOAT: ">f4", PGPU_DOUBLE: ">f8"}
NATIVE = {PGPU_INT: np.int32, PGPU_LONG: np.int64, PGPU_FLOAT: np.float32, PGPU_DOUBLE: np.float64}


def bits_per_value(cardinality: int) -> int:
    """PinotDataBitSet.getNumBitsPerValue(cardinality - 1) (PinotDataBitSet.java:59-71)."""
    m = cardinality - 1
    return 1 if m <= 1 else int(m).bit_length()


# ---- fixed-bit forward index ------------------------------------------------------------------------------------
def pack_fixed_bit(ids: np.ndarray, bits: int) -> bytes:
    """FixedBitSVForwardIndexWriter output for dict ids `ids` (chunks of 2^20 docs keep memory bounded)."""
    ids = np.asarray(ids, dtype=np.uint32)
    n = len(ids)
    out = bytearray()
    chunk = 1 << 20  # multiple of 8 docs -> every chunk ends on a byte boundary
    for s in range(0, n, chunk):
        v = ids[s:s + chunk]
        if bits < 32 and v.size and int(v.max()) >> bits:
            raise ValueError("dict id does not fit the bit width")
        b = np.unpackbits(v.astype(">u4").view(np.uint8).reshape(-1, 4), axis=1)[:, 32 - bits:]
        out += np.packbits(b.reshape(-1)).tobytes()
    need = (n * bits + 7) // 8
    assert len(out) == need, (len(out), need)
    return bytes(out)


def unpack_fixed_bit(data: bytes, bits: int, num_docs: int) -> np.ndarray:
    """PinotDataBitSet.readInt for docs 0..num_docs-1 (vectorised)."""
    out = np.empty(num_docs, dtype=np.int64)
    raw = np.frombuffer(data, dtype=np.uint8)
    chunk = 1 << 20
    w = (1 << np.arange(bits - 1, -1, -1, dtype=np.int64))
    for s in range(0, num_docs, chunk):
        e = min(num_docs, s + chunk)
        b0 = s * bits // 8
        b1 = (e * bits + 7) // 8
        bitsarr = np.unpackbits(raw[b0:b1])[: (e - s) * bits].reshape(-1, bits).astype(np.int64)
        out[s:e] = bitsarr @ w
    return out


def read_int(data: bytes, index: int, bits: int) -> int:
    """Scalar PinotDataBitSet.readInt(index, numBitsPerValue) (PinotDataBitSet.java:78-97)."""
    bit = index * bits
    byte, off = bit // 8, bit % 8
    cur = data[byte] & (0xFF >> off)
    left = bits - (8 - off)
    if left <= 0:
        return cur >> -left
    while left > 8:
        byte += 1
        cur = (cur << 8) | data[byte]
        left -= 8
    return (cur << left) | (data[byte + 1] >> (8 - left))


# ---- multi-value forward index ---------------------------------------------------------------------------------
def mv_docs_per_chunk(num_docs: int, num_values: int) -> int:
    """FixedBitMVForwardIndexWriter.java:77-78: ceil(2048 / (float)(totalNumValues / numDocs)), integer division
    inside (the reader repeats it, FixedBitMVForwardIndexReader.java:61)."""
    avg = num_values // num_docs
    return int(np.ceil(np.float32(2048) / np.float32(avg)))


def write_mv_forward(rows: Sequence[np.ndarray], bits: int) -> bytes:
    """FixedBitMVForwardIndexWriter file of per-row dict-id arrays (every row holds at least one value, as the
    segment creator's null-default placeholder guarantees)."""
    num_docs = len(rows)
    lens = np.fromiter((len(r) for r in rows), dtype=np.int64, count=num_docs)
    if num_docs == 0 or np.any(lens == 0):
        raise ValueError("multi-value rows must hold at least one value")
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    num_values = int(lens.sum())
    per = mv_docs_per_chunk(num_docs, num_values)
    chunks = starts[::per].astype(">i4").tobytes()
    bitmap = np.zeros((num_values + 7) // 8 * 8, dtype=np.uint8)
    bitmap[starts] = 1
    ids = np.concatenate([np.asarray(r, dtype=np.int64) for r in rows])
    return chunks + np.packbits(bitmap).tobytes() + pack_fixed_bit(ids, bits)


def read_mv_forward(data: bytes, num_docs: int, num_values: int, bits: int):
    """(offsets[num_docs + 1], dict ids[num_values]) of a FixedBitMVForwardIndexWriter file, found through the
    row-start bitmap as FixedBitMVForwardIndexReader.getDictIdMV finds a row (its chunk offsets only speed that up;
    they are checked here)."""
    per = mv_docs_per_chunk(num_docs, num_values)
    nchunks = (num_docs + per - 1) // per
    hdr = 4 * nchunks
    nb = (num_values + 7) // 8
    bm = np.unpackbits(np.frombuffer(data, dtype=np.uint8, count=nb, offset=hdr))[:num_values]
    starts = np.flatnonzero(bm)
    if len(starts) != num_docs or (num_docs and starts[0] != 0):
        raise ValueError("row-start bitmap does not hold one start per row")
    chunks = np.frombuffer(data, dtype=">i4", count=nchunks)
    if not np.array_equal(chunks.astype(np.int64), starts[::per]):
        raise ValueError("chunk offsets disagree with the row-start bitmap")
    ids = unpack_fixed_bit(data[hdr + nb:], bits, num_values)
    return np.concatenate([starts, [num_values]]).astype(np.int64), ids


# ---- dictionaries ----------------------------------------------------------------------------------------------
def build_dictionary(values: Sequence, data_type: int):
    """Sorted unique values + dict id per row (SegmentDictionaryCreator + indexOfSV)."""
    if data_type == PGPU_STRING:
        uniq = sorted(set(values))
        pos = {v: i for i, v in enumerate(uniq)}
        ids = np.fromiter((pos[v] for v in values), dtype=np.int32, count=len(values))
        return uniq, ids
    arr = np.asarray(values, dtype=NATIVE[data_type])
    uniq, ids = np.unique(arr, return_inverse=True)
    return uniq, ids.astype(np.int32)


def dictionary_bytes(uniq, data_type: int) -> Optional[bytes]:
    if data_type == PGPU_STRING:
        return None
    return np.asarray(uniq).astype(_BE[data_type]).tobytes()


def sorted_index_bytes(ids: np.ndarray, cardinality: int) -> bytes:
    """Per dict id (first doc, last doc) of a sorted column."""
    ids = np.asarray(ids)
    if len(ids) and np.any(np.diff(ids) < 0):
        raise ValueError("column is not sorted")
    starts = np.searchsorted(ids, np.arange(cardinality), side="left")
    ends = np.searchsorted(ids, np.arange(cardinality), side="right") - 1
    return np.stack([starts, ends], axis=1).astype(">i4").tobytes()


# ---- Roaring portable format -----------------------------------------------------------------------------------
SERIAL_COOKIE_NO_RUNCONTAINER = 12346
SERIAL_COOKIE = 12347
NO_OFFSET_THRESHOLD = 4


def _runs(low: np.ndarray) -> np.ndarray:
    """(start, length-1) pairs of the maximal runs of a sorted uint16 array."""
    if low.size == 0:
        return np.zeros((0, 2), dtype=np.int64)
    brk = np.nonzero(np.diff(low.astype(np.int64)) != 1)[0]
    starts = np.concatenate([[0], brk + 1])
    ends = np.concatenate([brk, [low.size - 1]])
    return np.stack([low[starts].astype(np.int64), (low[ends].astype(np.int64) - low[starts])], axis=1)


def roaring_serialize(doc_ids: Iterable[int], allow_runs: bool = True, force: Optional[str] = None) -> bytes:
    """Portable serialization of a sorted doc-id set.  `force` in {None, 'array', 'bitmap', 'run'} overrides the
    container choice (tests use it to exercise every container type)."""
    d = np.unique(np.asarray(list(doc_ids) if not isinstance(doc_ids, np.ndarray) else doc_ids, dtype=np.int64))
    if d.size and (d[0] < 0 or d[-1] >= 1 << 31):
        raise ValueError("doc ids out of range")
    keys = (d >> 16).astype(np.int64)
    containers = []  # (key, card, kind, payload bytes)
    if d.size:
        bounds = np.nonzero(np.diff(keys))[0] + 1
        for part in np.split(d, bounds):
            key = int(part[0] >> 16)
            low = (part & 0xFFFF).astype(np.uint16)
            card = int(low.size)
            runs = _runs(low)
            if force is not None:
                kind = force
            else:
                kind = "array" if card <= 4096 else "bitmap"
                plain = 2 * card if kind == "array" else 8192
                if allow_runs and 2 + 4 * len(runs) < plain:
                    kind = "run"
            if kind == "array":
                if card > 4096:
                    raise ValueError("array container above 4096 values")
                payload = low.astype("<u2").tobytes()
            elif kind == "bitmap":
                if card <= 4096 and force is None:
                    raise AssertionError
                bits = np.zeros(65536, dtype=np.uint8)
                bits[low] = 1
                payload = np.packbits(bits, bitorder="little").tobytes()
            else:
                payload = struct.pack("<H", len(runs)) + runs.astype("<u2").tobytes()
            containers.append((key, card, kind, payload))
    size = len(containers)
    has_run = any(c[2] == "run" for c in containers)
    out = bytearray()
    if has_run:
        out += struct.pack("<I", SERIAL_COOKIE | ((size - 1) << 16))
        flags = bytearray((size + 7) // 8)
        for i, c in enumerate(containers):
            if c[2] == "run":
                flags[i // 8] |= 1 << (i % 8)
        out += flags
    else:
        out += struct.pack("<II", SERIAL_COOKIE_NO_RUNCONTAINER, size)
    for key, card, _, _ in containers:
        out += struct.pack("<HH", key, card - 1)
    if not has_run or size >= NO_OFFSET_THRESHOLD:
        pos = len(out) + 4 * size
        for c in containers:
            out += struct.pack("<I", pos)
            pos += len(c[3])
    for c in containers:
        out += c[3]
    return bytes(out)


def roaring_deserialize(buf: bytes) -> np.ndarray:
    """Inverse of roaring_serialize (independent parser used by the round-trip tests)."""
    cookie = struct.unpack_from("<I", buf, 0)[0]
    if cookie & 0xFFFF == SERIAL_COOKIE:
        size = (cookie >> 16) + 1
        flags = buf[4:4 + (size + 7) // 8]
        pos = 4 + (size + 7) // 8
        has_run = True
    elif cookie == SERIAL_COOKIE_NO_RUNCONTAINER:
        size = struct.unpack_from("<I", buf, 4)[0]
        flags = b""
        pos = 8
        has_run = False
    else:
        raise ValueError(f"bad cookie {cookie}")
    kc = [struct.unpack_from("<HH", buf, pos + 4 * i) for i in range(size)]
    pos += 4 * size
    if not has_run or size >= NO_OFFSET_THRESHOLD:
        pos += 4 * size
    parts = []
    for i, (key, cm1) in enumerate(kc):
        card = cm1 + 1
        is_run = has_run and (flags[i // 8] >> (i % 8)) & 1
        if is_run:
            n = struct.unpack_from("<H", buf, pos)[0]
            pos += 2
            r = np.frombuffer(buf, dtype="<u2", count=2 * n, offset=pos).reshape(-1, 2).astype(np.int64)
            pos += 4 * n
            low = np.concatenate([np.arange(s, s + l + 1) for s, l in r]) if n else np.zeros(0, np.int64)
        elif card > 4096:
            bits = np.unpackbits(np.frombuffer(buf, dtype=np.uint8, count=8192, offset=pos), bitorder="little")
            pos += 8192
            low = np.nonzero(bits)[0]
        else:
            low = np.frombuffer(buf, dtype="<u2", count=card, offset=pos).astype(np.int64)
            pos += 2 * card
        if len(low) != card:
            raise ValueError("container cardinality mismatch")
        parts.append((key << 16) + low)
    return np.concatenate(parts) if parts else np.zeros(0, np.int64)


def inverted_index_bytes(ids: np.ndarray, cardinality: int, allow_runs: bool = True,
                         force: Optional[str] = None) -> bytes:
    """BitmapInvertedIndexWriter file for a column's dict ids."""
    ids = np.asarray(ids)
    order = np.argsort(ids, kind="stable")
    sorted_ids = ids[order]
    bounds = np.searchsorted(sorted_ids, np.arange(cardinality + 1))
    blobs = [roaring_serialize(order[bounds[i]:bounds[i + 1]], allow_runs, force) for i in range(cardinality)]
    header = 4 * (cardinality + 1)
    offs = [header]
    for b in blobs:
        offs.append(offs[-1] + len(b))
    return np.asarray(offs, dtype=">i4").tobytes() + b"".join(blobs)


def read_inverted_bitmap(data: bytes, cardinality: int, dict_id: int) -> np.ndarray:
    """BitmapInvertedIndexReader.getDocIds (reader subtracts the first offset)."""
    offs = np.frombuffer(data, dtype=">i4", count=cardinality + 1)
    first = int(offs[0])
    header = 4 * (cardinality + 1)
    s, e = int(offs[dict_id]) - first, int(offs[dict_id + 1]) - first
    return roaring_deserialize(data[header + s:header + e])


# ---- segment builder ------------------------------------------------------------------------------------------
def build_segment(name: str, columns: Dict[str, tuple], inverted: Iterable[str] = (),
                  sorted_columns: Optional[Iterable[str]] = None, allow_runs: bool = True,
                  raw: Iterable[str] = (), raw_codec: int = 0, raw_version: int = 2,
                  range_index: Iterable[str] = (), range_index_version: int = 2,
                  raw_min_max: bool = True, mv: Iterable[str] = ()) -> SegmentData:
    """Build an immutable segment from raw column values.

    `columns`: name -> (data_type, values).  A column is stored with a sorted index when its dict ids are
    non-decreasing (the segment creator's isSorted detection) unless `sorted_columns` restricts the set.
    `inverted`: columns whose inverted index is loaded (IndexLoadingConfig.getInvertedIndexColumns).
    `raw`: no-dictionary columns (noDictionaryColumns), written as FixedByteChunkSVForwardIndexWriter files with
    `raw_codec` / `raw_version` (oracle/rawfwd.py); `raw_min_max` records their metadata min / max.
    `range_index`: columns with a range index (rangeIndexColumns) of `range_index_version` (header only, see
    oracle.rawfwd.range_index_header).
    `mv`: multi-value columns; their values are a sequence of per-row value arrays (FixedBitMVForwardIndexWriter;
    an inverted index lists every doc holding the id)."""
    from .rawfwd import range_index_header, write_raw_forward
    inverted = set(inverted)
    raw = set(raw)
    range_index = set(range_index)
    mv = set(mv)
    n = None
    seg = None
    for cname, (dt, values) in columns.items():
        if n is None:
            n = len(values)
            seg = SegmentData(name, n)
        if len(values) != n:
            raise ValueError("ragged columns")
        if cname in mv:
            rows = [np.asarray(r, dtype=NATIVE[dt]) if dt != PGPU_STRING else list(r) for r in values]
            flat = np.concatenate(rows) if dt != PGPU_STRING else [v for r in rows for v in r]
            uniq, ids = build_dictionary(flat, dt)
            card = len(uniq)
            lens = np.fromiter((len(r) for r in rows), dtype=np.int64, count=n)
            starts = np.concatenate([[0], np.cumsum(lens)])
            id_rows = [ids[starts[i]:starts[i + 1]] for i in range(n)]
            col = ColumnIndexes(cname, dt, card, dictionary=(list(uniq) if dt == PGPU_STRING
                                                              else dictionary_bytes(uniq, dt)),
                                mv_forward=write_mv_forward(id_rows, bits_per_value(card)),
                                num_values=int(lens.sum()), max_values=int(lens.max()) if n else 0)
            if cname in inverted:
                docs = np.repeat(np.arange(n, dtype=np.int64), lens)
                pairs = np.unique(np.stack([ids.astype(np.int64), docs], axis=1), axis=0)
                order = np.argsort(pairs[:, 0], kind="stable")
                bounds = np.searchsorted(pairs[order, 0], np.arange(card + 1))
                blobs = [roaring_serialize(pairs[order[bounds[i]:bounds[i + 1]], 1], allow_runs)
                         for i in range(card)]
                offs = [4 * (card + 1)]
                for b in blobs:
                    offs.append(offs[-1] + len(b))
                col.inverted = np.asarray(offs, dtype=">i4").tobytes() + b"".join(blobs)
            seg.columns[cname] = col
            continue
        if cname in raw:
            vals = np.asarray(values, dtype=NATIVE[dt])
            col = ColumnIndexes(cname, dt, len(np.unique(vals)) if n else 0,
                                raw_forward=write_raw_forward(vals, dt, raw_codec, raw_version))
            if raw_min_max and n:
                col.min_value, col.max_value = vals.min().item(), vals.max().item()
            if cname in range_index:
                col.range_index = range_index_header(range_index_version, int(vals.min()) if n and dt < 2 else 0)
            seg.columns[cname] = col
            continue
        uniq, ids = build_dictionary(values, dt)
        card = len(uniq)
        is_sorted = bool(np.all(np.diff(ids) >= 0)) if n else True
        if sorted_columns is not None:
            is_sorted = is_sorted and cname in set(sorted_columns)
        col = ColumnIndexes(cname, dt, card, dictionary=(list(uniq) if dt == PGPU_STRING
                                                          else dictionary_bytes(uniq, dt)))
        if is_sorted:
            col.sorted_index = sorted_index_bytes(ids, card)
        else:
            col.forward = pack_fixed_bit(ids, bits_per_value(card))
        if cname in inverted:
            col.inverted = inverted_index_bytes(ids, card, allow_runs)
        if cname in range_index:
            col.range_index = range_index_header(range_index_version, 0)
        seg.columns[cname] = col
    return seg


# ---- on-disk segment directories (test infrastructure: feeds pinot_amd.loader) ---------------------------------
_TYPE_NAME = {PGPU_INT: "INT", PGPU_LONG: "LONG", PGPU_FLOAT: "FLOAT", PGPU_DOUBLE: "DOUBLE", PGPU_STRING: "STRING"}
_MAGIC = 0xDEADBEEFDEAFBEAD


def string_dictionary_bytes(values: Sequence[str], pad: bytes = b"\0"):
    """Fixed-width STRING dictionary: every value padded to the longest UTF-8 length
    (SegmentDictionaryCreator.java:92-156 with the segment's padding character)."""
    enc = [v.encode("utf-8") for v in values]
    width = max([len(b) for b in enc] + [1])
    return b"".join(b + pad * (width - len(b)) for b in enc), width


def write_segment_dir(seg: SegmentData, path: str, version: str = "v3", pad_char: str = "\0") -> str:
    """Write `seg` as a Pinot segment directory: metadata.properties plus either v1 files per index
    (V1Constants.Indexes extensions) or v3 columns.psf + index_map, each index behind the 8-byte magic marker
    (SingleFileIndexDirectory.allocNewBufferInternal :164-184, persistIndexMap :446-465).  Returns the
    directory holding metadata.properties."""
    import os
    os.makedirs(path, exist_ok=True)
    root = os.path.join(path, "v3") if version == "v3" else path
    os.makedirs(root, exist_ok=True)
    pad = pad_char.encode("utf-8")
    pad_text = "\\\\u0000" if pad_char == "\0" else pad_char
    meta = [f"segment.name = {seg.name}", "segment.table.name = testTable", f"segment.total.docs = {seg.num_docs}",
            f"segment.padding.character = {pad_text}", f"segment.index.version = {version}"]
    indexes = []  # (column, index name, v1 extension, bytes)
    for c in seg.columns.values():
        if c.raw_forward is not None:  # no-dictionary column (ColumnMetadataImpl hasDictionary = false)
            meta += [f"column.{c.name}.cardinality = {c.cardinality}", f"column.{c.name}.totalDocs = {seg.num_docs}",
                     f"column.{c.name}.dataType = {_TYPE_NAME[c.data_type]}",
                     f"column.{c.name}.bitsPerElement = {bits_per_value(max(c.cardinality, 1))}",
                     f"column.{c.name}.lengthOfEachEntry = 0", f"column.{c.name}.isSorted = false",
                     f"column.{c.name}.hasDictionary = false", f"column.{c.name}.hasInvertedIndex = false",
                     f"column.{c.name}.isSingleValues = true"]
            if c.min_value is not None and c.max_value is not None:
                meta += [f"column.{c.name}.minValue = {c.min_value!r}", f"column.{c.name}.maxValue = {c.max_value!r}"]
            indexes.append((c.name, "forward_index", ".sv.raw.fwd", bytes(c.raw_forward)))
            if c.range_index is not None:
                indexes.append((c.name, "range_index", ".bitmap.range", bytes(c.range_index)))
            continue
        if c.data_type == PGPU_STRING:
            dbytes, width = string_dictionary_bytes(list(c.dictionary), pad)
        else:
            dbytes, width = bytes(c.dictionary), 0
        if c.mv_forward is not None:  # multi-value column (isSingleValues = false)
            meta += [f"column.{c.name}.cardinality = {c.cardinality}", f"column.{c.name}.totalDocs = {seg.num_docs}",
                     f"column.{c.name}.dataType = {_TYPE_NAME[c.data_type]}",
                     f"column.{c.name}.bitsPerElement = {bits_per_value(c.cardinality)}",
                     f"column.{c.name}.lengthOfEachEntry = {width}", f"column.{c.name}.isSorted = false",
                     f"column.{c.name}.hasDictionary = true",
                     f"column.{c.name}.hasInvertedIndex = {'true' if c.inverted is not None else 'false'}",
                     f"column.{c.name}.isSingleValues = false",
                     f"column.{c.name}.maxNumberOfMultiValues = {c.max_values}",
                     f"column.{c.name}.totalNumberOfEntries = {c.num_values}"]
            indexes.append((c.name, "dictionary", ".dict", dbytes))
            indexes.append((c.name, "forward_index", ".mv.fwd", bytes(c.mv_forward)))
            if c.inverted is not None:
                indexes.append((c.name, "inverted_index", ".bitmap.inv", bytes(c.inverted)))
            continue
        sorted_col = c.sorted_index is not None
        meta += [f"column.{c.name}.cardinality = {c.cardinality}", f"column.{c.name}.totalDocs = {seg.num_docs}",
                 f"column.{c.name}.dataType = {_TYPE_NAME[c.data_type]}",
                 f"column.{c.name}.bitsPerElement = {bits_per_value(c.cardinality)}",
                 f"column.{c.name}.lengthOfEachEntry = {width}",
                 f"column.{c.name}.isSorted = {'true' if sorted_col else 'false'}",
                 f"column.{c.name}.hasDictionary = true",
                 f"column.{c.name}.hasInvertedIndex = {'true' if c.inverted is not None else 'false'}",
                 f"column.{c.name}.isSingleValues = true"]
        indexes.append((c.name, "dictionary", ".dict", dbytes))
        if sorted_col:
            indexes.append((c.name, "forward_index", ".sv.sorted.fwd", bytes(c.sorted_index)))
        else:
            indexes.append((c.name, "forward_index", ".sv.unsorted.fwd", bytes(c.forward)))
        if c.inverted is not None:
            indexes.append((c.name, "inverted_index", ".bitmap.inv", bytes(c.inverted)))
        if c.range_index is not None:
            indexes.append((c.name, "range_index", ".bitmap.range", bytes(c.range_index)))
    with open(os.path.join(root, "metadata.properties"), "w") as f:
        f.write("\n".join(meta) + "\n")
    if version == "v3":
        off, lines = 0, []
        with open(os.path.join(root, "columns.psf"), "wb") as f:
            for col, idx, _, data in indexes:
                f.write(struct.pack(">Q", _MAGIC))
                f.write(data)
                lines += [f"{col}.{idx}.startOffset = {off}", f"{col}.{idx}.size = {len(data) + 8}"]
                off += len(data) + 8
        with open(os.path.join(root, "index_map"), "w") as f:
            f.write("\n".join(lines) + "\n")
    else:
        for col, _, ext, data in indexes:
            with open(os.path.join(root, col + ext), "wb") as f:
                f.write(data)
    return root
