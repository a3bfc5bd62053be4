"""Raw (no-dictionary) forward index format, restated in Python (test infrastructure; see oracle/__init__.py).

* FixedByteChunkSVForwardIndexWriter (seglocal/io/writer/impl/FixedByteChunkSVForwardIndexWriter.java:39-104) on
  BaseChunkSVForwardIndexWriter (:71-194): header int32 version, numChunks, numDocsPerChunk, sizeOfEntry; from
  version 2 on also totalDocs, compressionType, dataHeaderStart; then one chunk offset per chunk (int32 for versions
  1-2, int64 for 3-4); then the chunks, each numDocsPerChunk big-endian values compressed on their own.  Version 4
  rounds numDocsPerChunk up to a power of two (normalizeDocsPerChunk).  SingleValueFixedByteRawIndexCreator
  writes 1000 docs per chunk (DEFAULT_NUM_DOCS_PER_CHUNK) at version 2 by default.
* Codecs (seglocal/io/compression/ChunkCompressorFactory.java, ChunkCompressionType ordinals PASS_THROUGH 0,
  SNAPPY 1, ZSTANDARD 2, LZ4 3, LZ4_LENGTH_PREFIXED 4).  SNAPPY and LZ4 are third-party (snappy-java, lz4-java;
  not vendored, not importable here): their published raw block formats are restated below, encoder and decoder.
  The encoders are simple greedy matchers -- any valid block decodes the same, which is all the readers rely on.
  ZSTANDARD (ZstandardCompressor / ZstandardDecompressor: zstd-jni 1.4.9-5, one zstd frame per chunk) is too large
  a format to restate; it goes through pyarrow's bundled zstd codec, an implementation independent of the system
  libzstd.so.1 the product decodes with.
* The reader half mirrors BaseChunkSVForwardIndexReader (seglocal/segment/index/readers/forward/
  BaseChunkSVForwardIndexReader.java:56-157) / FixedByteChunkSVForwardIndexReader.getInt/Long/Float/Double.
"""
from __future__ import annotations

import struct
from typing import Optional

import numpy as np

PASS_THROUGH, SNAPPY, ZSTANDARD, LZ4, LZ4_LENGTH_PREFIXED = range(5)
_BE = {0: ">i4", 1: ">i8", 2: ">f4", 3: ">f8"}   # PGPU_INT, PGPU_LONG, PGPU_FLOAT, PGPU_DOUBLE
DEFAULT_NUM_DOCS_PER_CHUNK = 1000                 # SingleValueFixedByteRawIndexCreator.java:40


# ---- snappy raw block ---------------------------------------------------------------------------------------------
def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def snappy_compress(data: bytes) -> bytes:
    out = bytearray(_varint(len(data)))
    n = len(data)
    table = {}
    lit_start = 0
    i = 0

    def literal(a: int, b: int):
        while a < b:
            k = min(b - a, 1 << 16)
            ln = k - 1
            if ln < 60:
                out.append(ln << 2)
            elif ln < 256:
                out.extend(bytes([60 << 2, ln]))
            else:
                out.extend(bytes([61 << 2, ln & 0xFF, ln >> 8]))
            out.extend(data[a:a + k])
            a += k

    while i + 4 <= n:
        key = data[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is not None and i - j < 65536:
            ln = 4
            while i + ln < n and data[j + ln] == data[i + ln] and ln < 64:
                ln += 1
            literal(lit_start, i)
            off = i - j
            if 4 <= ln <= 11 and off < 2048:
                out += bytes([1 | ((ln - 4) << 2) | ((off >> 8) << 5), off & 0xFF])
            else:
                out += bytes([2 | ((ln - 1) << 2), off & 0xFF, off >> 8])
            i += ln
            lit_start = i
        else:
            i += 1
    literal(lit_start, n)
    return bytes(out)


def snappy_decompress(buf: bytes) -> bytes:
    i, shift, n = 0, 0, 0
    while True:
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            break
    out = bytearray()
    while i < len(buf):
        tag = buf[i]
        i += 1
        t = tag & 3
        if t == 0:
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(buf[i:i + nb], "little")
                i += nb
            ln += 1
            out += buf[i:i + ln]
            i += ln
            continue
        if t == 1:
            ln, off = 4 + ((tag >> 2) & 7), ((tag >> 5) << 8) | buf[i]
            i += 1
        elif t == 2:
            ln, off = 1 + (tag >> 2), int.from_bytes(buf[i:i + 2], "little")
            i += 2
        else:
            ln, off = 1 + (tag >> 2), int.from_bytes(buf[i:i + 4], "little")
            i += 4
        for _ in range(ln):
            out.append(out[-off])
    assert len(out) == n
    return bytes(out)


# ---- LZ4 raw block --------------------------------------------------------------------------------------------------
_MFLIMIT, _LASTLITERALS = 12, 5


def lz4_compress(data: bytes) -> bytes:
    out = bytearray()
    n = len(data)
    table = {}
    anchor = i = 0

    def seq(lit_a: int, lit_b: int, off: int = 0, mlen: int = 0, last: bool = False):
        ll = lit_b - lit_a
        tok_l = min(ll, 15)
        tok_m = 0 if last else min(mlen - 4, 15)
        out.append((tok_l << 4) | tok_m)
        if ll >= 15:
            r = ll - 15
            while r >= 255:
                out.append(255)
                r -= 255
            out.append(r)
        out.extend(data[lit_a:lit_b])
        if last:
            return
        out.extend(struct.pack("<H", off))
        if mlen - 4 >= 15:
            r = mlen - 4 - 15
            while r >= 255:
                out.append(255)
                r -= 255
            out.append(r)

    while i + _MFLIMIT <= n:
        key = data[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is not None and i - j < 65536:
            ln = 4
            while i + ln < n - _LASTLITERALS and data[j + ln] == data[i + ln]:
                ln += 1
            seq(anchor, i, i - j, ln)
            i += ln
            anchor = i
        else:
            i += 1
    seq(anchor, n, last=True)
    return bytes(out)


def lz4_decompress(buf: bytes) -> bytes:
    out = bytearray()
    i = 0
    while i < len(buf):
        tok = buf[i]
        i += 1
        ll = tok >> 4
        if ll == 15:
            while True:
                b = buf[i]
                i += 1
                ll += b
                if b != 255:
                    break
        out += buf[i:i + ll]
        i += ll
        if i >= len(buf):
            break
        off = buf[i] | (buf[i + 1] << 8)
        i += 2
        ml = tok & 15
        if ml == 15:
            while True:
                b = buf[i]
                i += 1
                ml += b
                if b != 255:
                    break
        for _ in range(ml + 4):
            out.append(out[-off])
    return bytes(out)


def _compress(chunk: bytes, codec: int) -> bytes:
    if codec == PASS_THROUGH:
        return chunk
    if codec == SNAPPY:
        return snappy_compress(chunk)
    if codec == LZ4:
        return lz4_compress(chunk)
    if codec == LZ4_LENGTH_PREFIXED:  # LZ4CompressorWithLength: 4-byte little-endian length, then the block
        return struct.pack("<I", len(chunk)) + lz4_compress(chunk)
    if codec == ZSTANDARD:  # Zstd.compress(dst, src) at the default level: one frame with its content size
        return _zstd().compress(chunk, asbytes=True)
    raise ValueError(f"codec {codec} is not restated here")


def _decompress(chunk: bytes, codec: int) -> bytes:
    if codec == PASS_THROUGH:
        return chunk
    if codec == SNAPPY:
        return snappy_decompress(chunk)
    if codec == LZ4:
        return lz4_decompress(chunk)
    if codec == LZ4_LENGTH_PREFIXED:
        n = struct.unpack("<I", chunk[:4])[0]
        out = lz4_decompress(chunk[4:])
        assert len(out) == n
        return out
    if codec == ZSTANDARD:
        import pyarrow as pa
        n = _zstd_content_size(chunk)
        return _zstd().decompress(pa.py_buffer(chunk), decompressed_size=n, asbytes=True)
    raise ValueError(f"codec {codec} is not restated here")


def _zstd():
    import pyarrow as pa
    return pa.Codec("zstd", compression_level=3)  # zstd-jni's Zstd.compress default level (3)


def _zstd_content_size(frame: bytes) -> int:
    """Frame_Content_Size of a zstd frame header (RFC 8878 3.1.1.1): what Zstd.decompressedSize returns."""
    assert frame[:4] == b"\x28\xb5\x2f\xfd", "not a zstd frame"
    fhd = frame[4]
    fcs_flag, single, did_flag = fhd >> 6, (fhd >> 5) & 1, fhd & 3
    pos = 5 + (0 if single else 1) + (0, 1, 2, 4)[did_flag]
    size = (1 if single else 0, 2, 4, 8)[fcs_flag]
    assert size, "frame without a content size"
    v = int.from_bytes(frame[pos:pos + size], "little")
    return v + 256 if size == 2 else v


# ---- file ---------------------------------------------------------------------------------------------------------
def write_raw_forward(values: np.ndarray, data_type: int, codec: int = PASS_THROUGH, version: int = 2,
                      docs_per_chunk: int = DEFAULT_NUM_DOCS_PER_CHUNK) -> bytes:
    """The `<column>.sv.raw.fwd` bytes of `values` (doc order)."""
    be = np.ascontiguousarray(values, dtype=_BE[data_type])
    width = be.dtype.itemsize
    if version >= 4 and docs_per_chunk & (docs_per_chunk - 1):
        docs_per_chunk = 1 << (docs_per_chunk - 1).bit_length()
    total = len(be)
    nchunks = (total + docs_per_chunk - 1) // docs_per_chunk
    off_size = 8 if version >= 3 else 4
    # versions 2-4 (the writer's DEFAULT_VERSION 2 .. 4, BaseChunkSVForwardIndexWriter.java:74-75; version 1 files
    # predate it and are only read): seven header ints, dataHeaderStart = 28
    assert version in (2, 3, 4), version
    header = struct.pack(">iiiiiii", version, nchunks, docs_per_chunk, width, total, codec, 7 * 4)
    data_start = len(header) + nchunks * off_size
    chunks, offsets = [], []
    pos = data_start
    raw = be.tobytes()
    for c in range(nchunks):
        comp = _compress(raw[c * docs_per_chunk * width:(c + 1) * docs_per_chunk * width], codec)
        offsets.append(pos)
        chunks.append(comp)
        pos += len(comp)
    offs = b"".join(struct.pack(">q" if off_size == 8 else ">i", o) for o in offsets)
    return header + offs + b"".join(chunks)


def read_raw_forward(buf: bytes, data_type: int, num_docs: int) -> np.ndarray:
    """Values by doc id (native dtype), as FixedByteChunkSVForwardIndexReader returns them."""
    version, nchunks, per_chunk, width = struct.unpack(">iiii", buf[:16])
    codec, data_header = SNAPPY, 16
    if version > 1:
        codec, data_header = struct.unpack(">ii", buf[20:28])
    off_size = 8 if version >= 3 else 4
    offs = [struct.unpack(">q" if off_size == 8 else ">i", buf[data_header + k * off_size:
                                                                data_header + (k + 1) * off_size])[0]
            for k in range(nchunks)]
    parts = []
    for k in range(nchunks):
        end = offs[k + 1] if k + 1 < nchunks else len(buf)
        parts.append(_decompress(buf[offs[k]:end], codec))
    be = np.frombuffer(b"".join(parts), dtype=_BE[data_type])[:num_docs]
    assert len(be) == num_docs and be.dtype.itemsize == width
    return be.astype(be.dtype.newbyteorder("="))


def range_index_header(version: int = 2, min_value: int = 0) -> bytes:
    """The leading bytes of `<column>.bitmap.range`: BitSlicedRangeIndexCreator (version 2) writes int32 version,
    int64 min value, then its bit-slice bitmaps (BitSlicedRangeIndexCreator.java:115-125); the legacy
    RangeIndexCreator (version 1) starts with int32 version too (RangeIndexCreator.java:299-322).  The GPU path reads
    only the version (the doc sets come from the forward index), so test fixtures carry the header alone."""
    return struct.pack(">iq", version, min_value)


def maybe_codec_name(codec: Optional[int]) -> str:
    return {PASS_THROUGH: "PASS_THROUGH", SNAPPY: "SNAPPY", ZSTANDARD: "ZSTANDARD", LZ4: "LZ4",
            LZ4_LENGTH_PREFIXED: "LZ4_LENGTH_PREFIXED"}.get(codec, str(codec))
