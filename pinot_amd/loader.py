"""Immutable segment loader: a Pinot segment directory on disk -> ``SegmentData`` (host bytes for HBM upload).

Restates the parts of the server's load path this query path needs:

* segment directory resolution: ``<dir>/v3`` when present (SegmentDirectoryPaths.java:33,
  ``findSegmentDirectory``), else the v1 file-per-index layout;
* ``metadata.properties`` -> per-column metadata (segspi/index/metadata/ColumnMetadataImpl.java:130,
  ``fromPropertiesConfiguration`` :200-300; key names segspi/V1Constants.java:25-105);
* v1: one file per index, ``<col>.dict`` / ``.sv.unsorted.fwd`` / ``.sv.sorted.fwd`` / ``.bitmap.inv``
  (V1Constants.Indexes, FilePerIndexDirectory);
* v3: ``index_map`` (``<column>.<index>.startOffset|size``, parsed from the right because column names may
  contain '.') + ``columns.psf``, every index buffer preceded by the 8-byte magic marker 0xdeadbeefdeafbead
  (seglocal/segment/store/SingleFileIndexDirectory.java:71-75,214-260,290-316);
* STRING dictionaries: fixed-width values padded with ``segment.padding.character`` (legacy '%' when the key
  is absent, ColumnMetadataImpl.java:282-287), read back up to the first padding byte
  (seglocal/io/util/FixedByteValueReaderWriter.java:57-90).

* multi-value columns (``isSingleValues = false``): ``<col>.mv.fwd`` (FixedBitMVForwardIndexReader.java:58-75) with
  ``totalNumberOfEntries`` / ``maxNumberOfMultiValues`` from the metadata.

The loader only slices bytes; the GPU upload (``GpuSegment``) is the IndexingOverrides seam
(segspi/index/IndexingOverrides.java:82-92).  Shapes outside this path -- raw STRING / BYTES / JSON columns, raw
multi-value columns -- raise ``UnsupportedSegmentError`` so the server keeps its CPU readers for them.
"""
from __future__ import annotations

import io
import mmap
import os
import tarfile
from typing import Dict, Iterable, Optional

import numpy as np

from ._lib import PGPU_DOUBLE, PGPU_FLOAT, PGPU_INT, PGPU_LONG, PGPU_STRING
from .segment import ColumnIndexes, SegmentData, num_bits_per_value

MAGIC_MARKER = 0xDEADBEEFDEAFBEAD
MAGIC_MARKER_SIZE = 8
INDEX_MAP_FILE = "index_map"
INDEX_FILE = "columns.psf"
METADATA_FILE = "metadata.properties"
V3_SUBDIR = "v3"
LEGACY_PAD = "%"

# stored types the kernels read (FieldSpec.DataType.getStoredType: BOOLEAN -> INT, TIMESTAMP -> LONG)
_STORED_TYPE = {"INT": PGPU_INT, "BOOLEAN": PGPU_INT, "LONG": PGPU_LONG, "TIMESTAMP": PGPU_LONG,
                "FLOAT": PGPU_FLOAT, "DOUBLE": PGPU_DOUBLE, "STRING": PGPU_STRING}
_V1_EXT = {"dictionary": ".dict", "forward_unsorted": ".sv.unsorted.fwd", "forward_sorted": ".sv.sorted.fwd",
           "forward_raw": ".sv.raw.fwd", "forward_mv": ".mv.fwd", "inverted_index": ".bitmap.inv",
           "range_index": ".bitmap.range"}


class UnsupportedSegmentError(ValueError):
    """A column or layout this query path does not serve (the server keeps the CPU readers for it)."""


class SegmentFormatError(ValueError):
    """Corrupt or inconsistent segment files (missing magic marker, bad index_map, size mismatch)."""


def _unescape(s: str) -> str:
    r"""Java properties escapes: ``\\``, ``\uXXXX``, ``\t \n \r \f``, and escaped separators."""
    if "\\" not in s:
        return s
    out, i = [], 0
    while i < len(s):
        c = s[i]
        if c != "\\" or i + 1 == len(s):
            out.append(c)
            i += 1
            continue
        n = s[i + 1]
        if n == "u" and i + 6 <= len(s):
            out.append(chr(int(s[i + 2:i + 6], 16)))
            i += 6
            continue
        out.append({"t": "\t", "n": "\n", "r": "\r", "f": "\f"}.get(n, n))
        i += 2
    return "".join(out)


def read_properties(text: str) -> Dict[str, str]:
    """Parse a Java ``.properties`` file as commons-configuration does for Pinot's metadata (one logical line
    per key, ``key = value`` or ``key: value``, ``#`` / ``!`` comments, backslash line continuation)."""
    props: Dict[str, str] = {}
    lines = text.splitlines()
    i = 0
    while i < len(lines):
        line = lines[i].lstrip()
        i += 1
        if not line or line[0] in "#!":
            continue
        while line.endswith("\\") and not line.endswith("\\\\") and i < len(lines):
            line = line[:-1] + lines[i].lstrip()
            i += 1
        k = 0  # the key ends at the first unescaped '=', ':' or whitespace
        while k < len(line) and line[k] not in "=: \t\f":
            k += 2 if line[k] == "\\" else 1
        key = line[:k].rstrip()
        rest = line[k:].lstrip()
        if rest[:1] in ("=", ":"):
            rest = rest[1:].lstrip()
        props[_unescape(key)] = _unescape(rest)
    return props


def _java_unescape(s: str) -> str:
    """StringEscapeUtils.unescapeJava for the padding character value (a second escape level on top of the
    properties file's own: the file holds ``\\\\u0000``)."""
    return _unescape(s)


class _Source:
    """Files of one segment directory: a directory on disk or the members of a .tar.gz."""

    def __init__(self, path: str):
        self._tar: Optional[Dict[str, bytes]] = None
        if os.path.isdir(path):
            self.root = path
        elif tarfile.is_tarfile(path):
            self._tar = {}
            with tarfile.open(path, "r:*") as tf:
                for m in tf.getmembers():
                    if m.isfile():
                        f = tf.extractfile(m)
                        self._tar[os.path.normpath(m.name)] = f.read()
            tops = sorted({n.split(os.sep)[0] for n in self._tar})
            if len(tops) != 1:
                raise SegmentFormatError(f"{path}: expected one segment directory in the archive, got {tops}")
            self.root = tops[0]
        else:
            raise FileNotFoundError(path)
        if self.exists(os.path.join(self.root, V3_SUBDIR, METADATA_FILE)):
            self.root = os.path.join(self.root, V3_SUBDIR)

    def exists(self, p: str) -> bool:
        return os.path.normpath(p) in self._tar if self._tar is not None else os.path.isfile(p)

    def read(self, name: str) -> bytes:
        p = os.path.join(self.root, name)
        if self._tar is not None:
            try:
                return self._tar[os.path.normpath(p)]
            except KeyError:
                raise FileNotFoundError(p) from None
        with open(p, "rb") as f:
            return f.read()

    def has(self, name: str) -> bool:
        return self.exists(os.path.join(self.root, name))

    def map(self, name: str):
        """Whole-file view: mmap for files on disk (columns.psf can be GBs), bytes inside an archive."""
        if self._tar is not None:
            return memoryview(self.read(name))
        p = os.path.join(self.root, name)
        if os.path.getsize(p) == 0:
            return memoryview(b"")
        with open(p, "rb") as f:
            return memoryview(mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ))


def read_index_map(text: str) -> Dict[tuple, tuple]:
    """index_map -> {(column, index_name): (start_offset, size)} (SingleFileIndexDirectory.loadMap :214-260)."""
    entries: Dict[tuple, list] = {}
    for key, value in read_properties(text).items():
        last = key.rfind(".")
        if last < 0:
            raise SegmentFormatError(f"index_map: key separator not found: {key}")
        prop = key[last + 1:]
        sep = key.rfind(".", 0, last)
        if sep < 0:
            raise SegmentFormatError(f"index_map: index separator not found: {key}")
        ent = entries.setdefault((key[:sep], key[sep + 1:last].lower()), [-1, -1])
        if prop == "startOffset":
            ent[0] = int(value)
        elif prop == "size":
            ent[1] = int(value)
        else:
            raise SegmentFormatError(f"index_map: invalid key {key}")
    for k, (start, size) in entries.items():
        if start < 0 or size < 0:
            raise SegmentFormatError(f"index_map: invalid entry for {k}")
    return {k: (v[0], v[1]) for k, v in entries.items()}


def _col_meta(props: Dict[str, str], col: str, key: str, default=None):
    v = props.get(f"column.{col}.{key}", default)
    if v is None:
        raise SegmentFormatError(f"metadata.properties: missing column.{col}.{key}")
    return v


def _column_names(props: Dict[str, str]) -> list:
    names = []
    for k in props:
        if k.startswith("column.") and k.endswith(".cardinality"):
            names.append(k[len("column."):-len(".cardinality")])
    return names


def _string_values(buf: bytes, card: int, width: int, pad: bytes) -> list:
    if len(buf) != card * width:
        raise SegmentFormatError(f"STRING dictionary size {len(buf)} != {card} x {width}")
    out = []
    for i in range(card):
        v = buf[i * width:(i + 1) * width]
        j = v.find(pad)
        out.append((v if j < 0 else v[:j]).decode("utf-8"))
    return out


def load_segment(path: str, columns: Optional[Iterable[str]] = None) -> SegmentData:
    """Load an immutable segment (directory or .tar.gz; v1 or v3 layout) into ``SegmentData``.

    ``columns`` restricts the load to the columns a query references (the server loads all; HBM holds only what
    the GPU path reads).  Mirrors ImmutableSegmentLoader.load (seglocal/indexsegment/immutable/
    ImmutableSegmentLoader.java:153-214) for single-value dictionary-encoded columns."""
    src = _Source(path)
    props = read_properties(src.read(METADATA_FILE).decode("utf-8"))
    name = props.get("segment.name", os.path.basename(os.path.normpath(path)))
    num_docs = int(props["segment.total.docs"])
    pad_raw = props.get("segment.padding.character")
    pad_char = LEGACY_PAD if pad_raw is None else _java_unescape(pad_raw)[0]
    v3 = src.has(INDEX_MAP_FILE)
    if v3:
        index_map = read_index_map(src.read(INDEX_MAP_FILE).decode("utf-8"))
        psf = src.map(INDEX_FILE)

    def index_bytes(col: str, kind: str) -> Optional[bytes]:
        if v3:
            ikind = "forward_index" if kind.startswith("forward") else kind
            ent = index_map.get((col, ikind))
            if ent is None:
                return None
            start, size = ent
            if start + size > len(psf) or size < MAGIC_MARKER_SIZE:
                raise SegmentFormatError(f"{col}.{ikind}: entry [{start}, +{size}) outside {INDEX_FILE}")
            marker = int.from_bytes(psf[start:start + MAGIC_MARKER_SIZE], "big")
            if marker != MAGIC_MARKER:
                raise SegmentFormatError(f"missing magic marker in {INDEX_FILE} at position {start} ({col}.{ikind})")
            return bytes(psf[start + MAGIC_MARKER_SIZE:start + size])
        fname = col + _V1_EXT[kind]
        return src.read(fname) if src.has(fname) else None

    wanted = list(columns) if columns is not None else _column_names(props)
    seg = SegmentData(name, num_docs)
    for col in wanted:
        card = int(_col_meta(props, col, "cardinality"))
        dtype_name = _col_meta(props, col, "dataType").upper()
        if dtype_name not in _STORED_TYPE:
            raise UnsupportedSegmentError(f"column {col}: data type {dtype_name} is not on the GPU path")
        mv = _col_meta(props, col, "isSingleValues", "true").lower() != "true"
        dt = _STORED_TYPE[dtype_name]
        if mv and _col_meta(props, col, "hasDictionary", "true").lower() != "true":
            raise UnsupportedSegmentError(f"column {col}: raw multi-value column")
        if mv and dt == PGPU_STRING:
            raise UnsupportedSegmentError(f"column {col}: multi-value STRING column")
        if _col_meta(props, col, "hasDictionary", "true").lower() != "true":
            # raw (no-dictionary) column: FixedByteChunkSVForwardIndexReader bytes, decoded in the library
            if dt == PGPU_STRING:
                raise UnsupportedSegmentError(f"column {col}: raw STRING (var-byte) forward index")
            fwd = index_bytes(col, "forward_raw")
            if fwd is None:
                raise SegmentFormatError(f"column {col}: raw forward index not found")
            c = ColumnIndexes(col, dt, card, raw_forward=fwd, range_index=index_bytes(col, "range_index"))
            mn, mx = props.get(f"column.{col}.minValue"), props.get(f"column.{col}.maxValue")
            if mn is not None and mx is not None:  # ColumnMetadataImpl min / max (the non-scan MIN / MAX)
                c.min_value, c.max_value = float(mn), float(mx)
            seg.columns[col] = c
            continue
        is_sorted = _col_meta(props, col, "isSorted", "false").lower() == "true"
        bits = int(_col_meta(props, col, "bitsPerElement", num_bits_per_value(card - 1)))
        if not is_sorted and bits != num_bits_per_value(card - 1):
            raise SegmentFormatError(f"column {col}: bitsPerElement {bits} != bits for cardinality {card}")
        dict_bytes = index_bytes(col, "dictionary")
        if dict_bytes is None:
            raise SegmentFormatError(f"column {col}: dictionary not found")
        c = ColumnIndexes(col, dt, card)
        if dt == PGPU_STRING:
            width = int(_col_meta(props, col, "lengthOfEachEntry"))
            c.dictionary = _string_values(dict_bytes, card, width, pad_char.encode("utf-8")[:1])
            c.pad_char, c.entry_width = pad_char, width
        else:
            if len(dict_bytes) != card * np.dtype(
                    {PGPU_INT: ">i4", PGPU_LONG: ">i8", PGPU_FLOAT: ">f4", PGPU_DOUBLE: ">f8"}[dt]).itemsize:
                raise SegmentFormatError(f"column {col}: dictionary size {len(dict_bytes)} for cardinality {card}")
            c.dictionary = dict_bytes
        if mv:
            fwd = index_bytes(col, "forward_mv")
            nv = int(_col_meta(props, col, "totalNumberOfEntries"))
            if fwd is None:
                raise SegmentFormatError(f"column {col}: multi-value forward index not found")
            if num_docs <= 0 or nv < num_docs:
                raise SegmentFormatError(f"column {col}: {nv} entries for {num_docs} docs")
            c.mv_forward, c.num_values = fwd, nv
            c.max_values = int(_col_meta(props, col, "maxNumberOfMultiValues", "0"))
        elif is_sorted:
            fwd = index_bytes(col, "forward_sorted")
            if fwd is None or len(fwd) < 8 * card:
                raise SegmentFormatError(f"column {col}: sorted index missing or short")
            c.sorted_index = fwd[:8 * card]
        else:
            fwd = index_bytes(col, "forward_unsorted")
            need = (num_docs * bits + 7) // 8
            if fwd is None or len(fwd) < need:
                raise SegmentFormatError(f"column {col}: forward index missing or shorter than {need} bytes")
            c.forward = fwd
        c.inverted = index_bytes(col, "inverted_index")
        c.range_index = index_bytes(col, "range_index")
        seg.columns[col] = c
    return seg
