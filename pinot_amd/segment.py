"""Immutable segment model and HBM residency (the IndexingOverrides seam).

``SegmentData`` holds, per column, exactly the bytes a Pinot server has in its ``PinotDataBuffer``s after
``ImmutableSegmentLoader.load`` (seglocal/indexsegment/immutable/ImmutableSegmentLoader.java:153-214):

* dictionary      ``<col>.dict``             sorted unique values, big-endian (BaseImmutableDictionary.java:40-322)
* forward index   ``<col>.sv.unsorted.fwd``  fixed-bit, MSB-first (FixedBitSVForwardIndexReaderV2.java:62-96)
* sorted index    ``<col>.sv.sorted.fwd``    (start, end) per dict id (SortedIndexReaderImpl.java:37-121)
* inverted index  ``<col>.bitmap.inv``       offsets + Roaring bitmaps (BitmapInvertedIndexReader.java:45-61)
* raw forward     ``<col>.sv.raw.fwd``       no-dictionary values in chunks (BaseChunkSVForwardIndexReader.java:56-101)
* range index     ``<col>.bitmap.range``     only its version is used (BitSlicedRangeIndexReader.java:41-55)
* MV forward      ``<col>.mv.fwd``           chunk offsets, row-start bitmap, fixed-bit ids
                                             (FixedBitMVForwardIndexReader.java:58-140)

(file names: segspi/V1Constants.java:25-105).  ``GpuSegment`` copies them to HBM once
(``pgpu_segment_add_*``), the analogue of an ``IndexingOverride`` wrapping ``newForwardIndexReader`` /
``newInvertedIndexReader`` / ``newSortedIndexReader`` (segspi/index/IndexingOverrides.java:82-92).  The host keeps
the decoded dictionary values: predicates are evaluated against them on the host, as the reference's
PredicateEvaluators do (core/operator/filter/predicate/PredicateEvaluatorProvider.java:38-89).
"""
from __future__ import annotations

import ctypes as C
import itertools
import weakref
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Union

import numpy as np

from . import _lib
from ._lib import PGPU_DOUBLE, PGPU_FLOAT, PGPU_INT, PGPU_LONG, PGPU_STRING

TYPE_NAMES = {"INT": PGPU_INT, "LONG": PGPU_LONG, "FLOAT": PGPU_FLOAT, "DOUBLE": PGPU_DOUBLE, "STRING": PGPU_STRING}
_BE_DTYPE = {PGPU_INT: ">i4", PGPU_LONG: ">i8", PGPU_FLOAT: ">f4", PGPU_DOUBLE: ">f8"}
_NATIVE = {PGPU_INT: np.int32, PGPU_LONG: np.int64, PGPU_FLOAT: np.float32, PGPU_DOUBLE: np.float64}


def num_bits_per_value(max_value: int) -> int:
    """PinotDataBitSet.getNumBitsPerValue (seglocal/io/util/PinotDataBitSet.java:59-71)."""
    if max_value <= 1:
        return 1
    return int(max_value).bit_length()


@dataclass
class ColumnIndexes:
    """Per-column index buffers of one immutable segment (PhysicalColumnIndexContainer wiring)."""

    name: str
    data_type: int
    cardinality: int
    dictionary: Union[bytes, Sequence[str], None] = None  # BE bytes (numeric) or sorted strings
    forward: Optional[bytes] = None          # fixed-bit forward index (unsorted columns)
    sorted_index: Optional[bytes] = None     # sorted columns: also their forward index
    inverted: Optional[bytes] = None
    forward_device: Optional[int] = None     # device pointer alternative to `forward` (PGPU_MEM_DEVICE)
    forward_device_bytes: int = 0
    pad_char: str = "\0"                    # STRING dictionaries: segment.padding.character (legacy '%')
    entry_width: int = 0                     # STRING dictionaries: lengthOfEachEntry (bytes per padded value)
    raw_forward: Optional[bytes] = None      # no-dictionary column: the FixedByteChunkSVForwardIndexWriter file
    range_index: Optional[bytes] = None      # `<col>.bitmap.range` (its header version decides the leaf's stats)
    min_value: Optional[float] = None        # metadata min / max (raw columns: the non-scan MIN / MAX answer,
    max_value: Optional[float] = None        # NonScanBasedAggregationOperator via DataSourceMetadata)
    mv_forward: Optional[bytes] = None       # multi-value column: the FixedBitMVForwardIndexWriter file `<col>.mv.fwd`
    num_values: int = 0                      # multi-value: totalNumberOfEntries
    max_values: int = 0                      # multi-value: maxNumberOfMultiValues

    @property
    def is_mv(self) -> bool:
        return self.mv_forward is not None

    @property
    def is_raw(self) -> bool:
        return self.raw_forward is not None

    @property
    def range_index_version(self) -> int:
        if self.range_index is None:
            return 0
        return int.from_bytes(self.range_index[:4], "big")

    @property
    def bits_per_value(self) -> int:
        return num_bits_per_value(self.cardinality - 1)

    @property
    def is_sorted(self) -> bool:
        return self.sorted_index is not None

    def dictionary_values(self) -> Union[np.ndarray, List[str], None]:
        if self.is_raw:
            return None
        if self.data_type == PGPU_STRING:
            return list(self.dictionary)
        return np.frombuffer(self.dictionary, dtype=_BE_DTYPE[self.data_type]).astype(_NATIVE[self.data_type])


@dataclass
class SegmentData:
    name: str
    num_docs: int
    columns: Dict[str, ColumnIndexes] = field(default_factory=dict)

    def column(self, name: str) -> ColumnIndexes:
        try:
            return self.columns[name]
        except KeyError:
            raise KeyError(f"segment {self.name} has no column {name!r}") from None


class GpuContext:
    """One HIP device (one process per GPU); wraps pgpu_init / pgpu_shutdown."""

    def __init__(self, device: int = 0, _handle: Optional[C.c_void_p] = None):
        self._lib = _lib.load()
        self.owned = _handle is None  # a node's contexts are shut down by pgpu_node_shutdown
        if _handle is None:
            _handle = C.c_void_p()
            _lib.check(self._lib.pgpu_init(device, C.byref(_handle)))
        self.handle = _handle
        self.device = device
        self._remap_cache: Dict[tuple, "DeviceBuffer"] = {}
        self._remap_refs: Dict[tuple, int] = {}  # holders of each cached remap table (remap / unref_remap)
        self._remap_bytes = 0
        # caches of per-segment derived state (plan makers' global dictionaries, executors' agreements) that must
        # forget a segment when it is released: objects with a segment_released(uid) method, held weakly
        self._listeners: "weakref.WeakSet" = weakref.WeakSet()

    def add_listener(self, obj) -> None:
        self._listeners.add(obj)

    def set_derived_budget(self, nbytes: int) -> None:
        """HBM the derived copies of this context's segments may take (pgpu_context_set_derived_budget)."""
        _lib.check(self._lib.pgpu_context_set_derived_budget(self.handle, int(nbytes)))

    def derived_bytes(self):
        """(bytes held by derived copies, budget)."""
        used, budget = C.c_uint64(), C.c_uint64()
        _lib.check(self._lib.pgpu_context_derived_bytes(self.handle, C.byref(used), C.byref(budget)))
        return used.value, budget.value

    def segment_released(self, uid: int) -> None:
        """A segment left HBM: drop its remap tables and every cache entry naming it (bounded host / HBM state
        in a server whose pruning yields a different segment set per query)."""
        for k in [k for k in self._remap_cache if k[0] == uid]:
            self._drop_remap(k)
        for obj in list(self._listeners):
            obj.segment_released(uid)

    def _drop_remap(self, key: tuple) -> None:
        buf = self._remap_cache.pop(key)
        self._remap_refs.pop(key, None)
        self._remap_bytes -= buf.nbytes
        buf.release()

    def unref_remap(self, key: tuple) -> None:
        """One holder of a remap table (a cached global dictionary) let it go: freed when none is left."""
        n = self._remap_refs.get(key)
        if n is None:
            return  # already dropped with its segment
        if n <= 1:
            self._drop_remap(key)
        else:
            self._remap_refs[key] = n - 1

    def remap_bytes(self) -> int:
        """HBM held by cached group-key remap tables."""
        return self._remap_bytes

    def close(self) -> None:
        if self.handle:
            for b in self._remap_cache.values():
                b.release()
            self._remap_cache.clear()
            self._remap_refs.clear()
            self._remap_bytes = 0
            if self.owned:
                self._lib.pgpu_shutdown(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def kernel_geometry(self):
        g, t, b = C.c_int32(), C.c_int32(), C.c_int32()
        _lib.check(self._lib.pgpu_kernel_geometry(self.handle, C.byref(g), C.byref(t), C.byref(b)))
        return g.value, t.value, b.value

    def remap(self, key: tuple, table: np.ndarray) -> "DeviceBuffer":
        """The remap table cached under `key` (uploaded on first use); the caller holds a reference until
        unref_remap(key) or the release of the segment key[0]."""
        buf = self._remap_cache.get(key)
        if buf is None:
            buf = self._upload_remap(table)
            self._remap_cache[key] = buf
            self._remap_bytes += buf.nbytes
        self._remap_refs[key] = self._remap_refs.get(key, 0) + 1
        return buf

    def _upload_remap(self, table: np.ndarray) -> "DeviceBuffer":
        return DeviceBuffer.upload_int32(self, table)


class DeviceBuffer:
    def __init__(self, ctx: GpuContext, handle: C.c_void_p, nbytes: int = 0):
        self.ctx = ctx
        self.handle = handle
        self.nbytes = nbytes

    @staticmethod
    def upload_int32(ctx: GpuContext, arr: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(arr, dtype=np.int32)
        h = C.c_void_p()
        _lib.check(ctx._lib.pgpu_remap_upload(ctx.handle, a.ctypes.data_as(C.POINTER(C.c_int32)), len(a),
                                              C.byref(h)))
        return DeviceBuffer(ctx, h, 4 * len(a))

    def release(self) -> None:
        if self.handle:
            self.ctx._lib.pgpu_buffer_release(self.handle)
            self.handle = None


_UIDS = itertools.count(1)

MV_ROW_COLUMNS = ("len", "sum", "min", "max")


def mv_row_column(column: str, kind: str) -> str:
    """Slot name of a multi-value column's per-row reduction (GpuSegment._add_row_columns)."""
    return f"{column}$mv{kind}"


DOCID_COLUMN = "$docId"  # GpuSegment.docid_view


def group_dict_column(column: str) -> str:
    """Slot name of a raw column's on-the-fly group dictionary (GpuSegment.group_view)."""
    return f"{column}$gdict"


class GpuSegment:
    """An immutable segment resident in HBM plus the host-side dictionaries used for predicate evaluation.

    ``uid`` is unique for the life of the process (never reused, unlike ``id()``): host-side caches of derived
    per-segment state (global group dictionaries, remap tables) key on it."""

    def __init__(self, ctx: GpuContext, data: SegmentData, columns: Optional[Sequence[str]] = None,
                 _incremental: bool = False, derived: Optional[Dict[str, int]] = None):
        """``derived``: column -> PGPU_DERIVE_* flags of the copies seal builds for it (the table's GPU filter /
        metric columns, GpuExecutorConfig.derived_flags); columns it does not name get both (the default)."""
        self.ctx = ctx
        self.uid = next(_UIDS)
        self.data = data
        self.name = data.name
        self.num_docs = data.num_docs
        names = list(columns) if columns is not None else list(data.columns)
        self.slots: Dict[str, int] = {}
        self.dictionaries: Dict[str, Union[np.ndarray, List[str]]] = {}
        # multi-value columns' per-row reductions (mv_row_columns): raw columns of their own slots
        self.derived: Dict[str, ColumnIndexes] = {}
        nmv = 0 if _incremental else sum(1 for n in names if data.column(n).is_mv)
        # one spare slot per raw column for its on-the-fly group dictionary (group_view), filled on first use
        nraw = 0 if _incremental else sum(1 for n in names if data.column(n).is_raw)
        lib = ctx._lib
        h = C.c_void_p()
        # + the doc-id column's slot (docid_view), filled on first use
        nslots = len(names) + len(MV_ROW_COLUMNS) * nmv + nraw + (0 if _incremental else 1)
        _lib.check(lib.pgpu_segment_create(ctx.handle, data.num_docs, nslots, C.byref(h)))
        self.handle = h
        self._capacity = nslots
        self._gdict_free = list(range(nslots - nraw - 1, nslots - 1))  # spare slots (after every column's own)
        self._docid_slot = None if _incremental else nslots - 1
        self._derived_flags = dict(derived or {})
        if _incremental:
            return
        try:
            for n in names:
                self.add_column(data.column(n))
            self.seal()
        except Exception:
            self.release()
            raise

    @classmethod
    def begin(cls, ctx: GpuContext, name: str, num_docs: int, num_columns: int,
              derived: Optional[Dict[str, int]] = None) -> "GpuSegment":
        """Incremental upload: add_column() per column, then seal()."""
        data = SegmentData(name, num_docs)
        return cls(ctx, data, columns=[f"_{i}" for i in range(num_columns)], _incremental=True, derived=derived)

    def add_column(self, col: ColumnIndexes) -> None:
        need = 1 + (len(MV_ROW_COLUMNS) if col.is_mv else 0)
        if len(self.slots) + need > self._capacity:
            raise ValueError("segment column capacity exceeded")
        slot = len(self.slots)
        self._upload_column(slot, col)
        if col.name in self._derived_flags:
            _lib.check(self.ctx._lib.pgpu_segment_set_derived(self.handle, slot, int(self._derived_flags[col.name])))
        self.slots[col.name] = slot
        self.dictionaries[col.name] = col.dictionary_values()
        self.data.columns[col.name] = col
        if col.is_mv:
            self._add_row_columns(slot, col)

    def _add_row_columns(self, slot: int, col: ColumnIndexes) -> None:
        """COUNTMV / SUMMV / MINMV / MAXMV / AVGMV read per-row reductions of the column (pgpu_segment_add_mv_row_columns):
        raw columns named ``<column>$mv<kind>``."""
        d = col.dictionary_values()
        fp = col.data_type in (PGPU_FLOAT, PGPU_DOUBLE)
        kinds = {"len": PGPU_INT, "sum": PGPU_DOUBLE if fp else PGPU_LONG, "min": col.data_type, "max": col.data_type}
        slots = {}
        for k in MV_ROW_COLUMNS:
            slots[k] = len(self.slots)
            name = mv_row_column(col.name, k)
            self.slots[name] = slots[k]
            self.dictionaries[name] = None
            # min / max metadata: the dictionary's ends (the non-scan MINMV / MAXMV answer)
            self.derived[name] = ColumnIndexes(name, kinds[k], 0, raw_forward=b"",
                                               min_value=float(d[0]) if len(d) else None,
                                               max_value=float(d[-1]) if len(d) else None)
        _lib.check(self.ctx._lib.pgpu_segment_add_mv_row_columns(self.handle, slot, slots["len"], slots["sum"],
                                                                 slots["min"], slots["max"]))

    def seal(self) -> None:
        _lib.check(self.ctx._lib.pgpu_segment_seal(self.handle))

    def _upload_column(self, slot: int, col: ColumnIndexes) -> None:
        lib = self.ctx._lib
        seg = self.handle
        card = col.cardinality
        if col.is_raw:
            r = col.raw_forward
            _lib.check(lib.pgpu_segment_add_raw_forward_index(seg, slot, col.data_type, r, len(r)))
            if col.range_index is not None:
                _lib.check(lib.pgpu_segment_add_range_index(seg, slot, col.range_index, len(col.range_index)))
            return
        if col.data_type == PGPU_STRING:
            if col.is_mv:
                raise _lib.UnsupportedPlanError(_lib.PGPU_E_UNSUPPORTED, f"multi-value STRING column {col.name}")
            _lib.check(lib.pgpu_segment_add_dictionary(seg, slot, PGPU_STRING, None, 0, card))
        else:
            d = col.dictionary
            _lib.check(lib.pgpu_segment_add_dictionary(seg, slot, col.data_type, d, len(d), card))
        if col.is_mv:
            f = col.mv_forward
            _lib.check(lib.pgpu_segment_add_mv_forward_index(seg, slot, f, len(f), col.bits_per_value, card,
                                                             col.num_values))
        elif col.sorted_index is not None:
            s = col.sorted_index
            _lib.check(lib.pgpu_segment_add_sorted_index(seg, slot, s, len(s), card))
        elif col.forward_device is not None:
            _lib.check(lib.pgpu_segment_add_forward_index(seg, slot, C.c_void_p(col.forward_device),
                                                          col.forward_device_bytes, col.bits_per_value, card,
                                                          _lib.PGPU_MEM_DEVICE))
        elif col.forward is not None:
            f = col.forward
            _lib.check(lib.pgpu_segment_add_forward_index(seg, slot, f, len(f), col.bits_per_value, card,
                                                          _lib.PGPU_MEM_HOST))
        if col.inverted is not None:
            inv = col.inverted
            _lib.check(lib.pgpu_segment_add_inverted_index(seg, slot, inv, len(inv), card))
        if col.range_index is not None:
            _lib.check(lib.pgpu_segment_add_range_index(seg, slot, col.range_index, len(col.range_index)))

    def group_view(self, name: str) -> str:
        """The column a GROUP BY on `name` reads in this segment: the column itself when it is dictionary-encoded;
        for a raw (no-dictionary) column its on-the-fly group dictionary (pgpu_segment_add_group_dictionary: the
        distinct values as a sorted dictionary + a fixed-bit id per doc, built on the GPU on first use and kept
        with the segment), the analogue of NoDictionary*GroupKeyGenerator's value -> id maps."""
        col = self.column(name)
        if not col.is_raw:
            return name
        gname = group_dict_column(name)
        if gname in self.slots:
            return gname
        if not self._gdict_free:
            raise _lib.UnsupportedPlanError(_lib.PGPU_E_UNSUPPORTED,
                                            f"no spare slot for the group dictionary of raw column {name!r}")
        slot = self._gdict_free.pop(0)
        lib = self.ctx._lib
        card = C.c_int32()
        _lib.check(lib.pgpu_segment_add_group_dictionary(self.handle, self.slots[name], slot, C.byref(card)))
        nb = C.c_uint64()
        _lib.check(lib.pgpu_segment_dictionary_values(self.handle, slot, None, 0, C.byref(nb)))
        buf = np.empty(nb.value, dtype=np.uint8)
        _lib.check(lib.pgpu_segment_dictionary_values(self.handle, slot, buf.ctypes.data, nb.value, C.byref(nb)))
        vals = buf.view(_NATIVE[col.data_type]).copy()
        self.slots[gname] = slot
        self.dictionaries[gname] = vals
        self.derived[gname] = ColumnIndexes(gname, col.data_type, card.value,
                                            dictionary=vals.astype(_BE_DTYPE[col.data_type]).tobytes())
        return gname

    def docid_view(self) -> str:
        """The doc-id column (pgpu_segment_add_docid_column: a raw INT column whose value at doc d is d), added on
        first use: MIN over it is each group's first doc, the order of the reference's first-seen group ids."""
        if DOCID_COLUMN in self.slots:
            return DOCID_COLUMN
        if self._docid_slot is None:
            raise _lib.UnsupportedPlanError(_lib.PGPU_E_UNSUPPORTED, "no doc-id slot (incrementally built segment)")
        _lib.check(self.ctx._lib.pgpu_segment_add_docid_column(self.handle, self._docid_slot))
        self.slots[DOCID_COLUMN] = self._docid_slot
        self.dictionaries[DOCID_COLUMN] = None
        self.derived[DOCID_COLUMN] = ColumnIndexes(DOCID_COLUMN, PGPU_INT, self.num_docs, raw_forward=b"",
                                                   min_value=0.0, max_value=float(max(self.num_docs - 1, 0)))
        return DOCID_COLUMN

    def mv_row(self, name: str, doc: int) -> np.ndarray:
        """Dict ids of doc `doc` of a multi-value column, in value order (pgpu_segment_mv_row)."""
        cap = max(1, self.column(name).max_values or 64)
        while True:
            out = np.empty(cap, dtype=np.int32)
            n = C.c_int32()
            _lib.check(self.ctx._lib.pgpu_segment_mv_row(self.handle, self.slots[name], int(doc),
                                                         out.ctypes.data_as(C.POINTER(C.c_int32)), cap, C.byref(n)))
            if n.value <= cap:
                return out[: n.value]
            cap = n.value

    def column(self, name: str) -> ColumnIndexes:
        c = self.derived.get(name)
        return c if c is not None else self.data.column(name)

    def sorted_dictionary(self, name: str):
        """Host dictionary used by the predicate evaluators (built once per segment column)."""
        cache = self.__dict__.setdefault("_sorted_dicts", {})
        d = cache.get(name)
        if d is None:
            from .predicate import SortedDictionary
            col = self.column(name)
            d = SortedDictionary(self.dictionaries[name], col.data_type, pad_char=col.pad_char,
                                 entry_width=col.entry_width)
            cache[name] = d
        return d

    def min_max(self, name: str):
        """(min, max) of a column as the non-scan plan reads them: the sorted dictionary's ends, or a raw column's
        metadata min / max (None when the metadata has none: the segment is then scanned)."""
        col = self.column(name)
        if col.is_raw:
            if col.min_value is None or col.max_value is None:
                return None
            return float(col.min_value), float(col.max_value)
        d = self.dictionaries[name]
        return float(d[0]), float(d[-1])

    def sorted_pairs(self, name: str) -> np.ndarray:
        cache = self.__dict__.setdefault("_sorted_pairs", {})
        p = cache.get(name)
        if p is None:
            p = np.frombuffer(self.column(name).sorted_index, dtype=">i4").reshape(-1, 2).astype(np.int64)
            cache[name] = p
        return p

    def has_column(self, name: str) -> bool:
        return name in self.slots

    def device_bytes(self) -> int:
        n = C.c_uint64()
        _lib.check(self.ctx._lib.pgpu_segment_device_bytes(self.handle, C.byref(n)))
        return n.value

    def device_bytes_by_kind(self) -> Dict[str, int]:
        """HBM bytes by kind: the reference's indexes and the derived copies (pgpu_segment_device_bytes_ex)."""
        b = _lib.SegmentBytes()
        _lib.check(self.ctx._lib.pgpu_segment_device_bytes_ex(self.handle, C.byref(b)))
        return {n: int(getattr(b, n)) for n, _ in _lib.SegmentBytes._fields_}

    def release(self) -> None:
        if self.handle:
            self.ctx.segment_released(self.uid)
            self.ctx._lib.pgpu_segment_release(self.handle)
            self.handle = None
