"""ctypes binding of libpinotgpu.so (include/pinot_gpu.h).

This is the host-side view of the drop-in boundary: the same entry points a Pinot server binds through JNI
(INTEGRATION.md).  The library is built in-tree by ``__graft_entry__.build()``; importing this module on a machine
without the built library, or calling into it without a gfx950 device, raises — there is no CPU fallback on the
product path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpinotgpu.so")
PROF_LIB_PATH = os.path.join(_HERE, "libpinotgpu_prof.so")  # in-kernel phase counters (PGPU_PROFILE=1)
SYNTH_LIB_PATH = os.path.join(_HERE, "libpinotgpu_synth.so")

# ---- constants (mirror include/pinot_gpu.h) ------------------------------------------------------------------
PGPU_OK = 0
PGPU_MAX_SECTIONS = 17  # include/pinot_gpu.h: count + 16 value sections
PGPU_E_INVALID = -1
PGPU_E_HIP = -2
PGPU_E_UNSUPPORTED = -3
PGPU_E_NOT_FOUND = -4
PGPU_E_TIMEOUT = -5
PGPU_E_CANCELLED = -6
PGPU_E_GROUPS_LIMIT = -7

PGPU_INT, PGPU_LONG, PGPU_FLOAT, PGPU_DOUBLE, PGPU_STRING = range(5)
PGPU_MEM_HOST, PGPU_MEM_DEVICE = 0, 1

(PGPU_F_MATCH_ALL, PGPU_F_EMPTY, PGPU_F_SCAN, PGPU_F_INVERTED, PGPU_F_SORTED, PGPU_F_AND_BEGIN,
 PGPU_F_AND_CHILD_END, PGPU_F_AND_END, PGPU_F_OR_BEGIN, PGPU_F_OR_CHILD_END, PGPU_F_OR_END, PGPU_F_NOT,
 PGPU_F_RAW_SCAN, PGPU_F_RANGE_INDEX) = range(14)
PGPU_PRED_RANGE, PGPU_PRED_SET = 0, 1
PGPU_AGG_COUNT, PGPU_AGG_SUM, PGPU_AGG_MIN, PGPU_AGG_MAX, PGPU_AGG_AVG = range(5)
PGPU_RED_SUM_I64, PGPU_RED_SUM_F64, PGPU_RED_MIN_I64, PGPU_RED_MAX_I64 = range(4)
PGPU_Q_STATS, PGPU_Q_PARTITION, PGPU_Q_PART_SPILL, PGPU_Q_SUM_SPLIT, PGPU_Q_HASH = 1, 2, 4, 8, 16
PGPU_Q_EXACT_FILTER_STATS = 32
PGPU_KEYS_DENSE, PGPU_KEYS_HASH = 0, 1
PGPU_PART_BITS = 21  # split integer SUM: three sections of 21-bit parts (include/pinot_gpu.h)
PGPU_SUM_EXP_F64 = 32767  # pgpu_table_layout.agg_sum_exp of a float64 SUM section
PGPU_SUM_EXP_ZERO = -32767  # ... of a fixed-point SUM over a column holding only zeros
PGPU_MAX_FIXED_PARTS = 6  # widest fixed-point window (21-bit parts) of a floating SUM
PGPU_FIXED_TOL_BITS = 40
ABI_VERSION = 12


class PinotGpuError(RuntimeError):
    """Non-zero status from libpinotgpu (the IntermediateResultsBlock(Exception) path of the reference)."""

    def __init__(self, code: int, message: str):
        super().__init__(f"libpinotgpu status {code}: {message}")
        self.code = code


class UnsupportedPlanError(PinotGpuError):
    """PGPU_E_UNSUPPORTED: the server keeps the reference CPU plan for this query."""


class GroupsLimitError(UnsupportedPlanError):
    """PGPU_E_GROUPS_LIMIT: a segment met more distinct group keys than numGroupsLimit; the reference keeps its
    first-seen keys only (GpuPlanMaker.execute re-runs such segments with their first docs, or the server keeps the
    CPU plan -- an UnsupportedPlanError to callers that know no better)."""


class QueryTimeoutError(PinotGpuError):
    """PGPU_E_TIMEOUT: the query passed its deadline (QueryException.EXECUTION_TIMEOUT_ERROR,
    BaseCombineOperator.java:194-203)."""


class QueryCancelledError(PinotGpuError):
    """PGPU_E_CANCELLED: pgpu_query_cancel stopped the query."""


# ---- structs -------------------------------------------------------------------------------------------------
class FilterNode(C.Structure):
    _fields_ = [("op", C.c_int32), ("column", C.c_int32), ("pred", C.c_int32), ("negate", C.c_int32),
                ("lo", C.c_int32), ("hi", C.c_int32), ("ids", C.POINTER(C.c_int32)), ("num_ids", C.c_int32),
                ("reserved", C.c_int32), ("values", C.c_void_p)]


class Agg(C.Structure):
    _fields_ = [("fn", C.c_int32), ("column", C.c_int32)]


class SegmentPlan(C.Structure):
    _fields_ = [("segment", C.c_void_p), ("column_map", C.POINTER(C.c_int32)), ("filter", C.POINTER(FilterNode)),
                ("num_filter_nodes", C.c_int32), ("reserved", C.c_int32), ("group_remap", C.POINTER(C.c_void_p))]


class QueryDesc(C.Structure):
    _fields_ = [("num_columns", C.c_int32), ("num_segments", C.c_int32), ("segments", C.POINTER(SegmentPlan)),
                ("num_aggs", C.c_int32), ("num_group_columns", C.c_int32), ("aggs", C.POINTER(Agg)),
                ("group_columns", C.POINTER(C.c_int32)), ("group_cardinalities", C.POINTER(C.c_int32)),
                ("flags", C.c_uint64), ("reduce_docs", C.c_int64), ("num_groups_limit", C.c_int32),
                ("array_based_threshold", C.c_int32), ("deadline_ms", C.c_int64),
                ("sum_exp", C.POINTER(C.c_int32)), ("sum_parts", C.POINTER(C.c_int32))]


class TableLayout(C.Structure):
    _fields_ = [("num_keys", C.c_uint64), ("num_sections", C.c_int32), ("section_op", C.c_int32 * 17),
                ("agg_section", C.c_int32 * 16), ("agg_value_type", C.c_int32 * 16),
                ("agg_sum_parts", C.c_int32 * 16), ("agg_sum_exp", C.c_int32 * 16), ("key_kind", C.c_int32),
                ("key_words", C.c_int32),
                ("key_split", C.c_int32), ("reserved", C.c_int32)]


class SegmentBytes(C.Structure):
    """pgpu_segment_bytes: HBM bytes of a segment by kind (pgpu_segment_device_bytes_ex)."""
    _fields_ = [(n, C.c_uint64) for n in ("forward", "dictionary", "sorted", "inverted", "multi_value", "sliced",
                                           "value_planes", "total")]


# pgpu_query_stats.kernel_variant
PGPU_KV_RING, PGPU_KV_DIRECT, PGPU_KV_RDIRECT, PGPU_KV_RSTREAM, PGPU_KV_RPROG, PGPU_KV_RKEY, PGPU_KV_CAND, PGPU_KV_PSCAN, \
    PGPU_KV_RFSM = range(9)

# derived copies seal may build per column (pgpu_segment_set_derived)
PGPU_DERIVE_SLICED, PGPU_DERIVE_VALUE_PLANES, PGPU_DERIVE_ALL = 1, 2, 3


class QueryStats(C.Structure):
    _fields_ = [("num_docs_scanned", C.c_int64), ("num_entries_scanned_in_filter", C.c_int64),
                ("num_total_docs", C.c_int64), ("num_segments_matched", C.c_int64),
                ("sparse_sector_bytes", C.c_int64), ("dense_bytes", C.c_int64), ("kernel_ms", C.c_double),
                ("filter_stats_exact", C.c_int64), ("num_groups_limit_reached", C.c_int64),
                ("kernel_variant", C.c_int64)]


PGPU_TOPK_AGG, PGPU_TOPK_GROUP = 0, 1


class TopK(C.Structure):
    _fields_ = [("source", C.c_int32), ("agg_fn", C.c_int32), ("agg_index", C.c_int32), ("group_index", C.c_int32),
                ("descending", C.c_int32), ("num_group_columns", C.c_int32),
                ("group_cardinalities", C.POINTER(C.c_int32)), ("k", C.c_uint64), ("key_base", C.c_uint64)]


PGPU_X_PRED, PGPU_X_AND, PGPU_X_OR, PGPU_X_NOT = range(4)
PGPU_P_EQ, PGPU_P_NOT_EQ, PGPU_P_IN, PGPU_P_NOT_IN, PGPU_P_RANGE = range(5)


class Literal(C.Structure):
    _fields_ = [("i", C.c_int64), ("d", C.c_double), ("is_integral", C.c_int32), ("reserved", C.c_int32)]


class ExprNode(C.Structure):
    _fields_ = [("op", C.c_int32), ("num_children", C.c_int32), ("column", C.c_int32), ("pred", C.c_int32),
                ("lower_unbounded", C.c_int32), ("upper_unbounded", C.c_int32), ("lower_inclusive", C.c_int32),
                ("upper_inclusive", C.c_int32), ("num_values", C.c_int32), ("reserved", C.c_int32),
                ("values", C.POINTER(Literal))]


# exported symbols and their signatures: (name, restype, argtypes)
_P = C.c_void_p
SIGNATURES = [
    ("pgpu_abi_version", C.c_int, []),
    ("pgpu_init", C.c_int, [C.c_int, C.POINTER(_P)]),
    ("pgpu_shutdown", C.c_int, [_P]),
    ("pgpu_last_error", C.c_int, [C.c_char_p, C.c_size_t]),
    ("pgpu_segment_create", C.c_int, [_P, C.c_int32, C.c_int32, C.POINTER(_P)]),
    ("pgpu_segment_add_forward_index", C.c_int, [_P, C.c_int32, _P, C.c_uint64, C.c_int32, C.c_int32, C.c_int32]),
    ("pgpu_segment_add_sorted_index", C.c_int, [_P, C.c_int32, _P, C.c_uint64, C.c_int32]),
    ("pgpu_segment_add_dictionary", C.c_int, [_P, C.c_int32, C.c_int32, _P, C.c_uint64, C.c_int32]),
    ("pgpu_segment_add_inverted_index", C.c_int, [_P, C.c_int32, _P, C.c_uint64, C.c_int32]),
    ("pgpu_segment_add_raw_forward_index", C.c_int, [_P, C.c_int32, C.c_int32, _P, C.c_uint64]),
    ("pgpu_segment_add_range_index", C.c_int, [_P, C.c_int32, _P, C.c_uint64]),
    ("pgpu_segment_add_mv_forward_index", C.c_int, [_P, C.c_int32, _P, C.c_uint64, C.c_int32, C.c_int32, C.c_int64]),
    ("pgpu_segment_add_mv_row_columns", C.c_int, [_P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    ("pgpu_segment_seal", C.c_int, [_P]),
    ("pgpu_segment_add_group_dictionary", C.c_int, [_P, C.c_int32, C.c_int32, C.POINTER(C.c_int32)]),
    ("pgpu_segment_add_docid_column", C.c_int, [_P, C.c_int32]),
    ("pgpu_segment_dictionary_values", C.c_int, [_P, C.c_int32, _P, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("pgpu_segment_device_bytes", C.c_int, [_P, C.POINTER(C.c_uint64)]),
    ("pgpu_segment_device_bytes_ex", C.c_int, [_P, C.POINTER(SegmentBytes)]),
    ("pgpu_segment_set_derived", C.c_int, [_P, C.c_int32, C.c_int32]),
    ("pgpu_context_set_derived_budget", C.c_int, [_P, C.c_uint64]),
    ("pgpu_context_derived_bytes", C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("pgpu_segment_release", C.c_int, [_P]),
    ("pgpu_remap_upload", C.c_int, [_P, C.POINTER(C.c_int32), C.c_int32, C.POINTER(_P)]),
    ("pgpu_buffer_release", C.c_int, [_P]),
    ("pgpu_table_layout_of", C.c_int, [C.POINTER(QueryDesc), C.POINTER(TableLayout)]),
    ("pgpu_fixed_sum_layout", None, [C.c_double, C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("pgpu_sum_layout_agree", C.c_int, [C.POINTER(TableLayout), C.c_int32, C.c_int32, C.POINTER(C.c_int32),
                                        C.POINTER(C.c_int32)]),
    ("pgpu_table_bytes", C.c_uint64, [C.POINTER(TableLayout)]),
    ("pgpu_query_launch", C.c_int, [_P, C.POINTER(QueryDesc), _P, _P, C.c_uint64, C.POINTER(_P)]),
    ("pgpu_query_wait", C.c_int, [_P, C.POINTER(QueryStats)]),
    ("pgpu_query_release", C.c_int, [_P]),
    ("pgpu_query_cancel", C.c_int, [_P]),
    ("pgpu_query_matched_segments", C.c_int, [_P, C.POINTER(C.c_uint8), C.c_int32]),
    ("pgpu_segment_mv_row", C.c_int, [_P, C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.c_int32,
                                      C.POINTER(C.c_int32)]),
    ("pgpu_table_compact", C.c_int, [_P, C.POINTER(TableLayout), _P, _P, C.POINTER(C.c_int64),
                                     C.POINTER(C.c_int64), C.c_uint64, C.POINTER(C.c_uint64)]),
    ("pgpu_table_topk", C.c_int, [_P, C.POINTER(TableLayout), _P, _P, C.POINTER(TopK), C.POINTER(C.c_int64),
                                  C.POINTER(C.c_int64), C.c_uint64, C.POINTER(C.c_uint64)]),
    ("pgpu_query_collect_topk", C.c_int, [_P, C.POINTER(TopK), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                          C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(QueryStats)]),
    ("pgpu_query_submit", C.c_int, [_P, C.POINTER(QueryDesc), C.POINTER(_P)]),
    ("pgpu_query_collect", C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_uint64,
                                     C.POINTER(C.c_uint64), C.POINTER(QueryStats)]),
    ("pgpu_query_submit_expr", C.c_int, [_P, C.POINTER(QueryDesc), C.POINTER(ExprNode), C.c_int32, C.POINTER(_P)]),
    ("pgpu_query_submit_ordered", C.c_int, [_P, C.POINTER(QueryDesc), C.POINTER(ExprNode), C.c_int32,
                                            C.POINTER(TopK), C.POINTER(_P)]),
    ("pgpu_query_launch_expr", C.c_int, [_P, C.POINTER(QueryDesc), C.POINTER(ExprNode), C.c_int32, _P, _P,
                                         C.c_uint64, C.POINTER(_P)]),
    ("pgpu_query_execute", C.c_int, [_P, C.POINTER(QueryDesc), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                     C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(QueryStats)]),
    ("pgpu_decode_minmax_key", C.c_double, [C.c_int64, C.c_int32]),
    ("pgpu_node_init", C.c_int, [C.POINTER(C.c_int32), C.c_int32, C.POINTER(_P)]),
    ("pgpu_node_context", C.c_int, [_P, C.c_int32, C.POINTER(_P)]),
    ("pgpu_node_shutdown", C.c_int, [_P]),
    ("pgpu_node_query", C.c_int, [_P, C.POINTER(C.POINTER(QueryDesc)), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                  C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(QueryStats), C.POINTER(TableLayout)]),
    ("pgpu_node_query_topk", C.c_int, [_P, C.POINTER(C.POINTER(QueryDesc)), C.POINTER(TopK), C.POINTER(C.c_int64),
                                       C.POINTER(C.c_int64), C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(QueryStats),
                                       C.POINTER(TableLayout)]),
    ("pgpu_node_submit", C.c_int, [_P, C.POINTER(C.POINTER(QueryDesc)), C.POINTER(_P)]),
    ("pgpu_node_submit_expr", C.c_int, [_P, C.POINTER(C.POINTER(QueryDesc)), C.POINTER(C.POINTER(ExprNode)),
                                        C.POINTER(C.c_int32), C.POINTER(_P)]),
    ("pgpu_node_collect", C.c_int, [_P, C.POINTER(TopK), C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_uint64,
                                    C.POINTER(C.c_uint64), C.POINTER(QueryStats), C.POINTER(TableLayout)]),
    ("pgpu_slice_of", None, [C.c_uint64, C.c_int32, C.c_int32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("pgpu_key_owner", C.c_int32, [C.POINTER(C.c_int64), C.c_int32, C.c_int32]),
    ("pgpu_filter_entries_scanned", C.c_int, [C.POINTER(FilterNode), C.c_int32, C.POINTER(C.POINTER(C.c_uint32)),
                                             C.c_int32, C.c_int32, C.POINTER(C.c_int64)]),
    ("pgpu_kernel_geometry", C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
]

_lib = None


def load(path: str = None) -> C.CDLL:
    """Load libpinotgpu.so (fails loudly when it was not built); PGPU_PROFILE=1 selects the profiling build."""
    global _lib
    if _lib is not None:
        return _lib
    if path is None:
        path = PROF_LIB_PATH if os.environ.get("PGPU_PROFILE") == "1" else LIB_PATH
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    lib = C.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.pgpu_abi_version() != ABI_VERSION:
        raise ImportError("libpinotgpu ABI version mismatch")
    _lib = lib
    return lib


def last_error() -> str:
    lib = load()
    buf = C.create_string_buffer(2048)
    lib.pgpu_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(rc: int) -> None:
    if rc != PGPU_OK:
        msg = last_error()
        if rc == PGPU_E_UNSUPPORTED:
            raise UnsupportedPlanError(rc, msg)
        if rc == PGPU_E_GROUPS_LIMIT:
            raise GroupsLimitError(rc, msg)
        if rc == PGPU_E_TIMEOUT:
            raise QueryTimeoutError(rc, msg)
        if rc == PGPU_E_CANCELLED:
            raise QueryCancelledError(rc, msg)
        raise PinotGpuError(rc, msg)


def table_bytes(layout: TableLayout) -> int:
    return int(load().pgpu_table_bytes(C.byref(layout)))


def decode_minmax_key(key: int, value_type: int) -> float:
    return load().pgpu_decode_minmax_key(key, value_type)
