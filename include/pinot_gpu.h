/*
 * pinot_gpu.h — C ABI of libpinotgpu.so, the MI355X segment query path for Apache Pinot.
 *
 * This is the drop-in boundary.  A Pinot server binds these entry points (JNI stub in INTEGRATION.md) from
 *   - an IndexingOverride (segspi/index/IndexingOverrides.java:82-92) that uploads the forward index, dictionary,
 *     sorted index and bitmap inverted index bytes of every immutable segment to HBM once, at load time
 *     (seglocal/indexsegment/immutable/ImmutableSegmentLoader.java:186-187), and
 *   - a GpuPlanMaker (core/plan/maker/PlanMaker.java:36-59) whose per-query combine operator replaces
 *     BaseCombineOperator + AggregationOperator / AggregationGroupByOrderByOperator for the segments it owns
 *     (core/plan/CombinePlanNode.java:85-196, core/operator/combine/BaseCombineOperator.java:79-227).
 *
 * Rules of the ABI:
 *   - plain C types, pointers and sizes only; no C++ exceptions cross it;
 *   - every function returns PGPU_OK (0) or a negative PGPU_E* status; the message of the last failure on the
 *     calling thread is available through pgpu_last_error (thread-local), mirroring the processing-exception
 *     path of BaseCombineOperator.onException (core/operator/combine/BaseCombineOperator.java:177-179);
 *   - segment handles are immutable after pgpu_segment_seal and may be shared by concurrent queries;
 *   - queries are re-entrant: each takes its own workspace; submitted queries run in submission order on the
 *     context's query stream (each kernel fills the GPU, so serialising them loses nothing).
 *
 * Dictionary ids are segment-local, exactly as in the reference: the host evaluates predicates against each
 * segment's dictionary (core/operator/filter/predicate/<X>PredicateEvaluatorFactory.java) and passes dict-id ranges /
 * sets per segment.  Group-by keys are made global by per-segment remap tables (see pgpu_remap_upload).
 */
#ifndef PINOT_GPU_H
#define PINOT_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGPU_ABI_VERSION 12

/* ---- status codes ---------------------------------------------------------------------------------------- */
#define PGPU_OK 0
#define PGPU_E_INVALID (-1)     /* bad argument / malformed plan or index bytes */
#define PGPU_E_HIP (-2)         /* HIP runtime failure (out of memory, launch failure, ...) */
#define PGPU_E_UNSUPPORTED (-3) /* plan shape this build does not run on the GPU: caller keeps the CPU plan */
#define PGPU_E_NOT_FOUND (-4)
/* The query passed its deadline (pgpu_query_desc.deadline_ms) before it finished: the reference's combine stops
 * polling for results blocks and answers QueryException.EXECUTION_TIMEOUT_ERROR
 * (core/operator/combine/BaseCombineOperator.java:194-203).  Its kernels are told to stop (as by
 * pgpu_query_cancel) and have drained when the call returns; the context stays usable. */
#define PGPU_E_TIMEOUT (-5)
/* pgpu_query_cancel was called before the query finished (the reference cancels the segment tasks' futures,
 * BaseCombineOperator.getNextBlock); results and stats are partial and must be discarded. */
#define PGPU_E_CANCELLED (-6)
/* A segment whose group-key holder is map-based met more distinct keys than pgpu_query_desc.num_groups_limit: the
 * reference keeps only the first-seen keys in doc order (DictionaryBasedGroupKeyGenerator.java:384-463, 991-1016;
 * new keys beyond the limit get INVALID_ID and their docs are not aggregated).  The launch's table is discarded; the
 * caller re-runs such segments with MIN over the doc-id column (pgpu_segment_add_docid_column) and keeps the
 * num_groups_limit keys of smallest first doc (pinot_amd/plan.py), or keeps the CPU plan. */
#define PGPU_E_GROUPS_LIMIT (-7)

/* ---- stored data types (spi/data/FieldSpec.java DataType, stored type) -------------------------------------- */
#define PGPU_INT 0
#define PGPU_LONG 1
#define PGPU_FLOAT 2
#define PGPU_DOUBLE 3
#define PGPU_STRING 4 /* dictionary values stay on the host; ids only on the device */

/* ---- memory kinds for upload sources --------------------------------------------------------------------- */
#define PGPU_MEM_HOST 0
#define PGPU_MEM_DEVICE 1 /* source already in this device's HBM (e.g. a staged loader); copied D2D */

typedef struct pgpu_context pgpu_context;
typedef struct pgpu_segment pgpu_segment;
typedef struct pgpu_buffer pgpu_buffer;

/* ---- lifecycle ------------------------------------------------------------------------------------------- */
int pgpu_abi_version(void);
/* Open device `device_ordinal` (HIP ordinal, one process per GPU). */
int pgpu_init(int device_ordinal, pgpu_context** out_ctx);
int pgpu_shutdown(pgpu_context* ctx);
/* Copies the calling thread's last error message (NUL-terminated, truncated to len). Returns its full length. */
int pgpu_last_error(char* buf, size_t len);

/* ---- segment upload (IndexingOverrides seam) -------------------------------------------------------------
 * One pgpu_segment per immutable segment, one column slot per column the queries may touch.  All byte sources
 * are in the reference's on-disk layouts and are COPIED (the caller may unmap after return):
 *   forward index : FixedBitSVForwardIndexWriter layout — value i in bits [i*b, (i+1)*b) of an MSB-first,
 *                   big-endian bit stream, ceil(numDocs*b/8) bytes
 *                   (seglocal/io/writer/impl/FixedBitSVForwardIndexWriter.java:39-47,
 *                    seglocal/io/util/PinotDataBitSet.java:78-165)
 *   sorted index  : 2 big-endian int32 (startDocId, endDocId inclusive) per dict id; also the forward index of a
 *                   sorted column (seglocal/segment/index/readers/sorted/SortedIndexReaderImpl.java:37-121)
 *   dictionary    : sorted unique values, big-endian fixed width (4 B INT/FLOAT, 8 B LONG/DOUBLE)
 *                   (seglocal/segment/index/readers/BaseImmutableDictionary.java:40-322,
 *                    seglocal/io/util/FixedByteValueReaderWriter.java:37-53)
 *   inverted index: (card+1) big-endian int32 offsets followed by one Roaring portable-format bitmap per dict id
 *                   (seglocal/segment/creator/impl/inv/BitmapInvertedIndexWriter.java:35-124,
 *                    seglocal/segment/index/readers/BitmapInvertedIndexReader.java:45-61)
 */
int pgpu_segment_create(pgpu_context* ctx, int32_t num_docs, int32_t num_columns, pgpu_segment** out_seg);
/* bits_per_value = PinotDataBitSet.getNumBitsPerValue(cardinality - 1) (PinotDataBitSet.java:59-71), 1..31 */
int pgpu_segment_add_forward_index(pgpu_segment* seg, int32_t column, const void* bytes, uint64_t num_bytes,
                                   int32_t bits_per_value, int32_t cardinality, int32_t mem_kind);
int pgpu_segment_add_sorted_index(pgpu_segment* seg, int32_t column, const void* bytes, uint64_t num_bytes,
                                  int32_t cardinality);
/* data_type PGPU_STRING: pass bytes=NULL; only the cardinality is recorded. */
int pgpu_segment_add_dictionary(pgpu_segment* seg, int32_t column, int32_t data_type, const void* bytes,
                                uint64_t num_bytes, int32_t cardinality);
int pgpu_segment_add_inverted_index(pgpu_segment* seg, int32_t column, const void* bytes, uint64_t num_bytes,
                                    int32_t cardinality);
/* Raw (no-dictionary) single-value column of a fixed-width type (INT / LONG / FLOAT / DOUBLE): the file
 * FixedByteChunkSVForwardIndexWriter writes (`<column>.sv.raw.fwd`, seglocal/io/writer/impl/
 * FixedByteChunkSVForwardIndexWriter.java:39-104, header BaseChunkSVForwardIndexWriter.java:125-160), versions 1-4,
 * chunks PASS_THROUGH / SNAPPY / ZSTANDARD / LZ4 / LZ4_LENGTH_PREFIXED (ChunkCompressionType ordinals 0-4; ZSTANDARD
 * frames are decoded by the system's libzstd.so.1, and return PGPU_E_UNSUPPORTED when it cannot be loaded).  Decoded once into HBM as the values by doc id, replacing FixedByteChunkSVForwardIndexReader /
 * FixedBytePower2ChunkSVForwardIndexReader (seglocal/segment/index/readers/forward/BaseChunkSVForwardIndexReader.java:56-157).
 * Such a column has no dictionary (do not call pgpu_segment_add_dictionary); it may be aggregated (SUM / MIN / MAX /
 * AVG), filtered through PGPU_F_RAW_SCAN / PGPU_F_RANGE_INDEX leaves, and grouped on through its on-the-fly group
 * dictionary (pgpu_segment_add_group_dictionary). */
int pgpu_segment_add_raw_forward_index(pgpu_segment* seg, int32_t column, int32_t data_type, const void* bytes,
                                       uint64_t num_bytes);
/* Range index of a column (`<column>.bitmap.range`): only its header is read -- version 2 is the exact bit-sliced
 * index (BitSlicedRangeIndexCreator.java:38,115-125; BitSlicedRangeIndexReader.java:41-55), version 1 the legacy
 * RangeIndexReaderImpl with partial matches.  The GPU answers range-index leaves from the forward index (same doc set);
 * the version decides the leaf's statistics (see PGPU_F_RANGE_INDEX). */
int pgpu_segment_add_range_index(pgpu_segment* seg, int32_t column, const void* bytes, uint64_t num_bytes);
/* Multi-value dictionary-encoded column: the file FixedBitMVForwardIndexWriter writes (`<column>.mv.fwd`,
 * seglocal/io/writer/impl/FixedBitMVForwardIndexWriter.java:73-159): big-endian chunk offsets, a row-start bitmap
 * over the value index, the values' dict ids fixed-bit (`bits_per_value`), `num_values` = the column metadata's
 * totalNumberOfEntries.  Replaces FixedBitMVForwardIndexReader.getDictIdMV (seglocal/segment/index/readers/forward/
 * FixedBitMVForwardIndexReader.java:58-140): the row offsets are found once at upload, the ids stay packed in HBM.
 * Add the dictionary first (pgpu_segment_add_dictionary; numeric types) and optionally an inverted index.  A SCAN
 * leaf on such a column has applyMV semantics (BaseDictionaryBasedPredicateEvaluator.java:133-149): a row matches
 * when any of its values is in the leaf's dict-id set / range, and `negate` keeps the rows none of whose values is
 * (the exclusive NEQ / NOT IN forms); it counts each row's length towards numEntriesScannedInFilter
 * (MVScanDocIdIterator.java:56-100).  GROUP BY on the column expands each matched doc into one key per value
 * (DictionaryBasedGroupKeyGenerator.java:472-544, processMultiValue), with first-seen numGroupsLimit truncation as in
 * the single-value case.  It cannot be aggregated directly (PGPU_E_UNSUPPORTED): the *MV aggregation functions read
 * its row columns (below). */
int pgpu_segment_add_mv_forward_index(pgpu_segment* seg, int32_t column, const void* bytes, uint64_t num_bytes,
                                      int32_t bits_per_value, int32_t cardinality, int64_t num_values);
/* Dict ids of one row of a multi-value column, in value order (*out_len = the row's length; at most `capacity` ids
 * are written).  The host side of the first-seen numGroupsLimit cut on multi-value group keys: the new keys of the
 * doc where the limit is reached get ids in the order DictionaryBasedGroupKeyGenerator.processMultiValue meets
 * them (DictionaryBasedGroupKeyGenerator.java:186-199, IntGroupIdMap.getGroupId :991-1016). */
int pgpu_segment_mv_row(pgpu_segment* seg, int32_t column, int32_t doc, int32_t* out_ids, int32_t capacity,
                        int32_t* out_len);
/* Per-row reductions of a multi-value column, installed as raw columns in other slots of the same segment (-1 skips
 * one): len_column = values per row (INT), sum_column = the row's sum (LONG for INT / LONG, DOUBLE for FLOAT /
 * DOUBLE values), min_column / max_column = the row's smallest / largest value (the column's type).  COUNTMV /
 * SUMMV / MINMV / MAXMV / AVGMV (CountMV..AvgMVAggregationFunction: every value of every matched row) are then
 * SUM(len) / SUM(sum) / MIN(min) / MAX(max) / SUM(sum) / SUM(len) over the matched rows. */
int pgpu_segment_add_mv_row_columns(pgpu_segment* seg, int32_t column, int32_t len_column, int32_t sum_column,
                                    int32_t min_column, int32_t max_column);
int pgpu_segment_seal(pgpu_segment* seg);
/* GROUP BY on a raw (no-dictionary) column: its on-the-fly dictionary, the replacement of the value -> id maps of
 * NoDictionarySingleColumnGroupKeyGenerator / NoDictionaryMultiColumnGroupKeyGenerator
 * (core/query/aggregation/groupby/NoDictionarySingleColumnGroupKeyGenerator.java:70-118, 199-235;
 * NoDictionaryMultiColumnGroupKeyGenerator.java:90-150).  Built on the GPU from `raw_column`'s values into the empty
 * slot `dict_column` (callable before or after seal, once): the distinct values sorted ascending (Float.compare order;
 * FLOAT / DOUBLE values distinct by floatToIntBits / doubleToLongBits, as the reference's primitive maps key them:
 * -0.0 and 0.0 apart, one NaN) as a numeric dictionary, and every doc's id as a fixed-bit forward index.  The slot then
 * groups like any dictionary-encoded column; *out_cardinality = its distinct values. */
int pgpu_segment_add_group_dictionary(pgpu_segment* seg, int32_t raw_column, int32_t dict_column,
                                      int32_t* out_cardinality);
/* The little-endian numeric dictionary of a column (pgpu_segment_add_dictionary or _add_group_dictionary):
 * *out_bytes = its size; copied into `out` when non-NULL (capacity_bytes >= *out_bytes). */
int pgpu_segment_dictionary_values(const pgpu_segment* seg, int32_t column, void* out, uint64_t capacity_bytes,
                                   uint64_t* out_bytes);
/* The doc-id column: fills the empty slot `column` (before or after seal, once) with a raw INT column whose value at
 * doc d is d.  MIN over it is each group's first doc, the order in which the reference's map-based group-key holders
 * assign group ids (first-seen truncation at numGroupsLimit, PGPU_E_GROUPS_LIMIT).  4 bytes of HBM per doc. */
int pgpu_segment_add_docid_column(pgpu_segment* seg, int32_t column);
/* HBM bytes held by the segment (all columns, including padding and container directories). */
int pgpu_segment_device_bytes(const pgpu_segment* seg, uint64_t* out_bytes);
/* The same, by kind: the reference's own indexes (forward incl. raw values, dictionary, sorted, inverted,
 * multi-value) and the derived copies seal builds (bit-sliced forward indexes, value planes). */
typedef struct {
  uint64_t forward, dictionary, sorted, inverted, multi_value, sliced, value_planes, total;
} pgpu_segment_bytes;
int pgpu_segment_device_bytes_ex(const pgpu_segment* seg, pgpu_segment_bytes* out);
/* ---- HBM residency of derived copies (IndexLoadingConfig seam) -------------------------------------------------
 * pgpu_segment_seal derives two copies of a column's forward index that only this path reads: a bit-sliced copy
 * (PGPU_DERIVE_SLICED, same bytes as the forward index; scan-filter leaves streamed as bit planes) and, for INT /
 * LONG dictionaries of <= 32 value bits, value planes (PGPU_DERIVE_VALUE_PLANES, vbits bits per doc; aggregation of
 * densely matched metrics without dictionary gathers).  As the reference loads only the indexes a table's
 * IndexLoadingConfig names (seglocal/segment/index/column/PhysicalColumnIndexContainer.java:80,151-156), a server
 * names per column which copies to build -- its GPU filter columns and metric columns
 * (pinot.server.query.executor.gpu.sliced.columns / .value.planes.columns) -- before seal; the default is both.
 * Every copy is also built only while the context's derived bytes stay within its budget (default half of the
 * device's memory; 0 = none).  Queries plan around a missing copy (packed streams, dictionary gathers): results are
 * the same, only the kernel chosen differs. */
#define PGPU_DERIVE_SLICED 1
#define PGPU_DERIVE_VALUE_PLANES 2
#define PGPU_DERIVE_ALL 3
int pgpu_segment_set_derived(pgpu_segment* seg, int32_t column, int32_t flags);
int pgpu_context_set_derived_budget(pgpu_context* ctx, uint64_t bytes);
int pgpu_context_derived_bytes(pgpu_context* ctx, uint64_t* out_used, uint64_t* out_budget);
int pgpu_segment_release(pgpu_segment* seg);

/* ---- group-key remap tables ------------------------------------------------------------------------------
 * Per-segment int32 table: local dict id -> global group id (global dictionary = sorted union of the group
 * column's segment dictionaries).  Uploaded once and cached by the host; NULL in a plan means identity. */
int pgpu_remap_upload(pgpu_context* ctx, const int32_t* map, int32_t length, pgpu_buffer** out_buf);
int pgpu_buffer_release(pgpu_buffer* buf);

/* ---- query plan ------------------------------------------------------------------------------------------
 * The filter of each segment is a flat program in prefix order (the operator tree the reference builds in
 * core/plan/FilterPlanNode.java:192-313 after FilterOperatorUtils leaf choice and AND re-ordering,
 * core/operator/filter/FilterOperatorUtils.java:42-221):
 *   AND_BEGIN  c1 .. cn  AND_END      (each child is followed by AND_CHILD_END)
 *   OR_BEGIN   c1 .. cn  OR_END       (each child is followed by OR_CHILD_END)
 *   NOT c
 *   SCAN  leaf : ScanBasedFilterOperator over the forward index (ScanBasedFilterOperator.java:46-54)
 *   INVERTED leaf: BitmapBasedFilterOperator, OR of the bitmaps of `ids` (BitmapBasedFilterOperator.java:66-110)
 *   SORTED leaf: SortedIndexBasedFilterOperator, inclusive doc ranges (SortedIndexBasedFilterOperator.java:51-219)
 *   MATCH_ALL / EMPTY: MatchAllFilterOperator / EmptyFilterOperator
 * `negate` on a leaf complements it within [0, numDocs) — the NEQ / NOT IN / NOT BETWEEN forms
 * (BitmapBasedFilterOperator.java:82-100).  SCAN predicates are dict-id forms of the reference evaluators:
 *   PGPU_PRED_RANGE: lo <= dictId < hi   (SortedDictionaryBasedRangePredicateEvaluator.applySV,
 *                    RangePredicateEvaluatorFactory.java:174-177; EQ is [id, id+1))
 *   PGPU_PRED_SET  : dictId in ids[]     (DictionaryBasedInPredicateEvaluator, InPredicateEvaluatorFactory.java:142-182)
 */
#define PGPU_F_MATCH_ALL 0
#define PGPU_F_EMPTY 1
#define PGPU_F_SCAN 2
#define PGPU_F_INVERTED 3
#define PGPU_F_SORTED 4
#define PGPU_F_AND_BEGIN 5
#define PGPU_F_AND_CHILD_END 6
#define PGPU_F_AND_END 7
#define PGPU_F_OR_BEGIN 8
#define PGPU_F_OR_CHILD_END 9
#define PGPU_F_OR_END 10
#define PGPU_F_NOT 11
/* Raw-value leaves (columns uploaded with pgpu_segment_add_raw_forward_index):
 *   RAW_SCAN   : ScanBasedFilterOperator with a RawValueBased*PredicateEvaluator (its entries count towards
 *                numEntriesScannedInFilter like a dictionary scan's)
 *   RANGE_INDEX: RangeIndexBasedFilterOperator (FilterOperatorUtils.java:57-64: RANGE predicates on a column with a
 *                range index, AND priority 2).  On a dictionary column it carries the dict-id range [lo, hi) like a
 *                SCAN leaf; on a raw column raw values as below.  An exact (version 2) range index scans no entries;
 *                its raw-column bounds are used inclusively whatever the predicate's flags, as the reference's
 *                Int/Long/Float/DoubleRangeEvaluator pass getLowerBound / getUpperBound to the index
 *                (RangeIndexBasedFilterOperator.java:165-290), and floating values compare by FPOrdering ordinals
 *                (NaN = -infinity).
 * Raw values are given in `values`: 8-byte int64 for INT / LONG columns, IEEE double for FLOAT / DOUBLE columns (the
 * literal parsed as the evaluator parses it: Integer.parseInt, Float.parseFloat, ...).
 *   PGPU_PRED_RANGE: values[0] lower, values[1] upper bound; lo = 1 when the lower bound is inclusive, hi = 1 when
 *                    the upper is (an unbounded side is the type's extreme, inclusive)
 *   PGPU_PRED_SET  : num_ids values (EQ: one); negate for NOT_EQ / NOT_IN */
#define PGPU_F_RAW_SCAN 12
#define PGPU_F_RANGE_INDEX 13

#define PGPU_PRED_RANGE 0
#define PGPU_PRED_SET 1

typedef struct {
  int32_t op;         /* PGPU_F_* */
  int32_t column;     /* query column index (leaf ops) */
  int32_t pred;       /* PGPU_PRED_* (SCAN) */
  int32_t negate;     /* leaf complement within [0, numDocs) */
  int32_t lo, hi;     /* RANGE: [lo, hi) */
  const int32_t* ids; /* SET / INVERTED: dict ids; SORTED: 2*num_ids ints (start, end inclusive) */
  int32_t num_ids;
  int32_t reserved;
  const void* values; /* RAW_SCAN / raw RANGE_INDEX: the predicate's values (see PGPU_F_RAW_SCAN) */
} pgpu_filter_node;

/* aggregation functions (core/query/aggregation/function/<X>AggregationFunction.java) */
#define PGPU_AGG_COUNT 0 /* CountAggregationFunction.java:74-141; column = -1 */
#define PGPU_AGG_SUM 1   /* SumAggregationFunction.java:55-129 */
#define PGPU_AGG_MIN 2   /* MinAggregationFunction.java:55-138, empty = +inf */
#define PGPU_AGG_MAX 3   /* MaxAggregationFunction.java:55-138, empty = -inf */
#define PGPU_AGG_AVG 4   /* AvgAggregationFunction.java:58-190 + AvgPair */

typedef struct {
  int32_t fn;
  int32_t column; /* query column index, -1 for COUNT(*) */
} pgpu_agg;

typedef struct {
  const pgpu_segment* segment;
  const int32_t* column_map;          /* query column index -> segment column slot (num_columns entries) */
  const pgpu_filter_node* filter;     /* prefix-order program; NULL or 0 nodes = match all */
  int32_t num_filter_nodes;
  int32_t reserved;
  const pgpu_buffer* const* group_remap; /* per group-by column; NULL array or NULL entry = identity */
} pgpu_segment_plan;

typedef struct {
  int32_t num_columns;                /* query columns referenced by filter / aggregations / group-by */
  int32_t num_segments;
  const pgpu_segment_plan* segments;
  int32_t num_aggs;
  int32_t num_group_columns;          /* 0 = aggregation only */
  const pgpu_agg* aggs;
  const int32_t* group_columns;       /* query column indexes, key = sum_j gid_j * prod_{k<j} card_k */
  const int32_t* group_cardinalities; /* global cardinality per group column */
  uint64_t flags;                     /* PGPU_Q_* */
  /* Docs the partial table is reduced over (the whole node / cluster for a multi-GPU combine); 0 = the docs of
   * this launch.  Bounds integer SUM cells: with max|dictionary value| x reduce_docs >= 2^62 an INT / LONG SUM
   * is carried as three exact 21-bit-part sums (see pgpu_table_layout.agg_sum_parts). */
  int64_t reduce_docs;
  /* Group-key holder limits (InstancePlanMakerImplV2 num.groups.limit / max.init.group.holder.capacity,
   * core/plan/maker/InstancePlanMakerImplV2.java:66-88).  A segment whose local cardinality product exceeds both
   * can meet more than num_groups_limit distinct keys; the reference then keeps only the first-seen ones
   * (DictionaryBasedGroupKeyGenerator.java:137-164, :384-463).  Such segments' distinct keys are counted on the
   * GPU, and a segment that really exceeds the limit makes the query return PGPU_E_UNSUPPORTED (the server keeps
   * the CPU plan, which reproduces the truncation).  0 = no limit. */
  int32_t num_groups_limit;
  int32_t array_based_threshold;
  /* End time in milliseconds since the Unix epoch (QueryContext.getEndTimeMs: the broker's timeoutMs from the
   * query's arrival, System.currentTimeMillis clock); 0 = none.  Passed when the query is waited for (or already
   * at launch), the query is cancelled and pgpu_query_wait / _collect / _execute / pgpu_node_query return
   * PGPU_E_TIMEOUT. */
  int64_t deadline_ms;
  /* Per aggregation (num_aggs entries), or both NULL: the fixed-point layout (exponent, part count) of each FLOAT /
   * DOUBLE SUM / AVG agreed across the launches whose tables are combined (ranks, devices), as
   * pgpu_sum_layout_agree returns it from their own layouts (pgpu_table_layout.agg_sum_exp / agg_sum_parts).  The
   * launch takes it verbatim (PGPU_SUM_EXP_F64, or more than PGPU_MAX_FIXED_PARTS parts: a float64 section), so every
   * table has one layout; it fails with PGPU_E_INVALID when the agreed window does not cover its own values at its
   * own precision.  Entries of other aggregations are ignored. */
  const int32_t* sum_exp;
  const int32_t* sum_parts;
} pgpu_query_desc;

#define PGPU_Q_STATS 1ull /* count touched 32-B sectors of sparse column reads (roofline accounting) */
/* Group-by strategy for large key spaces: from 65,536 keys up, matched docs are written as records into
 * per-(key partition, workgroup) regions and each partition is then aggregated in an LDS table (one aggregated
 * column of a 4-byte type at most; otherwise HBM atomics).  These flags force it for any group-by shape the
 * partitioned path supports, and shrink its regions so that the spill path runs (tests and tuning). */
#define PGPU_Q_PARTITION 2ull
#define PGPU_Q_PART_SPILL 4ull
/* Carry every INT / LONG SUM / AVG as three 21-bit-part sums whatever the bound says (multi-GPU callers set it
 * on every rank when any rank's bound needs it, so that all ranks share one table layout). */
#define PGPU_Q_SUM_SPLIT 8ull
/* Group-by through the hash table (PGPU_KEYS_HASH) whatever the key space; chosen by default for key spaces
 * above 2^31 keys, for sparse occupancy, and when a segment's distinct keys must be counted (num_groups_limit). */
#define PGPU_Q_HASH 16ull
/* numEntriesScannedInFilter exactly as the reference's iterators count it (see pgpu_filter_entries_scanned):
 * every leaf of every segment's filter is also evaluated over all docs into a bitmap, and the iterator tree is
 * replayed on the host in pgpu_query_wait.  Without it the statistic is the GPU's own count of evaluated
 * forward-index entries, which equals the reference's except under leap-frogging iterators (an AND of several
 * scan leaves, an OR / NOT advanced by a parent AND); pgpu_query_stats.filter_stats_exact tells which. */
#define PGPU_Q_EXACT_FILTER_STATS 32ull

/* ---- partial-result table ----------------------------------------------------------------------------------
 * A query produces a dense table over G = prod(group_cardinalities) keys (G = 1 for aggregation only), laid out
 * as sections of G 8-byte cells so that RCCL can reduce each section with one op:
 *   section 0                : count      int64, SUM   (docs per key; COUNT(*) and the AVG count)
 *   one section per agg slot : SUM of INT/LONG column   -> int64   SUM (exact; == the reference's double sum
 *                                                                    while |partial sums| < 2^53)
 *                              ... whose bound max|value| x docs reaches 2^62 (or PGPU_Q_SUM_SPLIT):
 *                                  three int64 SUM sections s, s+1, s+2 holding the sums of bits [0,21),
 *                                  [21,42) (unsigned parts) and [42,64) (arithmetic shift) of every value:
 *                                  SUM = c[s] + c[s+1] * 2^21 + c[s+2] * 2^42, exact for < 2^42 docs
 *                                  (SumAggregationFunction.java:55-92 adds doubles in doc order and never
 *                                  wraps; an int64 cell would)
 *                              SUM of FLOAT/DOUBLE      -> P = agg_sum_parts (3..PGPU_MAX_FIXED_PARTS) int64 SUM
 *                                                          sections of the values in fixed point: |v| -> the
 *                                                          integer I = rint(|v| * 2^-e) (e = agg_sum_exp), section
 *                                                          s+k sums sign(v) * (bits [21k, 21k+21) of I), so that
 *                                                          integer adds make the sum independent of the order the
 *                                                          GPU adds in (a float64 SUM of atomics is not).  SUM =
 *                                                          round(sum_k c[s+k] * 2^(21k)) * 2^e.  e and P come from
 *                                                          the column's values (pgpu_fixed_sum_layout): each value
 *                                                          is exact, or rounded by at most 2^-41 of itself, so the
 *                                                          result is within 2^-41 * sum|v| of the exact sum (the
 *                                                          reference's doc-order double adds: (n-1) * 2^-53 *
 *                                                          sum|v|).  A NaN or infinity in the column, a value range
 *                                                          needing more than PGPU_MAX_FIXED_PARTS parts, or no
 *                                                          section budget keeps one float64 SUM section
 *                                                          (agg_sum_exp = PGPU_SUM_EXP_F64)
 *                              MIN / MAX                -> int64 MIN / MAX of an order-preserving key
 *                              AVG                      -> as SUM (count comes from section 0)
 *                              COUNT                    -> no section (section 0)
 * pgpu_table_layout describes it; pgpu_decode_minmax_key turns MIN/MAX keys back into doubles.
 */
#define PGPU_MAX_SECTIONS 17 /* count + 16 value sections (a split SUM takes 3; more than 16 -> UNSUPPORTED) */
#define PGPU_RED_SUM_I64 0
#define PGPU_RED_SUM_F64 1
#define PGPU_RED_MIN_I64 2
#define PGPU_RED_MAX_I64 3
#define PGPU_SUM_EXP_F64 32767 /* agg_sum_exp of a float64 SUM section */
#define PGPU_SUM_EXP_ZERO (-32767) /* agg_sum_exp of a fixed-point SUM over a column holding no nonzero value */
#define PGPU_MAX_FIXED_PARTS 6  /* 126-bit fixed-point window of a floating SUM */
#define PGPU_FIXED_TOL_BITS 40  /* a value may be rounded by at most 2^-(TOL+1) of itself */

/* key_kind of a table layout */
#define PGPU_KEYS_DENSE 0 /* cell index = global raw key: sum_j gid_j * prod_{k<j} card_k (< 2^31) */
#define PGPU_KEYS_HASH 1  /* cell index = hash slot; the slot's key words follow the sections (below) */

typedef struct {
  uint64_t num_keys;       /* G: keys (dense) or hash slots (hash) */
  int32_t num_sections;
  int32_t section_op[PGPU_MAX_SECTIONS]; /* PGPU_RED_* per section (section 0 = count) */
  int32_t agg_section[16]; /* section of agg i, or 0 for COUNT */
  int32_t agg_value_type[16]; /* stored type of the agg column (PGPU_INT..), -1 for COUNT */
  int32_t agg_sum_parts[16];  /* SUM / AVG: 1 = one int64 (or float64) section, > 1 = that many 21-bit-part sections
                                 (3 for a split integer SUM, 3..PGPU_MAX_FIXED_PARTS for a fixed-point floating SUM) */
  int32_t agg_sum_exp[16];    /* SUM / AVG of FLOAT / DOUBLE in fixed point: value = (exact part sum) * 2^exp
                                 (PGPU_SUM_EXP_ZERO: the column holds only zeros); PGPU_SUM_EXP_F64 = a float64
                                 section; 0 for integer columns (whether a SUM is fixed point is decided by
                                 agg_value_type and agg_sum_parts, never by this exponent) */
  /* Group keys.  Dense: the cell index is the key.  Hash: key_words int64 words per slot follow the sections
   * (word w of slot i at int64 index (num_sections + w) * num_keys + i; an empty slot holds -1).  Word 0 is the
   * mixed-radix key of group columns [0, key_split), word 1 (when key_words == 2, key spaces above 2^63, the
   * reference's ArrayMapBasedHolder, DictionaryBasedGroupKeyGenerator.java:137-146) that of [key_split, n). */
  int32_t key_kind;
  int32_t key_words;
  int32_t key_split;
  int32_t reserved;
} pgpu_table_layout;

/* Bytes of the partial table of a layout: 8 * (num_sections [+ key_words when hash]) * num_keys. */
uint64_t pgpu_table_bytes(const pgpu_table_layout* layout);

int pgpu_table_layout_of(const pgpu_query_desc* q, pgpu_table_layout* out);
/* The fixed-point window of a FLOAT / DOUBLE SUM over values with max |v| = max_abs, smallest nonzero |v| of binary
 * exponent min_exp and lowest significand bit 2^min_lsb (the layout's own choice, exposed for callers and tests):
 * *out_parts 21-bit parts at exponent *out_exp, or PGPU_SUM_EXP_F64 / PGPU_SUM_EXP_ZERO. */
void pgpu_fixed_sum_layout(double max_abs, int32_t min_exp, int32_t min_lsb, int32_t* out_exp, int32_t* out_parts);
/* One fixed-point layout for tables combined across launches: from each launch's own layout (pgpu_table_layout_of
 * without sum_exp) the window spanning all of them at the finest exponent any needs, per aggregation (out_exp /
 * out_parts: num_aggs entries, passed back as pgpu_query_desc.sum_exp / sum_parts).  A float64 layout anywhere stays
 * float64 everywhere; a window wider than PGPU_MAX_FIXED_PARTS parts makes every launch take float64. */
int pgpu_sum_layout_agree(const pgpu_table_layout* layouts, int32_t num_layouts, int32_t num_aggs, int32_t* out_exp,
                          int32_t* out_parts);

typedef struct {
  int64_t num_docs_scanned;              /* docs matching the filter (AggregationOperator.java:82-87) */
  int64_t num_entries_scanned_in_filter; /* GPU-evaluated forward-index entries, or the reference's count */
  int64_t num_total_docs;
  int64_t num_segments_matched;          /* segments with at least one matching doc (CombineOperatorUtils.java:64-67) */
  int64_t sparse_sector_bytes;           /* PGPU_Q_STATS: 32-B sectors touched by sparse reads * 32 */
  int64_t dense_bytes;                   /* forward-index bytes streamed in dense (staged) mode */
  double kernel_ms;                      /* every kernel reading the segments: leaf bitmaps, query kernel, group-by phases, filter-statistic kernels (HIP events on the query stream) */
  int64_t filter_stats_exact;            /* 1: num_entries_scanned_in_filter is the reference's figure */
  int64_t num_groups_limit_reached;      /* 1: a segment met >= num_groups_limit distinct group keys
                                            (AggregationGroupByOrderByOperator.java:111) */
  int64_t kernel_variant;                /* PGPU_KV_*: the query kernel the runtime chose (diagnostic) */
} pgpu_query_stats;
#define PGPU_KV_RING 0       /* loader + consumer waves through an LDS ring */
#define PGPU_KV_DIRECT 1     /* self-loading waves, LDS-DMA slots */
#define PGPU_KV_RDIRECT 2    /* one bit-sliced fast leaf in VGPRs */
#define PGPU_KV_RSTREAM 3    /* two fast leaves and value planes in VGPRs */
#define PGPU_KV_RPROG 4      /* index-only program as a truth table over expanded leaf bitmaps */
#define PGPU_KV_RKEY 5       /* index-only program over Roaring containers read into LDS per container key */
#define PGPU_KV_CAND 6       /* candidates from a sparse leading inverted leaf's containers */
#define PGPU_KV_PSCAN 7      /* partitioned group-by, phase-1 scan + phase-2 reduce */
#define PGPU_KV_RFSM 8       /* two bit-sliced leaves in VGPRs with the exact filter statistic's tile maps */

/* Enqueue the query on `stream` (hipStream_t; NULL = the context's own stream) and leave the partial table in
 * caller-provided device memory `dev_table` (table_bytes >= pgpu_table_bytes(layout)).  Does not synchronize.
 * Used for multi-GPU combine: the caller RCCL-reduces the sections of a dense table (hash tables are compacted
 * first and merged by key), then calls pgpu_table_compact.  Stats become valid after pgpu_query_wait, which
 * returns PGPU_E_UNSUPPORTED when a segment met more distinct group keys than num_groups_limit. */
typedef struct pgpu_query pgpu_query;
int pgpu_query_launch(pgpu_context* ctx, const pgpu_query_desc* q, void* stream, void* dev_table,
                      uint64_t table_bytes, pgpu_query** out_query);
int pgpu_query_wait(pgpu_query* query, pgpu_query_stats* out_stats);
int pgpu_query_release(pgpu_query* query);
/* Ask a launched / submitted query to stop (thread-safe; returns at once, from any thread, also while another
 * thread blocks in pgpu_query_wait / _collect).  Every kernel of the query polls the flag per range of tiles
 * (the ring kernel's loaders, the self-loading waves, the partitioned group-by's phase-1 steps and phase-2
 * regions) and skips the rest of its work; the wait then returns PGPU_E_CANCELLED (PGPU_E_TIMEOUT when the
 * deadline fired it), and the query must still be released / collected. */
int pgpu_query_cancel(pgpu_query* query);
/* Per-segment numDocsScanned > 0 flags of a launched / submitted query: when the query's stats become valid
 * (pgpu_query_wait / _collect) out[i] = 1 if segment i of the descriptor matched at least one doc, else 0.  `out`
 * must hold the descriptor's num_segments bytes and outlive the wait.  Replaces the per-operator test of
 * CombineOperatorUtils.setExecutionStatistics (:64-67) where several passes (filtered aggregations) share the
 * segments and their numSegmentsMatched is the union, not the sum. */
int pgpu_query_matched_segments(pgpu_query* query, uint8_t* out, int32_t num_segments);

/* Compact a (reduced) table: copy every key with count > 0 to the host (dense: ascending by key; hash: in slot
 * order).
 *   out_keys  : int64[capacity * key_words]   (global raw key words, row-major; key_words = 1 for dense)
 *   out_cells : int64[capacity * num_sections] row-major (section 0 = count, then sections in layout order;
 *               float64 sections are bit-cast into the int64 cells)
 * *out_num_groups receives the number of non-empty keys; if it exceeds capacity nothing beyond is written
 * and PGPU_E_INVALID is returned with the needed count. Synchronizes `stream`. */
int pgpu_table_compact(pgpu_context* ctx, const pgpu_table_layout* layout, const void* dev_table, void* stream,
                       int64_t* out_keys, int64_t* out_cells, uint64_t capacity, uint64_t* out_num_groups);

/* ---- ORDER BY ... LIMIT trim on the GPU ------------------------------------------------------------------------
 * GroupByOrderByCombineOperator keeps an IndexedTable whose finish() hands the broker only the top
 * trimSize = max(5 * limit, 5000) records by the first ORDER BY expression (GroupByUtils.getTableCapacity,
 * core/util/GroupByUtils.java:24-41; TableResizer.getTopRecords, core/data/table/TableResizer.java; IndexedTable.finish,
 * core/data/table/IndexedTable.java:135-156).  Here the non-empty groups of a (reduced) table are ranked on the GPU
 * by one order key -- an aggregation's final value (extractFinalResult as a double: SUM, MIN, MAX, AVG = sum / count;
 * COUNT as an integer) or a group column's value (its global dictionary id: global dictionaries are sorted) -- and
 * the best k are compacted: every group whose key is at least as good as the k-th best's, so ties at the boundary are
 * all kept and the caller's full ORDER BY ... LIMIT over the returned rows equals the one over the whole table.
 * Radix select over 64-bit order keys (8 passes of 8 bits), no host round trip between passes. */
#define PGPU_TOPK_AGG 0
#define PGPU_TOPK_GROUP 1
typedef struct {
  int32_t source;                     /* PGPU_TOPK_AGG / PGPU_TOPK_GROUP */
  int32_t agg_fn;                     /* AGG: PGPU_AGG_* of the aggregation */
  int32_t agg_index;                  /* AGG: its index in the query (layout agg_section / agg_sum_parts / type) */
  int32_t group_index;                /* GROUP: its position among the group columns */
  int32_t descending;
  int32_t num_group_columns;          /* GROUP: the query's group columns ... */
  const int32_t* group_cardinalities; /* ... and global cardinalities (mixed-radix decode of the key) */
  uint64_t k;                         /* keep the best k groups (ties with the k-th kept too); 0 = keep all */
  uint64_t key_base;                  /* dense tables: global key of cell 0 (a reduce-scatter slice), else 0 */
} pgpu_topk;

/* pgpu_table_compact restricted to the best groups by `order` (out_num_groups = the rows returned). */
int pgpu_table_topk(pgpu_context* ctx, const pgpu_table_layout* layout, const void* dev_table, void* stream,
                    const pgpu_topk* order, int64_t* out_keys, int64_t* out_cells, uint64_t capacity,
                    uint64_t* out_num_groups);
/* pgpu_query_collect returning only the best groups by `order` (NULL = all, as pgpu_query_collect). */
int pgpu_query_collect_topk(pgpu_query* query, const pgpu_topk* order, int64_t* out_keys, int64_t* out_cells,
                            uint64_t capacity, uint64_t* out_num_groups, pgpu_query_stats* out_stats);

/* Single-GPU asynchronous form (the combine operator of one server: BaseCombineOperator.getNextBlock submits the
 * segments' work and blocks in mergeResults, core/operator/combine/BaseCombineOperator.java:79-146):
 *   pgpu_query_submit  packs the plan, enqueues the query on a context-owned stream with its own partial table
 *                      (and, for tables <= 8 MiB, the copy of the whole table to pinned host memory) and returns
 *                      without synchronising; the caller's descriptor memory may be freed on return.
 *   pgpu_query_collect waits, compacts the non-empty keys into out_keys / out_cells (as pgpu_table_compact) and
 *                      releases the query (also on error).
 * Several queries may be in flight on one context; each owns its workspace. */
int pgpu_query_submit(pgpu_context* ctx, const pgpu_query_desc* q, pgpu_query** out_query);
int pgpu_query_collect(pgpu_query* query, int64_t* out_keys, int64_t* out_cells, uint64_t capacity,
                       uint64_t* out_num_groups, pgpu_query_stats* out_stats);

/* ---- per-segment filter planning inside the library (numeric columns) ----------------------------------------
 * The same query with the filter given once, as literals, instead of one dict-id program per segment: for every
 * segment the library evaluates the predicates against that segment's (host copy of the) dictionary
 * (<X>PredicateEvaluatorFactory, BaseImmutableDictionary.insertionIndexOf) and builds the physical filter as
 * FilterPlanNode / FilterOperatorUtils do (EMPTY / MATCH_ALL folding, leaf choice sorted > inverted > scan,
 * stable AND re-ordering) -- the host work of core/plan/FilterPlanNode.java:192-313 per segment, without a
 * round trip per segment through the caller.  Expression nodes in prefix order:
 *   PGPU_X_AND / PGPU_X_OR (num_children children follow), PGPU_X_NOT (one child follows), PGPU_X_PRED.
 * PRED literals: EQ / NOT_EQ one value, IN / NOT_IN num_values values, RANGE [lower, upper] with unbounded /
 * inclusive flags (a missing bound still occupies its slot).  Literal = the SQL literal parsed once:
 * is_integral with i exact (integer columns compare exactly; a fractional literal is never equal and inserts
 * by its double value), d for FLOAT (rounded to float) / DOUBLE columns.  A STRING column returns
 * PGPU_E_UNSUPPORTED (the caller plans that query per segment itself).  segments[i].filter is ignored. */
#define PGPU_X_PRED 0
#define PGPU_X_AND 1
#define PGPU_X_OR 2
#define PGPU_X_NOT 3
#define PGPU_P_EQ 0
#define PGPU_P_NOT_EQ 1
#define PGPU_P_IN 2
#define PGPU_P_NOT_IN 3
#define PGPU_P_RANGE 4

typedef struct {
  int64_t i;           /* exact value of an integral literal */
  double d;            /* the literal as a double */
  int32_t is_integral;
  int32_t reserved;
} pgpu_literal;

typedef struct {
  int32_t op;           /* PGPU_X_* */
  int32_t num_children; /* AND / OR */
  int32_t column;       /* PRED: query column index */
  int32_t pred;         /* PRED: PGPU_P_* */
  int32_t lower_unbounded, upper_unbounded, lower_inclusive, upper_inclusive; /* RANGE */
  int32_t num_values;
  int32_t reserved;
  const pgpu_literal* values;
} pgpu_expr_node;

int pgpu_query_submit_expr(pgpu_context* ctx, const pgpu_query_desc* q, const pgpu_expr_node* expr,
                           int32_t num_nodes, pgpu_query** out_query);
int pgpu_query_launch_expr(pgpu_context* ctx, const pgpu_query_desc* q, const pgpu_expr_node* expr,
                           int32_t num_nodes, void* stream, void* dev_table, uint64_t table_bytes,
                           pgpu_query** out_query);

/* pgpu_query_submit (expr == NULL: the descriptor's per-segment programs) or pgpu_query_submit_expr, with the
 * server's ORDER BY ... LIMIT trim known up front (`order`, as for pgpu_query_collect_topk; NULL = every group):
 * tables above 8 MiB are ranked and compacted on the GPU right behind the query's kernels, on its own stream, so
 * pgpu_query_collect(_topk) only copies the kept rows out -- a collect never waits behind the next query's kernel
 * (GroupByOrderByCombineOperator.mergeResults + IndexedTable.finish, core/operator/combine/
 * GroupByOrderByCombineOperator.java:127-248; trimSize = GroupByUtils.getTableCapacity).  Pass the same order to
 * pgpu_query_collect_topk (any other order selects again from the intact table). */
int pgpu_query_submit_ordered(pgpu_context* ctx, const pgpu_query_desc* q, const pgpu_expr_node* expr,
                              int32_t num_nodes, const pgpu_topk* order, pgpu_query** out_query);

/* ---- node-level combine: one process, several GPUs, RCCL inside the library ------------------------------------
 * For a server that drives all GPUs of a node from one process (a JVM): contexts for the given HIP ordinals and
 * one RCCL communicator clique over them (RCCL is loaded on first use).  Segments are uploaded through each
 * device's context (pgpu_node_context).  pgpu_node_query runs descs[i] (device i's segments, the same aggregations,
 * group columns and global group cardinalities on every device) on every device and merges the partial tables over
 * xGMI with the collectives of the one-process-per-GPU combine (pinot_amd/combine.py):
 *   dense, aggregation only or < 1 MiB : grouped ncclReduce per run of same-op sections to device 0;
 *   dense, larger                      : reduce-scatter -- device d owns the final cells of keys
 *                                        pgpu_slice_of(G, n, d) -- and every device trims its own slice;
 *   hash                               : each device's rows go to the device pgpu_key_owner names (peer copies)
 *                                        and are merged there in a fresh hash table, then trimmed there.
 * The rows come back like pgpu_query_collect's (out_layout receives the layout the cells follow); with `order`
 * (pgpu_node_query_topk) each device keeps only its best order->k rows by the ORDER BY key, ties kept -- exact,
 * because every row a device holds is final -- and the caller's ORDER BY ... LIMIT over the union equals the one
 * over all groups.  Replaces the host-side combine (AggregationOnlyCombineOperator.java:47-57,
 * GroupByOrderByCombineOperator.java:127-248, trim size GroupByUtils.getTableCapacity, GroupByUtils.java:24-41). */
typedef struct pgpu_node pgpu_node;
int pgpu_node_init(const int32_t* device_ordinals, int32_t num_devices, pgpu_node** out_node);
int pgpu_node_context(pgpu_node* node, int32_t index, pgpu_context** out_ctx);
int pgpu_node_shutdown(pgpu_node* node);
int pgpu_node_query(pgpu_node* node, const pgpu_query_desc* const* descs, int64_t* out_keys, int64_t* out_cells,
                    uint64_t capacity, uint64_t* out_num_groups, pgpu_query_stats* out_stats,
                    pgpu_table_layout* out_layout);
int pgpu_node_query_topk(pgpu_node* node, const pgpu_query_desc* const* descs, const pgpu_topk* order,
                         int64_t* out_keys, int64_t* out_cells, uint64_t capacity, uint64_t* out_num_groups,
                         pgpu_query_stats* out_stats, pgpu_table_layout* out_layout);
/* The same in two steps, so that several node queries can be in flight (the host plans and merges query i while
 * the devices run query i + 1): pgpu_node_submit agrees the table layout and launches every device into a table set
 * of the query's own; pgpu_node_collect waits for the devices, merges (on per-device merge streams, so a merge
 * never queues behind later queries' kernels), compacts or trims, and releases the query (also on failure).
 * Collect node queries in the order they were submitted.  Replaces the same combine as pgpu_node_query
 * (BaseCombineOperator.java:79-227: the query's segments run while earlier results merge). */
typedef struct pgpu_node_pending pgpu_node_pending;
int pgpu_node_submit(pgpu_node* node, const pgpu_query_desc* const* descs, pgpu_node_pending** out_query);
/* ... with each device's filter as a pgpu_expr_node program (pgpu_query_submit_expr's form: planned per segment
 * inside the library from the literals); exprs[i] == NULL keeps descs[i]'s own per-segment filter trees. */
int pgpu_node_submit_expr(pgpu_node* node, const pgpu_query_desc* const* descs, const pgpu_expr_node* const* exprs,
                          const int32_t* num_nodes, pgpu_node_pending** out_query);
int pgpu_node_collect(pgpu_node_pending* query, const pgpu_topk* order, int64_t* out_keys, int64_t* out_cells,
                      uint64_t capacity, uint64_t* out_num_groups, pgpu_query_stats* out_stats,
                      pgpu_table_layout* out_layout);
/* The partition arithmetic both multi-GPU combines share (host only, no device needed): the key slice
 * [first, first + count) of a dense table of num_keys keys that rank `rank` of `world` owns after the
 * reduce-scatter (slices of ceil(num_keys / world) keys, the last one shorter), and the rank owning a hash-table
 * group key of num_key_words words (-1 on bad arguments). */
void pgpu_slice_of(uint64_t num_keys, int32_t world, int32_t rank, uint64_t* first, uint64_t* count);
int32_t pgpu_key_owner(const int64_t* key_words, int32_t num_key_words, int32_t world);

/* Convenience: submit + collect. */
int pgpu_query_execute(pgpu_context* ctx, const pgpu_query_desc* q, int64_t* out_keys, int64_t* out_cells,
                       uint64_t capacity, uint64_t* out_num_groups, pgpu_query_stats* out_stats);

/* ---- reference execution statistics ---------------------------------------------------------------------
 * numEntriesScannedInFilter as the reference's iterators count it (SVScanDocIdIterator.java:57-98 under
 * AndDocIdSet.java:60-146 / OrDocIdSet.java:58-110 and the And / Or / Not iterators): the segment's filter program
 * (prefix order, as in pgpu_segment_plan) driven over host bitmaps of its leaves' matches -- leaf k in prefix order,
 * doc d at bit d % 32 of leaf_bits[k][d / 32].  The query path computes the same figure itself when the query
 * carries PGPU_Q_EXACT_FILTER_STATS (leaf bitmaps made on the GPU); this entry point is the host routine it uses. */
int pgpu_filter_entries_scanned(const pgpu_filter_node* nodes, int32_t num_nodes, const uint32_t* const* leaf_bits,
                                int32_t num_leaves, int32_t num_docs, int64_t* out);

/* MIN/MAX order-preserving key -> double (value_type = stored type of the aggregated column). */
double pgpu_decode_minmax_key(int64_t key, int32_t value_type);

/* ---- introspection --------------------------------------------------------------------------------------- */
/* Number of workgroups the query kernel launches and the docs per tile (for roofline accounting). */
int pgpu_kernel_geometry(pgpu_context* ctx, int32_t* out_grid, int32_t* out_tile_docs, int32_t* out_block);

#ifdef __cplusplus
}
#endif
#endif /* PINOT_GPU_H */
