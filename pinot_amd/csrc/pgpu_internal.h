// Shared host/device structures of libpinotgpu.so (not part of the ABI).
//
// HBM layout of one uploaded segment column (all copies made once at segment load):
//   fwd       : the FixedBitSVForwardIndexWriter byte stream, unchanged (big-endian, MSB-first, b bits per doc),
//               padded with zeros to a whole number of PGPU_TILE docs + 16 B so every 2048-doc tile is a whole,
//               16-B aligned run of 256*b bytes; words are byte-swapped in registers while decoding.
//   sorted    : SortedIndexReaderImpl pairs converted to little-endian int32 (start, end) per dict id.
//   dict      : dictionary values converted to little-endian native width (int32/int64/float/double).
//   inverted  : the Roaring portable bytes of every bitmap, unchanged (little-endian), plus a container directory
//               built on the host at upload: per dict id a [first, last) range of DevContainer records.
//
// Query kernel geometry (pgpu_kernels.hip): one workgroup per CU.  The first waves are LOADERS: they stream
// the "staged" forward-index columns of the workgroup's tiles into a ring of LDS slots with global_load_lds and
// publish each slot behind a counted vmcnt.  The other waves are CONSUMERS: consumer c takes tiles c, c+NCONS, ... of the
// workgroup's contiguous tile range, decodes the staged columns out of LDS (lane l owns docs [32l, 32l+32) of the
// 2048-doc tile), runs the dense filter program on 32-bit mask words, and either aggregates straight from the
// decoded ids (dense aggregation) or queues candidate doc ids for batched per-doc gathers (residual filter +
// sparse aggregation).  The loader's DMA queue never waits behind a consumer's gathers (separate waves, separate
// vmcnt), which is what keeps enough bytes in flight per CU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PGPU_TILE 4096          // forward-index padding granularity in docs
#define PGPU_WT 2048            // docs per tile: lane l owns docs [32l, 32l+32); 256*b bytes, 16-B aligned
#define PGPU_WAVE_TILE PGPU_WT
// Two kernel variants.  DENSE (some segment aggregates straight from staged tiles; register-heavy): 512 threads =
// 2 loader + 6 consumer waves.  SPARSE (filter + candidate queue only): 1024 threads = 4 loader + 12 consumer
// waves -- small-bit tiles need more loader issue slots and more consumer waves to hide per-tile latency.
#define PGPU_THREADS(dense) ((dense) ? 512 : 1024)
#define PGPU_WAVES_OF(dense) (PGPU_THREADS(dense) / 64)
#define PGPU_NLOAD_OF(dense) ((dense) ? 2 : 4)   // loader waves (each keeps its own 63-instruction vmcnt budget)
#define PGPU_NCONS_OF(dense) (PGPU_WAVES_OF(dense) - PGPU_NLOAD_OF(dense))
#define PGPU_MAX_SLOTS 8        // per-consumer mask rows (filter slots + 1 scratch row)
#define PGPU_MAX_AGGS 16
#define PGPU_MAX_GCOLS 16
#define PGPU_MAX_STAGE 6        // staged (LDS-streamed) columns per segment
#define PGPU_RING_MAX 64        // ring slots (flag arrays are sized for this)
#define PGPU_CQ_CAP 1024        // candidate-queue entries (uint16: consumer-tile index << 11 | doc in tile):
                                // a tile that does not fit behind the queued entries is flushed, then queued
                                // and flushed in two halves of <= 1024
#define PGPU_CQ_FLUSH 256       // candidate-queue flush threshold
#define PGPU_CQ_TILES 32        // a queue spans at most 32 of the consumer's tiles (5-bit tile index)
#define PGPU_AGG_LIST 1024      // dense-agg key / value list entries (int32 each, DENSE variant)
#define PGPU_DOC_U 4            // candidate docs per lane per flush round
#define PGPU_LDS_LIMIT 163840   // gfx950 LDS per CU
#define PGPU_LDS_TABLE_BYTES (32 * 1024)
#define PGPU_SLICE_RANGES 4       // dict-id ranges per bit-sliced fast leaf (RANGE = 1; small IN sets = runs)
#define PGPU_MAX_STAGE_INSTRS 31  // DMA instructions per tile (so two tiles always fit the 6-bit vmcnt)

// per-consumer LDS area: mask rows | list (candidate queue; DENSE: also the key / value lists) | accumulators
#define PGPU_CONS_LIST_BYTES_OF(dense) ((dense) ? 2 * PGPU_AGG_LIST * 4 + 1024 : PGPU_CQ_CAP * 2)
#define PGPU_CONS_ACC_BYTES (PGPU_MAX_AGGS * 8)
// consumer LDS area: mask rows (only as many as the query's programs use, + 1 scratch row), list, partials
#define PGPU_CONS_BYTES(dense, mask_rows) \
  ((mask_rows) * 256 + PGPU_CONS_LIST_BYTES_OF(dense) + PGPU_CONS_ACC_BYTES + PGPU_CQ_TILES * 4)
#define PGPU_FLAG_BYTES (3 * PGPU_RING_MAX * 4)

// column kinds
#define PGPU_COL_NONE 0
#define PGPU_COL_FIXED_BIT 1
#define PGPU_COL_SORTED 2
// Raw (no-dictionary) column: DevColumn::dict holds the values by doc id (little-endian, decoded from the
// FixedByteChunkSVForwardIndexWriter chunks at upload), so a raw column's "dict id" of doc d is d itself and every
// dictionary gather of the aggregation paths reads the value directly.  Predicates on it become per-segment match
// bitmaps (rawpred_kernel) read by PGPU_I_BITS leaves.
#define PGPU_COL_RAW 3
// Multi-value dictionary column: DevColumn::fwd holds the values' dict ids fixed-bit (value index order); its row
// offsets live beside it.  SCAN leaves on it become per-segment match bitmaps (mvpred_kernel) read as PGPU_I_BITS.
#define PGPU_COL_MV 4

// Roaring container types
#define PGPU_CT_ARRAY 0
#define PGPU_CT_BITMAP 1
#define PGPU_CT_RUN 2

struct DevContainer {
  uint32_t key;     // high 16 bits of the doc ids in the container
  uint32_t type;    // PGPU_CT_*
  uint32_t card;    // ARRAY: #values, RUN: #runs, BITMAP: cardinality
  uint32_t offset;  // byte offset of the payload (past the run-count for RUN) in inv_data
};

struct DevColumn {
  const uint32_t* fwd;            // fixed-bit words (raw big-endian bytes)
  const int32_t* sorted;          // (start, end) per dict id, LE
  const void* dict;               // LE values
  const uint32_t* inv_dir;        // card+1 container indexes
  const DevContainer* inv_ct;     // containers
  const uint8_t* inv_data;        // Roaring payload bytes
  const uint32_t* sliced;         // FIXED_BIT: bit-sliced copy (pgpu_bitslice_kernel), nullptr = none
  const uint32_t* vsliced;        // FIXED_BIT over an INT / LONG dictionary: bit planes of each doc's VALUE minus
                                  // vmin (vbits planes per tile, same layout as `sliced`; vslice_kernel), or nullptr
  int64_t vmin;
  int32_t vbits;
  int32_t kind;                   // PGPU_COL_*
  int32_t bits;
  int32_t card;
  int32_t dict_type;              // PGPU_INT .. PGPU_STRING
  int32_t pad_;
};

// Aggregation plan of a segment
#define PGPU_AM_COUNT 0   // COUNT(*) only, no group-by: matched docs are only counted
#define PGPU_AM_DENSE 1   // group / agg column ids decoded from the staged LDS slot
#define PGPU_AM_SPARSE 2  // matched docs queued; ids gathered per doc
#define PGPU_AM_SLICED 3  // aggregation-only: agg columns staged bit-sliced, matched docs' ids read from the planes
                          // in registers, values gathered from the dictionary (query_kernel_direct only)

#define PGPU_PREBITS 4
#define PGPU_FOR_MAX_BITS 16  // frame-of-reference dictionaries: widest per-block offset
struct DevSeg {
  int32_t num_docs;
  int32_t tile_begin;             // first global tile of this segment
  int32_t ntiles;
  int32_t col_begin;              // index of its first DevColumn (ncols per segment)
  int32_t remap_begin;            // index of its first remap pointer (ngcols per segment)
  int32_t prog_begin, prog_len;   // dense program: mask words of 32 consecutive docs per lane
  int32_t rprog_begin, rprog_len; // residual program: evaluated per queued candidate doc (0 = none)
  int32_t nstage;                 // staged columns
  int32_t stage_instrs;           // DMA instructions per tile for the staged columns
  int32_t agg_mode;               // PGPU_AM_*
  int32_t nreg;                   // AM_DENSE: columns decoded into registers before the slot is released
                                  //           (-1: the slot is held for the whole tile)
  int32_t reg_col[2];             // query columns of the register copies
  int32_t fast;                   // dense program is 1 staged SCAN leaf or an AND of 2 (RANGE / MASK predicates):
                                  // evaluated in registers, without the interpreter (0 = interpret)
  int32_t stage_col[PGPU_MAX_STAGE];   // query column of staged column j
  int32_t stage_off[PGPU_MAX_STAGE];   // byte offset of its region in a ring slot
  int32_t fast_ins[2];            // the fast leaves: instruction index within the dense program
  int32_t stage_sliced;           // bit j: staged column j is streamed from its bit-sliced copy
  // fast leaf j evaluated on bit planes (staged sliced): f_nr[j] ranges [lo, hi) of dict ids, OR-ed, then
  // negated when f_sneg[j] (0 ranges = the leaf decodes the packed layout)
  int32_t f_nr[2];
  int32_t f_sneg[2];
  int32_t f_nostat[2];            // fast leaf j does not count towards numEntriesScannedInFilter (range-index leaf)
  uint32_t f_rng[2][PGPU_SLICE_RANGES][2];
  int32_t track;                  // HASH mode: 1 + row of this segment's distinct-key bitmap (0 = not counted)
  // PGPU_Q_EXACT_FILTER_STATS: the leaves of the segment's whole (unsplit) filter program, in prefix order --
  // instruction indexes at pool[leaf_begin, +leaf_len); leaf k's match bits at leaf_bits[leaf_bits_off +
  // k * ntiles * 64 + tile * 64 + lane] (leafbits_kernel)
  int32_t leaf_len;
  int32_t leaf_begin;
  int32_t single_bits;            // the dense program is one precomputed BITS leaf (progbits_kernel's output):
                                  // a tile's match word is one load, no interpreter
  int64_t leaf_bits_off;
  // BITS leaves of the dense program (their instructions' n = slot): the query kernel loads their words for a
  // tile together before interpreting the program, one round trip instead of one per leaf
  int32_t nbits;
  int32_t pad2_;
  const uint32_t* bits_w[PGPU_PREBITS];
  // register-direct prefix pre-filter (DevParams::rd_pfx planes): the residual SCAN leaf's query column (-1: none)
  // and the ranges [lo, hi) of its ids' top rd_pfx bits that can match, OR-ed -- a candidate outside them cannot
  // match the leaf, so it is never gathered
  int32_t pfx_col;
  int32_t pfx_nr;
  uint32_t pfx_rng[PGPU_SLICE_RANGES][2];
  // PGPU_AM_SLICED with every aggregation from value planes (self-loading kernel): the aggregated columns' value
  // planes are DMA'd into the slot beside the staged filter columns (query column, byte offset in the slot)
  int32_t nvstage;
  int32_t vstage_col[2];
  int32_t vstage_off[2];
  // index-only dense program as a truth table (register streaming, DevParams::direct == 4): bit t = the program's
  // result when leaf i has the value of bit i of t; leaves 0 .. nbits - 1 are the BITS slots, then the SORTED leaves
  // at instruction indexes psorted[0 .. pnsorted) (absolute, into DevParams::instrs)
  uint32_t ptt;
  int32_t pnsorted;
  int32_t psorted[2];
  // query_kernel_rkey (DevParams::direct == 5): the segment's first (segment, container key) unit, and for each BITS
  // slot the inverted leaf it stands for (index into DevParams::invx)
  // query_kernel_cand (direct == 6) units are the containers of the leading inverted leaf (or the sorted leaf's
  // ranges) instead: unit_begin is the segment's first, cand_leaf the inverted leaf (index into DevParams::invx; -1
  // for a sorted one)
  int32_t unit_begin;
  int32_t inv_leaf[PGPU_PREBITS];
  int32_t cand_leaf;
  int32_t pad5_[2];
};
#define PGPU_PFX_PLANES 3  // top bit planes of the residual column streamed beside the fast leaf (DevParams::rd_pfx)

// Filter instruction with statically resolved mask slots.
#define PGPU_I_ALL 0
#define PGPU_I_EMPTY 1
#define PGPU_I_SCAN 2
#define PGPU_I_INV 3
#define PGPU_I_SORTED 4
#define PGPU_I_AND_BEGIN 5
#define PGPU_I_AND_CHILD 6
#define PGPU_I_AND_END 7
#define PGPU_I_OR_BEGIN 8
#define PGPU_I_OR_CHILD 9
#define PGPU_I_OR_END 10
#define PGPU_I_NOT 11
// match bits precomputed per doc (raw-value leaves: rawpred_kernel output at DevInstr::fwd, bit d % 32 of word d / 32)
#define PGPU_I_BITS 12

struct DevInstr {
  int32_t op;
  int32_t col;      // query column
  int32_t pred;     // 0 RANGE, 1 SET (bitset in the pool), 2 LIST (<= 8 ids inline)
  int32_t negate;
  int32_t lo, hi;
  int32_t pool_off; // int32 pool offset (SET bitset, bitmap ids, doc ranges)
  int32_t n;        // ids / ranges
  int32_t dst;      // written slot
  int32_t src;      // read slot (child / operand)
  int32_t care;     // care slot, -1 = valid docs
  int32_t jump;     // AND short-circuit target (instruction index within the program)
  // SCAN leaves carry their column so one scalar load has everything the leaf needs
  int32_t stage_off;  // byte offset of the staged region in a ring slot, -1 = read from HBM
  int32_t bits;
  int32_t kind;       // PGPU_COL_*
  int32_t card;
  const uint32_t* fwd;
  const int32_t* sorted;
  uint32_t ids[8];    // LIST ids
  // leaf entries do not count towards numEntriesScannedInFilter: RangeIndexBasedFilterOperator (an exact bit-sliced
  // range index) answers the leaf from its bitmaps (RangeIndexBasedFilterOperator.java:58-64); on the GPU the same
  // doc set comes from the forward index
  int32_t nostat;
  int32_t pad_[3];
};
static_assert(sizeof(DevInstr) == 128, "DevInstr layout");

// One raw-value filter leaf of one segment (ScanBasedFilterOperator with a RawValueBased*PredicateEvaluator, or
// RangeIndexBasedFilterOperator over a raw column): rawpred_kernel evaluates it over every doc into a bitmap before
// the query kernel runs (PGPU_I_BITS reads it).
struct RawLeaf {
  const void* values;   // the column's little-endian values (DevColumn::dict of a PGPU_COL_RAW column)
  uint32_t* out;        // ntiles * 64 words; bit d % 32 of word d / 32, 0 past num_docs
  int32_t num_docs;
  int32_t words;
  int32_t vtype;        // PGPU_INT .. PGPU_DOUBLE
  int32_t pred;         // PGPU_PRED_RANGE / PGPU_PRED_SET
  int32_t flags;        // RANGE: bit 0 lower inclusive, bit 1 upper inclusive (unbounded = inclusive type extreme)
  int32_t negate;       // NOT_EQ / NOT_IN
  int32_t nvals;        // SET: values at vals
  int32_t pad_;
  int64_t lo, hi;       // RANGE bounds: int64 (INT / LONG) or double bits (FLOAT / DOUBLE)
  const int64_t* vals;  // SET: int64 values ascending (INT / LONG) or order-preserving keys of the doubles ascending
};
// A SCAN leaf on a multi-value column (applyMV): bit d set when any value of row d is in [lo, hi) (RANGE) or in the
// id set (SET), complemented within [0, num_docs) when negate.
struct MvLeaf {
  const uint32_t* fwd;  // the values' dict ids, fixed-bit MSB-first (the file's raw-data section), padded
  const int32_t* off;   // num_docs + 1 row offsets into the value index
  const uint32_t* set;  // SET: membership bits over dict ids (bit id % 32 of word id / 32); null for RANGE
  uint32_t* out;        // ntiles * 64 words; bit d % 32 of word d / 32, 0 past num_docs
  int32_t num_docs;
  int32_t words;
  int32_t bits;
  int32_t lo, hi;       // RANGE: lo <= id < hi
  int32_t negate;
};

// An inverted-index leaf expanded into a doc bitmap before the query kernel (invexp_kernel): one workgroup per
// (leaf, 65,536-doc container key) ORs the key's container of every id, complemented within [0, num_docs) when negate.
// An index-only dense program evaluated once per query over all of a segment's tiles (progbits_kernel), its
// match words then read by the query kernel as one BITS leaf: the interpreter and the leaves' per-tile loads leave
// the query kernel's critical path.
struct ProgJob {
  int32_t seg;                // query segment
  int32_t prog_begin, prog_len;  // the original program
  int32_t tile0;              // first tile of this job in the progbits grid
  int32_t ntiles;
  int32_t nbits;              // its BITS leaves' bitmaps (instruction n = slot), loaded together per tile
  uint32_t* out;              // ntiles * 64 words (a workspace bitmap)
  const uint32_t* bits_w[PGPU_PREBITS];
};

struct InvLeafX {
  const uint32_t* dir;     // DevColumn::inv_dir
  const DevContainer* ct;  // DevColumn::inv_ct
  const uint8_t* data;     // DevColumn::inv_data
  const int32_t* ids;      // the leaf's dict ids
  uint32_t* out;           // ntiles * 64 words; bit d % 32 of word d / 32, 0 past num_docs
  int32_t nids;
  int32_t negate;
  int32_t num_docs;
  int32_t words;
  int32_t nkeys;           // 65,536-doc container keys of the segment
  int32_t ctab_off;        // query_kernel_rkey: its (id, key) records in DevParams::rk_ctab, id-major
  int32_t skip;            // not expanded (query_kernel_cand iterates its containers and nothing reads `out`)
  int32_t pad_;
};
#define PGPU_RKEY_PAIRS 64  // query_kernel_rkey: (leaf, id) pairs of one segment's program at most

#define PGPU_RAW_RANGE_LO_INCL 1
#define PGPU_RAW_RANGE_HI_INCL 2
#define PGPU_RAW_RANGE_ORDINAL 4  // range-index semantics for FLOAT / DOUBLE: NaN orders as -infinity (FPOrdering)

struct DevAgg {
  int32_t fn;       // PGPU_AGG_*
  int32_t col;      // query column (-1 COUNT)
  int32_t sec;      // table section (0 for COUNT)
  int32_t op;       // PGPU_RED_* of the section
  int32_t vtype;    // dictionary type
  int32_t emit;     // PART mode: this aggregation's column is the one carried in the records (first such agg)
  int32_t part;     // split integer SUM (pgpu_table_layout.agg_sum_parts == 3): 0 whole value, 1 bits [0,21),
                    // 2 bits [21,42), 3 bits [42,64) (arithmetic) -- each a SUM_I64 section of its own
  int32_t fxe;      // FLOAT / DOUBLE SUM_I64 (fixed point): the value's cell is rint(v * 2^-fxe) before the part split
};
#define PGPU_PART_BITS 21

#define PGPU_MODE_AGG 0
#define PGPU_MODE_LDS 1
#define PGPU_MODE_GLOBAL 2
// Large key spaces (G >= PGPU_PART_MIN_KEYS): the query kernel appends (key[, raw value]) records to per
// (key partition, workgroup) regions in HBM, then part_reduce_kernel aggregates each partition in an LDS table.
// Replaces one HBM atomic per (doc, section) with plain record stores + LDS atomics.
#define PGPU_MODE_PART 3
#define PGPU_PART_MIN_KEYS 65536
#define PGPU_PART_LDS_BYTES (128 * 1024)   // phase-2 LDS table per partition (keys x sections x 8 B)
#define PGPU_PART_MAX_PARTS 8192           // phase-1 LDS cursors (4 B each) must fit PGPU_LDS_TABLE_BYTES
#define PGPU_PART_MAX_SECTIONS 5           // count + up to 4 value sections (part_reduce_kernel<NS>)
#define PGPU_PSCAN_MAX_PARTS 2048          // part_scan_kernel: LDS rings of at most this many partitions
// Hash group-by (PGPU_KEYS_HASH): the table's cells are indexed by an open-addressing slot (linear probing,
// lock-free 64-bit CAS insert).  Keys of more than 63 bits are interned in two levels: word 0 (columns
// [0, key_split)) gets a slot s0 in a first table, then the slot of (s0 << 32 | word 1) is the cell index.
#define PGPU_MODE_HASH 4
#define PGPU_HASH_EMPTY (~0ull)

// Owner of a group key in the node-level / multi-rank combine of hash tables: the key words chained with the
// golden-ratio multiplier, two murmur3 fmix64 steps, modulo the device count -- bit for bit the routing of
// pinot_amd/combine.py (_hash_merge_topk), so both combines send a key to the same rank.
__host__ __device__ inline uint32_t pgpu_key_owner_of(const int64_t* key, int kw, int world) {
  uint64_t h = (uint64_t)key[0];
  for (int w = 1; w < kw; ++w) h = h * 0x9E3779B97F4A7C15ull + (uint64_t)key[w];
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return (uint32_t)(h % (uint64_t)world);
}
// Section ops of a table, by value (node merge kernel)
struct NodeOps {
  int32_t op[PGPU_MAX_SECTIONS];
};

#define PGPU_STAT_MATCHED 0
#define PGPU_STAT_SCANNED 1
#define PGPU_STAT_SECTOR_BYTES 2
#define PGPU_STAT_DENSE_BYTES 3
#define PGPU_NSTATS 4
// a ring slot's FULL flag with this bit: the loader saw the query cancelled and loaded nothing -- skip the tile
#define PGPU_SLOT_SKIP 0x40000000
#define PGPU_CANCEL_POLL 16   // tiles (per loader / self-loading wave) or phase-1 steps between polls

struct DevParams {
  const DevSeg* segs;
  const DevInstr* instrs;
  const DevColumn* cols;
  const int32_t* pool;
  const int32_t* const* remaps;   // [nseg * ngcols], nullptr = identity
  int64_t* table;                 // [nsec][G]
  int64_t* slab;                  // AGG mode: [waves][nsec]
  int64_t* stats;                 // [waves][PGPU_NSTATS]
  int64_t* prof;                  // [waves][PGPU_NPROF] (PGPU_FLAG_PROFILE)
  uint64_t G;
  int32_t nseg;
  int32_t total_tiles;
  int32_t ncols;
  int32_t nagg;
  int32_t ngcols;
  int32_t nsec;
  int32_t mode;
  int32_t flags;
  int32_t ring_slots;             // R
  int32_t slot_bytes;             // S (multiple of 16)
  int32_t inflight;               // loader's published-behind window (slots)
  int32_t ltab_bytes;             // LDS group table bytes (MODE_LDS)
  int32_t max_instrs;             // max DMA instructions of one tile (loader vmcnt budget)
  int32_t dense;                  // kernel variant (PGPU_THREADS)
  // PART mode: records of rw uint32 words {global key[, raw 4-byte dictionary value of column pcol]}; region of
  // (partition q, workgroup w) = records [(w * nparts + q) * rcap, +rcap); rcount[q * grid + w] = records written
  uint32_t* recs;
  uint32_t* rcount;
  int32_t pshift;                 // keys per partition = 1 << pshift
  int32_t nparts;
  int32_t rcap;
  int32_t rw;
  int32_t pcol;                   // query column carried in the records (-1: COUNT only)
  int32_t rec_idbits;             // > 0: one-word records ((key & partition mask) << rec_idbits | dict id) -- every
                                  // segment shares pcol's dictionary (pdict); 0: {key, raw 4-byte value} records
  const void* pdict;              // rec_idbits > 0: the shared dictionary of pcol
  int32_t pscan;                  // > 0: phase 1 by part_scan_kernel (dense filter programs) with LDS rings of
                                  // this many records per partition (a power of two, >= two 128-B lines)
  int32_t pscan_wave_bytes;       // its per-wave LDS area (filter mask rows)
  int32_t pscan_kb, pscan_vb;     // > 0: every segment's key and carried column are fixed-bit of these widths (no
                                  // filter, one group column): phase 1 reads the next tile's words a step ahead
  int32_t mask_rows;              // mask rows per consumer (filter slots used + 1 scratch row)
  int32_t cons_bytes;             // PGPU_CONS_BYTES(dense, mask_rows)
  int32_t direct;                 // query_kernel_direct: self-loading waves (every staged column a sliced fast leaf)
  int32_t dslots;                 // direct: LDS slots per wave (dslots - 1 tiles in flight while one is filtered)
  int32_t min_instrs;             // direct: fewest DMA instructions of any segment's tile (counted vmcnt waits)
  // PART with one-word records: ldict = phase 2 reads SUM values from pdict copied into LDS beside its table
  // (1 << slice_shift >= pdict_n entries)
  int32_t slice_shift;
  int32_t ldict;                  // 1: pdict copied whole; 2: its frame-of-reference image pfor (PGPU_FOR_*)
  uint32_t pdict_n;               // pdict entries
  const uint32_t* pfor;           // ldict 2: int32 base per 32-id block, then for_bits-bit offsets packed LSB-first
  int32_t for_bits;
  int32_t for_nblk;
  uint32_t cancel_gen;            // this launch's generation (see cancel)
  // PART region sizing (part_scan phase 1): a sampled counting pass (psample = tile stride) fills pcount, then
  // part_plan_kernel sizes each partition's region in proportion (pcap / poff within a workgroup's block of
  // pblock records) and splits heavy partitions across several phase-2 workgroups (p2work: {q, w0, w1, split}
  // per phase-2 workgroup, q < 0 = idle).  pcap == nullptr: uniform regions of rcap records.
  uint32_t* pcount;
  uint32_t* pcap;
  uint32_t* poff;
  int32_t* p2work;
  uint64_t pblock;
  int32_t psample;
  int32_t p2grid;
  // HASH mode: key words follow the sections in `table` (word 0 at table + nsec * G; two-level keys: the
  // interned word-0 values at + G); segmask = distinct-key bitmaps of the tracked segments ([rows][G / 32]);
  // hflag[0] = a probe sequence ran out of slots (query fails)
  uint32_t* segmask;
  int32_t* hflag;
  uint32_t* leaf_bits;            // PGPU_Q_EXACT_FILTER_STATS (see DevSeg::leaf_bits_off)
  uint32_t* segany;               // [nseg] set to 1 by any wave that matched a doc of the segment (numSegmentsMatched);
                                  // zero between queries (finalize_kernel resets the words it reads)
  const int32_t* cancel;          // == cancel_gen: stop (pgpu_query_cancel / deadline); HBM word, polled per tile range
  int32_t key_words;
  int32_t key_split;
  int32_t segmask_rows;
  int32_t cancel_poll;            // self-loading waves: tiles between cancel polls (PGPU_CANCEL_POLL, env override)
  int32_t rd_planes;              // register-direct: planes per tile held in VGPRs (>= every leaf's width; 8/10/12/16)
  int32_t mv_gmask;               // bit g: group column g is multi-value (sparse_agg_mv expands each doc's values)
  int32_t rd_pfx;                 // register-direct: prefix planes of every segment's residual leaf (0 or PGPU_PFX_PLANES)
  int32_t rs_vplanes;             // register streaming (direct == 3): value planes held per tile (16 or 24)
  int32_t total_units;            // query_kernel_rkey: (segment, 65,536-doc container key) units; query_kernel_cand:
                                  // (segment, container) units
  int32_t rk_leaves;              // query_kernel_rkey: leaf images per LDS buffer (max BITS slots of a segment)
  int32_t rk_ids;                 // query_kernel_rkey: stream the aggregated 16-bit columns' packed ids, gather values
  const struct InvLeafX* invx;    // query_kernel_rkey: the inverted leaves (containers read per unit)
  const struct DevContainer* rk_ctab;  // query_kernel_rkey: container record per (leaf, id, key) (rkey_ctab_kernel)
  const uint32_t* cand_ct;        // query_kernel_cand: per unit {segment, its container's index in InvLeafX::ct
                                  // (~0u: a sorted leaf's doc range), first doc, last doc}
  uint32_t* fsm_fn;               // query_kernel_rfsm (direct == 8): per-tile transducer maps for andfsm_segment_kernel
  uint64_t gstride64[PGPU_MAX_GCOLS];  // HASH: mixed-radix stride of group column g within its key word
  DevAgg aggs[PGPU_MAX_AGGS];
  int32_t gcols[PGPU_MAX_GCOLS];
  uint32_t gstride[PGPU_MAX_GCOLS];
  int32_t sec_op[PGPU_MAX_SECTIONS];
};
static_assert(sizeof(DevParams) <= 4096, "DevParams is a kernel argument");

#define PGPU_FLAG_STATS 1
#define PGPU_FLAG_PROFILE 2   // per-wave phase cycle counters into DevParams::prof (PGPU_PROFILE=1)
#define PGPU_FLAG_NT 4        // direct kernel: tile DMAs with the non-temporal policy (default; PGPU_DIRECT_NT=0 off)
#define PGPU_NPROF 12
// loader phases
#define PGPU_P_L_TOTAL 0
#define PGPU_P_L_FREE 1     // waiting for a free ring slot
#define PGPU_P_L_PUB 2      // counted vmcnt waits before publishing
#define PGPU_P_L_ISSUE 3    // DMA issue
// consumer phases
#define PGPU_P_C_TOTAL 4
#define PGPU_P_C_FULL 5     // waiting for a published slot
#define PGPU_P_C_FILTER 6   // dense filter program
#define PGPU_P_C_AGG 7      // register copies, dense aggregation, queue pushes
#define PGPU_P_C_FLUSH 8    // candidate-queue flushes
#define PGPU_P_C_TILES 9    // tiles processed
#define PGPU_P_C_FETCH 10   // filter: instruction fetch (scalar loads)
#define PGPU_P_C_DECODE 11  // filter: SCAN leaf decode + predicate

// LDS bytes of the query kernel for a given ring / table configuration.
inline uint32_t pgpu_lds_fixed_bytes(int dense, int ltab_bytes, int mask_rows) {
  return (uint32_t)(PGPU_FLAG_BYTES + PGPU_NCONS_OF(dense) * PGPU_CONS_BYTES(dense, mask_rows) +
                    ((ltab_bytes + 15) & ~15));
}
inline uint32_t pgpu_lds_bytes(int dense, int ring_slots, int slot_bytes, int ltab_bytes, int mask_rows) {
  return pgpu_lds_fixed_bytes(dense, ltab_bytes, mask_rows) + (uint32_t)(ring_slots * slot_bytes);
}

// Bytes of one staged column's region in a ring slot and its DMA instruction count.  Widths that are multiples of
// 8 bits get 16 B of padding per lane record so the consumers' ds_read_b128 are bank-conflict free.
// A bit-sliced column is staged as its plain 256*b tile bytes (b planes x 64 lane words: no padding needed).
inline int pgpu_stage_region_bytes(int bits, bool sliced = false) {
  return (bits % 8 == 0 && !sliced) ? 64 * (4 * bits + 16) : 256 * bits;
}
inline int pgpu_stage_instrs(int bits, bool sliced = false) {
  return (bits % 8 == 0 && !sliced) ? bits / 4 + 1 : (bits + 3) / 4;
}

// ---- GPU ORDER BY ... LIMIT trim (pgpu_table_topk) ----------------------------------------------------------------
// Order key of one table row, shared by the device selection (topk_* kernels) and the host path of small tables:
// an unsigned 64-bit key, larger = better, whose order (and ties) equal the host's final-value ORDER BY order
// (plan.py GroupColumns.order_and_limit): doubles of the final values (-0.0 folded into 0.0), integer counts,
// group ids.  Every function compiles for both sides (this header is only included by hipcc-built files).
#define PGPU_TK_COUNT 0
#define PGPU_TK_SUM_I64 1
#define PGPU_TK_SUM_SPLIT 2   // TopkDev::parts 21-bit-part sections, exact as a 256-bit integer
#define PGPU_TK_SUM_F64 3
#define PGPU_TK_MINMAX_INT 4  // order-preserving cell = the integer value
#define PGPU_TK_MINMAX_FP 5   // order-preserving cell = key of the double
#define PGPU_TK_AVG_I64 6
#define PGPU_TK_AVG_SPLIT 7
#define PGPU_TK_AVG_F64 8
#define PGPU_TK_GROUP 9
struct TopkDev {
  int32_t mode;
  int32_t sec;       // first value section
  int32_t desc;
  int32_t word;      // GROUP, hash tables: key word (0 / 1) holding the column
  uint64_t stride;   // GROUP: id = (word / stride) % card
  uint64_t card;
  uint64_t G;
  int32_t nsec;
  int32_t kw;        // 0 dense (cell index = key), 1 one hash key word, 2 two-level hash key
  uint64_t key_base; // dense: key of cell 0
  int32_t fxe;       // SUM / AVG split of a fixed-point floating SUM: value = part sum * 2^fxe (0: integer)
  int32_t parts;     // SUM / AVG split: part sections
};
struct TopkState {  // radix-select state: the best-k threshold's high bits found so far
  uint64_t prefix, mask, kleft;
};

__host__ __device__ inline uint64_t pgpu_tk_double(double d) {
  d = d + 0.0;  // -0.0 -> 0.0: equal doubles, equal keys
  int64_t b;
  __builtin_memcpy(&b, &d, 8);
  const int64_t k = b >= 0 ? b : (b ^ 0x7FFFFFFFFFFFFFFFll);
  return (uint64_t)k ^ 0x8000000000000000ull;
}
// sum_p c[p] * 2^(21 p) over `parts` signed int64 part sums (a split integer SUM, a fixed-point floating SUM) as a
// 256-bit two's-complement integer, rounded once to the nearest double (ties to even): a 64-bit window below the
// leading bit with a sticky bit for everything under it (> 11 guard bits remain below the 53-bit mantissa).
__host__ __device__ inline double pgpu_parts_to_double(const int64_t* c, int parts) {
  uint64_t w[4] = {0, 0, 0, 0};
  for (int p = 0; p < parts; ++p) {
    const uint64_t src[4] = {(uint64_t)c[p], c[p] < 0 ? ~0ull : 0ull, c[p] < 0 ? ~0ull : 0ull, c[p] < 0 ? ~0ull : 0ull};
    const int sh = PGPU_PART_BITS * p, limb = sh / 64, bit = sh % 64;
    uint64_t carry = 0;
    for (int i = 0; i < 4; ++i) {
      uint64_t a = 0;
      if (i >= limb) {
        a = bit ? (src[i - limb] << bit) : src[i - limb];
        if (bit && i - limb - 1 >= 0) a |= src[i - limb - 1] >> (64 - bit);
      }
      const uint64_t s1 = w[i] + a;
      const uint64_t c1 = s1 < a ? 1u : 0u;
      w[i] = s1 + carry;
      carry = c1 + (w[i] < s1 ? 1u : 0u);
    }
  }
  const bool neg = (int64_t)w[3] < 0;
  if (neg) {  // negate
    uint64_t carry = 1;
    for (int i = 0; i < 4; ++i) {
      w[i] = ~w[i] + carry;
      carry = (carry && w[i] == 0) ? 1u : 0u;
    }
  }
  int k = 3;
  while (k > 0 && w[k] == 0) --k;
  double d;
  if (k == 0) {
    d = (double)w[0];
  } else {
    const int lz = __builtin_clzll(w[k]);
    uint64_t m = lz ? ((w[k] << lz) | (w[k - 1] >> (64 - lz))) : w[k];
    bool sticky = lz ? (w[k - 1] << lz) != 0 : w[k - 1] != 0;
    for (int i = 0; i < k - 1; ++i) sticky = sticky || w[i] != 0;
    if (sticky) m |= 1;
    d = ldexp((double)m, 64 * (k - 1) + (64 - lz));
  }
  return neg ? -d : d;
}
__host__ __device__ inline double pgpu_tk_split_sum(const int64_t* t, uint64_t G, int sec, int parts, uint64_t row) {
  int64_t c[PGPU_MAX_FIXED_PARTS];
  for (int p = 0; p < parts && p < PGPU_MAX_FIXED_PARTS; ++p) c[p] = t[(uint64_t)(sec + p) * G + row];
  return pgpu_parts_to_double(c, parts < PGPU_MAX_FIXED_PARTS ? parts : PGPU_MAX_FIXED_PARTS);
}
__host__ __device__ inline uint64_t pgpu_topk_key(const int64_t* t, const TopkDev& s, uint64_t row) {
  const uint64_t G = s.G;
  const int64_t cnt = t[row];
  uint64_t u = 0;
  switch (s.mode) {
    case PGPU_TK_COUNT: u = (uint64_t)cnt ^ 0x8000000000000000ull; break;
    case PGPU_TK_SUM_I64: u = pgpu_tk_double((double)t[(uint64_t)s.sec * G + row]); break;
    case PGPU_TK_SUM_SPLIT: u = pgpu_tk_double(ldexp(pgpu_tk_split_sum(t, G, s.sec, s.parts, row), s.fxe)); break;
    case PGPU_TK_SUM_F64: {
      double d;
      __builtin_memcpy(&d, &t[(uint64_t)s.sec * G + row], 8);
      u = pgpu_tk_double(d);
      break;
    }
    case PGPU_TK_MINMAX_INT: u = pgpu_tk_double((double)t[(uint64_t)s.sec * G + row]); break;
    case PGPU_TK_MINMAX_FP: {
      const int64_t k = t[(uint64_t)s.sec * G + row];
      const int64_t b = k >= 0 ? k : (k ^ 0x7FFFFFFFFFFFFFFFll);
      double d;
      __builtin_memcpy(&d, &b, 8);
      u = pgpu_tk_double(d);
      break;
    }
    case PGPU_TK_AVG_I64: u = pgpu_tk_double((double)t[(uint64_t)s.sec * G + row] / (double)cnt); break;
    case PGPU_TK_AVG_SPLIT:
      u = pgpu_tk_double(ldexp(pgpu_tk_split_sum(t, G, s.sec, s.parts, row), s.fxe) / (double)cnt);
      break;
    case PGPU_TK_AVG_F64: {
      double d;
      __builtin_memcpy(&d, &t[(uint64_t)s.sec * G + row], 8);
      u = pgpu_tk_double(d / (double)cnt);
      break;
    }
    default: {  // PGPU_TK_GROUP
      uint64_t w;
      if (s.kw == 0) {
        w = s.key_base + row;
      } else {
        const int64_t* w0 = t + (uint64_t)s.nsec * G;
        if (s.kw == 1) {
          w = (uint64_t)w0[row];
        } else {
          const uint64_t c = (uint64_t)w0[row];
          w = s.word == 0 ? (uint64_t)w0[G + (c >> 32)] : (c & 0xFFFFFFFFull);
        }
      }
      u = (w / s.stride) % s.card;
      break;
    }
  }
  return s.desc ? u : ~u;  // best = largest key: the largest values (DESC) or the smallest (ASC)
}
