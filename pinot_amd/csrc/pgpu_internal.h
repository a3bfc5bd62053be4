// Shared host/device structures of libpinotgpu.so (not part of the ABI).
//
// HBM layout of one uploaded segment column (all copies made once at segment load):
//   fwd       : the FixedBitSVForwardIndexWriter byte stream, unchanged (big-endian, MSB-first, b bits per doc),
//               padded with zeros to a whole number of query tiles + 16 B so a tile is always a full 16-B-aligned
//               read; words are byte-swapped inside the kernel (v_perm) while staging.
//   sorted    : SortedIndexReaderImpl pairs converted to little-endian int32 (start, end) per dict id.
//   dict      : dictionary values converted to little-endian native width (int32/int64/float/double).
//   inverted  : the Roaring portable bytes of every bitmap, unchanged (little-endian), plus a container directory
//               built on the host at upload: per dict id a [first, last) range of DevContainer records.
#pragma once
#include <stdint.h>

#define PGPU_TILE 4096          // forward-index padding granularity in docs (whole tiles are always readable)
#define PGPU_WAVE_TILE 2048     // docs per wave tile: lane l owns docs [32l, 32l+32); 256*b bytes, 16-B aligned
#define PGPU_BLOCK 256          // threads per workgroup (4 independent waves of 64)
#define PGPU_WAVES (PGPU_BLOCK / 64)
#define PGPU_GROUPS (PGPU_TILE / 64)
#define PGPU_MAX_SLOTS 8        // per-lane mask words (7 filter slots + 1 scratch row)
#define PGPU_MAX_AGGS 16
#define PGPU_MAX_GCOLS 8
#define PGPU_LDS_TABLE_BYTES (16 * 1024)

// column kinds
#define PGPU_COL_NONE 0
#define PGPU_COL_FIXED_BIT 1
#define PGPU_COL_SORTED 2

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
  int32_t kind;                   // PGPU_COL_*
  int32_t bits;
  int32_t card;
  int32_t dict_type;              // PGPU_INT .. PGPU_STRING
};

struct DevSeg {
  int32_t num_docs;
  int32_t tile_begin;             // first global tile of this segment
  int32_t prog_begin;             // first instruction
  int32_t prog_len;
  int32_t col_begin;              // index of its first DevColumn (ncols per segment)
  int32_t remap_begin;            // index of its first remap pointer (ngcols per segment)
  int32_t pf_pc;                  // instruction whose column is register-prefetched one tile ahead (-1: none)
  int32_t pad1;
};

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

struct DevInstr {
  int32_t op;
  int32_t col;      // query column
  int32_t pred;     // 0 RANGE, 1 SET (bitset in the pool), 2 LIST (<= 8 ids in the pool)
  int32_t negate;
  int32_t lo, hi;
  int32_t pool_off; // int32 pool offset (SET bitset, id list, doc ranges)
  int32_t n;        // ids / ranges
  int32_t dst;      // written slot
  int32_t src;      // read slot (child / operand)
  int32_t care;     // care slot, -1 = valid docs
  int32_t jump;     // AND short-circuit target (instruction index within the segment program)
};

struct DevAgg {
  int32_t fn;       // PGPU_AGG_*
  int32_t col;      // query column (-1 COUNT)
  int32_t sec;      // table section (0 for COUNT)
  int32_t op;       // PGPU_RED_* of the section
  int32_t vtype;    // dictionary type
  int32_t pad;
};

#define PGPU_MODE_AGG 0
#define PGPU_MODE_LDS 1
#define PGPU_MODE_GLOBAL 2

#define PGPU_STAT_MATCHED 0
#define PGPU_STAT_SCANNED 1
#define PGPU_STAT_SECTOR_BYTES 2
#define PGPU_STAT_DENSE_BYTES 3
#define PGPU_NSTATS 4

struct DevParams {
  const DevSeg* segs;
  const DevInstr* instrs;
  const DevColumn* cols;
  const int32_t* pool;
  const int32_t* const* remaps;   // [nseg * ngcols], nullptr = identity
  int64_t* table;                 // [nsec][G]
  int64_t* slab;                  // AGG mode: [waves][nsec]
  int64_t* stats;                 // [waves][PGPU_NSTATS]
  uint64_t G;
  int32_t nseg;
  int32_t total_tiles;
  int32_t ncols;
  int32_t nagg;
  int32_t ngcols;
  int32_t nsec;
  int32_t mode;
  int32_t flags;
  int32_t pf_words;               // words of the driving column per wave tile (64 * max bits), 0 = no prefetch
  int32_t pad0;
  DevAgg aggs[PGPU_MAX_AGGS];
  int32_t gcols[PGPU_MAX_GCOLS];
  uint32_t gstride[PGPU_MAX_GCOLS];
  int32_t sec_op[PGPU_MAX_AGGS + 1];
};

#define PGPU_FLAG_STATS 1
