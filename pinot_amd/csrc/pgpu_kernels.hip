// HIP kernels of the MI355X segment query path (gfx950 / CDNA4).
//
// One launch runs a whole query over every segment a GPU owns.  A persistent grid of workgroups strides over
// (segment, 4096-doc tile) pairs; per tile a workgroup
//   1. interprets the segment's filter program (K1: fixed-bit unpack fused with dict-id RANGE/SET predicates;
//      K2: Roaring array/bitmap/run containers OR-ed into tile masks; sorted-index doc ranges; AND/OR/NOT on
//      64-bit ballot masks in LDS),
//   2. compacts the matching doc ids of the tile into an LDS list,
//   3. computes group keys from the group-by columns' dict ids (remapped to global ids) and
//   4. aggregates COUNT/SUM/MIN/MAX/AVG into per-thread registers (aggregation only), an LDS-privatised dense
//      table (small key spaces) or the global dense table (large key spaces)  (K3).
// Columns are read in one of two modes, chosen per tile from the density of the docs that still matter:
//   dense : the tile's bytes of the forward index are streamed into LDS with 16-B coalesced loads and
//           byte-swapped once; each lane then unpacks doc (64*g + lane) with one v_alignbit.
//   sparse: only the docs of the care mask fetch their two words from HBM (sector-granular traffic).
//
// Reference hot loops this replaces (file:line under pinot-core/... and pinot-segment-local/...):
//   FixedBitIntReader.read32 / PinotDataBitSet.readInt           seglocal/io/util/PinotDataBitSet.java:78-165
//   SVScanDocIdIterator.next / applyAnd                           core/operator/dociditerators/SVScanDocIdIterator.java:57-94
//   AndDocIdSet / OrDocIdSet / NotDocIdIterator                   core/operator/docidsets/AndDocIdSet.java:60-146, OrDocIdSet.java:58-110
//   BitmapBasedFilterOperator (Roaring or + flip)                 core/operator/filter/BitmapBasedFilterOperator.java:66-110
//   SortedIndexBasedFilterOperator                                core/operator/filter/SortedIndexBasedFilterOperator.java:51-219
//   Sum/Min/Max/Avg/CountAggregationFunction.aggregate*           core/query/aggregation/function/*.java
//   DictionaryBasedGroupKeyGenerator (raw key = mixed radix)      core/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:275-322
//   AggregationOnlyCombineOperator / GroupByOrderByCombineOperator core/operator/combine/*.java (partials merged in HBM)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pinot_gpu.h"
#include "pgpu_internal.h"

#define TILE PGPU_TILE
#define NT PGPU_BLOCK
#define NW PGPU_WAVES
#define NG PGPU_GROUPS

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct __attribute__((aligned(16))) Smem {
  uint32_t stage[TILE + 16];             // staged forward-index words of one column (byte-swapped), at +4
  uint64_t masks[PGPU_MAX_SLOTS][NG];    // filter mask slots
  uint64_t valid[NG];                    // docs < num_docs
  uint16_t list[TILE];                   // compacted matching doc offsets
  int32_t goff[NG + 1];                  // exclusive prefix of per-group match counts
  int32_t slot_count[PGPU_MAX_SLOTS];    // popcount of each AND accumulator
  int32_t nvalid;
  uint32_t sectors[TILE / 256 * 32 / 32 + 16];  // touched 32-B sectors of a sparse read (stats mode)
  int64_t accw[NW][PGPU_MAX_AGGS];       // AGG mode: per-wave accumulators
  int64_t bstats[PGPU_NSTATS];
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint32_t lowmask(uint32_t b) { return 0xFFFFFFFFu >> (32u - b); }

// Value whose last bit is stream bit e-1 (MSB-first), from byte-swapped words st[] (st[-1] readable).
__device__ __forceinline__ uint32_t extract_lds(const uint32_t* st, uint32_t e, uint32_t b) {
  uint32_t we = (e - 1u) >> 5;
  uint32_t r = e - (we << 5);  // 1..32 bits of the value in word we
  uint32_t lo = st[(int)we - 1];
  uint32_t hi = st[we];
  return __builtin_amdgcn_alignbit(lo, hi, 32u - r) & lowmask(b);
}

// Same from the raw big-endian words in HBM; e is the segment-level end bit.
__device__ __forceinline__ uint32_t extract_global(const uint32_t* __restrict__ words, uint64_t e, uint32_t b) {
  uint64_t we = (e - 1u) >> 5;
  uint32_t r = (uint32_t)(e - (we << 5));
  uint32_t hi = bswap32(words[we]);
  uint32_t lo = we ? bswap32(words[we - 1]) : 0u;
  return __builtin_amdgcn_alignbit(lo, hi, 32u - r) & lowmask(b);
}

// SortedIndexReaderImpl.getDictId: last dict id whose start <= doc (binary search over the start offsets).
__device__ __forceinline__ uint32_t sorted_dict_id(const int32_t* __restrict__ pairs, int32_t card, int32_t doc) {
  int32_t lo = 0, hi = card - 1;
  while (lo <= hi) {
    int32_t mid = (lo + hi) >> 1;
    if (pairs[2 * mid] <= doc) lo = mid + 1; else hi = mid - 1;
  }
  return (uint32_t)hi;
}

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(v, o, 64); v = t < v ? t : v; }
  return v;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(v, o, 64); v = t > v ? t : v; }
  return v;
}
__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Order-preserving int64 key of a dictionary value (MIN/MAX sections).
__device__ __forceinline__ int64_t minmax_key(const void* dict, int32_t vtype, uint32_t id) {
  switch (vtype) {
    case PGPU_INT: return (int64_t)((const int32_t*)dict)[id];
    case PGPU_LONG: return ((const int64_t*)dict)[id];
    case PGPU_FLOAT: {
      double d = (double)((const float*)dict)[id];
      int64_t b = __double_as_longlong(d);
      return b >= 0 ? b : (b ^ 0x7FFFFFFFFFFFFFFFll);
    }
    default: {
      int64_t b = __double_as_longlong(((const double*)dict)[id]);
      return b >= 0 ? b : (b ^ 0x7FFFFFFFFFFFFFFFll);
    }
  }
}
__device__ __forceinline__ int64_t value_i64(const void* dict, int32_t vtype, uint32_t id) {
  return vtype == PGPU_INT ? (int64_t)((const int32_t*)dict)[id] : ((const int64_t*)dict)[id];
}
__device__ __forceinline__ double value_f64(const void* dict, int32_t vtype, uint32_t id) {
  return vtype == PGPU_FLOAT ? (double)((const float*)dict)[id] : ((const double*)dict)[id];
}

__device__ __forceinline__ int64_t sec_identity(int32_t op) {
  return op == PGPU_RED_MIN_I64 ? INT64_MAX : (op == PGPU_RED_MAX_I64 ? INT64_MIN : 0);
}

// ---- staging -------------------------------------------------------------------------------------------------
// Copy the tile's ceil(TILE*b/128) 16-B chunks of the forward index into Smem.stage (+4 words), byte-swapped.
__device__ __forceinline__ void stage_column(Smem& sm, const uint32_t* __restrict__ fwd, int32_t tile_in_seg,
                                             uint32_t b) {
  const u32x4* src = (const u32x4*)(fwd + (size_t)tile_in_seg * (TILE / 32) * b);
  u32x4* dst = (u32x4*)(sm.stage + 4);
  const int n16 = (TILE / 128) * b;
  for (int i = threadIdx.x; i < n16; i += NT) {
    u32x4 v = src[i];
    v.x = bswap32(v.x); v.y = bswap32(v.y); v.z = bswap32(v.z); v.w = bswap32(v.w);
    dst[i] = v;
  }
}

struct TileCtx {
  const DevSeg* seg;
  int32_t tile_in_seg;
  int32_t doc0;      // first doc of the tile (segment-local)
  int32_t ndocs;     // docs of the tile inside the segment
};

// Dict id of tile-relative doc j of column c, from the staged copy (dense) or HBM (sparse).
__device__ __forceinline__ uint32_t get_id(const Smem& sm, const DevColumn& c, const TileCtx& t, int j,
                                           bool staged) {
  if (c.kind == PGPU_COL_SORTED) return sorted_dict_id(c.sorted, c.card, t.doc0 + j);
  const uint32_t b = (uint32_t)c.bits;
  if (staged) return extract_lds(sm.stage + 4, (uint32_t)(j + 1) * b, b);
  return extract_global(c.fwd, (uint64_t)(t.doc0 + j + 1) * b, b);
}

__device__ __forceinline__ bool eval_pred(const DevInstr& in, const int32_t* __restrict__ pool, uint32_t id) {
  bool m;
  if (in.pred == PGPU_PRED_RANGE) {
    m = (id - (uint32_t)in.lo) < (uint32_t)(in.hi - in.lo);
  } else {
    m = (pool[in.pool_off + (id >> 5)] >> (id & 31)) & 1;
  }
  return m != (in.negate != 0);
}

// Block-wide popcount of mask slot `s` (wave 0 computes, result in sm.slot_count[s]); caller syncs.
__device__ __forceinline__ void count_slot(Smem& sm, int s) {
  if (threadIdx.x < 64) {
    int c = __popcll(sm.masks[s][threadIdx.x]);
    c = wave_sum_i32(c);
    if (threadIdx.x == 0) sm.slot_count[s] = c;
  }
}

__device__ __forceinline__ const uint64_t* care_mask(const Smem& sm, int care) {
  return care < 0 ? sm.valid : sm.masks[care];
}
__device__ __forceinline__ int care_count(const Smem& sm, int care) {
  return care < 0 ? sm.nvalid : sm.slot_count[care];
}

// Sector bookkeeping for a sparse read of doc j (stats mode): bytes [j*b/8, ((j+1)*b-1)/8] of the tile.
__device__ __forceinline__ void mark_sectors(Smem& sm, int j, uint32_t b) {
  uint32_t s0 = ((uint32_t)j * b) >> 8;             // 32-B sector = 256 bits
  uint32_t s1 = ((uint32_t)(j + 1) * b - 1u) >> 8;
  atomicOr(&sm.sectors[s0 >> 5], 1u << (s0 & 31));
  if (s1 != s0) atomicOr(&sm.sectors[s1 >> 5], 1u << (s1 & 31));
}

// OR the tile slice of one Roaring bitmap (dict id `id` of column c) into mask slot `dst` (LDS atomics).
__device__ void or_bitmap(Smem& sm, const DevColumn& c, const TileCtx& t, uint32_t id, int dst) {
  const uint32_t key = (uint32_t)t.doc0 >> 16;
  const uint32_t lo16 = (uint32_t)t.doc0 & 0xFFFFu;  // tile start within the 65536-doc chunk
  int32_t a = (int32_t)c.inv_dir[id], z = (int32_t)c.inv_dir[id + 1] - 1;
  int32_t ci = -1;
  while (a <= z) {  // containers are sorted by key
    int32_t mid = (a + z) >> 1;
    uint32_t k = c.inv_ct[mid].key;
    if (k == key) { ci = mid; break; }
    if (k < key) a = mid + 1; else z = mid - 1;
  }
  if (ci < 0) return;
  const DevContainer ct = c.inv_ct[ci];
  if (ct.type == PGPU_CT_BITMAP) {
    const uint64_t* w = (const uint64_t*)(c.inv_data + ct.offset) + (lo16 >> 6);
    for (int g = threadIdx.x; g < NG; g += NT) {
      uint64_t v = w[g];
      if (v) atomicOr((unsigned long long*)&sm.masks[dst][g], (unsigned long long)v);
    }
  } else if (ct.type == PGPU_CT_ARRAY) {
    const uint16_t* v = (const uint16_t*)(c.inv_data + ct.offset);
    // first index with v >= lo16 and first with v >= lo16 + TILE
    int32_t l = 0, h = (int32_t)ct.card;
    while (l < h) { int32_t m = (l + h) >> 1; if (v[m] < lo16) l = m + 1; else h = m; }
    int32_t first = l;
    h = (int32_t)ct.card;
    while (l < h) { int32_t m = (l + h) >> 1; if ((uint32_t)v[m] < lo16 + TILE) l = m + 1; else h = m; }
    for (int32_t i = first + threadIdx.x; i < l; i += NT) {
      uint32_t off = (uint32_t)v[i] - lo16;
      atomicOr((unsigned long long*)&sm.masks[dst][off >> 6], 1ull << (off & 63));
    }
  } else {  // RUN: pairs (start, length-1)
    const uint16_t* r = (const uint16_t*)(c.inv_data + ct.offset);
    int32_t l = 0, h = (int32_t)ct.card;
    // first run whose end >= lo16
    while (l < h) {
      int32_t m = (l + h) >> 1;
      if ((uint32_t)r[2 * m] + r[2 * m + 1] < lo16) l = m + 1; else h = m;
    }
    for (int32_t i = l + threadIdx.x; i < (int32_t)ct.card; i += NT) {
      uint32_t s = r[2 * i], e = s + r[2 * i + 1];  // inclusive
      if (s >= lo16 + TILE) break;
      uint32_t s2 = s < lo16 ? 0u : s - lo16;
      uint32_t e2 = (e >= lo16 + TILE ? lo16 + TILE - 1 : e) - lo16;
      for (uint32_t w = s2 >> 6; w <= (e2 >> 6); ++w) {
        uint32_t bs = w == (s2 >> 6) ? (s2 & 63) : 0u;
        uint32_t be = w == (e2 >> 6) ? (e2 & 63) : 63u;
        uint64_t mk = (~0ull >> (63 - be)) & (~0ull << bs);
        atomicOr((unsigned long long*)&sm.masks[dst][w], (unsigned long long)mk);
      }
    }
  }
}

// Compact the docs of `mask` (tile-relative) into sm.list (ascending); zeroes mask slot `zero_slot` on the way
// (>= 0).  Returns the count.  Contains two __syncthreads().
__device__ __forceinline__ int compact_mask(Smem& sm, const uint64_t* mask, int zero_slot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x < 64) {
    const int g = threadIdx.x;
    const int c = __popcll(mask[g]);
    int x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    sm.goff[g] = x - c;
    if (g == 63) sm.goff[NG] = x;
  }
  __syncthreads();
  for (int g = wave; g < NG; g += NW) {
    const uint64_t m = mask[g];
    if ((m >> lane) & 1ull) {
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      sm.list[sm.goff[g] + below] = (uint16_t)(g * 64 + lane);
    }
  }
  if (zero_slot >= 0 && threadIdx.x < 64) sm.masks[zero_slot][threadIdx.x] = 0ull;
  __syncthreads();
  return sm.goff[NG];
}

// ---- filter program ------------------------------------------------------------------------------------------
// Returns with the final match mask in sm.masks[0] (or sm.valid when the program is empty) -> *final_slot.
__device__ int run_filter(Smem& sm, const DevParams& p, const TileCtx& t, const DevColumn* cols,
                          int64_t& scanned, int64_t& sector_bytes, int64_t& dense_bytes) {
  const DevSeg& s = *t.seg;
  if (s.prog_len == 0) return -1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int pc = 0;
  while (pc < s.prog_len) {
    const DevInstr in = p.instrs[s.prog_begin + pc];
    int next = pc + 1;
    switch (in.op) {
      case PGPU_I_ALL:
      case PGPU_I_EMPTY:
        if (threadIdx.x < 64) sm.masks[in.dst][threadIdx.x] = in.op == PGPU_I_ALL ? sm.valid[threadIdx.x] : 0ull;
        __syncthreads();
        break;
      case PGPU_I_SCAN: {
        const DevColumn& c = cols[in.col];
        const uint64_t* care = care_mask(sm, in.care);
        const int ncare = care_count(sm, in.care);
        const uint32_t b = (uint32_t)c.bits;
        const bool prestaged = pc == s.pf_pc;
        const bool dense = prestaged || (c.kind == PGPU_COL_FIXED_BIT && ncare * 32 >= t.ndocs);
        if (dense) {
          if (!prestaged) {
            stage_column(sm, c.fwd, t.tile_in_seg, b);
            __syncthreads();
          }
          if (threadIdx.x == 0) {
            scanned += t.ndocs;
            dense_bytes += ((int64_t)t.ndocs * b + 7) / 8;
          }
          for (int g = wave; g < NG; g += NW) {
            const int j = g * 64 + lane;
            bool m = false;
            if (j < t.ndocs) {
              uint32_t id = extract_lds(sm.stage + 4, (uint32_t)(j + 1) * b, b);
              m = eval_pred(in, p.pool, id);
            }
            uint64_t bal = __ballot(m);
            if (lane == 0) sm.masks[in.dst][g] = bal;
          }
        } else {
          const bool stats = (p.flags & PGPU_FLAG_STATS) && c.kind == PGPU_COL_FIXED_BIT;
          if (stats) {
            for (int i = threadIdx.x; i < (int)(sizeof(sm.sectors) / 4); i += NT) sm.sectors[i] = 0;
            __syncthreads();
          }
          if (threadIdx.x == 0) scanned += ncare;
          // Compact the care docs (fewer than ndocs/32 <= 128 here) into sm.list, then one thread per candidate
          // fetches its two words: a single memory round trip for the whole tile, no per-group serialisation.
          const int nc = compact_mask(sm, care, in.dst);
          for (int k = threadIdx.x; k < nc; k += NT) {
            const int j = sm.list[k];
            const uint32_t id = get_id(sm, c, t, j, false);
            if (eval_pred(in, p.pool, id))
              atomicOr((unsigned long long*)&sm.masks[in.dst][j >> 6], 1ull << (j & 63));
            if (stats) mark_sectors(sm, j, b);
          }
          if (stats) {
            __syncthreads();
            if (threadIdx.x < 64) {
              int cnt = 0;
              for (int i = threadIdx.x; i < (int)(sizeof(sm.sectors) / 4); i += 64) cnt += __popc(sm.sectors[i]);
              cnt = wave_sum_i32(cnt);
              if (threadIdx.x == 0) sector_bytes += 32ll * cnt;
            }
          }
        }
        __syncthreads();
        break;
      }
      case PGPU_I_INV: {
        const DevColumn& c = cols[in.col];
        if (threadIdx.x < 64) sm.masks[in.dst][threadIdx.x] = 0ull;
        __syncthreads();
        for (int i = 0; i < in.n; ++i) or_bitmap(sm, c, t, (uint32_t)p.pool[in.pool_off + i], in.dst);
        __syncthreads();
        if (in.negate) {
          if (threadIdx.x < 64) sm.masks[in.dst][threadIdx.x] = ~sm.masks[in.dst][threadIdx.x] & sm.valid[threadIdx.x];
          __syncthreads();
        }
        break;
      }
      case PGPU_I_SORTED: {
        if (threadIdx.x < 64) {
          const int g = threadIdx.x;
          const int32_t d0 = t.doc0 + g * 64, d1 = d0 + 63;
          const int32_t* rg = p.pool + in.pool_off;
          // first range whose end >= d0
          int32_t l = 0, h = in.n;
          while (l < h) { int32_t m = (l + h) >> 1; if (rg[2 * m + 1] < d0) l = m + 1; else h = m; }
          uint64_t mk = 0;
          for (int32_t i = l; i < in.n; ++i) {
            int32_t s0 = rg[2 * i], e0 = rg[2 * i + 1];
            if (s0 > d1) break;
            int32_t bs = s0 < d0 ? 0 : s0 - d0;
            int32_t be = e0 > d1 ? 63 : e0 - d0;
            mk |= (~0ull >> (63 - be)) & (~0ull << bs);
          }
          if (in.negate) mk = ~mk;
          sm.masks[in.dst][g] = mk & sm.valid[g];
        }
        __syncthreads();
        break;
      }
      case PGPU_I_AND_BEGIN:
        if (threadIdx.x < 64) sm.masks[in.dst][threadIdx.x] = care_mask(sm, in.care)[threadIdx.x];
        if (threadIdx.x == 0) sm.slot_count[in.dst] = care_count(sm, in.care);
        __syncthreads();
        break;
      case PGPU_I_AND_CHILD:
        if (threadIdx.x < 64) sm.masks[in.dst][threadIdx.x] &= sm.masks[in.src][threadIdx.x];
        count_slot(sm, in.dst);
        __syncthreads();
        if (sm.slot_count[in.dst] == 0) next = in.jump;
        break;
      case PGPU_I_OR_BEGIN:
        if (threadIdx.x < 64) sm.masks[in.dst][threadIdx.x] = 0ull;
        __syncthreads();
        break;
      case PGPU_I_OR_CHILD:
        if (threadIdx.x < 64) sm.masks[in.dst][threadIdx.x] |= sm.masks[in.src][threadIdx.x];
        __syncthreads();
        break;
      case PGPU_I_NOT:
        if (threadIdx.x < 64)
          sm.masks[in.dst][threadIdx.x] = ~sm.masks[in.src][threadIdx.x] & care_mask(sm, in.care)[threadIdx.x];
        __syncthreads();
        break;
      default:  // AND_END / OR_END: result already in dst
        break;
    }
    pc = next;
  }
  return 0;
}

// ---- register prefetch of the driving scan column -------------------------------------------------------------
// The first SCAN of a segment's program (under AND_BEGINs only) is evaluated densely on every tile; its bytes
// for the NEXT tile are loaded into registers while the current tile runs, then written to LDS at the top of
// the next iteration, so the workgroup's dominant stream is always in flight (T14-style issue-early/write-late).
#define PF_REGS 4  // ceil(32 * 32 / NT) 16-B chunks per thread for b <= 32

__device__ __forceinline__ int seg_of_tile(const DevParams& p, int tile) {
  int lo = 0, hi = p.nseg - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (p.segs[mid].tile_begin <= tile) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ int prefetch_regs(const DevParams& p, int tile, u32x4 (&pf)[PF_REGS]) {
  if (tile >= p.total_tiles) return 0;
  const DevSeg& sg = p.segs[seg_of_tile(p, tile)];
  if (sg.pf_pc < 0) return 0;
  const DevInstr& in = p.instrs[sg.prog_begin + sg.pf_pc];
  const DevColumn& c = p.cols[sg.col_begin + in.col];
  const int b = c.bits;
  const u32x4* src = (const u32x4*)(c.fwd + (size_t)(tile - sg.tile_begin) * (TILE / 32) * b);
  const int n16 = (TILE / 128) * b;
#pragma unroll
  for (int k = 0; k < PF_REGS; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < n16) pf[k] = src[i];
  }
  return b;
}

__device__ __forceinline__ void write_prefetched(Smem& sm, const u32x4 (&pf)[PF_REGS], int b) {
  const int n16 = (TILE / 128) * b;
  u32x4* dst = (u32x4*)(sm.stage + 4);
#pragma unroll
  for (int k = 0; k < PF_REGS; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < n16) {
      u32x4 v = pf[k];
      v.x = bswap32(v.x); v.y = bswap32(v.y); v.z = bswap32(v.z); v.w = bswap32(v.w);
      dst[i] = v;
    }
  }
}

// ---- the query kernel ----------------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(NT) void query_kernel(DevParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  __shared__ Smem sm;
  uint32_t* keys = (uint32_t*)dyn_smem;                 // MODE != AGG: group key per compacted entry
  int64_t* ltab = (int64_t*)(dyn_smem + TILE * 4);      // MODE == LDS: [nsec][G]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

  if (MODE == PGPU_MODE_LDS) {
    const int n = p.nsec * (int)p.G;
    for (int i = threadIdx.x; i < n; i += NT) ltab[i] = sec_identity(p.sec_op[i / (int)p.G]);
  }
  if (MODE == PGPU_MODE_AGG) {
    for (int i = threadIdx.x; i < NW * PGPU_MAX_AGGS; i += NT) {
      int a = i % PGPU_MAX_AGGS;
      sm.accw[i / PGPU_MAX_AGGS][a] = a < p.nagg ? sec_identity(p.aggs[a].op) : 0;
    }
  }
  int64_t matched = 0, scanned = 0, sector_bytes = 0, dense_bytes = 0;  // thread 0 owns these
  u32x4 pf[PF_REGS];
  int pf_bits = prefetch_regs(p, blockIdx.x, pf);
  __syncthreads();

  for (int tile = blockIdx.x; tile < p.total_tiles; tile += gridDim.x) {
    TileCtx t;
    t.seg = &p.segs[seg_of_tile(p, tile)];
    if (pf_bits) write_prefetched(sm, pf, pf_bits);   // this tile's driving column -> LDS
    pf_bits = prefetch_regs(p, tile + gridDim.x, pf);  // next tile's bytes stay in flight during this tile
    t.tile_in_seg = tile - t.seg->tile_begin;
    t.doc0 = t.tile_in_seg * TILE;
    t.ndocs = min(TILE, t.seg->num_docs - t.doc0);
    const DevColumn* cols = p.cols + t.seg->col_begin;

    if (threadIdx.x < 64) {
      const int g = threadIdx.x;
      const int rem = t.ndocs - g * 64;
      sm.valid[g] = rem >= 64 ? ~0ull : (rem <= 0 ? 0ull : (~0ull >> (64 - rem)));
    }
    if (threadIdx.x == 0) sm.nvalid = t.ndocs;
    __syncthreads();

    const int fslot = run_filter(sm, p, t, cols, scanned, sector_bytes, dense_bytes);
    const uint64_t* fmask = fslot < 0 ? sm.valid : sm.masks[0];

    // compaction of matching docs -> sm.list (final masks never exceed the valid docs)
    const int nm = compact_mask(sm, fmask, -1);
    if (threadIdx.x == 0) matched += nm;
    if (nm == 0) continue;  // uniform
    const bool dense_post = nm * 32 >= t.ndocs;

    // group keys
    if (MODE != PGPU_MODE_AGG) {
      for (int gc = 0; gc < p.ngcols; ++gc) {
        const DevColumn& c = cols[p.gcols[gc]];
        const int32_t* remap = p.remaps[t.seg->remap_begin + gc];
        const bool staged = dense_post && c.kind == PGPU_COL_FIXED_BIT;
        if (staged) {
          stage_column(sm, c.fwd, t.tile_in_seg, (uint32_t)c.bits);
          __syncthreads();
          if (threadIdx.x == 0) dense_bytes += ((int64_t)t.ndocs * c.bits + 7) / 8;
        }
        const uint32_t stride = p.gstride[gc];
        for (int k = threadIdx.x; k < nm; k += NT) {
          uint32_t id = get_id(sm, c, t, sm.list[k], staged);
          uint32_t gid = remap ? (uint32_t)remap[id] : id;
          keys[k] = (gc == 0 ? 0u : keys[k]) + gid * stride;
        }
        __syncthreads();
      }
      // COUNT section (section 0)
      for (int k = threadIdx.x; k < nm; k += NT) {
        const uint32_t key = keys[k];
        if (MODE == PGPU_MODE_LDS) atomicAdd((unsigned long long*)&ltab[key], 1ull);
        else atomicAdd((unsigned long long*)&p.table[key], 1ull);
      }
    }

    // aggregations
    int staged_col = -1;
    for (int a = 0; a < p.nagg; ++a) {
      const DevAgg ag = p.aggs[a];
      if (ag.fn == PGPU_AGG_COUNT) continue;
      const DevColumn& c = cols[ag.col];
      const bool staged = dense_post && c.kind == PGPU_COL_FIXED_BIT;
      if (staged && staged_col != ag.col) {
        __syncthreads();
        stage_column(sm, c.fwd, t.tile_in_seg, (uint32_t)c.bits);
        __syncthreads();
        staged_col = ag.col;
        if (threadIdx.x == 0) dense_bytes += ((int64_t)t.ndocs * c.bits + 7) / 8;
      }
      if (MODE == PGPU_MODE_AGG) {
        int64_t acc = sec_identity(ag.op);
        double dacc = 0.0;
        for (int k = threadIdx.x; k < nm; k += NT) {
          uint32_t id = get_id(sm, c, t, sm.list[k], staged);
          if (ag.op == PGPU_RED_SUM_I64) acc += value_i64(c.dict, ag.vtype, id);
          else if (ag.op == PGPU_RED_SUM_F64) dacc += value_f64(c.dict, ag.vtype, id);
          else {
            int64_t kk = minmax_key(c.dict, ag.vtype, id);
            acc = ag.op == PGPU_RED_MIN_I64 ? (kk < acc ? kk : acc) : (kk > acc ? kk : acc);
          }
        }
        if (ag.op == PGPU_RED_SUM_I64) acc = wave_sum_i64(acc);
        else if (ag.op == PGPU_RED_SUM_F64) dacc = wave_sum_f64(dacc);
        else if (ag.op == PGPU_RED_MIN_I64) acc = wave_min_i64(acc);
        else acc = wave_max_i64(acc);
        if (lane == 0) {
          int64_t& cell = sm.accw[wave][a];
          if (ag.op == PGPU_RED_SUM_I64) cell += acc;
          else if (ag.op == PGPU_RED_SUM_F64) cell = __double_as_longlong(__longlong_as_double(cell) + dacc);
          else if (ag.op == PGPU_RED_MIN_I64) cell = acc < cell ? acc : cell;
          else cell = acc > cell ? acc : cell;
        }
      } else {
        int64_t* secp = (MODE == PGPU_MODE_LDS ? ltab : p.table) + (size_t)ag.sec * p.G;
        for (int k = threadIdx.x; k < nm; k += NT) {
          uint32_t id = get_id(sm, c, t, sm.list[k], staged);
          const uint32_t key = keys[k];
          if (ag.op == PGPU_RED_SUM_I64)
            atomicAdd((unsigned long long*)&secp[key], (unsigned long long)value_i64(c.dict, ag.vtype, id));
          else if (ag.op == PGPU_RED_SUM_F64)
            atomicAdd((double*)&secp[key], value_f64(c.dict, ag.vtype, id));
          else if (ag.op == PGPU_RED_MIN_I64)
            atomicMin((long long*)&secp[key], (long long)minmax_key(c.dict, ag.vtype, id));
          else
            atomicMax((long long*)&secp[key], (long long)minmax_key(c.dict, ag.vtype, id));
        }
      }
    }
    __syncthreads();
  }

  // ---- block epilogue ----
  __syncthreads();
  if (MODE == PGPU_MODE_AGG) {
    // slab[block][sec]: section 0 = matched count
    int64_t* slab = p.slab + (size_t)blockIdx.x * p.nsec;
    if (threadIdx.x == 0) slab[0] = matched;
    if (threadIdx.x < p.nagg) {
      const int a = threadIdx.x;
      const DevAgg ag = p.aggs[a];
      if (ag.fn != PGPU_AGG_COUNT) {
        int64_t v = sm.accw[0][a];
        for (int w = 1; w < NW; ++w) {
          const int64_t x = sm.accw[w][a];
          if (ag.op == PGPU_RED_SUM_I64) v += x;
          else if (ag.op == PGPU_RED_SUM_F64) v = __double_as_longlong(__longlong_as_double(v) + __longlong_as_double(x));
          else if (ag.op == PGPU_RED_MIN_I64) v = x < v ? x : v;
          else v = x > v ? x : v;
        }
        slab[ag.sec] = v;
      }
    }
  } else if (MODE == PGPU_MODE_LDS) {
    const int G = (int)p.G;
    for (int key = threadIdx.x; key < G; key += NT) {
      const int64_t cnt = ltab[key];
      if (cnt == 0) continue;
      atomicAdd((unsigned long long*)&p.table[key], (unsigned long long)cnt);
      for (int s = 1; s < p.nsec; ++s) {
        const int64_t v = ltab[s * G + key];
        int64_t* dst = &p.table[(size_t)s * p.G + key];
        switch (p.sec_op[s]) {
          case PGPU_RED_SUM_I64: atomicAdd((unsigned long long*)dst, (unsigned long long)v); break;
          case PGPU_RED_SUM_F64: atomicAdd((double*)dst, __longlong_as_double(v)); break;
          case PGPU_RED_MIN_I64: atomicMin((long long*)dst, (long long)v); break;
          default: atomicMax((long long*)dst, (long long)v); break;
        }
      }
    }
  }
  if (threadIdx.x == 0) {
    int64_t* st = p.stats + (size_t)blockIdx.x * PGPU_NSTATS;
    st[PGPU_STAT_MATCHED] = matched;
    st[PGPU_STAT_SCANNED] = scanned;
    st[PGPU_STAT_SECTOR_BYTES] = sector_bytes;
    st[PGPU_STAT_DENSE_BYTES] = dense_bytes;
  }
}

// Table init: count/sum sections 0, MIN +max, MAX -max.
__global__ void table_init_kernel(int64_t* table, uint64_t G, int32_t nsec, DevParams p) {
  const uint64_t n = G * (uint64_t)nsec;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    table[i] = sec_identity(p.sec_op[i / G]);
}

// Reduce AGG-mode slabs (in block order: deterministic) into the G=1 table; reduce stats.
__global__ void finalize_kernel(DevParams p, int32_t nblocks, int64_t* stats_out) {
  const int s = threadIdx.x;
  if (p.mode == PGPU_MODE_AGG && s < p.nsec) {
    const int op = p.sec_op[s];
    int64_t v = sec_identity(op);
    for (int b = 0; b < nblocks; ++b) {
      const int64_t x = p.slab[(size_t)b * p.nsec + s];
      if (op == PGPU_RED_SUM_I64) v += x;
      else if (op == PGPU_RED_SUM_F64) v = __double_as_longlong(__longlong_as_double(v) + __longlong_as_double(x));
      else if (op == PGPU_RED_MIN_I64) v = x < v ? x : v;
      else v = x > v ? x : v;
    }
    p.table[s] = v;
  }
  if (s < PGPU_NSTATS) {
    int64_t v = 0;
    for (int b = 0; b < nblocks; ++b) v += p.stats[(size_t)b * PGPU_NSTATS + s];
    stats_out[s] = v;
  }
}

// ---- compaction of a dense table (keys with count > 0) ----------------------------------------------------
#define CMP_BLOCK 256
#define CMP_PER_BLOCK 4096

__global__ void compact_count_kernel(const int64_t* table, uint64_t G, int32_t* block_counts) {
  const uint64_t base = (uint64_t)blockIdx.x * CMP_PER_BLOCK;
  int c = 0;
  for (int i = threadIdx.x; i < CMP_PER_BLOCK; i += CMP_BLOCK) {
    const uint64_t k = base + i;
    if (k < G && table[k] > 0) ++c;
  }
  c = wave_sum_i32(c);
  __shared__ int ws[CMP_BLOCK / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < CMP_BLOCK / 64; ++w) t += ws[w];
    block_counts[blockIdx.x] = t;
  }
}

__global__ void compact_scan_kernel(int32_t* block_counts, int32_t nblocks, int64_t* total) {
  // single thread: nblocks <= a few 10^4
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    int64_t run = 0;
    for (int b = 0; b < nblocks; ++b) {
      const int32_t c = block_counts[b];
      block_counts[b] = (int32_t)run;
      run += c;
    }
    *total = run;
  }
}

__global__ void compact_write_kernel(const int64_t* table, uint64_t G, int32_t nsec, const int32_t* block_offsets,
                                     int64_t* out_keys, int64_t* out_cells) {
  const uint64_t base = (uint64_t)blockIdx.x * CMP_PER_BLOCK;
  __shared__ int wbase[CMP_BLOCK / 64 + 1];
  __shared__ int running;
  if (threadIdx.x == 0) running = block_offsets[blockIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i0 = 0; i0 < CMP_PER_BLOCK; i0 += CMP_BLOCK) {
    const uint64_t k = base + i0 + threadIdx.x;
    const bool f = k < G && table[k] > 0;
    const uint64_t bal = __ballot(f);
    const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    if (lane == 0) wbase[wave] = __popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) {
      int r = running;
      for (int w = 0; w < CMP_BLOCK / 64; ++w) { int c = wbase[w]; wbase[w] = r; r += c; }
      running = r;
    }
    __syncthreads();
    if (f) {
      const int pos = wbase[wave] + below;
      out_keys[pos] = (int64_t)k;
      for (int s = 0; s < nsec; ++s) out_cells[(size_t)pos * nsec + s] = table[(size_t)s * G + k];
    }
    __syncthreads();
  }
}

}  // namespace

// ---- host-side launch helpers (called by pgpu_runtime.cpp) ----------------------------------------------------
size_t pgpu_static_smem_bytes() { return sizeof(Smem); }

hipError_t pgpu_occupancy(int mode, size_t dyn_smem, int* blocks_per_cu) {
  switch (mode) {
    case PGPU_MODE_AGG:
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, query_kernel<PGPU_MODE_AGG>, NT, dyn_smem);
    case PGPU_MODE_LDS:
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, query_kernel<PGPU_MODE_LDS>, NT, dyn_smem);
    default:
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, query_kernel<PGPU_MODE_GLOBAL>, NT, dyn_smem);
  }
}

hipError_t pgpu_launch_table_init(const DevParams& p, hipStream_t st) {
  const uint64_t n = p.G * (uint64_t)p.nsec;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(table_init_kernel, dim3(blocks), dim3(256), 0, st, p.table, p.G, p.nsec, p);
  return hipGetLastError();
}

hipError_t pgpu_launch_query(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st) {
  switch (p.mode) {
    case PGPU_MODE_AGG:
      hipLaunchKernelGGL(query_kernel<PGPU_MODE_AGG>, dim3(grid), dim3(NT), dyn_smem, st, p);
      break;
    case PGPU_MODE_LDS:
      hipLaunchKernelGGL(query_kernel<PGPU_MODE_LDS>, dim3(grid), dim3(NT), dyn_smem, st, p);
      break;
    default:
      hipLaunchKernelGGL(query_kernel<PGPU_MODE_GLOBAL>, dim3(grid), dim3(NT), dyn_smem, st, p);
      break;
  }
  return hipGetLastError();
}

hipError_t pgpu_launch_finalize(const DevParams& p, int nblocks, int64_t* stats_out, hipStream_t st) {
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, st, p, nblocks, stats_out);
  return hipGetLastError();
}

hipError_t pgpu_launch_compact(const int64_t* table, uint64_t G, int32_t nsec, int32_t* block_counts,
                               int64_t* total, int64_t* out_keys, int64_t* out_cells, bool count_only,
                               hipStream_t st) {
  const int nb = (int)((G + CMP_PER_BLOCK - 1) / CMP_PER_BLOCK);
  if (count_only) {
    hipLaunchKernelGGL(compact_count_kernel, dim3(nb), dim3(CMP_BLOCK), 0, st, table, G, block_counts);
    hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(64), 0, st, block_counts, nb, total);
  } else {
    hipLaunchKernelGGL(compact_write_kernel, dim3(nb), dim3(CMP_BLOCK), 0, st, table, G, nsec, block_counts,
                       out_keys, out_cells);
  }
  return hipGetLastError();
}
