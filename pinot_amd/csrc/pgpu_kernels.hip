// HIP kernels of the MI355X segment query path (gfx950 / CDNA4).
//
// One launch runs a whole query over every segment a GPU owns.  Work unit = a WAVE TILE of 2048 consecutive docs
// of one segment; every wave of the persistent grid walks its own wave tiles independently (no workgroup barrier
// in the main loop), and inside a wave tile LANE l OWNS DOCS [32l, 32l+32): the 32*b bits of a lane are exactly b
// consecutive big-endian words of the FixedBitSVForwardIndexWriter stream, so a lane unpacks its 32 dict ids with
// compile-time shifts (one template instantiation per bit width) and every filter mask is one 32-bit word per lane.
//
//   K1  fixed-bit unpack fused with dict-id RANGE / SET / LIST predicates:
//         dense  — the lane's b words (the "driving" column of the filter is DMA'd into LDS one wave tile ahead
//                  with global_load_lds; other columns are loaded straight to VGPRs),
//         sparse — when the docs that still matter are < 1/32 of the tile, only those docs gather their two
//                  words (32-B-sector-granular traffic).
//   K2  Roaring array / bitmap / run containers (BitmapBasedFilterOperator), sorted-index doc ranges, and the
//       AND / OR / NOT algebra on the per-lane mask words (short-circuit of AND when a wave tile empties).
//   K3  COUNT / SUM / MIN / MAX / AVG: per-lane register accumulators + wave reduction (aggregation only), or
//       group keys (mixed-radix global dict ids) with atomics into an LDS-privatised dense table (small key
//       spaces) or the HBM dense table (large key spaces).
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

#define NT PGPU_BLOCK
#define NW PGPU_WAVES
#define WT PGPU_WAVE_TILE  // 2048 docs per wave tile
#define MAXS PGPU_MAX_SLOTS

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Loads through the global address space: segment pointers reach the kernel inside structs in HBM, so the
// compiler only sees generic pointers and would emit flat_* (which also count against lgkmcnt and stall LDS).
#define GAS __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ T gld(const T* p, size_t i) { return ((const GAS T*)p)[i]; }
__device__ __forceinline__ uint32_t lowmask(uint32_t b) { return 0xFFFFFFFFu >> (32u - b); }
// Bit i of a lane mask word as v_bfe_u32 with inline operands (a `1u << i` test makes the compiler keep 32
// materialised constants live in VGPRs across the unrolled doc loops).
__device__ __forceinline__ uint32_t lane_bit(uint32_t m, int i) { return __builtin_amdgcn_ubfe(m, (uint32_t)i, 1u); }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
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
// Wave-uniform total (readfirstlane: callers branch on it as a scalar).
__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return __builtin_amdgcn_readfirstlane(v);
}

// Order-preserving int64 key of a dictionary value (MIN/MAX sections).
__device__ __forceinline__ int64_t minmax_key(const void* dict, int32_t vtype, uint32_t id) {
  switch (vtype) {
    case PGPU_INT: return (int64_t)gld((const int32_t*)dict, id);
    case PGPU_LONG: return gld((const int64_t*)dict, id);
    case PGPU_FLOAT: {
      int64_t b = __double_as_longlong((double)gld((const float*)dict, id));
      return b >= 0 ? b : (b ^ 0x7FFFFFFFFFFFFFFFll);
    }
    default: {
      int64_t b = __double_as_longlong(gld((const double*)dict, id));
      return b >= 0 ? b : (b ^ 0x7FFFFFFFFFFFFFFFll);
    }
  }
}
__device__ __forceinline__ int64_t value_i64(const void* dict, int32_t vtype, uint32_t id) {
  return vtype == PGPU_INT ? (int64_t)gld((const int32_t*)dict, id) : gld((const int64_t*)dict, id);
}
__device__ __forceinline__ double value_f64(const void* dict, int32_t vtype, uint32_t id) {
  return vtype == PGPU_FLOAT ? (double)gld((const float*)dict, id) : gld((const double*)dict, id);
}
__device__ __forceinline__ int64_t sec_identity(int32_t op) {
  return op == PGPU_RED_MIN_I64 ? INT64_MAX : (op == PGPU_RED_MAX_I64 ? INT64_MIN : 0);
}

// ---- per-wave LDS carve ----------------------------------------------------------------------------------------
// dynamic LDS of a workgroup: [NW][MAXS][64] slot words | [NW][pf_words] driving-column buffers |
//                             [NW][MAX_AGGS] int64 accumulators | LDS group table [nsec][G] (mode LDS)
struct Carve {
  uint32_t* slots;   // this wave's [MAXS][64]
  uint32_t* pf;      // this wave's driving-column buffer (pf_words)
  int64_t* accw;     // this wave's [MAX_AGGS]
  int64_t* ltab;     // workgroup table
  bool* pf_have;     // a DMA into pf is in flight
  int pf_words;
};

__device__ __forceinline__ uint32_t& slot(const Carve& cv, int s) { return cv.slots[s * 64 + (threadIdx.x & 63)]; }

struct WTile {
  const DevSeg* seg;
  const DevColumn* cols;
  int32_t tile_in_seg;
  int32_t doc0;      // first doc of the wave tile (segment-local)
  int32_t ndocs;     // docs of the wave tile inside the segment (1..2048)
  uint32_t valid;    // this lane's valid-doc word
  int32_t lane_doc0; // doc0 + 32 * lane
};

// ---- fixed-bit extraction (compile-time bit width) -------------------------------------------------------------
// w[] = the lane's B words, byte-swapped (MSB-first bit order); value i occupies bits [i*B, (i+1)*B).
template <int B>
__device__ __forceinline__ uint32_t extract_c(const uint32_t (&w)[B], int i) {
  const int o = i * B;
  const int k = o >> 5, sh = o & 31;
  if (sh + B <= 32) return (w[k] >> (32 - sh - B)) & lowmask(B);
  return __builtin_amdgcn_alignbit(w[k], w[k + 1], 64 - sh - B) & lowmask(B);
}

// This lane's index, opaque to loop-invariant code motion: the per-bit-width lane offsets (lane * B for 31
// widths) would otherwise be hoisted out of the tile loop and pin ~30 VGPRs for the kernel's lifetime.
__device__ __forceinline__ uint32_t opaque_lane() {
  uint32_t l;
  asm volatile("v_and_b32 %0, 63, %1" : "=v"(l) : "v"(threadIdx.x));
  return l;
}

// The lane's B words of column `fwd` in wave tile `tile_in_seg`, straight from HBM (byte-swapped).
template <int B>
__device__ __forceinline__ void load_lane_words(const uint32_t* __restrict__ fwd, int tile_in_seg, uint32_t (&w)[B]) {
  const GAS uint32_t* src = (const GAS uint32_t*)fwd + ((size_t)tile_in_seg * 64 + opaque_lane()) * B;
  if constexpr (B % 4 == 0) {
#pragma unroll
    for (int k = 0; k < B; k += 4) {
      const u32x4 v = *(const GAS u32x4*)(src + k);
      w[k] = v.x; w[k + 1] = v.y; w[k + 2] = v.z; w[k + 3] = v.w;
    }
  } else if constexpr (B % 2 == 0) {
#pragma unroll
    for (int k = 0; k < B; k += 2) {
      const u32x2 v = *(const GAS u32x2*)(src + k);
      w[k] = v.x; w[k + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < B; ++k) w[k] = src[k];
  }
#pragma unroll
  for (int k = 0; k < B; ++k) w[k] = bswap32(w[k]);
}

// The lane's B words from the LDS copy of the wave tile (linear stream order, raw big-endian).
template <int B>
__device__ __forceinline__ void lds_lane_words(const uint32_t* buf, uint32_t (&w)[B]) {
  const uint32_t* src = buf + opaque_lane() * B;
#pragma unroll
  for (int k = 0; k < B; ++k) w[k] = bswap32(src[k]);
}

// ---- fixed-bit decode: ONE inlined dispatch site per source keeps the 31 bit-width variants out of every consumer
template <int B>
__device__ __forceinline__ void unpack_b(const uint32_t (&w)[B], uint32_t (&ids)[32]) {
#pragma unroll
  for (int i = 0; i < 32; ++i) ids[i] = extract_c<B>(w, i);
}
template <int B>
__device__ __forceinline__ void decode_hbm_b(const uint32_t* fwd, int tile_in_seg, uint32_t (&ids)[32]) {
  uint32_t w[B];
  load_lane_words<B>(fwd, tile_in_seg, w);
  unpack_b<B>(w, ids);
}
template <int B>
__device__ __forceinline__ void decode_lds_b(const uint32_t* buf, uint32_t (&ids)[32]) {
  uint32_t w[B];
  lds_lane_words<B>(buf, w);
  unpack_b<B>(w, ids);
}

#define PGPU_DISPATCH_B(b, CALL)                                                                     \
  switch (b) {                                                                                       \
    case 1: CALL(1); break;   case 2: CALL(2); break;   case 3: CALL(3); break;   case 4: CALL(4); break;   \
    case 5: CALL(5); break;   case 6: CALL(6); break;   case 7: CALL(7); break;   case 8: CALL(8); break;   \
    case 9: CALL(9); break;   case 10: CALL(10); break; case 11: CALL(11); break; case 12: CALL(12); break; \
    case 13: CALL(13); break; case 14: CALL(14); break; case 15: CALL(15); break; case 16: CALL(16); break; \
    case 17: CALL(17); break; case 18: CALL(18); break; case 19: CALL(19); break; case 20: CALL(20); break; \
    case 21: CALL(21); break; case 22: CALL(22); break; case 23: CALL(23); break; case 24: CALL(24); break; \
    case 25: CALL(25); break; case 26: CALL(26); break; case 27: CALL(27); break; case 28: CALL(28); break; \
    case 29: CALL(29); break; case 30: CALL(30); break; default: CALL(31); break;                   \
  }

// The lane's 32 dict ids of column c in the wave tile, from HBM.
__device__ __forceinline__ void decode_hbm(const DevColumn& c, int tile_in_seg, uint32_t (&ids)[32]) {
#define DEC_CALL(B) decode_hbm_b<B>(c.fwd, tile_in_seg, ids)
  PGPU_DISPATCH_B(c.bits, DEC_CALL)
#undef DEC_CALL
}
// ... from the LDS copy of the wave tile (the prefetched driving column).
__device__ __forceinline__ void decode_lds(int bits, const uint32_t* buf, uint32_t (&ids)[32]) {
#define DEC_CALL(B) decode_lds_b<B>(buf, ids)
  PGPU_DISPATCH_B(bits, DEC_CALL)
#undef DEC_CALL
}

// ---- predicates -----------------------------------------------------------------------------------------------
#define PRED_RANGE 0
#define PRED_SET 1   // bitset over dict ids in the pool
#define PRED_LIST 2  // up to 8 ids in the pool

struct Pred {
  int kind;
  uint32_t lo, span;         // RANGE: (id - lo) < span
  const uint32_t* bits;      // SET
  uint32_t ids[8];           // LIST
  bool negate;
};

__device__ __forceinline__ Pred make_pred(const DevInstr& in, const int32_t* pool) {
  Pred p;
  p.kind = in.pred;
  p.negate = in.negate != 0;
  p.lo = (uint32_t)in.lo;
  p.span = (uint32_t)(in.hi - in.lo);
  p.bits = (const uint32_t*)(pool + in.pool_off);
#pragma unroll
  for (int k = 0; k < 8; ++k) p.ids[k] = (p.kind == PRED_LIST && k < in.n) ? (uint32_t)pool[in.pool_off + k] : 0xFFFFFFFFu;
  return p;
}

__device__ __forceinline__ bool eval_pred(const Pred& p, uint32_t id) {
  bool m;
  if (p.kind == PRED_RANGE) {
    m = (id - p.lo) < p.span;
  } else if (p.kind == PRED_LIST) {
    m = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) m |= id == p.ids[k];
  } else {
    m = (gld(p.bits, id >> 5) >> (id & 31)) & 1u;
  }
  return m != p.negate;
}

// The lane's 32 predicate bits for its decoded ids.
__device__ __forceinline__ uint32_t pred_ids(const uint32_t (&ids)[32], const Pred& p) {
  // bits are shifted in from doc 31 down to doc 0 (v_lshl_or with inline operands)
  uint32_t m = 0;
  if (p.kind == PRED_RANGE) {
#pragma unroll
    for (int i = 31; i >= 0; --i) m = (m << 1) | (uint32_t)((ids[i] - p.lo) < p.span);
  } else if (p.kind == PRED_LIST) {
#pragma unroll
    for (int i = 31; i >= 0; --i) {
      bool h = false;
#pragma unroll
      for (int k = 0; k < 8; ++k) h |= ids[i] == p.ids[k];
      m = (m << 1) | (uint32_t)h;
    }
  } else {
#pragma unroll
    for (int i = 31; i >= 0; --i) m = (m << 1) | ((gld(p.bits, ids[i] >> 5) >> (ids[i] & 31)) & 1u);
  }
  return p.negate ? ~m : m;
}

// ---- sparse access --------------------------------------------------------------------------------------------
// SortedIndexReaderImpl.getDictId: last dict id whose start <= doc.
__device__ __forceinline__ uint32_t sorted_dict_id(const int32_t* __restrict__ pairs, int32_t card, int32_t doc) {
  int32_t lo = 0, hi = card - 1;
  while (lo <= hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (gld(pairs, 2 * (size_t)mid) <= doc) lo = mid + 1; else hi = mid - 1;
  }
  return (uint32_t)hi;
}

// Dict id of segment doc `d` gathered from HBM (two big-endian words around its bits).
__device__ __forceinline__ uint32_t gather_id(const DevColumn& c, int32_t d) {
  if (c.kind == PGPU_COL_SORTED) return sorted_dict_id(c.sorted, c.card, d);
  const uint32_t b = (uint32_t)c.bits;
  const uint64_t e = (uint64_t)(d + 1) * b;
  const uint64_t we = (e - 1u) >> 5;
  const uint32_t r = (uint32_t)(e - (we << 5));
  const uint32_t hi = bswap32(gld(c.fwd, we));
  const uint32_t lo = we ? bswap32(gld(c.fwd, we - 1)) : 0u;
  return __builtin_amdgcn_alignbit(lo, hi, 32u - r) & lowmask(b);
}

__device__ __forceinline__ void mark_sectors(uint32_t* sect, uint32_t j, uint32_t b) {
  const uint32_t s0 = (j * b) >> 8, s1 = ((j + 1) * b - 1) >> 8;  // 32-B sector = 256 bits
  atomicOr(&sect[s0 >> 5], 1u << (s0 & 31));
  if (s1 != s0) atomicOr(&sect[s1 >> 5], 1u << (s1 & 31));
}

// Sparse scan: predicate bits for the docs of `care` only, two candidates per round trip.
__device__ __forceinline__ uint32_t scan_sparse(const DevColumn& c, const WTile& t, const Pred& p, uint32_t care,
                                                uint32_t* sect) {
  uint32_t m = 0, left = care;
  const uint32_t jbase = (uint32_t)(t.lane_doc0 - t.doc0);
  while (__ballot(left != 0)) {
    const bool h0 = left != 0;
    const int i0 = h0 ? __builtin_ctz(left) : 0;
    left &= left - 1;
    const bool h1 = left != 0;
    const int i1 = h1 ? __builtin_ctz(left) : 0;
    left &= left - 1;
    uint32_t id0 = 0, id1 = 0;
    if (h0) id0 = gather_id(c, t.lane_doc0 + i0);
    if (h1) id1 = gather_id(c, t.lane_doc0 + i1);
    if (h0 && eval_pred(p, id0)) m |= 1u << i0;
    if (h1 && eval_pred(p, id1)) m |= 1u << i1;
    if (sect) {
      if (h0) mark_sectors(sect, jbase + i0, (uint32_t)c.bits);
      if (h1) mark_sectors(sect, jbase + i1, (uint32_t)c.bits);
    }
  }
  return m;
}

// ---- Roaring containers / sorted ranges ---------------------------------------------------------------------------
// Bits of the wave tile covered by one Roaring bitmap (dict id `id`), for this lane's 32 docs.
__device__ __noinline__ uint32_t bitmap_word(const DevColumn& c, const WTile& t, uint32_t id, uint32_t* lds_words) {
  const uint32_t key = (uint32_t)t.doc0 >> 16;
  const uint32_t lo16 = (uint32_t)t.doc0 & 0xFFFFu;  // multiple of 2048
  const int lane = threadIdx.x & 63;
  int32_t a = (int32_t)c.inv_dir[id], z = (int32_t)c.inv_dir[id + 1] - 1;
  int32_t ci = -1;
  while (a <= z) {
    const int32_t mid = (a + z) >> 1;
    const uint32_t k = c.inv_ct[mid].key;
    if (k == key) { ci = mid; break; }
    if (k < key) a = mid + 1; else z = mid - 1;
  }
  if (ci < 0) return 0u;
  const DevContainer ct = c.inv_ct[ci];
  const uint32_t my0 = lo16 + 32u * lane;  // my first doc within the container
  if (ct.type == PGPU_CT_BITMAP) {
    return ((const uint32_t*)(c.inv_data + ct.offset))[my0 >> 5];
  }
  if (ct.type == PGPU_CT_RUN) {
    const uint16_t* r = (const uint16_t*)(c.inv_data + ct.offset);
    int32_t l = 0, h = (int32_t)ct.card;
    while (l < h) {  // first run whose end >= lo16
      const int32_t m = (l + h) >> 1;
      if ((uint32_t)r[2 * m] + r[2 * m + 1] < lo16) l = m + 1; else h = m;
    }
    uint32_t w = 0;
    for (int32_t i = l; i < (int32_t)ct.card; ++i) {  // uniform loop over the runs overlapping the tile
      const uint32_t s = r[2 * i], e = s + r[2 * i + 1];
      if (s >= lo16 + WT) break;
      if (e >= my0 && s <= my0 + 31) {
        const uint32_t bs = s > my0 ? s - my0 : 0u, be = e < my0 + 31 ? e - my0 : 31u;
        w |= (0xFFFFFFFFu >> (31 - be)) & (0xFFFFFFFFu << bs);
      }
    }
    return w;
  }
  // ARRAY: values in [lo16, lo16 + WT) scattered to their owner lanes through LDS
  const uint16_t* v = (const uint16_t*)(c.inv_data + ct.offset);
  int32_t l = 0, h = (int32_t)ct.card;
  while (l < h) { const int32_t m = (l + h) >> 1; if (v[m] < lo16) l = m + 1; else h = m; }
  const int32_t first = l;
  h = (int32_t)ct.card;
  while (l < h) { const int32_t m = (l + h) >> 1; if ((uint32_t)v[m] < lo16 + WT) l = m + 1; else h = m; }
  lds_words[lane] = 0u;
  wave_sync();
  for (int32_t i = first + lane; i < l; i += 64) {
    const uint32_t off = (uint32_t)v[i] - lo16;
    atomicOr(&lds_words[off >> 5], 1u << (off & 31));
  }
  wave_sync();
  const uint32_t w = lds_words[lane];
  wave_sync();
  return w;
}

__device__ __noinline__ uint32_t sorted_ranges_word(const int32_t* rg, int n, const WTile& t) {
  const int32_t d0 = t.lane_doc0, d1 = d0 + 31;
  const int32_t w0 = t.doc0, w1 = t.doc0 + WT - 1;
  int32_t l = 0, h = n;
  while (l < h) { const int32_t m = (l + h) >> 1; if (rg[2 * m + 1] < w0) l = m + 1; else h = m; }
  uint32_t w = 0;
  for (int32_t i = l; i < n; ++i) {  // uniform over the ranges overlapping the wave tile
    const int32_t s = rg[2 * i], e = rg[2 * i + 1];
    if (s > w1) break;
    if (e >= d0 && s <= d1) {
      const int32_t bs = s > d0 ? s - d0 : 0, be = e < d1 ? e - d0 : 31;
      w |= (0xFFFFFFFFu >> (31 - be)) & (0xFFFFFFFFu << bs);
    }
  }
  return w;
}

// ---- driving-column prefetch (LDS DMA one wave tile ahead) ---------------------------------------------------------
__device__ __forceinline__ int seg_of_tile(const DevParams& p, int tile) {
  int lo = 0, hi = p.nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (p.segs[mid].tile_begin <= tile) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Issue global_load_lds (16 B per lane, 1 KiB per instruction) of the driving column of wave tile `tile` into
// `buf`; returns false when that tile's segment has no driving column.  The caller has finished reading `buf`.
__device__ __forceinline__ bool prefetch_tile(const DevParams& p, int tile, uint32_t* buf) {
  if (tile >= p.total_tiles) return false;
  const DevSeg& sg = p.segs[seg_of_tile(p, tile)];
  if (sg.pf_pc < 0) return false;
  const DevInstr& in = p.instrs[sg.prog_begin + sg.pf_pc];
  const DevColumn& c = p.cols[sg.col_begin + in.col];
  const int b = c.bits;
  const char* src = (const char*)(c.fwd + (size_t)(tile - sg.tile_begin) * 64 * b);
  const int lane = threadIdx.x & 63;
  const int chunks = (b + 3) >> 2;  // 1 KiB chunks of the 256*b-byte wave tile (last one may be partial)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // earlier LDS reads of buf are complete (WAR)
  for (int k = 0; k < chunks; ++k) {
    const int byte = k * 1024 + lane * 16;
    if (byte < 256 * b) {
      __builtin_amdgcn_global_load_lds((const void*)(src + byte),
                                       (__attribute__((address_space(3))) void*)(buf + k * 256), 16, 0, 0);
    }
  }
  return true;
}

// ---- filter program ------------------------------------------------------------------------------------------------
// Returns this lane's match word for the wave tile.  The driving column (instruction pf_pc) of this tile is in
// cv.pf; once it is decoded the DMA of the next tile (`next_tile`) is issued into the same buffer (*pf_issued).
__device__ __forceinline__ uint32_t run_filter(const DevParams& p, const Carve& cv, const WTile& t, int next_tile,
                                               bool* pf_issued, uint32_t* scratch_words, int64_t& scanned,
                                               int64_t& sector_bytes, int64_t& dense_bytes) {
  const DevSeg& s = *t.seg;
  if (s.prog_len == 0) return t.valid;
  const bool stats = p.flags & PGPU_FLAG_STATS;
  const int lane = threadIdx.x & 63;
  int pc = 0;
  while (pc < s.prog_len) {
    const DevInstr in = p.instrs[s.prog_begin + pc];
    int next = pc + 1;
    const uint32_t care = in.care < 0 ? t.valid : slot(cv, in.care);
    switch (in.op) {
      case PGPU_I_ALL: slot(cv, in.dst) = t.valid; break;
      case PGPU_I_EMPTY: slot(cv, in.dst) = 0u; break;
      case PGPU_I_SCAN: {
        const DevColumn& c = t.cols[in.col];
        const Pred pr = make_pred(in, p.pool);
        const bool prestaged = pc == s.pf_pc;
        int ncare = 0;
        if (!prestaged) ncare = wave_sum_i32(__popc(care));
        const bool dense = prestaged || (c.kind == PGPU_COL_FIXED_BIT && ncare * 32 >= t.ndocs);
        uint32_t m;
        if (dense) {
          uint32_t ids[32];
          if (prestaged) {
            decode_lds(c.bits, cv.pf, ids);
            *pf_issued = true;
            cv.pf_have[0] = prefetch_tile(p, next_tile, cv.pf);
          } else {
            decode_hbm(c, t.tile_in_seg, ids);
          }
          m = pred_ids(ids, pr) & t.valid;
          if (lane == 0) {
            scanned += t.ndocs;
            dense_bytes += ((int64_t)t.ndocs * c.bits + 7) / 8;
          }
        } else {
          uint32_t* sect = nullptr;
          if (stats && c.kind == PGPU_COL_FIXED_BIT) {
            sect = scratch_words;
            scratch_words[lane] = 0u;  // 64 words = 2048 sectors >= 2048 docs * 31 bits / 256
            wave_sync();
          }
          m = scan_sparse(c, t, pr, care, sect);
          if (sect) {
            wave_sync();
            const int cnt = wave_sum_i32(__popc(scratch_words[lane]));
            if (lane == 0) sector_bytes += 32ll * cnt;
            wave_sync();
          }
          if (lane == 0) scanned += ncare;
        }
        slot(cv, in.dst) = m & care;
        break;
      }
      case PGPU_I_INV: {
        const DevColumn& c = t.cols[in.col];
        uint32_t m = 0;
        for (int i = 0; i < in.n; ++i) m |= bitmap_word(c, t, (uint32_t)p.pool[in.pool_off + i], scratch_words);
        if (in.negate) m = ~m;
        slot(cv, in.dst) = m & t.valid;
        break;
      }
      case PGPU_I_SORTED: {
        uint32_t m = sorted_ranges_word(p.pool + in.pool_off, in.n, t);
        if (in.negate) m = ~m;
        slot(cv, in.dst) = m & t.valid;
        break;
      }
      case PGPU_I_AND_BEGIN: slot(cv, in.dst) = care; break;
      case PGPU_I_AND_CHILD: {
        const uint32_t a = slot(cv, in.dst) & slot(cv, in.src);
        slot(cv, in.dst) = a;
        if (!__ballot(a != 0u)) next = in.jump;
        break;
      }
      case PGPU_I_OR_BEGIN: slot(cv, in.dst) = 0u; break;
      case PGPU_I_OR_CHILD: slot(cv, in.dst) |= slot(cv, in.src); break;
      case PGPU_I_NOT: slot(cv, in.dst) = ~slot(cv, in.src) & care; break;
      default: break;  // AND_END / OR_END
    }
    pc = next;
  }
  return slot(cv, 0);
}

// ---- aggregation ---------------------------------------------------------------------------------------------------
struct Acc {
  int64_t i;
  double d;
};

__device__ __forceinline__ void acc_add(Acc& a, const DevAgg& ag, const DevColumn& c, uint32_t id) {
  if (ag.op == PGPU_RED_SUM_I64) a.i += value_i64(c.dict, ag.vtype, id);
  else if (ag.op == PGPU_RED_SUM_F64) a.d += value_f64(c.dict, ag.vtype, id);
  else {
    const int64_t k = minmax_key(c.dict, ag.vtype, id);
    a.i = ag.op == PGPU_RED_MIN_I64 ? (k < a.i ? k : a.i) : (k > a.i ? k : a.i);
  }
}

// table update for one doc: `tab` = LDS or HBM dense table, section-major
__device__ __forceinline__ void table_update(int64_t* tab, uint64_t G, const DevAgg& ag, const DevColumn& c,
                                             uint32_t key, uint32_t id) {
  int64_t* cell = tab + (size_t)ag.sec * G + key;
  if (ag.op == PGPU_RED_SUM_I64) atomicAdd((unsigned long long*)cell, (unsigned long long)value_i64(c.dict, ag.vtype, id));
  else if (ag.op == PGPU_RED_SUM_F64) atomicAdd((double*)cell, value_f64(c.dict, ag.vtype, id));
  else if (ag.op == PGPU_RED_MIN_I64) atomicMin((long long*)cell, (long long)minmax_key(c.dict, ag.vtype, id));
  else atomicMax((long long*)cell, (long long)minmax_key(c.dict, ag.vtype, id));
}

// ---- the query kernel ----------------------------------------------------------------------------------------------
template <int MODE>
// amdgpu_waves_per_eu(4): 128 VGPRs -> 4 waves per SIMD (16 per CU) to keep enough sparse gathers in flight
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4, 8))) void query_kernel(DevParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  // the wave index through readfirstlane: everything derived from it (tile, segment, program, columns, bit
  // widths) is then provably wave-uniform and lives in SGPRs, and the bit-width switch is a scalar branch
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  Carve cv;
  {
    unsigned char* base = dyn_smem;
    cv.slots = (uint32_t*)base + wave * MAXS * 64;
    base += NW * MAXS * 64 * 4;
    cv.pf_words = p.pf_words;
    cv.pf = (uint32_t*)base + wave * (size_t)p.pf_words;
    base += NW * (size_t)p.pf_words * 4;
    cv.accw = (int64_t*)base + wave * PGPU_MAX_AGGS;
    base += NW * PGPU_MAX_AGGS * 8;
    cv.ltab = (int64_t*)base;
  }
  uint32_t* scratch = cv.slots + (MAXS - 1) * 64;  // the last slot row doubles as per-wave LDS scratch
  if (MODE == PGPU_MODE_LDS) {
    const int n = p.nsec * (int)p.G;
    for (int i = threadIdx.x; i < n; i += NT) cv.ltab[i] = sec_identity(p.sec_op[i / (int)p.G]);
  }
  if (MODE == PGPU_MODE_AGG && lane < PGPU_MAX_AGGS) cv.accw[lane] = lane < p.nagg ? sec_identity(p.aggs[lane].op) : 0;
  __syncthreads();

  int64_t matched = 0, scanned = 0, sector_bytes = 0, dense_bytes = 0;  // lane 0 of each wave owns these
  const int gw = blockIdx.x * NW + wave, nwaves = gridDim.x * NW;
  bool have[1];
  cv.pf_have = have;
  have[0] = prefetch_tile(p, gw, cv.pf);
  for (int tile = gw; tile < p.total_tiles; tile += nwaves) {
    const int sidx = seg_of_tile(p, tile);
    WTile t;
    t.seg = &p.segs[sidx];
    t.cols = p.cols + t.seg->col_begin;
    t.tile_in_seg = tile - t.seg->tile_begin;
    t.doc0 = t.tile_in_seg * WT;
    t.ndocs = min(WT, t.seg->num_docs - t.doc0);
    t.lane_doc0 = t.doc0 + 32 * lane;
    {
      const int rem = t.ndocs - 32 * lane;
      t.valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
    }
    // this tile's driving column has landed in cv.pf (issued one tile ago)
    if (have[0]) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    bool issued = false;
    const uint32_t mm = run_filter(p, cv, t, tile + nwaves, &issued, scratch, scanned, sector_bytes, dense_bytes);
    if (!issued) have[0] = prefetch_tile(p, tile + nwaves, cv.pf);
    const int nm = wave_sum_i32(__popc(mm));
    if (lane == 0) matched += nm;
    if (nm == 0) continue;  // uniform
    const bool dense_post = nm * 32 >= t.ndocs;

    if (MODE == PGPU_MODE_AGG) {
      for (int a = 0; a < p.nagg; ++a) {
        const DevAgg ag = p.aggs[a];
        if (ag.fn == PGPU_AGG_COUNT) continue;
        const DevColumn& c = t.cols[ag.col];
        Acc acc;
        acc.i = sec_identity(ag.op);
        acc.d = 0.0;
        if (dense_post && c.kind == PGPU_COL_FIXED_BIT) {
          uint32_t ids[32];
          decode_hbm(c, t.tile_in_seg, ids);
#pragma unroll
          for (int i = 0; i < 32; ++i)
            if (lane_bit(mm, i)) acc_add(acc, ag, c, ids[i]);
        } else {
          for (uint32_t left = mm; left; left &= left - 1)
            acc_add(acc, ag, c, gather_id(c, t.lane_doc0 + __builtin_ctz(left)));
        }
        if (ag.op == PGPU_RED_SUM_I64) acc.i = wave_sum_i64(acc.i);
        else if (ag.op == PGPU_RED_SUM_F64) acc.d = wave_sum_f64(acc.d);
        else if (ag.op == PGPU_RED_MIN_I64) acc.i = wave_min_i64(acc.i);
        else acc.i = wave_max_i64(acc.i);
        if (lane == 0) {
          int64_t& cell = cv.accw[a];
          if (ag.op == PGPU_RED_SUM_I64) cell += acc.i;
          else if (ag.op == PGPU_RED_SUM_F64) cell = __double_as_longlong(__longlong_as_double(cell) + acc.d);
          else if (ag.op == PGPU_RED_MIN_I64) cell = acc.i < cell ? acc.i : cell;
          else cell = acc.i > cell ? acc.i : cell;
        }
      }
    } else {
      int64_t* tab = MODE == PGPU_MODE_LDS ? cv.ltab : p.table;
      bool all_fixed = true;
      for (int gc = 0; gc < p.ngcols; ++gc) all_fixed &= t.cols[p.gcols[gc]].kind == PGPU_COL_FIXED_BIT;
      for (int a = 0; a < p.nagg; ++a)
        if (p.aggs[a].fn != PGPU_AGG_COUNT) all_fixed &= t.cols[p.aggs[a].col].kind == PGPU_COL_FIXED_BIT;
      if (dense_post && all_fixed) {
        // one pass over [group columns..., aggregations...]: a single decode site for all of them
        uint32_t key[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) key[i] = 0u;
        const int nops = p.ngcols + (p.nagg > 0 ? p.nagg : 1);
        for (int op = 0; op < nops; ++op) {
          if (op == p.ngcols) {
#pragma unroll
            for (int i = 0; i < 32; ++i)
              if (lane_bit(mm, i)) atomicAdd((unsigned long long*)&tab[key[i]], 1ull);
          }
          const bool is_key = op < p.ngcols;
          DevAgg ag;
          int col;
          if (is_key) {
            col = p.gcols[op];
          } else {
            if (op - p.ngcols >= p.nagg) break;
            ag = p.aggs[op - p.ngcols];
            if (ag.fn == PGPU_AGG_COUNT) continue;
            col = ag.col;
          }
          const DevColumn& c = t.cols[col];
          uint32_t ids[32];
          decode_hbm(c, t.tile_in_seg, ids);
          if (is_key) {
            const int32_t* remap = p.remaps[t.seg->remap_begin + op];
            const uint32_t stride = p.gstride[op];
#pragma unroll
            for (int i = 0; i < 32; ++i)
              if (lane_bit(mm, i)) key[i] += (remap ? (uint32_t)gld(remap, ids[i]) : ids[i]) * stride;
          } else {
#pragma unroll
            for (int i = 0; i < 32; ++i)
              if (lane_bit(mm, i)) table_update(tab, p.G, ag, c, key[i], ids[i]);
          }
        }
      } else {
        for (uint32_t left = mm; __ballot(left != 0); left &= left - 1) {
          if (!left) continue;
          const int32_t d = t.lane_doc0 + __builtin_ctz(left);
          uint32_t key = 0;
          for (int gc = 0; gc < p.ngcols; ++gc) {
            const DevColumn& c = t.cols[p.gcols[gc]];
            const int32_t* remap = p.remaps[t.seg->remap_begin + gc];
            const uint32_t id = gather_id(c, d);
            key += (remap ? (uint32_t)gld(remap, id) : id) * p.gstride[gc];
          }
          atomicAdd((unsigned long long*)&tab[key], 1ull);
          for (int a = 0; a < p.nagg; ++a) {
            const DevAgg ag = p.aggs[a];
            if (ag.fn == PGPU_AGG_COUNT) continue;
            const DevColumn& c = t.cols[ag.col];
            table_update(tab, p.G, ag, c, key, gather_id(c, d));
          }
        }
      }
    }
  }
  if (have[0]) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue ----
  if (lane == 0) {
    int64_t* st = p.stats + (size_t)(blockIdx.x * NW + wave) * PGPU_NSTATS;
    st[PGPU_STAT_MATCHED] = matched;
    st[PGPU_STAT_SCANNED] = scanned;
    st[PGPU_STAT_SECTOR_BYTES] = sector_bytes;
    st[PGPU_STAT_DENSE_BYTES] = dense_bytes;
  }
  if (MODE == PGPU_MODE_AGG) {
    // slab[wave][sec]: section 0 = matched count; reduced in wave order by finalize_kernel (deterministic)
    int64_t* slab = p.slab + (size_t)(blockIdx.x * NW + wave) * p.nsec;
    if (lane == 0) slab[0] = matched;
    if (lane < p.nagg && p.aggs[lane].fn != PGPU_AGG_COUNT) slab[p.aggs[lane].sec] = cv.accw[lane];
  } else if (MODE == PGPU_MODE_LDS) {
    __syncthreads();
    const int G = (int)p.G;
    for (int key = threadIdx.x; key < G; key += NT) {
      const int64_t cnt = cv.ltab[key];
      if (cnt == 0) continue;
      atomicAdd((unsigned long long*)&p.table[key], (unsigned long long)cnt);
      for (int s = 1; s < p.nsec; ++s) {
        const int64_t v = cv.ltab[s * G + key];
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
}

// Table init: count/sum sections 0, MIN +max, MAX -max.
__global__ void table_init_kernel(int64_t* table, uint64_t G, int32_t nsec, DevParams p) {
  const uint64_t n = G * (uint64_t)nsec;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    table[i] = sec_identity(p.sec_op[i / G]);
}

// Reduce AGG-mode slabs into the G=1 table and the per-wave stats: block x reduces column x (a section, then the
// PGPU_NSTATS stats) over all waves with a fixed-shape tree, so double sums are deterministic.
__global__ __launch_bounds__(256) void finalize_kernel(DevParams p, int32_t nslabs, int64_t* stats_out) {
  __shared__ int64_t red[256];
  const int col = blockIdx.x;
  const bool is_stat = col >= p.nsec;
  if (!is_stat && p.mode != PGPU_MODE_AGG) return;
  const int op = is_stat ? PGPU_RED_SUM_I64 : p.sec_op[col];
  const int64_t* src = is_stat ? p.stats + (col - p.nsec) : p.slab + col;
  const int stride = is_stat ? PGPU_NSTATS : p.nsec;
  int64_t v = sec_identity(op);
  for (int b = threadIdx.x; b < nslabs; b += 256) {
    const int64_t x = src[(size_t)b * stride];
    if (op == PGPU_RED_SUM_I64) v += x;
    else if (op == PGPU_RED_SUM_F64) v = __double_as_longlong(__longlong_as_double(v) + __longlong_as_double(x));
    else if (op == PGPU_RED_MIN_I64) v = x < v ? x : v;
    else v = x > v ? x : v;
  }
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const int64_t x = red[threadIdx.x + o];
      int64_t y = red[threadIdx.x];
      if (op == PGPU_RED_SUM_I64) y += x;
      else if (op == PGPU_RED_SUM_F64) y = __double_as_longlong(__longlong_as_double(y) + __longlong_as_double(x));
      else if (op == PGPU_RED_MIN_I64) y = x < y ? x : y;
      else y = x > y ? x : y;
      red[threadIdx.x] = y;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (is_stat) stats_out[col - p.nsec] = red[0];
    else p.table[col] = red[0];
  }
}

// ---- compaction of a dense table (keys with count > 0) -------------------------------------------------------------
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

// ---- host-side launch helpers (called by pgpu_runtime.cpp) --------------------------------------------------------
size_t pgpu_dyn_smem_bytes(int mode, int pf_words, uint64_t table_bytes) {
  size_t n = (size_t)NW * MAXS * 64 * 4 + (size_t)NW * pf_words * 4 + (size_t)NW * PGPU_MAX_AGGS * 8;
  if (mode == PGPU_MODE_LDS) n += table_bytes;
  return n;
}

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

hipError_t pgpu_launch_finalize(const DevParams& p, int nslabs, int64_t* stats_out, hipStream_t st) {
  hipLaunchKernelGGL(finalize_kernel, dim3(p.nsec + PGPU_NSTATS), dim3(256), 0, st, p, nslabs, stats_out);
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
