// HIP kernels of the MI355X segment query path (gfx950 / CDNA4).
//
// One launch runs a whole query over every segment a GPU owns.  Geometry (pgpu_internal.h): one workgroup per CU
// (grid = min(#CUs, #tiles)) owns a contiguous range of 2048-doc tiles; two variants, chosen on the host:
//   SPARSE  1024 threads = 4 loader + 12 consumer waves (~90 VGPRs) -- selective filters, candidate queues
//   DENSE    512 threads = 2 loader +  6 consumer waves (~190 VGPRs) -- most docs survive, wide aggregation
//
//   LOADERS              stream each tile's "staged" forward-index columns (the scan columns of the dense part of
//                        the filter, plus the group / aggregation columns when most docs survive) into a ring of
//                        LDS slots with global_load_lds (16 B per lane, 1 KiB per instruction), and publish slot k
//                        behind a counted `s_waitcnt vmcnt` once its bytes have landed.  A loader only ever waits
//                        for its own DMAs, so ~64 KiB stay in flight per CU regardless of what the consumers do.
//   CONSUMERS            consumer c takes tiles c, c+NCONS, ...  Lane l owns docs [32l, 32l+32): its 32*b bits are b
//                        consecutive big-endian words, read with the widest bank-conflict-free ds_read and unpacked
//                        with compile-time shifts (one template instantiation per bit width) into 32 dict ids.
//
//   K1  fixed-bit unpack fused with dict-id RANGE / SET / LIST predicates -> one 32-bit match word per lane.
//   K2  Roaring array / bitmap / run containers (BitmapBasedFilterOperator), sorted-index doc ranges, AND / OR / NOT
//       on the match words (short-circuit of AND when a tile empties).
//   K3  COUNT / SUM / MIN / MAX / AVG and dictionary-id GROUP BY: matched docs are compacted into an LDS list so
//       every dictionary / remap gather and every table update runs with full lanes; per-lane partials + wave
//       reductions (aggregation only), LDS-privatised dense tables (small key spaces) or HBM tables.
//   Sparse work (a filter child too selective to stream, or aggregation columns under a selective filter) goes
//   through a per-consumer candidate queue of doc ids, flushed in rounds of 64 lanes x U docs with every gather of
//   a round issued before the first wait.
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

#include <algorithm>

#include "../../include/pinot_gpu.h"
#include "pgpu_internal.h"

// The file is compiled as several translation units in parallel (__graft_entry__.build): -DPGPU_TU=k keeps only
// the kernels of one aggregation mode (0 AGG, 1 LDS, 2 GLOBAL, 3 PART, 4 HASH) or the common kernels and the
// dispatchers (5).  Every query-kernel instantiation inlines all 31 bit widths, so one TU would take minutes.
#ifndef PGPU_TU
#define PGPU_TU -1  // everything
#endif
#define PGPU_TU_COMMON 5
#define TU_HAS(k) (PGPU_TU < 0 || PGPU_TU == (k))

#define WT PGPU_WT
#define MAXS PGPU_MAX_SLOTS
#define U PGPU_DOC_U
#define FI __device__ __forceinline__

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Loads through the global address space: segment pointers reach the kernel inside structs in HBM, so the
// compiler only sees generic pointers and would emit flat_* (which also count against lgkmcnt and stall LDS).
#define GAS __attribute__((address_space(1)))
#define LAS __attribute__((address_space(3)))
template <class T>
FI T gld(const T* p, size_t i) { return ((const GAS T*)p)[i]; }
// Query metadata (segments, columns, instructions, pool) is read through the constant address space with
// wave-uniform addresses so it becomes s_load (lgkmcnt) -- never a vector load that a vmcnt wait would order
// behind the loader's DMAs -- and is never copied into a private array (dynamic indexing spills to scratch).
#define CAS __attribute__((address_space(4)))
template <class T>
FI T cld(const T* p) {
  if constexpr (sizeof(T) > 8) {  // structs: dword by dword (no copy constructor from an address-space lvalue)
    static_assert(sizeof(T) % 4 == 0, "dword-sized metadata");
    uint32_t w[sizeof(T) / 4];
#pragma unroll
    for (unsigned i = 0; i < sizeof(T) / 4; ++i) w[i] = ((const CAS uint32_t*)p)[i];
    T v;
    __builtin_memcpy(&v, w, sizeof(T));
    return v;
  } else {
    return *(const CAS T*)p;
  }
}
template <class T>
FI T cld(const T* p, size_t i) { return ((const CAS T*)p)[i]; }
FI int sgpr(int v) { return __builtin_amdgcn_readfirstlane(v); }
// Phase timers: shader clock via s_memtime, accumulated per wave.  Compiled in only for the profiling build
// (libpinotgpu_prof.so, -DPGPU_PROFILE_BUILD, loaded when PGPU_PROFILE=1): the counters cost SGPRs the product
// build needs for the consumer's state.
#ifdef PGPU_PROFILE_BUILD
struct Prof {
  bool on;
  int64_t t[PGPU_NPROF];
};
FI int64_t now(const Prof& pf) { return pf.on ? (int64_t)__builtin_amdgcn_s_memtime() : 0; }
#define PROF_ADD(pf, k, since) do { if ((pf).on) (pf).t[k] += (int64_t)__builtin_amdgcn_s_memtime() - (since); } while (0)
#define PROF_ON(pf) ((pf).on)
#else
struct Prof {
  static constexpr bool on = false;
  int64_t t[1];
};
FI int64_t now(const Prof&) { return 0; }
#define PROF_ADD(pf, k, since) do { (void)(since); } while (0)
#define PROF_ON(pf) false
#endif
FI uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
FI uint32_t lowmask(uint32_t b) { return 0xFFFFFFFFu >> (32u - b); }
// Bit i of a mask word as v_bfe_u32 with inline operands.
FI uint32_t lane_bit(uint32_t m, int i) { return __builtin_amdgcn_ubfe(m, (uint32_t)i, 1u); }
FI int lane_id() { return threadIdx.x & 63; }

FI void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

FI int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
FI double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
FI int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(v, o, 64); v = t < v ? t : v; }
  return v;
}
FI int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { int64_t t = __shfl_xor(v, o, 64); v = t > v ? t : v; }
  return v;
}
// DPP lane moves (VALU, no LDS round trip).  Callers run with all 64 lanes active.
#define DPP_QUAD_1032 0xB1
#define DPP_QUAD_2301 0x4E
#define DPP_ROW_SHR(n) (0x110 + (n))
#define DPP_ROW_MIRROR 0x140
#define DPP_ROW_HALF_MIRROR 0x141
#define DPP_ROW_BCAST15 0x142
#define DPP_ROW_BCAST31 0x143
template <int CTRL, int ROWS = 0xF>
FI int dpp(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xF, true); }

// Wave-uniform total (an SGPR value: callers branch on it as a scalar).
FI int wave_sum_i32(int v) {
  v += dpp<DPP_QUAD_1032>(v);
  v += dpp<DPP_QUAD_2301>(v);
  v += dpp<DPP_ROW_HALF_MIRROR>(v);
  v += dpp<DPP_ROW_MIRROR>(v);  // every lane of a 16-lane row holds the row total
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}
// Exclusive prefix sum over the wave's lanes (row scans + row broadcasts).
FI int wave_excl_scan(int v) {
  int x = v;
  x += dpp<DPP_ROW_SHR(1)>(x);
  x += dpp<DPP_ROW_SHR(2)>(x);
  x += dpp<DPP_ROW_SHR(4)>(x);
  x += dpp<DPP_ROW_SHR(8)>(x);
  x += __builtin_amdgcn_update_dpp(0, x, DPP_ROW_BCAST15, 0xA, 0xF, false);
  x += __builtin_amdgcn_update_dpp(0, x, DPP_ROW_BCAST31, 0xC, 0xF, false);
  return x - v;
}

// ---- LDS flags (ring hand-off between the loader and the consumers) ----------------------------------------------
FI int flag_load(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
FI void flag_store(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
// The loader's flag accesses as inline asm: the compiler would otherwise guard every LDS access of the loader
// with `s_waitcnt vmcnt(0)` (it cannot prove the flags do not alias the in-flight LDS-DMA destinations).
FI uint32_t lds_off(const void* p) { return (uint32_t)(size_t)(const LAS void*)p; }
FI int loader_flag_load(const int* p) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_off(p)) : "memory");
  return sgpr(v);
}
FI void loader_flag_store(int* p, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_off(p)), "v"(v) : "memory");
}

// The query's cancel word (HBM, written by pgpu_query_cancel through a side-stream memset): one uncached load.
FI bool query_cancelled(const DevParams& p) {
  if (!p.cancel) return false;
  const int v = __hip_atomic_load(p.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return (uint32_t)__builtin_amdgcn_readfirstlane(v) == p.cancel_gen;
}

// s_waitcnt vmcnt(n) for a runtime n in [0, 63] (the immediate must be a constant).
FI void wait_vmcnt(int n) {
#define VMC(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
  switch (n) {
    VMC(0) VMC(1) VMC(2) VMC(3) VMC(4) VMC(5) VMC(6) VMC(7) VMC(8) VMC(9) VMC(10) VMC(11) VMC(12) VMC(13) VMC(14)
    VMC(15) VMC(16) VMC(17) VMC(18) VMC(19) VMC(20) VMC(21) VMC(22) VMC(23) VMC(24) VMC(25) VMC(26) VMC(27)
    VMC(28) VMC(29) VMC(30) VMC(31) VMC(32) VMC(33) VMC(34) VMC(35) VMC(36) VMC(37) VMC(38) VMC(39) VMC(40)
    VMC(41) VMC(42) VMC(43) VMC(44) VMC(45) VMC(46) VMC(47) VMC(48) VMC(49) VMC(50) VMC(51) VMC(52) VMC(53)
    VMC(54) VMC(55) VMC(56) VMC(57) VMC(58) VMC(59) VMC(60) VMC(61) VMC(62)
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
  }
#undef VMC
}

// Order-preserving int64 key of a dictionary value (MIN/MAX sections).
FI int64_t minmax_key(const void* dict, int32_t vtype, uint32_t id) {
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
FI int64_t sec_identity(int32_t op) {
  return op == PGPU_RED_MIN_I64 ? INT64_MAX : (op == PGPU_RED_MAX_I64 ? INT64_MIN : 0);
}

// Dictionary values dict[idx[r]] as the 8-byte cells their section reduces: int64 for integer SUM, float64 bits
// for floating SUM, order-preserving key for MIN/MAX.  The (uniform) type dispatch sits outside the unrolled
// gathers so all N loads are in flight before the first use.
FI int64_t key_of_double(double d) {
  const int64_t b = __double_as_longlong(d);
  return b >= 0 ? b : (b ^ 0x7FFFFFFFFFFFFFFFll);
}
template <int N>
FI void gather_cells(const void* dict, int32_t vtype, int32_t op, const uint32_t (&idx)[N], int64_t (&out)[N]) {
  if (vtype == PGPU_INT || vtype == PGPU_FLOAT) {
    uint32_t raw[N];
#pragma unroll
    for (int r = 0; r < N; ++r) raw[r] = gld((const uint32_t*)dict, idx[r]);
    if (vtype == PGPU_INT) {
#pragma unroll
      for (int r = 0; r < N; ++r) out[r] = (int64_t)(int32_t)raw[r];  // SUM_I64 value == MIN/MAX key
    } else {
#pragma unroll
      for (int r = 0; r < N; ++r) {
        const double d = (double)__uint_as_float(raw[r]);
        out[r] = op == PGPU_RED_MIN_I64 || op == PGPU_RED_MAX_I64 ? key_of_double(d) : __double_as_longlong(d);
      }
    }
  } else {
    int64_t raw[N];
#pragma unroll
    for (int r = 0; r < N; ++r) raw[r] = gld((const int64_t*)dict, idx[r]);
    if (vtype == PGPU_LONG) {
#pragma unroll
      for (int r = 0; r < N; ++r) out[r] = raw[r];
    } else {
#pragma unroll
      for (int r = 0; r < N; ++r)
        out[r] = op == PGPU_RED_MIN_I64 || op == PGPU_RED_MAX_I64 ? key_of_double(__longlong_as_double(raw[r])) : raw[r];
    }
  }
}
// Split integer SUM (DevAgg::part): the agg's cell sums one 21-bit part of every value, so that no int64 cell can
// wrap (pgpu_table_layout.agg_sum_parts).
FI int64_t part_of(int64_t v, int32_t part) {
  if (part == 1) return v & ((1ll << PGPU_PART_BITS) - 1);
  if (part == 2) return (v >> PGPU_PART_BITS) & ((1ll << PGPU_PART_BITS) - 1);
  if (part == 3) return v >> (2 * PGPU_PART_BITS);
  return v;
}
// Fixed-point floating SUM (DevAgg::fxe / part, pgpu_table_layout.agg_sum_exp / agg_sum_parts): the double v as
// the integer I = rint(|v| * 2^-fxe) (< 2^(21 * parts) by the layout's choice), and this section's share of it:
// sign(v) * bits [21 (part-1), 21 part) of I.  Integer adds make the sums order-independent.  Bits of I above the
// double's own significand come from shifting it (exact); only a value finer than 2^fxe is rounded.
FI int64_t fixed_part(int64_t bits, int32_t fxe, int32_t part) {
  const uint64_t mag = (uint64_t)bits & 0x7FFFFFFFFFFFFFFFull;
  if (mag == 0) return 0;
  const int be = (int)(mag >> 52);
  const uint64_t m = be ? ((mag & 0xFFFFFFFFFFFFFull) | (1ull << 52)) : mag;  // |v| = m * 2^((be ? be : 1) - 1075)
  const int s = (be ? be : 1) - 1075 - fxe;                                  // I = m * 2^s
  const int lo = PGPU_PART_BITS * (part - 1);
  uint64_t d;
  if (s < 0) {  // below the window's last bit: round (I < 2^53)
    const uint64_t i = (uint64_t)__builtin_rint(__builtin_ldexp(__longlong_as_double((int64_t)mag), -fxe));
    d = lo < 64 ? (i >> lo) : 0;
  } else {
    const int t = lo - s;  // bits [lo, lo + 21) of m << s = bits [t, t + 21) of m
    d = t >= 0 ? (t < 64 ? (m >> t) : 0) : (-t < PGPU_PART_BITS ? (m << -t) : 0);
  }
  d &= (1ull << PGPU_PART_BITS) - 1;
  return bits < 0 ? -(int64_t)d : (int64_t)d;
}
// gather_cells' SUM values -> the agg's cells: a floating value's fixed-point part, or an integer's part section
template <int N>
FI void apply_part(int64_t (&v)[N], const DevAgg& ag) {
  if (ag.op == PGPU_RED_SUM_I64 && (ag.vtype == PGPU_FLOAT || ag.vtype == PGPU_DOUBLE)) {
#pragma unroll
    for (int r = 0; r < N; ++r) v[r] = fixed_part(v[r], ag.fxe, ag.part);
    return;
  }
  if (ag.part == 0) return;
#pragma unroll
  for (int r = 0; r < N; ++r) v[r] = part_of(v[r], ag.part);
}
FI int64_t cell_combine(int32_t op, int64_t a, int64_t b) {
  if (op == PGPU_RED_SUM_I64) return a + b;
  if (op == PGPU_RED_SUM_F64) return __double_as_longlong(__longlong_as_double(a) + __longlong_as_double(b));
  if (op == PGPU_RED_MIN_I64) return b < a ? b : a;
  return b > a ? b : a;
}
FI int64_t wave_combine(int32_t op, int64_t v) {
  if (op == PGPU_RED_SUM_I64) return wave_sum_i64(v);
  if (op == PGPU_RED_SUM_F64) return __double_as_longlong(wave_sum_f64(__longlong_as_double(v)));
  if (op == PGPU_RED_MIN_I64) return wave_min_i64(v);
  return wave_max_i64(v);
}
// Atomic table update (LDS or HBM cell).
FI void cell_atomic(int64_t* cell, int32_t op, int64_t v) {
  if (op == PGPU_RED_SUM_I64) atomicAdd((unsigned long long*)cell, (unsigned long long)v);
  else if (op == PGPU_RED_SUM_F64) atomicAdd((double*)cell, __longlong_as_double(v));
  else if (op == PGPU_RED_MIN_I64) atomicMin((long long*)cell, (long long)v);
  else atomicMax((long long*)cell, (long long)v);
}
// PART mode: a record carries the raw 4-byte dictionary value; each aggregation derives its cell from it.
FI int64_t raw_to_cell(uint32_t raw, int32_t vtype, int32_t op) {
  if (vtype == PGPU_INT) return (int64_t)(int32_t)raw;
  const double d = (double)__uint_as_float(raw);
  return op == PGPU_RED_SUM_F64 ? __double_as_longlong(d) : key_of_double(d);
}
template <int N>
FI void gather_raw(const void* dict, const uint32_t (&idx)[N], uint32_t (&out)[N]) {
#pragma unroll
  for (int r = 0; r < N; ++r) out[r] = gld((const uint32_t*)dict, idx[r]);
}

// ---- fixed-bit extraction (compile-time bit width) -------------------------------------------------------------
// w[] = the lane's B words, byte-swapped (MSB-first bit order); value i occupies bits [i*B, (i+1)*B).
template <int B>
FI uint32_t extract_c(const uint32_t (&w)[B], int i) {
  const int o = i * B;
  const int k = o >> 5, sh = o & 31;
  if (sh + B <= 32) return (w[k] >> (32 - sh - B)) & lowmask(B);
  return __builtin_amdgcn_alignbit(w[k], w[k + 1], 64 - sh - B) & lowmask(B);
}
template <int B>
FI void unpack_b(const uint32_t (&w)[B], uint32_t (&ids)[32]) {
#pragma unroll
  for (int i = 0; i < 32; ++i) ids[i] = extract_c<B>(w, i);
}

// This lane's index, opaque to loop-invariant code motion (per-bit-width lane offsets would otherwise be hoisted
// out of the tile loop and pin ~30 VGPRs for the kernel's lifetime).
FI uint32_t opaque_lane() {
  uint32_t l;
  asm volatile("v_and_b32 %0, 63, %1" : "=v"(l) : "v"(threadIdx.x));
  return l;
}

// The lane's B words of a staged column region in a ring slot.  Record stride: B dwords, +4 when B % 8 == 0
// (pgpu_stage_region_bytes); read width: b128 when B % 4 == 0, b64 when B % 2 == 0, b32 otherwise -- every
// combination is bank-conflict free for a wave's lane groups.
template <int B>
FI void slot_lane_words(const uint32_t* region, uint32_t (&w)[B]) {
  constexpr int stride = (B % 8 == 0) ? B + 4 : B;
  const LAS uint32_t* src = (const LAS uint32_t*)region + opaque_lane() * stride;
  if constexpr (B % 4 == 0) {
#pragma unroll
    for (int k = 0; k < B; k += 4) {
      const u32x4 v = *(const LAS u32x4*)(src + k);
      w[k] = v.x; w[k + 1] = v.y; w[k + 2] = v.z; w[k + 3] = v.w;
    }
  } else if constexpr (B % 2 == 0) {
#pragma unroll
    for (int k = 0; k < B; k += 2) {
      const u32x2 v = *(const LAS u32x2*)(src + k);
      w[k] = v.x; w[k + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < B; ++k) w[k] = src[k];
  }
#pragma unroll
  for (int k = 0; k < B; ++k) w[k] = bswap32(w[k]);
}
// The lane's B words of tile `tile_in_seg` straight from HBM (fallback for a dense column that is not staged).
template <int B>
FI void hbm_lane_words(const uint32_t* fwd, int tile_in_seg, uint32_t (&w)[B]) {
  const GAS uint32_t* src = (const GAS uint32_t*)fwd + ((size_t)tile_in_seg * 64 + opaque_lane()) * B;
#pragma unroll
  for (int k = 0; k < B; ++k) w[k] = bswap32(src[k]);
}

// ... raw (big-endian as stored: a caller unpacks later), for loads issued ahead of their use
template <int B>
FI void hbm_lane_raw(const uint32_t* fwd, int tile_in_seg, uint32_t (&w)[B]) {
  const GAS uint32_t* src = (const GAS uint32_t*)fwd + ((size_t)tile_in_seg * 64 + opaque_lane()) * B;
#pragma unroll
  for (int k = 0; k < B; ++k) w[k] = src[k];
}

template <int B>
FI void decode_b(const uint32_t* region, const uint32_t* fwd, int tile_in_seg, uint32_t (&ids)[32]) {
  uint32_t w[B];
  if (region) slot_lane_words<B>(region, w);
  else hbm_lane_words<B>(fwd, tile_in_seg, w);
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

// The lane's 32 dict ids of a column: from its staged slot region (region != nullptr) or from HBM.  Callers keep
// the number of call sites (each inlines all 31 widths) to three: filter scan, register copies, aggregation.
FI void decode_ids(int bits, const uint32_t* region, const uint32_t* fwd, int tile_in_seg, uint32_t (&ids)[32]) {
#define DEC_CALL(B) decode_b<B>(region, fwd, tile_in_seg, ids)
  PGPU_DISPATCH_B(bits, DEC_CALL)
#undef DEC_CALL
}
// The lane's 32 "ids" of an aggregation / group column: dict ids, or for a raw (no-dictionary) column the doc ids
// themselves -- its value array takes the dictionary's place (DevColumn::dict), so every gather serves both.
FI void column_ids(int kind, int bits, const uint32_t* region, const uint32_t* fwd, int tile_in_seg,
                   uint32_t (&ids)[32]) {
  if (kind == PGPU_COL_RAW) {
    const uint32_t d0 = (uint32_t)tile_in_seg * WT + 32u * (uint32_t)lane_id();
#pragma unroll
    for (int i = 0; i < 32; ++i) ids[i] = d0 + (uint32_t)i;
    return;
  }
  decode_ids(bits, region, fwd, tile_in_seg, ids);
}

// ---- predicates -----------------------------------------------------------------------------------------------
#define PRED_RANGE 0
#define PRED_SET 1   // bitset over dict ids in the pool
#define PRED_LIST 2  // up to 8 ids in the pool
#define PRED_MASK 3  // columns of <= 64 ids: bit id of the 64-bit mask (lo | span << 32)

struct Pred {
  int kind;
  uint32_t lo, span;         // RANGE: (id - lo) < span
  const uint32_t* bits;      // SET
  uint32_t ids[8];           // LIST
  bool negate;
};

FI Pred make_pred(const DevInstr& in, const int32_t* pool) {
  Pred p;
  p.kind = in.pred;
  p.negate = in.negate != 0;
  p.lo = (uint32_t)in.lo;
  p.span = in.pred == PRED_MASK ? (uint32_t)in.hi : (uint32_t)(in.hi - in.lo);
  p.bits = (const uint32_t*)(pool + in.pool_off);
#pragma unroll
  for (int k = 0; k < 8; ++k) p.ids[k] = in.ids[k];  // unused entries are 0xFFFFFFFF (host)
  return p;
}

FI bool eval_pred(const Pred& p, uint32_t id) {
  bool m;
  if (p.kind == PRED_RANGE) {
    m = (id - p.lo) < p.span;
  } else if (p.kind == PRED_MASK) {
    m = (uint32_t)((((uint64_t)p.span << 32) | p.lo) >> (id & 63)) & 1u;
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
FI uint32_t pred_ids(const uint32_t (&ids)[32], const Pred& p) {
  uint32_t m = 0;
  if (p.kind == PRED_RANGE) {
#pragma unroll
    for (int i = 31; i >= 0; --i) m = (m << 1) | (uint32_t)((ids[i] - p.lo) < p.span);
  } else if (p.kind == PRED_MASK) {
    const uint64_t mask = ((uint64_t)p.span << 32) | p.lo;
#pragma unroll
    for (int i = 31; i >= 0; --i) m = (m << 1) | ((uint32_t)(mask >> (ids[i] & 63)) & 1u);
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

// ---- per-doc access ---------------------------------------------------------------------------------------------
// SortedIndexReaderImpl.getDictId: last dict id whose start <= doc.
FI uint32_t sorted_dict_id(const int32_t* __restrict__ pairs, int32_t card, int32_t doc) {
  int32_t lo = 0, hi = card - 1;
  while (lo <= hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (gld(pairs, 2 * (size_t)mid) <= doc) lo = mid + 1; else hi = mid - 1;
  }
  return (uint32_t)hi;
}

// Dict ids of segment docs d[u] gathered from HBM: two big-endian words around each doc's bits, all 2N loads
// (unconditional loads of valid addresses) issued before the first use.
struct ColRef {
  const uint32_t* fwd;
  const int32_t* sorted;
  int32_t kind, bits, card;
};
template <int N>
FI void gather_ids(const ColRef& c, const int32_t (&d)[N], uint32_t (&id)[N]) {
  if (c.kind == PGPU_COL_RAW) {  // the value array is indexed by doc id
#pragma unroll
    for (int u = 0; u < N; ++u) id[u] = (uint32_t)d[u];
    return;
  }
  if (c.kind == PGPU_COL_SORTED) {
#pragma unroll
    for (int u = 0; u < N; ++u) id[u] = sorted_dict_id(c.sorted, c.card, d[u]);
    return;
  }
  const uint32_t b = (uint32_t)c.bits;
  uint32_t hi[N], lo[N], r[N];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const uint64_t e = (uint64_t)(d[u] + 1) * b;
    const uint64_t we = (e - 1u) >> 5;
    r[u] = (uint32_t)(e - (we << 5));
    hi[u] = gld(c.fwd, we);
    lo[u] = we ? gld(c.fwd, we - 1) : 0u;
  }
#pragma unroll
  for (int u = 0; u < N; ++u) id[u] = __builtin_amdgcn_alignbit(bswap32(lo[u]), bswap32(hi[u]), 32u - r[u]) & lowmask(b);
}
FI ColRef colref(const DevColumn& c) { return ColRef{c.fwd, c.sorted, c.kind, c.bits, c.card}; }
FI ColRef colref(const DevInstr& in) { return ColRef{in.fwd, in.sorted, in.kind, in.bits, in.card}; }
template <int N>
FI void remap_ids(const int32_t* remap, uint32_t (&id)[N]) {
  if (!remap) return;
#pragma unroll
  for (int u = 0; u < N; ++u) id[u] = (uint32_t)gld(remap, id[u]);
}

// ---- hash group-by (PGPU_MODE_HASH) --------------------------------------------------------------------------------
FI uint64_t hmix(uint64_t k) {  // 64-bit finaliser (murmur3 fmix64)
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
// Slot keys change once (empty -> key), by CAS; agent-scope loads see other XCDs' claims.  A stale empty read only
// costs a failed CAS.
FI uint64_t hload(const uint64_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Slot of every live key in the open-addressing table `keys` (mask + 1 slots, linear probing): the slot already
// holding the key, or the empty slot this lane claims with a 64-bit CAS.  Every first probe is issued before the
// first compare.  A probe sequence that runs through the whole table sets hflag (the query fails, never hangs).
template <int N>
FI void hash_insert(uint64_t* keys, uint64_t mask, const uint64_t (&key)[N], uint32_t live, uint32_t (&slot)[N],
                    int32_t* hflag) {
  uint64_t h[N], cur[N];
#pragma unroll
  for (int r = 0; r < N; ++r) {
    h[r] = hmix(key[r]) & mask;
    cur[r] = ((live >> r) & 1u) ? hload(keys + h[r]) : 0ull;
  }
#pragma unroll
  for (int r = 0; r < N; ++r) {
    slot[r] = 0;
    if (!((live >> r) & 1u)) continue;
    uint64_t hh = h[r], c = cur[r];
    for (uint64_t it = 0;; ++it) {
      if (c == key[r]) break;
      if (c == PGPU_HASH_EMPTY) {
        const uint64_t prev = atomicCAS((unsigned long long*)(keys + hh), (unsigned long long)PGPU_HASH_EMPTY,
                                        (unsigned long long)key[r]);
        if (prev == PGPU_HASH_EMPTY || prev == key[r]) break;
      }
      if (it >= mask) {
        __hip_atomic_store(hflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        hh = 0;
        break;
      }
      hh = (hh + 1) & mask;
      c = hload(keys + hh);
    }
    slot[r] = (uint32_t)hh;
  }
}
// Cell slots of the live docs' group keys (words k0 / k1, see PGPU_MODE_HASH), then the segment's distinct-key bit.
template <int N>
FI void hash_slots(const DevParams& p, const uint64_t (&k0)[N], const uint64_t (&k1)[N], uint32_t live,
                   int32_t track, uint32_t (&slot)[N]) {
  uint64_t* w0 = (uint64_t*)(p.table + (size_t)p.nsec * p.G);
  const uint64_t mask = p.G - 1;
  if (p.key_words == 2) {
    uint32_t s0[N];
    hash_insert(w0 + p.G, mask, k0, live, s0, p.hflag);  // intern word 0
    uint64_t c[N];
#pragma unroll
    for (int r = 0; r < N; ++r) c[r] = ((uint64_t)s0[r] << 32) | k1[r];
    hash_insert(w0, mask, c, live, slot, p.hflag);
  } else {
    hash_insert(w0, mask, k0, live, slot, p.hflag);
  }
  if (track) {
    uint32_t* row = p.segmask + (size_t)(track - 1) * (p.G >> 5);
#pragma unroll
    for (int r = 0; r < N; ++r)
      if ((live >> r) & 1u) atomicOr(row + (slot[r] >> 5), 1u << (slot[r] & 31));
  }
}

// Roaring probe for one doc (per-doc filter leaves): is `d` in the bitmap of dict id `id`?
struct InvIndex {
  const uint32_t* dir;
  const DevContainer* ct;
  const uint8_t* data;
};
__device__ __noinline__ bool bitmap_contains(InvIndex c, uint32_t id, uint32_t d) {
  const uint32_t key = d >> 16, lo16 = d & 0xFFFFu;
  int32_t a = (int32_t)gld(c.dir, id), z = (int32_t)gld(c.dir, id + 1) - 1;
  while (a <= z) {
    const int32_t mid = (a + z) >> 1;
    const DevContainer ct = c.ct[mid];
    if (ct.key == key) {
      if (ct.type == PGPU_CT_BITMAP) return (gld((const uint32_t*)(c.data + ct.offset), lo16 >> 5) >> (lo16 & 31)) & 1u;
      if (ct.type == PGPU_CT_RUN) {
        const uint16_t* r = (const uint16_t*)(c.data + ct.offset);
        int32_t l = 0, h = (int32_t)ct.card - 1;
        while (l <= h) {  // last run whose start <= lo16
          const int32_t m = (l + h) >> 1;
          if (r[2 * m] <= lo16) l = m + 1; else h = m - 1;
        }
        return h >= 0 && lo16 <= (uint32_t)r[2 * h] + r[2 * h + 1];
      }
      const uint16_t* v = (const uint16_t*)(c.data + ct.offset);
      int32_t l = 0, h = (int32_t)ct.card - 1;
      while (l <= h) {
        const int32_t m = (l + h) >> 1;
        if (v[m] == lo16) return true;
        if (v[m] < lo16) l = m + 1; else h = m - 1;
      }
      return false;
    }
    if (ct.key < key) a = mid + 1; else z = mid - 1;
  }
  return false;
}

// ---- Roaring containers / sorted ranges for a whole tile -------------------------------------------------------
// Container of bitmap `id` holding key `key` (index into c.ct, -1 if none): uniform scalar loads; a bitmap that
// has a container for every key (dense) is hit directly at first + key, others fall back to a binary search.
FI int32_t find_container(const InvIndex& c, uint32_t id, uint32_t key) {
  int32_t a = (int32_t)cld(c.dir + id), z = (int32_t)cld(c.dir + id + 1) - 1;
  if (a > z) return -1;
  const int32_t g = a + (int32_t)key;
  if (g <= z && cld(&c.ct[g].key) == key) return g;
  while (a <= z) {
    const int32_t mid = (a + z) >> 1;
    const uint32_t k = cld(&c.ct[mid].key);
    if (k == key) return mid;
    if (k < key) a = mid + 1; else z = mid - 1;
  }
  return -1;
}
// Number of values of the sorted uint16 array v[0, n) below x (n <= 4096), by two rounds of a 64-way wave
// search instead of a 12-step chain of dependent loads: round 1 tests every step-th value (step = ceil(n / 64))
// and a ballot finds the block holding the boundary; round 2 tests that block's values.
FI int32_t lower_bound64(const uint16_t* v, int32_t n, uint32_t x) {
  const int lane = lane_id();
  const int32_t step = (n + 63) >> 6;
  const int32_t p = lane * step;
  const int c = __popcll(__ballot(p < n && (uint32_t)gld(v, p) < x));
  if (c == 0) return 0;
  const int32_t b = (c - 1) * step + 1;  // v[b - 1] < x; v[b + step - 1] >= x when that index exists
  const int32_t q = b + lane;
  return b + __popcll(__ballot(lane < step && q < n && (uint32_t)gld(v, q) < x));
}

// ---- Roaring containers / sorted ranges for a whole tile -------------------------------------------------------
// Bits of the tile covered by one Roaring bitmap (dict id `id`), for this lane's 32 docs.
__device__ __noinline__ uint32_t bitmap_word(InvIndex c, int32_t doc0, uint32_t id, uint32_t* lds_words) {
  const uint32_t key = (uint32_t)doc0 >> 16;
  const uint32_t lo16 = (uint32_t)doc0 & 0xFFFFu;  // multiple of 2048
  const int lane = lane_id();
  const int32_t ci = find_container(c, id, key);
  if (ci < 0) return 0u;
  const uint32_t type = cld(&c.ct[ci].type), card = cld(&c.ct[ci].card), offset = cld(&c.ct[ci].offset);
  const uint32_t my0 = lo16 + 32u * lane;  // my first doc within the container
  if (type == PGPU_CT_BITMAP) return gld((const uint32_t*)(c.data + offset), my0 >> 5);
  if (type == PGPU_CT_RUN) {
    const uint16_t* r = (const uint16_t*)(c.data + offset);
    int32_t l = 0, h = (int32_t)card;
    while (l < h) {  // first run whose end >= lo16
      const int32_t m = (l + h) >> 1;
      if ((uint32_t)gld(r, 2 * m) + gld(r, 2 * m + 1) < lo16) l = m + 1; else h = m;
    }
    uint32_t w = 0;
    for (int32_t i = l; i < (int32_t)card; ++i) {  // uniform loop over the runs overlapping the tile
      const uint32_t s = gld(r, 2 * i), e = s + gld(r, 2 * i + 1);
      if (s >= lo16 + WT) break;
      if (e >= my0 && s <= my0 + 31) {
        const uint32_t bs = s > my0 ? s - my0 : 0u, be = e < my0 + 31 ? e - my0 : 31u;
        w |= (0xFFFFFFFFu >> (31 - be)) & (0xFFFFFFFFu << bs);
      }
    }
    return w;
  }
  // ARRAY: values in [lo16, lo16 + WT) scattered to their owner lanes through LDS
  const uint16_t* v = (const uint16_t*)(c.data + offset);
  const int32_t first = lower_bound64(v, (int32_t)card, lo16);
  const int32_t last = lower_bound64(v, (int32_t)card, lo16 + WT);
  lds_words[lane] = 0u;
  wave_sync();
  for (int32_t i = first + lane; i < last; i += 64) {
    const uint32_t off = (uint32_t)gld(v, i) - lo16;
    atomicOr(&lds_words[off >> 5], 1u << (off & 31));
  }
  wave_sync();
  const uint32_t w = lds_words[lane];
  wave_sync();
  return w;
}

__device__ __noinline__ uint32_t sorted_ranges_word(const int32_t* rg, int n, int32_t doc0) {
  const int32_t d0 = doc0 + 32 * lane_id(), d1 = d0 + 31;
  const int32_t w0 = doc0, w1 = doc0 + WT - 1;
  int32_t l = 0, h = n;
  while (l < h) { const int32_t m = (l + h) >> 1; if (rg[2 * m + 1] < w0) l = m + 1; else h = m; }
  uint32_t w = 0;
  for (int32_t i = l; i < n; ++i) {  // uniform over the ranges overlapping the tile
    const int32_t s = rg[2 * i], e = rg[2 * i + 1];
    if (s > w1) break;
    if (e >= d0 && s <= d1) {
      const int32_t bs = s > d0 ? s - d0 : 0, be = e < d1 ? e - d0 : 31;
      w |= (0xFFFFFFFFu >> (31 - be)) & (0xFFFFFFFFu << bs);
    }
  }
  return w;
}

FI bool in_sorted_ranges(const int32_t* rg, int n, int32_t d) {
  int32_t l = 0, h = n;
  while (l < h) { const int32_t m = (l + h) >> 1; if (rg[2 * m + 1] < d) l = m + 1; else h = m; }
  return l < n && rg[2 * l] <= d;
}

// ---- workgroup LDS carve ------------------------------------------------------------------------------------------
// [full flags | free flags | loader instr counts] | 7 x consumer area | LDS group table | ring slots
struct Lds {
  int* full;
  int* freef;
  int* icnt;
  unsigned char* cons;
  int64_t* ltab;
  unsigned char* ring;
};

template <int DENSE>
FI Lds carve(unsigned char* base, const DevParams& p) {
  Lds L;
  L.full = (int*)base;
  L.freef = L.full + PGPU_RING_MAX;
  L.icnt = L.freef + PGPU_RING_MAX;
  L.cons = base + PGPU_FLAG_BYTES;
  L.ltab = (int64_t*)(L.cons + PGPU_NCONS_OF(DENSE) * p.cons_bytes);
  L.ring = (unsigned char*)L.ltab + ((p.ltab_bytes + 15) & ~15);
  return L;
}

// Segment / tile cursor over a contiguous global tile range (the segment's tile count is cached: advancing costs
// a scalar load only when it crosses into the next segment).
struct Cursor {
  int seg;
  int tile_in_seg;
  int ntiles;
};

FI Cursor cursor_at(const DevParams& p, int tile) {
  int lo = 0, hi = p.nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cld(&p.segs[mid].tile_begin) <= tile) lo = mid; else hi = mid - 1;
  }
  Cursor c;
  c.seg = lo;
  c.tile_in_seg = tile - cld(&p.segs[lo].tile_begin);
  c.ntiles = cld(&p.segs[lo].ntiles);
  return c;
}
// Returns true when the cursor moved into another segment.
FI bool cursor_advance(const DevParams& p, Cursor& c, int k) {
  c.tile_in_seg += k;
  bool moved = false;
  while (c.tile_in_seg >= c.ntiles && c.seg < p.nseg - 1) {
    c.tile_in_seg -= c.ntiles;
    ++c.seg;
    c.ntiles = cld(&p.segs[c.seg].ntiles);
    moved = true;
  }
  return moved;
}

// ================================================================================================================
// LOADER
// ================================================================================================================
// The loader's copy of its current segment's staging plan, in SGPRs (fixed-size, statically indexed).
struct StageCache {
  int nst;   // staged columns, the value-plane regions (DevSeg::nvstage) included
  int instrs;
  int lin;  // bit j: column j is bit-sliced (plain 256*b tile copy)
  const char* fwd[PGPU_MAX_STAGE];
  int bits[PGPU_MAX_STAGE];
  int off[PGPU_MAX_STAGE];
};
FI void load_stage(const DevParams& p, int seg, StageCache& sc) {
  const DevSeg* sg = p.segs + seg;
  sc.nst = cld(&sg->nstage);
  sc.instrs = cld(&sg->stage_instrs);
  sc.lin = cld(&sg->stage_sliced);
  const DevColumn* cols = p.cols + cld(&sg->col_begin);
  const int nv = cld(&sg->nvstage);
#pragma unroll
  for (int j = 0; j < PGPU_MAX_STAGE; ++j) {
    if (j < sc.nst) {
      const int qc = cld(&sg->stage_col[j]);
      sc.fwd[j] = (sc.lin >> j) & 1 ? (const char*)cld(&cols[qc].sliced) : (const char*)cld(&cols[qc].fwd);
      sc.bits[j] = cld(&cols[qc].bits);
      sc.off[j] = cld(&sg->stage_off[j]);
    } else if (j < sc.nst + nv) {  // value planes: a plain copy of vbits 256-B rows per tile
      const int qc = cld(&sg->vstage_col[j - sc.nst]);
      sc.fwd[j] = (const char*)cld(&cols[qc].vsliced);
      sc.bits[j] = cld(&cols[qc].vbits);
      sc.off[j] = cld(&sg->vstage_off[j - sc.nst]);
      sc.lin |= 1 << j;
    } else {
      sc.fwd[j] = nullptr;
      sc.bits[j] = 0;
      sc.off[j] = 0;
    }
  }
  sc.nst += nv;
}

// DMA the staged columns of one tile into `slot` (16 B per lane, 1 KiB per instruction; widths that are multiples
// of 8 bits skip one 16-B pad chunk per lane record, pgpu_stage_region_bytes).
FI void issue_tile(const StageCache& sc, int tile_in_seg, unsigned char* slot) {
  const int lane = lane_id();
#pragma unroll
  for (int j = 0; j < PGPU_MAX_STAGE; ++j) {
    if (j >= sc.nst) break;
    const int b = sc.bits[j];
    const char* src = sc.fwd[j] + (size_t)tile_in_seg * 256 * b;
    unsigned char* dst = slot + sc.off[j];
    if (b % 8 != 0 || ((sc.lin >> j) & 1)) {
      const int ninstr = (b + 3) >> 2;
      const char* ls = src + 16 * lane;
      for (int k = 0; k < ninstr; ++k) {
        if (64 * k + lane < 16 * b)
          __builtin_amdgcn_global_load_lds((const void*)(ls + 1024 * k), (LAS void*)(dst + 1024 * k), 16, 0, 0);
      }
    } else {
      const int q = b >> 2, ninstr = q + 1;  // q chunks + 1 pad chunk per lane record
      for (int k = 0; k < ninstr; ++k) {
        const int pos = 64 * k + lane;
        const int r = pos / (q + 1), s = pos - r * (q + 1);
        if (s < q)
          __builtin_amdgcn_global_load_lds((const void*)(src + 16 * (r * q + s)), (LAS void*)(dst + 1024 * k), 16, 0,
                                           0);
      }
    }
  }
}

// Loader `li` streams tiles li, li + NLOAD, ... of the workgroup's range into ring slot (seq % R).  Slot k is
// published (FULL = k+1) once its DMAs have landed, which the loader learns from a counted vmcnt: it keeps at most
// `inflight` of its own unpublished tiles and 63 instructions queued.
template <int NLOAD>
FI void loader(const DevParams& p, const Lds& L, int li, int t0, int ntiles, Prof& pf) {
  if (li >= ntiles) return;
  const int64_t t_start = now(pf);
  const int R = p.ring_slots, S = p.slot_bytes, P = p.inflight, budget = 63 - p.max_instrs;
  // issue cursor and its staging plan; publish cursor (instruction count of the oldest unpublished tile)
  Cursor ci = cursor_at(p, t0 + li), cp = ci;
  StageCache sc;
  load_stage(p, ci.seg, sc);
  int cp_instrs = sc.instrs;
  int seq = li, pub = li, pend = 0, slot = li % R, pslot = slot, nunpub = 0;
  auto publish_one = [&]() {
    const int64_t t0w = now(pf);
    wait_vmcnt(pend - cp_instrs);
    PROF_ADD(pf, PGPU_P_L_PUB, t0w);
    loader_flag_store(&L.full[pslot], pub + 1);
    pend -= cp_instrs;
    --nunpub;
    pub += NLOAD;
    pslot += NLOAD;
    while (pslot >= R) pslot -= R;
    if (pub < ntiles && cursor_advance(p, cp, NLOAD)) cp_instrs = cld(&p.segs[cp.seg].stage_instrs);
  };
  bool cx = false;  // cancelled: publish the remaining tiles as skipped, load nothing
  for (;;) {
    while (nunpub > 0 && (nunpub > P || pend > budget || seq >= ntiles)) publish_one();
    if (seq >= ntiles) break;
    if (!cx && ((seq - li) / NLOAD) % PGPU_CANCEL_POLL == PGPU_CANCEL_POLL - 1 && query_cancelled(p)) cx = true;
    if (cx)
      while (nunpub > 0) publish_one();
    if (seq >= R) {
      // the slot's previous tile must have been consumed; publish what is in flight while waiting
      const int64_t t0f = now(pf);
      for (int nap = 0; loader_flag_load(&L.freef[slot]) < seq - R + 1;) {
        if (nunpub > 0) {
          publish_one();
        } else {
          if (nap == 0) __builtin_amdgcn_s_sleep(2);
          else __builtin_amdgcn_s_sleep(6);
          nap = 1;
        }
      }
      PROF_ADD(pf, PGPU_P_L_FREE, t0f);
    }
    if (cx) {
      loader_flag_store(&L.full[slot], (seq + 1) | PGPU_SLOT_SKIP);
      seq += NLOAD;
      slot += NLOAD;
      while (slot >= R) slot -= R;
      continue;
    }
    const int64_t t0i = now(pf);
    issue_tile(sc, ci.tile_in_seg, L.ring + (size_t)slot * S);
    PROF_ADD(pf, PGPU_P_L_ISSUE, t0i);
    pend += sc.instrs;
    ++nunpub;
    seq += NLOAD;
    slot += NLOAD;
    while (slot >= R) slot -= R;
    if (seq < ntiles && cursor_advance(p, ci, NLOAD)) load_stage(p, ci.seg, sc);
  }
  PROF_ADD(pf, PGPU_P_L_TOTAL, t_start);
}

// ================================================================================================================
// CONSUMERS
// ================================================================================================================
struct Cons {
  uint32_t* masks;  // [mask_rows][64]
  uint16_t* queue;  // candidate queue [PGPU_CQ_CAP]
  int32_t* klist;   // DENSE: dense-agg keys [PGPU_AGG_LIST] (aliases the queue)
  int32_t* vlist;   // DENSE: dense-agg values [PGPU_AGG_LIST]
  int64_t* acc;     // [MAX_AGGS]  aggregation-only partials of this wave
  int32_t* qtiles;  // [PGPU_CQ_TILES] tile (in segment) of each queue tile index
};

// Scalars of the consumer's current segment (SGPRs); arrays stay behind `sg` and are read with cld.
struct SegState {
  const DevSeg* sg;
  int32_t track;  // HASH: distinct-key bitmap row + 1 (0 = not counted)
  int32_t single_bits;  // DevSeg::single_bits
  int32_t nvstage;      // DevSeg::nvstage
  const DevColumn* cols;
  const int32_t* const* remaps;
  int32_t num_docs, nstage, prog_begin, prog_len, rprog_begin, rprog_len, agg_mode, nreg, reg_col0, reg_col1;
  // fast dense program (DevSeg::fast): per leaf bit width, staged offset, predicate kind / lo / span, negate
  int32_t fast;
  int32_t f_bits[2], f_off[2], f_kind[2], f_neg[2];
  int32_t f_nr[2];  // bit-sliced leaf: number of dict-id ranges (0 = packed layout)
  uint32_t f_r0lo[2], f_r0hi[2];  // its first range (the only one of a RANGE leaf), kept in SGPRs
  int32_t f_sneg[2];
  uint32_t f_lo[2], f_span[2];
};
// numSegmentsMatched (CombineOperatorUtils.java:64-67: a segment counts when its numDocsScanned > 0): a plain store of
// 1 by lane 0 of any wave that matched docs of the segment (same value from every writer, no atomic needed).  `any`
// must be wave-uniform.
FI void mark_seg(const DevParams& p, const SegState& ss, bool any) {
  if (any && lane_id() == 0) p.segany[ss.sg - p.segs] = 1u;
}
FI void load_seg(const DevParams& p, int seg, SegState& ss) {
  const DevSeg* sg = p.segs + seg;
  ss.sg = sg;
  ss.cols = p.cols + cld(&sg->col_begin);
  ss.remaps = p.remaps + cld(&sg->remap_begin);
  ss.num_docs = cld(&sg->num_docs);
  ss.nstage = cld(&sg->nstage);
  ss.prog_begin = cld(&sg->prog_begin);
  ss.prog_len = cld(&sg->prog_len);
  ss.rprog_begin = cld(&sg->rprog_begin);
  ss.rprog_len = cld(&sg->rprog_len);
  ss.agg_mode = cld(&sg->agg_mode);
  ss.nreg = cld(&sg->nreg);
  ss.reg_col0 = cld(&sg->reg_col[0]);
  ss.reg_col1 = cld(&sg->reg_col[1]);
  ss.fast = cld(&sg->fast);
  ss.track = cld(&sg->track);
  ss.single_bits = cld(&sg->single_bits);
  ss.nvstage = cld(&sg->nvstage);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    ss.f_bits[j] = ss.f_off[j] = ss.f_kind[j] = ss.f_neg[j] = 0;
    ss.f_lo[j] = ss.f_span[j] = 0;
    ss.f_nr[j] = 0;
    ss.f_r0lo[j] = ss.f_r0hi[j] = 0;
    ss.f_sneg[j] = 0;
    if (j < ss.fast) {
      ss.f_nr[j] = cld(&sg->f_nr[j]);
      ss.f_r0lo[j] = cld(&sg->f_rng[j][0][0]);
      ss.f_r0hi[j] = cld(&sg->f_rng[j][0][1]);
      ss.f_sneg[j] = cld(&sg->f_sneg[j]);
      const DevInstr* in = p.instrs + ss.prog_begin + cld(&sg->fast_ins[j]);
      ss.f_bits[j] = cld(&in->bits);
      ss.f_off[j] = cld(&in->stage_off);
      ss.f_kind[j] = cld(&in->pred) | (cld(&in->nostat) ? 0x100 : 0);
      ss.f_neg[j] = cld(&in->negate);
      const int32_t lo = cld(&in->lo), hi = cld(&in->hi);
      ss.f_lo[j] = (uint32_t)lo;
      ss.f_span[j] = (ss.f_kind[j] & 0xFF) == PRED_MASK ? (uint32_t)hi : (uint32_t)(hi - lo);
    }
  }
}
FI DevColumn col_of(const SegState& ss, int col) { return cld(ss.cols + col); }

FI uint32_t& mrow(const Cons& c, int s) { return c.masks[s * 64 + lane_id()]; }

// Staged-region pointer of query column `col` in `slot` (nullptr: not staged / slot released).
FI const uint32_t* staged_region(const SegState& ss, const unsigned char* slot, int col) {
  if (!slot) return nullptr;
  for (int j = 0; j < ss.nstage; ++j)
    if (cld(&ss.sg->stage_col[j]) == col) return (const uint32_t*)(slot + cld(&ss.sg->stage_off[j]));
  return nullptr;
}

// Filter program interpreter over mask words.  Leaf evaluation is delegated to a context:
//   TileCtx - word = this lane's 32 consecutive docs of a tile (dense program)
//   DocCtx  - word = this lane's U queued candidate docs (residual program)
struct TileCtx {
  const SegState* ss;
  const unsigned char* slot;
  int tile_in_seg;
  int32_t doc0;
  int32_t lane_doc0;
  uint32_t valid;
};
struct DocCtx {
  const SegState* ss;
  int32_t doc[U];
  uint32_t valid;
};

FI uint32_t leaf_scan(const DevParams& p, const TileCtx& t, const DevInstr& in, uint32_t care, int64_t& dense_bytes) {
  const Pred pr = make_pred(in, p.pool);
  if (in.kind == PGPU_COL_FIXED_BIT) {
    const uint32_t* region = in.stage_off >= 0 && t.slot ? (const uint32_t*)(t.slot + in.stage_off) : nullptr;
    if (!region && lane_id() == 0) dense_bytes += (int64_t)WT * in.bits / 8;
    uint32_t ids[32];
    decode_ids(in.bits, region, in.fwd, t.tile_in_seg, ids);
    return pred_ids(ids, pr) & care;
  }
  // sorted column scanned: per-doc binary search for the care docs
  uint32_t m = 0;
  for (uint32_t left = care; left; left &= left - 1) {
    const int i = __builtin_ctz(left);
    if (eval_pred(pr, sorted_dict_id(in.sorted, in.card, t.lane_doc0 + i))) m |= 1u << i;
  }
  return m;
}
FI uint32_t leaf_scan(const DevParams& p, const DocCtx& t, const DevInstr& in, uint32_t care, int64_t&) {
  const Pred pr = make_pred(in, p.pool);
  uint32_t ids[U];
  gather_ids(colref(in), t.doc, ids);
  uint32_t m = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) m |= (uint32_t)eval_pred(pr, ids[u]) << u;
  return m & care;
}
FI uint32_t leaf_inv(const DevParams& p, const TileCtx& t, const DevInstr& in, uint32_t* scratch) {
  const DevColumn c = col_of(*t.ss, in.col);
  uint32_t m = 0;
  const InvIndex ix{c.inv_dir, c.inv_ct, c.inv_data};
  for (int i = 0; i < in.n; ++i) m |= bitmap_word(ix, t.doc0, (uint32_t)cld(p.pool, in.pool_off + i), scratch);
  return in.negate ? ~m : m;
}
FI uint32_t leaf_inv(const DevParams& p, const DocCtx& t, const DevInstr& in, uint32_t*) {
  const DevColumn c = col_of(*t.ss, in.col);
  uint32_t m = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    bool h = false;
    if ((t.valid >> u) & 1u)
      for (int i = 0; i < in.n && !h; ++i)
        h = bitmap_contains(InvIndex{c.inv_dir, c.inv_ct, c.inv_data}, (uint32_t)cld(p.pool, in.pool_off + i), (uint32_t)t.doc[u]);
    m |= (uint32_t)h << u;
  }
  return in.negate ? ~m : m;
}
// precomputed match bits (raw-value leaves): the lane's 32 docs are one word of the segment's bitmap
FI uint32_t leaf_bits(const TileCtx& t, const DevInstr& in) { return gld(in.fwd, (size_t)(t.doc0 >> 5) + lane_id()); }
FI uint32_t leaf_bits(const DocCtx& t, const DevInstr& in) {
  uint32_t w[U];
#pragma unroll
  for (int u = 0; u < U; ++u) w[u] = gld(in.fwd, (size_t)(t.doc[u] >> 5));
  uint32_t m = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) m |= ((w[u] >> (t.doc[u] & 31)) & 1u) << u;
  return m;
}
// The lane's 32 docs against doc ranges [s, e] inline in the instruction (n <= 4, pgpu_runtime convert_filter).
FI uint32_t inline_ranges_word(const DevInstr& in, int32_t doc0) {
  const int32_t d0 = doc0 + 32 * lane_id(), d1 = d0 + 31;
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k >= in.n) break;
    const int32_t s = (int32_t)in.ids[2 * k], e = (int32_t)in.ids[2 * k + 1];
    if (e >= d0 && s <= d1) {
      const int32_t bs = s > d0 ? s - d0 : 0, be = e < d1 ? e - d0 : 31;
      w |= (0xFFFFFFFFu >> (31 - be)) & (0xFFFFFFFFu << bs);
    }
  }
  return w;
}
FI uint32_t leaf_sorted(const DevParams& p, const TileCtx& t, const DevInstr& in) {
  const uint32_t m = in.n <= 4 ? inline_ranges_word(in, t.doc0) : sorted_ranges_word(p.pool + in.pool_off, in.n, t.doc0);
  return in.negate ? ~m : m;
}
FI uint32_t leaf_sorted(const DevParams& p, const DocCtx& t, const DevInstr& in) {
  uint32_t m = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) m |= (uint32_t)in_sorted_ranges(p.pool + in.pool_off, in.n, t.doc[u]) << u;
  return in.negate ? ~m : m;
}

// The dense program's precomputed-bitmap (BITS) leaves for one tile, loaded together up front (DevSeg::bits_w).
struct PreBits {
  uint32_t w[PGPU_PREBITS];
  FI uint32_t get(int k) const {
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < PGPU_PREBITS; ++j) v = k == j ? w[j] : v;
    return v;
  }
};
FI void prebits_load(const TileCtx& t, int begin, int ss_prog_begin, PreBits& pb) {
  const DevSeg* sg = t.ss->sg;
  const int nb = begin == ss_prog_begin ? cld(&sg->nbits) : 0;
  const size_t wi = (size_t)(t.doc0 >> 5) + lane_id();
#pragma unroll
  for (int j = 0; j < PGPU_PREBITS; ++j) pb.w[j] = j < nb ? gld((const uint32_t*)cld(&sg->bits_w[j]), wi) : 0u;
}
FI void prebits_load(const DocCtx&, int, int, PreBits&) {}
FI void prebits_load_job(const TileCtx& t, const ProgJob* job, PreBits& pb) {
  const int nb = job->nbits;
  const size_t wi = (size_t)(t.doc0 >> 5) + lane_id();
#pragma unroll
  for (int j = 0; j < PGPU_PREBITS; ++j) pb.w[j] = j < nb ? gld(job->bits_w[j], wi) : 0u;
}
FI void prebits_load_job(const DocCtx&, const ProgJob*, PreBits&) {}
FI uint32_t bits_leaf(const TileCtx& t, const DevInstr& in, const PreBits& pb) {
  return in.n >= 0 ? pb.get(in.n) : leaf_bits(t, in);
}
FI uint32_t bits_leaf(const DocCtx& t, const DevInstr& in, const PreBits&) { return leaf_bits(t, in); }

template <class Ctx>
FI uint32_t run_program(const DevParams& p, const Cons& cv, int begin, int len, const Ctx& t, int64_t& scanned,
                        int64_t& dense_bytes, Prof& pf, const ProgJob* job = nullptr) {
  uint32_t* scratch = cv.masks + (p.mask_rows - 1) * 64;
  PreBits pb;
  if (job) prebits_load_job(t, job, pb);  // progbits_kernel: the job's leaf bitmaps (bits_w names its output)
  else prebits_load(t, begin, t.ss->prog_begin, pb);
  int pc = 0;
  while (pc < len) {
    const int64_t tfe = now(pf);
    const DevInstr in = cld(p.instrs + begin + pc);
    if (PROF_ON(pf)) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      PROF_ADD(pf, PGPU_P_C_FETCH, tfe);
    }
    int next = pc + 1;
    const uint32_t care = in.care < 0 ? t.valid : mrow(cv, in.care);
    switch (in.op) {
      case PGPU_I_ALL: mrow(cv, in.dst) = t.valid; break;
      case PGPU_I_EMPTY: mrow(cv, in.dst) = 0u; break;
      case PGPU_I_SCAN: {
        const int n = wave_sum_i32(__popc(care));
        uint32_t m = 0;
        const int64_t tde = now(pf);
        if (n) m = leaf_scan(p, t, in, care, dense_bytes);
        if (PROF_ON(pf)) {
          m = sgpr(m) == 0xdeadbeefu ? m + 1 : m;  // force completion before the timestamp
          PROF_ADD(pf, PGPU_P_C_DECODE, tde);
        }
        if (lane_id() == 0 && !in.nostat) scanned += n;
        mrow(cv, in.dst) = m;
        break;
      }
      case PGPU_I_BITS: {
        if (!in.nostat) {
          const int n = wave_sum_i32(__popc(care));
          if (lane_id() == 0) scanned += n;
        }
        mrow(cv, in.dst) = bits_leaf(t, in, pb) & care;
        break;
      }
      case PGPU_I_INV: mrow(cv, in.dst) = leaf_inv(p, t, in, scratch) & t.valid; break;
      case PGPU_I_SORTED: mrow(cv, in.dst) = leaf_sorted(p, t, in) & t.valid; break;
      case PGPU_I_AND_BEGIN: mrow(cv, in.dst) = care; break;
      case PGPU_I_AND_CHILD: {
        const uint32_t a = mrow(cv, in.dst) & mrow(cv, in.src);
        mrow(cv, in.dst) = a;
        if (!__ballot(a != 0u)) next = in.jump;
        break;
      }
      case PGPU_I_OR_BEGIN: mrow(cv, in.dst) = 0u; break;
      case PGPU_I_OR_CHILD: mrow(cv, in.dst) |= mrow(cv, in.src); break;
      case PGPU_I_NOT: mrow(cv, in.dst) = ~mrow(cv, in.src) & care; break;
      default: break;  // AND_END / OR_END
    }
    pc = next;
  }
  return mrow(cv, 0);
}

// Fast dense program (SegState::fast leaves ANDed, RANGE / MASK predicates on staged columns): evaluated in
// registers -- no instruction fetch, no mask-row LDS round trips.  Same result and scan accounting as
// run_program on the equivalent AND program (a leaf is evaluated only while some doc of the wave survives).
// ---- bit-sliced predicates ----------------------------------------------------------------------------------------
// Bit-sliced tile layout (pgpu_bitslice_kernel): plane k of lane l = bit k of the dict ids of docs [32l, 32l+32),
// doc 32l+i in bit i, at dword k*64 + l of the tile's 256*b bytes.  x < c for a wave-uniform constant c is the
// borrow out of x - c, carried LSB -> MSB through the planes: borrow' = maj(~x_k, c_k, borrow), one v_bitop3 per
// plane for 32 docs (the packed layout needs an extract + compare + pack per doc).  x_k sits in the middle operand,
// so the table (0xB2) is symmetric in the outer two and does not depend on the operand-order convention.
template <int B>
FI uint32_t sliced_lt(const uint32_t (&x)[B], uint32_t c) {
  if (c >> B) return ~0u;  // c = 2^B: past the largest id
  uint32_t br = 0;
#pragma unroll
  for (int k = 0; k < B; ++k) br = __builtin_amdgcn_bitop3_b32((uint32_t)-(int32_t)((c >> k) & 1u), x[k], br, 0xB2);
  return br;
}
template <int B>
FI uint32_t sliced_ranges_b(const uint32_t* region, const DevSeg* sg, int j, int nr, uint32_t lo0, uint32_t hi0) {
  const LAS uint32_t* src = (const LAS uint32_t*)region + opaque_lane();
  uint32_t x[B];
#pragma unroll
  for (int k = 0; k < B; ++k) x[k] = src[64 * k];
  uint32_t m = sliced_lt<B>(x, hi0) & ~sliced_lt<B>(x, lo0);
  for (int r = 1; r < nr; ++r) {
    const uint32_t lo = cld(&sg->f_rng[j][r][0]), hi = cld(&sg->f_rng[j][r][1]);
    m |= sliced_lt<B>(x, hi) & ~sliced_lt<B>(x, lo);
  }
  return m;
}
FI uint32_t sliced_ranges(int bits, const uint32_t* region, const DevSeg* sg, int j, int nr, uint32_t lo0,
                          uint32_t hi0) {
  uint32_t m = 0;
#define SL_CALL(B) m = sliced_ranges_b<B>(region, sg, j, nr, lo0, hi0)
  PGPU_DISPATCH_B(bits, SL_CALL)
#undef SL_CALL
  return m;
}

// The scanned-entries count stays per lane (reduced once per wave at the end) and the empty-tile exit is a ballot:
// a tile costs no cross-lane reduction here.
FI uint32_t fast_filter(const SegState& ss, const TileCtx& t, uint32_t& lane_scanned) {
  uint32_t m = t.valid;
#pragma unroll 1
  for (int j = 0; j < ss.fast; ++j) {
    if (j > 0 && __builtin_amdgcn_ballot_w64(m != 0) == 0) return 0u;
    const int kind_ns = j ? ss.f_kind[1] : ss.f_kind[0];  // predicate kind | nostat << 8
    if (!(kind_ns >> 8)) lane_scanned += __popc(m);
    const int kind = kind_ns & 0xFF;
    const int bits = j ? ss.f_bits[1] : ss.f_bits[0];
    const int off = j ? ss.f_off[1] : ss.f_off[0];
    const uint32_t lo = j ? ss.f_lo[1] : ss.f_lo[0];
    const uint32_t span = j ? ss.f_span[1] : ss.f_span[0];
    const bool neg = (j ? ss.f_neg[1] : ss.f_neg[0]) != 0;
    const int nr = j ? ss.f_nr[1] : ss.f_nr[0];
    if (nr > 0) {
      // bit-sliced leaf: OR of dict-id ranges evaluated on the lane's bit planes (32 docs per word op)
      const uint32_t r = sliced_ranges(bits, (const uint32_t*)(t.slot + off), ss.sg, j, nr,
                                       j ? ss.f_r0lo[1] : ss.f_r0lo[0], j ? ss.f_r0hi[1] : ss.f_r0hi[0]);
      m &= (j ? ss.f_sneg[1] : ss.f_sneg[0]) ? ~r : r;
      continue;
    }
    uint32_t ids[32];
    decode_ids(bits, (const uint32_t*)(t.slot + off), nullptr, t.tile_in_seg, ids);
    uint32_t r = 0;
    if (kind == PRED_MASK) {
      const uint64_t mask = ((uint64_t)span << 32) | lo;
#pragma unroll
      for (int i = 31; i >= 0; --i) r = (r << 1) | ((uint32_t)(mask >> (ids[i] & 63)) & 1u);
    } else {
#pragma unroll
      for (int i = 31; i >= 0; --i) r = (r << 1) | (uint32_t)((ids[i] - lo) < span);
    }
    m &= neg ? ~r : r;
  }
  return m;
}

// ---- aggregation helpers ------------------------------------------------------------------------------------------
// Fold this lane's partial `v` of agg slot `a` into the wave's LDS accumulator (aggregation-only mode).
FI void acc_commit(const Cons& cv, int a, int32_t op, int64_t v) {
  const int64_t r = wave_combine(op, v);
  if (lane_id() == 0) cv.acc[a] = cell_combine(op, cv.acc[a], r);
}
// Per-lane register partials of the first NREG_ACC aggregations (reduced across the wave once, at the end);
// further aggregations fold into the LDS accumulator immediately.
#define NREG_ACC 4
struct LaneAcc {
  int64_t v[NREG_ACC];
};
FI void lacc_add(LaneAcc& la, const Cons& cv, int a, int32_t op, int64_t part) {
  if (a < NREG_ACC) {
#pragma unroll
    for (int k = 0; k < NREG_ACC; ++k)
      if (k == a) la.v[k] = cell_combine(op, la.v[k], part);
  } else {
    acc_commit(cv, a, op, part);
  }
}


template <int MODE>
FI int64_t* table_base(const DevParams& p, const Lds& L) {
  return MODE == PGPU_MODE_LDS ? L.ltab : p.table;
}

// PART mode: region of (partition q, phase-1 workgroup w) = records [part_base, + part_cap).  A workgroup's
// regions are one contiguous block of pblock records, so its record streams stay within a few pages (one region
// per partition would put every store on a different page); sized per partition by part_plan_kernel, or uniform.
FI size_t part_base(const DevParams& p, uint32_t q, uint32_t w) {
  return (size_t)w * p.pblock + (p.poff ? (size_t)p.poff[q] : (size_t)q * (uint32_t)p.rcap);
}
FI uint32_t part_cap(const DevParams& p, uint32_t q) { return p.pcap ? p.pcap[q] : (uint32_t)p.rcap; }

// PART mode: append the records {key[, raw]} of the live entries to this workgroup's region of each key's
// partition.  All N slot reservations (LDS cursor atomics) are issued before the first store.  A full region
// spills the doc straight into the HBM table with atomics: correct, only slower.
FI void part_spill(const DevParams& p, uint32_t key, uint32_t raw) {
  if (p.rec_idbits) raw = gld((const uint32_t*)p.pdict, raw);  // one-word records carry the dict id
  atomicAdd((unsigned long long*)&p.table[key], 1ull);
  for (int a = 0; a < p.nagg; ++a) {
    const DevAgg ag = p.aggs[a];
    if (ag.fn == PGPU_AGG_COUNT) continue;
    cell_atomic(&p.table[(size_t)ag.sec * p.G + key], ag.op, raw_to_cell(raw, ag.vtype, ag.op));
  }
}
template <int N>
FI void part_emit(const DevParams& p, const Lds& L, const uint32_t (&key)[N], const uint32_t (&raw)[N], uint32_t live) {
  uint32_t* cur = (uint32_t*)L.ltab;
  uint32_t slot[N];
#pragma unroll
  for (int r = 0; r < N; ++r) slot[r] = ((live >> r) & 1u) ? atomicAdd(cur + (key[r] >> p.pshift), 1u) : 0u;
  const uint32_t cap = (uint32_t)p.rcap;
  uint32_t spill = 0;
#pragma unroll
  for (int r = 0; r < N; ++r) {
    if (!((live >> r) & 1u)) continue;
    if (slot[r] < cap) {
      const size_t rec = part_base(p, key[r] >> p.pshift, blockIdx.x) + slot[r];
      if (p.rw == 1)
        p.recs[rec] = p.rec_idbits ? ((key[r] & ((1u << p.pshift) - 1)) << p.rec_idbits) | raw[r] : key[r];
      else *(u32x2*)(p.recs + 2 * rec) = u32x2{key[r], raw[r]};
    } else {
      spill |= 1u << r;
    }
  }
  if (spill)
#pragma unroll
    for (int r = 0; r < N; ++r)
      if ((spill >> r) & 1u) part_spill(p, key[r], raw[r]);
}

// GROUP BY with multi-value group columns (p.mv_gmask): every survivor adds to one cell per element of the
// cartesian product of its group columns' values, duplicates included (DictionaryBasedGroupKeyGenerator
// processMultiValue / getIntRawKeys, DictionaryBasedGroupKeyGenerator.java:325-336, 472-544; every aggregation's
// aggregateGroupByMV adds the doc's value once per key, e.g. SumAggregationFunction.java:105-114).  A multi-value
// column's DevColumn holds the values' packed ids in `fwd` and the rows' offsets into them in `sorted`.  Dense
// (LDS / GLOBAL) or hashed key spaces; one lane per doc, table atomics per expanded key.
template <int MODE>
FI void sparse_agg_mv(const DevParams& p, const Lds& L, const SegState& ss, const int32_t (&doc)[U], uint32_t m) {
  constexpr bool HASH = MODE == PGPU_MODE_HASH;
  int64_t* tab = table_base<MODE>(p, L);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!((m >> u) & 1u)) continue;
    const int32_t d = doc[u];
    uint64_t b0 = 0, b1 = 0;  // the single-value columns' part of the key (dense: b0 only; HASH: two key words)
    uint32_t total = 1;
    for (int g = 0; g < p.ngcols; ++g) {
      const DevColumn c = col_of(ss, p.gcols[g]);
      if ((p.mv_gmask >> g) & 1) {
        total *= (uint32_t)(gld(c.sorted, d + 1) - gld(c.sorted, d));
        continue;
      }
      const int32_t dd[1] = {d};
      uint32_t id[1];
      gather_ids(colref(c), dd, id);
      remap_ids(cld(ss.remaps, g), id);
      if (HASH) (g < p.key_split ? b0 : b1) += (uint64_t)id[0] * p.gstride64[g];
      else b0 += (uint64_t)(id[0] * p.gstride[g]);
    }
    for (uint32_t j = 0; j < total; ++j) {
      uint64_t k0 = b0, k1 = b1;
      uint32_t r = j;
      for (int g = 0; g < p.ngcols; ++g) {
        if (!((p.mv_gmask >> g) & 1)) continue;
        const DevColumn c = col_of(ss, p.gcols[g]);
        const int32_t s0 = gld(c.sorted, d), n = gld(c.sorted, d + 1) - s0;
        const int32_t vi[1] = {s0 + (int32_t)(r % (uint32_t)n)};
        r /= (uint32_t)n;
        uint32_t id[1];
        gather_ids(ColRef{c.fwd, nullptr, PGPU_COL_FIXED_BIT, c.bits, c.card}, vi, id);
        remap_ids(cld(ss.remaps, g), id);
        if (HASH) (g < p.key_split ? k0 : k1) += (uint64_t)id[0] * p.gstride64[g];
        else k0 += (uint64_t)(id[0] * p.gstride[g]);
      }
      uint32_t key;
      if (HASH) {
        const uint64_t a0[1] = {k0}, a1[1] = {k1};
        uint32_t slot[1];
        hash_slots(p, a0, a1, 1u, ss.track, slot);
        key = slot[0];
      } else {
        key = (uint32_t)k0;
      }
      atomicAdd((unsigned long long*)&tab[key], 1ull);
      for (int a = 0; a < p.nagg; ++a) {
        const DevAgg ag = p.aggs[a];
        if (ag.fn == PGPU_AGG_COUNT) continue;
        const DevColumn c = col_of(ss, ag.col);
        const int32_t dd[1] = {d};
        uint32_t id[1];
        gather_ids(colref(c), dd, id);
        int64_t v[1];
        gather_cells(c.dict, ag.vtype, ag.op, id, v);
        apply_part(v, ag);
        cell_atomic(tab + (size_t)ag.sec * p.G + key, ag.op, v[0]);
      }
    }
  }
}

// Sparse (per-doc) aggregation of the survivors `m` among this lane's U docs: group key = mixed radix of the
// remapped group ids, COUNT into section 0, every other aggregation gathers its id and dictionary value.
// MV: the kernel may meet multi-value group columns (only the ring kernel: the expansion's loops and gathers would
// cost the self-loading kernels' register budget -- 1.1 KB of scratch and a wave per SIMD -- the runtime never
// sends such a query to them).
template <int MODE, bool MV>
FI void sparse_agg(const DevParams& p, const Lds& L, const Cons& cv, LaneAcc& la, const SegState& ss,
                   const int32_t (&doc)[U], uint32_t m) {
  if constexpr (MV && (MODE == PGPU_MODE_LDS || MODE == PGPU_MODE_GLOBAL || MODE == PGPU_MODE_HASH)) {
    if (p.mv_gmask) {
      sparse_agg_mv<MODE>(p, L, ss, doc, m);
      return;
    }
  }
  uint32_t key[U];
#pragma unroll
  for (int u = 0; u < U; ++u) key[u] = 0;
  if (MODE == PGPU_MODE_HASH) {
    // 64-bit mixed-radix key words, then their hash slots: from here on the slot is the cell index
    uint64_t k0[U], k1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) k0[u] = k1[u] = 0;
    for (int g = 0; g < p.ngcols; ++g) {
      const DevColumn c = col_of(ss, p.gcols[g]);
      const int32_t* remap = cld(ss.remaps, g);
      uint32_t id[U];
      gather_ids(colref(c), doc, id);
#pragma unroll
      for (int u = 0; u < U; ++u) id[u] = ((m >> u) & 1u) ? id[u] : 0u;
      remap_ids(remap, id);
      const uint64_t st = p.gstride64[g];
      if (g < p.key_split) {
#pragma unroll
        for (int u = 0; u < U; ++u) k0[u] += (uint64_t)id[u] * st;
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) k1[u] += (uint64_t)id[u] * st;
      }
    }
    hash_slots(p, k0, k1, m, ss.track, key);
  } else if (MODE != PGPU_MODE_AGG) {
    for (int g = 0; g < p.ngcols; ++g) {
      const DevColumn c = col_of(ss, p.gcols[g]);
      const int32_t* remap = cld(ss.remaps, g);
      uint32_t id[U];
      gather_ids(colref(c), doc, id);
#pragma unroll
      for (int u = 0; u < U; ++u) id[u] = ((m >> u) & 1u) ? id[u] : 0u;
      remap_ids(remap, id);
#pragma unroll
      for (int u = 0; u < U; ++u) key[u] += id[u] * p.gstride[g];
    }
  }
  if (MODE != PGPU_MODE_AGG) {
    if (MODE == PGPU_MODE_PART) {
      uint32_t raw[U];
#pragma unroll
      for (int u = 0; u < U; ++u) raw[u] = 0;
      if (p.pcol >= 0) {
        const DevColumn c = col_of(ss, p.pcol);
        uint32_t id[U];
        gather_ids(colref(c), doc, id);
#pragma unroll
        for (int u = 0; u < U; ++u) id[u] = ((m >> u) & 1u) ? id[u] : 0u;
        if (p.rec_idbits) {
#pragma unroll
          for (int u = 0; u < U; ++u) raw[u] = id[u];
        } else {
          gather_raw(c.dict, id, raw);
        }
      }
      part_emit(p, L, key, raw, m);
      return;
    }
    int64_t* tab = table_base<MODE>(p, L);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if ((m >> u) & 1u) atomicAdd((unsigned long long*)&tab[key[u]], 1ull);
  }
  for (int a = 0; a < p.nagg; ++a) {
    const DevAgg ag = p.aggs[a];
    if (ag.fn == PGPU_AGG_COUNT) continue;
    const DevColumn c = col_of(ss, ag.col);
    uint32_t id[U];
    gather_ids(colref(c), doc, id);
#pragma unroll
    for (int u = 0; u < U; ++u) id[u] = ((m >> u) & 1u) ? id[u] : 0u;
    if (MODE == PGPU_MODE_AGG && (ag.op == PGPU_RED_MIN_I64 || ag.op == PGPU_RED_MAX_I64) && c.kind != PGPU_COL_RAW) {
      // sorted dictionary + order-preserving cell key: one value gather per lane, at the extreme live id
      const bool is_min = ag.op == PGPU_RED_MIN_I64;
      uint32_t best = is_min ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if ((m >> u) & 1u) best = is_min ? min(best, id[u]) : max(best, id[u]);
      int64_t part = sec_identity(ag.op);
      if (m) {
        const uint32_t idx[1] = {best};
        int64_t v1[1];
        gather_cells(c.dict, ag.vtype, ag.op, idx, v1);
        part = v1[0];
      }
      lacc_add(la, cv, a, ag.op, part);
      continue;
    }
    int64_t v[U];
    gather_cells(c.dict, ag.vtype, ag.op, id, v);
    apply_part(v, ag);
    if (MODE == PGPU_MODE_AGG) {
      int64_t part = sec_identity(ag.op);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if ((m >> u) & 1u) part = cell_combine(ag.op, part, v[u]);
      lacc_add(la, cv, a, ag.op, part);
    } else {
      int64_t* tab = table_base<MODE>(p, L) + (size_t)ag.sec * p.G;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if ((m >> u) & 1u) cell_atomic(&tab[key[u]], ag.op, v[u]);
    }
  }
}

// 32-B sectors of a b-bit column first touched by `doc` after `prev_doc` (ascending entries; stats pass only).
FI int new_sectors(uint32_t b, int32_t doc, bool live, int32_t prev_doc, bool prev_live) {
  if (!live) return 0;
  const int64_t s0 = ((int64_t)doc * b) >> 8, s1 = ((int64_t)(doc + 1) * b - 1) >> 8;
  int64_t from = s0;
  if (prev_live) {
    const int64_t pe = ((int64_t)(prev_doc + 1) * b - 1) >> 8;
    if (pe + 1 > from) from = pe + 1;
  }
  return s1 >= from ? (int)(s1 - from + 1) : 0;
}

// Flush the candidate queue (doc ids of one segment, ascending): residual filter per doc, then sparse aggregation.
template <int MODE, int NCONS, bool MV = false>
FI void flush_queue(const DevParams& p, const Lds& L, const Cons& cv, LaneAcc& la, const SegState& ss, int n,
                    int64_t& matched, int64_t& scanned, int64_t& sector_bytes, int64_t& dense_bytes, Prof& pf) {
  const int lane = lane_id();
  const bool stats = p.flags & PGPU_FLAG_STATS;
  wave_sync();
  for (int base = 0; base < n; base += 64 * U) {
    DocCtx d;
    d.ss = &ss;
    d.valid = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * 64 + lane;
      const bool ok = e < n;
      const uint32_t q = ok ? (uint32_t)cv.queue[e] : 0u;
      d.doc[u] = ok ? cv.qtiles[q >> 11] * WT + (int)(q & (WT - 1)) : 0;
      d.valid |= (uint32_t)ok << u;
    }
    uint32_t m = d.valid;
    if (ss.rprog_len > 0) m = run_program(p, cv, ss.rprog_begin, ss.rprog_len, d, scanned, dense_bytes, pf);
    const int nm = wave_sum_i32(__popc(m));
    if (lane == 0) matched += nm;
    mark_seg(p, ss, nm != 0);
    if (stats) {
      // 32-B sectors of every gathered forward index: residual scan columns over the candidates,
      // aggregation / group columns over the survivors
      int sec = 0;
      for (int pc = 0; pc < ss.rprog_len; ++pc) {
        const DevInstr in = cld(p.instrs + ss.rprog_begin + pc);
        if (in.op != PGPU_I_SCAN || in.kind != PGPU_COL_FIXED_BIT) continue;
        const uint32_t b = (uint32_t)in.bits;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int32_t pd = __shfl_up(d.doc[u], 1, 64);
          sec += new_sectors(b, d.doc[u], (d.valid >> u) & 1u, pd, lane > 0);
        }
      }
      if (nm && ss.agg_mode == PGPU_AM_SPARSE) {
        for (int k = 0; k < p.ncols; ++k) {
          bool used = false;
          for (int g = 0; g < p.ngcols; ++g) used |= p.gcols[g] == k;
          for (int a = 0; a < p.nagg; ++a) used |= p.aggs[a].fn != PGPU_AGG_COUNT && p.aggs[a].col == k;
          if (!used) continue;
          const DevColumn c = col_of(ss, k);
          if (c.kind != PGPU_COL_FIXED_BIT && c.kind != PGPU_COL_RAW) continue;
          const uint32_t b = c.kind == PGPU_COL_RAW ? (c.dict_type == PGPU_INT || c.dict_type == PGPU_FLOAT ? 32u : 64u)
                                                   : (uint32_t)c.bits;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const bool live = (m >> u) & 1u;
            const int32_t pd = __shfl_up(d.doc[u], 1, 64);
            const bool pl = lane > 0 && __shfl_up((int)live, 1, 64);
            sec += new_sectors(b, d.doc[u], live, pd, pl);
          }
        }
      }
      const int tot = wave_sum_i32(sec);
      if (lane == 0) sector_bytes += 32ll * tot;
    }
    if (nm && ss.agg_mode == PGPU_AM_SPARSE) sparse_agg<MODE, MV>(p, L, cv, la, ss, d.doc, m);
  }
  // a wait hipcc sees: its scoreboard then holds no pending gather, so it does not guard the next tile's LDS reads
  // with vmcnt(0) (which would also drain the direct kernel's prefetched tiles)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  wave_sync();
}

// Dense aggregation of this lane's matched docs `mm` of the tile from decoded ids (registers or the held slot).
// Per half tile (16 docs per lane): compact keys and ids of the matched docs into the LDS lists, then gather
// dictionary values with full lanes (4 rounds in flight) and fold them into partials / table cells.
// Aggregation-only, every aggregated column already in registers: the whole tile's matched ids are compacted into
// the consumer's 2048-entry list (klist + vlist are contiguous), so all of the tile's dictionary gathers are in
// flight together -- one gather latency per tile instead of one per half.
FI bool agg_cols_in_regs(const DevParams& p, const SegState& ss) {
  if (ss.nreg <= 0) return false;
  for (int a = 0; a < p.nagg; ++a) {
    const DevAgg ag = p.aggs[a];
    if (ag.fn == PGPU_AGG_COUNT) continue;
    if (ag.col != ss.reg_col0 && !(ss.nreg > 1 && ag.col == ss.reg_col1)) return false;
  }
  return true;
}
FI void dense_agg_tile(const DevParams& p, const Cons& cv, LaneAcc& la, const SegState& ss, uint32_t mm,
                       const uint32_t (&ra)[32], const uint32_t (&rb)[32]) {
  const int lane = lane_id();
  const int cnt = __popc(mm);
  const int nt = wave_sum_i32(cnt);
  const int off = wave_excl_scan(cnt);
  int32_t* list = cv.klist;  // [2 * PGPU_AGG_LIST] >= PGPU_WT
  for (int a = 0; a < p.nagg; ++a) {
    const DevAgg ag = p.aggs[a];
    if (ag.fn == PGPU_AGG_COUNT) continue;
    const bool r0 = ag.col == ss.reg_col0;
    const DevColumn c = col_of(ss, ag.col);
    if ((ag.op == PGPU_RED_MIN_I64 || ag.op == PGPU_RED_MAX_I64) && c.kind != PGPU_COL_RAW) {
      // dictionaries are sorted ascending and the MIN / MAX cell key is order-preserving, so the extreme value
      // sits at the extreme dict id: reduce the ids in registers, then gather one value per lane
      const bool is_min = ag.op == PGPU_RED_MIN_I64;
      uint32_t best = is_min ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const uint32_t id = r0 ? ra[i] : rb[i];
        if (lane_bit(mm, i)) best = is_min ? min(best, id) : max(best, id);
      }
      int64_t part = sec_identity(ag.op);
      if (mm) {  // lanes without survivors keep the identity (and never index with the sentinel id)
        const uint32_t idx[1] = {best};
        int64_t v[1];
        gather_cells(c.dict, ag.vtype, ag.op, idx, v);
        part = v[0];
      }
      lacc_add(la, cv, a, ag.op, part);  // wave-uniform call: acc_commit reduces across the wave
      continue;
    }
    {
      int k = off;
#pragma unroll
      for (int i = 0; i < 32; ++i)
        if (lane_bit(mm, i)) list[k++] = (int32_t)(r0 ? ra[i] : rb[i]);
    }
    wave_sync();
    int64_t part = sec_identity(ag.op);
    for (int b0 = 0; b0 < nt; b0 += 64 * 8) {
      uint32_t idx[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int e = b0 + lane + 64 * r;
        idx[r] = e < nt ? (uint32_t)list[e] : 0u;
      }
      int64_t v[8];
      gather_cells(c.dict, ag.vtype, ag.op, idx, v);
      apply_part(v, ag);
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (b0 + lane + 64 * r < nt) part = cell_combine(ag.op, part, v[r]);
    }
    lacc_add(la, cv, a, ag.op, part);
    wave_sync();
  }
}

template <int MODE>
FI void dense_agg(const DevParams& p, const Lds& L, const Cons& cv, LaneAcc& la, const SegState& ss, const TileCtx& t,
                  uint32_t mm, const uint32_t (&ra)[32], const uint32_t (&rb)[32]) {
  if (MODE == PGPU_MODE_AGG && agg_cols_in_regs(p, ss)) {
    dense_agg_tile(p, cv, la, ss, mm, ra, rb);
    return;
  }
  const int lane = lane_id();
  int32_t* klist = cv.klist;  // keys   [PGPU_AGG_LIST]
  int32_t* vlist = cv.vlist;  // values [PGPU_AGG_LIST]
#pragma unroll 1
  for (int h = 0; h < 2; ++h) {
    const uint32_t hm = (mm >> (16 * h)) & 0xFFFFu;
    const int cnt = __popc(hm);
    const int nh = wave_sum_i32(cnt);
    if (nh == 0) continue;
    const int off = wave_excl_scan(cnt);
    // operand list: group columns first (keys), then the non-COUNT aggregations
    uint32_t key[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) key[i] = 0;
    const int nops = (MODE != PGPU_MODE_AGG ? p.ngcols : 0) + p.nagg;
    for (int op = 0; op < nops; ++op) {
      const bool is_key = MODE != PGPU_MODE_AGG && op < p.ngcols;
      const int ai = op - (MODE != PGPU_MODE_AGG ? p.ngcols : 0);
      DevAgg ag;
      int col;
      if (is_key) {
        col = p.gcols[op];
      } else {
        ag = p.aggs[ai];
        if (ag.fn == PGPU_AGG_COUNT) continue;
        if (MODE == PGPU_MODE_PART && !ag.emit) continue;  // derived in phase 2 from the emitted column
        col = ag.col;
      }
      uint32_t lo[16];
      {
        uint32_t ids[32];
        if (ss.nreg > 0 && col == ss.reg_col0) {
#pragma unroll
          for (int i = 0; i < 32; ++i) ids[i] = ra[i];
        } else if (ss.nreg > 1 && col == ss.reg_col1) {
#pragma unroll
          for (int i = 0; i < 32; ++i) ids[i] = rb[i];
        } else {
          const DevColumn c = col_of(ss, col);
          column_ids(c.kind, c.bits, staged_region(ss, t.slot, col), c.fwd, t.tile_in_seg, ids);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) lo[i] = h ? ids[16 + i] : ids[i];
      }
      if (is_key) {
        const int32_t* remap = cld(ss.remaps, op);
        if (remap) {
#pragma unroll
          for (int i = 0; i < 16; ++i) lo[i] = lane_bit(hm, i) ? lo[i] : 0u;
          remap_ids(remap, lo);
        }
        const uint32_t st = p.gstride[op];
#pragma unroll
        for (int i = 0; i < 16; ++i) key[i] += lo[i] * st;
        if (op == p.ngcols - 1) {
          int k = off;
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (lane_bit(hm, i)) klist[k++] = (int32_t)key[i];
          wave_sync();
          if (MODE == PGPU_MODE_PART) {
            if (p.pcol < 0)
              for (int r0 = 0; r0 * 64 < nh; r0 += 8) {
                uint32_t kk[8], raw[8], live = 0;
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                  const int e = lane + 64 * (r0 + r);
                  kk[r] = e < nh ? (uint32_t)klist[e] : 0u;
                  raw[r] = 0u;
                  live |= (uint32_t)(e < nh) << r;
                }
                part_emit(p, L, kk, raw, live);
              }
          } else {
            int64_t* tab = table_base<MODE>(p, L);
            for (int e = lane; e < nh; e += 64) atomicAdd((unsigned long long*)&tab[(uint32_t)klist[e]], 1ull);
          }
        }
        continue;
      }
      const DevColumn c = col_of(ss, col);
      {
        int k = off;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (lane_bit(hm, i)) vlist[k++] = (int32_t)lo[i];
      }
      wave_sync();
      if (MODE == PGPU_MODE_PART) {
        for (int r0 = 0; r0 * 64 < nh; r0 += 8) {
          uint32_t idx[8], raw[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int e = lane + 64 * (r0 + r);
            idx[r] = e < nh ? (uint32_t)vlist[e] : 0u;
          }
          if (p.rec_idbits) {
#pragma unroll
            for (int r = 0; r < 8; ++r) raw[r] = idx[r];
          } else {
            gather_raw(c.dict, idx, raw);
          }
          uint32_t kk[8], live = 0;
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int e = lane + 64 * (r0 + r);
            kk[r] = e < nh ? (uint32_t)klist[e] : 0u;
            live |= (uint32_t)(e < nh) << r;
          }
          part_emit(p, L, kk, raw, live);
        }
        wave_sync();
        continue;
      }
      int64_t part = sec_identity(ag.op);
      int64_t* tab = table_base<MODE>(p, L) + (size_t)ag.sec * p.G;
      for (int r0 = 0; r0 * 64 < nh; r0 += 8) {
        uint32_t idx[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int e = lane + 64 * (r0 + r);
          idx[r] = e < nh ? (uint32_t)vlist[e] : 0u;
        }
        int64_t v[8];
        gather_cells(c.dict, ag.vtype, ag.op, idx, v);
        apply_part(v, ag);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int e = lane + 64 * (r0 + r);
          if (e < nh) {
            if (MODE == PGPU_MODE_AGG) part = cell_combine(ag.op, part, v[r]);
            else cell_atomic(&tab[(uint32_t)klist[e]], ag.op, v[r]);
          }
        }
      }
      if (MODE == PGPU_MODE_AGG) lacc_add(la, cv, ai, ag.op, part);
      wave_sync();
    }
    wave_sync();
  }
}

struct Stats {
  int64_t matched, scanned, sector_bytes, dense_bytes;
};

template <int MODE, int DENSE>
FI Stats consumer(const DevParams& p, const Lds& L, int cidx, int t0, int ntiles, Prof& pf) {
  constexpr int NCONS = PGPU_NCONS_OF(DENSE);
  const int64_t t_start = now(pf);
  const int lane = lane_id();
  const int R = p.ring_slots, S = p.slot_bytes;
  Cons cv;
  {
    unsigned char* base = L.cons + (size_t)cidx * p.cons_bytes;
    cv.masks = (uint32_t*)base;
    cv.queue = (uint16_t*)(base + p.mask_rows * 256);
    cv.klist = (int32_t*)(base + p.mask_rows * 256);
    cv.vlist = cv.klist + PGPU_AGG_LIST;
    cv.acc = (int64_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(DENSE));
    cv.qtiles = (int32_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(DENSE) + PGPU_CONS_ACC_BYTES);
  }
  if (MODE == PGPU_MODE_AGG && lane < PGPU_MAX_AGGS) cv.acc[lane] = lane < p.nagg ? sec_identity(p.aggs[lane].op) : 0;
  wave_sync();
  int64_t matched = 0, scanned = 0, sector_bytes = 0, dense_bytes = 0;
  uint32_t lane_scanned = 0;  // fast-path scanned entries, per lane (reduced at the end)
  LaneAcc la;
#pragma unroll
  for (int k = 0; k < NREG_ACC; ++k) la.v[k] = k < p.nagg ? sec_identity(p.aggs[k].op) : 0;
  int qn = 0;  // candidate-queue entries (all of segment `ss`)
  int qt = 0;  // tiles in the queue's tile table (cv.qtiles)
  SegState ss;
  int cseg = -1;
  Cursor cur;
  cur.seg = 0;
  cur.tile_in_seg = 0;
  cur.ntiles = 0;
  int prev = -1, slot_i = 0;
  // Tiles are claimed dynamically, in order, from the workgroup's LDS counter: a consumer busy with a queue
  // flush holds no claimed tile, so it never blocks the ring slot the loaders need next.
  for (;;) {
    if (qn && (qn >= PGPU_CQ_FLUSH || qt >= PGPU_CQ_TILES)) {
      const int64_t tq = now(pf);
      flush_queue<MODE, NCONS, true>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
      PROF_ADD(pf, PGPU_P_C_FLUSH, tq);
      qn = qt = 0;
    }
    int claim = 0;
    if (lane == 0) claim = __hip_atomic_fetch_add(L.icnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const int seq = __builtin_amdgcn_readlane(claim, 0);
    const bool end = seq >= ntiles;
    if (!end) {
      if (prev < 0) {
        cur = cursor_at(p, t0 + seq);
        slot_i = seq % R;
      } else {
        cursor_advance(p, cur, seq - prev);
        slot_i += seq - prev;
        while (slot_i >= R) slot_i -= R;
      }
      prev = seq;
    }
    const bool segchg = !end && cur.seg != cseg;
    if (qn && (end || segchg)) {
      const int64_t tq = now(pf);
      flush_queue<MODE, NCONS, true>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
      PROF_ADD(pf, PGPU_P_C_FLUSH, tq);
      qn = qt = 0;
    }
    if (end) break;
    if (segchg) {
      cseg = cur.seg;
      load_seg(p, cseg, ss);
    }
    unsigned char* slot = L.ring + (size_t)slot_i * S;
    const int64_t tw = now(pf);
    // poll with back-off: the scalar ALU is shared by every wave of the CU
    int fl;
    for (int nap = 0; ((fl = flag_load(&L.full[slot_i])) & ~PGPU_SLOT_SKIP) != seq + 1; nap = nap < 3 ? nap + 1 : 3) {
      if (nap == 0) __builtin_amdgcn_s_sleep(1);
      else if (nap == 1) __builtin_amdgcn_s_sleep(2);
      else if (nap == 2) __builtin_amdgcn_s_sleep(4);
      else __builtin_amdgcn_s_sleep(8);
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    PROF_ADD(pf, PGPU_P_C_FULL, tw);
    if (fl & PGPU_SLOT_SKIP) {  // cancelled: nothing was loaded into the slot; hand it back
      if (lane == 0) flag_store(&L.freef[slot_i], seq + 1);
      continue;
    }
    const int64_t tf = now(pf);
#ifdef PGPU_PROFILE_BUILD
    if (pf.on) pf.t[PGPU_P_C_TILES] += 1;
#endif

    TileCtx t;
    t.ss = &ss;
    t.slot = slot;
    t.tile_in_seg = cur.tile_in_seg;
    t.doc0 = cur.tile_in_seg * WT;
    t.lane_doc0 = t.doc0 + 32 * lane;
    {
      const int ndocs = min(WT, ss.num_docs - t.doc0);
      const int rem = ndocs - 32 * lane;
      t.valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
      if (p.flags & PGPU_FLAG_STATS)
        for (int j = 0; j < ss.nstage; ++j) {
          const int b = col_of(ss, cld(&ss.sg->stage_col[j])).bits;
          if (lane == 0) dense_bytes += ((int64_t)ndocs * b + 7) / 8;
        }
    }
    uint32_t mm = t.valid;
    if (ss.fast) mm = fast_filter(ss, t, lane_scanned);
    else if (ss.prog_len > 0) mm = run_program(p, cv, ss.prog_begin, ss.prog_len, t, scanned, dense_bytes, pf);
    const int nm = wave_sum_i32(__popc(mm));
    PROF_ADD(pf, PGPU_P_C_FILTER, tf);
    const int64_t ta = now(pf);
    const bool dense = DENSE && ss.agg_mode == PGPU_AM_DENSE && nm;
    uint32_t ra[32], rb[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) ra[i] = rb[i] = 0;
    if (DENSE && dense) {
      // copy up to two aggregation / group columns to registers, then hand the slot back to the loader
      for (int j = 0; j < ss.nreg; ++j) {
        const int col = j == 0 ? ss.reg_col0 : ss.reg_col1;
        const DevColumn c = col_of(ss, col);
        uint32_t ids[32];
        column_ids(c.kind, c.bits, staged_region(ss, slot, col), c.fwd, t.tile_in_seg, ids);
#pragma unroll
        for (int i = 0; i < 32; ++i) {
          if (j == 0) ra[i] = ids[i];
          else rb[i] = ids[i];
        }
      }
    }
    const bool hold = dense && ss.nreg < 0;
    if (!hold) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) flag_store(&L.freef[slot_i], seq + 1);
      t.slot = nullptr;
    }
    if (nm) {
      if (DENSE && dense) {
        if (lane == 0) matched += nm;
        mark_seg(p, ss, true);
        dense_agg<MODE>(p, L, cv, la, ss, t, mm, ra, rb);
      } else if (ss.rprog_len == 0 && ss.agg_mode == PGPU_AM_COUNT) {
        if (lane == 0) matched += nm;
        mark_seg(p, ss, true);
      } else if (qn + nm <= PGPU_CQ_CAP) {
        // queue the candidates (ascending: lane order, then bit order) as queue-tile index << 11 | doc in tile
        if (lane == 0) cv.qtiles[qt] = cur.tile_in_seg;
        const uint32_t tag = (uint32_t)qt << 11;
        ++qt;
        int k = qn + wave_excl_scan(__popc(mm));
        for (uint32_t left = mm; left; left &= left - 1)
          cv.queue[k++] = (uint16_t)(tag | (uint32_t)(32 * lane + __builtin_ctz(left)));
        qn += nm;
      } else {
        // a dense tile does not fit behind the queued entries: flush them, then queue and flush the tile in two
        // halves (lanes 0-31, 32-63: <= 1024 entries each)
        if (qn) {
          flush_queue<MODE, NCONS, true>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
          qn = qt = 0;
        }
        if (lane == 0) cv.qtiles[0] = cur.tile_in_seg;
        for (int half = 0; half < 2; ++half) {
          const uint32_t mh = (lane >> 5) == half ? mm : 0u;
          const int nh = wave_sum_i32(__popc(mh));
          if (nh == 0) continue;
          int k = wave_excl_scan(__popc(mh));
          for (uint32_t left = mh; left; left &= left - 1)
            cv.queue[k++] = (uint16_t)(32 * lane + __builtin_ctz(left));
          flush_queue<MODE, NCONS, true>(p, L, cv, la, ss, nh, matched, scanned, sector_bytes, dense_bytes, pf);
        }
      }
    }
    if (hold) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) flag_store(&L.freef[slot_i], seq + 1);
    }
    PROF_ADD(pf, PGPU_P_C_AGG, ta);
  }
  PROF_ADD(pf, PGPU_P_C_TOTAL, t_start);
  {
    const int64_t ls = wave_sum_i64((int64_t)lane_scanned);
    if (lane == 0) scanned += ls;
  }
  if (MODE == PGPU_MODE_AGG) {
#pragma unroll
    for (int a = 0; a < NREG_ACC; ++a)
      if (a < p.nagg && p.aggs[a].fn != PGPU_AGG_COUNT) acc_commit(cv, a, p.aggs[a].op, la.v[a]);
  }
  Stats s;
  s.matched = matched;
  s.scanned = scanned;
  s.sector_bytes = sector_bytes;
  s.dense_bytes = dense_bytes;
  return s;
}

// ================================================================================================================
// DIRECT (self-loading) variant: every staged column is a bit-sliced fast leaf and no segment aggregates densely
// (PGPU_AM_COUNT / PGPU_AM_SPARSE).  Such tiles are small (256 * b bytes) and their filter is a handful of VALU ops
// per 32 docs, so the loader -> ring -> consumer hand-off (flag polls, per-tile cursor work on a shared scalar unit)
// would dominate.  Here each wave streams its own tiles: it DMAs tile i+1 into one of two private LDS slots, waits
// for tile i with a counted vmcnt and filters it; 256-thread workgroups, several per CU.  The DMAs are issued from
// inline asm so that hipcc does not guard the wave's other LDS accesses with vmcnt(0) (in-order completion keeps
// hipcc's own counted waits conservative).
// ================================================================================================================
#define PGPU_DIRECT_THREADS 256
#define PGPU_DIRECT_WAVES (PGPU_DIRECT_THREADS / 64)
#ifndef PGPU_DIRECT_MIN_WAVES
#define PGPU_DIRECT_MIN_WAVES 5  // waves per SIMD the register budget must allow (<= 96 VGPRs; the other modes
                                 // keep 4: their accumulators / table paths would spill to scratch)
#endif

// saddr form: wave-uniform base in an SGPR pair + this lane's byte offset (a VGPR that lives for the whole kernel),
// so no VGPR is written right before the DMA -- a freshly written address VGPR draws a conservative vmcnt(0) from
// hipcc, which would drain this wave's prefetches.
FI void glds16_asm(uint32_t voff, const void* sbase, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_dst));
}
// Non-temporal form (PGPU_FLAG_NT): once-read tile bytes need not stay in L2 (MI355X_MICROARCH.md nt-weights).
FI void glds16_asm_nt(uint32_t voff, const void* sbase, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_dst));
}
FI const void* uniform_ptr(const void* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = (uint32_t)sgpr((int)(uint32_t)v), hi = (uint32_t)sgpr((int)(uint32_t)(v >> 32));
  return (const void*)(((uint64_t)hi << 32) | lo);
}
// The tile's staged (bit-sliced, linear) regions into `slot`: 16 B per lane, 1 KiB per instruction.
FI void issue_tile_direct(const StageCache& sc, int tile_in_seg, unsigned char* slot, uint32_t voff16, bool nt) {
  const int lane = lane_id();
#pragma unroll
  for (int j = 0; j < PGPU_MAX_STAGE; ++j) {
    if (j >= sc.nst) break;
    const int b = sc.bits[j];
    const char* base = sc.fwd[j] + (size_t)tile_in_seg * 256 * b;
    const uint32_t dst = sgpr((int)lds_off(slot + sc.off[j]));
    const int ninstr = (b + 3) >> 2;
    for (int k = 0; k < ninstr; ++k) {
      if (64 * k + lane < 16 * b) {
        if (nt) glds16_asm_nt(voff16, uniform_ptr(base + 1024 * k), dst + 1024 * k);
        else glds16_asm(voff16, uniform_ptr(base + 1024 * k), dst + 1024 * k);
      }
    }
  }
}

// PGPU_AM_SLICED (aggregation-only): after the filter, each aggregated column's planes for the tile are loaded
// straight into VGPRs from its bit-sliced copy (plane k of lane l at dword (tile * B + k) * 64 + l: one coalesced
// 256-B row per plane, so the column streams at the filter's rate instead of one 128-B line per gathered value),
// and each matched doc's id is read bit by bit from the lane's planes.  Ids of columns of <= 16 bits go to the
// wave's LDS queue (the candidate queue's space, unused here: one sub-queue per column) and their dictionary values
// are gathered in batches when it fills (many gathers in flight per lane); wider columns gather per tile.
template <int B>
FI void sliced_load(const uint32_t* sl, int tile, uint32_t (&x)[B]) {
  const uint32_t* src = sl + (size_t)tile * 64 * B + lane_id();
#pragma unroll
  for (int k = 0; k < B; ++k) x[k] = __builtin_nontemporal_load(src + 64 * k);
}
template <int B>
FI uint32_t sliced_id(const uint32_t (&x)[B], int i) {
  uint32_t id = 0;
#pragma unroll
  for (int k = 0; k < B; ++k) id |= ((x[k] >> i) & 1u) << k;
  return id;
}
// ids of this lane's matched docs of column c into queue q at [at, ...)
template <int B>
FI void sliced_enqueue_b(const DevColumn& c, int tile, uint32_t mm, uint16_t* q, int at) {
  uint32_t x[B];
  sliced_load<B>(c.sliced, tile, x);
  for (uint32_t left = mm; left; left &= left - 1) q[at++] = (uint16_t)sliced_id<B>(x, __builtin_ctz(left));
}
// Columns queued by the wave (<= 2 non-COUNT aggregations over <= 16-bit columns) and each one's queue capacity.
FI int sliced_queued(const DevParams& p, const SegState& ss) {
  int n = 0;
  for (int a = 0; a < p.nagg; ++a) {
    if (p.aggs[a].fn == PGPU_AGG_COUNT) continue;
    if (col_of(ss, p.aggs[a].col).bits > 16) return 0;
    ++n;
  }
  return n <= 2 ? n : 0;
}
// Gather and fold the queued ids' values (segment `ss`'s dictionaries), eight per lane in flight.
FI void sliced_flush(const DevParams& p, const Cons& cv, LaneAcc& la, const SegState& ss, int n) {
  if (n <= 0) return;
  wave_sync();
  const int cap = PGPU_CQ_CAP / 2;
  int slot = 0;
  for (int a = 0; a < p.nagg; ++a) {
    const DevAgg ag = p.aggs[a];
    if (ag.fn == PGPU_AGG_COUNT) continue;
    const DevColumn c = col_of(ss, ag.col);
    const uint16_t* q = cv.queue + slot++ * cap;
    int64_t part = sec_identity(ag.op);
    for (int base = 0; base < n; base += 8 * 64) {
      uint32_t idx[8];
      uint32_t live = 0;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int e = base + r * 64 + lane_id();
        idx[r] = e < n ? (uint32_t)q[e] : 0u;
        live |= (uint32_t)(e < n) << r;
      }
      int64_t v[8];
      gather_cells(c.dict, ag.vtype, ag.op, idx, v);
      apply_part(v, ag);
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if ((live >> r) & 1u) part = cell_combine(ag.op, part, v[r]);
    }
    lacc_add(la, cv, a, ag.op, part);
  }
  wave_sync();
}
// Aggregations answered from the value planes (bit-sliced index): SUM of whole int64 cells, MIN, MAX.
#define BSI_MAXB 24  // value planes held in VGPRs per tile (wider values: the id path; the direct kernel stays spill-free)
FI bool bsi_agg(const DevAgg& ag, const DevColumn& c) {
  return c.vsliced && c.vbits >= 1 && c.vbits <= BSI_MAXB &&
         ((ag.op == PGPU_RED_SUM_I64 && ag.part == 0) || ag.op == PGPU_RED_MIN_I64 || ag.op == PGPU_RED_MAX_I64);
}
template <int NB>
FI void bsi_fold(const Cons& cv, LaneAcc& la, const DevColumn& c, const DevAgg& ag, int a, const uint32_t (&x)[NB],
                 uint32_t mm) {
  const int vb = c.vbits;
  int64_t part;
  if (ag.op == PGPU_RED_SUM_I64) {
    uint64_t u = 0;
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (k < vb) u += (uint64_t)__popc(x[k] & mm) << k;
    part = (int64_t)u + (int64_t)__popc(mm) * c.vmin;
  } else {
    // MSB first: keep the matched docs whose value has the bit set (MAX) / clear (MIN) while any does
    const bool mx = ag.op == PGPU_RED_MAX_I64;
    uint32_t cand = mm, u = 0;
#pragma unroll
    for (int k = NB - 1; k >= 0; --k) {
      if (k >= vb) continue;
      const uint32_t t = cand & (mx ? x[k] : ~x[k]);
      if (t) cand = t;
      if ((t != 0) == mx) u |= 1u << k;
    }
    part = mm ? c.vmin + (int64_t)u : sec_identity(ag.op);
  }
  lacc_add(la, cv, a, ag.op, part);
}
template <int NB>
FI void bsi_load(const DevColumn& c, int tile, uint32_t (&x)[NB]) {
  const int vb = c.vbits;
  const uint32_t* src = c.vsliced + (size_t)tile * 64 * vb + lane_id();
#pragma unroll
  for (int k = 0; k < NB; ++k) x[k] = k < vb ? __builtin_nontemporal_load(src + 64 * k) : 0u;
}
FI void bsi_tile(const Cons& cv, LaneAcc& la, const DevColumn& c, const DevAgg& ag, int a, int tile, uint32_t mm) {
  uint32_t x[BSI_MAXB];
  bsi_load<BSI_MAXB>(c, tile, x);
  bsi_fold<BSI_MAXB>(cv, la, c, ag, a, x, mm);
}
// Value planes staged in the slot (DevSeg::nvstage: the self-loading kernel DMAs them with the tile's filter planes,
// so one counted vmcnt wait covers both -- a plain load issued behind the DMAs and used at once would wait for all of
// them, vmcnt retiring in order)
FI void bsi_tile_staged(const DevParams& p, const Cons& cv, LaneAcc& la, const SegState& ss, const unsigned char* slot,
                        uint32_t mm) {
  for (int a = 0; a < p.nagg; ++a) {
    if (p.aggs[a].fn == PGPU_AGG_COUNT) continue;
    const DevAgg ag = p.aggs[a];
    const int j = cld(&ss.sg->vstage_col[0]) == ag.col ? 0 : 1;
    const uint32_t* pl = (const uint32_t*)(slot + cld(&ss.sg->vstage_off[j])) + lane_id();
    const DevColumn c = col_of(ss, ag.col);
    const int vb = c.vbits;
    int64_t part;
    if (ag.op == PGPU_RED_SUM_I64) {  // planes read as they are folded (no 24-register plane array)
      uint64_t u = 0;
      for (int k = 0; k < vb; ++k) u += (uint64_t)__popc(pl[64 * k] & mm) << k;
      part = (int64_t)u + (int64_t)__popc(mm) * c.vmin;
    } else {
      const bool mx = ag.op == PGPU_RED_MAX_I64;
      uint32_t cand = mm, u = 0;
      for (int k = vb - 1; k >= 0; --k) {
        const uint32_t x = pl[64 * k];
        const uint32_t t = cand & (mx ? x : ~x);
        if (t) cand = t;
        if ((t != 0) == mx) u |= 1u << k;
      }
      part = mm ? c.vmin + (int64_t)u : sec_identity(ag.op);
    }
    lacc_add(la, cv, a, ag.op, part);
  }
}

FI void sliced_tile(const DevParams& p, const Cons& cv, LaneAcc& la, const SegState& ss, int tile, uint32_t mm,
                    int& sn) {
  bool all_bsi = true;
  for (int a = 0; a < p.nagg; ++a)
    if (p.aggs[a].fn != PGPU_AGG_COUNT) all_bsi = all_bsi && bsi_agg(p.aggs[a], col_of(ss, p.aggs[a].col));
  if (all_bsi) {
    for (int a = 0; a < p.nagg; ++a)
      if (p.aggs[a].fn != PGPU_AGG_COUNT) bsi_tile(cv, la, col_of(ss, p.aggs[a].col), p.aggs[a], a, tile, mm);
    return;
  }
  // (the planner sends a segment here only when its aggregations are all bit-sliced-index ones, or at most two over
  // <= 16-bit columns: sliced_queued)
  const int cap = PGPU_CQ_CAP / 2;
  // a tile with more matches than a sub-queue holds goes in quarters of 16 lanes (<= 512 docs each)
  const int cnt_all = __popc(mm);
  const int nm_all = wave_sum_i32(cnt_all);
  const int parts = nm_all <= cap ? 1 : 4;
  for (int part = 0; part < parts; ++part) {
    const uint32_t mp = parts == 1 ? mm : ((lane_id() >> 4) == part ? mm : 0u);
    const int cnt = __popc(mp);
    const int ex = wave_excl_scan(cnt);
    const int nm = __builtin_amdgcn_readlane(ex + cnt, 63);
    if (nm == 0) continue;
    if (sn + nm > cap) {
      sliced_flush(p, cv, la, ss, sn);
      sn = 0;
    }
    int slot = 0;
    for (int a = 0; a < p.nagg; ++a) {
      if (p.aggs[a].fn == PGPU_AGG_COUNT) continue;
      const DevColumn c = col_of(ss, p.aggs[a].col);
      uint16_t* q = cv.queue + slot++ * cap;
#define SQ_CALL(B) sliced_enqueue_b<B>(c, tile, mp, q, sn + ex)
      switch (c.bits) {
        case 1: SQ_CALL(1); break;   case 2: SQ_CALL(2); break;   case 3: SQ_CALL(3); break;   case 4: SQ_CALL(4); break;
        case 5: SQ_CALL(5); break;   case 6: SQ_CALL(6); break;   case 7: SQ_CALL(7); break;   case 8: SQ_CALL(8); break;
        case 9: SQ_CALL(9); break;   case 10: SQ_CALL(10); break; case 11: SQ_CALL(11); break; case 12: SQ_CALL(12); break;
        case 13: SQ_CALL(13); break; case 14: SQ_CALL(14); break; case 15: SQ_CALL(15); break; default: SQ_CALL(16); break;
      }
#undef SQ_CALL
    }
    sn += nm;
  }
}

// A self-loading wave's filtered tile: count it (COUNT-only segment), or queue its candidate docs for the residual
// filter and the sparse aggregation (a tile that does not fit behind the queued entries is flushed in two halves).
template <int MODE, int NW>
FI void direct_candidates(const DevParams& p, const Lds& L, const Cons& cv, LaneAcc& la, const SegState& ss,
                          int tile_in_seg, uint32_t mm, int& qn, int& qt, uint32_t& lane_matched, int64_t& matched,
                          int64_t& scanned, int64_t& sector_bytes, int64_t& dense_bytes, Prof& pf,
                          int* sn = nullptr, const unsigned char* slot = nullptr) {
  const int lane = lane_id();
  if (ss.rprog_len == 0 && ss.agg_mode == PGPU_AM_COUNT) {
    lane_matched += __popc(mm);
    mark_seg(p, ss, __builtin_amdgcn_ballot_w64(mm != 0) != 0);
  } else if (MODE == PGPU_MODE_AGG && ss.agg_mode == PGPU_AM_SLICED) {  // planner: no residual program
    lane_matched += __popc(mm);
    const bool any = __builtin_amdgcn_ballot_w64(mm != 0) != 0;
    mark_seg(p, ss, any);
    if (any && slot && ss.nvstage > 0) bsi_tile_staged(p, cv, la, ss, slot, mm);  // planes DMA'd with the tile
    else if (any && sn) sliced_tile(p, cv, la, ss, tile_in_seg, mm, *sn);
    if (any && (p.flags & PGPU_FLAG_STATS) && lane == 0)  // the aggregated columns' planes of this tile
      for (int a = 0; a < p.nagg; ++a)
        if (p.aggs[a].fn != PGPU_AGG_COUNT) {
          const DevColumn c = col_of(ss, p.aggs[a].col);
          dense_bytes += (int64_t)WT * (bsi_agg(p.aggs[a], c) ? c.vbits : c.bits) / 8;
        }
  } else if (__builtin_amdgcn_ballot_w64(mm != 0) != 0) {
    const int cnt = __popc(mm);
    const int ex = wave_excl_scan(cnt);
    const int nm = __builtin_amdgcn_readlane(ex + cnt, 63);
    if (qn + nm <= PGPU_CQ_CAP) {
      if (lane == 0) cv.qtiles[qt] = tile_in_seg;
      const uint32_t tag = (uint32_t)qt << 11;
      ++qt;
      int q = qn + ex;
      for (uint32_t left = mm; left; left &= left - 1)
        cv.queue[q++] = (uint16_t)(tag | (uint32_t)(32 * lane + __builtin_ctz(left)));
      qn += nm;
    } else {
      if (qn) {
        flush_queue<MODE, NW>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
        qn = qt = 0;
      }
      if (lane == 0) cv.qtiles[0] = tile_in_seg;
      for (int half = 0; half < 2; ++half) {
        const uint32_t mh = (lane >> 5) == half ? mm : 0u;
        const int nh = wave_sum_i32(__popc(mh));
        if (nh == 0) continue;
        int q = wave_excl_scan(__popc(mh));
        for (uint32_t left = mh; left; left &= left - 1) cv.queue[q++] = (uint16_t)(32 * lane + __builtin_ctz(left));
        flush_queue<MODE, NW>(p, L, cv, la, ss, nh, matched, scanned, sector_bytes, dense_bytes, pf);
      }
    }
  }
}

template <int MODE>
FI Stats direct_consumer(const DevParams& p, const Lds& L, int cidx, int t0, int ntiles, Prof& pf) {
  constexpr int NW = PGPU_DIRECT_WAVES;
  const int64_t t_start = now(pf);
  const int lane = lane_id();
  const int S = p.slot_bytes;
  Cons cv;
  {
    unsigned char* base = L.cons + (size_t)cidx * p.cons_bytes;
    cv.masks = (uint32_t*)base;
    cv.queue = (uint16_t*)(base + p.mask_rows * 256);
    cv.klist = (int32_t*)(base + p.mask_rows * 256);
    cv.vlist = cv.klist + PGPU_AGG_LIST;
    cv.acc = (int64_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0));
    cv.qtiles = (int32_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0) + PGPU_CONS_ACC_BYTES);
  }
  unsigned char* slots = L.ring + (size_t)cidx * p.dslots * S;
  if (MODE == PGPU_MODE_AGG && lane < PGPU_MAX_AGGS) cv.acc[lane] = lane < p.nagg ? sec_identity(p.aggs[lane].op) : 0;
  wave_sync();
  int64_t matched = 0, scanned = 0, sector_bytes = 0, dense_bytes = 0;
  uint32_t lane_scanned = 0, lane_matched = 0;  // per-lane counts (< 2^32 per lane), reduced at the end
  LaneAcc la;
#pragma unroll
  for (int k = 0; k < NREG_ACC; ++k) la.v[k] = k < p.nagg ? sec_identity(p.aggs[k].op) : 0;
  int qn = 0, qt = 0;
  int sn = 0;  // PGPU_AM_SLICED: ids queued per column (sliced_tile)
  SegState ss;
  int cseg = -1;
  if (cidx < ntiles) {
    // issue cursor `ci` runs up to D - 1 of this wave's tiles ahead of the processing cursor `cur`
    const int D = p.dslots;
    const int own = (ntiles - cidx + NW - 1) / NW;  // this wave's tiles: cidx, cidx + NW, ...
    Cursor ci = cursor_at(p, t0 + cidx), cur = ci;
    StageCache sc;
    load_stage(p, ci.seg, sc);
    int issued = 0, islot = 0, pslot = 0;
    int poll = p.cancel_poll;
    uint32_t voff16;
    asm volatile("v_lshlrev_b32 %0, 4, %1" : "=v"(voff16) : "v"(opaque_lane()));  // lane * 16, kept live
    uint32_t bw_next = 0;
    bool bw_have = false;
    auto issue_upto = [&](int upto) {
      while (issued < own && issued < upto) {
        if (issued > 0 && cursor_advance(p, ci, NW)) load_stage(p, ci.seg, sc);
        issue_tile_direct(sc, ci.tile_in_seg, slots + (size_t)islot * S, voff16, (p.flags & PGPU_FLAG_NT) != 0);
        ++issued;
        if (++islot == D) islot = 0;
      }
    };
    for (int k = 0; k < own; ++k) {
      issue_upto(k + D);
      if (--poll == 0) {
        poll = p.cancel_poll;
        if (query_cancelled(p)) break;  // in-flight DMAs drain below
      }
      const int next_instrs = (issued - k - 1) * p.min_instrs;  // lower bound of the DMAs issued after tile k
      if (k > 0) cursor_advance(p, cur, NW);
      if (qn && (qn >= PGPU_CQ_FLUSH || qt >= PGPU_CQ_TILES || cur.seg != cseg)) {
        const int64_t tq = now(pf);
        flush_queue<MODE, NW>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
        PROF_ADD(pf, PGPU_P_C_FLUSH, tq);
        qn = qt = 0;
      }
      if (cur.seg != cseg) {
        if (MODE == PGPU_MODE_AGG && sn) {  // queued ids are the previous segment's
          sliced_flush(p, cv, la, ss, sn);
          sn = 0;
        }
        cseg = cur.seg;
        load_seg(p, cseg, ss);
      }
      const int64_t tw = now(pf);
      // this tile's DMAs have landed (later tiles' may be in flight)
      if (ss.nstage + ss.nvstage > 0) wait_vmcnt(next_instrs);
      PROF_ADD(pf, PGPU_P_C_FULL, tw);
      const int64_t tf = now(pf);
#ifdef PGPU_PROFILE_BUILD
      if (pf.on) pf.t[PGPU_P_C_TILES] += 1;
#endif
      TileCtx t;
      t.ss = &ss;
      t.slot = slots + (size_t)pslot * S;
      if (++pslot == D) pslot = 0;
      t.tile_in_seg = cur.tile_in_seg;
      t.doc0 = cur.tile_in_seg * WT;
      t.lane_doc0 = t.doc0 + 32 * lane;
      {
        const int ndocs = min(WT, ss.num_docs - t.doc0);
        const int rem = ndocs - 32 * lane;
        t.valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
        if (p.flags & PGPU_FLAG_STATS)
          for (int j = 0; j < ss.nstage; ++j) {
            const int b = col_of(ss, cld(&ss.sg->stage_col[j])).bits;
            if (lane == 0) dense_bytes += ((int64_t)ndocs * b + 7) / 8;
          }
      }
      // a segment whose index-only program was evaluated by progbits_kernel reads one word per lane; the next
      // tile's word of the same segment is loaded one iteration ahead
      uint32_t bits_word = 0;
      if (ss.single_bits) {
        const uint32_t* bw = (const uint32_t*)cld(&ss.sg->bits_w[0]);
        bits_word = bw_have ? bw_next : gld(bw, (size_t)cur.tile_in_seg * 64 + lane);
        bw_have = false;
        if (k + 1 < own) {
          Cursor nx = cur;
          cursor_advance(p, nx, NW);
          if (nx.seg == cseg) {
            bw_next = gld(bw, (size_t)nx.tile_in_seg * 64 + lane);
            bw_have = true;
          }
        }
      }
      // fast sliced leaves in registers; a segment with nothing staged (bitmap / sorted / BITS leaves only) runs
      // its program through the interpreter -- no slot is read
      const uint32_t mm = ss.fast ? fast_filter(ss, t, lane_scanned)
                                  : ss.single_bits ? bits_word & t.valid
                                  : (ss.prog_len > 0 ? run_program(p, cv, ss.prog_begin, ss.prog_len, t, scanned,
                                                                   dense_bytes, pf)
                                                     : t.valid);
      // the slot's planes have been read (lgkmcnt): it is rewritten by the issue of tile k + D, after this point
      PROF_ADD(pf, PGPU_P_C_FILTER, tf);
      const int64_t ta = now(pf);
      direct_candidates<MODE, NW>(p, L, cv, la, ss, cur.tile_in_seg, mm, qn, qt, lane_matched, matched, scanned,
                                  sector_bytes, dense_bytes, pf, &sn, t.slot);
      PROF_ADD(pf, PGPU_P_C_AGG, ta);
    }
    if (qn) flush_queue<MODE, NW>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
    if (MODE == PGPU_MODE_AGG && sn) sliced_flush(p, cv, la, ss, sn);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  {
    const int64_t ls = wave_sum_i64((int64_t)lane_scanned), lm = wave_sum_i64((int64_t)lane_matched);
    if (lane == 0) {
      scanned += ls;
      matched += lm;
    }
  }
  PROF_ADD(pf, PGPU_P_C_TOTAL, t_start);
  if (MODE == PGPU_MODE_AGG) {
#pragma unroll
    for (int a = 0; a < NREG_ACC; ++a)
      if (a < p.nagg && p.aggs[a].fn != PGPU_AGG_COUNT) acc_commit(cv, a, p.aggs[a].op, la.v[a]);
  }
  Stats st;
  st.matched = matched;
  st.scanned = scanned;
  st.sector_bytes = sector_bytes;
  st.dense_bytes = dense_bytes;
  return st;
}

// LDS of the direct kernel: consumer areas | group table / partition cursors | two slots per wave.
FI Lds carve_direct(unsigned char* base, const DevParams& p) {
  Lds L;
  L.full = L.freef = L.icnt = nullptr;
  L.cons = base;
  L.ltab = (int64_t*)(L.cons + PGPU_DIRECT_WAVES * p.cons_bytes);
  L.ring = (unsigned char*)L.ltab + ((p.ltab_bytes + 15) & ~15);
  return L;
}

template <int MODE>
FI void direct_epilogue(const DevParams& p, const Lds& L, const Stats& st, int wave, int lane, Prof& pf);

template <int MODE>
__global__ __launch_bounds__(PGPU_DIRECT_THREADS, (MODE == PGPU_MODE_GLOBAL || MODE == PGPU_MODE_HASH) ? PGPU_DIRECT_MIN_WAVES : 4) void query_kernel_direct(DevParams p) {
  constexpr int NT = PGPU_DIRECT_THREADS, NWAVES = PGPU_DIRECT_WAVES;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Lds L = carve_direct(dyn_smem, p);
  if (MODE == PGPU_MODE_LDS) {
    const int n = p.nsec * (int)p.G;
    for (int i = threadIdx.x; i < n; i += NT) L.ltab[i] = sec_identity(p.sec_op[i / (int)p.G]);
  }
  if (MODE == PGPU_MODE_PART)
    for (int i = threadIdx.x; i < p.nparts; i += NT) ((uint32_t*)L.ltab)[i] = 0u;
  __syncthreads();
  // contiguous tile range per workgroup, one contiguous run of workgroups per XCD (see query_kernel)
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int t0 = (int)(((int64_t)p.total_tiles * lb) / nb);
  const int t1 = (int)(((int64_t)p.total_tiles * (lb + 1)) / nb);
  Prof pf;
#ifdef PGPU_PROFILE_BUILD
  pf.on = (p.flags & PGPU_FLAG_PROFILE) != 0;
#pragma unroll
  for (int k = 0; k < PGPU_NPROF; ++k) pf.t[k] = 0;
#endif
  const Stats st = direct_consumer<MODE>(p, L, wave, t0, t1 - t0, pf);
  direct_epilogue<MODE>(p, L, st, wave, lane, pf);
}

// Per-wave statistics and partials of a self-loading kernel, then the workgroup's table flush (LDS / PART modes).
template <int MODE>
FI void direct_epilogue(const DevParams& p, const Lds& L, const Stats& st, int wave, int lane, Prof& pf) {
  constexpr int NT = PGPU_DIRECT_THREADS, NWAVES = PGPU_DIRECT_WAVES;
  const size_t w = (size_t)blockIdx.x * NWAVES + wave;
#ifdef PGPU_PROFILE_BUILD
  if (pf.on && lane == 0) {
    int64_t* o = p.prof + w * PGPU_NPROF;
#pragma unroll
    for (int k = 0; k < PGPU_NPROF; ++k) o[k] = pf.t[k];
  }
#endif
  if (lane == 0) {
    int64_t* o = p.stats + w * PGPU_NSTATS;
    o[PGPU_STAT_MATCHED] = st.matched;
    o[PGPU_STAT_SCANNED] = st.scanned;
    o[PGPU_STAT_SECTOR_BYTES] = st.sector_bytes;
    o[PGPU_STAT_DENSE_BYTES] = st.dense_bytes;
  }
  if (MODE == PGPU_MODE_AGG) {
    int64_t* slab = p.slab + w * p.nsec;
    if (lane == 0) slab[0] = st.matched;
    if (lane < p.nagg && p.aggs[lane].fn != PGPU_AGG_COUNT) {
      const int64_t* acc = (const int64_t*)(L.cons + (size_t)wave * p.cons_bytes + p.mask_rows * 256 +
                                            PGPU_CONS_LIST_BYTES_OF(0));
      slab[p.aggs[lane].sec] = acc[lane];
    }
  } else if (MODE == PGPU_MODE_LDS) {
    __syncthreads();
    const int G = (int)p.G;
    for (int key = threadIdx.x; key < G; key += NT) {
      const int64_t cnt = L.ltab[key];
      if (cnt == 0) continue;
      atomicAdd((unsigned long long*)&p.table[key], (unsigned long long)cnt);
      for (int s = 1; s < p.nsec; ++s) cell_atomic(&p.table[(size_t)s * p.G + key], p.sec_op[s], L.ltab[s * G + key]);
    }
  } else if (MODE == PGPU_MODE_PART) {
    __syncthreads();
    for (int q = threadIdx.x; q < p.nparts; q += NT) {
      const uint32_t n = ((const uint32_t*)L.ltab)[q];
      p.rcount[(size_t)q * gridDim.x + blockIdx.x] = n < (uint32_t)p.rcap ? n : (uint32_t)p.rcap;
    }
  }
}

// ================================================================================================================
// REGISTER-DIRECT variant (p.direct == 2): every segment's only staged column is one bit-sliced fast leaf of at most
// PL = p.rd_planes bits (8, 10, 12 or 16: the borrow chains cost one v_bitop3 per plane, so PL tracks the width).  Its planes go straight into VGPRs -- plane k of lane l is one coalesced 4-B load per
// lane, 256 B per wave-instruction -- with RD tiles in flight per wave (a register ring, unrolled), no LDS staging
// at all: tools/stream_bench.hip reads such a stream at 5.6-6.0 TB/s where the LDS-DMA self-loading kernel
// streamed 3.8 TB/s (its in-flight bytes are bounded by the LDS slots).  Candidate handling as in direct_consumer.
// ================================================================================================================
#define PGPU_RDIRECT_DEPTH 2
struct RdIssue {  // the issue cursor's segment: its sliced column (and the prefix column's)
  const uint32_t* sliced;
  int bits;
  const uint32_t* psliced;
  int pbits;
};
FI void rd_load_issue(const DevParams& p, int seg, RdIssue& is) {
  const DevSeg* sg = p.segs + seg;
  const DevColumn* cols = p.cols + cld(&sg->col_begin);
  const int qc = cld(&sg->stage_col[0]);
  is.sliced = (const uint32_t*)cld(&cols[qc].sliced);
  is.bits = cld(&cols[qc].bits);
  const int pc = cld(&sg->pfx_col);
  is.psliced = pc >= 0 ? (const uint32_t*)cld(&cols[pc].sliced) : nullptr;
  is.pbits = pc >= 0 ? cld(&cols[pc].bits) : 0;
}
template <int PL>
FI void rd_load_tile(const RdIssue& is, int tile_in_seg, uint32_t (&x)[PL]) {
  const uint32_t* src = is.sliced + (size_t)tile_in_seg * is.bits * 64 + lane_id();
#pragma unroll
  for (int k = 0; k < PL; ++k)
    x[k] = k < is.bits ? __builtin_nontemporal_load(src + 64 * k) : 0u;  // planes past the width: 0 (inert below)
}
// The residual column's top PK planes (plane j of the prefix = bit pbits - PK + j of the id)
template <int PK>
FI void rd_load_prefix(const RdIssue& is, int tile_in_seg, uint32_t (&y)[PK]) {
  const uint32_t* src = is.psliced + ((size_t)tile_in_seg * is.pbits + (is.pbits - PK)) * 64 + lane_id();
#pragma unroll
  for (int k = 0; k < PK; ++k) y[k] = __builtin_nontemporal_load(src + 64 * k);
}
// The fast leaf on register planes: OR of dict-id ranges [lo, hi) (x < c as a borrow chain; planes past the
// column's width are 0 and leave the chain unchanged, and c = 2^bits sets the borrow there), then negated.
template <int PL>
FI uint32_t rd_lt(const uint32_t (&x)[PL], uint32_t c) {
  uint32_t br = 0;
#pragma unroll
  for (int k = 0; k < PL; ++k)
    br = __builtin_amdgcn_bitop3_b32((uint32_t)-(int32_t)((c >> k) & 1u), x[k], br, 0xB2);
  return (c >> PL) ? ~0u : br;
}
template <int PL>
FI uint32_t rd_filter(const SegState& ss, const uint32_t (&x)[PL], uint32_t valid,
                      uint32_t& lane_scanned) {
  if (!(ss.f_kind[0] >> 8)) lane_scanned += __popc(valid);
  uint32_t m = rd_lt(x, ss.f_r0hi[0]) & ~rd_lt(x, ss.f_r0lo[0]);
  for (int r = 1; r < ss.f_nr[0]; ++r) {
    const uint32_t lo = cld(&ss.sg->f_rng[0][r][0]), hi = cld(&ss.sg->f_rng[0][r][1]);
    m |= rd_lt(x, hi) & ~rd_lt(x, lo);
  }
  return valid & (ss.f_sneg[0] ? ~m : m);
}
// Prefix pre-filter of the candidates `mm`: those whose residual-column id has its top PK bits in a matching range.
// The rest are rejected here, never gathered; each still counts as one entry the residual leaf scans
// (SVScanDocIdIterator over the AND's candidates).
template <int PK>
FI uint32_t rd_prefix(const SegState& ss, const uint32_t (&y)[PK], uint32_t mm, uint32_t& lane_scanned) {
  uint32_t pm = 0;
  const int nr = cld(&ss.sg->pfx_nr);
  for (int r = 0; r < nr; ++r) {
    const uint32_t lo = cld(&ss.sg->pfx_rng[r][0]), hi = cld(&ss.sg->pfx_rng[r][1]);
    pm |= rd_lt(y, hi) & ~rd_lt(y, lo);
  }
  lane_scanned += __popc(mm & ~pm);
  return mm & pm;
}

template <int MODE, int PL, int PK>
FI Stats rdirect_consumer(const DevParams& p, const Lds& L, int cidx, int t0, int ntiles, Prof& pf) {
  constexpr int NW = PGPU_DIRECT_WAVES, RD = PGPU_RDIRECT_DEPTH;
  const int64_t t_start = now(pf);
  const int lane = lane_id();
  Cons cv;
  {
    unsigned char* base = L.cons + (size_t)cidx * p.cons_bytes;
    cv.masks = (uint32_t*)base;
    cv.queue = (uint16_t*)(base + p.mask_rows * 256);
    cv.klist = (int32_t*)(base + p.mask_rows * 256);
    cv.vlist = cv.klist + PGPU_AGG_LIST;
    cv.acc = (int64_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0));
    cv.qtiles = (int32_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0) + PGPU_CONS_ACC_BYTES);
  }
  if (MODE == PGPU_MODE_AGG && lane < PGPU_MAX_AGGS) cv.acc[lane] = lane < p.nagg ? sec_identity(p.aggs[lane].op) : 0;
  wave_sync();
  int64_t matched = 0, scanned = 0, sector_bytes = 0, dense_bytes = 0;
  uint32_t lane_scanned = 0, lane_matched = 0;
  LaneAcc la;
#pragma unroll
  for (int k = 0; k < NREG_ACC; ++k) la.v[k] = k < p.nagg ? sec_identity(p.aggs[k].op) : 0;
  int qn = 0, qt = 0;
  SegState ss;
  int cseg = -1;
  if (cidx < ntiles) {
    const int own = (ntiles - cidx + NW - 1) / NW;  // this wave's tiles: cidx, cidx + NW, ...
    Cursor ci = cursor_at(p, t0 + cidx), cur = ci;
    RdIssue is;
    rd_load_issue(p, ci.seg, is);
    uint32_t x[RD][PL];
    uint32_t y[RD][PK > 0 ? PK : 1];
#pragma unroll
    for (int s = 0; s < RD; ++s) {
      if (s < own) {
        if (s > 0 && cursor_advance(p, ci, NW)) rd_load_issue(p, ci.seg, is);
        rd_load_tile(is, ci.tile_in_seg, x[s]);
        if constexpr (PK > 0) rd_load_prefix<PK>(is, ci.tile_in_seg, y[s]);
      }
    }
    int poll = p.cancel_poll;
    bool stop = false;
    for (int k0 = 0; k0 < own && !stop; k0 += RD) {
#pragma unroll
      for (int s = 0; s < RD; ++s) {
        const int k = k0 + s;
        if (k >= own || stop) break;
        if (--poll == 0) {
          poll = p.cancel_poll;
          if (query_cancelled(p)) {
            stop = true;
            break;
          }
        }
        if (k > 0) cursor_advance(p, cur, NW);
        if (qn && (qn >= PGPU_CQ_FLUSH || qt >= PGPU_CQ_TILES || cur.seg != cseg)) {
          const int64_t tq = now(pf);
          flush_queue<MODE, NW>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
          PROF_ADD(pf, PGPU_P_C_FLUSH, tq);
          qn = qt = 0;
        }
        if (cur.seg != cseg) {
          cseg = cur.seg;
          load_seg(p, cseg, ss);
        }
        const int64_t tf = now(pf);
#ifdef PGPU_PROFILE_BUILD
        if (pf.on) pf.t[PGPU_P_C_TILES] += 1;
#endif
        const int doc0 = cur.tile_in_seg * WT;
        uint32_t valid;
        {
          const int ndocs = min(WT, ss.num_docs - doc0);
          const int rem = ndocs - 32 * lane;
          valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
          if ((p.flags & PGPU_FLAG_STATS) && lane == 0) dense_bytes += ((int64_t)ndocs * (ss.f_bits[0] + PK) + 7) / 8;
        }
        uint32_t mm = rd_filter(ss, x[s], valid, lane_scanned);
        if constexpr (PK > 0) mm = rd_prefix<PK>(ss, y[s], mm, lane_scanned);
        // refill this register slot with the tile RD ahead (its loads overlap this tile's candidate handling)
        if (k + RD < own) {
          if (cursor_advance(p, ci, NW)) rd_load_issue(p, ci.seg, is);
          rd_load_tile(is, ci.tile_in_seg, x[s]);
          if constexpr (PK > 0) rd_load_prefix<PK>(is, ci.tile_in_seg, y[s]);
        }
        PROF_ADD(pf, PGPU_P_C_FILTER, tf);
        const int64_t ta = now(pf);
        direct_candidates<MODE, NW>(p, L, cv, la, ss, cur.tile_in_seg, mm, qn, qt, lane_matched, matched, scanned,
                                    sector_bytes, dense_bytes, pf);
        PROF_ADD(pf, PGPU_P_C_AGG, ta);
      }
    }
    if (qn && !stop) flush_queue<MODE, NW>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
  }
  {
    const int64_t ls = wave_sum_i64((int64_t)lane_scanned), lm = wave_sum_i64((int64_t)lane_matched);
    if (lane == 0) {
      scanned += ls;
      matched += lm;
    }
  }
  PROF_ADD(pf, PGPU_P_C_TOTAL, t_start);
  if (MODE == PGPU_MODE_AGG) {
#pragma unroll
    for (int a = 0; a < NREG_ACC; ++a)
      if (a < p.nagg && p.aggs[a].fn != PGPU_AGG_COUNT) acc_commit(cv, a, p.aggs[a].op, la.v[a]);
  }
  Stats st;
  st.matched = matched;
  st.scanned = scanned;
  st.sector_bytes = sector_bytes;
  st.dense_bytes = dense_bytes;
  return st;
}

template <int MODE, int PL, int PK>
__global__ __launch_bounds__(PGPU_DIRECT_THREADS) void query_kernel_rdirect(DevParams p) {
  constexpr int NT = PGPU_DIRECT_THREADS, NWAVES = PGPU_DIRECT_WAVES;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Lds L = carve_direct(dyn_smem, p);
  if (MODE == PGPU_MODE_LDS) {
    const int n = p.nsec * (int)p.G;
    for (int i = threadIdx.x; i < n; i += NT) L.ltab[i] = sec_identity(p.sec_op[i / (int)p.G]);
  }
  if (MODE == PGPU_MODE_PART)
    for (int i = threadIdx.x; i < p.nparts; i += NT) ((uint32_t*)L.ltab)[i] = 0u;
  __syncthreads();
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int t0 = (int)(((int64_t)p.total_tiles * lb) / nb);
  const int t1 = (int)(((int64_t)p.total_tiles * (lb + 1)) / nb);
  Prof pf;
#ifdef PGPU_PROFILE_BUILD
  pf.on = (p.flags & PGPU_FLAG_PROFILE) != 0;
#pragma unroll
  for (int k = 0; k < PGPU_NPROF; ++k) pf.t[k] = 0;
#endif
  const Stats st = rdirect_consumer<MODE, PL, PK>(p, L, wave, t0, t1 - t0, pf);
  direct_epilogue<MODE>(p, L, st, wave, lane, pf);
}

// ================================================================================================================
// EXACT FILTER STATISTICS IN THE REGISTER STREAM (p.direct == 8).  With the reference's numEntriesScannedInFilter
// requested and every segment's filter an AND of two bit-sliced scan leaves (config 5's shape), the count needs each
// leaf's match word at every doc (AndDocIdIterator.java:40-67 leap-frogs SVScanDocIdIterator.java:57-71 over both
// leaves), so both leaves' planes are streamed in full anyway.  This kernel streams them once -- RD tiles ahead in a
// register ring, as query_kernel_rdirect does -- and from the same words (1) ANDs the leaves and aggregates the
// matched docs through the candidate queue (no residual program left to run) and (2) writes the tile's transducer
// map for andfsm_segment_kernel (the andfsm encoding), replacing query_kernel_rdirect + andfsm_tile_kernel, which
// read the first leaf twice.
// ================================================================================================================
#ifndef PGPU_ANDFSM_WORDS
#define PGPU_ANDFSM_WORDS 8  // per tile: next-state bits (2 per start state), then H per start state
#endif
struct RfIssue {  // the issue cursor's segment: both leaves' bit-sliced columns
  const uint32_t* s0;
  const uint32_t* s1;
  int b0, b1;
};
FI void rf_load_issue(const DevParams& p, int seg, RfIssue& is) {
  const DevSeg* sg = p.segs + seg;
  const DevColumn* cols = p.cols + cld(&sg->col_begin);
  const int lb = cld(&sg->leaf_begin);
  const int c0 = cld(&p.instrs[cld(p.pool, lb)].col), c1 = cld(&p.instrs[cld(p.pool, lb + 1)].col);
  is.s0 = (const uint32_t*)cld(&cols[c0].sliced);
  is.b0 = cld(&cols[c0].bits);
  is.s1 = (const uint32_t*)cld(&cols[c1].sliced);
  is.b1 = cld(&cols[c1].bits);
}
template <int P>
FI void rf_load(const uint32_t* sl, int bits, int tile_in_seg, uint32_t (&x)[P]) {
  const uint32_t* src = sl + (size_t)tile_in_seg * bits * 64 + lane_id();
#pragma unroll
  for (int k = 0; k < P; ++k) x[k] = k < bits ? __builtin_nontemporal_load(src + 64 * k) : 0u;
}
// A scan leaf on its register planes (planes past the column's width are 0): a dict-id range, an id mask or <= 4 ids
// (the shapes andfsm's fsm_sliced_ok admits), then negated for exclusive predicates.
template <int P>
FI uint32_t rf_leaf(const uint32_t (&x)[P], const DevInstr& in) {
  uint32_t m;
  if (in.pred == PRED_RANGE) {
    m = rd_lt(x, (uint32_t)in.hi) & ~rd_lt(x, (uint32_t)in.lo);
  } else if (in.pred == PRED_MASK) {
    m = 0;
    for (uint64_t mk = ((uint64_t)(uint32_t)in.hi << 32) | (uint32_t)in.lo; mk; mk &= mk - 1) {
      const uint32_t id = (uint32_t)__builtin_ctzll(mk);
      m |= rd_lt(x, id + 1u) & ~rd_lt(x, id);
    }
  } else {
    m = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < in.n) m |= rd_lt(x, in.ids[j] + 1u) & ~rd_lt(x, in.ids[j]);
  }
  return in.negate ? ~m : m;
}
// The tile's map of the two-iterator leap-frog: state s = the iterator scanning; per lane over its 32 docs, then
// composed across lanes in doc order; lane 0 writes {next states, hand-offs per start state} (andfsm's encoding,
// states 2 and 3 the identity).
FI void rf_tile_map(uint32_t m0, uint32_t m1, uint32_t* fn_tile) {
  const int lane = lane_id();
  uint32_t nxt = (2u << 4) | (3u << 6), h[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int s0 = 0; s0 < 2; ++s0) {
    int st = s0;
    uint32_t hh = 0;
    int pos = 0;
    while (pos < 32) {
      const uint32_t w = (st ? m1 : m0) >> pos;
      if (!w) break;
      const int d = pos + __builtin_ctz(w);
      ++hh;  // the other iterator advances to d (one entry)
      st = (((st ? m0 : m1) >> d) & 1u) ? 0 : 1 - st;  // both match: a result, iterator 0 leads again
      pos = d + 1;
    }
    nxt |= (uint32_t)st << (2 * s0);
    h[s0] = hh;
  }
  // (two live states: 2 and 3 stay the identity with no hand-offs, so only states 0 and 1 are composed)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t rn = (uint32_t)__shfl_down((int)nxt, o, 64);
    const uint32_t r0 = (uint32_t)__shfl_down((int)h[0], o, 64), r1 = (uint32_t)__shfl_down((int)h[1], o, 64);
    if ((lane & (2 * o - 1)) == 0 && lane + o < 64) {
      const uint32_t m0 = nxt & 3u, m1 = (nxt >> 2) & 3u;  // (each 0 or 1)
      h[0] += m0 ? r1 : r0;
      h[1] += m1 ? r1 : r0;
      nxt = (nxt & 0xF0u) | ((rn >> (2 * m0)) & 3u) | (((rn >> (2 * m1)) & 3u) << 2);
    }
  }
  if (lane == 0) {
    fn_tile[0] = nxt;
    fn_tile[1] = h[0];
    fn_tile[2] = h[1];
    fn_tile[3] = 0u;
    fn_tile[4] = 0u;
  }
}

template <int MODE, int P0, int P1>
FI Stats rfsm_consumer(const DevParams& p, const Lds& L, int cidx, int t0, int ntiles, Prof& pf) {
  constexpr int NW = PGPU_DIRECT_WAVES, RD = PGPU_RDIRECT_DEPTH;
  const int64_t t_start = now(pf);
  const int lane = lane_id();
  Cons cv;
  {
    unsigned char* base = L.cons + (size_t)cidx * p.cons_bytes;
    cv.masks = (uint32_t*)base;
    cv.queue = (uint16_t*)(base + p.mask_rows * 256);
    cv.klist = (int32_t*)(base + p.mask_rows * 256);
    cv.vlist = cv.klist + PGPU_AGG_LIST;
    cv.acc = (int64_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0));
    cv.qtiles = (int32_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0) + PGPU_CONS_ACC_BYTES);
  }
  if (MODE == PGPU_MODE_AGG && lane < PGPU_MAX_AGGS) cv.acc[lane] = lane < p.nagg ? sec_identity(p.aggs[lane].op) : 0;
  wave_sync();
  int64_t matched = 0, scanned = 0, sector_bytes = 0, dense_bytes = 0;
  uint32_t lane_matched = 0;
  LaneAcc la;
#pragma unroll
  for (int k = 0; k < NREG_ACC; ++k) la.v[k] = k < p.nagg ? sec_identity(p.aggs[k].op) : 0;
  int qn = 0, qt = 0;
  SegState ss;
  int cseg = -1;
  DevInstr in0, in1;
  if (cidx < ntiles) {
    const int own = (ntiles - cidx + NW - 1) / NW;  // this wave's tiles: cidx, cidx + NW, ...
    Cursor ci = cursor_at(p, t0 + cidx), cur = ci;
    RfIssue is;
    rf_load_issue(p, ci.seg, is);
    uint32_t x0[RD][P0], x1[RD][P1];
#pragma unroll
    for (int s = 0; s < RD; ++s) {
      if (s < own) {
        if (s > 0 && cursor_advance(p, ci, NW)) rf_load_issue(p, ci.seg, is);
        rf_load<P0>(is.s0, is.b0, ci.tile_in_seg, x0[s]);
        rf_load<P1>(is.s1, is.b1, ci.tile_in_seg, x1[s]);
      }
    }
    int poll = p.cancel_poll;
    bool stop = false;
    for (int k0 = 0; k0 < own && !stop; k0 += RD) {
#pragma unroll
      for (int s = 0; s < RD; ++s) {
        const int k = k0 + s;
        if (k >= own || stop) break;
        if (--poll == 0) {
          poll = p.cancel_poll;
          if (query_cancelled(p)) {
            stop = true;
            break;
          }
        }
        if (k > 0) cursor_advance(p, cur, NW);
        if (qn && (qn >= PGPU_CQ_FLUSH || qt >= PGPU_CQ_TILES || cur.seg != cseg)) {
          flush_queue<MODE, NW>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
          qn = qt = 0;
        }
        if (cur.seg != cseg) {
          cseg = cur.seg;
          load_seg(p, cseg, ss);
          ss.rprog_len = 0;  // both leaves are evaluated here: the queue carries results, not candidates
          const int lb = cld(&ss.sg->leaf_begin);
          in0 = cld(p.instrs + cld(p.pool, lb));
          in1 = cld(p.instrs + cld(p.pool, lb + 1));
        }
        const int64_t tf = now(pf);
        const int doc0 = cur.tile_in_seg * WT;
        uint32_t valid;
        {
          const int ndocs = min(WT, ss.num_docs - doc0);
          const int rem = ndocs - 32 * lane;
          valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
          if ((p.flags & PGPU_FLAG_STATS) && lane == 0) dense_bytes += ((int64_t)ndocs * (in0.bits + in1.bits) + 7) / 8;
        }
        const uint32_t m0 = rf_leaf<P0>(x0[s], in0) & valid, m1 = rf_leaf<P1>(x1[s], in1) & valid;
        // refill this register slot with the tile RD ahead (its loads overlap this tile's map and aggregation)
        if (k + RD < own) {
          if (cursor_advance(p, ci, NW)) rf_load_issue(p, ci.seg, is);
          rf_load<P0>(is.s0, is.b0, ci.tile_in_seg, x0[s]);
          rf_load<P1>(is.s1, is.b1, ci.tile_in_seg, x1[s]);
        }
        rf_tile_map(m0, m1, p.fsm_fn + (size_t)(t0 + cidx + k * NW) * PGPU_ANDFSM_WORDS);
        PROF_ADD(pf, PGPU_P_C_FILTER, tf);
        const int64_t ta = now(pf);
        direct_candidates<MODE, NW>(p, L, cv, la, ss, cur.tile_in_seg, m0 & m1, qn, qt, lane_matched, matched,
                                    scanned, sector_bytes, dense_bytes, pf);
        PROF_ADD(pf, PGPU_P_C_AGG, ta);
      }
    }
    if (qn && !stop) flush_queue<MODE, NW>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
  }
  {
    const int64_t lm = wave_sum_i64((int64_t)lane_matched);
    if (lane == 0) matched += lm;
  }
  PROF_ADD(pf, PGPU_P_C_TOTAL, t_start);
  if (MODE == PGPU_MODE_AGG) {
#pragma unroll
    for (int a = 0; a < NREG_ACC; ++a)
      if (a < p.nagg && p.aggs[a].fn != PGPU_AGG_COUNT) acc_commit(cv, a, p.aggs[a].op, la.v[a]);
  }
  Stats st;
  st.matched = matched;
  st.scanned = 0;  // (the reference's count comes from the tile maps: andfsm_segment_kernel)
  st.sector_bytes = sector_bytes;
  st.dense_bytes = dense_bytes;
  return st;
}

template <int MODE, int P0, int P1>
__global__ __launch_bounds__(PGPU_DIRECT_THREADS) void query_kernel_rfsm(DevParams p) {
  constexpr int NT = PGPU_DIRECT_THREADS;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Lds L = carve_direct(dyn_smem, p);
  if (MODE == PGPU_MODE_LDS) {
    const int n = p.nsec * (int)p.G;
    for (int i = threadIdx.x; i < n; i += NT) L.ltab[i] = sec_identity(p.sec_op[i / (int)p.G]);
  }
  __syncthreads();
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int t0 = (int)(((int64_t)p.total_tiles * lb) / nb);
  const int t1 = (int)(((int64_t)p.total_tiles * (lb + 1)) / nb);
  Prof pf;
#ifdef PGPU_PROFILE_BUILD
  pf.on = (p.flags & PGPU_FLAG_PROFILE) != 0;
#pragma unroll
  for (int k = 0; k < PGPU_NPROF; ++k) pf.t[k] = 0;
#endif
  const Stats st = rfsm_consumer<MODE, P0, P1>(p, L, wave, t0, t1 - t0, pf);
  direct_epilogue<MODE>(p, L, st, wave, lane, pf);
}

// ================================================================================================================
// REGISTER STREAMING (p.direct == 3, aggregation-only mode): every segment's filter is an AND of two bit-sliced fast
// leaves -- one of <= 16 bits ("wide"), one of <= PN bits ("narrow") -- and every aggregation is answered from one
// column's value planes (PGPU_AM_SLICED, no residual program).  All three plane sets of a tile stream into VGPRs
// RD tiles ahead, so the aggregation reads registers that were loaded with the filter planes: no LDS slot, no
// candidate queue, and no plain load issued behind a later one (vmcnt retires in order) -- one coalesced read of
// (wide + narrow + value) planes per tile, the shape tools/stream_bench.hip reads at 5.6-6.0 TB/s.  The value
// planes of a tile without a match are read too: the planner chose SLICED because nearly every line holds one.
// ================================================================================================================
struct RsIssue {
  const uint32_t* sw;  // the wide leaf's planes (bw per tile), the narrow leaf's, the value column's
  const uint32_t* sn;
  const uint32_t* sv;
  int bw, bn, vb;
};
// Leaf j of the segment's fast program (its instruction's query column).
FI int rs_leaf_col(const DevParams& p, const DevSeg* sg, int j) {
  return cld(&p.instrs[cld(&sg->prog_begin) + cld(&sg->fast_ins[j])].col);
}
FI void rs_load_issue(const DevParams& p, int seg, int vcol, RsIssue& is) {
  const DevSeg* sg = p.segs + seg;
  const DevColumn* cols = p.cols + cld(&sg->col_begin);
  const int c0 = rs_leaf_col(p, sg, 0), c1 = rs_leaf_col(p, sg, 1);
  const int b0 = cld(&cols[c0].bits), b1 = cld(&cols[c1].bits);
  const bool w0 = b0 >= b1;  // (rstream_consumer makes the same choice)
  is.sw = (const uint32_t*)cld(&cols[w0 ? c0 : c1].sliced);
  is.sn = (const uint32_t*)cld(&cols[w0 ? c1 : c0].sliced);
  is.bw = w0 ? b0 : b1;
  is.bn = w0 ? b1 : b0;
  is.sv = (const uint32_t*)cld(&cols[vcol].vsliced);
  is.vb = cld(&cols[vcol].vbits);
}
template <int PL>
FI void rs_load_planes(const uint32_t* sl, int bits, int tile_in_seg, uint32_t (&x)[PL]) {
  const uint32_t* src = sl + (size_t)tile_in_seg * bits * 64 + lane_id();
#pragma unroll
  for (int k = 0; k < PL; ++k) x[k] = k < bits ? __builtin_nontemporal_load(src + 64 * k) : 0u;
}
// Fast leaf j on register planes: OR of its dict-id ranges, then its negation (fast_filter's sliced branch).
template <int PL>
FI uint32_t rs_leaf(const SegState& ss, int j, const uint32_t (&x)[PL]) {
  uint32_t m = rd_lt(x, j ? ss.f_r0hi[1] : ss.f_r0hi[0]) & ~rd_lt(x, j ? ss.f_r0lo[1] : ss.f_r0lo[0]);
  const int nr = j ? ss.f_nr[1] : ss.f_nr[0];
  for (int r = 1; r < nr; ++r) {
    const uint32_t lo = cld(&ss.sg->f_rng[j][r][0]), hi = cld(&ss.sg->f_rng[j][r][1]);
    m |= rd_lt(x, hi) & ~rd_lt(x, lo);
  }
  return (j ? ss.f_sneg[1] : ss.f_sneg[0]) ? ~m : m;
}
// The matched docs' aggregations from the value planes (bsi_fold with the segment's width and offset cached).
template <int NV>
FI void rs_fold(const DevParams& p, const Cons& cv, LaneAcc& la, const uint32_t (&x)[NV], uint32_t mm, int vb,
                int64_t vmin, int vcol) {
  for (int a = 0; a < p.nagg; ++a) {
    if (p.aggs[a].fn == PGPU_AGG_COUNT || p.aggs[a].col != vcol) continue;
    const int32_t op = p.aggs[a].op;
    int64_t part;
    if (op == PGPU_RED_SUM_I64) {
      uint32_t u = 0;  // < 32 * 2^24
#pragma unroll
      for (int k = 0; k < NV; ++k)
        if (k < vb) u += (uint32_t)__popc(x[k] & mm) << k;
      part = (int64_t)u + (int64_t)__popc(mm) * vmin;
    } else {
      const bool mx = op == PGPU_RED_MAX_I64;
      uint32_t cand = mm, u = 0;
#pragma unroll
      for (int k = NV - 1; k >= 0; --k) {
        if (k >= vb) continue;
        const uint32_t t = cand & (mx ? x[k] : ~x[k]);
        if (t) cand = t;
        if ((t != 0) == mx) u |= 1u << k;
      }
      part = mm ? vmin + (int64_t)u : sec_identity(op);
    }
    lacc_add(la, cv, a, op, part);
  }
}

template <int PN, int NV>
FI Stats rstream_consumer(const DevParams& p, const Lds& L, int cidx, int t0, int ntiles, Prof& pf) {
  constexpr int NW = PGPU_DIRECT_WAVES, RD = PGPU_RDIRECT_DEPTH, PW = 16;
  const int64_t t_start = now(pf);
  const int lane = lane_id();
  Cons cv;
  {
    unsigned char* base = L.cons + (size_t)cidx * p.cons_bytes;
    cv.masks = (uint32_t*)base;
    cv.queue = (uint16_t*)(base + p.mask_rows * 256);
    cv.klist = (int32_t*)(base + p.mask_rows * 256);
    cv.vlist = cv.klist + PGPU_AGG_LIST;
    cv.acc = (int64_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0));
    cv.qtiles = (int32_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0) + PGPU_CONS_ACC_BYTES);
  }
  if (lane < PGPU_MAX_AGGS) cv.acc[lane] = lane < p.nagg ? sec_identity(p.aggs[lane].op) : 0;
  wave_sync();
  int64_t matched = 0, scanned = 0, dense_bytes = 0;
  uint32_t lane_scanned = 0, lane_matched = 0;
  LaneAcc la;
#pragma unroll
  for (int k = 0; k < NREG_ACC; ++k) la.v[k] = k < p.nagg ? sec_identity(p.aggs[k].op) : 0;
  int vcol = 0;  // the one value column (runtime: every non-COUNT aggregation reads it)
  for (int a = 0; a < p.nagg; ++a)
    if (p.aggs[a].fn != PGPU_AGG_COUNT) vcol = p.aggs[a].col;
  SegState ss;
  int cseg = -1, jw = 0, vb = 0;
  int64_t vmin = 0, vbytes = 0;
  if (cidx < ntiles) {
    const int own = (ntiles - cidx + NW - 1) / NW;  // this wave's tiles: cidx, cidx + NW, ...
    Cursor ci = cursor_at(p, t0 + cidx), cur = ci;
    RsIssue is;
    rs_load_issue(p, ci.seg, vcol, is);
    uint32_t xw[RD][PW], xn[RD][PN], xv[RD][NV];
#pragma unroll
    for (int s = 0; s < RD; ++s) {
      if (s < own) {
        if (s > 0 && cursor_advance(p, ci, NW)) rs_load_issue(p, ci.seg, vcol, is);
        rs_load_planes(is.sw, is.bw, ci.tile_in_seg, xw[s]);
        rs_load_planes(is.sn, is.bn, ci.tile_in_seg, xn[s]);
        rs_load_planes(is.sv, is.vb, ci.tile_in_seg, xv[s]);
      }
    }
    int poll = p.cancel_poll;
    bool stop = false;
    for (int k0 = 0; k0 < own && !stop; k0 += RD) {
#pragma unroll
      for (int s = 0; s < RD; ++s) {
        const int k = k0 + s;
        if (k >= own || stop) break;
        if (--poll == 0) {
          poll = p.cancel_poll;
          if (query_cancelled(p)) {
            stop = true;
            break;
          }
        }
        if (k > 0) cursor_advance(p, cur, NW);
        if (cur.seg != cseg) {
          cseg = cur.seg;
          load_seg(p, cseg, ss);
          jw = cld(&ss.cols[rs_leaf_col(p, ss.sg, 0)].bits) >= cld(&ss.cols[rs_leaf_col(p, ss.sg, 1)].bits) ? 0 : 1;
          vb = cld(&ss.cols[vcol].vbits);
          vmin = cld(&ss.cols[vcol].vmin);
          vbytes = 0;  // the aggregated columns' planes per matched tile (direct_candidates' dense-bytes model)
          for (int a = 0; a < p.nagg; ++a)
            if (p.aggs[a].fn != PGPU_AGG_COUNT) vbytes += (int64_t)WT * vb / 8;
        }
        const int64_t tf = now(pf);
#ifdef PGPU_PROFILE_BUILD
        if (pf.on) pf.t[PGPU_P_C_TILES] += 1;
#endif
        const int doc0 = cur.tile_in_seg * WT;
        uint32_t valid;
        {
          const int ndocs = min(WT, ss.num_docs - doc0);
          const int rem = ndocs - 32 * lane;
          valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
          if ((p.flags & PGPU_FLAG_STATS) && lane == 0) dense_bytes += ((int64_t)ndocs * (ss.f_bits[0] + ss.f_bits[1]) + 7) / 8;
        }
        // the AND in program order for the scanned-entries count: leaf 0 reads every doc, leaf 1 leaf 0's matches
        const uint32_t mw = rs_leaf(ss, jw, xw[s]), mn = rs_leaf(ss, 1 - jw, xn[s]);
        const uint32_t m0 = valid & (jw == 0 ? mw : mn);
        if (!(ss.f_kind[0] >> 8)) lane_scanned += __popc(valid);
        if (!(ss.f_kind[1] >> 8)) lane_scanned += __popc(m0);
        const uint32_t mm = m0 & mw & mn;
        PROF_ADD(pf, PGPU_P_C_FILTER, tf);
        const int64_t ta = now(pf);
        lane_matched += __popc(mm);
        const bool any = __builtin_amdgcn_ballot_w64(mm != 0) != 0;
        mark_seg(p, ss, any);
        if (any) {
          rs_fold<NV>(p, cv, la, xv[s], mm, vb, vmin, vcol);
          if ((p.flags & PGPU_FLAG_STATS) && lane == 0) dense_bytes += vbytes;
        }
        PROF_ADD(pf, PGPU_P_C_AGG, ta);
        // refill this register slot with the tile RD ahead (its loads overlap the next tile's work)
        if (k + RD < own) {
          if (cursor_advance(p, ci, NW)) rs_load_issue(p, ci.seg, vcol, is);
          rs_load_planes(is.sw, is.bw, ci.tile_in_seg, xw[s]);
          rs_load_planes(is.sn, is.bn, ci.tile_in_seg, xn[s]);
          rs_load_planes(is.sv, is.vb, ci.tile_in_seg, xv[s]);
        }
      }
    }
  }
  {
    const int64_t ls = wave_sum_i64((int64_t)lane_scanned), lm = wave_sum_i64((int64_t)lane_matched);
    if (lane == 0) {
      scanned += ls;
      matched += lm;
    }
  }
  PROF_ADD(pf, PGPU_P_C_TOTAL, t_start);
#pragma unroll
  for (int a = 0; a < NREG_ACC; ++a)
    if (a < p.nagg && p.aggs[a].fn != PGPU_AGG_COUNT) acc_commit(cv, a, p.aggs[a].op, la.v[a]);
  Stats st;
  st.matched = matched;
  st.scanned = scanned;
  st.sector_bytes = 0;
  st.dense_bytes = dense_bytes;
  return st;
}

template <int PN, int NV>
__global__ __launch_bounds__(PGPU_DIRECT_THREADS) void query_kernel_rstream(DevParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Lds L = carve_direct(dyn_smem, p);
  __syncthreads();
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int t0 = (int)(((int64_t)p.total_tiles * lb) / nb);
  const int t1 = (int)(((int64_t)p.total_tiles * (lb + 1)) / nb);
  Prof pf;
#ifdef PGPU_PROFILE_BUILD
  pf.on = (p.flags & PGPU_FLAG_PROFILE) != 0;
#pragma unroll
  for (int k = 0; k < PGPU_NPROF; ++k) pf.t[k] = 0;
#endif
  const Stats st = rstream_consumer<PN, NV>(p, L, wave, t0, t1 - t0, pf);
  direct_epilogue<PGPU_MODE_AGG>(p, L, st, wave, lane, pf);
}

// ================================================================================================================
// REGISTER STREAMING OF INDEX-ONLY PROGRAMS (p.direct == 4, aggregation-only mode): every segment's dense program
// reads only precomputed bitmaps (BITS leaves: inverted-index leaves expanded by invexp_kernel, raw-value leaves)
// and sorted-column doc ranges, <= 5 leaves, none counted as scanned entries; its aggregations come from <= 2
// columns' value planes.  The runtime turns the program into a truth table over its leaves (DevSeg::ptt), so a
// tile's match word is a 31-deep v_bfi mux tree over the leaf words -- no instruction fetch, no LDS mask rows -- and
// the leaves' bitmap words ride in the register ring with the value planes (as in query_kernel_rstream).
// ================================================================================================================
#define PGPU_RPROG_LEAVES 5
struct RpIssue {
  const uint32_t* bw[PGPU_PREBITS];
  const uint32_t* sv[2];
  int nb, vb[2];
};
FI void rp_load_issue(const DevParams& p, int seg, int vc0, int vc1, RpIssue& is) {
  const DevSeg* sg = p.segs + seg;
  const DevColumn* cols = p.cols + cld(&sg->col_begin);
  is.nb = cld(&sg->nbits);
#pragma unroll
  for (int j = 0; j < PGPU_PREBITS; ++j) is.bw[j] = (const uint32_t*)cld(&sg->bits_w[j]);
  is.sv[0] = (const uint32_t*)cld(&cols[vc0].vsliced);
  is.vb[0] = cld(&cols[vc0].vbits);
  is.sv[1] = vc1 >= 0 ? (const uint32_t*)cld(&cols[vc1].vsliced) : nullptr;
  is.vb[1] = vc1 >= 0 ? cld(&cols[vc1].vbits) : 0;
}
template <int NA, int NV>
FI void rp_load(const RpIssue& is, int tile_in_seg, uint32_t (&w)[PGPU_PREBITS], uint32_t (&x)[NA][NV]) {
  const size_t wi = (size_t)tile_in_seg * (WT / 32) + lane_id();  // the lane's 32 docs: one word of each bitmap
#pragma unroll
  for (int j = 0; j < PGPU_PREBITS; ++j) w[j] = j < is.nb ? __builtin_nontemporal_load(is.bw[j] + wi) : 0u;
#pragma unroll
  for (int c = 0; c < NA; ++c) rs_load_planes(is.sv[c], is.vb[c], tile_in_seg, x[c]);
}
// f(w) for the 5-input truth table T (bit t = f at leaf values t): a mux tree, leaf 0 first.
FI uint32_t tt_eval(uint32_t T, const uint32_t (&w)[PGPU_RPROG_LEAVES]) {
  uint32_t g[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t one = 0u - ((T >> (2 * j + 1)) & 1u), zero = 0u - ((T >> (2 * j)) & 1u);
    g[j] = (w[0] & one) | (~w[0] & zero);
  }
#pragma unroll
  for (int lv = 1; lv < PGPU_RPROG_LEAVES; ++lv) {
#pragma unroll
    for (int j = 0; j < (16 >> lv); ++j) g[j] = (w[lv] & g[2 * j + 1]) | (~w[lv] & g[2 * j]);
  }
  return g[0];
}

template <int NA, int NV>
FI Stats rprog_consumer(const DevParams& p, const Lds& L, int cidx, int t0, int ntiles, Prof& pf) {
  constexpr int NW = PGPU_DIRECT_WAVES, RD = PGPU_RDIRECT_DEPTH;
  const int64_t t_start = now(pf);
  const int lane = lane_id();
  Cons cv;
  {
    unsigned char* base = L.cons + (size_t)cidx * p.cons_bytes;
    cv.masks = (uint32_t*)base;
    cv.queue = (uint16_t*)(base + p.mask_rows * 256);
    cv.klist = (int32_t*)(base + p.mask_rows * 256);
    cv.vlist = cv.klist + PGPU_AGG_LIST;
    cv.acc = (int64_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0));
    cv.qtiles = (int32_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0) + PGPU_CONS_ACC_BYTES);
  }
  if (lane < PGPU_MAX_AGGS) cv.acc[lane] = lane < p.nagg ? sec_identity(p.aggs[lane].op) : 0;
  wave_sync();
  int64_t matched = 0, dense_bytes = 0;
  uint32_t lane_matched = 0;
  LaneAcc la;
#pragma unroll
  for (int k = 0; k < NREG_ACC; ++k) la.v[k] = k < p.nagg ? sec_identity(p.aggs[k].op) : 0;
  int vc0 = -1, vc1 = -1;  // the value columns, in first-use order (runtime: at most NA)
  for (int a = 0; a < p.nagg; ++a) {
    const int c = p.aggs[a].col;
    if (p.aggs[a].fn == PGPU_AGG_COUNT || c == vc0) continue;
    if (vc0 < 0) vc0 = c;
    else vc1 = c;
  }
  SegState ss;
  int cseg = -1, nb = 0, nsorted = 0, ps0 = 0, ps1 = 0, vb0 = 0, vb1 = 0;
  uint32_t T = 0;
  int64_t vmin0 = 0, vmin1 = 0, vbytes = 0;
  if (cidx < ntiles) {
    const int own = (ntiles - cidx + NW - 1) / NW;  // this wave's tiles: cidx, cidx + NW, ...
    Cursor ci = cursor_at(p, t0 + cidx), cur = ci;
    RpIssue is;
    rp_load_issue(p, ci.seg, vc0, vc1, is);
    uint32_t pw[RD][PGPU_PREBITS], xv[RD][NA][NV];
#pragma unroll
    for (int s = 0; s < RD; ++s) {
      if (s < own) {
        if (s > 0 && cursor_advance(p, ci, NW)) rp_load_issue(p, ci.seg, vc0, vc1, is);
        rp_load<NA, NV>(is, ci.tile_in_seg, pw[s], xv[s]);
      }
    }
    int poll = p.cancel_poll;
    bool stop = false;
    for (int k0 = 0; k0 < own && !stop; k0 += RD) {
#pragma unroll
      for (int s = 0; s < RD; ++s) {
        const int k = k0 + s;
        if (k >= own || stop) break;
        if (--poll == 0) {
          poll = p.cancel_poll;
          if (query_cancelled(p)) {
            stop = true;
            break;
          }
        }
        if (k > 0) cursor_advance(p, cur, NW);
        if (cur.seg != cseg) {
          cseg = cur.seg;
          load_seg(p, cseg, ss);
          T = cld(&ss.sg->ptt);
          nb = cld(&ss.sg->nbits);
          nsorted = cld(&ss.sg->pnsorted);
          ps0 = cld(&ss.sg->psorted[0]);
          ps1 = cld(&ss.sg->psorted[1]);
          vb0 = cld(&ss.cols[vc0].vbits);
          vmin0 = cld(&ss.cols[vc0].vmin);
          vb1 = vc1 >= 0 ? cld(&ss.cols[vc1].vbits) : 0;
          vmin1 = vc1 >= 0 ? cld(&ss.cols[vc1].vmin) : 0;
          vbytes = 0;  // the aggregated columns' planes per matched tile (direct_candidates' dense-bytes model)
          for (int a = 0; a < p.nagg; ++a)
            if (p.aggs[a].fn != PGPU_AGG_COUNT) vbytes += (int64_t)WT * (p.aggs[a].col == vc0 ? vb0 : vb1) / 8;
        }
        const int64_t tf = now(pf);
#ifdef PGPU_PROFILE_BUILD
        if (pf.on) pf.t[PGPU_P_C_TILES] += 1;
#endif
        TileCtx t;
        t.ss = &ss;
        t.slot = nullptr;
        t.tile_in_seg = cur.tile_in_seg;
        t.doc0 = cur.tile_in_seg * WT;
        t.lane_doc0 = t.doc0 + 32 * lane;
        {
          const int rem = min(WT, ss.num_docs - t.doc0) - 32 * lane;
          t.valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
        }
        const uint32_t sw0 = nsorted > 0 ? leaf_sorted(p, t, cld(p.instrs + ps0)) : 0u;
        const uint32_t sw1 = nsorted > 1 ? leaf_sorted(p, t, cld(p.instrs + ps1)) : 0u;
        uint32_t w[PGPU_RPROG_LEAVES];
#pragma unroll
        for (int i = 0; i < PGPU_RPROG_LEAVES; ++i)
          w[i] = (i < PGPU_PREBITS && i < nb) ? pw[s][i < PGPU_PREBITS ? i : 0] : (i == nb ? sw0 : (i == nb + 1 ? sw1 : 0u));
        const uint32_t mm = tt_eval(T, w) & t.valid;
        PROF_ADD(pf, PGPU_P_C_FILTER, tf);
        const int64_t ta = now(pf);
        lane_matched += __popc(mm);
        const bool any = __builtin_amdgcn_ballot_w64(mm != 0) != 0;
        mark_seg(p, ss, any);
        if (any) {
          rs_fold<NV>(p, cv, la, xv[s][0], mm, vb0, vmin0, vc0);
          if constexpr (NA > 1) rs_fold<NV>(p, cv, la, xv[s][NA - 1], mm, vb1, vmin1, vc1);
          if ((p.flags & PGPU_FLAG_STATS) && lane == 0) dense_bytes += vbytes;
        }
        PROF_ADD(pf, PGPU_P_C_AGG, ta);
        if (k + RD < own) {  // refill this register slot with the tile RD ahead
          if (cursor_advance(p, ci, NW)) rp_load_issue(p, ci.seg, vc0, vc1, is);
          rp_load<NA, NV>(is, ci.tile_in_seg, pw[s], xv[s]);
        }
      }
    }
  }
  {
    const int64_t lm = wave_sum_i64((int64_t)lane_matched);
    if (lane == 0) matched += lm;
  }
  PROF_ADD(pf, PGPU_P_C_TOTAL, t_start);
#pragma unroll
  for (int a = 0; a < NREG_ACC; ++a)
    if (a < p.nagg && p.aggs[a].fn != PGPU_AGG_COUNT) acc_commit(cv, a, p.aggs[a].op, la.v[a]);
  Stats st;
  st.matched = matched;
  st.scanned = 0;  // (the runtime admits only leaves that count no scanned entries)
  st.sector_bytes = 0;
  st.dense_bytes = dense_bytes;
  return st;
}

template <int NA, int NV>
__global__ __launch_bounds__(PGPU_DIRECT_THREADS) void query_kernel_rprog(DevParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Lds L = carve_direct(dyn_smem, p);
  __syncthreads();
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int t0 = (int)(((int64_t)p.total_tiles * lb) / nb);
  const int t1 = (int)(((int64_t)p.total_tiles * (lb + 1)) / nb);
  Prof pf;
#ifdef PGPU_PROFILE_BUILD
  pf.on = (p.flags & PGPU_FLAG_PROFILE) != 0;
#pragma unroll
  for (int k = 0; k < PGPU_NPROF; ++k) pf.t[k] = 0;
#endif
  const Stats st = rprog_consumer<NA, NV>(p, L, wave, t0, t1 - t0, pf);
  direct_epilogue<PGPU_MODE_AGG>(p, L, st, wave, lane, pf);
}

// ================================================================================================================
// INDEX-ONLY PROGRAMS OVER ROARING CONTAINERS IN LDS (p.direct == 5): query_kernel_rprog's shape when every BITS
// leaf of every segment is an inverted-index leaf.  Instead of expanding those leaves into HBM bitmaps first
// (invexp_kernel: one write and one read of a doc bitmap per leaf), a workgroup takes one (segment, 65,536-doc
// container key) unit at a time, ORs the key's container of each leaf's ids into an 8 KiB LDS image per leaf
// (BitmapBasedFilterOperator.java:66-110: bitmap containers copied, array values and runs set with LDS atomics,
// NOT IN / <> complemented within the segment), then its four waves evaluate the unit's 32 tiles from those
// images -- the truth table over the leaf words and sorted ranges, the value planes in a register ring that runs
// ahead across units, so the next unit's planes are in flight while its containers are read.
// ================================================================================================================
FI int unit_segment(const DevParams& p, int u) {
  int lo = 0, hi = p.nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cld(&p.segs[mid].unit_begin) <= u) lo = mid; else hi = mid - 1;
  }
  return lo;
}
// A wave's tile sequence over the units [u, u1): unit u's tiles wave, wave + NW, ... of its <= 32.
struct UnitCursor {
  int u, u1, seg, key, k, nt;  // unit, end, its segment, container key, next tile index in unit, tiles in unit
  int ntiles_seg, unit0;
};
FI void unit_enter(const DevParams& p, UnitCursor& c) {
  c.seg = unit_segment(p, c.u);
  c.unit0 = cld(&p.segs[c.seg].unit_begin);
  c.ntiles_seg = cld(&p.segs[c.seg].ntiles);
  c.key = c.u - c.unit0;
  c.nt = min(32, c.ntiles_seg - 32 * c.key);
}
// advance to this wave's next tile (true: *tile_in_seg / *seg set); false past the end
FI bool unit_next(const DevParams& p, UnitCursor& c, int wave, int* seg, int* tile_in_seg) {
  while (c.u < c.u1) {
    if (c.k < c.nt) {
      *seg = c.seg;
      *tile_in_seg = 32 * c.key + c.k;
      c.k += PGPU_DIRECT_WAVES;
      return true;
    }
    if (++c.u >= c.u1) break;
    unit_enter(p, c);
    c.k = wave;
  }
  return false;
}
// IDS: the aggregated columns' packed 16-bit dict ids stream instead of their value planes (16 words per lane and
// tile instead of vbits planes); the matched docs' ids go to the wave's LDS queue and their values are gathered from
// the (L2-resident) dictionaries when it fills (sliced_flush) -- fewer bytes than the value planes when few docs match.
// Every aggregation's column of an IDS launch is a 16-bit fixed-bit dictionary column (the runtime checks).
// The lane's matched docs' ids (docs 2k, 2k + 1 are the MSB-first halves of big-endian word k) into q[at, ...).
// The word is picked with constant register indices: a register array indexed by a doc number would live in
// scratch, and walking all 16 words unrolled per aggregation costs ~100 VGPRs.
FI uint32_t pick16(const uint32_t (&w)[16], uint32_t k) {
  uint32_t x = 0;  // (an OR of masked words: a select tree gets folded back into an indexed scratch load)
#pragma unroll
  for (int j = 0; j < 16; ++j) x |= w[j] & (0u - (uint32_t)(k == (uint32_t)j));
  return x;
}
FI void packed16_enqueue(const uint32_t (&w)[16], uint32_t mm, uint16_t* q, int at) {
  for (uint32_t left = mm; left; left &= left - 1) {
    const uint32_t i = (uint32_t)__builtin_ctz(left);
    const uint32_t x = bswap32(pick16(w, i >> 1));
    q[at++] = (uint16_t)((i & 1u) ? (x & 0xFFFFu) : (x >> 16));
  }
}
template <int NA, int NV, bool IDS = false>
__global__ __launch_bounds__(PGPU_DIRECT_THREADS) void query_kernel_rkey(DevParams p) {
  constexpr int NW = PGPU_DIRECT_WAVES, RD = PGPU_RDIRECT_DEPTH, NT = PGPU_DIRECT_THREADS;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Lds L = carve_direct(dyn_smem, p);
  int& rk_stop = *(int*)L.ring;  // the query was cancelled: every wave leaves at the same unit
  DevContainer* recs = (DevContainer*)(L.ring + 16);  // [PGPU_RKEY_PAIRS] the unit's container per (leaf, id)
  uint32_t* img = (uint32_t*)(L.ring + 16 + 16 * PGPU_RKEY_PAIRS);  // [nbits][2048]: the unit's leaf images
  Prof pf;
#ifdef PGPU_PROFILE_BUILD
  pf.on = (p.flags & PGPU_FLAG_PROFILE) != 0;
#pragma unroll
  for (int k = 0; k < PGPU_NPROF; ++k) pf.t[k] = 0;
#endif
  const int64_t t_start = now(pf);
  Cons cv;
  {
    unsigned char* base = L.cons + (size_t)wave * p.cons_bytes;
    cv.masks = (uint32_t*)base;
    cv.queue = (uint16_t*)(base + p.mask_rows * 256);
    cv.klist = (int32_t*)(base + p.mask_rows * 256);
    cv.vlist = cv.klist + PGPU_AGG_LIST;
    cv.acc = (int64_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0));
    cv.qtiles = (int32_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0) + PGPU_CONS_ACC_BYTES);
  }
  if (lane < PGPU_MAX_AGGS) cv.acc[lane] = lane < p.nagg ? sec_identity(p.aggs[lane].op) : 0;
  LaneAcc la;
#pragma unroll
  for (int k = 0; k < NREG_ACC; ++k) la.v[k] = k < p.nagg ? sec_identity(p.aggs[k].op) : 0;
  int vc0 = -1, vc1 = -1;  // the value columns, in first-use order (runtime: at most NA)
  for (int a = 0; a < p.nagg; ++a) {
    const int c = p.aggs[a].col;
    if (p.aggs[a].fn == PGPU_AGG_COUNT || c == vc0) continue;
    if (vc0 < 0) vc0 = c;
    else vc1 = c;
  }
  // this workgroup's contiguous run of units (XCD-aware order, as the tile ranges of the other kernels)
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int u0 = (int)(((int64_t)p.total_units * lb) / nb);
  const int u1 = (int)(((int64_t)p.total_units * (lb + 1)) / nb);
  int64_t dense_bytes = 0;
  uint32_t lane_matched = 0;
  // the value-plane ring: issue cursor `ci` runs RD tiles ahead of the consumed sequence
  uint32_t xv[RD][NA][NV];
  UnitCursor ci{u0, u1, 0, 0, wave, 0, 0, 0};
  if (u0 < u1) unit_enter(p, ci);
  int have = 0;  // tiles issued into the ring and not yet consumed
#define RK_ISSUE(S)                                                                                          \
  do {                                                                                                       \
    int sseg, stile;                                                                                         \
    if (unit_next(p, ci, wave, &sseg, &stile)) {                                                             \
      const DevColumn* pc = p.cols + cld(&p.segs[sseg].col_begin);                                           \
      if constexpr (IDS) {                                                                                   \
        hbm_lane_raw<NV>(cld(&pc[vc0].fwd), stile, xv[S][0]);                                               \
        if constexpr (NA > 1) hbm_lane_raw<NV>(cld(&pc[vc1].fwd), stile, xv[S][NA - 1]);                     \
      } else {                                                                                               \
        rs_load_planes(cld(&pc[vc0].vsliced), cld(&pc[vc0].vbits), stile, xv[S][0]);                        \
        if constexpr (NA > 1) rs_load_planes(cld(&pc[vc1].vsliced), cld(&pc[vc1].vbits), stile, xv[S][NA - 1]); \
      }                                                                                                      \
      ++have;                                                                                                \
    }                                                                                                        \
  } while (0)
#pragma unroll
  for (int s = 0; s < RD; ++s) RK_ISSUE(s);
  SegState ss;
  int cseg = -1, nbits = 0, nsorted = 0, ps0 = 0, ps1 = 0, vb0 = 0, vb1 = 0;
  uint32_t T = 0, negm = 0;
  int64_t vmin0 = 0, vmin1 = 0, vbytes = 0;
  int nid[PGPU_PREBITS] = {0, 0, 0, 0}, npairs = 0;  // ids per leaf, (leaf, id) pairs of the segment
  int slot = 0;
  int sn = 0;  // IDS: ids queued per aggregation (sliced_flush)
  for (int u = u0; u < u1; ++u) {
    const int seg = unit_segment(p, u);
    if (seg != cseg) {
      if (IDS && sn) {  // the queued ids are the old segment's: gather them from its dictionaries first
        sliced_flush(p, cv, la, ss, sn);
        sn = 0;
      }
      cseg = seg;
      load_seg(p, cseg, ss);
      T = cld(&ss.sg->ptt);
      nbits = cld(&ss.sg->nbits);
      nsorted = cld(&ss.sg->pnsorted);
      ps0 = cld(&ss.sg->psorted[0]);
      ps1 = cld(&ss.sg->psorted[1]);
      vb0 = cld(&ss.cols[vc0].vbits);
      vmin0 = cld(&ss.cols[vc0].vmin);
      vb1 = vc1 >= 0 ? cld(&ss.cols[vc1].vbits) : 0;
      vmin1 = vc1 >= 0 ? cld(&ss.cols[vc1].vmin) : 0;
      vbytes = 0;
      for (int a = 0; a < p.nagg; ++a)
        if (p.aggs[a].fn != PGPU_AGG_COUNT) vbytes += (int64_t)WT * (IDS ? 16 : (p.aggs[a].col == vc0 ? vb0 : vb1)) / 8;
      negm = 0;  // leaves of NOT IN / <> predicates: complemented within the segment
      npairs = 0;
      for (int j = 0; j < nbits; ++j) {
        negm |= (cld(&p.invx[cld(&ss.sg->inv_leaf[j])].negate) ? 1u : 0u) << j;
        nid[j] = cld(&p.invx[cld(&ss.sg->inv_leaf[j])].nids);
        npairs += nid[j];
      }
    }
    const int key = u - cld(&ss.sg->unit_begin);
    const int nt = min(32, cld(&ss.sg->ntiles) - 32 * key);
    // the unit's leaf images: every earlier reader is done, clear; the unit's container record of every (leaf, id)
    // from the query's container table (rkey_ctab_kernel: no container search here), then OR the containers in
    const int64_t tf = now(pf);
    __syncthreads();
    if (threadIdx.x == 0) rk_stop = query_cancelled(p) ? 1 : 0;
    if (threadIdx.x < npairs) {
      int j = 0, k = threadIdx.x;
      while (j + 1 < nbits && k >= nid[j]) k -= nid[j++];
      const InvLeafX X = p.invx[cld(&ss.sg->inv_leaf[j])];
      recs[threadIdx.x] = p.rk_ctab[(size_t)X.ctab_off + (size_t)k * X.nkeys + key];
    }
    __syncthreads();
    if (rk_stop) break;
    // Pass 1: each leaf's image = the OR of its bitmap containers, built in registers (thread t owns words t + NT*m)
    // and stored once -- no clearing pass and no LDS atomics; every container word load of the leaf is issued
    // before the first OR, so the loads overlap instead of paying one HBM round trip each.
    constexpr int WPT = 2048 / NT;  // image words per thread
    for (int t2 = 0, j = 0; j < nbits; ++j) {
      uint32_t acc[WPT];
#pragma unroll
      for (int m = 0; m < WPT; ++m) acc[m] = 0u;
      const uint8_t* data = (const uint8_t*)cld(&p.invx[cld(&ss.sg->inv_leaf[j])].data);
      for (int e = t2 + nid[j]; t2 < e; ++t2) {
        const DevContainer rc = recs[t2];
        if (sgpr(rc.type) != PGPU_CT_BITMAP || sgpr(rc.card) == 0) continue;
        const uint32_t* bm = (const uint32_t*)(data + sgpr(rc.offset));
        uint32_t v[WPT];
#pragma unroll
        for (int m = 0; m < WPT; ++m) v[m] = gld(bm, threadIdx.x + NT * m);
#pragma unroll
        for (int m = 0; m < WPT; ++m) acc[m] |= v[m];
      }
#pragma unroll
      for (int m = 0; m < WPT; ++m) img[j * 2048 + threadIdx.x + NT * m] = acc[m];
    }
    __syncthreads();
    // Pass 2: array values and runs set with LDS atomics, their 16-bit values loaded AB at a time per thread first
    for (int t2 = 0, j = 0, left = nbits > 0 ? nid[0] : 0; t2 < npairs; ++t2) {
      while (left == 0) left = nid[++j];
      --left;
      const DevContainer rc = recs[t2];
      const uint32_t type = sgpr(rc.type), card = sgpr(rc.card), offset = sgpr(rc.offset);
      if (card == 0 || type == PGPU_CT_BITMAP) continue;  // (no container of this id under this key / pass 1)
      uint32_t* w = img + j * 2048;
      const uint8_t* data = (const uint8_t*)cld(&p.invx[cld(&ss.sg->inv_leaf[j])].data);
      constexpr int AB = 8;
      if (type == PGPU_CT_RUN) {
        const uint16_t* r = (const uint16_t*)(data + offset);
        for (uint32_t q0 = 0; q0 < card; q0 += NT * AB) {
          uint32_t st[AB], ln[AB];
#pragma unroll
          for (int b = 0; b < AB; ++b) {
            const uint32_t q = q0 + threadIdx.x + NT * b;
            st[b] = q < card ? gld(r, 2 * q) : 1u;
            ln[b] = q < card ? gld(r, 2 * q + 1) : 0u;
          }
#pragma unroll
          for (int b = 0; b < AB; ++b) {
            if (q0 + threadIdx.x + NT * b >= card) continue;
            const uint32_t s0 = st[b], e0 = s0 + ln[b];  // inclusive
            const uint32_t a = s0 >> 5, z = e0 >> 5;
            for (uint32_t x = a; x <= z; ++x) {
              const uint32_t lo = x == a ? (s0 & 31) : 0u, hi = x == z ? (e0 & 31) : 31u;
              atomicOr(&w[x], (0xFFFFFFFFu >> (31 - hi)) & (0xFFFFFFFFu << lo));
            }
          }
        }
      } else {
        const uint16_t* v = (const uint16_t*)(data + offset);
        for (uint32_t q0 = 0; q0 < card; q0 += NT * AB) {
          uint32_t x[AB];
#pragma unroll
          for (int b = 0; b < AB; ++b) {
            const uint32_t q = q0 + threadIdx.x + NT * b;
            x[b] = q < card ? gld(v, q) : 0xFFFFFFFFu;
          }
#pragma unroll
          for (int b = 0; b < AB; ++b)
            if (x[b] != 0xFFFFFFFFu) atomicOr(&w[x[b] >> 5], 1u << (x[b] & 31));
        }
      }
    }
    __syncthreads();
    PROF_ADD(pf, PGPU_P_C_FETCH, tf);
    for (int k = wave; k < nt; k += NW) {
      if (have == 0) break;  // (never: the ring was issued over the same sequence)
      const int64_t tt = now(pf);
      TileCtx t;
      t.ss = &ss;
      t.slot = nullptr;
      t.tile_in_seg = 32 * key + k;
      t.doc0 = t.tile_in_seg * WT;
      t.lane_doc0 = t.doc0 + 32 * lane;
      {
        const int rem = min(WT, ss.num_docs - t.doc0) - 32 * lane;
        t.valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
      }
      const uint32_t sw0 = nsorted > 0 ? leaf_sorted(p, t, cld(p.instrs + ps0)) : 0u;
      const uint32_t sw1 = nsorted > 1 ? leaf_sorted(p, t, cld(p.instrs + ps1)) : 0u;
      uint32_t w[PGPU_RPROG_LEAVES];
#pragma unroll
      for (int i = 0; i < PGPU_RPROG_LEAVES; ++i) {
        uint32_t x = 0u;
        if (i < PGPU_PREBITS && i < nbits) {
          x = img[i * 2048 + k * 64 + lane];
          if ((negm >> i) & 1u) x = ~x & t.valid;
        } else if (i == nbits) {
          x = sw0;
        } else if (i == nbits + 1) {
          x = sw1;
        }
        w[i] = x;
      }
      const uint32_t mm = tt_eval(T, w) & t.valid;
      PROF_ADD(pf, PGPU_P_C_FILTER, tt);
      const int64_t ta = now(pf);
      lane_matched += __popc(mm);
      const bool any = __builtin_amdgcn_ballot_w64(mm != 0) != 0;
      mark_seg(p, ss, any);
      // the ring slot holding this tile (issued in the same per-wave order)
#pragma unroll
      for (int s = 0; s < RD; ++s) {
        if (s != slot) continue;
        if (any) {
          if constexpr (IDS) {
            // the matched docs' ids into the queue, one sub-queue per aggregation (a tile with more matches than a
            // sub-queue holds goes in quarters of 16 lanes), gathered when full
            constexpr int cap = PGPU_CQ_CAP / 2;
            const int nm_all = wave_sum_i32(__popc(mm));
            const int parts = nm_all <= cap ? 1 : 4;
            for (int part = 0; part < parts; ++part) {
              const uint32_t mp = parts == 1 ? mm : ((lane >> 4) == part ? mm : 0u);
              const int cnt = __popc(mp);
              const int ex = wave_excl_scan(cnt);
              const int nm = __builtin_amdgcn_readlane(ex + cnt, 63);
              if (nm == 0) continue;
              if (sn + nm > cap) {
                sliced_flush(p, cv, la, ss, sn);
                sn = 0;
              }
              int q = 0;
              for (int a = 0; a < p.nagg; ++a) {
                if (p.aggs[a].fn == PGPU_AGG_COUNT) continue;
                uint16_t* qq = cv.queue + q++ * cap;
                if (p.aggs[a].col == vc0) packed16_enqueue(xv[s][0], mp, qq, sn + ex);
                else packed16_enqueue(xv[s][NA - 1], mp, qq, sn + ex);
              }
              sn += nm;
            }
          } else {
            rs_fold<NV>(p, cv, la, xv[s][0], mm, vb0, vmin0, vc0);
            if constexpr (NA > 1) rs_fold<NV>(p, cv, la, xv[s][NA - 1], mm, vb1, vmin1, vc1);
          }
          if ((p.flags & PGPU_FLAG_STATS) && lane == 0) dense_bytes += vbytes;
        }
        --have;
        RK_ISSUE(s);
      }
      slot = slot + 1 == RD ? 0 : slot + 1;
      PROF_ADD(pf, PGPU_P_C_AGG, ta);
    }
  }
#undef RK_ISSUE
  if (IDS && sn && !rk_stop) sliced_flush(p, cv, la, ss, sn);
  {
    const int64_t lm = wave_sum_i64((int64_t)lane_matched);
    PROF_ADD(pf, PGPU_P_C_TOTAL, t_start);
#pragma unroll
    for (int a = 0; a < NREG_ACC; ++a)
      if (a < p.nagg && p.aggs[a].fn != PGPU_AGG_COUNT) acc_commit(cv, a, p.aggs[a].op, la.v[a]);
    Stats st;
    st.matched = lane == 0 ? lm : 0;
    st.scanned = 0;
    st.sector_bytes = 0;
    st.dense_bytes = dense_bytes;
    direct_epilogue<PGPU_MODE_AGG>(p, L, st, wave, lane, pf);
  }
}

// ================================================================================================================
// CANDIDATE ITERATION from a sparse leading index leaf (p.direct == 6).  AndDocIdSet.iterator iterates the index
// child's bitmap and applies the scan children to those docs only (AndDocIdSet.java:87-140, SVScanDocIdIterator
// .applyAnd :79-94).  When every segment's dense program is one inclusive inverted or sorted leaf holding few docs,
// the launch runs over that leaf's Roaring containers (or sorted doc ranges split at 65,536-doc keys) -- one unit
// each -- instead of over tiles: a wave turns its unit's docs into candidate-queue entries (array values as they
// are, bitmap and run containers through a private 8 KiB LDS image, ranges counted out), and flush_queue applies the
// residual program and the sparse aggregation to them.  Tiles holding no doc of the leaf are never visited.  A single-value column's ids have disjoint doc sets, so
// no doc is queued twice (the runtime takes a multi-value column here with one id only).
// ================================================================================================================
template <int MODE>
__global__ __launch_bounds__(PGPU_DIRECT_THREADS) void query_kernel_cand(DevParams p) {
  constexpr int NT = PGPU_DIRECT_THREADS, NW = PGPU_DIRECT_WAVES;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Lds L = carve_direct(dyn_smem, p);
  if (MODE == PGPU_MODE_LDS) {
    const int n = p.nsec * (int)p.G;
    for (int i = threadIdx.x; i < n; i += NT) L.ltab[i] = sec_identity(p.sec_op[i / (int)p.G]);
  }
  __syncthreads();
  Prof pf;
#ifdef PGPU_PROFILE_BUILD
  pf.on = (p.flags & PGPU_FLAG_PROFILE) != 0;
#pragma unroll
  for (int k = 0; k < PGPU_NPROF; ++k) pf.t[k] = 0;
#endif
  const int64_t t_start = now(pf);
  Cons cv;
  {
    unsigned char* base = L.cons + (size_t)wave * p.cons_bytes;
    cv.masks = (uint32_t*)base;
    cv.queue = (uint16_t*)(base + p.mask_rows * 256);
    cv.klist = (int32_t*)(base + p.mask_rows * 256);
    cv.vlist = cv.klist + PGPU_AGG_LIST;
    cv.acc = (int64_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0));
    cv.qtiles = (int32_t*)(base + p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(0) + PGPU_CONS_ACC_BYTES);
  }
  uint32_t* img = (uint32_t*)(L.ring + (size_t)wave * 8192);  // [2048] this wave's container image
  if (MODE == PGPU_MODE_AGG && lane < PGPU_MAX_AGGS) cv.acc[lane] = lane < p.nagg ? sec_identity(p.aggs[lane].op) : 0;
  wave_sync();
  LaneAcc la;
#pragma unroll
  for (int k = 0; k < NREG_ACC; ++k) la.v[k] = k < p.nagg ? sec_identity(p.aggs[k].op) : 0;
  int64_t matched = 0, scanned = 0, sector_bytes = 0, dense_bytes = 0;
  SegState ss;
  int cseg = -1;
  const DevContainer* ct = nullptr;
  const uint8_t* data = nullptr;
  const int nwaves = gridDim.x * NW;
  int poll = 0;
  for (int u = blockIdx.x * NW + wave; u < p.total_units; u += nwaves) {
    if ((poll++ & 7) == 0 && query_cancelled(p)) break;
    const int64_t tf = now(pf);
    const uint32_t* ur = p.cand_ct + 4 * (size_t)u;
    const int seg = sgpr((int)cld(ur));
    const uint32_t ci = (uint32_t)sgpr((int)cld(ur + 1));
    if (seg != cseg) {
      cseg = seg;
      load_seg(p, cseg, ss);
      const int leaf = cld(&ss.sg->cand_leaf);
      if (leaf >= 0) {
        ct = (const DevContainer*)cld(&p.invx[leaf].ct);
        data = (const uint8_t*)cld(&p.invx[leaf].data);
      }
    }
    if (ci == ~0u) {  // a sorted leaf's doc range [lo, hi] within one 65,536-doc key
      const uint32_t lo = (uint32_t)sgpr((int)cld(ur + 2)), hi = (uint32_t)sgpr((int)cld(ur + 3));
      if (lane < PGPU_CQ_TILES) cv.qtiles[lane] = (int)(lo >> 16) * PGPU_CQ_TILES + lane;
      PROF_ADD(pf, PGPU_P_C_FETCH, tf);
      const int64_t tq = now(pf);
      for (uint32_t b = lo; b <= hi; b += PGPU_CQ_CAP) {
        const int n = (int)min((uint32_t)PGPU_CQ_CAP, hi - b + 1);
        for (int i = lane; i < n; i += 64) cv.queue[i] = (uint16_t)((b + i) & 0xFFFFu);
        flush_queue<MODE, NW>(p, L, cv, la, ss, n, matched, scanned, sector_bytes, dense_bytes, pf);
      }
      PROF_ADD(pf, PGPU_P_C_FLUSH, tq);
      continue;
    }
    const uint32_t key = (uint32_t)sgpr((int)cld(&ct[ci].key)), type = (uint32_t)sgpr((int)cld(&ct[ci].type));
    const uint32_t card = (uint32_t)sgpr((int)cld(&ct[ci].card)), off = (uint32_t)sgpr((int)cld(&ct[ci].offset));
    // the container spans 32 tiles: queue entry = tile index << 11 | doc in tile = the doc's low 16 bits
    if (lane < PGPU_CQ_TILES) cv.qtiles[lane] = (int)key * PGPU_CQ_TILES + lane;
    PROF_ADD(pf, PGPU_P_C_FETCH, tf);
    const int64_t tq = now(pf);
    if (type != PGPU_CT_BITMAP && type != PGPU_CT_RUN) {  // array: the sorted low 16 bits themselves
      const uint16_t* v = (const uint16_t*)(data + off);
      for (uint32_t b = 0; b < card; b += PGPU_CQ_CAP) {
        const int n = (int)min((uint32_t)PGPU_CQ_CAP, card - b);
        for (int i = lane; i < n; i += 64) cv.queue[i] = gld(v, b + i);
        flush_queue<MODE, NW>(p, L, cv, la, ss, n, matched, scanned, sector_bytes, dense_bytes, pf);
      }
      PROF_ADD(pf, PGPU_P_C_FLUSH, tq);
      continue;
    }
    if (type == PGPU_CT_BITMAP) {
      const uint32_t* bm = (const uint32_t*)(data + off);
      for (int i = lane; i < 2048; i += 64) img[i] = gld(bm, i);
    } else {
      for (int i = lane; i < 2048; i += 64) img[i] = 0u;
      wave_sync();
      const uint16_t* r = (const uint16_t*)(data + off);
      for (uint32_t q = lane; q < card; q += 64) {
        const uint32_t s0 = gld(r, 2 * q), e0 = s0 + gld(r, 2 * q + 1);  // inclusive
        const uint32_t a = s0 >> 5, z = e0 >> 5;
        for (uint32_t x = a; x <= z; ++x) {
          const uint32_t lo = x == a ? (s0 & 31) : 0u, hi = x == z ? (e0 & 31) : 31u;
          atomicOr(&img[x], (0xFFFFFFFFu >> (31 - hi)) & (0xFFFFFFFFu << lo));
        }
      }
    }
    wave_sync();
    // the image's set bits in doc order, PGPU_CQ_CAP entries per flush
    int qn = 0;
    for (int w0 = 0; w0 < 2048; w0 += 64) {
      uint32_t x = img[w0 + lane];
      const int c = __popc(x);
      const int tot = sgpr(wave_sum_i32(c));
      if (tot == 0) continue;
      if (tot > PGPU_CQ_CAP) {  // more than a queue's worth in these 2,048 docs: two halves of <= 1,024 each
        for (int h = 0; h < 2; ++h) {
          const bool mine = (lane >> 5) == h;
          const int ch = mine ? c : 0;
          const int th = sgpr(wave_sum_i32(ch));
          if (qn + th > PGPU_CQ_CAP) {
            flush_queue<MODE, NW>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
            qn = 0;
          }
          int at = qn + wave_excl_scan(ch);
          uint32_t y = mine ? x : 0u;
          while (y) {
            const int bit = __ffs(y) - 1;
            y &= y - 1u;
            cv.queue[at++] = (uint16_t)((w0 + lane) * 32 + bit);
          }
          qn += th;
        }
        continue;
      }
      if (qn + tot > PGPU_CQ_CAP) {
        flush_queue<MODE, NW>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
        qn = 0;
      }
      int at = qn + wave_excl_scan(c);
      while (x) {
        const int bit = __ffs(x) - 1;
        x &= x - 1u;
        cv.queue[at++] = (uint16_t)((w0 + lane) * 32 + bit);
      }
      qn += tot;
    }
    if (qn) flush_queue<MODE, NW>(p, L, cv, la, ss, qn, matched, scanned, sector_bytes, dense_bytes, pf);
    PROF_ADD(pf, PGPU_P_C_FLUSH, tq);
  }
  PROF_ADD(pf, PGPU_P_C_TOTAL, t_start);
  if (MODE == PGPU_MODE_AGG) {
#pragma unroll
    for (int a = 0; a < NREG_ACC; ++a)
      if (a < p.nagg && p.aggs[a].fn != PGPU_AGG_COUNT) acc_commit(cv, a, p.aggs[a].op, la.v[a]);
  }
  Stats st;
  st.matched = matched;
  st.scanned = scanned;
  st.sector_bytes = sector_bytes;
  st.dense_bytes = dense_bytes;
  direct_epilogue<MODE>(p, L, st, wave, lane, pf);
}

// ---- the query kernel ----------------------------------------------------------------------------------------------
template <int MODE, int DENSE>
__global__ __launch_bounds__(PGPU_THREADS(DENSE), 1) void query_kernel(DevParams p) {
  constexpr int NT = PGPU_THREADS(DENSE), NWAVES = PGPU_WAVES_OF(DENSE), NLOAD = PGPU_NLOAD_OF(DENSE);
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Lds L = carve<DENSE>(dyn_smem, p);
  for (int i = threadIdx.x; i < 3 * PGPU_RING_MAX; i += NT) L.full[i] = 0;
  if (MODE == PGPU_MODE_LDS) {
    const int n = p.nsec * (int)p.G;
    for (int i = threadIdx.x; i < n; i += NT) L.ltab[i] = sec_identity(p.sec_op[i / (int)p.G]);
  }
  if (MODE == PGPU_MODE_PART)
    for (int i = threadIdx.x; i < p.nparts; i += NT) ((uint32_t*)L.ltab)[i] = 0u;
  __syncthreads();
  // this workgroup's contiguous tile range
  // XCD-aware placement: workgroups are dealt round-robin to the 8 XCDs, so logical rank (b % 8) * (grid / 8) +
  // b / 8 gives each XCD one contiguous run of tiles -- a few segments, whose dictionaries then stay in that
  // XCD's L2 instead of every XCD cycling through all of them
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int t0 = (int)(((int64_t)p.total_tiles * lb) / nb);
  const int t1 = (int)(((int64_t)p.total_tiles * (lb + 1)) / nb);
  Stats st;
  st.matched = st.scanned = st.sector_bytes = st.dense_bytes = 0;
  Prof pf;
#ifdef PGPU_PROFILE_BUILD
  pf.on = (p.flags & PGPU_FLAG_PROFILE) != 0;
#pragma unroll
  for (int k = 0; k < PGPU_NPROF; ++k) pf.t[k] = 0;
#endif
  if (wave < NLOAD) loader<NLOAD>(p, L, wave, t0, t1 - t0, pf);
  else st = consumer<MODE, DENSE>(p, L, wave - NLOAD, t0, t1 - t0, pf);
  const size_t w = (size_t)blockIdx.x * NWAVES + wave;
#ifdef PGPU_PROFILE_BUILD
  if (pf.on && lane == 0) {
    int64_t* o = p.prof + w * PGPU_NPROF;
#pragma unroll
    for (int k = 0; k < PGPU_NPROF; ++k) o[k] = pf.t[k];
  }
#endif

  // ---- epilogue ----
  if (lane == 0) {
    int64_t* o = p.stats + w * PGPU_NSTATS;
    o[PGPU_STAT_MATCHED] = st.matched;
    o[PGPU_STAT_SCANNED] = st.scanned;
    o[PGPU_STAT_SECTOR_BYTES] = st.sector_bytes;
    o[PGPU_STAT_DENSE_BYTES] = st.dense_bytes;
  }
  if (MODE == PGPU_MODE_AGG) {
    // slab[wave][sec]: section 0 = matched count; reduced in wave order by finalize_kernel (deterministic)
    int64_t* slab = p.slab + w * p.nsec;
    if (lane == 0) slab[0] = st.matched;
    if (lane < p.nagg && p.aggs[lane].fn != PGPU_AGG_COUNT) {
      const int64_t* acc =
          (const int64_t*)(L.cons + (size_t)(wave >= NLOAD ? wave - NLOAD : 0) * p.cons_bytes +
                           p.mask_rows * 256 + PGPU_CONS_LIST_BYTES_OF(DENSE));
      slab[p.aggs[lane].sec] = wave < NLOAD ? sec_identity(p.aggs[lane].op) : acc[lane];
    }
  } else if (MODE == PGPU_MODE_LDS) {
    __syncthreads();
    const int G = (int)p.G;
    for (int key = threadIdx.x; key < G; key += NT) {
      const int64_t cnt = L.ltab[key];
      if (cnt == 0) continue;
      atomicAdd((unsigned long long*)&p.table[key], (unsigned long long)cnt);
      for (int s = 1; s < p.nsec; ++s) cell_atomic(&p.table[(size_t)s * p.G + key], p.sec_op[s], L.ltab[s * G + key]);
    }
  } else if (MODE == PGPU_MODE_PART) {
    __syncthreads();
    for (int q = threadIdx.x; q < p.nparts; q += NT) {
      const uint32_t n = ((const uint32_t*)L.ltab)[q];
      p.rcount[(size_t)q * gridDim.x + blockIdx.x] = n < (uint32_t)p.rcap ? n : (uint32_t)p.rcap;
    }
  }
}

// ---- PART mode, phase 1 without the ring: part_scan_kernel ------------------------------------------------------
// Used when every segment's filter is a dense program (no candidate queue): each wave reads its tiles' columns
// straight from HBM (lane l's b consecutive words of each column: the whole tile is one contiguous read per column)
// and appends the matched docs' records to its workgroup's region of each key partition through an LDS
// write-combining ring per partition (p.pscan records, >= two 128-B lines).  Steps are workgroup-synchronous:
//   insert  every wave takes a slot per record on the partition's LDS tail (the slot IS the record's position in
//           the region) and writes the record into the ring, or straight to HBM when the ring is full;
//   flush   the ring's complete 128-B lines (all of them at the end) are written out, two lines per store
//           instruction (lanes 0-31 / 32-63) -- HBM sees whole lines instead of one 4-B store per record.
#if TU_HAS(3)
#define PGPU_PSCAN_THREADS 256
#define PGPU_PSCAN_WAVES (PGPU_PSCAN_THREADS / 64)

// one record to its region position `slot`, or into the HBM table when the region is full
FI void pscan_put(const DevParams& p, uint32_t q, uint32_t slot, uint32_t cap, uint32_t r0, uint32_t r1) {
  if (slot < cap) {
    const size_t at = part_base(p, q, blockIdx.x) + slot;
    if (p.rw == 1) p.recs[at] = r0;
    else *(u32x2*)(p.recs + 2 * at) = u32x2{r0, r1};
  } else if (p.rw == 2) {
    part_spill(p, r0, r1);
  } else if (p.rec_idbits) {
    part_spill(p, (q << p.pshift) | (r0 >> p.rec_idbits), r0 & ((1u << p.rec_idbits) - 1u));
  } else {
    part_spill(p, r0, 0u);
  }
}

// Flush this wave's share of the partitions (64 per pass): every complete 128-B line of a ring (every record when
// `final`).  A lane first settles its partition's range [H, E) and head.  Whole lines below the region's end go
// out eight partitions per step: 8 lanes per line, one 16-B ds_read_b128 / global_store_dwordx4 each, offsets in
// 32 bits from the workgroup's region block.  The rest -- a line's head or tail piece (after a ring overflow, and
// at the end) and records past a full region -- are walked one flagged partition at a time.
FI void pscan_flush(const DevParams& p, uint32_t* ht, const uint32_t* ring,
                    const uint32_t* lcap, const uint32_t* loff, uint32_t RC, int wave, bool final) {
  const int lane = lane_id(), np = p.nparts, g = lane >> 3, sub = lane & 7;
  const uint32_t rw = (uint32_t)p.rw, lsh = rw == 1 ? 5u : 4u, line = 1u << lsh;  // records per 128-B line
  uint32_t* wrec = p.recs + (size_t)blockIdx.x * p.pblock * rw;  // this workgroup's block (part_base)
  for (int qb = wave * 64; qb < np; qb += 64 * PGPU_PSCAN_WAVES) {
    const int q = qb + lane;
    uint32_t H = 0, E = 0, cap = 0, off = 0;
    if (q < np) {
      H = ht[2 * q + 1];
      cap = lcap[q];
      off = loff[q];
      const uint32_t T = ht[2 * q];
      if (T - H > RC) {  // the ring overflowed this step: it holds [H, H + RC), the rest went straight to HBM
        E = H + RC;
        ht[2 * q + 1] = T;
      } else {
        E = final ? T : (T & ~(line - 1u));
        if (E < H) E = H;
        ht[2 * q + 1] = E;
      }
    }
    if (!__ballot(E > H)) continue;
    // whole lines [FL, LL) (line numbers) inside the region
    const uint32_t FL = (H + line - 1u) >> lsh;
    uint32_t LL = min(E, cap) >> lsh;
    if (LL < FL) LL = FL;
    const bool rest = E > H && ((FL << lsh) != H || (LL << lsh) != E);
#pragma unroll 2
    for (int pb = 0; pb < 64; pb += 8) {
      const int src = pb + g;
      const uint32_t fl = (uint32_t)__shfl((int)FL, src, 64), ll = (uint32_t)__shfl((int)LL, src, 64);
      const uint32_t of = (uint32_t)__shfl((int)off, src, 64);
      const uint32_t qq = (uint32_t)(qb + src);
      for (uint32_t l = fl; l < ll; ++l) {
        const uint32_t s = l << lsh;
        const u32x4 v = *(const u32x4*)(ring + (qq * RC + (s & (RC - 1))) * rw + 4 * sub);
        *(u32x4*)(wrec + (of + s) * rw + 4 * sub) = v;
      }
    }
    // head / tail pieces and records past the region's end, one flagged partition at a time (a ring overflows in a
    // few partitions per step: walking every partition here cost half of phase 1): its values in SGPRs, lane l takes
    // dword l of the 256 bytes from the piece's first line on
    uint64_t todo = __ballot(rest);
    uint64_t spill = 0;
    while (todo) {
      const int src = __builtin_ctzll(todo);
      todo &= todo - 1;
      const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)H, src);
      const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)E, src);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)FL, src) << lsh;
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)LL, src) << lsh;
      const uint32_t cp = (uint32_t)__builtin_amdgcn_readlane((int)cap, src);
      const uint32_t of = (uint32_t)__builtin_amdgcn_readlane((int)off, src);
      const uint32_t qq = (uint32_t)(qb + src);
      bool full = false;
      for (uint32_t s0 = h & ~(line - 1u); s0 < e; s0 += 64u / rw) {
        const uint32_t s = s0 + (uint32_t)lane / rw;
        if (s < h || s >= e || (s >= lo && s < hi)) continue;
        if (s < cp) wrec[(of + s) * rw + (lane & (rw - 1))] = ring[(qq * RC + (s & (RC - 1))) * rw + (lane & (rw - 1))];
        else full = true;
      }
      if (__ballot(full)) spill |= 1ull << src;
    }
    // region full (rare): the records past the region's end go to the HBM table with atomics
    while (spill) {
      const int src = __builtin_ctzll(spill);
      spill &= spill - 1;
      const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)H, src);
      const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)E, src);
      const uint32_t cp = (uint32_t)__builtin_amdgcn_readlane((int)cap, src);
      const uint32_t qq = (uint32_t)(qb + src);
      for (uint32_t s0 = std::max(h, cp); s0 < e; s0 += 64u) {
        const uint32_t s = s0 + (uint32_t)lane;
        if (s >= e) continue;
        const uint32_t* r = ring + (qq * RC + (s & (RC - 1))) * rw;
        pscan_put(p, qq, s, cp, r[0], rw == 2 ? r[1] : 0u);
      }
      __builtin_amdgcn_s_waitcnt(0);  // nothing of this rare path stays pending into the store loops above
    }
  }
}

// COUNT: the sizing pass -- every psample-th tile, matched records counted per partition into pcount, nothing
// written.  Otherwise phase 1 proper.
// KB, VB > 0 (phase 1 proper only): every segment's group key and carried column are fixed-bit columns of KB / VB
// bits and there is no filter -- the next step's tile words are loaded a step ahead, raw, into VGPRs (phase 1 runs
// two waves per SIMD, bound by its LDS rings, so the registers are free), and the step's own HBM latency overlaps
// the previous step's inserts, flush and barriers.
template <bool COUNT, int KB = 0, int VB = 0>
__global__ __launch_bounds__(PGPU_PSCAN_THREADS, 2) void part_scan_kernel(DevParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int np = p.nparts;
  const uint32_t RC = (uint32_t)p.pscan;  // ring records per partition (power of two)
  const int npad = (np + 64 + 2) & ~1;   // + the cancel word; keeps the ring 16-B aligned
  // [npad] pairs {tail, head} (one 8-B word per partition: a record's slot and the partition's head come back from
  // one 64-bit LDS atomic): tail = slots taken (records of this workgroup in the partition), head = first slot not
  // yet written out; the 64 lanes' dummy partitions follow the real ones, then the cancel word (head of np + 64)
  uint32_t* ht = (uint32_t*)dyn_smem;
  uint32_t* lcap = ht + 2 * npad;         // [npad] region capacity / offset in the block per partition
  uint32_t* loff = lcap + npad;
  uint32_t* ring = loff + npad;           // [np][RC * rw], then one dummy record per lane
  Cons cv;
  cv.masks = (uint32_t*)((unsigned char*)(ring + ((size_t)np * RC + 64) * p.rw) + (size_t)wave * p.pscan_wave_bytes);
  cv.queue = nullptr;
  cv.klist = cv.vlist = nullptr;
  cv.acc = nullptr;
  cv.qtiles = nullptr;
  for (int i = threadIdx.x; i < 2 * npad; i += PGPU_PSCAN_THREADS) ht[i] = 0u;
  // the hottest partition of the sampling pass (skewed keys): its records take their slots with one atomic per wave
  // instruction (a ballot over the lanes that hit it) instead of 64 atomics on one LDS address
  uint32_t hq = 0xFFFFFFFFu;
  if (!COUNT && p.pcap) {  // every wave reduces the sampled counts itself (no LDS: the rings have it all)
    uint64_t best = 0;     // (count << 32 | partition): the largest count wins
    for (int q = lane; q < np; q += 64) best = std::max(best, ((uint64_t)p.pcount[q] << 32) | (uint32_t)q);
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t x = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(best >> 32), o, 64) << 32) |
                         (uint32_t)__shfl_xor((int)(uint32_t)best, o, 64);
      best = std::max(best, x);
    }
    uint64_t tot = 0;
    for (int q = lane; q < np; q += 64) tot += p.pcount[q];
    tot = (uint64_t)wave_sum_i64((int64_t)tot);
    // only a really hot partition (>= 4x the mean: skewed keys) -- for even keys the ballots cost more than the
    // same-address atomics they save
    if ((best >> 32) && (best >> 32) * (uint64_t)np >= 4 * tot)
      hq = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)best);
  }
  if (!COUNT)
    for (int i = threadIdx.x; i < np; i += PGPU_PSCAN_THREADS) {
      lcap[i] = part_cap(p, i);
      loff[i] = p.poff ? p.poff[i] : (uint32_t)i * (uint32_t)p.rcap;
    }
  __syncthreads();
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int S = COUNT ? p.psample : 1;
  const int ntl = COUNT ? (p.total_tiles + S - 1) / S : p.total_tiles;  // tiles of this pass
  const int t0 = (int)(((int64_t)ntl * lb) / nb);
  const int t1 = (int)(((int64_t)ntl * (lb + 1)) / nb);
  const uint32_t pmask = (1u << p.pshift) - 1u;
  const int idbits = p.rec_idbits;
  int64_t matched = 0, scanned = 0, dense_bytes = 0;
  Prof pf;
#ifdef PGPU_PROFILE_BUILD
  pf.on = !COUNT && (p.flags & PGPU_FLAG_PROFILE) != 0;
#pragma unroll
  for (int k = 0; k < PGPU_NPROF; ++k) pf.t[k] = 0;
#endif
  const int64_t t_all = now(pf);
  SegState ss;
  int cseg = -1;
  const int nsteps = (t1 - t0 + PGPU_PSCAN_WAVES - 1) / PGPU_PSCAN_WAVES;
  constexpr bool PF = KB > 0 && VB > 0 && !COUNT;
  uint32_t nkw[PF ? KB : 1], nvw[PF ? VB : 1];  // the next step's raw words (PF)
  auto prefetch = [&](int ptile) {
    if constexpr (PF) {
      if (ptile < t1 && ptile < p.total_tiles) {
        const Cursor cn = cursor_at(p, ptile);
        const DevColumn* pc = p.cols + cld(&p.segs[cn.seg].col_begin);
        hbm_lane_raw<KB>(cld(&pc[p.gcols[0]].fwd), cn.tile_in_seg, nkw);
        hbm_lane_raw<VB>(cld(&pc[p.pcol].fwd), cn.tile_in_seg, nvw);
      }
    }
  };
  prefetch(t0 + wave);
  for (int step = 0; step < nsteps; ++step) {
    const int tile = (t0 + step * PGPU_PSCAN_WAVES + wave) * S;
    int64_t tp = now(pf);
    uint32_t ckw[PF ? KB : 1], cvw[PF ? VB : 1];
    if constexpr (PF) {
#pragma unroll
      for (int k = 0; k < KB; ++k) ckw[k] = nkw[k];
#pragma unroll
      for (int k = 0; k < VB; ++k) cvw[k] = nvw[k];
      prefetch(tile + PGPU_PSCAN_WAVES);
    }
    if (tile < t1 * S && tile < p.total_tiles) {
      if (pf.on) pf.t[PGPU_P_C_TILES] += 1;
      const Cursor cu = cursor_at(p, tile);
      if (cu.seg != cseg) {
        cseg = cu.seg;
        load_seg(p, cseg, ss);
      }
      TileCtx t;
      t.ss = &ss;
      t.slot = nullptr;
      t.tile_in_seg = cu.tile_in_seg;
      t.doc0 = cu.tile_in_seg * WT;
      t.lane_doc0 = t.doc0 + 32 * lane;
      const int ndocs = min(WT, ss.num_docs - t.doc0);
      {
        const int rem = ndocs - 32 * lane;
        t.valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
      }
      uint32_t mm = t.valid;
      if (ss.prog_len > 0) mm = run_program(p, cv, ss.prog_begin, ss.prog_len, t, scanned, dense_bytes, pf);
      const int nm = wave_sum_i32(__popc(mm));
      if (lane == 0) matched += nm;
      if (!COUNT) mark_seg(p, ss, nm != 0);
      if (nm) {
        // group keys (mixed radix of remapped ids) and the carried value / dict id, in registers
        uint32_t key[32], val[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) key[i] = val[i] = 0;
        if constexpr (PF) {  // (one group column; ngcols is 1)
#pragma unroll
          for (int k = 0; k < KB; ++k) ckw[k] = bswap32(ckw[k]);
          uint32_t ids[32];
          unpack_b<KB>(ckw, ids);
          const int32_t* remap = cld(ss.remaps, 0);
          if (remap) {
#pragma unroll
            for (int i = 0; i < 32; ++i) ids[i] = lane_bit(mm, i) ? (uint32_t)gld(remap, ids[i]) : 0u;
          }
          const uint32_t st = p.gstride[0];
#pragma unroll
          for (int i = 0; i < 32; ++i) key[i] = ids[i] * st;
          if ((p.flags & PGPU_FLAG_STATS) && lane == 0) dense_bytes += ((int64_t)ndocs * KB + 7) / 8;
        }
        for (int g = 0; g < (PF ? 0 : p.ngcols); ++g) {
          const DevColumn c = col_of(ss, p.gcols[g]);
          if ((p.flags & PGPU_FLAG_STATS) && lane == 0) dense_bytes += ((int64_t)ndocs * c.bits + 7) / 8;
          uint32_t ids[32];
          column_ids(c.kind, c.bits, nullptr, c.fwd, t.tile_in_seg, ids);
          const int32_t* remap = cld(ss.remaps, g);
          if (remap) {
#pragma unroll
            for (int i = 0; i < 32; ++i) ids[i] = lane_bit(mm, i) ? (uint32_t)gld(remap, ids[i]) : 0u;
          }
          const uint32_t st = p.gstride[g];
#pragma unroll
          for (int i = 0; i < 32; ++i) key[i] += ids[i] * st;
        }
        if (COUNT) {
#pragma unroll
          for (int i = 0; i < 32; ++i)
            if (lane_bit(mm, i)) atomicAdd(&ht[2 * (key[i] >> p.pshift)], 1u);
        } else {
        if (p.pcol >= 0) {
          const DevColumn c = col_of(ss, p.pcol);
          if ((p.flags & PGPU_FLAG_STATS) && lane == 0) dense_bytes += ((int64_t)ndocs * c.bits + 7) / 8;
          if constexpr (PF) {
#pragma unroll
            for (int k = 0; k < VB; ++k) cvw[k] = bswap32(cvw[k]);
            unpack_b<VB>(cvw, val);
          } else {
            column_ids(c.kind, c.bits, nullptr, c.fwd, t.tile_in_seg, val);
          }
          if (!idbits) {
#pragma unroll
            for (int i = 0; i < 32; ++i) val[i] = lane_bit(mm, i) ? gld((const uint32_t*)c.dict, val[i]) : 0u;
          }
        }
        PROF_ADD(pf, PGPU_P_C_FILTER, tp);  // loads, filter, decode
        tp = now(pf);
        // slots first (all LDS atomics in flight together), then the ring writes.  Branch-free per doc: a doc
        // that does not match takes its slot on the lane's own dummy partition (np + lane) and writes the
        // lane's dummy ring entry; only records whose ring is full (rare) take the branch to an HBM store
        const uint32_t dq = (uint32_t)(np + lane);
        uint32_t spm = 0;  // docs whose region is full
        // eight docs at a time: their slots and the partitions' heads come back in one LDS round trip
#pragma unroll
        for (int g8 = 0; g8 < 4; ++g8) {
          uint32_t qq[8], slot[8], hd[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int i = 8 * g8 + j;
            qq[j] = lane_bit(mm, i) ? (key[i] >> p.pshift) : dq;
          }
          uint64_t o[8], hm[8];
          if (hq == 0xFFFFFFFFu) {
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = atomicAdd((unsigned long long*)(ht + 2 * qq[j]), 1ull);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              slot[j] = (uint32_t)o[j];
              hd[j] = (uint32_t)(o[j] >> 32);
            }
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) hm[j] = __ballot(qq[j] == hq);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const bool hot = (hm[j] >> lane) & 1u;
              const int leader = hm[j] ? __builtin_ctzll(hm[j]) : 0;
              o[j] = 0;
              if (!hot || lane == leader)
                o[j] = atomicAdd((unsigned long long*)(ht + 2 * qq[j]), hot ? (unsigned long long)__popcll(hm[j]) : 1ull);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              if (hm[j]) {  // the hot lanes' slots: the leader's base + their rank among the hot lanes
                const int leader = __builtin_ctzll(hm[j]);
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)o[j], leader);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(o[j] >> 32), leader);
                if ((hm[j] >> lane) & 1u)
                  o[j] = ((uint64_t)hi << 32) | (lo + (uint32_t)__popcll(hm[j] & ((1ull << lane) - 1ull)));
              }
              slot[j] = (uint32_t)o[j];
              hd[j] = (uint32_t)(o[j] >> 32);
            }
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int i = 8 * g8 + j;
            const bool live = lane_bit(mm, i);
            const bool in = live && slot[j] - hd[j] < RC;
            const uint32_t r0 = p.rw == 1 ? (idbits ? ((key[i] & pmask) << idbits) | val[i] : key[i]) : key[i];
            const uint32_t at = in ? qq[j] * RC + (slot[j] & (RC - 1)) : (uint32_t)np * RC + lane;
            if (p.rw == 1) ring[at] = r0;
            else *(u32x2*)(ring + 2 * at) = u32x2{r0, val[i]};
            if (live && !in) {  // the partition's ring is full: straight to the region (a store, nothing to wait on)
              if (slot[j] < lcap[qq[j]]) {
                const size_t rec = (size_t)blockIdx.x * p.pblock + loff[qq[j]] + slot[j];
                if (p.rw == 1) p.recs[rec] = r0;
                else *(u32x2*)(p.recs + 2 * rec) = u32x2{r0, val[i]};
              } else {
                spm |= 1u << i;
              }
            }
          }
        }
        // region full (rare): HBM-table atomics, kept out of the loops above so that their dictionary loads put
        // no vmcnt waits on the stores there
        if (__ballot(spm != 0)) {
#pragma unroll
          for (int i = 0; i < 32; ++i)
            if ((spm >> i) & 1u) part_spill(p, key[i], p.pcol >= 0 ? val[i] : 0u);
          __builtin_amdgcn_s_waitcnt(0);
        }
        }
      }
    }
    if (COUNT) continue;
    PROF_ADD(pf, PGPU_P_C_AGG, tp);  // inserts (0 when the tile had no match)
    tp = now(pf);
    __syncthreads();
    PROF_ADD(pf, PGPU_P_C_FULL, tp);  // barrier waits
    tp = now(pf);
    pscan_flush(p, ht, ring, lcap, loff, RC, wave, false);
    if (wave == 0 && step % PGPU_CANCEL_POLL == PGPU_CANCEL_POLL - 1 && query_cancelled(p) && lane == 0) ht[2 * (np + 64) + 1] = 1u;
    PROF_ADD(pf, PGPU_P_C_FLUSH, tp);
    tp = now(pf);
    __syncthreads();
    PROF_ADD(pf, PGPU_P_C_FULL, tp);
    if (ht[2 * (np + 64) + 1]) break;  // cancelled: the workgroup stops together (the word was set before the barrier)
  }
  if (COUNT) {
    __syncthreads();
    for (int q = threadIdx.x; q < np; q += PGPU_PSCAN_THREADS)
      if (ht[2 * q]) atomicAdd(&p.pcount[q], ht[2 * q]);
    return;
  }
  pscan_flush(p, ht, ring, lcap, loff, RC, wave, true);
  const size_t w = (size_t)blockIdx.x * PGPU_PSCAN_WAVES + wave;
  PROF_ADD(pf, PGPU_P_C_TOTAL, t_all);
#ifdef PGPU_PROFILE_BUILD
  if (pf.on && lane == 0) {
    int64_t* o = p.prof + w * PGPU_NPROF;
#pragma unroll
    for (int k = 0; k < PGPU_NPROF; ++k) o[k] = pf.t[k];
  }
#endif
  if (lane == 0) {
    int64_t* o = p.stats + w * PGPU_NSTATS;
    o[PGPU_STAT_MATCHED] = matched;
    o[PGPU_STAT_SCANNED] = scanned;
    o[PGPU_STAT_SECTOR_BYTES] = 0;
    o[PGPU_STAT_DENSE_BYTES] = dense_bytes;
  }
  for (int q = threadIdx.x; q < np; q += PGPU_PSCAN_THREADS)
    p.rcount[(size_t)q * gridDim.x + blockIdx.x] = ht[2 * q] < lcap[q] ? ht[2 * q] : lcap[q];
}

// Region sizing and phase-2 work split from the sampled counts (one 1024-thread workgroup):
//   pcap[q] = the workgroup block's pblock records shared in proportion to count[q] (smoothed so that a
//             partition the sample missed still gets lines), in whole 128-B lines; poff = their prefix sums;
//   p2work  = phase-2 workgroups: partition q gets 1 + its share of the p2grid - np spare workgroups in
//             proportion to its excess over the mean count, each taking a contiguous run of phase-1 regions.
FI uint32_t block_excl_scan(uint32_t v, uint32_t* scratch) {  // 1024 threads; scratch >= 16 words
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t x = (uint32_t)wave_excl_scan((int)v);
  if (lane == 63) scratch[wave] = x + v;
  __syncthreads();
  uint32_t base = 0;
  for (int w = 0; w < wave; ++w) base += scratch[w];
  __syncthreads();
  return base + x;
}

__global__ __launch_bounds__(1024) void part_plan_kernel(DevParams p, int grid1) {
  __shared__ uint32_t scratch[32];
  __shared__ uint64_t tot[2];
  const int np = p.nparts, t = threadIdx.x;
  const uint32_t line = 32u / (uint32_t)p.rw;
  if (t < 2) tot[t] = 0;
  __syncthreads();
  // two partitions per thread (np <= PGPU_PSCAN_MAX_PARTS = 2048)
  uint32_t c[2];
  for (int k = 0; k < 2; ++k) c[k] = 2 * t + k < np ? p.pcount[2 * t + k] : 0u;
  atomicAdd((unsigned long long*)&tot[0], (unsigned long long)(c[0] + c[1]));
  __syncthreads();
  const uint64_t sum = tot[0];
  const uint64_t smooth = sum / (8ull * (uint64_t)np) + 1;  // cold partitions keep ~1/8 of the mean share
  const double wsum = (double)sum + (double)smooth * np;
  // every partition keeps one line; the rest of the block is shared out (floors: the caps never exceed pblock)
  const uint64_t rest = p.pblock > (uint64_t)np * line ? p.pblock - (uint64_t)np * line : 0;
  uint32_t cap[2];
  for (int k = 0; k < 2; ++k) {
    const double share = ((double)c[k] + (double)smooth) / wsum;
    const uint64_t cp = (uint64_t)((double)rest * share) / line * line;
    cap[k] = 2 * t + k < np ? (uint32_t)(line + cp) : 0u;
  }
  const uint32_t off = block_excl_scan(cap[0] + cap[1], scratch);
  for (int k = 0; k < 2; ++k)
    if (2 * t + k < np) {
      p.pcap[2 * t + k] = cap[k];
      p.poff[2 * t + k] = off + (k ? cap[0] : 0u);
    }
  // phase-2 split: a partition of r times the mean count gets round(r) workgroups, scaled into the spare ones
  const double mean = (double)sum / np;
  const int spare = max(0, p.p2grid - np);
  uint32_t ns[2];
  __shared__ uint32_t extra;
  if (t == 0) extra = 0;
  __syncthreads();
  for (int k = 0; k < 2; ++k) {
    uint32_t s = 2 * t + k < np ? 1u : 0u;
    if (s && mean > 0) s = max(1u, (uint32_t)((double)c[k] / mean + 0.5));
    ns[k] = s;
    if (s > 1) atomicAdd(&extra, s - 1);
  }
  __syncthreads();
  for (int k = 0; k < 2; ++k) {
    if (ns[k] > 1 && extra > (uint32_t)spare) ns[k] = 1 + (uint32_t)((uint64_t)(ns[k] - 1) * spare / extra);
  }
  const uint32_t w0 = block_excl_scan(ns[0] + ns[1], scratch);
  for (int k = 0; k < 2; ++k) {
    const uint32_t first = w0 + (k ? ns[0] : 0u);
    for (uint32_t j = 0; j < ns[k]; ++j) {  // share j of ns of the partition's records (RegionWalk)
      int32_t* wk = p.p2work + 4 * (first + j);
      wk[0] = 2 * t + k;
      wk[1] = (int32_t)j;
      wk[2] = (int32_t)ns[k];
      wk[3] = ns[k] > 1;
    }
  }
  // idle tail of the phase-2 grid
  __shared__ uint32_t nused;
  if (t == 1023) nused = w0 + ns[0] + ns[1];
  __syncthreads();
  for (int i = (int)nused + t; i < p.p2grid; i += 1024) p.p2work[4 * i] = -1;
}
#endif  // TU_HAS(3)

// PART mode, phase 2: workgroup q aggregates the records of key partition q (from every phase-1 workgroup's
// region) into an LDS table [nsec][K], then folds it into the HBM table, which holds the identities plus the
// phase-1 spills.  NS = value sections (all reduce the records' one value column); ONE = one-word records.
// SUM values of one-word records come from the shared dictionary (pdict), per LDM:
//   0  gathered from L2 -- one 128-B line per 4-B lookup (~300 G lookups/s chip-wide for a 256-KiB dictionary,
//      tools/gather_bench.hip), the bound of this kernel when the dictionary is large;
//   1  the whole dictionary copied into LDS beside the table (~3,200 G lookups/s).
// Each wave walks its own regions in chunks of R x 64 records; loads are unconditional (clamped indices), so a
// chunk's R loads are in flight together; section ops are uniform, so a chunk runs one branch-free atomic loop
// per section.
// A value of the frame-of-reference dictionary image in LDS: block base + the id's fbits-bit offset (it may straddle
// two words).
FI uint32_t for_value(const uint32_t* fimg, int fnblk, int fbits, uint32_t id) {
  const uint32_t blk = id >> 5, bit = (id & 31u) * (uint32_t)fbits;
  const uint32_t* wds = fimg + fnblk + (size_t)blk * fbits + (bit >> 5);
  const uint64_t two = (uint64_t)wds[0] | ((uint64_t)wds[1] << 32);
  return fimg[blk] + (uint32_t)((two >> (bit & 31u)) & ((1ull << fbits) - 1ull));
}

template <int NS, int R>
FI void part_reduce_batch(int64_t* ptab, uint32_t K, const int32_t (&op)[NS > 0 ? NS : 1], int32_t vt, int idbits,
                          const uint32_t (&k)[R], const uint32_t (&raw)[R], const uint32_t (&val)[R],
                          const bool (&ok)[R]) {
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (ok[r]) atomicAdd((unsigned long long*)&ptab[k[r]], 1ull);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    int64_t* sec = ptab + (size_t)(1 + s) * K;
    if (op[s] == PGPU_RED_SUM_I64) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (ok[r]) atomicAdd((unsigned long long*)&sec[k[r]], (unsigned long long)(int64_t)(int32_t)val[r]);
    } else if (op[s] == PGPU_RED_SUM_F64) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (ok[r]) atomicAdd((double*)&sec[k[r]], (double)__uint_as_float(val[r]));
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (!ok[r]) continue;
        const int64_t c = idbits ? (int64_t)raw[r] : raw_to_cell(raw[r], vt, op[s]);
        if (op[s] == PGPU_RED_MIN_I64) atomicMin((long long*)&sec[k[r]], (long long)c);
        else atomicMax((long long*)&sec[k[r]], (long long)c);
      }
    }
  }
}

// Phase 2 of a partition split over several workgroups (part_plan_kernel): workgroup j of ns takes the records
// [j * T / ns, (j + 1) * T / ns) of the partition's T records, counted across the phase-1 regions in region order,
// so a heavy partition's share does not depend on how its records fell into regions.  Each wave walks the regions
// round-robin (region w to wave w % nwaves) and gets (region base + first record, record count) per region it
// holds a non-empty piece of.
struct RegionWalk {
  const DevParams* p;
  uint32_t q;
  int nwg, wave, nwaves;
  // all: every wave walks every piece and the caller deals each piece's chunks out across the waves.  A split
  // partition's share is a few large pieces (Zipf(1.1): ~2 phase-1 regions of ~2.7 M records per workgroup), so
  // dealing whole pieces to waves left 14 of 16 waves idle; an unsplit partition's are many small pieces, dealt whole.
  bool all;
  uint64_t r0, r1;     // this workgroup's record range in the partition
  uint64_t run;        // records of the regions before the current chunk of 64
  int wb;              // current chunk's first region
  uint64_t todo;       // lanes (regions) of the chunk left for this wave
  uint64_t excl;       // lane's region: first record (partition-wide)
  uint32_t cnt;        // lane's region: records
  size_t base;         // out: first record's index in p.recs
  uint32_t n;          // out: records
  int visited;
  FI RegionWalk(const DevParams& pp, uint32_t qq, int j, int ns, int nw, int wv, int nwv)
      : p(&pp), q(qq), nwg(nw), wave(wv), nwaves(nwv), all(ns > 1), run(0), wb(-64), todo(0), excl(0), cnt(0), base(0),
        n(0), visited(0) {
    r0 = 0;
    r1 = ~0ull;
    if (ns > 1) {
      uint64_t t = 0;
      for (int w = lane_id(); w < nwg; w += 64) t += pp.rcount[(size_t)qq * nwg + w];
      t = (uint64_t)wave_sum_i64((int64_t)t);
      r0 = t * (uint64_t)j / (uint64_t)ns;
      r1 = t * (uint64_t)(j + 1) / (uint64_t)ns;
    }
  }
  FI bool next() {
    while (!todo) {
      wb += 64;
      if (wb >= nwg) return false;
      const int w = wb + lane_id();
      const uint32_t c = w < nwg ? p->rcount[(size_t)q * nwg + w] : 0u;
      // 64-bit prefix of 32-bit counts: the high and low halves scanned apart (each sum < 2^22)
      excl = run + ((uint64_t)(uint32_t)wave_excl_scan((int)(c >> 16)) << 16) +
             (uint64_t)(uint32_t)wave_excl_scan((int)(c & 0xFFFFu));
      run += (uint64_t)wave_sum_i64((int64_t)c);
      cnt = c;
      const bool mine = w < nwg && (all || w % nwaves == wave) && excl < r1 && excl + c > r0;
      todo = __ballot(mine);
    }
    const int l = __builtin_ctzll(todo);
    todo &= todo - 1;
    const uint64_t e = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(excl >> 32), l) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)excl, l);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cnt, l);
    const uint64_t a = e > r0 ? e : r0, b2 = e + c < r1 ? e + c : r1;
    base = part_base(*p, q, (uint32_t)(wb + l)) + (size_t)(a - e);
    n = (uint32_t)(b2 - a);
    ++visited;
    return true;
  }
};

template <int NS, bool ONE, int LDM>
__global__ __launch_bounds__(1024) void part_reduce_kernel(DevParams p, int nwg) {
  extern __shared__ __attribute__((aligned(16))) int64_t ptab[];
  uint32_t* sdict = (uint32_t*)(ptab + (size_t)(NS + 1) * (1u << p.pshift));  // LDM 1: [1 << slice_shift]
  const uint32_t K = 1u << p.pshift;
  // this workgroup's partition and run of phase-1 regions [w0, w1) (part_plan_kernel), or all of partition blockIdx.x
  uint32_t q = blockIdx.x;
  int pj = 0, pns = 1;  // this workgroup's share j of ns of the partition's records
  bool split = false;
  if (p.p2work) {
    const int32_t* wk = p.p2work + 4 * blockIdx.x;
    if (wk[0] < 0) return;
    q = (uint32_t)wk[0];
    pj = wk[1];
    pns = wk[2];
    split = wk[3] != 0;
  }
  const uint64_t key0 = (uint64_t)q * K;
  const uint32_t nk = (uint32_t)min((uint64_t)K, p.G - key0);
  const int lane = lane_id(), wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  int32_t op[NS > 0 ? NS : 1];
#pragma unroll
  for (int s = 0; s < NS; ++s) op[s] = p.sec_op[1 + s];
  if constexpr (LDM == 2) {
    int32_t vt = PGPU_INT;
    for (int a = 0; a < p.nagg; ++a)
      if (p.aggs[a].fn != PGPU_AGG_COUNT) vt = p.aggs[a].vtype;
    // compact table beside the frame-of-reference dictionary: count u32, SUM sections int64, MIN / MAX sections
    // u32 dict ids (one-word records reduce ids), so 4096 keys and a 64K-value image fit the LDS together
    unsigned char* base = (unsigned char*)ptab;
    uint32_t* cnt = (uint32_t*)base;
    uint32_t soff[NS > 0 ? NS : 1];
    uint32_t at = 4u * K;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      soff[s] = at;
      at += (op[s] == PGPU_RED_SUM_I64 || op[s] == PGPU_RED_SUM_F64) ? 8u * K : 4u * K;
    }
    uint32_t* fimg = (uint32_t*)(base + at);
    const int fbits = p.for_bits, fnblk = p.for_nblk;
    for (uint32_t i = threadIdx.x; i < K; i += blockDim.x) {
      cnt[i] = 0u;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if (op[s] == PGPU_RED_SUM_I64 || op[s] == PGPU_RED_SUM_F64) ((int64_t*)(base + soff[s]))[i] = 0;
        else ((uint32_t*)(base + soff[s]))[i] = op[s] == PGPU_RED_MIN_I64 ? 0xFFFFFFFFu : 0u;
      }
    }
    for (uint32_t i = threadIdx.x; i < (uint32_t)(fnblk * (1 + fbits) + 1); i += blockDim.x) fimg[i] = gld(p.pfor, i);
    __syncthreads();
    const int idbits = p.rec_idbits;
    const uint32_t idmask = (1u << idbits) - 1u;
    constexpr int R = 16;
    RegionWalk rwk(p, q, pj, pns, nwg, wave, nwaves);
    while (rwk.next()) {
      if (rwk.visited % 8 == 0 && query_cancelled(p)) break;
      const uint32_t n = rwk.n;
      const size_t rb = rwk.base;
      for (uint32_t i0 = (rwk.all ? wave : 0) * R * 64; i0 < n; i0 += (rwk.all ? nwaves : 1) * R * 64) {
        uint32_t k[R], id[R];
        bool ok[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint32_t i = i0 + r * 64 + lane;
          ok[r] = i < n;
          const uint32_t v = gld(p.recs, rb + (ok[r] ? i : n - 1));
          k[r] = v >> idbits;
          id[r] = v & idmask;
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (ok[r]) atomicAdd(&cnt[k[r]], 1u);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          if (op[s] == PGPU_RED_SUM_I64 || op[s] == PGPU_RED_SUM_F64) {
            unsigned long long* sec = (unsigned long long*)(base + soff[s]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
              if (!ok[r]) continue;
              atomicAdd(&sec[k[r]], (unsigned long long)(int64_t)(int32_t)for_value(fimg, fnblk, fbits, id[r]));
            }
          } else {
            uint32_t* sec = (uint32_t*)(base + soff[s]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
              if (!ok[r]) continue;
              if (op[s] == PGPU_RED_MIN_I64) atomicMin(&sec[k[r]], id[r]);
              else atomicMax(&sec[k[r]], id[r]);
            }
          }
        }
      }
    }
    __syncthreads();
    for (uint32_t kk = threadIdx.x; kk < nk; kk += blockDim.x) {
      if (cnt[kk] == 0u) continue;
      for (int s = 0; s <= NS; ++s) {
        int64_t v;
        if (s == 0) {
          v = (int64_t)cnt[kk];
        } else if (op[s - 1] == PGPU_RED_SUM_I64 || op[s - 1] == PGPU_RED_SUM_F64) {
          v = ((const int64_t*)(base + soff[s - 1]))[kk];
        } else {  // id -> cell key of its value
          v = raw_to_cell(gld((const uint32_t*)p.pdict, ((const uint32_t*)(base + soff[s - 1]))[kk]), vt, p.sec_op[s]);
        }
        int64_t* cell = &p.table[(size_t)s * p.G + key0 + kk];
        if (split) cell_atomic(cell, p.sec_op[s], v);
        else *cell = cell_combine(p.sec_op[s], *cell, v);
      }
    }
    return;
  }
  int32_t vt = PGPU_INT;
  for (int a = 0; a < p.nagg; ++a)
    if (p.aggs[a].fn != PGPU_AGG_COUNT) vt = p.aggs[a].vtype;
  for (uint32_t i = threadIdx.x; i < (uint32_t)(NS + 1) * K; i += blockDim.x)
    ptab[i] = sec_identity(p.sec_op[i >> p.pshift]);
  const uint32_t slice = 1u << p.slice_shift;
  if (LDM == 1)
    for (uint32_t i = threadIdx.x; i < slice; i += blockDim.x)
      sdict[i] = i < p.pdict_n ? gld((const uint32_t*)p.pdict, i) : 0u;
  const int fbits = p.for_bits, fnblk = p.for_nblk;
  if (LDM == 2)  // the frame-of-reference image: int32 block bases, then the packed offsets
    for (uint32_t i = threadIdx.x; i < (uint32_t)(fnblk * (1 + fbits) + 1); i += blockDim.x) sdict[i] = gld(p.pfor, i);
  __syncthreads();
  // one-word records: (in-partition key << idbits | dict id) over the shared dictionary; MIN / MAX sections reduce
  // the dict ids (sorted dictionary) and are turned into cell keys when folded into the HBM table
  const int idbits = ONE ? p.rec_idbits : 0;
  const uint32_t idmask = idbits ? (1u << idbits) - 1u : 0u;
  bool need_val = false;
#pragma unroll
  for (int s = 0; s < NS; ++s) need_val |= op[s] == PGPU_RED_SUM_I64 || op[s] == PGPU_RED_SUM_F64;
  {
    constexpr int R = 16;
    RegionWalk rwk(p, q, pj, pns, nwg, wave, nwaves);
    while (rwk.next()) {
      if (rwk.visited % 8 == 0 && query_cancelled(p)) break;
      const uint32_t n = rwk.n;
      const size_t base = rwk.base;
      for (uint32_t i0 = (rwk.all ? wave : 0) * R * 64; i0 < n; i0 += (rwk.all ? nwaves : 1) * R * 64) {
        uint32_t k[R], raw[R], val[R];
        bool ok[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint32_t i = i0 + r * 64 + lane;
          ok[r] = i < n;
          const size_t at = base + (ok[r] ? i : n - 1);
          if (ONE) {
            const uint32_t v = gld(p.recs, at);
            k[r] = idbits ? v >> idbits : v - (uint32_t)key0;
            raw[r] = v & idmask;
          } else {
            const u32x2 v = gld((const u32x2*)p.recs, at);
            k[r] = v.x - (uint32_t)key0;
            raw[r] = v.y;
          }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) val[r] = raw[r];
        if (idbits && need_val) {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            if (LDM == 1) {
              val[r] = sdict[raw[r] & (slice - 1)];
            } else if (LDM == 2) {
              // value = block base + the id's fbits-bit offset (may straddle two words)
              const uint32_t id = ok[r] ? raw[r] : 0u, blk = id >> 5, bit = (id & 31u) * (uint32_t)fbits;
              const uint32_t* wds = sdict + fnblk + (size_t)blk * fbits + (bit >> 5);
              const uint64_t two = (uint64_t)wds[0] | ((uint64_t)wds[1] << 32);
              val[r] = sdict[blk] + (uint32_t)((two >> (bit & 31u)) & ((1ull << fbits) - 1ull));
            } else {
              val[r] = gld((const uint32_t*)p.pdict, raw[r]);
            }
          }
        }
        part_reduce_batch<NS, R>(ptab, K, op, vt, idbits, k, raw, val, ok);
      }
    }
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < nk; k += blockDim.x) {
    if (ptab[k] == 0) continue;
#pragma unroll
    for (int s = 0; s <= NS; ++s) {
      int64_t* cell = &p.table[(size_t)s * p.G + key0 + k];
      int64_t v = ptab[(size_t)s * K + k];
      if (idbits && s > 0 && (p.sec_op[s] == PGPU_RED_MIN_I64 || p.sec_op[s] == PGPU_RED_MAX_I64))
        v = raw_to_cell(gld((const uint32_t*)p.pdict, (uint32_t)v), vt, p.sec_op[s]);  // id -> cell key
      if (split) cell_atomic(cell, p.sec_op[s], v);  // several workgroups share the partition
      else *cell = cell_combine(p.sec_op[s], *cell, v);
    }
  }
}

#if TU_HAS(PGPU_TU_COMMON)
// Table init: count/sum sections 0, MIN +max, MAX -max.
__global__ void table_init_kernel(int64_t* table, uint64_t G, int32_t nsec, DevParams p) {
  const uint64_t n = G * (uint64_t)nsec;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    table[i] = sec_identity(p.sec_op[i / G]);
}

// Reduce AGG-mode slabs into the G=1 table and the per-wave stats: block x reduces column x (a section, then the
// PGPU_NSTATS stats) over all waves with a fixed-shape tree, so double sums are deterministic.
// The query's epilogue, one launch: blocks [0, nsec + NSTATS) reduce the AGG-mode slabs (also into the pinned host
// table) and the per-wave statistics (finalize); the next nseg_blocks turn the numSegmentsMatched words into pinned
// host flags and reset them; the rest copy a non-AGG table into pinned host memory (the three are independent).
__global__ __launch_bounds__(256) void finalize_kernel(DevParams p, int32_t nslabs, int64_t* stats_out, uint8_t* seg_out,
                                                       int32_t nseg_blocks, int64_t* host_table, uint64_t table_words) {
  __shared__ int64_t red[256];
  const int nfin = p.nsec + PGPU_NSTATS;
  if ((int)blockIdx.x >= nfin) {
    const int b = (int)blockIdx.x - nfin;
    if (b < nseg_blocks) {
      for (int i = b * 256 + threadIdx.x; i < p.nseg; i += nseg_blocks * 256) {
        seg_out[i] = p.segany[i] != 0u ? 1 : 0;
        p.segany[i] = 0u;
      }
    } else {
      const int nb = (int)gridDim.x - nfin - nseg_blocks;
      for (uint64_t i = (uint64_t)(b - nseg_blocks) * 256ull + threadIdx.x; i < table_words; i += nb * 256ull)
        host_table[i] = p.table[i];
    }
    return;
  }
  const int col = blockIdx.x;
  const bool is_stat = col >= p.nsec;
  if (!is_stat && p.mode != PGPU_MODE_AGG) return;
  const int op = is_stat ? PGPU_RED_SUM_I64 : p.sec_op[col];
  const int64_t* src = is_stat ? p.stats + (col - p.nsec) : p.slab + col;
  const int stride = is_stat ? PGPU_NSTATS : p.nsec;
  int64_t v = sec_identity(op);
  for (int b = threadIdx.x; b < nslabs; b += 256) v = cell_combine(op, v, src[(size_t)b * stride]);
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] = cell_combine(op, red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (is_stat) {
      stats_out[col - p.nsec] = red[0];
    } else {
      p.table[col] = red[0];
      if (host_table) host_table[col] = red[0];
    }
  }
}

// ---- host <-> device transfers as kernels ---------------------------------------------------------------------------
// Per-query metadata and results move through pinned host memory read / written by kernels (zero-copy), not
// through DMA-engine copies: a DMA copy queued between two query kernels was measured to hold the next kernel
// back by ~0.13 ms.
// Prologue: blocks [0, ncopy) copy the packed metadata arena from pinned host memory into HBM, the remaining
// blocks initialise the table (count / sum sections 0, MIN +max, MAX -max).
__global__ __launch_bounds__(256) void prologue_kernel(const u32x4* __restrict__ src, u32x4* dst, uint32_t n16,
                                                        int32_t ncopy, DevParams p) {
  if ((int)blockIdx.x < ncopy) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += ncopy * 256) dst[i] = src[i];
    return;
  }
  // table sections (identities), then HASH key words (empty = -1; two-level keys: both tables), then the
  // distinct-key bitmaps of the tracked segments
  const uint64_t n = p.G * (uint64_t)p.nsec;
  const uint64_t nk = p.mode == PGPU_MODE_HASH ? p.G * (uint64_t)p.key_words : 0;
  const uint64_t nm = p.segmask ? (uint64_t)p.segmask_rows * (p.G >> 5) : 0;
  const uint64_t nb = gridDim.x - ncopy;
  for (uint64_t i = (blockIdx.x - ncopy) * 256ull + threadIdx.x; i < n + nk + nm; i += nb * 256) {
    if (i < n) p.table[i] = sec_identity(p.sec_op[i / p.G]);
    else if (i < n + nk) p.table[i] = -1;
    else p.segmask[i - n - nk] = 0u;
  }
}

// Index-only dense programs (ProgJob): one wave per tile evaluates the segment's original program (bitmap / sorted /
// inverted leaves, AND / OR / NOT) and writes the tile's match words; the query kernel then reads one word per lane.
__global__ __launch_bounds__(256) void progbits_kernel(DevParams p, const ProgJob* jobs, int njobs, int total) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  // each wave walks a contiguous run of the jobs' tiles (XCD-aware workgroup order): the job and its segment state
  // are looked up once per run and per job change, not per tile
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int64_t nw = (int64_t)nb * 4, gw = (int64_t)lb * 4 + wave;
  const int gb = (int)((int64_t)total * gw / nw), ge = (int)((int64_t)total * (gw + 1) / nw);
  if (gb >= ge) return;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cld(&jobs[mid].tile0) <= gb) lo = mid; else hi = mid - 1;
  }
  Cons cv;
  cv.masks = (uint32_t*)(dyn_smem + (size_t)wave * p.mask_rows * 256);
  cv.queue = nullptr;
  cv.klist = cv.vlist = nullptr;
  cv.acc = nullptr;
  cv.qtiles = nullptr;
  SegState ss;
  ProgJob jb = cld(jobs + lo);
  load_seg(p, jb.seg, ss);
  for (int g = gb; g < ge; ++g) {
    while (g >= jb.tile0 + jb.ntiles && lo + 1 < njobs) {
      jb = cld(jobs + ++lo);
      load_seg(p, jb.seg, ss);
    }
    const int tile = g - jb.tile0;
    TileCtx t;
    t.ss = &ss;
    t.slot = nullptr;
    t.tile_in_seg = tile;
    t.doc0 = tile * WT;
    t.lane_doc0 = t.doc0 + 32 * lane;
    {
      const int rem = min(WT, ss.num_docs - t.doc0) - 32 * lane;
      t.valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
    }
    int64_t scanned = 0, dense_bytes = 0;
    Prof pf;
    const uint32_t m = run_program(p, cv, jb.prog_begin, jb.prog_len, t, scanned, dense_bytes, pf, &jb);
    jb.out[(size_t)tile * 64 + lane] = m & t.valid;
  }
}

// PGPU_Q_EXACT_FILTER_STATS: the match bits of every leaf of every segment's whole filter program over all its
// docs (one wave per tile, leaves read straight from HBM), for the host replay of the reference's iterators
// (pgpu_iterstats.cpp).
__global__ __launch_bounds__(256) void leafbits_kernel(DevParams p) {
  __shared__ uint32_t scratch[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = (int)blockIdx.x * 4 + wave;
  if (tile >= p.total_tiles) return;
  const Cursor c = cursor_at(p, tile);
  SegState ss;
  load_seg(p, c.seg, ss);
  const int nleaf = cld(&ss.sg->leaf_len);
  if (nleaf == 0) return;
  const int leaf_begin = cld(&ss.sg->leaf_begin);
  const int64_t off = cld(&ss.sg->leaf_bits_off);
  TileCtx t;
  t.ss = &ss;
  t.slot = nullptr;
  t.tile_in_seg = c.tile_in_seg;
  t.doc0 = c.tile_in_seg * WT;
  t.lane_doc0 = t.doc0 + 32 * lane;
  {
    const int rem = min(WT, ss.num_docs - t.doc0) - 32 * lane;
    t.valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
  }
  int64_t dummy = 0;
  for (int k = 0; k < nleaf; ++k) {
    const DevInstr in = cld(p.instrs + cld(p.pool, leaf_begin + k));
    uint32_t m = 0;
    if (in.op == PGPU_I_SCAN) m = leaf_scan(p, t, in, t.valid, dummy);
    else if (in.op == PGPU_I_INV) m = leaf_inv(p, t, in, scratch[wave]) & t.valid;
    else if (in.op == PGPU_I_SORTED) m = leaf_sorted(p, t, in) & t.valid;
    else if (in.op == PGPU_I_BITS) m = leaf_bits(t, in) & t.valid;
    p.leaf_bits[off + (int64_t)k * c.ntiles * 64 + (int64_t)c.tile_in_seg * 64 + lane] = m;
  }
}

// ---- PGPU_Q_EXACT_FILTER_STATS on the GPU: AndDocIdIterator over scan iterators as a finite-state transducer ------
// For a segment whose filter is one AND of k <= 4 SCAN leaves (AndDocIdSet.java:140-143: no index child, so the
// reference leap-frogs AndDocIdIterator over the SVScanDocIdIterators), the reference's numEntriesScannedInFilter is
// numDocs + H.  Every doc is read once by the iterator that is scanning when the walk reaches it, and H counts the
// hand-offs: each advance(target) that starts on a doc another iterator has just read (AndDocIdIterator.java:40-67,
// SVScanDocIdIterator.java:57-71).  The walk's state entering a doc is the scanning iterator s alone: when leaf s
// matches doc d, iterators j = 0..k-1 (j != s) read d in turn (H += 1 each) until one misses -- that one scans on
// (state j) -- or all match (an AND match: next() resumes iterator 0 at d + 1, state 0).  So each doc is a map
// state -> (state', H increment); a tile's map is the composition of its docs' maps (per lane over its 32 docs, then
// across lanes), a segment's the composition of its tiles' maps, evaluated from state 0.
#define PGPU_ANDFSM_WORDS 8  // per tile: next-state bits (2 per start state), then H per start state
FI uint32_t sel4(const uint32_t (&v)[4], int i) { return i == 0 ? v[0] : i == 1 ? v[1] : i == 2 ? v[2] : v[3]; }

template <int B>
FI void sliced_load_fsm(const uint32_t* sl, int tile, uint32_t (&x)[B]) {
  const uint32_t* src = sl + (size_t)tile * 64 * B + lane_id();
#pragma unroll
  for (int k = 0; k < B; ++k) x[k] = __builtin_nontemporal_load(src + 64 * k);
}
// A SCAN leaf's words for the transducer from the column's bit-sliced copy (plane k of lane l at dword
// (tile * B + k) * 64 + l): a dict-id range is lt(hi) & ~lt(lo) (sliced_lt), an id list an OR of [id, id + 1).  A
// (The MSB-first early exit of an EQ leaf -- a wave stops once no doc can match -- measured slower: its dependent
// four-plane rounds leave each tile's loads latency-bound.)
template <int B>
FI uint32_t fsm_sliced_b(const uint32_t* sl, int tile, const DevInstr& in) {
  uint32_t x[B];
  sliced_load_fsm<B>(sl, tile, x);  // every plane in flight at once: one round trip per tile
  uint32_t m;
  if (in.pred == PRED_RANGE) {
    m = sliced_lt<B>(x, (uint32_t)in.hi) & ~sliced_lt<B>(x, (uint32_t)in.lo);
  } else if (in.pred == PRED_MASK) {  // <= 64 ids: one [id, id + 1) per member of the mask
    m = 0;
    for (uint64_t mk = ((uint64_t)(uint32_t)in.hi << 32) | (uint32_t)in.lo; mk; mk &= mk - 1) {
      const uint32_t id = (uint32_t)__builtin_ctzll(mk);
      m |= sliced_lt<B>(x, id + 1u) & ~sliced_lt<B>(x, id);
    }
  } else {
    m = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)  // (fsm_sliced_ok: <= 4 ids; a constant index keeps ids[] out of scratch)
      if (j < in.n) m |= sliced_lt<B>(x, in.ids[j] + 1u) & ~sliced_lt<B>(x, in.ids[j]);
  }
  return in.negate ? ~m : m;
}
// Runtime-width forms (FSM_MAXB planes, each guarded by k < bits: constant register indices, no dispatch), so that
// the planes of several leaves can be in flight together.
#define FSM_MAXB 24
FI void fsm_load_planes(const uint32_t* sl, int bits, int tile, uint32_t (&x)[FSM_MAXB]) {
  const uint32_t* src = sl + (size_t)tile * 64 * bits + lane_id();
#pragma unroll
  for (int k = 0; k < FSM_MAXB; ++k) x[k] = k < bits ? __builtin_nontemporal_load(src + 64 * k) : 0u;
}
FI uint32_t fsm_lt(const uint32_t (&x)[FSM_MAXB], int bits, uint32_t c) {
  if (c >> bits) return ~0u;  // past the largest id
  uint32_t br = 0;
#pragma unroll
  for (int k = 0; k < FSM_MAXB; ++k)
    if (k < bits) br = __builtin_amdgcn_bitop3_b32((uint32_t)-(int32_t)((c >> k) & 1u), x[k], br, 0xB2);
  return br;
}
FI uint32_t fsm_eval_planes(const uint32_t (&x)[FSM_MAXB], const DevInstr& in) {
  const int b = in.bits;
  uint32_t m;
  if (in.pred == PRED_RANGE) {
    m = fsm_lt(x, b, (uint32_t)in.hi) & ~fsm_lt(x, b, (uint32_t)in.lo);
  } else if (in.pred == PRED_MASK) {
    m = 0;
    for (uint64_t mk = ((uint64_t)(uint32_t)in.hi << 32) | (uint32_t)in.lo; mk; mk &= mk - 1) {
      const uint32_t id = (uint32_t)__builtin_ctzll(mk);
      m |= fsm_lt(x, b, id + 1u) & ~fsm_lt(x, b, id);
    }
  } else {
    m = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < in.n) m |= fsm_lt(x, b, in.ids[j] + 1u) & ~fsm_lt(x, b, in.ids[j]);
  }
  return in.negate ? ~m : m;
}
FI bool fsm_sliced_ok(const DevInstr& in, const DevColumn& c) {
  return in.op == PGPU_I_SCAN && in.kind == PGPU_COL_FIXED_BIT && c.sliced && in.bits >= 1 && in.bits <= 24 &&
         (in.pred == PRED_RANGE || in.pred == PRED_MASK || (in.pred == PRED_LIST && in.n >= 1 && in.n <= 4));
}
FI uint32_t fsm_sliced(const uint32_t* sl, int bits, int tile, const DevInstr& in) {
  uint32_t m = 0;
#define FS_CALL(B) m = fsm_sliced_b<B>(sl, tile, in)
  switch (bits) {
    case 1: FS_CALL(1); break;   case 2: FS_CALL(2); break;   case 3: FS_CALL(3); break;   case 4: FS_CALL(4); break;
    case 5: FS_CALL(5); break;   case 6: FS_CALL(6); break;   case 7: FS_CALL(7); break;   case 8: FS_CALL(8); break;
    case 9: FS_CALL(9); break;   case 10: FS_CALL(10); break; case 11: FS_CALL(11); break; case 12: FS_CALL(12); break;
    case 13: FS_CALL(13); break; case 14: FS_CALL(14); break; case 15: FS_CALL(15); break; case 16: FS_CALL(16); break;
    case 17: FS_CALL(17); break; case 18: FS_CALL(18); break; case 19: FS_CALL(19); break; case 20: FS_CALL(20); break;
    case 21: FS_CALL(21); break; case 22: FS_CALL(22); break; case 23: FS_CALL(23); break; default: FS_CALL(24); break;
  }
#undef FS_CALL
  return m;
}

// S2: every segment's filter is an AND of exactly two bit-sliced leaves (the runtime checks fsm_sliced_ok on each),
// so the generic leaf path is compiled out and the kernel fits four waves per SIMD; the general build needs ~226
// VGPRs (two waves).
template <bool S2>
__global__ __launch_bounds__(256, S2 ? 4 : 1) void andfsm_tile_kernel(DevParams p, uint32_t* fn) {
  // each wave walks a contiguous run of tiles (XCD-aware workgroup order), so the segment's state and leaf
  // instructions are loaded once per segment rather than once per tile
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int64_t nw = (int64_t)nb * 4, gw = (int64_t)lb * 4 + wave;
  const int tb = (int)((int64_t)p.total_tiles * gw / nw), te = (int)((int64_t)p.total_tiles * (gw + 1) / nw);
  if (tb >= te) return;
  Cursor c = cursor_at(p, tb);
  int cseg = -1;
  SegState ss;
  int k = 0, leaf_begin = 0;
  DevInstr in0, in1;  // the first two leaves, and whether they are evaluated on bit planes
  bool sl0 = false, sl1 = false;
  const uint32_t *sp0 = nullptr, *sp1 = nullptr;
  for (int tile = tb; tile < te; ++tile) {
  if (tile > tb) cursor_advance(p, c, 1);
  if (c.seg != cseg) {
    cseg = c.seg;
    load_seg(p, cseg, ss);
    k = S2 ? 2 : cld(&ss.sg->leaf_len);
    leaf_begin = cld(&ss.sg->leaf_begin);
    sl0 = sl1 = false;
    if (k > 0) {
      in0 = cld(p.instrs + cld(p.pool, leaf_begin));
      const DevColumn c0 = col_of(ss, in0.col);
      sl0 = fsm_sliced_ok(in0, c0);
      sp0 = c0.sliced;
    }
    if (k > 1) {
      in1 = cld(p.instrs + cld(p.pool, leaf_begin + 1));
      const DevColumn c1 = col_of(ss, in1.col);
      sl1 = fsm_sliced_ok(in1, c1);
      sp1 = c1.sliced;
    }
  }
  TileCtx t;
  t.ss = &ss;
  t.slot = nullptr;
  t.tile_in_seg = c.tile_in_seg;
  t.doc0 = c.tile_in_seg * WT;
  t.lane_doc0 = t.doc0 + 32 * lane;
  {
    const int rem = min(WT, ss.num_docs - t.doc0) - 32 * lane;
    t.valid = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
  }
  int64_t dummy = 0;
  uint32_t m[4] = {0u, 0u, 0u, 0u};
  // the first two leaves, when bit-sliced: every plane of both is loaded before either is evaluated (one round trip
  // per tile instead of one per leaf)
  uint32_t x0[FSM_MAXB], x1[FSM_MAXB];
  if (sl0) fsm_load_planes(sp0, in0.bits, t.tile_in_seg, x0);
  if (sl1) fsm_load_planes(sp1, in1.bits, t.tile_in_seg, x1);
  if (sl0) m[0] = fsm_eval_planes(x0, in0) & t.valid;
  if (sl1) m[1] = fsm_eval_planes(x1, in1) & t.valid;
#pragma unroll
  for (int j = 0; j < (S2 ? 0 : 4); ++j) {
    if (j >= k) break;
    if ((j == 0 && sl0) || (j == 1 && sl1)) continue;
    const DevInstr in = cld(p.instrs + cld(p.pool, leaf_begin + j));
    const DevColumn col = col_of(ss, in.col);
    if (fsm_sliced_ok(in, col)) m[j] = fsm_sliced(col.sliced, in.bits, t.tile_in_seg, in) & t.valid;
    else m[j] = (in.op == PGPU_I_SCAN ? leaf_scan(p, t, in, t.valid, dummy) : leaf_bits(t, in)) & t.valid;
  }
  // this lane's map over its 32 docs, per start state
  uint32_t nxt = 0, h[4] = {0u, 0u, 0u, 0u};
  for (int s0 = 0; s0 < k; ++s0) {
    int st = s0;
    uint32_t hh = 0;
    int pos = 0;
    while (pos < 32) {
      const uint32_t w = sel4(m, st) >> pos;
      if (!w) break;
      const int d = pos + __builtin_ctz(w);
      int ns = -1;
      for (int j = 0; j < k; ++j) {
        if (j == st) continue;
        ++hh;
        if (!((sel4(m, j) >> d) & 1u)) {
          ns = j;
          break;
        }
      }
      st = ns < 0 ? 0 : ns;
      pos = d + 1;
    }
    nxt |= (uint32_t)st << (2 * s0);
    if (s0 == 0) h[0] = hh;
    else if (s0 == 1) h[1] = hh;
    else if (s0 == 2) h[2] = hh;
    else h[3] = hh;
  }
  for (int s0 = k; s0 < 4; ++s0) nxt |= (uint32_t)s0 << (2 * s0);  // unused states: identity
  // compose across lanes in doc order: lane l's map first, then lane l + o's
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t rn = (uint32_t)__shfl_down((int)nxt, o, 64);
    uint32_t rh[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) rh[s] = (uint32_t)__shfl_down((int)h[s], o, 64);
    if ((lane & (2 * o - 1)) == 0 && lane + o < 64) {
      uint32_t nn = 0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int mid = (int)((nxt >> (2 * s)) & 3u);
        nn |= ((rn >> (2 * mid)) & 3u) << (2 * s);
        h[s] += sel4(rh, mid);
      }
      nxt = nn;
    }
  }
  if (lane == 0) {
    uint32_t* o = fn + (size_t)tile * PGPU_ANDFSM_WORDS;
    o[0] = nxt;
#pragma unroll
    for (int s = 0; s < 4; ++s) o[1 + s] = h[s];
  }
  }  // tiles
}

// One workgroup per segment: compose its tiles' maps in order and write numDocs + H (from state 0) -- the
// reference's numEntriesScannedInFilter of the segment -- into pinned host memory.
// (1024 threads: a 2^25-doc segment's 16,384 tile maps are 16 sequential compositions per thread, then a 10-level
// tree -- 256 threads left a 64-long dependent chain of loads per thread, 44 us per query on config 5)
#define FSM_SEG_THREADS 1024
__global__ __launch_bounds__(FSM_SEG_THREADS) void andfsm_segment_kernel(DevParams p, const uint32_t* fn, int64_t* out) {
  __shared__ uint32_t s_n[FSM_SEG_THREADS];
  __shared__ uint64_t s_h[FSM_SEG_THREADS][4];
  const int seg = blockIdx.x, t = threadIdx.x;
  const int nt = cld(&p.segs[seg].ntiles), t0 = cld(&p.segs[seg].tile_begin);
  const int per = (nt + FSM_SEG_THREADS - 1) / FSM_SEG_THREADS;
  uint32_t nxt = 0xE4u;  // identity: state s -> s
  uint64_t h[4] = {0, 0, 0, 0};
  // eight maps loaded before the first is composed: the loads overlap instead of one round trip per map
  const int i1 = min(nt, (t + 1) * per);
  for (int i0 = t * per; i0 < i1; i0 += 8) {
    u32x4 a[8];
    uint32_t f4[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t* f = fn + (size_t)(t0 + min(i0 + j, i1 - 1)) * PGPU_ANDFSM_WORDS;  // (32-B records)
      a[j] = *(const u32x4*)f;
      f4[j] = f[4];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (i0 + j >= i1) break;
      const uint32_t rn = a[j].x;
      uint32_t nn = 0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int mid = (int)((nxt >> (2 * s)) & 3u);
        nn |= ((rn >> (2 * mid)) & 3u) << (2 * s);
        h[s] += mid == 0 ? a[j].y : mid == 1 ? a[j].z : mid == 2 ? a[j].w : f4[j];
      }
      nxt = nn;
    }
  }
  s_n[t] = nxt;
#pragma unroll
  for (int s = 0; s < 4; ++s) s_h[t][s] = h[s];
  __syncthreads();
  for (int o = 1; o < FSM_SEG_THREADS; o <<= 1) {
    if ((t & (2 * o - 1)) == 0) {
      const uint32_t ln = s_n[t], rn = s_n[t + o];
      uint32_t nn = 0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int mid = (int)((ln >> (2 * s)) & 3u);
        nn |= ((rn >> (2 * mid)) & 3u) << (2 * s);
        s_h[t][s] += s_h[t + o][mid];
      }
      s_n[t] = nn;
    }
    __syncthreads();
  }
  // no scan leaf (match-all / empty filter): no entries
  if (t == 0) out[seg] = nt > 0 && cld(&p.segs[seg].leaf_len) > 0 ? (int64_t)cld(&p.segs[seg].num_docs) + (int64_t)s_h[0][0] : 0;
}

// Distinct group keys of each tracked segment: popcount of its bitmap row (HASH mode, num_groups_limit).
__global__ __launch_bounds__(256) void segcount_kernel(DevParams p, int64_t* out) {
  const uint32_t* row = p.segmask + (size_t)blockIdx.x * (p.G >> 5);
  int64_t c = 0;
  for (uint64_t i = threadIdx.x; i < (p.G >> 5); i += 256) c += __popc(row[i]);
  __shared__ int64_t red[256];
  red[threadIdx.x] = c;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}
// numSegmentsMatched: the per-segment match words into pinned host memory (one byte per segment), each word reset to
// 0 for the workspace's next query.
// Copy `words` int64 of a finished table into pinned host memory.

// ---- compaction of a dense table (keys with count > 0) -------------------------------------------------------------
#define CMP_BLOCK 256
#define CMP_PER_BLOCK 4096

// A row is kept when its count is > 0 and, under a top-k selection (okey != nullptr), its order key reaches the
// selected threshold (TopkState::prefix after the last radix pass).
__device__ inline bool cmp_keep(const int64_t* table, uint64_t G, uint64_t k, const uint64_t* okey,
                                const TopkState* ts) {
  return k < G && table[k] > 0 && (!okey || okey[k] >= ts->prefix);
}
__global__ void compact_count_kernel(const int64_t* table, uint64_t G, int32_t* block_counts, const uint64_t* okey,
                                     const TopkState* ts) {
  const uint64_t base = (uint64_t)blockIdx.x * CMP_PER_BLOCK;
  int c = 0;
  for (int i = threadIdx.x; i < CMP_PER_BLOCK; i += CMP_BLOCK) {
    const uint64_t k = base + i;
    if (cmp_keep(table, G, k, okey, ts)) ++c;
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

// Output keys: the cell index (dense), or the slot's key words (hash: kw = 1 plain; kw = 2 two-level, word 0
// interned in the second key table).
__device__ inline void write_key(const int64_t* table, uint64_t G, int32_t nsec, int32_t kw, uint64_t k,
                                 int64_t* out) {
  if (kw == 0) {
    out[0] = (int64_t)k;
    return;
  }
  const int64_t* w0 = table + (size_t)nsec * G;
  if (kw == 1) {
    out[0] = w0[k];
    return;
  }
  const uint64_t c = (uint64_t)w0[k];
  out[0] = w0[G + (c >> 32)];
  out[1] = (int64_t)(c & 0xFFFFFFFFull);
}

__global__ void compact_write_kernel(const int64_t* table, uint64_t G, int32_t nsec, int32_t kw,
                                     const int32_t* block_offsets, int64_t* out_keys, int64_t* out_cells,
                                     const uint64_t* okey, const TopkState* ts) {
  const uint64_t base = (uint64_t)blockIdx.x * CMP_PER_BLOCK;
  __shared__ int wbase[CMP_BLOCK / 64 + 1];
  __shared__ int running;
  if (threadIdx.x == 0) running = block_offsets[blockIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i0 = 0; i0 < CMP_PER_BLOCK; i0 += CMP_BLOCK) {
    const uint64_t k = base + i0 + threadIdx.x;
    const bool f = cmp_keep(table, G, k, okey, ts);
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
      write_key(table, G, nsec, kw, k, out_keys + (size_t)pos * (kw > 1 ? kw : 1));
      for (int s = 0; s < nsec; ++s) out_cells[(size_t)pos * nsec + s] = table[(size_t)s * G + k];
    }
    __syncthreads();
  }
}

// ---- node-level combine of hash tables (pgpu_node.cpp) --------------------------------------------------------------
// Compacted rows (key words, then cells) go to the device owning their key (pgpu_key_owner_of): owners counted, rows
// grouped by owner into a send buffer, copied peer to peer, and merged on the owner into a fresh hash table of the
// query's layout (open addressing on the key words as the hash group-by interns them), cells by the section ops.
__global__ void node_owner_kernel(const int64_t* keys, uint64_t n, int32_t kw, int32_t world, uint8_t* owner,
                                  uint32_t* counts) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t o = pgpu_key_owner_of(keys + i * kw, kw, world);
    owner[i] = (uint8_t)o;
    atomicAdd(&counts[o], 1u);
  }
}
__global__ void node_scatter_kernel(const int64_t* keys, const int64_t* cells, uint64_t n, int32_t kw, int32_t nsec,
                                    const uint8_t* owner, uint32_t* cursor, int64_t* rows) {
  const int width = kw + nsec;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t at = atomicAdd(&cursor[owner[i]], 1u);
    int64_t* r = rows + (size_t)at * width;
    for (int w = 0; w < kw; ++w) r[w] = keys[i * kw + w];
    for (int s = 0; s < nsec; ++s) r[kw + s] = cells[i * nsec + s];
  }
}
__global__ void node_init_kernel(int64_t* table, uint64_t P, int32_t nsec, int32_t kw, NodeOps ops) {
  const uint64_t n = P * (uint64_t)(nsec + (kw == 2 ? 2 : 1));
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    table[i] = i < P * nsec ? sec_identity(ops.op[i / P]) : (int64_t)PGPU_HASH_EMPTY;
}
__global__ void node_merge_kernel(const int64_t* rows, uint64_t n, int32_t kw, int32_t nsec, int64_t* table,
                                  uint64_t P, NodeOps ops, int32_t* hflag) {
  const int width = kw + nsec;
  uint64_t* w0 = (uint64_t*)(table + (size_t)nsec * P);
  const uint64_t mask = P - 1;
  const uint64_t n64 = (n + 63) & ~63ull;  // whole waves: hash_insert's probes are per lane, ballots per wave
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n64; i += (uint64_t)gridDim.x * blockDim.x) {
    const bool live = i < n;
    const int64_t* r = rows + (size_t)(live ? i : 0) * width;
    uint32_t slot[1];
    if (kw == 2) {
      const uint64_t k0[1] = {(uint64_t)r[0]};
      uint32_t s0[1];
      hash_insert(w0 + P, mask, k0, live ? 1u : 0u, s0, hflag);  // intern word 0
      const uint64_t c[1] = {((uint64_t)s0[0] << 32) | (uint64_t)r[1]};
      hash_insert(w0, mask, c, live ? 1u : 0u, slot, hflag);
    } else {
      const uint64_t k[1] = {(uint64_t)r[0]};
      hash_insert(w0, mask, k, live ? 1u : 0u, slot, hflag);
    }
    if (!live) continue;
    for (int s = 0; s < nsec; ++s) cell_atomic(&table[(size_t)s * P + slot[0]], ops.op[s], r[kw + s]);
  }
}

#endif  // TU_HAS(PGPU_TU_COMMON)

}  // namespace

// ---- host-side launch helpers (called by pgpu_runtime.cpp) --------------------------------------------------------
template <int M, int PL, int PK>
static hipError_t rd_attr(size_t lds_bytes) {
  return hipFuncSetAttribute((const void*)query_kernel_rdirect<M, PL, PK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds_bytes);
}
// (the prefix variants stop at 12 planes: 16 + 3 planes per tile in flight would pass 128 VGPRs -- one wave per
// SIMD less -- so the runtime sets rd_pfx only for fast leaves of <= 12 bits)
template <int M, int PK>
static void rd_launch(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st) {
  if (p.rd_planes <= 8)
    hipLaunchKernelGGL((query_kernel_rdirect<M, 8, PK>), dim3(grid), dim3(PGPU_DIRECT_THREADS), dyn_smem, st, p);
  else if (p.rd_planes <= 10)
    hipLaunchKernelGGL((query_kernel_rdirect<M, 10, PK>), dim3(grid), dim3(PGPU_DIRECT_THREADS), dyn_smem, st, p);
  else if (PK > 0 || p.rd_planes <= 12)
    hipLaunchKernelGGL((query_kernel_rdirect<M, 12, PK>), dim3(grid), dim3(PGPU_DIRECT_THREADS), dyn_smem, st, p);
  else
    hipLaunchKernelGGL((query_kernel_rdirect<M, 16, 0>), dim3(grid), dim3(PGPU_DIRECT_THREADS), dyn_smem, st, p);
}
template <int M, int PK>
static hipError_t rd_attrs(size_t lds_bytes) {
  hipError_t e = rd_attr<M, 8, PK>(lds_bytes);
  if (e == hipSuccess) e = rd_attr<M, 10, PK>(lds_bytes);
  if (e == hipSuccess) e = rd_attr<M, 12, PK>(lds_bytes);
  if (e == hipSuccess && PK == 0) e = rd_attr<M, 16, 0>(lds_bytes);
  return e;
}
// register streaming: narrow-leaf planes 4 / 8, value planes 16 / 24
template <int PN, int NV>
static hipError_t rs_attr(size_t lds_bytes) {
  return hipFuncSetAttribute((const void*)query_kernel_rstream<PN, NV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds_bytes);
}
[[maybe_unused]] static hipError_t rs_attrs(size_t lds_bytes) {
  hipError_t e = rs_attr<4, 16>(lds_bytes);
  if (e == hipSuccess) e = rs_attr<4, 24>(lds_bytes);
  if (e == hipSuccess) e = rs_attr<8, 16>(lds_bytes);
  if (e == hipSuccess) e = rs_attr<8, 24>(lds_bytes);
  return e;
}
template <int NA, int NV>
static hipError_t rp_attr(size_t lds_bytes) {
  return hipFuncSetAttribute((const void*)query_kernel_rprog<NA, NV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds_bytes);
}
template <int NA, int NV, bool IDS = false>
static hipError_t rk_attr(size_t lds_bytes) {
  return hipFuncSetAttribute((const void*)query_kernel_rkey<NA, NV, IDS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds_bytes);
}
[[maybe_unused]] static hipError_t rp_attrs(size_t lds_bytes) {
  hipError_t e = rp_attr<1, 16>(lds_bytes);
  if (e == hipSuccess) e = rk_attr<1, 16>(lds_bytes);
  if (e == hipSuccess) e = rk_attr<1, 24>(lds_bytes);
  if (e == hipSuccess) e = rk_attr<2, 16>(lds_bytes);
  if (e == hipSuccess) e = rk_attr<2, 20>(lds_bytes);
  if (e == hipSuccess) e = rk_attr<2, 24>(lds_bytes);
  if (e == hipSuccess) e = rk_attr<1, 16, true>(lds_bytes);
  if (e == hipSuccess) e = rk_attr<2, 16, true>(lds_bytes);
  if (e == hipSuccess) e = rp_attr<1, 24>(lds_bytes);
  if (e == hipSuccess) e = rp_attr<2, 16>(lds_bytes);
  if (e == hipSuccess) e = rp_attr<2, 20>(lds_bytes);
  if (e == hipSuccess) e = rp_attr<2, 24>(lds_bytes);
  return e;
}
// (index-only register streaming: rd_planes = value columns 1 / 2, rs_vplanes = value planes 16 / 20 / 24; two
// columns of <= 20 planes keep three waves per SIMD, of 24 two)
[[maybe_unused]] static void rp_launch(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st) {
  const dim3 g(grid), b(PGPU_DIRECT_THREADS);
  if (p.direct == 5) {  // the inverted leaves' containers read into LDS per unit (query_kernel_rkey)
    const dim3 kb(PGPU_DIRECT_THREADS);
    if (p.rk_ids) {  // the aggregated columns' packed 16-bit ids, values gathered for the matched docs
      if (p.rd_planes <= 1) hipLaunchKernelGGL((query_kernel_rkey<1, 16, true>), g, kb, dyn_smem, st, p);
      else hipLaunchKernelGGL((query_kernel_rkey<2, 16, true>), g, kb, dyn_smem, st, p);
      return;
    }
    if (p.rd_planes <= 1 && p.rs_vplanes <= 16) hipLaunchKernelGGL((query_kernel_rkey<1, 16>), g, kb, dyn_smem, st, p);
    else if (p.rd_planes <= 1) hipLaunchKernelGGL((query_kernel_rkey<1, 24>), g, kb, dyn_smem, st, p);
    else if (p.rs_vplanes <= 16) hipLaunchKernelGGL((query_kernel_rkey<2, 16>), g, kb, dyn_smem, st, p);
    else if (p.rs_vplanes <= 20) hipLaunchKernelGGL((query_kernel_rkey<2, 20>), g, kb, dyn_smem, st, p);
    else hipLaunchKernelGGL((query_kernel_rkey<2, 24>), g, kb, dyn_smem, st, p);
    return;
  }
  if (p.rd_planes <= 1 && p.rs_vplanes <= 16) hipLaunchKernelGGL((query_kernel_rprog<1, 16>), g, b, dyn_smem, st, p);
  else if (p.rd_planes <= 1) hipLaunchKernelGGL((query_kernel_rprog<1, 24>), g, b, dyn_smem, st, p);
  else if (p.rs_vplanes <= 16) hipLaunchKernelGGL((query_kernel_rprog<2, 16>), g, b, dyn_smem, st, p);
  else if (p.rs_vplanes <= 20) hipLaunchKernelGGL((query_kernel_rprog<2, 20>), g, b, dyn_smem, st, p);
  else hipLaunchKernelGGL((query_kernel_rprog<2, 24>), g, b, dyn_smem, st, p);
}
// (fused exact statistics: rd_planes = the first leaf's planes held (10 / 12 / 16), rs_vplanes = the second's (20 / 24))
template <int M>
[[maybe_unused]] static void rf_launch(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st) {
  const dim3 g(grid), b(PGPU_DIRECT_THREADS);
  if (p.rd_planes <= 10 && p.rs_vplanes <= 20) hipLaunchKernelGGL((query_kernel_rfsm<M, 10, 20>), g, b, dyn_smem, st, p);
  else if (p.rd_planes <= 12 && p.rs_vplanes <= 20) hipLaunchKernelGGL((query_kernel_rfsm<M, 12, 20>), g, b, dyn_smem, st, p);
  else hipLaunchKernelGGL((query_kernel_rfsm<M, 16, 24>), g, b, dyn_smem, st, p);
}
template <int M>
[[maybe_unused]] static hipError_t rf_attrs(size_t lds_bytes) {
  hipError_t e = hipFuncSetAttribute((const void*)query_kernel_rfsm<M, 10, 20>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)query_kernel_rfsm<M, 12, 20>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_bytes);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)query_kernel_rfsm<M, 16, 24>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_bytes);
  return e;
}
[[maybe_unused]] static void rs_launch(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st) {
  const dim3 g(grid), b(PGPU_DIRECT_THREADS);
  if (p.rd_planes <= 4 && p.rs_vplanes <= 16) hipLaunchKernelGGL((query_kernel_rstream<4, 16>), g, b, dyn_smem, st, p);
  else if (p.rd_planes <= 4) hipLaunchKernelGGL((query_kernel_rstream<4, 24>), g, b, dyn_smem, st, p);
  else if (p.rs_vplanes <= 16) hipLaunchKernelGGL((query_kernel_rstream<8, 16>), g, b, dyn_smem, st, p);
  else hipLaunchKernelGGL((query_kernel_rstream<8, 24>), g, b, dyn_smem, st, p);
}
// Per aggregation mode (one translation unit each): launch the ring or direct query kernel, set its LDS attribute.
#define PGPU_MODE_FUNCS(M, NAME)                                                                                  \
  hipError_t pgpu_launch_query_##NAME(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st) {          \
    if (p.dense) hipLaunchKernelGGL((query_kernel<M, 1>), dim3(grid), dim3(PGPU_THREADS(1)), dyn_smem, st, p);   \
    else hipLaunchKernelGGL((query_kernel<M, 0>), dim3(grid), dim3(PGPU_THREADS(0)), dyn_smem, st, p);           \
    return hipGetLastError();                                                                                   \
  }                                                                                                             \
  hipError_t pgpu_launch_direct_##NAME(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st) {         \
    if (p.direct == 6) {                                                                                        \
      if constexpr (M != PGPU_MODE_PART)                                                                        \
        hipLaunchKernelGGL((query_kernel_cand<M>), dim3(grid), dim3(PGPU_DIRECT_THREADS), dyn_smem, st, p);     \
      else                                                                                                      \
        return hipErrorInvalidValue;                                                                            \
    } else if (p.direct == 8) {                                                                                 \
      if constexpr (M != PGPU_MODE_PART) rf_launch<M>(p, grid, dyn_smem, st);                                   \
      else return hipErrorInvalidValue;                                                                         \
    } else if (p.direct >= 3) {                                                                                 \
      if constexpr (M == PGPU_MODE_AGG) {                                                                       \
        if (p.direct == 3) rs_launch(p, grid, dyn_smem, st);                                                    \
        else rp_launch(p, grid, dyn_smem, st);                                                                  \
      } else                                                                                                    \
        return hipErrorInvalidValue;                                                                            \
    } else if (p.direct == 2) {                                                                                 \
      if (p.rd_pfx) rd_launch<M, PGPU_PFX_PLANES>(p, grid, dyn_smem, st);                                       \
      else rd_launch<M, 0>(p, grid, dyn_smem, st);                                                              \
    } else                                                                                                      \
      hipLaunchKernelGGL((query_kernel_direct<M>), dim3(grid), dim3(PGPU_DIRECT_THREADS), dyn_smem, st, p);     \
    return hipGetLastError();                                                                                   \
  }                                                                                                             \
  hipError_t pgpu_prepare_##NAME(size_t lds_bytes) {                                                            \
    hipError_t e = hipFuncSetAttribute((const void*)query_kernel<M, 0>,                                         \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);            \
    if (e == hipSuccess)                                                                                        \
      e = hipFuncSetAttribute((const void*)query_kernel<M, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,      \
                              (int)lds_bytes);                                                                  \
    if (e == hipSuccess)                                                                                        \
      e = hipFuncSetAttribute((const void*)query_kernel_direct<M>, hipFuncAttributeMaxDynamicSharedMemorySize,  \
                              (int)lds_bytes);                                                                  \
    if constexpr (M != PGPU_MODE_PART)                                                                          \
      if (e == hipSuccess)                                                                                      \
        e = hipFuncSetAttribute((const void*)query_kernel_cand<M>, hipFuncAttributeMaxDynamicSharedMemorySize,  \
                                (int)lds_bytes);                                                                \
    if constexpr (M != PGPU_MODE_PART)                                                                          \
      if (e == hipSuccess) e = rf_attrs<M>(lds_bytes);                                                          \
    if (e == hipSuccess) e = rd_attrs<M, 0>(lds_bytes);                                                         \
    if (e == hipSuccess) e = rd_attrs<M, PGPU_PFX_PLANES>(lds_bytes);                                           \
    if constexpr (M == PGPU_MODE_AGG)                                                                           \
      if (e == hipSuccess) e = rs_attrs(lds_bytes);                                                             \
    if constexpr (M == PGPU_MODE_AGG)                                                                           \
      if (e == hipSuccess) e = rp_attrs(lds_bytes);                                                             \
    return e;                                                                                                   \
  }
#define PGPU_MODE_DECLS(NAME)                                                                   \
  hipError_t pgpu_launch_query_##NAME(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st);  \
  hipError_t pgpu_launch_direct_##NAME(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st); \
  hipError_t pgpu_prepare_##NAME(size_t lds_bytes);
PGPU_MODE_DECLS(agg) PGPU_MODE_DECLS(lds) PGPU_MODE_DECLS(global) PGPU_MODE_DECLS(part) PGPU_MODE_DECLS(hash)

#if TU_HAS(0)
PGPU_MODE_FUNCS(PGPU_MODE_AGG, agg)
#endif
#if TU_HAS(1)
PGPU_MODE_FUNCS(PGPU_MODE_LDS, lds)
#endif
#if TU_HAS(2)
PGPU_MODE_FUNCS(PGPU_MODE_GLOBAL, global)
#endif
#if TU_HAS(4)
PGPU_MODE_FUNCS(PGPU_MODE_HASH, hash)
#endif
#if TU_HAS(3)
PGPU_MODE_FUNCS(PGPU_MODE_PART, part)

hipError_t pgpu_prepare_part_reduce() {
  hipError_t e = hipSuccess;
#define PART_ATTR_1(NS, ONE, LDM)                                                               \
  if (e == hipSuccess)                                                                          \
    e = hipFuncSetAttribute((const void*)part_reduce_kernel<NS, ONE, LDM>,                      \
                            hipFuncAttributeMaxDynamicSharedMemorySize, PGPU_LDS_LIMIT);
#define PART_ATTR(NS) PART_ATTR_1(NS, true, 0) PART_ATTR_1(NS, true, 1) PART_ATTR_1(NS, true, 2) PART_ATTR_1(NS, false, 0)
  PART_ATTR(0) PART_ATTR(1) PART_ATTR(2) PART_ATTR(3) PART_ATTR(4)
#undef PART_ATTR_1
#undef PART_ATTR
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)part_scan_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            PGPU_LDS_LIMIT);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)part_scan_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            PGPU_LDS_LIMIT);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)part_scan_kernel<false, 20, 16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            PGPU_LDS_LIMIT);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)part_scan_kernel<false, 16, 16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            PGPU_LDS_LIMIT);
  return e;
}

// Phase 1 by part_scan_kernel; with per-partition regions (p.pcap), first the sampled counting pass and the
// sizing / phase-2 plan, all on the stream (no host round trip).
hipError_t pgpu_launch_part_scan(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st) {
  if (p.pcap) {
    hipError_t e = hipMemsetAsync(p.pcount, 0, 4ull * p.nparts, st);
    if (e != hipSuccess) return e;
    const int sampled = (p.total_tiles + p.psample - 1) / p.psample;
    const int cg = max(1, min(grid, (sampled + PGPU_PSCAN_WAVES - 1) / PGPU_PSCAN_WAVES));
    hipLaunchKernelGGL(part_scan_kernel<true>, dim3(cg), dim3(PGPU_PSCAN_THREADS), dyn_smem, st, p);
    hipLaunchKernelGGL(part_plan_kernel, dim3(1), dim3(1024), 0, st, p, grid);
  }
  if (p.pscan_kb == 20 && p.pscan_vb == 16)
    hipLaunchKernelGGL((part_scan_kernel<false, 20, 16>), dim3(grid), dim3(PGPU_PSCAN_THREADS), dyn_smem, st, p);
  else if (p.pscan_kb == 16 && p.pscan_vb == 16)
    hipLaunchKernelGGL((part_scan_kernel<false, 16, 16>), dim3(grid), dim3(PGPU_PSCAN_THREADS), dyn_smem, st, p);
  else
    hipLaunchKernelGGL(part_scan_kernel<false>, dim3(grid), dim3(PGPU_PSCAN_THREADS), dyn_smem, st, p);
  return hipGetLastError();
}
bool pgpu_pscan_prefetch_ok(int kb, int vb) { return (kb == 20 || kb == 16) && vb == 16; }

hipError_t pgpu_launch_part_reduce(const DevParams& p, int nwg, hipStream_t st) {
  size_t lds = (size_t)p.nsec * ((size_t)1 << p.pshift) * 8 + (p.ldict == 1 ? (size_t)4 << p.slice_shift : 0);
  if (p.ldict == 2) {  // compact table (count and MIN / MAX ids in 4 B, SUM in 8 B) + the dictionary image
    lds = (size_t)4 << p.pshift;
    for (int s = 1; s < p.nsec; ++s)
      lds += (p.sec_op[s] == PGPU_RED_SUM_I64 || p.sec_op[s] == PGPU_RED_SUM_F64 ? (size_t)8 : (size_t)4) << p.pshift;
    lds += (size_t)4 * ((size_t)p.for_nblk * (1 + p.for_bits) + 1);
  }
  const dim3 g(p.p2work ? p.p2grid : p.nparts);
  switch (p.nsec - 1) {
#define PART_LAUNCH(NS)                                                                                    \
  case NS:                                                                                                 \
    if (p.rw == 1 && p.ldict == 1) hipLaunchKernelGGL((part_reduce_kernel<NS, true, 1>), g, dim3(1024), lds, st, p, nwg); \
    else if (p.rw == 1 && p.ldict == 2) hipLaunchKernelGGL((part_reduce_kernel<NS, true, 2>), g, dim3(1024), lds, st, p, nwg); \
    else if (p.rw == 1) hipLaunchKernelGGL((part_reduce_kernel<NS, true, 0>), g, dim3(1024), lds, st, p, nwg); \
    else hipLaunchKernelGGL((part_reduce_kernel<NS, false, 0>), g, dim3(1024), lds, st, p, nwg); \
    return hipGetLastError();
    PART_LAUNCH(0) PART_LAUNCH(1) PART_LAUNCH(2) PART_LAUNCH(3) PART_LAUNCH(4)
#undef PART_LAUNCH
    default:
      return hipErrorInvalidValue;
  }
}
#endif  // TU_HAS(3)

#if TU_HAS(PGPU_TU_COMMON)
hipError_t pgpu_prepare_part_reduce();

// Bit-sliced copy of a fixed-bit forward index (built once per column at segment seal): thread (tile, lane) unpacks
// its 32 dict ids from the big-endian packed words and writes plane k = bit k of each id (doc 32l+i in bit i) at
// dword (tile * b + k) * 64 + lane.  Same bytes per tile as the packed stream, so staging costs are unchanged.
template <int B>
__device__ void bitslice_b(const uint32_t* fwd, uint32_t* out, int64_t tile, int lane) {
  uint32_t w[B], ids[32];
  const uint32_t* src = fwd + ((size_t)tile * 64 + lane) * B;
#pragma unroll
  for (int k = 0; k < B; ++k) w[k] = bswap32(src[k]);
  unpack_b<B>(w, ids);
  uint32_t* dst = out + (size_t)tile * B * 64 + lane;
#pragma unroll
  for (int k = 0; k < B; ++k) {
    uint32_t pl = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) pl |= ((ids[i] >> k) & 1u) << i;
    dst[(size_t)k * 64] = pl;
  }
}
// Value planes (DevColumn::vsliced): per tile and lane the 32 docs' dictionary values minus vmin, bit k of doc 32l+i
// in bit i of dword k * 64 + l of the tile's 256 * vbits bytes.
template <int B>
__device__ void vslice_b(const uint32_t* fwd, const void* dict, int dict_type, int64_t vmin, int vbits, uint32_t* out,
                         int64_t tile, int lane) {
  uint32_t w[B], ids[32];
  const uint32_t* src = fwd + ((size_t)tile * 64 + lane) * B;
#pragma unroll
  for (int k = 0; k < B; ++k) w[k] = bswap32(src[k]);
  unpack_b<B>(w, ids);
  uint32_t u[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int64_t v = dict_type == PGPU_INT ? (int64_t)gld((const int32_t*)dict, ids[i]) : gld((const int64_t*)dict, ids[i]);
    u[i] = (uint32_t)((uint64_t)v - (uint64_t)vmin);
  }
  uint32_t* dst = out + (size_t)tile * vbits * 64 + lane;
  for (int k = 0; k < vbits; ++k) {
    uint32_t pl = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) pl |= ((u[i] >> k) & 1u) << i;
    dst[(size_t)k * 64] = pl;
  }
}
__global__ __launch_bounds__(256) void vslice_kernel(const uint32_t* fwd, const void* dict, int dict_type, int64_t vmin,
                                                     int bits, int vbits, uint32_t* out, int64_t ntiles) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tile = g >> 6;
  const int lane = (int)(g & 63);
  if (tile >= ntiles) return;
#define VS_CALL(B) vslice_b<B>(fwd, dict, dict_type, vmin, vbits, out, tile, lane)
  PGPU_DISPATCH_B(bits, VS_CALL)
#undef VS_CALL
}
__global__ __launch_bounds__(256) void bitslice_kernel(const uint32_t* fwd, uint32_t* out, int bits, int64_t ntiles) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tile = g >> 6;
  const int lane = (int)(g & 63);
  if (tile >= ntiles) return;
#define BS_CALL(B) bitslice_b<B>(fwd, out, tile, lane)
  PGPU_DISPATCH_B(bits, BS_CALL)
#undef BS_CALL
}

// ---- raw-value filter leaves ---------------------------------------------------------------------------------------
// Predicate of a leaf over a raw (no-dictionary) column, exactly as the reference's raw-value evaluators apply it
// per doc: Int/Long/Float/DoubleRawValueBasedRangePredicateEvaluator.applySV (RangePredicateEvaluatorFactory.java:
// 273-460: inclusive / exclusive bounds, unbounded = the type's extreme, inclusive), the raw EQ / NOT_EQ evaluators
// (EqualsPredicateEvaluatorFactory / NotEqualsPredicateEvaluatorFactory: primitive ==) and the raw IN / NOT_IN sets
// (InPredicateEvaluatorFactory / NotInPredicateEvaluatorFactory: fastutil open hash sets, i.e. float / double
// members compared by their bits -- here by the order-preserving key of the value, a bijection of the bits).
FI bool raw_set_has(const int64_t* vals, int n, int64_t k) {
  int a = 0, z = n - 1;
  while (a <= z) {
    const int m = (a + z) >> 1;
    const int64_t v = gld(vals, (size_t)m);
    if (v == k) return true;
    if (v < k) a = m + 1; else z = m - 1;
  }
  return false;
}
FI bool raw_match(const RawLeaf& L, uint64_t bits) {
  bool r;
  if (L.vtype == PGPU_INT || L.vtype == PGPU_LONG) {
    const int64_t x = L.vtype == PGPU_INT ? (int64_t)(int32_t)(uint32_t)bits : (int64_t)bits;
    if (L.pred == PGPU_PRED_RANGE)
      r = ((L.flags & PGPU_RAW_RANGE_LO_INCL) ? x >= L.lo : x > L.lo) && ((L.flags & PGPU_RAW_RANGE_HI_INCL) ? x <= L.hi : x < L.hi);
    else
      r = raw_set_has(L.vals, L.nvals, x);
  } else {
    double x = L.vtype == PGPU_FLOAT ? (double)__uint_as_float((uint32_t)bits) : __longlong_as_double((int64_t)bits);
    if (L.pred == PGPU_PRED_RANGE) {
      if ((L.flags & PGPU_RAW_RANGE_ORDINAL) && x != x) x = -__builtin_inf();  // FPOrdering.ordinalOf(NaN) = 0
      const double lo = __longlong_as_double(L.lo), hi = __longlong_as_double(L.hi);
      r = ((L.flags & PGPU_RAW_RANGE_LO_INCL) ? lo <= x : lo < x) && ((L.flags & PGPU_RAW_RANGE_HI_INCL) ? hi >= x : hi > x);
    } else {
      r = raw_set_has(L.vals, L.nvals, key_of_double(x));
    }
  }
  return r != (L.negate != 0);
}
// One wave per 1024 docs of leaf blockIdx.y: 16 coalesced value loads per lane in flight, one ballot per 64 docs,
// lanes 0..31 write the chunk's 32 match words (docs past num_docs never match).  An HBM streaming kernel: 4 or 8
// bytes read per doc, 1 bit written.
template <int W>
__device__ void rawpred_wave(const RawLeaf& L, int64_t c, int lane) {
  constexpr int NU = 16;
  const int64_t d0 = c * 1024;
  uint64_t v[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const size_t d = (size_t)(d0 + u * 64 + lane);
    v[u] = W == 4 ? (uint64_t)gld((const uint32_t*)L.values, d) : (uint64_t)gld((const uint64_t*)L.values, d);
  }
  uint64_t bal[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const bool live = d0 + u * 64 + lane < L.num_docs;
    bal[u] = __builtin_amdgcn_ballot_w64(live && raw_match(L, v[u]));
  }
  if (lane < 32) {
    uint64_t b = 0;
#pragma unroll
    for (int u = 0; u < NU; ++u) b = (lane >> 1) == u ? bal[u] : b;
    L.out[c * 32 + lane] = (uint32_t)(b >> (32 * (lane & 1)));
  }
}
__global__ __launch_bounds__(256) void rawpred_kernel(const RawLeaf* leaves) {
  const RawLeaf L = cld(leaves + blockIdx.y);
  const int lane = threadIdx.x & 63;
  const int64_t nchunks = L.words / 32;
  const bool w4 = L.vtype == PGPU_INT || L.vtype == PGPU_FLOAT;
  for (int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < nchunks; c += (int64_t)gridDim.x * 4) {
    if (w4) rawpred_wave<4>(L, c, lane);
    else rawpred_wave<8>(L, c, lane);
  }
}

// ---- multi-value SCAN leaves: one lane per row, 64 rows per ballot ------------------------------------------------
// PinotDataBitSet.readInt of value v (MSB-first): the 64-bit big-endian window of the two 32-bit words holding it.
FI uint32_t mv_read(const uint32_t* fwd, int64_t bit, int bits) {
  const int64_t w = bit >> 5;
  const uint64_t hi = __builtin_bswap32(__builtin_nontemporal_load(fwd + w));
  const uint64_t lo = __builtin_bswap32(__builtin_nontemporal_load(fwd + w + 1));
  const uint64_t win = (hi << 32) | lo;
  return (uint32_t)((win >> (64 - (int)(bit & 31) - bits)) & ((1ull << bits) - 1));
}

__global__ __launch_bounds__(256) void mvpred_kernel(const MvLeaf* leaves) {
  const MvLeaf L = cld(leaves + blockIdx.y);
  const int lane = threadIdx.x & 63;
  const int64_t nblk = L.words / 2;  // 64 rows per block
  for (int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); b < nblk; b += (int64_t)gridDim.x * 4) {
    const int64_t d = b * 64 + lane;
    bool hit = false;
    if (d < L.num_docs) {
      const int32_t s = L.off[d], e = L.off[d + 1];
      for (int32_t v = s; v < e && !hit; ++v) {  // applyMV: the first matching value decides
        const uint32_t id = mv_read(L.fwd, (int64_t)v * L.bits, L.bits);
        hit = L.set ? ((L.set[id >> 5] >> (id & 31)) & 1u) != 0 : ((int32_t)id >= L.lo && (int32_t)id < L.hi);
      }
      hit = hit != (L.negate != 0);
    }
    const uint64_t m = __ballot(hit);
    if (lane < 2) L.out[2 * b + lane] = (uint32_t)(lane ? (m >> 32) : m);
  }
}

hipError_t pgpu_launch_mvpred(const MvLeaf* dev_leaves, int nleaves, int64_t max_words, hipStream_t st) {
  if (nleaves <= 0) return hipSuccess;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(4096, (max_words / 2 + 3) / 4));
  hipLaunchKernelGGL(mvpred_kernel, dim3((unsigned)blocks, (unsigned)nleaves), dim3(256), 0, st, dev_leaves);
  return hipGetLastError();
}

// ---- inverted-index leaves expanded to doc bitmaps ---------------------------------------------------------------
// BitmapBasedFilterOperator's OR of the ids' bitmaps (BitmapBasedFilterOperator.java:66-101), one container key per
// workgroup: the 64K-doc word range is assembled in LDS (bitmap containers copied, array values and runs set with
// LDS atomics), then written out in whole lines.  The query kernel reads the result as a BITS leaf: one word per
// lane and tile instead of a per-tile container search and array scan on the consumer's critical path.
__global__ __launch_bounds__(256) void invexp_kernel(const InvLeafX* leaves) {
  __shared__ uint32_t w[2048];
  const InvLeafX L = cld(leaves + blockIdx.y);
  const uint32_t key = blockIdx.x;
  const int64_t word0 = (int64_t)key * 2048;
  if (word0 >= L.words || L.skip) return;
  const int t = threadIdx.x;
  for (int i = t; i < 2048; i += 256) w[i] = 0u;
  __syncthreads();
  const InvIndex ix{L.dir, L.ct, L.data};
  for (int k = 0; k < L.nids; ++k) {
    const int32_t ci = find_container(ix, (uint32_t)cld(L.ids + k), key);
    if (ci < 0) continue;
    const uint32_t type = cld(&L.ct[ci].type), card = cld(&L.ct[ci].card), offset = cld(&L.ct[ci].offset);
    if (type == PGPU_CT_BITMAP) {
      const uint32_t* b = (const uint32_t*)(L.data + offset);
      for (int i = t; i < 2048; i += 256) w[i] |= gld(b, i);
    } else if (type == PGPU_CT_RUN) {
      const uint16_t* r = (const uint16_t*)(L.data + offset);
      for (uint32_t j = t; j < card; j += 256) {
        const uint32_t s0 = gld(r, 2 * j), e0 = s0 + gld(r, 2 * j + 1);  // inclusive
        const uint32_t a = s0 >> 5, z = e0 >> 5;
        for (uint32_t x = a; x <= z; ++x) {
          const uint32_t lo = x == a ? (s0 & 31) : 0u, hi = x == z ? (e0 & 31) : 31u;
          atomicOr(&w[x], (0xFFFFFFFFu >> (31 - hi)) & (0xFFFFFFFFu << lo));
        }
      }
    } else {
      const uint16_t* v = (const uint16_t*)(L.data + offset);
      for (uint32_t j = t; j < card; j += 256) {
        const uint32_t x = gld(v, j);
        atomicOr(&w[x >> 5], 1u << (x & 31));
      }
    }
    __syncthreads();
  }
  const int64_t nw = min((int64_t)2048, (int64_t)L.words - word0);
  for (int i = t; i < nw; i += 256) {
    uint32_t x = w[i];
    if (L.negate) {
      const int64_t d0 = (word0 + i) * 32;
      const int64_t left = (int64_t)L.num_docs - d0;
      const uint32_t valid = left >= 32 ? 0xFFFFFFFFu : (left <= 0 ? 0u : ((1u << left) - 1u));
      x = ~x & valid;
    }
    L.out[word0 + i] = x;
  }
}

// query_kernel_rkey's container table: for every inverted leaf, id and 65,536-doc container key, the id's container
// of that key (card 0: none) -- the container searches done once per query, all in parallel, so the query kernel's
// units read one record per (leaf, id) instead of a chain of dependent directory loads.
__global__ __launch_bounds__(256) void rkey_ctab_kernel(const InvLeafX* leaves, DevContainer* out) {
  const InvLeafX L = cld(leaves + blockIdx.y);
  const int64_t n = (int64_t)L.nids * L.nkeys;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint32_t k = (uint32_t)(i / L.nkeys), key = (uint32_t)(i % L.nkeys);
    const uint32_t id = (uint32_t)gld(L.ids, k);
    int32_t a = (int32_t)gld(L.dir, id), z = (int32_t)gld(L.dir, id + 1) - 1;
    DevContainer r{key, 0u, 0u, 0u};
    while (a <= z) {
      const int32_t mid = (a + z) >> 1;
      const DevContainer c = L.ct[mid];
      if (c.key == key) {
        r = c;
        break;
      }
      if (c.key < key) a = mid + 1; else z = mid - 1;
    }
    out[(size_t)L.ctab_off + (size_t)i] = r;
  }
}

hipError_t pgpu_launch_rkey_ctab(const InvLeafX* dev_leaves, int nleaves, int64_t max_pairs, DevContainer* out,
                                 hipStream_t st) {
  if (nleaves <= 0) return hipSuccess;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(256, (max_pairs + 255) / 256));
  hipLaunchKernelGGL(rkey_ctab_kernel, dim3((unsigned)blocks, (unsigned)nleaves), dim3(256), 0, st, dev_leaves, out);
  return hipGetLastError();
}

hipError_t pgpu_launch_invexp(const InvLeafX* dev_leaves, int nleaves, int64_t max_words, hipStream_t st) {
  if (nleaves <= 0) return hipSuccess;
  const int64_t keys = (max_words + 2047) / 2048;
  hipLaunchKernelGGL(invexp_kernel, dim3((unsigned)std::max<int64_t>(1, keys), (unsigned)nleaves), dim3(256), 0, st,
                     dev_leaves);
  return hipGetLastError();
}

hipError_t pgpu_launch_rawpred(const RawLeaf* dev_leaves, int nleaves, int64_t max_words, hipStream_t st) {
  if (nleaves <= 0) return hipSuccess;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(2048, (max_words / 32 + 3) / 4));
  hipLaunchKernelGGL(rawpred_kernel, dim3((unsigned)blocks, (unsigned)nleaves), dim3(256), 0, st, dev_leaves);
  return hipGetLastError();
}

hipError_t pgpu_launch_vslice(const uint32_t* fwd, const void* dict, int dict_type, int64_t vmin, int bits, int vbits,
                              uint32_t* out, int64_t ntiles, hipStream_t st) {
  if (ntiles <= 0) return hipSuccess;
  const int64_t blocks = (ntiles * 64 + 255) / 256;
  hipLaunchKernelGGL(vslice_kernel, dim3((unsigned)blocks), dim3(256), 0, st, fwd, dict, dict_type, vmin, bits, vbits,
                     out, ntiles);
  return hipGetLastError();
}

hipError_t pgpu_launch_bitslice(const uint32_t* fwd, uint32_t* out, int bits, int64_t ntiles, hipStream_t st) {
  if (ntiles <= 0) return hipSuccess;
  const int64_t blocks = (ntiles * 64 + 255) / 256;
  hipLaunchKernelGGL(bitslice_kernel, dim3((unsigned)blocks), dim3(256), 0, st, fwd, out, bits, ntiles);
  return hipGetLastError();
}

hipError_t pgpu_prepare_query_kernels(size_t lds_bytes) {
  hipError_t e = pgpu_prepare_agg(lds_bytes);
  if (e == hipSuccess) e = pgpu_prepare_lds(lds_bytes);
  if (e == hipSuccess) e = pgpu_prepare_global(lds_bytes);
  if (e == hipSuccess) e = pgpu_prepare_part(lds_bytes);
  if (e == hipSuccess) e = pgpu_prepare_hash(lds_bytes);
  if (e == hipSuccess) e = pgpu_prepare_part_reduce();
  return e;
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
    case PGPU_MODE_AGG: return pgpu_launch_query_agg(p, grid, dyn_smem, st);
    case PGPU_MODE_LDS: return pgpu_launch_query_lds(p, grid, dyn_smem, st);
    case PGPU_MODE_GLOBAL: return pgpu_launch_query_global(p, grid, dyn_smem, st);
    case PGPU_MODE_PART: return pgpu_launch_query_part(p, grid, dyn_smem, st);
    case PGPU_MODE_HASH: return pgpu_launch_query_hash(p, grid, dyn_smem, st);
    default: return hipErrorInvalidValue;
  }
}

// Direct variant (p.direct): PGPU_DIRECT_THREADS per workgroup, several workgroups per CU.
hipError_t pgpu_launch_query_direct(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st) {
  switch (p.mode) {
    case PGPU_MODE_AGG: return pgpu_launch_direct_agg(p, grid, dyn_smem, st);
    case PGPU_MODE_LDS: return pgpu_launch_direct_lds(p, grid, dyn_smem, st);
    case PGPU_MODE_GLOBAL: return pgpu_launch_direct_global(p, grid, dyn_smem, st);
    case PGPU_MODE_PART: return pgpu_launch_direct_part(p, grid, dyn_smem, st);
    case PGPU_MODE_HASH: return pgpu_launch_direct_hash(p, grid, dyn_smem, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t pgpu_launch_leafbits(const DevParams& p, hipStream_t st) {
  if (p.total_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(leafbits_kernel, dim3((p.total_tiles + 3) / 4), dim3(256), 0, st, p);
  return hipGetLastError();
}

hipError_t pgpu_launch_andfsm(const DevParams& p, bool s2, uint32_t* fn, int64_t* out, hipStream_t st) {
  if (p.nseg <= 0) return hipSuccess;
  if (p.total_tiles > 0 && p.direct != 8) {  // (query_kernel_rfsm has written the tile maps)  // ~8 workgroups per CU, each wave over a contiguous run of tiles
    const dim3 g(std::min(2048, (p.total_tiles + 3) / 4));
    if (s2) hipLaunchKernelGGL(andfsm_tile_kernel<true>, g, dim3(256), 0, st, p, fn);
    else hipLaunchKernelGGL(andfsm_tile_kernel<false>, g, dim3(256), 0, st, p, fn);
  }
  hipLaunchKernelGGL(andfsm_segment_kernel, dim3(p.nseg), dim3(FSM_SEG_THREADS), 0, st, p, (const uint32_t*)fn, out);
  return hipGetLastError();
}

hipError_t pgpu_launch_progbits(const DevParams& p, const ProgJob* jobs, int njobs, int total, hipStream_t st) {
  if (njobs <= 0 || total <= 0) return hipSuccess;
  hipLaunchKernelGGL(progbits_kernel, dim3(std::min(2048, (total + 3) / 4)), dim3(256), (size_t)4 * p.mask_rows * 256, st, p, jobs,
                     njobs, total);
  return hipGetLastError();
}


hipError_t pgpu_launch_segcount(const DevParams& p, int64_t* out, hipStream_t st) {
  if (!p.segmask || p.segmask_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(segcount_kernel, dim3(p.segmask_rows), dim3(256), 0, st, p, out);
  return hipGetLastError();
}

hipError_t pgpu_launch_prologue(const DevParams& p, const void* host_arena, void* dev_arena, size_t bytes,
                                bool init_table, hipStream_t st) {
  const uint32_t n16 = (uint32_t)((bytes + 15) / 16);
  const int ncopy = std::max(1, std::min(16, (int)((n16 + 255) / 256)));
  int ninit = 0;
  if (init_table) {
    const uint64_t n = p.G * (uint64_t)(p.nsec + (p.mode == PGPU_MODE_HASH ? p.key_words : 0)) +
                       (p.segmask ? (uint64_t)p.segmask_rows * (p.G >> 5) : 0);
    ninit = (int)std::min<uint64_t>(4096, (n + 255) / 256);
    if (ninit < 1) ninit = 1;
  }
  hipLaunchKernelGGL(prologue_kernel, dim3(ncopy + ninit), dim3(256), 0, st, (const u32x4*)host_arena,
                     (u32x4*)dev_arena, n16, ncopy, p);
  return hipGetLastError();
}


hipError_t pgpu_launch_finalize(const DevParams& p, int nslabs, int64_t* stats_out, uint8_t* seg_out,
                                int64_t* host_table, uint64_t table_words, hipStream_t st) {
  const int nseg_blocks = p.nseg > 0 ? std::min(64, (p.nseg + 255) / 256) : 0;
  const bool copy = host_table && p.mode != PGPU_MODE_AGG;  // (AGG: finalize writes the host cells itself)
  const int nexp = copy ? (int)std::max<uint64_t>(1, std::min<uint64_t>(64, (table_words + 255) / 256)) : 0;
  hipLaunchKernelGGL(finalize_kernel, dim3(p.nsec + PGPU_NSTATS + nseg_blocks + nexp), dim3(256), 0, st, p, nslabs,
                     stats_out, seg_out, nseg_blocks, host_table, copy ? table_words : (uint64_t)0);
  return hipGetLastError();
}

hipError_t pgpu_launch_compact(const int64_t* table, uint64_t G, int32_t nsec, int32_t kw, int32_t* block_counts,
                               int64_t* total, int64_t* out_keys, int64_t* out_cells, bool count_only,
                               hipStream_t st, const uint64_t* okey, const TopkState* ts) {
  const int nb = (int)((G + CMP_PER_BLOCK - 1) / CMP_PER_BLOCK);
  if (count_only) {
    hipLaunchKernelGGL(compact_count_kernel, dim3(nb), dim3(CMP_BLOCK), 0, st, table, G, block_counts, okey, ts);
    hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(64), 0, st, block_counts, nb, total);
  } else {
    hipLaunchKernelGGL(compact_write_kernel, dim3(nb), dim3(CMP_BLOCK), 0, st, table, G, nsec, kw, block_counts,
                       out_keys, out_cells, okey, ts);
  }
  return hipGetLastError();
}

// ---- top-k selection (pgpu_table_topk): order keys, then 8 radix passes of 8 bits from the top ----------------
__global__ __launch_bounds__(256) void topk_key_kernel(const int64_t* table, TopkDev s, uint64_t* okey) {
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < s.G; k += (uint64_t)gridDim.x * 256)
    okey[k] = table[k] > 0 ? pgpu_topk_key(table, s, k) : 0ull;
}
__global__ void topk_init_kernel(TopkState* ts, uint32_t* hist, uint64_t k) {
  if (threadIdx.x == 0) {
    ts->prefix = 0;
    ts->mask = 0;
    ts->kleft = k;
  }
  hist[threadIdx.x] = 0;
}
// Histogram of digit (key >> shift) & 255 over the non-empty rows whose higher digits equal the prefix so far.
__global__ __launch_bounds__(256) void topk_hist_kernel(const int64_t* table, const uint64_t* okey, uint64_t G,
                                                        const TopkState* ts, int shift, uint32_t* hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t prefix = ts->prefix, mask = ts->mask;
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < G; k += (uint64_t)gridDim.x * 256) {
    const uint64_t u = okey[k];
    if (table[k] > 0 && (u & mask) == prefix) atomicAdd(&h[(u >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
// The digit holding the kleft-th best key: walk the bins from 255 down (one thread; 256 bins).
__global__ void topk_pick_kernel(TopkState* ts, uint32_t* hist, int shift) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = hist[threadIdx.x];
  hist[threadIdx.x] = 0;  // ready for the next pass
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint64_t kleft = ts->kleft, cum = 0;
  int d = 255;
  for (; d > 0; --d) {
    if (cum + h[d] >= kleft) break;
    cum += h[d];
  }
  // fewer than kleft rows under the prefix: d = 0 keeps every one of them (the threshold's low bits stay 0)
  ts->kleft = kleft > cum ? kleft - cum : 1;
  ts->prefix |= (uint64_t)d << shift;
  ts->mask |= 255ull << shift;
}

hipError_t pgpu_launch_node_route(const int64_t* keys, const int64_t* cells, uint64_t n, int32_t kw, int32_t nsec,
                                  int32_t world, uint8_t* owner, uint32_t* counts, uint32_t* cursor, int64_t* rows,
                                  bool scatter, hipStream_t st) {
  const int blocks = (int)std::min<uint64_t>(4096, std::max<uint64_t>(1, (n + 255) / 256));
  if (!scatter)
    hipLaunchKernelGGL(node_owner_kernel, dim3(blocks), dim3(256), 0, st, keys, n, kw, world, owner, counts);
  else
    hipLaunchKernelGGL(node_scatter_kernel, dim3(blocks), dim3(256), 0, st, keys, cells, n, kw, nsec, owner, cursor,
                       rows);
  return hipGetLastError();
}
hipError_t pgpu_launch_node_merge(const int64_t* rows, uint64_t n, int32_t kw, int32_t nsec, int64_t* table,
                                  uint64_t P, const NodeOps& ops, int32_t* hflag, hipStream_t st) {
  const int ib = (int)std::min<uint64_t>(4096, (P * (uint64_t)(nsec + 2) + 255) / 256);
  hipLaunchKernelGGL(node_init_kernel, dim3(ib), dim3(256), 0, st, table, P, nsec, kw, ops);
  if (n) {
    const int blocks = (int)std::min<uint64_t>(4096, (n + 255) / 256);
    hipLaunchKernelGGL(node_merge_kernel, dim3(blocks), dim3(256), 0, st, rows, n, kw, nsec, table, P, ops, hflag);
  }
  return hipGetLastError();
}
hipError_t pgpu_launch_topk(const int64_t* table, const TopkDev& s, uint64_t k, uint64_t* okey, TopkState* ts,
                            uint32_t* hist, hipStream_t st) {
  const int blocks = (int)std::max<uint64_t>(1, std::min<uint64_t>(2048, (s.G + 255) / 256));
  hipLaunchKernelGGL(topk_key_kernel, dim3(blocks), dim3(256), 0, st, table, s, okey);
  hipLaunchKernelGGL(topk_init_kernel, dim3(1), dim3(256), 0, st, ts, hist, k);
  for (int shift = 56; shift >= 0; shift -= 8) {
    hipLaunchKernelGGL(topk_hist_kernel, dim3(blocks), dim3(256), 0, st, table, okey, s.G, ts, shift, hist);
    hipLaunchKernelGGL(topk_pick_kernel, dim3(1), dim3(256), 0, st, ts, hist, shift);
  }
  return hipGetLastError();
}
#endif  // TU_HAS(PGPU_TU_COMMON)
