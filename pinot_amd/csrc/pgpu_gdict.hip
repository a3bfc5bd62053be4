// On-the-fly group dictionary of a raw (no-dictionary) column, built on the GPU once per (segment, column) the first
// time a query groups on it.  The reference groups raw columns with NoDictionarySingleColumnGroupKeyGenerator /
// NoDictionaryMultiColumnGroupKeyGenerator (core/query/aggregation/groupby/NoDictionarySingleColumnGroupKeyGenerator
// .java:70-118, NoDictionaryMultiColumnGroupKeyGenerator.java:90-150): a value -> id hash map per column (its
// `_onTheFlyDictionaries`), keys equal when their values are equal as Java's primitive maps compare them -- by
// value for INT / LONG, by Float.floatToIntBits / Double.doubleToLongBits for FLOAT / DOUBLE (fastutil's float and
// double maps), so -0.0 and 0.0 are two keys and every NaN is one.
//
// Here the distinct values become a sorted dictionary (ascending by Float.compare order, the order of any Pinot
// dictionary) and every doc's id a fixed-bit forward index in the reference's MSB-first big-endian layout, so the
// column then groups exactly like a dictionary-encoded one (global dictionary, remap, every table strategy):
//   keys     one order-preserving uint64 per doc (floating values canonicalised: one NaN)
//   sort     rocprim radix sort of the keys, then rocprim::unique -> the dictionary's keys and cardinality
//   encode   each doc's id = lower_bound of its key; 32-bit big-endian words packed MSB first
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>

#include "../../include/pinot_gpu.h"

namespace {

// order-preserving unsigned key of a value (sign bit flipped; negative floats bit-inverted)
__device__ inline uint64_t gkey(const void* vals, int32_t dtype, int64_t i) {
  if (dtype == PGPU_INT) return (uint64_t)(int64_t)((const int32_t*)vals)[i] ^ 0x8000000000000000ull;
  if (dtype == PGPU_LONG) return (uint64_t)((const int64_t*)vals)[i] ^ 0x8000000000000000ull;
  if (dtype == PGPU_FLOAT) {
    uint32_t b = ((const uint32_t*)vals)[i];
    if ((b & 0x7F800000u) == 0x7F800000u && (b & 0x007FFFFFu)) b = 0x7FC00000u;  // Float.floatToIntBits: one NaN
    return (uint64_t)((b & 0x80000000u) ? ~b : (b | 0x80000000u));
  }
  uint64_t b = ((const uint64_t*)vals)[i];
  if ((b & 0x7FF0000000000000ull) == 0x7FF0000000000000ull && (b & 0x000FFFFFFFFFFFFFull)) b = 0x7FF8000000000000ull;
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

__global__ __launch_bounds__(256) void gdict_key_kernel(const void* vals, int32_t dtype, int64_t n, uint64_t* keys) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) keys[i] = gkey(vals, dtype, i);
}

// dictionary value of a key (inverse of gkey), little-endian
__global__ __launch_bounds__(256) void gdict_value_kernel(const uint64_t* uniq, int32_t card, int32_t dtype, void* dict) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < card; i += (int64_t)gridDim.x * 256) {
    const uint64_t k = uniq[i];
    if (dtype == PGPU_INT) ((int32_t*)dict)[i] = (int32_t)(int64_t)(k ^ 0x8000000000000000ull);
    else if (dtype == PGPU_LONG) ((int64_t*)dict)[i] = (int64_t)(k ^ 0x8000000000000000ull);
    else if (dtype == PGPU_FLOAT) {
      const uint32_t b = (uint32_t)k;
      ((uint32_t*)dict)[i] = (b & 0x80000000u) ? (b & 0x7FFFFFFFu) : ~b;
    } else {
      ((uint64_t*)dict)[i] = (k & 0x8000000000000000ull) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    }
  }
}

// id of every doc: lower_bound of its key among the card sorted distinct keys (it is there)
__global__ __launch_bounds__(256) void gdict_id_kernel(const uint64_t* keys, int64_t n, const uint64_t* uniq,
                                                       int32_t card, uint32_t* ids) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint64_t k = keys[i];
    int32_t lo = 0, hi = card;
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      if (uniq[mid] < k) lo = mid + 1; else hi = mid;
    }
    ids[i] = (uint32_t)lo;
  }
}

// word w of the MSB-first stream holds bits [32w, 32w + 32): the ids overlapping it, stored big-endian
__global__ __launch_bounds__(256) void gdict_pack_kernel(const uint32_t* ids, int64_t n, int bits, uint32_t* words,
                                                         int64_t nwords) {
  for (int64_t w = blockIdx.x * 256ll + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * 256) {
    const int64_t b0 = 32 * w, b1 = b0 + 32;
    uint32_t v = 0;
    for (int64_t d = b0 / bits; d < n && d * bits < b1; ++d) {
      const int64_t s = d * bits;  // the id's first bit; bit j of the id (MSB first) is stream bit s + j
      const uint64_t id = ids[d];
      // place the id's bits [s, s + bits) into this word's [b0, b1): shift relative to the word's MSB
      const int64_t sh = (b1 - (s + bits));  // left shift of the id inside a 32-bit window ending at b1
      if (sh >= 0) v |= (uint32_t)((id << sh) & 0xFFFFFFFFull);
      else v |= (uint32_t)(id >> (-sh));
    }
    words[w] = __builtin_bswap32(v);
  }
}

int grid_of(int64_t n) { return (int)std::min<int64_t>(4096, std::max<int64_t>(1, (n + 255) / 256)); }

}  // namespace

// Scratch bytes the sort + unique of n keys needs (rocprim's two-call convention).
size_t pgpu_gdict_temp_bytes(int64_t n) {
  size_t a = 0, b = 0;
  (void)rocprim::radix_sort_keys(nullptr, a, (uint64_t*)nullptr, (uint64_t*)nullptr, (size_t)n);
  (void)rocprim::unique(nullptr, b, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr, (size_t)n);
  return std::max(a, b);
}

// keys, sorted copy and distinct keys of the n values; *d_card (device) = the cardinality.
hipError_t pgpu_gdict_sort_unique(const void* vals, int32_t dtype, int64_t n, uint64_t* keys, uint64_t* sorted,
                                  uint64_t* uniq, uint32_t* d_card, void* temp, size_t temp_bytes, hipStream_t st) {
  hipLaunchKernelGGL(gdict_key_kernel, dim3(grid_of(n)), dim3(256), 0, st, vals, dtype, n, keys);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t tb = temp_bytes;
  e = rocprim::radix_sort_keys(temp, tb, keys, sorted, (size_t)n, 0, 64, st);
  if (e != hipSuccess) return e;
  tb = temp_bytes;
  return rocprim::unique(temp, tb, sorted, uniq, d_card, (size_t)n, rocprim::equal_to<uint64_t>(), st);
}

// the dictionary values (little-endian), each doc's id, and the packed forward index (nwords big-endian words).
hipError_t pgpu_gdict_encode(const uint64_t* keys, int64_t n, const uint64_t* uniq, int32_t card, int32_t dtype,
                             int bits, void* dict, uint32_t* ids, uint32_t* words, int64_t nwords, hipStream_t st) {
  hipLaunchKernelGGL(gdict_value_kernel, dim3(grid_of(card)), dim3(256), 0, st, uniq, card, dtype, dict);
  hipLaunchKernelGGL(gdict_id_kernel, dim3(grid_of(n)), dim3(256), 0, st, keys, n, uniq, card, ids);
  hipLaunchKernelGGL(gdict_pack_kernel, dim3(grid_of(nwords)), dim3(256), 0, st, ids, n, bits, words, nwords);
  return hipGetLastError();
}
