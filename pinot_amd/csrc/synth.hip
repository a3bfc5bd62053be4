// libpinotgpu_synth.so — synthetic segment generator for bench.py and the GPU tests (not part of the query path).
//
// Writes a fixed-bit forward index (the FixedBitSVForwardIndexWriter layout: MSB-first, big-endian, b bits per doc,
// seglocal/io/writer/impl/FixedBitSVForwardIndexWriter.java:39-47) straight into HBM, so a 1B-row segment set
// does not have to be generated on the host and pushed over PCIe.  Dict ids come from a counter-based hash that
// pinot_amd/synth.py restates in numpy (and oracle/ in C), so every generated segment can be rebuilt on the CPU:
//   id(doc) = ((splitmix64(seed ^ (doc * 0xD1B54A32D192ED03)) >> 32) * card) >> 32        (uniform)
//   id(doc) = first k with cdf[k] > u(doc)                                                  (table distribution)
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ uint32_t synth_id(uint64_t seed, uint64_t doc, uint32_t card, const uint32_t* cdf) {
  const uint32_t u = (uint32_t)(splitmix64(seed ^ (doc * 0xD1B54A32D192ED03ull)) >> 32);
  if (!cdf) return (uint32_t)(((uint64_t)u * card) >> 32);
  uint32_t lo = 0, hi = card - 1;  // first k with cdf[k] > u
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (cdf[mid] > u) hi = mid; else lo = mid + 1;
  }
  return lo;
}

// One workgroup = 256 threads x 32 docs; thread t packs docs [32t, 32t+32) of the block into b words in LDS,
// then the block writes its 256*b words coalesced (byte-swapped to big-endian).
__global__ __launch_bounds__(256) void synth_fixed_bit_kernel(uint32_t* out, int64_t num_docs, int32_t bits,
                                                             uint32_t card, uint64_t seed, const uint32_t* cdf) {
  __shared__ uint32_t words[256 * 32];
  const int64_t block_doc0 = (int64_t)blockIdx.x * 8192;
  const int64_t doc0 = block_doc0 + threadIdx.x * 32;
  const uint32_t b = (uint32_t)bits;
  uint32_t* w = words + threadIdx.x * b;
  for (uint32_t i = 0; i < b; ++i) w[i] = 0;
  for (int i = 0; i < 32; ++i) {
    const int64_t doc = doc0 + i;
    const uint32_t v = doc < num_docs ? synth_id(seed, (uint64_t)doc, card, cdf) : 0u;
    // bits [i*b, (i+1)*b) of this thread's group, MSB-first
    const uint32_t bit = (uint32_t)i * b;
    const uint32_t wi = bit >> 5, off = bit & 31;  // value starts at MSB-offset off of word wi
    const uint64_t sh = (uint64_t)v << (64 - b - off);  // aligned within a 64-bit window {w[wi], w[wi+1]}
    w[wi] |= (uint32_t)(sh >> 32);
    if (off + b > 32) w[wi + 1] |= (uint32_t)sh;
  }
  __syncthreads();
  const int64_t total_words = (num_docs * b + 31) / 32;
  const int64_t base = block_doc0 / 32 * b;
  for (int i = threadIdx.x; i < 256 * (int)b; i += 256) {
    const int64_t gw = base + i;
    if (gw < total_words) out[gw] = __builtin_bswap32(words[i]);
  }
}

}  // namespace

// Scratch buffers come from this library's HIP runtime (the one libpinotgpu.so uses), never from another
// runtime that may be loaded in the same process (e.g. a framework's bundled HIP).
extern "C" void* synth_alloc(uint64_t bytes) {
  void* p = nullptr;
  return hipMalloc(&p, bytes) == hipSuccess ? p : nullptr;
}
extern "C" int synth_free(void* p) { return hipFree(p) == hipSuccess ? 0 : -1; }
extern "C" int synth_sync(void) { return hipDeviceSynchronize() == hipSuccess ? 0 : -1; }
extern "C" int synth_copy_to_host(void* dst, const void* src, uint64_t bytes) {
  return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

extern "C" int synth_copy_from_host(void* dst, const void* src, uint64_t bytes) {
  return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

extern "C" int synth_fixed_bit(void* dev_out, int64_t num_docs, int32_t bits, int32_t card, uint64_t seed,
                               const void* dev_cdf, void* stream) {
  if (!dev_out || num_docs < 0 || bits < 1 || bits > 32 || card < 1) return -1;
  const int64_t blocks = (num_docs + 8191) / 8192;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(synth_fixed_bit_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (uint32_t*)dev_out, num_docs, bits, (uint32_t)card, seed, (const uint32_t*)dev_cdf);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
