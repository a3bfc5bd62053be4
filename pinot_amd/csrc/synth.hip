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

// ---- bitmap inverted index of a synthetic column (host) --------------------------------------------------------
// Builds the BitmapInvertedIndexWriter file (seglocal/segment/creator/impl/inv/BitmapInvertedIndexWriter.java:
// 35-124) for the dict ids held in a fixed-bit forward index (MSB-first, `bits` per doc): (card + 1) big-endian
// absolute int32 offsets, then one RoaringBitmap 0.9.26 portable serialization per dict id, with the
// container choice of RoaringBitmapWriter + runOptimize (array if <= 4096 values else bitmap; run when
// 2 + 4 * runs bytes is smaller).  Used to give the bench's inverted-index workload real index bytes; the CPU
// tests check it byte for byte against the oracle's writer.  *out is malloc'ed; release with synth_host_free.
#include <stdlib.h>
#include <string.h>
#include <vector>

namespace {
void put16(std::vector<uint8_t>& o, uint32_t v) {
  o.push_back((uint8_t)v);
  o.push_back((uint8_t)(v >> 8));
}
void put32le(std::vector<uint8_t>& o, uint32_t v) {
  for (int k = 0; k < 4; ++k) o.push_back((uint8_t)(v >> (8 * k)));
}
void roaring_of(const uint32_t* d, size_t n, std::vector<uint8_t>& out) {
  struct Ct {
    uint32_t key, card, kind;  // kind 0 array, 1 bitmap, 2 run
    size_t begin, end, runs;
  };
  std::vector<Ct> cts;
  for (size_t i = 0; i < n;) {
    const uint32_t key = d[i] >> 16;
    size_t j = i;
    size_t runs = 0;
    while (j < n && (d[j] >> 16) == key) {
      if (j == i || d[j] != d[j - 1] + 1) ++runs;
      ++j;
    }
    Ct c{key, (uint32_t)(j - i), 0, i, j, runs};
    c.kind = c.card <= 4096 ? 0 : 1;
    const size_t plain = c.kind == 0 ? 2 * (size_t)c.card : 8192;
    if (2 + 4 * runs < plain) c.kind = 2;
    cts.push_back(c);
    i = j;
  }
  const size_t size = cts.size();
  const size_t base = out.size();  // offsets are relative to this bitmap's first byte
  bool has_run = false;
  for (const Ct& c : cts) has_run |= c.kind == 2;
  if (has_run) {
    put32le(out, 12347u | (uint32_t)((size - 1) << 16));
    std::vector<uint8_t> flags((size + 7) / 8, 0);
    for (size_t i = 0; i < size; ++i)
      if (cts[i].kind == 2) flags[i / 8] |= (uint8_t)(1u << (i % 8));
    out.insert(out.end(), flags.begin(), flags.end());
  } else {
    put32le(out, 12346u);
    put32le(out, (uint32_t)size);
  }
  for (const Ct& c : cts) {
    put16(out, c.key);
    put16(out, c.card - 1);
  }
  auto payload_bytes = [](const Ct& c) -> size_t {
    return c.kind == 0 ? 2 * (size_t)c.card : (c.kind == 1 ? 8192 : 2 + 4 * c.runs);
  };
  if (!has_run || size >= 4) {
    size_t pos = out.size() - base + 4 * size;
    for (const Ct& c : cts) {
      put32le(out, (uint32_t)pos);
      pos += payload_bytes(c);
    }
  }
  for (const Ct& c : cts) {
    if (c.kind == 0) {
      for (size_t k = c.begin; k < c.end; ++k) put16(out, d[k] & 0xFFFF);
    } else if (c.kind == 1) {
      uint64_t w[1024];
      memset(w, 0, sizeof(w));
      for (size_t k = c.begin; k < c.end; ++k) w[(d[k] & 0xFFFF) >> 6] |= 1ull << (d[k] & 63);
      for (int k = 0; k < 1024; ++k)
        for (int b = 0; b < 8; ++b) out.push_back((uint8_t)(w[k] >> (8 * b)));
    } else {
      put16(out, (uint32_t)c.runs);
      size_t k = c.begin;
      while (k < c.end) {
        size_t e = k;
        while (e + 1 < c.end && d[e + 1] == d[e] + 1) ++e;
        put16(out, d[k] & 0xFFFF);
        put16(out, (uint32_t)(e - k));
        k = e + 1;
      }
    }
  }
}
}  // namespace

extern "C" int synth_inverted_index(const uint8_t* fwd, int64_t num_docs, int32_t bits, int32_t card,
                                    uint8_t** out, uint64_t* out_len) {
  if (!fwd || !out || !out_len || bits < 1 || bits > 31 || card < 1 || num_docs < 0) return -1;
  std::vector<uint32_t> count((size_t)card + 1, 0), ids((size_t)num_docs);
  for (int64_t i = 0; i < num_docs; ++i) {
    // value i: bits [i*b, (i+1)*b) of the big-endian bit stream
    const uint64_t bit = (uint64_t)i * bits;
    uint64_t v = 0;
    for (int k = 0; k < 5; ++k) v = (v << 8) | fwd[(bit >> 3) + k];
    const uint32_t id = (uint32_t)((v >> (40 - (bit & 7) - bits)) & ((1ull << bits) - 1));
    if (id >= (uint32_t)card) return -2;
    ids[(size_t)i] = id;
    ++count[id + 1];
  }
  for (int c = 0; c < card; ++c) count[c + 1] += count[c];
  std::vector<uint32_t> docs((size_t)num_docs), pos(count.begin(), count.end() - 1);
  for (int64_t i = 0; i < num_docs; ++i) docs[pos[ids[(size_t)i]]++] = (uint32_t)i;
  std::vector<uint8_t> blob;
  std::vector<uint32_t> offs((size_t)card + 1);
  const uint32_t header = 4u * (uint32_t)(card + 1);
  for (int c = 0; c < card; ++c) {
    offs[c] = header + (uint32_t)blob.size();
    roaring_of(docs.data() + count[c], count[c + 1] - count[c], blob);
  }
  offs[card] = header + (uint32_t)blob.size();
  const uint64_t total = header + blob.size();
  uint8_t* o = (uint8_t*)malloc(total);
  if (!o) return -3;
  for (int c = 0; c <= card; ++c) {
    o[4 * c] = (uint8_t)(offs[c] >> 24);
    o[4 * c + 1] = (uint8_t)(offs[c] >> 16);
    o[4 * c + 2] = (uint8_t)(offs[c] >> 8);
    o[4 * c + 3] = (uint8_t)offs[c];
  }
  memcpy(o + header, blob.data(), blob.size());
  *out = o;
  *out_len = total;
  return 0;
}

extern "C" void synth_host_free(void* p) { free(p); }
