// Micro-benchmark: random 4-B dictionary gathers on gfx950 -- lookups/s against the table size (L1 / L2 /
// Infinity Cache resident) and against how many distinct lines one wave-instruction touches.  Informs the
// PART phase-2 dictionary gather design.  Build: hipcc --offload-arch=gfx950 -O3 tools/gather_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ inline uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  return x ^ (x >> 16);
}

// every lane does `iters` rounds of R gathers; ids = hash & mask; `spread` > 0: ids of one wave-instruction fall in
// a window of `spread` consecutive entries (a sorted-bucket stand-in)
template <int R>
__global__ __launch_bounds__(256) void gather_kernel(const uint32_t* __restrict__ dict, uint32_t mask, int iters,
                                                     uint32_t spread, uint32_t* out) {
  uint32_t acc = 0, seed = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  for (int it = 0; it < iters; ++it) {
    uint32_t id[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t h = mix(seed + (uint32_t)(it * R + r) * 0x9E3779B9u);
      if (spread) {
        const uint32_t base = mix(__builtin_amdgcn_readfirstlane(h) ^ 0x1234567u) & mask;
        id[r] = (base + (h % spread)) & mask;
      } else {
        id[r] = h & mask;
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) acc += dict[id[r]];
  }
  if (acc == 0x12345678u) out[0] = acc + lane;
}

template <int R>
__global__ __launch_bounds__(256) void lds_kernel(const uint32_t* __restrict__ dict, uint32_t mask, int iters,
                                                  uint32_t* out) {
  extern __shared__ uint32_t sd[];
  for (uint32_t i = threadIdx.x; i <= mask; i += 256) sd[i] = dict[i];
  __syncthreads();
  uint32_t acc = 0, seed = blockIdx.x * 256 + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc += sd[mix(seed + (uint32_t)(it * R + r) * 0x9E3779B9u) & mask];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const int cus = 256, wgs = cus * 8, iters = 64;
  uint32_t* d;
  uint32_t* o;
  hipMalloc(&d, 64u << 20);
  hipMalloc(&o, 64);
  std::vector<uint32_t> h(16u << 20);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)i * 16u;
  hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipFuncSetAttribute((const void*)lds_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double lookups = (double)wgs * 256 * iters * 16;
  auto run = [&](const char* what, uint32_t entries, uint32_t spread, bool lds) {
    float best = 1e9f;
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(a);
      if (lds)
        hipLaunchKernelGGL(lds_kernel<16>, dim3(wgs / 4), dim3(256), entries * 4, 0, d, entries - 1, iters * 4, o);
      else
        hipLaunchKernelGGL(gather_kernel<16>, dim3(wgs), dim3(256), 0, 0, d, entries - 1, iters, spread, o);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep) best = ms < best ? ms : best;
    }
    printf("%-8s table %8u entries (%7u KiB) spread %6u: %7.3f ms  %7.1f G lookups/s\n", what, entries,
           entries / 256, spread, best, lookups / best / 1e6);
  };
  for (uint32_t e : {1u << 10, 1u << 12, 1u << 13, 1u << 14, 1u << 16, 1u << 18, 1u << 20, 1u << 24})
    run("global", e, 0, false);
  for (uint32_t s : {64u, 256u, 1024u, 4096u}) run("global", 1u << 16, s, false);
  for (uint32_t e : {1u << 12, 1u << 14, 1u << 15}) run("lds", e, 0, true);
  return 0;
}
