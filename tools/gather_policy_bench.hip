// Micro-benchmark: random 4-B gathers from an HBM-resident column (2.5 GiB, past the Infinity Cache) -- what one
// gather costs in DRAM bandwidth under each load policy / allocation kind, alone and beside a coalesced stream of
// the shape of config 5's plane stream.  Informs the candidate-gather design of the register-direct kernel
// (DESIGN.md 4.1).  Build: hipcc --offload-arch=gfx950 -O3 tools/gather_policy_bench.hip -o tools/gather_policy_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ inline uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  return x ^ (x >> 16);
}

// POL 0: default; 1: nontemporal; 2: sc0 sc1 (system scope) via asm; 3: sc1 only
template <int POL>
__device__ inline uint32_t ld(const uint32_t* p) {
  if constexpr (POL == 0) return *p;
  if constexpr (POL == 1) return __builtin_nontemporal_load(p);
  uint32_t v;  // no wait here: the caller waits once for all R loads (asm_wait)
  if constexpr (POL == 2) asm volatile("global_load_dword %0, %1, off sc0 sc1" : "=v"(v) : "v"(p) : "memory");
  else asm volatile("global_load_dword %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// every lane: `rounds` x R random gathers over `words` words; optional stream of `splanes` words per round
template <int POL, int R>
__global__ __launch_bounds__(256) void gather_kernel(const uint32_t* __restrict__ col, uint64_t words, int rounds,
                                                     const uint32_t* __restrict__ stream, uint64_t swords,
                                                     int splanes, uint32_t* out) {
  uint32_t acc = 0, seed = blockIdx.x * 256 + threadIdx.x;
  const uint64_t gw = (uint64_t)blockIdx.x * 256 + threadIdx.x, nthr = (uint64_t)gridDim.x * 256;
  for (int it = 0; it < rounds; ++it) {
    uint32_t v[R];
    if (POL <= 1) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint64_t h = ((uint64_t)mix(seed + (uint32_t)(it * R + r) * 0x9E3779B9u) << 8) ^ mix(seed * 7 + it * R + r);
        v[r] = ld<POL>(col + h % words);
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint64_t h = ((uint64_t)mix(seed + (uint32_t)(it * R + r) * 0x9E3779B9u) << 8) ^ mix(seed * 7 + it * R + r);
        v[r] = ld<POL>(col + h % words);
      }
      static_assert(R == 4, "asm wait ties four registers");
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]) :: "memory");
    }
    uint32_t s[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < splanes) s[k] = __builtin_nontemporal_load(stream + ((gw + ((uint64_t)it * 16 + k) * nthr) % swords));
#pragma unroll
    for (int r = 0; r < R; ++r) acc += v[r];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < splanes) acc ^= s[k];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t bytes = 2560ull << 20, words = bytes / 4;
  const uint64_t sbytes = 2048ull << 20, swords = sbytes / 4;
  uint32_t *col, *colu, *stream, *o;
  hipMalloc(&col, bytes);
  hipExtMallocWithFlags((void**)&colu, bytes, hipDeviceMallocUncached);
  hipMalloc(&stream, sbytes);
  hipMalloc(&o, 64);
  hipMemset(col, 1, bytes);
  hipMemset(colu, 1, bytes);
  hipMemset(stream, 2, sbytes);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int wgs = 256 * 8, rounds = 32;
  constexpr int R = 4;
  auto run = [&](const char* what, auto kern, const uint32_t* c, int splanes) {
    float best = 1e9f;
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(a);
      hipLaunchKernelGGL(kern, dim3(wgs), dim3(256), 0, 0, c, words, rounds, stream, swords, splanes, o);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep) best = ms < best ? ms : best;
    }
    const double g = (double)wgs * 256 * rounds * R, sb = (double)wgs * 256 * rounds * splanes * 4;
    printf("%-22s stream %2d planes: %7.3f ms  %6.1f G gathers/s  stream %6.0f GB/s  (at 128 B/gather + stream: %5.0f GB/s)\n",
           what, splanes, best, g / best / 1e6, sb / best / 1e6, (g * 128 + sb) / best / 1e6);
  };
  for (int sp : {0, 4, 16}) {
    run("default", gather_kernel<0, R>, col, sp);
    run("nt", gather_kernel<1, R>, col, sp);
    run("sc0 sc1", gather_kernel<2, R>, col, sp);
    run("sc1", gather_kernel<3, R>, col, sp);
    run("uncached alloc", gather_kernel<0, R>, colu, sp);
    run("uncached alloc nt", gather_kernel<1, R>, colu, sp);
  }
  return 0;
}
