// Micro-benchmark: the config-5 filter stream (a 10-bit bit-sliced column, 2048-doc tiles of 10 planes x 256 B)
// read straight into VGPRs -- plane k of lane l is one coalesced 4-B load per lane, 256 B per wave-instruction --
// with D tiles in flight per wave, against the LDS-DMA self-loading kernel's measured rate (query_kernel_direct).
// Each wave evaluates the RANGE predicate on the planes (v_bitop3 borrow chains) and counts matches, as the
// direct kernel's COUNT path does.  Build: hipcc --offload-arch=gfx950 -O3 tools/stream_bench.hip -o stream_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define B 10
#define TILE_BYTES (256 * B)

__device__ inline uint32_t lt_const(const uint32_t (&x)[B], uint32_t c) {
  uint32_t br = 0;
#pragma unroll
  for (int k = 0; k < B; ++k) br = __builtin_amdgcn_bitop3_b32((uint32_t)-(int32_t)((c >> k) & 1u), x[k], br, 0xB2);
  return br;
}

// wave w of the grid takes a contiguous run of tiles; D tiles in flight (register ring, fully unrolled)
template <int D, bool NT>
__global__ __launch_bounds__(256) void stream_kernel(const uint32_t* __restrict__ planes, int64_t ntiles,
                                                     uint32_t lo, uint32_t hi, unsigned long long* out) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  // XCD-aware: workgroups are dealt round-robin to 8 XCDs; give each XCD a contiguous block
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int64_t w = (int64_t)lb * 4 + (threadIdx.x >> 6);
  const int64_t t0 = ntiles * w / nwaves, t1 = ntiles * (w + 1) / nwaves;
  uint32_t x[D][B];
  auto load = [&](int s, int64_t t) {
    const uint32_t* src = planes + t * (TILE_BYTES / 4) + lane;
#pragma unroll
    for (int k = 0; k < B; ++k) {
      if (NT) x[s][k] = __builtin_nontemporal_load(src + 64 * k);
      else x[s][k] = src[64 * k];
    }
  };
  uint32_t cnt = 0;
#pragma unroll
  for (int s = 0; s < D; ++s)
    if (t0 + s < t1) load(s, t0 + s);
  for (int64_t t = t0; t < t1; t += D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
      if (t + s < t1) {
        const uint32_t m = lt_const(x[s], hi) & ~lt_const(x[s], lo);
        cnt += __popc(m);
        if (t + s + D < t1) load(s, t + s + D);
      }
    }
  }
  atomicAdd(out, (unsigned long long)cnt);
}

int main(int argc, char** argv) {
  const int64_t ntiles = 491520;  // 30 x 2^25 docs / 2048
  const size_t bytes = (size_t)ntiles * TILE_BYTES;
  uint32_t* d;
  unsigned long long* o;
  hipMalloc(&d, bytes);
  hipMalloc(&o, 8);
  {
    std::vector<uint32_t> h(bytes / 4);
    uint32_t s = 12345;
    for (auto& v : h) { s = s * 1664525u + 1013904223u; v = s; }
    hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, auto kern, int wgs_per_cu) {
    const int grid = 256 * wgs_per_cu;
    float best = 1e9f;
    for (int rep = 0; rep < 6; ++rep) {
      hipMemset(o, 0, 8);
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, d, ntiles, 349u, 357u, o);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep) best = ms < best ? ms : best;
    }
    unsigned long long c;
    hipMemcpy(&c, o, 8, hipMemcpyDeviceToHost);
    printf("%-10s wg/cu %2d  %.4f ms  %7.1f GB/s  (count %llu)\n", name, wgs_per_cu, best, bytes / best / 1e6, c);
  };
  for (int w : {2, 4, 5, 6, 8}) {
    run("D2", stream_kernel<2, false>, w);
    run("D3", stream_kernel<3, false>, w);
    run("D4", stream_kernel<4, false>, w);
    run("D6", stream_kernel<6, false>, w);
    run("D4nt", stream_kernel<4, true>, w);
  }
  hipFree(d);
  hipFree(o);
  return 0;
}
