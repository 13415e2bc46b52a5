// Probe: the LDS-DMA weight-tile primitive of the decoder weight feed (cet_v4.hpp dma_tile) in isolation.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/dma_probe.hip -o tools/probe/dma_probe && tools/probe/dma_probe
// Each wave of a 512-thread workgroup DMAs T 1-KiB tiles (buffer_load_dwordx4 … lds, M0 = the wave-uniform LDS
// destination, lane l's 16 bytes at dst + 16·l) from a blob into its own LDS slots, waits with a counted
// s_waitcnt vmcnt, reads its slots back with ds_read_b128 and stores them: the host checks every byte.  The
// s_memtime span from the first issue to the vmcnt(0) retire is reported per wave (L2-warm on the second pass).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <vector>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void dma_tile(v4u rsrc, uint32_t soff, uint32_t dst, int voff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(dst), "s"(soff)
      : "memory");
}

constexpr int T = 6;   // tiles per wave

__global__ void __launch_bounds__(512) probe(const float* blob, float* out, unsigned long long* cyc, int pass) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const uint64_t p = (uint64_t)blob;
  const v4u r = {(unsigned)p, (unsigned)(p >> 32) & 0xffffu, 0x7ffffff0u, 0x00020000u};
  const int lane = threadIdx.x & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wg = blockIdx.x;
  // poison the wave's slots first (the read-back must see the DMA's bytes, not stale ones)
  for (int t = 0; t < T; ++t) reinterpret_cast<float4*>(lds + (w * T + t) * 1024)[lane] = float4{-1.f, -1.f, -1.f, -1.f};
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int t = 0; t < T; ++t)
    dma_tile(r, (uint32_t)((((wg * 8 + w) * T) + t) * 1024u), (uint32_t)((w * T + t) * 1024u), lane * 16);
  // the oldest tile first (counted), then all
  asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  const float4 first = reinterpret_cast<const float4*>(lds + (w * T) * 1024)[lane];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < T; ++t) {
    float4 v = reinterpret_cast<const float4*>(lds + (w * T + t) * 1024)[lane];
    if (t == 0) v = first;
    reinterpret_cast<float4*>(out)[((wg * 8 + w) * T + t) * 64 + lane] = v;
  }
  if (lane == 0) cyc[(pass * gridDim.x + wg) * 8 + w] = t1 - t0;
}

int main() {
  const int nwg = 512, n = nwg * 8 * T * 256;
  std::vector<float> h(n);
  for (int i = 0; i < n; ++i) h[i] = (float)(i % 100003) * 0.5f;
  float *d, *o;
  unsigned long long* c;
  hipMalloc(&d, n * 4);
  hipMalloc(&o, n * 4);
  hipMalloc(&c, 2 * nwg * 8 * 8);
  hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  for (int pass = 0; pass < 2; ++pass) {
    hipMemset(o, 0, n * 4);
    probe<<<nwg, 512, 8 * T * 1024>>>(d, o, c, pass);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("launch failed\n");
      return 1;
    }
    std::vector<float> g(n);
    hipMemcpy(g.data(), o, n * 4, hipMemcpyDeviceToHost);
    long bad = 0;
    for (int i = 0; i < n; ++i) bad += g[i] != h[i];
    std::vector<unsigned long long> cy(nwg * 8);
    hipMemcpy(cy.data(), c + pass * nwg * 8, nwg * 8 * 8, hipMemcpyDeviceToHost);
    double m = 0;
    for (auto v : cy) m += (double)v;
    printf("pass %d: %ld mismatching floats of %d; issue -> vmcnt(0) of %d tiles: mean %.0f cycles per wave\n", pass,
           bad, n, T, m / cy.size());
    if (bad) return 2;
  }
  printf("dma probe ok\n");
  return 0;
}
