// Probe: does v_permlane16/32_swap_b32 give the butterfly partner's value when its operands live in
// VGPRs above v127?  Each lane sums its value with the xor-16 / xor-32 partner through the swap on a
// low register pair (v0, v1) and on a high pair (v200, v201), with wait states around the swap, over
// many waves; mismatches against the exact partner sum are counted.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define SWAP(NAME, INST, R0, R1)                                                                            \
  __device__ __forceinline__ float NAME(float v) {                                                          \
    float r;                                                                                                 \
    asm volatile("v_mov_b32 " R0 ", %1\n\tv_mov_b32 " R1 ", %1\n\ts_nop 1\n\t" INST " " R0 ", " R1          \
                 "\n\ts_nop 1\n\tv_add_f32 %0, " R0 ", " R1                                                  \
                 : "=v"(r) : "v"(v) : R0, R1);                                                               \
    return r;                                                                                                \
  }
SWAP(lo16, "v_permlane16_swap_b32", "v0", "v1")
SWAP(lo32, "v_permlane32_swap_b32", "v0", "v1")
SWAP(hi16, "v_permlane16_swap_b32", "v200", "v201")
SWAP(hi32, "v_permlane32_swap_b32", "v200", "v201")

__global__ void probe(const float* in, int* bad, int iters) {
  const int lane = threadIdx.x & 63;
  const float* p = in + (size_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63);
  int b0 = 0, b1 = 0, b2 = 0, b3 = 0;
  for (int it = 0; it < iters; ++it) {
    const float v = p[lane] + it;
    const float e16 = v + (p[lane ^ 16] + it), e32 = v + (p[lane ^ 32] + it);
    b0 += lo16(v) != e16;
    b1 += lo32(v) != e32;
    b2 += hi16(v) != e16;
    b3 += hi32(v) != e32;
  }
  atomicAdd(bad + 0, b0);
  atomicAdd(bad + 1, b1);
  atomicAdd(bad + 2, b2);
  atomicAdd(bad + 3, b3);
}

int main() {
  const int blocks = 1024, threads = 512, iters = 64;
  std::vector<float> h((size_t)blocks * threads);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 0.25f;
  float* d;
  int* bad;
  hipMalloc(&d, h.size() * 4);
  hipMalloc(&bad, 16);
  hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipMemset(bad, 0, 16);
  hipLaunchKernelGGL(probe, dim3(blocks), dim3(threads), 0, 0, d, bad, iters);
  int hb[4];
  hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost);
  printf("mismatches of %lld: lo16 %d lo32 %d hi16 %d hi32 %d\n", (long long)blocks * threads * iters, hb[0], hb[1],
         hb[2], hb[3]);
  return 0;
}
