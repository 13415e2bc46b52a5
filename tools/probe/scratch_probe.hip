// Probe: does a private-memory (scratch) reload ever return a stale value?  (the ab8 candidate)
//   hipcc --offload-arch=gfx950 -O3 tools/probe/scratch_probe.hip -o tools/probe/scratch_probe && tools/probe/scratch_probe
// Every lane keeps a 256-byte array of 16-byte slots in private memory (runtime-indexed, so it cannot live in
// registers: scratch_store_dwordx4 / scratch_load_dwordx4, as the ab8 build's K/V weight struct).  For each of L
// "layers" the lane overwrites every slot with a layer-specific value, then reloads every slot R times (each reload
// checked), with global loads and LDS traffic in between like the attention's.  Two 512-thread workgroups per CU
// (80 KiB of LDS each), one wave of workgroups per launch.  Any reload that returns a value other than the last
// one stored counts as an error; the first few are reported with the lane, the slot and the layer it came from.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <vector>

constexpr int SLOTS = 16;

__device__ __forceinline__ uint4 val(int l, int i, unsigned gid) {
  return make_uint4(0x10000u * (unsigned)l + (unsigned)i, gid, (unsigned)(l * 7 + i), 0xA5000000u ^ gid);
}

__global__ void __launch_bounds__(512) probe(const uint4* noise, uint4* sink, unsigned* err, uint4* first, int L,
                                             int R, int s_st, int s_ld) {
  extern __shared__ uint4 lds[];
  uint4 buf[SLOTS];
  const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nerr = 0;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int l = 0; l < L; ++l) {
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) buf[(i + s_st) & (SLOTS - 1)] = val(l, i, gid);
    // global and LDS traffic between the stores and the reloads (the attention's pattern)
    const uint4 g = noise[(gid * 7u + (unsigned)l * 131u) & 65535u];
    lds[threadIdx.x + 512 * (l & 7)] = g;
    __syncthreads();
    const uint4 h = lds[(threadIdx.x * 3u + 17u) & 4095u];
    acc.x += g.x ^ h.y;
    acc.y += h.x;
    for (int r = 0; r < R; ++r) {
#pragma unroll
      for (int i = 0; i < SLOTS; ++i) {
        const uint4 v = buf[(i + s_ld) & (SLOTS - 1)];
        const uint4 e = val(l, i, gid);
        if (v.x != e.x || v.y != e.y || v.z != e.z || v.w != e.w) {
          if (nerr < 1) first[gid] = make_uint4(v.x, (unsigned)i, (unsigned)l, gid & 63u);
          ++nerr;
        }
        acc.z += v.z;
      }
      asm volatile("" ::: "memory");
    }
    __syncthreads();
  }
  err[gid] = nerr;
  sink[gid] = acc;
}

int main(int argc, char** argv) {
  const int L = argc > 1 ? atoi(argv[1]) : 64, R = argc > 2 ? atoi(argv[2]) : 4, reps = argc > 3 ? atoi(argv[3]) : 20;
  const int nblk = 512, nthr = 512, n = nblk * nthr;
  const size_t lds = 80 * 1024;
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  uint4 *noise, *sink, *first;
  unsigned* err;
  hipMalloc(&noise, 65536 * sizeof(uint4));
  hipMalloc(&sink, n * sizeof(uint4));
  hipMalloc(&first, n * sizeof(uint4));
  hipMalloc(&err, n * sizeof(unsigned));
  hipMemset(noise, 0x3c, 65536 * sizeof(uint4));
  std::vector<unsigned> h(n);
  std::vector<uint4> hf(n);
  unsigned long long total = 0;
  int shown = 0;
  for (int rep = 0; rep < reps; ++rep) {
    hipMemset(err, 0, n * sizeof(unsigned));
    hipLaunchKernelGGL(probe, dim3(nblk), dim3(nthr), lds, 0, noise, sink, err, first, L, R, 0, 0);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("launch failed\n");
      return 1;
    }
    hipMemcpy(h.data(), err, n * sizeof(unsigned), hipMemcpyDeviceToHost);
    hipMemcpy(hf.data(), first, n * sizeof(uint4), hipMemcpyDeviceToHost);
    unsigned long long e = 0;
    for (int i = 0; i < n; ++i) {
      e += h[i];
      if (h[i] && shown < 8) {
        printf("  rep %d thread %d lane %u: slot %u layer %u got x=%08x (layer %u slot %u)\n", rep, i, hf[i].w,
               hf[i].y, hf[i].z, hf[i].x, hf[i].x >> 16, hf[i].x & 0xffffu);
        ++shown;
      }
    }
    total += e;
  }
  const double checks = (double)reps * n * L * R * SLOTS;
  printf("scratch_probe: %d launches x %d threads, %d layers x %d reloads x %d slots: %llu stale of %.3g reloads\n",
         reps, n, L, R, SLOTS, total, checks);
  return total ? 2 : 0;
}
