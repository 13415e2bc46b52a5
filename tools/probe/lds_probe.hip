// Probe: LDS bank conflicts of the fused kernel's access patterns, one kernel per pattern, measured with
//   rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -- ./lds_probe
// (conflict cycles ÷ LDS instructions per kernel).  The addresses follow cet_v4.hpp: activation images
// (Img::ld — the GEMM B operand, LoadCirc3EO — the distil conv input, Img::st4 — every image write), the
// LayerNorm partials (ln_publish / ln_row_stats), the ProbSparse count rows (attention_head phase A, at the
// round-4 row stride of 96 B and the round-5 104 B) and the decoder's mix-scrambled context writes
// (ctx_st4), for the image row layouts (template SWZ)
//   0: RS 272 (the default layout: 256 B of bf16 features + 16 B pad)
//   1: RS 256 with the 16-byte chunk index XOR-ed with the row's low 4 bits
//   2: RS 288 with byte bits 4-5 XOR-ed with row bits 2-3 (cet_v4.hpp Img::off under -DCET_IMG_SWZ)
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 64;

template <int RS, int SWZ>
__device__ __forceinline__ int img_addr(int row, int byte) {
  if constexpr (SWZ == 0) return row * RS + byte;
  if constexpr (SWZ == 1) return row * 256 + ((((byte >> 4) ^ row) & 15) << 4) + (byte & 15);
  return row * 288 + (byte & ~48) + ((byte & 48) ^ ((row << 2) & 48));
}

__device__ __forceinline__ int lane_() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// GEMM B operand: lane (g, c) reads row mt·16 + c, features ks·32 + 8g .. +7 (ds_read_b128)
template <int RS, int SWZ>
__global__ void __launch_bounds__(512) gemm_read(float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int l = lane_(), g = l >> 4, c = l & 15;
  float4 acc = {0, 0, 0, 0};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int mt = 0; mt < 6; ++mt)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const float4 v = *reinterpret_cast<const float4*>(lds + img_addr<RS, SWZ>(mt * 16 + c, 2 * (ks * 32 + 8 * g)));
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    __builtin_amdgcn_s_barrier();
  }
  out[blockIdx.x * 512 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

// the distil conv's input in even/odd position order (LoadCirc3EO, L = 90)
template <int RS, int SWZ>
__global__ void __launch_bounds__(512) conv_read(float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int l = lane_(), g = l >> 4, c = l & 15;
  const int L = 90;
  float4 acc = {0, 0, 0, 0};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int mt = 0; mt < 6; ++mt)
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        const int m = mt * 16 + c;
        const int pos = ((mt >> 1) << 5) + ((m & 15) << 1) + (mt & 1);
        const int k0 = k * 32 + 8 * g, tap = k0 >> 7, ch = k0 & 127;
        int r = pos - 1 + tap;
        r = r < 0 ? r + L : r;
        r = r >= L ? r - L : r;
        r = r >= L ? L - 1 : r;
        const float4 v = *reinterpret_cast<const float4*>(lds + img_addr<RS, SWZ>(r, 2 * ch));
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    __builtin_amdgcn_s_barrier();
  }
  out[blockIdx.x * 512 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

// image write (Img::st4): lane (g, c) of wave w writes row mt·16 + c, features 16w + 4g .. +3 (ds_write_b64)
template <int RS, int SWZ>
__global__ void __launch_bounds__(512) img_write(float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int l = lane_(), g = l >> 4, c = l & 15, w = threadIdx.x >> 6;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int mt = 0; mt < 6; ++mt) {
      const uint2 v = {(unsigned)(it + mt), (unsigned)l};
      *reinterpret_cast<uint2*>(lds + img_addr<RS, SWZ>(mt * 16 + c, 2 * (16 * w + 4 * g))) = v;
    }
    __builtin_amdgcn_s_barrier();
  }
  out[blockIdx.x * 512 + threadIdx.x] = (float)lds[threadIdx.x];
}

// LayerNorm partials: (Σx, Σx²) publish (ds_write_b32, lanes g and g + 2 same word) and the row
// statistics' four ds_read_b128 per row (LN_STRIDE = 20 floats)
__global__ void __launch_bounds__(512) ln_part(float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* part = reinterpret_cast<float*>(lds);
  const int l = lane_(), g = l >> 4, c = l & 15, w = threadIdx.x >> 6;
  float acc = 0.f;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int mt = 0; mt < 6; ++mt) part[(mt * 16 + c) * 20 + 2 * w + (g & 1)] = (float)(it + l);
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int mt = 0; mt < 6; ++mt) {
      const float* pr = part + (mt * 16 + c) * 20;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 p = *reinterpret_cast<const float4*>(pr + 4 * j);
        acc += p.x + p.y + p.z + p.w;
      }
    }
    __builtin_amdgcn_s_barrier();
  }
  out[blockIdx.x * 512 + threadIdx.x] = acc;
}

// ProbSparse phase A: lane (g, c) reads three u64 count words of row q = qt·16 + c at byte g·24 (row stride ST)
template <int ST>
__global__ void __launch_bounds__(512) cnt_read(float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int l = lane_(), g = l >> 4, c = l & 15;
  unsigned acc = 0;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int qt = 0; qt < 6; ++qt) {
      const uint2* crow = reinterpret_cast<const uint2*>(lds + (qt * 16 + c) * ST + g * 24);
      const uint2 a = crow[0], b = crow[1], d = crow[2];
      acc += a.x ^ a.y ^ b.x ^ b.y ^ d.x ^ d.y;
    }
    __builtin_amdgcn_s_barrier();
  }
  out[blockIdx.x * 512 + threadIdx.x] = (float)acc;
}

// the decoder self-attention's mix-scrambled context writes: head w, query c (LQ = 15), features 4g .. +3
// at flat index w·LQ·16 + q·16 + 4g of the (H, L, E) view → image row f >> 7, feature f & 127
template <int RS, int SWZ>
__global__ void __launch_bounds__(512) ctx_mix(float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int l = lane_(), g = l >> 4, c = l & 15, w = threadIdx.x >> 6;
  for (int it = 0; it < ITERS; ++it) {
    const int f = w * 15 * 16 + c * 16 + 4 * g;
    const uint2 v = {(unsigned)it, (unsigned)l};
    if (c < 15) *reinterpret_cast<uint2*>(lds + img_addr<RS, SWZ>(f >> 7, 2 * (f & 127))) = v;
    __builtin_amdgcn_s_barrier();
  }
  out[blockIdx.x * 512 + threadIdx.x] = (float)lds[threadIdx.x];
}

int main() {
  const int blocks = 512;
  float* d;
  hipMalloc(&d, (size_t)blocks * 512 * 4);
  const int shm = 96 * 288 + 256;
#define RUN(K) hipLaunchKernelGGL(K, dim3(blocks), dim3(512), shm, 0, d)
#define RUN3(K) RUN((K<272, 0>)); RUN((K<256, 1>)); RUN((K<288, 2>))
  RUN3(gemm_read);
  RUN3(conv_read);
  RUN3(img_write);
  RUN3(ctx_mix);
  RUN(ln_part);
  RUN(cnt_read<96>);
  RUN(cnt_read<104>);
  const hipError_t e = hipDeviceSynchronize();
  printf("lds_probe: %s\n", hipGetErrorString(e));
  hipFree(d);
  return e == hipSuccess ? 0 : 1;
}
