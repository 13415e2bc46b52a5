// Stage helpers shared by the fused kernels (dense layers with their epilogues, staging, dumps).
#pragma once
#include "cet_attention.hpp"
#include "cet_plan.hpp"

namespace cet {

constexpr int NW = 8;              // waves per workgroup: one per attention head
constexpr int NTHREADS = NW * WAVE;

__device__ __forceinline__ f32x4 affine(const float* __restrict__ P, const GemmDesc d, int n0, f32x4 acc) {
  if (d.scale != NONE) acc *= *reinterpret_cast<const f32x4*>(P + d.scale + n0);
  if (d.bias != NONE) acc += *reinterpret_cast<const f32x4*>(P + d.bias + n0);
  return acc;
}

__device__ __forceinline__ void zero_lds(char* lds, int bytes) {
  f32x4* p = reinterpret_cast<f32x4*>(lds);
  for (int i = threadIdx.x; i < bytes / 16; i += NTHREADS) p[i] = f32x4{0.f, 0.f, 0.f, 0.f};
}

__device__ __forceinline__ void stage_input(const float* __restrict__ src, float* dst, int L, int C, int CS) {
  for (int i = threadIdx.x; i < L * C; i += NTHREADS) {
    const int t = i / C, c = i - t * C;
    dst[t * CS + c] = src[i];
  }
}

__device__ __forceinline__ void dump_rows(const float* X, int rows, float* dst) {
  for (int i = threadIdx.x; i < rows * DMODEL; i += NTHREADS) {
    const int m = i >> 7, n = i & 127;
    dst[i] = X[m * XS + n];
  }
}

// Q/K/V projection of `rows` positions of fp32 X: Q, K row-major bf16, V transposed.
template <class BL>
__device__ __forceinline__ void qkv_projection(const float* __restrict__ P, const bf16x8* __restrict__ W,
                                               const GemmDesc d, BL&& bl, int rows, __bf16* Q, __bf16* K,
                                               __bf16* Vt, int vts) {
  const int mt = (rows + 15) >> 4;
  gemm_t<4, 3, NW>(W + d.w, 24, mt, bl, [&](int m, int n0, f32x4 acc) {
    if (m >= rows) return;
    const f32x4 v = affine(P, d, n0, acc);
    if (n0 < 128) {
      *reinterpret_cast<bf16x4*>(Q + m * BS + n0) = cvt4(v);
    } else if (n0 < 256) {
      *reinterpret_cast<bf16x4*>(K + m * BS + n0 - 128) = cvt4(v);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) Vt[(n0 - 256 + r) * vts + m] = (__bf16)v[r];
    }
  });
}

// X[m][:] += W·src[m] + b  for m < rows   (out_projection / FFN conv2 + residual)
template <int KS, class BL>
__device__ __forceinline__ void residual_gemm(const float* __restrict__ P, const bf16x8* __restrict__ W,
                                              const GemmDesc d, BL&& bl, float* X, int rows) {
  gemm_t<KS, 1, NW>(W + d.w, 8, (rows + 15) >> 4, bl, [&](int m, int n0, f32x4 acc) {
    if (m >= rows) return;
    f32x4* px = reinterpret_cast<f32x4*>(X + m * XS + n0);
    *px = *px + affine(P, d, n0, acc);
  });
}

// FFN hidden = act(W1·X + b1) as bf16 rows (encoder.py:52-53, decoder.py:37)
template <int DFF, class BL>
__device__ __forceinline__ void ffn_hidden(const float* __restrict__ P, const bf16x8* __restrict__ W,
                                           const GemmDesc d, BL&& bl, int rows, __bf16* H, int relu) {
  gemm_t<4, 1, NW>(W + d.w, DFF / 16, (rows + 15) >> 4, bl, [&](int m, int n0, f32x4 acc) {
    if (m >= rows) return;
    f32x4 v = affine(P, d, n0, acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = relu ? fmaxf(v[r], 0.f) : gelu_erf(v[r]);
    *reinterpret_cast<bf16x4*>(H + m * BS + n0) = cvt4(v);
  });
}

}  // namespace cet
