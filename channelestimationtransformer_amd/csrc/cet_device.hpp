// Device-side building blocks of the fused channel-predictor kernels (gfx950 / CDNA4).
//
// Conventions used by every kernel in this directory:
//  * One workgroup = one channel sequence; NWAVES waves of 64 lanes.
//  * Activations live in LDS for the whole forward.  The residual stream X is
//    fp32 [rows][XS] (XS = 132 floats, +16 B/row so 16 consecutive rows start on
//    distinct 4-bank slots); GEMM operands/results that only feed MFMAs are bf16
//    [rows][BS] (BS = 136).  V is kept transposed (Vt[feature][key]) so it is the
//    A operand of the P·V product without a transpose.
//  * Dense layers are computed TRANSPOSED: Yᵀ[n][m] = W[n][k] · Xᵀ[k][m] on
//    v_mfma_f32_16x16x32_bf16.  W (the A operand) is pre-packed on the host in
//    fragment order [n_tile][k_step][lane][8] so one wave loads a 16×32 weight
//    tile with one fully coalesced 1 KiB global_load_dwordx4; X (the B operand)
//    is read from LDS rows; the C tile lands as 4 consecutive output features of
//    one sequence position per lane (one 16/8-byte LDS store).
//  * Attention runs one wave per head on v_mfma_f32_16x16x16_bf16 with scores
//    computed as Sᵀ = K·Qᵀ (key on the register axis, query on the lane axis), so
//    softmax reductions are in-register plus two cross-lane steps, and the
//    exponentiated tile is directly the B operand of Oᵀ = Vᵀ·Pᵀ.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cet_plan.hpp"

namespace cet {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

constexpr int WAVE = 64;
constexpr float NEG_INF = -__builtin_inff();

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16x16x16(const bf16x4& a, const bf16x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(short4_t, a),
                                                   __builtin_bit_cast(short4_t, b), c, 0, 0, 0);
}

typedef __attribute__((ext_vector_type(8))) float f32x8;
typedef __attribute__((ext_vector_type(2))) unsigned long long u64x2;

// fp32 → bf16 (round to nearest even): vector conversions lower to one v_cvt_pk_bf16_f32 per pair
__device__ __forceinline__ bf16x8 cvt8(const f32x4& lo, const f32x4& hi) {
  const f32x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_convertvector(v, bf16x8);
}
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
// 4-wide as two 2-wide conversions: a 4-wide convertvector is scalarised into four single-value
// v_cvt_pk_bf16_f32 plus two v_perm_b32 (6 VALU); this is two v_cvt_pk_bf16_f32
__device__ __forceinline__ bf16x4 cvt4(const f32x4& v) {
#ifdef CET_CVT4_VEC
  return __builtin_convertvector(v, bf16x4);
#else
  const bf16x2 a = __builtin_convertvector((f32x2{v[0], v[1]}), bf16x2);
  const bf16x2 b = __builtin_convertvector((f32x2{v[2], v[3]}), bf16x2);
  return __builtin_bit_cast(bf16x4, (u32x2{__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b)}));
#endif
}

// XOR-butterfly reductions across the lane axis.  The 16- and 32-lane exchanges use gfx950's
// v_permlane16_swap / v_permlane32_swap (one VALU op, no LDS); with both operands = v the two
// results are v and its partner, in some order per lane, so their sum/max is the butterfly.
__device__ __forceinline__ float swap_pair_sum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap_pair_sum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap_pair_max16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float swap_pair_max32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor_sum(float v, int m) {
  if (m == 16) return swap_pair_sum16(v);
  if (m == 32) return swap_pair_sum32(v);
  return v + __shfl_xor(v, m, 64);
}
__device__ __forceinline__ float xor_max(float v, int m) {
  if (m == 16) return swap_pair_max16(v);
  if (m == 32) return swap_pair_max32(v);
  return fmaxf(v, __shfl_xor(v, m, 64));
}

// Order LDS traffic of one wave: all earlier LDS ops of this wave complete before later ones
// are issued, and the compiler may not move memory ops across.  Used where lanes of one wave
// hand data to other lanes of the same wave through LDS (no workgroup barrier needed).
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// erf on [-4, 4] (±1 beyond, as in fp32) as an odd/even rational in x²: branch-free, one reciprocal;
// |error| ≤ 4.2e-7 against the exact erf (GELU's absolute error ≤ 7e-7; tools/erf_check.py).
__device__ __forceinline__ float erf_rational(float a) {
  const float x = __builtin_amdgcn_fmed3f(a, -4.0f, 4.0f);
  const float x2 = x * x;
  float p = fmaf(x2, -2.72614225801306e-10f, 2.77068142495902e-08f);
  p = fmaf(p, x2, -2.10102402082508e-06f);
  p = fmaf(p, x2, -5.69250639462346e-05f);
  p = fmaf(p, x2, -7.34990630326855e-04f);
  p = fmaf(p, x2, -2.95459980854025e-03f);
  p = fmaf(p, x2, -1.60960333262415e-02f);
  float q = fmaf(x2, -1.45660718464996e-05f, -2.13374055278905e-04f);
  q = fmaf(q, x2, -1.68282697438203e-03f);
  q = fmaf(q, x2, -7.37332916720468e-03f);
  q = fmaf(q, x2, -1.42647390514189e-02f);
  return x * p * __builtin_amdgcn_rcpf(q);
}
#if defined(CET_ABL_GELU)
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x; }   // ablation (wrong results)
#elif defined(CET_OCML_ERF)
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
#else
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_rational(x * 0.70710678118654752f)); }
#endif
// exp(x) - 1 on v_exp_f32: absolute error ~1e-7 near 0, far inside the parity bar
__device__ __forceinline__ float elu1(float x) { return x > 0.f ? x : __expf(x) - 1.0f; }

// ---------------------------------------------------------------------------------------------
// Dense layer on MFMA:  for m < rows, n < N:  Y[m][n] = Σ_k W[n][k] X[m][k]   (then epilogue).
//   Wf      : packed weights [N/16][KS][64 lanes] of bf16x8 (host-packed fragment order)
//   NT      : n-tiles (16 columns) per wave work unit (all of them kept in registers)
//   bload   : functor (m, k0) -> bf16x8 of X[m][k0 .. k0+7]
//   epi     : functor (m, n0, f32x4 acc) consuming Y[m][n0 .. n0+3]
// Work units = (group of NT n-tiles) × (m split); waves take units round-robin.
// ---------------------------------------------------------------------------------------------
template <int KS, int NT, int NWAVES, class BLoad, class Epi>
__device__ __forceinline__ void gemm_t(const bf16x8* __restrict__ Wf, int n_tiles, int m_tiles,
                                       BLoad&& bload, Epi&& epi) {
  const int lane = lane_id();
  const int wave = wave_id();
  const int n_groups = n_tiles / NT;
  int m_split = NWAVES / (n_groups > 0 ? n_groups : 1);
  if (m_split < 1) m_split = 1;
  if (m_split > m_tiles) m_split = m_tiles;
  const int units = n_groups * m_split;
  const int mrow = lane & 15;
  const int kq = (lane >> 4) * 8;
  const int nq = (lane >> 4) * 4;
  for (int unit = wave; unit < units; unit += NWAVES) {
    const int g = unit % n_groups;
    const int ms = unit / n_groups;
    bf16x8 a[NT][KS];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) a[t][ks] = Wf[((size_t)((g * NT + t) * KS + ks)) * WAVE + lane];
    for (int mt = ms; mt < m_tiles; mt += m_split) {
      f32x4 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int m = mt * 16 + mrow;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 b = bload(m, ks * 32 + kq);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x32(a[t][ks], b, acc[t]);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) epi(m, (g * NT + t) * 16 + nq, acc[t]);
    }
  }
}

// B-operand loaders -------------------------------------------------------------------------

// fp32 X rows in LDS, converted to bf16 on the fly.
struct LoadF32 {
  const float* X;  // LDS, stride XS
  __device__ __forceinline__ bf16x8 operator()(int m, int k0) const {
    const f32x4* p = reinterpret_cast<const f32x4*>(X + m * XS + k0);
    return cvt8(p[0], p[1]);
  }
};

// bf16 rows in LDS (stride BS).
struct LoadBF16 {
  const __bf16* X;
  __device__ __forceinline__ bf16x8 operator()(int m, int k0) const {
    return *reinterpret_cast<const bf16x8*>(X + m * BS + k0);
  }
};

// Circular k=3 convolution over time on fp32 X rows:  A[m][tap·D + c] = X[(m-1+tap) mod L][c].
template <int D>
struct LoadCirc3F32 {
  const float* X;
  int L;
  __device__ __forceinline__ bf16x8 operator()(int m, int k0) const {
    const int tap = k0 / D, c = k0 - tap * D;
    int r = m - 1 + tap;
    r = r < 0 ? r + L : (r >= L ? r - L : r);
    r = r >= L ? r % L : r;  // padded rows m >= L
    const f32x4* p = reinterpret_cast<const f32x4*>(X + r * XS + c);
    return cvt8(p[0], p[1]);
  }
};

// Token embedding input: staged x[t][C] fp32 (row stride CS), A[m][tap·C + c], zero past 3·C.
struct LoadEmbed {
  const float* X;
  int L, C, CS;
  __device__ __forceinline__ bf16x8 operator()(int m, int k0) const {
    const int tap = k0 / C, c = k0 - tap * C;
    if (tap >= 3) return bf16x8{};
    int r = m - 1 + tap;
    r = r < 0 ? r + L : r;
    r = r % L;
    const f32x4* p = reinterpret_cast<const f32x4*>(X + r * CS + c);
    return cvt8(p[0], p[1]);
  }
};

// ---------------------------------------------------------------------------------------------
// LayerNorm over 128 features of fp32 rows (in place or to another fp32 buffer), 16 lanes per
// row, 4 rows per wave-iteration.  torch.nn.LayerNorm semantics (biased variance, eps inside
// the sqrt).  If `unbiased_std` the reference Transformer's LayerNormalization is applied
// instead: alpha·(x-mean)/(std_unbiased + eps) + bias (buildingblocks.py:23-30).
// Optionally also writes a bf16 copy (dst_b, stride BS).
// ---------------------------------------------------------------------------------------------
template <int NWAVES>
__device__ __forceinline__ void layer_norm_rows(const float* src, float* dst, __bf16* dst_b, int rows,
                                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                                float eps, bool unbiased_std) {
  const int lane = lane_id();
  const int wave = wave_id();
  const int sub = lane >> 4;       // row within the wave's group of 4
  const int c0 = (lane & 15) * 8;  // 8 features per lane
  const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + c0);
  const f32x4 g1 = *reinterpret_cast<const f32x4*>(gamma + c0 + 4);
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(beta + c0);
  const f32x4 b1 = *reinterpret_cast<const f32x4*>(beta + c0 + 4);
  for (int rb = wave * 4; rb < rows; rb += NWAVES * 4) {
    const int r = rb + sub;
    const int rr = r < rows ? r : rows - 1;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(src + rr * XS + c0);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(src + rr * XS + c0 + 4);
    float s = (v0[0] + v0[1]) + (v0[2] + v0[3]) + (v1[0] + v1[1]) + (v1[2] + v1[3]);
    s = xor_sum(s, 1); s = xor_sum(s, 2); s = xor_sum(s, 4); s = xor_sum(s, 8);
    const float mean = s * (1.0f / 128.0f);
    f32x4 d0 = v0 - mean, d1 = v1 - mean;
    float q = d0[0] * d0[0] + d0[1] * d0[1] + d0[2] * d0[2] + d0[3] * d0[3] +
              d1[0] * d1[0] + d1[1] * d1[1] + d1[2] * d1[2] + d1[3] * d1[3];
    q = xor_sum(q, 1); q = xor_sum(q, 2); q = xor_sum(q, 4); q = xor_sum(q, 8);
    float inv;
    if (unbiased_std) inv = 1.0f / (sqrtf(q * (1.0f / 127.0f)) + eps);
    else inv = 1.0f / sqrtf(q * (1.0f / 128.0f) + eps);
    const f32x4 y0 = d0 * inv * g0 + b0;
    const f32x4 y1 = d1 * inv * g1 + b1;
    if (r < rows) {
      if (dst) {
        *reinterpret_cast<f32x4*>(dst + r * XS + c0) = y0;
        *reinterpret_cast<f32x4*>(dst + r * XS + c0 + 4) = y1;
      }
      if (dst_b) *reinterpret_cast<bf16x8*>(dst_b + r * BS + c0) = cvt8(y0, y1);
    }
  }
}

}  // namespace cet
