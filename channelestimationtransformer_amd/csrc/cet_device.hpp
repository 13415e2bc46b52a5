// Device-side building blocks of the fused channel-predictor kernels (gfx950 / CDNA4).
//
// Conventions shared by the fused kernels (cet_v4.hpp, cet_transformer4.hip):
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
typedef __attribute__((ext_vector_type(2))) int i32x2;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;

constexpr int WAVE = 64;
constexpr float NEG_INF = -__builtin_inff();

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
// Thread index the compiler cannot hoist: loop-invariant per-lane addresses of once-per-call copies
// (count tables, sampler state) would otherwise be computed at the encoder loop's entry and live, spilled,
// across the whole kernel.
__device__ __forceinline__ int tid_op() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  __builtin_assume(t >= 0 && t < 1024);
  return t;
}

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
// Caution: a butterfly is only right when every lane takes part, and the compiler once sank such swaps
// into EXEC-narrowed code (the retired two-sequence kernel, profiles/r03/bisect_*.txt).  Every call sits
// at full EXEC in the source; tools/exec_scan.py checks the built code objects for a swap reached under
// a narrowed EXEC (tests/test_isa_guard.py, CPU suite).
// max of three as one v_max3_f32 (NaN-free operands; fmaxf trees get re-paired by the compiler)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
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

}  // namespace cet
