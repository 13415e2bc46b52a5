// Layer-wise engine for shapes outside the fused kernels (any d_model, n_heads with d_k = d_model //
// n_heads, d_ff, sequence lengths up to LW_LMAX): one launch per operator, activations fp32 in HBM,
// every contraction on the fp32-input MFMA (v_mfma_f32_16x16x4_f32: exact fp32 products, the
// reference's own arithmetic class, so the ProbSparse top-u selection matches it).
//
// Operators (reference behaviour they restate):
//   lw_gemm       Linear / Conv1d(k=1) / circular Conv1d(k=3) (TokenEmbedding embed.py:30-49, ConvLayer
//                 encoder.py:22-28) with bias, folded BatchNorm, positional table, activation and residual
//   lw_layernorm  nn.LayerNorm over the rows (encoder.py:49-56, decoder.py:33-40), output rows remappable
//                 (EncoderStack concatenation, encoder.py:95-106)
//   lw_maxpool    MaxPool1d(3, 2, 1) (encoder.py:20,27)
//   lw_window     x[:, -L:] of EncoderStack (encoder.py:102-104)
//   lw_attention  ProbAttention (attn.py:73-175) and FullAttention (attn.py:37-70) per (sequence, head),
//                 with the AttentionLayer mix re-view (attn.py:205-206) and the optional attns maps
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cet_lw.h"

namespace cet {
bool ensure_lds_attr(const void* kern);   // cet_api.cpp
}

namespace cet {
namespace lw {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float gelu(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

// ------------------------------------------------------------------------------------ GEMM
// C[m][n] = epi(Σ_k A(m, k) · W[n][k]); 64 × 64 output tile per 256-thread workgroup; wave w computes
// rows 16w..16w+15 × the tile's 64 columns (4 accumulators).  K is staged through LDS in chunks of 32:
// each thread fetches two 4-float runs of A and two of W per chunk (vector loads where the rows allow),
// the next chunk's runs are in registers while this chunk's MFMAs run, one barrier pair per chunk.
// LDS rows are 34 floats: the MFMA reads (lanes 0-15: rows r, column k; lanes 16-31: rows r, k + 1)
// hit 32 distinct banks.
constexpr int GT = 64, GK = 32, GKS = GK + 2;

__device__ __forceinline__ float load_a(const GemmOp& op, int m, int k) {
  if (m >= op.M || k >= op.K) return 0.f;
  if (op.amode == 0) return op.A[(size_t)m * op.lda + k];
  // circular k=3 conv over each sequence: m = b·L + t, k = tap·C + c → src row (t − 1 + tap) mod L
  const int b = m / op.L, t = m - b * op.L;
  const int tap = k / op.Cin, c = k - tap * op.Cin;
  int r = t - 1 + tap;
  r = r < 0 ? r + op.L : (r >= op.L ? r - op.L : r);
  return op.A[((size_t)b * op.Ls + op.off + r) * op.lda + c];
}
// A row of the GEMM as a fetch sees it: row m = b·L + t split once (the divisions stay out of the K loop)
struct ARow {
  int m, b, t;
};
__device__ __forceinline__ ARow arow(const GemmOp& op, int m) {
  const int b = m / op.L;
  return ARow{m, b, m - b * op.L};
}
// four consecutive k of row m (k0 a multiple of 4): one 16-byte load when the run is inside the row and
// aligned (lda % 4 == 0), else element by element.  amode 1 (circular k=3 conv): the run stays inside one
// tap (Cin % 4 == 0), so it is four consecutive channels of one source row.
__device__ __forceinline__ f32x4 load_a4(const GemmOp& op, const ARow& ra, int k0, bool vec) {
  if (ra.m >= op.M || k0 >= op.K) return f32x4{0.f, 0.f, 0.f, 0.f};
  if (op.amode == 0) {
    const float* p = op.A + (size_t)ra.m * op.lda + k0;
    if (vec && k0 + 3 < op.K) return *reinterpret_cast<const f32x4*>(p);
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = k0 + i < op.K ? p[i] : 0.f;
    return v;
  }
  const int tap = k0 / op.Cin, c = k0 - tap * op.Cin;
  int r = ra.t - 1 + tap;
  r = r < 0 ? r + op.L : (r >= op.L ? r - op.L : r);
  const float* p = op.A + ((size_t)ra.b * op.Ls + op.off + r) * op.lda + c;
  if (vec && (op.Cin & 3) == 0 && k0 + 3 < op.K) return *reinterpret_cast<const f32x4*>(p);
  f32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = load_a(op, ra.m, k0 + i);
  return v;
}
__device__ __forceinline__ f32x4 load_w4(const GemmOp& op, int n, int k0, bool vec) {
  if (n >= op.N) return f32x4{0.f, 0.f, 0.f, 0.f};
  const float* w = op.W + (size_t)n * op.K;
  if (vec && k0 + 3 < op.K) return *reinterpret_cast<const f32x4*>(w + k0);
  f32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = k0 + i < op.K ? w[k0 + i] : 0.f;
  return r;
}

// The K loop of one 64 × 64 tile (rows m0.., columns n0..) into acc (staging in As / Ws).
__device__ __forceinline__ void gemm_acc(const GemmOp& op, int m0, int n0, float (*As)[GKS], float (*Ws)[GKS],
                                         f32x4 (&acc)[4]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool avec = (op.lda & 3) == 0 && ((reinterpret_cast<uintptr_t>(op.A) & 15) == 0);
  const bool wvec = (op.K & 3) == 0 && ((reinterpret_cast<uintptr_t>(op.W) & 15) == 0);
  // this thread's runs: row (tid >> 3) and (tid >> 3) + 32, columns 4·(tid & 7) .. +3 of the chunk
  const int fr = tid >> 3, fc = 4 * (tid & 7);
  const ARow far[2] = {arow(op, m0 + fr), arow(op, m0 + fr + 32)};
  f32x4 ra[2], rw[2];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ra[i] = load_a4(op, far[i], k0 + fc, avec);
      rw[i] = load_w4(op, n0 + fr + 32 * i, k0 + fc, wvec);
    }
  };
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  fetch(0);
  for (int k0 = 0; k0 < op.K; k0 += GK) {
    __syncthreads();   // the previous chunk has been read
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        As[fr + 32 * i][fc + c] = ra[i][c];
        Ws[fr + 32 * i][fc + c] = rw[i][c];
      }
    }
    __syncthreads();
    if (k0 + GK < op.K) fetch(k0 + GK);
#pragma unroll
    for (int kk = 0; kk < GK; kk += 4) {
      const float a = As[16 * w + (lane & 15)][kk + (lane >> 4)];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float b = Ws[16 * j + (lane & 15)][kk + (lane >> 4)];
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
      }
    }
  }
}

// The tile's epilogue (scale, bias, positional rows, activation, residual, row map or fused LayerNorm).
__device__ __forceinline__ void gemm_epi(const GemmOp& op, int m0, int n0, const f32x4 (&acc)[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // epilogue: lane holds rows 4(lane>>4)+r of the wave's 16, column lane&15 of each 16-wide group.
  // Every epilogue operand (scale, bias, positional row, residual) is loaded before the first store:
  // Y may alias R (in-place residual), so a load placed after a store cannot be hoisted above it, and
  // the 16 dependent L2 round trips per lane were most of the kernel's time.
  float pv[4][4], rv[4][4], sc[4], bi[4];
  ARow er[4];   // the lane's four output rows, split once
#pragma unroll
  for (int r = 0; r < 4; ++r) er[r] = arow(op, m0 + 16 * w + 4 * (lane >> 4) + r);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + 16 * j + (lane & 15);
    const bool nv = n < op.N;
    sc[j] = nv && op.scale ? op.scale[n] : 1.f;
    bi[j] = nv && op.bias ? op.bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = er[r].m;
      const bool v = nv && m < op.M;
      pv[j][r] = v && op.pe ? op.pe[(size_t)er[r].t * op.N + n] : 0.f;
      rv[j][r] = v && op.R ? op.R[(size_t)m * op.ldr + n] : 0.f;
    }
  }
  if (op.ln_g) {
    // x + sublayer(x) of whole rows (N ≤ 64: n0 = 0, the tile holds every column), then the LayerNorm
    // the next layer reads (in place: the pre-norm sum is not read again)
    float y[4][4], gg[4], bb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = 16 * j + (lane & 15);
      const bool nv = n < op.N;
      gg[j] = nv ? op.ln_g[n] : 0.f;
      bb[j] = nv ? op.ln_b[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[j][r] * sc[j] + bi[j];
        if (op.pe) v += pv[j][r];
        if (op.act == 1) v = gelu(v);
        else if (op.act == 2) v = fmaxf(v, 0.f);
        else if (op.act == 3) v = v > 0.f ? v : expm1f(v);
        if (op.R) v += rv[j][r];
        y[j][r] = nv ? v : 0.f;
      }
    }
    const float invN = 1.0f / (float)op.N;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s = (y[0][r] + y[1][r]) + (y[2][r] + y[3][r]);
      for (int o = 8; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);   // the 16 lanes of row r
      const float mean = s * invN;
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = 16 * j + (lane & 15) < op.N ? y[j][r] - mean : 0.f;
        q = fmaf(d, d, q);
      }
      for (int o = 8; o >= 1; o >>= 1) q += __shfl_xor(q, o, 64);
      const float inv = 1.0f / sqrtf(q * invN + 1e-5f);
      const int m = er[r].m;
      if (m >= op.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 16 * j + (lane & 15);
        if (n < op.N) op.Y[(size_t)m * op.ldy + n] = (y[j][r] - mean) * inv * gg[j] + bb[j];
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + 16 * j + (lane & 15);
    if (n >= op.N) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = er[r].m;
      if (m >= op.M) continue;
      float y = acc[j][r] * sc[j] + bi[j];
      const int b = er[r].b, t = er[r].t;
      if (op.pe) y += pv[j][r];
      if (op.act == 1) y = gelu(y);
      else if (op.act == 2) y = fmaxf(y, 0.f);
      else if (op.act == 3) y = y > 0.f ? y : expm1f(y);
      if (op.R) y += rv[j][r];
      if (op.row_t0 > 0) {   // keep rows t ≥ t0 of every sequence, written as [b][t − t0]
        if (t < op.row_t0) continue;
        op.Y[((size_t)b * (op.L - op.row_t0) + (t - op.row_t0)) * op.ldy + n] = y;
      } else {
        op.Y[(size_t)m * op.ldy + n] = y;
      }
    }
  }
}

__global__ void __launch_bounds__(256) lw_gemm(GemmOp op) {
  __shared__ float As[GT][GKS];
  __shared__ float Ws[GT][GKS];
  const int m0 = blockIdx.x * GT, n0 = blockIdx.y * GT;
  f32x4 acc[4];
  gemm_acc(op, m0, n0, As, Ws, acc);
  gemm_epi(op, m0, n0, acc);
}

// The FFN pair of one 64-row tile in one launch when d_model, d_ff ≤ 64 (encoder.py:50-53,
// decoder.py:50-53): h = act(x·W1ᵀ + b1) stays in LDS, then y = h·W2ᵀ + b2 + x with the LayerNorm of g2.
constexpr int HS = GT + 2;   // hidden rows: 66 floats (the MFMA reads hit 32 distinct banks)
__global__ void __launch_bounds__(256) lw_ffn(GemmOp g1, GemmOp g2) {
  __shared__ float As[GT][GKS];
  __shared__ float Ws[GT][GKS];
  __shared__ float Hs[GT][HS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * GT;
  f32x4 acc[4];
  gemm_acc(g1, m0, 0, As, Ws, acc);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = 16 * j + (lane & 15);
    const bool nv = n < g1.N;
    const float sc = nv && g1.scale ? g1.scale[n] : 1.f;
    const float bi = nv && g1.bias ? g1.bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float y = acc[j][r] * sc + bi;
      if (g1.act == 1) y = gelu(y);
      else if (g1.act == 2) y = fmaxf(y, 0.f);
      Hs[16 * w + 4 * (lane >> 4) + r][n] = nv ? y : 0.f;
    }
  }
  // second product: A = the hidden rows in LDS, W2 staged in chunks of 32
  const bool wvec = (g2.K & 3) == 0 && ((reinterpret_cast<uintptr_t>(g2.W) & 15) == 0);
  const int fr = tid >> 3, fc = 4 * (tid & 7);
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < g2.K; k0 += GK) {
    f32x4 rw[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) rw[i] = load_w4(g2, fr + 32 * i, k0 + fc, wvec);
    __syncthreads();   // Hs complete (first chunk) / the previous W chunk has been read
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) Ws[fr + 32 * i][fc + c] = rw[i][c];
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK; kk += 4) {
      const float a = k0 + kk + (lane >> 4) < GT ? Hs[16 * w + (lane & 15)][k0 + kk + (lane >> 4)] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Ws[16 * j + (lane & 15)][kk + (lane >> 4)], acc[j], 0, 0, 0);
    }
  }
  gemm_epi(g2, m0, 0, acc);
}

// Short-M variant (batch-1 latency: M = a few sequences' rows): a 16 × 64 tile per workgroup, so the
// ≈100-row GEMMs of one sequence spread over 6× more workgroups; K staged in chunks of 64 with the
// next chunk's global loads in flight during this chunk's MFMAs; two accumulation chains per wave.
constexpr int SM = 16, SK = 64;
__global__ void __launch_bounds__(256) lw_gemm_s(GemmOp op) {
  __shared__ float As[SM][SK + 1];
  __shared__ float Ws[GT][SK + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * SM, n0 = blockIdx.y * GT;
  float ra[SM * SK / 256], rw[GT * SK / 256];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < SM * SK / 256; ++i) {
      const int e = tid + 256 * i, r = e / SK, c = e % SK;
      ra[i] = load_a(op, m0 + r, k0 + c);
    }
#pragma unroll
    for (int i = 0; i < GT * SK / 256; ++i) {
      const int e = tid + 256 * i, r = e / SK, c = e % SK;
      const int n = n0 + r, k = k0 + c;
      rw[i] = n < op.N && k < op.K ? op.W[(size_t)n * op.K + k] : 0.f;
    }
  };
  fetch(0);
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  for (int k0 = 0; k0 < op.K; k0 += SK) {
    __syncthreads();   // the previous chunk has been read
#pragma unroll
    for (int i = 0; i < SM * SK / 256; ++i) {
      const int e = tid + 256 * i;
      As[e / SK][e % SK] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < GT * SK / 256; ++i) {
      const int e = tid + 256 * i;
      Ws[e / SK][e % SK] = rw[i];
    }
    __syncthreads();
    if (k0 + SK < op.K) fetch(k0 + SK);
#pragma unroll
    for (int kk = 0; kk < SK; kk += 8) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(As[lane & 15][kk + (lane >> 4)],
                                                  Ws[16 * w + (lane & 15)][kk + (lane >> 4)], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(As[lane & 15][kk + 4 + (lane >> 4)],
                                                  Ws[16 * w + (lane & 15)][kk + 4 + (lane >> 4)], acc1, 0, 0, 0);
    }
  }
  const f32x4 acc = acc0 + acc1;
  const int n = n0 + 16 * w + (lane & 15);
  if (n >= op.N) return;
  const float sc = op.scale ? op.scale[n] : 1.f;
  const float bi = op.bias ? op.bias[n] : 0.f;
  float pv[4], rv[4];   // loaded before the first store (Y may alias R), as in lw_gemm
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + 4 * (lane >> 4) + r;
    const bool v = m < op.M;
    pv[r] = v && op.pe ? op.pe[(size_t)(m - (m / op.L) * op.L) * op.N + n] : 0.f;
    rv[r] = v && op.R ? op.R[(size_t)m * op.ldr + n] : 0.f;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + 4 * (lane >> 4) + r;
    if (m >= op.M) continue;
    float y = acc[r] * sc + bi;
    const int b = m / op.L, t = m - b * op.L;
    if (op.pe) y += pv[r];
    if (op.act == 1) y = gelu(y);
    else if (op.act == 2) y = fmaxf(y, 0.f);
    else if (op.act == 3) y = y > 0.f ? y : expm1f(y);
    if (op.R) y += rv[r];
    if (op.row_t0 > 0) {
      if (t < op.row_t0) continue;
      op.Y[((size_t)b * (op.L - op.row_t0) + (t - op.row_t0)) * op.ldy + n] = y;
    } else {
      op.Y[(size_t)m * op.ldy + n] = y;
    }
  }
}

// ------------------------------------------------------------------------------- LayerNorm
// One wave per row; Y[out_row(m)] = (X[m] − mean) / sqrt(var + eps) · g + b  (biased variance).
__global__ void __launch_bounds__(256) lw_layernorm(LnOp op) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= op.M) return;
  const float* x = op.X + (size_t)m * op.D;
  float v[LW_DMAX / 64];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LW_DMAX / 64; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < op.D ? x[c] : 0.f;
    s += v[i];
  }
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / (float)op.D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LW_DMAX / 64; ++i) {
    const int c = lane + 64 * i;
    const float d = c < op.D ? v[i] - mean : 0.f;
    q = fmaf(d, d, q);
  }
  for (int o = 32; o >= 1; o >>= 1) q += __shfl_xor(q, o, 64);
  const float inv = 1.0f / sqrtf(q / (float)op.D + 1e-5f);
  const int b = m / op.L, t = m - b * op.L;
  float* y = op.Y + ((size_t)b * op.Lo + op.off + t) * op.D;
#pragma unroll
  for (int i = 0; i < LW_DMAX / 64; ++i) {
    const int c = lane + 64 * i;
    if (c < op.D) y[c] = (v[i] - mean) * inv * op.g[c] + op.b[c];
  }
}

// ---------------------------------------------------------------------- MaxPool / window copy
__global__ void lw_maxpool(const float* __restrict__ X, float* __restrict__ Y, int B, int L, int Lo, int D) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * Lo * D) return;
  const int c = (int)(i % D);
  const int64_t r = i / D;
  const int t = (int)(r % Lo), b = (int)(r / Lo);
  const float* x = X + (size_t)b * L * D + c;
  float v = x[(size_t)(2 * t) * D];
  if (2 * t + 1 < L) v = fmaxf(v, x[(size_t)(2 * t + 1) * D]);
  if (2 * t - 1 >= 0) v = fmaxf(v, x[(size_t)(2 * t - 1) * D]);
  Y[i] = v;
}

__global__ void lw_window(const float* __restrict__ X, float* __restrict__ Y, int B, int L0, int L, int D) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * L * D) return;
  const int c = (int)(i % D);
  const int64_t r = i / D;
  const int t = (int)(r % L), b = (int)(r / L);
  Y[i] = X[((size_t)b * L0 + (L0 - L) + t) * D + c];
}

// ------------------------------------------------------------------------------- attention
// One 256-thread workgroup per (sequence, head).  S = Q_h·K_hᵀ for every (query, key) pair in LDS,
// accumulated over feature chunks of 32 on the f32 MFMA; then per query row: ProbSparse M from the
// sampled pairs (attn.py:89-105, sum divided by L_K), exact top-u by rank (ties to the lower index),
// the initial context (mean(V) or cumsum(V) if masked, :116-125), and softmax(scale·S)·V for the
// selected (or all) rows with the causal mask (:127-146, ProbMask :23-34 / TriangularCausalMask
// :10-20).  scale = 1/sqrt(d_k) (attn.py:81,163).
constexpr int AC = 32;   // feature chunk
__global__ void __launch_bounds__(256) lw_attention(AttnOp op) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int LQ = op.LQ, LK = op.LK, E = op.E;
  const int LQp = (LQ + 15) & ~15, LKp = (LK + 15) & ~15;
  float* S = sm;                                   // [LQp][LKp + 1]
  const int SS = LKp + 1;
  float* Qc = S + LQp * SS;                        // [LQp][AC + 1]
  float* Kc = Qc + LQp * (AC + 1);                 // [LKp][AC + 1]
  float* Mv = Kc + LKp * (AC + 1);                 // [LQp] sparsity measure
  int* sel = reinterpret_cast<int*>(Mv + LQp);     // [LQp] selected query of rank r
  int* flag = sel + LQp;                           // [LQp] row selected
  const int b = blockIdx.x / op.H, h = blockIdx.x - (blockIdx.x / op.H) * op.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* Qg = op.Q + (size_t)b * LQ * op.ldq + (size_t)h * E;
  const float* Kg = op.K + (size_t)b * LK * op.ldk + (size_t)h * E;
  const float* Vg = op.V + (size_t)b * LK * op.ldv + (size_t)h * E;
  const int nqt = LQp / 16, nkt = LKp / 16;

  // ---- S = Q·Kᵀ, tile (qt, kt) owned by wave (qt·nkt + kt) mod 4, accumulated in LDS across chunks
  for (int i = tid; i < LQp * SS; i += 256) S[i] = 0.f;
  for (int e0 = 0; e0 < E; e0 += AC) {
    const int ec = ((E - e0 < AC ? E - e0 : AC) + 3) & ~3;   // features of this chunk, padded to 4
    __syncthreads();
    for (int i = tid; i < LQp * AC; i += 256) {
      const int r = i / AC, c = i - r * AC;
      Qc[r * (AC + 1) + c] = r < LQ && e0 + c < E ? Qg[(size_t)r * op.ldq + e0 + c] : 0.f;
    }
    for (int i = tid; i < LKp * AC; i += 256) {
      const int r = i / AC, c = i - r * AC;
      Kc[r * (AC + 1) + c] = r < LK && e0 + c < E ? Kg[(size_t)r * op.ldk + e0 + c] : 0.f;
    }
    __syncthreads();
    for (int t = w; t < nqt * nkt; t += 4) {
      const int qt = t / nkt, kt = t - qt * nkt;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int kk = 0; kk < ec; kk += 4) {
        const float a = Qc[(16 * qt + (lane & 15)) * (AC + 1) + kk + (lane >> 4)];
        const float bb = Kc[(16 * kt + (lane & 15)) * (AC + 1) + kk + (lane >> 4)];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bb, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) S[(16 * qt + 4 * (lane >> 4) + r) * SS + 16 * kt + (lane & 15)] += acc[r];
    }
  }
  __syncthreads();

  const bool sparse = op.prob && op.u < LQ;
  // ---- ProbSparse: M per query from its sampled keys, then the top-u by rank
  if (sparse) {
    for (int q = tid; q < LQ; q += 256) {
      const int32_t* ix = op.idx + (size_t)q * op.U;
      float mx = -INFINITY, sum = 0.f;
      for (int j = 0; j < op.U; ++j) {
        const float s = S[q * SS + ix[j]];
        mx = fmaxf(mx, s);
        sum += s;
      }
      Mv[q] = mx - sum / (float)LK;
    }
    __syncthreads();
    for (int q = tid; q < LQ; q += 256) {
      const float m = Mv[q];
      int rank = 0;
      for (int j = 0; j < LQ; ++j) {
        const float o = Mv[j];
        rank += (o > m) || (o == m && j < q);
      }
      flag[q] = rank < op.u;
      if (rank < op.u) sel[rank] = q;
    }
    __syncthreads();
  }
  const int nsel = sparse ? op.u : LQ;
  const float scale = 1.0f / sqrtf((float)E);

  // output placement: (query i, head h, feature e) → ctx; mix re-views (L, H, E) as (H, L, E)
  auto ctx_ptr = [&](int i) -> float* {
    if (!op.mix) return op.O + ((size_t)b * LQ + i) * op.ldo + (size_t)h * E;
    return op.O + (size_t)b * LQ * op.ldo + (size_t)h * LQ * E + (size_t)i * E;
  };

  // ---- softmax rows of the selected queries (P written over S in place): RL lanes per row, so a wave
  //      takes 64 / RL rows at once (short rows: 16 lanes, 4 rows per wave pass)
  const int RL = LK <= 32 ? 16 : 64, RPW = 64 / RL;
  const int sub = lane / RL, ll = lane - sub * RL;
  for (int r0 = w * RPW; r0 < nsel; r0 += 4 * RPW) {
    const int r = r0 + sub;
    const bool active = r < nsel;
    const int q = active ? (sparse ? sel[r] : r) : 0;
    float* Srow = S + q * SS;
    const int kmax = !active ? 0 : (op.causal ? q + 1 : LK);   // keys j > q masked
    float mx = -INFINITY;
    for (int j = ll; j < kmax; j += RL) mx = fmaxf(mx, Srow[j] * scale);
    for (int o = RL / 2; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float sum = 0.f;
    const int kend = active ? LK : 0;
    for (int j = ll; j < kend; j += RL) {
      const float p = j < kmax ? expf(Srow[j] * scale - mx) : 0.f;
      Srow[j] = p;
      sum += p;
    }
    for (int o = RL / 2; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
    const float inv = 1.0f / sum;
    for (int j = ll; j < kend; j += RL) Srow[j] *= inv;
    if (op.attns && active) {
      float* A = op.attns + (size_t)b * op.attn_bstride + ((size_t)h * LQ + q) * LK;
      for (int j = ll; j < LK; j += RL) A[j] = Srow[j];
    }
  }
  if (sparse && op.attns) {
    float* A = op.attns + (size_t)b * op.attn_bstride + (size_t)h * LQ * LK;
    for (int i = tid; i < LQ * LK; i += 256)
      if (!flag[i / LK]) A[i] = 1.0f / (float)LK;
  }
  // ---- per 32-feature chunk of V (staged in LDS): the initial context of the unselected rows, and
  //      O = P·V for the selected rows on the f32 MFMA (16 selected rows × 16 features per tile)
  const int nrt = (nsel + 15) / 16;
  for (int e0 = 0; e0 < E; e0 += AC) {
    const int nct = ((E - e0 < AC ? E - e0 : AC) + 15) / 16;   // 16-feature output tiles of this chunk
    __syncthreads();   // P complete (first chunk) / the previous chunk's V no longer read
    for (int i = tid; i < LKp * AC; i += 256) {
      const int r = i / AC, c = i - r * AC;
      Kc[r * (AC + 1) + c] = r < LK && e0 + c < E ? Vg[(size_t)r * op.ldv + e0 + c] : 0.f;
    }
    __syncthreads();
    if (sparse && tid < AC && e0 + tid < E) {
      const int c = tid, e = e0 + tid;
      if (!op.causal) {   // mean over keys (attn.py:116-119)
        float sv = 0.f;
        for (int j = 0; j < LK; ++j) sv += Kc[j * (AC + 1) + c];
        const float mean = sv / (float)LK;
        for (int q = 0; q < LQ; ++q)
          if (!flag[q]) ctx_ptr(q)[e] = mean;
      } else {            // cumsum over keys (attn.py:120-125)
        float sv = 0.f;
        for (int q = 0; q < LQ; ++q) {
          sv += Kc[q * (AC + 1) + c];
          if (!flag[q]) ctx_ptr(q)[e] = sv;
        }
      }
    }
    for (int t = w; t < nrt * nct; t += 4) {
      const int rt = t / nct, et = t - rt * nct;
      const int rs = 16 * rt + (lane & 15);
      const int qa = sparse ? sel[rs < nsel ? rs : nsel - 1] : (rs < nsel ? rs : nsel - 1);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k0 = 0; k0 < LKp; k0 += 4) {
        const float a = S[qa * SS + k0 + (lane >> 4)];
        const float bb = Kc[(k0 + (lane >> 4)) * (AC + 1) + 16 * et + (lane & 15)];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bb, acc, 0, 0, 0);
      }
      const int e = e0 + 16 * et + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 16 * rt + 4 * (lane >> 4) + r;
        if (rr < nsel && e < E) ctx_ptr(sparse ? sel[rr] : rr)[e] = acc[r];
      }
    }
  }
}

size_t attn_lds_bytes(int LQ, int LK) {
  const int LQp = (LQ + 15) & ~15, LKp = (LK + 15) & ~15;
  return sizeof(float) * ((size_t)LQp * (LKp + 1) + (size_t)LQp * (AC + 1) + (size_t)LKp * (AC + 1) + LQp) +
         sizeof(int) * 2 * (size_t)LQp;
}

// ---------------------------------------------------------------------------------- launchers
int launch_gemm(const GemmOp& op, hipStream_t st) {
  if (op.M <= 0 || op.N <= 0) return 0;
  if (op.ln_g && (op.N > GT || op.row_t0 > 0)) return -3;
  if (op.M <= 1024 && !op.ln_g) {   // few rows (batch-1 latency): more, shorter workgroups
    hipLaunchKernelGGL(lw_gemm_s, dim3((op.M + SM - 1) / SM, (op.N + GT - 1) / GT), dim3(256), 0, st, op);
  } else {
    hipLaunchKernelGGL(lw_gemm, dim3((op.M + GT - 1) / GT, (op.N + GT - 1) / GT), dim3(256), 0, st, op);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int launch_ffn(const GemmOp& g1, const GemmOp& g2, hipStream_t st) {
  if (g1.N > GT || g2.N > GT || g2.K > GT || g1.M != g2.M || g1.amode || g2.row_t0 || g1.R || g1.pe)
    return -3;
  hipLaunchKernelGGL(lw_ffn, dim3((g1.M + GT - 1) / GT), dim3(256), 0, st, g1, g2);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int launch_layernorm(const LnOp& op, hipStream_t st) {
  if (op.D > LW_DMAX) return -3;
  hipLaunchKernelGGL(lw_layernorm, dim3((op.M + 3) / 4), dim3(256), 0, st, op);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int launch_maxpool(const float* X, float* Y, int B, int L, int Lo, int D, hipStream_t st) {
  const int64_t n = (int64_t)B * Lo * D;
  hipLaunchKernelGGL(lw_maxpool, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, X, Y, B, L, Lo, D);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int launch_window(const float* X, float* Y, int B, int L0, int L, int D, hipStream_t st) {
  const int64_t n = (int64_t)B * L * D;
  hipLaunchKernelGGL(lw_window, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, X, Y, B, L0, L, D);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int prepare_attention() {
  // once per (device, kernel), thread-safe (cet_api.cpp)
  return cet::ensure_lds_attr(reinterpret_cast<const void*>(lw_attention)) ? 0 : -1;
}
int launch_attention(const AttnOp& op, int B, hipStream_t st) {
  if (op.LQ > LW_LMAX || op.LK > LW_LMAX) return -3;
  if (prepare_attention()) return -1;
  hipLaunchKernelGGL(lw_attention, dim3(B * op.H), dim3(256), attn_lds_bytes(op.LQ, op.LK), st, op);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace lw
}  // namespace cet
