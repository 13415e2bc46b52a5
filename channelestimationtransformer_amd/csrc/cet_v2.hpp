// "v2" building blocks: 4-wave workgroups, residual stream and per-head Q/K/V in registers.
//
// Register-resident residual stream (Resid):
//   wave w owns output features [32w, 32w+32) = n-tiles 2w, 2w+1 of every residual-producing
//   dense layer; for m-tile mt its lane l holds X[16·mt + (l&15)][16·(2w+t) + 4·(l>>4) + r]
//   in v[t][mt][r] — exactly the C fragment of the transposed dense layer Yᵀ = W·Xᵀ on
//   v_mfma_f32_16x16x32_bf16, so epilogues add straight into it.
// LDS holds only the bf16 image Xb of the current activation (B operand of the next dense
// layer), the attention context / FFN hidden, the encoder-stack output and small scratch.
//
// Per-head attention in registers (attention_head2):
//   Kᵀ tile   = Wk_h · Xᵀ  → C[e][key]  = A fragment of Sᵀ = K·Qᵀ  (16x16x16)
//   Qᵀ tile   = Wq_h · Xᵀ  → C[e][q]    = B fragment of Sᵀ
//   V  tile   = X · Wv_hᵀ  → C[key][e]  = A fragment of Oᵀ = Vᵀ·Pᵀ
//   exp(Sᵀ)   tile          → B fragment of Oᵀ (query on the lane axis)
// so no Q/K/V tensor ever goes through LDS.
#pragma once
#include "cet_attention.hpp"

namespace cet {
namespace v2 {

constexpr int NW = 4;
constexpr int NTHREADS = NW * WAVE;
constexpr int MT = 6;  // max 16-row tiles (96 positions)

template <int N>
struct ResidT {
  f32x4 v[2][N];
};
using Resid = ResidT<MT>;

__device__ __forceinline__ f32x4 load4(const float* __restrict__ p) { return *reinterpret_cast<const f32x4*>(p); }

__device__ __forceinline__ f32x4 affine4(const float* __restrict__ P, const GemmDesc d, int n0, f32x4 acc) {
  if (d.scale != NONE) acc *= load4(P + d.scale + n0);
  if (d.bias != NONE) acc += load4(P + d.bias + n0);
  return acc;
}
__device__ __forceinline__ float affine1(const float* __restrict__ P, const GemmDesc d, int n, float acc) {
  if (d.scale != NONE) acc *= P[d.scale + n];
  if (d.bias != NONE) acc += P[d.bias + n];
  return acc;
}

template <int KS>
__device__ __forceinline__ void load_frags(const bf16x8* __restrict__ W, int nt, bf16x8 (&a)[KS]) {
  const int lane = lane_id();
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) a[ks] = W[((size_t)(nt * KS + ks)) * WAVE + lane];
}

// Dense layer whose output n-tiles 2w, 2w+1 land in the wave's residual fragments.  The
// epilogue vectors (LSQ/BN scale, bias) are loaded once, before the m-tile loop, and applied
// here; epi(t, mt, n0, f32x4 y) receives the finished value.
template <int KS, class BL, class Epi>
__device__ __forceinline__ void gemm_wave2(const bf16x8* __restrict__ W, const float* __restrict__ P, const GemmDesc d,
                                           int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_id(), w = wave_id();
  bf16x8 a0[KS], a1[KS];
  load_frags<KS>(W + d.w, 2 * w, a0);
  load_frags<KS>(W + d.w, 2 * w + 1, a1);
  const int n0 = 32 * w + (lane >> 4) * 4, n1 = n0 + 16;
  f32x4 s0 = {1.f, 1.f, 1.f, 1.f}, s1 = s0, b0 = {0.f, 0.f, 0.f, 0.f}, b1 = b0;
  if (d.scale != NONE) { s0 = load4(P + d.scale + n0); s1 = load4(P + d.scale + n1); }
  if (d.bias != NONE) { b0 = load4(P + d.bias + n0); b1 = load4(P + d.bias + n1); }
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    if (mt < nmt) {
      f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 b = bl(mt * 16 + mrow, ks * 32 + kq);
        c0 = mfma16x16x32(a0[ks], b, c0);
        c1 = mfma16x16x32(a1[ks], b, c1);
      }
      epi(0, mt, n0, c0 * s0 + b0);
      epi(1, mt, n1, c1 * s1 + b1);
    }
  }
}

// Same, one of the two n-tiles at a time (halves the fragment registers for deep K).
template <int KS, class BL, class Epi>
__device__ __forceinline__ void gemm_wave2_split(const bf16x8* __restrict__ W, const float* __restrict__ P,
                                                 const GemmDesc d, int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_id(), w = wave_id();
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    bf16x8 a[KS];
    load_frags<KS>(W + d.w, 2 * w + t, a);
    const int n0 = 32 * w + 16 * t + (lane >> 4) * 4;
    f32x4 sc = {1.f, 1.f, 1.f, 1.f}, bi = {0.f, 0.f, 0.f, 0.f};
    if (d.scale != NONE) sc = load4(P + d.scale + n0);
    if (d.bias != NONE) bi = load4(P + d.bias + n0);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      if (mt < nmt) {
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) c = mfma16x16x32(a[ks], bl(mt * 16 + mrow, ks * 32 + kq), c);
        epi(t, mt, n0, c * sc + bi);
      }
    }
  }
}

template <int KS, int NMT, int T, class BL, class Epi>
__device__ __forceinline__ void gemm_kouter_tile(const bf16x8* __restrict__ W, const float* __restrict__ P,
                                                 const GemmDesc d, BL&& bl, Epi&& epi) {
  const int lane = lane_id(), w = wave_id();
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
  bf16x8 a[KS];
  load_frags<KS>(W + d.w, 2 * w + T, a);
  const int n0 = 32 * w + 16 * T + (lane >> 4) * 4;
  f32x4 sc = {1.f, 1.f, 1.f, 1.f}, bi = {0.f, 0.f, 0.f, 0.f};
  if (d.scale != NONE) sc = load4(P + d.scale + n0);
  if (d.bias != NONE) bi = load4(P + d.bias + n0);
  f32x4 c[NMT];
  bf16x8 b[NMT];
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    c[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    b[mt] = bl(mt * 16 + mrow, kq);
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8 bn[NMT];
    if (ks + 1 < KS) {
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt) bn[mt] = bl(mt * 16 + mrow, (ks + 1) * 32 + kq);
    }
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) c[mt] = mfma16x16x32(a[ks], b[mt], c[mt]);
    if (ks + 1 < KS) {
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt) b[mt] = bn[mt];
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the prefetch distance at one k-step
  }
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) epi(T, mt, n0, c[mt] * sc + bi);
}

// Deep-K dense layer (the distil conv, K = 384) in k-outer order with a compile-time m-tile count:
// one accumulator per m-tile, and the B fragments of every m-tile for step ks+1 are requested
// before step ks's MFMAs, so LDS latency overlaps the matrix work instead of preceding each MFMA.
// The n-tile index is a template parameter too, so every residual index the epilogue touches is
// static (a runtime index would demote the residual to scratch).
template <int KS, int NMT, class BL, class Epi>
__device__ __forceinline__ void gemm_wave2_kouter(const bf16x8* __restrict__ W, const float* __restrict__ P,
                                                  const GemmDesc d, BL&& bl, Epi&& epi) {
  gemm_kouter_tile<KS, NMT, 0>(W, P, d, bl, epi);
  gemm_kouter_tile<KS, NMT, 1>(W, P, d, bl, epi);
}

// Calls f(std::integral_constant<int, n>) for the runtime m-tile count n in [1, MT].
template <class F>
__device__ __forceinline__ void with_nmt(int n, F&& f) {
  switch (n) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: f(std::integral_constant<int, 5>{}); break;
    default: f(std::integral_constant<int, 6>{}); break;
  }
}

// Compile-time m-tile-count forms of gemm_wave2 / gemm_tiles (the decoder runs on 1..3 tiles): no
// per-tile branches, and the B fragments of tile mt+1 are requested before the MFMAs of tile mt.
template <int KS, int NMT, class BL, class Epi>
__device__ __forceinline__ void gemm_wave2_n(const bf16x8* __restrict__ W, const float* __restrict__ P, const GemmDesc d,
                                             BL&& bl, Epi&& epi) {
  const int lane = lane_id(), w = wave_id();
  bf16x8 a0[KS], a1[KS];
  load_frags<KS>(W + d.w, 2 * w, a0);
  load_frags<KS>(W + d.w, 2 * w + 1, a1);
  const int n0 = 32 * w + (lane >> 4) * 4, n1 = n0 + 16;
  f32x4 s0 = {1.f, 1.f, 1.f, 1.f}, s1 = s0, b0 = {0.f, 0.f, 0.f, 0.f}, b1 = b0;
  if (d.scale != NONE) { s0 = load4(P + d.scale + n0); s1 = load4(P + d.scale + n1); }
  if (d.bias != NONE) { b0 = load4(P + d.bias + n0); b1 = load4(P + d.bias + n1); }
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
  bf16x8 b[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) b[ks] = bl(mrow, ks * 32 + kq);
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    bf16x8 bn[KS];
    if (mt + 1 < NMT) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) bn[ks] = bl((mt + 1) * 16 + mrow, ks * 32 + kq);
    }
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      c0 = mfma16x16x32(a0[ks], b[ks], c0);
      c1 = mfma16x16x32(a1[ks], b[ks], c1);
    }
    epi(0, mt, n0, c0 * s0 + b0);
    epi(1, mt, n1, c1 * s1 + b1);
    if (mt + 1 < NMT) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) b[ks] = bn[ks];
    }
  }
}

template <int KS, int NMT, class BL, class Epi>
__device__ __forceinline__ void gemm_tiles_n(const bf16x8* __restrict__ W, const float* __restrict__ P,
                                             const GemmDesc d, int n_tiles, BL&& bl, Epi&& epi) {
  const int lane = lane_id(), w = wave_id();
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
  for (int nt = w; nt < n_tiles; nt += NW) {
    bf16x8 a[KS];
    load_frags<KS>(W + d.w, nt, a);
    const int n0 = nt * 16 + (lane >> 4) * 4;
    f32x4 sc = {1.f, 1.f, 1.f, 1.f}, bi = {0.f, 0.f, 0.f, 0.f};
    if (d.scale != NONE) sc = load4(P + d.scale + n0);
    if (d.bias != NONE) bi = load4(P + d.bias + n0);
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) {
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) c = mfma16x16x32(a[ks], bl(mt * 16 + mrow, ks * 32 + kq), c);
      epi(mt, n0, c * sc + bi);
    }
  }
}

// Dense layer over an arbitrary set of n-tiles (nt = w, w + NW, ...) — FFN hidden, projection.
template <int KS, class BL, class Epi>
__device__ __forceinline__ void gemm_tiles(const bf16x8* __restrict__ W, const float* __restrict__ P, const GemmDesc d,
                                           int n_tiles, int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_id(), w = wave_id();
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
  for (int nt = w; nt < n_tiles; nt += NW) {
    bf16x8 a[KS];
    load_frags<KS>(W + d.w, nt, a);
    const int n0 = nt * 16 + (lane >> 4) * 4;
    f32x4 sc = {1.f, 1.f, 1.f, 1.f}, bi = {0.f, 0.f, 0.f, 0.f};
    if (d.scale != NONE) sc = load4(P + d.scale + n0);
    if (d.bias != NONE) bi = load4(P + d.bias + n0);
    for (int mt = 0; mt < nmt; ++mt) {
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) c = mfma16x16x32(a[ks], bl(mt * 16 + mrow, ks * 32 + kq), c);
      epi(mt, n0, c * sc + bi);
    }
  }
}

// LayerNorm of the register residual over all 128 features (4 waves × 32).  Each wave reduces
// its 32 features per row to (mean_w, M2_w), the pairs meet in LDS, and Chan's combination
// gives the exact row mean / variance.  Writes the normalised rows to X (registers) and the
// bf16 image rows < `rows` to Xb (and optionally a second bf16 copy, e.g. the encoder output).
// torch.nn.LayerNorm (biased var, eps in the sqrt) or, if unbiased_std, the reference
// Transformer's LayerNormalization (alpha·(x-mean)/(std_unbiased+eps)+bias).
// Contains one workgroup barrier; the caller adds one before Xb is read.
template <int N>
__device__ __forceinline__ void ln_resid(ResidT<N>& X, int nmt, int rows, const float* __restrict__ gamma,
                                         const float* __restrict__ beta, float eps, bool unbiased_std, float* part,
                                         __bf16* Xb, __bf16* Xb2 = nullptr) {
  const int lane = lane_id(), w = wave_id(), g = lane >> 4, c = lane & 15;
  const int nb = 32 * w + 4 * g;
  const f32x4 g0 = load4(gamma + nb), g1 = load4(gamma + nb + 16);   // issued before the barrier
  const f32x4 b0 = load4(beta + nb), b1 = load4(beta + nb + 16);
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t) s += (X.v[t][mt][0] + X.v[t][mt][1]) + (X.v[t][mt][2] + X.v[t][mt][3]);
      s = xor_sum(s, 16);
      s = xor_sum(s, 32);
      const float mw = s * (1.0f / 32.0f);
      float q = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = X.v[t][mt][r] - mw;
          q = fmaf(d, d, q);
        }
      q = xor_sum(q, 16);
      q = xor_sum(q, 32);
      if (g == 0) *reinterpret_cast<f32x2*>(part + (mt * 16 + c) * 8 + 2 * w) = f32x2{mw, q};
    }
  }
  __syncthreads();
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      const int m = mt * 16 + c;
      const f32x4 p0 = load4(part + m * 8), p1 = load4(part + m * 8 + 4);
      const float mean = 0.25f * ((p0[0] + p0[2]) + (p1[0] + p1[2]));
      const float d0 = p0[0] - mean, d1 = p0[2] - mean, d2 = p1[0] - mean, d3 = p1[2] - mean;
      const float M2 = (p0[1] + p0[3]) + (p1[1] + p1[3]) + 32.0f * (d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
      // v_rsq_f32 / v_rcp_f32 (1 ulp) instead of the IEEE division expansion
      const float inv = unbiased_std ? __builtin_amdgcn_rcpf(sqrtf(M2 * (1.0f / 127.0f)) + eps)
                                     : __builtin_amdgcn_rsqf(M2 * (1.0f / 128.0f) + eps);
      X.v[0][mt] = (X.v[0][mt] - mean) * inv * g0 + b0;
      X.v[1][mt] = (X.v[1][mt] - mean) * inv * g1 + b1;
      if (m < rows) {
        const bf16x4 y0 = cvt4(X.v[0][mt]), y1 = cvt4(X.v[1][mt]);
        *reinterpret_cast<bf16x4*>(Xb + m * BS + nb) = y0;
        *reinterpret_cast<bf16x4*>(Xb + m * BS + nb + 16) = y1;
        if (Xb2) {
          *reinterpret_cast<bf16x4*>(Xb2 + m * BS + nb) = y0;
          *reinterpret_cast<bf16x4*>(Xb2 + m * BS + nb + 16) = y1;
        }
      }
    }
  }
}

// bf16 image of the register residual (rows < rows).
template <int N>
__device__ __forceinline__ void store_xb(const ResidT<N>& X, int nmt, int rows, __bf16* Xb) {
  const int lane = lane_id(), w = wave_id();
  const int nb = 32 * w + 4 * (lane >> 4);
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      const int m = mt * 16 + (lane & 15);
      if (m < rows) {
        *reinterpret_cast<bf16x4*>(Xb + m * BS + nb) = cvt4(X.v[0][mt]);
        *reinterpret_cast<bf16x4*>(Xb + m * BS + nb + 16) = cvt4(X.v[1][mt]);
      }
    }
  }
}

// fp32 dump of the register residual rows < rows into dst[rows][128] (debug only).
template <int N>
__device__ __forceinline__ void dump_resid(const ResidT<N>& X, int nmt, int rows, float* dst) {
  const int lane = lane_id(), w = wave_id();
  const int nb = 32 * w + 4 * (lane >> 4);
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      const int m = mt * 16 + (lane & 15);
      if (m < rows) {
        *reinterpret_cast<f32x4*>(dst + m * DMODEL + nb) = X.v[0][mt];
        *reinterpret_cast<f32x4*>(dst + m * DMODEL + nb + 16) = X.v[1][mt];
      }
    }
  }
}

// MaxPool1d(kernel 3, stride 2, padding 1) over positions of a register-resident tile set:
// out row t' = max(x[2t'-1], x[2t'], x[2t'+1]) over rows in [0, L).  Rows live on the 16-lane
// axis, so the 2:1 gather is a within-row ds_bpermute from tiles 2j-1, 2j, 2j+1.
__device__ __forceinline__ void maxpool_resid(const Resid& in, int L, Resid& out) {
  const int lane = lane_id();
  const int c = lane & 15, base = lane & 48;
  const int s0 = base | ((2 * c) & 15), s1 = base | ((2 * c + 1) & 15), sm = base | ((2 * c - 1) & 15);
#pragma unroll
  for (int j = 0; j < MT / 2; ++j) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a0 = __shfl(in.v[t][2 * j][r], s0, 64);
        const float b0 = __shfl(in.v[t][2 * j + 1][r], s0, 64);
        const float a1 = __shfl(in.v[t][2 * j][r], s1, 64);
        const float b1 = __shfl(in.v[t][2 * j + 1][r], s1, 64);
        const float a2 = __shfl(in.v[t][2 * j][r], sm, 64);
        const float b2 = __shfl(in.v[t][2 * j + 1][r], sm, 64);
        const float c2 = j > 0 ? __shfl(in.v[t][(2 * j - 1 < 0) ? 0 : 2 * j - 1][r], sm, 64) : NEG_INF;
        const int row0 = 32 * j + 2 * c;
        float v = c < 8 ? a0 : b0;                          // row 2t'   (always < L for t' < L_out)
        const float v1 = c < 8 ? a1 : b1;                   // row 2t'+1
        const float vm = c == 0 ? c2 : (c <= 8 ? a2 : b2);  // row 2t'-1
        if (row0 + 1 < L) v = fmaxf(v, v1);
        if (row0 - 1 >= 0) v = fmaxf(v, vm);
        out.v[t][j][r] = v;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = MT / 2; j < MT; ++j) out.v[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// ------------------------------------------------------------------------------ attention
struct HeadIO {
  const __bf16* Xq;           // LDS rows feeding the queries (bf16, stride BS)
  const __bf16* Xkv;          // LDS rows feeding keys / values
  const bf16x8* Wq;           // packed fragments, n-tile 0 of the query projection
  const bf16x8* Wk;
  const bf16x8* Wv;
  GemmDesc dq, dk, dv;        // epilogue vectors (bias/scale offsets already at the part's start)
  __bf16* ctx;                // LDS [LQ][BS]
  int LQ, LK, prob, causal, mix, u;
  const uint8_t* cnt;
  int cnt_stride;
  float* scr;                 // per-wave scratch: keys [96] u64, sel [96] int16, flag [96] bytes
  float* attn_out;            // global [H][LQ][LK] of this sequence or nullptr
  float* m_dbg;               // global [H][LQ] or nullptr
  unsigned long long* st;     // diagnostics: sub-phase s_memtime stamps of head 0, or nullptr
};

template <int MQ = MT, int MK = MT>
__device__ __forceinline__ void attention_head2(const HeadIO& io, const float* __restrict__ P, int h) {
  const int lane = lane_id();
  const int col = lane & 15, g = lane >> 4;
  const int LQ = io.LQ, LK = io.LK;
  const int nkt = (LK + 15) >> 4, nqt = (LQ + 15) >> 4;
  const bool sparse = io.prob && io.u < LQ;
  uint64_t* keys = reinterpret_cast<uint64_t*>(io.scr);
  int16_t* sel = reinterpret_cast<int16_t*>(io.scr + 192);
  uint8_t* flag = reinterpret_cast<uint8_t*>(io.scr + 240);
  auto SUB = [&](int k) {
    if (io.st && h == 0 && lane == 0) io.st[k] = __builtin_amdgcn_s_memtime();
  };
  SUB(0);

  // epilogue vectors: q/k features 16h + 4g + r (C rows), v feature 16h + col (C column)
  const int fq = 16 * h + 4 * g;
  const int kq = g * 8;
  bf16x4 Kf[MK], Vf[MK], Qf[MQ];
  {
    // pass 1: K and V tiles from the key/value rows (only wk, wv live)
    bf16x8 wk[4], wv[4];
    load_frags<4>(io.Wk, h, wk);
    load_frags<4>(io.Wv, h, wv);
    f32x4 sk = {1.f, 1.f, 1.f, 1.f}, bk = {0.f, 0.f, 0.f, 0.f};
    if (io.dk.scale != NONE) sk = load4(P + io.dk.scale + fq);
    if (io.dk.bias != NONE) bk = load4(P + io.dk.bias + fq);
    const float sv = io.dv.scale != NONE ? P[io.dv.scale + 16 * h + col] : 1.f;
    const float bv = io.dv.bias != NONE ? P[io.dv.bias + 16 * h + col] : 0.f;
#pragma unroll
    for (int mt = 0; mt < MK; ++mt) {
      Kf[mt] = bf16x4{};
      Vf[mt] = bf16x4{};
      if (mt < nkt) {
        f32x4 k = {0.f, 0.f, 0.f, 0.f}, v = k;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const bf16x8 bx = *reinterpret_cast<const bf16x8*>(io.Xkv + (mt * 16 + col) * BS + ks * 32 + kq);
          k = mfma16x16x32(wk[ks], bx, k);
          v = mfma16x16x32(bx, wv[ks], v);
        }
        Kf[mt] = cvt4(k * sk + bk);
        Vf[mt] = cvt4(v * sv + bv);
      }
    }
  }
  SUB(1);
  // pass 2: Q tiles (wq stays live: selected queries are re-projected in phase C)
  bf16x8 wq[4];
  load_frags<4>(io.Wq, h, wq);
  f32x4 sq = {1.f, 1.f, 1.f, 1.f}, bq = {0.f, 0.f, 0.f, 0.f};
  if (io.dq.scale != NONE) sq = load4(P + io.dq.scale + fq);
  if (io.dq.bias != NONE) bq = load4(P + io.dq.bias + fq);
#pragma unroll
  for (int mt = 0; mt < MQ; ++mt) {
    Qf[mt] = bf16x4{};
    if (mt < nqt) {
      f32x4 q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        q = mfma16x16x32(wq[ks], *reinterpret_cast<const bf16x8*>(io.Xq + (mt * 16 + col) * BS + ks * 32 + kq), q);
      Qf[mt] = cvt4(q * sq + bq);
    }
  }

  SUB(2);
  if (sparse) {
    // ---- sparsity measurement M (attn.py:95-105) from key multiplicities (LDS-staged table)
    const float invLK = 1.0f / (float)LK;
#pragma unroll 1
    for (int qt = 0; qt < nqt; ++qt) {
      bf16x4 qf = Qf[0];
#pragma unroll
      for (int t = 1; t < MQ; ++t) qf = qt == t ? Qf[t] : qf;
      {
        const int q = qt * 16 + col;
        // this lane's six count words (keys 16kt + 4g + r, kt = 0..5) are contiguous: cnt_pos()
        const uint2* crow = reinterpret_cast<const uint2*>(io.cnt + (size_t)q * io.cnt_stride + g * 24);
        const uint2 c01 = crow[0], c23 = crow[1], c45 = crow[2];
        const uint32_t cws[MT] = {c01.x, c01.y, c23.x, c23.y, c45.x, c45.y};
        float sum = 0.f, mx = NEG_INF;
#pragma unroll
        for (int kt = 0; kt < MK; ++kt) {
          if (kt < nkt) {
            const f32x4 s = mfma16x16x16(Kf[kt], qf, f32x4{0.f, 0.f, 0.f, 0.f});
            const uint32_t cw = cws[kt];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              // rows past L are stale-but-finite bf16 images in v2, so 0·s is exact zero
              const float cf = (float)((cw >> (8 * r)) & 0xffu);
              sum = fmaf(cf, s[r], sum);
              mx = fmaxf(mx, cf != 0.f ? s[r] : NEG_INF);
            }
          }
        }
        sum = xor_sum(sum, 16);
        sum = xor_sum(sum, 32);
        mx = xor_max(mx, 16);
        mx = xor_max(mx, 32);
        const float M = mx - sum * invLK;
        // selection key: order-preserving image of M above, ~q below — a total order in which
        // equal M go to the lower index (torch leaves topk's tie order unspecified); 0 = padding
        const uint32_t mu = __float_as_uint(M);
        const uint32_t hi = (mu & 0x80000000u) ? ~mu : (mu | 0x80000000u);
        const uint64_t key = q < LQ ? ((uint64_t)hi << 32) | (uint32_t)(0xffff - q) : 0ull;
        if (g == 0) {
          keys[q] = key;
          if (io.m_dbg && q < LQ) io.m_dbg[h * LQ + q] = M;
        }
      }
    }
    wave_lds_sync();
    SUB(3);
    // ---- exact top-u by rank: rank(q) = #{j : key_j > key_q}; q is selected iff rank < u and
    //      lands in sel[rank].  Lane group g counts over keys [g·J, g·J + J), J = 4·nqt.
    uint64_t myk[MQ];
    int rank[MQ];
#pragma unroll
    for (int qt = 0; qt < MQ; ++qt) {
      myk[qt] = qt < nqt ? keys[qt * 16 + col] : ~0ull;
      rank[qt] = 0;
    }
    const int J = 4 * nqt;
    const uint64_t* kg = keys + g * J;
#pragma unroll 2
    for (int j = 0; j < J; j += 2) {
      const u64x2 kk = *reinterpret_cast<const u64x2*>(kg + j);
#pragma unroll
      for (int qt = 0; qt < MQ; ++qt) rank[qt] += (int)(kk[0] > myk[qt]) + (int)(kk[1] > myk[qt]);
    }
    const int uu = io.u;
#pragma unroll
    for (int qt = 0; qt < MQ; ++qt) {
      if (qt < nqt) {
        int r = rank[qt];
        r = (int)xor_sum((float)r, 16);     // counts < 2^24: exact in fp32
        r = (int)xor_sum((float)r, 32);
        const int q = qt * 16 + col;
        if (g == 0 && q < LQ) {
          const bool s = r < uu;
          flag[q] = s;
          if (s) sel[r] = (int16_t)q;
        }
      }
    }
    wave_lds_sync();
  }
  if (sparse && !io.causal) {
    // ---- unselected rows keep the initial context, mean(V) (attn.py:116-119): written to every
    //      row here, then the selected rows are overwritten below (same wave, LDS in order)
    float part = 0.f;
#pragma unroll
    for (int kt = 0; kt < MK; ++kt)
      if (kt < nkt)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          part += (kt * 16 + g * 4 + j < LK) ? (float)Vf[kt][j] : 0.f;
    part = xor_sum(part, 16);
    part = xor_sum(part, 32);
    const __bf16 mean = (__bf16)(part / (float)LK);
    if (!io.mix) {
      for (int q = g; q < LQ; q += 4) io.ctx[q * BS + h * 16 + col] = mean;
    } else {
      for (int q = g; q < LQ; q += 4) {
        const int f = h * LQ * 16 + q * 16 + col;
        io.ctx[(f >> 7) * BS + (f & 127)] = mean;
      }
    }
  }
  SUB(4);

  // ---- softmax(scale·q·Kᵀ [mask])·V for the selected queries (attn.py:109-138 / 57-65)
  const float scale = 0.25f;
  const int nsel = sparse ? io.u : LQ;
  const int nst = (nsel + 15) >> 4;
#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    const int i = st * 16 + col;
    const int ic = i < nsel ? i : nsel - 1;
    int qi;
    bf16x4 qs;
    if (sparse) {
      // selected queries: re-project their rows (gathered from the bf16 image) — cheaper than
      // keeping Q in LDS
      qi = sel[ic];
      f32x4 q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        q = mfma16x16x32(wq[ks], *reinterpret_cast<const bf16x8*>(io.Xq + qi * BS + ks * 32 + kq), q);
      qs = cvt4(q * sq + bq);
    } else {
      qi = ic;
      qs = Qf[0];
#pragma unroll
      for (int t = 1; t < MQ; ++t) qs = st == t ? Qf[t] : qs;
    }
    // two sweeps over the key tiles (row max, then exp·V): the 16x16x16 score MFMAs are
    // recomputed rather than kept live (registers are the scarce resource at 2 waves/SIMD)
    float mx = NEG_INF;
#pragma unroll
    for (int kt = 0; kt < MK; ++kt) {
      if (kt < nkt) {
        const f32x4 a = mfma16x16x16(Kf[kt], qs, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt * 16 + g * 4 + r;
          const bool masked = key >= LK || (io.causal && key > qi);
          mx = masked ? mx : fmaxf(mx, a[r] * scale);
        }
      }
    }
    mx = xor_max(mx, 16);
    mx = xor_max(mx, 32);
    float sum = 0.f;
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < MK; ++kt) {
      if (kt < nkt) {
        f32x4 p = mfma16x16x16(Kf[kt], qs, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt * 16 + g * 4 + r;
          const bool masked = key >= LK || (io.causal && key > qi);
          p[r] = masked ? 0.f : __expf(p[r] * scale - mx);
          sum += p[r];
        }
        o = mfma16x16x16(Vf[kt], cvt4(p), o);
      }
    }
    sum = xor_sum(sum, 16);
    sum = xor_sum(sum, 32);
    const float inv = __builtin_amdgcn_rcpf(sum);
    if (i < nsel) {
      store_ctx4(io.ctx, io.mix, LQ, h, qi, g * 4, o * inv);
      if (io.attn_out) {
        float* arow = io.attn_out + ((size_t)h * LQ + qi) * LK;
#pragma unroll
        for (int kt = 0; kt < MK; ++kt)
          if (kt < nkt) {
            const f32x4 p = mfma16x16x16(Kf[kt], qs, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int key = kt * 16 + g * 4 + r;
              const bool masked = key >= LK || (io.causal && key > qi);
              if (key < LK) arow[key] = masked ? 0.f : __expf(p[r] * scale - mx) * inv;
            }
          }
      }
    }
  }

  SUB(5);
  if (sparse) {
    if (io.causal) {
      // masked: unselected rows keep cumsum(V) (attn.py:120-125) = Vᵀ·Tᵀ with T[q][key] = [key <= q],
      // the same MFMA with an indicator P
#pragma unroll
      for (int qt = 0; qt < MQ; ++qt) {
        if (qt < nqt) {
          const int q = qt * 16 + col;
          f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kt = 0; kt < MK; ++kt) {
            if (kt < nkt) {
              f32x4 ind;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int key = kt * 16 + g * 4 + r;
                ind[r] = (key <= q && key < LK) ? 1.f : 0.f;
              }
              o = mfma16x16x16(Vf[kt], cvt4(ind), o);
            }
          }
          if (q < LQ && !flag[q]) {
            int off;
            if (!io.mix) off = q * BS + h * 16 + g * 4;
            else { const int f = h * LQ * 16 + q * 16 + g * 4; off = (f >> 7) * BS + (f & 127); }
            *reinterpret_cast<bf16x4*>(io.ctx + off) = cvt4(o);
          }
        }
      }
    }
    if (io.attn_out) {
      const float invL = 1.0f / (float)LK;
      for (int q = 0; q < LQ; ++q)
        if (!flag[q]) {
          float* arow = io.attn_out + ((size_t)h * LQ + q) * LK;
          for (int k = lane; k < LK; k += WAVE) arow[k] = invL;
        }
    }
  }
  SUB(6);
}

}  // namespace v2
}  // namespace cet
