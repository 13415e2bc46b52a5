// "v3" building blocks: 8-wave (512-thread) workgroups, one 16-feature n-tile of the residual
// stream and one attention head per wave.
//
// Why: at the C2 batch (512 sequences on 256 CUs) every CU holds exactly two sequences, so the
// kernel time IS one sequence's latency.  v2 ran a sequence on 4 waves (2 per SIMD with two
// sequences per CU) and its phases were latency chains — 2 heads one after the other per wave,
// 2 n-tiles per dense layer.  v3 spreads the same work over 8 waves (4 per SIMD), halving every
// per-wave chain and giving each SIMD twice the independent streams to interleave; the register
// budget per wave halves with it (≤128 VGPRs), which the smaller per-wave state fits.
//
// Register-resident residual (Res<N>): wave w owns features [16w, 16w+16) = n-tile w of every
// residual-producing dense layer; for m-tile mt its lane l holds
// X[16·mt + (l&15)][16w + 4·(l>>4) + r] in v[mt][r] — the C fragment of Yᵀ = W·Xᵀ on
// v_mfma_f32_16x16x32_bf16 (the v2 layout with one n-tile per wave instead of two).
#pragma once
#include "cet_v2.hpp"

namespace cet {
namespace v3 {

using v2::load4;   // LDS / generic fp32x4 loads
using v2::with_nmt;

// Weights and parameters are read through buffer resources: a uniform byte offset (SGPR) plus a
// 32-bit per-lane offset, so no fragment or epilogue-vector load needs 64-bit VALU address math.
struct Mem {
  __amdgpu_buffer_rsrc_t w;   // packed bf16 fragments [n_tile][k_step][lane][8]
  __amdgpu_buffer_rsrc_t p;   // fp32 parameter blob
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7ffffff0, 0x00020000);
}
// this lane's bf16x8 of the 1 KiB wave tile at uniform byte offset `off`
__device__ __forceinline__ bf16x8 wfrag(const Mem& m, uint32_t off, int lane) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(m.w, lane * 16, (int)off, 0));
}
// fp32 parameters: uniform float offset `so` + per-lane float offset `vo`
__device__ __forceinline__ f32x4 pload4(const Mem& m, uint32_t so, int vo) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(m.p, vo * 4, (int)(so * 4u), 0));
}
__device__ __forceinline__ float pload1(const Mem& m, uint32_t so, int vo) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(m.p, vo * 4, (int)(so * 4u), 0));
}

// Lane index the compiler cannot hoist: every lane-derived address is recomputed inside the
// phase that uses it (a few VALU) instead of being hoisted to the kernel entry and kept live —
// at 128 VGPRs per wave the hoisted per-tile row addresses were what spilled to scratch.
__device__ __forceinline__ int lane_op() {
  int l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}

// The KS k-step fragments of n-tile nt of the layer whose fragments start at `base` (bf16x8
// units, as GemmDesc::w).
template <int KS>
__device__ __forceinline__ void load_frags(const Mem& m, uint32_t base, int nt, bf16x8 (&a)[KS]) {
  const int lane = lane_op();
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) a[ks] = wfrag(m, base * 16u + (uint32_t)(nt * KS + ks) * 1024u, lane);
}
__device__ __forceinline__ void epi_vecs(const Mem& m, const GemmDesc& d, int n0, f32x4& sc, f32x4& bi) {
  sc = f32x4{1.f, 1.f, 1.f, 1.f};
  bi = f32x4{0.f, 0.f, 0.f, 0.f};
  if (d.scale != NONE) sc = pload4(m, d.scale, n0);
  if (d.bias != NONE) bi = pload4(m, d.bias, n0);
}

constexpr int NW = 8;
constexpr int NTHREADS = NW * WAVE;
constexpr int MT = 6;             // max 16-row tiles (96 positions)
constexpr int LN_STRIDE = LN3_STRIDE;   // floats per LayerNorm-partials row (cet_plan.hpp)

template <int N>
struct Res {
  f32x4 v[N];
};

// A dense layer's per-wave operands — the KS weight fragments of n-tile w and the epilogue
// vectors — requested ahead of time: callers issue them before the workgroup barrier that
// precedes the layer, so their L2 latency overlaps the barrier wait instead of following it.
template <int KS>
struct WPre {
  bf16x8 a[KS];
  f32x4 sc, bi;
};
template <int KS>
__device__ __forceinline__ WPre<KS> prefetch_res(const Mem& m, const GemmDesc d) {
  WPre<KS> p;
  const int lane = lane_op(), w = wave_id();
  load_frags<KS>(m, d.w, w, p.a);
  epi_vecs(m, d, 16 * w + (lane >> 4) * 4, p.sc, p.bi);
  return p;
}

// Dense layer whose output n-tile w lands in the wave's residual fragments.
// epi(mt, n0, f32x4 y) receives the finished (scaled, biased) value.
template <int KS, int N, class BL, class Epi>
__device__ __forceinline__ void gemm_res(const WPre<KS>& p, int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_op(), w = wave_id();
  const int n0 = 16 * w + (lane >> 4) * 4;
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) c = mfma16x16x32(p.a[ks], bl(mt * 16 + mrow, ks * 32 + kq), c);
      epi(mt, n0, c * p.sc + p.bi);
    }
  }
}
template <int KS, int N, class BL, class Epi>
__device__ __forceinline__ void gemm_res(const Mem& m, const GemmDesc d, int nmt, BL&& bl, Epi&& epi) {
  gemm_res<KS, N>(prefetch_res<KS>(m, d), nmt, bl, epi);
}

// Compile-time m-tile count: no per-tile branch, B fragments of tile mt+1 requested before the
// MFMAs of tile mt.
template <int KS, int NMT, class BL, class Epi>
__device__ __forceinline__ void gemm_res_n(const WPre<KS>& p, BL&& bl, Epi&& epi) {
  const int lane = lane_op(), w = wave_id();
  const int n0 = 16 * w + (lane >> 4) * 4;
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
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) c = mfma16x16x32(p.a[ks], b[ks], c);
    epi(mt, n0, c * p.sc + p.bi);
    if (mt + 1 < NMT) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) b[ks] = bn[ks];
    }
  }
}
template <int KS, int NMT, class BL, class Epi>
__device__ __forceinline__ void gemm_res_n(const Mem& m, const GemmDesc d, BL&& bl, Epi&& epi) {
  gemm_res_n<KS, NMT>(prefetch_res<KS>(m, d), bl, epi);
}

// Dense layer over an arbitrary n-tile count (FFN hidden, projection), output through epi only.
// n_tiles ≥ NW: wave w takes n-tiles w, w+NW, ... over every m-tile; otherwise the waves split
// into NW / n_tiles groups per n-tile and a group takes every (NW / n_tiles)-th m-tile, so each
// wave loads its weight fragments once.
template <int KS, class BL, class Epi>
__device__ __forceinline__ void gemm_tiles(const Mem& m, const GemmDesc d, int n_tiles, int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_op(), w = wave_id();
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
  int nt0 = w, nt_step = NW, mt0 = 0, mt_step = 1;
  if (n_tiles < NW) {
    const int per = NW / n_tiles;
    if (w >= per * n_tiles) return;
    nt0 = w % n_tiles;
    nt_step = n_tiles;
    mt0 = w / n_tiles;
    mt_step = per;
  }
  for (int nt = nt0; nt < n_tiles; nt += nt_step) {
    bf16x8 a[KS];
    load_frags<KS>(m, d.w, nt, a);
    const int n0 = nt * 16 + (lane >> 4) * 4;
    f32x4 sc, bi;
    epi_vecs(m, d, n0, sc, bi);
    for (int mt = mt0; mt < nmt; mt += mt_step) {
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) c = mfma16x16x32(a[ks], bl(mt * 16 + mrow, ks * 32 + kq), c);
      epi(mt, n0, c * sc + bi);
    }
  }
}

// gemm_tiles for n_tiles ≤ NW (every wave owns at most one n-tile, so its operands can be
// prefetched): wave w takes n-tile w mod n_tiles and every (NW / n_tiles)-th m-tile from w / n_tiles.
template <int KS>
__device__ __forceinline__ WPre<KS> prefetch_tiles(const Mem& m, const GemmDesc d, int n_tiles) {
  WPre<KS> p;
  const int lane = lane_op(), w = wave_id();
  const int nt = w % n_tiles;
  load_frags<KS>(m, d.w, nt, p.a);
  epi_vecs(m, d, nt * 16 + (lane >> 4) * 4, p.sc, p.bi);
  return p;
}
template <int KS, class BL, class Epi>
__device__ __forceinline__ void gemm_tiles1(const WPre<KS>& p, int n_tiles, int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_op(), w = wave_id();
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
  const int per = NW / n_tiles;
  if (w >= per * n_tiles) return;
  const int nt = w % n_tiles, mt_step = per;
  const int n0 = nt * 16 + (lane >> 4) * 4;
  for (int mt = w / n_tiles; mt < nmt; mt += mt_step) {
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) c = mfma16x16x32(p.a[ks], bl(mt * 16 + mrow, ks * 32 + kq), c);
    epi(mt, n0, c * p.sc + p.bi);
  }
}

// Deep-K dense layer (the distil conv, K = 384) in k-outer order with a compile-time m-tile count:
// one accumulator per m-tile, the B fragments of step ks+1 requested before step ks's MFMAs, and
// the weight fragments loaded in halves of KH k-steps (keeps the wave under 128 VGPRs).
// The first KH of KS k-steps of n-tile w and the epilogue vectors of a deep-K layer.
template <int KS, int KH>
__device__ __forceinline__ WPre<KH> prefetch_kouter(const Mem& m, const GemmDesc d) {
  WPre<KH> p;
  const int lane = lane_op(), w = wave_id();
#pragma unroll
  for (int ks = 0; ks < KH; ++ks) p.a[ks] = wfrag(m, d.w * 16u + (uint32_t)(w * KS + ks) * 1024u, lane);
  epi_vecs(m, d, 16 * w + (lane >> 4) * 4, p.sc, p.bi);
  return p;
}
// `p` holds the first KH k-steps' fragments and the epilogue vectors (prefetch_kouter).
template <int KS, int KH, int NMT, class BL, class Epi>
__device__ __forceinline__ void gemm_kouter_res(const WPre<KH>& p, const Mem& m, const GemmDesc d, BL&& bl,
                                                Epi&& epi) {
  static_assert(KS % KH == 0, "k-steps split into equal halves");
  const int lane = lane_op(), w = wave_id();
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
  const int n0 = 16 * w + (lane >> 4) * 4;
  const f32x4 sc = p.sc, bi = p.bi;
  f32x4 c[NMT];
  bf16x8 b[NMT];
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    c[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    b[mt] = bl(mt * 16 + mrow, kq);
  }
  const uint32_t t0 = d.w * 16u + (uint32_t)(w * KS) * 1024u;
#pragma unroll
  for (int hf = 0; hf < KS / KH; ++hf) {
    bf16x8 a[KH];
#pragma unroll
    for (int ks = 0; ks < KH; ++ks)
      a[ks] = hf == 0 ? p.a[ks] : wfrag(m, t0 + (uint32_t)(hf * KH + ks) * 1024u, lane);
#pragma unroll
    for (int ks = 0; ks < KH; ++ks) {
      const int kk = hf * KH + ks;
      bf16x8 bn[NMT];
      if (kk + 1 < KS) {
#pragma unroll
        for (int mt = 0; mt < NMT; ++mt) bn[mt] = bl(mt * 16 + mrow, (kk + 1) * 32 + kq);
      }
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt) c[mt] = mfma16x16x32(a[ks], b[mt], c[mt]);
      if (kk + 1 < KS) {
#pragma unroll
        for (int mt = 0; mt < NMT; ++mt) b[mt] = bn[mt];
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch distance at one k-step
    }
  }
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) epi(mt, n0, c[mt] * sc + bi);
}

// LayerNorm of the register residual over all 128 features (8 waves × 16).  Each wave reduces
// its 16 features per row to (mean_w, M2_w), the 8 pairs meet in LDS (`part`, LN_STRIDE floats
// per row), and Chan's combination gives the exact row mean / variance.  Normalised rows go to X
// (registers) and rows < `rows` to the bf16 image Xb (and optionally Xb2).
// torch.nn.LayerNorm (biased var, eps in the sqrt) or, if unbiased_std, the reference
// Transformer's LayerNormalization (alpha·(x-mean)/(std_unbiased+eps)+bias).
// Contains one workgroup barrier; the caller adds one before Xb is read.
template <int N>
__device__ __forceinline__ void ln_res(Res<N>& X, int nmt, int rows, const Mem& mm, const LNDesc ln, float eps,
                                       bool unbiased_std, float* part, __bf16* Xb, __bf16* Xb2 = nullptr) {
  const int lane = lane_op(), w = wave_id(), g = lane >> 4, c = lane & 15;
  const int nb = 16 * w + 4 * g;
  const f32x4 g0 = pload4(mm, ln.g, nb), b0 = pload4(mm, ln.b, nb);   // issued before the barrier
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      float s = (X.v[mt][0] + X.v[mt][1]) + (X.v[mt][2] + X.v[mt][3]);
      s = xor_sum(s, 16);
      s = xor_sum(s, 32);
      const float mw = s * (1.0f / 16.0f);
      float q = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = X.v[mt][r] - mw;
        q = fmaf(d, d, q);
      }
      q = xor_sum(q, 16);
      q = xor_sum(q, 32);
      if (g == 0) *reinterpret_cast<f32x2*>(part + (mt * 16 + c) * LN_STRIDE + 2 * w) = f32x2{mw, q};
    }
  }
  __syncthreads();
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      const int m = mt * 16 + c;
      const float* pr = part + m * LN_STRIDE;
      const f32x4 p0 = load4(pr), p1 = load4(pr + 4), p2 = load4(pr + 8), p3 = load4(pr + 12);
      const float mean = 0.125f * (((p0[0] + p0[2]) + (p1[0] + p1[2])) + ((p2[0] + p2[2]) + (p3[0] + p3[2])));
      const float d0 = p0[0] - mean, d1 = p0[2] - mean, d2 = p1[0] - mean, d3 = p1[2] - mean;
      const float d4 = p2[0] - mean, d5 = p2[2] - mean, d6 = p3[0] - mean, d7 = p3[2] - mean;
      const float M2 = (((p0[1] + p0[3]) + (p1[1] + p1[3])) + ((p2[1] + p2[3]) + (p3[1] + p3[3]))) +
                       16.0f * ((d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3) + (d4 * d4 + d5 * d5 + d6 * d6 + d7 * d7));
      const float inv = unbiased_std ? __builtin_amdgcn_rcpf(sqrtf(M2 * (1.0f / 127.0f)) + eps)
                                     : __builtin_amdgcn_rsqf(M2 * (1.0f / 128.0f) + eps);
      X.v[mt] = (X.v[mt] - mean) * inv * g0 + b0;
      if (m < rows) {
        const bf16x4 y = cvt4(X.v[mt]);
        *reinterpret_cast<bf16x4*>(Xb + m * BS + nb) = y;
        if (Xb2) *reinterpret_cast<bf16x4*>(Xb2 + m * BS + nb) = y;
      }
    }
  }
}

// bf16 image of the register residual (rows < rows).
template <int N>
__device__ __forceinline__ void store_res(const Res<N>& X, int nmt, int rows, __bf16* Xb) {
  const int lane = lane_op(), w = wave_id();
  const int nb = 16 * w + 4 * (lane >> 4);
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      const int m = mt * 16 + (lane & 15);
      if (m < rows) *reinterpret_cast<bf16x4*>(Xb + m * BS + nb) = cvt4(X.v[mt]);
    }
  }
}

// fp32 dump of the register residual rows < rows into dst[rows][128] (debug only).
template <int N>
__device__ __forceinline__ void dump_res(const Res<N>& X, int nmt, int rows, float* dst) {
  const int lane = lane_op(), w = wave_id();
  const int nb = 16 * w + 4 * (lane >> 4);
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      const int m = mt * 16 + (lane & 15);
      if (m < rows) *reinterpret_cast<f32x4*>(dst + m * DMODEL + nb) = X.v[mt];
    }
  }
}

// MaxPool1d(kernel 3, stride 2, padding 1) over positions of a register-resident tile set:
// out row t' = max(x[2t'-1], x[2t'], x[2t'+1]) over rows in [0, L).  Rows live on the 16-lane
// axis, so the 2:1 gather is a within-row ds_bpermute from tiles 2j-1, 2j, 2j+1.
template <int NIN>
__device__ __forceinline__ void maxpool_res(const Res<NIN>& in, int L, Res<MT>& out) {
  const int lane = lane_op();
  const int c = lane & 15, base = lane & 48;
  const int s0 = base | ((2 * c) & 15), s1 = base | ((2 * c + 1) & 15), sm = base | ((2 * c - 1) & 15);
  constexpr int NOUT = (NIN + 1) / 2;
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a0 = __shfl(in.v[2 * j][r], s0, 64);
      const float a1 = __shfl(in.v[2 * j][r], s1, 64);
      const float a2 = __shfl(in.v[2 * j][r], sm, 64);
      float b0 = 0.f, b1 = 0.f, b2 = 0.f;   // tile 2j+1 absent: only padded output rows read it
      if (2 * j + 1 < NIN) {
        b0 = __shfl(in.v[2 * j + 1][r], s0, 64);
        b1 = __shfl(in.v[2 * j + 1][r], s1, 64);
        b2 = __shfl(in.v[2 * j + 1][r], sm, 64);
      }
      const float c2 = j > 0 ? __shfl(in.v[(2 * j - 1 < 0) ? 0 : 2 * j - 1][r], sm, 64) : NEG_INF;
      const int row0 = 32 * j + 2 * c;
      float v = c < 8 ? a0 : b0;                          // row 2t'   (always < L for t' < L_out)
      const float v1 = c < 8 ? a1 : b1;                   // row 2t'+1
      const float vm = c == 0 ? c2 : (c <= 8 ? a2 : b2);  // row 2t'-1
      if (row0 + 1 < L) v = fmaxf(v, v1);
      if (row0 - 1 >= 0) v = fmaxf(v, vm);
      out.v[j][r] = v;
    }
  }
#pragma unroll
  for (int j = NOUT; j < MT; ++j) out.v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// ------------------------------------------------------------------------------ attention
// One head per wave, everything in registers (the v2 scheme, cet_v2.hpp attention_head2):
//   Kᵀ = Wk_h·Xᵀ (A of Sᵀ = K·Qᵀ), Qᵀ = Wq_h·Xᵀ (B of Sᵀ), V = X·Wv_hᵀ (A of Oᵀ = Vᵀ·Pᵀ), and
//   the exponentiated Sᵀ tile is the B fragment of Oᵀ.  Reference: attn.py:73-175 (ProbAttention),
//   :37-70 (FullAttention), :195-209 (AttentionLayer incl. mix).
struct HeadIO {
  const __bf16* Xq;           // LDS rows feeding the queries (bf16, stride BS)
  const __bf16* Xkv;          // LDS rows feeding keys / values
  uint32_t wq, wk, wv;        // weight-blob offsets (bf16x8 units) of n-tile 0 of each projection
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
__device__ __forceinline__ void attention_head(const HeadIO& io, const Mem& m, int h) {
  const int lane = lane_op();
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
  bf16x4 Kf[MK], Vf[MK];
  {
    // pass 1: K and V tiles from the key/value rows (only wk, wv live)
    bf16x8 wk[4], wv[4];
    load_frags<4>(m, io.wk, h, wk);
    load_frags<4>(m, io.wv, h, wv);
    f32x4 sk, bk;
    epi_vecs(m, io.dk, fq, sk, bk);
    const float sv = io.dv.scale != NONE ? pload1(m, io.dv.scale, 16 * h + col) : 1.f;
    const float bv = io.dv.bias != NONE ? pload1(m, io.dv.bias, 16 * h + col) : 0.f;
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
  // Q tiles are projected where they are consumed (per query tile in M, per selected tile in the
  // softmax) instead of being kept: wq and its epilogue vectors are the only Q state that lives
  bf16x8 wq[4];
  load_frags<4>(m, io.wq, h, wq);
  f32x4 sq, bq;
  epi_vecs(m, io.dq, fq, sq, bq);
  auto project_q = [&](int row) __attribute__((always_inline)) {
    f32x4 q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      q = mfma16x16x32(wq[ks], *reinterpret_cast<const bf16x8*>(io.Xq + row * BS + ks * 32 + kq), q);
    return cvt4(q * sq + bq);
  };

  SUB(2);
  if (sparse) {
    // ---- sparsity measurement M (attn.py:95-105) from key multiplicities (LDS-staged table)
    const float invLK = 1.0f / (float)LK;
#pragma unroll
    for (int qt = 0; qt < MQ; ++qt) {
      if (qt >= nqt) break;
      const int q = qt * 16 + col;
      const bf16x4 qf = project_q(q);
      // this lane's six count words (keys 16kt + 4g + r, kt = 0..5) are contiguous: cnt_pos_v2()
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
            // rows past L are stale-but-finite bf16 images, so 0·s is exact zero
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
    // selected queries (sparse) are gathered rows of the bf16 image; re-projected here
    const int qi = sparse ? (int)sel[ic] : ic;
    const bf16x4 qs = project_q(qi);
    // two sweeps over the key tiles (row max, then exp·V): the 16x16x16 score MFMAs are
    // recomputed rather than kept live
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

}  // namespace v3
}  // namespace cet
