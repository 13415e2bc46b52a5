// Fused InformerStack forward, v2: 256-thread workgroups, register-resident residual stream
// and per-head attention (cet_v2.hpp), ~62 KB of LDS so two sequences share a CU.
//
// Reference: FullPrecision/InformerModel/model.py:142-271, encoder.py:6-106, decoder.py:6-56,
// attn.py:37-209, embed.py:8-135 (see cet_informer.hip for the v1 kernel and DESIGN.md).
#include "cet_kernels.h"
#include "cet_mt.hpp"
#include "cet_v2.hpp"

namespace cet {
namespace v2 {

template <int N>
using IC = std::integral_constant<int, N>;

// Token-embedding input for output row m = position m + off (EncoderStack window):
// A[m][tap·C + c] = x[(m + off - 1 + tap) mod L][c], zero past 3·C.  C is a power of two
// (CSH = log2 C) and the wrap is add/subtract — no integer division on the hot path.
struct LoadEmbedOff {
  const float* X;
  int L, CSH, CS, off;
  __device__ __forceinline__ bf16x8 operator()(int m, int k0) const {
    const int tap = k0 >> CSH, c = k0 & ((1 << CSH) - 1);
    if (tap >= 3) return bf16x8{};
    int r = m + off - 1 + tap;
    r = r < 0 ? r + L : r;
    r = r >= L ? r - L : r;
    r = r >= L ? L - 1 : r;  // padded rows (m >= L) only: any valid row
    const f32x4* p = reinterpret_cast<const f32x4*>(X + r * CS + c);
    return cvt8(p[0], p[1]);
  }
};

// Circular k=3 conv input from the bf16 image: A[m][tap·128 + c] = Xb[(m-1+tap) mod L][c].
struct LoadCirc3BF16 {
  const __bf16* X;
  int L;
  __device__ __forceinline__ bf16x8 operator()(int m, int k0) const {
    const int tap = k0 >> 7, c = k0 & 127;
    int r = m - 1 + tap;
    r = r < 0 ? r + L : r;
    r = r >= L ? r - L : r;
    r = r >= L ? L - 1 : r;  // padded rows only
    return *reinterpret_cast<const bf16x8*>(X + r * BS + c);
  }
};

__device__ __forceinline__ void stage(const float* __restrict__ src, float* dst, int L, int C, int CS) {
  for (int i = threadIdx.x; i < L * C; i += NTHREADS) {
    const int t = i / C, c = i - t * C;
    dst[t * CS + c] = src[i];
  }
}

__device__ __forceinline__ GemmDesc part_of(GemmDesc d, int off) {
  if (d.bias != NONE) d.bias += off;
  if (d.scale != NONE) d.scale += off;
  return d;
}

template <int DFF>
__global__ void __launch_bounds__(NTHREADS, 2) informer_forward_v2(InformerArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const InformerPlan& pl = *a.plan;
  const float* __restrict__ P = a.params;
  const bf16x8* __restrict__ W = reinterpret_cast<const bf16x8*>(a.weights);
  const int b = blockIdx.x;
  if (b >= a.B) return;
  const int w = wave_id();

  __bf16* Xb = reinterpret_cast<__bf16*>(lds + pl.lds2_XB);
  __bf16* CTX = reinterpret_cast<__bf16*>(lds + pl.lds2_CTX);   // attention context / FFN hidden
  __bf16* ENC = reinterpret_cast<__bf16*>(lds + pl.lds2_ENC);
  float* LNP = reinterpret_cast<float*>(lds + pl.lds2_LN);
  uint8_t* CNT = reinterpret_cast<uint8_t*>(lds + pl.lds2_CNT);
  MTState gen{reinterpret_cast<uint32_t*>(lds + pl.lds2_MT), MT_N};
  float* SCR = reinterpret_cast<float*>(lds + pl.lds2_SCR) + w * V2_SCR_FLOATS;
  float* IN = reinterpret_cast<float*>(lds + pl.lds2_CTX);      // staged raw input (aliases CTX)
  float* dbg = a.dbg ? a.dbg + (size_t)b * pl.dbg_stride : nullptr;

  for (int i = threadIdx.x; i < pl.lds2_bytes / 16; i += NTHREADS)
    reinterpret_cast<f32x4*>(lds)[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int C = pl.C, L0 = pl.seq_len, CS = pl.in_stride;
  constexpr int FRAGS_PER_TILE4 = 4 * WAVE;   // bf16x8 per n-tile at K = 128
  Resid X;
  // diagnostics: s_memtime at phase boundaries (wave 0, lane 0), off unless a.stamps is set
  unsigned long long* stamps = a.stamps ? a.stamps + (size_t)b * MAX_STAMPS : nullptr;
  int sid = 0;
  auto STAMP = [&]() {
    if (stamps) {
      if (threadIdx.x == 0 && sid < MAX_STAMPS) stamps[sid] = __builtin_amdgcn_s_memtime();
      ++sid;
    }
  };
  if (a.mt_in) {
    __syncthreads();   // LDS zeroing above is done before the state lands in it
    mt_load<NTHREADS>(gen, a.mt_in);
  }   // device-resident sampler (cet_mt.hpp)
  // fine-grained stamps inside encoder layer 0 (slots 116..127, diagnostics)
  auto FINE = [&](int layer, int k) {
    if (stamps && layer == 0 && threadIdx.x == 0) stamps[116 + k] = __builtin_amdgcn_s_memtime();
  };
  STAMP();

  // MQc / MKc: compile-time bounds on the query / key tiles (std::integral_constant)
  auto attend = [&](auto MQc, auto MKc, const __bf16* Xq, const __bf16* Xkv, const bf16x8* Wq, const bf16x8* Wk,
                    const bf16x8* Wv, GemmDesc dq, GemmDesc dk, GemmDesc dv, int LQ, int LK, int prob, int causal,
                    int mix, int call, float* attn_out) {
    constexpr int MQ_ = decltype(MQc)::value, MK_ = decltype(MKc)::value;
    HeadIO io;
    io.Xq = Xq; io.Xkv = Xkv; io.Wq = Wq; io.Wk = Wk; io.Wv = Wv;
    io.dq = dq; io.dk = dk; io.dv = dv;
    io.ctx = CTX; io.LQ = LQ; io.LK = LK; io.prob = prob; io.causal = causal; io.mix = mix; io.u = LQ;
    io.cnt = nullptr; io.cnt_stride = 0; io.scr = SCR; io.attn_out = attn_out; io.m_dbg = nullptr;
    // sub-phase stamps of the first two sparse calls land in slots 100.. / 108.. (diagnostics)
    io.st = (stamps && call >= 0 && call < 2) ? stamps + 100 + 8 * call : nullptr;
    if (call >= 0) {
      const AttnCall& c = pl.calls[call];
      io.u = c.u;
      io.cnt_stride = c.cnt_stride;
      if (dbg && c.m_dbg >= 0) io.m_dbg = dbg + c.m_dbg;
      const bool sparse = c.u < c.LQ;
      if (a.mt_in) {
        // replay this call's draws from the resident mt19937 stream into the LDS table
        mt_replay<NTHREADS>(gen, c.LQ, c.U, c.LK, sparse ? reinterpret_cast<uint32_t*>(CNT) : nullptr,
                            c.cnt_stride);
        if (call == pl.n_calls - 1 && b == 0) mt_store<NTHREADS>(gen, a.mt_out);
      } else if (sparse) {
        // stage the host-built table in LDS (one L2 round trip per layer instead of one per
        // query tile and key tile)
        const int bytes = ((c.LQ + 15) & ~15) * c.cnt_stride;
        const f32x4* src = reinterpret_cast<const f32x4*>(a.cnt + c.cnt_off);
        f32x4* dst = reinterpret_cast<f32x4*>(CNT);
        for (int i = threadIdx.x; i < bytes / 16; i += NTHREADS) dst[i] = src[i];
        __syncthreads();
      }
      if (sparse) io.cnt = CNT;
    }
    if constexpr (MQ_ * MK_ >= 4) {
#pragma unroll 1
      for (int hh = 0; hh < 2; ++hh) attention_head2<MQ_, MK_>(io, P, 2 * w + hh);
    } else {
      // small tiles: both heads in one straight-line block, so their loads and MFMAs overlap
      attention_head2<MQ_, MK_>(io, P, 2 * w);
      attention_head2<MQ_, MK_>(io, P, 2 * w + 1);
    }
  };

  for (int e = 0; e < pl.n_enc; ++e) {
    stage(a.x_enc + (size_t)b * L0 * C, IN, L0, C, CS);
    __syncthreads();
    // ---- DataEmbedding (embed.py:132-135) on the EncoderStack window x[:, -L:] (encoder.py:95-106)
    int L = L0 >> e;
    const int off = L0 - L;
    int nmt = (L + 15) >> 4;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) X.v[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      const GemmDesc d = pl.emb_enc;
      gemm_wave2<2>(W, P, d, nmt, LoadEmbedOff{IN, L0, pl.C_shift, CS, off}, [&](int t, int mt, int n0, f32x4 y) {
        const int m = mt * 16 + (lane_id() & 15);
        const int prow = m + off < LMAX ? m + off : LMAX - 1;
        X.v[t][mt] = y + load4(P + pl.pe_enc + prow * DMODEL + n0);
      });
    }
    __syncthreads();                       // IN (aliases CTX) fully read
    store_xb(X, nmt, L, Xb);
    __syncthreads();
    if (dbg && e == 0) dump_resid(X, nmt, L, dbg + pl.dbg_emb);
    STAMP();  // embedding

    const int first = pl.enc_first[e];
    for (int l = 0; l < pl.enc_layers[e]; ++l) {
      const EncLayerDesc& ld = pl.enc[first + l];
      L = ld.L_in;
      nmt = (L + 15) >> 4;
      // ---- AttentionLayer + ProbAttention / FullAttention, two heads per wave, context → CTX
      {
        const GemmDesc q = ld.qkv;
        attend(IC<MT>{}, IC<MT>{}, Xb, Xb, W + q.w, W + q.w + 8 * FRAGS_PER_TILE4, W + q.w + 16 * FRAGS_PER_TILE4,
               part_of(q, 0), part_of(q, 128), part_of(q, 256), L, L, pl.prob, 0, 0, ld.call,
               a.attns ? a.attns + ld.attn_off + (size_t)b * ld.attn_stride : nullptr);
      }
      __syncthreads();
      STAMP();  // encoder attention
      {
        const GemmDesc d = ld.o;   // x = x + new_x (encoder.py:49)
        gemm_wave2<4>(W, P, d, nmt, LoadBF16{CTX}, [&](int t, int mt, int n0, f32x4 y) {
          X.v[t][mt] += y;
        });
      }
      FINE(l, 0);
      ln_resid(X, nmt, L, P + ld.ln1.g, P + ld.ln1.b, 1e-5f, false, LNP, Xb);
      __syncthreads();
      STAMP();  // out-projection + LN1
      {
        const GemmDesc d = ld.f1;  // conv1 (k=1) + activation (encoder.py:52)
        const int relu = pl.act_relu;
        gemm_tiles<4>(W, P, d, DFF / 16, nmt, LoadBF16{Xb}, [&](int mt, int n0, f32x4 v) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = relu ? fmaxf(v[r], 0.f) : gelu_erf(v[r]);
          *reinterpret_cast<bf16x4*>(CTX + (mt * 16 + (lane_id() & 15)) * BS + n0) = cvt4(v);
        });
      }
      FINE(l, 1);
      __syncthreads();
      FINE(l, 2);
      {
        const GemmDesc d = ld.f2;  // conv2 (k=1) + residual (encoder.py:53-56)
        gemm_wave2<DFF / 32>(W, P, d, nmt, LoadBF16{CTX}, [&](int t, int mt, int n0, f32x4 y) {
          X.v[t][mt] += y;
        });
      }
      FINE(l, 3);
      ln_resid(X, nmt, L, P + ld.ln2.g, P + ld.ln2.b, 1e-5f, false, LNP, Xb);
      __syncthreads();
      STAMP();  // FFN + LN2
      if (dbg && ld.dbg_layer >= 0) dump_resid(X, nmt, L, dbg + ld.dbg_layer);
      FINE(l, 4);
      if (ld.conv.n) {
        // ---- ConvLayer (encoder.py:22-28): circular conv, BN(eval) folded, ELU, MaxPool(3,2,1)
        const GemmDesc d = ld.conv;
        // Cv lives inside each m-tile-count instantiation and only X leaves it: stores into a
        // shared Cv would be sunk behind the dispatch through a pointer phi, demoting Cv to scratch
        with_nmt(nmt, [&](auto NMT) __attribute__((always_inline)) {
          Resid Cv;
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) Cv.v[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
          gemm_wave2_kouter<12, decltype(NMT)::value>(W, P, d, LoadCirc3BF16{Xb, L},
                                                      [&](int t, int mt, int n0, f32x4 v) __attribute__((always_inline)) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = elu1(v[r]);
            Cv.v[t][mt] = v;
          });
          FINE(l, 5);
          maxpool_resid(Cv, L, X);
        });
        FINE(l, 6);
        L = ld.L_out;
        nmt = (L + 15) >> 4;
        __syncthreads();                   // every wave finished reading Xb
        FINE(l, 7);
        store_xb(X, nmt, L, Xb);
        __syncthreads();
        STAMP();  // distil conv + pool
        if (dbg && ld.dbg_conv >= 0) dump_resid(X, nmt, L, dbg + ld.dbg_conv);
      }
    }
    // ---- Encoder.norm (encoder.py:83-84) → this encoder's rows of the stack output (ENC)
    const int rows = pl.enc_rows[e];
    ln_resid(X, nmt, rows, P + pl.enc_norm[e].g, P + pl.enc_norm[e].b, 1e-5f, false, LNP, Xb,
             ENC + pl.enc_row_off[e] * BS);
    __syncthreads();
    if (dbg && pl.enc_dbg[e] >= 0) dump_resid(X, nmt, rows, dbg + pl.enc_dbg[e]);
    STAMP();  // encoder norm
  }

  // ================================ decoder (decoder.py:43-56), instantiated for its compile-time
  // tile count (dec_len ≤ 48): a 1..3-tile residual, branch-free GEMMs, the two heads of a wave
  // interleaved — the decoder's 15-row layers are latency, not work
  const int Ld = pl.dec_len, S = pl.S;
  stage(a.x_dec + (size_t)b * Ld * C, IN, Ld, C, CS);
  __syncthreads();
  auto decoder = [&](auto NMDc) __attribute__((always_inline)) {
    constexpr int NMD = decltype(NMDc)::value;
    const int nmd = NMD;
    ResidT<NMD> XD;
    {
      const GemmDesc d = pl.emb_dec;
      gemm_wave2_n<2, NMD>(W, P, d, LoadEmbedOff{IN, Ld, pl.C_shift, CS, 0}, [&](int t, int mt, int n0, f32x4 y) {
        const int m = mt * 16 + (lane_id() & 15);
        const int prow = m < LMAX ? m : LMAX - 1;
        XD.v[t][mt] = y + load4(P + pl.pe_dec + prow * DMODEL + n0);
      });
    }
    __syncthreads();
    store_xb(XD, nmd, Ld, Xb);
    __syncthreads();
    if (dbg) dump_resid(XD, nmd, Ld, dbg + pl.dbg_dec_emb);
    STAMP();  // decoder embedding

    for (int l = 0; l < pl.d_layers; ++l) {
      const DecLayerDesc& ld = pl.dec[l];
      {
        // masked self-attention with the mix scramble (model.py:211-222)
        const GemmDesc q = ld.qkv;
        attend(IC<NMD>{}, IC<NMD>{}, Xb, Xb, W + q.w, W + q.w + 8 * FRAGS_PER_TILE4, W + q.w + 16 * FRAGS_PER_TILE4,
               part_of(q, 0), part_of(q, 128), part_of(q, 256), Ld, Ld, pl.prob, 1, pl.mix, ld.call, nullptr);
      }
      __syncthreads();
      STAMP();  // decoder self-attention
      {
        const GemmDesc d = ld.o;
        gemm_wave2_n<4, NMD>(W, P, d, LoadBF16{CTX}, [&](int t, int mt, int n0, f32x4 y) { XD.v[t][mt] += y; });
      }
      ln_resid(XD, nmd, Ld, P + ld.ln1.g, P + ld.ln1.b, 1e-5f, false, LNP, Xb);
      __syncthreads();
      {
        // cross-attention: FullAttention over the encoder-stack output, mix=False
        const GemmDesc cq = ld.cq, ckv = ld.ckv;
        attend(IC<NMD>{}, IC<MT>{}, Xb, ENC, W + cq.w, W + ckv.w, W + ckv.w + 8 * FRAGS_PER_TILE4, part_of(cq, 0),
               part_of(ckv, 0), part_of(ckv, 128), Ld, S, 0, 0, 0, -1, nullptr);
      }
      __syncthreads();
      STAMP();  // cross-attention
      {
        const GemmDesc d = ld.co;
        gemm_wave2_n<4, NMD>(W, P, d, LoadBF16{CTX}, [&](int t, int mt, int n0, f32x4 y) { XD.v[t][mt] += y; });
      }
      ln_resid(XD, nmd, Ld, P + ld.ln2.g, P + ld.ln2.b, 1e-5f, false, LNP, Xb);
      __syncthreads();
      {
        const GemmDesc d = ld.f1;
        const int relu = pl.act_relu;
        gemm_tiles_n<4, NMD>(W, P, d, DFF / 16, LoadBF16{Xb}, [&](int mt, int n0, f32x4 v) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = relu ? fmaxf(v[r], 0.f) : gelu_erf(v[r]);
          *reinterpret_cast<bf16x4*>(CTX + (mt * 16 + (lane_id() & 15)) * BS + n0) = cvt4(v);
        });
      }
      __syncthreads();
      {
        const GemmDesc d = ld.f2;
        gemm_wave2_n<DFF / 32, NMD>(W, P, d, LoadBF16{CTX}, [&](int t, int mt, int n0, f32x4 y) { XD.v[t][mt] += y; });
      }
      ln_resid(XD, nmd, Ld, P + ld.ln3.g, P + ld.ln3.b, 1e-5f, false, LNP, Xb);
      __syncthreads();
      STAMP();  // decoder O/LN1 + cross O/LN2 + FFN/LN3
      if (dbg && ld.dbg >= 0) dump_resid(XD, nmd, Ld, dbg + ld.dbg);
    }
    ln_resid(XD, nmd, Ld, P + pl.dec_norm.g, P + pl.dec_norm.b, 1e-5f, false, LNP, Xb);
    __syncthreads();
    if (dbg) dump_resid(XD, nmd, Ld, dbg + pl.dbg_dec_out);
    {
      // projection (model.py:264) on the last pred_len rows → out[b]
      const GemmDesc d = pl.proj;
      const int first_row = Ld - pl.pred_len, co = pl.c_out;
      float* out = a.out + (size_t)b * pl.pred_len * co;
      gemm_tiles_n<4, NMD>(W, P, d, d.n / 16, LoadBF16{Xb}, [&](int mt, int n0, f32x4 v) {
        const int m = mt * 16 + (lane_id() & 15);
        if (m < first_row || m >= Ld) return;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n0 + r < co) out[(m - first_row) * co + n0 + r] = v[r];
      });
    }
    STAMP();  // final norm + projection
  };
  switch ((Ld + 15) >> 4) {
    case 1: decoder(IC<1>{}); break;
    case 2: decoder(IC<2>{}); break;
    default: decoder(IC<3>{}); break;
  }
}

}  // namespace v2
}  // namespace cet

extern "C" int cet_launch_informer_v2(const cet::InformerArgs* a, int dff, int lds_bytes, hipStream_t stream) {
  using namespace cet;
  if (a->B <= 0) return 0;
  auto launch = [&](auto kern) -> int {
    static bool attr_done = false;
    if (!attr_done) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024) != hipSuccess)
        return -1;
      attr_done = true;
    }
    hipLaunchKernelGGL(kern, dim3(a->B), dim3(v2::NTHREADS), lds_bytes, stream, *a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  };
  switch (dff) {
    case 64: return launch(v2::informer_forward_v2<64>);
    case 128: return launch(v2::informer_forward_v2<128>);
    default: return -3;
  }
}
