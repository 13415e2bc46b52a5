// Fused InformerStack / Informer inference forward — one workgroup per channel sequence.
//
// Reference: FullPrecision/InformerModel/model.py:142-271 (InformerStack.forward :247-271),
// encoder.py:6-106, decoder.py:6-56, attn.py:37-209, embed.py:8-135.
//
// The whole forward of a sequence (embedding → encoder stack with ProbSparse attention and
// distilling ConvLayers → decoder with masked/mixed self-attention and cross-attention →
// projection) runs inside one launch with every activation resident in LDS; weights stream
// from L2/MALL as pre-packed MFMA fragments.  See cet_device.hpp for the conventions.
#include "cet_kernels.h"
#include "cet_stages.hpp"

namespace cet {

template <int DFF>
__global__ void __launch_bounds__(NTHREADS, 1) informer_forward(InformerArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const InformerPlan& pl = *a.plan;
  const float* __restrict__ P = a.params;
  const bf16x8* __restrict__ W = reinterpret_cast<const bf16x8*>(a.weights);
  const int b = blockIdx.x;
  if (b >= a.B) return;

  float* X = reinterpret_cast<float*>(lds + pl.lds_X);
  __bf16* Qb = reinterpret_cast<__bf16*>(lds + pl.lds_Q);
  __bf16* Kb = reinterpret_cast<__bf16*>(lds + pl.lds_K);
  __bf16* Vt = reinterpret_cast<__bf16*>(lds + pl.lds_VT);
  __bf16* ENC = reinterpret_cast<__bf16*>(lds + pl.lds_ENC);
  __bf16* CTX = reinterpret_cast<__bf16*>(lds + pl.lds_CTX);
  float* T = reinterpret_cast<float*>(lds + pl.lds_Q);      // conv output: spans Q+K
  float* IN = reinterpret_cast<float*>(lds + pl.lds_K);     // staged raw input
  float* Msh = reinterpret_cast<float*>(lds + pl.lds_M);
  int16_t* SEL = reinterpret_cast<int16_t*>(lds + pl.lds_SEL);
  uint8_t* FLAG = reinterpret_cast<uint8_t*>(lds + pl.lds_FLAG);
  const int vts = pl.vts;
  const int wave = wave_id();
  float* dbg = a.dbg ? a.dbg + (size_t)b * pl.dbg_stride : nullptr;

  zero_lds(lds, pl.lds_bytes);
  const int C = pl.C;
  const int L0 = pl.seq_len;

  for (int e = 0; e < pl.n_enc; ++e) {
    stage_input(a.x_enc + (size_t)b * L0 * C, IN, L0, C, pl.in_stride);
    __syncthreads();
    // ---- DataEmbedding (embed.py:132-135) restricted to the encoder's input window
    //      x[:, -inp_len:] (EncoderStack, encoder.py:95-106)
    int L = L0 >> e;
    const int off = L0 - L;
    {
      const GemmDesc d = pl.emb_enc;
      gemm_t<2, 1, NW>(W + d.w, 8, (L0 + 15) >> 4, LoadEmbed{IN, L0, C, pl.in_stride}, [&](int m, int n0, f32x4 acc) {
        if (m < off || m >= L0) return;
        f32x4 v = affine(P, d, n0, acc) + *reinterpret_cast<const f32x4*>(P + pl.pe_enc + m * DMODEL + n0);
        *reinterpret_cast<f32x4*>(X + (m - off) * XS + n0) = v;
      });
    }
    __syncthreads();
    if (dbg && e == 0) { dump_rows(X, L0, dbg + pl.dbg_emb); __syncthreads(); }

    const int first = pl.enc_first[e];
    for (int l = 0; l < pl.enc_layers[e]; ++l) {
      const EncLayerDesc& ld = pl.enc[first + l];
      L = ld.L_in;
      // ---- AttentionLayer (attn.py:195-209): projections
      qkv_projection(P, W, ld.qkv, LoadF32{X}, L, Qb, Kb, Vt, vts);
      __syncthreads();
      // ---- ProbAttention / FullAttention, one wave per head; context overwrites Q in place
      {
        AttnIO io;
        io.Q = Qb; io.K = Kb; io.Vt = Vt; io.vts = vts; io.ctx = Qb;
        io.LQ = L; io.LK = L; io.prob = pl.prob; io.causal = 0; io.mix = 0;
        io.Msh = Msh; io.sel = SEL; io.flag = FLAG;
        io.cnt = nullptr; io.cnt_stride = 0; io.u = L; io.m_dbg = nullptr;
        if (ld.call >= 0) {
          const AttnCall& c = pl.calls[ld.call];
          io.u = c.u;
          io.cnt = a.cnt + c.cnt_off;
          io.cnt_stride = c.cnt_stride;
          if (dbg && c.m_dbg >= 0) io.m_dbg = dbg + c.m_dbg;
        }
        io.attn_out = a.attns ? a.attns + ld.attn_off + (size_t)b * ld.attn_stride : nullptr;
        attention_head(io, wave);
      }
      __syncthreads();
      residual_gemm<4>(P, W, ld.o, LoadBF16{Qb}, X, L);   // x = x + new_x   (encoder.py:49)
      __syncthreads();
      layer_norm_rows<NW>(X, X, nullptr, L, P + ld.ln1.g, P + ld.ln1.b, 1e-5f, false);
      __syncthreads();
      ffn_hidden<DFF>(P, W, ld.f1, LoadF32{X}, L, Kb, pl.act_relu);
      __syncthreads();
      residual_gemm<DFF / 32>(P, W, ld.f2, LoadBF16{Kb}, X, L);
      __syncthreads();
      layer_norm_rows<NW>(X, X, nullptr, L, P + ld.ln2.g, P + ld.ln2.b, 1e-5f, false);
      __syncthreads();
      if (dbg && ld.dbg_layer >= 0) { dump_rows(X, L, dbg + ld.dbg_layer); __syncthreads(); }
      if (ld.conv.n) {
        // ---- ConvLayer (encoder.py:22-28): circular conv → BN(eval, folded) → ELU → MaxPool(3,2,1)
        const GemmDesc d = ld.conv;
        gemm_t<12, 1, NW>(W + d.w, 8, (L + 15) >> 4, LoadCirc3F32<DMODEL>{X, L}, [&](int m, int n0, f32x4 acc) {
          if (m >= L) return;
          f32x4 v = affine(P, d, n0, acc);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = elu1(v[r]);
          *reinterpret_cast<f32x4*>(T + m * XS + n0) = v;
        });
        __syncthreads();
        const int Lo = ld.L_out;
        for (int i = threadIdx.x; i < Lo * 32; i += NTHREADS) {
          const int t = i >> 5, c4 = (i & 31) * 4;
          f32x4 v = *reinterpret_cast<const f32x4*>(T + (2 * t) * XS + c4);
          if (2 * t - 1 >= 0) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(T + (2 * t - 1) * XS + c4);
            v = f32x4{fmaxf(v[0], w[0]), fmaxf(v[1], w[1]), fmaxf(v[2], w[2]), fmaxf(v[3], w[3])};
          }
          if (2 * t + 1 < L) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(T + (2 * t + 1) * XS + c4);
            v = f32x4{fmaxf(v[0], w[0]), fmaxf(v[1], w[1]), fmaxf(v[2], w[2]), fmaxf(v[3], w[3])};
          }
          *reinterpret_cast<f32x4*>(X + t * XS + c4) = v;
        }
        __syncthreads();
        if (dbg && ld.dbg_conv >= 0) { dump_rows(X, Lo, dbg + ld.dbg_conv); __syncthreads(); }
      }
    }
    // ---- Encoder.norm (encoder.py:83-84) → this encoder's slice of the stack output (bf16)
    const int rows = pl.enc_rows[e];
    layer_norm_rows<NW>(X, X, ENC + pl.enc_row_off[e] * BS, rows, P + pl.enc_norm[e].g, P + pl.enc_norm[e].b,
                        1e-5f, false);
    __syncthreads();
    if (dbg && pl.enc_dbg[e] >= 0) { dump_rows(X, rows, dbg + pl.enc_dbg[e]); __syncthreads(); }
  }

  // ================================ decoder (decoder.py:43-56)
  const int Ld = pl.dec_len;
  const int S = pl.S;
  stage_input(a.x_dec + (size_t)b * Ld * C, IN, Ld, C, pl.in_stride);
  __syncthreads();
  {
    const GemmDesc d = pl.emb_dec;
    gemm_t<2, 1, NW>(W + d.w, 8, (Ld + 15) >> 4, LoadEmbed{IN, Ld, C, pl.in_stride}, [&](int m, int n0, f32x4 acc) {
      if (m >= Ld) return;
      f32x4 v = affine(P, d, n0, acc) + *reinterpret_cast<const f32x4*>(P + pl.pe_dec + m * DMODEL + n0);
      *reinterpret_cast<f32x4*>(X + m * XS + n0) = v;
    });
  }
  __syncthreads();
  if (dbg) { dump_rows(X, Ld, dbg + pl.dbg_dec_emb); __syncthreads(); }

  for (int l = 0; l < pl.d_layers; ++l) {
    const DecLayerDesc& ld = pl.dec[l];
    // ---- masked self-attention, mix=True (model.py:211-222)
    qkv_projection(P, W, ld.qkv, LoadF32{X}, Ld, Qb, Kb, Vt, vts);
    __syncthreads();
    {
      AttnIO io;
      io.Q = Qb; io.K = Kb; io.Vt = Vt; io.vts = vts; io.ctx = CTX;
      io.LQ = Ld; io.LK = Ld; io.prob = pl.prob; io.causal = 1; io.mix = pl.mix;
      io.Msh = Msh; io.sel = SEL; io.flag = FLAG;
      io.cnt = nullptr; io.cnt_stride = 0; io.u = Ld; io.m_dbg = nullptr; io.attn_out = nullptr;
      if (ld.call >= 0) {
        const AttnCall& c = pl.calls[ld.call];
        io.u = c.u;
        io.cnt = a.cnt + c.cnt_off;
        io.cnt_stride = c.cnt_stride;
        if (dbg && c.m_dbg >= 0) io.m_dbg = dbg + c.m_dbg;
      }
      attention_head(io, wave);
    }
    __syncthreads();
    residual_gemm<4>(P, W, ld.o, LoadBF16{CTX}, X, Ld);
    __syncthreads();
    layer_norm_rows<NW>(X, X, nullptr, Ld, P + ld.ln1.g, P + ld.ln1.b, 1e-5f, false);
    __syncthreads();
    // ---- cross-attention (FullAttention, no mask, mix=False) over the stack output
    {
      const GemmDesc dq = ld.cq;
      gemm_t<4, 1, NW>(W + dq.w, 8, (Ld + 15) >> 4, LoadF32{X}, [&](int m, int n0, f32x4 acc) {
        if (m >= Ld) return;
        *reinterpret_cast<bf16x4*>(Qb + m * BS + n0) = cvt4(affine(P, dq, n0, acc));
      });
      const GemmDesc dkv = ld.ckv;
      gemm_t<4, 2, NW>(W + dkv.w, 16, (S + 15) >> 4, LoadBF16{ENC}, [&](int m, int n0, f32x4 acc) {
        if (m >= S) return;
        const f32x4 v = affine(P, dkv, n0, acc);
        if (n0 < 128) {
          *reinterpret_cast<bf16x4*>(Kb + m * BS + n0) = cvt4(v);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) Vt[(n0 - 128 + r) * vts + m] = (__bf16)v[r];
        }
      });
    }
    __syncthreads();
    {
      AttnIO io;
      io.Q = Qb; io.K = Kb; io.Vt = Vt; io.vts = vts; io.ctx = CTX;
      io.LQ = Ld; io.LK = S; io.prob = 0; io.causal = 0; io.mix = 0; io.u = Ld;
      io.Msh = Msh; io.sel = SEL; io.flag = FLAG;
      io.cnt = nullptr; io.cnt_stride = 0; io.m_dbg = nullptr; io.attn_out = nullptr;
      attention_head(io, wave);
    }
    __syncthreads();
    residual_gemm<4>(P, W, ld.co, LoadBF16{CTX}, X, Ld);
    __syncthreads();
    layer_norm_rows<NW>(X, X, nullptr, Ld, P + ld.ln2.g, P + ld.ln2.b, 1e-5f, false);
    __syncthreads();
    ffn_hidden<DFF>(P, W, ld.f1, LoadF32{X}, Ld, Kb, pl.act_relu);
    __syncthreads();
    residual_gemm<DFF / 32>(P, W, ld.f2, LoadBF16{Kb}, X, Ld);
    __syncthreads();
    layer_norm_rows<NW>(X, X, nullptr, Ld, P + ld.ln3.g, P + ld.ln3.b, 1e-5f, false);
    __syncthreads();
    if (dbg && ld.dbg >= 0) { dump_rows(X, Ld, dbg + ld.dbg); __syncthreads(); }
  }
  layer_norm_rows<NW>(X, X, nullptr, Ld, P + pl.dec_norm.g, P + pl.dec_norm.b, 1e-5f, false);
  __syncthreads();
  if (dbg) { dump_rows(X, Ld, dbg + pl.dbg_dec_out); __syncthreads(); }

  // ---- projection (model.py:264), last pred_len rows → out[b]
  {
    const GemmDesc d = pl.proj;
    const int first_row = Ld - pl.pred_len;
    const int co = pl.c_out;
    float* out = a.out + (size_t)b * pl.pred_len * co;
    gemm_t<4, 1, NW>(W + d.w, d.n / 16, (Ld + 15) >> 4, LoadF32{X}, [&](int m, int n0, f32x4 acc) {
      if (m < first_row || m >= Ld) return;
      const f32x4 v = affine(P, d, n0, acc);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n0 + r < co) out[(m - first_row) * co + n0 + r] = v[r];
    });
  }
}

}  // namespace cet

extern "C" int cet_launch_informer(const cet::InformerArgs* a, int dff, int lds_bytes, hipStream_t stream) {
  using namespace cet;
  if (a->B <= 0) return 0;
  auto launch = [&](auto kern) -> int {
    if (!ensure_lds_attr(reinterpret_cast<const void*>(kern))) return -1;
    hipLaunchKernelGGL(kern, dim3(a->B), dim3(NTHREADS), lds_bytes, stream, *a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  };
  switch (dff) {
    case 64: return launch(informer_forward<64>);
    case 128: return launch(informer_forward<128>);
    default: return -3;
  }
}
