// Fused models/Transformer inference forward — one workgroup per channel sequence.
//
// Reference: models/Transformer/model.py:76-87 (Transformer.forward), encoder.py:41-69,
// decoder.py:117-179, buildingblocks.py (LayerNormalization :23-30 with unbiased std and eps
// on the std, FeedForwardBlock :54-65 ReLU, MultiHeadAttentionBlock :152-192 bias-free, no
// masks, ResidualConnection :214-226 pre-LN), embed.py (circular conv k=3 + positional add).
#include "cet_kernels.h"
#include "cet_stages.hpp"

namespace cet {

// `plan` is a.plan again as a noalias parameter, so uniform descriptor reads become scalar loads.
template <int DFF>
__global__ void __launch_bounds__(NTHREADS, 1) transformer_forward(TransformerArgs a,
                                                                   const TransformerPlan* __restrict__ plan) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const TransformerPlan& pl = *plan;
  const float* __restrict__ P = a.params;
  const bf16x8* __restrict__ W = reinterpret_cast<const bf16x8*>(a.weights);
  const int b = blockIdx.x;
  if (b >= a.B) return;

  float* X = reinterpret_cast<float*>(lds + pl.lds_X);
  __bf16* Qb = reinterpret_cast<__bf16*>(lds + pl.lds_Q);
  __bf16* Kb = reinterpret_cast<__bf16*>(lds + pl.lds_K);
  __bf16* Vt = reinterpret_cast<__bf16*>(lds + pl.lds_VT);
  __bf16* ENC = reinterpret_cast<__bf16*>(lds + pl.lds_ENC);
  __bf16* XN = reinterpret_cast<__bf16*>(lds + pl.lds_ENC);   // encoder phase: LN output
  __bf16* XND = reinterpret_cast<__bf16*>(lds + pl.lds_XN);   // decoder phase: LN output
  float* IN = reinterpret_cast<float*>(lds + pl.lds_K);
  const int vts = pl.vts;
  const int wave = wave_id();
  float* dbg = a.dbg ? a.dbg + (size_t)b * pl.dbg_stride : nullptr;
  const float eps = 1e-6f;

  zero_lds(lds, pl.lds_bytes);
  const int C = pl.C;
  const int L = pl.src_len;

  auto attend = [&](const __bf16* Q, const __bf16* K, int LQ, int LK, __bf16* ctx) {
    AttnIO io;
    io.Q = Q; io.K = K; io.Vt = Vt; io.vts = vts; io.ctx = ctx;
    io.LQ = LQ; io.LK = LK; io.prob = 0; io.causal = 0; io.mix = 0; io.u = LQ;
    io.cnt = nullptr; io.cnt_stride = 0; io.Msh = nullptr; io.sel = nullptr; io.flag = nullptr;
    io.attn_out = nullptr; io.m_dbg = nullptr;
    attention_head(io, wave);
  };

  // ---- encode (model.py:27-30)
  stage_input(a.x_enc + (size_t)b * L * C, IN, L, C, pl.in_stride);
  __syncthreads();
  {
    const GemmDesc d = pl.emb_src;
    gemm_t<2, 1, NW>(W + d.w, 8, (L + 15) >> 4, LoadEmbed{IN, L, C, pl.in_stride}, [&](int m, int n0, f32x4 acc) {
      if (m >= L) return;
      *reinterpret_cast<f32x4*>(X + m * XS + n0) =
          affine(P, d, n0, acc) + *reinterpret_cast<const f32x4*>(P + pl.pe_src + m * DMODEL + n0);
    });
  }
  __syncthreads();
  if (dbg) { dump_rows(X, L, dbg + pl.dbg_emb); __syncthreads(); }
  for (int l = 0; l < pl.N; ++l) {
    const auto& ld = pl.enc[l];
    layer_norm_rows<NW>(X, nullptr, XN, L, P + ld.ln0.g, P + ld.ln0.b, eps, true);
    __syncthreads();
    qkv_projection(P, W, ld.qkv, LoadBF16{XN}, L, Qb, Kb, Vt, vts);
    __syncthreads();
    attend(Qb, Kb, L, L, Qb);
    __syncthreads();
    residual_gemm<4>(P, W, ld.o, LoadBF16{Qb}, X, L);
    __syncthreads();
    layer_norm_rows<NW>(X, nullptr, XN, L, P + ld.ln1.g, P + ld.ln1.b, eps, true);
    __syncthreads();
    ffn_hidden<DFF>(P, W, ld.f1, LoadBF16{XN}, L, Kb, 1);
    __syncthreads();
    residual_gemm<DFF / 32>(P, W, ld.f2, LoadBF16{Kb}, X, L);
    __syncthreads();
    if (dbg && ld.dbg >= 0) { dump_rows(X, L, dbg + ld.dbg); __syncthreads(); }
  }
  layer_norm_rows<NW>(X, dbg ? X : nullptr, ENC, L, P + pl.enc_norm.g, P + pl.enc_norm.b, eps, true);
  __syncthreads();
  if (dbg) { dump_rows(X, L, dbg + pl.dbg_enc_out); __syncthreads(); }

  // ---- decode (model.py:32-41)
  const int Ld = pl.tgt_len;
  stage_input(a.x_dec + (size_t)b * Ld * C, IN, Ld, C, pl.in_stride);
  __syncthreads();
  {
    const GemmDesc d = pl.emb_tgt;
    gemm_t<2, 1, NW>(W + d.w, 8, (Ld + 15) >> 4, LoadEmbed{IN, Ld, C, pl.in_stride}, [&](int m, int n0, f32x4 acc) {
      if (m >= Ld) return;
      *reinterpret_cast<f32x4*>(X + m * XS + n0) =
          affine(P, d, n0, acc) + *reinterpret_cast<const f32x4*>(P + pl.pe_tgt + m * DMODEL + n0);
    });
  }
  __syncthreads();
  if (dbg) { dump_rows(X, Ld, dbg + pl.dbg_dec_emb); __syncthreads(); }
  for (int l = 0; l < pl.N; ++l) {
    const auto& ld = pl.dec[l];
    layer_norm_rows<NW>(X, nullptr, XND, Ld, P + ld.ln0.g, P + ld.ln0.b, eps, true);
    __syncthreads();
    qkv_projection(P, W, ld.qkv, LoadBF16{XND}, Ld, Qb, Kb, Vt, vts);
    __syncthreads();
    attend(Qb, Kb, Ld, Ld, Qb);   // tgt_mask = None in the reference forward
    __syncthreads();
    residual_gemm<4>(P, W, ld.o, LoadBF16{Qb}, X, Ld);
    __syncthreads();
    layer_norm_rows<NW>(X, nullptr, XND, Ld, P + ld.ln1.g, P + ld.ln1.b, eps, true);
    __syncthreads();
    {
      const GemmDesc dq = ld.cq;
      gemm_t<4, 1, NW>(W + dq.w, 8, (Ld + 15) >> 4, LoadBF16{XND}, [&](int m, int n0, f32x4 acc) {
        if (m >= Ld) return;
        *reinterpret_cast<bf16x4*>(Qb + m * BS + n0) = cvt4(affine(P, dq, n0, acc));
      });
      const GemmDesc dkv = ld.ckv;
      gemm_t<4, 2, NW>(W + dkv.w, 16, (L + 15) >> 4, LoadBF16{ENC}, [&](int m, int n0, f32x4 acc) {
        if (m >= L) return;
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
    attend(Qb, Kb, Ld, L, Qb);
    __syncthreads();
    residual_gemm<4>(P, W, ld.co, LoadBF16{Qb}, X, Ld);
    __syncthreads();
    layer_norm_rows<NW>(X, nullptr, XND, Ld, P + ld.ln2.g, P + ld.ln2.b, eps, true);
    __syncthreads();
    ffn_hidden<DFF>(P, W, ld.f1, LoadBF16{XND}, Ld, Kb, 1);
    __syncthreads();
    residual_gemm<DFF / 32>(P, W, ld.f2, LoadBF16{Kb}, X, Ld);
    __syncthreads();
    if (dbg && ld.dbg >= 0) { dump_rows(X, Ld, dbg + ld.dbg); __syncthreads(); }
  }
  layer_norm_rows<NW>(X, X, nullptr, Ld, P + pl.dec_norm.g, P + pl.dec_norm.b, eps, true);
  __syncthreads();
  if (dbg) { dump_rows(X, Ld, dbg + pl.dbg_dec_out); __syncthreads(); }
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

extern "C" int cet_launch_transformer(const cet::TransformerArgs* a, int dff, int lds_bytes, hipStream_t stream) {
  using namespace cet;
  if (a->B <= 0) return 0;
  auto launch = [&](void (*kern)(TransformerArgs, const TransformerPlan*), int) -> int {
    if (!ensure_lds_attr(reinterpret_cast<const void*>(kern))) return -1;
    hipLaunchKernelGGL(kern, dim3(a->B), dim3(NTHREADS), lds_bytes, stream, *a, a->plan);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  };
  switch (dff) {
    case 64: return launch(transformer_forward<64>, 0);
    case 128: return launch(transformer_forward<128>, 1);
    default: return -3;
  }
}
