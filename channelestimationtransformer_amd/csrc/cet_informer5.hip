// Fused InformerStack forward, v5: TWO sequences per 512-thread workgroup, one workgroup per CU, 256
// VGPRs (cet_v5.hpp).  Same phase order, arithmetic and outputs as the v4 production instance
// (cet_informer4.hpp), which still serves the split-bf16 policy, the diagnostic outputs and the
// small-batch encoder split.
//
// Reference: FullPrecision/InformerModel/model.py:142-271 (InformerStack), :11-139 (Informer),
// encoder.py:6-106, decoder.py:6-56, attn.py:37-209, embed.py:8-135; FullPrecision/metrics.py:26-30
// (the fused NMSE_Split epilogue).
#include "cet_kernels.h"
#include "cet_mt.hpp"
#include "cet_sampler.hpp"
#include "cet_v5.hpp"

namespace cet {
namespace v5 {

// DIAG: the instance that honours the activation dumps (a.dbg, cet_set_debug), for per-stage parity
template <int DFF, int P, bool DIAG>
__device__ __forceinline__ void informer_forward_v5_body(const InformerArgs& a, const InformerPlan* __restrict__ plan) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
#define PL (*fresh(plan))
#define ELD (PL.enc[first + l])
#define DLD (PL.dec[l])
  constexpr int NS = 2;
  constexpr int PP = plain_of<P>();
  using LY = L5<P>;
  constexpr int RS = Geo<P>::RS;
  const Mem M{make_rsrc(a.weights), make_rsrc(a.params), a.wlo};
  const int b0 = (int)blockIdx.x * NS;
  if (b0 >= a.B) return;
  // the last workgroup of an odd batch repeats its first sequence in slot 1 and stores nothing for it
  const bool has1 = b0 + 1 < a.B;
  const int b1 = has1 ? b0 + 1 : b0;
  auto bseq = [b0, b1](int s) __attribute__((always_inline)) { return s == 0 ? b0 : b1; };
  const int w = wave_id();
  // per-stage fp32 dumps of each sequence's residual rows (the v4 debug layout, cet_debug_layout)
  auto DUMP = [&](const auto& Xs, int s, int nmt_, int rows, int off) __attribute__((always_inline)) {
    if constexpr (DIAG) {
      if (a.dbg && off >= 0 && (s == 0 || has1)) dump_res(Xs, nmt_, rows, a.dbg + (size_t)bseq(s) * PL.dbg_stride + off);
    }
  };
  // per-phase s_memtime stamps of the workgroup (the v4 phase points, tools/stamps.py), in its first
  // sequence's row of a.stamps
  unsigned long long* stamps = DIAG && a.stamps ? a.stamps + (size_t)b0 * MAX_STAMPS : nullptr;
  int sid = 0;
  auto STAMP = [&]() __attribute__((always_inline)) {
    if constexpr (DIAG) {
      if (stamps) {
        if (threadIdx.x == 0 && sid < MAX_STAMPS) stamps[sid] = __builtin_amdgcn_s_memtime();
        ++sid;
      }
    }
  };
#ifndef CET_NO_SETPRIO
  if (w >= 4) __builtin_amdgcn_s_setprio(1);   // the younger half (MI355X_MICROARCH "Two waves per SIMD" 4)
#endif

  auto XB = [&](int s) __attribute__((always_inline)) { return Img<P>{lds + LY::xb(s), 0}; };
  auto CTX = [&](int s) __attribute__((always_inline)) { return Img<P>{lds + LY::ctx(s), 0}; };
  auto FIN = [&](int s) __attribute__((always_inline)) { return Img<PP>{lds + LY::ctx(s), 0}; };
  auto ENC = [&](int s) __attribute__((always_inline)) {
    return Img<P>{lds + PL.lds5_enc + s * PL.lds5_enc_stride, 0};
  };
  auto IN = [&](int s) __attribute__((always_inline)) { return reinterpret_cast<float*>(lds + LY::ctx(s)); };
  auto XDEC = [&](int s) __attribute__((always_inline)) {
    return reinterpret_cast<float*>(lds + PL.lds5_xdec + s * PL.lds5_xdec_stride);
  };
  auto LAB = [&](int s) __attribute__((always_inline)) {
    return reinterpret_cast<float*>(lds + PL.lds5_lab + s * PL.lds5_lab_stride);
  };
  auto LNP = [&](int s) __attribute__((always_inline)) { return reinterpret_cast<float*>(lds + LY::scr(s)); };
  auto SCR = [&](int s) __attribute__((always_inline)) {
    return reinterpret_cast<float*>(lds + LY::scr(s)) + w * SCR_FLOATS;
  };
  uint8_t* CNT = reinterpret_cast<uint8_t*>(lds + LY::cnt(NS));

  const int C = PL.C, L0 = PL.seq_len, CS = PL.in_stride, Ld = PL.dec_len;
  // both sequences' inputs and labels are requested first (one f32x4 per thread each; the launcher
  // checks L·C ≤ 4·512), so their HBM latency overlaps the LDS zeroing
  const int t4 = 4 * (int)threadIdx.x;
  const int nlab = PL.pred_len * PL.c_out;
  f32x4 xe4[NS], xd4[NS], lb4[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    xe4[s] = xd4[s] = lb4[s] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t4 < L0 * C) xe4[s] = *reinterpret_cast<const f32x4*>(a.x_enc + (size_t)bseq(s) * L0 * C + t4);
    if (t4 < Ld * C) xd4[s] = *reinterpret_cast<const f32x4*>(a.x_dec + (size_t)bseq(s) * Ld * C + t4);
    if (a.label && t4 < nlab) lb4[s] = *reinterpret_cast<const f32x4*>(a.label + (size_t)bseq(s) * nlab + t4);
  }
  // zero the activation images: rows past L are read (never used) by MFMAs, and must be finite
  for (int i = threadIdx.x; i < PL.lds5_zero / 16; i += NTHREADS)
    reinterpret_cast<f32x4*>(lds)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  wg_sync();
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (t4 < L0 * C) *reinterpret_cast<f32x4*>(IN(s) + (t4 >> PL.C_shift) * CS + (t4 & (C - 1))) = xe4[s];
    if (t4 < Ld * C) *reinterpret_cast<f32x4*>(XDEC(s) + (t4 >> PL.C_shift) * CS + (t4 & (C - 1))) = xd4[s];
    if (a.label && t4 < nlab) *reinterpret_cast<f32x4*>(LAB(s) + t4) = lb4[s];
  }

  MTState gen{reinterpret_cast<uint32_t*>(lds + PL.lds5_mt), MT_N};
  if (a.mt_in && !a.cnt) {
    wg_sync();
    mt_load<NTHREADS>(gen, a.mt_in);
  }   // device-resident sampler (cet_mt.hpp)

  STAMP();
  constexpr int FRAGS_PER_TILE4 = 4 * WAVE;   // 16-byte lane fragments per n-tile at K = 128
  // one attention call (AttentionLayer, attn.py:178-209): one head per wave, both sequences
  auto attend = [&](auto MQc, auto MKc, auto&& Xq, auto&& Xkv, uint32_t Wq, uint32_t Wk, uint32_t Wv, GemmDesc dq,
                    GemmDesc dk, GemmDesc dv, int LQ, int LK, int prob, int causal, int mix, int call)
      __attribute__((always_inline)) {
    constexpr int MQ_ = decltype(MQc)::value, MK_ = decltype(MKc)::value;
    HeadIO2<P, NS> io;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      io.xq[s] = Xq(s);
      io.xkv[s] = Xkv(s);
      io.ctx[s] = CTX(s);
      io.scr[s] = SCR(s);
    }
    io.wq = Wq; io.wk = Wk; io.wv = Wv; io.dq = dq; io.dk = dk; io.dv = dv;
    io.LQ = LQ; io.LK = LK; io.prob = prob; io.causal = causal; io.mix = mix; io.u = LQ;
    io.cnt = nullptr; io.cnt_stride = 0;
    if (call >= 0) {
      const AttnCall& c = PL.calls[call];
      io.u = c.u;
      io.cnt_stride = c.cnt_stride;
      const bool sparse = c.u < c.LQ;
      if (!a.cnt) {
        // resident sampler: replay this call's draws into the (shared) LDS table (cet_mt.hpp)
        mt_replay<NTHREADS>(gen, c.LQ, c.U, c.LK, sparse ? reinterpret_cast<uint32_t*>(CNT) : nullptr,
                            c.cnt_stride);
        if (call == PL.n_calls - 1 && blockIdx.x == 0) mt_store<NTHREADS>(gen, a.mt_out);
      } else if (sparse) {
        const int bytes = ((c.LQ + 15) & ~15) * c.cnt_stride;
        const f32x4* src = reinterpret_cast<const f32x4*>(a.cnt + c.cnt_off);
        f32x4* dst = reinterpret_cast<f32x4*>(CNT);
        for (int i = threadIdx.x; i < bytes / 16; i += NTHREADS) dst[i] = src[i];
        wg_sync();
      }
      if (sparse) io.cnt = CNT;
    }
    attention_s<P, NS, MQ_, MK_>(io, M, w);
  };
  auto ldXB = [&](int s, int m, int k0) __attribute__((always_inline)) { return XB(s).ld(m, k0); };
  auto ldCTX = [&](int s, int m, int k0) __attribute__((always_inline)) { return CTX(s).ld(m, k0); };
  auto stXB = [&](int s, int m, int n0, const f32x4& y) __attribute__((always_inline)) { XB(s).st4(m, n0, y); };
  const int relu = PL.act_relu;
  auto ffn_act = [&](int s, int mt, int n0, f32x4 v) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = relu ? fmaxf(v[r], 0.f) : gelu_erf(v[r]);
    CTX(s).st4(mt * 16 + (lane_op() & 15), n0, v);
  };

  Res<MT> X[NS];
  for (int e = 0; e < PL.n_enc; ++e) {
    if (e > 0)   // CTX was reused by encoder e-1
#pragma unroll
      for (int s = 0; s < NS; ++s) stage(a.x_enc + (size_t)bseq(s) * L0 * C, IN(s), L0, C, CS);
    wg_sync();
    // ---- DataEmbedding (embed.py:132-135) on the EncoderStack window x[:, -L:] (encoder.py:95-106)
    int L = L0 >> e;
    const int off = L0 - L;
    int nmt = (L + 15) >> 4;
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) X[s].v[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      const GemmDesc d = PL.emb_enc;
      gemm_res_s<PP, 2, MT, NS>(
          prefetch_res<PP, 2>(M, d), nmt,
          [&](int s, int m, int k0) __attribute__((always_inline)) {
            return LoadEmbed<PP>{IN(s), L0, PL.C_shift, CS, off}(m, k0);
          },
          [&](int s, int mt, int n0, f32x4 y) __attribute__((always_inline)) {
            const int m = mt * 16 + (lane_op() & 15);
            const int prow = m + off < LMAX ? m + off : LMAX - 1;
            X[s].v[mt] = y + pload4(M, PL.pe_enc, prow * DMODEL + n0);
          });
    }
    wg_sync();                       // IN (aliases CTX) fully read
#pragma unroll
    for (int s = 0; s < NS; ++s) store_res(X[s], nmt, L, XB(s));
    wg_sync();
    if (e == 0)
#pragma unroll
      for (int s = 0; s < NS; ++s) DUMP(X[s], s, nmt, L, PL.dbg_emb);
    STAMP();  // embedding

    const int first = PL.enc_first[e];
    for (int l = 0; l < PL.enc_layers[e]; ++l) {
      L = ELD.L_in;
      nmt = (L + 15) >> 4;
      // ---- AttentionLayer + ProbAttention / FullAttention, one head per wave, context → CTX
      {
        const GemmDesc q = ELD.qkv;
        auto enc_attend = [&](auto NQ) __attribute__((always_inline)) {
          attend(NQ, NQ, XB, XB, q.w, q.w + 8 * FRAGS_PER_TILE4, q.w + 16 * FRAGS_PER_TILE4, part_of(q, 0),
                 part_of(q, 128), part_of(q, 256), L, L, PL.prob, 0, 0, ELD.call);
        };
        switch (nmt) {
          case 1: enc_attend(IC<1>{}); break;
          case 2: enc_attend(IC<2>{}); break;
          case 3: enc_attend(IC<3>{}); break;
          default: enc_attend(IC<MT>{}); break;
        }
      }
      const WPre<P, 4> po = prefetch_res<P, 4>(M, ELD.o);   // x = x + new_x (encoder.py:49)
      wg_sync();
      STAMP();  // encoder attention
      gemm_res_s<P, 4, MT, NS>(po, nmt, ldCTX, [&](int s, int mt, int n0, f32x4 y) __attribute__((always_inline)) {
        X[s].v[mt] += y;
      });
      static_assert(DFF / 16 <= NW, "FFN hidden n-tiles: at most one per wave");
      const WPre<P, 4> pf1 = prefetch_tiles<P, 4>(M, ELD.f1, DFF / 16);   // conv1 (k=1) + activation
      ln_res_s<NS, MT>(X, nmt, L, M, ELD.ln1, 1e-5f, false, LNP, stXB);
      wg_sync();
      STAMP();  // out-projection + LN1
      gemm_tiles1_s<P, 4, NS>(pf1, DFF / 16, nmt, ldXB, ffn_act);
      const WPre<P, DFF / 32> pf2 = prefetch_res<P, DFF / 32>(M, ELD.f2);  // conv2 (k=1) + residual
      wg_sync();
      gemm_res_s<P, DFF / 32, MT, NS>(pf2, nmt, ldCTX,
                                      [&](int s, int mt, int n0, f32x4 y) __attribute__((always_inline)) {
                                        X[s].v[mt] += y;
                                      });
      ln_res_s<NS, MT>(X, nmt, L, M, ELD.ln2, 1e-5f, false, LNP, stXB);
      wg_sync();
      STAMP();  // FFN + LN2
#pragma unroll
      for (int s = 0; s < NS; ++s) DUMP(X[s], s, nmt, L, ELD.dbg_layer);
      if (ELD.conv.n) {
        // ---- ConvLayer (encoder.py:22-28): circular conv, BN(eval) folded, ELU, MaxPool(3,2,1)
        // in even/odd position order, the pool an in-register max with a DPP row rotate
        const GemmDesc d = ELD.conv;
        with_nmt(nmt + (nmt & 1), [&](auto NMT) __attribute__((always_inline)) {
          constexpr int N_ = decltype(NMT)::value;
          if constexpr (N_ % 2 == 0) {
            Res<N_> Cv[NS];
            const WPre<P, 4> pcv = prefetch_kouter<P, 12, 4>(M, d);
            gemm_kouter_s<P, 12, 4, N_, NS>(
                pcv, M, d,
                [&](int s, int m, int k0) __attribute__((always_inline)) { return LoadCirc3EO<P>{XB(s), L}(m, k0); },
                [&](int s, int mt, int n0, f32x4 v) __attribute__((always_inline)) {
#pragma unroll
                  for (int r = 0; r < 4; ++r) v[r] = elu1(v[r]);
                  Cv[s].v[mt] = v;
                });
#pragma unroll
            for (int s = 0; s < NS; ++s) maxpool_eo<N_>(Cv[s], L, X[s]);
          }
        });
        L = ELD.L_out;
        nmt = (L + 15) >> 4;
        wg_sync();                   // every wave finished reading XB
#pragma unroll
        for (int s = 0; s < NS; ++s) store_res(X[s], nmt, L, XB(s));
        wg_sync();
        STAMP();  // distil conv + pool
#pragma unroll
        for (int s = 0; s < NS; ++s) DUMP(X[s], s, nmt, L, ELD.dbg_conv);
      }
    }
    // ---- Encoder.norm (encoder.py:83-84) → this encoder's rows of the stack output (ENC)
    const int rows = PL.enc_rows[e];
    const int roff = PL.enc_row_off[e] * RS;
    ln_res_s<NS, MT>(X, nmt, rows, M, PL.enc_norm[e], 1e-5f, false, LNP,
                     [&](int s, int m, int n0, const f32x4& y) __attribute__((always_inline)) {
                       Img<P>{ENC(s).base + roff, 0}.st4(m, n0, y);
                     });
    wg_sync();
#pragma unroll
    for (int s = 0; s < NS; ++s) DUMP(X[s], s, nmt, rows, PL.enc_dbg[e]);
    STAMP();  // encoder norm
  }

  // ================================ decoder (decoder.py:43-56), instantiated for its compile-time
  // tile count (dec_len ≤ 48); the staged decoder inputs are in XDEC
  const int S = PL.S;
  auto decoder = [&](auto NMDc, auto NMSc) __attribute__((always_inline)) {
    constexpr int NMS = decltype(NMSc)::value;
    constexpr int NMD = decltype(NMDc)::value;
    Res<NMD> XD[NS];
    {
      const GemmDesc d = PL.emb_dec;
      gemm_res_s<PP, 2, NMD, NS>(
          prefetch_res<PP, 2>(M, d), NMD,
          [&](int s, int m, int k0) __attribute__((always_inline)) {
            return LoadEmbed<PP>{XDEC(s), Ld, PL.C_shift, CS, 0}(m, k0);
          },
          [&](int s, int mt, int n0, f32x4 y) __attribute__((always_inline)) {
            const int m = mt * 16 + (lane_op() & 15);
            const int prow = m < LMAX ? m : LMAX - 1;
            XD[s].v[mt] = y + pload4(M, PL.pe_dec, prow * DMODEL + n0);
          });
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) store_res(XD[s], NMD, Ld, XB(s));
    wg_sync();
#pragma unroll
    for (int s = 0; s < NS; ++s) DUMP(XD[s], s, NMD, Ld, PL.dbg_dec_emb);
    STAMP();  // decoder embedding

    for (int l = 0; l < PL.d_layers; ++l) {
      // cross-attention K/V of this layer (encoder-stack output only): projected before the
      // self-attention, so their weight fetch overlaps it
      const GemmDesc cq = DLD.cq, ckv = DLD.ckv;
      HeadIO2<P, NS> cio;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        cio.xq[s] = XB(s);
        cio.xkv[s] = ENC(s);
        cio.ctx[s] = CTX(s);
        cio.scr[s] = SCR(s);
      }
      cio.wq = cq.w; cio.wk = ckv.w; cio.wv = ckv.w + 8 * FRAGS_PER_TILE4;
      cio.dq = part_of(cq, 0); cio.dk = part_of(ckv, 0); cio.dv = part_of(ckv, 128);
      cio.LQ = Ld; cio.LK = S; cio.prob = 0; cio.causal = 0; cio.mix = 0; cio.u = Ld;
      cio.cnt = nullptr; cio.cnt_stride = 0;
      AF<PP> CK[NS][NMS], CV[NS][NMS];
      project_kv_s<P, NS, NMS>(cio, M, w, CK, CV);
      {
        // masked self-attention with the mix scramble (model.py:211-222)
        const GemmDesc q = DLD.qkv;
        attend(IC<NMD>{}, IC<NMD>{}, XB, XB, q.w, q.w + 8 * FRAGS_PER_TILE4, q.w + 16 * FRAGS_PER_TILE4,
               part_of(q, 0), part_of(q, 128), part_of(q, 256), Ld, Ld, PL.prob, 1, PL.mix, DLD.call);
      }
      const WPre<P, 4> po = prefetch_res<P, 4>(M, DLD.o);
      wg_sync();
      STAMP();  // decoder self-attention
      gemm_res_s<P, 4, NMD, NS>(po, NMD, ldCTX, [&](int s, int mt, int n0, f32x4 y) __attribute__((always_inline)) {
        XD[s].v[mt] += y;
      });
      ln_res_s<NS, NMD>(XD, NMD, Ld, M, DLD.ln1, 1e-5f, false, LNP, stXB);
      wg_sync();
      // cross-attention: FullAttention over the encoder-stack output, mix=False
      attention_s<P, NS, NMD, NMS, true>(cio, M, w, CK, CV);
      const WPre<P, 4> pco = prefetch_res<P, 4>(M, DLD.co);
      wg_sync();
      STAMP();  // cross-attention
      gemm_res_s<P, 4, NMD, NS>(pco, NMD, ldCTX, [&](int s, int mt, int n0, f32x4 y) __attribute__((always_inline)) {
        XD[s].v[mt] += y;
      });
      const WPre<P, 4> pf1 = prefetch_tiles<P, 4>(M, DLD.f1, DFF / 16);
      ln_res_s<NS, NMD>(XD, NMD, Ld, M, DLD.ln2, 1e-5f, false, LNP, stXB);
      wg_sync();
      gemm_tiles1_s<P, 4, NS>(pf1, DFF / 16, NMD, ldXB, ffn_act);
      const WPre<P, DFF / 32> pf2 = prefetch_res<P, DFF / 32>(M, DLD.f2);
      wg_sync();
      gemm_res_s<P, DFF / 32, NMD, NS>(pf2, NMD, ldCTX,
                                       [&](int s, int mt, int n0, f32x4 y) __attribute__((always_inline)) {
                                         XD[s].v[mt] += y;
                                       });
      ln_res_s<NS, NMD>(XD, NMD, Ld, M, DLD.ln3, 1e-5f, false, LNP, stXB);
      wg_sync();
      STAMP();  // decoder O/LN1 + cross O/LN2 + FFN/LN3
#pragma unroll
      for (int s = 0; s < NS; ++s) DUMP(XD[s], s, NMD, Ld, DLD.dbg);
    }
    // final norm → the projection's input image (plain precision; CTX is free: FFN2 is done)
    ln_res_s<NS, NMD>(XD, NMD, Ld, M, PL.dec_norm, 1e-5f, false, LNP,
                      [&](int s, int m, int n0, const f32x4& y) __attribute__((always_inline)) { FIN(s).st4(m, n0, y); });
    wg_sync();
#pragma unroll
    for (int s = 0; s < NS; ++s) DUMP(XD[s], s, NMD, Ld, PL.dbg_dec_out);
    {
      // projection (model.py:264) on the last pred_len rows → out[b]
      const GemmDesc d = PL.proj;
      const int first_row = Ld - PL.pred_len, co = PL.c_out;
      const bool fuse = a.label != nullptr;   // the launcher guarantees c_out ≤ 16 (one n-tile)
      gemm_tiles_s<PP, 4, NS>(
          M, d, d.n / 16, NMD, [&](int s, int m, int k0) __attribute__((always_inline)) { return FIN(s).ld(m, k0); },
          [&](int s, int mt, int n0, f32x4 v) {
            if (s > 0 && !has1) return;   // the repeated sequence of an odd batch's last workgroup
            const int lane = lane_op();
            const int m = mt * 16 + (lane & 15);
            const bool valid = m >= first_row && m < Ld;
            const int bq = bseq(s);
            float* out = a.out + (size_t)bq * PL.pred_len * co;
            const float* lab = LAB(s);
            float se = 0.f, pw = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (valid && n0 + r < co) {
                out[(m - first_row) * co + n0 + r] = v[r];
                if (fuse) {   // NMSE_Split_cuda(x_hat = out, x = label): Σ(x − x̂)², Σ x̂² (metrics.py:26-30)
                  const float dx = lab[(m - first_row) * co + n0 + r] - v[r];
                  se = fmaf(dx, dx, se);
                  pw = fmaf(v[r], v[r], pw);
                }
              }
            if (fuse) {
              se = bp_sum(se, 16);   // over the 16 features of row m (4 lane groups)
              se = bp_sum(se, 32);
              pw = bp_sum(pw, 16);
              pw = bp_sum(pw, 32);
              if ((lane >> 4) == 0 && valid) {
                // write-through (sc1) so the last workgroup to finish reads it without a fence
                const float2 pr = make_float2(se, pw);
                __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.nmse_part + (size_t)bq * PL.pred_len +
                                                                         (m - first_row)),
                                   __builtin_bit_cast(unsigned long long, pr), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
              }
            }
          });
      if (fuse) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores are done
    }
    STAMP();  // final norm + projection
  };
  const bool s16 = S <= 16;
  switch ((Ld + 15) >> 4) {
    case 1: s16 ? decoder(IC<1>{}, IC<1>{}) : decoder(IC<1>{}, IC<MT>{}); break;
    case 2: s16 ? decoder(IC<2>{}, IC<1>{}) : decoder(IC<2>{}, IC<MT>{}); break;
    default: s16 ? decoder(IC<3>{}, IC<1>{}) : decoder(IC<3>{}, IC<MT>{}); break;
  }
  // ---- the first workgroup to finish prepares the NEXT forward's ProbSparse tables; the last one
  //      reduces the batch's NMSE_Split and re-arms the counter (as v4, over this grid's workgroups)
  if (a.ticket) {
    wg_sync();   // every wave's NMSE partials are written (each waited for its own stores)
    unsigned* tk = reinterpret_cast<unsigned*>(lds + LY::scr(0));
    const unsigned nwg = gridDim.x;
    if (threadIdx.x == 0) {
      // agent-scope acq_rel arrival: orders this workgroup's partial stores before the count, and the
      // last arrival's reads after it
      const unsigned t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (t + 1u == nwg) __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *tk = t;
    }
    wg_sync();   // the other waves load after this barrier (the adding wave has its value)
    const unsigned tw = __builtin_amdgcn_readfirstlane(*tk);
    if (a.label && tw + 1u == nwg) {
      // ---- last workgroup: the batch's NMSE_Split from every sequence's partials.  Thread i takes
      //      sequences i, i+512, ... (write-through partials, read with sc1 loads); then a fixed
      //      butterfly per wave and a fixed order over the waves: deterministic.
      const int T = PL.pred_len, lane = threadIdx.x & 63;
      double* red = reinterpret_cast<double*>(lds + LY::ctx(0));   // [NW][2][8]
      for (int t0 = 0; t0 < T; t0 += 8) {
        const int nt = T - t0 < 8 ? T - t0 : 8;
        double se[8], pw[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) se[j] = pw[j] = 0.0;
        for (int sq = threadIdx.x; sq < a.B; sq += NTHREADS) {
          const unsigned long long* src = reinterpret_cast<const unsigned long long*>(a.nmse_part + (size_t)sq * T + t0);
          unsigned long long u[8];
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < nt) u[j] = __hip_atomic_load(src + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < nt) {
              const float2 pr = __builtin_bit_cast(float2, u[j]);
              se[j] += (double)pr.x;
              pw[j] += (double)pr.y;
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1) {
            se[j] += __shfl_xor(se[j], o, 64);
            pw[j] += __shfl_xor(pw[j], o, 64);
          }
        if (lane == 0)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            red[(w * 2 + 0) * 8 + j] = se[j];
            red[(w * 2 + 1) * 8 + j] = pw[j];
          }
        wg_sync();
        if ((int)threadIdx.x < nt) {
          const int j = threadIdx.x;
          double a0 = 0.0, p0 = 0.0;
          for (int ww = 0; ww < NW; ++ww) {
            a0 += red[(ww * 2 + 0) * 8 + j];
            p0 += red[(ww * 2 + 1) * 8 + j];
          }
          if (a.nmse_sums) {
            a.nmse_sums[t0 + j] = a0;
            a.nmse_sums[T + t0 + j] = p0;
          }
          if (a.nmse_acc) a.nmse_acc[t0 + j] += (float)(a0 / p0);
        }
        wg_sync();
      }
    }
    const bool elected = tw == 0u;
    wg_sync();   // every wave has read the ticket before the replay reuses the LDS
    if (elected && a.cnt_next)
      replay_all<NTHREADS>(PL, a.mt_in, a.mt_out, a.cnt_next, lds, a.lds_bytes, reinterpret_cast<uint32_t*>(lds),
                           reinterpret_cast<uint32_t*>(lds + LY::ctx(0)));
  }
#undef PL
#undef ELD
#undef DLD
}

// one workgroup per CU: 8 waves, two per SIMD, up to 256 VGPRs each
template <int DFF, int P, bool DIAG>
__global__ void __launch_bounds__(NTHREADS, 2) informer_forward_v5(InformerArgs a, const InformerPlan* __restrict__ plan) {
  informer_forward_v5_body<DFF, P, DIAG>(a, plan);
}

}  // namespace v5
}  // namespace cet

// Two sequences per workgroup: grid = ceil(B / 2).  Production outputs, the activation dumps and the
// phase stamps (the caller routes the attention maps and the split-bf16 policy to v4).
extern "C" int cet_launch_informer_v5(const cet::InformerArgs* a, int prec, int dff, int lds_bytes, hipStream_t stream) {
  using namespace cet;
  if (a->B <= 0) return 0;
  if (a->attns || a->enc_split) return -3;
  using K = void (*)(InformerArgs, const InformerPlan*);
  K kern = nullptr;
  const bool diag = a->dbg != nullptr || a->stamps != nullptr;
  if (prec == v4::P_BF16) {
    if (dff == 64) kern = diag ? v5::informer_forward_v5<64, v4::P_BF16, true> : v5::informer_forward_v5<64, v4::P_BF16, false>;
    else if (dff == 128)
      kern = diag ? v5::informer_forward_v5<128, v4::P_BF16, true> : v5::informer_forward_v5<128, v4::P_BF16, false>;
  }
  if (!kern) return -3;
  if (!ensure_lds_attr(reinterpret_cast<const void*>(kern))) return -1;
  InformerArgs args = *a;
  args.lds_bytes = lds_bytes;
  const unsigned grid = (unsigned)((a->B + 1) / 2);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(v4::NTHREADS), lds_bytes, stream, args, a->plan);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
