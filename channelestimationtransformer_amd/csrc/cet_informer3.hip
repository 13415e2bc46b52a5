// Fused InformerStack forward, v3: 512-thread workgroups (8 waves), one residual n-tile and one
// attention head per wave (cet_v3.hpp), ≤80 KB of LDS and ≤128 VGPRs so two sequences share a CU
// at 4 waves per SIMD.
//
// Reference: FullPrecision/InformerModel/model.py:142-271, encoder.py:6-106, decoder.py:6-56,
// attn.py:37-209, embed.py:8-135 (the v2 kernel, cet_informer2.hip, has the same phase order).
#include "cet_kernels.h"
#include "cet_mt.hpp"
#include "cet_sampler.hpp"
#include "cet_v3.hpp"

namespace cet {
namespace v3 {

template <int N>
using IC = std::integral_constant<int, N>;

// Token-embedding input for output row m = position m + off (EncoderStack window):
// A[m][tap·C + c] = x[(m + off - 1 + tap) mod L][c], zero past 3·C (C a power of two).
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

// Plan access point: the plan is read through the constant address space (scalar loads that no
// store of the kernel can clobber).  The pointer is also hidden from the optimiser (asm), so
// each phase re-loads its descriptors instead of keeping them live in SGPRs: 724 instead of 2468
// SGPR spill/reload lane moves, ≈1.3% faster (V3_TRANSPARENT_PLAN restores the other behaviour).
// (The host pass of the compile only needs the declarations.)
#if defined(__HIP_DEVICE_COMPILE__)
template <class T>
using cptr = const __attribute__((address_space(4))) T*;
#else
template <class T>
using cptr = const T*;
#endif
template <class T>
__device__ __forceinline__ cptr<T> fresh(const T* p) {
  cptr<T> c = (cptr<T>)p;
#ifndef V3_TRANSPARENT_PLAN
  asm volatile("" : "+s"(c));
#endif
  return c;
}

__device__ __forceinline__ GemmDesc part_of(GemmDesc d, int off) {
  if (d.bias != NONE) d.bias += off;
  if (d.scale != NONE) d.scale += off;
  return d;
}

// DIAG: the instance that honours the optional outputs (attns maps, activation dump, phase stamps);
// the production instance compiles them out, which frees the scalar registers their pointers held.
// XE: the plan's layout has the x_dec region (staged at entry; cet_plan.hpp V3L_XDEC).
template <int DFF, bool DIAG, bool XE>
// `plan` is a.plan passed again as a noalias parameter: no store of the kernel can clobber it, so
// every uniform descriptor read becomes a scalar load (s_load into SGPRs) instead of a vector load
// plus v_readfirstlane.
__global__ void __launch_bounds__(NTHREADS, 4) informer_forward_v3(InformerArgs a,
                                                                  const InformerPlan* __restrict__ plan) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
#define PL (*fresh(plan))
#define ELD (PL.enc[first + l])
#define DLD (PL.dec[l])
  const Mem M{make_rsrc(a.weights), make_rsrc(a.params)};
  const int b = blockIdx.x;
  if (b >= a.B) return;
  const int w = wave_id();

  __bf16* Xb = reinterpret_cast<__bf16*>(lds + V3L_XB);
  __bf16* CTX = reinterpret_cast<__bf16*>(lds + V3L_CTX);   // attention context / FFN hidden
  __bf16* ENC = reinterpret_cast<__bf16*>(lds + (XE ? V3L_ENC_XE : V3L_ENC));
  float* LNP = reinterpret_cast<float*>(lds + V3L_SCR);      // LN partials (alias the scratch)
  uint8_t* CNT = reinterpret_cast<uint8_t*>(lds + V3L_CNT);
  MTState gen{reinterpret_cast<uint32_t*>(lds + V3L_MT), MT_N};
  float* SCR = reinterpret_cast<float*>(lds + V3L_SCR) + w * V2_SCR_FLOATS;
  float* IN = reinterpret_cast<float*>(lds + V3L_CTX);      // staged raw input (aliases CTX)
  float* dbg = DIAG && a.dbg ? a.dbg + (size_t)b * PL.dbg_stride : nullptr;

  // staged decoder input: its own region (XE, staged at entry) or CTX (staged when the decoder starts)
  float* XDEC = reinterpret_cast<float*>(lds + (XE ? V3L_XDEC : V3L_CTX));
  if (DIAG && a.stamps && threadIdx.x == 0) a.stamps[(size_t)b * MAX_STAMPS + 127] = __builtin_amdgcn_s_memtime();
  const int C = PL.C, L0 = PL.seq_len, CS = PL.in_stride, Ld = PL.dec_len;
  // this sequence's x_enc and x_dec rows are requested first (one f32x4 per thread each: L·C/4 ≤
  // 384), so their HBM latency overlaps the LDS zeroing instead of following it
  const int t4 = 4 * (int)threadIdx.x;
  f32x4 xe4 = {0.f, 0.f, 0.f, 0.f}, xd4 = xe4;
  if (t4 < L0 * C) xe4 = *reinterpret_cast<const f32x4*>(a.x_enc + (size_t)b * L0 * C + t4);
  if (XE && t4 < Ld * C) xd4 = *reinterpret_cast<const f32x4*>(a.x_dec + (size_t)b * Ld * C + t4);
  // zero the activation images: rows past L of Xb / CTX / ENC are read (never used) by MFMAs
  for (int i = threadIdx.x; i < V3L_CNT / 16; i += NTHREADS)
    reinterpret_cast<f32x4*>(lds)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = V3L_XDEC / 16 + (int)threadIdx.x; i < PL.lds3_bytes / 16; i += NTHREADS)
    reinterpret_cast<f32x4*>(lds)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();   // zeroing done before the staged rows land in CTX
  {
    const int cm = C - 1;
    if (t4 < L0 * C) *reinterpret_cast<f32x4*>(IN + (t4 >> PL.C_shift) * CS + (t4 & cm)) = xe4;
    if (XE && t4 < Ld * C) *reinterpret_cast<f32x4*>(XDEC + (t4 >> PL.C_shift) * CS + (t4 & cm)) = xd4;
  }

  constexpr int FRAGS_PER_TILE4 = 4 * WAVE;   // bf16x8 per n-tile at K = 128
  Res<MT> X;
  // diagnostics: s_memtime at phase boundaries (wave 0, lane 0), off unless a.stamps is set
  unsigned long long* stamps = DIAG && a.stamps ? a.stamps + (size_t)b * MAX_STAMPS : nullptr;
  int sid = 0;
  auto STAMP = [&]() {
    if (stamps) {
      if (threadIdx.x == 0 && sid < MAX_STAMPS) stamps[sid] = __builtin_amdgcn_s_memtime();
      ++sid;
    }
  };
  if (a.mt_in && !a.cnt) {
    __syncthreads();   // LDS zeroing above is done before the state lands in it
    mt_load<NTHREADS>(gen, a.mt_in);
  }   // device-resident sampler (cet_mt.hpp)
  auto FINE = [&](int layer, int k) {
    if (stamps && layer == 0 && threadIdx.x == 0) stamps[116 + k] = __builtin_amdgcn_s_memtime();
  };
  STAMP();

  // one head per wave; MQc / MKc: compile-time bounds on the query / key tiles
  auto attend = [&](auto MQc, auto MKc, const __bf16* Xq, const __bf16* Xkv, uint32_t Wq, uint32_t Wk,
                    uint32_t Wv, GemmDesc dq, GemmDesc dk, GemmDesc dv, int LQ, int LK, int prob, int causal,
                    int mix, int call, float* attn_out) {
    constexpr int MQ_ = decltype(MQc)::value, MK_ = decltype(MKc)::value;
    HeadIO io;
    io.Xq = Xq; io.Xkv = Xkv; io.wq = Wq; io.wk = Wk; io.wv = Wv;
    io.dq = dq; io.dk = dk; io.dv = dv;
    io.ctx = CTX; io.LQ = LQ; io.LK = LK; io.prob = prob; io.causal = causal; io.mix = mix; io.u = LQ;
    io.cnt = nullptr; io.cnt_stride = 0; io.scr = SCR; io.attn_out = attn_out; io.m_dbg = nullptr;
    io.st = (stamps && call >= 0 && call < 2) ? stamps + 100 + 8 * call : nullptr;
    if (call >= 0) {
      const AttnCall& c = PL.calls[call];
      io.u = c.u;
      io.cnt_stride = c.cnt_stride;
      if (dbg && c.m_dbg >= 0) io.m_dbg = dbg + c.m_dbg;
      const bool sparse = c.u < c.LQ;
      if (!a.cnt) {
        // resident sampler: replay this call's draws into the LDS table (cet_mt.hpp)
        mt_replay<NTHREADS>(gen, c.LQ, c.U, c.LK, sparse ? reinterpret_cast<uint32_t*>(CNT) : nullptr,
                            c.cnt_stride);
        if (call == PL.n_calls - 1 && b == 0) mt_store<NTHREADS>(gen, a.mt_out);
      } else if (sparse) {
        const int bytes = ((c.LQ + 15) & ~15) * c.cnt_stride;
        const f32x4* src = reinterpret_cast<const f32x4*>(a.cnt + c.cnt_off);
        f32x4* dst = reinterpret_cast<f32x4*>(CNT);
        for (int i = threadIdx.x; i < bytes / 16; i += NTHREADS) dst[i] = src[i];
        __syncthreads();
      }
      if (sparse) io.cnt = CNT;
    }
#ifndef V3_NO_ATTN
    attention_head<MQ_, MK_>(io, M, w);
#endif
  };

  auto ESTAMP = [&](int k) {   // embedding sub-phases of encoder 0 (slots 124..126)
    if (stamps && threadIdx.x == 0) stamps[124 + k] = __builtin_amdgcn_s_memtime();
  };
  for (int e = 0; e < PL.n_enc; ++e) {
    if (e > 0) stage(a.x_enc + (size_t)b * L0 * C, IN, L0, C, CS);   // CTX was reused by encoder e-1
    __syncthreads();
    if (e == 0) ESTAMP(0);
    // ---- DataEmbedding (embed.py:132-135) on the EncoderStack window x[:, -L:] (encoder.py:95-106)
    int L = L0 >> e;
    const int off = L0 - L;
    int nmt = (L + 15) >> 4;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) X.v[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      const GemmDesc d = PL.emb_enc;
      gemm_res<2, MT>(M, d, nmt, LoadEmbedOff{IN, L0, PL.C_shift, CS, off}, [&](int mt, int n0, f32x4 y) {
        const int m = mt * 16 + (lane_op() & 15);
        const int prow = m + off < LMAX ? m + off : LMAX - 1;
        X.v[mt] = y + pload4(M, PL.pe_enc, prow * DMODEL + n0);
      });
    }
    if (e == 0) ESTAMP(1);
    __syncthreads();                       // IN (aliases CTX) fully read
    store_res(X, nmt, L, Xb);
    __syncthreads();
    if (dbg && e == 0) dump_res(X, nmt, L, dbg + PL.dbg_emb);
    STAMP();  // embedding

    const int first = PL.enc_first[e];
    for (int l = 0; l < PL.enc_layers[e]; ++l) {
      L = ELD.L_in;
      nmt = (L + 15) >> 4;
      // ---- AttentionLayer + ProbAttention / FullAttention, one head per wave, context → CTX
      {
        const GemmDesc q = ELD.qkv;
        // instantiated for the layer's compile-time tile bound (distilled layers: 3, 2, 1 tiles)
        auto enc_attend = [&](auto NQ) __attribute__((always_inline)) {
          attend(NQ, NQ, Xb, Xb, q.w, q.w + 8 * FRAGS_PER_TILE4, q.w + 16 * FRAGS_PER_TILE4, part_of(q, 0),
                 part_of(q, 128), part_of(q, 256), L, L, PL.prob, 0, 0, ELD.call,
                 DIAG && a.attns ? a.attns + ELD.attn_off + (size_t)b * ELD.attn_stride : nullptr);
        };
        switch (nmt) {
          case 1: enc_attend(IC<1>{}); break;
          case 2: enc_attend(IC<2>{}); break;
          case 3: enc_attend(IC<3>{}); break;
          default: enc_attend(IC<MT>{}); break;
        }
      }
      const WPre<4> po = prefetch_res<4>(M, ELD.o);   // x = x + new_x (encoder.py:49)
      __syncthreads();
      STAMP();  // encoder attention
      gemm_res<4, MT>(po, nmt, LoadBF16{CTX}, [&](int mt, int n0, f32x4 y) { X.v[mt] += y; });
      FINE(l, 0);
      static_assert(DFF / 16 <= NW, "FFN hidden n-tiles: at most one per wave");
      const WPre<4> pf1 = prefetch_tiles<4>(M, ELD.f1, DFF / 16);   // conv1 (k=1) + activation (encoder.py:52)
      ln_res(X, nmt, L, M, ELD.ln1, 1e-5f, false, LNP, Xb);
      __syncthreads();
      STAMP();  // out-projection + LN1
      {
        const int relu = PL.act_relu;
        gemm_tiles1<4>(pf1, DFF / 16, nmt, LoadBF16{Xb}, [&](int mt, int n0, f32x4 v) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = relu ? fmaxf(v[r], 0.f) : gelu_erf(v[r]);
          *reinterpret_cast<bf16x4*>(CTX + (mt * 16 + (lane_op() & 15)) * BS + n0) = cvt4(v);
        });
      }
      FINE(l, 1);
      const WPre<DFF / 32> pf2 = prefetch_res<DFF / 32>(M, ELD.f2);  // conv2 (k=1) + residual (encoder.py:53-56)
      __syncthreads();
      FINE(l, 2);
      gemm_res<DFF / 32, MT>(pf2, nmt, LoadBF16{CTX}, [&](int mt, int n0, f32x4 y) { X.v[mt] += y; });
      FINE(l, 3);
      const int has_conv = ELD.conv.n;
#ifdef V3_PREFETCH_CONV
      WPre<4> pcv;
      if (has_conv) pcv = prefetch_kouter<12, 4>(M, ELD.conv);
#endif
      ln_res(X, nmt, L, M, ELD.ln2, 1e-5f, false, LNP, Xb);
      __syncthreads();
      STAMP();  // FFN + LN2
      if (dbg && ELD.dbg_layer >= 0) dump_res(X, nmt, L, dbg + ELD.dbg_layer);
      FINE(l, 4);
#ifndef V3_NO_CONV
      if (has_conv) {
        // ---- ConvLayer (encoder.py:22-28): circular conv, BN(eval) folded, ELU, MaxPool(3,2,1).
        // The conv output lives inside each m-tile-count instantiation and only X leaves it.
        const GemmDesc d = ELD.conv;
        with_nmt(nmt, [&](auto NMT) __attribute__((always_inline)) {
          constexpr int N_ = decltype(NMT)::value;
          Res<N_> Cv;
#ifndef V3_PREFETCH_CONV
          const WPre<4> pcv = prefetch_kouter<12, 4>(M, d);
#endif
          gemm_kouter_res<12, 4, N_>(pcv, M, d, LoadCirc3BF16{Xb, L},
                                     [&](int mt, int n0, f32x4 v) __attribute__((always_inline)) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = elu1(v[r]);
            Cv.v[mt] = v;
          });
          FINE(l, 5);
          maxpool_res<N_>(Cv, L, X);
        });
        FINE(l, 6);
        L = ELD.L_out;
        nmt = (L + 15) >> 4;
        __syncthreads();                   // every wave finished reading Xb
        FINE(l, 7);
        store_res(X, nmt, L, Xb);
        __syncthreads();
        STAMP();  // distil conv + pool
        if (dbg && ELD.dbg_conv >= 0) dump_res(X, nmt, L, dbg + ELD.dbg_conv);
      }
#endif
    }
    // ---- Encoder.norm (encoder.py:83-84) → this encoder's rows of the stack output (ENC)
    const int rows = PL.enc_rows[e];
    ln_res(X, nmt, rows, M, PL.enc_norm[e], 1e-5f, false, LNP, Xb,
           ENC + PL.enc_row_off[e] * BS);
    __syncthreads();
    if (dbg && PL.enc_dbg[e] >= 0) dump_res(X, nmt, rows, dbg + PL.enc_dbg[e]);
    STAMP();  // encoder norm
  }

  // ================================ decoder (decoder.py:43-56), instantiated for its compile-time
  // tile count (dec_len ≤ 48)
  const int S = PL.S;
  if (!XE) {   // no room to keep it since entry: stage it now (into CTX)
    stage(a.x_dec + (size_t)b * Ld * C, XDEC, Ld, C, CS);
    __syncthreads();
  }
  // NMSc: compile-time bound on the cross-attention key tiles (the encoder-stack output rows)
  auto decoder = [&](auto NMDc, auto NMSc) __attribute__((always_inline)) {
    constexpr int NMS = decltype(NMSc)::value;
    constexpr int NMD = decltype(NMDc)::value;
    const int nmd = NMD;
    Res<NMD> XD;
    {
      const GemmDesc d = PL.emb_dec;
      gemm_res_n<2, NMD>(M, d, LoadEmbedOff{XDEC, Ld, PL.C_shift, CS, 0}, [&](int mt, int n0, f32x4 y) {
        const int m = mt * 16 + (lane_op() & 15);
        const int prow = m < LMAX ? m : LMAX - 1;
        XD.v[mt] = y + pload4(M, PL.pe_dec, prow * DMODEL + n0);
      });
    }
    __syncthreads();
    store_res(XD, nmd, Ld, Xb);
    __syncthreads();
    if (dbg) dump_res(XD, nmd, Ld, dbg + PL.dbg_dec_emb);
    STAMP();  // decoder embedding

    for (int l = 0; l < PL.d_layers; ++l) {
      {
        // masked self-attention with the mix scramble (model.py:211-222)
        const GemmDesc q = DLD.qkv;
        attend(IC<NMD>{}, IC<NMD>{}, Xb, Xb, q.w, q.w + 8 * FRAGS_PER_TILE4, q.w + 16 * FRAGS_PER_TILE4,
               part_of(q, 0), part_of(q, 128), part_of(q, 256), Ld, Ld, PL.prob, 1, PL.mix, DLD.call, nullptr);
      }
      const WPre<4> po = prefetch_res<4>(M, DLD.o);
      __syncthreads();
      STAMP();  // decoder self-attention
      gemm_res_n<4, NMD>(po, LoadBF16{CTX}, [&](int mt, int n0, f32x4 y) { XD.v[mt] += y; });
      ln_res(XD, nmd, Ld, M, DLD.ln1, 1e-5f, false, LNP, Xb);
      __syncthreads();
      {
        // cross-attention: FullAttention over the encoder-stack output, mix=False
        const GemmDesc cq = DLD.cq, ckv = DLD.ckv;
        attend(IC<NMD>{}, IC<NMS>{}, Xb, ENC, cq.w, ckv.w, ckv.w + 8 * FRAGS_PER_TILE4, part_of(cq, 0),
               part_of(ckv, 0), part_of(ckv, 128), Ld, S, 0, 0, 0, -1, nullptr);
      }
      const WPre<4> pco = prefetch_res<4>(M, DLD.co);
      __syncthreads();
      STAMP();  // cross-attention
      gemm_res_n<4, NMD>(pco, LoadBF16{CTX}, [&](int mt, int n0, f32x4 y) { XD.v[mt] += y; });
      const WPre<4> pf1 = prefetch_tiles<4>(M, DLD.f1, DFF / 16);
      ln_res(XD, nmd, Ld, M, DLD.ln2, 1e-5f, false, LNP, Xb);
      __syncthreads();
      {
        const int relu = PL.act_relu;
        gemm_tiles1<4>(pf1, DFF / 16, nmd, LoadBF16{Xb}, [&](int mt, int n0, f32x4 v) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = relu ? fmaxf(v[r], 0.f) : gelu_erf(v[r]);
          *reinterpret_cast<bf16x4*>(CTX + (mt * 16 + (lane_op() & 15)) * BS + n0) = cvt4(v);
        });
      }
      const WPre<DFF / 32> pf2 = prefetch_res<DFF / 32>(M, DLD.f2);
      __syncthreads();
      gemm_res_n<DFF / 32, NMD>(pf2, LoadBF16{CTX}, [&](int mt, int n0, f32x4 y) { XD.v[mt] += y; });
      ln_res(XD, nmd, Ld, M, DLD.ln3, 1e-5f, false, LNP, Xb);
      __syncthreads();
      STAMP();  // decoder O/LN1 + cross O/LN2 + FFN/LN3
      if (dbg && DLD.dbg >= 0) dump_res(XD, nmd, Ld, dbg + DLD.dbg);
    }
    ln_res(XD, nmd, Ld, M, PL.dec_norm, 1e-5f, false, LNP, Xb);
    __syncthreads();
    if (dbg) dump_res(XD, nmd, Ld, dbg + PL.dbg_dec_out);
    {
      // projection (model.py:264) on the last pred_len rows → out[b]
      const GemmDesc d = PL.proj;
      const int first_row = Ld - PL.pred_len, co = PL.c_out;
      float* out = a.out + (size_t)b * PL.pred_len * co;
      gemm_tiles<4>(M, d, d.n / 16, nmd, LoadBF16{Xb}, [&](int mt, int n0, f32x4 v) {
        const int m = mt * 16 + (lane_op() & 15);
        if (m < first_row || m >= Ld) return;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n0 + r < co) out[(m - first_row) * co + n0 + r] = v[r];
      });
    }
    STAMP();  // final norm + projection
  };
#ifndef V3_NO_DEC
  switch ((Ld + 15) >> 4) {
    case 1: S <= 16 ? decoder(IC<1>{}, IC<1>{}) : decoder(IC<1>{}, IC<MT>{}); break;
    case 2: S <= 16 ? decoder(IC<2>{}, IC<1>{}) : decoder(IC<2>{}, IC<MT>{}); break;
    default: S <= 16 ? decoder(IC<3>{}, IC<1>{}) : decoder(IC<3>{}, IC<MT>{}); break;
  }
#endif
  // ---- the first workgroup to finish prepares the NEXT forward's ProbSparse tables from the
  //      resident sampler state (cet_sampler.hpp) while the rest of the grid drains; the last
  //      one to finish re-arms the counter for the next launch
  if (a.ticket) {
    __syncthreads();
    unsigned* tk = reinterpret_cast<unsigned*>(lds + V3L_SCR);
    if (threadIdx.x == 0) {
      const unsigned t = atomicAdd(a.ticket, 1u);
      if (t + 1u == (unsigned)a.B) atomicExch(a.ticket, 0u);
      *tk = t;
    }
    __syncthreads();
    const bool elected = __builtin_amdgcn_readfirstlane(*tk) == 0u;
    __syncthreads();   // every wave has read the ticket before the replay reuses the LDS
    if (elected && a.cnt_next)
      replay_all<NTHREADS>(PL, a.mt_in, a.mt_out, a.cnt_next, lds, PL.lds3_bytes,
                           reinterpret_cast<uint32_t*>(lds + V3L_MT), reinterpret_cast<uint32_t*>(lds + V3L_CNT));
  }
}

#undef PL
#undef ELD
#undef DLD

}  // namespace v3
}  // namespace cet

extern "C" int cet_launch_informer_v3(const cet::InformerArgs* a, int dff, int lds_bytes, int xdec_early,
                                      hipStream_t stream) {
  using namespace cet;
  if (a->B <= 0) return 0;
  auto launch = [&](void (*kern)(InformerArgs, const InformerPlan*), int) -> int {
    if (!ensure_lds_attr(reinterpret_cast<const void*>(kern))) return -1;
    hipLaunchKernelGGL(kern, dim3(a->B), dim3(v3::NTHREADS), lds_bytes, stream, *a, a->plan);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  };
  const bool diag = a->attns || a->dbg || a->stamps;
  const int slot = (dff == 128 ? 4 : 0) + (diag ? 2 : 0) + (xdec_early ? 1 : 0);
  using K = void (*)(InformerArgs, const InformerPlan*);
  static const K kerns[8] = {v3::informer_forward_v3<64, false, false>,  v3::informer_forward_v3<64, false, true>,
                             v3::informer_forward_v3<64, true, false>,   v3::informer_forward_v3<64, true, true>,
                             v3::informer_forward_v3<128, false, false>, v3::informer_forward_v3<128, false, true>,
                             v3::informer_forward_v3<128, true, false>,  v3::informer_forward_v3<128, true, true>};
  if (dff != 64 && dff != 128) return -3;
  return launch(kerns[slot], slot);
}

namespace cet {
namespace v3 {
// One-workgroup table preparation for the first forward after a (re)seed.
__global__ void __launch_bounds__(NTHREADS) sampler_prep(const InformerPlan* plan, const uint32_t* mt_in,
                                                         uint32_t* mt_out, uint8_t* tab_out, int lds_bytes) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  replay_all<NTHREADS>(*plan, mt_in, mt_out, tab_out, lds, lds_bytes, reinterpret_cast<uint32_t*>(lds),
                       reinterpret_cast<uint32_t*>(lds + MT_WORDS * 4));
}
}  // namespace v3
}  // namespace cet

extern "C" int cet_launch_sampler_prep(const cet::InformerPlan* plan, const uint32_t* mt_in, uint32_t* mt_out,
                                       uint8_t* tab_out, int lds_bytes, hipStream_t stream) {
  hipLaunchKernelGGL(cet::v3::sampler_prep, dim3(1), dim3(cet::v3::NTHREADS), lds_bytes, stream, plan, mt_in, mt_out,
                     tab_out, lds_bytes);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
