// One-wave-per-head attention for the fused kernels (ProbSparse and full).
//
// Reference semantics (FullPrecision/InformerModel/attn.py):
//  * ProbAttention.forward :148-175 — U_part / u = min(factor·ceil(ln L), L);
//    _prob_QK :89-114 — M[q] = max_j QK_sample[q,j] − Σ_j QK_sample[q,j] / L_K over the
//    U sampled keys (with multiplicity), then top-u queries;
//    _get_initial_context :116-125 — mean(V) (unmasked) or cumsum(V) (masked);
//    _update_context :127-146 — softmax(scale·q·Kᵀ) (ProbMask: key > query → −inf) · V
//    written into the selected rows; attns rows = attn, other rows 1/L_K.
//  * FullAttention.forward :52-70 — softmax(scale·QKᵀ [causal mask]) · V.
//  * AttentionLayer mix (:205-207) — output (B,L,H,E) viewed as (B,H,L,E) memory.
//
// The sampled-key multiplicities cnt[q][key] (from the host's torch-compatible index
// draw) turn the gather into a masked reduction over a full Sᵀ = K·Qᵀ tile computed on
// MFMA: Σ_j QK_sample = Σ_key cnt·S and max_j QK_sample = max_{cnt>0} S.
#pragma once
#include "cet_device.hpp"

namespace cet {

struct AttnIO {
  const __bf16* Q;        // LDS [LQ rows][BS]; head h occupies columns 16h..16h+15
  const __bf16* K;        // LDS [LK rows][BS]
  const __bf16* Vt;       // LDS [128][vts]  (V transposed: feature-major)
  int vts;
  __bf16* ctx;            // LDS [LQ][BS] output (may alias Q when !mix)
  int LQ, LK;
  int prob;               // 1: ProbSparse, 0: full attention
  int causal;             // mask_flag of the reference (decoder self-attention)
  int mix;                // AttentionLayer(mix=True) output scramble
  int u;                  // selected queries (prob); LQ for full
  const uint8_t* cnt;     // global [>= round16(LQ)][cnt_stride] key multiplicities (prob && u < LQ)
  int cnt_stride;
  float* Msh;             // LDS scratch [8][96]
  int16_t* sel;           // LDS scratch [8][96]
  uint8_t* flag;          // LDS scratch [8][96]
  float* attn_out;        // global [H][LQ][LK] for this sequence, or nullptr
  float* m_dbg;           // global [H][LQ] debug dump of M, or nullptr
};

constexpr int SCR = 96;   // per-head scratch entries (max padded L)

__device__ __forceinline__ void store_ctx4(__bf16* ctx, int mix, int LQ, int h, int q, int e0, const f32x4& v) {
  int off;
  if (!mix) {
    off = q * BS + h * 16 + e0;
  } else {
    const int f = h * LQ * 16 + q * 16 + e0;  // (L,H,E) values re-viewed as (H,L,E) memory
    off = (f >> 7) * BS + (f & 127);
  }
  *reinterpret_cast<bf16x4*>(ctx + off) = cvt4(v);
}

__device__ __forceinline__ bf16x4 ld_frag4(const __bf16* p) { return *reinterpret_cast<const bf16x4*>(p); }

// Executed by ONE wave for head h.  No workgroup barrier inside.
__device__ void attention_head(const AttnIO& io, int h) {
  const int lane = lane_id();
  const int col = lane & 15;   // query column of the S^T tile / row of A fragments
  const int grp = lane >> 4;   // 0..3
  const int LQ = io.LQ, LK = io.LK;
  const int nkt = (LK + 15) >> 4;
  const int nqt = (LQ + 15) >> 4;
  float* Msh = io.Msh ? io.Msh + h * SCR : nullptr;        // scratch: sparse mode only
  int16_t* sel = io.sel ? io.sel + h * SCR : nullptr;
  uint8_t* flag = io.flag ? io.flag + h * SCR : nullptr;
  const int hc = h * 16 + grp * 4;  // this lane's 4 head features in fragment loads
  const bool sparse = io.prob && io.u < LQ;
  const int nsel = sparse ? io.u : LQ;

  if (sparse) {
    // ---- sparsity measurement M for every query (attn.py:95-105)
    for (int qt = 0; qt < nqt; ++qt) {
      const int q = qt * 16 + col;
      const bf16x4 bq = ld_frag4(io.Q + q * BS + hc);
      const uint8_t* crow = io.cnt + (size_t)q * io.cnt_stride + grp * 4;
      float sum = 0.f, mx = NEG_INF;
      for (int kt = 0; kt < nkt; ++kt) {
        const bf16x4 ak = ld_frag4(io.K + (kt * 16 + col) * BS + hc);
        const f32x4 s = mfma16x16x16(ak, bq, f32x4{0.f, 0.f, 0.f, 0.f});
        const uint32_t cw = *reinterpret_cast<const uint32_t*>(crow + kt * 16);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // select, never multiply: rows past L hold stale bytes (the distil conv output
          // aliases Q/K in LDS) that can decode as bf16 NaN/Inf, and 0·NaN = NaN
          const uint32_t c = (cw >> (8 * r)) & 0xffu;
          sum = c ? fmaf((float)c, s[r], sum) : sum;
          mx = c ? fmaxf(mx, s[r]) : mx;
        }
      }
      sum = xor_sum(sum, 16); sum = xor_sum(sum, 32);
      mx = xor_max(mx, 16); mx = xor_max(mx, 32);
      const float M = mx - sum / (float)LK;
      if (grp == 0 && q < LQ) {
        Msh[q] = M;
        if (io.m_dbg) io.m_dbg[h * LQ + q] = M;
      }
    }
    wave_lds_sync();
    // ---- top-u by rank (ties: lower index first)
    for (int q = lane; q < LQ; q += WAVE) {
      const float mq = Msh[q];
      int rank = 0;
      for (int k = 0; k < LQ; ++k) {
        const float mk = Msh[k];
        rank += (mk > mq) || (mk == mq && k < q);
      }
      const bool s = rank < io.u;
      flag[q] = s;
      if (s) sel[rank] = (int16_t)q;
    }
    wave_lds_sync();
  }

  // ---- softmax(scale·q·Kᵀ)·V for the selected queries (attn.py:109-112, 127-138 / 57-65)
  const float scale = 0.25f;  // 1/sqrt(E), E = 16
  const int nst = (nsel + 15) >> 4;
  for (int st = 0; st < nst; ++st) {
    const int i = st * 16 + col;
    const int ic = i < nsel ? i : nsel - 1;
    const int qi = sparse ? (int)sel[ic] : ic;
    const bf16x4 bq = ld_frag4(io.Q + qi * BS + hc);
    f32x4 s[6];
    float mx = NEG_INF;
#pragma unroll
    for (int kt = 0; kt < 6; ++kt) {
      if (kt < nkt) {
        const bf16x4 ak = ld_frag4(io.K + (kt * 16 + col) * BS + hc);
        s[kt] = mfma16x16x16(ak, bq, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt * 16 + grp * 4 + r;
          const bool masked = key >= LK || (io.causal && key > qi);
          s[kt][r] = masked ? NEG_INF : s[kt][r] * scale;
          mx = fmaxf(mx, s[kt][r]);
        }
      }
    }
    mx = xor_max(mx, 16); mx = xor_max(mx, 32);
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 6; ++kt) {
      if (kt < nkt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[kt][r] = __expf(s[kt][r] - mx);
          sum += s[kt][r];
        }
      }
    }
    sum = xor_sum(sum, 16); sum = xor_sum(sum, 32);
    const float inv = 1.0f / sum;
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 6; ++kt) {
      if (kt < nkt) {
        const bf16x4 av = ld_frag4(io.Vt + (h * 16 + col) * io.vts + kt * 16 + grp * 4);
        o = mfma16x16x16(av, cvt4(s[kt]), o);
      }
    }
    // o: rows e = 4·grp + r, column = this lane's query
    // (the O tile's column index is the lane's col, rows are features) -> lane holds 4 features
    if (i < nsel) {
      store_ctx4(io.ctx, io.mix, LQ, h, qi, grp * 4, o * inv);
      if (io.attn_out) {
        float* arow = io.attn_out + ((size_t)h * LQ + qi) * LK;
#pragma unroll
        for (int kt = 0; kt < 6; ++kt) {
          if (kt < nkt) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int key = kt * 16 + grp * 4 + r;
              if (key < LK) arow[key] = s[kt][r] * inv;
            }
          }
        }
      }
    }
  }

  if (sparse) {
    // ---- rows that were not selected keep the initial context (attn.py:116-125)
    const int e = col;
    const __bf16* vrow = io.Vt + (h * 16 + e) * io.vts;
    if (!io.causal) {
      float part = 0.f;
      for (int k = grp; k < LK; k += 4) part += (float)vrow[k];
      part = xor_sum(part, 16); part = xor_sum(part, 32);
      const float mean = part / (float)LK;
      for (int qb = 0; qb < LQ; qb += 4) {
        const int q = qb + grp;
        if (q < LQ && !flag[q]) {
          int off;
          if (!io.mix) off = q * BS + h * 16 + e;
          else { const int f = h * LQ * 16 + q * 16 + e; off = (f >> 7) * BS + (f & 127); }
          io.ctx[off] = (__bf16)mean;
        }
      }
    } else if (grp == 0) {
      float run = 0.f;
      for (int q = 0; q < LQ; ++q) {
        run += (float)vrow[q];
        if (!flag[q]) {
          int off;
          if (!io.mix) off = q * BS + h * 16 + e;
          else { const int f = h * LQ * 16 + q * 16 + e; off = (f >> 7) * BS + (f & 127); }
          io.ctx[off] = (__bf16)run;
        }
      }
    }
    if (io.attn_out) {
      const float invL = 1.0f / (float)LK;
      for (int q = 0; q < LQ; ++q) {
        if (!flag[q]) {
          float* arow = io.attn_out + ((size_t)h * LQ + q) * LK;
          for (int k = lane; k < LK; k += WAVE) arow[k] = invL;
        }
      }
    }
  }
}

}  // namespace cet
