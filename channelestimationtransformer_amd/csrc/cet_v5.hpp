// "v5" building blocks: the v4 scheme (8 waves, wave w owns residual n-tile w and attention head w,
// the residual stream in registers) carrying NS sequences per workgroup.
//
// v4 puts ONE sequence in a 512-thread workgroup and two workgroups on a CU, at 128 VGPRs: every
// workgroup streams the whole weight blob from its XCD's L2 (2 MB per sequence), every LayerNorm and
// phase hand-off is a barrier of its own, and the register cap spills (profiles/r02).  v5 stacks the
// sequences of a CU under each weight fragment instead:
//   * a weight fragment fetched once feeds the MFMAs of all NS sequences (half the L2 traffic at NS = 2);
//   * one workgroup barrier serves every sequence (half the barriers per sequence);
//   * each wave interleaves NS independent dependency chains (the second sequence hides the first's
//     latencies instead of a second workgroup doing it through the SIMD arbiter);
//   * 256 VGPRs per wave (one workgroup per CU): no spills, room for the operand prefetches.
// Per-sequence state lives in arrays indexed by a compile-time sequence slot s < NS, so every LDS offset
// still folds into ds_* immediates.
//
// Reference: FullPrecision/InformerModel/attn.py:73-209, encoder.py:6-56, decoder.py:6-40.
#pragma once
#include "cet_v4.hpp"

namespace cet {
namespace v5 {

using namespace cet::v4;

// ------------------------------------------------------------------ LDS layout (compile time)
// per sequence: image XB | context CTX (also the staged input rows and the projection input) | the
// waves' attention scratch (aliased by the LayerNorm partials); then, shared by the sequences, the
// ProbSparse multiplicity table; then the plan-sized regions (cet_api.cpp plan_informer: the stack
// outputs, the staged decoder inputs and labels, the sampler state).
template <int P>
struct L5 {
  static_assert(P != P_X3, "split-bf16 operands need 256 VGPRs for one sequence: v4 only");
  static constexpr int IMG = v4_img(P);
  static constexpr int CTXB = v4_ctx_bytes(P);
  static constexpr int SCRB = 8 * V2_SCR_FLOATS * 4;
  static constexpr int SEQ = v5_seq(P);
  static constexpr int xb(int s) { return s * SEQ; }
  static constexpr int ctx(int s) { return s * SEQ + IMG; }
  static constexpr int scr(int s) { return s * SEQ + IMG + CTXB; }
  static constexpr int cnt(int ns) { return ns * SEQ; }
  static_assert(SEQ == IMG + CTXB + SCRB && v5_fixed(P, 2) == cnt(2) + LMAX * 96, "cet_plan.hpp v5 layout");
  static_assert(IMG % 16 == 0 && CTXB % 16 == 0 && SCRB % 16 == 0, "16-B regions");
};

// Workgroup barrier that is also a full compiler memory barrier: every cross-wave hand-off in v5 goes
// through LDS between two barriers, and the asm clobbers keep the optimiser from moving any memory
// access across one.
__device__ __forceinline__ void wg_sync() {
  asm volatile("" ::: "memory");
  __syncthreads();
  asm volatile("" ::: "memory");
}

// Lane-axis butterflies of v5 on ds_bpermute (__shfl_xor), not v_permlane16/32_swap.  In this kernel
// the compiler moved permlane-swap reductions below the point where EXEC narrows to the lanes that
// store the result (e.g. the fused-NMSE epilogue: the swaps ran after s_and_saveexec, so the partner
// lanes were inactive).  The symptom was a 1e-4 deviation of the first sequence slot whose configurations
// changed from build to build, with the result varying from run to run; the attention's reductions were
// the ones hit (bisected by call site).  ds_bpermute is a convergent operation the compiler keeps where
// it is written: every configuration then equals v4 bit for bit.
__device__ __forceinline__ float bp_sum(float v, int m) { return v + __shfl_xor(v, m, 64); }
__device__ __forceinline__ float bp_max(float v, int m) { return fmaxf(v, __shfl_xor(v, m, 64)); }

// ------------------------------------------------------------------ dense layers over NS sequences
// Output n-tile w of every sequence's residual; the weight fragments p are shared.  bl(s, m, k0) loads
// sequence s's B fragment, epi(s, mt, n0, y) consumes its accumulator.
template <int P, int KS, int N, int NS, class BL, class Epi>
__device__ __forceinline__ void gemm_res_s(const WPre<P, KS>& p, int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_op(), w = wave_id();
  const int n0 = 16 * w + (lane >> 4) * 4;
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      f32x4 c[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) c[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int s = 0; s < NS; ++s) c[s] = mma<P>(&p.a[ks], bl(s, mt * 16 + mrow, ks * 32 + kq), c[s]);
#pragma unroll
      for (int s = 0; s < NS; ++s) epi(s, mt, n0, c[s] * p.sc + p.bi);
    }
  }
}

// Dense layer over n_tiles ≤ NW n-tiles (the FFN hidden layer): the (m-tile, sequence) items of an
// n-tile are spread over the NW / n_tiles waves that share it.
template <int P, int KS, int NS, class BL, class Epi>
__device__ __forceinline__ void gemm_tiles1_s(const WPre<P, KS>& p, int n_tiles, int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_op(), w = wave_id();
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
  const int per = NW / n_tiles;
  if (w >= per * n_tiles) return;
  const int nt = w % n_tiles, mt_step = per;
  const int n0 = nt * 16 + (lane >> 4) * 4;
  for (int mt = w / n_tiles; mt < nmt; mt += mt_step) {
    f32x4 c[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) c[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int s = 0; s < NS; ++s) c[s] = mma<P>(&p.a[ks], bl(s, mt * 16 + mrow, ks * 32 + kq), c[s]);
#pragma unroll
    for (int s = 0; s < NS; ++s) epi(s, mt, n0, c[s] * p.sc + p.bi);
  }
}

// Dense layer over an arbitrary n-tile count (the projection): (n-tile, m-tile, sequence) items
// round-robin over the waves, output through epi only.
template <int P, int KS, int NS, class BL, class Epi>
__device__ __forceinline__ void gemm_tiles_s(const Mem& m, const GemmDesc d, int n_tiles, int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_op(), w = wave_id();
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
  const int items = n_tiles * nmt * NS;
  for (int it = w; it < items; it += NW) {
    const int s = it % NS, r = it / NS;
    const int nt = r % n_tiles, mt = r / n_tiles;
    WF<P> a[KS];
    load_frags<P, KS>(m, d.w, nt, a);
    const int n0 = nt * 16 + (lane >> 4) * 4;
    f32x4 sc, bi;
    epi_vecs(m, d, n0, sc, bi);
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) c = mma<P>(&a[ks], bl(s, mt * 16 + mrow, ks * 32 + kq), c);
    epi(s, mt, n0, c * sc + bi);
  }
}

// Deep-K dense layer (the distil conv, K = 384) in k-outer order with a compile-time m-tile count, for
// NS sequences: one accumulator per (sequence, m-tile), B fragments one k-step ahead, the weight
// fragments fetched in groups of KH k-steps and shared by the sequences.
template <int P, int KS, int KH, int NMT, int NS, class BL, class Epi>
__device__ __forceinline__ void gemm_kouter_s(const WPre<P, KH>& p, const Mem& m, const GemmDesc d, BL&& bl,
                                              Epi&& epi) {
  static_assert(KS % KH == 0, "k-steps split into equal groups");
  const int lane = lane_op(), w = wave_id();
  const int kq = (lane >> 4) * 8, mrow = lane & 15;
  const int n0 = 16 * w + (lane >> 4) * 4;
  f32x4 c[NS][NMT];
  XF<P> b[NS][NMT];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) {
      c[s][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      b[s][mt] = bl(s, mt * 16 + mrow, kq);
    }
  const uint32_t t0 = d.w * 16u + (uint32_t)(w * KS) * 1024u;
#pragma unroll
  for (int hf = 0; hf < KS / KH; ++hf) {
    WF<P> a[KH];
#pragma unroll
    for (int ks = 0; ks < KH; ++ks) a[ks] = hf == 0 ? p.a[ks] : wfrag<P>(m, t0 + (uint32_t)(hf * KH + ks) * 1024u, lane);
#pragma unroll
    for (int ks = 0; ks < KH; ++ks) {
      const int kk = hf * KH + ks;
      XF<P> bn[NS][NMT];
      if (kk + 1 < KS) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int mt = 0; mt < NMT; ++mt) bn[s][mt] = bl(s, mt * 16 + mrow, (kk + 1) * 32 + kq);
      }
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
        for (int s = 0; s < NS; ++s) c[s][mt] = mma<P>(&a[ks], b[s][mt], c[s][mt]);
      if (kk + 1 < KS) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int mt = 0; mt < NMT; ++mt) b[s][mt] = bn[s][mt];
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch distance at one k-step
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) epi(s, mt, n0, c[s][mt] * p.sc + p.bi);
}

// LayerNorm of NS register residuals over all 128 features (8 waves × 16), v4's three steps with one
// pair of workgroup barriers for every sequence: (1) per-wave (mean, M2) partials of each row into the
// sequence's partial area (part(s)); (2) the (sequence, m-tile) items, one per wave in turn, combine a
// row's 8 pairs (Chan) into (mean, 1/std); (3) every wave normalises its fragments.  Normalised rows go
// to X (INPLACE) and rows < `rows` through out(s, m, n0, y).  unbiased_std: the reference Transformer's
// LayerNormalization (buildingblocks.py:23-30) instead of torch.nn.LayerNorm.
template <int NS, int N, bool INPLACE = true, class Part, class Out>
__device__ __forceinline__ void ln_res_s(Res<N> (&X)[NS], int nmt, int rows, const Mem& mm, const LNDesc ln,
                                         float eps, bool unbiased_std, Part&& part, Out&& out) {
  const int lane = lane_op(), w = wave_id(), g = lane >> 4, c = lane & 15;
  const int nb = 16 * w + 4 * g;
  const f32x4 g0 = pload4(mm, ln.g, nb), b0 = pload4(mm, ln.b, nb);   // issued before the barriers
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    float* pa = part(s);
#pragma unroll
    for (int mt = 0; mt < N; ++mt) {
      if (mt < nmt) {
        float sm = (X[s].v[mt][0] + X[s].v[mt][1]) + (X[s].v[mt][2] + X[s].v[mt][3]);
        sm = bp_sum(sm, 16);
        sm = bp_sum(sm, 32);
        const float mw = sm * (1.0f / 16.0f);
        float q = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = X[s].v[mt][r] - mw;
          q = fmaf(d, d, q);
        }
        q = bp_sum(q, 16);
        q = bp_sum(q, 32);
        if (g == 0) *reinterpret_cast<f32x2*>(pa + (mt * 16 + c) * LN_STRIDE + 2 * w) = f32x2{mw, q};
      }
    }
  }
  wg_sync();
  for (int it = w; it < nmt * NS; it += NW) {
    const int s = it % NS, mtc = it / NS;
    float* pa = part(s);
    const int m = mtc * 16 + c;
    const float* pr = pa + m * LN_STRIDE;
    const f32x4 p0 = load4(pr), p1 = load4(pr + 4), p2 = load4(pr + 8), p3 = load4(pr + 12);
    const float mean = 0.125f * (((p0[0] + p0[2]) + (p1[0] + p1[2])) + ((p2[0] + p2[2]) + (p3[0] + p3[2])));
    const float d0 = p0[0] - mean, d1 = p0[2] - mean, d2 = p1[0] - mean, d3 = p1[2] - mean;
    const float d4 = p2[0] - mean, d5 = p2[2] - mean, d6 = p3[0] - mean, d7 = p3[2] - mean;
    const float M2 = (((p0[1] + p0[3]) + (p1[1] + p1[3])) + ((p2[1] + p2[3]) + (p3[1] + p3[3]))) +
                     16.0f * ((d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3) + (d4 * d4 + d5 * d5 + d6 * d6 + d7 * d7));
    const float inv = unbiased_std ? __builtin_amdgcn_rcpf(sqrtf(M2 * (1.0f / 127.0f)) + eps)
                                   : __builtin_amdgcn_rsqf(M2 * (1.0f / 128.0f) + eps);
    if (g == 0) *reinterpret_cast<f32x2*>(pa + LMAX * LN_STRIDE + 2 * m) = f32x2{mean, inv};
  }
  wg_sync();
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const float* stats = part(s) + LMAX * LN_STRIDE;
#pragma unroll
    for (int mt = 0; mt < N; ++mt) {
      if (mt < nmt) {
        const int m = mt * 16 + c;
        const f32x2 st = *reinterpret_cast<const f32x2*>(stats + 2 * m);
        const f32x4 y = (X[s].v[mt] - st[0]) * st[1] * g0 + b0;
        if (INPLACE) X[s].v[mt] = y;
        if (m < rows) out(s, m, nb, y);
      }
    }
  }
}

// ------------------------------------------------------------------------------ attention
// One head per wave for NS sequences (v4::attention_head per sequence, the head's weights fetched once;
// every sequence's chain interleaved).  Reference: attn.py:73-175 (ProbAttention), :37-70
// (FullAttention), :195-209 (AttentionLayer, mix).
template <int PD, int NS>
struct HeadIO2 {
  Img<PD> xq[NS], xkv[NS];    // images feeding the queries / keys+values, per sequence
  Img<PD> ctx[NS];            // attention context out (the O-projection's input image)
  float* scr[NS];             // per-wave scratch: keys [96] u64, sel [96] int16, flag [96] bytes
  uint32_t wq, wk, wv;        // weight-blob offsets (16-byte units) of n-tile 0 of each projection
  GemmDesc dq, dk, dv;        // epilogue vectors
  int LQ, LK, prob, causal, mix, u;
  const uint8_t* cnt;         // the call's multiplicity table (LDS, shared by the sequences) or nullptr
  int cnt_stride;
};

template <int PD, int NS, int MK>
__device__ __forceinline__ void project_kv_s(const HeadIO2<PD, NS>& io, const Mem& m, int h,
                                             AF<plain_of<PD>()> (&Kf)[NS][MK], AF<plain_of<PD>()> (&Vf)[NS][MK]) {
  constexpr int PA = plain_of<PD>();
  const int lane = lane_op();
  const int col = lane & 15, g = lane >> 4;
  const int nkt = (io.LK + 15) >> 4;
  const int fq = 16 * h + 4 * g;
  const int kq = g * 8;
  WF<PD> wk[4], wv[4];
  load_frags<PD, 4>(m, io.wk, h, wk);
  load_frags<PD, 4>(m, io.wv, h, wv);
  f32x4 sk, bk;
  epi_vecs(m, io.dk, fq, sk, bk);
  const float sv = io.dv.scale != NONE ? pload1(m, io.dv.scale, 16 * h + col) : 1.f;
  const float bv = io.dv.bias != NONE ? pload1(m, io.dv.bias, 16 * h + col) : 0.f;
#pragma unroll
  for (int mt = 0; mt < MK; ++mt) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      Kf[s][mt] = AF<PA>{};
      Vf[s][mt] = AF<PA>{};
    }
    if (mt < nkt) {
      f32x4 k[NS], v[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) k[s] = v[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const XF<PD> bx = io.xkv[s].ld(mt * 16 + col, ks * 32 + kq);
          k[s] = mma<PD>(&wk[ks], bx, k[s]);
          v[s] = mma_xw<PD>(bx, &wv[ks], v[s]);
        }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        Kf[s][mt] = split4<PA>(k[s] * sk + bk);
        Vf[s][mt] = split4<PA>(v[s] * sv + bv);
      }
    }
  }
}

// EXTKV: the K/V tiles come from the caller (kin / vin, project_kv_s) instead of being projected here.
template <int PD, int NS, int MQ = MT, int MK = MT, bool EXTKV = false>
__device__ __forceinline__ void attention_s(const HeadIO2<PD, NS>& io, const Mem& m, int h,
                                            const AF<plain_of<PD>()> (*kin)[MK] = nullptr,
                                            const AF<plain_of<PD>()> (*vin)[MK] = nullptr) {
  constexpr int PA = plain_of<PD>();
  const int lane = lane_op();
  const int col = lane & 15, g = lane >> 4;
  const int LQ = io.LQ, LK = io.LK;
  const int nkt = (LK + 15) >> 4, nqt = (LQ + 15) >> 4;
  const bool sparse = io.prob && io.u < LQ;
  const int fq = 16 * h + 4 * g;
  const int kq = g * 8;
  AF<PA> Kf[NS][MK], Vf[NS][MK];
  if constexpr (EXTKV) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int mt = 0; mt < MK; ++mt) {
        Kf[s][mt] = kin[s][mt];
        Vf[s][mt] = vin[s][mt];
      }
  } else {
    project_kv_s<PD, NS, MK>(io, m, h, Kf, Vf);
  }
  // Q tiles are projected where they are consumed; the Q weights are shared by the sequences
  WF<PD> wq[4];
  f32x4 sq, bq;
  load_frags<PD, 4>(m, io.wq, h, wq);
  epi_vecs(m, io.dq, fq, sq, bq);
  auto project_q = [&](int s, int row) __attribute__((always_inline)) {
    f32x4 q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) q = mma<PD>(&wq[ks], io.xq[s].ld(row, ks * 32 + kq), q);
    return split4<PA>(q * sq + bq);
  };

  if (sparse) {
    // ---- sparsity measurement M (attn.py:95-105) from the key multiplicities (shared table)
    const float invLK = 1.0f / (float)LK;
#pragma unroll
    for (int qt = 0; qt < MQ; ++qt) {
      if (qt >= nqt) break;
      const int q = qt * 16 + col;
      AF<PA> qf[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) qf[s] = project_q(s, q);
      // this lane's six count words (keys 16kt + 4g + r, kt = 0..5) are contiguous (cnt_pos_v2)
      const uint2* crow = reinterpret_cast<const uint2*>(io.cnt + (size_t)q * io.cnt_stride + g * 24);
      const uint2 c01 = crow[0], c23 = crow[1], c45 = crow[2];
      const uint32_t cws[MT] = {c01.x, c01.y, c23.x, c23.y, c45.x, c45.y};
      float sum[NS], mx[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sum[s] = 0.f;
        mx[s] = NEG_INF;
      }
#pragma unroll
      for (int kt = 0; kt < MK; ++kt) {
        if (kt < nkt) {
          const uint32_t cw = cws[kt];
          f32x4 sc[NS];
#pragma unroll
          for (int s = 0; s < NS; ++s) sc[s] = mma16<PA>(Kf[s][kt], qf[s], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float cf = (float)((cw >> (8 * r)) & 0xffu);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
              sum[s] = fmaf(cf, sc[s][r], sum[s]);
              mx[s] = fmaxf(mx[s], cf != 0.f ? sc[s][r] : NEG_INF);
            }
          }
        }
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        float su = bp_sum(sum[s], 16);
        su = bp_sum(su, 32);
        float mm = bp_max(mx[s], 16);
        mm = bp_max(mm, 32);
        const float Mv = mm - su * invLK;
        // selection key: order-preserving image of M above, ~q below — equal M go to the lower index
        const uint32_t mu = __float_as_uint(Mv);
        const uint32_t hi = (mu & 0x80000000u) ? ~mu : (mu | 0x80000000u);
        const uint64_t key = q < LQ ? ((uint64_t)hi << 32) | (uint32_t)(0xffff - q) : 0ull;
        if (g == 0) reinterpret_cast<uint64_t*>(io.scr[s])[q] = key;
      }
    }
    wave_lds_sync();
    // ---- exact top-u by rank: rank(q) = #{j : key_j > key_q}; q is selected iff rank < u and
    //      lands in sel[rank].  Lane group g counts over keys [g·J, g·J + J), J = 4·nqt.
    uint64_t myk[NS][MQ];
    int rank[NS][MQ];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int qt = 0; qt < MQ; ++qt) {
        myk[s][qt] = qt < nqt ? reinterpret_cast<const uint64_t*>(io.scr[s])[qt * 16 + col] : ~0ull;
        rank[s][qt] = 0;
      }
    const int J = 4 * nqt;
#pragma unroll 2
    for (int j = 0; j < J; j += 2) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const u64x2 kk = *reinterpret_cast<const u64x2*>(reinterpret_cast<const uint64_t*>(io.scr[s]) + g * J + j);
#pragma unroll
        for (int qt = 0; qt < MQ; ++qt) rank[s][qt] += (int)(kk[0] > myk[s][qt]) + (int)(kk[1] > myk[s][qt]);
      }
    }
    const int uu = io.u;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      int16_t* sel = reinterpret_cast<int16_t*>(io.scr[s] + 192);
      uint8_t* flag = reinterpret_cast<uint8_t*>(io.scr[s] + 240);
#pragma unroll
      for (int qt = 0; qt < MQ; ++qt) {
        if (qt < nqt) {
          int r = rank[s][qt];
          r = (int)bp_sum((float)r, 16);     // counts < 2^24: exact in fp32
          r = (int)bp_sum((float)r, 32);
          const int q = qt * 16 + col;
          if (g == 0 && q < LQ) {
            const bool sl = r < uu;
            flag[q] = sl;
            if (sl) sel[r] = (int16_t)q;
          }
        }
      }
    }
    wave_lds_sync();
  }
  auto ctx_st4 = [&](int s, int q, int e0, const f32x4& v) __attribute__((always_inline)) {
    if (!io.mix) {
      io.ctx[s].st4(q, h * 16 + e0, v);
    } else {
      const int f = h * LQ * 16 + q * 16 + e0;   // (L,H,E) values re-viewed as (H,L,E) memory
      io.ctx[s].st4(f >> 7, f & 127, v);
    }
  };
  if (sparse && !io.causal) {
    // ---- unselected rows keep the initial context, mean(V) (attn.py:116-119): written to every
    //      row here, then the selected rows are overwritten below (same wave, LDS in order)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      float part = 0.f;
#pragma unroll
      for (int kt = 0; kt < MK; ++kt)
        if (kt < nkt)
#pragma unroll
          for (int j = 0; j < 4; ++j) part += (kt * 16 + g * 4 + j < LK) ? (float)Vf[s][kt].h[j] : 0.f;
      part = bp_sum(part, 16);
      part = bp_sum(part, 32);
      const float mean = part / (float)LK;
      if (!io.mix) {
        for (int q = g; q < LQ; q += 4) io.ctx[s].st1(q, h * 16 + col, mean);
      } else {
        for (int q = g; q < LQ; q += 4) {
          const int f = h * LQ * 16 + q * 16 + col;
          io.ctx[s].st1(f >> 7, f & 127, mean);
        }
      }
    }
  }

  // ---- softmax(scale·q·Kᵀ [mask])·V for the selected queries (attn.py:109-138 / 57-65)
  const float scale = 0.25f;
  const int nsel = sparse ? io.u : LQ;
  const int nst = (nsel + 15) >> 4;
#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    const int i = st * 16 + col;
    const int ic = i < nsel ? i : nsel - 1;
    int qi[NS];
    AF<PA> qs[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      qi[s] = sparse ? (int)reinterpret_cast<const int16_t*>(io.scr[s] + 192)[ic] : ic;
      qs[s] = project_q(s, qi[s]);
    }
    float mx[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) mx[s] = NEG_INF;
#pragma unroll
    for (int kt = 0; kt < MK; ++kt) {
      if (kt < nkt) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const f32x4 a = mma16<PA>(Kf[s][kt], qs[s], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kt * 16 + g * 4 + r;
            const bool masked = key >= LK || (io.causal && key > qi[s]);
            mx[s] = masked ? mx[s] : fmaxf(mx[s], a[r] * scale);
          }
        }
      }
    }
    float sum[NS];
    f32x4 o[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      mx[s] = bp_max(mx[s], 16);
      mx[s] = bp_max(mx[s], 32);
      sum[s] = 0.f;
      o[s] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int kt = 0; kt < MK; ++kt) {
      if (kt < nkt) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          f32x4 p = mma16<PA>(Kf[s][kt], qs[s], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kt * 16 + g * 4 + r;
            const bool masked = key >= LK || (io.causal && key > qi[s]);
            p[r] = masked ? 0.f : __expf(p[r] * scale - mx[s]);
            sum[s] += p[r];
          }
          o[s] = mma16<PA>(Vf[s][kt], split4<PA>(p), o[s]);
        }
      }
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      float su = bp_sum(sum[s], 16);
      su = bp_sum(su, 32);
      const float inv = __builtin_amdgcn_rcpf(su);
      if (i < nsel) ctx_st4(s, qi[s], g * 4, o[s] * inv);
    }
  }

  if (sparse && io.causal) {
    // masked: unselected rows keep cumsum(V) (attn.py:120-125) = Vᵀ·Tᵀ with T[q][key] = [key <= q]
#pragma unroll
    for (int qt = 0; qt < MQ; ++qt) {
      if (qt < nqt) {
        const int q = qt * 16 + col;
        f32x4 o[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) o[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < MK; ++kt) {
          if (kt < nkt) {
            f32x4 ind;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int key = kt * 16 + g * 4 + r;
              ind[r] = (key <= q && key < LK) ? 1.f : 0.f;
            }
            const AF<PA> ia = split4<PA>(ind);
#pragma unroll
            for (int s = 0; s < NS; ++s) o[s] = mma16<PA>(Vf[s][kt], ia, o[s]);
          }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const uint8_t* flag = reinterpret_cast<const uint8_t*>(io.scr[s] + 240);
          if (q < LQ && !flag[q]) ctx_st4(s, q, g * 4, o[s]);
        }
      }
    }
  }
}

}  // namespace v5
}  // namespace cet
