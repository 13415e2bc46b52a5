// Fused InformerStack forward, v4: the v3 structure (512-thread workgroups, one residual n-tile and
// one attention head per wave, two sequences per CU) with the operand precision as a template
// policy (cet_v4.hpp) and a plan-sized LDS layout.  Instantiated per precision in
// cet_informer4_{bf16,x3,fp8}.hip (parallel builds).
//
// Reference: FullPrecision/InformerModel/model.py:142-271 (InformerStack), :11-139 (Informer),
// encoder.py:6-106, decoder.py:6-56, attn.py:37-209, embed.py:8-135; models/InformerLSQ/LSQ.py:65-74,
// 305-314 (LSQ weight grid, P_FP8 / P_X3 carriers).
#pragma once
#include "cet_kernels.h"
#include "cet_mt.hpp"
#include "cet_sampler.hpp"
#include "cet_v4.hpp"

namespace cet {
namespace v4 {

// P: precision of the dense (LSQ-quantisable) layers; DIAG: the instance that honours the optional
// outputs (attns maps, activation dumps, phase stamps) — the production instance compiles them out.
// SH: the plan's encoder rows as compile-time constants (cet_kernels.h v4_shape: 0 generic, 1 C2 — one encoder
// 90 → 45 → 23 → 12 —, 2 the TimingAnalysis stack e_layers [4, 3] with a ≤ 16-row decoder over its 24 stack rows).
// ST: a production instance that honours the phase stamps only (the C2 + stamps diagnostic build,
// -DCET_C2_STAMPS: per-phase cycles of the instance the bench times).
// FEED: the decoder's weights and bias / LayerNorm vectors arrive by the LDS-DMA weight feed (cet_v4.hpp; the host
// builds the parameter tiles and checks the plan: cet_api.cpp build_informer).
// PDEC: the decoder's operand precision — P, or split bf16 under a bf16 encoder (P_BF16 / P_X3, the "mixed"
// policy for genuinely sparse decoders: the encoder at the bf16 rate and two workgroups per CU, the decoder's
// ProbSparse selection from fp32-level Q·K).  Its images keep the bf16 layout: hi plane in rows 0-47, lo plane in
// rows 48-95 of XB and CTX; the stack output gets a second plane.
template <int DFF, bool DIAG, int P, bool SPLIT = false, int SH = 0, bool ST = false, bool FEED = false,
          int PDEC = P>
__device__ __forceinline__ void informer_forward_v4_body(const InformerArgs& a, const InformerPlan* __restrict__ plan) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
#define PL (*fresh(plan))
#define ELD (PL.enc[first + l])
#define DLD (PL.dec[l])
  constexpr int PP = plain_of<P>();       // embedding / projection precision
  using G = Geo<P>;
  const Mem M{make_rsrc(a.weights), make_rsrc(a.params), a.wlo};
  const int nsplit = SPLIT ? PL.n_enc : 1;
  const int b = SPLIT ? (int)blockIdx.x / nsplit : (int)blockIdx.x;
  const int my_e = SPLIT ? (int)blockIdx.x - b * nsplit : -1;   // the one encoder of this workgroup
  if (b >= a.B) return;
  if (a.poison) lds_poison<NTHREADS>(lds, a.lds_bytes);
  const int w = wave_id();
#ifdef CET_STAGGER
  // experiment: CET_STAGGER = mask·65536 + units: workgroups with (b & mask) != 0 idle units·64 cycles first
  if (a.stagger && (b & (a.stagger >> 16))) {
    for (int i = 0; i < (a.stagger & 0xffff); ++i) __builtin_amdgcn_s_sleep(1);
  }
#endif
#ifdef CET_SETPRIO
  // static priority for the younger half of the workgroup, the SIMD arbitration loser
  // (MI355X_MICROARCH "Two waves per SIMD" item 4): −0.7 µs at C2 with one batch in flight in round 2
  // (profiles/r02/ab_erf_setprio.log); with two batches in flight and round 4's kernel it costs 2 % of the
  // throughput at an equal kernel-alone time (profiles/r04/ab10/ab.log), so it is off by default
  if (w >= 4) __builtin_amdgcn_s_setprio(1);
#endif

  const Img<P> XB{lds + V4L_XB, G::IMG};
  const Img<P> CTXI{lds + v4_ctx(P), G::IMG};                           // attention context / FFN hidden
  // the decoder's precision and images (cet_informer4.hpp PDEC)
  constexpr int PD = PDEC, PPD = plain_of<PD>();
  constexpr bool MIXD = PD != P;
  static_assert(!MIXD || (P == P_BF16 && PD == P_X3), "mixed: bf16 encoder, split-bf16 decoder");
  constexpr int LOD = 48 * G::RS;   // the mixed decoder's lo plane: rows 48-95 of its image
  const Img<PD> XBd{lds + V4L_XB, MIXD ? LOD : Geo<PD>::IMG};
  const Img<PD> CTXd{lds + v4_ctx(P), MIXD ? LOD : Geo<PD>::IMG};
  const Img<PD> ENC{lds + v4_enc(P), PL.lds4_enc_lo};                   // encoder-stack output
  const Img<PPD> FIN{lds + v4_ctx(P), MIXD ? LOD : Geo<PPD>::IMG};       // decoder output (projection input)
  float* LNP = reinterpret_cast<float*>(lds + v4_scr(P));            // LN partials (alias the scratch)
#ifdef CET_LN_LAST
  unsigned* LNC = reinterpret_cast<unsigned*>(lds + PL.lds4_lncnt);  // LayerNorm arrival counter
  if (threadIdx.x == 0) *LNC = 0u;   // ordered before the first LayerNorm by the encoder loop's barriers
#else
  unsigned* LNC = nullptr;
#endif
  uint8_t* CNT = reinterpret_cast<uint8_t*>(lds + v4_cnt(P));
  MTState gen{reinterpret_cast<uint32_t*>(lds + PL.lds4_mt), MT_N};
  float* SCR = reinterpret_cast<float*>(lds + v4_scr(P)) + w * SCR_FLOATS;
  float* IN = reinterpret_cast<float*>(lds + v4_ctx(P));                // staged raw input (aliases CTX)
  float* dbg = DIAG && a.dbg ? a.dbg + (size_t)b * PL.dbg_stride : nullptr;

  if ((DIAG || ST) && a.stamps && threadIdx.x == 0) {
    a.stamps[(size_t)b * MAX_STAMPS + 127] = __builtin_amdgcn_s_memtime();
    // the constant 100 MHz clock, comparable across workgroups and XCDs (s_memtime is not)
    a.stamps[(size_t)b * MAX_STAMPS + 98] = __builtin_amdgcn_s_memrealtime();
    // where it ran: HW_ID (wave / SIMD / CU / SH / SE fields) and XCC_ID, hwreg(id, 0, 32)
    a.stamps[(size_t)b * MAX_STAMPS + 96] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    a.stamps[(size_t)b * MAX_STAMPS + 97] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
  }
  const int C = PL.C, L0 = PL.seq_len, CS = PL.in_stride, Ld = PL.dec_len;
  // this sequence's x_enc rows are requested first (one f32x4 per thread: L·C/4 ≤ 384), so their HBM
  // latency overlaps the LDS zeroing
  const int t4 = 4 * (int)threadIdx.x;
  const int xdec_off = PL.lds4_xdec;   // x_dec's own region (staged now) or -1 (staged before the decoder)
  float* XDEC = reinterpret_cast<float*>(lds + (xdec_off >= 0 ? xdec_off : v4_ctx(P)));
  f32x4 xe4 = {0.f, 0.f, 0.f, 0.f}, xd4 = xe4;
  if (t4 < L0 * C) xe4 = *reinterpret_cast<const f32x4*>(a.x_enc + (size_t)b * L0 * C + t4);
  if (xdec_off >= 0 && t4 < Ld * C) xd4 = *reinterpret_cast<const f32x4*>(a.x_dec + (size_t)b * Ld * C + t4);
  // fused NMSE: this sequence's labels (pred_len × c_out, c_out ≤ 16) staged with the inputs
  float* LAB = reinterpret_cast<float*>(lds + PL.lds4_lab);
  const int nlab = PL.pred_len * PL.c_out;
  f32x4 lb4 = {0.f, 0.f, 0.f, 0.f};
  if (a.label && t4 < nlab) {
    // nlab need not be a multiple of 4 (c_out ≤ 16 is any width): element loads, never past the batch
    const float* lp = a.label + (size_t)b * nlab + t4;
    if ((nlab & 3) == 0) {
      lb4 = *reinterpret_cast<const f32x4*>(lp);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) lb4[j] = t4 + j < nlab ? lp[j] : 0.f;
    }
  }
  // C2 with prepared (or host-staged) multiplicity tables: the first sparse call's table is requested with
  // the inputs at entry and stored into CNT with them, instead of a global copy + barrier at the head of the
  // first attention phase (104.4 vs 105.4 us kernel alone; staging calls 1-2's tables the same way during
  // the first layer's FFN / distil phases measured slower: DESIGN §3.0e).
#ifndef CET_NO_TAB_PRE
  constexpr bool PRE = SH != V4S_GENERIC;
#else
  constexpr bool PRE = false;
#endif
  f32x4 t0a = {0.f, 0.f, 0.f, 0.f}, t0b = t0a;
  int t0n = 0;   // 16-byte pieces of call 0's table (≤ 96 rows × 104 B / 16 = 624: two per thread)
  static_assert(LMAX * CNT_STRIDE / 16 <= 2 * NTHREADS, "call 0's table staged with two f32x4 per thread");
  static_assert(!FEED || (P == P_BF16 && DFF == 64 && !DIAG && SH != V4S_GENERIC), "the feed's plans (cet_api.cpp)");
  if constexpr (PRE) {
    const int c0 = PL.enc[PL.enc_first[0]].call;
    if (a.cnt && c0 >= 0 && PL.calls[c0].u < PL.calls[c0].LQ) {
      t0n = ((PL.calls[c0].LQ + 15) & ~15) * PL.calls[c0].cnt_stride / 16;
      const f32x4* src = reinterpret_cast<const f32x4*>(a.cnt + PL.calls[c0].cnt_off);
      const int i = tid_op();
      if (i < t0n) t0a = src[i];
      if (i + NTHREADS < t0n) t0b = src[i + NTHREADS];
    }
  }
#ifdef CET_ZERO_ALL
  // zero the activation images: rows past L are read (never used) by MFMAs
  for (int i = threadIdx.x; i < PL.lds4_zero / 16; i += NTHREADS)
    reinterpret_cast<f32x4*>(lds)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();   // zeroing done before the staged rows land in CTX
#else
  {
    // Zero only the rows an MFMA can read before anything writes them: XB and CTX past the first window this
    // workgroup embeds (rows L .. LMAX, L = seq_len, or its encoder's window under the encoder split, where no
    // earlier encoder wrote the rows below L0) and the stack output's padded rows (ENC rows S .. 16·⌈S/16⌉),
    // every plane.  Padded key / value rows must be finite (one NaN key row reaches every query through the
    // softmax); the rows below L are written by the first layer before any later layer or the decoder reads
    // them.  No barrier: the staged rows below land in other bytes (IN rows are 4·in_stride < RS bytes
    // apart), and the encoder loop's barrier orders both before any reader.
    constexpr int RS = G::RS, RQ = RS / 16;   // 16-byte slots per image row
    static_assert(RS % 16 == 0, "image rows of whole 16-byte slots");
    const int r0 = SPLIT ? L0 >> my_e : L0, S0 = PL.S;
    const int n_x = (LMAX - r0) * RQ, n_e = (((S0 + 15) & ~15) - S0) * RQ;   // slots per plane
    const int per = 2 * n_x + n_e;
    char* const enc0 = lds + v4_enc(P);
    for (int i = tid_op(); i < G::PLANES * per; i += NTHREADS) {
      const int pl = i >= per, j = i - pl * per;
      char* q = j < n_x       ? lds + V4L_XB + pl * G::IMG + r0 * RS + j * 16
                : j < 2 * n_x ? lds + v4_ctx(P) + pl * G::IMG + r0 * RS + (j - n_x) * 16
                              : enc0 + pl * PL.lds4_enc_lo + S0 * RS + (j - 2 * n_x) * 16;
      *reinterpret_cast<f32x4*>(q) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (MIXD) {
      // the stack output's lo-plane padded rows (the decoder's lo-plane rows 48-95 of XB / CTX hold the first
      // encoder layer's finite rows below 90 and the zeroed rows above before the decoder writes them)
      for (int i = tid_op(); i < n_e; i += NTHREADS)
        *reinterpret_cast<f32x4*>(enc0 + PL.lds4_enc_lo + S0 * RS + i * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
#endif
  if (t4 < L0 * C) *reinterpret_cast<f32x4*>(IN + (t4 >> PL.C_shift) * CS + (t4 & (C - 1))) = xe4;
  if (xdec_off >= 0 && t4 < Ld * C) *reinterpret_cast<f32x4*>(XDEC + (t4 >> PL.C_shift) * CS + (t4 & (C - 1))) = xd4;
  if (a.label && t4 < nlab) *reinterpret_cast<f32x4*>(LAB + t4) = lb4;
  if constexpr (PRE) {
    f32x4* dst = reinterpret_cast<f32x4*>(CNT);
    const int i = tid_op();
    if (i < t0n) dst[i] = t0a;
    if (i + NTHREADS < t0n) dst[i + NTHREADS] = t0b;
  }
  auto pre_table = [&](int l) -> const uint8_t* {   // the pre-staged table of encoder layer l's call, or null
    if constexpr (!PRE) return nullptr;
    return l == 0 && t0n ? CNT : nullptr;   // (encoder 0 only: enc_layer passes l = -1 for the others)
  };

  Res<MT> X;
  unsigned long long* stamps = (DIAG || ST) && a.stamps ? a.stamps + (size_t)b * MAX_STAMPS : nullptr;
  int sid = 0;
#ifdef CET_PRIO_SLICE
  // The two workgroups of a CU (blocks b and b + 256 at B = 512, tools/stamps.py) compete for VALU issue,
  // which goes to the older waves first: one finishes ≈21 µs before the other, which then runs alone on a
  // half-idle CU.  At every phase boundary each workgroup takes the high priority in alternate slices of
  // 2^CET_PRIO_SLICE ticks of the 100 MHz chip clock, the younger in the odd slices, so both progress alike.
  const unsigned young = ((unsigned)b >> 8) & 1u;
  auto prio = [&]() {
    const unsigned rt = (unsigned)__builtin_amdgcn_s_memrealtime();
    if (((rt >> CET_PRIO_SLICE) ^ young) & 1u)
      __builtin_amdgcn_s_setprio(1);
    else
      __builtin_amdgcn_s_setprio(0);
  };
#else
  auto prio = [&]() {};
#endif
  auto STAMP = [&]() {
    prio();
    if (stamps) {
      if (threadIdx.x == 0 && sid < MAX_STAMPS) stamps[sid] = __builtin_amdgcn_s_memtime();
      ++sid;
    }
  };
  if (a.mt_in && !a.cnt) {
    __syncthreads();
    mt_load<NTHREADS>(gen, a.mt_in);
  }   // device-resident sampler (cet_mt.hpp)
  auto FINE = [&](int layer, int k) {
    if (stamps && layer == 0 && threadIdx.x == 0) stamps[116 + k] = __builtin_amdgcn_s_memtime();
  };
  STAMP();

  constexpr int FRAGS_PER_TILE4 = 4 * WAVE;   // 16-byte lane fragments per n-tile at K = 128
  // the per-head operands of one attention call (AttentionLayer, attn.py:178-209)
  // (the images' precision: the encoder's, or the mixed decoder's with its own context image)
  auto head_io = [&](const auto& Xq, const auto& Xkv, uint32_t Wq, uint32_t Wk, uint32_t Wv, GemmDesc dq,
                     GemmDesc dk, GemmDesc dv, int LQ, int LK, int prob, int causal, int mix, float* attn_out) {
    constexpr int PX = std::decay_t<decltype(Xq)>::PREC;
    HeadIO<PX> io;
    io.xq = Xq; io.xkv = Xkv; io.wq = Wq; io.wk = Wk; io.wv = Wv;
    if constexpr (PX == P) io.ctx = CTXI;
    else io.ctx = CTXd;
    io.dq = dq; io.dk = dk; io.dv = dv;
    io.LQ = LQ; io.LK = LK; io.prob = prob; io.causal = causal; io.mix = mix; io.u = LQ;
    io.cnt = nullptr; io.cnt_stride = 0; io.scr = SCR; io.attn_out = attn_out; io.m_dbg = nullptr;
    io.st = nullptr;
    return io;
  };
  // the ProbSparse draws of one attention call: u, the multiplicity table (replayed in-kernel or staged)
  auto call_setup = [&](auto& io, int call, const uint8_t* pre) __attribute__((always_inline)) {
#ifndef CET_STAMP_DEC_CALL
    io.st = (stamps && call >= 0 && call < 2) ? stamps + 100 + 8 * call : nullptr;
#else   // diagnostic: sub-phases of the first encoder call and the first decoder self-attention call
    io.st = (stamps && (call == 0 || call == PL.n_calls - 3)) ? stamps + 100 + 8 * (call != 0) : nullptr;
#endif
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
        if (call == PL.n_calls - 1 && b == 0) {
          mt_store<NTHREADS>(gen, a.mt_out);
          if constexpr (FEED) vm_wait<0>();   // no store may stay in flight beside the feed's counted loads
        }
      } else if (sparse && pre) {
        // staged earlier (C2): already in LDS behind an earlier barrier
      } else if (sparse) {
        const int bytes = ((c.LQ + 15) & ~15) * c.cnt_stride;
        const f32x4* src = reinterpret_cast<const f32x4*>(a.cnt + c.cnt_off);
        f32x4* dst = reinterpret_cast<f32x4*>(CNT);
#ifndef CET_ABL_CNT
        for (int i = tid_op(); i < bytes / 16; i += NTHREADS) dst[i] = src[i];
        __syncthreads();
#else
        (void)bytes; (void)src; (void)dst;   // ablation (wrong results)
#endif
      }
      if (sparse) io.cnt = a.cnt && pre ? pre : CNT;
    }
  };
  // one head per wave; MQc / MKc: compile-time bounds on the query / key tiles; NKXc: whether MKc is
  // exactly ceil(LK / 16) (true for the encoder, which has a case for every nmt, and for the decoder
  // self-attention, whose bound is its own length; the un-hoisted cross-attention passes it per bound)
  auto attend = [&](auto MQc, auto MKc, auto NKXc, const auto& Xq, const auto& Xkv, uint32_t Wq, uint32_t Wk,
                    uint32_t Wv, GemmDesc dq, GemmDesc dk, GemmDesc dv, int LQ, int LK, int prob, int causal,
                    int mix, int call, float* attn_out, const uint8_t* pre = nullptr) {
    constexpr int MQ_ = decltype(MQc)::value, MK_ = decltype(MKc)::value;
    constexpr bool NKX_ = decltype(NKXc)::value;
    constexpr int PX = std::decay_t<decltype(Xq)>::PREC;
    HeadIO<PX> io = head_io(Xq, Xkv, Wq, Wk, Wv, dq, dk, dv, LQ, LK, prob, causal, mix, attn_out);
#if defined(CET_AB8)
    // reproduction of round 4's ab8 candidate: the early request below with the weight struct handed
    // to attention_head by address — the split-bf16 production instance then keeps it in private memory and
    // disagrees with its diagnostic instance
    const KVPre<PX> kvp = prefetch_kv<PX>(io, M, w);
    call_setup(io, call, pre);
    attention_head<PX, MQ_, MK_, false, NKX_>(io, M, w, nullptr, nullptr, nullptr, &kvp);
#elif !defined(CET_LATE_KV)
    // the head's K/V weights are requested before the call's table setup (its copy loop and barrier hide their L2
    // round trip), and the K/V tiles are projected here and handed to attention_head in registers: +1.4 % seq/s
    // at the driver's bench command, +1.6 % at 300 steps, kernel alone +0.8 µs (profiles/r06/early_kv/)
    const KVPre<PX> kvp = prefetch_kv<PX>(io, M, w);
    call_setup(io, call, pre);
    AF<plain_of<PX>()> Kf[MK_], Vf[MK_];
    project_kv<PX, MK_>(io, kvp, Kf, Vf);
    attention_head<PX, MQ_, MK_, true, NKX_>(io, M, w, Kf, Vf);
#else
    call_setup(io, call, pre);
    attention_head<PX, MQ_, MK_, false, NKX_>(io, M, w);
#endif
  };

  // ---- decoder weight feed (FEED; cet_v4.hpp).  Per decoder layer and wave, 38 weight tiles in the order the
  // layer consumes them — cross K (tiles 0-3), cross V (4-7), self K (8-11), self V (12-15), self Q (16-19),
  // O (20-23), cross Q (24-27), cross O (28-31), FFN1 (32-35, n-tile w mod 4), FFN2 (36-37) — each in ring slot
  // (2l + j) mod 6 of the wave, and the layer's parameter tile in the wave's parameter slot.  Past the last layer
  // the stream continues with the projection's four tiles (then repeats: the counts stay static).
  auto fd_rs = [&]() __attribute__((always_inline)) { return raw_rsrc(a.weights); };
  auto fd_off = [&](int l, auto Jc) __attribute__((always_inline)) -> uint32_t {
    constexpr int J = decltype(Jc)::value;
    const uint32_t wv = (uint32_t)w;
    if (l >= PL.d_layers) return PL.proj.w * 16u + (uint32_t)(J & 3) * 1024u;
    if constexpr (J < 4) return PL.dec[l].ckv.w * 16u + (wv * 4u + J) * 1024u;
    else if constexpr (J < 8) return PL.dec[l].ckv.w * 16u + ((8u + wv) * 4u + (J - 4)) * 1024u;
    else if constexpr (J < 12) return PL.dec[l].qkv.w * 16u + ((8u + wv) * 4u + (J - 8)) * 1024u;
    else if constexpr (J < 16) return PL.dec[l].qkv.w * 16u + ((16u + wv) * 4u + (J - 12)) * 1024u;
    else if constexpr (J < 20) return PL.dec[l].qkv.w * 16u + (wv * 4u + (J - 16)) * 1024u;
    else if constexpr (J < 24) return PL.dec[l].o.w * 16u + (wv * 4u + (J - 20)) * 1024u;
    else if constexpr (J < 28) return PL.dec[l].cq.w * 16u + (wv * 4u + (J - 24)) * 1024u;
    else if constexpr (J < 32) return PL.dec[l].co.w * 16u + (wv * 4u + (J - 28)) * 1024u;
    else if constexpr (J < 36) return PL.dec[l].f1.w * 16u + ((wv & 3u) * 4u + (J - 32)) * 1024u;
    else return PL.dec[l].f2.w * 16u + (wv * 2u + (J - 36)) * 1024u;
  };
  auto fd_slot = [&](int l, auto Jc) __attribute__((always_inline)) -> uint32_t {
    constexpr int J = decltype(Jc)::value;
    int k = (2 * l) % FEED_R + J % FEED_R;
    k = k >= FEED_R ? k - FEED_R : k;
    return feed_slot(FEED_R * w + k);
  };
  auto fd_issue = [&](int l, auto Tc) __attribute__((always_inline)) {   // tile T of layer l (T ≥ 38: of layer l + 1)
    constexpr int T = decltype(Tc)::value;
    if constexpr (T < 38) dma_tile(fd_rs(), fd_off(l, IC<T>{}), fd_slot(l, IC<T>{}), 16 * lane_op());
    else dma_tile(fd_rs(), fd_off(l + 1, IC<T - 38>{}), fd_slot(l + 1, IC<T - 38>{}), 16 * lane_op());
  };
  auto fd_issue_par = [&](int l) __attribute__((always_inline)) {   // layer l's parameter tile (past the last: its copy)
    const int lp = l < PL.d_layers ? l : PL.d_layers - 1;
    dma_tile(fd_rs(), PL.dec_par * 16u + (uint32_t)(lp * NW + w) * 1024u, feed_slot(48 + w), 16 * lane_op());
  };
  // take K tiles J0 .. J0 + K − 1 of layer l (the caller waited for them), then refill their slots with the tiles
  // six ahead in the stream
  auto fd_read = [&](int l, auto J0c, auto Kc, auto* out) __attribute__((always_inline)) {
    constexpr int J0 = decltype(J0c)::value, K = decltype(Kc)::value;
    const int lane = lane_op();
#pragma unroll
    for (int i = 0; i < K; ++i) {
      uint32_t sl;
      if (i == 0) sl = fd_slot(l, IC<J0>{});
      else if (i == 1) sl = fd_slot(l, IC<J0 + 1>{});
      else if (i == 2) sl = fd_slot(l, IC<J0 + 2>{});
      else sl = fd_slot(l, IC<J0 + 3>{});
      out[i].h = *reinterpret_cast<const bf16x8*>(lds + sl + 16 * lane);   // (bf16 fragments: FEED is P_BF16)
    }
  };
  auto fd_take = [&](int l, auto J0c, auto Kc, auto* out) __attribute__((always_inline)) {
    constexpr int J0 = decltype(J0c)::value, K = decltype(Kc)::value;
    fd_read(l, J0c, Kc, out);
    lgkm_wait0();   // the slots are read before they are refilled
    fd_issue(l, IC<J0 + FEED_R>{});
    fd_issue(l, IC<J0 + FEED_R + 1>{});
    if constexpr (K > 2) {
      fd_issue(l, IC<J0 + FEED_R + 2>{});
      fd_issue(l, IC<J0 + FEED_R + 3>{});
    }
  };
  auto fd_par4 = [&](int v) __attribute__((always_inline)) {   // block v, the lane group's four features
    return *reinterpret_cast<const f32x4*>(lds + feed_slot(48 + w) + (16 * v + 4 * (lane_op() >> 4)) * 4);
  };
  auto fd_par1 = [&](int v) __attribute__((always_inline)) {   // block v, feature (lane & 15)
    return *reinterpret_cast<const float*>(lds + feed_slot(48 + w) + (16 * v + (lane_op() & 15)) * 4);
  };
  // the stream's first six tiles and layer 0's parameter tile, issued well ahead of the decoder (the encoder
  // norm phase; under the encoder split after the stack-output exchange)
  auto fd_prefill = [&]() __attribute__((always_inline)) {
    fd_issue(0, IC<0>{});
    fd_issue(0, IC<1>{});
    fd_issue(0, IC<2>{});
    fd_issue(0, IC<3>{});
    fd_issue(0, IC<4>{});
    fd_issue(0, IC<5>{});
    fd_issue_par(0);
  };

  for (int e = 0; e < PL.n_enc; ++e) {
    if (SPLIT && e != my_e) continue;   // the entry staging of x_enc is still intact for it
    // CTX was reused by encoder e-1: re-stage x_enc (the window's embedding is recomputed over the whole
    // sequence's circular conv: embed.py runs once in the reference, model.py:257-258, encoder.py:95-106;
    // staging it under encoder 0's norm phase or with one f32x4 per thread measured no faster)
    if (!SPLIT && e > 0) stage(a.x_enc + (size_t)b * L0 * C, IN, L0, C, CS);
    // ---- DataEmbedding (embed.py:132-135) on the EncoderStack window x[:, -L:] (encoder.py:95-106)
    int L = L0 >> e;
    const int off = L0 - L;
    int nmt = (L + 15) >> 4;
#ifndef CET_NO_EMB_PRE
    // its operands (weight fragments, epilogue vectors, positional rows) requested before the barrier that
    // publishes the staged input: one L2 round trip under the barrier instead of one per m-tile after it
    const WPre<PP, 2> pemb = prefetch_res<PP, 2>(M, PL.emb_enc);
    f32x4 pe[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      pe[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (mt < nmt) {
        const int lane = lane_op();
        const int m = mt * 16 + (lane & 15);
        const int prow = m + off < LMAX ? m + off : LMAX - 1;
        pe[mt] = pload4(M, PL.pe_enc, prow * DMODEL + 16 * w + (lane >> 4) * 4);
      }
    }
#endif
    __syncthreads();
    if (stamps && e == 0 && threadIdx.x == 0) stamps[124] = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) X.v[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
#ifndef CET_NO_EMB_PRE
      gemm_res<PP, 2, MT>(pemb, nmt, LoadEmbed<PP>{IN, L0, PL.C_shift, CS, off},
                          [&](int mt, int n0, f32x4 y) { X.v[mt] = y + pe[mt]; });
#else
      const GemmDesc d = PL.emb_enc;
      auto emb_epi = [&](int mt, int n0, f32x4 y) {
        const int m = mt * 16 + (lane_op() & 15);
        const int prow = m + off < LMAX ? m + off : LMAX - 1;
        X.v[mt] = y + pload4(M, PL.pe_enc, prow * DMODEL + n0);
      };
      gemm_res<PP, 2, MT>(M, d, nmt, LoadEmbed<PP>{IN, L0, PL.C_shift, CS, off}, emb_epi);
#endif
    }
    if (stamps && e == 0 && threadIdx.x == 0) stamps[125] = __builtin_amdgcn_s_memtime();
#ifdef CET_EMB_BARRIER2
    __syncthreads();   // (not needed: the embedding reads IN in CTX, the store below writes XB)
#endif
    store_res(X, nmt, L, XB);
    __syncthreads();
    if (dbg && e == 0) dump_res(X, nmt, L, dbg + PL.dbg_emb);
    STAMP();  // embedding

    const int first = PL.enc_first[e];
    // one encoder layer on L rows (a compile-time constant in the C2 instance: its tile counts, LayerNorm
    // bounds and attention dispatch fold); returns the rows leaving its distil conv
    auto enc_layer = [&](auto Lc, int l) __attribute__((always_inline)) {
      const int L = Lc;
      const int nmt = (L + 15) >> 4;
      int Lout = L;
      // ---- AttentionLayer + ProbAttention / FullAttention, one head per wave, context → CTX
      {
        const GemmDesc q = ELD.qkv;
        auto enc_attend = [&](auto NQ) __attribute__((always_inline)) {
          attend(NQ, NQ, std::true_type{}, XB, XB, q.w, q.w + 8 * FRAGS_PER_TILE4, q.w + 16 * FRAGS_PER_TILE4, part_of(q, 0),
                 part_of(q, 128), part_of(q, 256), L, L, PL.prob, 0, 0, ELD.call,
                 DIAG && a.attns ? a.attns + ELD.attn_off + (size_t)b * ELD.attn_stride : nullptr,
                 pre_table(SH == V4S_C2 || e == 0 ? l : -1));   // C2: one encoder
        };
        switch (nmt) {
          case 1: enc_attend(IC<1>{}); break;
          case 2: enc_attend(IC<2>{}); break;
          case 3: enc_attend(IC<3>{}); break;
          case 4: enc_attend(IC<4>{}); break;
          case 5: enc_attend(IC<5>{}); break;
          default: enc_attend(IC<MT>{}); break;   // exactly MT tiles: every key-tile bound is exact
        }
      }
      const WPre<P, 4> po = prefetch_res<P, 4>(M, ELD.o);   // x = x + new_x (encoder.py:49)
      __syncthreads();
      STAMP();  // encoder attention
      gemm_res<P, 4, MT>(po, nmt, LoadImg<P>{CTXI}, [&](int mt, int n0, f32x4 y) { X.v[mt] += y; });
      FINE(l, 0);
      static_assert(DFF / 16 <= NW, "FFN hidden n-tiles: at most one per wave");
      const WPre<P, 4> pf1 = prefetch_tiles<P, 4>(M, ELD.f1, DFF / 16);   // conv1 (k=1) + activation
      ln_res(X, nmt, L, M, ELD.ln1, 1e-5f, false, LNP, XB, (const Img<P>*)nullptr,
             ST && stamps && e == 0 && l == 0 ? stamps + 32 : nullptr, LNC);   // L0 LN1 per-wave stamps: 32..63
      __syncthreads();
      STAMP();  // out-projection + LN1
      {
        const int relu = PL.act_relu;
        gemm_tiles1<P, 4>(pf1, DFF / 16, nmt, LoadImg<P>{XB}, [&](int mt, int n0, f32x4 v) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = relu ? fmaxf(v[r], 0.f) : gelu_erf(v[r]);
          CTXI.st4(mt * 16 + (lane_op() & 15), n0, v);
        });
      }
      FINE(l, 1);
      const WPre<P, DFF / 32> pf2 = prefetch_res<P, DFF / 32>(M, ELD.f2);  // conv2 (k=1) + residual
      __syncthreads();
      FINE(l, 2);
      gemm_res<P, DFF / 32, MT>(pf2, nmt, LoadImg<P>{CTXI}, [&](int mt, int n0, f32x4 y) { X.v[mt] += y; });
      FINE(l, 3);
      const int has_conv = ELD.conv.n;
      const bool last_of_stack = e == PL.n_enc - 1 && l == PL.enc_layers[e] - 1;
      ln_res(X, nmt, L, M, ELD.ln2, 1e-5f, false, LNP, XB, (const Img<P>*)nullptr,
             ST && stamps && e == 0 && l == 0 ? stamps + 64 : nullptr, LNC);   // L0 LN2: slots 64..95
      __syncthreads();
      STAMP();  // FFN + LN2
      if (dbg && ELD.dbg_layer >= 0) dump_res(X, nmt, L, dbg + ELD.dbg_layer);
      FINE(l, 4);
      if (has_conv) {
        // ---- ConvLayer (encoder.py:22-28): circular conv, BN(eval) folded, ELU, MaxPool(3,2,1)
        // The conv's m-tiles are computed in even/odd position order (pairs of tiles), so the pool
        // is an in-register max with a DPP row rotate.
        const GemmDesc d = ELD.conv;
        with_nmt(nmt + (nmt & 1), [&](auto NMT) __attribute__((always_inline)) {
          constexpr int N_ = decltype(NMT)::value;
          if constexpr (N_ % 2 == 0) {
            Res<N_> Cv;
            const WPre<P, 4> pcv = prefetch_kouter<P, 12, 4>(M, d);
            gemm_kouter_res<P, 12, 4, N_>(pcv, M, d, LoadCirc3EO<P>{XB, L},
                                          [&](int mt, int n0, f32x4 v) __attribute__((always_inline)) {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = elu1(v[r]);
              Cv.v[mt] = v;
            });
            FINE(l, 5);
            maxpool_eo<N_>(Cv, L, X);
          }
        });
        FINE(l, 6);
        Lout = ELD.L_out;
        __syncthreads();                   // every wave finished reading XB
        FINE(l, 7);
        store_res(X, (Lout + 15) >> 4, Lout, XB);
        __syncthreads();
        STAMP();  // distil conv + pool
        if (dbg && ELD.dbg_conv >= 0) dump_res(X, (Lout + 15) >> 4, Lout, dbg + ELD.dbg_conv);
      }
      (void)last_of_stack;
      return Lout;
    };
    if constexpr (SH == V4S_C2) {
      // C2 (BASELINE configs[1]): one encoder of four layers, rows 90 → 45 → 23 → 12 (the host checks the plan)
      enc_layer(IC<90>{}, 0);
      enc_layer(IC<45>{}, 1);
      enc_layer(IC<23>{}, 2);
      L = enc_layer(IC<12>{}, 3);
    } else if constexpr (SH == V4S_E43) {
      // the TimingAnalysis stack (TimingAnalysis/config.py e_layers [4, 3]): encoder 0 as C2's, encoder 1 on the
      // window x[:, -45:], rows 45 → 23 → 12
      if (e == 0) {
        enc_layer(IC<90>{}, 0);
        enc_layer(IC<45>{}, 1);
        enc_layer(IC<23>{}, 2);
        L = enc_layer(IC<12>{}, 3);
      } else {
        enc_layer(IC<45>{}, 0);
        enc_layer(IC<23>{}, 1);
        L = enc_layer(IC<12>{}, 2);
      }
    } else {
      for (int l = 0; l < PL.enc_layers[e]; ++l) L = enc_layer(ELD.L_in, l);
    }
    nmt = (L + 15) >> 4;
    // ---- Encoder.norm (encoder.py:83-84) → this encoder's rows of the stack output (ENC)
    const int rows = PL.enc_rows[e];
    if constexpr (FEED && !SPLIT) {
      if (e == PL.n_enc - 1) fd_prefill();
    }
    const ImgRows<PD> encw{ENC, PL.enc_row_off[e]};
    ln_res(X, nmt, rows, M, PL.enc_norm[e], 1e-5f, false, LNP, XB, &encw, nullptr, LNC);
    __syncthreads();
    if (dbg && PL.enc_dbg[e] >= 0) dump_res(X, nmt, rows, dbg + PL.enc_dbg[e]);
    STAMP();  // encoder norm
  }

  // ================================ decoder (decoder.py:43-56), instantiated for its compile-time
  // tile count (dec_len ≤ 48); the staged decoder input is in XDEC
  const int S = PL.S;
  if constexpr (SPLIT) {
    // ---- publish this encoder's rows of the stack output (write-through, like the NMSE partials),
    //      count the arrival; the last of the sequence's workgroups fetches the other rows and goes on
    constexpr int RW = G::RS / 8;   // u64 words per image row
    uint64_t* xchg = a.enc_xchg + (size_t)b * S * RW;
    const uint64_t* enc64 = reinterpret_cast<const uint64_t*>(ENC.base);
    {
      const int r0 = PL.enc_row_off[my_e], n = PL.enc_rows[my_e] * RW;
      for (int i = threadIdx.x; i < n; i += NTHREADS)
        __hip_atomic_store(xchg + r0 * RW + i, enc64[r0 * RW + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* tk = reinterpret_cast<unsigned*>(lds + v4_scr(P));
    if (threadIdx.x == 0) {
      // agent-scope acq_rel arrival: the rows published above are ordered before the count, and the
      // last arrival's reads of the other workgroups' rows after it (not only by the sc1 codegen)
      const unsigned t = __hip_atomic_fetch_add(a.enc_count + b, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (t + 1u == (unsigned)nsplit)   // re-arm for the next launch
        __hip_atomic_store(a.enc_count + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *tk = t;
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(*tk) + 1u != (unsigned)nsplit) return;   // uniform: the whole workgroup
    uint64_t* encw = reinterpret_cast<uint64_t*>(ENC.base);
    for (int e = 0; e < nsplit; ++e) {
      if (e == my_e) continue;
      const int r0 = PL.enc_row_off[e], n = PL.enc_rows[e] * RW;
      for (int i = threadIdx.x; i < n; i += NTHREADS)
        encw[r0 * RW + i] = __hip_atomic_load(xchg + r0 * RW + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if constexpr (FEED) fd_prefill();   // the exchange's stores are retired (vmcnt(0) above)
  }
  if (xdec_off < 0) {   // no room to keep it since entry: stage it now (into CTX, free after the encoder)
    stage(a.x_dec + (size_t)b * Ld * C, XDEC, Ld, C, CS);
    __syncthreads();
  }
  // ---- the decoder on the weight feed (FEED): the decoder below, with every weight tile taken from the wave's LDS
  //      ring (six tiles ahead) and every bias / LayerNorm vector from the layer's parameter tile — no global load
  //      of the decoder layers waits in a phase.  The counted waits follow the stream: entering a layer 7 loads
  //      are in flight (tiles 0-5, the parameter tile); each group of four leaves two in flight, FFN2's pair four.
  auto decoder_feed = [&](auto NMSc) __attribute__((always_inline)) {
   if constexpr (FEED) {
    constexpr int NMS = decltype(NMSc)::value;
    constexpr bool CROSS_EXACT = NMS == 1 || SH == V4S_E43;
    constexpr int NMD = 1;
    const int nmd = NMD;
    Res<NMD> XD;
    {
      const GemmDesc d = PL.emb_dec;
      gemm_res_n<PP, 2, NMD>(M, d, LoadEmbed<PP>{XDEC, Ld, PL.C_shift, CS, 0}, [&](int mt, int n0, f32x4 y) {
        const int m = mt * 16 + (lane_op() & 15);
        const int prow = m < LMAX ? m : LMAX - 1;
        XD.v[mt] = y + pload4(M, PL.pe_dec, prow * DMODEL + n0);
      });
    }
    __syncthreads();
    store_res(XD, nmd, Ld, XB);
    __syncthreads();
    STAMP();  // decoder embedding
    const f32x4 one4 = {1.f, 1.f, 1.f, 1.f};
    for (int l = 0; l < PL.d_layers; ++l) {
      // cross-attention K / V of this layer (the encoder-stack output only), projected first
      KVPre<P> ckv;
      vm_wait<3>();
      fd_take(l, IC<0>{}, IC<4>{}, ckv.k);
      vm_wait<2>();
      fd_take(l, IC<4>{}, IC<4>{}, ckv.v);
      ckv.sk = one4;
      ckv.bk = fd_par4(0);
      ckv.sv = 1.f;
      ckv.bv = fd_par1(1);
      const HeadIO<P> cio = head_io(XB, ENC, 0u, 0u, 0u, GemmDesc{}, GemmDesc{}, GemmDesc{}, Ld, S, 0, 0, 0, nullptr);
      AF<PP> CK[NMS], CV[NMS];
      project_kv<P, NMS>(cio, ckv, CK, CV);
      {
        // masked self-attention with the mix scramble (model.py:211-222); every query selected (u = L)
        HeadIO<P> sio = head_io(XB, XB, 0u, 0u, 0u, GemmDesc{}, GemmDesc{}, GemmDesc{}, Ld, Ld, PL.prob, 1, PL.mix,
                                nullptr);
        call_setup(sio, DLD.call, nullptr);   // the draws still advance the sampler stream
        KVPre<P> skv;
        vm_wait<2>();
        fd_take(l, IC<8>{}, IC<4>{}, skv.k);
        vm_wait<2>();
        fd_take(l, IC<12>{}, IC<4>{}, skv.v);
        skv.sk = one4;
        skv.bk = fd_par4(2);
        skv.sv = 1.f;
        skv.bv = fd_par1(3);
        AF<PP> SK[NMD], SV[NMD];
        project_kv<P, NMD>(sio, skv, SK, SV);
        WPre<P, 4> sq;
        vm_wait<2>();
        fd_take(l, IC<16>{}, IC<4>{}, sq.a);
        sq.sc = one4;
        sq.bi = fd_par4(4);
        attention_head<P, NMD, NMD, true, true>(sio, M, w, SK, SV, &sq);
      }
      WPre<P, 4> po;
      vm_wait<2>();
      fd_take(l, IC<20>{}, IC<4>{}, po.a);
      po.sc = one4;
      po.bi = fd_par4(5);
      __syncthreads();
      STAMP();  // decoder self-attention
      gemm_res_n<P, 4, NMD>(po, LoadImg<P>{CTXI}, [&](int mt, int n0, f32x4 y) { XD.v[mt] += y; });
      WPre<P, 4> pcq;
      vm_wait<2>();
      fd_take(l, IC<24>{}, IC<4>{}, pcq.a);
      pcq.sc = one4;
      pcq.bi = fd_par4(8);
      ln_res_gb(XD, nmd, Ld, fd_par4(6), fd_par4(7), 1e-5f, false, LNP, XB, (const Img<P>*)nullptr);
      __syncthreads();
      // cross-attention: FullAttention over the encoder-stack output, mix=False
      attention_head<P, NMD, NMS, true, CROSS_EXACT>(cio, M, w, CK, CV, &pcq);
      WPre<P, 4> pco;
      vm_wait<2>();
      fd_take(l, IC<28>{}, IC<4>{}, pco.a);
      pco.sc = one4;
      pco.bi = fd_par4(9);
      __syncthreads();
      STAMP();  // cross-attention
      gemm_res_n<P, 4, NMD>(pco, LoadImg<P>{CTXI}, [&](int mt, int n0, f32x4 y) { XD.v[mt] += y; });
      WPre<P, 4> pf1;
      vm_wait<2>();
      fd_take(l, IC<32>{}, IC<4>{}, pf1.a);   // refills the next layer's tiles 0-3 (or the projection's)
      pf1.sc = one4;
      pf1.bi = fd_par4(12);
      ln_res_gb(XD, nmd, Ld, fd_par4(10), fd_par4(11), 1e-5f, false, LNP, XB, (const Img<P>*)nullptr);
      __syncthreads();
      {
        const int relu = PL.act_relu;
        gemm_tiles1<P, 4>(pf1, DFF / 16, nmd, LoadImg<P>{XB}, [&](int mt, int n0, f32x4 v) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = relu ? fmaxf(v[r], 0.f) : gelu_erf(v[r]);
          CTXI.st4(mt * 16 + (lane_op() & 15), n0, v);
        });
      }
      WPre<P, DFF / 32> pf2;
      vm_wait<4>();
      fd_take(l, IC<36>{}, IC<2>{}, pf2.a);   // refills the next layer's tiles 4-5
      pf2.sc = one4;
      pf2.bi = fd_par4(13);
      __syncthreads();
      gemm_res_n<P, DFF / 32, NMD>(pf2, LoadImg<P>{CTXI}, [&](int mt, int n0, f32x4 y) { XD.v[mt] += y; });
      ln_res_gb(XD, nmd, Ld, fd_par4(14), fd_par4(15), 1e-5f, false, LNP, XB, (const Img<P>*)nullptr);
      lgkm_wait0();          // the parameter tile's last reads are done ...
      fd_issue_par(l + 1);   // ... before the next layer's tile replaces it
      __syncthreads();
      STAMP();  // decoder O/LN1 + cross O/LN2 + FFN/LN3
    }
    // final norm → the projection's input image (plain precision; CTX rows < 16 are free: FFN2 is done)
    ln_res(XD, nmd, Ld, M, PL.dec_norm, 1e-5f, false, LNP, FIN, (const Img<PP>*)nullptr);
    __syncthreads();
    {
      // projection (model.py:264) on the last pred_len rows → out[b]: the stream's four tiles past the last layer
      WF<P> pw[4];
      vm_wait<0>();   // the stream is drained (its last three loads are dummies): nothing stays in flight past here
      fd_read(PL.d_layers, IC<0>{}, IC<4>{}, pw);
      const GemmDesc d = PL.proj;
      const int first_row = Ld - PL.pred_len, co = PL.c_out;
      float* out = a.out + (size_t)b * PL.pred_len * co;
#ifdef V4_NO_FUSE
      constexpr bool fuse = false;
#else
      const bool fuse = a.label != nullptr;
#endif
      if (w == 0) {   // one n-tile (c_out ≤ 16), one m-tile: wave 0
        const int lane = lane_op();
        const int kq = kq_of<PP>(lane), mrow = lane & 15;
        const int n0 = (lane >> 4) * 4;
        f32x4 sc, bi;
        epi_vecs(M, d, n0, sc, bi);
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) c = mma<PP>(&pw[ks], FIN.ld(mrow, ks * 32 + kq), c);
        const f32x4 v = c * sc + bi;
        const int m = mrow;
        const bool valid = m >= first_row && m < Ld;
        float se = 0.f, pwr = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (valid && n0 + r < co) {
            out[(m - first_row) * co + n0 + r] = v[r];
            if (fuse) {   // NMSE_Split_cuda(x_hat = out, x = label): Σ(x − x̂)², Σ x̂² (metrics.py:26-30)
              const float dx = LAB[(m - first_row) * co + n0 + r] - v[r];
              se = fmaf(dx, dx, se);
              pwr = fmaf(v[r], v[r], pwr);
            }
          }
        if (fuse) {
          se = xor_sum(se, 16);
          se = xor_sum(se, 32);
          pwr = xor_sum(pwr, 16);
          pwr = xor_sum(pwr, 32);
          if ((lane >> 4) == 0 && valid) {
            const float2 pr = make_float2(se, pwr);
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.nmse_part + (size_t)b * PL.pred_len +
                                                                     (m - first_row)),
                               __builtin_bit_cast(unsigned long long, pr), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          }
        }
        if (fuse) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores are done
      }
    }
    STAMP();  // final norm + projection
    if (stamps && threadIdx.x == 0) stamps[99] = __builtin_amdgcn_s_memrealtime();
   }
  };
  auto decoder = [&](auto NMDc, auto NMSc) __attribute__((always_inline)) {
    constexpr int NMS = decltype(NMSc)::value;
    // the cross-attention's key-tile bound is exact for one tile (S ≤ 16) and in the E43 instance (S = 24)
    constexpr bool CROSS_EXACT = NMS == 1 || SH == V4S_E43;
    constexpr int NMD = decltype(NMDc)::value;
    const int nmd = NMD;
    Res<NMD> XD;
    {
      const GemmDesc d = PL.emb_dec;
      gemm_res_n<PPD, 2, NMD>(M, d, LoadEmbed<PPD>{XDEC, Ld, PL.C_shift, CS, 0}, [&](int mt, int n0, f32x4 y) {
        const int m = mt * 16 + (lane_op() & 15);
        const int prow = m < LMAX ? m : LMAX - 1;
        XD.v[mt] = y + pload4(M, PL.pe_dec, prow * DMODEL + n0);
      });
    }
    __syncthreads();
    store_res(XD, nmd, Ld, XBd);
    __syncthreads();
    if (dbg) dump_res(XD, nmd, Ld, dbg + PL.dbg_dec_emb);
    STAMP();  // decoder embedding

#ifdef CET_ABL_DEC
    for (int l = 0; l < 0; ++l) {   // ablation (wrong results)
#else
    for (int l = 0; l < PL.d_layers; ++l) {
#endif
#ifndef CET_NO_CROSS_HOIST
      // cross-attention K/V of this layer (encoder-stack output only): projected before the
      // self-attention, so their weight fetch overlaps it instead of following it (123.4 vs 124.3 us,
      // profiles/r02/ab_cross_hoist.log)
      const GemmDesc cq = DLD.cq, ckv = DLD.ckv;
      const HeadIO<PD> cio = head_io(XBd, ENC, cq.w, ckv.w, ckv.w + 8 * FRAGS_PER_TILE4, part_of(cq, 0), part_of(ckv, 0),
                                    part_of(ckv, 128), Ld, S, 0, 0, 0, nullptr);
      AF<PPD> CK[NMS], CV[NMS];
      project_kv<PD, NMS>(cio, M, w, CK, CV);
#endif
      {
        // masked self-attention with the mix scramble (model.py:211-222)
        const GemmDesc q = DLD.qkv;
        attend(IC<NMD>{}, IC<NMD>{}, std::true_type{}, XBd, XBd, q.w, q.w + 8 * FRAGS_PER_TILE4, q.w + 16 * FRAGS_PER_TILE4,
               part_of(q, 0), part_of(q, 128), part_of(q, 256), Ld, Ld, PL.prob, 1, PL.mix, DLD.call, nullptr);
      }
      const WPre<PD, 4> po = prefetch_res<PD, 4>(M, DLD.o);
      __syncthreads();
      STAMP();  // decoder self-attention
      gemm_res_n<PD, 4, NMD>(po, LoadImg<PD>{CTXd}, [&](int mt, int n0, f32x4 y) { XD.v[mt] += y; });
#ifndef CET_NO_CROSSQ_PRE
      // the cross-attention's Q weights of head w, requested before LN1's barrier (the decoder's residual
      // is one tile: the registers are free here)
      const WPre<PD, 4> pcq = prefetch_res<PD, 4>(M, cq);
      const WPre<PD, 4>* cqp = &pcq;
#else
      const WPre<PD, 4>* cqp = nullptr;
#endif
      ln_res(XD, nmd, Ld, M, DLD.ln1, 1e-5f, false, LNP, XBd, (const Img<PD>*)nullptr);
      __syncthreads();
      {
        // cross-attention: FullAttention over the encoder-stack output, mix=False
#ifndef CET_NO_CROSS_HOIST
        attention_head<PD, NMD, NMS, true, CROSS_EXACT>(cio, M, w, CK, CV, cqp);
#else
        const GemmDesc cq = DLD.cq, ckv = DLD.ckv;
        // the key-tile bound MT is exact only for S in 81-96; NMS == 1 is exact (S ≤ 16)
        attend(IC<NMD>{}, IC<NMS>{}, std::bool_constant<NMS == 1>{}, XBd, ENC, cq.w, ckv.w, ckv.w + 8 * FRAGS_PER_TILE4, part_of(cq, 0),
               part_of(ckv, 0), part_of(ckv, 128), Ld, S, 0, 0, 0, -1, nullptr);
#endif
      }
      const WPre<PD, 4> pco = prefetch_res<PD, 4>(M, DLD.co);
      __syncthreads();
      STAMP();  // cross-attention
      gemm_res_n<PD, 4, NMD>(pco, LoadImg<PD>{CTXd}, [&](int mt, int n0, f32x4 y) { XD.v[mt] += y; });
      const WPre<PD, 4> pf1 = prefetch_tiles<PD, 4>(M, DLD.f1, DFF / 16);
      ln_res(XD, nmd, Ld, M, DLD.ln2, 1e-5f, false, LNP, XBd, (const Img<PD>*)nullptr);
      __syncthreads();
      {
        const int relu = PL.act_relu;
        gemm_tiles1<PD, 4>(pf1, DFF / 16, nmd, LoadImg<PD>{XBd}, [&](int mt, int n0, f32x4 v) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = relu ? fmaxf(v[r], 0.f) : gelu_erf(v[r]);
          CTXd.st4(mt * 16 + (lane_op() & 15), n0, v);
        });
      }
      const WPre<PD, DFF / 32> pf2 = prefetch_res<PD, DFF / 32>(M, DLD.f2);
      __syncthreads();
      gemm_res_n<PD, DFF / 32, NMD>(pf2, LoadImg<PD>{CTXd}, [&](int mt, int n0, f32x4 y) { XD.v[mt] += y; });
      ln_res(XD, nmd, Ld, M, DLD.ln3, 1e-5f, false, LNP, XBd, (const Img<PD>*)nullptr);
      __syncthreads();
      STAMP();  // decoder O/LN1 + cross O/LN2 + FFN/LN3
      if (dbg && DLD.dbg >= 0) dump_res(XD, nmd, Ld, dbg + DLD.dbg);
    }
    // final norm → the projection's input image (plain precision; CTX is free: FFN2 is done)
    ln_res(XD, nmd, Ld, M, PL.dec_norm, 1e-5f, false, LNP, FIN, (const Img<PPD>*)nullptr);
    __syncthreads();
    if (dbg) dump_res(XD, nmd, Ld, dbg + PL.dbg_dec_out);
    {
      // projection (model.py:264) on the last pred_len rows → out[b]
      const GemmDesc d = PL.proj;
      const int first_row = Ld - PL.pred_len, co = PL.c_out;
      float* out = a.out + (size_t)b * PL.pred_len * co;
#ifdef V4_NO_FUSE
      constexpr bool fuse = false;
#else
      const bool fuse = a.label != nullptr;   // the launcher guarantees c_out ≤ 16 (one n-tile)
#endif
      gemm_tiles<PPD, 4>(M, d, d.n / 16, nmd, LoadImg<PPD>{FIN}, [&](int mt, int n0, f32x4 v) {
        const int lane = lane_op();
        const int m = mt * 16 + (lane & 15);
        const bool valid = m >= first_row && m < Ld;
        float se = 0.f, pw = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (valid && n0 + r < co) {
            out[(m - first_row) * co + n0 + r] = v[r];
            if (fuse) {   // NMSE_Split_cuda(x_hat = out, x = label): Σ(x − x̂)², Σ x̂² (metrics.py:26-30)
              const float dx = LAB[(m - first_row) * co + n0 + r] - v[r];
              se = fmaf(dx, dx, se);
              pw = fmaf(v[r], v[r], pw);
            }
          }
        if (fuse) {
          se = xor_sum(se, 16);   // over the 16 features of row m (4 lane groups)
          se = xor_sum(se, 32);
          pw = xor_sum(pw, 16);
          pw = xor_sum(pw, 32);
          if ((lane >> 4) == 0 && valid) {
            // write-through (sc1) so the last workgroup to finish reads it without a fence
            const float2 pr = make_float2(se, pw);
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.nmse_part + (size_t)b * PL.pred_len +
                                                                     (m - first_row)),
                               __builtin_bit_cast(unsigned long long, pr), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      });
      if (fuse) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores are done
    }
    STAMP();  // final norm + projection
    if (stamps && threadIdx.x == 0) stamps[99] = __builtin_amdgcn_s_memrealtime();
  };
  if constexpr (FEED) {
    // the host checks the plan (cet_api.cpp build_informer): a one-tile decoder; C2's stack output is one tile (S =
    // 12), the E43 stack's two (S = 24)
    decoder_feed(IC<SH == V4S_E43 ? 2 : 1>{});
  } else if constexpr (SH == V4S_E43) {
    decoder(IC<1>{}, IC<2>{});   // the host checks dec_len ≤ 16 and S = 24
  } else switch ((Ld + 15) >> 4) {
    case 1: S <= 16 ? decoder(IC<1>{}, IC<1>{}) : decoder(IC<1>{}, IC<MT>{}); break;
    case 2: S <= 16 ? decoder(IC<2>{}, IC<1>{}) : decoder(IC<2>{}, IC<MT>{}); break;
    default: S <= 16 ? decoder(IC<3>{}, IC<1>{}) : decoder(IC<3>{}, IC<MT>{}); break;
  }
  // ---- the first workgroup to finish prepares the NEXT forward's ProbSparse tables from the
  //      resident sampler state (cet_sampler.hpp) while the rest of the grid drains; the last one to
  //      finish re-arms the counter for the next launch
  if (a.ticket) {
    __syncthreads();   // every wave's NMSE partials are written (each waited for its own stores)
    unsigned* tk = reinterpret_cast<unsigned*>(lds + v4_scr(P));
    if (threadIdx.x == 0) {
      // agent-scope acq_rel arrival: this workgroup's NMSE partials are ordered before the count, and
      // the last arrival's reads of every partial after it
      const unsigned t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (t + 1u == (unsigned)a.B)   // re-arm for the next launch
        __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *tk = t;
    }
    __syncthreads();   // the other waves load after this barrier (the adding wave has its value)
    const unsigned tw = __builtin_amdgcn_readfirstlane(*tk);
#ifndef V4_NO_FUSE
    if (a.label && tw + 1u == (unsigned)a.B) {
      // ---- last workgroup: the batch's NMSE_Split from every sequence's partials.  Thread i takes
      //      sequences i, i+512, ... (write-through partials, read with sc1 loads); then a fixed
      //      butterfly per wave and a fixed order over the waves: deterministic.
      const int T = PL.pred_len, lane = threadIdx.x & 63;
      double* red = reinterpret_cast<double*>(lds + v4_ctx(P));   // [NW][2][8]
      for (int t0 = 0; t0 < T; t0 += 8) {
        const int nt = T - t0 < 8 ? T - t0 : 8;
        double se[8], pw[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) se[j] = pw[j] = 0.0;
        for (int s = threadIdx.x; s < a.B; s += NTHREADS) {
          const unsigned long long* src = reinterpret_cast<const unsigned long long*>(a.nmse_part + (size_t)s * T + t0);
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
        __syncthreads();
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
        __syncthreads();
      }
    }
#endif
    const bool elected = tw == 0u;
    __syncthreads();   // every wave has read the ticket before the replay reuses the LDS
    if (elected && a.cnt_next)
      replay_all<NTHREADS>(PL, a.mt_in, a.mt_out, a.cnt_next, lds, a.lds_bytes, reinterpret_cast<uint32_t*>(lds),
                           reinterpret_cast<uint32_t*>(lds + v4_ctx(P)));
  }
#undef PL
#undef ELD
#undef DLD
}

// X3 carries hi/lo operand pairs: 256 VGPRs, one workgroup per CU; the others fit 128 (two per CU).
template <int DFF, bool DIAG, int P, bool SPLIT = false, int SH = 0, bool ST = false, bool FEED = false,
          int PDEC = P>
__global__ void __launch_bounds__(NTHREADS, P == P_X3 ? 2 : 4)
    informer_forward_v4(InformerArgs a, const InformerPlan* __restrict__ plan) {
  informer_forward_v4_body<DFF, DIAG, P, SPLIT, SH, ST, FEED, PDEC>(a, plan);
}

template <int P>
int launch_v4(const InformerArgs* a, int dff, int lds_bytes, hipStream_t stream) {
  if (a->B <= 0) return 0;
  using K = void (*)(InformerArgs, const InformerPlan*);
  K kern = nullptr;
  const bool split = a->enc_split != 0;
  switch (v4_instance(*a, P, dff)) {
    case V4I_SPLIT:   // encoder split: bf16 policy, production instance only (the launcher checks the plan)
      if constexpr (P == P_BF16) {
        if (a->shape == V4S_E43)
          kern = a->feed ? informer_forward_v4<64, false, P, true, V4S_E43, false, true>
                         : informer_forward_v4<64, false, P, true, V4S_E43>;
        else kern = dff == 64 ? informer_forward_v4<64, false, P, true> : informer_forward_v4<128, false, P, true>;
      }
      break;
#ifdef CET_C2_STAMPS
    case V4I_SHAPE_STAMPS:   // the shape instance + phase stamps (diagnostic build)
      if constexpr (P == P_BF16) {
        if (a->feed)
          kern = a->shape == V4S_E43 ? informer_forward_v4<64, false, P, false, V4S_E43, true, true>
                                     : informer_forward_v4<64, false, P, false, V4S_C2, true, true>;
        else
          kern = a->shape == V4S_E43 ? informer_forward_v4<64, false, P, false, V4S_E43, true>
                                     : informer_forward_v4<64, false, P, false, V4S_C2, true>;
      }
      break;
#endif
    case V4I_SHAPE:   // the plan's rows at compile time
      if constexpr (P == P_BF16) {
        if (a->feed)   // the decoder on the LDS-DMA weight feed (the host checked the plan)
          kern = a->shape == V4S_E43 ? informer_forward_v4<64, false, P, false, V4S_E43, false, true>
                                     : informer_forward_v4<64, false, P, false, V4S_C2, false, true>;
        else
          kern = a->shape == V4S_E43 ? informer_forward_v4<64, false, P, false, V4S_E43>
                                     : informer_forward_v4<64, false, P, false, V4S_C2>;
      } else if constexpr (P == P_FP8) {
        kern = informer_forward_v4<64, false, P, false, V4S_C2>;
      }
      break;
    case V4I_DIAG: kern = dff == 64 ? informer_forward_v4<64, true, P> : informer_forward_v4<128, true, P>; break;
    case V4I_GENERIC: kern = dff == 64 ? informer_forward_v4<64, false, P> : informer_forward_v4<128, false, P>; break;
    default: break;
  }
  if (!kern) return -3;
  if (!ensure_lds_attr(reinterpret_cast<const void*>(kern))) return -1;
  InformerArgs args = *a;
  args.lds_bytes = lds_bytes;
  const unsigned grid = (unsigned)a->B * (split ? (unsigned)a->enc_split : 1u);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NTHREADS), lds_bytes, stream, args, a->plan);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// The mixed policy (host precision 4): the bf16 encoder with a split-bf16 decoder (PDEC = P_X3).
inline int launch_v4_mix(const InformerArgs* a, int dff, int lds_bytes, hipStream_t stream) {
  if (a->B <= 0) return 0;
  using K = void (*)(InformerArgs, const InformerPlan*);
  K kern = nullptr;
  switch (v4_instance(*a, 4, dff)) {
    case V4I_SHAPE: kern = informer_forward_v4<64, false, P_BF16, false, V4S_C2, false, false, P_X3>; break;
    case V4I_DIAG: kern = informer_forward_v4<64, true, P_BF16, false, V4S_GENERIC, false, false, P_X3>; break;
    case V4I_GENERIC: kern = informer_forward_v4<64, false, P_BF16, false, V4S_GENERIC, false, false, P_X3>; break;
    default: break;
  }
  if (!kern) return -3;
  if (!ensure_lds_attr(reinterpret_cast<const void*>(kern))) return -1;
  InformerArgs args = *a;
  args.lds_bytes = lds_bytes;
  hipLaunchKernelGGL(kern, dim3((unsigned)a->B), dim3(NTHREADS), lds_bytes, stream, args, a->plan);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace v4
}  // namespace cet
