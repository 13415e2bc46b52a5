// "v4" building blocks: the v3 scheme (8-wave workgroups, one 16-feature n-tile of the register
// residual and one attention head per wave) with the operand precision as a compile-time policy:
//
//   P_BF16  bf16 operands, fp32 accumulation (the C2 contract).
//   P_X3    split bf16: every operand x is carried as hi = bf16(x), lo = bf16(x − hi) and a product
//           is hi·hi + hi·lo + lo·hi on three MFMAs (≈16 significant bits per operand, fp32
//           accumulation): the fp32-parity mode, and the exact carrier of LSQ integer grids whose
//           |q| exceeds bf16's 256.
//   P_FP8   OCP e4m3 activations for the LSQ-quantised layers, the integer weight grid
//           q ∈ [−128, 127] carried exactly in e4m3 parts, the step size in the epilogue.  Default:
//           v_mfma_f32_16x16x32_fp8_fp8 with the grid as 16·⌊q/16⌋ and q mod 16, two MFMAs per
//           32-feature k-step.  (The block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 form — hi and lo in
//           one MFMA per 64 features, the ×16 in the E8M0 block scale — was removed in round 5: its
//           8-register operand tuples spill ≈270 VGPRs at the 128-VGPR cap and it ran C5 fp8 at 263.6 vs
//           219.3 µs, profiles/r05/fp8_scaled/; its lane/byte/scale layout, probed on MI355X, is kept in
//           tools/probe/mfma_scale_probe.hip and profiles/r03/mfma_scale_probe.txt.)
//           The layers the reference does not quantise (token embedding, projection) and the attention
//           products stay bf16.
//
// Fragment geometry: every policy uses v_mfma_f32_16x16x32_* (lane l holds A[row l&15]
// [k = 8(l>>4) .. +7] and B[k = 8(l>>4) .. +7][col l&15]; fp8: 8 e4m3 per lane).  The weight blob keeps
// 16 B per lane per 32-feature k-step for every policy, so the GEMM loops are shared (KR = 1 k-step of
// weight fragments per MFMA).
//
// Images (LDS): bf16 rows of 272 B (256 B of features + one 16-byte pad slot; -DCET_IMG_SWZ: 288 B with
// a row-bit XOR, Img::off), X3 adds a lo plane, fp8 rows are 144 B (conflict-free ds_read_b64).
#pragma once
#include <type_traits>

#include "cet_device.hpp"

namespace cet {
namespace v4 {

enum { P_BF16 = 0, P_X3 = 1, P_FP8 = 2 };
// precision of the layers the reference never quantises, and of the attention products
template <int P>
constexpr int plain_of() { return P == P_FP8 ? P_BF16 : P; }

constexpr int NW = 8;
constexpr int NTHREADS = NW * WAVE;
constexpr int MT = 6;                 // max 16-row tiles (96 positions)
constexpr int LN_STRIDE = LN3_STRIDE;
constexpr int SCR_FLOATS = V2_SCR_FLOATS;   // per-wave attention scratch (u64 keys | int16 sel | flags)

template <int P>
struct Geo {
  static constexpr int RS = v4_rs(P);                 // image row stride (bytes)
  static constexpr int PLANES = P == P_X3 ? 2 : 1;
  static constexpr int IMG = LMAX * RS;                // one plane of a LMAX-row image
};

// ------------------------------------------------------------------ fragments and products
template <int P>
struct XF {  // B-role (activation) fragment of one 16x16x32 k-step
  bf16x8 h;
};
template <>
struct XF<P_X3> {
  bf16x8 h, l;
};
template <int P>
struct WF {  // A-role (weight) fragment
  bf16x8 h;
};
template <>
struct WF<P_X3> {
  bf16x8 h, l;
};
// ---- fp8 on v_mfma_f32_16x16x32_fp8_fp8 (default): per 32-feature k-step the grid as 16·⌊q/16⌋ and
//      q mod 16 (both e4m3-exact), two MFMAs
template <>
struct XF<P_FP8> {
  long q;   // 8 e4m3: features k0 .. +7
};
template <>
struct WF<P_FP8> {
  long hi, lo;   // 16·⌊q/16⌋ and q mod 16, e4m3
};

// k-steps (32 features of weight fragments) one MFMA consumes (one for every policy), and the lane's
// activation k offset
template <int P>
constexpr int KR = 1;
template <int P>
__device__ __forceinline__ int kq_of(int lane) {
  return 8 * (lane >> 4);
}

__device__ __forceinline__ f32x4 mfma8(long a, long b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, c, 0, 0, 0);
}

// W·X (weights as A): the transposed dense layer Yᵀ = W·Xᵀ; a points at KR<P> weight fragments
template <int P>
__device__ __forceinline__ f32x4 mma(const WF<P>* a, const XF<P>& b, f32x4 c) {
  if constexpr (P == P_BF16) {
    return mfma16x16x32(a->h, b.h, c);
  } else if constexpr (P == P_X3) {
    c = mfma16x16x32(a->l, b.h, c);   // small terms first
    c = mfma16x16x32(a->h, b.l, c);
    return mfma16x16x32(a->h, b.h, c);
  } else {
    c = mfma8(a->lo, b.q, c);
    return mfma8(a->hi, b.q, c);
  }
}
// X·Wᵀ (activations as A): V = X·Wvᵀ, whose C fragment is the A operand of Oᵀ = Vᵀ·Pᵀ
template <int P>
__device__ __forceinline__ f32x4 mma_xw(const XF<P>& a, const WF<P>* b, f32x4 c) {
  if constexpr (P == P_BF16) {
    return mfma16x16x32(a.h, b->h, c);
  } else if constexpr (P == P_X3) {
    c = mfma16x16x32(a.l, b->h, c);
    c = mfma16x16x32(a.h, b->l, c);
    return mfma16x16x32(a.h, b->h, c);
  } else {
    c = mfma8(a.q, b->lo, c);
    return mfma8(a.q, b->hi, c);
  }
}

// 16x16x16 operands of the attention products (Sᵀ = K·Qᵀ, Oᵀ = Vᵀ·Pᵀ): bf16, or hi/lo pairs in X3
template <int P>
struct AF {
  bf16x4 h;
};
template <>
struct AF<P_X3> {
  bf16x4 h, l;
};
template <int P>
__device__ __forceinline__ AF<P> split4(const f32x4& v) {
  AF<P> r;
  r.h = cvt4(v);
  if constexpr (P == P_X3) r.l = cvt4(v - __builtin_convertvector(r.h, f32x4));
  return r;
}
template <int P>
__device__ __forceinline__ f32x4 mma16(const AF<P>& a, const AF<P>& b, f32x4 c) {
  if constexpr (P == P_X3) {
    c = mfma16x16x16(a.l, b.h, c);
    c = mfma16x16x16(a.h, b.l, c);
  }
  return mfma16x16x16(a.h, b.h, c);
}

// fp32 → operand conversions
template <int P>
__device__ __forceinline__ XF<P> split8(const f32x4& a, const f32x4& b) {
  XF<P> r;
  r.h = cvt8(a, b);
  if constexpr (P == P_X3) {
    const bf16x4 ha = {r.h[0], r.h[1], r.h[2], r.h[3]}, hb = {r.h[4], r.h[5], r.h[6], r.h[7]};
    r.l = cvt8(a - __builtin_convertvector(ha, f32x4), b - __builtin_convertvector(hb, f32x4));
  }
  return r;
}
__device__ __forceinline__ uint32_t fp8x4(const f32x4& v) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], w, true);
  return (uint32_t)w;
}

// ------------------------------------------------------------------ LDS images
// An activation image: `rows` × 128 features of plane(s) starting at byte `base` of the LDS window,
// RS bytes per row; the X3 lo plane sits `lo` bytes after the hi plane.
template <int P>
struct ImgBase {   // the lo-plane offset exists only where there is a lo plane
  char* base;
  int lo;
};
template <>
struct ImgBase<P_BF16> {
  char* base;
  static constexpr int lo = 0;
};
template <>
struct ImgBase<P_FP8> {
  char* base;
  static constexpr int lo = 0;
};
template <int P>
struct Img : ImgBase<P> {
  static constexpr int PREC = P;
  using ImgBase<P>::base;
  using ImgBase<P>::lo;
  __device__ __forceinline__ Img(char* b, int l) {
    base = b;
    if constexpr (P == P_X3) this->lo = l;
    (void)l;
  }
  __device__ __forceinline__ Img() = default;
#ifdef CET_IMG_SWZ
  static constexpr bool SWZ = P != P_FP8;
#else
  static constexpr bool SWZ = false;
#endif
  // byte offset of (row, byte) in a plane.  SWZ (RS = 288): byte bits 4-5 XOR-ed with row bits 2-3.  The
  // 32-byte row skew alone makes an MFMA operand read (ds_read_b128: lanes of rows c = 0-15 over two adjacent
  // 16-byte chunks per lane group) conflict-free but the image writes (ds_write_b64: 16 rows, one column, 32
  // banks) 4-way; the XOR spreads those rows back to 2-way and keeps the reads conflict-free
  // (tools/lds_bank_model.py, tools/probe/lds_probe.hip).  It touches neither bit 6-7 (the k-step, an
  // immediate offset) nor, for rows mt·16 + c, anything but c: one per-lane term per access pattern.  A view
  // must start on a row ≡ 0 (mod 16) of its image (ImgRows shifts rows instead)
  static __device__ __forceinline__ int off(int row, int byte) {
    constexpr int RS = Geo<P>::RS;
    // spelled so that the XOR sees only the lane-dependent parts (byte bits 4-5, row bits 2-3): for rows
    // mt·16 + c and bytes ks·64 + 16g the term is one per-lane value and mt, ks stay immediate offsets
    if constexpr (SWZ) return row * RS + (byte & ~48) + ((byte & 48) ^ ((row << 2) & 48));
    return row * RS + byte;
  }
  __device__ __forceinline__ XF<P> ld(int row, int k0) const {
    constexpr int RS = Geo<P>::RS;
#ifdef CET_ABL_LDSROW
    row &= ~15;   // ablation (wrong results): every lane group reads one row — conflict-free, same instructions
#endif
    XF<P> r;
    if constexpr (P == P_FP8) {
      r.q = *reinterpret_cast<const long*>(base + row * RS + k0);
    } else {
      const int o = off(row, 2 * k0);
      r.h = *reinterpret_cast<const bf16x8*>(base + o);
      if constexpr (P == P_X3) r.l = *reinterpret_cast<const bf16x8*>(base + lo + o);
    }
    return r;
  }
  __device__ __forceinline__ void st4(int row, int n0, const f32x4& v) const {
    constexpr int RS = Geo<P>::RS;
    if constexpr (P == P_FP8) {
      *reinterpret_cast<uint32_t*>(base + row * RS + n0) = fp8x4(v);
    } else {
      const bf16x4 h = cvt4(v);
      const int o = off(row, 2 * n0);
      *reinterpret_cast<bf16x4*>(base + o) = h;
      if constexpr (P == P_X3) *reinterpret_cast<bf16x4*>(base + lo + o) = cvt4(v - __builtin_convertvector(h, f32x4));
    }
  }
  __device__ __forceinline__ void st1(int row, int n, float v) const {
    constexpr int RS = Geo<P>::RS;
    if constexpr (P == P_FP8) {
      *reinterpret_cast<uint8_t*>(base + row * RS + n) = (uint8_t)__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false);
    } else {
      const __bf16 h = (__bf16)v;
      const int o = off(row, 2 * n);
      *reinterpret_cast<__bf16*>(base + o) = h;
      if constexpr (P == P_X3) *reinterpret_cast<__bf16*>(base + lo + o) = (__bf16)(v - (float)h);
    }
  }
};

// rows r0 .. of an image as a writer's rows 0 .. (the encoder norm's rows of the stack output)
template <int P>
struct ImgRows {
  Img<P> im;
  int r0;
  __device__ __forceinline__ void st4(int row, int n0, const f32x4& v) const { im.st4(row + r0, n0, v); }
};

// B-operand loaders
template <int P>
struct LoadImg {
  Img<P> im;
  __device__ __forceinline__ XF<P> operator()(int m, int k0) const { return im.ld(m, k0); }
};
// Circular k=3 conv input: A[m][tap·128 + c] = X[(m-1+tap) mod L][c]
template <int P>
struct LoadCirc3 {
  Img<P> im;
  int L;
  __device__ __forceinline__ XF<P> operator()(int m, int k0) const {
    const int tap = k0 >> 7, c = k0 & 127;
    int r = m - 1 + tap;
    r = r < 0 ? r + L : r;
    r = r >= L ? r - L : r;
    r = r >= L ? L - 1 : r;  // padded rows only
    return im.ld(r, c);
  }
};
// The same conv input with the m-tiles in even/odd position order (for the pooling that follows):
// tile 2j holds positions 32j + 2c, tile 2j+1 positions 32j + 2c + 1 (c = the tile row).
template <int P>
struct LoadCirc3EO {
  Img<P> im;
  int L;
  __device__ __forceinline__ XF<P> operator()(int m, int k0) const {
    const int mt = m >> 4;
    const int pos = ((mt >> 1) << 5) + ((m & 15) << 1) + (mt & 1);
    const int tap = k0 >> 7, c = k0 & 127;
    int r = pos - 1 + tap;
    r = r < 0 ? r + L : r;
    r = r >= L ? r - L : r;
    r = r >= L ? L - 1 : r;  // padded positions only
    return im.ld(r, c);
  }
};
// Token-embedding input for output row m = position m + off (EncoderStack window):
// A[m][tap·C + c] = x[(m + off - 1 + tap) mod L][c], zero past 3·C (C a power of two).  The embedding
// is never quantised: P here is plain_of<>.
template <int P>
struct LoadEmbed {
  const float* X;
  int L, CSH, CS, off;
  __device__ __forceinline__ XF<P> operator()(int m, int k0) const {
    const int tap = k0 >> CSH, c = k0 & ((1 << CSH) - 1);
    if (tap >= 3) return XF<P>{};
    int r = m + off - 1 + tap;
    r = r < 0 ? r + L : r;
    r = r >= L ? r - L : r;
    r = r >= L ? L - 1 : r;  // padded rows (m >= L) only: any valid row
    const f32x4* p = reinterpret_cast<const f32x4*>(X + r * CS + c);
    return split8<P>(p[0], p[1]);
  }
};

// ------------------------------------------------------------------ weights and parameters
struct Mem {
  __amdgpu_buffer_rsrc_t w;   // packed fragments [n_tile][k_step][lane][16 B]
  __amdgpu_buffer_rsrc_t p;   // fp32 parameter blob
  uint32_t wlo;               // X3: byte offset of the lo-fragment blob
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7ffffff0, 0x00020000);
}
__device__ __forceinline__ uint4 wload16(const Mem& m, uint32_t off, int lane) {
#ifdef CET_ABL_WL1
  off &= 0x3C00u;   // ablation (wrong results): every weight tile from one L1-resident 16 KiB window
#endif
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(m.w, lane * 16, (int)off, 0));
}
// this lane's fragment of the 1 KiB wave tile at uniform byte offset `off`
template <int P>
__device__ __forceinline__ WF<P> wfrag(const Mem& m, uint32_t off, int lane) {
  WF<P> r;
  const uint4 v = wload16(m, off, lane);
  if constexpr (P == P_FP8) {
    r.hi = (long)(((unsigned long long)v.y << 32) | v.x);
    r.lo = (long)(((unsigned long long)v.w << 32) | v.z);
  } else {
    r.h = __builtin_bit_cast(bf16x8, v);
    if constexpr (P == P_X3) r.l = __builtin_bit_cast(bf16x8, wload16(m, off + m.wlo, lane));
  }
  return r;
}
__device__ __forceinline__ f32x4 pload4(const Mem& m, uint32_t so, int vo) {
#ifdef CET_ABL_PL1
  so &= 0xFFu;   // ablation (wrong results): parameter vectors from one L1-resident window
#endif
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(m.p, vo * 4, (int)(so * 4u), 0));
}
__device__ __forceinline__ float pload1(const Mem& m, uint32_t so, int vo) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(m.p, vo * 4, (int)(so * 4u), 0));
}
__device__ __forceinline__ f32x4 load4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// Lane index the compiler cannot hoist (keeps lane-derived addresses from living across phases).
__device__ __forceinline__ int lane_op() {
  int l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
#ifndef CET_NO_LANE_ASSUME
  // the range survives the opaque move: lane-derived k offsets (< 32) fold into compile-time taps
  __builtin_assume(l >= 0 && l < 64);
#endif
  return l;
}

template <int P, int KS>
__device__ __forceinline__ void load_frags(const Mem& m, uint32_t base, int nt, WF<P> (&a)[KS]) {
  const int lane = lane_op();
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) a[ks] = wfrag<P>(m, base * 16u + (uint32_t)(nt * KS + ks) * 1024u, lane);
}
__device__ __forceinline__ void epi_vecs(const Mem& m, const GemmDesc& d, int n0, f32x4& sc, f32x4& bi) {
  sc = f32x4{1.f, 1.f, 1.f, 1.f};
  bi = f32x4{0.f, 0.f, 0.f, 0.f};
  if (d.scale != NONE) sc = pload4(m, d.scale, n0);
  if (d.bias != NONE) bi = pload4(m, d.bias, n0);
}

template <int N>
struct Res {
  f32x4 v[N];
};

// ------------------------------------------------------------------ decoder weight feed (LDS-DMA)
// The decoder's weight tiles (1 KiB wave tiles of the fragment blob) stream into per-wave LDS slots with
// buffer_load_dwordx4 … lds (no VGPR destination), six tiles ahead of their use, and its bias / LayerNorm
// vectors arrive the same way as one 1 KiB parameter tile per (layer, wave) (cet_api.cpp build_informer).  The
// slots live in LDS the decoder leaves unused (bf16 layout): image rows 16–95 of XB and of CTX, the LayerNorm
// partials past row 15 and the multiplicity table — 57 slots; wave w owns ring slots 6w .. 6w + 5 and
// parameter slot 48 + w.  hipcc does not count these loads: the issuing wave retires them with its own counted
// s_waitcnt vmcnt and reads only its own slots, so no barrier orders them.
typedef unsigned v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u32 raw_rsrc(const void* base) {   // the descriptor make_rsrc builds, as a value
  const uint64_t p = (uint64_t)base;
  return v4u32{(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)p),
               (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)(p >> 32) & 0xffffu)), 0x7ffffff0u, 0x00020000u};
}
// one 1 KiB wave tile at blob byte offset soff → LDS bytes [dst, dst + 1024): lane l's 16 bytes at dst + 16·l
__device__ __forceinline__ void dma_tile(v4u32 rsrc, uint32_t soff, uint32_t dst, int voff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(dst), "s"(soff)
      : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
constexpr int FEED_R = 6;   // ring tiles per wave
constexpr uint32_t FEED_XB = 16 * V4_RS16;                                  // XB rows 16..95: 21 slots
constexpr uint32_t FEED_CTX = (uint32_t)v4_ctx(0) + 16 * V4_RS16;           // CTX rows 16..95: 21 slots
constexpr uint32_t FEED_SCR = (uint32_t)v4_scr(0) + 16 * LN_STRIDE * 4;    // LN partials past row 15: 6 slots
constexpr uint32_t FEED_CNT = (uint32_t)v4_cnt(0);                          // the multiplicity table: 9 slots
static_assert(FEED_XB + 21 * 1024 <= (uint32_t)v4_ctx(0), "XB slots inside XB");
static_assert(FEED_CTX + 21 * 1024 <= (uint32_t)v4_scr(0), "CTX slots inside CTX");
static_assert(FEED_SCR + 6 * 1024 <= (uint32_t)v4_scr(0) + LMAX * LN_STRIDE * 4, "slots below the LN statistics");
static_assert(FEED_CNT + 8 * 1024 <= (uint32_t)v4_enc(0), "CNT slots inside the table");
__device__ __forceinline__ uint32_t feed_slot(int i) {
  return i < 21 ? FEED_XB + 1024u * i
       : i < 42 ? FEED_CTX + 1024u * (i - 21)
       : i < 48 ? FEED_SCR + 1024u * (i - 42)
                : FEED_CNT + 1024u * (i - 48);
}

// A dense layer's per-wave operands, requested ahead of the barrier that precedes the layer.
template <int P, int KS>
struct WPre {
  WF<P> a[KS];
  f32x4 sc, bi;
};
template <int P, int KS>
__device__ __forceinline__ WPre<P, KS> prefetch_res(const Mem& m, const GemmDesc d) {
  WPre<P, KS> p;
  const int lane = lane_op(), w = wave_id();
  load_frags<P, KS>(m, d.w, w, p.a);
  epi_vecs(m, d, 16 * w + (lane >> 4) * 4, p.sc, p.bi);
  return p;
}

// Dense layer whose output n-tile w lands in the wave's residual fragments (runtime m-tile count).
template <int P, int KS, int N, class BL, class Epi>
__device__ __forceinline__ void gemm_res(const WPre<P, KS>& p, int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_op(), w = wave_id();
  const int n0 = 16 * w + (lane >> 4) * 4;
  const int kq = kq_of<P>(lane), mrow = lane & 15;
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ks += KR<P>) c = mma<P>(&p.a[ks], bl(mt * 16 + mrow, ks * 32 + kq), c);
      epi(mt, n0, c * p.sc + p.bi);
    }
  }
}
template <int P, int KS, int N, class BL, class Epi>
__device__ __forceinline__ void gemm_res(const Mem& m, const GemmDesc d, int nmt, BL&& bl, Epi&& epi) {
  gemm_res<P, KS, N>(prefetch_res<P, KS>(m, d), nmt, bl, epi);
}

// Compile-time m-tile count: B fragments of tile mt+1 requested before the MFMAs of tile mt.
template <int P, int KS, int NMT, class BL, class Epi>
__device__ __forceinline__ void gemm_res_n(const WPre<P, KS>& p, BL&& bl, Epi&& epi) {
  const int lane = lane_op(), w = wave_id();
  const int n0 = 16 * w + (lane >> 4) * 4;
  const int kq = kq_of<P>(lane), mrow = lane & 15;
  XF<P> b[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ks += KR<P>) b[ks] = bl(mrow, ks * 32 + kq);
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    XF<P> bn[KS];
    if (mt + 1 < NMT) {
#pragma unroll
      for (int ks = 0; ks < KS; ks += KR<P>) bn[ks] = bl((mt + 1) * 16 + mrow, ks * 32 + kq);
    }
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ks += KR<P>) c = mma<P>(&p.a[ks], b[ks], c);
    epi(mt, n0, c * p.sc + p.bi);
    if (mt + 1 < NMT) {
#pragma unroll
      for (int ks = 0; ks < KS; ks += KR<P>) b[ks] = bn[ks];
    }
  }
}
template <int P, int KS, int NMT, class BL, class Epi>
__device__ __forceinline__ void gemm_res_n(const Mem& m, const GemmDesc d, BL&& bl, Epi&& epi) {
  gemm_res_n<P, KS, NMT>(prefetch_res<P, KS>(m, d), bl, epi);
}

// Dense layer over an arbitrary n-tile count (the projection), output through epi only.
template <int P, int KS, class BL, class Epi>
__device__ __forceinline__ void gemm_tiles(const Mem& m, const GemmDesc d, int n_tiles, int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_op(), w = wave_id();
  const int kq = kq_of<P>(lane), mrow = lane & 15;
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
    WF<P> a[KS];
    load_frags<P, KS>(m, d.w, nt, a);
    const int n0 = nt * 16 + (lane >> 4) * 4;
    f32x4 sc, bi;
    epi_vecs(m, d, n0, sc, bi);
    for (int mt = mt0; mt < nmt; mt += mt_step) {
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ks += KR<P>) c = mma<P>(&a[ks], bl(mt * 16 + mrow, ks * 32 + kq), c);
      epi(mt, n0, c * sc + bi);
    }
  }
}

// n_tiles ≤ NW (FFN hidden): wave w takes n-tile w mod n_tiles and every (NW / n_tiles)-th m-tile.
template <int P, int KS>
__device__ __forceinline__ WPre<P, KS> prefetch_tiles(const Mem& m, const GemmDesc d, int n_tiles) {
  WPre<P, KS> p;
  const int lane = lane_op(), w = wave_id();
  const int nt = w % n_tiles;
  load_frags<P, KS>(m, d.w, nt, p.a);
  epi_vecs(m, d, nt * 16 + (lane >> 4) * 4, p.sc, p.bi);
  return p;
}
template <int P, int KS, class BL, class Epi>
__device__ __forceinline__ void gemm_tiles1(const WPre<P, KS>& p, int n_tiles, int nmt, BL&& bl, Epi&& epi) {
  const int lane = lane_op(), w = wave_id();
  const int kq = kq_of<P>(lane), mrow = lane & 15;
  const int per = NW / n_tiles;
  if (w >= per * n_tiles) return;
  const int nt = w % n_tiles, mt_step = per;
  const int n0 = nt * 16 + (lane >> 4) * 4;
  for (int mt = w / n_tiles; mt < nmt; mt += mt_step) {
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ks += KR<P>) c = mma<P>(&p.a[ks], bl(mt * 16 + mrow, ks * 32 + kq), c);
    epi(mt, n0, c * p.sc + p.bi);
  }
}

// Deep-K dense layer (the distil conv, K = 384) in k-outer order with a compile-time m-tile count:
// one accumulator per m-tile, the B fragments of step ks+1 requested before step ks's MFMAs, and the
// weight fragments loaded in groups of KH k-steps.
template <int P, int KS, int KH>
__device__ __forceinline__ WPre<P, KH> prefetch_kouter(const Mem& m, const GemmDesc d) {
  WPre<P, KH> p;
  const int lane = lane_op(), w = wave_id();
#pragma unroll
  for (int ks = 0; ks < KH; ++ks) p.a[ks] = wfrag<P>(m, d.w * 16u + (uint32_t)(w * KS + ks) * 1024u, lane);
  epi_vecs(m, d, 16 * w + (lane >> 4) * 4, p.sc, p.bi);
  return p;
}
template <int P, int KS, int KH, int NMT, class BL, class Epi>
__device__ __forceinline__ void gemm_kouter_res(const WPre<P, KH>& p, const Mem& m, const GemmDesc d, BL&& bl,
                                                Epi&& epi) {
  static_assert(KS % KH == 0 && KH % KR<P> == 0, "k-steps split into equal groups");
  const int lane = lane_op(), w = wave_id();
  const int kq = kq_of<P>(lane), mrow = lane & 15;
  const int n0 = 16 * w + (lane >> 4) * 4;
  const f32x4 sc = p.sc, bi = p.bi;
  f32x4 c[NMT];
  XF<P> b[NMT];
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    c[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    b[mt] = bl(mt * 16 + mrow, kq);
  }
  const uint32_t t0 = d.w * 16u + (uint32_t)(w * KS) * 1024u;
#pragma unroll
  for (int hf = 0; hf < KS / KH; ++hf) {
    WF<P> a[KH];
#pragma unroll
    for (int ks = 0; ks < KH; ++ks) a[ks] = hf == 0 ? p.a[ks] : wfrag<P>(m, t0 + (uint32_t)(hf * KH + ks) * 1024u, lane);
#pragma unroll
    for (int ks = 0; ks < KH; ks += KR<P>) {
      const int kk = hf * KH + ks;
      XF<P> bn[NMT];
      if (kk + KR<P> < KS) {
#pragma unroll
        for (int mt = 0; mt < NMT; ++mt) bn[mt] = bl(mt * 16 + mrow, (kk + KR<P>) * 32 + kq);
      }
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt) c[mt] = mma<P>(&a[ks], b[mt], c[mt]);
      if (kk + KR<P> < KS) {
#pragma unroll
        for (int mt = 0; mt < NMT; ++mt) b[mt] = bn[mt];
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch distance at one k-step
    }
  }
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) epi(mt, n0, c[mt] * sc + bi);
}

// One-pass LayerNorm, step 1: each wave publishes (Σx, Σx²) over its 16 features per row.  The two
// butterflies share their swaps: permlane16_swap(s, q) leaves rows (s0+s1, q0+q1, s2+s3, q2+q3) after one
// add, and the 32-lane swap then gives Σs in rows 0 / 2 and Σq in rows 1 / 3 — lanes g and g + 2 store the
// same word to the same address, so the publish needs no branch.
template <int N>
__device__ __forceinline__ void ln_publish(const Res<N>& X, int nmt, float* part) {
  const int lane = lane_op(), w = wave_id(), g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      const f32x4 x = X.v[mt];
      // on the fragment's natural register pairs: packed math with no operand moves
      const f32x2 hs = x.xy + x.zw, hq = x.xy * x.xy + x.zw * x.zw;
      const float s = hs.x + hs.y, q = hq.x + hq.y;
      const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s), __float_as_uint(q), false, false);
      const float t = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(t), __float_as_uint(t), false, false);
      part[(mt * 16 + c) * LN_STRIDE + 2 * w + (g & 1)] = __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
    }
  }
}

// row statistics (mean, 1/std) of row m from the 8 waves' (Σx, Σx²)
__device__ __forceinline__ f32x2 ln_row_stats(const float* part, int m, float eps, bool unbiased_std) {
  const float* pr = part + m * LN_STRIDE;
  const f32x4 p0 = load4(pr), p1 = load4(pr + 4), p2 = load4(pr + 8), p3 = load4(pr + 12);
  // (Σx, Σx²) pairs summed as pairs (packed adds on the loaded register pairs)
  const f32x2 t = ((p0.xy + p0.zw) + (p1.xy + p1.zw)) + ((p2.xy + p2.zw) + (p3.xy + p3.zw));
  const float sx = t.x, sq = t.y;
  const float mean = sx * (1.0f / 128.0f);
  const float M2 = fmaxf(fmaf(-sx, mean, sq), 0.f);   // Σx² − (Σx)²/128
  const float inv = unbiased_std ? __builtin_amdgcn_rcpf(sqrtf(M2 * (1.0f / 127.0f)) + eps)
                                 : __builtin_amdgcn_rsqf(M2 * (1.0f / 128.0f) + eps);
  return f32x2{mean, inv};
}

// step 2 in the own-rows form: every wave combines the partials of the rows it holds and normalises them
template <int N, class Out, class Out2, bool INPLACE = true>
__device__ __forceinline__ void ln_apply_own(Res<N>& X, int nmt, int rows, f32x4 g0, f32x4 b0, float eps,
                                             bool unbiased_std, const float* part, const Out& out, const Out2* out2) {
  const int lane = lane_op(), w = wave_id(), c = lane & 15;
  const int nb = 16 * w + 4 * (lane >> 4);
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      const int m = mt * 16 + c;
      const f32x2 st = ln_row_stats(part, m, eps, unbiased_std);
      const f32x4 y = (X.v[mt] - st[0]) * st[1] * g0 + b0;
      if (INPLACE) X.v[mt] = y;
      if (m < rows) {
        out.st4(m, nb, y);
        if (out2) out2->st4(m, nb, y);
      }
    }
  }
}

// LayerNorm of the register residual over all 128 features (8 waves × 16).
//   1. each wave reduces its 16 features per row to (Σx, Σx²) and stores the pair (LDS partials);
//   2. wave w < nmt combines the 8 pairs of the rows of m-tile w into (mean, 1/std) per row — once per
//      row, not once per wave (-DCET_LN_TWOPASS: per-wave (mean, M2) and Chan's combination);
//   3. every wave normalises its fragments from those row statistics.
// Normalised rows go to X and rows < `rows` to the image `out` (and `out2`).  torch.nn.LayerNorm
// (biased var, eps in the sqrt) or, if unbiased_std, the reference Transformer's LayerNormalization.
// Two workgroup barriers inside; the caller adds one before the image is read.
// INPLACE = false (pre-LN residual blocks, models/Transformer buildingblocks.py:214-226): the
// normalised rows only go to the image(s); X keeps the residual.
// lst (diagnostics, the C2 + stamps build): per-wave s_memtime at entry, after each barrier and at exit, in
// lst[4·w + 0..3] — which part of a LayerNorm phase is the wave's own work and which is waiting for the others.
// ln_res_gb: γ / β of the wave's four features given (the decoder weight feed reads them from its parameter
// tile); ln_res below loads them from the parameter blob.
template <int N, class Out, class Out2, bool INPLACE = true>
__device__ __forceinline__ void ln_res_gb(Res<N>& X, int nmt, int rows, const f32x4 g0, const f32x4 b0, float eps,
                                          bool unbiased_std, float* part, const Out& out, const Out2* out2,
                                          unsigned long long* lst = nullptr, unsigned* arrive = nullptr) {
  const int lane = lane_op(), w = wave_id(), g = lane >> 4, c = lane & 15;
  const int nb = 16 * w + 4 * g;
  float* stats = part + LMAX * LN_STRIDE;   // [LMAX] (mean, 1/std): the scratch's last 768 bytes
  auto LST = [&](int k) __attribute__((always_inline)) {
    if (lst && lane == 0) lst[4 * w + k] = __builtin_amdgcn_s_memtime();
  };
  LST(0);
#ifdef CET_ABL_LN
  // ablation (wrong results): no row statistics, no barriers — the LayerNorm's own cost, measured by its absence
  (void)part; (void)stats; (void)eps; (void)unbiased_std;
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      const int m = mt * 16 + c;
      const f32x4 y = X.v[mt] * g0 + b0;
      if (INPLACE) X.v[mt] = y;
      if (m < rows) {
        out.st4(m, nb, y);
        if (out2) out2->st4(m, nb, y);
      }
    }
  }
  return;
#endif
#ifdef CET_LN_LAST
  if constexpr (N > 1) {
    if (arrive) {
      // one barrier instead of two: each wave counts itself in after publishing its partials (LDS executes a
      // wave's operations in order, so the count follows its stores), and the last to arrive combines every row
      // and re-arms the counter before the barrier
      ln_publish(X, nmt, part);
      unsigned t = 0;
      if (lane == 0) t = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
      t = (unsigned)__builtin_amdgcn_readfirstlane((int)t);
      if (t == (unsigned)(NW - 1)) {
        for (int m = lane; m < nmt * 16; m += WAVE)
          *reinterpret_cast<f32x2*>(stats + 2 * m) = ln_row_stats(part, m, eps, unbiased_std);
        if (lane == 0) __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __syncthreads();
      LST(1);
      LST(2);
#pragma unroll
      for (int mt = 0; mt < N; ++mt) {
        if (mt < nmt) {
          const int m = mt * 16 + c;
          const f32x2 st = *reinterpret_cast<const f32x2*>(stats + 2 * m);
          const f32x4 y = (X.v[mt] - st[0]) * st[1] * g0 + b0;
          if (INPLACE) X.v[mt] = y;
          if (m < rows) {
            out.st4(m, nb, y);
            if (out2) out2->st4(m, nb, y);
          }
        }
      }
      LST(3);
      return;
    }
  }
#endif
#ifndef CET_LN_TWOPASS
  ln_publish(X, nmt, part);
  __syncthreads();
  LST(1);
  auto row_stats = [&](int m) __attribute__((always_inline)) { return ln_row_stats(part, m, eps, unbiased_std); };
#ifndef CET_LN_TWO_BARRIER
#ifndef CET_LN_ONE_MAX
#define CET_LN_ONE_MAX 1
#endif
  if constexpr (N <= CET_LN_ONE_MAX) {
    // few m-tiles (the decoder's 15 rows): every wave combines its own rows' partials — no second
    // barrier; the caller's barrier after the LN orders these reads before the partials are rewritten.
    // For the encoder's 3-6 tiles the redundant combining costs more than the barrier it saves
    // (-DCET_LN_ONE_MAX=3 ±0, =6 +1.2 us; profiles/r04/ab9/ab.log)
    ln_apply_own<N, Out, Out2, INPLACE>(X, nmt, rows, g0, b0, eps, unbiased_std, part, out, out2);
    LST(3);
    return;
  }
#endif
  // wave w < nmt: the rows of m-tile w, once per row (every lane group stores the same pair)
  if (w < nmt) *reinterpret_cast<f32x2*>(stats + 2 * (w * 16 + c)) = row_stats(w * 16 + c);
#else
  // two passes (mean, then Σ(x − mean)²) per wave, Chan's combination over the waves
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
  if (w < nmt) {
    const int m = w * 16 + c;
    const float* pr = part + m * LN_STRIDE;
    const f32x4 p0 = load4(pr), p1 = load4(pr + 4), p2 = load4(pr + 8), p3 = load4(pr + 12);
    const float mean = 0.125f * (((p0[0] + p0[2]) + (p1[0] + p1[2])) + ((p2[0] + p2[2]) + (p3[0] + p3[2])));
    const float d0 = p0[0] - mean, d1 = p0[2] - mean, d2 = p1[0] - mean, d3 = p1[2] - mean;
    const float d4 = p2[0] - mean, d5 = p2[2] - mean, d6 = p3[0] - mean, d7 = p3[2] - mean;
    const float M2 = (((p0[1] + p0[3]) + (p1[1] + p1[3])) + ((p2[1] + p2[3]) + (p3[1] + p3[3]))) +
                     16.0f * ((d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3) + (d4 * d4 + d5 * d5 + d6 * d6 + d7 * d7));
    const float inv = unbiased_std ? __builtin_amdgcn_rcpf(sqrtf(M2 * (1.0f / 127.0f)) + eps)
                                   : __builtin_amdgcn_rsqf(M2 * (1.0f / 128.0f) + eps);
    if (g == 0) *reinterpret_cast<f32x2*>(stats + 2 * m) = f32x2{mean, inv};
  }
#endif
  __syncthreads();
  LST(2);
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      const int m = mt * 16 + c;
      const f32x2 st = *reinterpret_cast<const f32x2*>(stats + 2 * m);
      const f32x4 y = (X.v[mt] - st[0]) * st[1] * g0 + b0;
      if (INPLACE) X.v[mt] = y;
      if (m < rows) {
        out.st4(m, nb, y);
        if (out2) out2->st4(m, nb, y);
      }
    }
  }
  LST(3);
}
template <int N, class Out, class Out2, bool INPLACE = true>
__device__ __forceinline__ void ln_res(Res<N>& X, int nmt, int rows, const Mem& mm, const LNDesc ln, float eps,
                                       bool unbiased_std, float* part, const Out& out, const Out2* out2,
                                       unsigned long long* lst = nullptr, unsigned* arrive = nullptr) {
  const int nb = 16 * wave_id() + 4 * (lane_op() >> 4);
  const f32x4 g0 = pload4(mm, ln.g, nb), b0 = pload4(mm, ln.b, nb);   // issued before the barriers
  ln_res_gb<N, Out, Out2, INPLACE>(X, nmt, rows, g0, b0, eps, unbiased_std, part, out, out2, lst, arrive);
}

// Two torch.nn.LayerNorms under one barrier, both in the own-rows form: the fused decoder layer 0's LN1
// (decoder.py:31) beside the last encoder layer's LN1 (encoder.py:50) in the shape instances.  Each has its
// own partials; the caller's barrier after it orders the reads before either is rewritten.
template <int N1, int N2, class O1, class O2>
__device__ __forceinline__ void ln_res_pair(Res<N1>& X1, int nmt1, int rows1, const LNDesc ln1, float* part1,
                                            const O1& out1, Res<N2>& X2, int nmt2, int rows2, const LNDesc ln2,
                                            float* part2, const O2& out2, const Mem& mm, float eps) {
  const int lane = lane_op(), w = wave_id();
  const int nb = 16 * w + 4 * (lane >> 4);
  const f32x4 g1 = pload4(mm, ln1.g, nb), b1 = pload4(mm, ln1.b, nb);
  const f32x4 g2 = pload4(mm, ln2.g, nb), b2 = pload4(mm, ln2.b, nb);
  ln_publish(X1, nmt1, part1);
  ln_publish(X2, nmt2, part2);
  __syncthreads();
  ln_apply_own<N1, O1, O1>(X1, nmt1, rows1, g1, b1, eps, false, part1, out1, (const O1*)nullptr);
  ln_apply_own<N2, O2, O2>(X2, nmt2, rows2, g2, b2, eps, false, part2, out2, (const O2*)nullptr);
}

// image of the register residual (rows < rows)
template <int N, class Out>
__device__ __forceinline__ void store_res(const Res<N>& X, int nmt, int rows, const Out& out) {
  const int lane = lane_op(), w = wave_id();
  const int nb = 16 * w + 4 * (lane >> 4);
#pragma unroll
  for (int mt = 0; mt < N; ++mt) {
    if (mt < nmt) {
      const int m = mt * 16 + (lane & 15);
      if (m < rows) out.st4(m, nb, X.v[mt]);
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

// MaxPool1d(kernel 3, stride 2, padding 1) over even/odd-ordered tiles (LoadCirc3EO): pooled row
// t' = 16j + c = max(x[2t'], x[2t'+1], x[2t'-1]) = max(E_j[c], O_j[c], O_j[c-1]) where O_j[c-1] for
// c = 0 is O_{j-1}[15].  The one-row shift is a DPP row rotate (no LDS, no permute through LDS).
__device__ __forceinline__ float ror1(float v) {   // lane c of each 16-lane row gets lane (c-1) mod 16
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x121, 0xf, 0xf, false));
}
template <int NIN>
__device__ __forceinline__ void maxpool_eo(const Res<NIN>& in, int L, Res<MT>& out) {
  static_assert(NIN % 2 == 0, "even/odd tile pairs");
  constexpr int NOUT = NIN / 2;
  const int c = lane_op() & 15;
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
    const int t = 16 * j + c;
    const bool has_odd = 2 * t + 1 < L, has_prev = t > 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = in.v[2 * j][r], o = in.v[2 * j + 1][r];
      const float os = ror1(o);
      const float ps = j > 0 ? ror1(in.v[2 * j - 1][r]) : NEG_INF;
      const float m1 = c == 0 ? ps : os;
      float v = e;
      if (has_odd) v = fmaxf(v, o);
      if (has_prev) v = fmaxf(v, m1);
      out.v[j][r] = v;
    }
  }
#pragma unroll
  for (int j = NOUT; j < MT; ++j) out.v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

template <int N>
using IC = std::integral_constant<int, N>;

// Diagnostic (CET_LDS_POISON=1): every byte of the workgroup's dynamic LDS set to 0xFF — NaN as fp32, bf16 and
// e4m3 — before the kernel stages or zeroes anything, so a read of a byte nothing wrote in this launch is a
// deterministic NaN in the output instead of whatever the CU's previous workgroup left there.
template <int NT>
__device__ __forceinline__ void lds_poison(char* lds, int bytes) {
  for (int i = tid_op(); i < bytes / 16; i += NT) reinterpret_cast<uint4*>(lds)[i] = uint4{~0u, ~0u, ~0u, ~0u};
  __syncthreads();
}

__device__ __forceinline__ void stage(const float* __restrict__ src, float* dst, int L, int C, int CS) {
  for (int i = tid_op(); i < L * C; i += NTHREADS) {
    const int t = i / C, c = i - t * C;
    dst[t * CS + c] = src[i];
  }
}

// Plan access point: read through the constant address space behind an opaque pointer, so each
// phase re-loads its descriptors with scalar loads instead of keeping them live in SGPRs.
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
  asm volatile("" : "+s"(c));
  return c;
}

__device__ __forceinline__ GemmDesc part_of(GemmDesc d, int off) {
  if (d.bias != NONE) d.bias += off;
  if (d.scale != NONE) d.scale += off;
  return d;
}

// ------------------------------------------------------------------------------ attention
// One head per wave, everything in registers: Kᵀ = Wk_h·Xᵀ (A of Sᵀ = K·Qᵀ), Qᵀ = Wq_h·Xᵀ (B of Sᵀ),
// V = X·Wv_hᵀ (A of Oᵀ = Vᵀ·Pᵀ), and the exponentiated Sᵀ tile is the B fragment of Oᵀ.
// Reference: attn.py:73-175 (ProbAttention), :37-70 (FullAttention), :195-209 (AttentionLayer, mix).
// PD: precision of the Q/K/V projections (the model's dense policy); PA: of the attention products.
template <int PD>
struct HeadIO {
  Img<PD> xq, xkv;            // images feeding the queries / keys+values
  Img<PD> ctx;                // attention context out (the O-projection's input image)
  uint32_t wq, wk, wv;        // weight-blob offsets (16-byte units) of n-tile 0 of each projection
  GemmDesc dq, dk, dv;        // epilogue vectors (bias/scale offsets at the part's start)
  int LQ, LK, prob, causal, mix, u;
  const uint8_t* cnt;
  int cnt_stride;
  float* scr;                 // per-wave scratch: keys [96] u64, sel [96] int16, flag [96] bytes
  float* attn_out;            // global [H][LQ][LK] of this sequence or nullptr
  float* m_dbg;               // global [H][LQ] or nullptr
  unsigned long long* st;     // diagnostics: sub-phase s_memtime stamps of head 0, or nullptr
};

// The K and V weight fragments of head h and their epilogue vectors, requested ahead of their use.
template <int PD>
struct KVPre {
  WF<PD> k[4], v[4];
  f32x4 sk, bk;
  float sv, bv;
};
template <int PD>
__device__ __forceinline__ KVPre<PD> prefetch_kv(const HeadIO<PD>& io, const Mem& m, int h) {
  KVPre<PD> p;
  const int lane = lane_op();
  const int col = lane & 15, g = lane >> 4;
  load_frags<PD, 4>(m, io.wk, h, p.k);
  load_frags<PD, 4>(m, io.wv, h, p.v);
  epi_vecs(m, io.dk, 16 * h + 4 * g, p.sk, p.bk);
  p.sv = io.dv.scale != NONE ? pload1(m, io.dv.scale, 16 * h + col) : 1.f;
  p.bv = io.dv.bias != NONE ? pload1(m, io.dv.bias, 16 * h + col) : 0.f;
  return p;
}

// K and V tiles of head h from the key/value rows (attn.py:195-199): Kᵀ = Wk_h·Xᵀ as the A fragments
// of Sᵀ = K·Qᵀ, V = X·Wv_hᵀ as the A fragments of Oᵀ = Vᵀ·Pᵀ.
template <int PD, int MK>
__device__ __forceinline__ void project_kv(const HeadIO<PD>& io, const KVPre<PD>& w, AF<plain_of<PD>()> (&Kf)[MK],
                                           AF<plain_of<PD>()> (&Vf)[MK]) {
  constexpr int PA = plain_of<PD>();
  const int lane = lane_op();
  const int col = lane & 15;
  const int nkt = (io.LK + 15) >> 4;
  const int kq = kq_of<PD>(lane);
#pragma unroll
  for (int mt = 0; mt < MK; ++mt) {
    Kf[mt] = AF<PA>{};
    Vf[mt] = AF<PA>{};
    if (mt < nkt) {
      f32x4 k = {0.f, 0.f, 0.f, 0.f}, v = k;
#pragma unroll
      for (int ks = 0; ks < 4; ks += KR<PD>) {
        const XF<PD> bx = io.xkv.ld(mt * 16 + col, ks * 32 + kq);
        k = mma<PD>(&w.k[ks], bx, k);
        v = mma_xw<PD>(bx, &w.v[ks], v);
      }
#ifdef CET_MFMA_NOP
      // diagnostic (the ab8 investigation): 32 extra wait states between the K / V MFMA chains and
      // the VALU epilogue that reads their results
      asm volatile("s_nop 15\n\ts_nop 15" : "+v"(k), "+v"(v));
#endif
      Kf[mt] = split4<PA>(k * w.sk + w.bk);
      Vf[mt] = split4<PA>(v * w.sv + w.bv);
    }
  }
}
template <int PD, int MK>
__device__ __forceinline__ void project_kv(const HeadIO<PD>& io, const Mem& m, int h, AF<plain_of<PD>()> (&Kf)[MK],
                                           AF<plain_of<PD>()> (&Vf)[MK]) {
  project_kv<PD, MK>(io, prefetch_kv<PD>(io, m, h), Kf, Vf);
}

// EXTKV: the K/V tiles come from the caller (kin / vin, project_kv) instead of being projected here.
// NKX: the caller guarantees ceil(LK / 16) == MK (the key-tile bound is exact).
// qpre: the Q weight fragments and epilogue vectors of head h, requested by the caller ahead of time.
template <int PD, int MQ = MT, int MK = MT, bool EXTKV = false, bool NKX = false>
__device__ __forceinline__ void attention_head(const HeadIO<PD>& io, const Mem& m, int h,
                                               const AF<plain_of<PD>()>* kin = nullptr,
                                               const AF<plain_of<PD>()>* vin = nullptr,
                                               const WPre<PD, 4>* qpre = nullptr,
                                               const KVPre<PD>* kvpre = nullptr) {
  constexpr int PA = plain_of<PD>();
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
  const int fq = 16 * h + 4 * g;
  const int kq = kq_of<PD>(lane);
  AF<PA> Kf[MK], Vf[MK];
  // single-tile heads (the decoder's, and the last encoder layer's): few live registers, so the Q
  // weights could be requested with the K/V weights (one L2 round trip instead of two in sequence);
  // measured slower (126.5 vs 124.3 us, profiles/r02/ab_cross_hoist.log), so off unless CET_EARLYQ1
#ifdef CET_EARLYQ1
  constexpr bool EARLYQ = MQ == 1 && MK == 1;
#else
  constexpr bool EARLYQ = false;
#endif
  WF<PD> wq[4];
  f32x4 sq, bq;
  if constexpr (EARLYQ) {
    load_frags<PD, 4>(m, io.wq, h, wq);
    epi_vecs(m, io.dq, fq, sq, bq);
  }
  if constexpr (EXTKV) {
#pragma unroll
    for (int mt = 0; mt < MK; ++mt) {
      Kf[mt] = kin[mt];
      Vf[mt] = vin[mt];
    }
  } else if (kvpre) {
#ifdef CET_AB8_INV
    // diagnostic: invalidate the vector L1 before the caller's struct is read back from private
    // memory — does the ab8 build's wrong element come from a stale L1 line?
    asm volatile("buffer_inv sc1\n\ts_waitcnt vmcnt(0)" ::: "memory");
#endif
    project_kv<PD, MK>(io, *kvpre, Kf, Vf);   // weights requested by the caller (the CET_AB8 reproduction)
  } else {
    project_kv<PD, MK>(io, m, h, Kf, Vf);
  }
  SUB(1);
  // Q tiles are projected where they are consumed (per query tile in M, per selected tile in the
  // softmax): wq and its epilogue vectors are the only Q state that lives
  if constexpr (!EARLYQ) {
    if (qpre) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) wq[ks] = qpre->a[ks];
      sq = qpre->sc;
      bq = qpre->bi;
    } else {
      load_frags<PD, 4>(m, io.wq, h, wq);
      epi_vecs(m, io.dq, fq, sq, bq);
    }
  }
  auto project_q = [&](int row, float post = 1.f) __attribute__((always_inline)) {
    f32x4 q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ks += KR<PD>) q = mma<PD>(&wq[ks], io.xq.ld(row, ks * 32 + kq), q);
    return split4<PA>(post == 1.f ? q * sq + bq : (q * sq + bq) * post);
  };

  SUB(2);
  if (sparse) {
    // ---- sparsity measurement M (attn.py:95-105) from key multiplicities (LDS-staged table)
    const float invLK = 1.0f / (float)LK;
#pragma unroll
    for (int qt = 0; qt < MQ; ++qt) {
      if (qt >= nqt) break;
      const int q = qt * 16 + col;
      const AF<PA> qf = project_q(q);
      // this lane's six count words (keys 16kt + 4g + r, kt = 0..5) are contiguous (cnt_pos_v2)
      const uint2* crow = reinterpret_cast<const uint2*>(io.cnt + (size_t)q * io.cnt_stride + g * 24);
      const uint2 c01 = crow[0], c23 = crow[1], c45 = crow[2];
      const uint32_t cws[MT] = {c01.x, c01.y, c23.x, c23.y, c45.x, c45.y};
      // Σ count·score as two packed chains; the sampled maximum through min(score, bound) with the
      // bound count·2^64 − 2^63: ≥ 2^63 for a drawn key (the score passes), −2^63 for an undrawn one —
      // below every score, and every query row holds U ≥ 1 draws, so the row maximum is a drawn score
      constexpr float BND = 18446744073709551616.f, HALF = 9223372036854775808.f;
      f32x2 sum2 = {0.f, 0.f};
      float mx = -HALF;
#pragma unroll
      for (int kt = 0; kt < MK; ++kt) {
        if (kt < nkt) {
          const f32x4 s = mma16<PA>(Kf[kt], qf, f32x4{0.f, 0.f, 0.f, 0.f});
          const uint32_t cw = cws[kt];
          f32x4 cf;
#pragma unroll
          for (int r = 0; r < 4; ++r) cf[r] = (float)((cw >> (8 * r)) & 0xffu);
          sum2 = cf.xy * s.xy + sum2;
          sum2 = cf.zw * s.zw + sum2;
          const f32x4 bnd = cf * BND - HALF;
          // two keys per v_max3 (spelled out: the compiler re-pairs a max tree into three instructions)
          mx = max3f(mx, __builtin_fminf(s[0], bnd[0]), __builtin_fminf(s[1], bnd[1]));
          mx = max3f(mx, __builtin_fminf(s[2], bnd[2]), __builtin_fminf(s[3], bnd[3]));
        }
      }
      float sum = sum2.x + sum2.y;
      sum = xor_sum(sum, 16);
      sum = xor_sum(sum, 32);
      mx = xor_max(mx, 16);
      mx = xor_max(mx, 32);
      const float M = mx - sum * invLK;
      // selection key: order-preserving image of M above, ~q below — equal M go to the lower index
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
#ifdef CET_ABL_TOPU
    for (int qt = 0; qt < MQ; ++qt) rank[qt] = g == 0 ? qt * 16 + col : 0;   // ablation (wrong results)
    for (int j = 0; j < 0; j += 2) {
#else
#pragma unroll 2
    for (int j = 0; j < J; j += 2) {
#endif
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
  auto ctx_st4 = [&](int q, int e0, const f32x4& v) __attribute__((always_inline)) {
    if (!io.mix) {
      io.ctx.st4(q, h * 16 + e0, v);
    } else {
      const int f = h * LQ * 16 + q * 16 + e0;   // (L,H,E) values re-viewed as (H,L,E) memory
      io.ctx.st4(f >> 7, f & 127, v);
    }
  };
  if (sparse && !io.causal) {
    // ---- unselected rows keep the initial context, mean(V) (attn.py:116-119): written to every
    //      row here, then the selected rows are overwritten below (same wave, LDS in order).  The key
    //      sums come from the MFMA, Oᵀ = Vᵀ·I with I the indicator of the keys < L_K in every column:
    //      lane (g, c) then holds features 4g .. 4g+3 and stores them 4-wide into rows c, c + 16, …
    f32x4 vs = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < MK; ++kt)
      if (kt < nkt) {
        f32x4 ind;
#pragma unroll
        for (int j = 0; j < 4; ++j) ind[j] = kt * 16 + g * 4 + j < LK ? 1.f : 0.f;
        vs = mma16<PA>(Vf[kt], split4<PA>(ind), vs);
      }
    const f32x4 mean4 = vs * (1.0f / (float)LK);
    for (int q = col; q < LQ; q += 16) ctx_st4(q, g * 4, mean4);
  }
  SUB(4);

  // ---- softmax(scale·q·Kᵀ [mask])·V for the selected queries (attn.py:109-138 / 57-65).  The mask
  //      enters the score MFMA as its accumulator init (−inf on masked keys, 0 elsewhere), so neither
  //      sweep selects per score: the scores come out already scaled (2^-2 in the query operand) and
  //      exp2(−inf) = 0 zeroes the masked probabilities.  Non-causal calls mask only keys
  //      ≥ L_K, which lie in the last key tile (nkt == MK when NKX), computed once per call.
  const int nsel = sparse ? io.u : LQ;
  const int nst = (nsel + 15) >> 4;
  if constexpr (NKX) __builtin_assume(nkt == MK);
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  auto key_mask = [&](int kt, int lim) __attribute__((always_inline)) {   // keys ≥ lim → −inf
    f32x4 z;
#pragma unroll
    for (int r = 0; r < 4; ++r) z[r] = kt * 16 + g * 4 + r >= lim ? NEG_INF : 0.f;
    return z;
  };
  const f32x4 last_mask = key_mask(nkt - 1, LK);
#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    const int i = st * 16 + col;
    const int ic = i < nsel ? i : nsel - 1;
    const int qi = sparse ? (int)sel[ic] : ic;
    // the 1/√E = 2^-2 scale rides in the query operand (exact: a power of two)
    const AF<PA> qs = project_q(qi, 0.25f);
    const int lim = io.causal ? (qi + 1 < LK ? qi + 1 : LK) : LK;   // the first masked key of this query
    f32x4 init[MK];
#pragma unroll
    for (int kt = 0; kt < MK; ++kt) init[kt] = io.causal ? key_mask(kt, lim) : (kt == nkt - 1 ? last_mask : zero4);
    float mx = NEG_INF;
#pragma unroll
    for (int kt = 0; kt < MK; ++kt) {
      if (kt < nkt) {
        const f32x4 a = mma16<PA>(Kf[kt], qs, init[kt]);
        mx = __builtin_fmaxf(mx, __builtin_fmaxf(__builtin_fmaxf(a[0], a[1]), __builtin_fmaxf(a[2], a[3])));
      }
    }
    mx = xor_max(mx, 16);
    mx = xor_max(mx, 32);
    // p = exp2(s·log2e − max·log2e) on the scaled scores: one FMA and one v_exp_f32 per score
    constexpr float LOG2E = 1.4426950408889634f;
    mx *= LOG2E;
    auto prob = [&](float a) __attribute__((always_inline)) { return __builtin_amdgcn_exp2f(fmaf(a, LOG2E, -mx)); };
    float sum = 0.f;
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < MK; ++kt) {
      if (kt < nkt) {
        f32x4 p = mma16<PA>(Kf[kt], qs, init[kt]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[r] = prob(p[r]);
          sum += p[r];
        }
        o = mma16<PA>(Vf[kt], split4<PA>(p), o);
      }
    }
    sum = xor_sum(sum, 16);
    sum = xor_sum(sum, 32);
    const float inv = __builtin_amdgcn_rcpf(sum);
    if (i < nsel) {
      ctx_st4(qi, g * 4, o * inv);
      if (io.attn_out) {
        float* arow = io.attn_out + ((size_t)h * LQ + qi) * LK;
#pragma unroll
        for (int kt = 0; kt < MK; ++kt)
          if (kt < nkt) {
            const f32x4 p = mma16<PA>(Kf[kt], qs, init[kt]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int key = kt * 16 + g * 4 + r;
              if (key < LK) arow[key] = prob(p[r]) * inv;
            }
          }
      }
    }
  }

  SUB(5);
  if (sparse) {
    if (io.causal) {
      // masked: unselected rows keep cumsum(V) (attn.py:120-125) = Vᵀ·Tᵀ with T[q][key] = [key <= q]
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
              o = mma16<PA>(Vf[kt], split4<PA>(ind), o);
            }
          }
          if (q < LQ && !flag[q]) ctx_st4(q, g * 4, o);
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

}  // namespace v4
}  // namespace cet
