// Execution plans shared by the host runtime (cet_api.cpp) and the fused kernels.
// A plan is built once per engine on the host (shapes, weight offsets, LDS layout) and
// copied to device memory; the kernels read it through scalar loads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cet {

constexpr uint32_t NONE = 0xffffffffu;
constexpr int MAX_ENC = 4;
constexpr int MAX_ENC_LAYERS = 16;   // summed over the encoders of a stack
constexpr int MAX_DEC_LAYERS = 8;
constexpr int MAX_CALLS = MAX_ENC_LAYERS + MAX_DEC_LAYERS;
constexpr int LMAX = 96;             // longest (padded) sequence a workgroup keeps in LDS
constexpr int DMODEL = 128;
constexpr int NHEAD = 8;
constexpr int XS = 132;   // fp32 row stride (floats) of X-like LDS buffers (+16 B per row)
constexpr int BS = 136;
// v2 key-multiplicity row layout: key 16kt + 4g + r sits at byte 24g + 4kt + r of its 96-byte query
// row, so the lane holding keys 4g..4g+3 of every key tile reads one contiguous 24-byte run.
// (v1 rows are key-linear.)
__host__ __device__ inline int cnt_word_off(int key) { return ((key >> 2) & 3) * 24 + (key >> 4) * 4; }
__host__ __device__ inline int cnt_pos_v2(int key) { return cnt_word_off(key) + (key & 3); }
// v2 per-wave attention scratch: 96 u64 selection keys | 96 int16 selected rows | 96 flag bytes
constexpr int V2_SCR_FLOATS = 264;
// LayerNorm partials: floats per row (8 waves × (mean, M2) + pad; 80-byte rows put 16
// consecutive rows on distinct bank quads)
constexpr int LN3_STRIDE = 20;

// One dense layer: packed bf16 weights (fragment order) + fp32 epilogue vectors.
struct GemmDesc {
  uint32_t w;      // offset into the weight blob, in bf16x8 (16-byte) units
  uint32_t bias;   // float offset into the parameter blob (NONE: no bias)
  uint32_t scale;  // float offset of a per-output scale (NONE: 1.0) — LSQ step / BatchNorm fold
  uint16_t n;      // output features (padded to 16)
  uint16_t k;      // input features (padded to 32)
};

struct LNDesc {
  uint32_t g, b;   // float offsets of gamma / beta
};

struct EncLayerDesc {
  GemmDesc qkv, o, f1, f2;
  LNDesc ln1, ln2;
  GemmDesc conv;         // distil ConvLayer following this layer (n == 0: none)
  int L_in, L_out;       // rows entering the layer / leaving its ConvLayer
  int call;              // index into calls[] (ProbSparse) or -1
  uint32_t attn_off;     // float offset of this layer's attns map in the attns buffer (per batch 0)
  int attn_stride;       // floats per batch element of that map (H·L·L)
  int dbg_layer, dbg_conv;  // debug-dump float offsets (per sequence), -1: none
};

struct DecLayerDesc {
  GemmDesc qkv, o, cq, ckv, co, f1, f2;
  LNDesc ln1, ln2, ln3;
  int call;
  int dbg;
};

struct AttnCall {
  int LQ, LK, U, u;
  uint32_t cnt_off;      // byte offset into the per-forward multiplicity blob
  int cnt_stride;        // bytes per query row
  int m_dbg;             // debug float offset of M [H][LQ], -1: none
};

struct InformerPlan {
  int C, c_out, seq_len, dec_len, pred_len;
  int C_shift;              // log2(C)
  int n_enc;
  int enc_layers[MAX_ENC];
  int enc_first[MAX_ENC];   // index of the encoder's first layer in enc[]
  int enc_rows[MAX_ENC];    // output rows of each encoder
  int enc_row_off[MAX_ENC]; // row offset of each encoder's output in the concatenated stack output
  int enc_dbg[MAX_ENC];
  int d_layers, dff, prob, act_relu, mix, lsq;
  int S;                    // total encoder output rows (cross-attention keys)
  GemmDesc emb_enc, emb_dec, proj;
  uint32_t pe_enc, pe_dec;  // float offsets of the positional tables [LMAX][128]
  EncLayerDesc enc[MAX_ENC_LAYERS];
  LNDesc enc_norm[MAX_ENC];
  DecLayerDesc dec[MAX_DEC_LAYERS];
  LNDesc dec_norm;
  AttnCall calls[MAX_CALLS];
  int n_calls;
  uint32_t cnt_bytes;
  // v4 layout (cet_plan.hpp v4_*): the fixed regions, the encoder-stack output (planes × S_pad rows),
  // the staged x_dec and, for the in-kernel sampler replay, its state
  int lds4_enc, lds4_enc_lo, lds4_cnt, lds4_mt, lds4_zero, lds4_bytes, lds4_bytes_replay;
  int lds4_xdec;            // x_dec staged at kernel entry (byte offset), or -1: staged before the decoder
  int lds4_lab;             // labels of the fused NMSE (pred_len × c_out fp32), staged at kernel entry
  int lds4_lncnt;           // LayerNorm arrival counter (-DCET_LN_LAST: the last wave to publish combines the rows)
  int prec;                 // v4 operand precision of the dense layers (v4::P_BF16 / P_X3 / P_FP8)
  int stack;
  int in_stride;            // floats per staged input row
  int dbg_stride, dbg_emb, dbg_dec_emb, dbg_dec_out;
  int draws;                // mt19937 words one forward consumes (Σ LQ·U over every call)
  uint32_t dec_par;         // decoder weight feed: 16-byte-unit offset of the (layer, wave) parameter tiles, or NONE
};

// v4 LDS layout (precision P: 0 bf16, 1 split-bf16 hi/lo planes, 2 fp8); every offset the kernel
// uses in its phases is a compile-time constant (folded into ds_* immediates):
//   image XB | context / FFN hidden / staged input / projection input (CTX) | per-wave attention
//   scratch aliased by the LayerNorm partials | multiplicity table | stack output (plan-sized) |
//   [x_dec staged at entry] | [sampler state, in-kernel replay only]
// Image rows: bf16 272 B ( 288 B — conflict-free ds_read_b128 — measured no faster), fp8
// 144 B (conflict-free ds_read_b64).
#ifdef CET_IMG_SWZ
#define V4_RS16 288   // swizzled rows (cet_v4.hpp Img::off)
#endif
#ifndef V4_RS16
#define V4_RS16 272   // A/B knob: bf16 image row stride (bytes); 288 (conflict-free ds_read_b128) measured equal
#endif
constexpr int v4_rs(int P) { return P == 2 ? 144 : V4_RS16; }
constexpr int v4_planes(int P) { return P == 1 ? 2 : 1; }
constexpr int v4_img(int P) { return LMAX * v4_rs(P); }
constexpr int v4_max3(int a, int b, int c) { return a > b ? (a > c ? a : c) : (b > c ? b : c); }
constexpr int V4L_XB = 0;
constexpr int V4_LDS_2PERCU = 80 * 1024;   // two workgroups per CU
constexpr int v4_ctx(int P) { return v4_planes(P) * v4_img(P); }
constexpr int v4_ctx_bytes(int P) {
  // context image | staged fp32 input rows (LMAX × 20 floats) | the bf16 projection input (48 rows)
  return v4_max3(v4_planes(P) * v4_img(P), LMAX * 20 * 4, 48 * v4_rs(0) * v4_planes(P == 2 ? 0 : P));
}
constexpr int v4_scr(int P) { return v4_ctx(P) + v4_ctx_bytes(P); }
constexpr int v4_cnt(int P) { return v4_scr(P) + 8 * V2_SCR_FLOATS * 4; }   // multiplicity table, LMAX rows
// ProbSparse multiplicity-table rows: 96 count bytes (six key tiles) + 8 pad.  26 dwords ≡ 2 (mod 4): the
// 16 query rows one lane group reads (attention phase A, 8-byte reads) fall on 16 distinct bank pairs; at
// 96 bytes they fell on 4 (4-way, 24 extra LDS cycles per read; tools/probe/lds_probe.hip)
constexpr int CNT_STRIDE = 104;
constexpr int v4_enc(int P) { return v4_cnt(P) + LMAX * CNT_STRIDE; }       // stack output (plan-sized)
static_assert(LMAX * LN3_STRIDE * 4 + LMAX * 8 <= 8 * V2_SCR_FLOATS * 4,
              "LN partials and row statistics fit the scratch they alias");
static_assert(v4_ctx(0) % 16 == 0 && v4_scr(0) % 16 == 0 && v4_enc(1) % 16 == 0 && v4_enc(2) % 16 == 0, "16-B");

// LDS bytes of the three-pass sampler replay (cet_sampler.hpp replay_all_fast): the padded
// mt19937 state | the forward's tempered words | every call's multiplicity table.
constexpr int REPLAY_STATE_WORDS = 640;
__host__ __device__ inline int replay_fast_lds(const InformerPlan& pl) {
  return REPLAY_STATE_WORDS * 4 + ((pl.draws * 4 + 15) & ~15) + (int)pl.cnt_bytes;
}

struct TransformerPlan {
  int C, c_out, src_len, tgt_len, pred_len, N, dff;
  GemmDesc emb_src, emb_tgt, proj;
  uint32_t pe_src, pe_tgt;
  struct Enc { GemmDesc qkv, o, f1, f2; LNDesc ln0, ln1; int dbg; } enc[MAX_DEC_LAYERS];
  struct Dec { GemmDesc qkv, o, cq, ckv, co, f1, f2; LNDesc ln0, ln1, ln2; int dbg; } dec[MAX_DEC_LAYERS];
  LNDesc enc_norm, dec_norm;
  int lds_X, lds_XN, lds_Q, lds_K, lds_VT, lds_ENC, lds_bytes;
  int vts;
  int in_stride;
  int dbg_stride, dbg_emb, dbg_enc_out, dbg_dec_emb, dbg_dec_out;
  int lds4_bytes;           // v4 structure (cet_transformer4.hip): the fixed v4 regions + staged x_dec
};

}  // namespace cet
