// Layer-wise engine (cet_lw.hip, cet_lw_host.cpp): operator argument blocks and launchers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace cet {
namespace lw {

constexpr int LW_DMAX = 1024;   // widest LayerNorm row (d_model)
constexpr int LW_LMAX = 128;    // longest sequence an attention workgroup holds (S in LDS)

// Y[m][n] = epi(Σ_k A(m, k) · W[n][k]),  epi(y) = act(y·scale[n] + bias[n] + pe[t][n]) + R[m][n].
// Rows are sequence-major: m = b·L + t.  amode 0: A(m, k) = A[m·lda + k]; amode 1: circular k=3
// conv, A(m, tap·Cin + c) = A[(b·Ls + off + (t − 1 + tap) mod L)·lda + c].  row_t0 > 0 keeps only
// rows t ≥ row_t0, written densely as Y[b][t − row_t0].  act: 0 none, 1 GELU (erf), 2 ReLU, 3 ELU.
struct GemmOp {
  int M, N, K;
  const float* A;
  int lda, amode, L, Ls, off, Cin;
  const float* W;      // [N][K]
  const float* bias;   // [N] or null
  const float* scale;  // [N] or null
  const float* pe;     // [L][N] or null
  int act;
  const float* R;      // residual [M][ldr] or null (may alias Y)
  int ldr;
  float* Y;
  int ldy;
  int row_t0;
  // fused LayerNorm of the finished rows (eps 1e-5, biased variance; encoder.py:49-56) when the tile holds
  // whole rows (N ≤ 64): gamma / beta, or null
  const float* ln_g;
  const float* ln_b;
};

// LayerNorm of M rows of width D (eps 1e-5, biased variance); input row m = b·L + t goes to output
// row b·Lo + off + t (Lo = L, off = 0: in place or a plain copy).
struct LnOp {
  int M, D, L, Lo, off;
  const float* X;
  float* Y;
  const float* g;
  const float* b;
};

// Attention of every (sequence, head): Q rows b·LQ + i at column h·E (row stride ldq), K/V rows
// b·LK + j.  prob: ProbSparse with the call's draws idx[LQ][U] and u; causal: keys j > i masked
// (and cumsum(V) as the initial context); mix: the (L, H, E) → (H, L, E) re-view of the output
// (requires ldo = H·E).  attns: [B][H][LQ][LK] maps or null.
struct AttnOp {
  int H, E, LQ, LK;
  const float* Q;
  int ldq;
  const float* K;
  int ldk;
  const float* V;
  int ldv;
  float* O;
  int ldo;
  int prob, causal, mix, U, u;
  const int32_t* idx;
  float* attns;            // map of (b, h, i, j) at attns + b·attn_bstride + (h·LQ + i)·LK + j
  int64_t attn_bstride;
};

int launch_gemm(const GemmOp& op, hipStream_t st);
// the FFN pair in one launch (d_model, d_ff ≤ 64): g1 = conv1 + activation, g2 = conv2 + residual (+ LayerNorm)
int launch_ffn(const GemmOp& g1, const GemmOp& g2, hipStream_t st);
int launch_layernorm(const LnOp& op, hipStream_t st);
int launch_maxpool(const float* X, float* Y, int B, int L, int Lo, int D, hipStream_t st);
int launch_window(const float* X, float* Y, int B, int L0, int L, int D, hipStream_t st);
int launch_attention(const AttnOp& op, int B, hipStream_t st);
size_t attn_lds_bytes(int LQ, int LK);
int prepare_attention();   // dynamic-LDS attribute of lw_attention (before any capture)

// ------------------------------------------------------------- fused form (cet_lwf.hip)
// The whole forward of one sequence in one 256-thread workgroup with every activation in LDS, for
// models whose per-sequence working set fits (the d_model-64 MimoSimulation checkpoint: 77 KB, two
// workgroups per CU).  Same operators and arithmetic class as the layer-wise launches (fp32 operands on
// v_mfma_f32_16x16x4_f32); weights pre-packed in MFMA fragment order so every weight load of a wave is
// one coalesced 1 KB read: Wp[nt][kq][lane][j] = W[16nt + (lane & 15)][16kq + 4j + (lane >> 4)].
constexpr uint32_t FNONE = 0xffffffffu;
constexpr int F_MAX_ENC = 4, F_MAX_EL = 8, F_MAX_DEC = 4, F_MAX_CALLS = F_MAX_ENC * F_MAX_EL + F_MAX_DEC;
constexpr int F_LMAX = 128;   // rows per sequence (8 m-tiles)
struct FG {
  uint32_t w;      // packed weight (float offset into the packed blob)
  uint32_t wb;     // the same weight as bf16 fragments (16-byte offset into the bf16 blob; the bf16 instance)
  uint32_t b, s;   // bias / scale (float offsets into the model blob) or FNONE
  int N, K;
};
struct FEnc {
  FG qkv, o, f1, f2, cv;
  uint32_t g1, b1, g2, b2;
  int conv, Lo, call;
};
struct FDec {
  FG qkv, o, cq, ckv, co, f1, f2;
  uint32_t g1, b1, g2, b2, g3, b3;
  int call;
};
struct FPlan {
  int C, Cd, c_out, L0, Ld, pred, D, H, E, HE, dff, S, prob, mix, act, stack, nenc, ndec;
  int nl[F_MAX_ENC], eL0[F_MAX_ENC], eoff[F_MAX_ENC];
  uint32_t ng[F_MAX_ENC], nb[F_MAX_ENC];
  FG emb_e, emb_d, proj;
  uint32_t pe_e, pe_d, dng, dnb;
  int call_U[F_MAX_CALLS], call_u[F_MAX_CALLS];
  uint32_t call_off[F_MAX_CALLS];
  // LDS layout (float offsets) and row strides
  int oE1, e1_rows, oX, oT, oCTX, oENC, oXD, oSCR, scr_floats, lds_floats;   // E1: later stack windows' rows
  int attn_waves;   // 8, or 4 when eight attention scratches would not fit (cet_lw_host.cpp build_fused)
  int ldD, ldT, ldH, ldF, ldKV, ldIN, ldINd;
  FEnc enc[F_MAX_ENC][F_MAX_EL];
  FDec dec[F_MAX_DEC];
};
bool plan_is_d64(const FPlan& p);   // the plan equals the compile-time d_model-64 layout (cet_lwf.hip D64Plan)
// bf: GEMM operands in bf16 (v_mfma_f32_16x16x32_bf16, weights from pwb) instead of fp32
int launch_fused(const FPlan* d_plan, int D, bool fix, bool bf, size_t lds_bytes, const float* blob, const float* pw,
                 const void* pwb, const float* x_enc, const float* x_dec, float* out, const int32_t* idx, int B,
                 hipStream_t st);
int prepare_fused(int D, bool fix, bool bf);

// ------------------------------------------------------------------ host model (cet_lw_host.cpp)
// Weights as fp32 [N][K] matrices in one device blob (float offsets below); ProbSparse draws of a
// forward concatenated in call order (call c's [LQ][U] table at idx_off[c]).
struct EncLayer {
  size_t wqkv, bqkv, wo, bo, w1, b1, w2, b2, g1, be1, g2, be2;
  int conv;
  size_t wc, sc, sh;   // distil conv [D][3D] with BatchNorm(eval) folded into scale / shift
  int L_in, L_out, call;
  int64_t attn_off;
};
struct DecLayer {
  size_t wqkv, bqkv, wo, bo, wcq, bcq, wckv, bckv, wco, bco, w1, b1, w2, b2, g1, be1, g2, be2, g3, be3;
  int call;
};
struct Model {
  int C = 0, Cd = 0, c_out = 0, L0 = 0, Ld = 0, pred = 0, D = 0, H = 0, E = 0, HE = 0, dff = 0, S = 0;
  int prob = 0, mix = 0, act = 1, stack = 1, out_attn = 0;
  size_t emb_enc_w = 0, emb_enc_b = 0, pe_enc = 0, emb_dec_w = 0, emb_dec_b = 0, pe_dec = 0;
  std::vector<std::vector<EncLayer>> enc;
  std::vector<size_t> norm_g, norm_b;
  std::vector<int> enc_L0, enc_rows, enc_off;
  std::vector<DecLayer> dec;
  size_t dnorm_g = 0, dnorm_b = 0, proj_w = 0, proj_b = 0;
  std::vector<float> blob;             // host copy
  std::vector<int> call_LQ, call_LK, call_U, call_u;
  std::vector<size_t> idx_off;
  size_t idx_total = 0;
  int64_t attn_floats = 0;             // per sequence
  // device state
  float* d_blob = nullptr;
  size_t d_blob_n = 0;
  float* ws = nullptr;
  size_t ws_n = 0;
  int32_t* d_idx = nullptr;
  hipGraphExec_t gexec = nullptr;   // the operator sequence captured for batch gB
  int gB = 0;
  // the same sequence captured over the caller's own buffers (no staging copies), once the caller has
  // repeated a (x_enc, x_dec, out, draws, B) tuple: a serving loop over fixed buffers
  struct Key {
    const float* xe;
    const float* xd;
    float* out;
    const int32_t* idx;
    int B;
    bool operator==(const Key& o) const { return xe == o.xe && xd == o.xd && out == o.out && idx == o.idx && B == o.B; }
  };
  hipGraphExec_t dexec = nullptr;
  Key dkey{}, last{};
  hipStream_t cap = nullptr;        // capture stream
  // fused form (cet_lwf.hip): the plan, the packed weights; chosen for every forward without attention
  // maps when the per-sequence working set fits one workgroup's LDS (CET_LW_FUSED=0 turns it off)
  FPlan fplan{};
  bool fused_ok = false, use_fused = true, last_fused = false;
  size_t fused_lds = 0;
  bool fused_fix = false;   // the plan is the compile-time d_model-64 layout (launch_fused's FIX instance)
  // bf16 GEMM operands (cet_set_precision "bf16" on a layer-wise engine): the fused form only, for feature
  // counts that are multiples of 8 (a lane's 8 consecutive k never straddle a conv tap)
  bool bf16 = false, fused_bf_ok = false;
  // whether a forward with (or without) attention maps runs the fused form, and whether bf16 can run it
  bool will_fuse(const float* attns) const { return fused_ok && use_fused && !(attns && out_attn); }
  bool bf16_refused(const float* attns) const { return bf16 && !(will_fuse(attns) && fused_bf_ok); }
  std::vector<float> pblob;
  std::vector<uint16_t> pbblob;   // Wb[nt][ks][lane][j] = bf16(W[16nt + (lane & 15)][32ks + 8(lane >> 4) + j])
  FPlan* d_fplan = nullptr;
  float* d_pblob = nullptr;
  uint16_t* d_pbblob = nullptr;
  int build_fused();
  ~Model();
  size_t ws_floats(int B) const;
  int ensure_ws(int B);
  int enqueue(const float* x_enc, const float* x_dec, int B, float* out, float* attns, const int32_t* idx_dev,
              hipStream_t st);
  int upload();
  // x_enc [B][L0][C], x_dec [B][Ld][C] → out [B][pred][c_out]; idx_dev: this forward's draws (device)
  int forward(const float* x_enc, const float* x_dec, int B, float* out, float* attns, const int32_t* idx_dev,
              hipStream_t st);
  size_t push(const std::vector<float>& v);
};

}  // namespace lw
}  // namespace cet
