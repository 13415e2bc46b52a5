// Layer-wise engine, host side: the forward of InformerStack / Informer (FullPrecision/InformerModel/
// model.py:11-271) as a sequence of operator launches on the caller's stream (cet_lw.hip), for the
// shapes the fused kernels do not carry.  The model (weights as fp32 [N][K] matrices, the plan of
// layers) is built by cet_api.cpp (build_lw); this file owns the device side.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>

#include "cet_lw.h"

namespace cet {
namespace lw {

static uint16_t bf16_rne(float f) {   // fp32 → bf16, round to nearest even (finite weights)
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

Model::~Model() {
  if (gexec) (void)hipGraphExecDestroy(gexec);
  if (dexec) (void)hipGraphExecDestroy(dexec);
  if (cap) (void)hipStreamDestroy(cap);
  if (d_blob) (void)hipFree(d_blob);
  if (ws) (void)hipFree(ws);
  if (d_idx) (void)hipFree(d_idx);
  if (d_fplan) (void)hipFree(d_fplan);
  if (d_pblob) (void)hipFree(d_pblob);
  if (d_pbblob) (void)hipFree(d_pbblob);
}

size_t Model::push(const std::vector<float>& v) {
  while (blob.size() % 4) blob.push_back(0.f);
  const size_t off = blob.size();
  blob.insert(blob.end(), v.begin(), v.end());
  return off;
}

int Model::upload() {
  if (blob.size() > d_blob_n) {
    // the captured graphs hold the old blob's address: drop them with it
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (dexec) (void)hipGraphExecDestroy(dexec);
    gexec = dexec = nullptr;
    if (d_blob && hipFree(d_blob) != hipSuccess) return -1;
    d_blob = nullptr;
    if (hipMalloc((void**)&d_blob, blob.size() * sizeof(float)) != hipSuccess) return -1;
    d_blob_n = blob.size();
  }
  if (hipMemcpy(d_blob, blob.data(), blob.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return -1;
  if (!d_idx && idx_total && hipMalloc((void**)&d_idx, idx_total * sizeof(int32_t)) != hipSuccess) return -1;
  if (!cap && hipStreamCreateWithFlags(&cap, hipStreamNonBlocking) != hipSuccess) return -1;
  if (build_fused()) return -1;
  return prepare_attention() ? -1 : 0;
}

// The fused form's plan (cet_lw.h FPlan) and packed weights, rebuilt with every upload.  fused_ok stays
// false when the sequence's working set does not fit one workgroup's LDS (or a count exceeds the plan).
int Model::build_fused() {
  fused_ok = false;
  const char* env = std::getenv("CET_LW_FUSED");
  use_fused = !(env && std::strcmp(env, "0") == 0);
  const int nenc = (int)enc.size(), ndec = (int)dec.size();
  const int Lm = std::max(L0, Ld);
  const bool why = std::getenv("CET_LW_FUSED_WHY") != nullptr;
  if (why) fprintf(stderr, "lw fused: nenc %d ndec %d calls %zu Lm %d S %d\n", nenc, ndec, call_u.size(), Lm, S);
  if (nenc < 1 || nenc > F_MAX_ENC || ndec > F_MAX_DEC || (int)call_u.size() > F_MAX_CALLS) return 0;
  if (Lm > F_LMAX || S > F_LMAX || S < 1) return 0;
  // the validated range (tests/test_gpu_layerwise.py: up to 48 rows = 3 m-tiles, d_model ≤ 256 for the
  // 16-lane LayerNorm rows); wider shapes keep the operator launches
  if (Lm > 48 || S > 48 || D > 256) return 0;   // S: the cross-attention K/V GEMM runs over S rows
  for (const auto& e : enc)
    if ((int)e.size() > F_MAX_EL) return 0;
  auto r16 = [](int x) { return (x + 15) & ~15; };
  auto pad = [](int w) { return ((w + 31) & ~31) + 2; };   // ≡ 2 mod 32 floats
  FPlan& p = fplan;
  std::memset(&p, 0, sizeof(p));
  p.C = C; p.Cd = Cd; p.c_out = c_out; p.L0 = L0; p.Ld = Ld; p.pred = pred; p.D = D; p.H = H; p.E = E; p.HE = HE;
  p.dff = dff; p.S = S; p.prob = prob; p.mix = mix; p.act = act; p.stack = stack; p.nenc = nenc; p.ndec = ndec;
  p.ldD = pad(D); p.ldT = pad(3 * HE); p.ldH = pad(HE); p.ldF = pad(std::max(dff, D)); p.ldKV = pad(2 * HE);
  p.ldIN = C | 1; p.ldINd = Cd | 1;
  // E1: the rows of the later encoders' windows x[:, -L0/2:] (each later window is a suffix of it)
  p.e1_rows = stack && nenc >= 2 ? enc_L0[1] : 0;
  const size_t nE1 = (size_t)p.e1_rows * p.ldD, nX = (size_t)r16(L0) * p.ldD;
  const size_t nT = std::max({(size_t)r16(Lm) * p.ldT, (size_t)r16(Ld) * p.ldH + (size_t)r16(S) * p.ldKV,
                              (size_t)r16(Lm) * p.ldF, (size_t)r16(L0) * p.ldIN, (size_t)r16(Ld) * p.ldINd});
  const size_t nCTX = (size_t)r16(Lm) * p.ldH, nENC = (size_t)r16(S) * p.ldD, nXD = (size_t)r16(Ld) * p.ldD;
  // one head's scores (LQ rows of LK + 1 floats), M, sel and flag (cet_lwf.hip fattn)
  auto scr_of = [&](int LQ, int LK) { return (size_t)LQ * (LK + 1) + 3 * (size_t)r16(LQ); };
  size_t scr = std::max({scr_of(L0, L0), scr_of(Ld, Ld), scr_of(Ld, S)});
  scr = (scr + 3) & ~(size_t)3;
  size_t o = 0;
  auto place = [&](size_t n) {
    const size_t at = o;
    o += (n + 3) & ~(size_t)3;
    return (int)at;
  };
  p.oE1 = place(nE1); p.oX = place(nX); p.oT = place(nT); p.oCTX = place(nCTX); p.oENC = place(nENC);
  p.oXD = place(nXD);
  // attention on all 8 waves (one scratch each) unless only 4 scratches keep two workgroups per CU (80 KB)
  // or keep the workgroup within the CU's 160 KB at all
  const size_t base = o;
  auto fits = [&](int aw, size_t kb) { return (base + aw * scr) * sizeof(float) <= kb * 1024; };
  p.attn_waves = fits(8, 80) || (!fits(4, 80) && fits(8, 160)) ? 8 : 4;
  p.oSCR = place(p.attn_waves * scr);
  p.scr_floats = (int)scr;
  p.lds_floats = (int)o;
  fused_lds = o * sizeof(float);
  if (why) fprintf(stderr, "lw fused: lds %zu bytes, attention on %d waves\n", fused_lds, p.attn_waves);
  if (fused_lds > 160 * 1024) return 0;
  // packed weights: Wp[nt][kq][lane][j] = W[16nt + (lane & 15)][16kq + 4j + (lane >> 4)], and for the bf16
  // instance Wb[nt][ks][lane][j] = bf16(W[16nt + (lane & 15)][32ks + 8(lane >> 4) + j]) (round to nearest even)
  pblob.clear();
  pbblob.clear();
  auto pack = [&](size_t w, int N, int K, size_t bias, size_t scale) {
    const int NT = (N + 15) / 16, KQ = (K + 15) / 16;
    const size_t at = pblob.size();
    pblob.resize(at + (size_t)NT * KQ * 256, 0.f);
    for (int nt = 0; nt < NT; ++nt)
      for (int kq = 0; kq < KQ; ++kq)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 4; ++j) {
            const int n = 16 * nt + (lane & 15), k = 16 * kq + 4 * j + (lane >> 4);
            if (n < N && k < K) pblob[at + (((size_t)nt * KQ + kq) * 64 + lane) * 4 + j] = blob[w + (size_t)n * K + k];
          }
    const int KS = (K + 31) / 32;
    const size_t atb = pbblob.size();
    // the bf16 fragments only for a bf16 engine (the precision is fixed when the model is planned)
    if (bf16) pbblob.resize(atb + (size_t)NT * KS * 512, 0);
    for (int nt = 0; bf16 && nt < NT; ++nt)
      for (int ks = 0; ks < KS; ++ks)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int n = 16 * nt + (lane & 15), k = 32 * ks + 8 * (lane >> 4) + j;
            if (n < N && k < K) pbblob[atb + (((size_t)nt * KS + ks) * 64 + lane) * 8 + j] = bf16_rne(blob[w + (size_t)n * K + k]);
          }
    FG g;
    g.w = (uint32_t)at; g.wb = (uint32_t)(atb / 8); g.b = (uint32_t)bias; g.s = scale == (size_t)-1 ? FNONE : (uint32_t)scale; g.N = N; g.K = K;
    return g;
  };
  const size_t none = (size_t)-1;
  p.emb_e = pack(emb_enc_w, D, 3 * C, emb_enc_b, none);
  p.emb_d = pack(emb_dec_w, D, 3 * Cd, emb_dec_b, none);
  p.proj = pack(proj_w, c_out, D, proj_b, none);
  p.pe_e = (uint32_t)pe_enc; p.pe_d = (uint32_t)pe_dec; p.dng = (uint32_t)dnorm_g; p.dnb = (uint32_t)dnorm_b;
  for (int i = 0; i < nenc; ++i) {
    p.nl[i] = (int)enc[i].size(); p.eL0[i] = enc_L0[i]; p.eoff[i] = enc_off[i];
    p.ng[i] = (uint32_t)norm_g[i]; p.nb[i] = (uint32_t)norm_b[i];
    for (int l = 0; l < p.nl[i]; ++l) {
      const EncLayer& s = enc[i][l];
      FEnc& f = p.enc[i][l];
      f.qkv = pack(s.wqkv, 3 * HE, D, s.bqkv, none);
      f.o = pack(s.wo, D, HE, s.bo, none);
      f.f1 = pack(s.w1, dff, D, s.b1, none);
      f.f2 = pack(s.w2, D, dff, s.b2, none);
      if (s.conv) f.cv = pack(s.wc, D, 3 * D, s.sh, s.sc);
      f.g1 = (uint32_t)s.g1; f.b1 = (uint32_t)s.be1; f.g2 = (uint32_t)s.g2; f.b2 = (uint32_t)s.be2;
      f.conv = s.conv; f.Lo = s.L_out; f.call = s.call;
    }
  }
  for (int l = 0; l < ndec; ++l) {
    const DecLayer& s = dec[l];
    FDec& f = p.dec[l];
    f.qkv = pack(s.wqkv, 3 * HE, D, s.bqkv, none);
    f.o = pack(s.wo, D, HE, s.bo, none);
    f.cq = pack(s.wcq, HE, D, s.bcq, none);
    f.ckv = pack(s.wckv, 2 * HE, D, s.bckv, none);
    f.co = pack(s.wco, D, HE, s.bco, none);
    f.f1 = pack(s.w1, dff, D, s.b1, none);
    f.f2 = pack(s.w2, D, dff, s.b2, none);
    f.g1 = (uint32_t)s.g1; f.b1 = (uint32_t)s.be1; f.g2 = (uint32_t)s.g2; f.b2 = (uint32_t)s.be2;
    f.g3 = (uint32_t)s.g3; f.b3 = (uint32_t)s.be3; f.call = s.call;
  }
  for (size_t c = 0; c < call_u.size(); ++c) {
    p.call_U[c] = call_U[c]; p.call_u[c] = call_u[c]; p.call_off[c] = (uint32_t)idx_off[c];
  }
  if (blob.size() >= FNONE || pblob.size() >= FNONE || pbblob.size() / 8 >= FNONE) return 0;
  if (!d_fplan && hipMalloc((void**)&d_fplan, sizeof(FPlan)) != hipSuccess) return -1;
  if (d_pblob) (void)hipFree(d_pblob);
  d_pblob = nullptr;
  if (hipMalloc((void**)&d_pblob, pblob.size() * sizeof(float)) != hipSuccess) return -1;
  if (hipMemcpy(d_pblob, pblob.data(), pblob.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return -1;
  if (d_pbblob) (void)hipFree(d_pbblob);
  d_pbblob = nullptr;
  if (!pbblob.empty()) {
    if (hipMalloc((void**)&d_pbblob, pbblob.size() * sizeof(uint16_t)) != hipSuccess) return -1;
    if (hipMemcpy(d_pbblob, pbblob.data(), pbblob.size() * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess)
      return -1;
  }
  fused_bf_ok = C % 8 == 0 && Cd % 8 == 0 && D % 8 == 0 && HE % 8 == 0 && dff % 8 == 0;
  if (hipMemcpy(d_fplan, &p, sizeof(FPlan), hipMemcpyHostToDevice) != hipSuccess) return -1;
  const char* fenv = std::getenv("CET_LW_FUSED_FIX");
  fused_fix = plan_is_d64(p) && !(fenv && std::strcmp(fenv, "0") == 0);
  if (why) fprintf(stderr, "lw fused: compile-time d64 layout %s\n", fused_fix ? "yes" : "no");
  if (prepare_fused(D, fused_fix, bf16 && fused_bf_ok)) return -1;
  fused_ok = true;
  return 0;
}

size_t Model::ws_floats(int B) const {
  const int Lm = std::max(L0, Ld);
  const size_t BL0 = (size_t)B * L0, BLm = (size_t)B * std::max(Lm, S);
  return BL0 * D * 2 + BLm * 3 * HE + BLm * HE + BLm * std::max(dff, D) + (size_t)B * S * D + (size_t)B * Ld * D +
         (size_t)B * Ld * HE + BL0 * C + (size_t)B * Ld * Cd + (size_t)B * pred * c_out + 64;
}

int Model::ensure_ws(int B) {
  const size_t need = ws_floats(B);
  if (need <= ws_n) return 0;
  if (gexec) {
    (void)hipGraphExecDestroy(gexec);
    gexec = nullptr;
  }
  if (dexec) {
    (void)hipGraphExecDestroy(dexec);
    dexec = nullptr;
  }
  if (ws && hipFree(ws) != hipSuccess) return -1;
  ws = nullptr;
  if (hipMalloc((void**)&ws, need * sizeof(float)) != hipSuccess) return -1;
  ws_n = need;
  return 0;
}

// The operator sequence is captured once per batch size into a hipGraph over fixed workspace
// buffers; a forward then costs two input copies, one graph launch and one output copy on the
// caller's stream instead of ≈110 kernel launches (batch-1 latency is launch-bound).  A caller that
// repeats its buffers (a serving loop) gets a second graph captured over those buffers and skips the
// copies.  Forwards that materialise attention maps launch the operators directly.
static int capture(hipStream_t cap, hipGraphExec_t* exec, const std::function<int(hipStream_t)>& body) {
  hipGraph_t g = nullptr;
  // captured on a private stream (the caller's may be the null stream, which cannot capture); the
  // instantiated graph is launched on the caller's stream
  if (hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal) != hipSuccess) return -1;
  const int rc = body(cap);
  if (hipStreamEndCapture(cap, &g) != hipSuccess || rc) {
    if (g) (void)hipGraphDestroy(g);
    return -1;
  }
  const hipError_t ie = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  return ie == hipSuccess ? 0 : -1;
}

int Model::forward(const float* x_enc, const float* x_dec, int B, float* out, float* attns, const int32_t* idx_dev,
                   hipStream_t st) {
  // the fused form: one launch, no workspace, no staging copies
  last_fused = will_fuse(attns);
  if (bf16 && !(last_fused && fused_bf_ok)) return -7;   // bf16 operands exist in the fused form only
  if (last_fused)
    return launch_fused(d_fplan, D, fused_fix, bf16, fused_lds, d_blob, d_pblob, d_pbblob, x_enc, x_dec, out, idx_dev,
                        B, st);
  if (ensure_ws(B)) return -1;
  if (attns && out_attn) return enqueue(x_enc, x_dec, B, out, attns, idx_dev, st);
  const Key key{x_enc, x_dec, out, idx_dev, B};
  if (!(dexec && dkey == key) && last == key) {
    if (dexec) (void)hipGraphExecDestroy(dexec);
    dexec = nullptr;
    if (capture(cap, &dexec, [&](hipStream_t s) { return enqueue(x_enc, x_dec, B, out, nullptr, idx_dev, s); }))
      return -1;
    dkey = key;
  }
  last = key;
  if (dexec && dkey == key) return hipGraphLaunch(dexec, st) == hipSuccess ? 0 : -1;
  const size_t nXE = (size_t)B * L0 * C, nXDi = (size_t)B * Ld * Cd, nOUT = (size_t)B * pred * c_out;
  float* XE = ws + ws_floats(B) - 64 - nOUT - nXDi - nXE;
  float* XDi = XE + nXE;
  float* OUTb = XDi + nXDi;
  if (hipMemcpyAsync(XE, x_enc, nXE * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess) return -1;
  if (hipMemcpyAsync(XDi, x_dec, nXDi * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess) return -1;
  if (!gexec || gB != B) {
    if (gexec) (void)hipGraphExecDestroy(gexec);
    gexec = nullptr;
    if (capture(cap, &gexec, [&](hipStream_t s) { return enqueue(XE, XDi, B, OUTb, nullptr, idx_dev, s); }))
      return -1;
    gB = B;
  }
  if (hipGraphLaunch(gexec, st) != hipSuccess) return -1;
  return hipMemcpyAsync(out, OUTb, nOUT * sizeof(float), hipMemcpyDeviceToDevice, st) == hipSuccess ? 0 : -1;
}

int Model::enqueue(const float* x_enc, const float* x_dec, int B, float* out, float* attns, const int32_t* idx_dev,
                   hipStream_t st) {
  const int Lm = std::max(L0, Ld);
  const size_t BL0 = (size_t)B * L0, BLm = (size_t)B * std::max(Lm, S);
  // workspace: E0 | X | QKV | CTX | HID | ENC | XD | QC | (graph inputs / output)
  const size_t nE0 = BL0 * D, nX = BL0 * D, nQKV = BLm * 3 * HE, nCTX = BLm * HE,
               nHID = BLm * std::max(dff, D), nENC = (size_t)B * S * D, nXD = (size_t)B * Ld * D;
  float* E0 = ws;
  float* X = E0 + nE0;
  float* QKV = X + nX;
  float* CTX = QKV + nQKV;
  float* HID = CTX + nCTX;
  float* ENC = HID + nHID;
  float* XD = ENC + nENC;
  float* QC = XD + nXD;
  const float* P = d_blob;
  int rc = 0;
  auto gemm = [&](const float* A, int M, int N, int K, int lda, size_t w, size_t bias, float* Y, int ldy,
                  int Lrow) {
    GemmOp g{};
    g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.amode = 0; g.L = Lrow; g.Ls = Lrow; g.off = 0; g.Cin = 1;
    g.W = P + w; g.bias = P + bias; g.scale = nullptr; g.pe = nullptr; g.act = 0; g.R = nullptr; g.ldr = 0;
    g.Y = Y; g.ldy = ldy; g.row_t0 = 0;
    return g;
  };
  auto run = [&](const GemmOp& g) {
    if (!rc) rc = launch_gemm(g, st);
  };
  auto ln = [&](float* Xi, float* Yo, int M, int L, int Lo, int off, size_t g, size_t b) {
    LnOp o{M, D, L, Lo, off, Xi, Yo, P + g, P + b};
    if (!rc) rc = launch_layernorm(o, st);
  };
  // a residual GEMM whose in-place LayerNorm follows: fused into its epilogue when one 64-wide tile holds
  // whole rows (d_model ≤ 64), else the separate LayerNorm launch
  // the FFN pair (conv1 + activation, conv2 + residual + LayerNorm): one launch with the hidden rows in
  // LDS when d_model and d_ff ≤ 64, else two GEMMs
  auto run_ffn = [&](const GemmOp& g1, GemmOp g2, int L, size_t lg, size_t lb) {
    if (D <= 64 && dff <= 64) {
      g2.ln_g = P + lg;
      g2.ln_b = P + lb;
      if (!rc) rc = launch_ffn(g1, g2, st);
    } else {
      run(g1);
      run(g2);
      ln(g2.Y, g2.Y, g2.M, L, L, 0, lg, lb);
    }
  };
  auto run_ln = [&](GemmOp g, int L, size_t lg, size_t lb) {
    if (D <= 64) {
      g.ln_g = P + lg;
      g.ln_b = P + lb;
      run(g);
    } else {
      run(g);
      ln(g.Y, g.Y, g.M, L, L, 0, lg, lb);
    }
  };
  auto attend = [&](const float* Q, int ldq, const float* K, int ldk, const float* V, int ldv, float* O, int LQ,
                    int LK, int prob_, int causal, int mix_, int call, float* amap) {
    AttnOp a{};
    a.H = H; a.E = E; a.LQ = LQ; a.LK = LK; a.Q = Q; a.ldq = ldq; a.K = K; a.ldk = ldk; a.V = V; a.ldv = ldv;
    a.O = O; a.ldo = HE; a.prob = prob_; a.causal = causal; a.mix = mix_;
    a.U = call >= 0 ? call_U[call] : 0;
    a.u = call >= 0 ? call_u[call] : LQ;
    a.idx = call >= 0 ? idx_dev + idx_off[call] : nullptr;
    a.attns = amap;
    a.attn_bstride = attn_floats;
    if (!rc) rc = launch_attention(a, B, st);
  };

  // ---- DataEmbedding (embed.py:132-135): circular conv k=3 + pe[:L]
  {
    GemmOp g = gemm(x_enc, B * L0, D, 3 * C, C, emb_enc_w, emb_enc_b, stack ? E0 : X, D, L0);
    g.amode = 1; g.Cin = C; g.pe = P + pe_enc;
    run(g);
  }
  // ---- encoders (EncoderStack: encoder i on x[:, -L0/2^i:], encoder.py:95-106)
  for (size_t i = 0; i < enc.size(); ++i) {
    int L = enc_L0[i];
    if (stack && !rc) rc = launch_window(E0, X, B, L0, L, D, st);
    for (const EncLayer& ly : enc[i]) {
      const int M = B * L;
      run(gemm(X, M, 3 * HE, D, D, ly.wqkv, ly.bqkv, QKV, 3 * HE, L));
      attend(QKV, 3 * HE, QKV + HE, 3 * HE, QKV + 2 * HE, 3 * HE, CTX, L, L, prob, 0, 0, ly.call,
             attns && out_attn ? attns + ly.attn_off : nullptr);
      {
        GemmOp g = gemm(CTX, M, D, HE, HE, ly.wo, ly.bo, X, D, L);   // x = norm1(x + new_x) (encoder.py:49)
        g.R = X; g.ldr = D;
        run_ln(g, L, ly.g1, ly.be1);
      }
      {
        GemmOp g = gemm(X, M, dff, D, D, ly.w1, ly.b1, HID, dff, L);
        g.act = act;
        GemmOp g2 = gemm(HID, M, D, dff, dff, ly.w2, ly.b2, X, D, L);   // norm2(x + y)
        g2.R = X; g2.ldr = D;
        run_ffn(g, g2, L, ly.g2, ly.be2);
      }
      if (ly.conv) {   // ConvLayer (encoder.py:22-28)
        GemmOp g = gemm(X, M, D, 3 * D, D, ly.wc, ly.sh, HID, D, L);
        g.amode = 1; g.Cin = D; g.scale = P + ly.sc; g.act = 3;
        run(g);
        if (!rc) rc = launch_maxpool(HID, X, B, L, ly.L_out, D, st);
        L = ly.L_out;
      }
    }
    // Encoder.norm → rows [enc_off, enc_off + L) of the concatenated stack output
    ln(X, ENC, B * L, L, S, enc_off[i], norm_g[i], norm_b[i]);
  }
  // ---- decoder (decoder.py:43-56, model.py:211-225)
  {
    GemmOp g = gemm(x_dec, B * Ld, D, 3 * Cd, Cd, emb_dec_w, emb_dec_b, XD, D, Ld);
    g.amode = 1; g.Cin = Cd; g.pe = P + pe_dec;
    run(g);
  }
  const int Md = B * Ld;
  for (const DecLayer& ly : dec) {
    run(gemm(XD, Md, 3 * HE, D, D, ly.wqkv, ly.bqkv, QKV, 3 * HE, Ld));
    attend(QKV, 3 * HE, QKV + HE, 3 * HE, QKV + 2 * HE, 3 * HE, CTX, Ld, Ld, prob, 1, mix, ly.call, nullptr);
    {
      GemmOp g = gemm(CTX, Md, D, HE, HE, ly.wo, ly.bo, XD, D, Ld);   // norm1(x + self-attention)
      g.R = XD; g.ldr = D;
      run_ln(g, Ld, ly.g1, ly.be1);
    }
    run(gemm(XD, Md, HE, D, D, ly.wcq, ly.bcq, QC, HE, Ld));
    run(gemm(ENC, B * S, 2 * HE, D, D, ly.wckv, ly.bckv, QKV, 2 * HE, S));
    attend(QC, HE, QKV, 2 * HE, QKV + HE, 2 * HE, CTX, Ld, S, 0, 0, 0, -1, nullptr);
    {
      GemmOp g = gemm(CTX, Md, D, HE, HE, ly.wco, ly.bco, XD, D, Ld);   // norm2(x + cross-attention)
      g.R = XD; g.ldr = D;
      run_ln(g, Ld, ly.g2, ly.be2);
    }
    {
      GemmOp g = gemm(XD, Md, dff, D, D, ly.w1, ly.b1, HID, dff, Ld);
      g.act = act;
      GemmOp g2 = gemm(HID, Md, D, dff, dff, ly.w2, ly.b2, XD, D, Ld);   // norm3(x + y)
      g2.R = XD; g2.ldr = D;
      run_ffn(g, g2, Ld, ly.g3, ly.be3);
    }
  }
  ln(XD, XD, Md, Ld, Ld, 0, dnorm_g, dnorm_b);
  {
    // projection (model.py:264), the last pred_len rows of every sequence → out[B][pred][c_out]
    GemmOp g = gemm(XD, Md, c_out, D, D, proj_w, proj_b, out, c_out, Ld);
    g.row_t0 = Ld - pred;   // (0: every row kept, the plain row map)
    run(g);
  }
  return rc;
}

}  // namespace lw
}  // namespace cet
