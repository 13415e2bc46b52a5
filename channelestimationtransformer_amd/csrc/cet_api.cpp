// Host runtime behind include/cet.h: weight intake by reference key name, packing into
// MFMA fragment order, execution plans, the torch-compatible ProbSparse sampler and the
// per-forward key-multiplicity tables.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/cet.h"
#include "cet_kernels.h"
#include "cet_lw.h"
#include "cet_plan.hpp"

using namespace cet;

bool cet::ensure_lds_attr(const void* kern) {
  static std::mutex mu;
  static std::set<std::pair<int, const void*>> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> lk(mu);
  if (done.count({dev, kern})) return true;
  if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) return false;
  done.insert({dev, kern});
  return true;
}

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) return fail(CET_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

// ------------------------------------------------------------------ torch CPU generator
// torch.manual_seed(s) seeds an mt19937 with (uint32)s; CPU randint(L, shape) draws
// mt19937() % L sequentially (verified against torch in tests/test_rng_native.py).
struct MT19937 {
  uint32_t mt[624];
  int idx = 624;
  void seed(uint64_t s) {
    mt[0] = (uint32_t)(s & 0xffffffffu);
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    idx = 624;
  }
  uint32_t next() {
    if (idx >= 624) {
      for (int i = 0; i < 624; ++i) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
        mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      idx = 0;
    }
    uint32_t y = mt[idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
};

uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
float bf2f(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
// OCP e4m3fn (gfx950's fp8), round-half-even, saturating at ±448 (the packer only feeds it values it
// represents exactly: integers of magnitude ≤ 16 and multiples of 16 up to 128)
uint8_t f2e4m3(float f) {
  const uint8_t s = std::signbit(f) ? 0x80 : 0;
  const double a = std::fabs((double)f);
  if (a == 0.0) return s;
  int e2;
  const double m = std::frexp(a, &e2);   // a = m·2^e2, m ∈ [0.5, 1)
  int E = e2 - 1 + 7;                    // a = (2m)·2^(e2-1)
  if (E >= 1) {
    int mant = (int)std::nearbyint((2.0 * m - 1.0) * 8.0);
    if (mant == 8) { mant = 0; ++E; }
    if (E > 15 || (E == 15 && mant > 6)) return (uint8_t)(s | 0x7e);
    return (uint8_t)(s | (E << 3) | mant);
  }
  int mant = (int)std::nearbyint(a * 512.0);   // subnormal: mant·2^-9
  if (mant >= 8) return (uint8_t)(s | (1 << 3));
  return (uint8_t)(s | mant);
}

int r16(int x) { return (x + 15) & ~15; }
constexpr int MT_WORDS_HOST = 640;   // cet_mt.hpp MT_WORDS (state + index, padded)
int r32(int x) { return (x + 31) & ~31; }
int u_part(int factor, int L) {
  const int u = factor * (int)std::ceil(std::log((double)L));
  return u < L ? u : L;
}

struct Weight {
  std::vector<int64_t> shape;
  std::vector<float> data;
  bool loaded = false;
  bool required = true;
};

}  // namespace

struct cet_engine {
  int kind = 0;  // 0 informer, 1 transformer
  cet_informer_config icfg{};
  cet_transformer_config tcfg{};
  std::map<std::string, Weight> weights;
  std::vector<std::string> order;
  bool dirty = true;
  bool uploaded = false;
  int last_path = 0; // the fused kernel the last forward launched (CET_PATH_*), 0: none yet
  std::string last_kernel;   // its instance, as rocprofv3 names it (cet_last_kernel)
  bool enc_split_ok = true;   // v4 encoder split allowed (CET_NO_ENC_SPLIT at creation turns it off)
  bool feed_ok = false;       // the plan's decoder runs on the LDS-DMA weight feed (build_informer, FEED instances)
  int variant = 4;   // fused-kernel generation: 4 (one sequence per workgroup), the only one kept
  // shapes outside the fused kernels (d_model != 128, n_heads != 8, d_ff > 128, ...): the layer-wise
  // engine (cet_lw.hip), fp32 on the f32 MFMA, one launch per operator
  bool generic = false;
  std::unique_ptr<cet::lw::Model> lw;
  int32_t* h_lwidx[4] = {};   // pinned staging of each forward's draws (ring, events ev[])

  // packed blobs
  std::vector<uint16_t> wblob;
  std::vector<uint16_t> wblob_lo;   // v4 split-bf16: lo fragments (uploaded after wblob)
  int prec_req = -1;                // cet_set_precision: -1 auto, else v4::P_BF16 / P_X3 / P_FP8
  int prec = 0;                     // the precision the plan was built for
  std::vector<float> pblob;
  InformerPlan ip{};
  TransformerPlan tp{};
  void* d_plan = nullptr;
  void* d_w = nullptr;
  float* d_p = nullptr;
  size_t d_w_bytes = 0, d_p_bytes = 0;

  // ProbSparse sampling
  struct Call { int LK, LQ, U; };
  std::vector<Call> calls;
  std::vector<std::vector<int32_t>> idx;
  std::vector<bool> idx_set;
  bool native_rng = false;
  bool host_sampler = false;   // cet_set_sampler: native draws on the host, tables staged per forward
  MT19937 rng;
  // device-resident copy of the same stream (v2 kernel, cet_mt.hpp): two HBM slots of
  // 624 words + read index; the kernel reads slot mt_cur and writes the advanced state to the
  // other.  The host mirror lags by host_lag draws and catches up only when it is read.
  uint32_t* d_mt = nullptr;
  uint32_t* h_mt = nullptr;
  hipEvent_t ev_mt = nullptr;
  bool ev_mt_used = false;
  int mt_cur = 0;
  bool dev_mt_valid = false;
  int64_t host_lag = 0;
  int64_t draws_per_forward = 0;
  void sync_host_rng() {
    for (; host_lag > 0; --host_lag) (void)rng.next();
  }
  // v3 prepared tables: the multiplicity tables of the NEXT forward are built by the first
  // workgroup of the current forward to finish (or by cet_launch_sampler_prep after a reseed),
  // so no forward replays the stream on its critical path.  d_tab[tab_cur] holds the tables of
  // the next forward when tab_ready; d_mt[mt_cur] is then the state after their draws.
  uint8_t* d_tab[2] = {};
  int tab_cur = 0;
  bool tab_ready = false;
  unsigned* d_ticket = nullptr;
  // v4 encoder split (launch_fused): exchange image rows [B][S][RS / 8] and per-sequence arrival counts
  uint64_t* d_enc_xchg = nullptr;
  size_t enc_xchg_n = 0;
  unsigned* d_enc_count = nullptr;
  int enc_count_n = 0;
  float2* d_nmse_part = nullptr;   // fused NMSE: per-sequence partials [B][pred_len]
  size_t nmse_part_n = 0;
  static constexpr int PREP_MIN_B = 64;   // below this the first finisher has no slack to hide in

  // per-forward multiplicity tables (ring of pinned staging + device buffers)
  static constexpr int NSLOT = 4;
  uint8_t* h_cnt[NSLOT] = {};
  uint8_t* d_cnt[NSLOT] = {};
  hipEvent_t ev[NSLOT] = {};
  bool ev_used[NSLOT] = {};
  int slot = 0;
  size_t cnt_bytes = 0;

  float* dbg = nullptr;
  unsigned long long* stamps = nullptr;
  std::string dbg_json;

  // kernel timing: hipEvents bracketing one forward kernel launch in every `timing_every` on the
  // caller's stream (a sample keeps the events' own cost out of the launches between them)
  bool timing = false;
  int timing_every = 1;
  int64_t timing_seen = 0;
  std::vector<hipEvent_t> t_ev;
  size_t t_n = 0;
  int64_t attn_floats = 0;
  std::vector<std::pair<int64_t, int>> attn_layout;  // (offset, L) per encoder layer

  ~cet_engine() {
    for (auto ev_ : t_ev) (void)hipEventDestroy(ev_);
    if (d_plan) (void)hipFree(d_plan);
    if (d_w) (void)hipFree(d_w);
    if (d_p) (void)hipFree(d_p);
    for (int i = 0; i < NSLOT; ++i) {
      if (h_cnt[i]) (void)hipHostFree(h_cnt[i]);
      if (d_cnt[i]) (void)hipFree(d_cnt[i]);
      if (ev[i]) (void)hipEventDestroy(ev[i]);
    }
    if (d_mt) (void)hipFree(d_mt);
    for (auto* t : d_tab)
      if (t) (void)hipFree(t);
    if (d_ticket) (void)hipFree(d_ticket);
    if (d_enc_xchg) (void)hipFree(d_enc_xchg);
    if (d_enc_count) (void)hipFree(d_enc_count);
    if (d_nmse_part) (void)hipFree(d_nmse_part);
    if (h_mt) (void)hipHostFree(h_mt);
    for (auto* h : h_lwidx)
      if (h) (void)hipHostFree(h);
    if (ev_mt) (void)hipEventDestroy(ev_mt);
  }

  void add(const std::string& name, std::vector<int64_t> shape, bool required = true) {
    Weight w;
    w.shape = std::move(shape);
    w.required = required;
    weights[name] = std::move(w);
    order.push_back(name);
  }
  const std::vector<float>& W(const std::string& n) const { return weights.at(n).data; }
  float scalar(const std::string& n) const { return weights.at(n).data.at(0); }
  bool has(const std::string& n) const {
    auto it = weights.find(n);
    return it != weights.end() && it->second.loaded;
  }
};

namespace {

// ------------------------------------------------------------------ schema (mirrors spec.py)
void schema_embedding(cet_engine* e, const std::string& p, int c_in, int d) {
  e->add(p + ".value_embedding.tokenConv.weight", {d, c_in, 3});
  e->add(p + ".value_embedding.tokenConv.bias", {d});
  e->add(p + ".position_embedding.pe", {1, 5000, d});
  // temporal tables (embed.py:130-159) exist in checkpoints but are never used (embed.py:132-135)
  const char* names[4] = {"hour_embed", "weekday_embed", "day_embed", "month_embed"};
  const int rows[4] = {24, 7, 32, 13};
  for (int i = 0; i < 4; ++i) e->add(p + ".temporal_embedding." + names[i] + ".emb.weight", {rows[i], d}, false);
}

// AttentionLayer (attn.py:178-193): d_keys = d_values = d_model // n_heads; q/k/v project d_model →
// d_keys·n_heads, out projects d_values·n_heads → d_model
void schema_attn(cet_engine* e, const std::string& p, int d, int heads, bool lsq) {
  const int he = (d / heads) * heads;
  for (const char* n : {"query_projection", "key_projection", "value_projection", "out_projection"}) {
    const bool out = std::strcmp(n, "out_projection") == 0;
    e->add(p + "." + n + ".weight", {out ? d : he, out ? he : d});
    e->add(p + "." + n + ".bias", {out ? d : he});
    if (lsq) e->add(p + "." + n + ".step_size", {});
  }
}

void schema_ffn(cet_engine* e, const std::string& p, int d, int dff, bool lsq) {
  e->add(p + ".conv1.weight", {dff, d, 1});
  e->add(p + ".conv1.bias", {dff});
  if (lsq) e->add(p + ".conv1.step_size", {});
  e->add(p + ".conv2.weight", {d, dff, 1});
  e->add(p + ".conv2.bias", {d});
  if (lsq) e->add(p + ".conv2.step_size", {});
}

void schema_ln(cet_engine* e, const std::string& p, int d) {
  e->add(p + ".weight", {d});
  e->add(p + ".bias", {d});
}

void schema_informer(cet_engine* e) {
  const auto& c = e->icfg;
  const int d = c.d_model;
  const bool lsq = c.lsq_bits > 0;
  schema_embedding(e, "enc_embedding", c.enc_in, d);
  schema_embedding(e, "dec_embedding", c.dec_in, d);
  for (int i = 0; i < c.n_enc; ++i) {
    const std::string pre = c.stack ? "encoder.encoders." + std::to_string(i) : std::string("encoder");
    for (int l = 0; l < c.e_layers[i]; ++l) {
      const std::string p = pre + ".attn_layers." + std::to_string(l);
      schema_attn(e, p + ".attention", d, c.n_heads, lsq);
      schema_ffn(e, p, d, c.d_ff, lsq);
      schema_ln(e, p + ".norm1", d);
      schema_ln(e, p + ".norm2", d);
    }
    if (c.distil)
      for (int l = 0; l < c.e_layers[i] - 1; ++l) {
        const std::string p = pre + ".conv_layers." + std::to_string(l);
        e->add(p + ".downConv.weight", {d, d, 3});
        e->add(p + ".downConv.bias", {d});
        if (lsq) e->add(p + ".downConv.step_size", {});
        e->add(p + ".norm.weight", {d});
        e->add(p + ".norm.bias", {d});
        e->add(p + ".norm.running_mean", {d});
        e->add(p + ".norm.running_var", {d});
        e->add(p + ".norm.num_batches_tracked", {}, false);
      }
    schema_ln(e, pre + ".norm", d);
  }
  for (int l = 0; l < c.d_layers; ++l) {
    const std::string p = "decoder.layers." + std::to_string(l);
    schema_attn(e, p + ".self_attention", d, c.n_heads, lsq);
    schema_attn(e, p + ".cross_attention", d, c.n_heads, lsq);
    schema_ffn(e, p, d, c.d_ff, lsq);
    schema_ln(e, p + ".norm1", d);
    schema_ln(e, p + ".norm2", d);
    schema_ln(e, p + ".norm3", d);
  }
  schema_ln(e, "decoder.norm", d);
  e->add("projection.weight", {c.c_out, d});
  e->add("projection.bias", {c.c_out});
}

void schema_transformer(cet_engine* e) {
  const auto& c = e->tcfg;
  const int d = c.d_model;
  auto mha = [&](const std::string& p) {
    for (const char* n : {"w_q", "w_k", "w_v", "w_o"}) e->add(p + "." + n + ".weight", {d, d});
  };
  auto ff = [&](const std::string& p) {
    e->add(p + ".linear_1.weight", {c.d_ff, d});
    e->add(p + ".linear_1.bias", {c.d_ff});
    e->add(p + ".linear_2.weight", {d, c.d_ff});
    e->add(p + ".linear_2.bias", {d});
  };
  auto ln = [&](const std::string& p) {
    e->add(p + ".alpha", {d});
    e->add(p + ".bias", {d});
  };
  for (int l = 0; l < c.N; ++l) {
    const std::string p = "encoder.layers." + std::to_string(l);
    mha(p + ".self_attention_block");
    ff(p + ".feed_forward_block");
    for (int r = 0; r < 2; ++r) ln(p + ".residual_connections." + std::to_string(r) + ".norm");
  }
  ln("encoder.norm");
  for (int l = 0; l < c.N; ++l) {
    const std::string p = "decoder.layers." + std::to_string(l);
    mha(p + ".self_attention_block");
    mha(p + ".cross_attention_block");
    ff(p + ".feed_forward_block");
    for (int r = 0; r < 3; ++r) ln(p + ".residual_connections." + std::to_string(r) + ".norm");
  }
  ln("decoder.norm");
  e->add("src_embed.tokenEmbedding.weight", {d, c.src_vocab, 3});
  e->add("src_embed.tokenEmbedding.bias", {d});
  e->add("tgt_embed.tokenEmbedding.weight", {d, c.tgt_vocab, 3});
  e->add("tgt_embed.tokenEmbedding.bias", {d});
  e->add("src_pos.pe", {1, c.src_seq_len, d});
  e->add("tgt_pos.pe", {1, c.tgt_seq_len + c.label_len, d});
  e->add("projection_layer.proj.weight", {c.tgt_vocab, d});
  e->add("projection_layer.proj.bias", {c.tgt_vocab});
}

// ------------------------------------------------------------------ packing
struct Packer {
  std::vector<uint16_t>& wb;
  std::vector<float>& pb;
  std::vector<uint16_t>* wlo = nullptr;   // split-bf16 (v4 P_X3): the lo fragments, parallel to wb

  // W given as a row-major [N][K] fp32 matrix → fragment order [N/16][K/32][64][8] bf16 (and, with
  // `wlo`, the residuals bf16(w − hi) in the same order).
  GemmDesc gemm(const std::vector<float>& w, int N, int K, const float* bias, const float* scale) {
    GemmDesc d{};
    const int Np = r16(N), Kp = r32(K);
    d.w = (uint32_t)(wb.size() / 8);
    d.n = (uint16_t)Np;
    d.k = (uint16_t)Kp;
    for (int nt = 0; nt < Np / 16; ++nt)
      for (int ks = 0; ks < Kp / 32; ++ks)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int n = nt * 16 + (lane & 15), k = ks * 32 + 8 * (lane >> 4) + j;
            const float x = n < N && k < K ? w[(size_t)n * K + k] : 0.f;
            const uint16_t h = f2bf(x);
            wb.push_back(h);
            if (wlo) wlo->push_back(f2bf(x - bf2f(h)));
          }
    d.bias = bias ? vec(bias, N, Np) : NONE;
    d.scale = scale ? vec(scale, N, Np) : NONE;
    return d;
  }
  // An LSQ integer grid q ∈ [−128, 127] as e4m3 pairs (v4 P_FP8, default form): lane fragment = 8 bytes
  // of 16·⌊q/16⌋ then 8 bytes of q mod 16, both exact in e4m3; same 16 B per lane per k-step as bf16.
  GemmDesc gemm_fp8(const std::vector<float>& q, int N, int K, const float* bias, const float* scale) {
    GemmDesc d{};
    const int Np = r16(N), Kp = r32(K);
    d.w = (uint32_t)(wb.size() / 8);
    d.n = (uint16_t)Np;
    d.k = (uint16_t)Kp;
    for (int nt = 0; nt < Np / 16; ++nt)
      for (int ks = 0; ks < Kp / 32; ++ks)
        for (int lane = 0; lane < 64; ++lane) {
          uint8_t by[16];
          for (int j = 0; j < 8; ++j) {
            const int n = nt * 16 + (lane & 15), k = ks * 32 + 8 * (lane >> 4) + j;
            const int v = n < N && k < K ? (int)q[(size_t)n * K + k] : 0;
            const int hi = (int)std::floor(v / 16.0);
            by[j] = f2e4m3((float)(16 * hi));
            by[8 + j] = f2e4m3((float)(v - 16 * hi));
          }
          for (int j = 0; j < 8; ++j) wb.push_back((uint16_t)(by[2 * j] | (by[2 * j + 1] << 8)));
        }
    d.bias = bias ? vec(bias, N, Np) : NONE;
    d.scale = scale ? vec(scale, N, Np) : NONE;
    return d;
  }
  uint32_t vec(const float* v, int n, int npad) {
    while (pb.size() % 4) pb.push_back(0.f);
    const uint32_t off = (uint32_t)pb.size();
    for (int i = 0; i < npad; ++i) pb.push_back(i < n ? v[i] : 0.f);
    return off;
  }
  LNDesc ln(const std::vector<float>& g, const std::vector<float>& b) {
    LNDesc d;
    d.g = vec(g.data(), (int)g.size(), (int)g.size());
    d.b = vec(b.data(), (int)b.size(), (int)b.size());
    return d;
  }
};

// LSQ weight grid (LSQ.py:65-74): q = round_half_even(clamp(w/s, Qn, Qp)); w_q = q·s.  The
// integer q is packed and s is applied in the epilogue; q is exact in bf16 while |q| ≤ 256, which
// the LSQ initialisation s = mean|w|/√Qp keeps for every width up to 16 bits (|q| ≲ 2·√Qp).  Returns
// max |q| so the packer can refuse a grid bf16 cannot hold.
float lsq_grid(std::vector<float>& w, float s, int bits) {
  const float qn = -(float)(1 << (bits - 1)), qp = (float)((1 << (bits - 1)) - 1);
  float qmax = 0.f;
  for (auto& x : w) {
    float v = x / s;
    v = v < qn ? qn : (v > qp ? qp : v);
    x = std::nearbyint(v);
    qmax = std::max(qmax, std::fabs(x));
  }
  return qmax;
}

// Largest |q| of every LSQ integer grid the engine would pack (0 without LSQ).
float lsq_qmax(cet_engine* e) {
  float qmax = 0.f;
  if (e->icfg.lsq_bits <= 0) return qmax;
  for (const auto& kv : e->weights) {
    const std::string& n = kv.first;
    const std::string suf = ".step_size";
    if (n.size() <= suf.size() || n.compare(n.size() - suf.size(), suf.size(), suf) != 0 || !kv.second.loaded)
      continue;
    const std::string wn = n.substr(0, n.size() - suf.size()) + ".weight";
    if (!e->has(wn)) continue;
    std::vector<float> w = e->W(wn);
    qmax = std::max(qmax, lsq_grid(w, e->scalar(n), e->icfg.lsq_bits));
  }
  return qmax;
}

// The v4 operand precision (cet_v4.hpp): the requested one, or automatically split bf16 where
// bf16 cannot carry the model — an LSQ grid with |q| > 256, or a genuinely sparse masked decoder
// (u < L_dec), whose unselected rows take cumsum(V) so that a near-tie flip of the top-u selection
// moves the output by O(1): there the sparsity measure must be as exact as the reference's.
int resolve_precision(cet_engine* e, float qmax, int* out) {
  const auto& c = e->icfg;
  const int Ld = c.label_len + c.out_len;
  const bool sparse_dec = c.attn_prob && u_part(c.factor, Ld) < Ld;
  int P = e->prec_req;
  if (P < 0) P = (qmax > 256.f || sparse_dec) ? 1 : 0;
  if (P == 2) {
    if (c.lsq_bits <= 0 || c.lsq_bits > 8)
      return fail(CET_E_INVALID, "fp8 activations need an LSQ engine of at most 8 bits (integer grid in e4m3 pairs)");
    if (qmax > 128.f) return fail(CET_E_INVALID, "fp8 weight pairs hold |q| <= 128");
  }
  if ((P == 0 || P == 4) && qmax > 256.f)
    return fail(CET_E_INVALID, "LSQ grid with |q| = " + std::to_string((int)qmax) +
                                   " > 256 is not exact in bf16; use the split-bf16 precision");
  if (P == 4 && (c.d_ff != 64 || Ld > 48))
    return fail(CET_E_INVALID, "the mixed precision (bf16 encoder, split-bf16 decoder) needs d_ff 64 and <= 48 decoder rows");
  *out = P;
  return CET_OK;
}

int build_lw(cet_engine* e);

int build_informer(cet_engine* e) {
  if (e->generic) return build_lw(e);
  const auto& c = e->icfg;
  const int D = c.d_model;
  auto& wb = e->wblob;
  auto& pb = e->pblob;
  wb.clear();
  pb.clear();
  e->wblob_lo.clear();
  Packer pk{wb, pb};
  InformerPlan& p = e->ip;
  std::memset(&p, 0, sizeof(p));
  const bool lsq = c.lsq_bits > 0;
  const int bits = c.lsq_bits;
  float qmax = 0.f;   // largest |q| of the LSQ integer grids
  int P = 0;
  {
    const int rc = resolve_precision(e, lsq_qmax(e), &P);
    if (rc) return rc;
  }
  e->prec = P;
  p.prec = P;
  if (P == 1 || P == 4) pk.wlo = &e->wblob_lo;   // split bf16 (4: the decoder's layers; the encoder ignores them)

  auto lin = [&](const std::string& n) { return e->W(n + ".weight"); };
  // Linear/conv1x1 (possibly several concatenated along the output axis) → GemmDesc
  auto dense = [&](std::vector<std::string> names, int K, bool conv1x1) -> GemmDesc {
    std::vector<float> w, b, s;
    for (auto& n : names) {
      std::vector<float> wi = lin(n);
      const int Ni = (int)wi.size() / K;
      float step = 1.f;
      if (lsq && e->has(n + ".step_size")) {
        step = e->scalar(n + ".step_size");
        qmax = std::max(qmax, lsq_grid(wi, step, bits));
      }
      w.insert(w.end(), wi.begin(), wi.end());
      const auto& bi = e->W(n + ".bias");
      b.insert(b.end(), bi.begin(), bi.end());
      s.insert(s.end(), Ni, step);
    }
    (void)conv1x1;
    const int N = (int)w.size() / K;
    if (P == 2) return pk.gemm_fp8(w, N, K, b.data(), s.data());
    return pk.gemm(w, N, K, b.data(), lsq ? s.data() : nullptr);
  };

  p.C = c.enc_in;
  p.C_shift = c.enc_in == 8 ? 3 : 4;
  p.c_out = c.c_out;
  p.seq_len = c.seq_len;
  p.dec_len = c.label_len + c.out_len;
  p.pred_len = c.out_len;
  p.n_enc = c.n_enc;
  p.d_layers = c.d_layers;
  p.dff = c.d_ff;
  p.prob = c.attn_prob;
  p.act_relu = c.act_relu;
  p.mix = c.mix;
  p.lsq = lsq;

  // token embeddings: W[n][tap·C + c] = conv.weight[n][c][tap]   (embed.py:30-49)
  auto emb = [&](const std::string& pre, int C) {
    const auto& w = e->W(pre + ".value_embedding.tokenConv.weight");
    std::vector<float> m((size_t)D * 3 * C);
    for (int n = 0; n < D; ++n)
      for (int ch = 0; ch < C; ++ch)
        for (int tap = 0; tap < 3; ++tap) m[(size_t)n * 3 * C + tap * C + ch] = w[((size_t)n * C + ch) * 3 + tap];
    const auto& b = e->W(pre + ".value_embedding.tokenConv.bias");
    return pk.gemm(m, D, 3 * C, b.data(), nullptr);
  };
  p.emb_enc = emb("enc_embedding", c.enc_in);
  p.emb_dec = emb("dec_embedding", c.dec_in);
  {
    const auto& pe = e->W("enc_embedding.position_embedding.pe");
    p.pe_enc = pk.vec(pe.data(), LMAX * D, LMAX * D);
    const auto& pd = e->W("dec_embedding.position_embedding.pe");
    p.pe_dec = pk.vec(pd.data(), LMAX * D, LMAX * D);
  }

  int layer = 0, call = 0;
  int64_t dbg = 0;
  std::ostringstream js;
  js << "{\"stages\": [";
  bool firstj = true;
  auto jstage = [&](const std::string& name, int64_t off, int rows, int cols) {
    js << (firstj ? "" : ", ") << "[\"" << name << "\", " << off << ", " << rows << ", " << cols << "]";
    firstj = false;
  };
  p.dbg_emb = (int)dbg;
  jstage("enc_emb", dbg, c.seq_len, D);
  dbg += (int64_t)c.seq_len * D;
  e->calls.clear();
  e->attn_layout.clear();
  int64_t attn_off = 0;
  int S = 0;
  for (int i = 0; i < c.n_enc; ++i) {
    const std::string pre = c.stack ? "encoder.encoders." + std::to_string(i) : std::string("encoder");
    int L = c.stack ? (c.seq_len >> i) : c.seq_len;
    p.enc_layers[i] = c.e_layers[i];
    p.enc_first[i] = layer;
    for (int l = 0; l < c.e_layers[i]; ++l) {
      if (layer >= MAX_ENC_LAYERS) return fail(CET_E_INVALID, "too many encoder layers");
      EncLayerDesc& d = p.enc[layer];
      const std::string lp = pre + ".attn_layers." + std::to_string(l);
      d.qkv = dense({lp + ".attention.query_projection", lp + ".attention.key_projection",
                     lp + ".attention.value_projection"}, D, false);
      d.o = dense({lp + ".attention.out_projection"}, D, false);
      d.f1 = dense({lp + ".conv1"}, D, true);
      d.f2 = dense({lp + ".conv2"}, c.d_ff, true);
      d.ln1 = pk.ln(e->W(lp + ".norm1.weight"), e->W(lp + ".norm1.bias"));
      d.ln2 = pk.ln(e->W(lp + ".norm2.weight"), e->W(lp + ".norm2.bias"));
      d.L_in = L;
      d.call = -1;
      if (c.attn_prob) {
        if (call >= MAX_CALLS) return fail(CET_E_INVALID, "too many ProbSparse calls");
        d.call = call++;
        e->calls.push_back({L, L, u_part(c.factor, L)});
      }
      d.attn_off = (uint32_t)attn_off;
      if (c.output_attention) {
        e->attn_layout.push_back({attn_off, L});
        attn_off += (int64_t)NHEAD * L * L;
      }
      d.dbg_layer = (int)dbg;
      jstage("enc" + std::to_string(i) + "_layer" + std::to_string(l), dbg, L, D);
      dbg += (int64_t)L * D;
      d.dbg_conv = -1;
      d.conv.n = 0;
      if (c.distil && l < c.e_layers[i] - 1) {
        // ConvLayer: W[n][tap·D + c] = downConv.weight[n][c][tap]; BatchNorm(eval) folded into
        // a per-channel scale/shift applied after the conv (encoder.py:22-28).
        const std::string cp = pre + ".conv_layers." + std::to_string(l);
        std::vector<float> w = e->W(cp + ".downConv.weight");
        float step = 1.f;
        if (lsq && e->has(cp + ".downConv.step_size")) {
          step = e->scalar(cp + ".downConv.step_size");
          qmax = std::max(qmax, lsq_grid(w, step, bits));
        }
        std::vector<float> m((size_t)D * 3 * D);
        for (int n = 0; n < D; ++n)
          for (int ch = 0; ch < D; ++ch)
            for (int tap = 0; tap < 3; ++tap) m[(size_t)n * 3 * D + tap * D + ch] = w[((size_t)n * D + ch) * 3 + tap];
        const auto& cb = e->W(cp + ".downConv.bias");
        const auto& g = e->W(cp + ".norm.weight");
        const auto& bb = e->W(cp + ".norm.bias");
        const auto& rm = e->W(cp + ".norm.running_mean");
        const auto& rv = e->W(cp + ".norm.running_var");
        std::vector<float> sc(D), sh(D);
        for (int n = 0; n < D; ++n) {
          const double inv = (double)g[n] / std::sqrt((double)rv[n] + 1e-5);
          sc[n] = (float)(inv * step);
          sh[n] = (float)(((double)cb[n] - rm[n]) * inv + bb[n]);
        }
        d.conv = P == 2 ? pk.gemm_fp8(m, D, 3 * D, sh.data(), sc.data()) : pk.gemm(m, D, 3 * D, sh.data(), sc.data());
        d.L_out = (L - 1) / 2 + 1;
        d.dbg_conv = (int)dbg;
        jstage("enc" + std::to_string(i) + "_conv" + std::to_string(l), dbg, d.L_out, D);
        dbg += (int64_t)d.L_out * D;
        L = d.L_out;
      } else {
        d.L_out = L;
      }
      ++layer;
    }
    p.enc_norm[i] = pk.ln(e->W(pre + ".norm.weight"), e->W(pre + ".norm.bias"));
    p.enc_rows[i] = L;
    p.enc_row_off[i] = S;
    S += L;
    p.enc_dbg[i] = (int)dbg;
    jstage("enc" + std::to_string(i) + "_out", dbg, L, D);
    dbg += (int64_t)L * D;
  }
  p.S = S;
  (void)qmax;
  const int Ld = c.label_len + c.out_len;
  p.dbg_dec_emb = (int)dbg;
  jstage("dec_emb", dbg, Ld, D);
  dbg += (int64_t)Ld * D;
  for (int l = 0; l < c.d_layers; ++l) {
    DecLayerDesc& d = p.dec[l];
    const std::string lp = "decoder.layers." + std::to_string(l);
    d.qkv = dense({lp + ".self_attention.query_projection", lp + ".self_attention.key_projection",
                   lp + ".self_attention.value_projection"}, D, false);
    d.o = dense({lp + ".self_attention.out_projection"}, D, false);
    d.cq = dense({lp + ".cross_attention.query_projection"}, D, false);
    d.ckv = dense({lp + ".cross_attention.key_projection", lp + ".cross_attention.value_projection"}, D, false);
    d.co = dense({lp + ".cross_attention.out_projection"}, D, false);
    d.f1 = dense({lp + ".conv1"}, D, true);
    d.f2 = dense({lp + ".conv2"}, c.d_ff, true);
    d.ln1 = pk.ln(e->W(lp + ".norm1.weight"), e->W(lp + ".norm1.bias"));
    d.ln2 = pk.ln(e->W(lp + ".norm2.weight"), e->W(lp + ".norm2.bias"));
    d.ln3 = pk.ln(e->W(lp + ".norm3.weight"), e->W(lp + ".norm3.bias"));
    d.call = -1;
    if (c.attn_prob) {
      d.call = call++;
      e->calls.push_back({Ld, Ld, u_part(c.factor, Ld)});
    }
    d.dbg = (int)dbg;
    jstage("dec_layer" + std::to_string(l), dbg, Ld, D);
    dbg += (int64_t)Ld * D;
  }
  p.dec_norm = pk.ln(e->W("decoder.norm.weight"), e->W("decoder.norm.bias"));
  p.dbg_dec_out = (int)dbg;
  jstage("dec_out", dbg, Ld, D);
  dbg += (int64_t)Ld * D;
  {
    const auto& w = e->W("projection.weight");
    const auto& b = e->W("projection.bias");
    p.proj = pk.gemm(w, c.c_out, D, b.data(), nullptr);
  }
  // Decoder weight feed (cet_informer4.hpp FEED): the decoder's weight tiles stream into per-wave LDS slots by
  // LDS-DMA, and its bias and LayerNorm vectors come from one 1 KiB parameter tile per (layer, wave) packed here
  // after the weights, 16 blocks of the wave's 16 features: cross K / V, self K / V / Q, O biases, LN1 γ / β,
  // cross Q, cross O biases, LN2 γ / β, FFN1 (n-tile w mod 4), FFN2 biases, LN3 γ / β.  Plans it fits: bf16
  // operands, d_ff 64, a one-tile decoder (≤ 16 rows) whose ProbSparse calls select every query (u = L, the
  // decoder of every BASELINE Informer config), and no per-output scales (LSQ plans keep the register path).
  {
    p.dec_par = NONE;
    e->feed_ok = false;
    bool scales = false;
    for (int l = 0; l < c.d_layers; ++l) {
      const DecLayerDesc& d = p.dec[l];
      for (const GemmDesc* g : {&d.qkv, &d.o, &d.cq, &d.ckv, &d.co, &d.f1, &d.f2}) scales = scales || g->scale != NONE;
    }
    const bool dense_dec = !(c.attn_prob && u_part(c.factor, Ld) < Ld);
    if (P == 0 && !scales && c.d_ff == 64 && Ld <= 16 && dense_dec && D == 128) {
      while (wb.size() % 512) wb.push_back(0);   // 1 KiB aligned
      p.dec_par = (uint32_t)(wb.size() / 8);
      auto put = [&](float* t, int v, uint32_t off, int at) {
        for (int i = 0; i < 16; ++i) t[16 * v + i] = off == NONE ? 0.f : pb[off + at + i];
      };
      for (int l = 0; l < c.d_layers; ++l) {
        const DecLayerDesc& d = p.dec[l];
        for (int w = 0; w < 8; ++w) {
          float t[256];
          put(t, 0, d.ckv.bias, 16 * w);
          put(t, 1, d.ckv.bias, 128 + 16 * w);
          put(t, 2, d.qkv.bias, 128 + 16 * w);
          put(t, 3, d.qkv.bias, 256 + 16 * w);
          put(t, 4, d.qkv.bias, 16 * w);
          put(t, 5, d.o.bias, 16 * w);
          put(t, 6, d.ln1.g, 16 * w);
          put(t, 7, d.ln1.b, 16 * w);
          put(t, 8, d.cq.bias, 16 * w);
          put(t, 9, d.co.bias, 16 * w);
          put(t, 10, d.ln2.g, 16 * w);
          put(t, 11, d.ln2.b, 16 * w);
          put(t, 12, d.f1.bias, 16 * (w % 4));
          put(t, 13, d.f2.bias, 16 * w);
          put(t, 14, d.ln3.g, 16 * w);
          put(t, 15, d.ln3.b, 16 * w);
          for (int i = 0; i < 256; ++i) {
            uint32_t u;
            std::memcpy(&u, &t[i], 4);
            wb.push_back((uint16_t)(u & 0xffffu));
            wb.push_back((uint16_t)(u >> 16));
          }
        }
      }
      // opt-in (CET_FEED=1): measured slower than the register path — LDS-DMA fills ≈12 B/clk per CU against the
      // decoder's ≈40 B/clk of weights, and the weights' L2 latency is mostly hidden already
      e->feed_ok = std::getenv("CET_FEED") != nullptr;
    }
    if (pk.wlo) pk.wlo->resize(wb.size(), 0);   // split bf16: the lo blob stays parallel (no tiles there)
  }

  // ProbSparse calls: multiplicity table layout + M debug dumps
  p.n_calls = (int)e->calls.size();
  uint32_t coff = 0;
  js << "], \"m\": [";
  for (int k = 0; k < p.n_calls; ++k) {
    AttnCall& ac = p.calls[k];
    ac.LQ = e->calls[k].LQ;
    ac.LK = e->calls[k].LK;
    ac.U = e->calls[k].U;
    ac.u = u_part(c.factor, ac.LQ);
    ac.cnt_stride = CNT_STRIDE;   // fixed rows (cet_plan.hpp): every key tile of a query row is in bounds
    ac.cnt_off = coff;
    coff += (uint32_t)(r16(ac.LQ) * ac.cnt_stride);
    coff = (coff + 15) & ~15u;
    ac.m_dbg = (int)dbg;
    js << (k ? ", " : "") << "[" << dbg << ", " << NHEAD << ", " << ac.LQ << "]";
    dbg += (int64_t)NHEAD * ac.LQ;
  }
  js << "]}";
  p.cnt_bytes = coff;
  p.draws = 0;
  for (int k = 0; k < p.n_calls; ++k) p.draws += p.calls[k].LQ * p.calls[k].U;
  e->cnt_bytes = coff ? coff : 16;
  p.dbg_stride = (int)dbg;
  e->dbg_json = js.str();
  e->attn_floats = attn_off;
  for (int k = 0; k < MAX_ENC_LAYERS; ++k) p.enc[k].attn_stride = (int)attn_off;

  // LDS layout
  const int LP = r16(std::max(c.seq_len, Ld));
  const int SP = r16(S);
  auto al = [](int x) { return (x + 15) & ~15; };
  p.in_stride = c.enc_in + 4;
  int max_cnt = 0;
  for (int k = 0; k < p.n_calls; ++k)
    if (p.calls[k].u < p.calls[k].LQ) max_cnt = std::max(max_cnt, r16(p.calls[k].LQ) * p.calls[k].cnt_stride);
  if (max_cnt > LMAX * CNT_STRIDE || LP > LMAX || (c.enc_in & 3))
    return fail(CET_E_INVALID, "fused LDS layout: multiplicity table or sequence length out of range");
  // v4: fixed regions (cet_plan.hpp v4_*) | stack output | [x_dec staged at entry, when two sequences
  // per CU still fit with it: its HBM latency then overlaps the LDS zeroing; else it is requested
  // before the last encoder norm, into CTX] | [sampler state: in-kernel replay path only]
  {
    // 4 (mixed): the bf16 layout, the stack output with a lo plane for the split-bf16 decoder
    const int RS = v4_rs(P), planes = P == 4 ? 2 : v4_planes(P);
    p.lds4_cnt = v4_cnt(P);
    p.lds4_enc = v4_enc(P);
    p.lds4_enc_lo = SP * RS;
    p.lds4_zero = al(p.lds4_enc + planes * SP * RS);
    p.lds4_bytes = p.lds4_zero;
    p.lds4_xdec = -1;
    const int xdec_bytes = al(Ld * p.in_stride * 4);
    if (p.lds4_bytes + xdec_bytes <= V4_LDS_2PERCU || P == 1) {
      p.lds4_xdec = p.lds4_bytes;
      p.lds4_bytes += xdec_bytes;
    }
    p.lds4_lab = p.lds4_bytes;
    p.lds4_bytes = al(p.lds4_bytes + c.out_len * c.c_out * 4);
    p.lds4_lncnt = p.lds4_bytes;
    p.lds4_bytes = al(p.lds4_bytes + 16);
    p.lds4_mt = p.lds4_bytes;
    p.lds4_bytes_replay = al(p.lds4_mt + MT_WORDS_HOST * 4);
    if (LMAX * p.in_stride * 4 > v4_ctx_bytes(P) || Ld > 48 || p.lds4_bytes_replay > 160 * 1024)
      return fail(CET_E_INVALID, "v4 LDS layout: staged input, decoder length or LDS size out of range");
  }
  p.stack = c.stack;
  return CET_OK;
}

// The layer-wise model (cet_lw.h): weights as fp32 [N][K] matrices — LSQ grids fake-quantised on the
// host exactly as LSQ.py:65-74 (w_q = round_half_even(clamp(w/s, Qn, Qp))·s), BatchNorm(eval) of the
// distil ConvLayer folded into a per-channel scale / shift, conv kernels reordered to [n][tap·C + c].
int build_lw(cet_engine* e) {
  const auto& c = e->icfg;
  auto m = std::make_unique<lw::Model>();
  const int D = c.d_model, H = c.n_heads, E = D / H, HE = E * H;
  const bool lsq = c.lsq_bits > 0;
  m->C = c.enc_in;
  m->Cd = c.dec_in;
  m->c_out = c.c_out;
  m->L0 = c.seq_len;
  m->Ld = c.label_len + c.out_len;
  m->pred = c.out_len;
  m->D = D;
  m->H = H;
  m->E = E;
  m->HE = HE;
  m->dff = c.d_ff;
  m->prob = c.attn_prob;
  m->mix = c.mix;
  m->act = c.act_relu ? 2 : 1;
  m->stack = c.stack;
  m->out_attn = c.output_attention;
  // "bf16" on a layer-wise engine: bf16 GEMM operands in the fused form (cet_lwf.hip); "auto" stays fp32, the
  // reference's arithmetic class for these shapes
  m->bf16 = e->prec_req == 0;
  e->prec = m->bf16 ? 0 : 3;
  auto Wq = [&](const std::string& n) {   // a quantisable module's weight, LSQ applied
    std::vector<float> w = e->W(n + ".weight");
    if (lsq && e->has(n + ".step_size")) {
      const float st = e->scalar(n + ".step_size");
      (void)lsq_grid(w, st, c.lsq_bits);
      for (auto& x : w) x *= st;
    }
    return w;
  };
  auto dense = [&](std::vector<std::string> names, size_t& w, size_t& b) {
    std::vector<float> ww, bb;
    for (auto& n : names) {
      const auto wi = Wq(n);
      ww.insert(ww.end(), wi.begin(), wi.end());
      const auto& bi = e->W(n + ".bias");
      bb.insert(bb.end(), bi.begin(), bi.end());
    }
    w = m->push(ww);
    b = m->push(bb);
  };
  auto conv3 = [&](const std::vector<float>& w, int N, int Cin) {   // [n][c][tap] → [n][tap·Cin + c]
    std::vector<float> r((size_t)N * 3 * Cin);
    for (int n = 0; n < N; ++n)
      for (int ch = 0; ch < Cin; ++ch)
        for (int tap = 0; tap < 3; ++tap) r[(size_t)n * 3 * Cin + tap * Cin + ch] = w[((size_t)n * Cin + ch) * 3 + tap];
    return r;
  };
  auto vec = [&](const std::string& n) { return m->push(e->W(n)); };
  auto pe_rows = [&](const std::string& n, int L) {
    const auto& pe = e->W(n);
    return m->push(std::vector<float>(pe.begin(), pe.begin() + (size_t)L * D));
  };
  m->emb_enc_w = m->push(conv3(e->W("enc_embedding.value_embedding.tokenConv.weight"), D, c.enc_in));
  m->emb_enc_b = vec("enc_embedding.value_embedding.tokenConv.bias");
  m->pe_enc = pe_rows("enc_embedding.position_embedding.pe", c.seq_len);
  m->emb_dec_w = m->push(conv3(e->W("dec_embedding.value_embedding.tokenConv.weight"), D, c.dec_in));
  m->emb_dec_b = vec("dec_embedding.value_embedding.tokenConv.bias");
  m->pe_dec = pe_rows("dec_embedding.position_embedding.pe", m->Ld);
  int call = 0, S = 0;
  int64_t attn_off = 0;
  e->attn_layout.clear();
  for (int i = 0; i < c.n_enc; ++i) {
    const std::string pre = c.stack ? "encoder.encoders." + std::to_string(i) : std::string("encoder");
    int L = c.stack ? (c.seq_len >> i) : c.seq_len;   // inp_len = x.shape[1] // 2**i (encoder.py:102)
    m->enc_L0.push_back(L);
    std::vector<lw::EncLayer> layers;
    for (int l = 0; l < c.e_layers[i]; ++l) {
      lw::EncLayer d{};
      const std::string lp = pre + ".attn_layers." + std::to_string(l);
      dense({lp + ".attention.query_projection", lp + ".attention.key_projection", lp + ".attention.value_projection"},
            d.wqkv, d.bqkv);
      dense({lp + ".attention.out_projection"}, d.wo, d.bo);
      dense({lp + ".conv1"}, d.w1, d.b1);
      dense({lp + ".conv2"}, d.w2, d.b2);
      d.g1 = vec(lp + ".norm1.weight");
      d.be1 = vec(lp + ".norm1.bias");
      d.g2 = vec(lp + ".norm2.weight");
      d.be2 = vec(lp + ".norm2.bias");
      d.L_in = L;
      d.call = c.attn_prob ? call++ : -1;
      d.attn_off = attn_off;
      if (c.output_attention) {
        e->attn_layout.push_back({attn_off, L});
        attn_off += (int64_t)H * L * L;
      }
      d.conv = c.distil && l < c.e_layers[i] - 1;
      d.L_out = L;
      if (d.conv) {
        const std::string cp = pre + ".conv_layers." + std::to_string(l);
        float step = 1.f;
        std::vector<float> w = e->W(cp + ".downConv.weight");
        if (lsq && e->has(cp + ".downConv.step_size")) {
          step = e->scalar(cp + ".downConv.step_size");
          (void)lsq_grid(w, step, c.lsq_bits);   // the integer grid; the step joins the BN scale
        }
        d.wc = m->push(conv3(w, D, D));
        const auto& cb = e->W(cp + ".downConv.bias");
        const auto& g = e->W(cp + ".norm.weight");
        const auto& bb = e->W(cp + ".norm.bias");
        const auto& rm = e->W(cp + ".norm.running_mean");
        const auto& rv = e->W(cp + ".norm.running_var");
        std::vector<float> sc(D), sh(D);
        for (int n = 0; n < D; ++n) {
          const double inv = (double)g[n] / std::sqrt((double)rv[n] + 1e-5);
          sc[n] = (float)(inv * step);
          sh[n] = (float)(((double)cb[n] - rm[n]) * inv + bb[n]);
        }
        d.sc = m->push(sc);
        d.sh = m->push(sh);
        d.L_out = (L - 1) / 2 + 1;
        L = d.L_out;
      }
      layers.push_back(d);
    }
    m->enc.push_back(layers);
    m->norm_g.push_back(vec(pre + ".norm.weight"));
    m->norm_b.push_back(vec(pre + ".norm.bias"));
    m->enc_rows.push_back(L);
    m->enc_off.push_back(S);
    S += L;
  }
  m->S = S;
  for (int l = 0; l < c.d_layers; ++l) {
    lw::DecLayer d{};
    const std::string lp = "decoder.layers." + std::to_string(l);
    dense({lp + ".self_attention.query_projection", lp + ".self_attention.key_projection",
           lp + ".self_attention.value_projection"}, d.wqkv, d.bqkv);
    dense({lp + ".self_attention.out_projection"}, d.wo, d.bo);
    dense({lp + ".cross_attention.query_projection"}, d.wcq, d.bcq);
    dense({lp + ".cross_attention.key_projection", lp + ".cross_attention.value_projection"}, d.wckv, d.bckv);
    dense({lp + ".cross_attention.out_projection"}, d.wco, d.bco);
    dense({lp + ".conv1"}, d.w1, d.b1);
    dense({lp + ".conv2"}, d.w2, d.b2);
    d.g1 = vec(lp + ".norm1.weight");
    d.be1 = vec(lp + ".norm1.bias");
    d.g2 = vec(lp + ".norm2.weight");
    d.be2 = vec(lp + ".norm2.bias");
    d.g3 = vec(lp + ".norm3.weight");
    d.be3 = vec(lp + ".norm3.bias");
    d.call = c.attn_prob ? call++ : -1;
    m->dec.push_back(d);
  }
  m->dnorm_g = vec("decoder.norm.weight");
  m->dnorm_b = vec("decoder.norm.bias");
  m->proj_w = vec("projection.weight");
  m->proj_b = vec("projection.bias");
  size_t off = 0;
  for (const auto& cl : e->calls) {
    m->call_LQ.push_back(cl.LQ);
    m->call_LK.push_back(cl.LK);
    m->call_U.push_back(cl.U);
    m->call_u.push_back(u_part(c.factor, cl.LQ));
    m->idx_off.push_back(off);
    off += (size_t)cl.LQ * cl.U;
  }
  m->idx_total = off;
  m->attn_floats = attn_off;
  e->attn_floats = attn_off;
  e->dbg_json = "{\"stages\": [], \"m\": []}";
  std::memset(&e->ip, 0, sizeof(e->ip));
  e->ip.n_calls = (int)e->calls.size();
  e->lw = std::move(m);
  return CET_OK;
}

int build_transformer(cet_engine* e);

// Can the fused kernels (d_model 128, 8 heads of 16, d_ff 64 / 128, ≤ 96 rows) carry the model?
bool fused_supported(const cet_informer_config& c) {
  if (c.d_model != DMODEL || c.n_heads != NHEAD) return false;
  if (c.enc_in != c.dec_in || (c.enc_in != 8 && c.enc_in != 16)) return false;
  if (c.d_ff != 64 && c.d_ff != 128) return false;
  if (c.seq_len < 2 || c.seq_len > LMAX) return false;
  const int Ld = c.label_len + c.out_len;
  if (Ld > 48) return false;
  int S = 0;
  for (int i = 0; i < c.n_enc && i < MAX_ENC; ++i) {
    int L = c.stack ? (c.seq_len >> i) : c.seq_len;
    for (int l = 0; l < c.e_layers[i] - 1; ++l)
      if (c.distil) L = (L - 1) / 2 + 1;
    S += L;
  }
  return S <= LMAX && c.c_out <= 128;
}

int check_informer_config(const cet_informer_config& c) {
  if (c.d_model < 1 || c.d_model > lw::LW_DMAX) return fail(CET_E_INVALID, "d_model must be in [1, 1024]");
  if (c.n_heads < 1 || c.n_heads > c.d_model) return fail(CET_E_INVALID, "n_heads must be in [1, d_model]");
  if (c.enc_in < 1 || c.dec_in < 1 || c.enc_in > 1024 || c.dec_in > 1024) return fail(CET_E_INVALID, "enc_in / dec_in out of range");
  if (c.d_ff < 1 || c.d_ff > 8192) return fail(CET_E_INVALID, "d_ff must be in [1, 8192]");
  if (c.seq_len < 2 || c.seq_len > lw::LW_LMAX) return fail(CET_E_INVALID, "seq_len must be in [2, 128]");
  const int Ld = c.label_len + c.out_len;
  if (Ld < 1 || Ld > lw::LW_LMAX || c.out_len < 1 || c.out_len > Ld)
    return fail(CET_E_INVALID, "label_len+out_len must be in [1, 128]");
  if (c.n_enc < 1 || c.n_enc > MAX_ENC) return fail(CET_E_INVALID, "1..4 encoders");
  if (!c.stack && c.n_enc != 1) return fail(CET_E_INVALID, "Informer has one encoder");
  int S = 0, layers = 0;
  for (int i = 0; i < c.n_enc; ++i) {
    if (c.e_layers[i] < 1) return fail(CET_E_INVALID, "e_layers entries must be >= 1");
    int L = c.stack ? (c.seq_len >> i) : c.seq_len;
    if (L < 1) return fail(CET_E_INVALID, "encoder window is empty");
    layers += c.e_layers[i];
    for (int l = 0; l < c.e_layers[i] - 1; ++l)
      if (c.distil) L = (L - 1) / 2 + 1;
    S += L;
  }
  if (layers > MAX_ENC_LAYERS) return fail(CET_E_INVALID, "too many encoder layers");
  if (S > lw::LW_LMAX) return fail(CET_E_INVALID, "encoder stack output longer than 128 rows");
  if (c.d_layers < 1 || c.d_layers > MAX_DEC_LAYERS) return fail(CET_E_INVALID, "1..8 decoder layers");
  if (c.c_out < 1 || c.c_out > 1024) return fail(CET_E_INVALID, "c_out must be in [1, 1024]");
  if (c.factor < 1) return fail(CET_E_INVALID, "factor must be >= 1");
  if (c.lsq_bits < 0 || c.lsq_bits == 1 || c.lsq_bits > 16) return fail(CET_E_INVALID, "lsq_bits must be 0 or 2..16");
  return CET_OK;
}

int upload(cet_engine* e) {
  if (e->kind == 0 && e->generic) {
    if (e->lw->upload()) return fail(CET_E_HIP, "layer-wise weight upload failed");
    for (auto*& h : e->h_lwidx) {
      if (h) HIP_TRY(hipHostFree(h));
      HIP_TRY(hipHostMalloc((void**)&h, std::max<size_t>(e->lw->idx_total, 1) * sizeof(int32_t)));
    }
    for (int i = 0; i < cet_engine::NSLOT; ++i) {
      if (!e->ev[i]) HIP_TRY(hipEventCreateWithFlags(&e->ev[i], hipEventDisableTiming));
      e->ev_used[i] = false;
    }
    return CET_OK;
  }
  const void* plan = e->kind == 0 ? (const void*)&e->ip : (const void*)&e->tp;
  const size_t plan_bytes = e->kind == 0 ? sizeof(InformerPlan) : sizeof(TransformerPlan);
  if (!e->d_plan) HIP_TRY(hipMalloc(&e->d_plan, sizeof(InformerPlan) > sizeof(TransformerPlan)
                                                  ? sizeof(InformerPlan) : sizeof(TransformerPlan)));
  HIP_TRY(hipMemcpy(e->d_plan, plan, plan_bytes, hipMemcpyHostToDevice));
  const size_t hbytes = e->wblob.size() * 2, lbytes = e->wblob_lo.size() * 2;
  const size_t wbytes = hbytes + lbytes, pbytes = e->pblob.size() * 4;
  if (wbytes > e->d_w_bytes) {
    if (e->d_w) HIP_TRY(hipFree(e->d_w));
    HIP_TRY(hipMalloc(&e->d_w, wbytes));
    e->d_w_bytes = wbytes;
  }
  if (pbytes > e->d_p_bytes) {
    if (e->d_p) HIP_TRY(hipFree(e->d_p));
    HIP_TRY(hipMalloc((void**)&e->d_p, pbytes + 64));
    e->d_p_bytes = pbytes;
  }
  HIP_TRY(hipMemcpy(e->d_w, e->wblob.data(), hbytes, hipMemcpyHostToDevice));
  if (lbytes) HIP_TRY(hipMemcpy((char*)e->d_w + hbytes, e->wblob_lo.data(), lbytes, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_p, e->pblob.data(), pbytes, hipMemcpyHostToDevice));
  if (e->kind == 0) {
    for (int i = 0; i < cet_engine::NSLOT; ++i) {
      if (e->h_cnt[i]) HIP_TRY(hipHostFree(e->h_cnt[i]));
      if (e->d_cnt[i]) HIP_TRY(hipFree(e->d_cnt[i]));
      HIP_TRY(hipHostMalloc((void**)&e->h_cnt[i], e->cnt_bytes));
      HIP_TRY(hipMalloc((void**)&e->d_cnt[i], e->cnt_bytes));
      if (!e->ev[i]) HIP_TRY(hipEventCreateWithFlags(&e->ev[i], hipEventDisableTiming));
      e->ev_used[i] = false;
    }
    if (!e->d_mt) {
      HIP_TRY(hipMalloc((void**)&e->d_mt, 2 * 640 * sizeof(uint32_t)));
      HIP_TRY(hipHostMalloc((void**)&e->h_mt, 640 * sizeof(uint32_t)));
      HIP_TRY(hipEventCreateWithFlags(&e->ev_mt, hipEventDisableTiming));
      HIP_TRY(hipMalloc((void**)&e->d_ticket, 64));
      HIP_TRY(hipMemset(e->d_ticket, 0, 64));
    }
    for (auto*& t : e->d_tab) {
      if (t) HIP_TRY(hipFree(t));
      HIP_TRY(hipMalloc((void**)&t, e->cnt_bytes));
    }
    // Prepared tables pending: d_mt[mt_cur] is already past their draws, which no forward has
    // consumed yet.  Dropping them means the next forward must restart from the host mirror
    // (the state after the forwards actually launched), not from d_mt[mt_cur].
    if (e->tab_ready) e->dev_mt_valid = false;
    e->tab_ready = false;
    e->draws_per_forward = 0;
    for (const auto& c : e->calls) e->draws_per_forward += (int64_t)c.LQ * c.U;
  }
  return CET_OK;
}

// Host-side packing + plan (no device needed).
int finalize_host(cet_engine* e) {
  if (!e->dirty) return CET_OK;
  for (auto& n : e->order) {
    const Weight& w = e->weights[n];
    if (w.required && !w.loaded) return fail(CET_E_MISSING, "weight not loaded: " + n);
  }
  int rc = e->kind == 0 ? build_informer(e) : build_transformer(e);
  if (rc) return rc;
  e->dirty = false;
  e->uploaded = false;
  return CET_OK;
}

int finalize(cet_engine* e) {
  int rc = finalize_host(e);
  if (rc) return rc;
  if (e->uploaded) return CET_OK;
  rc = upload(e);
  if (rc) return rc;
  e->uploaded = true;
  return CET_OK;
}

int build_transformer(cet_engine* e) {
  const auto& c = e->tcfg;
  const int D = c.d_model;
  e->wblob.clear();
  e->pblob.clear();
  Packer pk{e->wblob, e->pblob};
  TransformerPlan& p = e->tp;
  std::memset(&p, 0, sizeof(p));
  p.C = c.src_vocab;
  p.c_out = c.tgt_vocab;
  p.src_len = c.src_seq_len;
  p.tgt_len = c.tgt_seq_len + c.label_len;
  p.pred_len = c.tgt_seq_len;
  p.N = c.N;
  p.dff = c.d_ff;
  // bias-free Q/K/V/O (buildingblocks.py:109-113), concatenated along the output axis
  auto mha = [&](std::vector<std::string> names) {
    std::vector<float> w;
    for (auto& n : names) {
      const auto& wi = e->W(n + ".weight");
      w.insert(w.end(), wi.begin(), wi.end());
    }
    return pk.gemm(w, (int)w.size() / D, D, nullptr, nullptr);
  };
  auto lin = [&](const std::string& n, int K) {
    const auto& w = e->W(n + ".weight");
    return pk.gemm(w, (int)w.size() / K, K, e->W(n + ".bias").data(), nullptr);
  };
  auto lnt = [&](const std::string& n) { return pk.ln(e->W(n + ".alpha"), e->W(n + ".bias")); };
  auto emb = [&](const std::string& pre, int C) {
    const auto& w = e->W(pre + ".weight");
    std::vector<float> m((size_t)D * 3 * C);
    for (int n = 0; n < D; ++n)
      for (int ch = 0; ch < C; ++ch)
        for (int tap = 0; tap < 3; ++tap) m[(size_t)n * 3 * C + tap * C + ch] = w[((size_t)n * C + ch) * 3 + tap];
    return pk.gemm(m, D, 3 * C, e->W(pre + ".bias").data(), nullptr);
  };
  p.emb_src = emb("src_embed.tokenEmbedding", c.src_vocab);
  p.emb_tgt = emb("tgt_embed.tokenEmbedding", c.tgt_vocab);
  p.pe_src = pk.vec(e->W("src_pos.pe").data(), p.src_len * D, p.src_len * D);
  p.pe_tgt = pk.vec(e->W("tgt_pos.pe").data(), p.tgt_len * D, p.tgt_len * D);
  int64_t dbg = 0;
  std::ostringstream js;
  js << "{\"stages\": [";
  bool firstj = true;
  auto jstage = [&](const std::string& name, int64_t off, int rows) {
    js << (firstj ? "" : ", ") << "[\"" << name << "\", " << off << ", " << rows << ", " << D << "]";
    firstj = false;
  };
  p.dbg_emb = (int)dbg;
  jstage("enc_emb", dbg, p.src_len);
  dbg += (int64_t)p.src_len * D;
  for (int l = 0; l < c.N; ++l) {
    const std::string lp = "encoder.layers." + std::to_string(l);
    auto& d = p.enc[l];
    d.qkv = mha({lp + ".self_attention_block.w_q", lp + ".self_attention_block.w_k", lp + ".self_attention_block.w_v"});
    d.o = mha({lp + ".self_attention_block.w_o"});
    d.f1 = lin(lp + ".feed_forward_block.linear_1", D);
    d.f2 = lin(lp + ".feed_forward_block.linear_2", c.d_ff);
    d.ln0 = lnt(lp + ".residual_connections.0.norm");
    d.ln1 = lnt(lp + ".residual_connections.1.norm");
    d.dbg = (int)dbg;
    jstage("enc_layer" + std::to_string(l), dbg, p.src_len);
    dbg += (int64_t)p.src_len * D;
  }
  p.enc_norm = lnt("encoder.norm");
  p.dbg_enc_out = (int)dbg;
  jstage("enc_out", dbg, p.src_len);
  dbg += (int64_t)p.src_len * D;
  p.dbg_dec_emb = (int)dbg;
  jstage("dec_emb", dbg, p.tgt_len);
  dbg += (int64_t)p.tgt_len * D;
  for (int l = 0; l < c.N; ++l) {
    const std::string lp = "decoder.layers." + std::to_string(l);
    auto& d = p.dec[l];
    d.qkv = mha({lp + ".self_attention_block.w_q", lp + ".self_attention_block.w_k", lp + ".self_attention_block.w_v"});
    d.o = mha({lp + ".self_attention_block.w_o"});
    d.cq = mha({lp + ".cross_attention_block.w_q"});
    d.ckv = mha({lp + ".cross_attention_block.w_k", lp + ".cross_attention_block.w_v"});
    d.co = mha({lp + ".cross_attention_block.w_o"});
    d.f1 = lin(lp + ".feed_forward_block.linear_1", D);
    d.f2 = lin(lp + ".feed_forward_block.linear_2", c.d_ff);
    d.ln0 = lnt(lp + ".residual_connections.0.norm");
    d.ln1 = lnt(lp + ".residual_connections.1.norm");
    d.ln2 = lnt(lp + ".residual_connections.2.norm");
    d.dbg = (int)dbg;
    jstage("dec_layer" + std::to_string(l), dbg, p.tgt_len);
    dbg += (int64_t)p.tgt_len * D;
  }
  p.dec_norm = lnt("decoder.norm");
  p.dbg_dec_out = (int)dbg;
  jstage("dec_out", dbg, p.tgt_len);
  dbg += (int64_t)p.tgt_len * D;
  p.proj = lin("projection_layer.proj", D);
  js << "], \"m\": []}";
  e->dbg_json = js.str();
  p.dbg_stride = (int)dbg;
  e->calls.clear();
  e->attn_floats = 0;
  e->attn_layout.clear();
  // LDS: X fp32 | Q | K (+FFN hidden, staged input) | Vt | ENC (= encoder-phase LN output) | decoder LN output
  const int LP = r16(std::max(p.src_len, p.tgt_len));
  auto al = [](int x) { return (x + 15) & ~15; };
  int o = 0;
  p.lds_X = o; o = al(o + LP * XS * 4);
  p.lds_Q = o; o = al(o + LP * BS * 2);
  p.lds_K = o; o = al(o + LP * BS * 2);
  p.vts = LP + 8;
  p.lds_VT = o; o = al(o + DMODEL * p.vts * 2);
  p.lds_ENC = o; o = al(o + LP * BS * 2);
  p.lds_XN = o; o = al(o + r16(p.tgt_len) * BS * 2);
  p.lds_bytes = o;
  p.in_stride = c.src_vocab + 4;
  if (o > 160 * 1024) return fail(CET_E_INVALID, "sequence too long for the LDS-resident Transformer kernel");
  p.lds4_bytes = v4_enc(0) + al(p.tgt_len * p.in_stride * 4);
  if (p.src_len > LMAX || p.tgt_len > 48 || LMAX * p.in_stride * 4 > v4_ctx_bytes(0))
    return fail(CET_E_INVALID, "v4 Transformer layout: sequence lengths out of range");
  return CET_OK;
}

// Record the "before" event of a timed launch (returns the pair index, or -1).
int timing_mark(cet_engine* e, hipStream_t st) {
  if (!e->timing) return -1;
  if (e->timing_seen++ % e->timing_every) return -1;
  if (e->t_n * 2 + 2 > e->t_ev.size()) {
    for (int i = 0; i < 64; ++i) {
      hipEvent_t ev_;
      if (hipEventCreate(&ev_) != hipSuccess) return -1;
      e->t_ev.push_back(ev_);
    }
  }
  const int k = (int)e->t_n++;
  (void)hipEventRecord(e->t_ev[2 * k], st);
  return k;
}

}  // namespace

// =================================================================== C ABI
extern "C" {

const char* cet_last_error(void) { return g_err.c_str(); }
int cet_version(void) { return 1; }

int cet_create_informer(const cet_informer_config* cfg, cet_engine** out) {
  if (!cfg || !out) return fail(CET_E_INVALID, "null argument");
  int rc = check_informer_config(*cfg);
  if (rc) return rc;
  auto e = std::make_unique<cet_engine>();
  e->kind = 0;
  e->icfg = *cfg;
  e->generic = !fused_supported(*cfg) || std::getenv("CET_LAYERWISE") != nullptr;
  e->enc_split_ok = std::getenv("CET_NO_ENC_SPLIT") == nullptr;
  schema_informer(e.get());
  // shapes of the ProbSparse draws are known before weights arrive
  const auto& c = *cfg;
  if (c.attn_prob) {
    for (int i = 0; i < c.n_enc; ++i) {
      int L = c.stack ? (c.seq_len >> i) : c.seq_len;
      for (int l = 0; l < c.e_layers[i]; ++l) {
        e->calls.push_back({L, L, u_part(c.factor, L)});
        if (c.distil && l < c.e_layers[i] - 1) L = (L - 1) / 2 + 1;
      }
    }
    const int Ld = c.label_len + c.out_len;
    for (int l = 0; l < c.d_layers; ++l) e->calls.push_back({Ld, Ld, u_part(c.factor, Ld)});
  }
  e->idx.assign(e->calls.size(), {});
  e->idx_set.assign(e->calls.size(), false);
  *out = e.release();
  return CET_OK;
}

int cet_create_transformer(const cet_transformer_config* cfg, cet_engine** out) {
  if (!cfg || !out) return fail(CET_E_INVALID, "null argument");
  const auto& c = *cfg;
  if (c.d_model != DMODEL || c.h != NHEAD) return fail(CET_E_INVALID, "this build supports d_model=128, h=8");
  if (c.src_vocab != c.tgt_vocab || (c.src_vocab % 8) || c.src_vocab > 21)
    return fail(CET_E_INVALID, "src_vocab == tgt_vocab, a multiple of 8, <= 21 required");
  if (c.d_ff != 64 && c.d_ff != 128) return fail(CET_E_INVALID, "d_ff must be 64 or 128 in this build");
  if (c.src_seq_len < 2 || c.src_seq_len > LMAX) return fail(CET_E_INVALID, "src_seq_len must be in [2, 96]");
  const int Ld = c.tgt_seq_len + c.label_len;
  if (c.tgt_seq_len < 1 || Ld > 48) return fail(CET_E_INVALID, "tgt_seq_len+label_len must be <= 48");
  if (c.N < 1 || c.N > MAX_DEC_LAYERS) return fail(CET_E_INVALID, "N must be in [1, 8]");
  auto e = std::make_unique<cet_engine>();
  e->kind = 1;
  e->tcfg = c;
  schema_transformer(e.get());
  *out = e.release();
  return CET_OK;
}

void cet_destroy(cet_engine* e) { delete e; }

int cet_load_weight(cet_engine* e, const char* name, const float* data, int64_t numel) {
  if (!e || !name || (!data && numel)) return fail(CET_E_INVALID, "null argument");
  auto it = e->weights.find(name);
  if (it == e->weights.end()) return fail(CET_E_INVALID, std::string("unexpected key: ") + name);
  int64_t n = 1;
  for (auto s : it->second.shape) n *= s;
  if (n != numel) return fail(CET_E_INVALID, std::string("size mismatch for ") + name);
  it->second.data.assign(data, data + numel);
  it->second.loaded = true;
  e->dirty = true;
  return CET_OK;
}

int cet_missing_weights(cet_engine* e, char* first_missing, int buflen) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  int n = 0;
  for (auto& name : e->order) {
    const Weight& w = e->weights[name];
    if (w.required && !w.loaded) {
      if (!n && first_missing && buflen > 0) std::snprintf(first_missing, buflen, "%s", name.c_str());
      ++n;
    }
  }
  return n;
}

int cet_prob_calls(cet_engine* e, int* shapes, int max) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  const int n = (int)e->calls.size();
  for (int i = 0; i < n && i < max && shapes; ++i) {
    shapes[3 * i] = e->calls[i].LK;
    shapes[3 * i + 1] = e->calls[i].LQ;
    shapes[3 * i + 2] = e->calls[i].U;
  }
  return n;
}

int cet_set_prob_indices(cet_engine* e, int call, const int32_t* idx, int L_Q, int U) {
  if (!e || !idx) return fail(CET_E_INVALID, "null argument");
  if (call < 0 || call >= (int)e->calls.size()) return fail(CET_E_INVALID, "call out of range");
  const auto& c = e->calls[call];
  if (c.LQ != L_Q || c.U != U) return fail(CET_E_INVALID, "index sample shape mismatch");
  for (int i = 0; i < L_Q * U; ++i)
    if (idx[i] < 0 || idx[i] >= c.LK) return fail(CET_E_INVALID, "index out of range");
  e->idx[call].assign(idx, idx + (size_t)L_Q * U);
  e->idx_set[call] = true;   // one-shot: consumed by the next forward; a seeded native stream is not touched
  return CET_OK;
}

int cet_seed(cet_engine* e, uint64_t seed) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  e->rng.seed(seed);
  e->native_rng = true;
  e->host_lag = 0;
  e->dev_mt_valid = false;
  return CET_OK;
}

int64_t cet_native_draw(cet_engine* e, int32_t* out, int64_t n_max) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  if (!e->native_rng) return fail(CET_E_STATE, "call cet_seed first");
  int64_t n = 0;
  for (const auto& c : e->calls) n += (int64_t)c.LQ * c.U;
  if (!out) return n;
  if (n_max < n) return fail(CET_E_INVALID, "buffer too small");
  e->sync_host_rng();
  e->dev_mt_valid = false;   // the host stream moved past the device copy
  int64_t k = 0;
  for (const auto& c : e->calls)
    for (int i = 0; i < c.LQ * c.U; ++i) out[k++] = (int32_t)(e->rng.next() % (uint32_t)c.LK);
  return n;
}

int64_t cet_peek_draw(cet_engine* e, int32_t* out, int64_t n_max) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  if (!e->native_rng) return fail(CET_E_STATE, "call cet_seed first");
  int64_t n = 0;
  for (const auto& c : e->calls) n += (int64_t)c.LQ * c.U;
  if (!out) return n;
  if (n_max < n) return fail(CET_E_INVALID, "buffer too small");
  e->sync_host_rng();        // the host mirror catches up with the launched forwards (device copy unaffected)
  MT19937 r = e->rng;        // draw from a copy: the stream does not move
  int64_t k = 0;
  for (const auto& c : e->calls)
    for (int i = 0; i < c.LQ * c.U; ++i) out[k++] = (int32_t)(r.next() % (uint32_t)c.LK);
  return n;
}

int64_t cet_attns_floats(cet_engine* e) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  int rc = finalize_host(e);
  if (rc) return rc;
  return e->attn_floats;
}

int cet_attns_layout(cet_engine* e, int64_t* offsets, int* lengths, int max) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  int rc = finalize_host(e);
  if (rc) return rc;
  const int n = (int)e->attn_layout.size();
  for (int i = 0; i < n && i < max; ++i) {
    if (offsets) offsets[i] = e->attn_layout[i].first;
    if (lengths) lengths[i] = e->attn_layout[i].second;
  }
  return n;
}

int cet_set_debug(cet_engine* e, float* dbg) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  e->dbg = dbg;
  return CET_OK;
}

int64_t cet_debug_floats(cet_engine* e) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  int rc = finalize_host(e);
  if (rc) return rc;
  return e->kind == 0 ? e->ip.dbg_stride : e->tp.dbg_stride;
}

int cet_debug_layout(cet_engine* e, char* json, int buflen) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  int rc = finalize_host(e);
  if (rc) return rc;
  if (json && buflen > 0) std::snprintf(json, buflen, "%s", e->dbg_json.c_str());
  return (int)e->dbg_json.size();
}

// The plan's compile-time instance (cet_kernels.h V4Shape): C2's encoder — one encoder of four layers on rows
// 90 → 45 → 23 → 12, the first three distilling — or the TimingAnalysis stack e_layers [4, 3] — that encoder and
// one on the window x[:, -45:] (45 → 23 → 12, the first two distilling), 24 stack rows, a decoder of ≤ 16 rows.
static bool encoder_rows_are(const InformerPlan& p, int e, int n, const int* lin, const int* lout) {
  if (p.enc_layers[e] != n) return false;
  for (int l = 0; l < n; ++l) {
    const auto& d = p.enc[p.enc_first[e] + l];
    if (d.L_in != lin[l] || d.L_out != lout[l] || (d.conv.n != 0) != (l < n - 1)) return false;
  }
  return true;
}
// CET_LDS_POISON=1: the v4 kernels fill their LDS with NaN at entry (diagnostic, tests/test_gpu_poison.py)
static int lds_poison_requested() {
  const char* v = std::getenv("CET_LDS_POISON");
  return v && std::strcmp(v, "0") != 0 ? 1 : 0;
}
static int plan_shape(const InformerPlan& p, int dff) {
  static const int lin4[4] = {90, 45, 23, 12}, lout4[4] = {45, 23, 12, 12};
  static const int lin3[3] = {45, 23, 12}, lout3[3] = {23, 12, 12};
  // the compile-time instances exist for d_ff 64 only: any other d_ff keeps the generic (and generic split) ones
  if (p.seq_len != 90 || dff != 64) return V4S_GENERIC;
  if (p.n_enc == 1 && encoder_rows_are(p, 0, 4, lin4, lout4)) return V4S_C2;
  if (p.n_enc == 2 && encoder_rows_are(p, 0, 4, lin4, lout4) && encoder_rows_are(p, 1, 3, lin3, lout3) && p.S == 24 &&
      p.dec_len <= 16)
    return V4S_E43;
  return V4S_GENERIC;
}

static int launch_fused(cet_engine* e, const InformerArgs& a, hipStream_t st) {
  const InformerPlan& p = e->ip;
  InformerArgs b = a;
  b.wlo = (uint32_t)(e->wblob.size() * 2);
  const char* c2env = std::getenv("CET_V4_C2");   // "0": the generic instance for every plan (A/B)
  b.shape = c2env && std::strcmp(c2env, "0") == 0 ? V4S_GENERIC : plan_shape(p, e->icfg.d_ff);
  b.stagger = 0;
  if (const char* sg = std::getenv("CET_STAGGER")) b.stagger = std::atoi(sg);
  b.poison = lds_poison_requested();
  b.feed = 0;
  b.enc_split = 0;
  b.enc_xchg = nullptr;
  b.enc_count = nullptr;
  const bool diag = a.attns || a.dbg || a.stamps;
  const bool replay = a.mt_in && !a.cnt;
  // encoder split (v4): the encoders of a stack are independent until the decoder, so at small batches
  // each runs on its own workgroup (bf16 policy, no ProbSparse draws, production outputs only, the
  // whole grid resident at two workgroups per CU)
  static const int64_t split_max = [] {   // CET_SPLIT_MAX: the largest B · n_enc split (A/B knob; default 512)
    const char* v = std::getenv("CET_SPLIT_MAX");
    return v ? (int64_t)std::atoll(v) : (int64_t)512;
  }();
  const bool split = e->enc_split_ok && e->prec == 0 && p.n_enc > 1 && p.n_calls == 0 && !diag &&
                     (int64_t)a.B * p.n_enc <= split_max;
  if (split) {
    const size_t words = (size_t)a.B * p.S * (v4_rs(0) / 8);
    if (words > e->enc_xchg_n) {
      if (e->d_enc_xchg) HIP_TRY(hipFree(e->d_enc_xchg));
      HIP_TRY(hipMalloc((void**)&e->d_enc_xchg, words * sizeof(uint64_t)));
      e->enc_xchg_n = words;
    }
    if (a.B > e->enc_count_n) {
      if (e->d_enc_count) HIP_TRY(hipFree(e->d_enc_count));
      HIP_TRY(hipMalloc((void**)&e->d_enc_count, (size_t)a.B * sizeof(unsigned)));
      e->enc_count_n = a.B;
      // zeroed on every (re)allocation, on this launch's stream; the kernel re-arms it after each use
      HIP_TRY(hipMemsetAsync(e->d_enc_count, 0, (size_t)a.B * sizeof(unsigned), st));
    }
    b.enc_split = p.n_enc;
    b.enc_xchg = e->d_enc_xchg;
    b.enc_count = e->d_enc_count;
  }
  e->last_path = split ? CET_PATH_V4_SPLIT : CET_PATH_V4;
  {
    // the instance launch_v4 takes (v4_instance: one decision for both sides)
    const int inst = v4_instance(b, e->prec, e->icfg.d_ff);
    const int kp = e->prec == 4 ? 0 : e->prec, kd = e->prec == 4 ? 1 : e->prec;   // encoder / decoder precision
    const int sh = inst == V4I_SHAPE || inst == V4I_SHAPE_STAMPS || (inst == V4I_SPLIT && b.shape == V4S_E43) ? b.shape : 0;
    // the decoder weight feed: the bf16 shape instances (and E43's split form) of a plan build_informer accepted
    b.feed = e->feed_ok && e->prec == 0 && sh != 0 ? 1 : 0;
    char nm[160];
    std::snprintf(nm, sizeof nm, "cet::v4::informer_forward_v4<%d, %s, %d, %s, %d, %s, %s, %d>", e->icfg.d_ff,
                  inst == V4I_DIAG ? "true" : "false", kp, inst == V4I_SPLIT ? "true" : "false", sh,
                  inst == V4I_SHAPE_STAMPS ? "true" : "false", b.feed ? "true" : "false", kd);
    e->last_kernel = inst == V4I_NONE ? std::string() : std::string(nm);
  }
  return cet_launch_informer_v4(&b, e->prec, e->icfg.d_ff, replay ? p.lds4_bytes_replay : p.lds4_bytes, st);
}

static int forward_impl(cet_engine* e, const float* x_enc, const float* x_dec, int B, float* out, float* attns,
                        const float* label, float* nmse_acc, double* nmse_sums, void* stream);

// Layer-wise forward: this forward's ProbSparse draws (explicit indices, or the native stream drawn
// on the host — the same torch.randint sequence) staged through a pinned ring, then the operator
// launches, then NMSE_Split if a label is given.
static int forward_lw(cet_engine* e, const float* x_enc, const float* x_dec, int B, float* out, float* attns,
                      const float* label, float* nmse_acc, double* nmse_sums, hipStream_t st) {
  const int n_calls = (int)e->calls.size();
  bool explicit_idx = n_calls > 0, any_idx = false;
  for (int c = 0; c < n_calls; ++c) {
    explicit_idx = explicit_idx && e->idx_set[c];
    any_idx = any_idx || e->idx_set[c];
  }
  if (any_idx && !explicit_idx) return fail(CET_E_STATE, "ProbSparse indices set for some calls only");
  // refused before any draw or timing event, so a refused forward leaves the RNG stream and the timing slots alone
  if (e->lw->bf16_refused(attns))
    return fail(CET_E_INVALID, "bf16 operands need the fused layer-wise form (no attention maps, a working set that "
                               "fits one workgroup, feature counts that are multiples of 8)");
  if (n_calls && !explicit_idx && !e->native_rng)
    return fail(CET_E_STATE, "ProbSparse indices not set (cet_set_prob_indices for every call, or cet_seed)");
  if (n_calls) {
    if (!explicit_idx) {
      e->sync_host_rng();
      e->dev_mt_valid = false;
    }
    const int k = e->slot;
    e->slot = (e->slot + 1) % cet_engine::NSLOT;
    if (e->ev_used[k]) HIP_TRY(hipEventSynchronize(e->ev[k]));
    int32_t* h = e->h_lwidx[k];
    size_t o = 0;
    for (int c = 0; c < n_calls; ++c) {
      const auto& sh = e->calls[c];
      const size_t n = (size_t)sh.LQ * sh.U;
      if (explicit_idx) {
        std::memcpy(h + o, e->idx[c].data(), n * sizeof(int32_t));
      } else {
        for (size_t i = 0; i < n; ++i) h[o + i] = (int32_t)(e->rng.next() % (uint32_t)sh.LK);
      }
      o += n;
    }
    if (explicit_idx) e->idx_set.assign(e->calls.size(), false);
    HIP_TRY(hipMemcpyAsync(e->lw->d_idx, h, o * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipEventRecord(e->ev[k], st));
    e->ev_used[k] = true;
  }
  const int tk = timing_mark(e, st);
  const int rc = e->lw->forward(x_enc, x_dec, B, out, attns, e->lw->d_idx, st);
  if (tk >= 0) (void)hipEventRecord(e->t_ev[2 * tk + 1], st);
  e->last_path = e->lw->last_fused ? CET_PATH_LW_FUSED : CET_PATH_LW;
  e->last_kernel = !e->lw->last_fused ? ""   // the operator path launches several kernels
                  : e->lw->bf16        ? "cet::lw::lw_fused (bf16 operands)"
                                       : "cet::lw::lw_fused";
  if (rc) return fail(CET_E_HIP, std::string("layer-wise launch failed: ") + hipGetErrorString(hipGetLastError()));
  if (label && cet_launch_nmse_split(out, label, B, e->icfg.out_len, e->icfg.c_out, nmse_acc, nullptr, 1, nmse_sums, st))
    return fail(CET_E_HIP, "nmse launch failed");
  return CET_OK;
}

int cet_forward(cet_engine* e, const float* x_enc, const float* x_dec, int B, float* out, float* attns,
                void* stream) {
  return forward_impl(e, x_enc, x_dec, B, out, attns, nullptr, nullptr, nullptr, stream);
}

int cet_forward_nmse(cet_engine* e, const float* x_enc, const float* x_dec, int B, float* out, const float* label,
                     float* nmse_acc, double* nmse_sums, void* stream) {
  if (!label || (!nmse_acc && !nmse_sums)) return fail(CET_E_INVALID, "null argument");
  if (e && e->kind != 0) return fail(CET_E_INVALID, "cet_forward_nmse: Informer engines only");
  return forward_impl(e, x_enc, x_dec, B, out, nullptr, label, nmse_acc, nmse_sums, stream);
}

static int forward_impl(cet_engine* e, const float* x_enc, const float* x_dec, int B, float* out, float* attns,
                        const float* label, float* nmse_acc, double* nmse_sums, void* stream) {
  if (!e || !x_enc || !x_dec || !out) return fail(CET_E_INVALID, "null argument");
  if (B < 0 || B > (1 << 24)) return fail(CET_E_INVALID, "bad batch size");
  int rc = finalize(e);
  if (rc) return rc;
  if (B == 0) return CET_OK;
  hipStream_t st = (hipStream_t)stream;
  if (e->kind == 1) {
    TransformerArgs a;
    a.plan = (const TransformerPlan*)e->d_plan;
    a.weights = e->d_w;
    a.params = e->d_p;
    a.x_enc = x_enc;
    a.x_dec = x_dec;
    a.out = out;
    a.dbg = e->dbg;
    a.B = B;
    a.poison = lds_poison_requested();
    const char* c3env = std::getenv("CET_V4_C3");
    a.c3 = e->tp.src_len == 90 && e->tp.tgt_len == 15 && !(c3env && std::strcmp(c3env, "0") == 0);
    {
      const bool tdiag = a.dbg != nullptr, c3 = e->tcfg.d_ff == 64 && a.c3 && !tdiag;
      char nm[128];
      std::snprintf(nm, sizeof nm, "cet::v4::transformer_forward_v4<%d, %s, %s>", e->tcfg.d_ff, tdiag ? "true" : "false",
                    c3 ? "true" : "false");
      e->last_kernel = nm;
    }
    const int tk = timing_mark(e, st);
    rc = cet_launch_transformer_v4(&a, e->tcfg.d_ff, e->tp.lds4_bytes, st);
    if (tk >= 0) (void)hipEventRecord(e->t_ev[2 * tk + 1], st);
    if (rc) return fail(CET_E_HIP, std::string("transformer launch failed: ") + hipGetErrorString(hipGetLastError()));
    return CET_OK;
  }
  if (e->generic) return forward_lw(e, x_enc, x_dec, B, out, attns, label, nmse_acc, nmse_sums, st);
  const InformerPlan& p = e->ip;
  InformerArgs a;
  a.plan = (const InformerPlan*)e->d_plan;
  a.weights = e->d_w;
  a.params = e->d_p;
  a.cnt = nullptr;
  a.mt_in = nullptr;
  a.mt_out = nullptr;
  a.cnt_next = nullptr;
  a.ticket = nullptr;
  a.x_enc = x_enc;
  a.x_dec = x_dec;
  a.out = out;
  a.attns = (attns && e->icfg.output_attention) ? attns : nullptr;
  a.dbg = e->dbg;
  a.stamps = e->stamps;
  a.B = B;
  a.wlo = 0;
  a.lds_bytes = 0;
  a.label = nullptr;
  a.nmse_part = nullptr;
  a.nmse_acc = nullptr;
  a.nmse_sums = nullptr;
  // NMSE_Split of this forward's output: fused into the v4 kernel's epilogue (one n-tile of outputs),
  // else the standalone reduction right after the forward on the same stream
  const bool fuse_nmse = label && e->icfg.c_out <= 16;
  if (fuse_nmse) {
    const size_t need = (size_t)B * e->icfg.out_len;
    if (need > e->nmse_part_n) {
      if (e->d_nmse_part) HIP_TRY(hipFree(e->d_nmse_part));
      HIP_TRY(hipMalloc((void**)&e->d_nmse_part, need * sizeof(float2)));
      e->nmse_part_n = need;
    }
    a.label = label;
    a.nmse_part = e->d_nmse_part;
    a.nmse_acc = nmse_acc;
    a.nmse_sums = nmse_sums;
    a.ticket = e->d_ticket;
  }
  auto finish_nmse = [&]() -> int {
    if (!label || fuse_nmse) return CET_OK;
    if (cet_launch_nmse_split(out, label, B, e->icfg.out_len, e->icfg.c_out, nmse_acc, nullptr, 1, nmse_sums,
                              (hipStream_t)stream))
      return fail(CET_E_HIP, "nmse launch failed");
    return CET_OK;
  };
  // explicit indices (cet_set_prob_indices for every call) win for this one forward
  bool explicit_idx = p.n_calls > 0, any_idx = false;
  for (int c = 0; c < p.n_calls; ++c) {
    explicit_idx = explicit_idx && e->idx_set[c];
    any_idx = any_idx || e->idx_set[c];
  }
  if (any_idx && !explicit_idx) return fail(CET_E_STATE, "ProbSparse indices set for some calls only");
  if (p.n_calls && !explicit_idx && !e->native_rng)
    return fail(CET_E_STATE, "ProbSparse indices not set (cet_set_prob_indices for every call, or cet_seed)");
  if (e->native_rng && p.n_calls && !e->host_sampler && !explicit_idx) {
    // ---- resident sampler: the kernel replays this forward's draws itself (cet_mt.hpp)
    if (!e->dev_mt_valid) {
      e->sync_host_rng();
      if (e->ev_mt_used) HIP_TRY(hipEventSynchronize(e->ev_mt));
      std::memcpy(e->h_mt, e->rng.mt, sizeof(e->rng.mt));
      e->h_mt[624] = (uint32_t)e->rng.idx;
      HIP_TRY(hipMemcpyAsync(e->d_mt + 640 * e->mt_cur, e->h_mt, 640 * sizeof(uint32_t), hipMemcpyHostToDevice, st));
      HIP_TRY(hipEventRecord(e->ev_mt, st));
      e->ev_mt_used = true;
      e->dev_mt_valid = true;
      e->tab_ready = false;
    }
    const bool prep = B >= cet_engine::PREP_MIN_B;
    if (prep && !e->tab_ready) {
      // first forward after a (re)seed: this forward's tables from a one-workgroup launch
      const int lds = std::max(640 * 4 + LMAX * CNT_STRIDE, std::min(replay_fast_lds(p), 64 * 1024));
      if (cet_launch_sampler_prep((const InformerPlan*)e->d_plan, e->d_mt + 640 * e->mt_cur,
                                  e->d_mt + 640 * (1 - e->mt_cur), e->d_tab[e->tab_cur], lds, st))
        return fail(CET_E_HIP, std::string("sampler prep launch failed: ") + hipGetErrorString(hipGetLastError()));
      e->mt_cur = 1 - e->mt_cur;
      e->tab_ready = true;
    }
    if (e->tab_ready) {
      // prepared tables: staged by this forward; a large one also prepares the next forward's
      // (d_mt[mt_cur] is the state after this forward's draws)
      a.cnt = e->d_tab[e->tab_cur];
      if (prep) {
        a.mt_in = e->d_mt + 640 * e->mt_cur;
        a.mt_out = e->d_mt + 640 * (1 - e->mt_cur);
        a.cnt_next = e->d_tab[1 - e->tab_cur];
        a.ticket = e->d_ticket;   // (also the fused NMSE's finish counter)
        e->mt_cur = 1 - e->mt_cur;
        e->tab_cur = 1 - e->tab_cur;
      } else {
        e->tab_ready = false;
      }
    } else {
      a.mt_in = e->d_mt + 640 * e->mt_cur;
      a.mt_out = e->d_mt + 640 * (1 - e->mt_cur);
      e->mt_cur = 1 - e->mt_cur;
    }
    e->host_lag += e->draws_per_forward;
    const int tk = timing_mark(e, st);
    rc = launch_fused(e, a, st);
    if (tk >= 0) (void)hipEventRecord(e->t_ev[2 * tk + 1], st);
    if (rc) return fail(CET_E_HIP, std::string("informer launch failed: ") + hipGetErrorString(hipGetLastError()));
    return finish_nmse();
  }
  // ---- this forward's ProbSparse draws → key multiplicity tables (host-built)
  const bool native_now = e->native_rng && !explicit_idx;
  if (native_now) {
    e->sync_host_rng();
    e->dev_mt_valid = false;
  }
  const int k = e->slot;
  e->slot = (e->slot + 1) % cet_engine::NSLOT;
  if (e->ev_used[k]) HIP_TRY(hipEventSynchronize(e->ev[k]));
  uint8_t* h = e->h_cnt[k];
  if (p.n_calls) {
    std::memset(h, 0, e->cnt_bytes);
    for (int c = 0; c < p.n_calls; ++c) {
      const auto& sh = e->calls[c];
      const AttnCall& ac = p.calls[c];
      uint8_t* tab = h + ac.cnt_off;
      if (native_now) {
        for (int q = 0; q < sh.LQ; ++q)
          for (int j = 0; j < sh.U; ++j) {
            const int key = (int)(e->rng.next() % (uint32_t)sh.LK);
            tab[q * ac.cnt_stride + cnt_pos_v2(key)]++;
          }
      } else {
        const int32_t* id = e->idx[c].data();
        for (int q = 0; q < sh.LQ; ++q)
          for (int j = 0; j < sh.U; ++j) {
            const int key = id[q * sh.U + j];
            tab[q * ac.cnt_stride + cnt_pos_v2(key)]++;
          }
      }
    }
    if (explicit_idx) e->idx_set.assign(e->calls.size(), false);
    HIP_TRY(hipMemcpyAsync(e->d_cnt[k], h, e->cnt_bytes, hipMemcpyHostToDevice, st));
    HIP_TRY(hipEventRecord(e->ev[k], st));
    e->ev_used[k] = true;
  }
  a.cnt = e->d_cnt[k];
  const int tk = timing_mark(e, st);
  rc = launch_fused(e, a, st);
  if (tk >= 0) (void)hipEventRecord(e->t_ev[2 * tk + 1], st);
  if (rc) return fail(CET_E_HIP, std::string("informer launch failed: ") + hipGetErrorString(hipGetLastError()));
  return finish_nmse();
}

int cet_set_stamps(cet_engine* e, uint64_t* stamps_dev) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  e->stamps = reinterpret_cast<unsigned long long*>(stamps_dev);
  return CET_OK;
}

int cet_set_precision(cet_engine* e, int prec) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  if (e->kind != 0) return fail(CET_E_INVALID, "precision modes are Informer-engine only");
  if (prec < -1 || prec > 4 || prec == 3)
    return fail(CET_E_INVALID, "precision must be -1 (auto), 0 (bf16), 1 (split bf16), 2 (fp8) or 4 (bf16 encoder, "
                               "split-bf16 decoder)");
  if (e->generic && prec != -1 && prec != 0)
    return fail(CET_E_INVALID, "the layer-wise engine (shapes outside the fused kernels) computes in fp32, or in bf16 "
                               "operands in its fused form");
  e->prec_req = prec;
  e->dirty = true;
  return CET_OK;
}

int cet_get_precision(cet_engine* e) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  if (e->kind != 0) return 0;
  const int rc = finalize_host(e);
  if (rc) return rc;
  return e->prec;
}

int cet_set_sampler(cet_engine* e, int on_host) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  if (on_host != 0 && on_host != 1) return fail(CET_E_INVALID, "on_host must be 0 or 1");
  e->host_sampler = on_host != 0;
  return CET_OK;
}

int cet_set_variant(cet_engine* e, int variant) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  if (variant != 4)
    return fail(CET_E_INVALID, "variant must be 4 (one sequence per workgroup); 1-3 and 5 are retired");
  e->variant = variant;
  return CET_OK;
}

int cet_last_path(cet_engine* e) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  return e->last_path;
}

int cet_last_kernel(cet_engine* e, char* name, int buflen) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  if (name && buflen > 0) std::snprintf(name, buflen, "%s", e->last_kernel.c_str());
  return (int)e->last_kernel.size();
}

int cet_timing(cet_engine* e, int enable) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  e->timing = enable != 0;
  e->timing_every = enable > 1 ? enable : 1;
  e->timing_seen = 0;
  e->t_n = 0;
  return CET_OK;
}

int cet_timing_read(cet_engine* e, double* total_ms, int64_t* launches) {
  if (!e) return fail(CET_E_INVALID, "null engine");
  double tot = 0.0;
  for (size_t k = 0; k < e->t_n; ++k) {
    HIP_TRY(hipEventSynchronize(e->t_ev[2 * k + 1]));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, e->t_ev[2 * k], e->t_ev[2 * k + 1]));
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = (int64_t)e->t_n;
  return CET_OK;
}

int cet_nmse_split(const float* pred, const float* label, int B, int T, int F, float* out, int accumulate,
                   void* stream) {
  if (!pred || !label || !out) return fail(CET_E_INVALID, "null argument");
  if (B <= 0 || T <= 0 || F <= 0 || T > 1024) return fail(CET_E_INVALID, "bad shape");
  int rc = cet_launch_nmse_split(pred, label, B, T, F, out, nullptr, accumulate, nullptr, (hipStream_t)stream);
  if (rc) return fail(CET_E_HIP, "nmse launch failed");
  return CET_OK;
}

int cet_nmse_split_sums(const float* pred, const float* label, int B, int T, int F, float* out, int accumulate,
                        double* sums, void* stream) {
  if (!pred || !label || (!out && !sums)) return fail(CET_E_INVALID, "null argument");
  if (B <= 0 || T <= 0 || F <= 0 || T > 1024) return fail(CET_E_INVALID, "bad shape");
  int rc = cet_launch_nmse_split(pred, label, B, T, F, out, nullptr, accumulate, sums, (hipStream_t)stream);
  if (rc) return fail(CET_E_HIP, "nmse launch failed");
  return CET_OK;
}

int cet_prepare_batch(const float* dataset, int64_t n_samples, int slots, int nr, int nt, const int32_t* sample_idx,
                      int64_t sample_base, const int32_t* start, const float* noise, uint64_t seed, uint64_t counter,
                      int B, int seq_len, int label_len, int pred_len, double snr_db, float* x_enc, float* x_dec,
                      float* label, int32_t* start_out, void* stream) {
  if (!dataset || !x_enc) return fail(CET_E_INVALID, "null argument");
  if (B < 0 || n_samples <= 0 || nr <= 0 || nt <= 0 || nr * nt > 64) return fail(CET_E_INVALID, "bad shape");
  if (seq_len <= 0 || pred_len < 0 || label_len < 0 || label_len > seq_len || slots < seq_len + pred_len)
    return fail(CET_E_INVALID, "window does not fit: need label_len <= seq_len and seq_len + pred_len <= slots");
  if (!sample_idx && (sample_base < 0 || sample_base + B > n_samples))
    return fail(CET_E_INVALID, "sample range outside the dataset");
  if ((int64_t)slots * nr * nt > (1ll << 30)) return fail(CET_E_INVALID, "sample too large");
  if (B == 0) return CET_OK;
  PrepArgs a;
  a.dataset = reinterpret_cast<const float2*>(dataset);
  a.n_samples = n_samples;
  a.slots = slots;
  a.E = nr * nt;
  a.sample_idx = sample_idx;
  a.sample_base = sample_base;
  a.start = start;
  a.noise = reinterpret_cast<const float2*>(noise);
  a.seed = seed;
  a.counter = counter;
  a.B = B;
  a.seq_len = seq_len;
  a.label_len = label_len;
  a.pred_len = pred_len;
  a.noise_scale = (float)std::sqrt(std::pow(10.0, -snr_db / 10.0) / 2.0);   // np.sqrt(sigma / 2) → complex64
  a.x_enc = x_enc;
  a.x_dec = x_dec;
  a.label = label;
  a.start_out = start_out;
  if (cet_launch_prepare_batch(&a, (hipStream_t)stream)) return fail(CET_E_HIP, "prepare_batch launch failed");
  return CET_OK;
}

int cet_synth_channels(const float* alpha, const float* phi, const float* gain, int n, int slots, int nr, int nt,
                       int paths, double doppler, float* out, void* stream) {
  if (!alpha || !phi || !gain || !out) return fail(CET_E_INVALID, "null argument");
  if (n < 0 || slots <= 0 || nr <= 0 || nt <= 0 || paths <= 0 || nr * nt > 64) return fail(CET_E_INVALID, "bad shape");
  if (n == 0) return CET_OK;
  SynthArgs a;
  a.alpha = alpha;
  a.phi = phi;
  a.gain = reinterpret_cast<const float2*>(gain);
  a.n = n;
  a.slots = slots;
  a.E = nr * nt;
  a.paths = paths;
  a.doppler = (float)doppler;
  a.out = reinterpret_cast<float2*>(out);
  if (cet_launch_synth(&a, (hipStream_t)stream)) return fail(CET_E_HIP, "synth launch failed");
  return CET_OK;
}

}  // extern "C"
