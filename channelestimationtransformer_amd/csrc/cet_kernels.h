// Kernel argument blocks and launchers shared by the host runtime and the .hip units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cet_plan.hpp"

namespace cet {

constexpr int MAX_STAMPS = 128;

struct InformerArgs {
  const InformerPlan* plan;   // device copy of the plan
  const void* weights;        // packed bf16 fragment blob
  const float* params;        // fp32 blob: biases, scales, LN, positional tables
  const uint8_t* cnt;         // per-forward ProbSparse key multiplicities (host-built), or
  const uint32_t* mt_in;      // resident mt19937 state slot to replay the draws from, and
  uint32_t* mt_out;           //     the slot workgroup 0 writes the advanced state to
  uint8_t* cnt_next;          // where the first workgroup to finish writes the next forward's tables
  unsigned* ticket;           // finish counter for that election (the last finisher re-arms it)
  const float* x_enc;         // [B][seq_len][C]
  const float* x_dec;         // [B][dec_len][C]
  float* out;                 // [B][pred_len][c_out]
  float* attns;               // optional encoder attention maps
  float* dbg;                 // optional per-stage activation dump
  unsigned long long* stamps; // optional per-phase s_memtime stamps [B][CET_MAX_STAMPS] (diagnostics)
  int B;
  uint32_t wlo;               // v4 split-bf16: byte offset of the lo weight fragments in `weights`
  int lds_bytes;              // dynamic LDS of the launch (set by the launcher)
  // v4 fused NMSE_Split (FullPrecision/metrics.py:26-30) of (out, label) over the batch, or label = null
  const float* label;         // [B][pred_len][c_out] (c_out ≤ 16)
  float2* nmse_part;          // [B][pred_len] per-sequence (Σ(x−x̂)², Σx̂²), written write-through (sc1)
  float* nmse_acc;            // [pred_len] ratio, accumulated (+=) by the last workgroup, or null
  double* nmse_sums;          // [2][pred_len] global sums (overwritten) by the last workgroup, or null
  // v4 encoder split (stacks, no ProbSparse calls, small batches): workgroup (b, e) runs encoder e of
  // sequence b, publishes its rows of the stack output, and the last of a sequence's workgroups to finish
  // runs the decoder; the others exit
  int enc_split;              // 0 / 1
  uint64_t* enc_xchg;         // [B][S rows][row stride / 8] bf16 stack-output image rows
  unsigned* enc_count;        // [B] arrivals (the last arrival re-arms it)
  int stagger;                // experiment (CET_STAGGER=mask:units): workgroups with (b & mask) != 0 sleep units·64
                              // cycles at entry (-DCET_STAGGER builds only)
  int shape;                  // v4_shape of the plan (V4S_*): the bf16 production launch takes the instance with its
                              // encoder rows as compile-time constants
  int poison;                 // diagnostic (CET_LDS_POISON=1): every LDS byte NaN at entry, before anything is staged
  int feed;                   // the plan's decoder runs on the LDS-DMA weight feed (the FEED instances)
};

// Plans with a compile-time instance (cet_api.cpp plan_shape): C2's encoder (one encoder, rows 90 → 45 → 23 → 12,
// the first three distilling) and the TimingAnalysis stack (e_layers [4, 3]: that encoder plus one on the window
// x[:, -45:], rows 45 → 23 → 12; 24 stack rows, a decoder of at most 16 rows).
enum V4Shape { V4S_GENERIC = 0, V4S_C2 = 1, V4S_E43 = 2 };

// The v4 Informer instance a launch takes.  launch_v4 (cet_informer4.hpp) launches exactly this choice and
// the host reports it (cet_last_kernel), so the two agree by construction.  prec: 0 bf16, 1 split bf16, 2 fp8.
enum V4Instance { V4I_NONE = 0, V4I_GENERIC = 1, V4I_DIAG = 2, V4I_SHAPE = 3, V4I_SPLIT = 4, V4I_SHAPE_STAMPS = 5 };
__host__ __device__ inline int v4_instance(const InformerArgs& a, int prec, int dff) {
  const bool diag = a.attns || a.dbg || a.stamps;
  if (dff != 64 && dff != 128) return V4I_NONE;
  if (a.enc_split) return prec == 0 && !diag && (a.shape != V4S_E43 || dff == 64) ? V4I_SPLIT : V4I_NONE;
#ifdef CET_C2_STAMPS
  if (dff == 64 && a.shape != V4S_GENERIC && a.stamps && !a.attns && !a.dbg && prec == 0) return V4I_SHAPE_STAMPS;
#endif
  // compile-time rows: C2 for bf16 and fp8, E43 for bf16
  if (dff == 64 && !diag && ((a.shape == V4S_C2 && prec != 1) || (a.shape == V4S_E43 && prec == 0))) return V4I_SHAPE;
  if (prec == 4 && dff != 64) return V4I_NONE;   // the mixed instances exist for d_ff 64
  return diag ? V4I_DIAG : V4I_GENERIC;
}

// device channel pipeline (cet_data.hip)
struct PrepArgs {
  const float2* dataset;   // [n_samples][slots][E] complex64, E = Nr·Nt
  int64_t n_samples;
  int slots, E;
  const int32_t* sample_idx;   // [B] or null: sample = sample_base + b
  int64_t sample_base;
  const int32_t* start;        // [B] window starts or null: drawn on device
  const float2* noise;         // [B][slots][E] (re, im) standard normals, or null: device Philox
  uint64_t seed, counter;
  int B, seq_len, label_len, pred_len;
  float noise_scale;           // sqrt(sigma / 2) rounded to fp32, sigma = 10^(-SNR/10)
  float* x_enc;                // [B][seq_len][2E]
  float* x_dec;                // [B][label_len + pred_len][2E] or null
  float* label;                // [B][pred_len][2E] or null
  int32_t* start_out;          // [B] the windows used, or null
};

struct SynthArgs {
  const float* alpha;
  const float* phi;
  const float2* gain;
  int n, slots, E, paths;
  float doppler;
  float2* out;   // [n][slots][E]
};

struct TransformerArgs {
  const TransformerPlan* plan;
  const void* weights;
  const float* params;
  const float* x_enc;
  const float* x_dec;
  float* out;
  float* dbg;
  int B;
  int c3;   // the plan is C3's (src_len 90, tgt_len 15): the production launch takes the instance with those
            // lengths at compile time
  int poison;      // diagnostic (CET_LDS_POISON=1): every LDS byte NaN at entry
  int lds_bytes;   // dynamic LDS of the launch (set by the launcher)
};

// hipFuncSetAttribute(MaxDynamicSharedMemorySize, 160 KiB) for `kern` on the CURRENT device,
// once per (device, kernel); thread-safe (cet_api.cpp).  Returns false if the runtime refuses.
bool ensure_lds_attr(const void* kern);

}  // namespace cet

extern "C" int cet_launch_sampler_prep(const cet::InformerPlan* plan, const uint32_t* mt_in, uint32_t* mt_out,
                                       uint8_t* tab_out, int lds_bytes, hipStream_t stream);
extern "C" int cet_launch_informer_v4(const cet::InformerArgs* a, int prec, int dff, int lds_bytes, hipStream_t stream);
extern "C" int cet_launch_prepare_batch(const void* args, hipStream_t stream);
extern "C" int cet_launch_synth(const void* args, hipStream_t stream);
extern "C" int cet_launch_transformer_v4(const cet::TransformerArgs* a, int dff, int lds_bytes, hipStream_t stream);
extern "C" int cet_launch_nmse_split(const float* pred, const float* label, int B, int T, int F, float* acc,
                                     float* last, int accumulate, double* sums, hipStream_t stream);
