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
  const uint32_t* mt_in;      // v2: resident mt19937 state slot to replay the draws from, and
  uint32_t* mt_out;           //     the slot workgroup 0 writes the advanced state to
  const float* x_enc;         // [B][seq_len][C]
  const float* x_dec;         // [B][dec_len][C]
  float* out;                 // [B][pred_len][c_out]
  float* attns;               // optional encoder attention maps
  float* dbg;                 // optional per-stage activation dump
  unsigned long long* stamps; // optional per-phase s_memtime stamps [B][CET_MAX_STAMPS] (diagnostics)
  int B;
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
};

}  // namespace cet

extern "C" int cet_launch_informer(const cet::InformerArgs* a, int dff, int lds_bytes, hipStream_t stream);
extern "C" int cet_launch_informer_v2(const cet::InformerArgs* a, int dff, int lds_bytes, hipStream_t stream);
extern "C" int cet_launch_transformer(const cet::TransformerArgs* a, int dff, int lds_bytes, hipStream_t stream);
extern "C" int cet_launch_nmse_split(const float* pred, const float* label, int B, int T, int F, float* acc,
                                     float* last, int accumulate, hipStream_t stream);
