// One-workgroup launch that prepares a forward's ProbSparse multiplicity tables from the resident
// mt19937 state (cet_sampler.hpp replay_all): used for the first forward after a (re)seed; later
// forwards get their tables from the previous forward's first workgroup to finish.
// Reference: FullPrecision/InformerModel/attn.py:96-98 (torch.randint per ProbAttention call).
#include "cet_kernels.h"
#include "cet_sampler.hpp"

namespace cet {
constexpr int PREP_THREADS = 512;

__global__ void __launch_bounds__(PREP_THREADS) sampler_prep(const InformerPlan* plan, const uint32_t* mt_in,
                                                             uint32_t* mt_out, uint8_t* tab_out, int lds_bytes) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  replay_all<PREP_THREADS>(*plan, mt_in, mt_out, tab_out, lds, lds_bytes, reinterpret_cast<uint32_t*>(lds),
                           reinterpret_cast<uint32_t*>(lds + MT_WORDS * 4));
}
}  // namespace cet

extern "C" int cet_launch_sampler_prep(const cet::InformerPlan* plan, const uint32_t* mt_in, uint32_t* mt_out,
                                       uint8_t* tab_out, int lds_bytes, hipStream_t stream) {
  if (!cet::ensure_lds_attr(reinterpret_cast<const void*>(cet::sampler_prep))) return -1;
  hipLaunchKernelGGL(cet::sampler_prep, dim3(1), dim3(cet::PREP_THREADS), lds_bytes, stream, plan, mt_in, mt_out,
                     tab_out, lds_bytes);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
