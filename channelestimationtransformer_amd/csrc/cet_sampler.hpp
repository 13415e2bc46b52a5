// Whole-forward ProbSparse table preparation (v3 "prepared tables" mode).
//
// The reference draws torch.randint(L_K, (L_Q, sample_k)) once per ProbAttention call from the
// global CPU generator (FullPrecision/InformerModel/attn.py:96-98); every workgroup of a forward
// needs the same key-multiplicity tables.  replay_all() advances the resident mt19937 state
// (cet_mt.hpp) through all of one forward's calls in order and writes each sparse call's table to
// global memory in the v2/v3 row layout (cnt_pos_v2).  It runs in one workgroup: either the
// sampler-prep kernel (first forward after a reseed) or the FIRST workgroup of a forward to
// finish, which prepares the next forward's tables while the rest of the grid drains.
#pragma once
#include "cet_mt.hpp"

namespace cet {

template <int NT>
__device__ __forceinline__ void replay_all(const InformerPlan& pl, const uint32_t* __restrict__ mt_in,
                                           uint32_t* __restrict__ mt_out, uint8_t* __restrict__ tab_out,
                                           uint32_t* st_lds, uint32_t* tab_lds) {
  MTState g{st_lds, MT_N};
  mt_load<NT>(g, mt_in);
  for (int c = 0; c < pl.n_calls; ++c) {
    const AttnCall& ac = pl.calls[c];
    const bool sparse = ac.u < ac.LQ;
    mt_replay<NT>(g, ac.LQ, ac.U, ac.LK, sparse ? tab_lds : nullptr, ac.cnt_stride);
    if (sparse) {
      const int n16 = ((ac.LQ + 15) & ~15) * ac.cnt_stride / 16;
      typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
      const u32x4* src = reinterpret_cast<const u32x4*>(tab_lds);
      u32x4* dst = reinterpret_cast<u32x4*>(tab_out + ac.cnt_off);
      for (int i = threadIdx.x; i < n16; i += NT) dst[i] = src[i];
      __syncthreads();   // the next call zeroes the LDS table
    }
  }
  mt_store<NT>(g, mt_out);
}

}  // namespace cet
