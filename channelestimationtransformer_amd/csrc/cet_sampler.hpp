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

static_assert(MT_WORDS == REPLAY_STATE_WORDS, "replay_fast_lds() assumes the padded state slot");

// Per-call replay (any plan): the calls in stream order, each one twisting as it goes.
template <int NT>
__device__ __forceinline__ void replay_all_calls(const InformerPlan& pl, const uint32_t* __restrict__ mt_in,
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
      for (int i = tid_op(); i < n16; i += NT) dst[i] = src[i];
      __syncthreads();   // the next call zeroes the LDS table
    }
  }
  mt_store<NT>(g, mt_out);
}

// Whole-forward replay in three workgroup-wide passes (needs replay_fast_lds bytes at `lds`):
//   1. the forward's pl.draws words of the stream, tempered, into LDS (the twists are the only
//      serial part), while the tables are zeroed;
//   2. every draw of every sparse call into its table at once (LDS packed-byte atomics; the
//      calls' tables are disjoint, so no barrier between calls);
//   3. one coalesced copy of all tables, and the advanced state, to global memory.
template <int NT>
__device__ __forceinline__ void replay_all_fast(const InformerPlan& pl, const uint32_t* __restrict__ mt_in,
                                                uint32_t* __restrict__ mt_out, uint8_t* __restrict__ tab_out,
                                                char* lds) {
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  uint32_t* st = reinterpret_cast<uint32_t*>(lds);
  uint32_t* words = st + MT_WORDS;
  uint32_t* tabs = words + ((pl.draws + 3) & ~3);
  const int tab16 = (int)pl.cnt_bytes / 16;
  for (int i = tid_op(); i < tab16; i += NT) reinterpret_cast<u32x4*>(tabs)[i] = u32x4{0u, 0u, 0u, 0u};
  MTState g{st, MT_N};
  mt_load<NT>(g, mt_in);
  const int total = pl.draws;
  int have = 0;
  while (have < total) {
    if (g.idx >= MT_N) {
      mt_twist<NT>(g.st);   // barriers on both sides: the previous block's readers are done
      g.idx = 0;
    }
    const int take = min(MT_N - g.idx, total - have);
    for (int t = tid_op(); t < take; t += NT) words[have + t] = mt_temper(g.st[g.idx + t]);
    have += take;
    g.idx += take;
  }
  __syncthreads();
  int base = 0;
  for (int c = 0; c < pl.n_calls; ++c) {
    const AttnCall& ac = pl.calls[c];
    const int n = ac.LQ * ac.U;
    if (ac.u < ac.LQ) {
      const float invU = 1.0f / (float)ac.U;
      uint32_t* tab = tabs + ac.cnt_off / 4;
      for (int d = tid_op(); d < n; d += NT) {
        const uint32_t key = words[base + d] % (uint32_t)ac.LK;
        const int q = (int)(((float)d + 0.5f) * invU);   // exact: d < 96·96, U ≤ 96
        atomicAdd(&tab[(q * ac.cnt_stride + cnt_word_off((int)key)) >> 2], 1u << ((key & 3u) * 8u));
      }
    }
    base += n;
  }
  __syncthreads();
  for (int i = tid_op(); i < tab16; i += NT)
    reinterpret_cast<u32x4*>(tab_out)[i] = reinterpret_cast<const u32x4*>(tabs)[i];
  mt_store<NT>(g, mt_out);
}

// One forward's tables from the resident state: the three-pass replay when `lds_avail` bytes of
// LDS hold it, else call by call.
template <int NT>
__device__ __forceinline__ void replay_all(const InformerPlan& pl, const uint32_t* __restrict__ mt_in,
                                           uint32_t* __restrict__ mt_out, uint8_t* __restrict__ tab_out,
                                           char* lds, int lds_avail, uint32_t* st_lds, uint32_t* tab_lds) {
  if (replay_fast_lds(pl) <= lds_avail)
    replay_all_fast<NT>(pl, mt_in, mt_out, tab_out, lds);
  else
    replay_all_calls<NT>(pl, mt_in, mt_out, tab_out, st_lds, tab_lds);
}

}  // namespace cet
