// Device-resident ProbSparse index sampler: the torch CPU generator's mt19937 stream, regenerated
// by every workgroup in LDS, so a forward needs no host draw and no host→device copy.
//
// The reference draws ``torch.randint(L_K, (L_Q, sample_k))`` once per ProbAttention call
// (FullPrecision/InformerModel/attn.py:57-60) from the global CPU generator: 32-bit mt19937
// outputs reduced ``% L_K``, consumed in call order.  The state (624 words + read index) lives in
// HBM in two ping-pong slots; every workgroup of a forward reads slot ``in``, replays the draws of
// each call into its LDS key-multiplicity table, and workgroup 0 stores the advanced state into
// slot ``out`` for the next forward.  The host mirror of the same generator is cet_api.cpp MT19937.
#pragma once
#include "cet_device.hpp"

namespace cet {

constexpr int MT_N = 624;
constexpr int MT_WORDS = 640;   // state + read index, padded (one HBM slot)

struct MTState {
  uint32_t* st;   // LDS copy of the 624-word state
  int idx;        // next word to temper (uniform across the workgroup); 624 = twist first
};

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// Twist with thread t owning words t, t+227 and t+454.  Sequentially, word i reads word i+1 while
// it is still old (except 623, which reads the new word 0) and word (i+397) mod 624, which is old
// for i < 227 and otherwise the word 227 places below, rewritten earlier in the same twist: for
// t+227 that is word t and for t+454 word t+227, both this thread's own results.  So all old
// words are read first and the update needs no exchange between threads.
__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt, uint32_t far) {
  const uint32_t y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
  return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

template <int NT>
__device__ __forceinline__ void mt_twist(uint32_t* st) {
  static_assert(NT >= 227, "one word per thread per third");
  const int t = tid_op();
  __syncthreads();   // every reader of the previous block is done
  uint32_t n0 = 0, n1 = 0, n2 = 0;
  if (t < 227) {
    n0 = mt_mix(st[t], st[t + 1], st[t + 397]);
    n1 = mt_mix(st[t + 227], st[t + 228], n0);
    if (t < 169) {
      n2 = mt_mix(st[t + 454], st[t + 455], n1);
    } else if (t == 169) {   // word 623 reads the new word 0
      const uint32_t w0 = mt_mix(st[0], st[1], st[397]);
      n2 = mt_mix(st[623], w0, n1);
    }
  }
  __syncthreads();
  if (t < 227) {
    st[t] = n0;
    st[t + 227] = n1;
    if (t < 170) st[t + 454] = n2;
  }
  __syncthreads();
}

// Replay one call's L_Q·U draws.  With ``tab`` (LDS, rows of ``stride`` bytes, zeroed here) each
// draw (q, key) increments tab[q][key]; without it the stream is only advanced (calls whose u ≥ L_Q
// attend over every query, but the reference still draws their samples).
template <int NT>
__device__ __forceinline__ void mt_replay(MTState& g, int LQ, int U, int LK, uint32_t* tab, int stride) {
  if (tab) {
    const int words = ((LQ + 15) & ~15) * stride / 4;
    for (int i = tid_op(); i < words; i += NT) tab[i] = 0u;
    __syncthreads();
  }
  const int n = LQ * U;
  const float invU = 1.0f / (float)U;
  int done = 0;
  while (done < n) {
    if (g.idx >= MT_N) {
      mt_twist<NT>(g.st);
      g.idx = 0;
    }
    const int take = min(MT_N - g.idx, n - done);
    if (tab) {
      for (int t = tid_op(); t < take; t += NT) {
        const uint32_t key = mt_temper(g.st[g.idx + t]) % (uint32_t)LK;
        const int q = (int)(((float)(done + t) + 0.5f) * invU);   // exact: p < 96·96, U ≤ 96
        atomicAdd(&tab[(q * stride + cnt_word_off((int)key)) >> 2], 1u << ((key & 3u) * 8u));   // counts ≤ U < 256
      }
    }
    done += take;
    g.idx += take;
  }
  __syncthreads();
}

template <int NT>
__device__ __forceinline__ void mt_load(MTState& g, const uint32_t* __restrict__ src) {
  for (int i = tid_op(); i < MT_N; i += NT) g.st[i] = src[i];
  g.idx = (int)src[MT_N];
  __syncthreads();
}

template <int NT>
__device__ __forceinline__ void mt_store(const MTState& g, uint32_t* __restrict__ dst) {
  for (int i = tid_op(); i < MT_N; i += NT) dst[i] = g.st[i];
  if (threadIdx.x == 0) dst[MT_N] = (uint32_t)g.idx;
}

}  // namespace cet
