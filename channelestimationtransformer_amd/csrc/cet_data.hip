// Device-side channel pipeline: the per-sample work of
// FullPrecision/dataset.py SeqData.__getitem__ (:124-152) — channelnorm (:77-88), complex AWGN
// (:54-74), the seq_len + pred_len window — followed by LoadBatch (:20-44) and the callers'
// decoder input (QuantizationAwareTraining.py:97-114), for a whole batch in one launch, straight
// from a device-resident dataset.  Plus a seeded sum-of-sinusoids (Jakes) channel source that
// stands in for the reference's absent CDL pickles.
//
// HBM-bound byte work: one workgroup per sample reads the sample once per pass (the two power
// means need the whole sample), writes x_enc / x_dec / label.  No LDS staging — the sample
// (≤ 32 KB) stays L2-resident between the passes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cet_kernels.h"

namespace cet {
namespace data {

constexpr int NT = 256;

// ------------------------------------------------------------------ Philox4x32-10 normals
struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0, h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    c = U4{h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Two standard normals from two uniforms (Box–Muller); u1 ∈ (0, 1].
__device__ __forceinline__ float2 box_muller(uint32_t a, uint32_t b) {
  const float u1 = ((float)a + 1.0f) * 2.3283064365386963e-10f;
  const float u2 = (float)b * 2.3283064365386963e-10f;
  const float r = sqrtf(-2.0f * logf(u1));
  float s, c;
  sincosf(6.283185307179586f * u2, &s, &c);
  return make_float2(r * c, r * s);
}

// Standard-normal pair for complex element e of sample (b) in batch `counter`: the real part and
// the imaginary part (torch.randn twice over the sample shape, dataset.py:65-66).
__device__ __forceinline__ float2 normal_pair(uint64_t seed, uint64_t counter, int b, int e) {
  const U4 r = philox4x32_10(U4{(uint32_t)e, (uint32_t)b, (uint32_t)counter, (uint32_t)(counter >> 32)},
                             (uint32_t)seed, (uint32_t)(seed >> 32));
  return box_muller(r.x, r.y);
}

__device__ __forceinline__ uint32_t uniform_u32(uint64_t seed, uint64_t counter, int b) {
  const U4 r = philox4x32_10(U4{0xFFFFFFFFu, (uint32_t)b, (uint32_t)counter, (uint32_t)(counter >> 32)},
                             (uint32_t)seed ^ 0x5bd1e995u, (uint32_t)(seed >> 32));
  return r.x;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) s += red[w];
  return s;
}

__global__ void __launch_bounds__(NT) prepare_batch_kernel(cet::PrepArgs a) {
  __shared__ float red[NT / 64];
  const int b = blockIdx.x;
  if (b >= a.B) return;
  const int64_t s = a.sample_idx ? (int64_t)a.sample_idx[b] : a.sample_base + b;
  const int n = a.slots * a.E, L = a.seq_len + a.pred_len;
  const float2* H = a.dataset + s * n;
  // window start: np.random.randint(0, slots - L + 1) (dataset.py:142)
  int st;
  if (a.start) st = a.start[b];
  else st = (int)(uniform_u32(a.seed, a.counter, b) % (uint32_t)(a.slots - L + 1));
  if (a.start_out && threadIdx.x == 0) a.start_out[b] = st;
  const int F = 2 * a.E, Ld = a.label_len + a.pred_len;
  float* xe = a.x_enc + (size_t)b * a.seq_len * F;
  float* xd = a.x_dec ? a.x_dec + (size_t)b * Ld * F : nullptr;
  float* lb = a.label ? a.label + (size_t)b * a.pred_len * F : nullptr;
  if (s < 0 || s >= a.n_samples || st < 0 || st > a.slots - L) {
    // never read outside the dataset: the sample's rows become NaN
    const float qnan = __uint_as_float(0x7fc00000u);
    for (int i = threadIdx.x; i < a.seq_len * F; i += NT) xe[i] = qnan;
    if (xd) for (int i = threadIdx.x; i < Ld * F; i += NT) xd[i] = qnan;
    if (lb) for (int i = threadIdx.x; i < a.pred_len * F; i += NT) lb[i] = qnan;
    return;
  }

  // channelnorm: H / sqrt(mean |H|^2) over the whole sample
  float p = 0.f;
  for (int i = threadIdx.x; i < n; i += NT) {
    const float2 h = H[i];
    p = fmaf(h.x, h.x, fmaf(h.y, h.y, p));
  }
  const float rms = sqrtf(block_sum(p, red) / (float)n);
  // noise(): n = sqrt(sigma/2)·(re + j·im)·sqrt(mean |Hn|^2), Hn the normalised sample
  float p2 = 0.f;
  for (int i = threadIdx.x; i < n; i += NT) {
    const float2 h = H[i];
    const float x = h.x / rms, y = h.y / rms;
    p2 = fmaf(x, x, fmaf(y, y, p2));
  }
  const float nrm = sqrtf(block_sum(p2, red) / (float)n);
  for (int i = threadIdx.x; i < L * a.E; i += NT) {
    const int t = i / a.E, e = i - t * a.E;
    const int src = (st + t) * a.E + e;
    const float2 h = H[src];
    const float x = h.x / rms, y = h.y / rms;
    if (t < a.seq_len) {
      // H_seq = H_noise[window][:seq_len] → LoadBatch interleave f = 2e + {re, im}
      float2 z;
      if (a.noise) z = a.noise[(size_t)b * n + src];
      else z = normal_pair(a.seed, a.counter, b, src);
      const float nx = (a.noise_scale * z.x) * nrm, ny = (a.noise_scale * z.y) * nrm;
      const float2 v = make_float2(x + nx, y + ny);
      *reinterpret_cast<float2*>(xe + t * F + 2 * e) = v;
      // decoder input: encoder rows seq_len - label_len .. seq_len, then pred_len zero rows
      const int td = t - (a.seq_len - a.label_len);
      if (xd && td >= 0) *reinterpret_cast<float2*>(xd + td * F + 2 * e) = v;
    } else {
      // H_pred = clean H[window][seq_len:]
      const int k = t - a.seq_len;
      if (lb) *reinterpret_cast<float2*>(lb + k * F + 2 * e) = make_float2(x, y);
      if (xd) *reinterpret_cast<float2*>(xd + (a.label_len + k) * F + 2 * e) = make_float2(0.f, 0.f);
    }
  }
}

// ------------------------------------------------------------------ Jakes channel source
// H[s][t][r·Nt + a] = Σ_p g_p·exp(j(2π·doppler·cos(α_p)·t + φ_p)) / sqrt(P), then unit mean
// power per sample.  Parameters [n][E][P] (α, φ) and [n][E][P] complex gains (SynthArgs).
__global__ void __launch_bounds__(NT) synth_kernel(cet::SynthArgs a) {
  __shared__ float red[NT / 64];
  const int s = blockIdx.x;
  if (s >= a.n) return;
  const int n = a.slots * a.E;
  float2* H = a.out + (size_t)s * n;
  const float inv_sqrt_p = rsqrtf((float)a.paths);
  float p = 0.f;
  for (int i = threadIdx.x; i < n; i += NT) {
    const int t = i / a.E, e = i - t * a.E;
    const size_t base = ((size_t)s * a.E + e) * a.paths;
    float re = 0.f, im = 0.f;
    for (int q = 0; q < a.paths; ++q) {
      const float ph = 6.283185307179586f * a.doppler * cosf(a.alpha[base + q]) * (float)t + a.phi[base + q];
      float sn, cs;
      sincosf(ph, &sn, &cs);
      const float2 g = a.gain[base + q];
      re += g.x * cs - g.y * sn;
      im += g.x * sn + g.y * cs;
    }
    re *= inv_sqrt_p;
    im *= inv_sqrt_p;
    H[i] = make_float2(re, im);
    p = fmaf(re, re, fmaf(im, im, p));
  }
  const float inv = rsqrtf(block_sum(p, red) / (float)n);
  for (int i = threadIdx.x; i < n; i += NT) {
    const float2 h = H[i];
    H[i] = make_float2(h.x * inv, h.y * inv);
  }
}

}  // namespace data
}  // namespace cet

extern "C" int cet_launch_prepare_batch(const void* args, hipStream_t stream) {
  const auto& a = *static_cast<const cet::PrepArgs*>(args);
  if (a.B <= 0) return 0;
  hipLaunchKernelGGL(cet::data::prepare_batch_kernel, dim3(a.B), dim3(cet::data::NT), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int cet_launch_synth(const void* args, hipStream_t stream) {
  const auto& a = *static_cast<const cet::SynthArgs*>(args);
  if (a.n <= 0) return 0;
  hipLaunchKernelGGL(cet::data::synth_kernel, dim3(a.n), dim3(cet::data::NT), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
