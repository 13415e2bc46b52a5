// NMSE_Split_cuda (FullPrecision/metrics.py:26-30): per prediction step t,
//   Σ_{b,f} (x − x̂)² / Σ_{b,f} x̂²   with x̂ = pred (the FIRST argument, as run_validation
// passes the model output first, QuantizationAwareTraining.py:122).  One workgroup per step,
// fp64 accumulation, optional running sum (the caller's `loss += ...`).
#include <hip/hip_runtime.h>

#include "cet_kernels.h"

namespace cet {

__global__ void __launch_bounds__(256) nmse_split_kernel(const float* __restrict__ pred, const float* __restrict__ label,
                                                         int B, int T, int F, float* out, float* last, int accumulate) {
  __shared__ double sm[2][4];
  const int t = blockIdx.x;
  double mse = 0.0, pw = 0.0;
  for (int i = threadIdx.x; i < B * F; i += blockDim.x) {
    const int b = i / F, f = i - b * F;
    const size_t o = ((size_t)b * T + t) * F + f;
    const double xh = pred[o], x = label[o];
    mse += (x - xh) * (x - xh);
    pw += xh * xh;
  }
  for (int m = 32; m >= 1; m >>= 1) {
    mse += __shfl_xor(mse, m, 64);
    pw += __shfl_xor(pw, m, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    sm[0][threadIdx.x >> 6] = mse;
    sm[1][threadIdx.x >> 6] = pw;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, p = 0.0;
    for (int w = 0; w < 4; ++w) { a += sm[0][w]; p += sm[1][w]; }
    const float r = (float)(a / p);
    out[t] = accumulate ? out[t] + r : r;
    if (last) last[t] = r;
  }
}

}  // namespace cet

extern "C" int cet_launch_nmse_split(const float* pred, const float* label, int B, int T, int F, float* acc,
                                     float* last, int accumulate, hipStream_t stream) {
  hipLaunchKernelGGL(cet::nmse_split_kernel, dim3(T), dim3(256), 0, stream, pred, label, B, T, F, acc, last,
                     accumulate);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
