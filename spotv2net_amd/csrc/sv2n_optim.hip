// Adam over one flat parameter buffer (the reference optimiser,
// 5_train_SpotV2Net.py:127 torch.optim.Adam(lr), amsgrad=False).
//
// All trainable parameters of the model are views of one flat fp32 buffer
// (spotv2net_amd.train), so one launch updates every parameter: 7 fp32
// streams of 4 B per parameter (read p, g, m, v; write p, m, v).  The step
// counter lives on the device (graph-capturable); the caller increments it
// before the launch, exactly like torch's capturable Adam.
//   m = β1 m + (1-β1) g ;  v = β2 v + (1-β2) g²
//   p -= lr/(1-β1^t) · m / (sqrt(v)/sqrt(1-β2^t) + eps)
#include "sv2n_common.h"

namespace sv2n {

__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, const float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v,
                                              int64_t n, const float* __restrict__ step, float lr,
                                              float b1, float b2, float eps, float wd) {
  const float t = *step;
  const float bc1 = 1.f - powf(b1, t);
  const float bc2 = 1.f - powf(b2, t);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 mv = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* pp = &pv.x;
    float* gp = &gv.x;
    float* mp = &mv.x;
    float* vp = &vv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = gp[k];
      if (wd != 0.f) gk = fmaf(wd, pp[k], gk);
      mp[k] = fmaf(b1, mp[k] - gk, gk);           // lerp(m, g, 1-b1)
      vp[k] = fmaf(b2, vp[k], (1.f - b2) * gk * gk);
      const float denom = sqrtf(vp[k]) / bc2s + eps;
      pp[k] = pp[k] - step_size * (mp[k] / denom);
    }
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(m)[i] = mv;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gk = g[i];
    if (wd != 0.f) gk = fmaf(wd, p[i], gk);
    m[i] = fmaf(b1, m[i] - gk, gk);
    v[i] = fmaf(b2, v[i], (1.f - b2) * gk * gk);
    p[i] = p[i] - step_size * (m[i] / (sqrtf(v[i]) / bc2s + eps));
  }
}

}  // namespace sv2n

using namespace sv2n;

extern "C" int sv2n_adam_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                             int64_t n, const float* step, float lr, float beta1, float beta2,
                             float eps, float weight_decay, hipStream_t stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || !step || n < 0) return SV2N_ERR_ARG;
  if (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) & 15)
    return SV2N_ERR_ALIGN;
  if (n == 0) return 0;
  const int64_t n4 = (n + 3) / 4;
  const int grid = (int)std::min<int64_t>(2048, (n4 + 255) / 256);
  hipLaunchKernelGGL(k_adam, dim3(grid), dim3(256), 0, stream, param, grad, exp_avg, exp_avg_sq,
                     n, step, lr, beta1, beta2, eps, weight_decay);
  return (int)hipGetLastError();
}
