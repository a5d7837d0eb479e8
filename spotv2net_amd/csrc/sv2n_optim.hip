// Adam over one flat parameter buffer (the reference optimiser,
// 5_train_SpotV2Net.py:127 torch.optim.Adam(lr), amsgrad=False).
//
// All trainable parameters of the model are views of one flat fp32 buffer
// (spotv2net_amd.train), so one launch updates every parameter: 7 fp32
// streams of 4 B per parameter (read p, g, m, v; write p, m, v).  The step
// counter lives on the device (graph-capturable): sv2n_adam_f32 expects it
// already incremented (like torch's capturable Adam), sv2n_adam_f32_step
// increments it in-kernel and zeroes the consumed gradient.
//   m = β1 m + (1-β1) g ;  v = β2 v + (1-β2) g²
//   p -= lr/(1-β1^t) · m / (sqrt(v)/sqrt(1-β2^t) + eps)
#include "sv2n_common.h"

namespace sv2n {

// STEP: the kernel advances the device step counter itself (t = *step + 1,
// written back by the last-arriving block, cnt = ticket counter) and zeroes
// the gradient it consumed, so a training step needs no separate increment
// or grad-zeroing launch.
template <bool STEP>
__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v,
                                              int64_t n, float* __restrict__ step, float lr,
                                              float b1, float b2, float eps, float wd,
                                              unsigned* __restrict__ cnt) {
  __shared__ int s_flag;
  const float t = STEP ? *step + 1.f : *step;
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
    if (STEP) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gk = g[i];
    if (wd != 0.f) gk = fmaf(wd, p[i], gk);
    m[i] = fmaf(b1, m[i] - gk, gk);
    v[i] = fmaf(b2, v[i], (1.f - b2) * gk * gk);
    p[i] = p[i] - step_size * (m[i] / (sqrtf(v[i]) / bc2s + eps));
    if (STEP) g[i] = 0.f;
  }
  // every block read *step at its start; once all have taken a ticket the
  // last one may advance it (nothing else is handed over: no fences)
  if (STEP && last_block_ticket2(cnt, gridDim.x, &s_flag) && threadIdx.x == 0) *step = t;
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
  hipLaunchKernelGGL(k_adam<false>, dim3(grid), dim3(256), 0, stream, param,
                     const_cast<float*>(grad), exp_avg, exp_avg_sq, n, const_cast<float*>(step),
                     lr, beta1, beta2, eps, weight_decay, nullptr);
  return (int)hipGetLastError();
}

extern "C" int sv2n_adam_f32_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq,
                                  int64_t n, float* step, uint32_t* counter, float lr,
                                  float beta1, float beta2, float eps, float weight_decay,
                                  hipStream_t stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || !step || !counter || n < 0)
    return SV2N_ERR_ARG;
  if (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) & 15)
    return SV2N_ERR_ALIGN;
  if (n == 0) return 0;
  const int64_t n4 = (n + 3) / 4;
  // the step counter's ticket is two-level (~grid/8 + 8 serialised atomics),
  // so the grid may exceed one block per CU: MI355X, round 6 (same box), C3
  // loop 469.7 / 469.9 K windows/s at 256 blocks, 471.9 / 473.3 K at 1,024,
  // 474.6 K at 2,048; C2's Adam 8.0 -> 7.8 us
#ifndef SV2N_ADAM_GRID
#define SV2N_ADAM_GRID 1024
#endif
  const int grid = (int)std::min<int64_t>(SV2N_ADAM_GRID, (n4 + 255) / 256);
  hipLaunchKernelGGL(k_adam<true>, dim3(grid), dim3(256), 0, stream, param, grad, exp_avg,
                     exp_avg_sq, n, step, lr, beta1, beta2, eps, weight_decay, counter);
  return (int)hipGetLastError();
}
