// Dropout uniforms from a counter-based generator, for the captured training
// step (spotv2net_amd.train.TrainStep).  The reference draws its post-layer
// dropout mask with torch's generator (F.dropout, reference
// utils/models.py:148); a hipGraph that captures a torch random op makes every
// replay launch two generator-state fills before the graph, and the draw is a
// launch of its own.  Here the uniforms are a pure function of
//   (seed, step, salt, element index)
// on Philox4x32-10 (Salmon et al., SC'11: the counter/key schedule cuRAND and
// torch use): key = seed, counter = (i/4 low, i/4 high, salt, step); element
// i takes word i%4 of its counter's block, u = (word >> 8)·2^-24 in [0, 1).
// `step` is read from device memory (the optimizer's step count, advanced by
// the captured Adam launch), so each replay draws fresh masks with no host
// work and nothing to reset; `salt` separates the draws of one step.
#include "sv2n_common.h"

namespace sv2n {

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ float word_uniform(uint32_t w) {
  return (float)(w >> 8) * (1.0f / 16777216.0f);
}

// one counter block (4 elements) per thread, grid-stride
__global__ __launch_bounds__(256) void k_dropout_uniform(float* __restrict__ u, int64_t n,
                                                         uint32_t k0, uint32_t k1,
                                                         const float* __restrict__ step,
                                                         uint32_t salt) {
  const uint32_t st = (uint32_t)*step;
  const int64_t nb = (n + 3) >> 2;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb;
       b += (int64_t)gridDim.x * blockDim.x) {
    const uint4 w = philox4x32_10(make_uint4((uint32_t)b, (uint32_t)(b >> 32), salt, st), k0, k1);
    const int64_t i = b << 2;
    if (i + 4 <= n) {
      *reinterpret_cast<float4*>(u + i) =
          make_float4(word_uniform(w.x), word_uniform(w.y), word_uniform(w.z), word_uniform(w.w));
    } else {
      const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
      for (int q = 0; i + q < n; ++q) u[i + q] = word_uniform(ws[q]);
    }
  }
}

}  // namespace sv2n

using namespace sv2n;

extern "C" int sv2n_dropout_uniform(float* u, int64_t n, uint64_t seed, const float* step,
                                    uint32_t salt, hipStream_t stream) {
  if (!u || !step || n < 0) return SV2N_ERR_ARG;
  if ((uintptr_t)u & 15) return SV2N_ERR_ALIGN;
  if (n == 0) return 0;
  const int64_t nb = (n + 3) / 4;
  const int grid = (int)std::min<int64_t>(4096, (nb + 255) / 256);
  hipLaunchKernelGGL(k_dropout_uniform, dim3(grid), dim3(256), 0, stream, u, n, (uint32_t)seed,
                     (uint32_t)(seed >> 32), step, salt);
  return (int)hipGetLastError();
}
