// Output head of GATModel: the final nn.Linear(h_last, out_ch) (reference
// utils/models.py:120, applied at :150) as two small kernels instead of three
// library GEMM launches with a skinny N (out_ch is 1 in the reference config,
// 14 for the multi-output models).
//   forward   out[i][o] = Σ_c x[i][c] · W[o][c] + b[o]
//   backward  dx[i][c]  = Σ_o dout[i][o] · W[o][c]
//             gW[o][c] += Σ_i dout[i][o] · x[i][c],  gb[o] += Σ_i dout[i][o]
// The weight gradient is reduced per workgroup into partial slabs and summed in
// a fixed order (deterministic), then ACCUMULATED into the .grad buffers.
#include "sv2n_common.h"

namespace sv2n {

constexpr int HEAD_MAX_OUT = 16;
constexpr int HEAD_ROWS = 256;  // rows per workgroup (one per thread)

// x rows staged through LDS so the global reads are coalesced
template <int OUT>
__global__ __launch_bounds__(256) void k_head_fwd(const float* __restrict__ x, int64_t N, int C,
                                                  const float* __restrict__ W,
                                                  const float* __restrict__ b,
                                                  float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float sx[];  // [256][C+1]
  __shared__ float sw[HEAD_MAX_OUT * 128];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * HEAD_ROWS;
  const int nr = (int)min((int64_t)HEAD_ROWS, N - r0);
  const int CP = C + 1;
  for (int k = t; k < OUT * C; k += 256) sw[k] = W[k];
  for (int k = t; k < nr * C; k += 256) {
    const int r = k / C;
    sx[r * CP + (k - r * C)] = x[r0 * C + k];
  }
  __syncthreads();
  if (t < nr) {
    float acc[OUT];
#pragma unroll
    for (int o = 0; o < OUT; ++o) acc[o] = 0.f;
    for (int c = 0; c < C; ++c) {
      const float xv = sx[t * CP + c];
#pragma unroll
      for (int o = 0; o < OUT; ++o) acc[o] = fmaf(xv, sw[o * C + c], acc[o]);
    }
#pragma unroll
    for (int o = 0; o < OUT; ++o) out[(r0 + t) * OUT + o] = acc[o] + (b ? b[o] : 0.f);
  }
}

// dx rows + per-block partial [OUT][C+1] (last column = bias partial)
template <int OUT>
__global__ __launch_bounds__(256) void k_head_bwd(const float* __restrict__ x, int64_t N, int C,
                                                  const float* __restrict__ W,
                                                  const float* __restrict__ dout,
                                                  float* __restrict__ dx,
                                                  float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float sx[];  // [256][C+1] x rows, then dx
  __shared__ float sw[HEAD_MAX_OUT * 128];
  __shared__ float sd[HEAD_ROWS][HEAD_MAX_OUT];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * HEAD_ROWS;
  const int nr = (int)min((int64_t)HEAD_ROWS, N - r0);
  const int CP = C + 1;
  for (int k = t; k < OUT * C; k += 256) sw[k] = W[k];
  for (int k = t; k < nr * C; k += 256) {
    const int r = k / C;
    sx[r * CP + (k - r * C)] = x[r0 * C + k];
  }
  for (int k = t; k < HEAD_ROWS * OUT; k += 256) {
    const int r = k / OUT;
    sd[r][k - r * OUT] = (r < nr) ? dout[(r0 + r) * OUT + (k - r * OUT)] : 0.f;
  }
  __syncthreads();
  // weight / bias partials: thread per (o, c) column, sum over the block's rows
  float* pb = part + (int64_t)blockIdx.x * OUT * CP;
  for (int oc = t; oc < OUT * CP; oc += 256) {
    const int o = oc / CP, c = oc - o * CP;
    float s = 0.f;
    if (c < C) {
      for (int r = 0; r < nr; ++r) s = fmaf(sd[r][o], sx[r * CP + c], s);
    } else {
      for (int r = 0; r < nr; ++r) s += sd[r][o];
    }
    pb[oc] = s;
  }
  // dx rows (coalesced store through the row-major global layout)
  for (int k = t; k < nr * C; k += 256) {
    const int r = k / C, c = k - r * C;
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < OUT; ++o) s = fmaf(sd[r][o], sw[o * C + c], s);
    dx[r0 * C + k] = s;
  }
}

// gW[o][c] += Σ_b part[b][o][c]; gb[o] += Σ_b part[b][o][C]
__global__ __launch_bounds__(256) void k_head_reduce(const float* __restrict__ part, int nparts,
                                                     int OUT, int C, float* __restrict__ gW,
                                                     float* __restrict__ gb) {
  const int CP = C + 1;
  const int oc = blockIdx.x * 256 + threadIdx.x;
  if (oc >= OUT * CP) return;
  float s0 = 0.f, s1 = 0.f;
  int b = 0;
  for (; b + 1 < nparts; b += 2) {
    s0 += part[(int64_t)b * OUT * CP + oc];
    s1 += part[(int64_t)(b + 1) * OUT * CP + oc];
  }
  if (b < nparts) s0 += part[(int64_t)b * OUT * CP + oc];
  const int o = oc / CP, c = oc - o * CP;
  if (c < C) {
    if (gW) gW[o * C + c] += s0 + s1;
  } else if (gb) {
    gb[o] += s0 + s1;
  }
}

}  // namespace sv2n

using namespace sv2n;

static int head_check(int64_t N, int C, int out_ch) {
  if (N <= 0 || C <= 0 || out_ch <= 0) return SV2N_ERR_ARG;
  if (out_ch > HEAD_MAX_OUT || C > 128 || out_ch * C > HEAD_MAX_OUT * 128) return SV2N_ERR_SHAPE;
  return 0;
}

#define SV2N_HEAD_CASE(KERNEL, O, ...) \
  case O: if (lds > 65536) raise_head_lds(KERNEL<O>); hipLaunchKernelGGL(KERNEL<O>, __VA_ARGS__); break;
#define SV2N_HEAD_DISPATCH(KERNEL, ...)                                                       \
  switch (out_ch) {                                                                           \
    SV2N_HEAD_CASE(KERNEL, 1, __VA_ARGS__) SV2N_HEAD_CASE(KERNEL, 2, __VA_ARGS__)             \
    SV2N_HEAD_CASE(KERNEL, 3, __VA_ARGS__) SV2N_HEAD_CASE(KERNEL, 4, __VA_ARGS__)             \
    SV2N_HEAD_CASE(KERNEL, 5, __VA_ARGS__) SV2N_HEAD_CASE(KERNEL, 6, __VA_ARGS__)             \
    SV2N_HEAD_CASE(KERNEL, 7, __VA_ARGS__) SV2N_HEAD_CASE(KERNEL, 8, __VA_ARGS__)             \
    SV2N_HEAD_CASE(KERNEL, 9, __VA_ARGS__) SV2N_HEAD_CASE(KERNEL, 10, __VA_ARGS__)            \
    SV2N_HEAD_CASE(KERNEL, 11, __VA_ARGS__) SV2N_HEAD_CASE(KERNEL, 12, __VA_ARGS__)           \
    SV2N_HEAD_CASE(KERNEL, 13, __VA_ARGS__) SV2N_HEAD_CASE(KERNEL, 14, __VA_ARGS__)           \
    SV2N_HEAD_CASE(KERNEL, 15, __VA_ARGS__) SV2N_HEAD_CASE(KERNEL, 16, __VA_ARGS__)           \
    default: return SV2N_ERR_SHAPE;                                                           \
  }

template <typename K>
static void raise_head_lds(K kernel) {
  (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            140 * 1024);
}

extern "C" int sv2n_head_fwd(const float* x, int64_t num_rows, int in_features,
                             const float* weight, const float* bias, int out_features,
                             float* out, hipStream_t stream) {
  const int out_ch = out_features;
  if (!x || !weight || !out) return SV2N_ERR_ARG;
  if (int rc = head_check(num_rows, in_features, out_ch)) return rc;
  const unsigned grid = (unsigned)((num_rows + HEAD_ROWS - 1) / HEAD_ROWS);
  const size_t lds = sizeof(float) * HEAD_ROWS * (in_features + 1);
  SV2N_HEAD_DISPATCH(k_head_fwd, dim3(grid), dim3(256), lds, stream, x, num_rows, in_features,
                     weight, bias, out)
  return (int)hipGetLastError();
}

extern "C" int64_t sv2n_head_bwd_workspace(int64_t num_rows, int in_features, int out_features) {
  return ((num_rows + HEAD_ROWS - 1) / HEAD_ROWS) * (int64_t)out_features * (in_features + 1);
}

extern "C" int sv2n_head_bwd(const float* x, int64_t num_rows, int in_features,
                             const float* weight, int out_features, const float* dout, float* dx,
                             float* g_weight, float* g_bias, float* workspace,
                             int64_t workspace_floats, hipStream_t stream) {
  const int out_ch = out_features;
  if (!x || !weight || !dout || !dx || !workspace) return SV2N_ERR_ARG;
  if (int rc = head_check(num_rows, in_features, out_ch)) return rc;
  const int64_t nb = (num_rows + HEAD_ROWS - 1) / HEAD_ROWS;
  if (workspace_floats < nb * out_ch * (in_features + 1)) return SV2N_ERR_WORKSPACE;
  const size_t lds = sizeof(float) * HEAD_ROWS * (in_features + 1);
  SV2N_HEAD_DISPATCH(k_head_bwd, dim3((unsigned)nb), dim3(256), lds, stream, x, num_rows,
                     in_features, weight, dout, dx, workspace)
  if (g_weight || g_bias) {
    const int tot = out_ch * (in_features + 1);
    hipLaunchKernelGGL(k_head_reduce, dim3((tot + 255) / 256), dim3(256), 0, stream, workspace,
                       (int)nb, out_ch, in_features, g_weight, g_bias);
  }
  return (int)hipGetLastError();
}
