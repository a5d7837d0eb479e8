// Device-side window builder: the CovarianceLaggedDataset
// graph layout (reference utils/dataset.py:200-282, multi-output targets
// :385-405) gathered straight from a device-resident matrix series into a
// batch's x / edge_attr / y_x buffers, one launch per batch, capturable.
//
//   x[b*n + v][c*S + t]          = vol[st_b + t][v][c]                      (:279)
//   edge_attr[b*E0 + e][0*S + t] = volvol[st_b + t][min(s,g)][max(s,g)]     (:243-245,
//                                   the upper-triangle value, duplicated for the swapped half)
//   edge_attr[b*E0 + e][1*S + t] = volvol[st_b + t][s][s]                   (:236, source)
//   edge_attr[b*E0 + e][2*S + t] = volvol[st_b + t][g][g]                   (target)
//   y[(b*n + v)*F + k]           = vol[st_b + S + k][v][v]                   (:262 / :385-390)
// with e -> (s = source, g = target) from the canonical table (target<<8 | source).
//
// Every output element is written once, coalesced; the reads are gathers from
// the window's S matrices (L2 / Infinity-Cache resident across the threads of
// a window).  HBM-bound by the writes: B*(n*n*S + 3*E0*S + n*F)*4 bytes.
#include "sv2n_common.h"

namespace sv2n {

__global__ __launch_bounds__(256) void k_window_gather(
    const float* __restrict__ vol, const float* __restrict__ volvol, int n,
    const int64_t* __restrict__ starts, int64_t B, int S, int F,
    const uint16_t* __restrict__ canon, float* __restrict__ x, float* __restrict__ ea,
    float* __restrict__ y) {
  const int64_t nn = (int64_t)n * n;
  const int E0 = n * (n - 1);
  const int64_t nx = B * nn * S, ne = B * (int64_t)E0 * 3 * S, ny = B * (int64_t)n * F;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nx + ne + ny;
       i += stride) {
    if (i < nx) {
      const int64_t row = i / (n * S);
      const int j = (int)(i - row * n * S);
      const int64_t b = row / n;
      const int v = (int)(row - b * n);
      const int c = j / S, t = j - c * S;
      x[i] = vol[(starts[b] + t) * nn + v * n + c];
    } else if (i < nx + ne) {
      const int64_t k0 = i - nx;
      const int64_t row = k0 / (3 * S);
      const int j = (int)(k0 - row * 3 * S);
      const int64_t b = row / E0;
      const int e = (int)(row - b * E0);
      const int kind = j / S, t = j - kind * S;
      const int code = canon[e];
      const int s = code & 0xff, g = code >> 8;
      int r, c;
      if (kind == 0) {
        r = min(s, g);
        c = max(s, g);
      } else {
        r = c = (kind == 1) ? s : g;
      }
      ea[k0] = volvol[(starts[b] + t) * nn + r * n + c];
    } else {
      const int64_t k0 = i - nx - ne;
      const int64_t row = k0 / F;
      const int k = (int)(k0 - row * F);
      const int64_t b = row / n;
      const int v = (int)(row - b * n);
      y[k0] = vol[(starts[b] + S + k) * nn + v * n + v];
    }
  }
}

}  // namespace sv2n

using namespace sv2n;

extern "C" int sv2n_window_gather(const float* vol, const float* volvol, int n,
                                  const int64_t* starts, int64_t num_windows, int seq_length,
                                  int future_steps, const uint16_t* canon, float* x,
                                  float* edge_attr, float* y, hipStream_t stream) {
  if (!vol || !volvol || !starts || !canon || !x || !edge_attr || !y) return SV2N_ERR_ARG;
  if (n < 2 || n > SV2N_MAX_N_TILED || num_windows < 1 || seq_length < 1 || future_steps < 1)
    return SV2N_ERR_SHAPE;
  const int64_t total = num_windows * ((int64_t)n * n * seq_length +
                                       (int64_t)n * (n - 1) * 3 * seq_length +
                                       (int64_t)n * future_steps);
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(k_window_gather, dim3((unsigned)blocks), dim3(256), 0, stream, vol, volvol,
                     n, starts, num_windows, seq_length, future_steps, canon, x, edge_attr, y);
  return (int)hipGetLastError();
}
