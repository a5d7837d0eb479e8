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
// A window whose matrices fall outside the series (starts[b] < 0 or
// starts[b] + S + F > T) reads nothing and is written as NaN (a device-side
// error that needs no host round trip; the op stays capturable).
#include "sv2n_common.h"

#ifndef SV2N_WINDOW_XCD
#define SV2N_WINDOW_XCD 1
#endif

namespace sv2n {

__global__ __launch_bounds__(256) void k_window_gather(
    const float* __restrict__ vol, const float* __restrict__ volvol, int n, int64_t T,
    const int64_t* __restrict__ starts, int64_t soff, int64_t B, int S, int F,
    const uint16_t* __restrict__ canon, float* __restrict__ x, float* __restrict__ ea,
    float* __restrict__ y) {
  const int64_t nn = (int64_t)n * n;
  const float qnan = __builtin_nanf("");
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
      const int64_t st = starts[b] < 0 ? -1 : starts[b] + soff;  // a negative index is out of range
      x[i] = (st >= 0 && st + S + F <= T) ? vol[(st + t) * nn + v * n + c] : qnan;
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
      const int64_t st = starts[b] < 0 ? -1 : starts[b] + soff;  // a negative index is out of range
      ea[k0] = (st >= 0 && st + S + F <= T) ? volvol[(st + t) * nn + r * n + c] : qnan;
    } else {
      const int64_t k0 = i - nx - ne;
      const int64_t row = k0 / F;
      const int k = (int)(k0 - row * F);
      const int64_t b = row / n;
      const int v = (int)(row - b * n);
      const int64_t st = starts[b] < 0 ? -1 : starts[b] + soff;  // a negative index is out of range
      y[k0] = (st >= 0 && st + S + F <= T) ? vol[(st + S + k) * nn + v * n + v] : qnan;
    }
  }
}

// One workgroup per (window b, node u): the S rows vol[st+t][u][:] and
// volvol[st+t][u][:] and the volvol diagonal are staged in LDS ([t][v]
// images, read along v = coalesced), then written transposed:
//   x row b*n+u                       (n*S floats, contiguous)
//   the edge rows of the upper pairs (u, w), w > u, and of their swapped
//   copies (canonical order: both runs are contiguous, 3S floats per row)
//   y[(b*n+u)*F .. +F)
// 3 * S * (n+1) floats of LDS.  diag (optional): diag[t][v] = volvol[t][v][v].
// cv_only (sv2n_window_gather_cv): of the edge rows only what the
// covariance-layout edge passes read (sv2n_edge.hip cv_var_row): the
// covariance columns of the upper rows, and in workgroup u = 0 the target
// variance columns of the pairs (0, w) and the source variance columns of
// pair (0, 1), plus the covariance columns of the lower rows the passes' last
// 16-row tile reaches — ≈ 1/6 of the edge bytes; the rest is not written.
__global__ __launch_bounds__(256) void k_window_rows(
    const float* __restrict__ vol, const float* __restrict__ volvol, int n, int64_t T,
    const int64_t* __restrict__ starts, int64_t soff, int S, int F,
    const float* __restrict__ diag, float* __restrict__ x, float* __restrict__ ea,
    float* __restrict__ y, unsigned short* __restrict__ xb, int64_t ldxb, int cv_only) {
  extern __shared__ float lds[];
  const int NP = n + 1;
  float* sv = lds;             // [S][NP] vol[t][u][v]
  float* sw = sv + S * NP;     // [S][NP] volvol[t][u][v]
  float* sd = sw + S * NP;     // [S][NP] volvol[t][v][v]
#if SV2N_WINDOW_XCD
  // XCD-aware order: blocks are dealt round-robin over the 8 XCDs, so block i
  // takes the (i % 8)-th contiguous eighth of the (window, node) range — a
  // window's n node blocks share one XCD's L2, and the series lines their rows
  // share (row u and u+1 of a matrix meet inside one 128-B line; the diagonal
  // every block reads) are fetched into one L2 instead of up to eight
  const int G = gridDim.x, gq = G >> 3, gr = G & 7, gi = blockIdx.x & 7;
  const int wb = gi * gq + min(gi, gr) + (blockIdx.x >> 3);
#else
  const int wb = blockIdx.x;
#endif
  const int u = wb % n;
  const int64_t b = wb / n;
  const int t = threadIdx.x;
  const int64_t nn = (int64_t)n * n;
  const int64_t st = starts[b] < 0 ? -1 : starts[b] + soff;  // a negative index is out of range
  const int E0 = n * (n - 1), P = E0 / 2;
  if (st < 0 || st + S + F > T) {  // window outside the series: NaN rows, no reads
    const float qnan = __builtin_nanf("");
    if (t < F) y[(b * n + u) * F + t] = qnan;
    if (x) {
      float* xr = x + (b * n + u) * (int64_t)n * S;
      for (int j = t; j < n * S; j += 256) xr[j] = qnan;
    }
    if (xb)
      for (int j = t; j < ldxb; j += 256)
        xb[(b * n + u) * ldxb + j] = j < n * S ? (unsigned short)0x7fc0 : (unsigned short)0;
    const int m = n - 1 - u, e0 = u * (2 * n - u - 1) / 2, RW = 3 * S;
    float* up = ea + (b * E0 + e0) * (int64_t)RW;
    float* lo = ea + (b * E0 + P + e0) * (int64_t)RW;
    for (int j = t; j < m * RW; j += 256) up[j] = lo[j] = qnan;
    return;
  }
  // staging: every load of a round issued before its LDS stores (the rolled
  // loop made one memory round trip per 256 elements: C3, S 42, 5 rounds)
  for (int k0 = 0; k0 < S * n; k0 += 8 * 256) {
    float a[8], w[8], d[8];
    int dst[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      // past the end: no load at all (the lanes' requests, not clamped
      // duplicates — at C3's S·n = 1260 three of the eight rounds are empty)
      const int k = k0 + t + 256 * r;
      const int tt = k / n, v = k - tt * n;
      const int64_t base = (st + tt) * nn;
      dst[r] = tt * NP + v;
      a[r] = w[r] = d[r] = 0.f;
      if (k < S * n) {
        a[r] = vol[base + (int64_t)u * n + v];
        w[r] = volvol[base + (int64_t)u * n + v];
        // the diagonal is only read for the pairs (u, w > u) — and of the
        // covariance-only edge rows only by node 0; from the series' diagonal
        // [T][n] when given (ABI 11: one line per matrix, not one per element)
        if (v > u && (!cv_only || u == 0))
          d[r] = diag ? diag[(st + tt) * n + v] : volvol[base + (int64_t)v * n + v];
      }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r)
      if (k0 + t + 256 * r < S * n) {
        sv[dst[r]] = a[r];
        sw[dst[r]] = w[r];
        sd[dst[r]] = d[r];
      }
  }
  if (t < F) y[(b * n + u) * F + t] = vol[(st + S + t) * nn + (int64_t)u * n + u];
  __syncthreads();
  // x[b*n+u][c*S + tt] = vol[tt][u][c]: 16-B stores when the row allows
  // (x NULL with xb: only the bf16 twin, ABI 21)
  float* xr = x ? x + (b * n + u) * (int64_t)n * S : nullptr;
  const int nxr = n * S;
  if ((nxr & 3) == 0 && (((uintptr_t)xr) & 15) == 0) {
    unsigned short* xbr = xb ? xb + (b * n + u) * ldxb : nullptr;
    for (int j4 = t; j4 < nxr / 4; j4 += 256) {
      f32x4 v;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int j = 4 * j4 + k, c = j / S, tt = j - c * S;
        v[k] = sv[tt * NP + c];
      }
      if (xr) *reinterpret_cast<f32x4*>(xr + 4 * j4) = v;
      if (xbr) {  // bf16(x) beside it (round to nearest even, as the GEMMs' staging)
        typedef __bf16 b4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<b4*>(xbr + 4 * j4) = __builtin_convertvector(v, b4);
      }
    }
    if (xbr)
      for (int j = nxr + t; j < ldxb; j += 256) xbr[j] = 0;
  } else {
    for (int j = t; j < nxr; j += 256) {
      const int c = j / S, tt = j - c * S;
      xr[j] = sv[tt * NP + c];
    }
  }
  // upper pairs (u, w > u): e = off(u) + (w - u - 1), off(u) = u*(2n-u-1)/2
  const int m = n - 1 - u;
  if (m == 0) return;
  const int e0 = u * (2 * n - u - 1) / 2;
  const int RW = 3 * S;
  float* up = ea + (b * E0 + e0) * (int64_t)RW;
  float* lo = ea + (b * E0 + P + e0) * (int64_t)RW;
  if (cv_only) {
    // the passes' last tile of 16 upper rows runs into the first lower rows
    // (their d-logits are zero there): those rows' covariance columns too, so
    // the products stay finite and bitwise those of the full gather
    const int pad = (16 - P % 16) % 16;
    const int lane = t & 63, wv = wave_id();
    for (int r = wv; r < m; r += 4) {
      const int w = u + 1 + r;
      const int qe = u == 0 ? RW : S;  // u > 0: the covariance columns only
      for (int q = lane; q < qe; q += 64) {
        const int kind = q / S, tt = q - kind * S;
        if (kind == 1 && r != 0) continue;  // source variance: pair (0, 1) only
        up[r * RW + q] = kind == 0 ? sw[tt * NP + w] : (kind == 1 ? sw[tt * NP + u] : sd[tt * NP + w]);
        if (kind == 0 && e0 + r < pad) lo[r * RW + q] = sw[tt * NP + w];
      }
    }
    return;
  }
  if ((S & 1) == 0 && RW <= 2 * 64 && (((uintptr_t)up) & 7) == 0 && (((uintptr_t)lo) & 7) == 0) {
    // one wave per edge row, two adjacent columns per lane (8-B stores; S even:
    // both columns have the same kind), (kind, t) decoded once
    const int lane = t & 63, wv = wave_id();
    const int q = 2 * lane, kind = q / S, tq = q - kind * S;
    const bool qv = q < RW;
    for (int r = wv; r < m; r += 4) {
      const int w = u + 1 + r;
      float cu[2], cl[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int tt = tq + k;
        // upper edge u -> w: (covol, var_u, var_w); swapped w -> u: (covol, var_w, var_u)
        const float cov = sw[tt * NP + w], du = sw[tt * NP + u], dw = sd[tt * NP + w];
        cu[k] = kind == 0 ? cov : (kind == 1 ? du : dw);
        cl[k] = kind == 0 ? cov : (kind == 1 ? dw : du);
      }
      if (qv) {
        *reinterpret_cast<float2*>(up + r * RW + q) = make_float2(cu[0], cu[1]);
        *reinterpret_cast<float2*>(lo + r * RW + q) = make_float2(cl[0], cl[1]);
      }
    }
    return;
  }
  if (RW <= 4 * 64) {
    // one wave per edge row, a lane's columns fixed: (kind, t) decoded once
    // (the flat element loop divided twice per element)
    const int lane = t & 63, wv = wave_id();
    int kind[4], tq[4];
#pragma unroll
    for (int qi = 0; qi < 4; ++qi) {
      const int q = lane + 64 * qi;
      kind[qi] = q / S;
      tq[qi] = q - kind[qi] * S;
    }
    for (int r = wv; r < m; r += 4) {
      const int w = u + 1 + r;
#pragma unroll
      for (int qi = 0; qi < 4; ++qi) {
        const int q = lane + 64 * qi;
        if (q < RW) {
          const int tt = tq[qi];
          const float cov = sw[tt * NP + w], du = sw[tt * NP + u], dw = sd[tt * NP + w];
          up[r * RW + q] = kind[qi] == 0 ? cov : (kind[qi] == 1 ? du : dw);
          lo[r * RW + q] = kind[qi] == 0 ? cov : (kind[qi] == 1 ? dw : du);
        }
      }
    }
    return;
  }
  for (int j = t; j < m * RW; j += 256) {
    const int r = j / RW, q = j - r * RW;
    const int kind = q / S, tt = q - kind * S;
    const int w = u + 1 + r;
    const float cov = sw[tt * NP + w];
    const float du = sw[tt * NP + u], dw = sd[tt * NP + w];
    up[j] = kind == 0 ? cov : (kind == 1 ? du : dw);
    lo[j] = kind == 0 ? cov : (kind == 1 ? dw : du);
  }
}

}  // namespace sv2n

using namespace sv2n;

extern "C" int sv2n_window_gather_bf16x(const float* vol, const float* volvol,
                                        const float* diag, int n, int64_t num_matrices,
                                        const int64_t* starts, int64_t start_offset,
                                        int64_t num_windows, int seq_length, int future_steps,
                                        const uint16_t* canon, float* x, uint16_t* x_bf16,
                                        int64_t ld_xb, float* edge_attr, float* y,
                                        hipStream_t stream) {
  if (!vol || !volvol || !starts || !canon || !x_bf16 || !edge_attr || !y)
    return SV2N_ERR_ARG;
  if (n < 2 || n > SV2N_MAX_N_TILED || num_windows < 1 || seq_length < 1 || future_steps < 1 ||
      num_matrices < 1)
    return SV2N_ERR_SHAPE;
  const size_t lds = sizeof(float) * 3 * (size_t)seq_length * (n + 1);
  // the row kernel's 16-B x path only (n·S % 4 == 0, 16-B aligned x rows)
  if (lds > 64 * 1024 || future_steps > 256 || ((int64_t)n * seq_length) % 4 ||
      ld_xb < (int64_t)n * seq_length || (ld_xb & 3) || ((uintptr_t)x & 15) ||
      ((uintptr_t)x_bf16 & 7))
    return SV2N_ERR_SHAPE;
  hipLaunchKernelGGL(k_window_rows, dim3((unsigned)(num_windows * n)), dim3(256), lds, stream,
                     vol, volvol, n, num_matrices, starts, start_offset, seq_length, future_steps,
                     diag, x, edge_attr, y, reinterpret_cast<unsigned short*>(x_bf16), ld_xb, 0);
  return (int)hipGetLastError();
}

extern "C" int sv2n_window_gather_cv(const float* vol, const float* volvol, const float* diag,
                                     int n, int64_t num_matrices, const int64_t* starts,
                                     int64_t start_offset, int64_t num_windows, int seq_length,
                                     int future_steps, const uint16_t* canon, float* x,
                                     uint16_t* x_bf16, int64_t ld_xb, float* edge_attr, float* y,
                                     hipStream_t stream) {
  if (!vol || !volvol || !starts || !canon || (!x && !x_bf16) || !edge_attr || !y)
    return SV2N_ERR_ARG;
  if (n < 2 || n > SV2N_MAX_N_TILED || num_windows < 1 || seq_length < 1 || future_steps < 1 ||
      num_matrices < 1)
    return SV2N_ERR_SHAPE;
  const size_t lds = sizeof(float) * 3 * (size_t)seq_length * (n + 1);
  if (lds > 64 * 1024 || future_steps > 256) return SV2N_ERR_SHAPE;
  if (x_bf16 && (((int64_t)n * seq_length) % 4 || ld_xb < (int64_t)n * seq_length ||
                 (ld_xb & 3) || ((uintptr_t)x & 15) || ((uintptr_t)x_bf16 & 7)))
    return SV2N_ERR_SHAPE;
  hipLaunchKernelGGL(k_window_rows, dim3((unsigned)(num_windows * n)), dim3(256), lds, stream,
                     vol, volvol, n, num_matrices, starts, start_offset, seq_length, future_steps,
                     diag, x, edge_attr, y, reinterpret_cast<unsigned short*>(x_bf16),
                     x_bf16 ? ld_xb : (int64_t)0, 1);
  return (int)hipGetLastError();
}

extern "C" int sv2n_window_gather_diag(const float* vol, const float* volvol,
                                       const float* diag, int n, int64_t num_matrices,
                                       const int64_t* starts, int64_t start_offset,
                                       int64_t num_windows, int seq_length, int future_steps,
                                       const uint16_t* canon, float* x, float* edge_attr,
                                       float* y, hipStream_t stream) {
  if (!vol || !volvol || !starts || !canon || !x || !edge_attr || !y) return SV2N_ERR_ARG;
  if (n < 2 || n > SV2N_MAX_N_TILED || num_windows < 1 || seq_length < 1 || future_steps < 1 ||
      num_matrices < 1)
    return SV2N_ERR_SHAPE;
  const int64_t total = num_windows * ((int64_t)n * n * seq_length +
                                       (int64_t)n * (n - 1) * 3 * seq_length +
                                       (int64_t)n * future_steps);
  const size_t lds = sizeof(float) * 3 * (size_t)seq_length * (n + 1);
  if (lds <= 64 * 1024 && future_steps <= 256) {
    hipLaunchKernelGGL(k_window_rows, dim3((unsigned)(num_windows * n)), dim3(256), lds, stream,
                       vol, volvol, n, num_matrices, starts, start_offset, seq_length, future_steps,
                       diag, x, edge_attr, y, (unsigned short*)nullptr, (int64_t)0, 0);
    return (int)hipGetLastError();
  }
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(k_window_gather, dim3((unsigned)blocks), dim3(256), 0, stream, vol, volvol,
                     n, num_matrices, starts, start_offset, num_windows, seq_length, future_steps,
                     canon, x, edge_attr, y);
  return (int)hipGetLastError();
}

extern "C" int sv2n_window_gather(const float* vol, const float* volvol, int n,
                                  int64_t num_matrices, const int64_t* starts,
                                  int64_t start_offset, int64_t num_windows, int seq_length,
                                  int future_steps, const uint16_t* canon, float* x,
                                  float* edge_attr, float* y, hipStream_t stream) {
  return sv2n_window_gather_diag(vol, volvol, nullptr, n, num_matrices, starts, start_offset,
                                 num_windows, seq_length, future_steps, canon, x, edge_attr, y,
                                 stream);
}
