// Output head of GATModel: the final nn.Linear(h_last, out_ch) (reference
// utils/models.py:120, applied at :150), and the same head fused with the
// training loss of 5_train_SpotV2Net.py:154 (nn.MSELoss, mean reduction).
//   forward   out[i][o] = Σ_c x[i][c] · W[o][c] + b[o]
//   backward  dx[i][c]  = Σ_o dout[i][o] · W[o][c]
//             gW[o][c] += Σ_i dout[i][o] · x[i][c],  gb[o] += Σ_i dout[i][o]
//   MSE       loss = mean((out - y)²),  dout = 2 (out - y) / (rows·out_ch) · dloss
// Reductions over rows go through per-workgroup partial slabs summed in a
// fixed order by the last-arriving workgroup of the same launch
// (last_block_sc1_2): deterministic, and no separate reduce launch.
//
// Workspace layout (floats): [0, 288) ticket counters (zero before the first
// call; every launch leaves it zero) | [288, ...) partial slabs.
//
// Rows per workgroup R = 256 for in_features <= 128 (one row per thread);
// wider heads (C1/C3: 500) stage fewer rows, R ∈ {128, 64, 32}, so the
// [R][C+1] image and the weights fit the 160 KiB LDS, and 256/R threads share
// a row (strided over c, partials added in a fixed order).
#include "sv2n_common.h"

namespace sv2n {

constexpr int HEAD_MAX_OUT = 16;
constexpr int HEAD_MAX_IN = 1024;
constexpr int HEAD_ROWS = 256;  // rows per workgroup at most (one per thread)
constexpr int HEAD_WS_HDR = SV2N_TICKET_WORDS;  // two-level ticket counters
constexpr size_t HEAD_LDS_BUDGET = 160 * 1024 - 20 * 1024;  // dynamic part (statics below)

// rows per workgroup for in_features C, out_features O, N rows (0: does not
// fit): the largest of 256 .. 32 whose [R][C+1] image and weights fit the LDS,
// lowered (down to 8) until the launch has ~256 workgroups (a C2 batch of
// 15,360 rows at R = 256 was 60 workgroups on 256 CUs)
__host__ __device__ inline int head_rows_per_block(int C, int O, int64_t N) {
  int R = 0;
  for (int r = 256; r >= 32; r >>= 1)
    if ((size_t)4 * ((size_t)r * (C + 1) + (size_t)O * C) <= HEAD_LDS_BUDGET) {
      R = r;
      break;
    }
  if (R == 0) return 0;
  // halve while the launch stays <= 256 workgroups and the weight-gradient
  // partials the last workgroup combines stay <= 128K floats (C3, 3,840 rows
  // of 500: 60 workgroups of 64 rows took 35 us; 240 of 16 rows)
  const int64_t tot = (int64_t)O * (C + 1);
  while (R > 8) {
    const int64_t nb = (N + R / 2 - 1) / (R / 2);
    if (nb > 256 || nb * tot > 131072) break;
    R >>= 1;
  }
  return R;
}
__host__ __device__ inline size_t head_lds_bytes(int C, int O, int64_t N) {
  return (size_t)4 * ((size_t)head_rows_per_block(C, O, N) * (C + 1) + (size_t)O * C);
}

// x rows staged through LDS so the global reads are coalesced.  The block's
// rows are one contiguous span of nr*C floats: it is read as 16-B buffer
// loads, 8 per thread in flight per round (a plain element loop of
// load -> LDS store is not pipelined by the compiler: one round trip per
// element), then scattered into the padded [row][C+1] image.
template <int OUT>
__device__ __forceinline__ void head_rows(const float* __restrict__ x, int64_t r0, int nr, int C,
                                          float* __restrict__ sx, const float* __restrict__ W,
                                          float* __restrict__ sw, int t) {
  const int CP = C + 1;
  for (int k = t; k < OUT * C; k += 256) sw[k] = W[k];
  const int n = nr * C;
  const float* base = x + r0 * C;
  if ((((uintptr_t)base) & 15) == 0) {
    const rsrc_t rx = make_rsrc(base, (uint32_t)n * 4u);
    const int nv = (n + 3) >> 2;
    for (int v0 = 0; v0 < nv; v0 += 8 * 256) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = v0 + t + 256 * u;
        v[u] = bld4(rx, q < nv ? q * 16 : OOB);  // tail floats past n read 0
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = v0 + t + 256 * u;
        if (q < nv) {
          int e = 4 * q, r = e / C, c = e - r * C;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (e + k < n) sx[r * CP + c] = v[u][k];
            if (++c == C) { c = 0; ++r; }
          }
        }
      }
    }
  } else {
    for (int k = t; k < n; k += 256) {
      const int r = k / C;
      sx[r * CP + (k - r * C)] = base[k];
    }
  }
}

// acc[o] = Σ_c x[row][c]·W[o][c] of the block's row r = t % R over the c of
// thread part q = t / R (c ≡ q mod 256/R); with more than one part per row the
// parts are added in a fixed order through s_part.  Returns true for the
// thread that holds row r's total (q == 0, r < nr).
template <int OUT>
__device__ __forceinline__ bool head_dot(const float* __restrict__ sx, const float* __restrict__ sw,
                                         int C, int R, int nr, int t, float (&acc)[OUT],
                                         float* __restrict__ s_part) {
  const int CP = C + 1;
  const int r = t % R, q = t / R, Q = 256 / R;
#pragma unroll
  for (int o = 0; o < OUT; ++o) acc[o] = 0.f;
  if (r < nr) {
    for (int c = q; c < C; c += Q) {
      const float xv = sx[r * CP + c];
#pragma unroll
      for (int o = 0; o < OUT; ++o) acc[o] = fmaf(xv, sw[o * C + c], acc[o]);
    }
  }
  if (Q == 1) return r < nr;
  __syncthreads();
#pragma unroll
  for (int o = 0; o < OUT; ++o) s_part[(q * R + r) * OUT + o] = acc[o];
  __syncthreads();
  if (q != 0) return false;
#pragma unroll
  for (int o = 0; o < OUT; ++o) {
    float v = 0.f;
    for (int k = 0; k < Q; ++k) v += s_part[(k * R + r) * OUT + o];
    acc[o] = v;
  }
  return r < nr;
}

template <int OUT>
__global__ __launch_bounds__(256) void k_head_fwd(const float* __restrict__ x, int64_t N, int C,
                                                  const float* __restrict__ W,
                                                  const float* __restrict__ b,
                                                  float* __restrict__ out, int R) {
  extern __shared__ __attribute__((aligned(16))) float sx[];  // [R][C+1] | sw [OUT][C]
  __shared__ float s_part[256 * OUT];
  float* sw = sx + R * (C + 1);
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int nr = (int)min((int64_t)R, N - r0);
  head_rows<OUT>(x, r0, nr, C, sx, W, sw, t);
  __syncthreads();
  float acc[OUT];
  if (head_dot<OUT>(sx, sw, C, R, nr, t, acc, s_part)) {
    const int r = t % R;
#pragma unroll
    for (int o = 0; o < OUT; ++o) out[(r0 + r) * OUT + o] = acc[o] + (b ? b[o] : 0.f);
  }
}

// head + MSE forward: diff = out - y (saved for the backward), optional
// prediction, loss = Σ diff² · inv_count (last-arriving block)
template <int OUT>
__global__ __launch_bounds__(256) void k_head_mse_fwd(
    const float* __restrict__ x, int64_t N, int C, const float* __restrict__ W,
    const float* __restrict__ b, const float* __restrict__ target, float* __restrict__ yhat,
    float* __restrict__ diff, float* __restrict__ ws, float* __restrict__ loss,
    float* __restrict__ loss_sum, float inv_count, int R) {
  extern __shared__ __attribute__((aligned(16))) float sx[];  // [R][C+1] | sw [OUT][C]
  __shared__ float s_part[256 * OUT];
  __shared__ float s_red[256];
  float* sw = sx + R * (C + 1);
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int nr = (int)min((int64_t)R, N - r0);
  head_rows<OUT>(x, r0, nr, C, sx, W, sw, t);
  __syncthreads();
  float sq = 0.f;
  float acc[OUT];
  if (head_dot<OUT>(sx, sw, C, R, nr, t, acc, s_part)) {
    const int r = t % R;
#pragma unroll
    for (int o = 0; o < OUT; ++o) {
      const int64_t k = (r0 + r) * OUT + o;
      const float v = acc[o] + (b ? b[o] : 0.f);
      if (yhat) yhat[k] = v;
      const float d = v - target[k];
      diff[k] = d;
      sq = fmaf(d, d, sq);
    }
  }
  s_red[t] = sq;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) s_red[t] += s_red[t + s];
    __syncthreads();
  }
  float* part = ws + HEAD_WS_HDR;
  if (t == 0) st_sc1(part + blockIdx.x, s_red[0]);
  int* s_flag = reinterpret_cast<int*>(s_part);
  if (last_block_sc1_2(reinterpret_cast<unsigned*>(ws), gridDim.x, s_flag)) {
    float a = 0.f;
    for (int k = t; k < (int)gridDim.x; k += 256) a += ld_sc1(part + k);
    s_red[t] = a;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (t < s) s_red[t] += s_red[t + s];
      __syncthreads();
    }
    if (t == 0) {
      loss[0] = s_red[0] * inv_count;
      if (loss_sum) loss_sum[0] += s_red[0] * inv_count;
    }
  }
}

// dx rows + per-block partial [OUT][C+1] (last column = bias partial); the
// last-arriving block ACCUMULATES Σ partials into gW / gb.  Both the
// per-block column sums (over 256 rows) and the combine (over the blocks)
// spread a column over RG = 256 / (OUT·(C+1)) thread groups (>= 1), then add
// the groups in a fixed order through LDS: deterministic, all threads busy.
// dout = src · scale (· *dscale when given): plain head backward with
// src = dout, scale = 1; MSE backward with src = diff, scale = 2/(rows·out),
// dscale = dloss.
template <int OUT>
__global__ __launch_bounds__(256) void k_head_bwd(const float* __restrict__ x, int64_t N, int C,
                                                  const float* __restrict__ W,
                                                  const float* __restrict__ src, float scale,
                                                  const float* __restrict__ dscale,
                                                  float* __restrict__ dx, float* __restrict__ ws,
                                                  float* __restrict__ gW, float* __restrict__ gb,
                                                  int R) {
  extern __shared__ __attribute__((aligned(16))) float sx[];  // [R][C+1] x rows | sw [OUT][C]
  __shared__ float sd[HEAD_ROWS][HEAD_MAX_OUT];
  __shared__ float s_grp[256];
  float* sw = sx + R * (C + 1);
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int nr = (int)min((int64_t)R, N - r0);
  const int CP = C + 1;
  const int tot = OUT * CP;
  const int RG = tot <= 256 ? 256 / tot : 1;
  const float sc = dscale ? scale * dscale[0] : scale;
  head_rows<OUT>(x, r0, nr, C, sx, W, sw, t);
  for (int k = t; k < R * OUT; k += 256) {
    const int r = k / OUT;
    sd[r][k - r * OUT] = (r < nr) ? src[(r0 + r) * OUT + (k - r * OUT)] * sc : 0.f;
  }
  __syncthreads();
  float* part = ws + HEAD_WS_HDR;
  float* pb = part + (int64_t)blockIdx.x * tot;
  if (RG > 1) {
    // column oc = t % tot summed over rows r ≡ g (mod RG), g = t / tot
    if (t < RG * tot) {
      const int oc = t % tot, g = t / tot;
      const int o = oc / CP, c = oc - o * CP;
      float s = 0.f;
      if (c < C) {
        for (int r = g; r < nr; r += RG) s = fmaf(sd[r][o], sx[r * CP + c], s);
      } else {
        for (int r = g; r < nr; r += RG) s += sd[r][o];
      }
      s_grp[t] = s;
    }
    __syncthreads();
    if (t < tot) {
      float s = 0.f;
      for (int g = 0; g < RG; ++g) s += s_grp[g * tot + t];
      st_sc1(pb + t, s);
    }
  } else {
    for (int oc = t; oc < tot; oc += 256) {
      const int o = oc / CP, c = oc - o * CP;
      float s = 0.f;
      if (c < C) {
        for (int r = 0; r < nr; ++r) s = fmaf(sd[r][o], sx[r * CP + c], s);
      } else {
        for (int r = 0; r < nr; ++r) s += sd[r][o];
      }
      st_sc1(pb + oc, s);
    }
  }
  // dx rows (coalesced store through the row-major global layout)
  for (int k = t; k < nr * C; k += 256) {
    const int r = k / C, c = k - r * C;
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < OUT; ++o) s = fmaf(sd[r][o], sw[o * C + c], s);
    dx[r0 * C + k] = s;
  }
  if (!gW && !gb) return;
  int* s_flag = reinterpret_cast<int*>(&sd[0][0]);
  __syncthreads();  // sd no longer needed: reuse one word as the flag
  if (last_block_sc1_2(reinterpret_cast<unsigned*>(ws), gridDim.x, s_flag)) {
    const int nparts = gridDim.x;
    for (int base = 0; base < tot; base += 256) {
      const int cols = min(256, tot - base);
      const int PG = 256 / cols;  // part groups
      if (t < PG * cols) {
        const int oc = base + t % cols, g = t / cols;
        float s = 0.f;
        // 8 independent loads in flight per round (a dependent chain of
        // agent-scope loads is one memory round trip per part)
        for (int b0 = g; b0 < nparts; b0 += 8 * PG) {
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int bb = b0 + u * PG;
            v[u] = bb < nparts ? ld_sc1(part + (int64_t)bb * tot + oc) : 0.f;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) s += v[u];
        }
        s_grp[t] = s;
      }
      __syncthreads();
      if (t < cols) {
        float s = 0.f;
        for (int g = 0; g < PG; ++g) s += s_grp[g * cols + t];
        const int oc = base + t;
        const int o = oc / CP, c = oc - o * CP;
        if (c < C) {
          if (gW) gW[o * C + c] += s;
        } else if (gb) {
          gb[o] += s;
        }
      }
      __syncthreads();
    }
  }
}

// Head + MSE forward AND backward in one launch, for a training step whose
// upstream loss gradient is 1 (train.TrainStep: loss.backward()): per block
// the rows' outputs, diff = out - target, the squared-error partial, dout =
// diff · 2/(rows·out), dx rows and the [OUT][C+1] weight/bias partial; the
// last-arriving block sums the loss partials and the weight / bias partials
// in a fixed order.  Replaces k_head_mse_fwd + k_head_bwd (x read once, one
// launch, one ticket).
template <int OUT>
__global__ __launch_bounds__(256) void k_head_mse_train(
    const float* __restrict__ x, int64_t N, int C, const float* __restrict__ W,
    const float* __restrict__ b, const float* __restrict__ target, float* __restrict__ dx,
    float* __restrict__ ws, float* __restrict__ gW, float* __restrict__ gb,
    float* __restrict__ loss, float* __restrict__ loss_sum, float inv_count, float scale, int R) {
  extern __shared__ __attribute__((aligned(16))) float sx[];  // [R][C+1] | sw [OUT][C]
  __shared__ float s_part[256 * OUT];
  __shared__ float sd[HEAD_ROWS][HEAD_MAX_OUT];
  __shared__ float s_grp[256];
  float* sw = sx + R * (C + 1);
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int nr = (int)min((int64_t)R, N - r0);
  const int CP = C + 1;
  const int tot = OUT * CP;
  head_rows<OUT>(x, r0, nr, C, sx, W, sw, t);
  for (int k = t; k < R * OUT; k += 256) sd[k / OUT][k - (k / OUT) * OUT] = 0.f;
  __syncthreads();
  float sq = 0.f;
  float acc[OUT];
  if (head_dot<OUT>(sx, sw, C, R, nr, t, acc, s_part)) {
    const int r = t % R;
#pragma unroll
    for (int o = 0; o < OUT; ++o) {
      const int64_t k = (r0 + r) * OUT + o;
      const float d = acc[o] + (b ? b[o] : 0.f) - target[k];
      sq = fmaf(d, d, sq);
      sd[r][o] = d * scale;
    }
  }
  // block loss partial: wave sums, then the 4 waves in order
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) sq += __shfl_xor(sq, m, 64);
  if ((t & 63) == 0) s_grp[t >> 6] = sq;
  __syncthreads();
  float* part = ws + HEAD_WS_HDR;
  float* pb = part + (int64_t)blockIdx.x * (tot + 1);
  if (t == 0) st_sc1(pb + tot, (s_grp[0] + s_grp[1]) + (s_grp[2] + s_grp[3]));
  __syncthreads();
  // weight / bias partial: column oc = t % tot over rows r = g (mod RG)
  const int RG = tot <= 256 ? 256 / tot : 1;
  if (RG > 1) {
    if (t < RG * tot) {
      const int oc = t % tot, g = t / tot;
      const int o = oc / CP, c = oc - o * CP;
      float s = 0.f;
      if (c < C) {
        for (int r = g; r < nr; r += RG) s = fmaf(sd[r][o], sx[r * CP + c], s);
      } else {
        for (int r = g; r < nr; r += RG) s += sd[r][o];
      }
      s_grp[t] = s;
    }
    __syncthreads();
    if (t < tot) {
      float s = 0.f;
      for (int g = 0; g < RG; ++g) s += s_grp[g * tot + t];
      st_sc1(pb + t, s);
    }
  } else {
    for (int oc = t; oc < tot; oc += 256) {
      const int o = oc / CP, c = oc - o * CP;
      float s = 0.f;
      if (c < C) {
        for (int r = 0; r < nr; ++r) s = fmaf(sd[r][o], sx[r * CP + c], s);
      } else {
        for (int r = 0; r < nr; ++r) s += sd[r][o];
      }
      st_sc1(pb + oc, s);
    }
  }
  // dx rows
  for (int k = t; k < nr * C; k += 256) {
    const int r = k / C, c = k - r * C;
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < OUT; ++o) s = fmaf(sd[r][o], sw[o * C + c], s);
    dx[r0 * C + k] = s;
  }
  int* s_flag = reinterpret_cast<int*>(s_part);
  __syncthreads();  // s_part free: one word as the flag
  if (last_block_sc1_2(reinterpret_cast<unsigned*>(ws), gridDim.x, s_flag)) {
    const int nparts = gridDim.x;
    const int stride = tot + 1;
    for (int base = 0; base < stride; base += 256) {
      const int cols = min(256, stride - base);
      const int PG = 256 / cols;  // part groups
      if (t < PG * cols) {
        const int oc = base + t % cols, g = t / cols;
        float s = 0.f;
        // 64 loads in flight: one round trip for up to 64·PG partials (C2: 240)
        for (int b0 = g; b0 < nparts; b0 += 64 * PG) {
          float v[64];
#pragma unroll
          for (int u = 0; u < 64; ++u) {
            const int bb = b0 + u * PG;
            v[u] = bb < nparts ? ld_sc1(part + (int64_t)bb * stride + oc) : 0.f;
          }
#pragma unroll
          for (int u = 0; u < 64; ++u) s += v[u];
        }
        s_grp[t] = s;
      }
      __syncthreads();
      if (t < cols) {
        float s = 0.f;
        for (int g = 0; g < PG; ++g) s += s_grp[g * cols + t];
        const int oc = base + t;
        if (oc == tot) {
          loss[0] = s * inv_count;
          if (loss_sum) loss_sum[0] += s * inv_count;
        } else {
          const int o = oc / CP, c = oc - o * CP;
          if (c < C) {
            if (gW) gW[o * C + c] += s;
          } else if (gb) {
            gb[o] += s;
          }
        }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// Head + MSE training launch, wave-per-rows form (out_features·ceil(C/64) <=
// 32; every SpotV2Net head: out 1, C 50 / 500).  Wave w of block b owns rows
// [(4b + w)·RW, +RW); lane l holds columns l + 64k (k < KC) of W in registers
// and of each row it reads (dword loads, 256 B per instruction; RB rows in
// flight).  Per row: the dot by a wave reduction, diff, the squared-error
// term, dx = dout ⊗ W (coalesced stores), and the weight / bias gradient
// partials in registers.  The block adds its 4 waves' partials in wave order
// through LDS and publishes one [OUT][C+1] + loss partial; the launch then
// reduces the partials in two levels (group_last_sc1 / top_last_sc1: group
// g = b % 8 sums blocks g, g + 8, ... in order, the last group finisher the 8
// groups in order).  The block-at-a-time kernel above read every partial in
// one workgroup: C3 (240 partials of 502 floats) spent most of its 33 us there.
// ---------------------------------------------------------------------------
// DEFER (sv2n_head_mse_train_rows): each block only publishes its partial
// (plain stores); k_head_mse_reduce_w sums them later, in the same order.
template <int OUT, int KC, bool DEFER = false>
__global__ __launch_bounds__(256) void k_head_mse_train_w(
    const float* __restrict__ x, int64_t N, int C, const float* __restrict__ W,
    const float* __restrict__ b, const float* __restrict__ target, float* __restrict__ dx,
    float* __restrict__ ws, float* __restrict__ gW, float* __restrict__ gb,
    float* __restrict__ loss, float* __restrict__ loss_sum, float inv_count, float scale,
    int RW) {
  constexpr int RB = KC >= 8 ? 4 : (KC >= 4 ? 8 : 16);  // rows in flight per wave
  extern __shared__ __attribute__((aligned(16))) float s_w4[];  // [4][stride] wave partials
  __shared__ int s_flag;
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int CP = C + 1, stride = OUT * CP + 1;  // [o][c], [o][C] bias, [OUT·CP] loss
  float w[OUT][KC], bo[OUT], gw[OUT][KC], gbs[OUT];
#pragma unroll
  for (int o = 0; o < OUT; ++o) {
    bo[o] = b ? b[o] : 0.f;
    gbs[o] = 0.f;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int c = lane + 64 * k;
      w[o][k] = c < C ? W[o * C + c] : 0.f;
      gw[o][k] = 0.f;
    }
  }
  float sq = 0.f;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * RW;
  const int nr = (int)max((int64_t)0, min((int64_t)RW, N - r0));
  for (int i0 = 0; i0 < nr; i0 += RB) {
    float xv[RB][KC], tv[RB][OUT];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const bool rv = i0 + u < nr;
      const int64_t r = r0 + i0 + u;
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const int c = lane + 64 * k;
        xv[u][k] = (rv && c < C) ? x[r * C + c] : 0.f;
      }
#pragma unroll
      for (int o = 0; o < OUT; ++o) tv[u][o] = rv ? target[r * OUT + o] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      if (i0 + u >= nr) continue;  // wave-uniform
      const int64_t r = r0 + i0 + u;
      float d[OUT];
#pragma unroll
      for (int o = 0; o < OUT; ++o) {
        float p = 0.f;
#pragma unroll
        for (int k = 0; k < KC; ++k) p = fmaf(xv[u][k], w[o][k], p);
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) p += __shfl_xor(p, m, 64);
        const float e = p + bo[o] - tv[u][o];
        sq = fmaf(e, e, sq);
        d[o] = e * scale;
        gbs[o] += d[o];
      }
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const int c = lane + 64 * k;
        float v = 0.f;
#pragma unroll
        for (int o = 0; o < OUT; ++o) {
          v = fmaf(d[o], w[o][k], v);
          gw[o][k] = fmaf(d[o], xv[u][k], gw[o][k]);
        }
        if (c < C) dx[r * C + c] = v;
      }
    }
  }
  // block partial: the 4 waves in order
  float* sp = s_w4 + wave * stride;
#pragma unroll
  for (int o = 0; o < OUT; ++o) {
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int c = lane + 64 * k;
      if (c < C) sp[o * CP + c] = gw[o][k];
    }
    if (lane == 0) sp[o * CP + C] = gbs[o];
  }
  if (lane == 0) sp[OUT * CP] = sq;  // every lane holds the same sum
  __syncthreads();
  float* part = ws + HEAD_WS_HDR;
  const unsigned nb = gridDim.x;
  if constexpr (DEFER) {
    for (int oc = t; oc < stride; oc += 256)
      part[(int64_t)blockIdx.x * stride + oc] =
          (s_w4[oc] + s_w4[stride + oc]) + (s_w4[2 * stride + oc] + s_w4[3 * stride + oc]);
    return;
  }
  for (int oc = t; oc < stride; oc += 256)
    st_sc1(part + (int64_t)blockIdx.x * stride + oc,
           (s_w4[oc] + s_w4[stride + oc]) + (s_w4[2 * stride + oc] + s_w4[3 * stride + oc]));
  if (!group_last_sc1(reinterpret_cast<unsigned*>(ws), nb, &s_flag)) return;
  // group g: blocks g, g + 8, ... in order -> group slab g
  float* gslab = part + (int64_t)nb * stride;
  const unsigned g = blockIdx.x & 7u, members = (nb - g + 7u) / 8u;
  for (int oc = t; oc < stride; oc += 256) {
    float s = 0.f;
    for (unsigned m0 = 0; m0 < members; m0 += 32) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u)
        v[u] = m0 + u < members ? ld_sc1(part + (int64_t)(g + 8u * (m0 + u)) * stride + oc) : 0.f;
#pragma unroll
      for (int u = 0; u < 32; ++u) s += v[u];
    }
    st_sc1(gslab + (int64_t)g * stride + oc, s);
  }
  if (!top_last_sc1(reinterpret_cast<unsigned*>(ws), nb, &s_flag)) return;
  const int groups = nb < 8u ? (int)nb : 8;
  for (int oc = t; oc < stride; oc += 256) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = u < groups ? ld_sc1(gslab + (int64_t)u * stride + oc) : 0.f;
    const float s = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    if (oc == OUT * CP) {
      loss[0] = s * inv_count;
      if (loss_sum) loss_sum[0] += s * inv_count;
    } else {
      const int o = oc / CP, c = oc - o * CP;
      if (c < C) {
        if (gW) gW[o * C + c] += s;
      } else if (gb) {
        gb[o] += s;
      }
    }
  }
}

// The deferred reduction of k_head_mse_train_w<..., true>'s nb block partials
// (a launch of its own, after the layer backwards that need only dx).  Block of 512 = 8 groups x 64 columns: thread (g, l) sums
// partials g, g + 8, ... of column oc in block order, as group_last_sc1's
// finisher does, and group 0 adds the 8 group sums as top_last_sc1's finisher
// does: the same floating-point order, so the same bits as the one-launch form.
__global__ __launch_bounds__(512) void k_head_mse_reduce_w(
    const float* __restrict__ ws, unsigned nb, int OUT, int C, float* __restrict__ gW,
    float* __restrict__ gb, float* __restrict__ loss, float* __restrict__ loss_sum,
    float inv_count) {
  __shared__ float s_g[8][64];
  const int t = threadIdx.x, g = t >> 6, l = t & 63;
  const int CP = C + 1, stride = OUT * CP + 1;
  const int oc = blockIdx.x * 64 + l;
  const float* part = ws + HEAD_WS_HDR;
  const unsigned members = (unsigned)g < nb ? (nb - (unsigned)g + 7u) / 8u : 0u;
  float s = 0.f;
  if (oc < stride) {
    for (unsigned m0 = 0; m0 < members; m0 += 32) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u)
        v[u] = m0 + u < members ? part[(int64_t)(g + 8u * (m0 + u)) * stride + oc] : 0.f;
#pragma unroll
      for (int u = 0; u < 32; ++u) s += v[u];
    }
  }
  s_g[g][l] = s;
  __syncthreads();
  if (g != 0 || oc >= stride) return;
  const int groups = nb < 8u ? (int)nb : 8;
  float v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = u < groups ? s_g[u][l] : 0.f;
  const float r = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
  if (oc == OUT * CP) {
    loss[0] = r * inv_count;
    if (loss_sum) loss_sum[0] += r * inv_count;
  } else {
    const int o = oc / CP, c = oc - o * CP;
    if (c < C) {
      if (gW) gW[o * C + c] += r;
    } else if (gb) {
      gb[o] += r;
    }
  }
}

// rows per wave of k_head_mse_train_w: enough waves to fill the chip once
// (<= 256 blocks of 4 waves)
static inline int head_w_rows(int64_t N) { return (int)std::max<int64_t>(1, (N + 1023) / 1024); }
static inline int head_w_kc(int C) {
  const int kc = (C + 63) / 64;
  return kc <= 1 ? 1 : kc <= 2 ? 2 : kc <= 4 ? 4 : kc <= 8 ? 8 : 16;
}
static inline bool head_w_ok(int C, int O) { return O <= 4 && O * head_w_kc(C) <= 32; }
static inline int64_t head_w_blocks(int64_t N) {
  const int64_t rw = head_w_rows(N);
  return (N + 4 * rw - 1) / (4 * rw);
}

}  // namespace sv2n

using namespace sv2n;

static int head_check(int64_t N, int C, int out_ch) {
  if (N <= 0 || C <= 0 || out_ch <= 0) return SV2N_ERR_ARG;
  if (out_ch > HEAD_MAX_OUT || C > HEAD_MAX_IN || head_rows_per_block(C, out_ch, N) == 0)
    return SV2N_ERR_SHAPE;
  if (N / head_rows_per_block(C, out_ch, N) >= 0x7fffffff) return SV2N_ERR_SHAPE;
  return 0;
}

template <typename K>
static void raise_head_lds(K kernel) {
  (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            140 * 1024);
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

extern "C" int sv2n_head_fwd(const float* x, int64_t num_rows, int in_features,
                             const float* weight, const float* bias, int out_features,
                             float* out, hipStream_t stream) {
  const int out_ch = out_features;
  if (!x || !weight || !out) return SV2N_ERR_ARG;
  if (int rc = head_check(num_rows, in_features, out_ch)) return rc;
  const int R = head_rows_per_block(in_features, out_ch, num_rows);
  const unsigned grid = (unsigned)((num_rows + R - 1) / R);
  const size_t lds = head_lds_bytes(in_features, out_ch, num_rows);
  SV2N_HEAD_DISPATCH(k_head_fwd, dim3(grid), dim3(256), lds, stream, x, num_rows, in_features,
                     weight, bias, out, R)
  return (int)hipGetLastError();
}

static int64_t head_bwd_blocks(int64_t num_rows, int C, int O) {
  const int R = head_rows_per_block(C, O, num_rows);
  return R ? (num_rows + R - 1) / R : 0;
}

extern "C" int64_t sv2n_head_bwd_workspace(int64_t num_rows, int in_features, int out_features) {
  return HEAD_WS_HDR + head_bwd_blocks(num_rows, in_features, out_features) *
                           (int64_t)out_features * (in_features + 1);
}

static int head_bwd_launch(const float* x, int64_t num_rows, int in_features, const float* weight,
                           int out_ch, const float* src, float scale, const float* dscale,
                           float* dx, float* g_weight, float* g_bias, float* workspace,
                           int64_t workspace_floats, hipStream_t stream) {
  if (!x || !weight || !src || !dx || !workspace) return SV2N_ERR_ARG;
  if (int rc = head_check(num_rows, in_features, out_ch)) return rc;
  const int64_t nb = head_bwd_blocks(num_rows, in_features, out_ch);
  if (workspace_floats < sv2n_head_bwd_workspace(num_rows, in_features, out_ch))
    return SV2N_ERR_WORKSPACE;
  if ((uintptr_t)workspace & 15) return SV2N_ERR_ALIGN;
  const int R = head_rows_per_block(in_features, out_ch, num_rows);
  const size_t lds = head_lds_bytes(in_features, out_ch, num_rows);
  SV2N_HEAD_DISPATCH(k_head_bwd, dim3((unsigned)nb), dim3(256), lds, stream, x, num_rows,
                     in_features, weight, src, scale, dscale, dx, workspace, g_weight, g_bias, R)
  return (int)hipGetLastError();
}

extern "C" int sv2n_head_bwd(const float* x, int64_t num_rows, int in_features,
                             const float* weight, int out_features, const float* dout, float* dx,
                             float* g_weight, float* g_bias, float* workspace,
                             int64_t workspace_floats, hipStream_t stream) {
  return head_bwd_launch(x, num_rows, in_features, weight, out_features, dout, 1.f, nullptr, dx,
                         g_weight, g_bias, workspace, workspace_floats, stream);
}

extern "C" int64_t sv2n_head_mse_workspace(int64_t num_rows, int in_features, int out_features) {
  const int64_t nb = head_bwd_blocks(num_rows, in_features, out_features);
  return std::max<int64_t>(sv2n_head_bwd_workspace(num_rows, in_features, out_features),
                           HEAD_WS_HDR + nb);
}

extern "C" int sv2n_head_mse_fwd(const float* x, int64_t num_rows, int in_features,
                                 const float* weight, const float* bias, int out_features,
                                 const float* target, float* yhat, float* diff, float* loss,
                                 float* loss_sum, float* workspace, int64_t workspace_floats,
                                 hipStream_t stream) {
  const int out_ch = out_features;
  if (!x || !weight || !target || !diff || !loss || !workspace) return SV2N_ERR_ARG;
  if (int rc = head_check(num_rows, in_features, out_ch)) return rc;
  if (workspace_floats < sv2n_head_mse_workspace(num_rows, in_features, out_ch))
    return SV2N_ERR_WORKSPACE;
  if ((uintptr_t)workspace & 15) return SV2N_ERR_ALIGN;
  const int R = head_rows_per_block(in_features, out_ch, num_rows);
  const unsigned grid = (unsigned)((num_rows + R - 1) / R);
  const size_t lds = head_lds_bytes(in_features, out_ch, num_rows);
  const float inv_count = 1.f / (float)(num_rows * out_ch);
  SV2N_HEAD_DISPATCH(k_head_mse_fwd, dim3(grid), dim3(256), lds, stream, x, num_rows,
                     in_features, weight, bias, target, yhat, diff, workspace, loss, loss_sum,
                     inv_count, R)
  return (int)hipGetLastError();
}

extern "C" int sv2n_head_mse_bwd(const float* x, int64_t num_rows, int in_features,
                                 const float* weight, int out_features, const float* diff,
                                 const float* grad_loss, float* dx, float* g_weight,
                                 float* g_bias, float* workspace, int64_t workspace_floats,
                                 hipStream_t stream) {
  const float scale = 2.f / (float)(num_rows * (int64_t)out_features);
  return head_bwd_launch(x, num_rows, in_features, weight, out_features, diff, scale, grad_loss,
                         dx, g_weight, g_bias, workspace, workspace_floats, stream);
}

extern "C" int64_t sv2n_head_mse_train_workspace(int64_t num_rows, int in_features,
                                                 int out_features) {
  const int64_t stride = (int64_t)out_features * (in_features + 1) + 1;
  if (head_w_ok(in_features, out_features))  // block partials + 8 group slabs
    return HEAD_WS_HDR + (head_w_blocks(num_rows) + 8) * stride;
  return HEAD_WS_HDR + head_bwd_blocks(num_rows, in_features, out_features) * stride;
}

template <bool DEFER>
static int head_w_launch(const float* x, int64_t num_rows, int C, const float* weight,
                         const float* bias, int out_ch, const float* target, float* loss,
                         float* loss_sum, float* dx, float* g_weight, float* g_bias,
                         float* workspace, hipStream_t stream) {
  const float inv_count = 1.f / (float)(num_rows * out_ch);
  const float scale = 2.f / (float)(num_rows * (int64_t)out_ch);
  const int RW = head_w_rows(num_rows), kc = head_w_kc(C);
  const unsigned grid = (unsigned)head_w_blocks(num_rows);
  const size_t lds = sizeof(float) * 4 * ((size_t)out_ch * (C + 1) + 1);
#define SV2N_HW(O, K)                                                                           \
  if (out_ch == O && kc == K) {                                                                 \
    hipLaunchKernelGGL((k_head_mse_train_w<O, K, DEFER>), dim3(grid), dim3(256), lds, stream,  \
                       x, num_rows, C, weight, bias, target, dx, workspace, g_weight, g_bias,   \
                       loss, loss_sum, inv_count, scale, RW);                                   \
    return (int)hipGetLastError();                                                              \
  }
  SV2N_HW(1, 1) SV2N_HW(1, 2) SV2N_HW(1, 4) SV2N_HW(1, 8) SV2N_HW(1, 16)
  SV2N_HW(2, 1) SV2N_HW(2, 2) SV2N_HW(2, 4) SV2N_HW(2, 8) SV2N_HW(2, 16)
  SV2N_HW(3, 1) SV2N_HW(3, 2) SV2N_HW(3, 4) SV2N_HW(3, 8)
  SV2N_HW(4, 1) SV2N_HW(4, 2) SV2N_HW(4, 4) SV2N_HW(4, 8)
#undef SV2N_HW
  return SV2N_ERR_SHAPE;
}

extern "C" int sv2n_head_mse_train_rows(const float* x, int64_t num_rows, int in_features,
                                        const float* weight, const float* bias, int out_features,
                                        const float* target, float* dx, float* workspace,
                                        int64_t workspace_floats, hipStream_t stream) {
  const int out_ch = out_features;
  if (!x || !weight || !target || !dx || !workspace) return SV2N_ERR_ARG;
  if (int rc = head_check(num_rows, in_features, out_ch)) return rc;
  if (!head_w_ok(in_features, out_ch)) return SV2N_ERR_SHAPE;
  if (workspace_floats < sv2n_head_mse_train_workspace(num_rows, in_features, out_ch))
    return SV2N_ERR_WORKSPACE;
  if ((uintptr_t)workspace & 15) return SV2N_ERR_ALIGN;
  return head_w_launch<true>(x, num_rows, in_features, weight, bias, out_ch, target, nullptr,
                             nullptr, dx, nullptr, nullptr, workspace, stream);
}

extern "C" int sv2n_head_mse_train_reduce(const float* workspace, int64_t workspace_floats,
                                          int64_t num_rows, int in_features, int out_features,
                                          float* loss, float* loss_sum, float* g_weight,
                                          float* g_bias, hipStream_t stream) {
  const int out_ch = out_features;
  if (!workspace || !loss) return SV2N_ERR_ARG;
  if (int rc = head_check(num_rows, in_features, out_ch)) return rc;
  if (!head_w_ok(in_features, out_ch)) return SV2N_ERR_SHAPE;
  if (workspace_floats < sv2n_head_mse_train_workspace(num_rows, in_features, out_ch))
    return SV2N_ERR_WORKSPACE;
  const int stride = out_ch * (in_features + 1) + 1;
  hipLaunchKernelGGL(k_head_mse_reduce_w, dim3((unsigned)((stride + 63) / 64)), dim3(512), 0,
                     stream, workspace, (unsigned)head_w_blocks(num_rows), out_ch, in_features,
                     g_weight, g_bias, loss, loss_sum, 1.f / (float)(num_rows * out_ch));
  return (int)hipGetLastError();
}

extern "C" int sv2n_head_mse_train(const float* x, int64_t num_rows, int in_features,
                                   const float* weight, const float* bias, int out_features,
                                   const float* target, float* loss, float* loss_sum, float* dx,
                                   float* g_weight, float* g_bias, float* workspace,
                                   int64_t workspace_floats, hipStream_t stream) {
  const int out_ch = out_features;
  if (!x || !weight || !target || !loss || !dx || !workspace) return SV2N_ERR_ARG;
  if (int rc = head_check(num_rows, in_features, out_ch)) return rc;
  if (workspace_floats < sv2n_head_mse_train_workspace(num_rows, in_features, out_ch))
    return SV2N_ERR_WORKSPACE;
  if ((uintptr_t)workspace & 15) return SV2N_ERR_ALIGN;
  const float inv_count = 1.f / (float)(num_rows * out_ch);
  const float scale = 2.f / (float)(num_rows * (int64_t)out_ch);
  if (head_w_ok(in_features, out_ch))
    return head_w_launch<false>(x, num_rows, in_features, weight, bias, out_ch, target, loss,
                                loss_sum, dx, g_weight, g_bias, workspace, stream);
  const int R = head_rows_per_block(in_features, out_ch, num_rows);
  const unsigned grid = (unsigned)((num_rows + R - 1) / R);
  const size_t lds = head_lds_bytes(in_features, out_ch, num_rows);
  SV2N_HEAD_DISPATCH(k_head_mse_train, dim3(grid), dim3(256), lds, stream, x, num_rows,
                     in_features, weight, bias, target, dx, workspace, g_weight, g_bias, loss,
                     loss_sum, inv_count, scale, R)
  return (int)hipGetLastError();
}
