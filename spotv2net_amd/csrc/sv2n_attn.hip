// Fused per-graph GAT attention (forward + backward) for graphs of n <= 32
// nodes — the dense-block form of PyG 2.3.0 GATConv message passing that
// SpotV2Net runs on its fully connected 30-asset graphs
// (reference utils/models.py:146 -> GATConv.forward).
//
// One workgroup (256 threads = 4 waves) owns one graph g.  Per head h the
// incoming edges of target i form row i of a 32-padded n x n matrix, so
// PyG's per-target softmax (scatter_max / scatter_sum over edge_index[1]) is a
// row softmax reduced inside one 32-lane half of a wave, the self loop with
// fill_value='mean' is the mean of the row's stored edge logits (linearity of
// lin_edge), and the scatter-add aggregation is the row-by-column product
// P(n x n) · xs_h(n x C) with P broadcast from LDS.
//
// HBM traffic per graph (fwd): xs rows n*ldx*4 B read once, ae slab n*n*H*4 B,
// y rows written once, P saved (n*n*H*4 B).
#include "sv2n_common.h"

namespace sv2n {

constexpr int ATT_THREADS = 256;

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
template <int ACT, bool CONCAT>
__global__ __launch_bounds__(ATT_THREADS) void k_attn_fwd(
    const float* __restrict__ xs, int ldx, const float* __restrict__ ae,
    const uint32_t* __restrict__ rowmask, const float* __restrict__ bias,
    const uint8_t* __restrict__ keep, float keep_scale, float* __restrict__ y,
    float* __restrict__ psave, int n, int H, int C, float slope) {
  __shared__ __attribute__((aligned(16))) float sPT[SV2N_MAX_HEADS][32][SV2N_PSTR];  // [h][j][i]
  __shared__ float sA[SV2N_MAX_HEADS][32];
  __shared__ float sD[SV2N_MAX_HEADS][32];

  const int g = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t row0 = (int64_t)g * n;
  const int HC = H * C;

  for (int idx = t; idx < H * 32; idx += ATT_THREADS) {
    const int h = idx >> 5, j = idx & 31;
    float as = 0.f, ad = 0.f;
    if (j < n) {
      const float* r = xs + (row0 + j) * ldx + HC;
      as = r[h];
      ad = r[H + h];
    }
    sA[h][j] = as;
    sD[h][j] = ad;
  }
  __syncthreads();

  // ---- per-target softmax, two rows per wave instruction ----
  const int R = H * n;
  const int half = lane >> 5, j = lane & 31;
  for (int rb = wave * 2; rb < R; rb += 8) {  // wave-uniform trip count
    const int r = rb + half;
    const bool rv = r < R;
    const int h = rv ? r / n : 0;
    const int i = rv ? r - h * n : 0;
    const uint32_t bits = row_bits(rowmask, row0 + i, n, i);
    const bool off = rv && j < n && j != i && ((bits >> j) & 1u);
    const bool valid = rv && j < n && (j == i || off);
    float s = sA[h][j] + sD[h][i];
    if (ae) {
      const float e = off ? ae[((row0 + i) * n + j) * H + h] : 0.f;
      const float esum = red32_sum(e);
      const int cnt = __popc(bits);
      const float loopv = cnt > 0 ? esum / (float)cnt : 0.f;
      s += (j == i) ? loopv : e;
    }
    const bool neg = !(s > 0.f);
    const float lr = neg ? s * slope : s;
    const float mx = red32_max(valid ? lr : -INFINITY);
    const float ex = valid ? expf(lr - mx) : 0.f;
    const float den = red32_sum(ex);
    const float p = ex / (den + 1e-16f);
    float pd = valid ? p : 0.f;
    if (rv && j < n) {  // absent edges store 0 so the backward reads finite P
      const int64_t pidx = (((int64_t)g * H + h) * n + i) * n + j;
      psave[pidx] = valid ? (neg ? -p : p) : 0.f;
      if (keep && valid) pd = keep[pidx] ? p * keep_scale : 0.f;
    }
    if (rv) sPT[h][j][i] = pd;
  }
  __syncthreads();

  // ---- aggregation + head combine + bias + activation ----
  const int OC = CONCAT ? HC : C;
  for (int oc = t; oc < OC; oc += ATT_THREADS) {
    float sum[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) sum[i] = 0.f;
    const int h0 = CONCAT ? oc / C : 0;
    const int h1 = CONCAT ? h0 + 1 : H;
    for (int h = h0; h < h1; ++h) {
      const int col = CONCAT ? oc : h * C + oc;
      float xv[32];
#pragma unroll
      for (int jj = 0; jj < 32; ++jj) xv[jj] = (jj < n) ? xs[(row0 + jj) * ldx + col] : 0.f;
      float acc[32];
#pragma unroll
      for (int i = 0; i < 32; ++i) acc[i] = 0.f;
#pragma unroll
      for (int jj = 0; jj < 32; ++jj) {
        if (jj < n) {
          const float4* pr = reinterpret_cast<const float4*>(&sPT[h][jj][0]);
#pragma unroll
          for (int i4 = 0; i4 < 8; ++i4) {
            const float4 pv = pr[i4];
            acc[4 * i4 + 0] = fmaf(pv.x, xv[jj], acc[4 * i4 + 0]);
            acc[4 * i4 + 1] = fmaf(pv.y, xv[jj], acc[4 * i4 + 1]);
            acc[4 * i4 + 2] = fmaf(pv.z, xv[jj], acc[4 * i4 + 2]);
            acc[4 * i4 + 3] = fmaf(pv.w, xv[jj], acc[4 * i4 + 3]);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 32; ++i) sum[i] += acc[i];
    }
    const float b = bias ? bias[oc] : 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      if (i < n) {
        const float z = (CONCAT ? sum[i] : sum[i] / (float)H) + b;
        y[(row0 + i) * OC + oc] = act_fwd<ACT>(z);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward
// dynamic LDS (floats): sPd[H][32][PSTR] | sG[H][32][PSTR] | sO[H][CK][PSTR] | sX[H][CK][PSTR]
// ---------------------------------------------------------------------------
constexpr int BWD_CK = 16;

template <int ACT, bool CONCAT>
__global__ __launch_bounds__(ATT_THREADS) void k_attn_bwd(
    const float* __restrict__ dy, const float* __restrict__ y, const float* __restrict__ xs,
    int ldx, const float* __restrict__ psave, const uint8_t* __restrict__ keep, float keep_scale,
    const uint32_t* __restrict__ rowmask, float* __restrict__ dxs, float* __restrict__ dae,
    float* __restrict__ dbias_part, int n, int H, int C, float slope) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int PS = 32 * SV2N_PSTR;
  float* sPd = smem;                       // post-dropout P   [h][i][j]
  float* sG = sPd + H * PS;                // dP, then dL      [h][i][j]
  float* sO = sG + H * PS;                 // dOut chunk       [h][c][i]
  float* sX = sO + H * BWD_CK * SV2N_PSTR; // xs chunk         [h][c][j]

  const int g = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t row0 = (int64_t)g * n;
  const int HC = H * C;
  const int OC = CONCAT ? HC : C;
  const float invH = 1.f / (float)H;
  const int64_t pbase = (int64_t)g * H * n * n;

  // phase 1: post-dropout probabilities
  for (int idx = t; idx < H * n * n; idx += ATT_THREADS) {
    const int h = idx / (n * n);
    const int rem = idx - h * n * n;
    const int i = rem / n, j = rem - i * n;
    const float p = fabsf(psave[pbase + idx]);
    float pd = p;
    if (keep) pd = keep[pbase + idx] ? p * keep_scale : 0.f;
    sPd[h * PS + i * SV2N_PSTR + j] = pd;
  }

  // phase 2: dP[h][i][j] = Σ_c dOut[i][h][c] · xs[j][h][c], 4x4 register tiles
  const int ntile = H * 64;
  float acc0[16], acc1[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) { acc0[k] = 0.f; acc1[k] = 0.f; }
  for (int c0 = 0; c0 < C; c0 += BWD_CK) {
    const int ck = min(BWD_CK, C - c0);
    __syncthreads();
    for (int idx = t; idx < H * 32 * BWD_CK; idx += ATT_THREADS) {
      const int c = idx % BWD_CK;
      const int i = (idx / BWD_CK) & 31;
      const int h = idx / (BWD_CK * 32);
      float vo = 0.f, vx = 0.f;
      if (i < n && c < ck) {
        const int col = h * C + c0 + c;
        vx = xs[(row0 + i) * ldx + col];
        const int oc = CONCAT ? col : c0 + c;
        const float dz = act_bwd<ACT>(dy[(row0 + i) * OC + oc], y[(row0 + i) * OC + oc]);
        vo = CONCAT ? dz : dz * invH;
      }
      sO[(h * BWD_CK + c) * SV2N_PSTR + i] = vo;
      sX[(h * BWD_CK + c) * SV2N_PSTR + i] = vx;
    }
    __syncthreads();
#pragma unroll
    for (int rep = 0; rep < 2; ++rep) {
      const int tt = t + rep * ATT_THREADS;
      if (tt < ntile) {
        const int h = tt >> 6, ib = (tt >> 3) & 7, jb = tt & 7;
        float* acc = rep == 0 ? acc0 : acc1;
        for (int c = 0; c < ck; ++c) {
          const float4 a = *reinterpret_cast<const float4*>(sO + (h * BWD_CK + c) * SV2N_PSTR + 4 * ib);
          const float4 b = *reinterpret_cast<const float4*>(sX + (h * BWD_CK + c) * SV2N_PSTR + 4 * jb);
          const float av[4] = {a.x, a.y, a.z, a.w};
          const float bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int z = 0; z < 4; ++z) acc[4 * x + z] = fmaf(av[x], bv[z], acc[4 * x + z]);
        }
      }
    }
  }
#pragma unroll
  for (int rep = 0; rep < 2; ++rep) {
    const int tt = t + rep * ATT_THREADS;
    if (tt < ntile) {
      const int h = tt >> 6, ib = (tt >> 3) & 7, jb = tt & 7;
      const float* acc = rep == 0 ? acc0 : acc1;
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int z = 0; z < 4; ++z) sG[h * PS + (4 * ib + x) * SV2N_PSTR + 4 * jb + z] = acc[4 * x + z];
    }
  }
  __syncthreads();

  // phase 3: softmax + leaky_relu backward per target row, self-loop share,
  //          dAE, d a_dst
  const int R = H * n;
  const int half = lane >> 5, j = lane & 31;
  for (int rb = wave * 2; rb < R; rb += 8) {
    const int r = rb + half;
    const bool rv = r < R;
    const int h = rv ? r / n : 0;
    const int i = rv ? r - h * n : 0;
    const uint32_t bits = row_bits(rowmask, row0 + i, n, i);
    const bool off = rv && j < n && j != i && ((bits >> j) & 1u);
    const bool valid = rv && j < n && (j == i || off);
    const int64_t pidx = pbase + ((int64_t)h * n + i) * n + j;
    const float ps = valid ? psave[pidx] : 0.f;
    const float p = fabsf(ps);
    const bool neg = signbit(ps);
    float dp = valid ? sG[h * PS + i * SV2N_PSTR + j] : 0.f;
    if (keep) dp = (valid && keep[pidx]) ? dp * keep_scale : 0.f;
    const float tsum = red32_sum(p * dp);
    const float ds = p * (dp - tsum);
    const float dl = valid ? (neg ? ds * slope : ds) : 0.f;
    const float dad = red32_sum(dl);
    const float dlii = __shfl(dl, (lane & 32) | i, 64);
    if (dae && rv && j < n) {
      const int cnt = __popc(bits);
      const float share = cnt > 0 ? dlii / (float)cnt : 0.f;
      dae[((row0 + i) * n + j) * H + h] = off ? dl + share : 0.f;
    }
    if (rv && j == 0) dxs[(row0 + i) * ldx + HC + H + h] = dad;
    if (rv) sG[h * PS + i * SV2N_PSTR + j] = dl;
  }
  __syncthreads();

  // phase 4: d a_src[j][h] = Σ_i dL[h][i][j]; zero the padding columns
  for (int idx = t; idx < H * 32; idx += ATT_THREADS) {
    const int h = idx >> 5, jj = idx & 31;
    if (jj < n) {
      float s = 0.f;
      for (int i = 0; i < n; ++i) s += sG[h * PS + i * SV2N_PSTR + jj];
      dxs[(row0 + jj) * ldx + HC + h] = s;
    }
  }
  const int npad = ldx - (HC + 2 * H);
  for (int idx = t; idx < n * npad; idx += ATT_THREADS) {
    const int rr = idx / npad;
    dxs[(row0 + rr) * ldx + HC + 2 * H + (idx - rr * npad)] = 0.f;
  }

  // phase 5: dxs[j][h*C+c] = Σ_i Pd[h][i][j] · dOut[i][h][c]; bias partials
  for (int oc = t; oc < HC; oc += ATT_THREADS) {
    const int h = oc / C;
    const int c = oc - h * C;
    const int ycol = CONCAT ? oc : c;
    float dz[32];
#pragma unroll
    for (int i = 0; i < 32; ++i)
      dz[i] = (i < n) ? act_bwd<ACT>(dy[(row0 + i) * OC + ycol], y[(row0 + i) * OC + ycol]) : 0.f;
    if (CONCAT || h == 0) {
      float bsum = 0.f;
#pragma unroll
      for (int i = 0; i < 32; ++i) bsum += dz[i];
      dbias_part[(int64_t)g * OC + ycol] = bsum;
    }
    float acc[32];
#pragma unroll
    for (int jj = 0; jj < 32; ++jj) acc[jj] = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      if (i < n) {
        const float d = CONCAT ? dz[i] : dz[i] * invH;
        const float4* pr = reinterpret_cast<const float4*>(sPd + h * PS + i * SV2N_PSTR);
#pragma unroll
        for (int j4 = 0; j4 < 8; ++j4) {
          const float4 pv = pr[j4];
          acc[4 * j4 + 0] = fmaf(pv.x, d, acc[4 * j4 + 0]);
          acc[4 * j4 + 1] = fmaf(pv.y, d, acc[4 * j4 + 1]);
          acc[4 * j4 + 2] = fmaf(pv.z, d, acc[4 * j4 + 2]);
          acc[4 * j4 + 3] = fmaf(pv.w, d, acc[4 * j4 + 3]);
        }
      }
    }
#pragma unroll
    for (int jj = 0; jj < 32; ++jj)
      if (jj < n) dxs[(row0 + jj) * ldx + oc] = acc[jj];
  }
}

}  // namespace sv2n

// ============================ C-ABI ========================================
using namespace sv2n;

template <int ACT, bool CONCAT>
static void launch_fwd(int64_t B, hipStream_t st, const float* xs, int ldx, const float* ae,
                       const uint32_t* rowmask, const float* bias, const uint8_t* keep,
                       float keep_scale, float* y, float* psave, int n, int H, int C, float slope) {
  hipLaunchKernelGGL((k_attn_fwd<ACT, CONCAT>), dim3((unsigned)B), dim3(ATT_THREADS), 0, st, xs,
                     ldx, ae, rowmask, bias, keep, keep_scale, y, psave, n, H, C, slope);
}

template <int ACT, bool CONCAT>
static void launch_bwd(int64_t B, hipStream_t st, size_t lds, const float* dy, const float* y,
                       const float* xs, int ldx, const float* psave, const uint8_t* keep,
                       float keep_scale, const uint32_t* rowmask, float* dxs, float* dae,
                       float* dbias, int n, int H, int C, float slope) {
  static bool raised = false;
  if (!raised && lds > 65536) {
    (void)hipFuncSetAttribute((const void*)k_attn_bwd<ACT, CONCAT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    raised = true;
  }
  hipLaunchKernelGGL((k_attn_bwd<ACT, CONCAT>), dim3((unsigned)B), dim3(ATT_THREADS), lds, st, dy,
                     y, xs, ldx, psave, keep, keep_scale, rowmask, dxs, dae, dbias, n, H, C, slope);
}

static int check_attn_args(int64_t B, int n, int H, int C, int ldx, int act) {
  if (B <= 0 || C <= 0) return SV2N_ERR_ARG;
  if (n < 1 || n > SV2N_MAX_N || H < 1 || H > SV2N_MAX_HEADS || act < 0 || act > 3)
    return SV2N_ERR_SHAPE;
  if (ldx < H * C + 2 * H) return SV2N_ERR_SHAPE;
  return 0;
}

#define SV2N_DISPATCH_ACT(FN, CONCAT, ...)              \
  switch (act) {                                        \
    case 0: FN<0, CONCAT>(__VA_ARGS__); break;          \
    case 1: FN<1, CONCAT>(__VA_ARGS__); break;          \
    case 2: FN<2, CONCAT>(__VA_ARGS__); break;          \
    default: FN<3, CONCAT>(__VA_ARGS__); break;         \
  }

extern "C" int sv2n_gat_attn_fwd(const float* xs, int ldx, const float* ae,
                                 const uint32_t* rowmask, const float* bias, const uint8_t* keep,
                                 float keep_scale, float* y, float* psave, int64_t num_graphs,
                                 int n, int heads, int channels, int concat, int act,
                                 float negative_slope, hipStream_t stream) {
  if (!xs || !y || !psave) return SV2N_ERR_ARG;
  if (int rc = check_attn_args(num_graphs, n, heads, channels, ldx, act)) return rc;
  if (concat) {
    SV2N_DISPATCH_ACT(launch_fwd, true, num_graphs, stream, xs, ldx, ae, rowmask, bias, keep,
                      keep_scale, y, psave, n, heads, channels, negative_slope)
  } else {
    SV2N_DISPATCH_ACT(launch_fwd, false, num_graphs, stream, xs, ldx, ae, rowmask, bias, keep,
                      keep_scale, y, psave, n, heads, channels, negative_slope)
  }
  return (int)hipGetLastError();
}

extern "C" int sv2n_gat_attn_bwd(const float* dy, const float* y, const float* xs, int ldx,
                                 const float* psave, const uint8_t* keep, float keep_scale,
                                 const uint32_t* rowmask, float* dxs, float* dae,
                                 float* dbias_partial, int64_t num_graphs, int n, int heads,
                                 int channels, int concat, int act, float negative_slope,
                                 hipStream_t stream) {
  if (!dy || !y || !xs || !psave || !dxs || !dbias_partial) return SV2N_ERR_ARG;
  if (int rc = check_attn_args(num_graphs, n, heads, channels, ldx, act)) return rc;
  const size_t lds = sizeof(float) * (size_t)heads * (2 * 32 * SV2N_PSTR + 2 * BWD_CK * SV2N_PSTR);
  if (lds > 160 * 1024) return SV2N_ERR_SHAPE;
  if (concat) {
    SV2N_DISPATCH_ACT(launch_bwd, true, num_graphs, stream, lds, dy, y, xs, ldx, psave, keep,
                      keep_scale, rowmask, dxs, dae, dbias_partial, n, heads, channels,
                      negative_slope)
  } else {
    SV2N_DISPATCH_ACT(launch_bwd, false, num_graphs, stream, lds, dy, y, xs, ldx, psave, keep,
                      keep_scale, rowmask, dxs, dae, dbias_partial, n, heads, channels,
                      negative_slope)
  }
  return (int)hipGetLastError();
}
