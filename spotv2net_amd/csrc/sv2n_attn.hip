// Fused per-graph GAT attention (forward + backward) for graphs of n <= 32
// nodes — the dense-block form of PyG 2.3.0 GATConv message passing that
// SpotV2Net runs on its fully connected 30-asset graphs
// (reference utils/models.py:146 -> GATConv.forward).
//
// One workgroup (256 threads = 4 waves) owns one graph g.  Per head h the
// incoming edges of target i form row i of a 32-padded n x n matrix, so
// PyG's per-target softmax (scatter_max / scatter_sum over edge_index[1]) is a
// row softmax reduced inside one 32-lane half of a wave, and the self loop with
// fill_value='mean' is the mean of the row's stored edge logits (linearity of
// lin_edge).  The message passing products are 32x32 MFMA tiles
// (v_mfma_f32_32x32x2_f32: exact f32, k-ordered fma chains):
//   forward    out_h   = P_h (n x n) · xs_h (n x C)             (scatter-add, a10)
//   backward   dP_hᵀ   = xs_h · dOut_hᵀ                        (message bwd)
//              dxs_h   = P_hᵀ · dOut_h                         (gather bwd)
// with P in LDS as [h][i][j] (row stride 33 floats: conflict-free for row and
// column fragment reads) and xs / dOut rows read coalesced from HBM.
//
// Saved probabilities / keep masks use a padded [g][h][32][32] layout
// (16-B aligned rows); the sign bit of a saved probability records
// leaky_relu's negative side for the backward.
#include "sv2n_common.h"

namespace sv2n {

constexpr int ATT_THREADS = 256;
constexpr int TS = 33;  // LDS tile row stride (floats)

typedef float floatx16 __attribute__((ext_vector_type(16)));

// C/D row of accumulator register r for lane half hf (32x32 MFMA layout)
__device__ __forceinline__ int crow(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------------------
// forward
// LDS: sP[H][32][TS] | sA[H][32] | sD[H][32]
// ---------------------------------------------------------------------------
template <int ACT, bool CONCAT>
__global__ __launch_bounds__(ATT_THREADS) void k_attn_fwd(
    const float* __restrict__ xs, int ldx, const float* __restrict__ ae,
    const uint32_t* __restrict__ rowmask, const float* __restrict__ bias,
    const uint8_t* __restrict__ keep, float keep_scale, float* __restrict__ y,
    float* __restrict__ psave, int n, int H, int C, float slope) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sP = smem;
  float* sA = sP + H * 32 * TS;
  float* sD = sA + H * 32;

  const int g = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int half = lane >> 5, l32 = lane & 31;
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
    sA[idx] = as;
    sD[idx] = ad;
  }
  __syncthreads();

  // ---- per-target softmax over all 32 (padded) rows of every head ----
  const int j = l32;
  for (int rb = wave * 2; rb < H * 32; rb += 8) {
    const int r = rb + half;
    const int h = r >> 5, i = r & 31;
    const bool rv = i < n;
    const uint32_t bits = rv ? row_bits(rowmask, row0 + i, n, i) : 0u;
    const bool off = rv && j < n && j != i && ((bits >> j) & 1u);
    const bool valid = rv && j < n && (j == i || off);
    float s = sA[h * 32 + j] + sD[h * 32 + i];
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
    if (rv) {
      const int64_t pidx = (((int64_t)g * H + h) * 32 + i) * 32 + j;
      psave[pidx] = valid ? (neg ? -p : p) : 0.f;
      if (keep && valid) pd = keep[pidx] ? p * keep_scale : 0.f;
    }
    sP[(h * 32 + i) * TS + j] = pd;
  }
  __syncthreads();

  // ---- aggregation on MFMA: acc[i][c] = Σ_j P[h][i][j] · xs[j][h*C + c] ----
  const int nck = (C + 31) / 32;
  const int items = CONCAT ? H * nck : nck;
  const int OC = CONCAT ? HC : C;
  const float invH = 1.f / (float)H;
  for (int it = wave; it < items; it += 4) {
    const int hb = CONCAT ? it / nck : 0;
    const int c0 = 32 * (CONCAT ? it - hb * nck : it);
    const int he = CONCAT ? hb + 1 : H;
    const int c = c0 + l32;
    const bool cok = c < C;
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    for (int h = hb; h < he; ++h) {
      float bv[16];
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const int jj = 2 * kk + half;
        bv[kk] = (jj < n && cok) ? xs[(row0 + jj) * ldx + h * C + c] : 0.f;
      }
      const float* prow = sP + (h * 32 + l32) * TS + half;
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(prow[2 * kk], bv[kk], acc, 0, 0, 0);
    }
    if (cok) {
      const int oc = CONCAT ? hb * C + c : c;
      const float b = bias ? bias[oc] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = crow(r, half);
        if (i < n) {
          const float z = (CONCAT ? acc[r] : acc[r] * invH) + b;
          y[(row0 + i) * OC + oc] = act_fwd<ACT>(z);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward
// LDS: sP[H][32][TS] (post-dropout P) | per wave: tO[32][TS] (dOut chunk, [i][c]),
//      tX[32][TS] (xs chunk [j][c], later dLᵀ [j][i])
// ---------------------------------------------------------------------------
template <int ACT, bool CONCAT>
__global__ __launch_bounds__(ATT_THREADS) void k_attn_bwd(
    const float* __restrict__ dy, const float* __restrict__ y, const float* __restrict__ xs,
    int ldx, const float* __restrict__ psave, const uint8_t* __restrict__ keep, float keep_scale,
    const uint32_t* __restrict__ rowmask, float* __restrict__ dxs, float* __restrict__ dae,
    float* __restrict__ dbias_part, int n, int H, int C, float slope) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int g = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int64_t row0 = (int64_t)g * n;
  const int HC = H * C;
  const int OC = CONCAT ? HC : C;
  const float invH = 1.f / (float)H;
  const int64_t pbase = (int64_t)g * H * 1024;
  float* sP = smem;
  float* tO = sP + H * 32 * TS + wave * 2 * 32 * TS;
  float* tX = tO + 32 * TS;

  for (int idx = t; idx < H * 1024; idx += ATT_THREADS) {
    const int h = idx >> 10, i = (idx >> 5) & 31, jj = idx & 31;
    float pd = 0.f;
    if (i < n) {
      pd = fabsf(psave[pbase + idx]);
      if (keep) pd = keep[pbase + idx] ? pd * keep_scale : 0.f;
    }
    sP[(h * 32 + i) * TS + jj] = pd;
  }
  __syncthreads();

  for (int h = wave; h < H; h += 4) {
    floatx16 G;  // dPᵀ: G[j][i] = Σ_c xs[j][c] · dOut[i][c]
#pragma unroll
    for (int r = 0; r < 16; ++r) G[r] = 0.f;
    for (int c0 = 0; c0 < C; c0 += 32) {
      const int c = c0 + l32;
      const bool cok = c < C;
      const int ycol = CONCAT ? h * C + c : c;
      float bsum = 0.f;
#pragma unroll 4
      for (int s = 0; s < 16; ++s) {
        const int rr = half + 2 * s;
        const bool ok = rr < n && cok;
        const float dz = ok ? act_bwd<ACT>(dy[(row0 + rr) * OC + ycol], y[(row0 + rr) * OC + ycol])
                            : 0.f;
        bsum += dz;
        tO[rr * TS + l32] = CONCAT ? dz : dz * invH;
        tX[rr * TS + l32] = ok ? xs[(row0 + rr) * ldx + h * C + c] : 0.f;
      }
      bsum += __shfl_xor(bsum, 32, 64);
      if (half == 0 && cok && (CONCAT || h == 0)) dbias_part[(int64_t)g * OC + ycol] = bsum;
      lds_fence();
      // G += X · Oᵀ   (A[j][c] = tX[j][c], B[c][i] = tO[i][c])
      const float* xr = tX + l32 * TS + half;
      const float* orow = tO + l32 * TS + half;
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
        G = __builtin_amdgcn_mfma_f32_32x32x2f32(xr[2 * kk], orow[2 * kk], G, 0, 0, 0);
      // dxs chunk = Pdᵀ · O   (A[j][i] = sP[h][i][j], B[i][c] = tO[i][c])
      floatx16 D2;
#pragma unroll
      for (int r = 0; r < 16; ++r) D2[r] = 0.f;
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const int ii = 2 * kk + half;
        D2 = __builtin_amdgcn_mfma_f32_32x32x2f32(sP[(h * 32 + ii) * TS + l32], tO[ii * TS + l32],
                                                  D2, 0, 0, 0);
      }
      if (cok) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int jr = crow(r, half);
          if (jr < n) dxs[(row0 + jr) * ldx + h * C + c] = D2[r];
        }
      }
      lds_fence();  // tile reads retired before the next chunk overwrites them
    }

    // ---- softmax + leaky_relu backward on G: lane column i, rows j = crow(r, half) ----
    const int i = l32;
    const bool iv = i < n;
    const uint32_t bits = iv ? row_bits(rowmask, row0 + i, n, i) : 0u;
    const int64_t prow = pbase + ((int64_t)h * 32 + i) * 32;
    float ps[16];
    uint32_t kp[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int jb = 8 * q + 4 * half;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (iv) v = *reinterpret_cast<const float4*>(psave + prow + jb);
      ps[4 * q + 0] = v.x;
      ps[4 * q + 1] = v.y;
      ps[4 * q + 2] = v.z;
      ps[4 * q + 3] = v.w;
      kp[q] = (keep && iv) ? *reinterpret_cast<const uint32_t*>(keep + prow + jb) : 0u;
    }
    float dp[16];
    float tl = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jr = crow(r, half);
      const bool valid = iv && jr < n && (jr == i || ((bits >> jr) & 1u));
      float d = valid ? G[r] : 0.f;
      if (keep) d = ((kp[r >> 2] >> (8 * (r & 3))) & 0xffu) ? d * keep_scale : 0.f;
      dp[r] = d;
      tl += fabsf(ps[r]) * d;
    }
    tl += __shfl_xor(tl, 32, 64);
    float dl[16];
    float dad = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jr = crow(r, half);
      const bool valid = iv && jr < n && (jr == i || ((bits >> jr) & 1u));
      const float p = fabsf(ps[r]);
      const float ds = p * (dp[r] - tl);
      dl[r] = valid ? (signbit(ps[r]) ? ds * slope : ds) : 0.f;
      dad += dl[r];
    }
    dad += __shfl_xor(dad, 32, 64);
    if (half == 0 && iv) dxs[(row0 + i) * ldx + HC + H + h] = dad;
    // dl[i][i] sits in half (i>>2)&1, register (i&3) + 4*(i>>3)
    const int hi = (i >> 2) & 1, ri = (i & 3) + 4 * (i >> 3);
    float mine = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) mine = (r == ri) ? dl[r] : mine;
    const float other = __shfl_xor(mine, 32, 64);
    const float dlii = (half == hi) ? mine : other;
    if (dae && iv) {
      const int cnt = __popc(bits);
      const float share = cnt > 0 ? dlii / (float)cnt : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int jr = crow(r, half);
        if (jr < n)
          dae[((row0 + i) * n + jr) * H + h] =
              (jr != i && ((bits >> jr) & 1u)) ? dl[r] + share : 0.f;
      }
    }
    // d a_src[j] = Σ_i dL[i][j]: transpose through LDS (tX as [j][i])
#pragma unroll
    for (int r = 0; r < 16; ++r) tX[crow(r, half) * TS + i] = dl[r];
    lds_fence();
    if (lane < 32 && lane < n) {
      float s = 0.f;
      for (int ii = 0; ii < 32; ++ii) s += tX[lane * TS + ii];
      dxs[(row0 + lane) * ldx + HC + h] = s;
    }
    lds_fence();
  }

  const int npad = ldx - (HC + 2 * H);
  for (int idx = t; idx < n * npad; idx += ATT_THREADS) {
    const int rr = idx / npad;
    dxs[(row0 + rr) * ldx + HC + 2 * H + (idx - rr * npad)] = 0.f;
  }
}

}  // namespace sv2n

// ============================ C-ABI ========================================
using namespace sv2n;

static size_t fwd_lds(int H) { return sizeof(float) * ((size_t)H * 32 * TS + 2 * (size_t)H * 32); }
static size_t bwd_lds(int H) { return sizeof(float) * ((size_t)H * 32 * TS + 4 * 2 * 32 * TS); }

template <typename K>
static void raise_lds(K kernel, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
}

template <int ACT, bool CONCAT>
static void launch_fwd(int64_t B, hipStream_t st, const float* xs, int ldx, const float* ae,
                       const uint32_t* rowmask, const float* bias, const uint8_t* keep,
                       float keep_scale, float* y, float* psave, int n, int H, int C, float slope) {
  const size_t lds = fwd_lds(H);
  raise_lds(k_attn_fwd<ACT, CONCAT>, lds);
  hipLaunchKernelGGL((k_attn_fwd<ACT, CONCAT>), dim3((unsigned)B), dim3(ATT_THREADS), lds, st, xs,
                     ldx, ae, rowmask, bias, keep, keep_scale, y, psave, n, H, C, slope);
}

template <int ACT, bool CONCAT>
static void launch_bwd(int64_t B, hipStream_t st, const float* dy, const float* y,
                       const float* xs, int ldx, const float* psave, const uint8_t* keep,
                       float keep_scale, const uint32_t* rowmask, float* dxs, float* dae,
                       float* dbias, int n, int H, int C, float slope) {
  const size_t lds = bwd_lds(H);
  raise_lds(k_attn_bwd<ACT, CONCAT>, lds);
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
  if (concat) {
    SV2N_DISPATCH_ACT(launch_bwd, true, num_graphs, stream, dy, y, xs, ldx, psave, keep,
                      keep_scale, rowmask, dxs, dae, dbias_partial, n, heads, channels,
                      negative_slope)
  } else {
    SV2N_DISPATCH_ACT(launch_bwd, false, num_graphs, stream, dy, y, xs, ldx, psave, keep,
                      keep_scale, rowmask, dxs, dae, dbias_partial, n, heads, channels,
                      negative_slope)
  }
  return (int)hipGetLastError();
}
