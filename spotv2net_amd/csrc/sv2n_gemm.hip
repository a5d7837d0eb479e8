// f32-input MFMA GEMM for the GATConv projections (PyG lin_src, SURVEY §8a
// row a6) and their backward products.
//
//   C[M][N] = Σ_k A(m,k) · B(n,k)
//   A(m,k) = A[m*lda + k]  (a_kmajor = 1)   or  A[k*lda + m]  (a_kmajor = 0)
//   B(n,k) = B[n*ldb + k]  (b_kmajor = 1)   or  B[k*ldb + n]  (b_kmajor = 0)
//
// gfx950 has exact f32 MFMA (v_mfma_f32_16x16x4_f32: one rounding per product,
// k-ordered fma chain) at the f32 vector peak (157 TF).  Tiling:
//   kernel template: sv2n_gemm_kernel.h.  Configuration chosen with
//   tools/gemm_tune.hip on MI355X over the five C2 projection shapes
//   (profiles/gemm_tune_r01.txt): 8 waves x 16 rows (BM = 128), BN = 208
//   (NT = 13) for widths > 256 else 128, K-step 16, two register prefetch
//   sets, split-K up to 32 slices aiming at ~480 workgroups for the long-K
//   weight gradients (deterministic slab reduce).  103 TF/s on the layer-0
//   projection (M 15360, N 408, K 1260) vs 76 TF/s for hipBLASLt fp32 on the
//   same box (tools/gemm_ref_blas.py).
#include "sv2n_common.h"
#include "sv2n_gemm_kernel.h"
#include "sv2n_gemm3_kernel.h"
#include "sv2n_gemm_tt.h"
#include "sv2n_gemm_bw.h"
#include <algorithm>

namespace sv2n {

struct GemmPlan {
  int nt, pf, splitk;
  int64_t kslice;
};

static GemmPlan plan_gemm(int64_t M, int64_t N, int64_t K) {
  constexpr int BM = 128;
  GemmPlan p{};
  const int64_t pad128 = (N + 127) / 128 * 128, pad208 = (N + 207) / 208 * 208;
  p.nt = (N > 256 && pad208 <= pad128) ? 13 : 8;
  const int64_t bn = 16 * p.nt;
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + bn - 1) / bn);
  int64_t sk = 1;
  if (tiles < 240 && K >= 2048) {
    constexpr int64_t target = 480;  // workgroups aimed at
    sk = std::min<int64_t>(32, (target + tiles - 1) / tiles);
    sk = std::min<int64_t>(sk, std::max<int64_t>(1, K / 256));
  }
  int64_t ks = (K + sk - 1) / sk;
  ks = (ks + 15) / 16 * 16;
  p.splitk = (int)((K + ks - 1) / ks);
  p.kslice = ks;
  p.pf = 2;
  return p;
}


// ---------------------------------------------------------------------------
// Fused weight-gradient epilogue of one GAT layer (the
// backward of lin_src and of the att_src / att_dst folds, plus the bias).
// The split-K GEMM's slabs are summed in a fixed order by one contiguous
// streaming pass (k_splitk_reduce) into T = dWaugᵀ [F][ldt] (ldt = the
// projection width; columns HC.. hold the fold rows).  One launch of
// independent blocks then does
//   tile blocks   gW[o][f]   += T[f][o] + T[f][HC+h]·att_s[o] + T[f][HC+H+h]·att_d[o]
//                 (16 f x 64 o, transposed through LDS, gW written along f)
//   att blocks    g_att_s[o] += Σ_f T[f][HC+h] · W[o][f]   (one wave per o,
//                 same for dst; o = h*C+c)
//   bias blocks   g_bias[o]  += Σ_b dbias_partial[b][o]
// with every sum in a fixed order and no hand-off between blocks (tiles
// summing their att partials through a shared ticket serialised on the
// counter: 25 us).  Every load is a buffer load (out-of-range offsets read
// 0): nothing sits behind a branch, each batch is one memory round trip.
// ---------------------------------------------------------------------------
constexpr int WG_FT = 16, WG_OT = 64;

// Att-vector gradients of one layer: g_att_s[o] += Σ_f T[f][HC+h]·W[o][f]
// (and dst), h = o / C.  A block owns ATT_RB consecutive rows o (their heads
// [h0, h1]); it stages those heads' fold columns of T (strided by ldt) into
// LDS once, [q][h - h0][f], then each wave takes ATT_RB/4 rows and reads W
// rows coalesced, all of them in flight at once.  (Per-wave loads of the
// strided columns — one 64-line gather per lane slot, once per row — cost
// 41 us at C3, HC 3000 x F 1260.)  Sums in a fixed order.
constexpr int ATT_RB = 8;            // rows per block
constexpr int ATT_RW = ATT_RB / 4;   // rows per wave
constexpr int ATT_FPL = 24;          // f per lane per pass (F <= 1536: one pass)

// SLABS = false: the fold columns are columns HC.. of T [F][ldt].  SLABS =
// true (bf16 path, k_wgrad_epi_t): they are rows HC.. of nslab split-K slabs
// [ldt][F] (ldt = rows), summed here in slab order.
template <bool SLABS>
__device__ __forceinline__ void wgrad_att_block(int blk, const float* __restrict__ T, int ldt,
                                                const float* __restrict__ W, int H, int C, int F,
                                                float* __restrict__ g_as, float* __restrict__ g_ad,
                                                float* __restrict__ s_fold, int nslab = 1) {
  // s_fold: [2][nh][F] (dynamic LDS)
  const int HC = H * C, t = threadIdx.x, lane = t & 63, wv = wave_id();
  const int o0 = blk * ATT_RB, o1 = min(HC, o0 + ATT_RB);
  const int h0 = o0 / C, nh = (o1 - 1) / C - h0 + 1;
  const rsrc_t rt = make_rsrc(T, (uint32_t)F * (uint32_t)ldt * 4u * (uint32_t)nslab);
  {
    const int n = 2 * nh * F;
    for (int k0 = 0; k0 < n; k0 += 8 * 256) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + t + 256 * u;
        const int q = k / (nh * F), r = k - q * nh * F, hh = r / F, f = r - hh * F;
        if constexpr (SLABS) {
          const int off = ((HC + q * H + h0 + hh) * F + f) * 4;
          v[u] = bld(rt, k < n ? off : OOB);
          for (int sl = 1; sl < nslab; ++sl)
            v[u] += bld(rt, k < n ? off + sl * F * ldt * 4 : OOB);
        } else {
          v[u] = bld(rt, k < n ? (f * ldt + HC + q * H + h0 + hh) * 4 : OOB);
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k0 + t + 256 * u < n) s_fold[k0 + t + 256 * u] = v[u];
    }
  }
  __syncthreads();
  const int ob = o0 + wv * ATT_RW;
  float as[ATT_RW], ad[ATT_RW];
#pragma unroll
  for (int r = 0; r < ATT_RW; ++r) as[r] = ad[r] = 0.f;
  for (int f0 = 0; f0 < F; f0 += 64 * ATT_FPL) {
    float w[ATT_RW][ATT_FPL];
#pragma unroll
    for (int r = 0; r < ATT_RW; ++r) {
      const int o = ob + r;
      const rsrc_t rw = make_rsrc(W + (int64_t)min(o, HC - 1) * F, o < o1 ? (uint32_t)F * 4u : 0u);
#pragma unroll
      for (int u = 0; u < ATT_FPL; ++u) {
        const int f = f0 + lane + 64 * u;
        w[r][u] = bld(rw, f < F ? f * 4 : OOB);
      }
    }
#pragma unroll
    for (int r = 0; r < ATT_RW; ++r) {
      const int hh = min(ob + r, o1 - 1) / C - h0;
      const float* gs = s_fold + hh * F;
      const float* gd = s_fold + (nh + hh) * F;
#pragma unroll
      for (int u = 0; u < ATT_FPL; ++u) {
        const int f = min(f0 + lane + 64 * u, F - 1);  // w is 0 past F
        as[r] = fmaf(gs[f], w[r][u], as[r]);
        ad[r] = fmaf(gd[f], w[r][u], ad[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < ATT_RW; ++r) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      as[r] += __shfl_xor(as[r], m, 64);
      ad[r] += __shfl_xor(ad[r], m, 64);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < ATT_RW; ++r) {
      const int o = ob + r;
      if (o < o1) {
        if (g_as) g_as[o] += as[r];
        if (g_ad) g_ad[o] += ad[r];
      }
    }
  }
}

// g_bias[o] += Σ_b dbp[b][o] for 16 columns o: 16 row groups, 8 loads in
// flight each, the groups added in order
__device__ __forceinline__ void wgrad_bias_block(int blk, const float* __restrict__ dbp, int nparts,
                                                 int OC, float* __restrict__ g_bias,
                                                 float (*s_red)[17]) {
  const int t = threadIdx.x;
  const rsrc_t rb = make_rsrc(dbp, (uint32_t)nparts * (uint32_t)OC * 4u);
  const int lo = t & 15, grp = t >> 4;
  const int o = blk * 16 + lo;
  float a = 0.f;
  for (int q0 = 0; q0 < nparts; q0 += 16 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int q = q0 + grp + 16 * u;
      v[u] = bld(rb, (o < OC && q < nparts) ? (q * OC + o) * 4 : OOB);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) a += v[u];
  }
  s_red[grp][lo] = a;
  __syncthreads();
  if (grp == 0 && o < OC) {
    float sb = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) sb += s_red[k][lo];
    g_bias[o] += sb;
  }
}

__global__ __launch_bounds__(256) void k_wgrad_epi(
    const float* __restrict__ T, int ldt, const float* __restrict__ W,
    const float* __restrict__ att_s, const float* __restrict__ att_d, int H, int C, int F,
    float* __restrict__ gW, float* __restrict__ g_as, float* __restrict__ g_ad, int ntile,
    int nft, int natt, const float* __restrict__ dbp, int nparts, int OC,
    float* __restrict__ g_bias) {
  __shared__ float tile[WG_FT][WG_OT + 1];
  __shared__ float sfold[WG_FT][2 * SV2N_MAX_HEADS];
  __shared__ float s_red[16][17];
  const int HC = H * C;
  const int t = threadIdx.x;
  // dispatch order: the att blocks (the longest) first, then the gW tiles,
  // then the bias blocks; b is the block's number in tile/att/bias order
  const int bx = blockIdx.x;
  const int b = bx < natt ? ntile + bx : (bx < natt + ntile ? bx - natt : bx);
  const rsrc_t rt = make_rsrc(T, (uint32_t)F * (uint32_t)ldt * 4u);
  if (b >= ntile + natt) {  // ---- bias column sums ----
    wgrad_bias_block(b - ntile - natt, dbp, nparts, OC, g_bias, s_red);
    return;
  }
  if (b >= ntile) {  // att blocks (dispatched first)
    extern __shared__ float s_dyn[];
    wgrad_att_block<false>(b - ntile, T, ldt, W, H, C, F, g_as, g_ad, s_dyn);
    return;
  }
  // ---- gW tile: 16 f x 64 o ----
  const int ft = b % nft, ot = b / nft;
  const int f0 = ft * WG_FT, o0 = ot * WG_OT;
  {
    const int ol = t & 63, fr = t >> 6;
    const int o = o0 + ol;
    constexpr int R = WG_FT / 4;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int f = f0 + fr + 4 * r;
      tile[fr + 4 * r][ol] = bld(rt, (o < HC && f < F) ? (f * ldt + o) * 4 : OOB);
    }
    if (t < WG_FT * 2 * H) {  // 16 x 2H <= 256
      const int fl = t / (2 * H), k = t - fl * 2 * H;
      const int f = f0 + fl;
      sfold[fl][k] = bld(rt, f < F ? (f * ldt + HC + k) * 4 : OOB);
    }
  }
  __syncthreads();
  const int fl = t & (WG_FT - 1), og = t / WG_FT;  // 256 / WG_FT o-rows per pass
  const int f = f0 + fl;
  constexpr int OPP = 256 / WG_FT, Q = WG_OT / OPP;
  const rsrc_t rg = make_rsrc(gW, (uint32_t)HC * (uint32_t)F * 4u);
  const rsrc_t ras = make_rsrc(att_s, (uint32_t)HC * 4u), rad = make_rsrc(att_d, (uint32_t)HC * 4u);
  float gv[Q], av[Q], dv[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {  // all loads first
    const int o = o0 + og + OPP * q;
    gv[q] = bld(rg, (o < HC && f < F) ? (o * F + f) * 4 : OOB);
    av[q] = bld(ras, o < HC ? o * 4 : OOB);
    dv[q] = bld(rad, o < HC ? o * 4 : OOB);
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int orow = og + OPP * q, o = o0 + orow;
    const int h = min(o, HC - 1) / C;
    const float v = gv[q] + (tile[fl][orow] + sfold[fl][h] * av[q] + sfold[fl][H + h] * dv[q]);
    bst(rg, (o < HC && f < F) ? (o * F + f) * 4 : OOB, v);
  }
}

// ---------------------------------------------------------------------------
// bf16 path: the GEMM writes dWaug itself (rows o' = the ldt projection rows,
// F columns) as nslab split-K slabs S[s][o'][f], and this one launch sums the
// slabs while applying the fold (no reduce launch, no transposition):
//   row blocks  gW[o][f] += (Σ_s S[s][o][f]) + fs_h[f]·att_s[o] + fd_h[f]·att_d[o],
//               fs_h / fd_h = Σ_s S[s][HC+h][f] / Σ_s S[s][HC+H+h][f], h = o / C;
//               a block = WT_RB rows x 256 f, a wave per row, float4 per lane
//   att blocks  as in k_wgrad_epi, the fold rows summed from the slabs
//   bias blocks as in k_wgrad_epi
// ---------------------------------------------------------------------------
constexpr int WT_RB = 32;

__global__ __launch_bounds__(256) void k_wgrad_epi_t(
    const float* __restrict__ S, int nslab, int ldt, const float* __restrict__ W,
    const float* __restrict__ att_s, const float* __restrict__ att_d, int H, int C, int F,
    float* __restrict__ gW, float* __restrict__ g_as, float* __restrict__ g_ad, int nrow,
    int nfc, int natt, const float* __restrict__ dbp, int nparts, int OC,
    float* __restrict__ g_bias) {
  __shared__ float s_red[16][17];
  const int HC = H * C;
  const int t = threadIdx.x, lane = t & 63, wv = wave_id();
  const int bx = blockIdx.x;  // att blocks first, then the row blocks, then bias
  if (bx < natt) {
    extern __shared__ float s_dyn[];
    wgrad_att_block<true>(bx, S, ldt, W, H, C, F, g_as, g_ad, s_dyn, nslab);
    return;
  }
  const int b = bx - natt;
  if (b >= nrow * nfc) {
    wgrad_bias_block(b - nrow * nfc, dbp, nparts, OC, g_bias, s_red);
    return;
  }
  const int fc = b % nfc, rg = b / nfc;
  const int o0 = rg * WT_RB, o1 = min(HC, o0 + WT_RB);
  const int f = 4 * (fc * 64 + lane);
  const bool fv = f < F;
  const int64_t sstride = (int64_t)ldt * F;
  const rsrc_t rs = make_rsrc(S, (uint32_t)(sstride * nslab * 4));
  const rsrc_t rg_ = make_rsrc(gW, (uint32_t)HC * (uint32_t)F * 4u);
  // fold rows of the (at most two) heads the block's rows touch
  const int ha = o0 / C, hb = (o1 - 1) / C;
  f32x4 fs[2], fd[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int h = k ? hb : ha;
    const int offs = ((HC + h) * F + f) * 4, offd = ((HC + H + h) * F + f) * 4;
    fs[k] = bld4(rs, fv ? offs : OOB);
    fd[k] = bld4(rs, fv ? offd : OOB);
    for (int sl = 1; sl < nslab; ++sl) {
      fs[k] += bld4(rs, fv ? offs + (int)(sl * sstride * 4) : OOB);
      fd[k] += bld4(rs, fv ? offd + (int)(sl * sstride * 4) : OOB);
    }
  }
  constexpr int RPW = WT_RB / 4;  // rows per wave
  f32x4 gv[RPW], tv[RPW];
  float av[RPW], dv[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {  // every load of the wave's rows in flight
    const int o = o0 + wv + 4 * r;
    const bool ov = o < o1 && fv;
    const int off = (o * F + f) * 4;
    gv[r] = bld4(rg_, ov ? off : OOB);
    tv[r] = bld4(rs, ov ? off : OOB);
    for (int sl = 1; sl < nslab; ++sl) tv[r] += bld4(rs, ov ? off + (int)(sl * sstride * 4) : OOB);
    av[r] = o < o1 ? att_s[o] : 0.f;
    dv[r] = o < o1 ? att_d[o] : 0.f;
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int o = o0 + wv + 4 * r;
    if (o < o1 && fv) {
      const int k = (o / C) == ha ? 0 : 1;
      f32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = gv[r][j] + (tv[r][j] + fs[k][j] * av[r] + fd[k][j] * dv[r]);
      bst4(rg_, (o * F + f) * 4, v);
    }
  }
}
}  // namespace sv2n

using namespace sv2n;

extern "C" int64_t sv2n_gemm_f32_workspace(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const GemmPlan p = plan_gemm(M, N, K);
  return p.splitk > 1 ? (int64_t)p.splitk * M * N : 0;
}

template <int NT, int PF>
static void dispatch_layout(int a_kmajor, int b_kmajor, const GemmPlan& p, hipStream_t st,
                            const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                            int64_t ldc, int64_t M, int64_t N, int64_t K, bool avec, bool bvec,
                            float* part) {
  if (a_kmajor && b_kmajor)
    launch_gemm_cfg<8, 1, NT, 16, true, true, PF>(p.splitk, p.kslice, st, A, lda, B, ldb, C, ldc,
                                                  M, N, K, avec, bvec, part);
  else if (a_kmajor)
    launch_gemm_cfg<8, 1, NT, 16, true, false, PF>(p.splitk, p.kslice, st, A, lda, B, ldb, C, ldc,
                                                   M, N, K, avec, bvec, part);
  else if (b_kmajor)
    launch_gemm_cfg<8, 1, NT, 16, false, true, PF>(p.splitk, p.kslice, st, A, lda, B, ldb, C, ldc,
                                                   M, N, K, avec, bvec, part);
  else
    launch_gemm_cfg<8, 1, NT, 16, false, false, PF>(p.splitk, p.kslice, st, A, lda, B, ldb, C,
                                                    ldc, M, N, K, avec, bvec, part);
}

extern "C" int sv2n_gemm_f32(int a_kmajor, int b_kmajor, const float* A, int64_t lda,
                             const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M,
                             int64_t N, int64_t K, float* workspace, int64_t workspace_floats,
                             hipStream_t stream) {
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0) return SV2N_ERR_ARG;
  if (ldc < N || lda < (a_kmajor ? K : M) || ldb < (b_kmajor ? K : N)) return SV2N_ERR_SHAPE;
  const GemmPlan p = plan_gemm(M, N, K);
  float* part = nullptr;
  if (p.splitk > 1) {
    if (!workspace || workspace_floats < (int64_t)p.splitk * M * N) return SV2N_ERR_WORKSPACE;
    part = workspace;
  }
  const bool avec = ((uintptr_t)A % 16 == 0) && (lda % 4 == 0);
  const bool bvec = ((uintptr_t)B % 16 == 0) && (ldb % 4 == 0);
  if (p.nt == 13) {
    if (p.pf == 2)
      dispatch_layout<13, 2>(a_kmajor, b_kmajor, p, stream, A, lda, B, ldb, C, ldc, M, N, K, avec,
                             bvec, part);
    else
      dispatch_layout<13, 1>(a_kmajor, b_kmajor, p, stream, A, lda, B, ldb, C, ldc, M, N, K, avec,
                             bvec, part);
  } else {
    if (p.pf == 2)
      dispatch_layout<8, 2>(a_kmajor, b_kmajor, p, stream, A, lda, B, ldb, C, ldc, M, N, K, avec,
                            bvec, part);
    else
      dispatch_layout<8, 1>(a_kmajor, b_kmajor, p, stream, A, lda, B, ldb, C, ldc, M, N, K, avec,
                            bvec, part);
  }
  return (int)hipGetLastError();
}

// How the slab GEMM of a weight gradient runs.  kind 0: exact-f32 kernel
// (k_gemm_f32, XR slices); kind 1 / 2: bf16x3 k_gemm_tt3w<13, kind>.  For the
// 208-column tiling the split count follows the bf16x3 kernel's rule — one
// round of 144 KiB / 98 KiB workgroups balanced over the 8 XCDs (a multiple
// of 8 slices, tiles x slices <= 256; MI355X, C2 L0 dWᵀ 1260 x 408 x 15360:
// 24 slices 92 us, 16: 126 us, 32: 130 us), at most 256 slices of >= 256 rows
// (sv2n_gat_wgrad_node_workspace covers both plans); unaligned operands run
// the f32 kernel on the same slices.
struct SlabPlan {
  int kind, nt, splitk;  // kind: 0 f32 kernel; 1 / 2: tt3w<13, MT>; 3 / 4: tt3w<9, MT>
  int64_t kslice;
};
static SlabPlan slab_plan(int64_t F, int64_t N, int64_t K, bool vec, int64_t lda, int64_t ldb) {
  const GemmPlan p = plan_gemm(F, N, K);
  SlabPlan sp{0, p.nt, p.splitk, p.kslice};
  if (p.splitk <= 1) return sp;
  // column tiles of 208 (C2: N = 408, 208) or 144 (C5: N = 144), at most 25 % padding
  int bn = 0;
  for (const int w : {208, 144})
    if ((N + w - 1) / w * w * 4 <= 5 * N) {
      bn = w;
      break;
    }
  if (bn == 0) return sp;
  const int64_t ntile = (N + bn - 1) / bn;
  const int mt = ((F + 255) / 256) * ntile >= 8 ? 2 : 1;  // row tiles per wave
  const int64_t tiles = ((F + 128 * mt - 1) / (128 * mt)) * ntile;
  int64_t sk = 8 * std::max<int64_t>(1, 256 / (8 * tiles));
  sk = std::min<int64_t>(sk, std::min<int64_t>(256, std::max<int64_t>(8, K / 256 / 8 * 8)));
  int64_t ks = (K + sk - 1) / sk;
  ks = (ks + 31) / 32 * 32;
  sp.splitk = (int)((K + ks - 1) / ks);
  sp.kslice = ks;
  const bool ok = vec && (F % 4) == 0 && K * std::max(lda, ldb) * 4 <= 0x7fffffff;
  sp.kind = ok ? (bn == 208 ? 0 : 2) + mt : 0;
  return sp;
}

template <int NT, int MT>
static void launch_tt3w(const SlabPlan& p, hipStream_t stream, const float* x, int64_t ld_x,
                        const float* dxs, int64_t ldx, int64_t F, int64_t N, int64_t K,
                        float* out) {
  using Cfg = GemmTT3WCfg<NT, MT>;
  using CfgY = GemmTT3YCfg<NT, MT>;
  // tt3y where it measured faster: the 208-column tilings (C2 L0 dWᵀ 92.9 ->
  // 91.0 us, step 0.5476 -> 0.5424 ms); C5's 144-column one: 524 vs 530 us
  if constexpr (NT == 13 && CfgY::LDS <= 160 * 1024) {
    static bool attr_y = [] {
      (void)hipFuncSetAttribute((const void*)k_gemm_tt3y<NT, MT>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)CfgY::LDS);
      return true;
    }();
    (void)attr_y;
    const dim3 gy((unsigned)((F + Cfg::BM - 1) / Cfg::BM), (unsigned)((N + Cfg::BN - 1) / Cfg::BN),
                  (unsigned)((p.splitk + 7) / 8 * 8));
    hipLaunchKernelGGL((k_gemm_tt3y<NT, MT>), gy, dim3(Cfg::THREADS), CfgY::LDS, stream, x,
                       ld_x, dxs, ldx, out, F, N, K, p.kslice, p.splitk);
    return;
  }
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_gemm_tt3w<NT, MT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)Cfg::LDS);
    return true;
  }();
  (void)attr;
  const dim3 grid((unsigned)((F + Cfg::BM - 1) / Cfg::BM), (unsigned)((N + Cfg::BN - 1) / Cfg::BN),
                  (unsigned)((p.splitk + 7) / 8 * 8));
  hipLaunchKernelGGL((k_gemm_tt3w<NT, MT>), grid, dim3(Cfg::THREADS), Cfg::LDS, stream, x, ld_x,
                     dxs, ldx, out, F, N, K, p.kslice, p.splitk);
}

static void launch_wgrad_slabs(const SlabPlan& p, hipStream_t stream, const float* x,
                               int64_t ld_x, const float* dxs, int64_t ldx, int64_t F, int64_t N,
                               int64_t K, bool avec, bool bvec, float* out) {
  if (p.kind == 2) {
    launch_tt3w<13, 2>(p, stream, x, ld_x, dxs, ldx, F, N, K, out);
  } else if (p.kind == 1) {
    launch_tt3w<13, 1>(p, stream, x, ld_x, dxs, ldx, F, N, K, out);
  } else if (p.kind == 4) {
    launch_tt3w<9, 2>(p, stream, x, ld_x, dxs, ldx, F, N, K, out);
  } else if (p.kind == 3) {
    launch_tt3w<9, 1>(p, stream, x, ld_x, dxs, ldx, F, N, K, out);
  } else if (p.nt == 13) {
    launch_gemm_slabs<8, 1, 13, 16, false, false, 2, 0, true>(p.splitk, p.kslice, stream, x, ld_x,
                                                              dxs, ldx, F, N, K, avec, bvec, out);
  } else {
    launch_gemm_slabs<8, 1, 8, 16, false, false, 2, 0, true>(p.splitk, p.kslice, stream, x, ld_x,
                                                             dxs, ldx, F, N, K, avec, bvec, out);
  }
}

// ---- the split-K GEMM alone: C's K slices left as slabs [nsplit][M][N] ------
// (what sv2n_gat_wgrad_node runs before its reduce; exposed for consumers that
// fuse the reduction, and so the kernel can be timed by itself)
extern "C" int sv2n_gemm_f32_slabs_count(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  // enough for either plan (the non-k-major weight-gradient case follows slab_plan)
  return std::max(plan_gemm(M, N, K).splitk, slab_plan(M, N, K, true, M, N).splitk);
}

extern "C" int sv2n_gemm_f32_slabs(int a_kmajor, int b_kmajor, const float* A, int64_t lda,
                                   const float* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
                                   float* slabs, int64_t slab_floats, hipStream_t stream) {
  if (!A || !B || !slabs || M <= 0 || N <= 0 || K <= 0) return SV2N_ERR_ARG;
  if (lda < (a_kmajor ? K : M) || ldb < (b_kmajor ? K : N)) return SV2N_ERR_SHAPE;
  const GemmPlan p = plan_gemm(M, N, K);
  if (slab_floats < (int64_t)p.splitk * M * N) return SV2N_ERR_WORKSPACE;
  const bool avec = ((uintptr_t)A % 16 == 0) && (lda % 4 == 0);
  const bool bvec = ((uintptr_t)B % 16 == 0) && (ldb % 4 == 0);
#define SV2N_SLABS(NT, AK, BK)                                                                    \
  launch_gemm_slabs<8, 1, NT, 16, AK, BK, 2, 0, true>(p.splitk, p.kslice, stream, A, lda, B, ldb, \
                                                    M, N, K, \
                                             avec, bvec, slabs)
  if (!a_kmajor && !b_kmajor) {
    const SlabPlan sp = slab_plan(M, N, K, avec && bvec, lda, ldb);
    if (slab_floats < (int64_t)sp.splitk * M * N) return SV2N_ERR_WORKSPACE;
    launch_wgrad_slabs(sp, stream, A, lda, B, ldb, M, N, K, avec, bvec, slabs);
    return (int)hipGetLastError();
  }
  if (p.nt == 13) {
    if (a_kmajor && b_kmajor) SV2N_SLABS(13, true, true);
    else if (a_kmajor) SV2N_SLABS(13, true, false);
    else if (b_kmajor) SV2N_SLABS(13, false, true);
    else SV2N_SLABS(13, false, false);
  } else {
    if (a_kmajor && b_kmajor) SV2N_SLABS(8, true, true);
    else if (a_kmajor) SV2N_SLABS(8, true, false);
    else if (b_kmajor) SV2N_SLABS(8, false, true);
    else SV2N_SLABS(8, false, false);
  }
#undef SV2N_SLABS
  return (int)hipGetLastError();
}

// ---- weight gradients of one layer: split-K GEMM + fused epilogue ----------
// The slab GEMM of a weight gradient, T[f][o] = Σ_k x[k][f] · dxs[k][o] (both
// operands k-strided): the bf16x3 kernel k_gemm_tt3w where it applies (208-
// column tiles, split-K, 16-B aligned operands), else the exact-f32 kernel; K
// slices grouped per XCD either way (C2 L0: HBM fetch 374 -> 122 MB).
static int64_t wgrad_slab_floats(int64_t n_nodes, int F, int ldt) {
  const GemmPlan p = plan_gemm(F, ldt, n_nodes);
  const SlabPlan sp = slab_plan(F, ldt, n_nodes, true, F, ldt);
  const int sk = std::max(p.splitk, sp.splitk);
  return sk > 1 ? (int64_t)sk * F * ldt : 0;
}

extern "C" int64_t sv2n_gat_wgrad_node_workspace(int64_t num_nodes, int in_features, int ldx,
                                                 int heads, int channels) {
  if (num_nodes <= 0 || in_features <= 0 || ldx <= 0 || heads <= 0 || channels <= 0) return 0;
  return (int64_t)in_features * ldx + wgrad_slab_floats(num_nodes, in_features, ldx);
}

// bf16-operand weight-gradient GEMM: k_gemm_tt<128, 128, 1> (transposed LDS
// reads, sv2n_gemm_tt.h), K slices of multiples of 32 aiming at ~480
// workgroups (tools/gemm_tt_tune.hip: C3 dWaugᵀ 1260 x 3012 x 3840 in 78 us,
// 374 TF/s, vs 340 us for the split kernel k_gemm3_t)
constexpr int TT_BM = 128, TT_BN = 128;
static GemmPlan plan_gemm_bf16t(int64_t M, int64_t N, int64_t K) {
  GemmPlan p{};
  p.nt = TT_BN / 16;
  const int64_t tiles = ((M + TT_BM - 1) / TT_BM) * ((N + TT_BN - 1) / TT_BN);
  int64_t sk = 1;
  if (tiles < 400 && K >= 512) {
    sk = std::min<int64_t>(32, (480 + tiles - 1) / tiles);
    sk = std::min<int64_t>(sk, std::max<int64_t>(1, K / 256));
  }
  int64_t ks = (K + sk - 1) / sk;
  ks = (ks + 31) / 32 * 32;
  p.splitk = (int)((K + ks - 1) / ks);
  p.kslice = ks;
  p.pf = 1;
  return p;
}

static void launch_wgrad_bf16(const GemmPlan& p, hipStream_t st, const float* x, int64_t ld_x,
                              const float* dxs, int64_t ldx, int64_t F, int64_t K, float* out) {
  using Cfg = GemmTTCfg<TT_BM, TT_BN, 1>;
  constexpr size_t lds = Cfg::LDS;
  static_assert(lds <= 64 * 1024, "LDS budget");
  const dim3 grid((unsigned)((F + TT_BM - 1) / TT_BM), (unsigned)((ldx + TT_BN - 1) / TT_BN),
                  (unsigned)p.splitk);
  hipLaunchKernelGGL((k_gemm_tt<TT_BM, TT_BN, 1>), grid, dim3(256), lds, st, x, ld_x, dxs, ldx,
                     out, ldx, F, ldx, K, p.kslice);
}

// the same product transposed, dWaug = dxsᵀ·x [ldx][F] (operands swapped):
// the epilogue (k_wgrad_epi_t) then works along rows of gW.  Round 4: the
// large-tile kernel k_gemm_bw<128, 256, TN> (sv2n_gemm_bw.h; K slices of
// multiples of 64 aiming at one round of ~240 workgroups).  C3 shape (M 3012,
// N 1260, K 3840, tools/gemm_bw_tune.hip): 128 x 256 split 2 68.3 us, the
// round-3 k_gemm_tt<128, 128, 1> 75.1, 256 x 128 117.6, 256 x 192 247.7
constexpr int BWT_BM = 128, BWT_BN = 256;
// both operands already bf16 in memory (sv2n_gat_wgrad_node_bf16b): 128 x 128
// tiles, split 2 on the C3 shape (48.6 us; 128 x 256: 51.1)
constexpr int BWB_BM = 128, BWB_BN = 128;
static GemmPlan plan_wgrad_bw(int64_t ldx, int64_t F, int64_t K, int BM = BWT_BM,
                              int BN = BWT_BN) {
  GemmPlan p{};
  const int64_t tiles = ((ldx + BM - 1) / BM) * ((F + BN - 1) / BN);
  int64_t sk = std::max<int64_t>(1, (240 + tiles / 2) / tiles);
  sk = std::min<int64_t>(sk, std::max<int64_t>(1, K / 512));
  sk = std::min<int64_t>(sk, 8);
  int64_t ks = (K + sk - 1) / sk;
  ks = (ks + 63) / 64 * 64;
  p.splitk = (int)((K + ks - 1) / ks);
  p.kslice = ks;
  return p;
}
static void launch_wgrad_bf16_t(const GemmPlan& p, hipStream_t st, const float* x, int64_t ld_x,
                                const float* dxs, int64_t ldx, int64_t F, int64_t K, float* out) {
  using Cfg = GemmBWCfg<BWT_BM, BWT_BN, true, true, true>;
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_gemm_bw<BWT_BM, BWT_BN, true, true, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)Cfg::LDS);
    return true;
  }();
  (void)attr;
  const int nm = (int)((ldx + BWT_BM - 1) / BWT_BM), nn = (int)((F + BWT_BN - 1) / BWT_BN);
  const dim3 grid((unsigned)(((nm + 7) / 8) * 8 * nn), 1, (unsigned)p.splitk);
  hipLaunchKernelGGL((k_gemm_bw<BWT_BM, BWT_BN, true, true, true>), grid, dim3(Cfg::THREADS),
                     Cfg::LDS, st, (const void*)dxs, ldx, (const void*)x, ld_x, out, F, ldx, F, K,
                     p.kslice, nm, nn);
}

static void launch_wgrad_bf16b(const GemmPlan& p, hipStream_t st, const unsigned short* xb,
                               int64_t ld_xb, const unsigned short* db, int64_t ld_db,
                               int64_t ldx, int64_t F, int64_t K, float* out) {
  using Cfg = GemmBWCfg<BWB_BM, BWB_BN, true, false, false>;
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_gemm_bw<BWB_BM, BWB_BN, true, false, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)Cfg::LDS);
    return true;
  }();
  (void)attr;
  const int nm = (int)((ldx + BWB_BM - 1) / BWB_BM), nn = (int)((F + BWB_BN - 1) / BWB_BN);
  const dim3 grid((unsigned)(((nm + 7) / 8) * 8 * nn), 1, (unsigned)p.splitk);
  hipLaunchKernelGGL((k_gemm_bw<BWB_BM, BWB_BN, true, false, false>), grid, dim3(Cfg::THREADS),
                     Cfg::LDS, st, (const void*)db, ld_db, (const void*)xb, ld_xb, out, F, ldx, F,
                     K, p.kslice, nm, nn);
}

// bf16 operands in memory (precision 1 with xb / db set): x_bf16 [K][ld_xb],
// dxs_bf16 [K][ld_db]
struct Bf16Ops {
  const unsigned short* xb;
  int64_t ld_xb;
  const unsigned short* db;
  int64_t ld_db;
};

static int wgrad_node(int precision, const float* x, int64_t ld_x, const float* dxs, int ldx,
                      int64_t num_nodes, int in_features, const float* W, const float* att_src,
                      const float* att_dst, int heads, int channels, const float* dbias_partial,
                      int num_parts, int bias_len, float* gW, float* g_att_src, float* g_att_dst,
                      float* g_bias, float* workspace, int64_t workspace_floats,
                      hipStream_t stream, const Bf16Ops& bo = Bf16Ops{});

extern "C" int sv2n_gat_wgrad_node(const float* x, int64_t ld_x, const float* dxs, int ldx,
                                   int64_t num_nodes, int in_features, const float* W,
                                   const float* att_src, const float* att_dst, int heads,
                                   int channels, const float* dbias_partial, int num_parts,
                                   int bias_len, float* gW, float* g_att_src, float* g_att_dst,
                                   float* g_bias, float* workspace, int64_t workspace_floats,
                                   hipStream_t stream) {
  return wgrad_node(0, x, ld_x, dxs, ldx, num_nodes, in_features, W, att_src, att_dst, heads,
                    channels, dbias_partial, num_parts, bias_len, gW, g_att_src, g_att_dst,
                    g_bias, workspace, workspace_floats, stream);
}

extern "C" int64_t sv2n_gat_wgrad_node_bf16_workspace(int64_t num_nodes, int in_features, int ldx,
                                                      int heads, int channels) {
  if (num_nodes <= 0 || in_features <= 0 || ldx <= 0 || heads <= 0 || channels <= 0) return 0;
  const GemmPlan p = plan_gemm_bf16t(in_features, ldx, num_nodes);
  const int sk = std::max({p.splitk, plan_wgrad_bw(ldx, in_features, num_nodes).splitk,
                           plan_wgrad_bw(ldx, in_features, num_nodes, BWB_BM, BWB_BN).splitk});
  return (int64_t)in_features * ldx * (sk > 1 ? 1 + sk : 1);
}

extern "C" int sv2n_gat_wgrad_node_bf16b(const uint16_t* x_bf16, int64_t ld_xb,
                                         const uint16_t* dxs_bf16, int64_t ld_db,
                                         int64_t num_nodes, int in_features, int ldx,
                                         const float* W, const float* att_src,
                                         const float* att_dst, int heads, int channels,
                                         const float* dbias_partial, int num_parts, int bias_len,
                                         float* gW, float* g_att_src, float* g_att_dst,
                                         float* g_bias, float* workspace,
                                         int64_t workspace_floats, hipStream_t stream) {
  if (!x_bf16 || !dxs_bf16) return SV2N_ERR_ARG;
  if (ld_xb < in_features || ld_db < ldx || (ld_xb & 7) || (ld_db & 7)) return SV2N_ERR_SHAPE;
  if (((uintptr_t)x_bf16 & 15) || ((uintptr_t)dxs_bf16 & 15)) return SV2N_ERR_ALIGN;
  if (!gW) return SV2N_ERR_ARG;  // the bf16-operand form always produces the weight gradient
  const Bf16Ops bo{reinterpret_cast<const unsigned short*>(x_bf16), ld_xb,
                   reinterpret_cast<const unsigned short*>(dxs_bf16), ld_db};
  return wgrad_node(1, nullptr, in_features, nullptr, ldx, num_nodes, in_features, W, att_src,
                    att_dst, heads, channels, dbias_partial, num_parts, bias_len, gW, g_att_src,
                    g_att_dst, g_bias, workspace, workspace_floats, stream, bo);
}

extern "C" int sv2n_gat_wgrad_node_bf16(const float* x, int64_t ld_x, const float* dxs, int ldx,
                                        int64_t num_nodes, int in_features, const float* W,
                                        const float* att_src, const float* att_dst, int heads,
                                        int channels, const float* dbias_partial, int num_parts,
                                        int bias_len, float* gW, float* g_att_src,
                                        float* g_att_dst, float* g_bias, float* workspace,
                                        int64_t workspace_floats, hipStream_t stream) {
  return wgrad_node(1, x, ld_x, dxs, ldx, num_nodes, in_features, W, att_src, att_dst, heads,
                    channels, dbias_partial, num_parts, bias_len, gW, g_att_src, g_att_dst,
                    g_bias, workspace, workspace_floats, stream);
}

static int wgrad_node(int precision, const float* x, int64_t ld_x, const float* dxs, int ldx,
                      int64_t num_nodes, int in_features, const float* W, const float* att_src,
                      const float* att_dst, int heads, int channels, const float* dbias_partial,
                      int num_parts, int bias_len, float* gW, float* g_att_src, float* g_att_dst,
                      float* g_bias, float* workspace, int64_t workspace_floats,
                      hipStream_t stream, const Bf16Ops& bo) {
  const bool weights = gW || g_att_src || g_att_dst;
  const bool bfin = bo.xb != nullptr;
  const int F = in_features, H = heads, C = channels, HC = heads * channels;
  if (H < 1 || C < 1 || F < 1 || num_nodes < 1) return SV2N_ERR_ARG;
  if (H > SV2N_MAX_HEADS || ldx < HC + 2 * H) return SV2N_ERR_SHAPE;
  if (weights && ((!bfin && (!x || !dxs)) || !W || !att_src || !att_dst)) return SV2N_ERR_ARG;
  if (weights && ld_x < F) return SV2N_ERR_SHAPE;
  if ((int64_t)F * ldx >= (int64_t)1 << 29 || (int64_t)HC * F >= (int64_t)1 << 29)
    return SV2N_ERR_SHAPE;  // 32-bit buffer offsets
  const bool bias = g_bias && dbias_partial && bias_len > 0 && num_parts > 0;
  if (!weights && !bias) return 0;
  if ((int64_t)num_parts * bias_len >= (int64_t)1 << 29) return SV2N_ERR_SHAPE;
  const int64_t need = precision ? sv2n_gat_wgrad_node_bf16_workspace(num_nodes, F, ldx, H, C)
                                 : sv2n_gat_wgrad_node_workspace(num_nodes, F, ldx, H, C);
  if (!workspace || workspace_floats < need) return SV2N_ERR_WORKSPACE;
  float* T = workspace;  // reduced dWaugᵀ [F][ldx]
  float* slabs = T + (int64_t)F * ldx;
  if (weights && precision) {
    // bf16 operands: both k-strided, rounded while staged (k_gemm_tt, NP = 1)
    if (!bfin && (((uintptr_t)x & 15) || (ld_x & 3) || ((uintptr_t)dxs & 15) || (ldx & 3) ||
                  F < 4 || ldx < 4))
      return SV2N_ERR_ALIGN;
    if (num_nodes * std::max<int64_t>(ld_x, ldx) * 4 > 0x7fffffff) return SV2N_ERR_SHAPE;
    if (bfin && ((F & 3) != 0 || !gW)) return SV2N_ERR_SHAPE;
    const GemmPlan p = plan_gemm_bf16t(F, ldx, num_nodes);
    if ((F & 3) == 0 && gW) {
      // dWaug [ldx][F] as pt.splitk slabs, summed by the epilogue launch itself
      const GemmPlan pt = bfin ? plan_wgrad_bw(ldx, F, num_nodes, BWB_BM, BWB_BN)
                               : plan_wgrad_bw(ldx, F, num_nodes);
      float* S = pt.splitk > 1 ? slabs : T;
      if (bfin)
        launch_wgrad_bf16b(pt, stream, bo.xb, bo.ld_xb, bo.db, bo.ld_db, ldx, F, num_nodes, S);
      else
        launch_wgrad_bf16_t(pt, stream, x, ld_x, dxs, ldx, F, num_nodes, S);
      const int nfc = (F / 4 + 63) / 64, nrow = (HC + WT_RB - 1) / WT_RB;
      const int natt = (g_att_src || g_att_dst) ? (HC + ATT_RB - 1) / ATT_RB : 0;
      size_t lds = 0;
      if (natt) {
        const int nh_max = std::min(H, (ATT_RB - 1) / C + 2);
        lds = sizeof(float) * 2 * (size_t)nh_max * F;
        if (lds > 140 * 1024) return SV2N_ERR_SHAPE;
        static bool attr = [] {
          (void)hipFuncSetAttribute((const void*)k_wgrad_epi_t,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 140 * 1024);
          return true;
        }();
        (void)attr;
      }
      const int nbias = bias ? (bias_len + 15) / 16 : 0;
      hipLaunchKernelGGL(k_wgrad_epi_t, dim3((unsigned)(natt + nrow * nfc + nbias)), dim3(256),
                         lds, stream, S, pt.splitk, ldx, W, att_src, att_dst, H, C, F, gW,
                         g_att_src, g_att_dst, nrow, nfc, natt, dbias_partial, num_parts,
                         bias_len, g_bias);
      return (int)hipGetLastError();
    }
    float* out = p.splitk > 1 ? slabs : T;
    launch_wgrad_bf16(p, stream, x, ld_x, dxs, ldx, F, num_nodes, out);
    if (p.splitk > 1) {
      splitk_reduce(stream, slabs, p.splitk, (int64_t)F, (int64_t)ldx, T, (int64_t)ldx);
    }
  } else if (weights) {
    // T[f][o] = Σ_k x[k][f] · dxs[k][o]   (both operands k-strided)
    const bool avec = ((uintptr_t)x % 16 == 0) && (ld_x % 4 == 0);
    const bool bvec = ((uintptr_t)dxs % 16 == 0) && (ldx % 4 == 0);
    const SlabPlan p = slab_plan(F, ldx, num_nodes, avec && bvec, ld_x, ldx);
    float* out = p.splitk > 1 ? slabs : T;
    launch_wgrad_slabs(p, stream, x, ld_x, dxs, ldx, F, ldx, num_nodes, avec, bvec, out);
    if (p.splitk > 1) {
      splitk_reduce(stream, slabs, p.splitk, (int64_t)F, (int64_t)ldx, T, (int64_t)ldx);
    }
  }
  const int nft = (F + WG_FT - 1) / WG_FT, not_ = (HC + WG_OT - 1) / WG_OT;
  const int ntile = gW ? nft * not_ : 0;
  const int natt = (g_att_src || g_att_dst) ? (HC + ATT_RB - 1) / ATT_RB : 0;
  size_t lds = 0;
  if (natt) {
    const int nh_max = std::min(H, (ATT_RB - 1) / C + 2);
    lds = sizeof(float) * 2 * (size_t)nh_max * F;
    if (lds > 140 * 1024) return SV2N_ERR_SHAPE;
    static bool attr = [] {
      (void)hipFuncSetAttribute((const void*)k_wgrad_epi,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 140 * 1024);
      return true;
    }();
    (void)attr;
  }
  const int nbias = bias ? (bias_len + 15) / 16 : 0;
  hipLaunchKernelGGL(k_wgrad_epi, dim3((unsigned)(ntile + natt + nbias)), dim3(256), lds, stream, T,
                     ldx, W, att_src, att_dst, H, C, F, gW, g_att_src, g_att_dst, ntile, nft, natt,
                     dbias_partial, num_parts, bias_len, g_bias);
  return (int)hipGetLastError();
}
