// Fused GAT attention for dense-block graphs of 32 < n <= 256 nodes (the
// SURVEY.md §8d C5 stress shapes and any larger block batch) — the same PyG
// 2.3.0 GATConv semantics as sv2n_attn.hip (reference utils/models.py:146 ->
// GATConv.forward), re-tiled for rows that no
// longer fit one 32-lane half.
//
// Edge logits come as per-layer head planes [H][E] in edge order (what
// sv2n_edge_logits_fwd_planes writes with fully coalesced stores).  In the
// canonical order (reference utils/dataset.py:216-226) the logit of (target
// i <- source j) sits at
//     j > i:  U + off(i) + (j-i-1)   — contiguous along the row's sources,
//     j < i:  off(j) + (i-j-1)       — contiguous along the block's targets,
// (U = n(n-1)/2, off(u) = u(2n-u-1)/2), so the lanes that own a row load its
// logits straight into registers with one add per element (off(j)-j-1 is a
// per-lane constant): row runs for the upper part, 16-B runs shared by the
// four rows of a wave for the lower part, which the block's other waves
// complete from the same lines.  No LDS staging of the logits.  Block
// layouts (any order, missing edges) read an [N][n] edge-id map instead.
//
// * one workgroup (4 waves) per (graph g, head h); blockIdx is remapped so the
//   H head-workgroups of a graph run on the same XCD (shared L2 for the xs
//   rows they all read);
// * targets are walked in blocks of TB = 16 rows; within a block, 16-lane
//   group gq of wave w owns target row r = 4w + gq and lane q of the group
//   sources j = 64c + 4q + s (c, s = 0..3): four b128 loads per row, the
//   softmax max / sums are 16-lane DPP reductions (row_ror 8, 4, quad xor);
// * a_src of the lane's 16 sources stays in registers for the whole graph;
// * the products run on v_mfma_f32_16x16x4_f32 (exact f32) from LDS:
//     forward   out_h[i]  = Σ_j P[i][j] · xs_h[j]        (TB x C, K = n, split over waves)
//     backward  dP[i][j]  = Σ_c dOut[i][c] · xs_h[j][c]  (TB x n, K = C)
//               dxs_h[j] += Σ_i P[i][j] · dOut[i]        (n x C, K = TB per block,
//                                                         accumulated in VGPRs)
// * the next block's logit rows (and, backward, its dy / y rows) are loaded
//   into registers while the current block is computed; the backward's
//   d-logit rows go out as b128 stores after the next block's loads were
//   issued (gfx950 retires loads and stores on one in-order vmcnt);
// * nothing is saved between forward and backward except the layer output:
//   the backward recomputes P from xs and the logits (its HBM cost equals
//   reading a saved P, and the forward skips writing one);
// * concat = False (mean over heads) needs a cross-head sum: the forward then
//   writes per-head aggregates to a workspace and k_head_mean finishes
//   mean + bias + activation.
#include "sv2n_common.h"

#include <algorithm>

namespace sv2n {

constexpr int TT = 256;        // threads per workgroup
constexpr int TB = 16;         // target rows per block
constexpr int TILED_MAX_N = 256;
constexpr int TILED_MAX_C = 64;

typedef float f4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int round_up(int a, int m) { return (a + m - 1) / m * m; }

// 16-lane row reductions: row_ror 8, row_ror 4, then quad xor 2 and 1.  Every
// lane of the row ends with the same bits (each step adds two equal pairs).
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dppf<0x128>(v);
  v += dppf<0x124>(v);
  v += dppf<0x4E>(v);
  v += dppf<0xB1>(v);
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dppf<0x128>(v));
  v = fmaxf(v, dppf<0x124>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0xB1>(v));
  return v;
}

// blockIdx -> (graph, head) so that consecutive heads of a graph land on the
// same XCD (hardware round-robins blockIdx over the 8 XCDs); identity when the
// grid is not a multiple of 8.
__device__ __forceinline__ void block_gh(int H, int64_t& g, int& h) {
  const int64_t nb = (int64_t)gridDim.x;
  int64_t b = blockIdx.x;
  if ((nb & 7) == 0) b = (b & 7) * (nb >> 3) + (b >> 3);
  g = b / H;
  h = (int)(b - g * H);
}

// source of element k (0..15) of lane q
__device__ __forceinline__ int src_of(int q, int k) { return 64 * (k >> 2) + 4 * q + (k & 3); }

__device__ __forceinline__ int tri_off(int n, int u) { return u * (2 * n - u - 1) / 2; }

// Per-lane constants of the graph: a_src of the lane's sources (0 past n)
// and kmax, the number of the lane's sources below n (src_of rises with k).
struct LaneConst {
  float as[16];
  int kmax;
};

__device__ __forceinline__ void init_lane_const(LaneConst& K, rsrc_t rxs, int n, int q, int ldx,
                                                int asoff) {
  K.kmax = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int j = src_of(q, k);
    K.as[k] = bld(rxs, j < n ? 4 * (j * ldx + asoff) : OOB);
    K.kmax += j < n ? 1 : 0;
  }
}

// in-plane offset (floats) of (target i <- source j) in canonical order, or
// -1 for the self slot / past n.  Selects only: a divergent early return per
// element made the compiler emit an exec-masked branch region per element.
__device__ __forceinline__ int canon_logit_id(int upb, int i, int j, int n) {
  const int id = j > i ? upb + j : tri_off(n, j) - j - 1 + i;
  return (i < n && j < n && j != i) ? id : -1;
}
// the same through an edge-id map row (erow = (g*n + i)*n).  The load is
// unconditional (a branch per element costs an exec-masked region); a row
// past n (the padding rows of a graph's last target block, which for the
// last graph lie past the end of the map) reads element 0 instead.
__device__ __forceinline__ int eid_logit_id(const int32_t* __restrict__ eid, int64_t erow, int i,
                                            int j, int n, int64_t ext = 0) {
  const bool ok = i < n && j < n && j != i;
  if (ok) SV2N_CHK(101, erow + j, ext);  // ext: N·n, the map's entries
  const int e = eid[ok ? erow + j : 0];
  return ok ? e : -1;
}

// One target row's inputs, loaded one block ahead.
struct RowIn {
  float e[16];  // logits of the lane's sources
  float ad;     // a_dst[i]
};

// rae spans the graph's slice of the head plane (canonical) or the whole
// plane (edge-id map: erow = (g*n + i)*n).
__device__ __forceinline__ void load_row(RowIn& R, rsrc_t rae, rsrc_t rxs, const LaneConst& K,
                                         const int32_t* __restrict__ eid, int64_t erow, int i,
                                         int n, int U, int q, int adoff, int ldx,
                                         int64_t ext = 0) {
  int id[16];
  if (eid) {
#pragma unroll
    for (int k = 0; k < 16; ++k) id[k] = eid_logit_id(eid, erow, i, src_of(q, k), n, ext);
  } else {
    const int upb = U + tri_off(n, i) - i - 1;
#pragma unroll
    for (int k = 0; k < 16; ++k) id[k] = canon_logit_id(upb, i, src_of(q, k), n);
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) R.e[k] = bld(rae, id[k] >= 0 ? 4 * id[k] : OOB);
  R.ad = bld(rxs, i < n ? 4 * (i * ldx + adoff) : OOB);
}

__device__ __forceinline__ void unpack(float (&e)[16], const RowIn& R) {
#pragma unroll
  for (int k = 0; k < 16; ++k) e[k] = R.e[k];
}

// What the softmax of one row yields.  e[] is consumed (zeroed where absent);
// bit k of negm is leaky_relu's negative branch of element k (backward).
struct RowSoft {
  float p[16];
  uint32_t negm;
  float cnt;
  int kd;  // this lane's element index of the self loop, -1 if none
};

// general: a rowmask is given (absent edges are selected away); otherwise
// every off-diagonal source below n is an edge.
__device__ __forceinline__ void row_softmax(RowSoft& S, float (&e)[16], const LaneConst& K,
                                            float ad, int i, int n, int q, bool general,
                                            const uint32_t* __restrict__ rowmask, int64_t grow,
                                            bool has_ae, float slope, int64_t nrows = 0) {
  const int kd = ((i >> 2) & 15) == q ? 4 * (i >> 6) + (i & 3) : -1;
  S.kd = kd;
  float esum = 0.f;
  uint32_t valid;
  if (general) {
    uint32_t pres = 0u;
    const int W = (n + 31) >> 5;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int j = src_of(q, k);
      const bool in = i < n && j < n && j != i;
      if (rowmask && in) SV2N_CHK(102, grow * W + (j >> 5), nrows * W);
      // rows past n (last graph: past the end of the mask) read word 0
      const uint32_t w = rowmask ? rowmask[in ? grow * W + (j >> 5) : 0] : ~0u;
      pres |= ((in && ((w >> (j & 31)) & 1u)) ? 1u : 0u) << k;
    }
    valid = pres | (kd >= 0 ? (1u << kd) : 0u);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      e[k] = ((pres >> k) & 1u) ? e[k] : 0.f;
      esum += e[k];
    }
    S.cnt = row16_sum((float)__popc(pres));
  } else {
    // sources past n and the (never stored) self slot load 0
    valid = (1u << K.kmax) - 1u;
    esum = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) esum += e[k];
    S.cnt = (float)(n - 1);
  }
  esum = row16_sum(esum);
  const float loopv = (has_ae && S.cnt > 0.f) ? esum / S.cnt : 0.f;
  float mx = -INFINITY;
  S.negm = 0u;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    float v = K.as[k] + ad;
    v += (k == kd) ? loopv : e[k];
    const bool pos = v > 0.f;
    S.negm |= pos ? 0u : (1u << k);
    const float lr = pos ? v : v * slope;
    const float s = ((valid >> k) & 1u) ? lr : -INFINITY;
    S.p[k] = s;
    mx = fmaxf(mx, s);
  }
  mx = row16_max(mx);
  float den = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    S.p[k] = expf(S.p[k] - mx);  // exp(-inf) = 0 for masked sources
    den += S.p[k];
  }
  den = row16_sum(den);
  const float inv = 1.f / (den + 1e-16f);
#pragma unroll
  for (int k = 0; k < 16; ++k) S.p[k] *= inv;
}

// keep[((g*H+h)*n + i)*n + j] of the lane's 16 sources (dropout on attention)
__device__ __forceinline__ uint32_t keep_bits(const uint8_t* __restrict__ keep, int64_t base,
                                              int i, int n, int q, int64_t ext = 0) {
  uint32_t kb = 0u;
  if (i < n) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int j = src_of(q, k);
      if (j < n) SV2N_CHK(103, base + (int64_t)i * n + j, ext);
      if (j < n && keep[base + (int64_t)i * n + j]) kb |= 1u << k;
    }
  }
  return kb;
}

// head plane h of a layer: the graph's slice (canonical order) or the whole
// plane (edge-id map); a null plane reads 0 / drops stores
__device__ __forceinline__ rsrc_t plane_rsrc(const float* planes, int64_t E,
                                             const int32_t* eid, int64_t g, int h, int n) {
  if (!planes) return make_rsrc(nullptr, 0u);
  const float* p = planes + (int64_t)h * E;
  if (eid) return make_rsrc(p, (uint32_t)(4 * E));
  const int64_t E0 = (int64_t)n * (n - 1);
  return make_rsrc(p + g * E0, (uint32_t)(4 * E0));
}

// d(edge logit) rows of target block [i0, i0+TB), staged in s[r][j] (row
// stride PS), to the canonical-order plane slice: the block is cut into 16x16
// source tiles, tile k = t>>4 served by 16 threads (q = t&15):
//   above the block's diagonal tile: element m = (r = m, j = 16k+q) -> lanes along j
//   at or below it:                  element m = (r = q, j = 16k+m) -> lanes along i
// so every store instruction writes 16-lane runs of consecutive ids (64 B).
__device__ __forceinline__ void store_block_dae(const float* __restrict__ sl, int PS, int i0,
                                                int t, rsrc_t rdae, int n, int U, int NP) {
  const int k = t >> 4, q = t & 15;
  if (16 * k >= NP) return;
  const bool along_j = k > (i0 >> 4);
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int r = along_j ? m : q, j = 16 * k + (along_j ? q : m);
    const int i = i0 + r;
    const int id = canon_logit_id(U + tri_off(n, i) - i - 1, i, j, n);
    bst(rdae, id >= 0 ? 4 * id : OOB, sl[r * PS + j]);
  }
}

__device__ __forceinline__ void store_row4(float* __restrict__ dst, int NP, int q, bool rv,
                                           const float (&v)[16]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int j0 = 64 * c + 4 * q;
    if (j0 < NP)
      *reinterpret_cast<f4*>(dst + j0) =
          rv ? f4{v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]} : f4{0.f, 0.f, 0.f, 0.f};
  }
}

// ---------------------------------------------------------------------------
// forward
// LDS: sXT [CW][XT] xs_hᵀ (B operand, b128 along sources) | sP [TB][PS] P rows
//      (A operand, b128 along sources) | sR [4][CW][SRS] K-split partials,
//      column-major (one 16-B store per tile: the row-major scalar form was
//      miscompiled into ds_write2 with wrong offsets by this toolchain at CT = 4)
// ---------------------------------------------------------------------------
template <int ACT, bool CONCAT, int CT>
__global__ __launch_bounds__(TT) void k_attn_tiled_fwd(
    const float* __restrict__ xs, int ldx, const float* __restrict__ ae_planes, int64_t E,
    const int32_t* __restrict__ eid, const uint32_t* __restrict__ rowmask,
    const float* __restrict__ bias, const uint8_t* __restrict__ keep, float keep_scale,
    float* __restrict__ out, int n, int H, int C, float slope) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int CW = 16 * CT;
  constexpr int SRS = TB + 4;
  const int NP = round_up(n, 16);
  const int XT = NP + 4, PS = NP + 4;
  float* sXT = smem;              // [CW][XT]
  float* sP = sXT + CW * XT;      // [TB][PS]
  float* sR = sP + TB * PS;       // [4][CW][SRS]

  int64_t g;
  int h;
  block_gh(H, g, h);
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int gq = lane >> 4, q = lane & 15;
  const int64_t row0 = g * n;
  const int HC = H * C;
  const bool general = rowmask != nullptr;
  const bool has_ae = ae_planes != nullptr;
  const rsrc_t rae = plane_rsrc(ae_planes, E, eid, g, h, n);
  const rsrc_t rxs = make_rsrc(xs + row0 * ldx, (uint32_t)(4 * n * ldx));
  const int U = (n * (n - 1)) / 2;
  const int64_t Nrows = (int64_t)gridDim.x / H * n;  // bound checks (SV2N_CHK) only

  LaneConst K;
  init_lane_const(K, rxs, n, q, ldx, HC + h);
  RowIn R;
  load_row(R, rae, rxs, K, eid, (row0 + wave * 4 + gq) * n, wave * 4 + gq, n, U, q, HC + H + h,
           ldx, Nrows * n);
  for (int idx = t; idx < NP * CW; idx += TT) {
    const int j = idx / CW, c = idx - j * CW;
    if (j < n && c < C) SV2N_CHK(104, (row0 + j) * ldx + h * C + c, Nrows * ldx);
    sXT[c * XT + j] = (j < n && c < C) ? xs[(row0 + j) * ldx + h * C + c] : 0.f;
  }
  const int64_t kbase = (g * H + h) * (int64_t)n * n;

  const int li = lane & 15, lk = lane >> 4;
  const int kq = NP / 4;  // K-split: wave w sums sources [w*kq, (w+1)*kq), kq % 4 == 0
  for (int i0 = 0; i0 < n; i0 += TB) {
    const int r = wave * 4 + gq, i = i0 + r;
    // ---- softmax of row i (16-lane group), P -> sP ----
    {
      float e[16];
      unpack(e, R);
      const float ad = R.ad;
      if (i0 + TB < n)
        load_row(R, rae, rxs, K, eid, (row0 + i + TB) * n, i + TB, n, U, q, HC + H + h, ldx,
                 Nrows * n);
      RowSoft S;
      row_softmax(S, e, K, ad, i, n, q, general, rowmask, row0 + i, has_ae, slope, Nrows);
      if (keep) {
        const uint32_t kb = keep_bits(keep, kbase, i, n, q, Nrows * H * n);
#pragma unroll
        for (int k = 0; k < 16; ++k) S.p[k] = ((kb >> k) & 1u) ? S.p[k] * keep_scale : 0.f;
      }
      store_row4(sP + r * PS, NP, q, i < n, S.p);
    }
    __syncthreads();
    // ---- out[i][c] = Σ_j P[i][j] xs_h[j][c], K split over the 4 waves ----
    {
      f4 acc[CT];
#pragma unroll
      for (int b = 0; b < CT; ++b) acc[b] = f4{0.f, 0.f, 0.f, 0.f};
      // lane (li, lk) feeds k = k0 + 4lk + s at MFMA step s of a 16-wide k
      // chunk (every k of the chunk once: the order of the sum is permuted)
      for (int k0 = wave * kq; k0 < (wave + 1) * kq; k0 += 16) {
        const int kk = min(k0 + 4 * lk, NP - 4);
        const bool kin = k0 + 4 * lk < (wave + 1) * kq;
        const f4 a = kin ? *reinterpret_cast<const f4*>(sP + li * PS + kk) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b = 0; b < CT; ++b) {
          const f4 bb = *reinterpret_cast<const f4*>(sXT + (16 * b + li) * XT + kk);
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bb.x, acc[b], 0, 0, 0);
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bb.y, acc[b], 0, 0, 0);
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bb.z, acc[b], 0, 0, 0);
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bb.w, acc[b], 0, 0, 0);
        }
      }
      // D layout: acc[b][rr] = out[row 4lk + rr][col 16b + li]
#pragma unroll
      for (int b = 0; b < CT; ++b)
        *reinterpret_cast<f4*>(sR + (wave * CW + 16 * b + li) * SRS + 4 * lk) = acc[b];
    }
    __syncthreads();
    for (int idx = t; idx < TB * CW; idx += TT) {
      const int rr = idx / CW, c = idx - rr * CW;
      const int ii = i0 + rr;
      if (ii < n && c < C) {
        SV2N_CHK(105, (row0 + ii) * HC + h * C + c, Nrows * HC);
        const float* pr = sR + c * SRS + rr;
        const float v = (pr[0] + pr[CW * SRS]) + (pr[2 * CW * SRS] + pr[3 * CW * SRS]);
        if (CONCAT) {
          const float b = bias ? bias[h * C + c] : 0.f;
          out[(row0 + ii) * HC + h * C + c] = act_fwd<ACT>(v + b);
        } else {
          out[(row0 + ii) * HC + h * C + c] = v;  // workspace, per head
        }
      }
    }
    // sP is rewritten only after every wave passed this block's second
    // barrier; sR only after the next block's first
  }
}

// mean over heads + bias + activation (concat = False)
template <int ACT>
__global__ __launch_bounds__(256) void k_head_mean(const float* __restrict__ ws,
                                                   const float* __restrict__ bias,
                                                   float* __restrict__ y, int64_t N, int H,
                                                   int C) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= N * C) return;
  const int64_t row = idx / C;
  const int c = (int)(idx - row * C);
  const float* w = ws + row * H * C + c;
  SV2N_CHK(106, row * H * C + c + (H - 1) * C, N * H * C);
  float s = 0.f;
  for (int h = 0; h < H; ++h) s += w[h * C];
  y[idx] = act_fwd<ACT>(s * (1.f / (float)H) + (bias ? bias[c] : 0.f));
}

// ---------------------------------------------------------------------------
// backward
//   dz = act'(y)·dy; dOut_h = dz (concat slice h) or dz / H (mean);
//   P recomputed; dPd = dOut·xs_hᵀ; dP = dropout-bwd(dPd);
//   dS = P ⊙ (dP − Σ_j P dP); dL = dS · leaky'(s);
//   dae[i][j] = dL[i][j] + dL[i][i] / cnt  (present j),  a_d[i] += Σ_j dL,
//   a_s[j] += Σ_i dL[i][j],  dxs_h[j] += Σ_i Pd[i][j] dOut[i]
// LDS: sX [NP][XR] xs_h rows (dPd's B, b128 along c) | sP [TB][PS] Pd rows |
//      sL [TB][PS] dPd rows | sO [2][TB][OS] dOut (double-buffered)
// ---------------------------------------------------------------------------
template <int ACT, bool CONCAT, int CT>
__global__ __launch_bounds__(TT, 2) void k_attn_tiled_bwd(
    const float* __restrict__ dy, const float* __restrict__ y, const float* __restrict__ xs,
    int ldx, const float* __restrict__ ae_planes, int64_t E, const int32_t* __restrict__ eid,
    const uint8_t* __restrict__ keep, float keep_scale, const uint32_t* __restrict__ rowmask,
    float* __restrict__ dxs, float* __restrict__ dae_planes, float* __restrict__ dbias, int n,
    int H, int C, float slope) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int CW = 16 * CT;
  constexpr int XR = CW + 4;
  constexpr int OS = CW + 4;
  const int NP = round_up(n, 16);
  const int PS = NP + 4;
  float* sX = smem;               // [NP][XR]
  float* sP = sX + NP * XR;       // [TB][PS]
  float* sL = sP + TB * PS;       // [TB][PS]
  float* sO = sL + TB * PS;       // [2][TB][OS]

  int64_t g;
  int h;
  block_gh(H, g, h);
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int gq = lane >> 4, q = lane & 15;
  const int64_t row0 = g * n;
  const int HC = H * C;
  const int OC = CONCAT ? HC : C;
  const int oc0 = CONCAT ? h * C : 0;
  const float oscale = CONCAT ? 1.f : 1.f / (float)H;
  const bool general = rowmask != nullptr;
  const bool has_ae = ae_planes != nullptr;
  const rsrc_t rae = plane_rsrc(ae_planes, E, eid, g, h, n);
  const rsrc_t rdae = plane_rsrc(dae_planes, E, eid, g, h, n);
  const int U = (n * (n - 1)) / 2;
  const rsrc_t rxs = make_rsrc(xs + row0 * ldx, (uint32_t)(4 * n * ldx));
  const rsrc_t rdy = make_rsrc(dy + row0 * OC, (uint32_t)(4 * n * OC));
  const rsrc_t ry = make_rsrc(y + row0 * OC, (uint32_t)(4 * n * OC));
  const int64_t Nrows = (int64_t)gridDim.x / H * n;  // bound checks (SV2N_CHK) only

  // dOut rows of a block: TB*CW values, CT per thread
  float pdy[CT], py[CT];
  auto load_dout = [&](int i0n) {
#pragma unroll
    for (int m = 0; m < CT; ++m) {
      const int idx = t + TT * m, rr = idx / CW, c = idx - rr * CW, ii = i0n + rr;
      const int off = (ii < n && c < C) ? 4 * (ii * OC + oc0 + c) : OOB;
      pdy[m] = bld(rdy, off);
      py[m] = bld(ry, off);
    }
  };

  LaneConst K;
  init_lane_const(K, rxs, n, q, ldx, HC + h);
  RowIn R;
  load_row(R, rae, rxs, K, eid, (row0 + wave * 4 + gq) * n, wave * 4 + gq, n, U, q, HC + H + h,
           ldx, Nrows * n);
  load_dout(0);
  for (int idx = t; idx < NP * CW; idx += TT) {
    const int j = idx / CW, c = idx - j * CW;
    if (j < n && c < C) SV2N_CHK(107, (row0 + j) * ldx + h * C + c, Nrows * ldx);
    sX[j * XR + c] = (j < n && c < C) ? xs[(row0 + j) * ldx + h * C + c] : 0.f;
  }
  const int64_t kbase = (g * H + h) * (int64_t)n * n;

  // dxs accumulators: wave w owns row tiles jt = w, w+4, ... (NP/16 <= 16) x CT column tiles
  constexpr int MAXJT = TILED_MAX_N / 16 / 4;
  f4 dacc[MAXJT][CT];
#pragma unroll
  for (int a = 0; a < MAXJT; ++a)
#pragma unroll
    for (int b = 0; b < CT; ++b) dacc[a][b] = f4{0.f, 0.f, 0.f, 0.f};
  float das[16];  // Σ_i dL[i][j] over this lane group's rows, per source of the lane
#pragma unroll
  for (int k = 0; k < 16; ++k) das[k] = 0.f;
  float dbias_acc = 0.f;  // thread t < C owns bias column t of this head's slice
  const int li = lane & 15, lk = lane >> 4;
  const int njt = NP / 16;

  int buf = 0;
  for (int i0 = 0; i0 < n; i0 += TB, buf ^= 1) {
    float* sOb = sO + buf * TB * OS;
    // ---- stage dOut (prefetched) ----
#pragma unroll
    for (int m = 0; m < CT; ++m) {
      const int idx = t + TT * m, rr = idx / CW, c = idx - rr * CW;
      sOb[rr * OS + c] = act_bwd<ACT>(pdy[m], py[m]) * oscale;
    }
    __syncthreads();
    if (t < C && (CONCAT || h == 0)) {
      float s = 0.f;
      for (int rr = 0; rr < TB; ++rr) s += sOb[rr * OS + t];
      dbias_acc += s / oscale;  // = Σ dz
    }
    // ---- dPd[i][j] = Σ_c dOut[i][c] xs_h[j][c]: tiles over j, waves stride ----
    for (int jt = wave; jt < njt; jt += 4) {
      f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < CW; kb += 16) {
        const f4 a = *reinterpret_cast<const f4*>(sOb + li * OS + kb + 4 * lk);
        const f4 bb = *reinterpret_cast<const f4*>(sX + (16 * jt + li) * XR + kb + 4 * lk);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bb.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bb.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bb.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bb.w, acc, 0, 0, 0);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) sL[(4 * lk + rr) * PS + 16 * jt + li] = acc[rr];
    }
    __syncthreads();
    // ---- rows: recompute P, softmax / leaky / dropout backward ----
    {
      const int r = wave * 4 + gq, i = i0 + r;
      const bool rv = i < n;
      float e[16];
      unpack(e, R);
      const float ad = R.ad;
      if (i0 + TB < n) {
        load_row(R, rae, rxs, K, eid, (row0 + i + TB) * n, i + TB, n, U, q, HC + H + h, ldx,
                 Nrows * n);
        load_dout(i0 + TB);
      }
      RowSoft S;
      row_softmax(S, e, K, ad, i, n, q, general, rowmask, row0 + i, has_ae, slope, Nrows);
      float d[16];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int j0 = 64 * c + 4 * q;
        const f4 v = j0 < NP ? *reinterpret_cast<const f4*>(sL + r * PS + j0)
                             : f4{0.f, 0.f, 0.f, 0.f};
        d[4 * c] = v.x;
        d[4 * c + 1] = v.y;
        d[4 * c + 2] = v.z;
        d[4 * c + 3] = v.w;
      }
      float pd[16];
      if (keep) {
        const uint32_t kb = keep_bits(keep, kbase, i, n, q, Nrows * H * n);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const bool kp = (kb >> k) & 1u;
          d[k] = kp ? d[k] * keep_scale : 0.f;
          pd[k] = kp ? S.p[k] * keep_scale : 0.f;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) pd[k] = S.p[k];
      }
      float dot = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) dot = fmaf(S.p[k], d[k], dot);
      dot = row16_sum(dot);
      float rsum = 0.f, dloop = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float ds = S.p[k] * (d[k] - dot);
        const float dl = ((S.negm >> k) & 1u) ? ds * slope : ds;
        d[k] = rv ? dl : 0.f;
        rsum += d[k];
        dloop = (k == S.kd) ? d[k] : dloop;
        das[k] += d[k];
      }
      rsum = row16_sum(rsum);
      dloop = row16_sum(dloop);  // one lane holds it, the others add 0
      if (rv && q == 0) SV2N_CHK(108, (row0 + i) * ldx + HC + H + h, Nrows * ldx);
      if (rv && q == 0) dxs[(row0 + i) * ldx + HC + H + h] = rsum;  // d a_dst
      const float dshare = (has_ae && S.cnt > 0.f) ? dloop / S.cnt : 0.f;
      // d(edge logit) of every present edge of the row: with an edge-id map
      // straight from the lanes; in canonical order staged in this group's own
      // sL row (its dPd was read above) and written tile-wise below
      if (dae_planes && eid) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          // eid holds -1 for absent edges (rowmask agrees)
          const int id = eid_logit_id(eid, (row0 + i) * n, i, src_of(q, k), n, Nrows * n);
          bst(rdae, id >= 0 ? 4 * id : OOB, d[k] + dshare);
        }
      } else if (dae_planes) {
        float dv[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) dv[k] = d[k] + dshare;
        store_row4(sL + r * PS, NP, q, rv, dv);
      }
      store_row4(sP + r * PS, NP, q, rv, pd);
    }
    __syncthreads();
    if (dae_planes && !eid) store_block_dae(sL, PS, i0, t, rdae, n, U, NP);
    // ---- dxs_h += Pdᵀ · dOut ----
#pragma unroll
    for (int a = 0; a < MAXJT; ++a) {
      const int jt = wave + 4 * a;
      if (jt < njt) {
        const float* pa = sP + lk * PS + 16 * jt + li;  // Pᵀ[j][i] = P[i][j]
#pragma unroll
        for (int b = 0; b < CT; ++b) {
          const float* ob = sOb + lk * OS + 16 * b + li;
#pragma unroll
          for (int k = 0; k < TB; k += 4)
            dacc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[k * PS], ob[k * OS], dacc[a][b],
                                                              0, 0, 0);
        }
      }
    }
    // sP / sL are rewritten only after the next block's first barrier, sO
    // is double-buffered
  }
  // ---- d a_src: sum das over the 4 lane groups of each wave, then the waves ----
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    das[k] += __shfl_xor(das[k], 16, 64);
    das[k] += __shfl_xor(das[k], 32, 64);
  }
  __syncthreads();
  float* sDa = sP;  // [4][NP] <= 2 * TB * PS floats (sP, sL are free now)
  if (gq == 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int j = src_of(q, k);
      if (j < NP) sDa[wave * NP + j] = das[k];
    }
  }
  __syncthreads();
  for (int j = t; j < n; j += TT) {
    SV2N_CHK(109, (row0 + j) * ldx + HC + h, Nrows * ldx);
    dxs[(row0 + j) * ldx + HC + h] = (sDa[j] + sDa[NP + j]) + (sDa[2 * NP + j] + sDa[3 * NP + j]);
  }
  // ---- write dxs_h, padding columns, bias partial ----
#pragma unroll
  for (int a = 0; a < MAXJT; ++a) {
    const int jt = wave + 4 * a;
    if (jt < njt) {
#pragma unroll
      for (int b = 0; b < CT; ++b) {
        const int c = 16 * b + li;
        if (c < C) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int j = 16 * jt + 4 * lk + rr;
            if (j < n) SV2N_CHK(110, (row0 + j) * ldx + h * C + c, Nrows * ldx);
            if (j < n) dxs[(row0 + j) * ldx + h * C + c] = dacc[a][b][rr];
          }
        }
      }
    }
  }
  if (h == 0) {
    const int padc = ldx - HC - 2 * H;
    for (int idx = t; idx < n * padc; idx += TT) {
      const int j = idx / padc;
      SV2N_CHK(111, (row0 + j) * ldx + HC + 2 * H + (idx - j * padc), Nrows * ldx);
      dxs[(row0 + j) * ldx + HC + 2 * H + (idx - j * padc)] = 0.f;
    }
  }
  if (t < C && (CONCAT || h == 0)) SV2N_CHK(112, g * OC + oc0 + t, Nrows / n * OC);
  if (t < C && (CONCAT || h == 0)) dbias[g * OC + oc0 + t] = dbias_acc;
}

}  // namespace sv2n

SV2N_CHK_EXPORT(tiled)

// ============================ C-ABI ========================================
using namespace sv2n;

static int ct_of(int C) { return (C + 15) / 16; }

static size_t tiled_fwd_lds(int n, int C) {
  const int CW = 16 * ct_of(C), NP = round_up(n, 16);
  return sizeof(float) *
         ((size_t)CW * (NP + 4) + (size_t)TB * (NP + 4) + (size_t)4 * CW * (TB + 4));
}
static size_t tiled_bwd_lds(int n, int C) {
  const int CW = 16 * ct_of(C), NP = round_up(n, 16);
  return sizeof(float) * ((size_t)NP * (CW + 4) + 2 * (size_t)TB * (NP + 4) +
                          2 * (size_t)TB * (CW + 4));
}

template <typename K>
static void raise_lds_tiled(K kernel, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
}

static int check_tiled(int64_t B, int n, int H, int C, int ldx, int act) {
  if (B <= 0 || C <= 0 || n <= 0) return SV2N_ERR_ARG;
  if (n > TILED_MAX_N || H < 1 || H > SV2N_MAX_HEADS || C > TILED_MAX_C || act < 0 || act > 3)
    return SV2N_ERR_SHAPE;
  if (ldx < H * C + 2 * H) return SV2N_ERR_SHAPE;
  if (B * H > 0x7fffffff) return SV2N_ERR_SHAPE;
  if ((int64_t)n * ldx * 4 > 0x7fffffff) return SV2N_ERR_SHAPE;  // 32-bit buffer offsets
  return 0;
}

template <int ACT, bool CONCAT, int CT>
static void tiled_fwd_launch(int64_t B, hipStream_t st, const float* xs, int ldx, const float* ae,
                             int64_t E, const int32_t* eid, const uint32_t* rowmask,
                             const float* bias, const uint8_t* keep, float ks, float* out, int n,
                             int H, int C, float slope) {
  const size_t lds = tiled_fwd_lds(n, C);
  raise_lds_tiled(k_attn_tiled_fwd<ACT, CONCAT, CT>, lds);
  hipLaunchKernelGGL((k_attn_tiled_fwd<ACT, CONCAT, CT>), dim3((unsigned)(B * H)), dim3(TT), lds,
                     st, xs, ldx, ae, E, eid, rowmask, bias, keep, ks, out, n, H, C, slope);
}

template <int ACT, bool CONCAT, int CT>
static void tiled_bwd_launch(int64_t B, hipStream_t st, const float* dy, const float* y,
                             const float* xs, int ldx, const float* ae, int64_t E,
                             const int32_t* eid, const uint8_t* keep, float ks,
                             const uint32_t* rowmask, float* dxs, float* dae, float* dbias, int n,
                             int H, int C, float slope) {
  const size_t lds = tiled_bwd_lds(n, C);
  raise_lds_tiled(k_attn_tiled_bwd<ACT, CONCAT, CT>, lds);
  hipLaunchKernelGGL((k_attn_tiled_bwd<ACT, CONCAT, CT>), dim3((unsigned)(B * H)), dim3(TT), lds,
                     st, dy, y, xs, ldx, ae, E, eid, keep, ks, rowmask, dxs, dae, dbias, n, H, C,
                     slope);
}

#define SV2N_TILED_CT(FN, ACT, CONCAT, ...)                 \
  switch (ct_of(C)) {                                       \
    case 1: FN<ACT, CONCAT, 1>(__VA_ARGS__); break;         \
    case 2: FN<ACT, CONCAT, 2>(__VA_ARGS__); break;         \
    case 3: FN<ACT, CONCAT, 3>(__VA_ARGS__); break;         \
    default: FN<ACT, CONCAT, 4>(__VA_ARGS__); break;        \
  }
#define SV2N_TILED_ACT(FN, CONCAT, ...)                     \
  switch (act) {                                            \
    case 0: SV2N_TILED_CT(FN, 0, CONCAT, __VA_ARGS__) break; \
    case 1: SV2N_TILED_CT(FN, 1, CONCAT, __VA_ARGS__) break; \
    case 2: SV2N_TILED_CT(FN, 2, CONCAT, __VA_ARGS__) break; \
    default: SV2N_TILED_CT(FN, 3, CONCAT, __VA_ARGS__) break; \
  }

extern "C" int64_t sv2n_gat_attn_tiled_workspace(int64_t num_graphs, int n, int heads,
                                                 int channels, int concat) {
  return concat ? 0 : num_graphs * n * (int64_t)heads * channels;
}

// planes are addressed with 32-bit byte offsets
static int check_planes(const float* ae, int64_t num_edges, const int32_t* eid, int64_t B, int n) {
  if (!ae) return 0;
  if (!eid && num_edges != B * (int64_t)n * (n - 1)) return SV2N_ERR_SHAPE;
  if (num_edges * 4 > 0x7fffff00LL) return SV2N_ERR_SHAPE;
  return 0;
}

extern "C" int sv2n_gat_attn_tiled_fwd(const float* xs, int ldx, const float* ae,
                                       int64_t num_edges, const int32_t* eid,
                                       const uint32_t* rowmask, const float* bias,
                                       const uint8_t* keep, float keep_scale, float* y,
                                       float* workspace, int64_t workspace_floats,
                                       int64_t num_graphs, int n, int heads, int channels,
                                       int concat, int act, float negative_slope,
                                       hipStream_t stream) {
  if (!xs || !y) return SV2N_ERR_ARG;
  const int C = channels;
  if (int rc = check_tiled(num_graphs, n, heads, C, ldx, act)) return rc;
  if (int rc = check_planes(ae, num_edges, eid, num_graphs, n)) return rc;
  if (concat) {
    SV2N_TILED_ACT(tiled_fwd_launch, true, num_graphs, stream, xs, ldx, ae, num_edges, eid,
                   rowmask, bias, keep, keep_scale, y, n, heads, C, negative_slope)
  } else {
    const int64_t need = sv2n_gat_attn_tiled_workspace(num_graphs, n, heads, C, 0);
    if (!workspace || workspace_floats < need) return SV2N_ERR_WORKSPACE;
    SV2N_TILED_CT(tiled_fwd_launch, 0, false, num_graphs, stream, xs, ldx, ae, num_edges, eid,
                  rowmask, nullptr, keep, keep_scale, workspace, n, heads, C, negative_slope)
    const int64_t tot = num_graphs * n * (int64_t)C;
    const unsigned grid = (unsigned)((tot + 255) / 256);
    const int64_t N = num_graphs * n;
    switch (act) {
      case 0: hipLaunchKernelGGL(k_head_mean<0>, dim3(grid), dim3(256), 0, stream, workspace, bias, y, N, heads, C); break;
      case 1: hipLaunchKernelGGL(k_head_mean<1>, dim3(grid), dim3(256), 0, stream, workspace, bias, y, N, heads, C); break;
      case 2: hipLaunchKernelGGL(k_head_mean<2>, dim3(grid), dim3(256), 0, stream, workspace, bias, y, N, heads, C); break;
      default: hipLaunchKernelGGL(k_head_mean<3>, dim3(grid), dim3(256), 0, stream, workspace, bias, y, N, heads, C); break;
    }
  }
  return (int)hipGetLastError();
}

extern "C" int sv2n_gat_attn_tiled_bwd(const float* dy, const float* y, const float* xs, int ldx,
                                       const float* ae, int64_t num_edges, const int32_t* eid,
                                       const uint8_t* keep, float keep_scale,
                                       const uint32_t* rowmask, float* dxs, float* dae,
                                       float* dbias_partial, int64_t num_graphs, int n,
                                       int heads, int channels, int concat, int act,
                                       float negative_slope, hipStream_t stream) {
  if (!dy || !y || !xs || !dxs || !dbias_partial) return SV2N_ERR_ARG;
  const int C = channels;
  if (int rc = check_tiled(num_graphs, n, heads, C, ldx, act)) return rc;
  if (int rc = check_planes(ae, num_edges, eid, num_graphs, n)) return rc;
  if (int rc = check_planes(dae, num_edges, eid, num_graphs, n)) return rc;
  const int OC = concat ? heads * C : C;
  if ((int64_t)n * OC * 4 > 0x7fffffff) return SV2N_ERR_SHAPE;
  if (concat) {
    SV2N_TILED_ACT(tiled_bwd_launch, true, num_graphs, stream, dy, y, xs, ldx, ae, num_edges,
                   eid, keep, keep_scale, rowmask, dxs, dae, dbias_partial, n, heads, C,
                   negative_slope)
  } else {
    SV2N_TILED_ACT(tiled_bwd_launch, false, num_graphs, stream, dy, y, xs, ldx, ae, num_edges,
                   eid, keep, keep_scale, rowmask, dxs, dae, dbias_partial, n, heads, C,
                   negative_slope)
  }
  return (int)hipGetLastError();
}
