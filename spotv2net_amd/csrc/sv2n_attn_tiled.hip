// Fused GAT attention for dense-block graphs of 32 < n <= 256 nodes (the
// SURVEY.md §8d C5 stress shapes and any larger block batch) — the same PyG
// 2.3.0 GATConv semantics as sv2n_attn.hip (reference utils/models.py:146 ->
// GATConv.forward), re-tiled for rows that no
// longer fit one 32-lane half:
//
// * one workgroup (4 waves) per (graph g, head h); blockIdx is remapped so the
//   H head-workgroups of a graph run on the same XCD (shared L2 for the xs
//   rows they all read);
// * edge logits come in per-layer head planes AE[h][e] in edge order (what
//   sv2n_edge_logits_fwd_planes writes with fully coalesced stores); edge e of
//   (target i, source j) is computed from the canonical order or read from an
//   eid map [g][i][j] (block layouts).  A target block's first-half edges
//   (sources j < i) are 16 consecutive edge ids per j, so the gathers stay
//   sector-coalesced across the block's rows;
// * targets are walked in blocks of TB = 16 rows; a wave owns a row at a time
//   and its lanes cover sources j = lane + 64q, so the self-loop mean, the
//   softmax max / sum are 64-lane wave reductions;
// * the products run on v_mfma_f32_16x16x4_f32 (exact f32) from LDS:
//     forward   out_h[i]  = Σ_j P[i][j] · xs_h[j]        (TB x C, K = n)
//     backward  dP[i][j]  = Σ_c dOut[i][c] · xs_h[j][c]  (TB x n, K = C)
//               dxs_h[j] += Σ_i P[i][j] · dOut[i]        (n x C, K = TB per block,
//                                                         accumulated in VGPRs)
// * nothing is saved between forward and backward except the layer output:
//   the backward recomputes P from xs and AE (its HBM cost equals reading a
//   saved P, and the forward skips writing one);
// * concat = False (mean over heads) needs a cross-head sum: the forward then
//   writes per-head aggregates to a workspace and k_head_mean finishes
//   mean + bias + activation.
//
// LDS images (floats):
//   sX [NP][XS]  xs_h rows (zero-padded to NP = round_up(n, 16) rows and
//                16*CT columns)
//   sP [TB][PS]  P rows
// ds_read_b32 banks are (addr/4) % 32 per 32-lane half (cdna_hip_programming.md
// §2).  A fragment read "row = lane&15, col = lane>>4" is conflict-free for a
// stride ≡ 2 (mod 32) or odd; "row = lane>>4, col = lane&15" for ≡ 16 (mod 32)
// (odd: one 2-way pair).  Strides below follow the role each image plays.
#include "sv2n_common.h"

#include <algorithm>

namespace sv2n {

constexpr int TT = 256;        // threads per workgroup
constexpr int TB = 16;         // target rows per block
constexpr int TILED_MAX_N = 256;
constexpr int TILED_MAX_C = 64;

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
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

__host__ __device__ constexpr int round_up(int a, int m) { return (a + m - 1) / m * m; }
__host__ __device__ constexpr int pad32(int a, int mod) {  // smallest s >= a, s % 32 == mod
  return a + ((mod - a % 32) + 32) % 32;
}

// In-graph edge index of (target i <- source j) in the CovarianceLaggedDataset
// order (reference utils/dataset.py:216-226: the row-major upper pairs (u < v)
// as u -> v, then the same pairs swapped).  32-bit: n(n-1) < 2^31.
__device__ __forceinline__ int canon_eid(int n, int i, int j) {
  const int u = j > i ? i : j, v = j > i ? j : i;
  return (j > i ? (n * (n - 1)) / 2 : 0) + u * (2 * n - u - 1) / 2 + (v - u - 1);
}

constexpr int RPW = TB / 4;  // rows per wave per target block
constexpr int SRS = TB + 4;  // K-split partial row stride (16-B aligned, fewer conflicts)

// Edge logits of one target block [i0, i0+TB) x sources [0, NP), staged into
// sE[r][j] (row stride SE; -inf where edge j->i is absent or j == i).
//
// In the canonical order (utils/dataset.py:216-226) an upper element (j > i)
// has the in-graph id U + off(i) + (j-i-1), contiguous in j, and a lower one
// (j < i) the id off(j) + (i-j-1), contiguous in i (U = n(n-1)/2,
// off(u) = u(2n-u-1)/2).  The block is cut into 16x16 tiles over sources,
// tile k = t>>4 served by 16 threads (q = t&15), 16 elements each:
//   k above the block's diagonal tile: element m = (r = m, j = 16k+q)  -> lanes along j
//   k at or below it:                  element m = (r = q, j = 16k+m)  -> lanes along i
// so every load instruction reads 16-lane runs of consecutive ids (64 B)
// instead of 64 scattered words, and each thread holds 16 values with 32-bit
// buffer offsets.  With an edge-id map (block layouts) every tile uses the
// first mapping (the eid row reads are then coalesced; the logit gather is
// arbitrary by nature).
__device__ __forceinline__ int tri_off(int n, int u) { return u * (2 * n - u - 1) / 2; }

__device__ __forceinline__ bool mask_bit(const uint32_t* __restrict__ rowmask, int64_t row, int W,
                                         int j) {
  return !rowmask || ((rowmask[row * W + (j >> 5)] >> (j & 31)) & 1u);
}

// element m of thread t in block i0 -> (r, j); `along_j` for the first mapping
__device__ __forceinline__ void tile_elem(int t, int m, bool along_j, int& r, int& j) {
  const int k = t >> 4, q = t & 15;
  r = along_j ? m : q;
  j = 16 * k + (along_j ? q : m);
}
__device__ __forceinline__ bool tile_along_j(int t, int i0, bool has_eid) {
  return has_eid || (t >> 4) > (i0 >> 4);
}

// canonical in-graph id of (i <- j), or -1 when the pair is not an edge slot
__device__ __forceinline__ int canon_id(int n, int U, int i, int j) {
  if (i >= n || j >= n || i == j) return -1;
  return j > i ? U + tri_off(n, i) + (j - i - 1) : tri_off(n, j) + (i - j - 1);
}

struct BlockLoad {
  float v[TB];
  uint32_t valid;  // bit m: element m is a present edge
};

__device__ __forceinline__ void load_block(BlockLoad& L, int i0, int t,
                                           const float* __restrict__ ae,
                                           const int32_t* __restrict__ eid,
                                           const uint32_t* __restrict__ rowmask, int64_t g, int n) {
  const int W = (n + 31) >> 5;
  const bool aj = tile_along_j(t, i0, eid != nullptr);
  L.valid = 0u;
  if (eid) {
#pragma unroll
    for (int m = 0; m < TB; ++m) {
      int r, j;
      tile_elem(t, m, aj, r, j);
      const int i = i0 + r;
      int e = -1;
      if (i < n && j < n && j != i) e = eid[(g * n + i) * n + j];
      L.v[m] = (e >= 0 && ae) ? ae[e] : 0.f;
      L.valid |= (e >= 0 ? 1u : 0u) << m;
    }
    return;
  }
  const int64_t E0 = (int64_t)n * (n - 1);
  const int U = (n * (n - 1)) / 2;
  const rsrc_t rs = make_rsrc(ae ? ae + g * E0 : nullptr, ae ? (uint32_t)(E0 * 4) : 0u);
#pragma unroll
  for (int m = 0; m < TB; ++m) {
    int r, j;
    tile_elem(t, m, aj, r, j);
    const int i = i0 + r;
    const int id = canon_id(n, U, i, j);
    const bool ok = id >= 0 && mask_bit(rowmask, g * n + i, W, j);
    L.v[m] = bld(rs, ok ? 4 * id : OOB);
    L.valid |= (ok ? 1u : 0u) << m;
  }
}

__device__ __forceinline__ void stage_block(const BlockLoad& L, float* __restrict__ sE, int SE,
                                            int i0, int t, bool has_eid, int NP) {
  const bool aj = tile_along_j(t, i0, has_eid);
  if ((t >> 4) < NP / 16) {
#pragma unroll
    for (int m = 0; m < TB; ++m) {
      int r, j;
      tile_elem(t, m, aj, r, j);
      sE[r * SE + j] = ((L.valid >> m) & 1u) ? L.v[m] : -INFINITY;
    }
  }
}

// d(edge logit) of one target block, staged in sE[r][j] by the rows phase,
// written to the head plane through the same tile mapping (canonical order,
// present edges only; other slots go to an out-of-range offset and drop).
__device__ __forceinline__ void store_block_dae(const float* __restrict__ sE, int SE, int i0,
                                                int t, float* __restrict__ dae,
                                                const uint32_t* __restrict__ rowmask, int64_t g,
                                                int n, int NP) {
  const int W = (n + 31) >> 5;
  const int64_t E0 = (int64_t)n * (n - 1);
  const int U = (n * (n - 1)) / 2;
  const bool aj = tile_along_j(t, i0, false);
  const rsrc_t rs = make_rsrc(dae + g * E0, (uint32_t)(E0 * 4));
  if ((t >> 4) < NP / 16) {
#pragma unroll
    for (int m = 0; m < TB; ++m) {
      int r, j;
      tile_elem(t, m, aj, r, j);
      const int i = i0 + r;
      const int id = canon_id(n, U, i, j);
      const bool ok = id >= 0 && mask_bit(rowmask, g * n + i, W, j);
      bst(rs, ok ? 4 * id : OOB, sE[r * SE + j]);
    }
  }
}

__device__ __forceinline__ int64_t edge_index_of(const int32_t* __restrict__ eid, int64_t g,
                                                 int n, int i, int j) {
  return eid ? (int64_t)eid[(g * n + i) * n + j]
             : g * ((int64_t)n * (n - 1)) + canon_eid(n, i, j);
}

// Softmax of RPW target rows at once (independent rows share every reduction
// round).  Lane owns sources j = lane + 64q.  On return p[rr][q] is the
// probability (0 where invalid), neg[rr][q] the leaky-negative flag,
// present[rr][q] whether edge j->i exists, cnt[rr] the in-degree.
struct Rows {
  float p[RPW][4];
  bool neg[RPW][4];
  bool present[RPW][4];
  float cnt[RPW];
};

__device__ __forceinline__ void rows_softmax(Rows& R, const float* __restrict__ sE, int SE,
                                             const float* __restrict__ sA,
                                             const float* __restrict__ sD, int rb, int i0, int n,
                                             int NP, bool has_ae, float slope, int lane) {
  float e[RPW][4], red[2 * RPW];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    float es = 0.f, c = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = lane + 64 * q;
      const float ev = j < NP ? sE[(rb + rr) * SE + j] : -INFINITY;
      const bool pr = ev != -INFINITY;
      R.present[rr][q] = pr;
      e[rr][q] = pr ? ev : 0.f;
      es += e[rr][q];
      c += pr ? 1.f : 0.f;
    }
    red[rr] = es;
    red[RPW + rr] = c;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
    for (int k = 0; k < 2 * RPW; ++k) red[k] += __shfl_xor(red[k], m, 64);
  float mx[RPW], s[RPW][4];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int i = i0 + rb + rr;
    R.cnt[rr] = red[RPW + rr];
    const float loopv = (has_ae && R.cnt[rr] > 0.f) ? red[rr] / R.cnt[rr] : 0.f;
    const float ad = i < n ? sD[i] : 0.f;
    mx[rr] = -INFINITY;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = lane + 64 * q;
      const bool valid = i < n && (R.present[rr][q] || j == i);
      float v = (j < NP ? sA[j] : 0.f) + ad;
      v += (j == i) ? loopv : e[rr][q];
      R.neg[rr][q] = !(v > 0.f);
      const float lr = R.neg[rr][q] ? v * slope : v;
      s[rr][q] = valid ? lr : -INFINITY;
      mx[rr] = fmaxf(mx[rr], s[rr][q]);
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) mx[rr] = fmaxf(mx[rr], __shfl_xor(mx[rr], m, 64));
  float den[RPW];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    den[rr] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      s[rr][q] = (s[rr][q] == -INFINITY) ? 0.f : expf(s[rr][q] - mx[rr]);
      den[rr] += s[rr][q];
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) den[rr] += __shfl_xor(den[rr], m, 64);
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const float inv = den[rr] + 1e-16f;
#pragma unroll
    for (int q = 0; q < 4; ++q) R.p[rr][q] = s[rr][q] / inv;
  }
}

// ---------------------------------------------------------------------------
// forward
// LDS: sX [NP][XS] | sP [TB][PS] | sA [NP] | sD [NP] | sE [TB][NP] (aliased by
//      the K-split partials sR [4][TB][CW] after the rows phase)
// ---------------------------------------------------------------------------
template <int ACT, bool CONCAT, int CT>
__global__ __launch_bounds__(TT) void k_attn_tiled_fwd(
    const float* __restrict__ xs, int ldx, const float* __restrict__ ae_planes, int64_t E,
    const int32_t* __restrict__ eid, const uint32_t* __restrict__ rowmask,
    const float* __restrict__ bias, const uint8_t* __restrict__ keep, float keep_scale,
    float* __restrict__ out, int n, int H, int C, float slope) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int CW = 16 * CT;
  constexpr int XS = pad32(CW, 16);  // B operand: row = lane>>4
  const int NP = round_up(n, 16);
  const int PS = pad32(NP, 2);       // A operand: row = lane&15
  float* sX = smem;               // [NP][XS]
  float* sP = sX + NP * XS;       // [TB][PS]
  float* sA = sP + TB * PS;       // [NP]
  float* sD = sA + NP;            // [NP]
  const int SE = NP + 1;          // conflict-free column-wise tile writes
  float* sE = sD + NP;            // [TB][SE], max(TB*SE, 4*CW*SRS) floats
  float* sR = sE;                 // [4][CW][SRS], after the rows phase

  int64_t g;
  int h;
  block_gh(H, g, h);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t row0 = g * n;
  const int HC = H * C;
  const float* ae = ae_planes ? ae_planes + (int64_t)h * E : nullptr;

  BlockLoad L;
  load_block(L, 0, t, ae, eid, rowmask, g, n);
  for (int idx = t; idx < NP * CW; idx += TT) {
    const int j = idx / CW, c = idx - j * CW;
    sX[j * XS + c] = (j < n && c < C) ? xs[(row0 + j) * ldx + h * C + c] : 0.f;
  }
  for (int j = t; j < NP; j += TT) {
    sA[j] = j < n ? xs[(row0 + j) * ldx + HC + h] : 0.f;
    sD[j] = j < n ? xs[(row0 + j) * ldx + HC + H + h] : 0.f;
  }

  const int li = lane & 15, lk = lane >> 4;
  const int kq = NP / 4;  // K-split: wave w sums sources [w*kq, (w+1)*kq)
  for (int i0 = 0; i0 < n; i0 += TB) {
    stage_block(L, sE, SE, i0, t, eid != nullptr, NP);
    __syncthreads();
    if (i0 + TB < n) load_block(L, i0 + TB, t, ae, eid, rowmask, g, n);
    // ---- P rows: wave w owns rows [4w, 4w+4) of the block ----
    {
      const int rb = wave * RPW;
      Rows R;
      rows_softmax(R, sE, SE, sA, sD, rb, i0, n, NP, ae != nullptr, slope, lane);
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const int i = i0 + rb + rr;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = lane + 64 * q;
          if (j < NP) {
            float pd = R.p[rr][q];
            if (keep && i < n && j < n)
              pd = keep[((g * H + h) * n + i) * n + j] ? pd * keep_scale : 0.f;
            sP[(rb + rr) * PS + j] = pd;
          }
        }
      }
    }
    __syncthreads();
    // ---- out[i][c] = Σ_j P[i][j] xs_h[j][c], K split over the 4 waves ----
    {
      f4 acc[CT];
#pragma unroll
      for (int b = 0; b < CT; ++b) acc[b] = f4{0.f, 0.f, 0.f, 0.f};
      const float* pa = sP + li * PS + lk;
      for (int k = wave * kq; k < (wave + 1) * kq; k += 4) {
        const float a = pa[k];
#pragma unroll
        for (int b = 0; b < CT; ++b)
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, sX[(k + lk) * XS + 16 * b + li],
                                                        acc[b], 0, 0, 0);
      }
      // partials column-major [wave][c][row]: one 16-B store per tile (the
      // row-major scalar form was miscompiled into ds_write2 with wrong
      // offsets by this toolchain at CT = 4)
#pragma unroll
      for (int b = 0; b < CT; ++b)
        *reinterpret_cast<f4*>(sR + (wave * CW + 16 * b + li) * SRS + 4 * lk) = acc[b];
    }
    __syncthreads();
    for (int idx = t; idx < TB * CW; idx += TT) {
      const int r = idx / CW, c = idx - r * CW;
      const int i = i0 + r;
      if (i < n && c < C) {
        const float* q = sR + c * SRS + r;
        const float v = (q[0] + q[CW * SRS]) + (q[2 * CW * SRS] + q[3 * CW * SRS]);
        if (CONCAT) {
          const float b = bias ? bias[h * C + c] : 0.f;
          out[(row0 + i) * HC + h * C + c] = act_fwd<ACT>(v + b);
        } else {
          out[(row0 + i) * HC + h * C + c] = v;  // workspace, per head
        }
      }
    }
    __syncthreads();
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
// LDS: sX [NP][XS] | sP [TB][PS] (Pd) | sL [TB][PS] (dP then dL) |
//      sO [TB][OS] (dOut) | sA [NP] | sD [NP] | sDa [NP] | sE [TB][NP]
// ---------------------------------------------------------------------------
template <int ACT, bool CONCAT, int CT>
__global__ __launch_bounds__(TT) void k_attn_tiled_bwd(
    const float* __restrict__ dy, const float* __restrict__ y, const float* __restrict__ xs,
    int ldx, const float* __restrict__ ae_planes, int64_t E, const int32_t* __restrict__ eid,
    const uint8_t* __restrict__ keep, float keep_scale, const uint32_t* __restrict__ rowmask,
    float* __restrict__ dxs, float* __restrict__ dae_planes, float* __restrict__ dbias, int n,
    int H, int C, float slope) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int CW = 16 * CT;
  constexpr int XS = CW + 1;         // dP's B operand: row = lane&15
  constexpr int OS = CW + 1;         // read both ways (dP's A, dxs's B)
  const int NP = round_up(n, 16);
  const int PS = pad32(NP, 16);      // Pᵀ operand: row = lane>>4
  float* sX = smem;               // [NP][XS]
  float* sP = sX + NP * XS;       // [TB][PS]
  float* sL = sP + TB * PS;       // [TB][PS]
  float* sO = sL + TB * PS;       // [TB][OS]
  float* sA = sO + TB * OS;       // [NP]
  float* sD = sA + NP;            // [NP]
  float* sDa = sD + NP;           // [NP]
  const int SE = NP + 1;          // conflict-free column-wise tile accesses
  float* sE = sDa + NP;           // [TB][SE]: edge logits, then d(edge logit)

  int64_t g;
  int h;
  block_gh(H, g, h);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t row0 = g * n;
  const int HC = H * C;
  const int OC = CONCAT ? HC : C;
  const int oc0 = CONCAT ? h * C : 0;
  const float oscale = CONCAT ? 1.f : 1.f / (float)H;
  const float* ae = ae_planes ? ae_planes + (int64_t)h * E : nullptr;
  float* dae = dae_planes ? dae_planes + (int64_t)h * E : nullptr;

  // dOut rows of the next block, prefetched in registers with its edge logits
  // (a load issued after this block's dae stores would wait for all of them)
  constexpr int OPT = TB * CW / TT;  // = CT
  float pdy[OPT], py[OPT];
  auto load_dout = [&](int i0n) {
#pragma unroll
    for (int m = 0; m < OPT; ++m) {
      const int idx = t + TT * m, r = idx / CW, c = idx - r * CW, i = i0n + r;
      const bool ok = i < n && c < C;
      const int64_t o = ok ? (row0 + i) * OC + oc0 + c : 0;
      pdy[m] = ok ? dy[o] : 0.f;
      py[m] = ok ? y[o] : 0.f;
    }
  };
  BlockLoad L;
  load_block(L, 0, t, ae, eid, rowmask, g, n);
  load_dout(0);
  for (int idx = t; idx < NP * CW; idx += TT) {
    const int j = idx / CW, c = idx - j * CW;
    sX[j * XS + c] = (j < n && c < C) ? xs[(row0 + j) * ldx + h * C + c] : 0.f;
  }
  for (int j = t; j < NP; j += TT) {
    sA[j] = j < n ? xs[(row0 + j) * ldx + HC + h] : 0.f;
    sD[j] = j < n ? xs[(row0 + j) * ldx + HC + H + h] : 0.f;
    sDa[j] = 0.f;
  }
  // dxs accumulators: wave w owns row tiles jt = w, w+4, ... (NP/16 <= 16) x CT column tiles
  constexpr int MAXJT = TILED_MAX_N / 16 / 4;  // 4 row tiles per wave
  f4 dacc[MAXJT][CT];
#pragma unroll
  for (int a = 0; a < MAXJT; ++a)
#pragma unroll
    for (int b = 0; b < CT; ++b) dacc[a][b] = f4{0.f, 0.f, 0.f, 0.f};
  float dbias_acc = 0.f;  // thread t < C owns bias column t of this head's slice
  const int li = lane & 15, lk = lane >> 4;
  const int njt = NP / 16;

  for (int i0 = 0; i0 < n; i0 += TB) {
    // ---- stage: edge logits of this block (prefetched), dOut rows ----
    stage_block(L, sE, SE, i0, t, eid != nullptr, NP);
#pragma unroll
    for (int m = 0; m < OPT; ++m) {
      const int idx = t + TT * m, r = idx / CW, c = idx - r * CW;
      sO[r * OS + c] = act_bwd<ACT>(pdy[m], py[m]) * oscale;
    }
    __syncthreads();
    if (i0 + TB < n) {
      load_block(L, i0 + TB, t, ae, eid, rowmask, g, n);
      load_dout(i0 + TB);
    }
    if (t < C && (CONCAT || h == 0)) {
      float s = 0.f;
      for (int r = 0; r < TB; ++r) s += sO[r * OS + t];
      dbias_acc += s / oscale;  // = Σ dz
    }
    // ---- dPd[i][j] = Σ_c dOut[i][c] xs_h[j][c]: tiles over j, waves stride ----
    for (int jt = wave; jt < njt; jt += 4) {
      f4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* oa = sO + li * OS + lk;
      const float* xb = sX + (16 * jt + li) * XS + lk;
#pragma unroll
      for (int k = 0; k < CW; k += 4)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(oa[k], xb[k], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) sL[(4 * lk + r) * PS + 16 * jt + li] = acc[r];
    }
    __syncthreads();
    // ---- rows: recompute P, softmax / leaky / dropout backward ----
    {
      const int rb = wave * RPW;
      Rows R;
      rows_softmax(R, sE, SE, sA, sD, rb, i0, n, NP, ae != nullptr, slope, lane);
      float dp[RPW][4], pd[RPW][4], red[3 * RPW];
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const int i = i0 + rb + rr;
        float dot = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = lane + 64 * q;
          const float p = R.p[rr][q];
          float d = (j < NP) ? sL[(rb + rr) * PS + j] : 0.f;
          pd[rr][q] = p;
          if (keep && i < n && j < n && (R.present[rr][q] || j == i)) {
            const bool kp = keep[((g * H + h) * n + i) * n + j] != 0;
            d = kp ? d * keep_scale : 0.f;
            pd[rr][q] = kp ? p * keep_scale : 0.f;
          }
          dp[rr][q] = p != 0.f ? d : 0.f;
          dot += p * dp[rr][q];
        }
        red[rr] = dot;
      }
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
        for (int k = 0; k < RPW; ++k) red[k] += __shfl_xor(red[k], m, 64);
      float dl[RPW][4];
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const int i = i0 + rb + rr;
        float rsum = 0.f, dloop = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = lane + 64 * q;
          const float ds = R.p[rr][q] * (dp[rr][q] - red[rr]);
          dl[rr][q] = R.neg[rr][q] ? ds * slope : ds;
          rsum += dl[rr][q];
          if (j == i) dloop = dl[rr][q];
        }
        red[RPW + rr] = rsum;
        red[2 * RPW + rr] = dloop;
      }
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
        for (int k = RPW; k < 3 * RPW; ++k) red[k] += __shfl_xor(red[k], m, 64);
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const int r = rb + rr, i = i0 + r;
        if (i < n && lane == 0) dxs[(row0 + i) * ldx + HC + H + h] = red[RPW + rr];  // d a_dst
        const float dshare =
            (ae && R.cnt[rr] > 0.f) ? red[2 * RPW + rr] / R.cnt[rr] : 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = lane + 64 * q;
          if (j < NP) {
            sP[r * PS + j] = pd[rr][q];
            sL[r * PS + j] = dl[rr][q];
          }
          if (eid) {
            if (dae && R.present[rr][q]) dae[edge_index_of(eid, g, n, i, j)] = dl[rr][q] + dshare;
          } else if (j < NP) {
            sE[r * SE + j] = dl[rr][q] + dshare;  // this wave's own rows of sE
          }
        }
      }
    }
    __syncthreads();
    if (dae && !eid) store_block_dae(sE, SE, i0, t, dae, rowmask, g, n, NP);
    // ---- column sums of dL (d a_src) and dxs_h += Pdᵀ · dOut ----
    for (int j = t; j < NP; j += TT) {
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < TB; ++r) s += sL[r * PS + j];
      sDa[j] += s;
    }
#pragma unroll
    for (int a = 0; a < MAXJT; ++a) {
      const int jt = wave + 4 * a;
      if (jt < njt) {
        const float* pa = sP + lk * PS + 16 * jt + li;  // Pᵀ[j][i] = P[i][j]
#pragma unroll
        for (int b = 0; b < CT; ++b) {
          const float* ob = sO + lk * OS + 16 * b + li;
#pragma unroll
          for (int k = 0; k < TB; k += 4)
            dacc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[k * PS], ob[k * OS], dacc[a][b],
                                                              0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // ---- write dxs_h, d a_src, padding columns, bias partial ----
#pragma unroll
  for (int a = 0; a < MAXJT; ++a) {
    const int jt = wave + 4 * a;
    if (jt < njt) {
#pragma unroll
      for (int b = 0; b < CT; ++b) {
        const int c = 16 * b + li;
        if (c < C) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int j = 16 * jt + 4 * lk + r;
            if (j < n) dxs[(row0 + j) * ldx + h * C + c] = dacc[a][b][r];
          }
        }
      }
    }
  }
  for (int j = t; j < n; j += TT) dxs[(row0 + j) * ldx + HC + h] = sDa[j];
  if (h == 0) {
    const int padc = ldx - HC - 2 * H;
    for (int idx = t; idx < n * padc; idx += TT) {
      const int j = idx / padc;
      dxs[(row0 + j) * ldx + HC + 2 * H + (idx - j * padc)] = 0.f;
    }
  }
  if (t < C && (CONCAT || h == 0)) dbias[g * OC + oc0 + t] = dbias_acc;
}

}  // namespace sv2n

// ============================ C-ABI ========================================
using namespace sv2n;

static int ct_of(int C) { return (C + 15) / 16; }

static size_t tiled_fwd_lds(int n, int C) {
  const int CW = 16 * ct_of(C), NP = round_up(n, 16);
  return sizeof(float) * ((size_t)NP * pad32(CW, 16) + (size_t)TB * pad32(NP, 2) + 2 * NP +
                          std::max((size_t)TB * (NP + 1), (size_t)4 * CW * SRS));
}
static size_t tiled_bwd_lds(int n, int C) {
  const int CW = 16 * ct_of(C), NP = round_up(n, 16);
  return sizeof(float) * ((size_t)NP * (CW + 1) + 2 * (size_t)TB * pad32(NP, 16) +
                          (size_t)TB * (CW + 1) + 3 * (size_t)NP + (size_t)TB * (NP + 1));
}

template <typename K>
static void raise_lds_tiled(K kernel, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
}

static int check_tiled(int64_t B, int n, int H, int C, int ldx, int act) {
  if (B <= 0 || C <= 0 || n <= 0) return SV2N_ERR_ARG;
  if (n > TILED_MAX_N || H < 1 || H > SV2N_MAX_HEADS || C > TILED_MAX_C || act < 0 || act > 3)
    return SV2N_ERR_SHAPE;
  if (ldx < H * C + 2 * H) return SV2N_ERR_SHAPE;
  if (B * H > 0x7fffffff) return SV2N_ERR_SHAPE;
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
  if (ae && !eid && num_edges != num_graphs * (int64_t)n * (n - 1)) return SV2N_ERR_SHAPE;
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
  if (ae && !eid && num_edges != num_graphs * (int64_t)n * (n - 1)) return SV2N_ERR_SHAPE;
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
