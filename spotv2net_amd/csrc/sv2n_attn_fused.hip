// Edge-fused GAT attention for dense-block graphs of 32 < n <= 256 nodes with
// narrow edge features (the SURVEY.md §8d C5 stress shapes: D = 12, 8 heads
// of 16 channels) — PyG 2.3.0 GATConv semantics (reference utils/models.py:146
// -> GATConv.forward), like sv2n_attn_tiled.hip,
// but the edge logits are never materialised:
//
//   logit(i <- j, h) = edge_attr[e(i,j)] · W̃[:, h] + a_src[j,h] + a_dst[i,h]
//
// is computed where it is consumed, from the D-float edge row, in every pass
// that needs it.  With D·4 bytes per edge below the 4·H bytes one layer's
// logit plane costs to write and to read back (and the same again for d-logit
// planes in the backward), re-reading edge_attr once per layer and direction
// moves fewer HBM bytes than any materialised form: per layer 2·4D bytes per
// edge against 16·H (C5: 96 vs 128, and no separate edge pass).
//
// Forward, one 8-wave workgroup per (graph, 32-target tile), XCD-aware block
// order (the tiles of a graph share an XCD, so the xs rows they all read hit L2):
//   * sources in blocks of 32: the block's edge rows and xs rows are loaded one
//     block ahead into registers (edge slots mapped so each wave reads
//     contiguous runs of the canonical order: along the targets below the
//     diagonal, along the sources above it);
//   * logits of all 8 head columns into LDS (packed FMAs); then wave h runs
//     head h's online softmax IN the MFMA A-operand layout (running max / sum
//     per row, row reductions over the 4 lanes of a row with permlane swaps),
//     keeping the sum of the raw edge logits for the mean-filled self loop;
//   * aggregation out_h = P_h · xs_h on v_mfma_f32_16x16x4_f32 (exact f32)
//     with P straight from registers, accumulators rescaled per row as the
//     max moves;
//   * self loop last (its logit needs the row's mean edge logit), then
//     normalisation, bias and activation; training saves the pre-bias head
//     aggregates and per-row softmax statistics (max, 1/sum, self logit, count).
//
// Backward, three launches per layer:
//   bprep  per node: dOut = act'(y)·dy (÷H for mean), r = dOut·agg
//          (= Σ_j p·dP, the softmax row term), the self loop's whole gradient,
//          and per-chunk bias partials;
//   bwd    one 8-wave workgroup per (graph, 32-source tile) walking all
//          targets in blocks of 16, wave h doing all of head h's work on a
//          block (k_fattn_bwd2): logits recomputed from the block's edge rows
//          (staged once in LDS, double-buffered: one barrier per block) in the
//          forward's summation order, dP = dOut·xsᵀ and dxs += Pᵀ·dOut on
//          MFMA, the softmax backward in the MFMA output layout, d a_src
//          complete in the workgroup, d a_dst partial per source tile, dW̃[:, h]
//          in registers; 128 VGPRs so two workgroups share a CU (round 3: the
//          three-phase form with logit / d-logit planes exchanged between
//          waves ran one workgroup per CU, 2.20 -> 1.63 ms per C5 layer);
//   finish d a_dst = Σ partials + self term, dW̃ = fixed-order sum of partials.
// No atomics; every sum has a fixed order (deterministic).
#include "sv2n_common.h"
#include <type_traits>

// tools/fattn_ablate.py builds forward variants with parts removed (timing
// only): 1 no edge_attr loads, 2 no softmax / MFMA phase, 3 no logit arithmetic
#ifndef SV2N_FATTN_ABLATE
#define SV2N_FATTN_ABLATE 0
#endif

namespace sv2n {
namespace fused {

constexpr int WT = 512;   // threads per workgroup of the attention kernels (8 waves)
constexpr int PT = 256;   // threads per workgroup of the per-node / reduction kernels
constexpr int MH = 8;     // max heads (one per wave in the MFMA phases)
constexpr int FT = 32;    // forward: targets per tile
constexpr int FS = 32;    // forward: sources per block
constexpr int BS = 32;    // backward: sources per tile
constexpr int BT = 16;    // backward: targets per block
constexpr int RS = 36;    // LDS stride (floats) of a 32-wide row (16-B aligned, b128 conflict-free)
constexpr int XW = 132;   // LDS stride of a [8 heads x 16] row
constexpr int XCHUNKS = 3;  // forward xs prefetch: ceil(32 rows x 34 chunks / 512)

typedef float f4 __attribute__((ext_vector_type(4)));

// 24-bit multiplies (full rate; the 32-bit v_mul_lo_u32 is quarter rate): u, n < 2^12
__device__ __forceinline__ int tri_off(int n, int u) { return __mul24(u, 2 * n - u - 1) >> 1; }

// canonical in-graph edge id of (target i <- source j) (reference
// utils/dataset.py:216-226: upper pairs u->w row-major, then swapped), -1 if
// (i, j) is not an edge
__device__ __forceinline__ int canon_id(int i, int j, int n) {
  const int U = __mul24(n, n - 1) >> 1;
  const int id = j > i ? U + tri_off(n, i) + (j - i - 1) : tri_off(n, j) + (i - j - 1);
  return (i < n && j < n && i != j) ? id : -1;
}

// blockIdx -> (graph, tile) with the tiles of a graph on one XCD
__device__ __forceinline__ void block_gt(int NT, int64_t& g, int& tile) {
  const int64_t nb = (int64_t)gridDim.x;
  int64_t b = blockIdx.x;
  if ((nb & 7) == 0) b = (b & 7) * (nb >> 3) + (b >> 3);
  g = b / NT;
  tile = (int)(b - g * NT);
}

// One edge row of D floats.  Canonical layouts: buffer loads at 32-bit
// offsets within the graph's edge rows (a miss reads 0).  Edge-id maps
// (block layouts): global edge ids, 64-bit addresses.
template <int D>
__device__ __forceinline__ void load_edge(float (&v)[D], rsrc_t rea, int cid,
                                          const float* __restrict__ ea, int64_t gid, bool eidm) {
  if (eidm) {
    const bool ok = gid >= 0;
    const float* p = ea + (ok ? gid : 0) * D;
    if constexpr (D % 4 == 0) {
#pragma unroll
      for (int q = 0; q < D / 4; ++q) {
        const f4 w = ok ? *reinterpret_cast<const f4*>(p + 4 * q) : f4{0.f, 0.f, 0.f, 0.f};
        v[4 * q] = w.x; v[4 * q + 1] = w.y; v[4 * q + 2] = w.z; v[4 * q + 3] = w.w;
      }
    } else {
#pragma unroll
      for (int d = 0; d < D; ++d) v[d] = ok ? p[d] : 0.f;
    }
  } else {
    if constexpr (D % 4 == 0) {
#pragma unroll
      for (int q = 0; q < D / 4; ++q) {
        const f32x4 w = bld4(rea, cid >= 0 ? 4 * (cid * D + 4 * q) : OOB);
        v[4 * q] = w.x; v[4 * q + 1] = w.y; v[4 * q + 2] = w.z; v[4 * q + 3] = w.w;
      }
    } else {
#pragma unroll
      for (int d = 0; d < D; ++d) v[d] = bld(rea, cid >= 0 ? 4 * (cid * D + d) : OOB);
    }
  }
}

__device__ __forceinline__ float act_fwd_rt(int act, float z) {
  switch (act) {
    case ACT_RELU: return act_fwd<ACT_RELU>(z);
    case ACT_TANH: return act_fwd<ACT_TANH>(z);
    case ACT_SIGMOID: return act_fwd<ACT_SIGMOID>(z);
    default: return z;
  }
}
__device__ __forceinline__ float act_bwd_rt(int act, float dy, float y) {
  switch (act) {
    case ACT_RELU: return act_bwd<ACT_RELU>(dy, y);
    case ACT_TANH: return act_bwd<ACT_TANH>(dy, y);
    case ACT_SIGMOID: return act_bwd<ACT_SIGMOID>(dy, y);
    default: return dy;
  }
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// 16-lane row sum (every lane of the row ends with the same value)
__device__ __forceinline__ float row16_sum(float v) {
  v += dppf<0x128>(v);
  v += dppf<0x124>(v);
  v += dppf<0x4E>(v);
  v += dppf<0xB1>(v);
  return v;
}

// Half of an edge row: lane parity `half` holds floats [half*DH, half*DH + DH)
// (DH = ceil(D/2); past D reads 0).  The backward splits every edge row over a
// lane pair so that its dW̃ accumulators are D/2 x 8 per thread, not D x 8.
template <int D>
__device__ __forceinline__ void load_edge_half(float (&v)[(D + 1) / 2], rsrc_t rea, int cid,
                                               const float* __restrict__ ea, int64_t gid,
                                               bool eidm, int half) {
  constexpr int DH = (D + 1) / 2;
  const int d0 = half * DH;
  if (eidm) {
    const bool ok = gid >= 0;
    const float* p = ea + (ok ? gid : 0) * D + d0;
#pragma unroll
    for (int dd = 0; dd < DH; ++dd) v[dd] = (ok && d0 + dd < D) ? p[dd] : 0.f;
  } else if constexpr (DH % 2 == 0 && D % 2 == 0) {
#pragma unroll
    for (int q = 0; q < DH / 2; ++q) {
      const auto w = __builtin_amdgcn_raw_buffer_load_b64(
          rea, cid >= 0 ? 4 * (cid * D + d0 + 2 * q) : OOB, 0, 0);
      v[2 * q] = __uint_as_float(w[0]);
      v[2 * q + 1] = __uint_as_float(w[1]);
    }
  } else {
#pragma unroll
    for (int dd = 0; dd < DH; ++dd)
      v[dd] = (d0 + dd < D) ? bld(rea, cid >= 0 ? 4 * (cid * D + d0 + dd) : OOB) : 0.f;
  }
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
// Softmax arithmetic in base 2: scaled logits s = leaky(logit)·log2(e), p =
// exp2(s - m) on v_exp_f32; the saved row max m is in the same units.
constexpr float L2E = 1.4426950408889634f;
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

typedef float f2 __attribute__((ext_vector_type(2)));

// logits of K edge rows for all 8 head columns on packed FMAs: the row's
// floats in natural register pairs (d, d+1) times W̃ᵀ pairs from LDS (sWT
// [8][DP], broadcast b128 reads), the two halves summed at the end — no
// broadcast copies of the loaded values (which would make the compiler wait on
// the prefetch right after issuing it)
template <int D>
constexpr int dpad() { return (D + 3) / 4 * 4; }
template <int D, int K>
__device__ __forceinline__ void edge_logits_pk(float (&lg)[K][MH], const float (&ev)[K][D],
                                               const float* __restrict__ sWT) {
  constexpr int DP = dpad<D>();
#pragma unroll
  for (int h = 0; h < MH; ++h) {
    f2 a2[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a2[k] = f2{0.f, 0.f};
#pragma unroll
    for (int q = 0; q < DP / 4; ++q) {
      const f4 w4 = *reinterpret_cast<const f4*>(sWT + h * DP + 4 * q);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int d = 4 * q;
        const f2 e01 = f2{ev[k][d], d + 1 < D ? ev[k][d + 1] : 0.f};
        a2[k] = __builtin_elementwise_fma(e01, f2{w4.x, w4.y}, a2[k]);
        if (d + 2 < D) {
          const f2 e23 = f2{ev[k][d + 2], d + 3 < D ? ev[k][d + 3] : 0.f};
          a2[k] = __builtin_elementwise_fma(e23, f2{w4.z, w4.w}, a2[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) lg[k][h] = a2[k].x + a2[k].y;
  }
}

// max / sum over the 4 lanes li, li+16, li+32, li+48 of a wave (the rows of an
// MFMA A operand): gfx950 permlane swaps, no LDS round trip
__device__ __forceinline__ float lk_max(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float lk_sum(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

constexpr int FHS = FT * RS + 32;  // forward: LDS stride of a head's [32][RS] logit block

template <int D, bool EIDM, bool KEEP>
__global__ __launch_bounds__(WT, (EIDM || KEEP) ? 2 : 4) void k_fattn_fwd(
    const float* __restrict__ xs, int ldx, const float* __restrict__ ea,
    const float* __restrict__ wf, int hl_pad, int col0, const int32_t* __restrict__ eid,
    const float* __restrict__ bias, const uint8_t* __restrict__ keep, float keep_scale,
    float* __restrict__ y, float* __restrict__ agg, float* __restrict__ stats, int n, int H,
    int C, int act, int concat, float slope) {
  __shared__ __attribute__((aligned(16))) float sE[MH * FHS];       // edge logits of the block
  __shared__ __attribute__((aligned(16))) float sXT[MH * 16 * RS];  // xs_hᵀ of the block
  __shared__ __attribute__((aligned(16))) float sA[MH * FS];        // a_src of the block
  __shared__ __attribute__((aligned(16))) float sAl[MH * FT], sPs[MH * FT], sInv[MH * FT];
  __shared__ uint32_t sPres[2][FT];  // edge-id maps: present sources per target (by block parity)
  __shared__ __attribute__((aligned(16))) float sWT[MH * dpad<D>()];  // W̃ᵀ, zero padded

  const int NT = (n + FT - 1) / FT;
  int64_t g;
  int tile;
  block_gt(NT, g, tile);
  const int t = threadIdx.x, lane = t & 63, hh = t >> 6;  // wave hh: head hh in [B]
  const int li = lane & 15, lk = lane >> 4;
  const int i0 = tile * FT;
  const int HC = H * C;
  const int64_t row0 = g * n;
  const int E0 = n * (n - 1);
  constexpr bool eidm = EIDM;
  const rsrc_t rea = eidm ? make_rsrc(nullptr, 0u)
                          : make_rsrc(ea + g * (int64_t)E0 * D, (uint32_t)(4 * E0 * D));
  const rsrc_t rxs = make_rsrc(xs + row0 * ldx, (uint32_t)(4 * n * ldx));
  const int CQ = (HC + H + 3) >> 2;  // 16-B chunks of [xs | a_src] per row
  const float slope2 = slope * L2E;
  const bool hv = hh < H;
  const int64_t Nrows = (int64_t)gridDim.x / NT * n;  // bound checks (SV2N_CHK) only

  if (t < MH * dpad<D>()) {
    const int h = t / dpad<D>(), d = t - h * dpad<D>();
    if (h < H && d < D) SV2N_CHK(201, d * hl_pad + col0 + h, D * hl_pad);
    sWT[t] = (h < H && d < D) ? wf[d * hl_pad + col0 + h] : 0.f;
  }
  if (eidm && t < 2 * FT) sPres[t >> 5][t & 31] = 0u;
  // padding rows of xs_hᵀ (c >= C or h >= H) stay zero
  for (int idx = t; idx < MH * 16 * RS; idx += WT) {
    const int r = idx / RS;
    if ((r & 15) >= C || (r >> 4) >= H) sXT[idx] = 0.f;
  }
  // where this thread's xs chunks go in LDS (fixed over the blocks): -1 none;
  // < 2^20: 4 rows of sXT from there (stride RS); else a_src elements from
  // (xd & 0xffff), count (xd >> 20)
  int xdst[XCHUNKS];
#pragma unroll
  for (int q = 0; q < XCHUNKS; ++q) {
    const int u = t + WT * q, jl = u & 31, cq = u >> 5, cg = 4 * cq;
    xdst[q] = -1;
    if (cq < CQ) {
      if (cg < HC) {
        const int h = cg / C, c = cg - h * C;
        xdst[q] = (h * 16 + c) * RS + jl;
      } else {
        xdst[q] = (min(4, HC + H - cg) << 20) | ((cg - HC) * FS + jl);
      }
    }
  }

  // per row tile rt: state of row i = i0 + 16rt + li for head hh (replicated over lk)
  float ad[2], mrow[2], lrow[2], esum[2], cnt[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int i = i0 + 16 * rt + li;
    if (hv && i < n) SV2N_CHK(202, (row0 + i) * ldx + HC + H + hh, Nrows * ldx);
    ad[rt] = (hv && i < n) ? xs[(row0 + i) * ldx + HC + H + hh] : 0.f;
    mrow[rt] = -INFINITY;
    lrow[rt] = 0.f;  // this lane's share of the row sum
    esum[rt] = 0.f;
    cnt[rt] = 0.f;
  }
  __syncthreads();

  // edge rows and xs rows of the next block, loaded while this one is computed
  float ev[2][D];
  f32x4 xv[XCHUNKS];
  auto slot = [&](int k, int j0, int& il, int& jl) {
    const int s = k * WT + t;
    const bool along_i = !eidm && (j0 + FS <= i0);
    il = along_i ? (s & 31) : (s >> 5);
    jl = along_i ? (s >> 5) : (s & 31);
  };
  auto issue = [&](int j0) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      int il, jl;
      slot(k, j0, il, jl);
      const int i = i0 + il, j = j0 + jl;
      int cid = -1;
      int64_t gid = -1;
      if constexpr (eidm) {
        if (i < n && j < n && i != j) SV2N_CHK(203, (row0 + i) * n + j, Nrows * n);
        gid = (i < n && j < n && i != j) ? eid[(row0 + i) * n + j] : -1;
      } else {
        cid = canon_id(i, j, n);
      }
      if (SV2N_FATTN_ABLATE == 1) {
#pragma unroll
        for (int d = 0; d < D; ++d) ev[k][d] = (float)(cid & 7) * 0.01f;
      } else {
        load_edge<D>(ev[k], rea, cid, ea, gid, eidm);
      }
    }
#pragma unroll
    for (int q = 0; q < XCHUNKS; ++q) {
      const int u = t + WT * q, jl = u & 31, cq = u >> 5, j = j0 + jl;
      xv[q] = bld4(rxs, (cq < CQ && j < n) ? 4 * (j * ldx + 4 * cq) : OOB);
    }
  };

  f4 acc[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) acc[rt] = f4{0.f, 0.f, 0.f, 0.f};

  issue(0);
  int par = 0;
  for (int j0 = 0; j0 < n; j0 += FS, par ^= 1) {
    // ---- [A] logits of the block (all 8 head columns), xs rows into LDS ----
    {
      float lg[2][MH];
      if (SV2N_FATTN_ABLATE == 3) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int h = 0; h < MH; ++h) lg[k][h] = ev[k][h % D];
      } else {
        edge_logits_pk<D, 2>(lg, ev, sWT);
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        int il, jl;
        slot(k, j0, il, jl);
        float* dst = sE + il * RS + jl;
#pragma unroll
        for (int h = 0; h < MH; ++h) dst[h * FHS] = lg[k][h];
        if constexpr (eidm) {
          const int i = i0 + il, j = j0 + jl;
          if (i < n && j < n && i != j) SV2N_CHK(204, (row0 + i) * n + j, Nrows * n);
          const bool pres = i < n && j < n && i != j && eid[(row0 + i) * n + j] >= 0;
          if (pres) atomicOr(&sPres[par][il], 1u << jl);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < XCHUNKS; ++q) {
      const int xd = xdst[q];
      if (xd >= 0 && xd < (1 << 20)) {
        float* dst = sXT + xd;
        dst[0] = xv[q].x;
        dst[RS] = xv[q].y;
        dst[2 * RS] = xv[q].z;
        dst[3 * RS] = xv[q].w;
      } else if (xd >= 0) {
        float* dst = sA + (xd & 0xffff);
        const int cntq = xd >> 20;
        const float vv[4] = {xv[q].x, xv[q].y, xv[q].z, xv[q].w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (e < cntq) dst[e * FS] = vv[e];
      }
    }
    if (j0 + FS < n) issue(j0 + FS);
    __syncthreads();

    // ---- [B] wave hh: softmax of head hh in registers, MFMA aggregation ----
    if (hv && SV2N_FATTN_ABLATE != 2) {
      const bool clean = !eidm && j0 != i0 && j0 + FS <= n;
      const f4 as0 = *reinterpret_cast<const f4*>(sA + hh * FS + 4 * lk);
      const f4 as1 = *reinterpret_cast<const f4*>(sA + hh * FS + 16 + 4 * lk);
      const float asv[8] = {as0.x, as0.y, as0.z, as0.w, as1.x, as1.y, as1.z, as1.w};
      const f4 xb0 = *reinterpret_cast<const f4*>(sXT + (hh * 16 + li) * RS + 4 * lk);
      const f4 xb1 = *reinterpret_cast<const f4*>(sXT + (hh * 16 + li) * RS + 16 + 4 * lk);
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int il = 16 * rt + li, i = i0 + il;
        const float* er = sE + hh * FHS + il * RS;
        const f4 e0 = *reinterpret_cast<const f4*>(er + 4 * lk);
        const f4 e1 = *reinterpret_cast<const f4*>(er + 16 + 4 * lk);
        const float evv[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
        uint32_t vm = 0xffu;  // bit k: element k (source 4lk + (k&3) + 16(k>>2)) is an edge
        if (!clean) {
          uint32_t row = i < n ? 0xffffffffu : 0u;
          const int lim = n - j0;
          if (lim < 32) row &= (1u << lim) - 1u;
          if (i >= j0 && i < j0 + FS) row &= ~(1u << (i - j0));
          if constexpr (eidm) row &= sPres[par][il];
          vm = ((row >> (4 * lk)) & 0xfu) | (((row >> (16 + 4 * lk)) & 0xfu) << 4);
        }
        float sv[8], bm = -INFINITY, es = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const bool valid = (vm >> k) & 1u;
          es += valid ? evv[k] : 0.f;
          const float v = asv[k] + ad[rt] + evv[k];
          const float s2 = v * (v > 0.f ? L2E : slope2);
          sv[k] = valid ? s2 : -INFINITY;
          bm = fmaxf(bm, sv[k]);
        }
        esum[rt] += es;
        if constexpr (eidm) cnt[rt] += (float)__popc(vm);  // canonical: n - 1
        bm = lk_max(bm);
        const float mo = mrow[rt];
        const float mn = fmaxf(mo, bm);
        const float al = mn == -INFINITY ? 1.f : fexp2(mo - mn);
        const float mref = mn == -INFINITY ? 0.f : mn;
        float pk[8], ls = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float p = fexp2(sv[k] - mref);  // exp2(-inf) = 0
          ls += p;
          pk[k] = p;
          if constexpr (KEEP) {
            const int j = j0 + 4 * lk + (k & 3) + 16 * (k >> 2);
            if (i < n && j < n) SV2N_CHK(205, ((g * H + hh) * (int64_t)n + i) * n + j, Nrows * H * n);
            pk[k] = (i < n && j < n && keep[((g * H + hh) * (int64_t)n + i) * n + j]) ?
                        p * keep_scale : 0.f;
          }
        }
        lrow[rt] = lrow[rt] * al + ls;
        mrow[rt] = mn;
        // rescale factor of the accumulator rows 4lk + r (wave-local LDS exchange)
        if (lk == 0) sAl[hh * FT + il] = al;
        const f4 al4 = *reinterpret_cast<const f4*>(sAl + hh * FT + 16 * rt + 4 * lk);
        acc[rt].x *= al4.x;
        acc[rt].y *= al4.y;
        acc[rt].z *= al4.z;
        acc[rt].w *= al4.w;
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pk[0], xb0.x, acc[rt], 0, 0, 0);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pk[1], xb0.y, acc[rt], 0, 0, 0);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pk[2], xb0.z, acc[rt], 0, 0, 0);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pk[3], xb0.w, acc[rt], 0, 0, 0);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pk[4], xb1.x, acc[rt], 0, 0, 0);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pk[5], xb1.y, acc[rt], 0, 0, 0);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pk[6], xb1.z, acc[rt], 0, 0, 0);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pk[7], xb1.w, acc[rt], 0, 0, 0);
      }
    }
    if constexpr (eidm) {
      if (t < FT) sPres[par ^ 1][t] = 0u;  // the next block's buffer (last read two blocks ago)
    }
    __syncthreads();
  }

  // ---- self loop (logit = a_src + a_dst + mean edge logit), statistics ----
  if (hv) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int il = 16 * rt + li, i = i0 + il;
      const float l = lk_sum(lrow[rt]);
      const float es = lk_sum(esum[rt]);
      const float cn = eidm ? lk_sum(cnt[rt]) : (float)(n - 1);
      if (i < n) SV2N_CHK(206, (row0 + i) * ldx + HC + hh, Nrows * ldx);
      const float as_self = i < n ? xs[(row0 + i) * ldx + HC + hh] : 0.f;
      const float loopv = cn > 0.f ? es / cn : 0.f;
      const float vs = as_self + ad[rt] + loopv;
      const float lr = vs * (vs > 0.f ? L2E : slope2);
      const float mo = mrow[rt];
      const float mn = fmaxf(mo, lr);
      const float al = fexp2(mo - mn);
      const float ps = fexp2(lr - mn);
      const float lt = l * al + ps;
      const float inv = 1.f / (lt + 1e-16f);
      float pks = ps;
      if constexpr (KEEP)
        if (i < n) SV2N_CHK(207, ((g * H + hh) * (int64_t)n + i) * n + i, Nrows * H * n);
      if constexpr (KEEP) pks = (i < n && keep[((g * H + hh) * (int64_t)n + i) * n + i]) ?
                                    ps * keep_scale : 0.f;
      if (lk == 0) {
        sAl[hh * FT + il] = al;
        sPs[hh * FT + il] = pks;
        sInv[hh * FT + il] = inv;
        if (stats && i < n) {
          float* st = stats + (row0 + i) * 4 * H;
          st[hh] = mn;
          st[H + hh] = inv;
          st[2 * H + hh] = vs;
          st[3 * H + hh] = cn;
        }
      }
    }
  }
  __syncthreads();

  float* sOut = sE;  // [FT][HC] head aggregates (mean over heads)
  if (hv) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const float av[4] = {acc[rt].x, acc[rt].y, acc[rt].z, acc[rt].w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int il = 16 * rt + 4 * lk + r, i = i0 + il, c = li;
        if (i < n && c < C) {
          const int q = hh * FT + il;
          const int64_t row = row0 + i;
          SV2N_CHK(208, row * ldx + hh * C + c, Nrows * ldx);
          SV2N_CHK(209, row * HC + hh * C + c, Nrows * HC);
          const float xv1 = xs[row * ldx + hh * C + c];
          const float out = fmaf(av[r], sAl[q], sPs[q] * xv1) * sInv[q];
          if (agg) agg[row * HC + hh * C + c] = out;
          if (concat) {
            const float b = bias ? bias[hh * C + c] : 0.f;
            y[row * HC + hh * C + c] = act_fwd_rt(act, out + b);
          } else {
            sOut[il * HC + hh * C + c] = out;
          }
        }
      }
    }
  }
  if (!concat) {
    __syncthreads();
    const float invH = 1.f / (float)H;
    for (int idx = t; idx < FT * C; idx += WT) {
      const int il = idx / C, c = idx - il * C, i = i0 + il;
      if (i < n) {
        float s = 0.f;
        for (int h = 0; h < H; ++h) s += sOut[il * HC + h * C + c];
        SV2N_CHK(210, (row0 + i) * C + c, Nrows * C);
        y[(row0 + i) * C + c] = act_fwd_rt(act, s * invH + (bias ? bias[c] : 0.f));
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward: per-node preparation
//   dout [N][HC]  dOut_h (concat slice, or dz / H for every head)
//   rs   [N][4H]  r | d logit of the self loop | its kept prob. | that ÷ count
//   dbp  [B*NT][OC] bias partials (Σ dz over the chunk's rows)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(PT) void k_fattn_bprep(
    const float* __restrict__ dy, const float* __restrict__ y, const float* __restrict__ agg,
    const float* __restrict__ stats, const float* __restrict__ xs, int ldx,
    const uint8_t* __restrict__ keep, float keep_scale, float* __restrict__ dout,
    float* __restrict__ rs, float* __restrict__ dbp, int n, int H, int C, int act, int concat,
    float slope) {
  __shared__ float sRt[FT * 128], sDp[FT * 128];
  __shared__ float sDb[2 * 128];
  const int NT = (n + FT - 1) / FT;
  const int64_t g = blockIdx.x / NT;
  const int chunk = (int)(blockIdx.x - g * NT);
  const int i0 = chunk * FT;
  const int t = threadIdx.x;
  const int HC = H * C, OC = concat ? HC : C;
  const int64_t row0 = g * n;
  const int hc = t & 127, rh = t >> 7;
  const int h = hc / C, c = hc - (hc / C) * C;
  const int oc = concat ? hc : c;
  const bool colv = hc < HC;
  const float oscale = concat ? 1.f : 1.f / (float)H;

  float vdy[FT / 2], vy[FT / 2], vag[FT / 2], vx[FT / 2];
#pragma unroll
  for (int q = 0; q < FT / 2; ++q) {
    const int i = i0 + rh + 2 * q;
    const bool ok = colv && i < n;
    const int64_t row = row0 + (ok ? i : 0);
    if (ok) SV2N_CHK(211, row * ldx + hc, (int64_t)gridDim.x / NT * n * ldx);
    if (ok) SV2N_CHK(212, row * HC + hc, (int64_t)gridDim.x / NT * n * HC);
    vdy[q] = ok ? dy[row * OC + oc] : 0.f;
    vy[q] = ok ? y[row * OC + oc] : 0.f;
    vag[q] = ok ? agg[row * HC + hc] : 0.f;
    vx[q] = ok ? xs[row * ldx + hc] : 0.f;
  }
  float db = 0.f;
#pragma unroll
  for (int q = 0; q < FT / 2; ++q) {
    const int il = rh + 2 * q, i = i0 + il;
    const bool ok = colv && i < n;
    const float dz = act_bwd_rt(act, vdy[q], vy[q]);
    const float d = dz * oscale;
    if (ok) SV2N_CHK(213, (row0 + i) * HC + hc, (int64_t)gridDim.x / NT * n * HC);
    if (ok) dout[(row0 + i) * HC + hc] = d;
    sRt[il * 128 + hc] = ok ? d * vag[q] : 0.f;
    sDp[il * 128 + hc] = ok ? d * vx[q] : 0.f;
    if (ok && (concat || h == 0)) db += dz;
  }
  sDb[rh * 128 + hc] = db;
  __syncthreads();
  {
    const int il = t >> 3, hh = t & 7, i = i0 + il;
    if (hh < H && i < n) {
      float r = 0.f, dp = 0.f;
      for (int cc = 0; cc < C; ++cc) {
        r += sRt[il * 128 + hh * C + cc];
        dp += sDp[il * 128 + hh * C + cc];
      }
      const int64_t row = row0 + i;
      const float* st = stats + row * 4 * H;
      const float mx = st[hh], inv = st[H + hh], vs = st[2 * H + hh], cnt = st[3 * H + hh];
      const float lr = vs * (vs > 0.f ? L2E : slope * L2E);  // base-2 units, as the forward
      const float ps = fexp2(lr - mx) * inv;
      float pd = ps, dP = dp;
      if (keep) {
        const bool kp = keep[((g * H + hh) * (int64_t)n + i) * n + i] != 0;
        pd = kp ? ps * keep_scale : 0.f;
        dP = kp ? dp * keep_scale : 0.f;
      }
      const float ds = ps * (dP - r);
      const float dl = vs > 0.f ? ds : ds * slope;
      float* o = rs + row * 4 * H;
      o[hh] = r;
      o[H + hh] = dl;
      o[2 * H + hh] = pd;
      o[3 * H + hh] = cnt > 0.f ? dl / cnt : 0.f;
    }
  }
  if (t < OC) dbp[(g * NT + chunk) * OC + t] = sDb[t] + sDb[128 + t];
}

// ---------------------------------------------------------------------------
// backward, head-per-wave form: one 8-wave workgroup per (graph, 32-source
// tile), walking the targets in blocks of 16 like k_fattn_bwd, but wave h
// does ALL of head h's work on a block: its logits from the block's edge rows
// (staged once in LDS for every head, double-buffered: one barrier per
// block), the softmax / leaky / dropout backward in the MFMA output layout,
// dW̃[:, h] accumulated in registers (D per lane), d a_src / d a_dst, and
// dxs_h.  No logit or d-logit planes cross between waves, the xs rows and the
// W̃ column of the wave's head live in registers, and the logits are summed
// in the forward's order (even / odd d on packed FMAs), so the recomputed
// probabilities are the forward's bit for bit.  Two workgroups fit a CU (128
// VGPRs, 71 KB of LDS): the next block's rows are loaded after this block's
// work, their latency covered by the other workgroup.
// LDS: sEA[2][BT·BS][DP] edge rows | sO[2][BT][XW] dOut rows | sV[2][5][MH·BT]
//      per-target vectors (max, 1/sum, r, a_dst, self-loop share) | sPres[2][BT]
// ---------------------------------------------------------------------------
template <int D, bool EIDM, bool KEEP>
__global__ __launch_bounds__(WT, 4) void k_fattn_bwd2(
    const float* __restrict__ xs, int ldx, const float* __restrict__ ea,
    const float* __restrict__ wf, int hl_pad, int col0, const int32_t* __restrict__ eid,
    const uint8_t* __restrict__ keep, float keep_scale, const float* __restrict__ dout,
    const float* __restrict__ stats, const float* __restrict__ rs, float* __restrict__ dxs,
    float* __restrict__ adst_part, float* __restrict__ wpart, int n, int H, int C, float slope) {
  constexpr int DP = dpad<D>(), EV = DP / 4, DH = (D + 1) / 2;
  // edge rows of one target: BS·DP floats + 16 of padding (the along-i staging
  // writes of 16 consecutive targets then spread over the banks; the row
  // loop's b128 reads stay conflict-free)
  constexpr int ES = BS * DP + 16;
  // one LDS block, the small per-block arrays first (their reads in the row
  // loop take immediate offsets from one base register)
  constexpr int O_V = 0, O_WT = O_V + 2 * 5 * MH * BT, O_PR = O_WT + MH * DP;
  constexpr int O_O = (O_PR + 2 * BT + 3) & ~3, O_EA = O_O + 2 * BT * XW;
  __shared__ __attribute__((aligned(16))) float smem[O_EA + 2 * BT * ES];
  float(*const sV)[5][MH * BT] = reinterpret_cast<float(*)[5][MH * BT]>(smem + O_V);
  float* const sWT = smem + O_WT;  // W̃ columns, [h][d]
  uint32_t(*const sPres)[BT] = reinterpret_cast<uint32_t(*)[BT]>(smem + O_PR);
  float(*const sO)[BT * XW] = reinterpret_cast<float(*)[BT * XW]>(smem + O_O);
  float(*const sEA)[BT * ES] = reinterpret_cast<float(*)[BT * ES]>(smem + O_EA);

  const int NS = (n + BS - 1) / BS;
  int64_t g;
  int js;
  block_gt(NS, g, js);
  const int t = threadIdx.x, lane = t & 63, hh = t >> 6;  // wave hh: head hh
  for (int k = t; k < MH * DP; k += WT) {
    const int h = k / DP, d = k - h * DP;
    sWT[k] = (h < H && d < D) ? wf[d * hl_pad + col0 + h] : 0.f;
  }
  const int li = lane & 15, lk = lane >> 4;
  const int j0 = js * BS;
  const int HC = H * C;
  const int64_t row0 = g * n;
  const int64_t Ntot = (int64_t)gridDim.x / NS * n;
  const int E0 = n * (n - 1);
  const rsrc_t rea = EIDM ? make_rsrc(nullptr, 0u)
                          : make_rsrc(ea + g * (int64_t)E0 * D, (uint32_t)(4 * E0 * D));
  const rsrc_t rdo = make_rsrc(dout + row0 * HC, (uint32_t)(4 * n * HC));
  const rsrc_t rst = make_rsrc(stats + row0 * 4 * H, (uint32_t)(16 * n * H));
  const rsrc_t rrs = make_rsrc(rs + row0 * 4 * H, (uint32_t)(16 * n * H));
  const rsrc_t rxs = make_rsrc(xs + row0 * ldx, (uint32_t)(4 * n * ldx));
  const int HQ = HC >> 2;  // 16-B chunks per dOut row
  const float slope2 = slope * L2E;
  const bool hv = hh < H;
  float* const adst_row = adst_part + ((int64_t)js * Ntot + row0) * H + hh;  // + i*H

  for (int idx = t; idx < 2 * BT * XW; idx += WT) (&sO[0][0])[idx] = 0.f;  // padding stays 0
  // this wave's head: xs_h of the tile's sources (the B operand of dP, channels
  // 4lk..4lk+3 of source 16jt + li) and a_src, and the W̃ column, in registers
  f4 xb[2];
  float asrc[2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    const int j = j0 + 16 * jt + li;
    const bool ok = hv && j < n;
    xb[jt] = (ok && 4 * lk < C) ? bld4(rxs, 4 * (j * ldx + hh * C + 4 * lk)) : f4{0.f, 0.f, 0.f, 0.f};
    asrc[jt] = ok ? bld(rxs, 4 * (j * ldx + HC + hh)) : 0.f;
  }

  // prefetch registers: this thread's edge slot of the next block, a dOut
  // chunk and a per-target vector
  f32x4 evn[EV];
  bool presn = false;
  int sil = 0, sjl = 0;
  f32x4 don;
  float vecn[5];
  auto issue = [&](int i0) {
    const bool along_i = !EIDM && (j0 + BS <= i0);  // contiguous canonical runs
    sil = along_i ? (t & 15) : (t >> 5);
    sjl = along_i ? (t >> 4) : (t & 31);
    const int i = i0 + sil, j = j0 + sjl;
    if constexpr (EIDM) {
      if (i < n && j < n && i != j) SV2N_CHK(214, (row0 + i) * n + j, Ntot * n);
      const int64_t gid = (i < n && j < n && i != j) ? eid[(row0 + i) * n + j] : -1;
      presn = gid >= 0;
      const float* p = ea + (presn ? gid : 0) * D;
#pragma unroll
      for (int q = 0; q < EV; ++q)
#pragma unroll
        for (int c = 0; c < 4; ++c) evn[q][c] = (presn && 4 * q + c < D) ? p[4 * q + c] : 0.f;
    } else {
      const int cid = canon_id(i, j, n);
      if constexpr (D % 4 == 0) {
#pragma unroll
        for (int q = 0; q < EV; ++q) evn[q] = bld4(rea, cid >= 0 ? 4 * (cid * D + 4 * q) : OOB);
      } else {
#pragma unroll
        for (int q = 0; q < EV; ++q)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            evn[q][c] = 4 * q + c < D ? bld(rea, cid >= 0 ? 4 * (cid * D + 4 * q + c) : OOB) : 0.f;
      }
    }
    {
      const int r = t / HQ, cq = t - r * HQ, i2 = i0 + r;
      don = bld4(rdo, (r < BT && i2 < n) ? 4 * (i2 * HC + 4 * cq) : OOB);
    }
    if (t < MH * BT) {
      const int h = t >> 4, il = t & 15, i2 = i0 + il;
      const bool ok = h < H && i2 < n;
      const int o4 = ok ? 4 * (__mul24(i2, 4 * H) + h) : OOB;
      const int ox = ok ? 4 * (__mul24(i2, ldx) + HC + H + h) : OOB;
      vecn[0] = bld(rst, o4);
      vecn[1] = bld(rst, ok ? o4 + 4 * H : OOB);
      vecn[2] = bld(rrs, o4);
      vecn[3] = bld(rxs, ox);
      vecn[4] = bld(rrs, ok ? o4 + 12 * H : OOB);
    }
  };
  auto stage = [&](int buf) {
#pragma unroll
    for (int q = 0; q < EV; ++q)
      *reinterpret_cast<f32x4*>(&sEA[buf][sil * ES + sjl * DP + 4 * q]) = evn[q];
    {
      const int r = t / HQ, cq = t - r * HQ;
      if (r < BT) {
        const int cg = 4 * cq, h = cg / C, c = cg - h * C;
        *reinterpret_cast<f32x4*>(&sO[buf][r * XW + h * 16 + c]) = don;
      }
    }
    if (t < MH * BT) {
#pragma unroll
      for (int k = 0; k < 5; ++k) sV[buf][k][t] = vecn[k];
    }
    if constexpr (EIDM) {  // row sil = 32 consecutive threads: one ballot per half-wave
      const uint64_t m = __ballot(presn);
      if ((lane & 31) == 0) sPres[buf][sil] = (uint32_t)(m >> (lane & 32));
    }
  };

  f2 wacc[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) wacc[d] = f2{0.f, 0.f};
  f4 dacc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  float das[2] = {0.f, 0.f};

  issue(0);
  stage(0);
  __syncthreads();
  int par = 0;
  for (int i0 = 0; i0 < n; i0 += BT, par ^= 1) {
    // the block's work for this wave's head; CLEAN: no diagonal, no edge-id
    // map, no partial tile (every (target, source) pair is an edge)
    auto head_block = [&](auto clean_tag) __attribute__((always_inline)) {
      constexpr bool CLEAN = decltype(clean_tag)::value;
      const float* sEAb = sEA[par];
      const float* sOb = sO[par];
      // dP[i][j] = dOut_h[i] · xs_h[j]: rows i = 4lk + r, columns j = 16jt + li
      f4 pacc[2];
      const f4 oa = *reinterpret_cast<const f4*>(sOb + li * XW + hh * 16 + 4 * lk);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        f4 pa = {0.f, 0.f, 0.f, 0.f};
        pa = __builtin_amdgcn_mfma_f32_16x16x4f32(oa.x, xb[jt].x, pa, 0, 0, 0);
        pa = __builtin_amdgcn_mfma_f32_16x16x4f32(oa.y, xb[jt].y, pa, 0, 0, 0);
        pa = __builtin_amdgcn_mfma_f32_16x16x4f32(oa.z, xb[jt].z, pa, 0, 0, 0);
        pa = __builtin_amdgcn_mfma_f32_16x16x4f32(oa.w, xb[jt].w, pa, 0, 0, 0);
        pacc[jt] = pa;
      }
      const int q0 = hh * BT + 4 * lk;
      const f4* wt = reinterpret_cast<const f4*>(sWT + hh * DP);  // broadcast reads
      // target rows r of the lane one at a time (rolled: only the two edges of
      // one row are live), each finishing its d a_dst partial and its k-slice
      // of dxs += Pᵀ·dOut right away
#pragma unroll 1
      for (int r = 0; r < 4; ++r) {
        const int il = 4 * lk + r, i = i0 + il;
        const float* vr = &sV[par][0][q0 + r];
        const float mv = vr[0], iv = vr[MH * BT], rv = vr[2 * MH * BT];
        const float av = vr[3 * MH * BT], shv = vr[4 * MH * BT];
        const float ob = sOb[il * XW + hh * 16 + li];  // dOut_h[i][c = li]
        float rowacc = 0.f;
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
          const int jl = 16 * jt + li, j = j0 + jl;
          bool valid = true;
          if constexpr (!CLEAN) {
            valid = i < n && j < n && i != j;
            if constexpr (EIDM) valid = valid && ((sPres[par][il] >> jl) & 1u);
          }
          // the edge row and its logit, in the forward's order (even / odd d)
          const f4* er = reinterpret_cast<const f4*>(sEAb + il * ES + jl * DP);
          float ev[DP];
#pragma unroll
          for (int q = 0; q < EV; ++q) {
            const f4 w = er[q];
            ev[4 * q] = w.x; ev[4 * q + 1] = w.y; ev[4 * q + 2] = w.z; ev[4 * q + 3] = w.w;
          }
          f2 a2 = f2{0.f, 0.f};
#pragma unroll
          for (int q = 0; q < EV; ++q) {
            const f4 w4 = wt[q];
            if (4 * q < D)
              a2 = __builtin_elementwise_fma(f2{ev[4 * q], 4 * q + 1 < D ? ev[4 * q + 1] : 0.f},
                                             f2{w4.x, w4.y}, a2);
            if (4 * q + 2 < D)
              a2 = __builtin_elementwise_fma(
                  f2{ev[4 * q + 2], 4 * q + 3 < D ? ev[4 * q + 3] : 0.f}, f2{w4.z, w4.w}, a2);
          }
          const float v = (asrc[jt] + av) + (a2.x + a2.y);
          float p = fexp2(v * (v > 0.f ? L2E : slope2) - mv) * iv;
          if constexpr (!CLEAN) p = valid ? p : 0.f;
          const f4 pa = pacc[jt];
          float dP = r == 0 ? pa.x : (r == 1 ? pa.y : (r == 2 ? pa.z : pa.w));
          float pk = p;
          if constexpr (KEEP) {
            if (valid) SV2N_CHK(215, ((g * H + hh) * (int64_t)n + i) * n + j, Ntot * H * n);
            const bool kp = valid && keep[((g * H + hh) * (int64_t)n + i) * n + j] != 0;
            pk = kp ? p * keep_scale : 0.f;
            dP = kp ? dP * keep_scale : 0.f;
          }
          const float ds = p * (dP - rv);
          float dl = v > 0.f ? ds : ds * slope;
          if constexpr (!CLEAN) dl = valid ? dl : 0.f;
          das[jt] += dl;
          rowacc += dl;
          // dxs_h[j][c] += P[i][j] dOut_h[i][c]: this row's k-slice (A = P, lane (j, lk))
          dacc[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pk, ob, dacc[jt], 0, 0, 0);
          // dW̃[:, h] += edge row ⊗ (d logit + the self loop's share)
          float wsc = dl + shv;
          if constexpr (!CLEAN) wsc = valid ? wsc : 0.f;
#pragma unroll
          for (int d = 0; d < DH; ++d)
            wacc[d] = __builtin_elementwise_fma(f2{ev[2 * d], 2 * d + 1 < D ? ev[2 * d + 1] : 0.f},
                                                f2{wsc, wsc}, wacc[d]);
        }
        // d a_dst partial of this source tile: the row sum over the 16 lanes li
        const float s = row16_sum(rowacc);
        if (li == 0 && i < n)
          SV2N_CHK(216, ((int64_t)js * Ntot + row0 + i) * H + hh, (int64_t)NS * Ntot * H);
        if (li == 0 && i < n) adst_row[__mul24(i, H)] = s;
      }
    };
    if (hv) {
      if (!EIDM && (j0 + BS <= i0 || i0 + BT <= j0) && j0 + BS <= n && i0 + BT <= n)
        head_block(std::true_type{});
      else
        head_block(std::false_type{});
    }
    // the next block to the other buffer (last read before the previous
    // barrier); its loads wait here, under the other workgroup on the CU
    if (i0 + BT < n) {
      issue(i0 + BT);
      stage(par ^ 1);
    }
    __syncthreads();
  }

  // ---- d a_src (complete: every target was visited) + the self loop ----
  if (hv) {
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      const float s = lk_sum(das[jt]);
      const int j = j0 + 16 * jt + li;
      if (lk == 0 && j < n) {
        const int64_t row = row0 + j;
        SV2N_CHK(217, row * ldx + HC + hh, Ntot * ldx);
        SV2N_CHK(218, row * 4 * H + H + hh, Ntot * 4 * H);
        dxs[row * ldx + HC + hh] = s + rs[row * 4 * H + H + hh];
      }
    }
    // ---- dxs_h rows: accumulated products + the self loop's P·dOut ----
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      const float dv[4] = {dacc[jt].x, dacc[jt].y, dacc[jt].z, dacc[jt].w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = j0 + 16 * jt + 4 * lk + r, c = li;
        if (j < n && c < C) {
          const int64_t row = row0 + j;
          SV2N_CHK(219, row * ldx + hh * C + c, Ntot * ldx);
          SV2N_CHK(220, row * HC + hh * C + c, Ntot * HC);
          dxs[row * ldx + hh * C + c] =
              fmaf(rs[row * 4 * H + 2 * H + hh], dout[row * HC + hh * C + c], dv[r]);
        }
      }
    }
  }
  {
    const int padc = ldx - HC - 2 * H;
    for (int idx = t; idx < BS * padc; idx += WT) {
      const int jl = idx / padc, j = j0 + jl;
      if (j < n) SV2N_CHK(221, (row0 + j) * ldx + HC + 2 * H + (idx - jl * padc), Ntot * ldx);
      if (j < n) dxs[(row0 + j) * ldx + HC + 2 * H + (idx - jl * padc)] = 0.f;
    }
  }
  // ---- dW̃[:, h] partial of the workgroup: the wave's 64 lanes ----
  if (hv) {
    const int64_t P = (int64_t)gridDim.x;
    const int64_t part = g * NS + js;
#pragma unroll
    for (int d = 0; d < DH; ++d) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int dd = 2 * d + e;
        const float v = lk_sum(row16_sum(wacc[d][e]));
        if (lane == 0 && dd < D) wpart[(int64_t)(dd * H + hh) * P + part] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward: d a_dst (Σ over source tiles + self loop) and dW̃ (Σ of partials)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(PT) void k_fattn_bfinish(
    const float* __restrict__ adst_part, const float* __restrict__ rs, float* __restrict__ dxs,
    int ldx, int64_t N, int NS, int H, int HC, const float* __restrict__ wpart, int64_t P,
    float* __restrict__ dwf, int hl_pad, int col0, int64_t nA) {
  __shared__ float sred[PT];
  const int t = threadIdx.x;
  if ((int64_t)blockIdx.x < nA) {
    const int64_t idx = (int64_t)blockIdx.x * PT + t;
    if (idx < N * H) {
      const int64_t i = idx / H;
      const int h = (int)(idx - i * H);
      float s = 0.f;
      SV2N_CHK(222, ((NS - 1) * N + i) * H + h, (int64_t)NS * N * H);
      SV2N_CHK(223, i * ldx + HC + H + h, N * ldx);
      for (int q = 0; q < NS; ++q) s += adst_part[(q * N + i) * H + h];
      dxs[i * ldx + HC + H + h] = s + rs[i * 4 * H + H + h];
    }
    return;
  }
  const int q = (int)(blockIdx.x - nA);  // output (d, h) = q / H, q % H
  const float* src = wpart + (int64_t)q * P;
  float s = 0.f;
  for (int64_t k = t; k < P; k += PT) s += src[k];
  sred[t] = s;
  __syncthreads();
  for (int w = PT / 2; w > 0; w >>= 1) {
    if (t < w) sred[t] += sred[t + w];
    __syncthreads();
  }
  if (t == 0) {
    const int d = q / H, h = q - d * H;
    dwf[d * hl_pad + col0 + h] = sred[0];
  }
}

}  // namespace fused
}  // namespace sv2n

SV2N_CHK_EXPORT(fused)

// ============================ C-ABI ========================================
using namespace sv2n::fused;

#define SV2N_FVAR(M, DD)                       \
  if (eid) {                                     \
    if (keep) M(DD, true, true); else M(DD, true, false);  \
  } else {                                       \
    if (keep) M(DD, false, true); else M(DD, false, false); \
  }

extern "C" int sv2n_gat_attn_fused_supported(int n, int heads, int channels, int edge_dim) {
  const bool d_ok = edge_dim == 3 || edge_dim == 6 || edge_dim == 12;
  return (n > 32 && n <= 256 && heads >= 1 && heads <= MH && channels >= 4 && channels <= 16 &&
          channels % 4 == 0 && d_ok)
             ? 1
             : 0;
}

static int fused_check(const float* xs, int ldx, const float* ea, int edge_dim, const float* wf,
                       int hl_pad, int col0, int64_t B, int n, int H, int C, int act) {
  if (!xs || !ea || !wf || B <= 0) return SV2N_ERR_ARG;
  if (!sv2n_gat_attn_fused_supported(n, H, C, edge_dim) || act < 0 || act > 3)
    return SV2N_ERR_SHAPE;
  if (col0 < 0 || col0 + H > hl_pad) return SV2N_ERR_SHAPE;
  if (ldx < H * C + 2 * H || (ldx & 3) || ((uintptr_t)xs & 15)) return SV2N_ERR_ALIGN;
  if ((int64_t)n * ldx * 4 > 0x7fffffff) return SV2N_ERR_SHAPE;
  if ((int64_t)n * (n - 1) * edge_dim * 4 > 0x7fffff00LL) return SV2N_ERR_SHAPE;
  if (B * ((n + 31) / 32) > 0x7fffffffLL) return SV2N_ERR_SHAPE;
  return 0;
}

extern "C" int sv2n_gat_attn_fused_fwd(const float* xs, int ldx, const float* edge_attr,
                                       int edge_dim, const float* wfold, int hl_pad, int col0,
                                       const int32_t* eid, const float* bias, const uint8_t* keep,
                                       float keep_scale, float* y, float* agg, float* stats,
                                       int64_t num_graphs, int n, int heads, int channels,
                                       int concat, int act, float negative_slope,
                                       hipStream_t stream) {
  if (!y || ((agg == nullptr) != (stats == nullptr))) return SV2N_ERR_ARG;
  if (int rc = fused_check(xs, ldx, edge_attr, edge_dim, wfold, hl_pad, col0, num_graphs, n,
                           heads, channels, act))
    return rc;
  if (!eid && ((uintptr_t)edge_attr & 15)) return SV2N_ERR_ALIGN;
  const dim3 grid((unsigned)(num_graphs * ((n + FT - 1) / FT)));
#define SV2N_FFWD1(DD, EM, KP)                                                                  \
  hipLaunchKernelGGL((k_fattn_fwd<DD, EM, KP>), grid, dim3(WT), 0, stream, xs, ldx, edge_attr, wfold,     \
                     hl_pad, col0, eid, bias, keep, keep_scale, y, agg, stats, n, heads,        \
                     channels, act, concat, negative_slope)
  switch (edge_dim) {
    case 3: SV2N_FVAR(SV2N_FFWD1, 3) break;
    case 6: SV2N_FVAR(SV2N_FFWD1, 6) break;
    default: SV2N_FVAR(SV2N_FFWD1, 12) break;
  }
#undef SV2N_FFWD1
  return (int)hipGetLastError();
}

extern "C" int64_t sv2n_gat_attn_fused_bwd_workspace(int64_t num_graphs, int n, int heads,
                                                     int channels, int edge_dim) {
  const int64_t N = num_graphs * n;
  const int64_t NS = (n + BS - 1) / BS;
  return N * heads * channels        // dout
         + N * 4 * heads            // rs
         + NS * N * heads           // d a_dst partials
         + (int64_t)edge_dim * heads * num_graphs * NS;  // dW̃ partials
}

extern "C" int sv2n_gat_attn_fused_bwd(const float* dy, const float* y, const float* agg,
                                       const float* stats, const float* xs, int ldx,
                                       const float* edge_attr, int edge_dim, const float* wfold,
                                       int hl_pad, int col0, const int32_t* eid,
                                       const uint8_t* keep, float keep_scale, float* dxs,
                                       float* dbias_partial, float* dwfold, float* workspace,
                                       int64_t workspace_floats, int64_t num_graphs, int n,
                                       int heads, int channels, int concat, int act,
                                       float negative_slope, hipStream_t stream) {
  if (!dy || !y || !agg || !stats || !dxs || !dbias_partial || !dwfold || !workspace)
    return SV2N_ERR_ARG;
  if (int rc = fused_check(xs, ldx, edge_attr, edge_dim, wfold, hl_pad, col0, num_graphs, n,
                           heads, channels, act))
    return rc;
  if (!eid && ((uintptr_t)edge_attr & 15)) return SV2N_ERR_ALIGN;
  const int H = heads, C = channels, HC = H * C;
  if (((uintptr_t)dxs & 15)) return SV2N_ERR_ALIGN;
  const int64_t need = sv2n_gat_attn_fused_bwd_workspace(num_graphs, n, H, C, edge_dim);
  if (workspace_floats < need) return SV2N_ERR_WORKSPACE;
  const int64_t N = num_graphs * n;
  const int NT = (n + FT - 1) / FT, NS = (n + BS - 1) / BS;
  float* dout = workspace;
  float* rs = dout + N * HC;
  float* adst = rs + N * 4 * H;
  float* wpart = adst + (int64_t)NS * N * H;
  if (((uintptr_t)dout & 15)) return SV2N_ERR_ALIGN;
  hipLaunchKernelGGL(k_fattn_bprep, dim3((unsigned)(num_graphs * NT)), dim3(PT), 0, stream, dy,
                     y, agg, stats, xs, ldx, keep, keep_scale, dout, rs, dbias_partial, n, H, C,
                     act, concat, negative_slope);
  const dim3 grid((unsigned)(num_graphs * NS));
#define SV2N_FBWD1(DD, EM, KP)                                                                  \
  hipLaunchKernelGGL((k_fattn_bwd2<DD, EM, KP>), grid, dim3(WT), 0, stream, xs, ldx, edge_attr, wfold, \
                     hl_pad, col0, eid, keep, keep_scale, dout, stats, rs, dxs, adst, wpart, n, \
                     H, C, negative_slope)
  switch (edge_dim) {
    case 3: SV2N_FVAR(SV2N_FBWD1, 3) break;
    case 6: SV2N_FVAR(SV2N_FBWD1, 6) break;
    default: SV2N_FVAR(SV2N_FBWD1, 12) break;
  }
#undef SV2N_FBWD1
  const int64_t nA = (N * H + PT - 1) / PT;
  hipLaunchKernelGGL(k_fattn_bfinish, dim3((unsigned)(nA + edge_dim * H)), dim3(PT), 0, stream,
                     adst, rs, dxs, ldx, N, NS, H, HC, wpart, num_graphs * NS, dwfold, hl_pad,
                     col0, nA);
  return (int)hipGetLastError();
}
