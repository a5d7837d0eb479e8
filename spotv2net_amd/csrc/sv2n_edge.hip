// Edge-feature streaming kernels: the folded lin_edge·att_edge logits for all
// GAT layers in ONE pass over edge_attr, and the matching weight gradient.
//
// Reference semantics (PyG 2.3.0 GATConv.edge_update, used by
// utils/models.py:146 for every layer):
//     a_e[e,h] = Σ_c (edge_attr[e] · W_edge[h*C+c,:]) * att_edge[h,c]
// which is linear in edge_attr, so it is evaluated as edge_attr[e] · W̃[:,h]
// with W̃ = fold(W_edge, att_edge) built by the host (autograd-tracked).  The
// fold removes the [E, H*C] intermediate (737 MB per layer at batch 512) and
// divides the flops by C; what is left is an HBM stream of edge_attr.
//
// HBM layout: edge_attr [E][D] fp32 row-major (D = 3*seq_length), read once
// per pass with 16-B loads into an LDS chunk of 64 edges.
#include <cstdlib>
#include "sv2n_common.h"

namespace sv2n {

constexpr int EDGE_CHUNK = 64;
constexpr int EDGE_THREADS = 256;

struct LayerPtrs { float* p[SV2N_MAX_LAYERS]; };
struct LayerCPtrs { const float* p[SV2N_MAX_LAYERS]; };

// Both kernels are persistent (grid-stride over 64-edge chunks) and
// software-pipelined: the next chunk's edge rows (and, backward, its gathered
// dAE values) are loaded into registers while the current chunk is computed
// from LDS, so each workgroup keeps one chunk (32 KB at D = 126) in flight.
// RF = float4 registers per thread for a chunk: D <= 16*RF.
constexpr int EDGE_RF_MAX = 24;

__device__ __forceinline__ int rf_needed(int D) { return (EDGE_CHUNK * D / 4 + EDGE_THREADS - 1) / EDGE_THREADS; }

// native vector type: HIP's float4 struct copies lower to memcpy through a
// stack slot, which keeps the prefetch array in scratch
typedef float vf4 __attribute__((ext_vector_type(4)));

template <int RF>
struct ChunkRegs {
  vf4 v[RF];
  __device__ __forceinline__ void load(const float* __restrict__ ea, int64_t e0, int ne, int D,
                                       int t) {
    const vf4* s4 = reinterpret_cast<const vf4*>(ea + e0 * D);  // 16-B aligned (e0 % 64 == 0)
    const int last = max(((ne * D) >> 2) - 1, 0);
    // unconditional loads from clamped slots (the store side skips k >= nf4),
    // so the register array is always fully defined (no scratch, no branches)
#pragma unroll
    for (int s = 0; s < RF; ++s) v[s] = s4[min(t + s * EDGE_THREADS, last)];
  }
  // flat copy into an unpadded [64][D] image plus the (ne*D)%4 scalar tail.
  // The image holds RF*256 float4 slots, so every slot is stored without a
  // branch (surplus slots land in rows >= ne, which are never read).
  __device__ __forceinline__ void store_flat(float* __restrict__ s_ea, const float* __restrict__ ea,
                                             int64_t e0, int ne, int D, int t) const {
    const int nf = ne * D, nf4 = nf >> 2;
    vf4* d4 = reinterpret_cast<vf4*>(s_ea);
#pragma unroll
    for (int s = 0; s < RF; ++s) d4[t + s * EDGE_THREADS] = v[s];
    for (int k = (nf4 << 2) + t; k < nf; k += EDGE_THREADS) s_ea[k] = ea[e0 * D + k];
  }
  // scatter into a [64][DP] image with padded rows (DP = D rounded up to 4)
  __device__ __forceinline__ void store_padded(float* __restrict__ s_ea,
                                               const float* __restrict__ ea, int64_t e0, int ne,
                                               int D, int DP, int t) const {
    const int nf = ne * D, nf4 = nf >> 2;
#pragma unroll
    for (int s = 0; s < RF; ++s) {
      const int k = t + s * EDGE_THREADS;
      if (k < nf4) {
        const vf4 x = v[s];
        const int f = k << 2;
        int r = f / D, d = f - r * D;
        s_ea[r * DP + d] = x.x; if (++d == D) { d = 0; ++r; }
        s_ea[r * DP + d] = x.y; if (++d == D) { d = 0; ++r; }
        s_ea[r * DP + d] = x.z; if (++d == D) { d = 0; ++r; }
        s_ea[r * DP + d] = x.w;
      }
    }
    for (int f = (nf4 << 2) + t; f < nf; f += EDGE_THREADS) {
      const int r = f / D;
      s_ea[r * DP + (f - r * D)] = ea[e0 * D + f];
    }
    for (int k = t; k < ne * (DP - D); k += EDGE_THREADS) {
      const int r = k / (DP - D);
      s_ea[r * DP + D + (k - r * (DP - D))] = 0.f;
    }
  }
};

// ---------------------------------------------------------------------------
// forward: ae[l][g][i][j][h] = edge_attr[e] · wfold[:, l*H+h]
// per chunk, thread (el = t/4, q = t%4) sums d ≡ q (mod 4) for all hl_pad
// columns, quad-reduced through DPP, then written per layer.
// ---------------------------------------------------------------------------
template <int HLP, int RF, bool PLANES>
__global__ __launch_bounds__(EDGE_THREADS) void k_edge_fwd(
    const float* __restrict__ ea, int64_t E, int D, const int64_t* __restrict__ ei,
    const uint16_t* __restrict__ canon, int E0, const float* __restrict__ wf, LayerPtrs ae,
    int L, int H, int64_t B, int n) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s_wf = smem;                            // [D][HLP]
  float* s_ea = smem + D * HLP;                  // [64][D] (RF*1024 floats)
  float* s_out = s_ea + RF * EDGE_THREADS * 4;   // [64][HLP]
  __shared__ float* s_ptr[SV2N_MAX_LAYERS];

  const int t = threadIdx.x;
  if (t < SV2N_MAX_LAYERS) {
#pragma unroll
    for (int l = 0; l < SV2N_MAX_LAYERS; ++l)
      if (l == t) s_ptr[l] = ae.p[l];
  }
  {
    const float4* w4 = reinterpret_cast<const float4*>(wf);
    float4* sw4 = reinterpret_cast<float4*>(s_wf);
    for (int k = t; k < D * HLP / 4; k += EDGE_THREADS) sw4[k] = w4[k];
  }
  const int64_t nchunks = (E + EDGE_CHUNK - 1) / EDGE_CHUNK;
  const int el = t >> 2, q = t & 3;
  const int HL = L * H;
  ChunkRegs<RF> R;
  int64_t c = blockIdx.x;
  if (c < nchunks) R.load(ea, c * EDGE_CHUNK, (int)min((int64_t)EDGE_CHUNK, E - c * EDGE_CHUNK), D, t);
  for (; c < nchunks; c += gridDim.x) {
    const int64_t e0 = c * EDGE_CHUNK;
    const int ne = (int)min((int64_t)EDGE_CHUNK, E - e0);
    __syncthreads();  // previous chunk's LDS fully consumed
    R.store_flat(s_ea, ea, e0, ne, D, t);
    __syncthreads();
    const int64_t cn = c + gridDim.x;
    if (cn < nchunks)
      R.load(ea, cn * EDGE_CHUNK, (int)min((int64_t)EDGE_CHUNK, E - cn * EDGE_CHUNK), D, t);

    float acc[HLP];
#pragma unroll
    for (int k = 0; k < HLP; ++k) acc[k] = 0.f;
    if (el < ne) {
      const float* row = s_ea + el * D;
      for (int d = q; d < D; d += 4) {
        const float v = row[d];
        const float4* w4 = reinterpret_cast<const float4*>(s_wf + d * HLP);
#pragma unroll
        for (int k4 = 0; k4 < HLP / 4; ++k4) {
          const float4 w = w4[k4];
          acc[4 * k4 + 0] = fmaf(v, w.x, acc[4 * k4 + 0]);
          acc[4 * k4 + 1] = fmaf(v, w.y, acc[4 * k4 + 1]);
          acc[4 * k4 + 2] = fmaf(v, w.z, acc[4 * k4 + 2]);
          acc[4 * k4 + 3] = fmaf(v, w.w, acc[4 * k4 + 3]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < HLP; ++k) {
      acc[k] += dpp_xor1(acc[k]);
      acc[k] += dpp_xor2(acc[k]);
    }
    // lane q of the quad parks columns k ≡ q (mod 4) in LDS (compile-time index)
#pragma unroll
    for (int k = 0; k < HLP; ++k)
      if ((k & 3) == q) s_out[el * HLP + k] = acc[k];
    __syncthreads();
    if constexpr (PLANES) {  // [H][E] per layer: 64 consecutive edges per (layer, head)
      for (int idx = t; idx < ne * HL; idx += EDGE_THREADS) {
        const int k = idx / ne, le = idx - k * ne;
        const int l = k / H, h = k - l * H;
        s_ptr[l][(int64_t)h * E + e0 + le] = s_out[le * HLP + k];
      }
    } else if (!ei) {  // canonical batch: edge order [E][H] per layer, contiguous runs
      const int nh = ne * H;
      for (int idx = t; idx < L * nh; idx += EDGE_THREADS) {
        const int l = idx / nh, r = idx - l * nh;
        const int le = r / H, h = r - le * H;
        SV2N_CHK(402, e0 * H + r, E * H);
        s_ptr[l][e0 * H + r] = s_out[le * HLP + l * H + h];
      }
    } else {
      for (int idx = t; idx < ne * HL; idx += EDGE_THREADS) {
        const int le = idx / HL, k = idx - le * HL;
        int64_t g;
        int i, j;
        if (!decode_edge(e0 + le, ei, E, canon, E0, n, B, g, i, j)) continue;
        const int l = k / H, h = k - l * H;
        SV2N_CHK(401, ((g * n + i) * n + j) * H + h, B * n * n * H);
        s_ptr[l][((g * n + i) * n + j) * H + h] = s_out[le * HLP + k];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward: partial[b][d][k] = Σ_{e in block b's chunks} edge_attr[e][d] * dae_e[k]
// thread tile = 4 d x 4 k outer products, ES edge-groups per tile; block-level
// reduction at the end, then k_reduce_partials sums the per-block partials in
// a fixed order (deterministic).
// ---------------------------------------------------------------------------
template <int HLP, bool PLANES>
__device__ __forceinline__ void gather_dae(float (&gd)[(EDGE_CHUNK * HLP + EDGE_THREADS - 1) / EDGE_THREADS],
                                           const float* const* s_ptr, const int64_t* __restrict__ ei,
                                           int64_t E, const uint16_t* __restrict__ canon, int E0,
                                           int n, int64_t B, int HL, int H, int64_t e0, int ne,
                                           int t) {
  constexpr int GN = (EDGE_CHUNK * HLP + EDGE_THREADS - 1) / EDGE_THREADS;
#pragma unroll
  for (int s = 0; s < GN; ++s) {
    const int idx = t + s * EDGE_THREADS;
    float v = 0.f;
    if constexpr (PLANES) {  // edge fastest: coalesced reads of the [H][E] planes
      const int le = idx & (EDGE_CHUNK - 1), k = idx / EDGE_CHUNK;
      const int64_t e = e0 + le;
      if (le < ne && k < HL && !(ei && ei[e] == ei[E + e])) {
        const int l = k / H, h = k - l * H;
        v = s_ptr[l][(int64_t)h * E + e];
      }
    } else if (!ei) {  // canonical batch: edge order [E][H]
      const int le = idx / HLP, k = idx - le * HLP;
      if (le < ne && k < HL) {
        const int l = k / H, h = k - l * H;
        SV2N_CHK(404, (e0 + le) * H + h, E * H);
        v = s_ptr[l][(e0 + le) * H + h];
      }
    } else {
      const int le = idx / HLP, k = idx - le * HLP;
      int64_t g;
      int i, j;
      if (le < ne && k < HL && decode_edge(e0 + le, ei, E, canon, E0, n, B, g, i, j)) {
        const int l = k / H, h = k - l * H;
        SV2N_CHK(403, ((g * n + i) * n + j) * H + h, B * n * n * H);
        v = s_ptr[l][((g * n + i) * n + j) * H + h];
      }
    }
    gd[s] = v;
  }
}

// NT > 1 (wide shapes: (DP/4)·(HLP/4) thread tiles > 256, e.g. the HPO grid's
// seq_length 120 with 3 layers x 7 heads): every thread owns tiles t, t + 256,
// ... and walks every edge of the chunk (ES = 1).
template <int HLP, int RF, bool PLANES, int NT>
__global__ __launch_bounds__(EDGE_THREADS) void k_edge_bwd(
    const float* __restrict__ ea, int64_t E, int D, int DP, const int64_t* __restrict__ ei,
    const uint16_t* __restrict__ canon, int E0, LayerCPtrs dae, int L, int H, int64_t B, int n,
    float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s_ea = smem;                        // [64][DP]
  float* s_dae = smem + max(EDGE_CHUNK * DP, RF * EDGE_THREADS * 4);  // [64][HLP]
  __shared__ const float* s_ptr[SV2N_MAX_LAYERS];
  constexpr int GN = (EDGE_CHUNK * HLP + EDGE_THREADS - 1) / EDGE_THREADS;

  const int t = threadIdx.x;
  if (t < SV2N_MAX_LAYERS) {
#pragma unroll
    for (int l = 0; l < SV2N_MAX_LAYERS; ++l)
      if (l == t) s_ptr[l] = dae.p[l];
  }
  __syncthreads();
  const int KG = HLP / 4;
  const int T = (DP / 4) * KG;  // thread tiles
  const int ES = NT == 1 ? EDGE_THREADS / T : 1;
  const int tile = NT == 1 ? t % T : t, es = NT == 1 ? t / T : 0;
  const int HL = L * H;

  float acc[NT][16];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[j][k] = 0.f;

  const int64_t nchunks = (E + EDGE_CHUNK - 1) / EDGE_CHUNK;
  ChunkRegs<RF> R;
  float gd[GN];
  int64_t c = blockIdx.x;
  if (c < nchunks) {
    const int64_t e0 = c * EDGE_CHUNK;
    const int ne = (int)min((int64_t)EDGE_CHUNK, E - e0);
    R.load(ea, e0, ne, D, t);
    gather_dae<HLP, PLANES>(gd, s_ptr, ei, E, canon, E0, n, B, HL, H, e0, ne, t);
  }
  for (; c < nchunks; c += gridDim.x) {
    const int64_t e0 = c * EDGE_CHUNK;
    const int ne = (int)min((int64_t)EDGE_CHUNK, E - e0);
    __syncthreads();  // previous chunk fully consumed
    if (DP == D) R.store_flat(s_ea, ea, e0, ne, D, t);
    else R.store_padded(s_ea, ea, e0, ne, D, DP, t);
#pragma unroll
    for (int s = 0; s < GN; ++s) {
      const int idx = t + s * EDGE_THREADS;
      if (idx < EDGE_CHUNK * HLP)
        s_dae[PLANES ? (idx & (EDGE_CHUNK - 1)) * HLP + idx / EDGE_CHUNK : idx] = gd[s];
    }
    __syncthreads();
    const int64_t cn = c + gridDim.x;
    if (cn < nchunks) {
      const int64_t e1 = cn * EDGE_CHUNK;
      const int ne1 = (int)min((int64_t)EDGE_CHUNK, E - e1);
      R.load(ea, e1, ne1, D, t);
      gather_dae<HLP, PLANES>(gd, s_ptr, ei, E, canon, E0, n, B, HL, H, e1, ne1, t);
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int tj = tile + j * EDGE_THREADS;
      if (es < ES && tj < T) {
        const int dg = tj / KG, kg = tj - dg * KG;
        for (int le = es; le < ne; le += ES) {
          const float4 a = *reinterpret_cast<const float4*>(s_ea + le * DP + 4 * dg);
          const float4 b = *reinterpret_cast<const float4*>(s_dae + le * HLP + 4 * kg);
          const float av[4] = {a.x, a.y, a.z, a.w};
          const float bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y)
              acc[j][4 * x + y] = fmaf(av[x], bv[y], acc[j][4 * x + y]);
        }
      }
    }
  }
  // block reduction over the ES edge groups (reuse the chunk buffer)
  __syncthreads();
  float* s_red = smem;  // [ES][T][16]: <= max(256, T)*16 floats
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int tj = tile + j * EDGE_THREADS;
    if (es < ES && tj < T) {
#pragma unroll
      for (int k = 0; k < 16; ++k) s_red[(es * T + tj) * 16 + k] = acc[j][k];
    }
  }
  __syncthreads();
  const int O = D * HLP;
  for (int o = t; o < O; o += EDGE_THREADS) {
    const int d = o / HLP, k = o - d * HLP;
    const int tl = (d >> 2) * KG + (k >> 2);
    const int sub = (d & 3) * 4 + (k & 3);
    float s = 0.f;
    for (int g2 = 0; g2 < ES; ++g2) s += s_red[(g2 * T + tl) * 16 + sub];
    partial[(int64_t)blockIdx.x * O + o] = s;
  }
}

// out[o] = Σ_b partial[b][o] in a fixed order: a block owns 16 outputs, 16
// row groups each sum every 16th partial with 32 buffer loads in flight per
// round (out-of-range offsets read 0; round 4: 8 in flight took 5.7 us for
// the 1,024 partials of the C2 edge gradient, a chain of memory round trips),
// then combine through LDS.
__global__ __launch_bounds__(256) void k_reduce_partials(const float* __restrict__ partial,
                                                         int nparts, int O,
                                                         float* __restrict__ out) {
  constexpr int U = 32;
  __shared__ float s_red[16][17];
  const int lo = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int o = blockIdx.x * 16 + lo;
  const rsrc_t rp = make_rsrc(partial, (uint32_t)nparts * (uint32_t)O * 4u);
  float a = 0.f;
  for (int b0 = 0; b0 < nparts; b0 += 16 * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = b0 + grp + 16 * u;
      v[u] = bld(rp, (o < O && b < nparts) ? (b * O + o) * 4 : OOB);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) a += v[u];
  }
  s_red[grp][lo] = a;
  __syncthreads();
  if (grp == 0 && o < O) {
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) sm += s_red[k][lo];
    out[o] = sm;
  }
}

__global__ void k_block_rowmask(const int64_t* __restrict__ ei, int64_t E, int64_t N, int n,
                                uint32_t* __restrict__ rowmask) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int64_t s = ei[e], t = ei[E + e];
  if (s == t || t < 0 || t >= N) return;
  const int64_t g = t / n;
  const int64_t j = s - g * n;
  if (j < 0 || j >= n) return;
  const int W = (n + 31) >> 5;
  atomicOr(&rowmask[t * W + (j >> 5)], 1u << (int)(j & 31));
}

// rowmask plus validation without a host round trip: counts into *bad the
// edges the dense-block kernels cannot take (an end outside [0, N), source
// and target in different n-node blocks, a repeated (target, source) pair —
// the atomicOr that finds its bit already set)
__global__ void k_block_rowmask_checked(const int64_t* __restrict__ ei, int64_t E, int64_t N,
                                        int n, uint32_t* __restrict__ rowmask,
                                        int* __restrict__ bad) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int64_t s = ei[e], t = ei[E + e];
  if (s < 0 || s >= N || t < 0 || t >= N || s / n != t / n) {
    atomicAdd(bad, 1);
    return;
  }
  if (s == t) return;  // input self loops: PyG removes them
  const int64_t j = s - (t / n) * n;
  const int W = (n + 31) >> 5;
  const uint32_t bit = 1u << (int)(j & 31);
  if (atomicOr(&rowmask[t * W + (j >> 5)], bit) & bit) atomicAdd(bad, 1);
}

// ---------------------------------------------------------------------------
// narrow edge features (D <= 16, e.g. the C5 stress shapes, D = 12): a 64-edge
// chunk is only 3 KB there, too little in flight per workgroup, so one thread
// owns one edge row instead.
//   forward:  acc[k] = Σ_d ea[e][d] · W̃[d][k] (W̃ broadcast from LDS), stored
//             per (layer, head) — coalesced across the wave in the plane layout
//   backward: wave w owns columns k in [w*HLP/4, (w+1)*HLP/4) and accumulates
//             ea[e][d] · dAE[e][k] for its lanes' edges in registers over a
//             grid-stride loop; one wave reduction per (d, k) at the end, then
//             k_reduce_partials (fixed order, deterministic).
// ---------------------------------------------------------------------------
constexpr int EDGE_SMALL_D = 16;

// per-column output bases, built on the host: column k = l*H + h of layer l's
// AE lives at col[k][e] (planes) or col[k][((g*n+i)*n+j)*H] (dense block)
struct ColPtrs { float* p[32]; };
struct ColCPtrs { const float* p[32]; };

template <int DS>
__device__ __forceinline__ void load_row_small(float (&x)[DS], const float* __restrict__ ea,
                                               int64_t e, int D) {
#pragma unroll
  for (int d = 0; d < DS; ++d) x[d] = d < D ? ea[e * D + d] : 0.f;
}

template <int DS, int HLP, bool PLANES>
__global__ __launch_bounds__(256) void k_edge_fwd_small(
    const float* __restrict__ ea, int64_t E, int D, const int64_t* __restrict__ ei,
    const uint16_t* __restrict__ canon, int E0, const float* __restrict__ wf, ColPtrs col,
    int L, int H, int64_t B, int n) {
  __shared__ __attribute__((aligned(16))) float s_wf[DS * HLP];
  const int t = threadIdx.x;
  for (int k = t; k < DS * HLP; k += 256) s_wf[k] = k < D * HLP ? wf[k] : 0.f;
  __syncthreads();
  const int HL = L * H;
  const float4* w4 = reinterpret_cast<const float4*>(s_wf);
  for (int64_t e = (int64_t)blockIdx.x * 256 + t; e < E; e += (int64_t)gridDim.x * 256) {
    float x[DS];
    load_row_small<DS>(x, ea, e, D);
    int64_t off = e;
    if constexpr (!PLANES) {
      int64_t g;
      int i, j;
      if (!ei) {
        off = e * H;  // canonical batch: edge order
      } else {
        if (!decode_edge(e, ei, E, canon, E0, n, B, g, i, j)) continue;
        off = ((g * n + i) * n + j) * H;
      }
    }
    // 4 output columns at a time (not unrolled: W̃ stays in LDS as broadcast
    // reads instead of D*HLP live VGPRs)
#pragma unroll 1
    for (int k0 = 0; k0 < HL; k0 += 4) {
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
      for (int d = 0; d < DS; ++d) {
        const float4 w = w4[d * (HLP / 4) + (k0 >> 2)];
        a0 = fmaf(x[d], w.x, a0);
        a1 = fmaf(x[d], w.y, a1);
        a2 = fmaf(x[d], w.z, a2);
        a3 = fmaf(x[d], w.w, a3);
      }
      col.p[k0][off] = a0;
      if (k0 + 1 < HL) col.p[k0 + 1][off] = a1;
      if (k0 + 2 < HL) col.p[k0 + 2][off] = a2;
      if (k0 + 3 < HL) col.p[k0 + 3][off] = a3;
    }
  }
}

template <int DS, int HLP, bool PLANES>
__global__ __launch_bounds__(256) void k_edge_bwd_small(
    const float* __restrict__ ea, int64_t E, int D, const int64_t* __restrict__ ei,
    const uint16_t* __restrict__ canon, int E0, ColCPtrs col, int L, int H, int64_t B, int n,
    float* __restrict__ partial) {
  constexpr int KQ = HLP / 4;
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int HL = L * H;
  float acc[DS][KQ];
#pragma unroll
  for (int d = 0; d < DS; ++d)
#pragma unroll
    for (int q = 0; q < KQ; ++q) acc[d][q] = 0.f;
  for (int64_t e = (int64_t)blockIdx.x * 64 + lane; e < E; e += (int64_t)gridDim.x * 64) {
    int64_t off = e;
    bool ok;
    if constexpr (PLANES) {
      ok = !(ei && ei[e] == ei[E + e]);
    } else if (!ei) {
      ok = true;
      off = e * H;  // canonical batch: edge order
    } else {
      int64_t g;
      int i, j;
      ok = decode_edge(e, ei, E, canon, E0, n, B, g, i, j);
      off = ((g * n + i) * n + j) * H;
    }
    if (!ok) continue;
    float x[DS];
    load_row_small<DS>(x, ea, e, D);
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const int k = wave * KQ + q;  // wave-uniform
      const float v = k < HL ? col.p[k][off] : 0.f;
#pragma unroll
      for (int d = 0; d < DS; ++d) acc[d][q] = fmaf(x[d], v, acc[d][q]);
    }
  }
  // wave reduction, lane 0 writes this block's [D][HLP] slab entries of its columns
  float* pb = partial + (int64_t)blockIdx.x * D * HLP;
#pragma unroll
  for (int d = 0; d < DS; ++d)
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      float v = acc[d][q];
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
      if (lane == 0 && d < D) pb[d * HLP + wave * KQ + q] = v;
    }
}

// Head-plane backward on MFMA (D <= 16, E % 4 == 0, no input self loops):
//   partial[d][k] = Σ_e ea[e][d] · dAE_k[e]  =  (eaᵀ · dAE)[d][k]
// is a 16 x HLP output with K = E: each wave accumulates it in HLP/16
// v_mfma_f32_16x16x4_f32 tiles over its own grid-stride stream of 64-edge
// chunks.  Within a chunk lane group lk (= lane>>4) owns edges
// e0 + 16*lk + s, s = 0..15 (MFMA step s), so its dAE operand for four steps
// is one 16-B load from the plane and A (= ea[e][d], d = lane&15) is a
// column read of 16 consecutive rows.  The four waves' tiles are summed
// through LDS into one slab per block (k_reduce_partials finishes).
template <int HLP>
__global__ __launch_bounds__(256) void k_edge_bwd_mfma(const float* __restrict__ ea, int64_t E,
                                                       int D, ColCPtrs col, int HL,
                                                       float* __restrict__ partial) {
  constexpr int NT = HLP >= 16 ? HLP / 16 : 1;
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ float s_red[4][16 * NT * 16];
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, lk = lane >> 4;
  f4 acc[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) acc[q] = f4{0.f, 0.f, 0.f, 0.f};
  const float* bp[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) bp[q] = (16 * q + li < HL) ? col.p[16 * q + li] : nullptr;
  const int64_t nchunks = (E + 63) / 64;
  const int64_t stride = (int64_t)gridDim.x * 4;
  for (int64_t c = (int64_t)blockIdx.x * 4 + wave; c < nchunks; c += stride) {
    const int64_t eb = c * 64 + 16 * lk;  // this lane group's 16 edges
    float a[16];
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2)
      a[s2] = (li < D && eb + s2 < E) ? ea[(eb + s2) * D + li] : 0.f;
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      f4 b[4];
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) {
        const int64_t e = eb + 4 * c4;
        b[c4] = (bp[q] && e < E) ? *reinterpret_cast<const f4*>(bp[q] + e) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2)
        acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], b[s2 >> 2][s2 & 3], acc[q], 0, 0, 0);
    }
  }
  // D layout: acc[q][r] = out[d = 4*lk + r][k = 16q + li]
#pragma unroll
  for (int q = 0; q < NT; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) s_red[wave][(4 * lk + r) * (16 * NT) + 16 * q + li] = acc[q][r];
  __syncthreads();
  float* pb = partial + (int64_t)blockIdx.x * D * HLP;
  for (int o = t; o < D * HLP; o += 256) {
    const int d = o / HLP, k = o - d * HLP;
    float v = 0.f;
    if (k < 16 * NT) v = (s_red[0][d * 16 * NT + k] + s_red[1][d * 16 * NT + k]) +
                         (s_red[2][d * 16 * NT + k] + s_red[3][d * 16 * NT + k]);
    pb[o] = v;
  }
}

// ---------------------------------------------------------------------------
// Canonical batches with wide edge rows (C2 / C3: D = 126), round 4: both
// passes as HBM streams whose inner products run on v_mfma_f32_16x16x4_f32
// (exact f32 products, f32 accumulation), so LDS carries each edge row at
// most once (the kernels above re-read every staged value 8-16 times from
// LDS: thread tiles of 4 d x 4 columns, W̃ broadcasts).  A wave owns tiles
// of MX_TE = 16 consecutive edges (grid-stride over tiles, adjacent waves on
// adjacent tiles); the next tile's loads are in flight while one is computed.
//
// forward:  logits[e][k] = Σ_d ea[e][d]·W̃[d][k]   (M = 16 edges, N = 16 >= HL
//   columns, K = d).  The MFMA A operand puts 16 rows on 4 lanes each, so the
//   tile (16·D contiguous floats) is loaded flat instead (dwordx2, 512
//   contiguous bytes per instruction; D even, so no float2 straddles a row)
//   into the wave's [17][132] LDS image (row 16 takes the lanes past the
//   tile; row i starts at bank 4i, so a half-wave's 32 b64 reads hit 64
//   distinct banks) and read back with ds_read_b64: MFMA (s, c) pairs lane
//   group g with d = 8s + 2g + c.  W̃ lives in 2·NS registers per lane.
// backward: partial[d][k] = Σ_e ea[e][d]·dAE[e][k]   (M = d, N = columns,
//   K = edges).  K step q takes edges 4g + q of the tile; M tile m holds
//   d = 32·(m/2) + 2i + (m&1), so lane (i, g) loads the A operands of M tiles
//   m, m + 1 as one float2 straight from HBM: an instruction reads 4 rows x
//   128 contiguous bytes, no LDS image at all.  dAE comes from the layers'
//   [E][H] buffers (4 dwords per lane per tile).  The wave accumulators are
//   summed in wave order through LDS into one [D][hl_pad] partial per
//   workgroup (k_reduce_partials finishes).
// ---------------------------------------------------------------------------
constexpr int MX_TE = 16, MX_PF = 132, MX_WAVES = 4;
// backward: tiles in flight per wave.  Round 4 A/B (C2 traced step, one box):
// 1 tile (95 VGPRs, 5 waves / SIMD) 52.0 us, 2 tiles (150 VGPRs, 3 waves /
// SIMD) 53.4 us; the round-3 LDS-tile kernel took 56.7 us in the same place.
constexpr int MX_DEPTH = 1;

// per lane: this column's output / input row pointer (column li = l·H + h)
template <typename T, typename P>
__device__ __forceinline__ T* mx_col_ptr(const P& lp, int li, int L, int H) {
  T* r = nullptr;
#pragma unroll
  for (int l = 0; l < SV2N_MAX_LAYERS; ++l)
    if (l < L && li >= l * H && li < (l + 1) * H) r = lp.p[l] + (li - l * H);
  return r;
}

// the tile's rows as a buffer (nothing past E or past the last tile)
__device__ __forceinline__ rsrc_t mx_tile_rsrc(const float* ea, int64_t t, int64_t ntiles,
                                               int64_t E, int D) {
  const int64_t e0 = t * MX_TE;
  const int64_t rows = t < ntiles ? min((int64_t)MX_TE, E - e0) : 0;
  return make_rsrc(ea + (t < ntiles ? e0 * D : 0), (uint32_t)(rows * D * 4));
}

template <int NS>
__global__ __launch_bounds__(256, 4) void k_edge_fwd_mx(const float* __restrict__ ea, int64_t E,
                                                        int D, const float* __restrict__ wf,
                                                        int hlp, LayerPtrs ae, int L, int H) {
  __shared__ __attribute__((aligned(16))) float s_img[MX_WAVES][(MX_TE + 1) * MX_PF];
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int li = lane & 15, g = lane >> 4;
  const int HL = L * H;
  float* img = s_img[wave];
  // columns D .. 8·NS of the 16 rows are read as operands: zero them once
  for (int k = lane; k < MX_TE * (8 * NS - D); k += 64) {
    const int r = k / (8 * NS - D);
    img[r * MX_PF + D + (k - r * (8 * NS - D))] = 0.f;
  }
  float wb[NS][2];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int d = 8 * s + 2 * g + c;
      wb[s][c] = (d < D && li < HL) ? wf[d * hlp + li] : 0.f;
    }
  float* outp = li < HL ? mx_col_ptr<float>(ae, li, L, H) : nullptr;
  // flat piece j of a tile: floats f = 128j + 2·lane -> tile byte offset, image offset
  int goff[NS], loff[NS];
  const int nf = MX_TE * D;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int f = 128 * j + 2 * lane;
    const int r = f / D;
    goff[j] = f < nf ? 4 * f : OOB;
    loff[j] = f < nf ? r * MX_PF + (f - r * D) : MX_TE * MX_PF + 2 * (lane & 31);
  }
  const int64_t ntiles = (E + MX_TE - 1) / MX_TE;
  const int64_t stride = (int64_t)gridDim.x * MX_WAVES;
  int64_t tile = (int64_t)blockIdx.x * MX_WAVES + wave;
  u32x2 v[NS];
  {
    const rsrc_t r = mx_tile_rsrc(ea, tile, ntiles, E, D);
#pragma unroll
    for (int j = 0; j < NS; ++j) v[j] = bld2_u32(r, goff[j]);
  }
  for (; tile < ntiles; tile += stride) {
#pragma unroll
    for (int j = 0; j < NS; ++j) *reinterpret_cast<u32x2*>(img + loff[j]) = v[j];
    {
      const rsrc_t r = mx_tile_rsrc(ea, tile + stride, ntiles, E, D);  // next tile in flight
#pragma unroll
      for (int j = 0; j < NS; ++j) v[j] = bld2_u32(r, goff[j]);
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const float2 a = *reinterpret_cast<const float2*>(img + li * MX_PF + 8 * s + 2 * g);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, wb[s][0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, wb[s][1], acc, 0, 0, 0);
    }
    if (outp) {
      const int64_t e0 = tile * MX_TE + 4 * g;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (e0 + r < E) {
          SV2N_CHK(405, (e0 + r) * H + (li - (li / H) * H), E * H);
          outp[(e0 + r) * H] = acc[r];
        }
    }
  }
}

// DEPTH tiles in flight per wave (register sets used in rotation)
template <int NS, int DEPTH>
__global__ __launch_bounds__(256, 4) void k_edge_bwd_mx(const float* __restrict__ ea,
                                                                  int64_t E, int D,
                                                                  LayerCPtrs dae, int L, int H,
                                                                  int hlp,
                                                                  float* __restrict__ partial) {
  constexpr int NM = NS / 2, NP = NM / 2;  // M tiles of 16 d; float2 pieces per row
  __shared__ __attribute__((aligned(16))) float s_red[MX_WAVES * 8 * NS * 16];
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int li = lane & 15, g = lane >> 4;
  const int HL = L * H;
  const float* inp = li < HL ? mx_col_ptr<const float>(dae, li, L, H) : nullptr;
  const int64_t ntiles = (E + MX_TE - 1) / MX_TE;
  const int64_t stride = (int64_t)gridDim.x * MX_WAVES;
  f32x4 acc[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x2 v[DEPTH][4][NP];
  float b[DEPTH][4];
  // lane (li, g): row 4g + q, columns 32·mm + 2li (+1); the row / column step
  // goes in the wave-uniform soffset, the last piece past D reads nothing
  const int vo = ((4 * g) * D + 2 * li) * 4;
  const int vo_last = 32 * (NP - 1) + 2 * li < D ? vo : OOB;
  auto load = [&](u32x2 (&w)[4][NP], float (&bb)[4], int64_t t) __attribute__((always_inline)) {
    const rsrc_t r = mx_tile_rsrc(ea, t, ntiles, E, D);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int mm = 0; mm < NP; ++mm)
        w[q][mm] = __builtin_amdgcn_raw_buffer_load_b64(r, mm == NP - 1 ? vo_last : vo,
                                                        (q * D + 32 * mm) * 4, 0);
    // this lane's column for edges 4g + q of the tile (0 past E / past HL;
    // per-lane pointers, so plain masked global loads, not a descriptor)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t e = t * MX_TE + 4 * g + q;
      if (inp && e < E) SV2N_CHK(406, e * H, E * H);
      bb[q] = (inp && e < E) ? inp[e * H] : 0.f;
    }
  };
  int64_t tile = (int64_t)blockIdx.x * MX_WAVES + wave;
#pragma unroll
  for (int k = 0; k < DEPTH; ++k) load(v[k], b[k], tile + k * stride);
  for (; tile < ntiles; tile += DEPTH * stride) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      const int64_t t = tile + k * stride;
      if (t >= ntiles) break;  // wave-uniform
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mm = 0; mm < NP; ++mm) {
          acc[2 * mm] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(v[k][q][mm][0]),
                                                              b[k][q], acc[2 * mm], 0, 0, 0);
          acc[2 * mm + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(
              __uint_as_float(v[k][q][mm][1]), b[k][q], acc[2 * mm + 1], 0, 0, 0);
        }
      load(v[k], b[k], t + DEPTH * stride);  // the tile DEPTH ahead (or nothing)
    }
  }
  // wave partials -> LDS [wave][8NS][16], summed in wave order
#pragma unroll
  for (int m = 0; m < NM; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int d = 32 * (m >> 1) + 2 * (4 * g + r) + (m & 1);
      s_red[(wave * 8 * NS + d) * 16 + li] = acc[m][r];
    }
  __syncthreads();
  float* pb = partial + (int64_t)blockIdx.x * D * hlp;
  for (int o = threadIdx.x; o < D * hlp; o += 256) {
    const int d = o / hlp, k = o - d * hlp;
    float sm = 0.f;
    if (k < 16) {
      sm = s_red[d * 16 + k];
#pragma unroll
      for (int w = 1; w < MX_WAVES; ++w) sm += s_red[(w * 8 * NS + d) * 16 + k];
    }
    pb[o] = sm;
  }
}

// eid[t*n + j] = e for every non-self edge s->t, j = s - g*n (caller fills -1)
__global__ void k_block_eid(const int64_t* __restrict__ ei, int64_t E, int64_t N, int n,
                            int32_t* __restrict__ eid) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int64_t s = ei[e], t = ei[E + e];
  if (s == t || t < 0 || t >= N) return;
  const int64_t j = s - (t / n) * n;
  if (j < 0 || j >= n) return;
  eid[t * n + j] = (int32_t)e;
}

// ---------------------------------------------------------------------------
// Edge features in the reference's covariance layout (utils/dataset.py:
// 228-243, stacked over the window at :279-282): the row of edge s -> t is
//   [cov_t'(s,t) | var_t'(s) | var_t'(t)]  for t' < S  (D = 3S),
// with cov symmetric (both directions carry adj[min][max]) and var a node
// quantity (the volvol diagonal).  Canonical complete graphs only (upper pairs
// p = (u, v), u < v, row-major, source u -> target v; then the same pairs
// swapped at P + p).  Every logit is then
//   ae[u->v][c] = A[p][c] + Vs[u][c] + Vt[v][c],   ae[v->u][c] = A[p][c] + Vs[v][c] + Vt[u][c]
//   A[p][c] = Σ cov_t'(p)·W̃[t'][c],  Vs[u][c] = Σ var_t'(u)·W̃[S+t'][c],  Vt: W̃[2S+t'][c]
// so a graph's pass reads the covariance columns of its P upper rows and
// one variance series per node (from the rows of pairs (0, u)): ≈ 1/6 of
// its edge_attr bytes.  The backward is the transpose:
//   dW̃[t'][c]    = Σ_p cov_t'(p)·(dae[p][c] + dae[P+p][c])
//   dW̃[S+t'][c]  = Σ_u var_t'(u)·Σ_{source u} dae[e][c]
//   dW̃[2S+t'][c] = Σ_u var_t'(u)·Σ_{target u} dae[e][c]
// One 256-thread workgroup per graph (grid-stride); the backward accumulates
// its graphs' dW̃ in registers and leaves one partial slab per workgroup
// (k_reduce_partials sums them in order).  The caller vouches for the layout
// (spotv2net_amd.layout.mark_cov_var: the builders that write it).
// ---------------------------------------------------------------------------
constexpr int CV_T = 256, CV_MAXN = 32, CV_MAXS = 64, CV_MAXC = 16, CV_PCH = 64;
constexpr int CV_BWD_GRID = 1024;

// node u's variance series: the source columns of pair (0, 1) for u = 0, the
// target columns of pair (0, u) (upper row u - 1) otherwise
__device__ __forceinline__ const float* cv_var_row(const float* gea, int u, int S, int D) {
  return u == 0 ? gea + S : gea + (int64_t)(u - 1) * D + 2 * S;
}

__device__ __forceinline__ float* cv_col(const LayerPtrs& lp, int c, int H) {
  float* r = nullptr;
#pragma unroll
  for (int l = 0; l < SV2N_MAX_LAYERS; ++l)
    if (c >= l * H && c < (l + 1) * H) r = lp.p[l] + (c - l * H);
  return r;
}
__device__ __forceinline__ const float* cv_col(const LayerCPtrs& lp, int c, int H) {
  const float* r = nullptr;
#pragma unroll
  for (int l = 0; l < SV2N_MAX_LAYERS; ++l)
    if (c >= l * H && c < (l + 1) * H) r = lp.p[l] + (c - l * H);
  return r;
}

// global -> LDS staging with 8 loads in flight per thread (a runtime-bounded
// loop would wait on each load before issuing the next)
template <typename LOAD, typename STORE>
__device__ __forceinline__ void cv_stage(int total, int t, LOAD load, STORE store) {
  for (int k0 = t; k0 < total; k0 += 8 * CV_T) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u * CV_T;
      v[u] = k < total ? load(k) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u * CV_T;
      if (k < total) store(k, v[u]);
    }
  }
}

// rows x cols (cols <= 64) row by row: wave w takes rows w, w + 4, ..., lane =
// column (coalesced rows, no index division), 8 rows in flight per wave
template <typename LOAD, typename STORE>
__device__ __forceinline__ void cv_stage_rows(int rows, int cols, LOAD load, STORE store) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool lv = lane < cols;
  for (int r0 = w; r0 < rows; r0 += 4 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = r0 + 4 * u;
      v[u] = (lv && r < rows) ? load(r, lane) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = r0 + 4 * u;
      if (lv && r < rows) store(r, lane, v[u]);
    }
  }
}

// Forward: one workgroup per (graph, CV_FSUB·CV_PCH upper pairs), four
// threads per pair and CV_FSUB pairs per thread group.  A thread's covariance
// loads (t' = cq, cq + 4, ...) are issued first and land while W̃ and the node
// variances are staged and the node terms formed; the four partial dot
// products of a pair are summed across its lanes (xor 1, 2).  NC: logit
// columns rounded up to 4.
constexpr int CV_FSUB = 4;
template <int NC>
__global__ __launch_bounds__(CV_T) void k_edge_fwd_cv(const float* __restrict__ ea, int n, int S,
                                                      const uint16_t* __restrict__ canon,
                                                      const float* __restrict__ wf, int hlp,
                                                      LayerPtrs ae, int L, int H) {
  __shared__ __attribute__((aligned(16))) float sW[3 * CV_MAXS][NC];
  __shared__ float sVar[CV_MAXN][CV_MAXS + 1];
  __shared__ float sVs[CV_MAXN][NC], sVt[CV_MAXN][NC];
  const int t = threadIdx.x, D = 3 * S, HL = L * H, E0 = n * (n - 1), P = E0 / 2;
  constexpr int CH = CV_FSUB * CV_PCH;
  const int nch = (P + CH - 1) / CH;
  const int64_t g = blockIdx.x / nch;
  const int p0 = (int)(blockIdx.x - g * nch) * CH;
  const int pl = t >> 2, cq = t & 3;
  const float* gea = ea + g * E0 * D;
  float x[CV_FSUB][CV_MAXS / 4];
#pragma unroll
  for (int sb = 0; sb < CV_FSUB; ++sb) {
    const int p = p0 + sb * CV_PCH + pl;
#pragma unroll
    for (int k = 0; k < CV_MAXS / 4; ++k) {
      const int tt = cq + 4 * k;
      x[sb][k] = (p < P && tt < S) ? gea[(int64_t)p * D + tt] : 0.f;
    }
  }
  cv_stage(D * NC, t,
           [&](int k) {
             const int d = k / NC, c = k - d * NC;
             return c < HL ? wf[d * hlp + c] : 0.f;
           },
           [&](int k, float v) { (&sW[0][0])[k] = v; });
  cv_stage_rows(n, S, [&](int r, int c) { return cv_var_row(gea, r, S, D)[c]; },
                [&](int r, int c, float v) { sVar[r][c] = v; });
  __syncthreads();
  // node terms: four lanes per (node, column), each a quarter of the lags
  for (int k = t; k < 4 * n * NC; k += CV_T) {
    const int q = k & 3, uc = k >> 2, u = uc / NC, c = uc - u * NC;
    float vs = 0.f, vt = 0.f;
    for (int tt = q; tt < S; tt += 4) {
      vs = fmaf(sVar[u][tt], sW[S + tt][c], vs);
      vt = fmaf(sVar[u][tt], sW[2 * S + tt][c], vt);
    }
    vs += __shfl_xor(vs, 1, 64);
    vt += __shfl_xor(vt, 1, 64);
    vs += __shfl_xor(vs, 2, 64);
    vt += __shfl_xor(vt, 2, 64);
    if (q == 0) {
      sVs[u][c] = vs;
      sVt[u][c] = vt;
    }
  }
  __syncthreads();  // sVs / sVt
#pragma unroll
  for (int sb = 0; sb < CV_FSUB; ++sb) {
    const int p = p0 + sb * CV_PCH + pl;
    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.f;
#pragma unroll
    for (int k = 0; k < CV_MAXS / 4; ++k) {
      const int tt = cq + 4 * k;
      if (tt < S) {
#pragma unroll
        for (int c = 0; c < NC; c += 4) {
          const float4 w = *reinterpret_cast<const float4*>(&sW[tt][c]);
          acc[c] = fmaf(x[sb][k], w.x, acc[c]);
          acc[c + 1] = fmaf(x[sb][k], w.y, acc[c + 1]);
          acc[c + 2] = fmaf(x[sb][k], w.z, acc[c + 2]);
          acc[c + 3] = fmaf(x[sb][k], w.w, acc[c + 3]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      acc[c] += __shfl_xor(acc[c], 1, 64);
      acc[c] += __shfl_xor(acc[c], 2, 64);
    }
    if (p < P) {
      const int pr = canon[p];  // (target << 8) | source of upper edge p
      const int u = pr & 0xff, v = pr >> 8;
      const int64_t eu = g * E0 + p, el = g * E0 + P + p;
#pragma unroll
      for (int i = 0; i < NC / 4; ++i) {
        const int c = cq + 4 * i;
        float a = acc[4 * i];
#pragma unroll
        for (int j = 1; j < 4; ++j) a = (j == cq) ? acc[4 * i + j] : a;
        if (c < HL) {
          float* col = cv_col(ae, c, H);
          col[eu * H] = a + sVs[u][c] + sVt[v][c];
          col[el * H] = a + sVs[v][c] + sVt[u][c];
        }
      }
    }
  }
}

// Backward: units of (graph, chunk of CV_PCH upper pairs), grid-stride.  A
// unit stages its pairs' covariance columns, the graph's variance series and
// the pairs' two d-logit rows; NG = 256 / S thread groups take every NG-th
// pair, each thread one t' and every column in registers:
//   cov row t':  x·(d_up + d_low)
//   src row t':  var_u·d_up + var_v·d_low      (u -> v is the upper edge)
//   tgt row t':  var_v·d_up + var_u·d_low
// accumulated over the workgroup's units; at the end the groups are added in
// group order and the workgroup leaves one [D][hlp] slab (k_reduce_partials).
template <int NC>
__global__ __launch_bounds__(CV_T) void k_edge_bwd_cv(const float* __restrict__ ea, int64_t B,
                                                      int n, int S,
                                                      const uint16_t* __restrict__ canon,
                                                      LayerCPtrs dae, int L, int H, int hlp,
                                                      float* __restrict__ partial) {
  __shared__ float sCov[CV_PCH * (CV_MAXS + 1)];
  __shared__ float sVar[CV_MAXN][CV_MAXS + 1];
  __shared__ __attribute__((aligned(16))) float sDu[CV_PCH][NC];
  __shared__ __attribute__((aligned(16))) float sDl[CV_PCH][NC];
  __shared__ int sPr[CV_PCH];
  static_assert(CV_T * NC <= CV_PCH * (CV_MAXS + 1), "group reduction area");
  const int t = threadIdx.x, D = 3 * S, HL = L * H, E0 = n * (n - 1), P = E0 / 2;
  const int NG = CV_T / S;
  const int grp = t / S, tt = t - grp * S;
  const bool act = grp < NG;
  const int nch = (P + CV_PCH - 1) / CV_PCH;
  const int64_t U = B * nch;
  float ac[NC], as_[NC], at_[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) ac[c] = as_[c] = at_[c] = 0.f;
  for (int64_t un = blockIdx.x; un < U; un += gridDim.x) {
    const int64_t g = un / nch;
    const int p0 = (int)(un - g * nch) * CV_PCH, np = min(CV_PCH, P - p0);
    const float* gea = ea + g * E0 * D;
    __syncthreads();  // the previous unit's LDS reads
    cv_stage_rows(np, S, [&](int r, int c) { return gea[(int64_t)(p0 + r) * D + c]; },
                  [&](int r, int c, float v) { sCov[r * (S + 1) + c] = v; });
    cv_stage_rows(n, S, [&](int r, int c) { return cv_var_row(gea, r, S, D)[c]; },
                  [&](int r, int c, float v) { sVar[r][c] = v; });
    cv_stage(2 * CV_PCH * NC, t,
             [&](int k) {
               const int lo = k >= CV_PCH * NC, r = k - lo * CV_PCH * NC;
               const int pl = r / NC, c = r - pl * NC;
               return (pl < np && c < HL)
                          ? cv_col(dae, c, H)[(g * E0 + (lo ? P : 0) + p0 + pl) * H]
                          : 0.f;
             },
             [&](int k, float v) {
               const int lo = k >= CV_PCH * NC, r = k - lo * CV_PCH * NC;
               (lo ? &sDl[0][0] : &sDu[0][0])[r] = v;
             });
    if (t < np) sPr[t] = canon[p0 + t];
    __syncthreads();
    if (act) {
      for (int pp = grp; pp < np; pp += NG) {
        const float x = sCov[pp * (S + 1) + tt];
        const int pr = sPr[pp];
        const float vu = sVar[pr & 0xff][tt], vv = sVar[pr >> 8][tt];
#pragma unroll
        for (int c = 0; c < NC; c += 4) {
          const float4 du = *reinterpret_cast<const float4*>(&sDu[pp][c]);
          const float4 dl = *reinterpret_cast<const float4*>(&sDl[pp][c]);
          ac[c] = fmaf(x, du.x + dl.x, ac[c]);
          ac[c + 1] = fmaf(x, du.y + dl.y, ac[c + 1]);
          ac[c + 2] = fmaf(x, du.z + dl.z, ac[c + 2]);
          ac[c + 3] = fmaf(x, du.w + dl.w, ac[c + 3]);
          as_[c] = fmaf(vu, du.x, fmaf(vv, dl.x, as_[c]));
          as_[c + 1] = fmaf(vu, du.y, fmaf(vv, dl.y, as_[c + 1]));
          as_[c + 2] = fmaf(vu, du.z, fmaf(vv, dl.z, as_[c + 2]));
          as_[c + 3] = fmaf(vu, du.w, fmaf(vv, dl.w, as_[c + 3]));
          at_[c] = fmaf(vv, du.x, fmaf(vu, dl.x, at_[c]));
          at_[c + 1] = fmaf(vv, du.y, fmaf(vu, dl.y, at_[c + 1]));
          at_[c + 2] = fmaf(vv, du.z, fmaf(vu, dl.z, at_[c + 2]));
          at_[c + 3] = fmaf(vv, du.w, fmaf(vu, dl.w, at_[c + 3]));
        }
      }
    }
  }
  // the slab: for each block q (cov, src, tgt) the groups' rows in group order
  float* pb = partial + (int64_t)blockIdx.x * D * hlp;
  float* sRed = sCov;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    __syncthreads();
    if (act) {
#pragma unroll
      for (int c = 0; c < NC; ++c)
        sRed[(grp * S + tt) * NC + c] = q == 0 ? ac[c] : (q == 1 ? as_[c] : at_[c]);
    }
    __syncthreads();
    for (int k = t; k < S * hlp; k += CV_T) {
      const int r = k / hlp, c = k - r * hlp;
      float v = 0.f;
      if (c < HL)
        for (int gq = 0; gq < NG; ++gq) v += sRed[(gq * S + r) * NC + c];
      pb[(int64_t)(q * S + r) * hlp + c] = v;
    }
  }
}


// ---------------------------------------------------------------------------
// Round 5 (even S): both covariance-layout passes with ONE workgroup of 8
// waves per graph and the inner products on v_mfma_f32_16x16x4_f32 (exact f32
// products, f32 sums).  The graph's P upper rows go in tiles of 16 pairs, tile
// k on wave k % 8.  What the round-4 passes spent their time on (PMC,
// profiles/r05_cv_pmc.txt): the covariance columns loaded 4 lanes x 16 B per
// row (16 rows per load instruction), the variance series re-read by every
// 64-pair unit, and per-unit staging phases between barriers.
//
// forward: every wave issues the covariance loads of ALL its tiles up front
//   (flat float2 pieces of the tile's 16 x S block: 512 contiguous bytes over
//   ~3 rows per instruction; a graph's ~73 KB in flight), after the small
//   loads the workgroup needs first (variance series, the fold's node rows,
//   the pair table), so waiting for those never waits for the stream.  The
//   node terms Vs = var·W̃[S..2S), Vt = var·W̃[2S..3S) are formed while the
//   stream lands (four lanes per (node, column)).  Per tile the wave writes
//   its rows into a private LDS image (row stride 8·NJ + 4 floats: the 16 rows
//   of a half-wave's b64 reads start on distinct 4-bank groups) and runs
//   A[p][c] = Σ_t cov[p][t]·W̃[t][c] (MFMA step (s, c') pairs lane group g with
//   t = 8s + 2g + c'), then writes A + Vs[u] + Vt[v] and A + Vs[v] + Vt[u]
//   (lane (c, g) stores column c of pair 4g + r: 4·H-byte runs per pair and
//   layer; staging the tile through LDS into contiguous 16·H-float runs
//   measured slower, 24.4 vs 22.4 µs).
// backward: per tile the A operands come straight from HBM (M tile m holds
//   t = 32(m/2) + 2i + (m&1): lane (i, g) loads the pieces of two M tiles as
//   one float2, 4 rows x 128 contiguous bytes per instruction), B = d_up +
//   d_low of the tile's pairs, the next tile's loads in flight; the d-logits
//   also go into an LDS table of the graph, from which the per-node sums of
//   the outgoing / incoming edges' d-logits are added in a fixed order, then
//   dW̃[S + t] = Σ_u var_t(u)·Σ_out(u), dW̃[2S + t] = Σ_u var_t(u)·Σ_in(u).
//   One [D][hl_pad] partial per workgroup (fixed summation order throughout),
//   k_reduce_partials finishes.
// ---------------------------------------------------------------------------
constexpr int CV2_WAVES = 8, CV2_T = 64 * CV2_WAVES, CV2_TW = 4;  // tiles of 16 pairs per wave
constexpr int CV2_BWD_GRID = 512;
static_assert(CV2_WAVES * CV2_TW * 16 >= CV_MAXN * (CV_MAXN - 1) / 2, "tiles cover every pair");
static_assert(CV2_BWD_GRID <= CV_BWD_GRID, "workspace of sv2n_edge_logits_bwd_cv_workspace");

// (u, v), u < v, of upper pair p: (v << 8) | u in the pair table
__device__ __forceinline__ int cv2_pair_index(int a, int b, int n) {  // a < b
  return a * (2 * n - a - 1) / 2 + (b - a - 1);
}

template <int NJ, int NC>
__global__ __launch_bounds__(CV2_T) void k_edge_fwd_cv2(const float* __restrict__ ea, int n, int S,
                                                        const uint16_t* __restrict__ canon,
                                                        const float* __restrict__ wf, int hlp,
                                                        LayerPtrs ae, int L, int H) {
  constexpr int RS = 8 * NJ + 4;       // image row stride (floats)
  constexpr int IMG = 16 * RS + 128;   // + where the pieces past the tile land
  __shared__ __attribute__((aligned(16))) float s_img[CV2_WAVES][IMG];
  __shared__ float sVar[CV_MAXN][CV_MAXS + 1];
  __shared__ float sWn[2 * CV_MAXS][NC];  // the fold's source / target rows
  __shared__ float sV[2][CV_MAXN][NC];    // node terms (source, target)
  __shared__ int sPr[CV_MAXN * (CV_MAXN - 1) / 2];
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, gq = lane >> 4;
  const int D = 3 * S, HL = L * H, E0 = n * (n - 1), P = E0 / 2, TP = (P + 15) / 16;
  const int S2 = S >> 1;
  const int64_t g = blockIdx.x;
  const rsrc_t rg = make_rsrc(ea + g * E0 * D, (uint32_t)(E0 * D) * 4u);

  // 1) the loads the workgroup needs first: variance series (node u: the
  //    source columns of upper row 0 for u = 0, the target columns of upper
  //    row u - 1 otherwise), the fold's node rows, the pair table
  u32x2 vv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int k = t + CV2_T * i, u = k / S2, c2 = k - u * S2;
    const int off = u == 0 ? S + 2 * c2 : (u - 1) * D + 2 * S + 2 * c2;
    vv[i] = __builtin_amdgcn_raw_buffer_load_b64(rg, k < n * S2 ? 4 * off : OOB, 0, 0);
  }
  float wn[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = t + CV2_T * i, d = k / NC, c = k - d * NC;
    wn[i] = (k < 2 * S * NC && c < HL) ? wf[(S + d) * hlp + c] : 0.f;
  }
  const int pr = t < P ? (int)canon[t] : 0;
  float wb[NJ][2];  // B operands: W̃[t][li], t = 8s + 2g + c
#pragma unroll
  for (int s = 0; s < NJ; ++s)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int tt = 8 * s + 2 * gq + c;
      wb[s][c] = (tt < S && li < HL) ? wf[tt * hlp + li] : 0.f;
    }
  // 2) the covariance stream: flat float2 pieces f = 128j + 2·lane of each
  //    of the wave's tiles (16 rows x S floats)
  int loff[NJ];
  u32x2 v[CV2_TW][NJ];
  {
    int goff[NJ];
    const int nf = 16 * S;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int f = 128 * j + 2 * lane, r = f / S, c = f - r * S;
      goff[j] = f < nf ? 4 * (r * D + c) : OOB;
      loff[j] = f < nf ? r * RS + c : 16 * RS + 2 * lane;
    }
#pragma unroll
    for (int k = 0; k < CV2_TW; ++k) {
      const int tile = wave + CV2_WAVES * k;
      const bool ok = tile < TP;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        v[k][j] = __builtin_amdgcn_raw_buffer_load_b64(rg, ok ? goff[j] : OOB,
                                                        ok ? tile * 16 * D * 4 : 0, 0);
    }
  }
  float* img = s_img[wave];
  for (int k = lane; k < 16 * (8 * NJ - S); k += 64) {  // lags S .. 8·NJ of the image: 0
    const int r = k / (8 * NJ - S);
    img[r * RS + S + (k - r * (8 * NJ - S))] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int k = t + CV2_T * i, u = k / S2, c2 = k - u * S2;
    if (k < n * S2) {
      sVar[u][2 * c2] = __uint_as_float(vv[i][0]);
      sVar[u][2 * c2 + 1] = __uint_as_float(vv[i][1]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = t + CV2_T * i;
    if (k < 2 * S * NC) (&sWn[0][0])[k] = wn[i];
  }
  if (t < P) sPr[t] = pr;
  __syncthreads();
  // 3) node terms, four lanes per (node, column), lags q, q + 4, ...
  for (int k0 = 0; k0 < 4 * n * NC; k0 += CV2_T) {
    const int k = k0 + t;
    const int q = k & 3, uc = k >> 2, u = min(uc / NC, n - 1), c = uc - (uc / NC) * NC;
    float vs = 0.f, vt = 0.f;
    for (int tt = q; tt < S; tt += 4) {
      vs = fmaf(sVar[u][tt], sWn[tt][c], vs);
      vt = fmaf(sVar[u][tt], sWn[S + tt][c], vt);
    }
    vs += __shfl_xor(vs, 1, 64);
    vt += __shfl_xor(vt, 1, 64);
    vs += __shfl_xor(vs, 2, 64);
    vt += __shfl_xor(vt, 2, 64);
    if (q == 0 && uc < n * NC) {
      sV[0][u][c] = vs;
      sV[1][u][c] = vt;
    }
  }
  __syncthreads();
  // 4) per tile: LDS image, MFMA, node terms, both directions out
  float* outp = li < HL ? mx_col_ptr<float>(ae, li, L, H) : nullptr;
  const int64_t gE0 = g * E0;
#pragma unroll
  for (int k = 0; k < CV2_TW; ++k) {
    const int tile = wave + CV2_WAVES * k;
    if (tile >= TP) break;  // wave-uniform
#pragma unroll
    for (int j = 0; j < NJ; ++j) *reinterpret_cast<u32x2*>(img + loff[j]) = v[k][j];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NJ; ++s) {
      const float2 a = *reinterpret_cast<const float2*>(img + li * RS + 8 * s + 2 * gq);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, wb[s][0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, wb[s][1], acc, 0, 0, 0);
    }
    if (outp) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = tile * 16 + 4 * gq + r;
        if (p < P) {
          const int pp = sPr[p], u = pp & 0xff, w = pp >> 8;
          SV2N_CHK(407, (gE0 + P + p) * H, (int64_t)gridDim.x * E0 * H);
          SV2N_CHK(408, u * 32 + w, n * 32);
          outp[(gE0 + p) * H] = acc[r] + sV[0][u][li] + sV[1][w][li];
          outp[(gE0 + P + p) * H] = acc[r] + sV[0][w][li] + sV[1][u][li];
        }
      }
    }
  }
}

// SPLIT (at most 8 logit columns): the B operand's 16 columns carry d_up of
// column c in lane column c and d_low in lane column 8 + c, so one MFMA per
// M tile serves both directions and each lane loads one d-logit per pair
// (the halves are added at the end); otherwise B = d_up + d_low.  The
// d-logits also go into an LDS table of the graph; after the tiles the
// per-node sums over the outgoing / incoming edges are read from it in a
// fixed order through a [node][partner] index table built once.
template <int NP, int NC>
__global__ __launch_bounds__(CV2_T) __attribute__((amdgpu_waves_per_eu(4))) void k_edge_bwd_cv2(
    const float* __restrict__ ea, int64_t B, int n, int S, const uint16_t* __restrict__ canon,
    LayerCPtrs dae, int L, int H, int hlp, float* __restrict__ partial) {
  constexpr bool SPLIT = NC <= 8;
  constexpr int NM = 2 * NP;  // M tiles of 16 lags
  constexpr int PMAX = CV_MAXN * (CV_MAXN - 1) / 2;
  // the graph's d-logits [2 · PMAX + 1][NC] ([0, PMAX) up u -> v, [PMAX,
  // 2·PMAX) low v -> u, the last row zero); at the end the waves' lag
  // accumulators [wave][32·NP lags][16 columns]
  constexpr int SD = (2 * PMAX + 1) * NC, SR = CV2_WAVES * 32 * NP * 16;
  constexpr int ZROW = 2 * PMAX;
  __shared__ float sVar[CV_MAXN][CV_MAXS + 1];
  __shared__ float sBuf[SD > SR ? SD : SR];
  __shared__ float sDn[2][CV_MAXN][NC];     // per node: Σ over outgoing [0] / incoming [1] edges
  __shared__ float sVarRes[2 * CV_MAXS][NC];
  // sOut[u][w]: row of sD holding the d-logit of edge u -> w (ZROW for w = u);
  // the edge w -> u is the other half of the same pair: row ± PMAX
  __shared__ short sOut[CV_MAXN][CV_MAXN];
  float* sRed = sBuf;
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, gq = lane >> 4;
  const int D = 3 * S, HL = L * H, E0 = n * (n - 1), P = E0 / 2, TP = (P + 15) / 16;
  const int S2 = S >> 1;
  // SPLIT: lane column li reads column li & 7 of the up (li < 8) or low rows
  const int col = SPLIT ? (li & 7) : li, low = SPLIT ? (li >> 3) : 0;
  const float* inp = col < HL ? mx_col_ptr<const float>(dae, col, L, H) : nullptr;
  const float* col0 = mx_col_ptr<const float>(dae, 0, L, H);
  for (int k = t; k < n * n; k += CV2_T) {
    const int u = k / n, w = k - u * n;
    sOut[u][w] = (short)(u == w ? ZROW : u < w ? cv2_pair_index(u, w, n)
                                               : PMAX + cv2_pair_index(w, u, n));
  }
  if (t < NC) sBuf[ZROW * NC + t] = 0.f;
  f32x4 acc[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the variance-term outputs this thread owns: o = t + 512·i over [2][S][NC]
  constexpr int KV = (2 * CV_MAXS * NC + CV2_T - 1) / CV2_T;
  float av[KV];
#pragma unroll
  for (int i = 0; i < KV; ++i) av[i] = 0.f;
  // lane (li, g): row 4g + q of a tile, lags 32·mm + 2li (+1)
  const int vo = ((4 * gq) * D + 2 * li) * 4;
  constexpr int ND = SPLIT ? 1 : 2;  // d-logit loads per pair and lane

  for (int64_t g = blockIdx.x; g < B; g += gridDim.x) {
    const rsrc_t rg = make_rsrc(ea + g * E0 * D, (uint32_t)(E0 * D) * 4u);
    // this graph's d-logits, this column.  The column's array differs per
    // lane (layer col / H), so no buffer descriptor (those are wave-uniform):
    // a plain load, unconditional (a lane past the logits or the pairs reads
    // column 0's first d-logit and drops it), so the compiler's wait counts
    // stay exact — a conditional load here waited vmcnt(0) per tile
    const float* ib = (inp ? inp : col0) + g * E0 * H;
    u32x2 vv[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = t + CV2_T * i, u = k / S2, c2 = k - u * S2;
      const int off = u == 0 ? S + 2 * c2 : (u - 1) * D + 2 * S + 2 * c2;
      vv[i] = __builtin_amdgcn_raw_buffer_load_b64(rg, k < n * S2 ? 4 * off : OOB, 0, 0);
    }
    u32x2 pc[4][NP];
    float dd[4][ND];
    auto load = [&](int tile) __attribute__((always_inline)) {
      const bool ok = tile < TP;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int mm = 0; mm < NP; ++mm)
          pc[q][mm] = __builtin_amdgcn_raw_buffer_load_b64(
              rg, (ok && 32 * mm + 2 * li < S) ? vo : OOB,
              ok ? ((tile * 16 + q) * D + 32 * mm) * 4 : 0, 0);
        const int p = tile * 16 + 4 * gq + q;
        const bool pv = ok && p < P && inp;
        if (pv) SV2N_CHK(409, (g * E0 + P + p) * H, B * E0 * H);
#pragma unroll
        for (int s = 0; s < ND; ++s) {
          const float v = ib[pv ? ((low | s) ? P + p : p) * H : 0];
          dd[q][s] = pv ? v : 0.f;
        }
      }
    };
    __syncthreads();  // the previous graph's sVar / sBuf / sDn reads (first: sOut)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = t + CV2_T * i, u = k / S2, c2 = k - u * S2;
      if (k < n * S2) {
        sVar[u][2 * c2] = __uint_as_float(vv[i][0]);
        sVar[u][2 * c2 + 1] = __uint_as_float(vv[i][1]);
      }
    }
    load(wave);
#pragma unroll 1
    for (int k = 0; k < CV2_TW; ++k) {
      const int tile = wave + CV2_WAVES * k;
      if (tile >= TP) break;  // wave-uniform
      float x[4][ND];
      u32x2 a[4][NP];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int s = 0; s < ND; ++s) x[q][s] = dd[q][s];
#pragma unroll
        for (int mm = 0; mm < NP; ++mm) a[q][mm] = pc[q][mm];
      }
      load(tile + CV2_WAVES);  // the next tile in flight (nothing past TP)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int p = tile * 16 + 4 * gq + q;
        if (p < P && col < NC) {
#pragma unroll
          for (int s = 0; s < ND; ++s) sBuf[(((low | s) ? PMAX : 0) + p) * NC + col] = x[q][s];
        }
        const float b = SPLIT ? x[q][0] : x[q][0] + x[q][ND - 1];
#pragma unroll
        for (int mm = 0; mm < NP; ++mm) {
          acc[2 * mm] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[q][mm][0]), b,
                                                             acc[2 * mm], 0, 0, 0);
          acc[2 * mm + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[q][mm][1]), b,
                                                                 acc[2 * mm + 1], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // the d-logit table and sVar complete
    // per-node sums in a fixed order (partners w = 0 .. n-1; the self row is
    // the zero row): outgoing [0] reads row sOut[u][w], incoming [1] the
    // pair's other half
    for (int k = t; k < 2 * n * NC; k += CV2_T) {
      const int side = k / (n * NC), uc = k - side * n * NC, u = uc / NC, c = uc - u * NC;
      float sm = 0.f;
#pragma unroll 8
      for (int w = 0; w < n; ++w) {
        int r = sOut[u][w];
        if (side) r = r == ZROW ? ZROW : (r >= PMAX ? r - PMAX : r + PMAX);
        sm += sBuf[r * NC + c];
      }
      sDn[side][u][c] = sm;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < KV; ++i) {
      const int o = t + CV2_T * i;
      if (o < 2 * S * NC) {
        const int side = o / (S * NC), r = o - side * S * NC, tt = r / NC, c = r - tt * NC;
        float sm = av[i];
        for (int u = 0; u < n; ++u) sm = fmaf(sVar[u][tt], sDn[side][u][c], sm);
        av[i] = sm;
      }
    }
  }
  // the workgroup's partial: covariance rows from the waves' accumulators
  // (added in wave order), variance rows from the threads' sums
  __syncthreads();
#pragma unroll
  for (int m = 0; m < NM; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tt = 32 * (m >> 1) + 2 * (4 * gq + r) + (m & 1);
      sRed[(wave * 32 * NP + tt) * 16 + li] = acc[m][r];
    }
#pragma unroll
  for (int i = 0; i < KV; ++i) {
    const int o = t + CV2_T * i;
    if (o < 2 * S * NC) (&sVarRes[0][0])[o] = av[i];
  }
  __syncthreads();
  float* pb = partial + (int64_t)blockIdx.x * D * hlp;
  for (int o = t; o < D * hlp; o += CV2_T) {
    const int d = o / hlp, c = o - d * hlp;
    float v = 0.f;
    if (c < HL) {
      if (d < S) {
        v = sRed[d * 16 + c];
#pragma unroll
        for (int w = 1; w < CV2_WAVES; ++w) v += sRed[(w * 32 * NP + d) * 16 + c];
        if constexpr (SPLIT) {  // + the low half (lane columns 8 + c)
          float vl = sRed[d * 16 + 8 + c];
#pragma unroll
          for (int w = 1; w < CV2_WAVES; ++w) vl += sRed[(w * 32 * NP + d) * 16 + 8 + c];
          v += vl;
        }
      } else {
        v = sVarRes[d - S][c];
      }
    }
    pb[o] = v;
  }
}

}  // namespace sv2n

SV2N_CHK_EXPORT(edge)

// ============================ C-ABI ========================================
using namespace sv2n;

static constexpr int EDGE_BWD_GRID = 768;
static constexpr int EDGE_FWD_GRID = 1024;
// persistent workgroup counts (MI355X sweeps: 512-6960 forward, 256-768
// backward within noise of these; the backward's bounds its workspace)
static constexpr int EDGE_SMALL_FWD_GRID = 4096;
static constexpr int EDGE_SMALL_BWD_GRID = 1024;
// MFMA streaming kernels (k_edge_fwd_mx / k_edge_bwd_mx): 4 workgroups of 4
// waves per CU (~36 KB LDS each)
static constexpr int EDGE_MX_GRID = 1024;

// canonical edge order (no edge_index, no planes), even D up to 128 (float2
// pieces never straddle a row), at most 16 logit columns (one MFMA N tile)
static bool edge_mx_ok(bool planes, const int64_t* edge_index, int edge_dim, int hl) {
  return !planes && !edge_index && edge_dim > EDGE_SMALL_D && (edge_dim & 1) == 0 &&
         edge_dim <= 128 && hl <= 16;
}

#define SV2N_SMALL_DISPATCH(KERNEL, GRID, ...)                                              \
  {                                                                                         \
    const int ds = (edge_dim + 3) & ~3;                                                     \
    switch (ds * 100 + hl_pad) {                                                            \
      case 404: hipLaunchKernelGGL((KERNEL<4, 4, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;   \
      case 408: hipLaunchKernelGGL((KERNEL<4, 8, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;   \
      case 416: hipLaunchKernelGGL((KERNEL<4, 16, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;  \
      case 432: hipLaunchKernelGGL((KERNEL<4, 32, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;  \
      case 804: hipLaunchKernelGGL((KERNEL<8, 4, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;   \
      case 808: hipLaunchKernelGGL((KERNEL<8, 8, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;   \
      case 816: hipLaunchKernelGGL((KERNEL<8, 16, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;  \
      case 832: hipLaunchKernelGGL((KERNEL<8, 32, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;  \
      case 1204: hipLaunchKernelGGL((KERNEL<12, 4, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break; \
      case 1208: hipLaunchKernelGGL((KERNEL<12, 8, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break; \
      case 1216: hipLaunchKernelGGL((KERNEL<12, 16, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;\
      case 1232: hipLaunchKernelGGL((KERNEL<12, 32, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;\
      case 1604: hipLaunchKernelGGL((KERNEL<16, 4, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break; \
      case 1608: hipLaunchKernelGGL((KERNEL<16, 8, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break; \
      case 1616: hipLaunchKernelGGL((KERNEL<16, 16, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;\
      case 1632: hipLaunchKernelGGL((KERNEL<16, 32, PL>), GRID, dim3(256), 0, stream, __VA_ARGS__); break;\
      default: return SV2N_ERR_SHAPE;                                                       \
    }                                                                                       \
  }

template <bool PL>
static int edge_fwd_small(const float* edge_attr, int64_t num_edges, int edge_dim,
                          const int64_t* edge_index, const uint16_t* canon, int E0,
                          const float* wfold, int hl_pad, const LayerPtrs& lp, int num_layers,
                          int heads, int64_t num_graphs, int n, hipStream_t stream) {
  const int64_t blocks = (num_edges + 255) / 256;
  const dim3 grid((unsigned)std::min<int64_t>(blocks, EDGE_SMALL_FWD_GRID));
  ColPtrs col{};
  for (int k = 0; k < num_layers * heads; ++k)
    col.p[k] = lp.p[k / heads] + (PL ? (int64_t)(k % heads) * num_edges : (int64_t)(k % heads));
  SV2N_SMALL_DISPATCH(k_edge_fwd_small, grid, edge_attr, num_edges, edge_dim, edge_index, canon,
                      E0, wfold, col, num_layers, heads, num_graphs, n)
  return (int)hipGetLastError();
}

template <bool PL>
static int edge_bwd_small(const float* edge_attr, int64_t num_edges, int edge_dim,
                          const int64_t* edge_index, const uint16_t* canon, int E0,
                          const LayerCPtrs& lp, int num_layers, int heads, int64_t num_graphs,
                          int n, float* workspace, int64_t workspace_floats, float* dwfold,
                          int hl_pad, hipStream_t stream) {
  const int O = edge_dim * hl_pad;
  if (PL && !edge_index && (num_edges & 3) == 0) {  // MFMA path (planes 16-B aligned)
    const int64_t blocks = (num_edges + 255) / 256;
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, EDGE_SMALL_BWD_GRID));
    if (workspace_floats < (int64_t)nb * O) return SV2N_ERR_WORKSPACE;
    ColCPtrs col{};
    for (int k = 0; k < num_layers * heads; ++k)
      col.p[k] = lp.p[k / heads] + (int64_t)(k % heads) * num_edges;
    const int HL = num_layers * heads;
    switch (hl_pad) {
      case 4: hipLaunchKernelGGL(k_edge_bwd_mfma<4>, dim3(nb), dim3(256), 0, stream, edge_attr, num_edges, edge_dim, col, HL, workspace); break;
      case 8: hipLaunchKernelGGL(k_edge_bwd_mfma<8>, dim3(nb), dim3(256), 0, stream, edge_attr, num_edges, edge_dim, col, HL, workspace); break;
      case 16: hipLaunchKernelGGL(k_edge_bwd_mfma<16>, dim3(nb), dim3(256), 0, stream, edge_attr, num_edges, edge_dim, col, HL, workspace); break;
      case 32: hipLaunchKernelGGL(k_edge_bwd_mfma<32>, dim3(nb), dim3(256), 0, stream, edge_attr, num_edges, edge_dim, col, HL, workspace); break;
      default: return SV2N_ERR_SHAPE;
    }
    hipLaunchKernelGGL(k_reduce_partials, dim3((O + 15) / 16), dim3(256), 0, stream, workspace,
                       nb, O, dwfold);
    return (int)hipGetLastError();
  }
  const int64_t blocks = (num_edges + 63) / 64;
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, EDGE_SMALL_BWD_GRID));
  if (workspace_floats < (int64_t)nb * O) return SV2N_ERR_WORKSPACE;
  ColCPtrs col{};
  for (int k = 0; k < num_layers * heads; ++k)
    col.p[k] = lp.p[k / heads] + (PL ? (int64_t)(k % heads) * num_edges : (int64_t)(k % heads));
  SV2N_SMALL_DISPATCH(k_edge_bwd_small, dim3(nb), edge_attr, num_edges, edge_dim, edge_index,
                      canon, E0, col, num_layers, heads, num_graphs, n, workspace)
  hipLaunchKernelGGL(k_reduce_partials, dim3((O + 15) / 16), dim3(256), 0, stream, workspace,
                     nb, O, dwfold);
  return (int)hipGetLastError();
}

// the dynamic LDS a launch asks for (not 160 KiB: the kernels also hold a
// little static LDS, and a limit whose sum with it exceeds the CU's 160 KiB is
// refused, leaving the 64 KiB default in place)
template <typename K>
static void raise_lds_limit(K kernel, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
}

static int edge_fwd_impl(const float* edge_attr, int64_t num_edges, int edge_dim,
                         const int64_t* edge_index, const uint16_t* canon, const float* wfold,
                         int hl_pad, float* const* ae_layers, int num_layers, int heads,
                         int64_t num_graphs, int n, bool planes, hipStream_t stream) {
  if (!edge_attr || !wfold || !ae_layers || num_edges < 0 || edge_dim <= 0 || num_graphs <= 0)
    return SV2N_ERR_ARG;
  if (num_edges == 0) return 0;  // nothing to project (e.g. single-node graphs)
  if (!planes && !edge_index && !canon) return SV2N_ERR_ARG;
  if (n < 1 || n > SV2N_MAX_N_TILED || heads < 1 || heads > SV2N_MAX_HEADS || num_layers < 1 ||
      num_layers > SV2N_MAX_LAYERS || num_layers * heads > hl_pad)
    return SV2N_ERR_SHAPE;
  if (((uintptr_t)edge_attr & 15) || ((uintptr_t)wfold & 15)) return SV2N_ERR_ALIGN;
  if (num_edges == 0) return 0;
  LayerPtrs lp{};
  for (int l = 0; l < num_layers; ++l) {
    if (!ae_layers[l]) return SV2N_ERR_ARG;
    lp.p[l] = ae_layers[l];
  }
  const int E0 = n * (n - 1);
  if (edge_dim <= EDGE_SMALL_D)
    return planes ? edge_fwd_small<true>(edge_attr, num_edges, edge_dim, edge_index, canon, E0,
                                         wfold, hl_pad, lp, num_layers, heads, num_graphs, n,
                                         stream)
                  : edge_fwd_small<false>(edge_attr, num_edges, edge_dim, edge_index, canon, E0,
                                          wfold, hl_pad, lp, num_layers, heads, num_graphs, n,
                                          stream);
  if (edge_mx_ok(planes, edge_index, edge_dim, num_layers * heads)) {
    const int64_t waves = (num_edges + MX_TE - 1) / MX_TE;
    const dim3 grid((unsigned)std::min<int64_t>((waves + MX_WAVES - 1) / MX_WAVES, EDGE_MX_GRID));
#define SV2N_MXF(NS)                                                                          \
  hipLaunchKernelGGL((k_edge_fwd_mx<NS>), grid, dim3(256), 0, stream, edge_attr, num_edges,    \
                     edge_dim, wfold, hl_pad, lp, num_layers, heads);
    switch ((edge_dim + 31) / 32) {
      case 1: SV2N_MXF(4) break;
      case 2: SV2N_MXF(8) break;
      case 3: SV2N_MXF(12) break;
      default: SV2N_MXF(16) break;
    }
#undef SV2N_MXF
    return (int)hipGetLastError();
  }
  const int64_t nchunks = (num_edges + EDGE_CHUNK - 1) / EDGE_CHUNK;
  constexpr int fwd_grid = EDGE_FWD_GRID;
  const unsigned grid = (unsigned)std::min<int64_t>(nchunks, fwd_grid);
  const int rf = (EDGE_CHUNK * edge_dim / 4 + EDGE_THREADS - 1) / EDGE_THREADS;
  if (rf > EDGE_RF_MAX) return SV2N_ERR_SHAPE;
  const int rfi = rf <= 2 ? 2 : rf <= 8 ? 8 : rf <= 16 ? 16 : 24;  // instantiated RF
  const size_t lds = sizeof(float) * ((size_t)edge_dim * hl_pad + (size_t)rfi * EDGE_THREADS * 4 +
                                      (size_t)EDGE_CHUNK * hl_pad);
  if (lds > 159 * 1024) return SV2N_ERR_SHAPE;  // room for the static LDS
#define SV2N_LAUNCH_EF2(HLP, RF, PL)                                                              \
  {                                                                                               \
    raise_lds_limit(k_edge_fwd<HLP, RF, PL>, lds);                                                \
    hipLaunchKernelGGL((k_edge_fwd<HLP, RF, PL>), dim3(grid), dim3(EDGE_THREADS), lds, stream,    \
                       edge_attr, num_edges, edge_dim, edge_index, canon, E0, wfold, lp,          \
                       num_layers, heads, num_graphs, n);                                         \
  }
#define SV2N_LAUNCH_EF(HLP, RF)                                  \
  {                                                              \
    if (planes) SV2N_LAUNCH_EF2(HLP, RF, true)                   \
    else SV2N_LAUNCH_EF2(HLP, RF, false)                         \
  }
#define SV2N_LAUNCH_EF_RF(HLP)                                   \
  case HLP:                                                      \
    if (rf <= 2) SV2N_LAUNCH_EF(HLP, 2)                          \
    else if (rf <= 8) SV2N_LAUNCH_EF(HLP, 8)                     \
    else if (rf <= 16) SV2N_LAUNCH_EF(HLP, 16)                   \
    else SV2N_LAUNCH_EF(HLP, 24)                                 \
    break;
  switch (hl_pad) {
    SV2N_LAUNCH_EF_RF(4)
    SV2N_LAUNCH_EF_RF(8)
    SV2N_LAUNCH_EF_RF(16)
    SV2N_LAUNCH_EF_RF(32)
    default:
      return SV2N_ERR_SHAPE;
  }
#undef SV2N_LAUNCH_EF_RF
#undef SV2N_LAUNCH_EF
#undef SV2N_LAUNCH_EF2
  return (int)hipGetLastError();
}

extern "C" int64_t sv2n_edge_logits_bwd_workspace(int edge_dim, int hl_pad) {
  return (int64_t)std::max(EDGE_MX_GRID, edge_dim <= EDGE_SMALL_D ? EDGE_SMALL_BWD_GRID
                                                                    : EDGE_BWD_GRID) *
         edge_dim * hl_pad;
}

static int edge_bwd_impl(const float* edge_attr, int64_t num_edges, int edge_dim,
                         const int64_t* edge_index, const uint16_t* canon,
                         const float* const* dae_layers, int num_layers, int heads,
                         int64_t num_graphs, int n, float* workspace, int64_t workspace_floats,
                         float* dwfold, int hl_pad, bool planes, hipStream_t stream) {
  if (!edge_attr || !dae_layers || !dwfold || !workspace || num_edges < 0 || edge_dim <= 0 ||
      num_graphs <= 0)
    return SV2N_ERR_ARG;
  if (!planes && !edge_index && !canon) return SV2N_ERR_ARG;
  if (n < 1 || n > SV2N_MAX_N_TILED || heads < 1 || heads > SV2N_MAX_HEADS || num_layers < 1 ||
      num_layers > SV2N_MAX_LAYERS || num_layers * heads > hl_pad)
    return SV2N_ERR_SHAPE;
  if ((uintptr_t)edge_attr & 15) return SV2N_ERR_ALIGN;
  const int DP = (edge_dim + 3) & ~3;
  const int tiles = (DP / 4) * (hl_pad / 4);  // 4x4 thread tiles of the [D][hl_pad] gradient
  if (tiles > 3 * EDGE_THREADS) return SV2N_ERR_SHAPE;
  const int nt = (tiles + EDGE_THREADS - 1) / EDGE_THREADS;
  LayerCPtrs lp{};
  for (int l = 0; l < num_layers; ++l) {
    if (!dae_layers[l]) return SV2N_ERR_ARG;
    lp.p[l] = dae_layers[l];
  }
  const int O = edge_dim * hl_pad;
  const int E0 = n * (n - 1);
  if (num_edges > 0 && edge_dim <= EDGE_SMALL_D)
    return planes ? edge_bwd_small<true>(edge_attr, num_edges, edge_dim, edge_index, canon, E0,
                                         lp, num_layers, heads, num_graphs, n, workspace,
                                         workspace_floats, dwfold, hl_pad, stream)
                  : edge_bwd_small<false>(edge_attr, num_edges, edge_dim, edge_index, canon, E0,
                                          lp, num_layers, heads, num_graphs, n, workspace,
                                          workspace_floats, dwfold, hl_pad, stream);
  if (num_edges > 0 && edge_mx_ok(planes, edge_index, edge_dim, num_layers * heads)) {
    const int64_t waves = (num_edges + MX_TE - 1) / MX_TE;
    const int grid = (int)std::min<int64_t>((waves + MX_WAVES - 1) / MX_WAVES, EDGE_MX_GRID);
    if (workspace_floats < (int64_t)grid * O) return SV2N_ERR_WORKSPACE;
    switch ((edge_dim + 31) / 32) {
      case 1: hipLaunchKernelGGL((k_edge_bwd_mx<4, MX_DEPTH>), dim3(grid), dim3(256), 0, stream, edge_attr, num_edges, edge_dim, lp, num_layers, heads, hl_pad, workspace); break;
      case 2: hipLaunchKernelGGL((k_edge_bwd_mx<8, MX_DEPTH>), dim3(grid), dim3(256), 0, stream, edge_attr, num_edges, edge_dim, lp, num_layers, heads, hl_pad, workspace); break;
      case 3: hipLaunchKernelGGL((k_edge_bwd_mx<12, MX_DEPTH>), dim3(grid), dim3(256), 0, stream, edge_attr, num_edges, edge_dim, lp, num_layers, heads, hl_pad, workspace); break;
      default: hipLaunchKernelGGL((k_edge_bwd_mx<16, MX_DEPTH>), dim3(grid), dim3(256), 0, stream, edge_attr, num_edges, edge_dim, lp, num_layers, heads, hl_pad, workspace); break;
    }
    hipLaunchKernelGGL(k_reduce_partials, dim3((O + 15) / 16), dim3(256), 0, stream, workspace,
                       grid, O, dwfold);
    return (int)hipGetLastError();
  }
  const int64_t nchunks = (num_edges + EDGE_CHUNK - 1) / EDGE_CHUNK;
  constexpr int bwd_grid = EDGE_BWD_GRID;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(bwd_grid, nchunks));
  if (workspace_floats < (int64_t)grid * O) return SV2N_ERR_WORKSPACE;
  const int rf = (EDGE_CHUNK * edge_dim / 4 + EDGE_THREADS - 1) / EDGE_THREADS;
  if (rf > EDGE_RF_MAX) return SV2N_ERR_SHAPE;
  const int rfi = rf <= 2 ? 2 : rf <= 8 ? 8 : rf <= 16 ? 16 : 24;  // instantiated RF
  const size_t ea_floats = std::max((size_t)EDGE_CHUNK * DP, (size_t)rfi * EDGE_THREADS * 4);
  size_t lds = sizeof(float) * (ea_floats + (size_t)EDGE_CHUNK * hl_pad);
  lds = std::max(lds, sizeof(float) * (size_t)std::max(EDGE_THREADS, tiles) * 16);
  if (lds > 159 * 1024) return SV2N_ERR_SHAPE;  // room for the static LDS
  if (num_edges == 0) return (int)hipMemsetAsync(dwfold, 0, sizeof(float) * O, stream);
#define SV2N_LAUNCH_EB3(HLP, RF, PL, NT)                                                          \
  {                                                                                               \
    raise_lds_limit(k_edge_bwd<HLP, RF, PL, NT>, lds);                                            \
    hipLaunchKernelGGL((k_edge_bwd<HLP, RF, PL, NT>), dim3(grid), dim3(EDGE_THREADS), lds,        \
                       stream, edge_attr, num_edges, edge_dim, DP, edge_index, canon, E0, lp,     \
                       num_layers, heads, num_graphs, n, workspace);                              \
  }
#define SV2N_LAUNCH_EB2(HLP, RF, PL)                                                              \
  {                                                                                               \
    if (nt == 1) SV2N_LAUNCH_EB3(HLP, RF, PL, 1)                                                  \
    else if constexpr (HLP >= 16 && RF >= 16) { /* tiles > 256 need DP > 4096 / HLP */           \
      if (nt == 2) SV2N_LAUNCH_EB3(HLP, RF, PL, 2)                                                \
      else SV2N_LAUNCH_EB3(HLP, RF, PL, 3)                                                        \
    } else return SV2N_ERR_SHAPE;                                                                 \
  }
#define SV2N_LAUNCH_EB(HLP, RF)                                  \
  {                                                              \
    if (planes) SV2N_LAUNCH_EB2(HLP, RF, true)                   \
    else SV2N_LAUNCH_EB2(HLP, RF, false)                         \
  }
#define SV2N_LAUNCH_EB_RF(HLP)                                   \
  case HLP:                                                      \
    if (rf <= 2) SV2N_LAUNCH_EB(HLP, 2)                          \
    else if (rf <= 8) SV2N_LAUNCH_EB(HLP, 8)                     \
    else if (rf <= 16) SV2N_LAUNCH_EB(HLP, 16)                   \
    else SV2N_LAUNCH_EB(HLP, 24)                                 \
    break;
  switch (hl_pad) {
    SV2N_LAUNCH_EB_RF(4)
    SV2N_LAUNCH_EB_RF(8)
    SV2N_LAUNCH_EB_RF(16)
    SV2N_LAUNCH_EB_RF(32)
    default:
      return SV2N_ERR_SHAPE;
  }
#undef SV2N_LAUNCH_EB_RF
#undef SV2N_LAUNCH_EB
#undef SV2N_LAUNCH_EB2
#undef SV2N_LAUNCH_EB3
  hipLaunchKernelGGL(k_reduce_partials, dim3((O + 15) / 16), dim3(256), 0, stream, workspace,
                     grid, O, dwfold);
  return (int)hipGetLastError();
}

extern "C" int sv2n_edge_logits_fwd(const float* edge_attr, int64_t num_edges, int edge_dim,
                                    const int64_t* edge_index, const uint16_t* canon,
                                    const float* wfold, int hl_pad, float* const* ae_layers,
                                    int num_layers, int heads, int64_t num_graphs, int n,
                                    hipStream_t stream) {
  return edge_fwd_impl(edge_attr, num_edges, edge_dim, edge_index, canon, wfold, hl_pad,
                       ae_layers, num_layers, heads, num_graphs, n, false, stream);
}

extern "C" int sv2n_edge_logits_bwd(const float* edge_attr, int64_t num_edges, int edge_dim,
                                    const int64_t* edge_index, const uint16_t* canon,
                                    const float* const* dae_layers, int num_layers, int heads,
                                    int64_t num_graphs, int n, float* workspace,
                                    int64_t workspace_floats, float* dwfold, int hl_pad,
                                    hipStream_t stream) {
  return edge_bwd_impl(edge_attr, num_edges, edge_dim, edge_index, canon, dae_layers,
                       num_layers, heads, num_graphs, n, workspace, workspace_floats, dwfold,
                       hl_pad, false, stream);
}

extern "C" int sv2n_edge_partials_reduce(const float* partial, int64_t num_parts, int64_t width,
                                         float* out, hipStream_t stream) {
  if (!partial || !out || num_parts <= 0 || width <= 0) return SV2N_ERR_ARG;
  if (num_parts * width * 4 > 0x7fffffff) return SV2N_ERR_SHAPE;
  hipLaunchKernelGGL(k_reduce_partials, dim3((unsigned)((width + 15) / 16)), dim3(256), 0, stream,
                     partial, (int)num_parts, (int)width, out);
  return (int)hipGetLastError();
}

extern "C" int sv2n_edge_logits_fwd_planes(const float* edge_attr, int64_t num_edges,
                                           int edge_dim, const float* wfold, int hl_pad,
                                           float* const* ae_layers, int num_layers, int heads,
                                           hipStream_t stream) {
  return edge_fwd_impl(edge_attr, num_edges, edge_dim, nullptr, nullptr, wfold, hl_pad,
                       ae_layers, num_layers, heads, 1, 1, true, stream);
}

extern "C" int sv2n_edge_logits_bwd_planes(const float* edge_attr, int64_t num_edges,
                                           int edge_dim, const int64_t* edge_index,
                                           const float* const* dae_layers, int num_layers,
                                           int heads, float* workspace,
                                           int64_t workspace_floats, float* dwfold, int hl_pad,
                                           hipStream_t stream) {
  return edge_bwd_impl(edge_attr, num_edges, edge_dim, edge_index, nullptr, dae_layers,
                       num_layers, heads, 1, 1, workspace, workspace_floats, dwfold, hl_pad, true,
                       stream);
}

extern "C" int sv2n_block_eid(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes,
                              int n, int32_t* eid, hipStream_t stream) {
  if (!edge_index || !eid || num_edges < 0 || num_nodes <= 0) return SV2N_ERR_ARG;
  if (n < 1 || n > SV2N_MAX_N_TILED || num_edges > 0x7fffffff) return SV2N_ERR_SHAPE;
  if (num_edges == 0) return 0;
  hipLaunchKernelGGL(k_block_eid, dim3((unsigned)((num_edges + 255) / 256)), dim3(256), 0,
                     stream, edge_index, num_edges, num_nodes, n, eid);
  return (int)hipGetLastError();
}

extern "C" int sv2n_block_rowmask(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes,
                                  int n, uint32_t* rowmask, hipStream_t stream) {
  if (!edge_index || !rowmask || num_edges < 0 || num_nodes <= 0) return SV2N_ERR_ARG;
  if (n < 1 || n > SV2N_MAX_N_TILED) return SV2N_ERR_SHAPE;
  if (num_edges == 0) return 0;
  hipLaunchKernelGGL(k_block_rowmask, dim3((unsigned)((num_edges + 255) / 256)), dim3(256), 0,
                     stream, edge_index, num_edges, num_nodes, n, rowmask);
  return (int)hipGetLastError();
}

extern "C" int sv2n_block_rowmask_checked(const int64_t* edge_index, int64_t num_edges,
                                          int64_t num_nodes, int n, uint32_t* rowmask,
                                          int32_t* violations, hipStream_t stream) {
  if (!edge_index || !rowmask || !violations || num_edges < 0 || num_nodes <= 0)
    return SV2N_ERR_ARG;
  if (n < 1 || n > SV2N_MAX_N_TILED) return SV2N_ERR_SHAPE;
  if (num_edges == 0) return 0;
  hipLaunchKernelGGL(k_block_rowmask_checked, dim3((unsigned)((num_edges + 255) / 256)),
                     dim3(256), 0, stream, edge_index, num_edges, num_nodes, n, rowmask,
                     violations);
  return (int)hipGetLastError();
}

// ---- covariance-layout edge features (k_edge_fwd_cv2 / k_edge_bwd_cv2; odd
// seq_length: k_edge_fwd_cv / k_edge_bwd_cv) ----
// SV2N_CV_ROUND4=1: the round-4 kernels for every seq_length (A/B switch)
static bool cv_round4() {
  static const bool v = [] {
    const char* e = std::getenv("SV2N_CV_ROUND4");
    return e && e[0] == '1';
  }();
  return v;
}
static int cv_check(const float* ea, int64_t B, int n, int S, const uint16_t* canon, int L,
                    int H, int hlp) {
  if (!ea || !canon || B < 0 || L < 1 || L > SV2N_MAX_LAYERS || H < 1) return SV2N_ERR_ARG;
  if (n < 2 || n > CV_MAXN || S < 1 || S > CV_MAXS || L * H > CV_MAXC || hlp < L * H)
    return SV2N_ERR_SHAPE;
  return 0;
}

extern "C" int sv2n_edge_logits_fwd_cv(const float* edge_attr, int64_t num_graphs, int n,
                                       int seq_length, const uint16_t* canon, const float* wfold,
                                       int hl_pad, float* const* ae_layers, int num_layers,
                                       int heads, hipStream_t stream) {
  if (int rc = cv_check(edge_attr, num_graphs, n, seq_length, canon, num_layers, heads, hl_pad))
    return rc;
  if (!wfold || !ae_layers) return SV2N_ERR_ARG;
  if (num_graphs == 0) return 0;
  LayerPtrs lp{};
  for (int l = 0; l < num_layers; ++l) {
    if (!ae_layers[l]) return SV2N_ERR_ARG;
    lp.p[l] = ae_layers[l];
  }
  if ((seq_length & 1) == 0 && !cv_round4()) {
    // round 5: one workgroup per graph, MFMA (even seq_length)
    if (num_graphs > 0x7fffffff) return SV2N_ERR_SHAPE;
    const int nj = seq_length <= 16 ? 2 : seq_length <= 32 ? 4 : seq_length <= 48 ? 6 : 8;
    const int nc = (num_layers * heads + 3) / 4;
#define SV2N_CVF2(NJ, NC)                                                                        \
  hipLaunchKernelGGL((k_edge_fwd_cv2<NJ, NC>), dim3((unsigned)num_graphs), dim3(CV2_T), 0, stream, \
                     edge_attr, n, seq_length, canon, wfold, hl_pad, lp, num_layers, heads)
#define SV2N_CVF2_NC(NJ)                                         \
  switch (nc) {                                                  \
    case 1: SV2N_CVF2(NJ, 4); break;                             \
    case 2: SV2N_CVF2(NJ, 8); break;                             \
    case 3: SV2N_CVF2(NJ, 12); break;                            \
    default: SV2N_CVF2(NJ, 16); break;                           \
  }
    switch (nj) {
      case 2: SV2N_CVF2_NC(2) break;
      case 4: SV2N_CVF2_NC(4) break;
      case 6: SV2N_CVF2_NC(6) break;
      default: SV2N_CVF2_NC(8) break;
    }
#undef SV2N_CVF2_NC
#undef SV2N_CVF2
    return (int)hipGetLastError();
  }
  const int64_t P = (int64_t)n * (n - 1) / 2, nch = (P + CV_FSUB * CV_PCH - 1) / (CV_FSUB * CV_PCH);
  if (num_graphs * nch > 0x7fffffff) return SV2N_ERR_SHAPE;
  const dim3 grid((unsigned)(num_graphs * nch));
  switch ((num_layers * heads + 3) / 4) {
    case 1: hipLaunchKernelGGL(k_edge_fwd_cv<4>, grid, dim3(CV_T), 0, stream, edge_attr, n,
                               seq_length, canon, wfold, hl_pad, lp, num_layers, heads); break;
    case 2: hipLaunchKernelGGL(k_edge_fwd_cv<8>, grid, dim3(CV_T), 0, stream, edge_attr, n,
                               seq_length, canon, wfold, hl_pad, lp, num_layers, heads); break;
    case 3: hipLaunchKernelGGL(k_edge_fwd_cv<12>, grid, dim3(CV_T), 0, stream, edge_attr, n,
                               seq_length, canon, wfold, hl_pad, lp, num_layers, heads); break;
    default: hipLaunchKernelGGL(k_edge_fwd_cv<16>, grid, dim3(CV_T), 0, stream, edge_attr, n,
                                seq_length, canon, wfold, hl_pad, lp, num_layers, heads); break;
  }
  return (int)hipGetLastError();
}

extern "C" int64_t sv2n_edge_logits_bwd_cv_workspace(int seq_length, int hl_pad) {
  return (int64_t)CV_BWD_GRID * 3 * seq_length * hl_pad;
}

extern "C" int sv2n_edge_logits_bwd_cv(const float* edge_attr, int64_t num_graphs, int n,
                                       int seq_length, const uint16_t* canon,
                                       const float* const* dae_layers, int num_layers, int heads,
                                       float* workspace, int64_t workspace_floats, float* dwfold,
                                       int hl_pad, hipStream_t stream) {
  if (int rc = cv_check(edge_attr, num_graphs, n, seq_length, canon, num_layers, heads, hl_pad))
    return rc;
  if (!dae_layers || !workspace || !dwfold) return SV2N_ERR_ARG;
  if (workspace_floats < sv2n_edge_logits_bwd_cv_workspace(seq_length, hl_pad))
    return SV2N_ERR_WORKSPACE;
  LayerCPtrs lp{};
  for (int l = 0; l < num_layers; ++l) {
    if (!dae_layers[l]) return SV2N_ERR_ARG;
    lp.p[l] = dae_layers[l];
  }
  const int D = 3 * seq_length, width = D * hl_pad;
  if ((seq_length & 1) == 0 && !cv_round4()) {
    // round 5: one workgroup per graph (grid-stride past CV2_BWD_GRID), MFMA
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(num_graphs, CV2_BWD_GRID));
    const int nc = (num_layers * heads + 3) / 4;
#define SV2N_CVB2(NP, NC)                                                                          \
  hipLaunchKernelGGL((k_edge_bwd_cv2<NP, NC>), dim3(grid), dim3(CV2_T), 0, stream, edge_attr,      \
                     num_graphs, n, seq_length, canon, lp, num_layers, heads, hl_pad, workspace)
#define SV2N_CVB2_NC(NP)                                         \
  switch (nc) {                                                  \
    case 1: SV2N_CVB2(NP, 4); break;                             \
    case 2: SV2N_CVB2(NP, 8); break;                             \
    case 3: SV2N_CVB2(NP, 12); break;                            \
    default: SV2N_CVB2(NP, 16); break;                           \
  }
    if (seq_length <= 32) SV2N_CVB2_NC(1)
    else SV2N_CVB2_NC(2)
#undef SV2N_CVB2_NC
#undef SV2N_CVB2
    hipLaunchKernelGGL(k_reduce_partials, dim3((unsigned)((width + 15) / 16)), dim3(256), 0, stream,
                       workspace, grid, width, dwfold);
    return (int)hipGetLastError();
  }
  const int64_t units = num_graphs * (((int64_t)n * (n - 1) / 2 + CV_PCH - 1) / CV_PCH);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(units, CV_BWD_GRID));
#define SV2N_CVB(NC)                                                                           \
  hipLaunchKernelGGL(k_edge_bwd_cv<NC>, dim3(grid), dim3(CV_T), 0, stream, edge_attr, num_graphs, \
                     n, seq_length, canon, lp, num_layers, heads, hl_pad, workspace)
  switch ((num_layers * heads + 3) / 4) {
    case 1: SV2N_CVB(4); break;
    case 2: SV2N_CVB(8); break;
    case 3: SV2N_CVB(12); break;
    default: SV2N_CVB(16); break;
  }
#undef SV2N_CVB
  hipLaunchKernelGGL(k_reduce_partials, dim3((unsigned)((width + 15) / 16)), dim3(256), 0, stream,
                     workspace, grid, width, dwfold);
  return (int)hipGetLastError();
}
