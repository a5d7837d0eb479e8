// GAT attention for graphs of n <= 32 nodes — the 30-asset volatility-
// spillover graphs of every SpotV2Net configuration (utils/dataset.py:216-226;
// PyG 2.3.0 GATConv inside utils/models.py:146).
// Same contract and saved state as k_attn_fwd / k_attn_bwd (sv2n_attn.hip, the
// round-1 kernels, kept behind SV2N_ATTN_CANON=0), with far fewer instructions
// per wave:
//
//  * the edge logits of a graph arrive as one contiguous block — [E0][H] in
//    the canonical edge order, or the dense [n][n][H] block of a row-mask
//    layout — and are copied into LDS as they lie (16-B loads and stores, no
//    per-element decode); the softmax lane of target i and source j finds a
//    canonical edge by the closed form of the order,
//      e(i, j) = T(j) + i - j - 1              (j < i: the upper pair (j, i))
//              = P + T(i) + j - i - 1          (j > i: the swapped pair),
//    T(x) = x(2n - x - 1)/2, P = n(n - 1)/2;
//  * lane (i, half) of a wave owns target row i and sources 16·half .. +15 in
//    the softmax; it writes their three bf16 planes (round 6; f32-accurate
//    bf16x3, as the projection GEMMs) to LDS, from where whichever wave
//    aggregates the head reads the A operand of v_mfma_f32_32x32x16_bf16
//    (two K steps of 16 sources, six products each; the backward still
//    aggregates on exact-f32 v_mfma_f32_32x32x2f32);
//  * the xs / dy / y operands are read straight from HBM in the MFMA operand
//    layouts (dword buffer loads, 128 B per half-wave, the row stride in a
//    scalar offset register), ahead of the MFMAs that use them.
#include "sv2n_common.h"

#include <cstdlib>

#include "sv2n_gemm3_kernel.h"  // split3_pk, bf16x8, u32x4_t

namespace sv2n {
namespace canon {

// Diagnostic builds only (make STAMPS=1): per-wave s_memtime / s_memrealtime
// stamps of the kernel phases, read back by sv2n_diag_stamps.
#ifdef SV2N_STAMPS
__device__ unsigned long long g_stamps[4096 * 4 * 16];
#define SV2N_STAMP(k, v) \
  if ((threadIdx.x & 63) == 0) g_stamps[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + (k)] = (v)
#define SV2N_T() __builtin_amdgcn_s_memtime()
#define SV2N_RT() __builtin_amdgcn_s_memrealtime()
#else
#define SV2N_STAMP(k, v)
#endif

// diagnostic timing builds only (results wrong; never in the library):
// SV2N_ATTN_ABL bit 1 drops the forward's y stores, bit 2 its xs loads, bit 4
// its psave stores
#ifndef SV2N_ATTN_ABL
#define SV2N_ATTN_ABL 0
#endif
constexpr int THREADS = 256;
constexpr int PS = SV2N_PSTR;  // LDS row stride of a probability row (floats)
constexpr int AEV = 8;         // 16-B slots per thread covering E0·H <= 992·8

typedef float floatx16 __attribute__((ext_vector_type(16)));

// Forward aggregation P·xs: 1 = f32-accurate bf16x3 on v_mfma_f32_32x32x16_bf16
// (P and xs split into three bf16 planes, the six products with plane orders
// p + q <= 2, as the projection GEMMs: 12 MFMAs of 32 cycles per 32 x 32
// tile); 0 = exact f32 on v_mfma_f32_32x32x2f32 (16 MFMAs of 64 cycles)
#ifndef SV2N_AGG_X3
#define SV2N_AGG_X3 1
#endif
// backward: G = xs·dZᵀ (the softmax's dP) on bf16x3 as well (1) or exact f32 (0)
#ifndef SV2N_BWD_G_X3
#define SV2N_BWD_G_X3 1
#endif
constexpr int PBR = 40;  // bf16 row stride of a probability plane row (80 B: distinct b128 bank slots)
// floats of the probability area sP of the forward: f32 rows, or three bf16 planes
__host__ __device__ constexpr int sp_floats(int H) {
  return SV2N_AGG_X3 ? 3 * H * 32 * PBR / 2 : H * 32 * PS;
}
// the six bf16x3 products of one 32 x 32 x 16 step (small terms first)
__device__ __forceinline__ floatx16 mfma32_x3(const bf16x8 (&a)[3], const bf16x8 (&b)[3],
                                              floatx16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
}
// eight floats -> their three bf16 planes (split3_pk pairs, low half first)
__device__ __forceinline__ void split8_x3(const float* v, bf16x8 (&h)[3]) {
  u32x4_t w0, w1, w2;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned a, b, c;
    split3_pk(v[2 * q], v[2 * q + 1], a, b, c);
    w0[q] = a;
    w1[q] = b;
    w2[q] = c;
  }
  h[0] = __builtin_bit_cast(bf16x8, w0);
  h[1] = __builtin_bit_cast(bf16x8, w1);
  h[2] = __builtin_bit_cast(bf16x8, w2);
}

// row of accumulator register r in lane half hf (32x32 MFMA C/D layout)
__device__ __forceinline__ int crow(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

// f32 -> bf16 bits, round to nearest even (v_cvt_pk_bf16_f32, as the bf16
// GEMMs' operand staging)
__device__ __forceinline__ unsigned short to_bf16(float x) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 v = {x, 0.f};
  return (unsigned short)(__builtin_bit_cast(unsigned, __builtin_convertvector(v, b2)) & 0xffffu);
}
__device__ __forceinline__ void bst16_s(rsrc_t r, int voff, int soff, float v) {
  __builtin_amdgcn_raw_buffer_store_b16(to_bf16(v), r, voff, soff, 0);
}

// dword buffer load / store with a wave-uniform scalar offset
__device__ __forceinline__ float bld_s(rsrc_t r, int voff, int soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ void bst_s(rsrc_t r, int voff, int soff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, soff, 0);
}

// ---------------------------------------------------------------------------
// forward: S 256-thread workgroups per graph (S = 1 when the batch alone
// fills the chip, C2; C3's 128 graphs of 6 x 500 columns run S = 4).  Each
// computes the whole softmax (cheap) and aggregates its share of the work
// items.  Block b -> graph 8·(b / 8S) + b % 8, split (b / 8) % S: the splits of
// a graph run on one XCD (they share its logits and xs rows through L2).
// LDS: sP (dropped-out probabilities, the MFMA A operand: three bf16 planes
//      [3][H][32][PBR], or f32 [H][32][PS] without SV2N_AGG_X3) |
//      sAS[H][32] a_src | sAD[H][32] a_dst | sAE[E0·H]
// Work items of wave slot u = 4s + w (after the softmax): concat — (head h,
// 32-column tile tc) pairs u, u + 4S, ...; mean — tiles tc = u, u + 4S, ...,
// each summed over the heads (sub-items h = 0..H-1 on one accumulator, in head
// order).  The saved probabilities are stored by split 0.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool graph_split(int64_t B, int S, int64_t& g, int& s) {
  const int64_t b = blockIdx.x;
  g = (b / (8 * S)) * 8 + (b & 7);
  s = (int)((b >> 3) % S);
  return g < B;
}

// HEAD (one workgroup per graph, the model's last GAT layer): the output head
// and the MSE loss of the training step are fused in (HeadFuse).  The layer
// output a = act(z) goes to LDS sY[32][OC + 1] instead of HBM; after a
// barrier, per row i: out_i = Σ_oc m·a·w[oc] + b (m the post-dropout factor),
// dout_i = 2/(B·n)·(out_i − target_i); then y receives dZ = act'(dout_i·w·m)
// (what the backward's activation step would produce, so the layer's
// backward runs with the identity and reads no y) and the graph's partials
// Σ_i dout_i·m·a (head weight), Σ_i dout_i (head bias), Σ_i diff² (loss)
// go to part[g] (k_head_fuse_finish sums them in graph order, accumulates
// the head gradients and writes the loss).
template <int ACT, bool CONCAT, bool KEEP, bool HEAD = false>
__global__ __launch_bounds__(THREADS) void k_fwd(
    const float* __restrict__ xs, int ldx, const float* __restrict__ ae, int ae_edge_order,
    const uint32_t* __restrict__ rowmask, const float* __restrict__ bias, const uint8_t* __restrict__ keep, float keep_scale,
    float* __restrict__ y, float* __restrict__ psave, const float* __restrict__ post_u,
    float post_p, float post_scale, float* __restrict__ post_out, int n, int H, int C, float slope,
    int S, int64_t B, HeadFuse hf) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sP = smem;  // SV2N_AGG_X3: three bf16 planes [3][H][32][PBR]
  unsigned short* sPb = reinterpret_cast<unsigned short*>(smem);
  const int PL = H * 32 * PBR;  // bf16 plane stride
  float* sAS = sP + sp_floats(H);
  float* sAD = sAS + H * 32;
  float* sAE = sAD + H * 32;

  SV2N_STAMP(0, SV2N_RT());
  SV2N_STAMP(1, SV2N_T());
  int64_t g;
  int split;
  if (!graph_split(B, S, g, split)) return;
  SV2N_CHK(301, g, B);  // every other access of the graph goes through its buffer descriptors
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int slot = 4 * split + wave, NS = 4 * S;
  const int l32 = lane & 31, half = lane >> 5;
  const int HC = H * C, OC = CONCAT ? HC : C;
  const int E0 = n * (n - 1), P = E0 / 2;
  const int nae = ae ? (ae_edge_order ? E0 : n * n) * H : 0;
  const int ntc = (C + 31) >> 5;
  const rsrc_t rx = make_rsrc(xs + (int64_t)g * n * ldx, (uint32_t)(n * ldx) * 4u);
  const rsrc_t ry = make_rsrc(y + (int64_t)g * n * OC, (uint32_t)(n * OC) * 4u);
  const rsrc_t rp = make_rsrc(psave + (int64_t)g * H * 1024, (uint32_t)H * 4096u);
  const rsrc_t rb = make_rsrc(bias, bias ? (uint32_t)OC * 4u : 0u);
  const bool post = post_u != nullptr;  // dropout after the layer, fused into the store
  const rsrc_t ru = make_rsrc(post ? post_u + g * n * OC : nullptr, post ? (uint32_t)(n * OC) * 4u : 0u);
  const rsrc_t ro = make_rsrc(post ? post_out + g * n * OC : nullptr,
                              post ? (uint32_t)(n * OC) * 4u : 0u);

  // ---- work items of this wave: q -> (head, tile), first / last sub-item ----
  const int nq = CONCAT ? max(0, (H * ntc - slot + NS - 1) / NS)
                        : max(0, (ntc - slot + NS - 1) / NS) * H;
  auto item = [&](int q, int& h, int& tc) {
    if constexpr (CONCAT) {
      const int s = slot + NS * q;
      h = s / ntc;
      tc = s - h * ntc;
    } else {
      const int k = q / H;
      h = q - k * H;
      tc = slot + NS * k;
    }
  };
  // xs rows 16·half + kk of head h's columns of tile tc: the B operand
  // branch-free: an item past the wave's last (q >= nq) reads 0 (OOB), so
  // the compiler's wait counts stay exact (a conditional load made the
  // softmax's first wait a vmcnt(0) on every xs load)
  // The item's bias value comes with its operands (loaded at the end of the
  // item, it was the youngest load there, and its wait a vmcnt(0) on the
  // later items' operands still in flight).
  auto load_b = [&](int q, float (&b)[16], float& bb) {
    int h, tc;
    item(q, h, tc);
    const int c = 32 * tc + l32;
    const bool ok = c < C && q < nq;
    bb = bld(rb, ok ? ((CONCAT ? h * C : 0) + c) * 4 : OOB);
#if SV2N_AGG_X3
    // element e: source 16·(e / 8) + 8·half + e % 8 (K step e / 8 of the
    // 32x32x16 B operand)
    const int voff = ok ? ((8 * half) * ldx + h * C + c) * 4 : OOB;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
      b[kk] = (SV2N_ATTN_ABL & 2) ? (float)(kk + voff) * 1e-3f
                                  : bld_s(rx, voff, (16 * (kk >> 3) + (kk & 7)) * ldx * 4);
#else
    const int voff = ok ? ((16 * half) * ldx + h * C + c) * 4 : OOB;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
      b[kk] = (SV2N_ATTN_ABL & 2) ? (float)(kk + voff) * 1e-3f : bld_s(rx, voff, kk * ldx * 4);
#endif
  };

  // ---- prologue: every load before any store ----
  f32x4 av[AEV];
  const rsrc_t ra = make_rsrc(ae ? ae + (int64_t)g * nae : nullptr, (uint32_t)nae * 4u);
  const int nv = (nae + 3) >> 2;
  const bool ae_vec = (nae & 3) == 0 && ((uintptr_t)ae & 15) == 0;
  if (ae_vec) {  // (uniform) unconditional loads, past the logits OOB (0)
#pragma unroll
    for (int q = 0; q < AEV; ++q) {
      const int k = t + THREADS * q;
      av[q] = bld4(ra, k < nv ? k * 16 : OOB);
    }
  } else {
#pragma unroll
    for (int q = 0; q < AEV; ++q) {
      const int k = t + THREADS * q;
#pragma unroll
      for (int c = 0; c < 4; ++c) av[q][c] = bld(ra, 4 * k + c < nae ? (4 * k + c) * 4 : OOB);
    }
  }
  float asd[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {  // (k, j) = a_src (k < H) / a_dst (k >= H) of node j
    const int idx = t + THREADS * s, k = idx >> 5, j = idx & 31;
    asd[s] = bld(rx, k < 2 * H ? (j * ldx + HC + k) * 4 : OOB);  // rows j >= n read 0
  }
  // sources of target row l32 (block layouts: the row mask; else all n) —
  // loaded BEFORE the xs operands: the softmax waits for it, and a load
  // issued after the 64 xs loads made that wait a vmcnt(0), i.e. the softmax
  // started only once the whole graph's xs had landed (round 6)
  const uint32_t allm = n >= 32 ? 0xffffffffu : ((1u << n) - 1u);
  const uint32_t rmw = bld_u32(make_rsrc(rowmask ? rowmask + (int64_t)g * n : nullptr,
                                          rowmask ? (uint32_t)n * 4u : 0u), l32 * 4);
  const uint32_t rbits = (rowmask ? rmw : allm) & ~(1u << l32);
  // HEAD: the output head's weights (OC <= 512: two per thread), staged into
  // LDS at the head phase (their loads in the prologue, ahead of the xs
  // operands: the head loops then read LDS instead of waiting on L2 per
  // column)
  float hw[2] = {0.f, 0.f};
  if constexpr (HEAD) {
    const rsrc_t rw = make_rsrc(hf.w, (uint32_t)OC * 4u);
#pragma unroll
    for (int k = 0; k < 2; ++k) hw[k] = bld(rw, t + THREADS * k < OC ? (t + THREADS * k) * 4 : OOB);
  }
  // B operands of the wave's first four work items (C2: all of them)
  float bq[4][16], bbq[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) load_b(u, bq[u], bbq[u]);

#pragma unroll
  for (int q = 0; q < AEV; ++q) {
    const int k = t + THREADS * q;
    if (q * THREADS < nv && k < nv) *reinterpret_cast<f32x4*>(sAE + 4 * k) = av[q];
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int idx = t + THREADS * s;
    if (idx < 2 * H * 32) sAS[idx] = asd[s];
  }
  __syncthreads();
  SV2N_STAMP(2, SV2N_T());

  // ---- per-target softmax: lane (i, half) = target i, sources 16·half + kk ----
  const int i = l32;
  const bool iv = i < n;
  // canonical edge ids of row i: e = Q(j) + i (j < i), e = Ehi + j (j > i), with
  // Q(j) = T(j) - j - 1 and Ehi = P + T(i) - i - 1 — no table, no branch
  const int Ehi = P + ((i * (2 * n - 1 - i)) >> 1) - i - 1;
  float pkeep[2][16];  // signed probabilities for psave, stored after the next loads
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int h = wave + 4 * s2;
    if (h >= H) break;  // wave-uniform
    uint32_t kw[4] = {~0u, ~0u, ~0u, ~0u};
    if constexpr (KEEP) {
      const u32x4 w4 = bld4_u32(make_rsrc(keep + ((int64_t)g * H + h) * 1024, 1024u),
                                (i * 32 + 16 * half));
      kw[0] = w4[0]; kw[1] = w4[1]; kw[2] = w4[2]; kw[3] = w4[3];
    }
    const float ad = sAD[h * 32 + i];
    const f32x4* asr = reinterpret_cast<const f32x4*>(sAS + h * 32 + 16 * half);
    f32x4 as4[4];
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) as4[k4] = asr[k4];
    float lg[16];
    float esum = 0.f;
    // the 16 edge logits of the lane's sources: every LDS address first, then
    // the 16 reads back to back and one wait.  Uniform choices (logits present,
    // edge order) are masks, not conditions: as conditions inside the loop
    // the compiler branched on them per source and waited lgkmcnt(0) after
    // each read — a serial chain of 16 LDS round trips (round 6).
    float av16[16];
    {
      const int j0 = 16 * half;
      const int eom = ae_edge_order ? -1 : 0;           // edge order vs dense [n][n]
      const uint32_t aem = ae ? 0xffffffffu : 0u;       // no logits: every source reads 0
      const uint32_t evb = iv ? (rbits & aem) : 0u;     // sources with a logit to read
      int elo = ((j0 * (2 * n - 1 - j0)) >> 1) - j0 - 1 + i;  // e(i, j) for j < i, j = j0
      int idx[16];
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const int j = j0 + kk;
        const int e_c = j < i ? elo : Ehi + j;
        const int e = (e_c & eom) | ((i * n + j) & ~eom);
        // masked by an AND (as a select the compiler branched around the multiply)
        idx[kk] = (__mul24(e, H) + h) & -(int)((evb >> j) & 1u);
        elo += n - 2 - j;  // T(j + 1) - T(j) - 1
      }
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) av16[kk] = sAE[idx[kk]];
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) av16[kk] = ((evb >> (j0 + kk)) & 1u) ? av16[kk] : 0.f;
    }
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const float a = av16[kk];
      esum += a;
      lg[kk] = as4[kk >> 2][kk & 3] + ad + a;
    }
    esum += __shfl_xor(esum, 32, 64);
    const int cnt = __popc(rbits);
    const float loopv = (ae && cnt > 0) ? esum / (float)cnt : 0.f;
    // the lane's valid sources kk (incoming edges and the self loop) as bits:
    // every step below is a select, not a branch (round 6: a conditional
    // expf made the compiler branch per source under exec masks, with its
    // masks spilled to VGPR lanes — 566 readlanes, the forward's softmax
    // phase 17.5K cycles)
    const uint32_t vbits = iv ? ((rbits | (1u << i)) >> (16 * half)) & 0xffffu : 0u;
    float mx = -INFINITY;
    uint32_t negm = 0u;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const int j = 16 * half + kk;
      float v = lg[kk] + (j == i ? loopv : 0.f);
      const bool neg = !(v > 0.f);
      negm |= neg ? (1u << kk) : 0u;
      v = neg ? v * slope : v;
      lg[kk] = v;
      mx = fmaxf(mx, ((vbits >> kk) & 1u) ? v : -INFINITY);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float den = 0.f;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const float ex = __expf(lg[kk] - mx);
      lg[kk] = ((vbits >> kk) & 1u) ? ex : 0.f;
      den += lg[kk];
    }
    den += __shfl_xor(den, 32, 64);
    const float inv = 1.f / (den + 1e-16f);
    float pdv[16];
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int kk = 4 * k4 + c;
        const float p = lg[kk] * inv;
        const bool valid = (vbits >> kk) & 1u;
        pkeep[s2][kk] = valid ? (((negm >> kk) & 1u) ? -p : p) : 0.f;
        float d = p;
        if constexpr (KEEP) d = ((kw[k4] >> (8 * c)) & 0xffu) ? d * keep_scale : 0.f;
        pdv[kk] = d;
      }
    }
#if SV2N_AGG_X3
    {  // row i, sources 16·half .. +15 of each plane: two 16-B pieces per plane
      unsigned short* prow = sPb + (h * 32 + i) * PBR + 16 * half;
#pragma unroll
      for (int k8 = 0; k8 < 2; ++k8) {
        bf16x8 pl[3];
        split8_x3(pdv + 8 * k8, pl);
#pragma unroll
        for (int pp = 0; pp < 3; ++pp)
          *reinterpret_cast<bf16x8*>(prow + pp * PL + 8 * k8) = pl[pp];
      }
    }
#else
    float* prow = sP + (h * 32 + i) * PS + 16 * half;
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4)
      *reinterpret_cast<f32x4*>(prow + 4 * k4) =
          f32x4{pdv[4 * k4], pdv[4 * k4 + 1], pdv[4 * k4 + 2], pdv[4 * k4 + 3]};
#endif
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int h = wave + 4 * s2;
    if (h >= H || split != 0) break;
    const int off = ((h * 32 + i) * 32 + 16 * half) * 4;
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4)
      if (!(SV2N_ATTN_ABL & 4) || pkeep[s2][4 * k4] == 1234.5f)
        bst4(rp, off + 16 * k4,
             f32x4{pkeep[s2][4 * k4], pkeep[s2][4 * k4 + 1], pkeep[s2][4 * k4 + 2],
                   pkeep[s2][4 * k4 + 3]});
  }
  SV2N_STAMP(3, SV2N_T());
  __syncthreads();  // sP complete
  SV2N_STAMP(4, SV2N_T());

  // ---- aggregation: out_h[i][c] = Σ_j P_h[i][j] · xs[j][h·C + c] ----
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const float invH = 1.f / (float)H;
  float* sY = sAE + ((nae + 3) & ~3);  // HEAD: the layer output [32][OC + 1]
  float uv[16];  // post-dropout draws of the work item's outputs (loaded at its first sub-item)
  auto run = [&](int q, const float (&b)[16], float bv) {
    int h, tc;
    item(q, h, tc);
    if (post && (CONCAT || h == 0)) {
      const int c = 32 * tc + l32;
      const int voff = c < C ? (4 * half * OC + (CONCAT ? h * C : 0) + c) * 4 : OOB;
#pragma unroll
      for (int r = 0; r < 16; ++r) uv[r] = bld_s(ru, voff, ((r & 3) + 8 * (r >> 2)) * OC * 4);
    }
#if SV2N_AGG_X3
    {  // K steps s = 0, 1 (sources 16s .. 16s + 15): lane (i, half) holds 8·half .. +7
      const unsigned short* pa = sPb + (h * 32 + l32) * PBR + 8 * half;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 a3[3], b3[3];
#pragma unroll
        for (int pp = 0; pp < 3; ++pp)
          a3[pp] = *reinterpret_cast<const bf16x8*>(pa + pp * PL + 16 * ks);
        split8_x3(b + 8 * ks, b3);
        acc = mfma32_x3(a3, b3, acc);
      }
    }
#else
    const f32x4* pa = reinterpret_cast<const f32x4*>(sP + (h * 32 + l32) * PS + 16 * half);
    f32x4 a4[4];
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) a4[k4] = pa[k4];
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[kk >> 2][kk & 3], b[kk], acc, 0, 0, 0);
#endif
    if (CONCAT || h == H - 1) {  // end of the work item: bias, activation, store
      const int c = 32 * tc + l32;
      const int oc = (CONCAT ? h * C : 0) + c;
      const bool cv = c < C;
      const int voff = cv ? (4 * half * OC + oc) * 4 : OOB;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float z = (CONCAT ? acc[r] : acc[r] * invH) + bv;
        const float a = act_fwd<ACT>(z);
        if constexpr (HEAD) {
          // unconditional (a branch per r otherwise): rows past n land in
          // sY's unread rows, columns past C in its unread padding column OC
          sY[crow(r, half) * (OC + 1) + (cv ? oc : OC)] = a;
        } else {
          if (!(SV2N_ATTN_ABL & 1) || a == 1234.5f)
            bst_s(ry, voff, ((r & 3) + 8 * (r >> 2)) * OC * 4, a);
          if (post)
            bst_s(ro, voff, ((r & 3) + 8 * (r >> 2)) * OC * 4,
                  uv[r] >= post_p ? a * post_scale : 0.f);
        }
        acc[r] = 0.f;
      }
    }
  };
  for (int q0 = 0; q0 < nq; q0 += 4) {  // (nq = 0: a split past the last tile)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = q0 + u;
      if (q < nq) {
        run(q, bq[u], bbq[u]);
        load_b(q + 4, bq[u], bbq[u]);  // past the last item: OOB (0), no branch
      }
    }
  }
  if constexpr (HEAD) {
    const int OC1 = OC + 1;
    float* sD = sY + 32 * OC1;  // dout per row
    float* sL = sD + 32;        // diff² per row
    float* sHw = sL + 32;       // the head weights [OC]
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (t + THREADS * k < OC) sHw[t + THREADS * k] = hw[k];
    // post-dropout factor of (row, oc): the forward's mask and scale
    auto mfac = [&](int row, int oc) {
      return post ? (bld(ru, (row * OC + oc) * 4) >= post_p ? post_scale : 0.f) : 1.f;
    };
    __syncthreads();  // sY complete
    {  // head output and residual: 8 threads per row, columns sub, sub + 8, ...
      const int row = t >> 3, sub = t & 7;
      float sacc = 0.f;
      if (row < n)
        for (int oc = sub; oc < OC; oc += 8)
          sacc = fmaf(sY[row * OC1 + oc] * mfac(row, oc), sHw[oc], sacc);
      sacc += __shfl_xor(sacc, 1, 64);
      sacc += __shfl_xor(sacc, 2, 64);
      sacc += __shfl_xor(sacc, 4, 64);
      if (sub == 0) {
        float dv = 0.f, lv = 0.f;
        if (row < n) {
          const float out = sacc + (hf.b ? hf.b[0] : 0.f);
          const float diff = out - hf.target[g * n + row];
          dv = diff * hf.inv_n2;
          lv = diff * diff;
        }
        sD[row] = dv;
        sL[row] = lv;
      }
    }
    __syncthreads();
    SV2N_STAMP(7, SV2N_T());
    // dZ in y's place (coalesced rows)
    const rsrc_t rz = make_rsrc(y + (int64_t)g * n * OC, (uint32_t)(n * OC) * 4u);
    for (int k = t; k < n * OC; k += THREADS) {
      const int row = k / OC, oc = k - row * OC;
      const float a = sY[row * OC1 + oc];
      bst(rz, k * 4, act_bwd<ACT>(sD[row] * sHw[oc] * mfac(row, oc), a));
    }
    SV2N_STAMP(8, SV2N_T());
    // the graph's partials (k_head_fuse_finish sums them in graph order:
    // round 4, summing them in this launch with two-level tickets made the C2
    // layer-1 forward 31.4 us against 24.9 + 4.9 for the forward and the
    // separate finish launch).  Column oc by G consecutive lanes, lane sub
    // summing rows sub, sub + G, ... in order, the G sums added in a fixed
    // xor tree (round 6: one lane per column walked all n rows, a serial LDS
    // chain of ~4 K cycles at the end of every workgroup)
    float* pg = hf.part + (int64_t)g * (OC + 2);
    const int G = OC <= THREADS / 8 ? 8 : (OC <= THREADS / 4 ? 4 : (OC <= THREADS / 2 ? 2 : 1));
    for (int oc0 = 0; oc0 < OC; oc0 += THREADS / G) {  // (uniform)
      const int oc = oc0 + t / G, sub = t & (G - 1);
      float sacc = 0.f;
      if (oc < OC)
        for (int row = sub; row < n; row += G)
          sacc = fmaf(sD[row], sY[row * OC1 + oc] * mfac(row, oc), sacc);
      for (int m = 1; m < G; m <<= 1) sacc += __shfl_xor(sacc, m, 64);
      if (sub == 0 && oc < OC) {
        SV2N_CHK(302, (int64_t)g * (OC + 2) + oc, B * (OC + 2));
        pg[oc] = sacc;
      }
    }
    if (wave == THREADS / 64 - 1) {  // Σ dout, Σ diff² over the rows: the last wave, a xor tree
      float sd = lane < n ? sD[lane] : 0.f, sl = lane < n ? sL[lane] : 0.f;
#pragma unroll
      for (int m = 1; m < 32; m <<= 1) {
        sd += __shfl_xor(sd, m, 64);
        sl += __shfl_xor(sl, m, 64);
      }
      if (lane == 0) {
        SV2N_CHK(303, (int64_t)g * (OC + 2) + OC + 1, B * (OC + 2));
        pg[OC] = sd;
        pg[OC + 1] = sl;
      }
    }
  }
  SV2N_STAMP(5, SV2N_T());
  SV2N_STAMP(6, SV2N_RT());
}


// Sums k_fwd<HEAD>'s per-graph partials part[B][OC + 2] in graph order:
// g_w[o] += Σ_g part[g][o] (o < OC), g_b[0] += Σ_g part[g][OC], loss[0] =
// Σ_g part[g][OC + 1] / (B·n) (and loss_sum[0] += loss[0]).  Block: 16
// columns x 16 graph groups, 32 loads in flight per thread.
__global__ __launch_bounds__(256) void k_head_fuse_finish(const float* __restrict__ part,
                                                          int64_t B, int OC, float inv_n,
                                                          float* __restrict__ g_w,
                                                          float* __restrict__ g_b,
                                                          float* __restrict__ loss,
                                                          float* __restrict__ loss_sum) {
  constexpr int U = 32;
  __shared__ float s_red[16][17];
  const int lo = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int o = blockIdx.x * 16 + lo, O = OC + 2;
  const rsrc_t rp = make_rsrc(part, (uint32_t)(B * O) * 4u);
  float a = 0.f;
  for (int64_t b0 = 0; b0 < B; b0 += 16 * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t b = b0 + grp + 16 * u;
      v[u] = bld(rp, (o < O && b < B) ? (int)(b * O + o) * 4 : OOB);
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
    if (o < OC) {
      if (g_w) g_w[o] += sm;
    } else if (o == OC) {
      if (g_b) g_b[0] += sm;
    } else {
      loss[0] = sm * inv_n;
      if (loss_sum) loss_sum[0] += sm * inv_n;
    }
  }
}

// ---------------------------------------------------------------------------
// backward: S workgroups per graph (graph_split), split s owning heads
// [s·HS, s·HS + HS), HS <= 4.  Its waves form 4/WPH groups of WPH waves;
// group q owns the split's head q and wave k of a group takes its chunks
// k, k + WPH, ...  Per head h (wave registers + the wave's LDS area):
//   dZ_h[i][c] = act'(dy, y) (· 1/H for the head mean),
//   G[j][i]    = Σ_c xs[j][h·C + c] · dZ_h[i][c]          (dP_dᵀ: lane i, rows j)
//   dxs[j][h·C + c] = Σ_i P_d[i][j] · dZ_h[i][c]
// over 32-column chunks staged through the wave's LDS area (xs and dZ rows,
// stride CS: conflict-free row and column operand reads); with WPH > 1 the
// group's partial G are added in wave order through LDS after a barrier.
// Then the dropout / softmax / leaky_relu backward of G in the MFMA output
// layout (lane i holds rows j = crow(r, half) — the positions its saved
// probabilities are loaded at) -> dl in sDL.  After a barrier: d ae of the
// split's heads in edge order (one decode per edge), d a_src = column sums
// of dl, d a_dst, zero padding (split 0).
// C3 (128 graphs, H 6 x 500 columns) runs S 6, HS 1, WPH 4; C2 (512 graphs,
// H 4) S 1, HS 4, WPH 1: one workgroup per graph, wave w owning head w; 8
// heads run at least two workgroups per graph.
// LDS: sP[HS][32][PB] (P_d, the A operand of dxs) | per wave 2 x [32][CS]
//      chunk area.  After the chunk loop (and a barrier) the chunk areas are
//      reused for sDL[HS][32][DS] | sSh[HS][32] (self-loop share of row i) |
//      sDad[HS][32] | sRB[32] | sDec[P] (pair p -> (u, w), u < w): 52 KB at
//      C2's HS = 4, three workgroups per CU (74 KB and two before).
//      HS <= 4 (canon_bwd_plan): each wave owns at most one head and keeps its
//      G in registers until then.
// ---------------------------------------------------------------------------
constexpr int CS = 36;  // chunk row stride (floats): 16-B rows, conflict-free b128 row reads
constexpr int AREA = 4 * 2 * 32 * CS;  // the four waves' chunk areas (floats)
constexpr int DS = 33;  // dl row stride (floats): conflict-free column sums
constexpr int PB = 32;  // P_d row stride: column reads only (conflict-free at any stride)

__host__ __device__ inline int canon_bwd_tail_floats(int HS) {  // sDL .. sDec
  return HS * 32 * DS + 2 * HS * 32 + 32 + (32 * 31 / 2 + 1) / 2;
}

// ---------------------------------------------------------------------------
// Edge-gradient tail (EdgeTail.ea != nullptr; canonical batches, one split per
// graph): the weight gradient of the folded edge logits of EVERY layer,
//   part[g][d][k] = Σ_{e of graph g} edge_attr[e][d] · dAE[e][k],
// k = l·H + h over the hl_pad columns of the edge pass (sv2n_edge.hip), with
// this layer's d-logits taken from LDS (never written to HBM) and the other
// layers' from their [E][H] edge-order buffers.  The graph's edge rows are
// streamed once; the caller sums the per-graph partials in graph order
// (k_reduce_partials).  This replaces the separate edge-gradient pass over
// edge_attr (k_edge_bwd) and its d-logit write / read for this layer.
// LDS: the tail region moves to the end of the chunk areas so that the
// d-logit table sE[E0][8] can span sP and the start of the areas; the wave
// partials reuse sE after the stream.
// ---------------------------------------------------------------------------

__host__ __device__ inline int canon_bwd_tail_off(bool edge, int HS) {
  return edge ? ((AREA - canon_bwd_tail_floats(HS)) & ~3) : 0;
}

// The tail proper (every thread of the workgroup; sDL / sSh / sDec complete).
__device__ __forceinline__ void edge_grad_tail(const EdgeTail& et, int64_t g, int n, int H,
                                               const float* sDL, const float* sSh,
                                               const uint16_t* sDec, float* smem) {
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int E0 = n * (n - 1), P = E0 / 2, D = et.D;
  float* sE = smem;  // [E0][ET_COLS]
  // this layer's d-logits (dl + the self-loop share of row ti), PyG's per-edge
  // gradient of the folded edge logit
  for (int p = t; p < P; p += THREADS) {
    const uint32_t uw = sDec[p];
    const int u = uw >> 8, w = uw & 0xff;
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int ti = side ? u : w, tj = side ? w : u, e = side ? P + p : p;
      for (int h = 0; h < H; ++h)
        sE[e * ET_COLS + et.own * H + h] = sDL[(h * 32 + ti) * DS + tj] + sSh[h * 32 + ti];
    }
  }
  // the other layers' columns (coalesced [E0][H] runs) and the zero padding
  for (int l = 0; l < et.L; ++l) {
    if (l == et.own) continue;
    const rsrc_t rd = make_rsrc(et.dae[l] + g * E0 * H, (uint32_t)(E0 * H) * 4u);
    for (int k = t; k < E0 * H; k += THREADS) {
      const int e = k / H, h = k - e * H;
      sE[e * ET_COLS + l * H + h] = bld(rd, k * 4);
    }
  }
  for (int k = t; k < E0 * (ET_COLS - et.L * H); k += THREADS) {
    const int w = ET_COLS - et.L * H, e = k / w;
    sE[e * ET_COLS + et.L * H + (k - e * w)] = 0.f;
  }
  __syncthreads();
  // stream the graph's edge rows: wave w takes edges w, w + 4, ...; lane l the
  // columns d = 2l, 2l + 1 (8-B loads: a row is one wave-instruction); two
  // register sets of U rows in flight
  constexpr int U = 8;
  const int d0 = 2 * lane;
  const bool dv = d0 < D;
  const rsrc_t rea = make_rsrc(et.ea + g * E0 * D, (uint32_t)(E0 * D) * 4u);
  float a0[ET_COLS], a1[ET_COLS];
#pragma unroll
  for (int c = 0; c < ET_COLS; ++c) a0[c] = a1[c] = 0.f;
  u32x2 va[U], vb[U];
  auto load = [&](u32x2 (&v)[U], int e0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + 4 * u;
      v[u] = bld2_u32(rea, (dv && e < E0) ? (e * D + d0) * 4 : OOB);
    }
  };
  auto fma_rows = [&](const u32x2 (&v)[U], int e0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + 4 * u;
      if (e < E0) {  // wave-uniform
        const f32x4 k0 = *reinterpret_cast<const f32x4*>(sE + e * ET_COLS);
        const f32x4 k1 = *reinterpret_cast<const f32x4*>(sE + e * ET_COLS + 4);
        const float x0 = __uint_as_float(v[u][0]), x1 = __uint_as_float(v[u][1]);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          a0[c] = fmaf(x0, k0[c], a0[c]);
          a1[c] = fmaf(x1, k0[c], a1[c]);
          a0[4 + c] = fmaf(x0, k1[c], a0[4 + c]);
          a1[4 + c] = fmaf(x1, k1[c], a1[4 + c]);
        }
      }
    }
  };
  int e0 = wave;
  load(va, e0);
  for (; e0 < E0; e0 += 8 * U) {
    load(vb, e0 + 4 * U);
    fma_rows(va, e0);
    load(va, e0 + 8 * U);
    fma_rows(vb, e0 + 4 * U);
  }
  __syncthreads();  // every wave is done with sE: it takes the wave partials
  float* sR = smem;  // [4][ET_COLS][128]
#pragma unroll
  for (int c = 0; c < ET_COLS; ++c) {
    sR[(wave * ET_COLS + c) * 128 + d0] = a0[c];
    sR[(wave * ET_COLS + c) * 128 + d0 + 1] = a1[c];
  }
  __syncthreads();
  const int O = D * et.hlp;
  const rsrc_t rp = make_rsrc(et.part + g * O, (uint32_t)O * 4u);
  for (int o = t; o < O; o += THREADS) {
    const int d = o / et.hlp, c = o - d * et.hlp;
    float s = sR[c * 128 + d];
#pragma unroll
    for (int w = 1; w < 4; ++w) s += sR[(w * ET_COLS + c) * 128 + d];
    bst(rp, o * 4, s);
  }
}

template <int ACT, bool CONCAT, bool KEEP, int DEPTH>
__global__ __launch_bounds__(THREADS) void k_bwd(
    const float* __restrict__ dy, const float* __restrict__ y, const float* __restrict__ xs,
    int ldx, const float* __restrict__ psave, const uint8_t* __restrict__ keep, float keep_scale,
    const float* __restrict__ post_u, float post_p, float post_scale,
    const uint32_t* __restrict__ rowmask, float* __restrict__ dxs, float* __restrict__ dae,
    int ae_edge_order, float* __restrict__ dbias_part, int n, int H, int C, float slope, int S,
    int HS, int WPH, int64_t B, EdgeTail et, unsigned short* __restrict__ dxb, int ldb) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sP = smem;
  float* sArea = sP + HS * 32 * PB;
  const bool etail = et.ea != nullptr;  // uniform
  float* sDL = sArea + canon_bwd_tail_off(etail, HS);  // after the chunk loop
  float* sSh = sDL + HS * 32 * DS;
  float* sDad = sSh + HS * 32;
  uint32_t* sRB = reinterpret_cast<uint32_t*>(sDad + HS * 32);  // source bits of row i
  uint16_t* sDec = reinterpret_cast<uint16_t*>(sRB + 32);        // pair p -> (u << 8 | w)

  SV2N_STAMP(0, SV2N_RT());
  SV2N_STAMP(1, SV2N_T());
  int64_t g;
  int split;
  if (!graph_split(B, S, g, split)) return;
  SV2N_CHK(301, g, B);  // every other access of the graph goes through its buffer descriptors
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int l32 = lane & 31, half = lane >> 5;
  const int HC = H * C, OC = CONCAT ? HC : C;
  const int E0 = n * (n - 1);
  const float invH = 1.f / (float)H;
  const int h0 = split * HS, nhs = min(HS, H - h0);  // this split's heads
  const rsrc_t rx = make_rsrc(xs + g * n * ldx, (uint32_t)(n * ldx) * 4u);
  // dxb != NULL (uniform): dxs goes out as bf16 [N][ldb] instead (the bf16
  // weight-gradient GEMM's operand, rounded as its staging would)
  const bool bfo = dxb != nullptr;
  const rsrc_t rdx = make_rsrc(bfo ? nullptr : dxs + g * n * ldx, bfo ? 0u : (uint32_t)(n * ldx) * 4u);
  const rsrc_t rdb16 = make_rsrc(bfo ? dxb + g * n * ldb : nullptr, bfo ? (uint32_t)(n * ldb) * 2u : 0u);
  auto put = [&](int j, int col, float v) __attribute__((always_inline)) {  // dxs[j][col]
    if (bfo)
      __builtin_amdgcn_raw_buffer_store_b16(to_bf16(v), rdb16, j < n ? (j * ldb + col) * 2 : OOB,
                                            0, 0);
    else
      bst(rdx, j < n ? (j * ldx + col) * 4 : OOB, v);
  };
  const rsrc_t rdy = make_rsrc(dy + g * n * OC, (uint32_t)(n * OC) * 4u);
  const rsrc_t ryy = make_rsrc(y + g * n * OC, (uint32_t)(n * OC) * 4u);
  const rsrc_t rps = make_rsrc(psave + g * H * 1024, (uint32_t)H * 4096u);
  const rsrc_t rdb = make_rsrc(dbias_part + g * OC, (uint32_t)OC * 4u);
  // dy is the gradient of the post-dropout output (never with DEPTH 3: its
  // register sets leave no room for the draws)
  const bool post = DEPTH < 3 && post_u != nullptr;
  const rsrc_t ru =
      make_rsrc(post ? post_u + g * n * OC : nullptr, post ? (uint32_t)(n * OC) * 4u : 0u);

  float* sX = sArea + wave * 2 * 32 * CS;
  float* sZ = sX + 32 * CS;
  const int nch = (C + 31) >> 5;
  const int cwb = (C + nch - 1) / nch;  // balanced chunk width (<= 32)
  const int grp = wave / WPH, sub = wave - grp * WPH;
  // chunk ch of the wave's head: columns [c0, c0 + cw).  When the dy / y rows
  // are 64-B aligned (OC % 16 == 0: C2's 400) the chunk edges sit on their
  // 64-B segments — the first chunk ends at the head's first segment edge past
  // 16 columns, then 32 columns each — so no segment is fetched by two chunks
  // (balanced 25-column chunks re-fetched every edge segment: PMC reads 1.9x
  // the algorithmic bytes).  Otherwise, or if that takes an extra chunk,
  // balanced widths.
  const int hoff = CONCAT ? (h0 + grp) * C : 0;
  const int al = (16 - (hoff & 15)) & 15;
  const int f1 = al == 0 ? 32 : al + 16;
  const bool seg = (OC & 15) == 0 && (C > f1 ? 1 + (C - f1 + 31) / 32 : 1) == nch;
  auto chunk_range = [&](int ch, int& c0, int& cw) {
    if (seg) {
      c0 = ch == 0 ? 0 : f1 + 32 * (ch - 1);
      cw = min(ch == 0 ? f1 : 32, C - c0);
    } else {
      c0 = cwb * ch;
      cw = min(cwb, C - c0);
    }
  };
  const int nhw = grp < nhs ? 1 : 0;                            // heads of this wave (HS <= NG)
  const int ncw = sub < nch ? (nch - sub + WPH - 1) / WPH : 0;  // chunks per head
  const int nseq = nhw * ncw;                                  // (head, chunk) steps

  // chunk step q: rows 2m + half, column l32 of the chunk (dword loads, the
  // row stride in the scalar offset).  DEPTH register sets: chunk q lives in
  // set q % DEPTH, so DEPTH chunks are in flight (C2: two, at 2 waves/SIMD;
  // three when ACT is the identity — dy arrives as dZ from the producer's
  // ReLU-masked store (sv2n_gemm_f32x3_relu) and no y is read; four sets
  // spill at the 256-register budget of 2 waves/SIMD).
  float rx_[DEPTH][16], rdy_[DEPTH][16], ry_[DEPTH][16], ru_[DEPTH][16];
  auto load_chunk = [&](int q, auto set_tag) __attribute__((always_inline)) {
    constexpr int b = decltype(set_tag)::value;
    const int ch = sub + WPH * q, h = h0 + grp;  // the wave's one head
    int c0, cw;
    chunk_range(ch, c0, cw);
    const int c = c0 + l32;
    const bool cv = l32 < cw && q < nseq;  // past the wave's last step: OOB (0), no branch
    const int xo = cv ? (half * ldx + h * C + c) * 4 : OOB;
    const int zo = cv ? (half * OC + (CONCAT ? h * C : 0) + c) * 4 : OOB;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      rx_[b][m] = bld_s(rx, xo, 2 * m * ldx * 4);
      rdy_[b][m] = bld_s(rdy, zo, 2 * m * OC * 4);
      if constexpr (ACT != ACT_ID) ry_[b][m] = bld_s(ryy, zo, 2 * m * OC * 4);
    }
    if (post) {  // (a uniform branch: unconditional loads of nothing cost C2's
                 // layer-1 backward 19.9 -> 21.4 us, more than the exact waits gain)
#pragma unroll
      for (int m = 0; m < 16; ++m) ru_[b][m] = bld_s(ru, zo, 2 * m * OC * 4);
    }
  };
  // saved probabilities / keep bytes of head h at lane i's output rows
  // j = crow(r, half): four 16-B pieces of row i
  f32x4 pr[4];
  uint32_t kb[4];
  auto load_p = [&](int h) {
    const int base = ((h * 32 + l32) * 32 + 4 * half) * 4;
#pragma unroll
    for (int m = 0; m < 4; ++m) pr[m] = bld4(rps, base + 32 * m);
    if constexpr (KEEP) {  // (h >= H: a wave without a head, nothing read)
      const rsrc_t rk = make_rsrc(h < H ? keep + (g * H + h) * 1024 : nullptr, h < H ? 1024u : 0u);
#pragma unroll
      for (int m = 0; m < 4; ++m) kb[m] = bld_u32(rk, (l32 * 32 + 4 * half) + 8 * m);
    }
  };

  // sources of target row l32 (block layouts: the row mask; else all n),
  // then the first chunks — every load unconditional (past the wave's steps,
  // or without a row mask, OOB: 0), so the compiler's wait counts stay exact.
  // Round 6: the row-mask select after conditional chunk loads made the
  // prologue wait vmcnt(0) on every chunk in flight (C2: all three), and
  // its later use a second vmcnt(0).
  const uint32_t allm = n >= 32 ? 0xffffffffu : ((1u << n) - 1u);
  const uint32_t rmw = bld_u32(make_rsrc(rowmask ? rowmask + g * n : nullptr,
                                          rowmask ? (uint32_t)n * 4u : 0u), l32 * 4);
  const uint32_t rbits = (rowmask ? rmw : allm) & ~(1u << l32);
  load_p(h0 + grp);  // a wave without a head (h >= H) reads past psave: 0
  load_chunk(0, std::integral_constant<int, 0>{});
  if constexpr (DEPTH > 1) load_chunk(1, std::integral_constant<int, 1>{});
  if constexpr (DEPTH > 2) load_chunk(2, std::integral_constant<int, 2>{});
  floatx16 G;
#pragma unroll
  for (int r = 0; r < 16; ++r) G[r] = 0.f;
  const int i = l32;
  const bool iv = i < n;

  // ---- softmax / leaky_relu backward of head h (local hl) from Gh: lane (i,
  //      half), rows j = crow(r, half) ----
  auto softmax_bwd = [&](int hl, const floatx16& Gh) {
    // validity as one per-lane bit mask and selects (round 6: the
    // short-circuit `iv && (jr == i || bit)` compiled to exec-mask branches
    // around every accumulator read, as the forward's conditional expf did)
    const uint32_t vmask = iv ? (rbits | (1u << i)) : 0u;
    float ps[16], dp[16];
    float tl = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jr = crow(r, half);
      ps[r] = pr[r >> 2][r & 3];
      const bool valid = (vmask >> jr) & 1u;
      const float gv = CONCAT ? Gh[r] : Gh[r] * invH;
      float d = valid ? gv : 0.f;
      if constexpr (KEEP) d = ((kb[r >> 2] >> (8 * (r & 3))) & 0xffu) ? d * keep_scale : 0.f;
      dp[r] = d;
      tl += fabsf(ps[r]) * d;
    }
    tl += __shfl_xor(tl, 32, 64);
    float dad = 0.f, mine = 0.f;
    const int ri = (i & 3) + 4 * (i >> 3), hi = (i >> 2) & 1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jr = crow(r, half);
      const bool valid = (vmask >> jr) & 1u;
      const float ds = fabsf(ps[r]) * (dp[r] - tl);
      const float dl = valid ? (signbit(ps[r]) ? ds * slope : ds) : 0.f;
      dad += dl;
      mine = (r == ri) ? dl : mine;
      sDL[(hl * 32 + i) * DS + jr] = dl;
    }
    dad += __shfl_xor(dad, 32, 64);
    const float other = __shfl_xor(mine, 32, 64);
    const float dlii = (half == hi) ? mine : other;
    if (half == 0) {
      sDad[hl * 32 + i] = iv ? dad : 0.f;
      const int cnt = __popc(rbits);
      sSh[hl * 32 + i] = (iv && cnt > 0) ? dlii / (float)cnt : 0.f;
    }
  };

  if (nhw > 0) {  // wave-uniform
    const int hl = grp, h = h0 + hl;
    auto chunk_step = [&](int chi, auto set_tag) __attribute__((always_inline)) {
      constexpr int b = decltype(set_tag)::value;
      const int q = chi, ch = sub + WPH * chi;
      int c0, cw;
      chunk_range(ch, c0, cw);
      if (chi == 0) {
        // P_d of head h -> sP rows (each lane: its 16 positions of row i).
        // With WPH > 1 every wave of the group writes the same values: each
        // reads only what it wrote itself.
        float* prow = sP + (hl * 32 + l32) * PB + 4 * half;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float a = fabsf(pr[m][e]);
            if constexpr (KEEP) a = ((kb[m] >> (8 * e)) & 0xffu) ? a * keep_scale : 0.f;
            v[e] = iv ? a : 0.f;
          }
          *reinterpret_cast<f32x4*>(prow + 8 * m) = v;
        }
      }
      // stage the chunk: sX[row][c] = xs, sZ[row][c] = act'(dy, y)
      SV2N_STAMP(2 + 2 * min(q, 3), SV2N_T());
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int row = 2 * m + half;
        sX[row * CS + l32] = rx_[b][m];
        const float d =
            post ? (ru_[b][m] >= post_p ? rdy_[b][m] * post_scale : 0.f) : rdy_[b][m];
        sZ[row * CS + l32] = ACT == ACT_ID ? d : act_bwd<ACT>(d, ry_[b][m]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own LDS writes, in order
      SV2N_STAMP(3 + 2 * min(q, 3), SV2N_T());
      load_chunk(q + DEPTH, set_tag);  // refill this set (past the last step: OOB)
      // bias partials: column sums of dz (concat: this head's columns; mean: once)
      if (CONCAT || h == 0) {
        float sb = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) sb += sZ[(16 * half + r) * CS + l32];
        sb += __shfl_xor(sb, 32, 64);
        bst(rdb, (half == 0 && l32 < cw) ? ((CONCAT ? h * C : 0) + c0 + l32) * 4 : OOB, sb);
      }
      // G[j][i] += Σ_c xs[j][c] · dZ[i][c]    (step kk pairs columns kk and 16 + kk;
      // the chunk's columns past cw are staged zeros)
      if constexpr (SV2N_BWD_G_X3 && ACT == ACT_ID && DEPTH <= 2) {
        // bf16x3: K steps of 16 columns, lane (row, half) holds columns 16s +
        // 8·half .. +7.  Identity-activation, two-chunk instances only: with
        // the activation's operands live the extra planes cost the C3 kernel
        // its second workgroup per CU, and at three chunks in flight (C2 L0)
        // it measured no faster (27.6 -> 27.8-28.0 us; C2 L1 19.8-20.2 ->
        // 18.7-18.9 us, profiles/r06_attn_bwd_g_bf16x3.txt)
        const float* xr = sX + l32 * CS + 8 * half;
        const float* zr = sZ + l32 * CS + 8 * half;
#pragma unroll 1
        for (int ks = 0; ks < 2; ++ks) {
          const f32x4 x0 = *reinterpret_cast<const f32x4*>(xr + 16 * ks);
          const f32x4 x1 = *reinterpret_cast<const f32x4*>(xr + 16 * ks + 4);
          const f32x4 z0 = *reinterpret_cast<const f32x4*>(zr + 16 * ks);
          const f32x4 z1 = *reinterpret_cast<const f32x4*>(zr + 16 * ks + 4);
          const float xv[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
          const float zv[8] = {z0[0], z0[1], z0[2], z0[3], z1[0], z1[1], z1[2], z1[3]};
          bf16x8 a3[3], b3[3];
          split8_x3(xv, a3);
          split8_x3(zv, b3);
          G = mfma32_x3(a3, b3, G);
        }
      } else {
        const f32x4* xa = reinterpret_cast<const f32x4*>(sX + l32 * CS + 16 * half);
        const f32x4* zb = reinterpret_cast<const f32x4*>(sZ + l32 * CS + 16 * half);
        f32x4 a4[4], b4[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          a4[m] = xa[m];
          b4[m] = zb[m];
        }
#pragma unroll
        for (int kk = 0; kk < 16; ++kk)
          G = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[kk >> 2][kk & 3], b4[kk >> 2][kk & 3], G,
                                                   0, 0, 0);
      }
      // dxs[j][c] = Σ_i P_d[i][j] · dZ[i][c]    (k: i = 16·half + kk)
      floatx16 D;
#pragma unroll
      for (int r = 0; r < 16; ++r) D[r] = 0.f;
      const float* pcol = sP + (hl * 32 + 16 * half) * PB + l32;
      const float* zcol = sZ + (16 * half) * CS + l32;
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
        D = __builtin_amdgcn_mfma_f32_32x32x2f32(pcol[kk * PB], zcol[kk * CS], D, 0, 0, 0);
      if (bfo) {
        const int voff = l32 < cw ? (4 * half * ldb + h * C + c0 + l32) * 2 : OOB;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          bst16_s(rdb16, voff, ((r & 3) + 8 * (r >> 2)) * ldb * 2, CONCAT ? D[r] : D[r] * invH);
      } else {
        const int voff = l32 < cw ? (4 * half * ldx + h * C + c0 + l32) * 4 : OOB;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          bst_s(rdx, voff, ((r & 3) + 8 * (r >> 2)) * ldx * 4, CONCAT ? D[r] : D[r] * invH);
      }
    };
    for (int chi = 0; chi < ncw; chi += DEPTH) {
      chunk_step(chi, std::integral_constant<int, 0>{});
      if constexpr (DEPTH > 1)
        if (chi + 1 < ncw) chunk_step(chi + 1, std::integral_constant<int, 1>{});
      if constexpr (DEPTH > 2)
        if (chi + 2 < ncw) chunk_step(chi + 2, std::integral_constant<int, 2>{});
    }
  }
  __syncthreads();  // every wave is done with the chunk areas (reused below)
  if (WPH > 1) {
    // one head per group: the group's partial G, added in wave order
    float* sG = sArea + wave * 2 * 32 * CS;
#pragma unroll
    for (int r = 0; r < 16; ++r) sG[r * 64 + lane] = G[r];
    __syncthreads();
    if (sub == 0 && nhw > 0) {
      for (int k = 1; k < WPH; ++k) {
        const float* o = sArea + (wave + k) * 2 * 32 * CS;
#pragma unroll
        for (int r = 0; r < 16; ++r) G[r] += o[r * 64 + lane];
      }
    }
    __syncthreads();  // partials read: the area now takes sDL
  }
  if (nhw > 0 && sub == 0) softmax_bwd(grp, G);  // pr still holds this head's P
  if (t < 32) sRB[t] = rbits;
  if ((dae || etail) && ae_edge_order && t < n) {  // row u of the pair table
    const int base = (t * (2 * n - 1 - t)) >> 1;
    for (int w = t + 1; w < n; ++w) sDec[base + w - t - 1] = (uint16_t)((t << 8) | w);
  }
  SV2N_STAMP(10, SV2N_T());
  __syncthreads();
  SV2N_STAMP(11, SV2N_T());

  // ---- d ae of this split's heads in canonical edge order [E0][H]: pair
  //      p = (u, w), u < w, is edge p (target w, source u) and edge P + p
  //      (target u, source w) ----
  const bool vec4 = H == 4 && nhs == 4, vec2 = nhs == 2 && (H & 1) == 0 && (h0 & 1) == 0;
  if (dae && !ae_edge_order) {
    // ---- dense [n][n][H] block (block layouts): zeros off the edge set ----
    const int nae = n * n * H;
    const rsrc_t rdae = make_rsrc(dae + g * nae, (uint32_t)nae * 4u);
    for (int k = t; k < n * n; k += THREADS) {
      const int ti = k / n, tj = k - ti * n;
      const bool e = tj != ti && ((sRB[ti] >> tj) & 1u);
      if (vec4) {
        f32x4 v;
#pragma unroll
        for (int h = 0; h < 4; ++h) v[h] = e ? sDL[(h * 32 + ti) * DS + tj] + sSh[h * 32 + ti] : 0.f;
        bst4(rdae, k * 16, v);
      } else if (vec2) {
        bst2(rdae, (k * H + h0) * 4, e ? sDL[ti * DS + tj] + sSh[ti] : 0.f,
             e ? sDL[(32 + ti) * DS + tj] + sSh[32 + ti] : 0.f);
      } else {
        for (int hl = 0; hl < nhs; ++hl)
          bst(rdae, (k * H + h0 + hl) * 4,
              e ? sDL[(hl * 32 + ti) * DS + tj] + sSh[hl * 32 + ti] : 0.f);
      }
    }
  } else if (dae) {
    const int P = E0 / 2, nae = E0 * H;
    const rsrc_t rdae = make_rsrc(dae + g * nae, (uint32_t)nae * 4u);
    for (int p = t; p < P; p += THREADS) {
      const uint32_t uw = sDec[p];
      const int u = uw >> 8, w = uw & 0xff;
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const int ti = side ? u : w, tj = side ? w : u, e = side ? P + p : p;
        if (vec4) {
          f32x4 v;
#pragma unroll
          for (int h = 0; h < 4; ++h) v[h] = sDL[(h * 32 + ti) * DS + tj] + sSh[h * 32 + ti];
          bst4(rdae, e * 16, v);
        } else if (vec2) {
          bst2(rdae, (e * H + h0) * 4, sDL[ti * DS + tj] + sSh[ti],
               sDL[(32 + ti) * DS + tj] + sSh[32 + ti]);
        } else {
          for (int hl = 0; hl < nhs; ++hl)
            bst(rdae, (e * H + h0 + hl) * 4, sDL[(hl * 32 + ti) * DS + tj] + sSh[hl * 32 + ti]);
        }
      }
    }
  }
  // ---- dxs columns [HC, ldx): d a_src[h][j] = Σ_i dl[h][i][j] (two lanes per
  //      column, 16 rows each), d a_dst, zero padding (split 0) ----
  for (int q = t; q < 2 * 32 * nhs; q += THREADS) {
    const int hl = q >> 6, j = (q >> 1) & 31, part = q & 1;
    const float* col = sDL + (hl * 32 + 16 * part) * DS + j;
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) v += col[r * DS];
    v += __shfl_xor(v, 1, 64);
    if (part == 0) put(j, HC + h0 + hl, v);
  }
  for (int q = t; q < 32 * nhs; q += THREADS) {
    const int j = q & 31, hl = q >> 5;
    put(j, HC + H + h0 + hl, sDad[hl * 32 + j]);
  }
  const int npad = (bfo ? ldb : ldx) - HC - 2 * H;
  if (split == 0)
    for (int q = t; q < 32 * npad; q += THREADS) {
      const int j = q & 31, c2 = q >> 5;
      put(j, HC + 2 * H + c2, 0.f);
    }
  if (etail) edge_grad_tail(et, g, n, H, sDL, sSh, sDec, smem);
  SV2N_STAMP(12, SV2N_T());
  SV2N_STAMP(13, SV2N_RT());
}

}  // namespace canon

#ifdef SV2N_STAMPS
extern "C" int sv2n_diag_stamps(unsigned long long* out, int64_t count) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(canon::g_stamps),
                                  sizeof(unsigned long long) * (size_t)count);
}
#endif

// ---- launchers (called by the C-ABI entry points in sv2n_attn.hip) ---------
// Workgroups per graph.  The batch alone fills the chip at >= 512 blocks
// (2 per CU: C2's 512 graphs ran slower split, 27.8 vs 21 us forward); below that a graph's work is split: forward by work items
// (every split recomputes the softmax), backward by heads and, inside a
// split, a head's chunks over WPH waves.
constexpr int64_t CANON_FILL = 512;
constexpr unsigned CANON_CUS = 256;  // MI355X compute units

static int canon_fwd_splits(int64_t B, int H, int C, bool concat) {
  const int ntc = (C + 31) >> 5, items = concat ? H * ntc : ntc;
  int S = 1;
  while (B * S < CANON_FILL && 4 * 2 * S <= items) S *= 2;
  return S;
}

struct CanonBwdPlan {
  int S, HS, WPH;
};
// single: the fewest splits (the edge-gradient tail needs a whole graph per
// workgroup, whatever B)
// SV2N_CANON_BWD_S=s: that many head splits where valid (A/B switch)
static int canon_bwd_forced_s() {
  static const int v = [] {
    const char* e = std::getenv("SV2N_CANON_BWD_S");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}
// mean (head-mean layers): every split re-reads the graph's dy / y / dropout
// draws, so the split count stops at 384 workgroups (C3, B 128: 3 splits of
// two heads, 44.9 µs in the loop against 51.3 for 6 splits of one,
// profiles/r05_c3_bwd_splits.txt)
constexpr int64_t CANON_FILL_MEAN = 384;
static CanonBwdPlan canon_bwd_plan(int64_t B, int H, int C, bool single = false,
                                   bool mean = false) {
  const int nch = (C + 31) >> 5;
  int S = 1;
  const int fs = single ? 0 : canon_bwd_forced_s();
  const int64_t fill = mean ? CANON_FILL_MEAN : CANON_FILL;
  for (int s = 1; s <= H; ++s) {
    const int hs = (H + s - 1) / s;
    if (hs > 4 || (H + hs - 1) / hs != s) continue;  // one head per wave; no empty split
    S = s;
    if (fs > 0 ? s >= fs : (single || B * s >= fill)) break;
  }
  const int HS = (H + S - 1) / S;
  const int WPH = max(1, min(4 / HS, nch));
  return {S, HS, WPH == 3 ? 2 : WPH};  // WPH divides 4
}

static unsigned canon_grid(int64_t B, int S) {
  return (unsigned)(S == 1 ? B : ((B + 7) / 8) * 8 * S);
}

size_t attn_canon_bwd_lds(int HS) {
  const int area = 4 * 2 * 32 * canon::CS;
  return sizeof(float) * ((size_t)HS * 32 * canon::PB +
                          (size_t)std::max(area, canon::canon_bwd_tail_floats(HS)));
}

template <int ACT, bool CONCAT, bool KEEP>
static void launch_canon_bwd(int64_t B, hipStream_t st, const float* dy, const float* y,
                             const float* xs, int ldx, const float* psave, const uint8_t* keep,
                             float keep_scale, const float* post_u, float post_p,
                             const uint32_t* rowmask, float* dxs, float* dae,
                             int ae_edge_order, float* dbias, int n, int H, int C, float slope,
                             const EdgeTail& et, unsigned short* dxb, int ldb) {
  const CanonBwdPlan pl = canon_bwd_plan(B, H, C, et.ea != nullptr, !CONCAT);
  const size_t lds = attn_canon_bwd_lds(pl.HS);
  const unsigned grid = canon_grid(B, pl.S);
  // two chunks in flight per wave when every workgroup is resident at 2 waves
  // per SIMD (the deeper register sets cost the third workgroup per CU)
  auto launch = [&](auto kern) {
    if (lds > 65536)
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(canon::THREADS), lds, st, dy, y, xs, ldx, psave,
                       keep, keep_scale, post_u, post_p,
                       post_u ? (float)(1.0 / (1.0 - (double)post_p)) : 1.f, rowmask, dxs, dae,
                       ae_edge_order, dbias, n, H, C, slope, pl.S, pl.HS, pl.WPH, B, et, dxb,
                       ldb);
  };
  const int nch = (C + 31) >> 5;
  const bool resident = grid <= 2 * CANON_CUS;
  if constexpr (ACT == ACT_ID) {
    if (resident && nch > 2 && !post_u) {
      launch(canon::k_bwd<ACT, CONCAT, KEEP, 3>);
      return;
    }
  }
  if (resident && nch > 1)
    launch(canon::k_bwd<ACT, CONCAT, KEEP, 2>);
  else
    launch(canon::k_bwd<ACT, CONCAT, KEEP, 1>);
}

// Whether the edge-gradient tail runs for this shape (canonical complete
// graphs, all heads in one workgroup, hl_pad <= 8 columns, even D <= 128 with
// 8-B aligned rows; the d-logit table and the moved tail fit the LDS).
bool attn_canon_edge_tail_ok(int64_t B, int n, int H, int C, int D, int hlp) {
  const CanonBwdPlan pl = canon_bwd_plan(B, H, C, true);
  if (pl.S != 1 || n < 2 || n > 32 || hlp > ET_COLS || hlp < H || D < 1 || D > 128 ||
      (D & 1))
    return false;
  const int E0 = n * (n - 1);
  const int room = pl.HS * 32 * canon::PB + canon::canon_bwd_tail_off(true, pl.HS);
  return E0 * ET_COLS <= room && 4 * ET_COLS * 128 <= room;
}

void attn_canon_bwd(int64_t B, hipStream_t st, const float* dy, const float* y, const float* xs,
                    int ldx, const float* psave, const uint8_t* keep, float keep_scale,
                    const float* post_u, float post_p, const uint32_t* rowmask, float* dxs,
                    float* dae, int ae_edge_order, float* dbias, int n, int H, int C, int concat,
                    int act, float slope, const EdgeTail& et, unsigned short* dxb, int ldb) {
#define SV2N_CB(A, CC, K)                                                                      \
  launch_canon_bwd<A, CC, K>(B, st, dy, y, xs, ldx, psave, keep, keep_scale, post_u, post_p,   \
                             rowmask, dxs, dae, ae_edge_order, dbias, n, H, C, slope, et, dxb, \
                             ldb)
#define SV2N_CB_ACT(CC, K)                 \
  switch (act) {                           \
    case 0: SV2N_CB(0, CC, K); break;      \
    case 1: SV2N_CB(1, CC, K); break;      \
    case 2: SV2N_CB(2, CC, K); break;      \
    default: SV2N_CB(3, CC, K); break;     \
  }
  if (concat) {
    if (keep) { SV2N_CB_ACT(true, true) } else { SV2N_CB_ACT(true, false) }
  } else {
    if (keep) { SV2N_CB_ACT(false, true) } else { SV2N_CB_ACT(false, false) }
  }
#undef SV2N_CB_ACT
#undef SV2N_CB
}

// HEAD: + the layer output [32][OC + 1], two [32] row vectors and the head weights [OC]
size_t attn_canon_fwd_lds(int n, int H, bool has_ae, bool edge_order, int head_oc) {
  const int nae = has_ae ? (edge_order ? n * (n - 1) : n * n) * H : 0;
  return sizeof(float) * ((size_t)canon::sp_floats(H) + 2 * (size_t)H * 32 +
                          (size_t)((nae + 3) & ~3) +
                          (head_oc > 0 ? (size_t)32 * (head_oc + 1) + 64 + head_oc : 0));
}

// the output head fuses into the layer's forward when one workgroup runs each
// graph (its rows and columns all in one place) and the layer output fits LDS
bool attn_canon_head_ok(int64_t B, int n, int H, int C, bool concat) {
  const int OC = concat ? H * C : C;
  // LDS with the layer output, for the larger (dense [n][n]) logit block
  return n >= 1 && n <= 32 && canon_fwd_splits(B, H, C, concat) == 1 && OC <= 512 &&
         attn_canon_fwd_lds(n, H, true, false, OC) <= 160 * 1024;
}

template <int ACT, bool CONCAT, bool KEEP, bool HEAD>
static void launch_canon_fwd(int64_t B, hipStream_t st, const float* xs, int ldx, const float* ae,
                             int ae_edge_order, const uint32_t* rowmask, const float* bias,
                             const uint8_t* keep, float keep_scale, float* y, float* psave,
                             const float* post_u, float post_p, float* post_out, int n, int H,
                             int C, float slope, const HeadFuse& hf) {
  const size_t lds = attn_canon_fwd_lds(n, H, ae != nullptr, ae_edge_order != 0,
                                        HEAD ? (CONCAT ? H * C : C) : 0);
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)canon::k_fwd<ACT, CONCAT, KEEP, HEAD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int S = HEAD ? 1 : canon_fwd_splits(B, H, C, CONCAT);
  hipLaunchKernelGGL((canon::k_fwd<ACT, CONCAT, KEEP, HEAD>), dim3(canon_grid(B, S)),
                     dim3(canon::THREADS), lds, st, xs, ldx, ae, ae_edge_order, rowmask, bias, keep,
                     keep_scale, y, psave, post_u, post_p,
                     post_u ? (float)(1.0 / (1.0 - (double)post_p)) : 1.f, post_out, n, H, C,
                     slope, S, B, hf);
}

void attn_canon_fwd(int64_t B, hipStream_t st, const float* xs, int ldx, const float* ae,
                    int ae_edge_order, const uint32_t* rowmask, const float* bias,
                    const uint8_t* keep, float keep_scale, float* y, float* psave,
                    const float* post_u, float post_p, float* post_out, int n, int H, int C,
                    int concat, int act, float slope, const HeadFuse& hf) {
#define SV2N_CF(A, CC, K)                                                                      \
  {                                                                                            \
    if (hf.w)                                                                                  \
      launch_canon_fwd<A, CC, K, true>(B, st, xs, ldx, ae, ae_edge_order, rowmask, bias, keep, \
                                       keep_scale, y, psave, post_u, post_p, post_out, n, H,   \
                                       C, slope, hf);                                          \
    else                                                                                       \
      launch_canon_fwd<A, CC, K, false>(B, st, xs, ldx, ae, ae_edge_order, rowmask, bias,      \
                                        keep, keep_scale, y, psave, post_u, post_p, post_out,  \
                                        n, H, C, slope, hf);                                   \
  }
#define SV2N_CF_ACT(CC, K)                 \
  switch (act) {                           \
    case 0: SV2N_CF(0, CC, K); break;      \
    case 1: SV2N_CF(1, CC, K); break;      \
    case 2: SV2N_CF(2, CC, K); break;      \
    default: SV2N_CF(3, CC, K); break;     \
  }
  if (concat) {
    if (keep) { SV2N_CF_ACT(true, true) } else { SV2N_CF_ACT(true, false) }
  } else {
    if (keep) { SV2N_CF_ACT(false, true) } else { SV2N_CF_ACT(false, false) }
  }
#undef SV2N_CF_ACT
#undef SV2N_CF
  if (hf.w) {
    const int OC = concat ? H * C : C;
    hipLaunchKernelGGL(canon::k_head_fuse_finish, dim3((unsigned)((OC + 2 + 15) / 16)),
                       dim3(256), 0, st, hf.part, B, OC, 0.5f * hf.inv_n2, hf.gw, hf.gb,
                       hf.loss, hf.loss_sum);
  }
}

}  // namespace sv2n

SV2N_CHK_EXPORT(canon)
