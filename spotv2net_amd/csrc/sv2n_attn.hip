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
#include <algorithm>
#include <cstdlib>

namespace sv2n {

constexpr int ATT_THREADS = 256;
constexpr int TS = 33;  // LDS tile row stride (floats)

typedef float floatx16 __attribute__((ext_vector_type(16)));

// C/D row of accumulator register r for lane half hf (32x32 MFMA layout)
__device__ __forceinline__ int crow(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------------------
// forward
// LDS: sP[H][32][TS] | sA[H][32] | sD[H][32] | sB[XS] (bias of the chunk) |
//      sU = sE[H][32][TS] (edge logits, one row per (head, target)) during the
//      softmax, then sX[32][XS] (one xs chunk: rows j, `span` columns)
// All global loads of a chunk are issued before any store of the launch, so
// no `s_waitcnt vmcnt` ever waits on an output store: gfx950 counts stores on
// the same in-order counter, and a wait for a load issued after a store drains
// the store too (measured: a bias load behind the y stores cost 6 of 33 µs).
// A chunk is heads [h0, h0+hpc) x columns [c0, c0+cw) of each head; the C2
// layers (H·C = 400 / 200) are one chunk, so the whole graph's inputs arrive
// in one memory round trip.
// ---------------------------------------------------------------------------
constexpr int XW = 512;                           // max xs columns per chunk
constexpr int XV = 32 * XW / 4 / ATT_THREADS;     // 16-B register slots per thread
constexpr int AEV = 32 * 32 * SV2N_MAX_HEADS / 4 / ATT_THREADS;  // covers n·n·H for all n, H
constexpr int RPT = SV2N_MAX_HEADS * 64 / ATT_THREADS;            // softmax lane-rows per thread

__host__ __device__ inline int ae_floats(int H) { return H * 32 * TS; }  // sE[h][i][TS]
// chunk row stride: room for a 32-column tile starting at any head slot
__host__ __device__ inline int x_stride(int span) { return ((span + 32 + 3) & ~3) + 4; }

struct FwdChunking {
  int hpc, cw;  // heads per chunk, columns per head per chunk
};
static inline FwdChunking fwd_chunking(int H, int C, bool concat) {
  if (H * C <= XW) return {H, C};
  if (!concat) return {H, (XW / H) & ~31};        // every head, a column window
  if (C <= XW) return {XW / C, C};                // whole heads
  return {1, XW};                                 // one head, a column window
}

template <int ACT, bool CONCAT>
__global__ __launch_bounds__(ATT_THREADS) void k_attn_fwd(
    const float* __restrict__ xs, int ldx, const float* __restrict__ ae, int ae_edge_order,
    const uint32_t* __restrict__ rowmask, const float* __restrict__ bias,
    const uint8_t* __restrict__ keep, float keep_scale, float* __restrict__ y,
    float* __restrict__ psave, int n, int H, int C, float slope, int hpc, int cw) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int XSmax = x_stride(hpc * cw);
  float* sP = smem;
  float* sA = sP + H * 32 * TS;
  float* sD = sA + H * 32;
  float* sB = sD + H * 32;
  float* sE = sB + XSmax;  // sE during the softmax, then sX
  float* sX = sE;

  const int g = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int64_t row0 = (int64_t)g * n;
  const int HC = H * C;
  const int OC = CONCAT ? HC : C;
  const int nhb = (H + hpc - 1) / hpc, ncb = (C + cw - 1) / cw;
  const int nchunk = CONCAT ? nhb * ncb : ncb;
  // chunk group: this workgroup takes chunks cg, cg + ncg, ... of graph g
  // (gridDim.y > 1 spreads one graph over several workgroups); with exactly
  // one head-aligned chunk per workgroup (concat) its softmax covers only
  // that chunk's heads [hs, hs + hn)
  const int cg = blockIdx.y, ncg = gridDim.y;
  const bool own_heads = CONCAT && ncg == nchunk && cw == C && ncg > 1;
  const int hs = own_heads ? (cg / ncb) * hpc : 0;
  const int hn = own_heads ? min(hpc, H - hs) : H;
  const bool write_psave = own_heads || cg == 0;
  const bool row_vec = ((ldx & 3) == 0) && ((((uintptr_t)xs) & 15) == 0);
  const bool contig = cw == C;  // a chunk = contiguous columns [h0*C, (h0+nh)*C) of a row

  // ---- chunk geometry and its loads (addresses clamped, never branched
  //      around: the compiler can then count vmcnt past them) ----
  struct Chunk { int h0, nh, c0, cwv, span; bool vec; };
  auto chunk_of = [&](int ch) {
    Chunk k;
    const int hb = CONCAT ? ch / ncb : 0, cb = CONCAT ? ch - hb * ncb : ch;
    k.h0 = hb * hpc;
    k.nh = min(hpc, H - k.h0);
    k.c0 = cb * cw;
    k.cwv = min(cw, C - k.c0);
    k.span = k.nh * cw;
    k.vec = row_vec && (contig ? (((k.h0 * C) | k.span) & 3) == 0 : (C & 3) == 0);
    return k;
  };
  float4 xr[XV];
  float br[XW / ATT_THREADS];
  const float* xg = xs + row0 * ldx;  // this graph's rows (32-bit offsets below)
  auto load_chunk = [&](const Chunk& k) {
    // opaque copy of the thread index: keeps the compiler from hoisting the
    // per-slot offsets out of the chunk loop (16+ VGPRs held across it)
    int tt = t;
    asm volatile("" : "+v"(tt));
    if (k.vec) {
      const int nq = k.span >> 2;                         // 16-B slots per row
      int j = tt / nq, o4 = tt - j * nq;
      const int dj = ATT_THREADS / nq, do4 = ATT_THREADS - dj * nq;
#pragma unroll
      for (int v = 0; v < XV; ++v) {
        const int o = 4 * o4;
        int col;
        bool ok = j < n;
        if (contig) {
          col = k.h0 * C + o;
        } else {
          const int hh = o / cw, cc = o - hh * cw;
          ok = ok && cc < k.cwv;
          col = (k.h0 + hh) * C + k.c0 + cc;
        }
        const float4 w = *reinterpret_cast<const float4*>(xg + (ok ? j * ldx + col : 0));
        xr[v] = ok ? w : make_float4(0.f, 0.f, 0.f, 0.f);
        o4 += do4;
        j += dj;
        if (o4 >= nq) { o4 -= nq; ++j; }
      }
    }
#pragma unroll
    for (int v = 0; v < XW / ATT_THREADS; ++v) {
      const int o = tt + ATT_THREADS * v;
      const int hh = o / cw, cc = o - hh * cw;
      const bool ok = bias && o < k.span && cc < k.cwv;
      // bias may be NULL (bias=False): read a valid address, discard the value
      const float* bsrc = bias ? bias : xs;
      const float b = bsrc[ok ? (CONCAT ? (k.h0 + hh) * C : 0) + k.c0 + cc : 0];
      br[v] = ok ? b : 0.f;
    }
  };
  // chunk -> sX[j][o] (row stride XS), bias -> sB
  auto store_chunk = [&](const Chunk& k, int XS) {
    int tt = t;
    asm volatile("" : "+v"(tt));
    if (k.vec) {
      const int nq = k.span >> 2;
      int j = tt / nq, o4 = tt - j * nq;
      const int dj = ATT_THREADS / nq, do4 = ATT_THREADS - dj * nq;
#pragma unroll
      for (int v = 0; v < XV; ++v) {
        if (j < 32) *reinterpret_cast<float4*>(sX + j * XS + 4 * o4) = xr[v];
        o4 += do4;
        j += dj;
        if (o4 >= nq) { o4 -= nq; ++j; }
      }
    } else {  // unaligned rows: straight from global (not register-staged)
      for (int e = t; e < 32 * k.span; e += ATT_THREADS) {
        const int j = e / k.span, o = e - j * k.span;
        const int hh = o / cw, cc = o - hh * cw;
        sX[j * XS + o] = (j < n && cc < k.cwv) ? xs[(row0 + j) * ldx + (k.h0 + hh) * C + k.c0 + cc]
                                               : 0.f;
      }
    }
#pragma unroll
    for (int v = 0; v < XW / ATT_THREADS; ++v) {
      const int o = t + ATT_THREADS * v;
      if (o < XS) sB[o] = br[v];
    }
  };

  // ---- every load of the softmax phase, then chunk 0's ----
  // AE block of the graph: canonical edge order [n(n-1)][H] (ae_edge_order,
  // what the edge pass writes for canonical batches: coalesced both ways) or
  // the dense [n][n][H] form (block layouts)
  const int E0 = n * (n - 1);
  const int nae = ae_edge_order ? E0 * H : n * n * H;
  const int nv = (nae + 3) >> 2;  // slots of four elements (the last may be partial)
  const float* aesrc = ae ? ae + (int64_t)g * nae : xs;
  const bool ae_vec = (((uintptr_t)aesrc) & 15) == 0 && (nae & 3) == 0;
  float4 av[AEV];
  if (ae) {
#pragma unroll
    for (int q = 0; q < AEV; ++q) {
      const int k = t + ATT_THREADS * q;
      const int kc = k < nv ? k : 0;
      float4 w;
      if (ae_vec) {
        w = reinterpret_cast<const float4*>(aesrc)[kc];
      } else {  // clamped scalar loads: the tail elements past nae are never scattered
        const int b0 = 4 * kc, lim = nae - 1;
        w.x = aesrc[min(b0, lim)];
        w.y = aesrc[min(b0 + 1, lim)];
        w.z = aesrc[min(b0 + 2, lim)];
        w.w = aesrc[min(b0 + 3, lim)];
      }
      av[q] = w;
    }
  }
  const int ha = t >> 5, ja = t & 31;  // sA/sD slot (t < H*32 <= 256)
  const bool aok = ha < H && ja < n;
  const float* arow = xs + (aok ? (row0 + ja) * ldx + HC + ha : 0);
  const float as_v = arow[0], ad_v = arow[aok ? H : 0];
  // softmax inputs from global: each lane-row's source bitmask and keep bytes
  // (clamped, unconditional loads)
  const int nlr = 64 * hn;  // lane-rows: two lanes per (head, target) row
  uint32_t rbits[RPT], kw[RPT][4];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int rr = t + ATT_THREADS * q;
    const int r = rr >> 1, i = r & 31, h = hs + (r >> 5);
    const bool ok = rr < nlr && i < n;
    const uint32_t* rm = rowmask ? rowmask : reinterpret_cast<const uint32_t*>(xs);
    const uint32_t w = rm[rowmask && ok ? row0 + i : 0];
    rbits[q] = !ok ? 0u : (rowmask ? w & ~(1u << i) : row_bits(nullptr, row0 + i, n, i));
    const uint8_t* kp = keep ? keep : reinterpret_cast<const uint8_t*>(xs);
    const int64_t kb = (keep && ok) ? ((((int64_t)g * H + h) * 32 + i) * 32 + 16 * (rr & 1)) : 0;
#pragma unroll
    for (int w4 = 0; w4 < 4; ++w4) kw[q][w4] = *reinterpret_cast<const uint32_t*>(kp + kb + 4 * w4);
  }

  Chunk cur = chunk_of(cg);  // issued last: only the aggregation waits for it
  load_chunk(cur);

  if (ae && ae_edge_order) {
    // element kk = e*H + h of the edge-ordered block -> sE[h][i][j]
#pragma unroll
    for (int q = 0; q < AEV; ++q) {
      const int kk0 = 4 * (t + ATT_THREADS * q);
      if (kk0 < nae) {
        const float* pa = &av[q].x;
        int e = kk0 / H, h2 = kk0 - e * H;
        CanonIt it;
        it.init(e, n);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (kk0 + c < nae) sE[(h2 * 32 + it.i()) * TS + it.j()] = pa[c];
          if (++h2 == H) { h2 = 0; it.next(n); }
        }
      }
    }
  } else if (ae) {
    // element kk = 4k + e of AE [n][n][H] -> (i, j, h), kk = (i*n + j)*H + h
    const int kb = 4 * t;
    int h = kb % H, ij = kb / H;
    int i = ij / n, jj = ij - i * n;
    const int step = 4 * ATT_THREADS;  // elements per q
    const int sh = step % H, sij = step / H;
    const int si = sij / n, sj = sij - si * n;
#pragma unroll
    for (int q = 0; q < AEV; ++q) {
      const float* pa = &av[q].x;
      int h2 = h, j2 = jj, i2 = i;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (i2 < n) sE[(h2 * 32 + i2) * TS + j2] = pa[e];
        if (++h2 == H) { h2 = 0; if (++j2 == n) { j2 = 0; ++i2; } }
      }
      h += sh;
      if (h >= H) { h -= H; ++jj; }
      jj += sj;
      if (jj >= n) { jj -= n; ++i; }
      i += si;
    }
  }
  if (ha < H) {
    sA[t] = aok ? as_v : 0.f;
    sD[t] = aok ? ad_v : 0.f;
  }
  __syncthreads();

  // ---- per-target softmax: two lanes per (head, target) row, 16 columns each;
  //      the signed probabilities stay in registers until the xs chunk has
  //      left them (a wait for its loads would otherwise drain these stores) ----
  float4 psv[RPT][4];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int rr = t + ATT_THREADS * q;
    if (q * ATT_THREADS >= nlr) break;
    if (rr >= nlr) continue;  // wave-uniform: nlr is a multiple of 64
    const int r = rr >> 1, part = rr & 1;
    const int h = hs + (r >> 5), i = r & 31;
    const int jb = 16 * part;
    const bool rv = i < n;
    const uint32_t bits = rbits[q];
    const uint32_t pb = bits >> jb;  // this lane's 16 columns
    const float* er = sE + (h * 32 + i) * TS + jb;
    const float* ar = sA + h * 32 + jb;
    const float ad = sD[h * 32 + i];
    float ev[16];
    float loopv = 0.f;
    if (ae) {
      float esum = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        ev[c] = ((pb >> c) & 1u) ? er[c] : 0.f;
        esum += ev[c];
      }
      esum += __shfl_xor(esum, 1, 64);
      const int cnt = __popc(bits);
      loopv = cnt > 0 ? esum / (float)cnt : 0.f;
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) ev[c] = 0.f;
    }
    const uint32_t validm = rv ? ((bits | (1u << i)) >> jb) : 0u;
    float lr[16];
    uint32_t negm = 0u;
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const float sv = ar[c] + ad + ((jb + c == i) ? loopv : ev[c]);
      const bool neg = !(sv > 0.f);
      negm |= neg ? (1u << c) : 0u;
      lr[c] = neg ? sv * slope : sv;
      if ((validm >> c) & 1u) mx = fmaxf(mx, lr[c]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
    float den = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      lr[c] = ((validm >> c) & 1u) ? expf(lr[c] - mx) : 0.f;
      den += lr[c];
    }
    den += __shfl_xor(den, 1, 64);
    const float inv = 1.f / (den + 1e-16f);
    float* prow = sP + (h * 32 + i) * TS + jb;
#pragma unroll
    for (int c4 = 0; c4 < 16; c4 += 4) {
      float sq[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = c4 + e;
        const float p = lr[c] * inv;
        const bool valid = (validm >> c) & 1u;
        sq[e] = valid ? (((negm >> c) & 1u) ? -p : p) : 0.f;
        float pd = valid ? p : 0.f;
        if (keep) pd = ((kw[q][c >> 2] >> (8 * (c & 3))) & 0xffu) ? pd * keep_scale : 0.f;
        prow[c] = pd;
      }
      psv[q][c4 >> 2] = make_float4(sq[0], sq[1], sq[2], sq[3]);
    }
  }
  __syncthreads();  // sE dead, sP complete
  store_chunk(cur, x_stride(cur.span));
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int rr = t + ATT_THREADS * q;
    const int r = rr >> 1, h = hs + (r >> 5), i = r & 31;
    if (write_psave && rr < nlr && i < n) {
      float4* dst = reinterpret_cast<float4*>(psave + (((int64_t)g * H + h) * 32 + i) * 32 + 16 * (rr & 1));
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) dst[c4] = psv[q][c4];
    }
  }

  // ---- aggregation per chunk: out[i][c] = Σ_j P[h][i][j] · xs[j][h*C + c] ----
  const float invH = 1.f / (float)H;
  for (int ch = cg; ch < nchunk; ch += ncg) {
    const Chunk k = cur;
    const int XS = x_stride(k.span);
    __syncthreads();
    if (ch + ncg < nchunk) {
      cur = chunk_of(ch + ncg);
      load_chunk(cur);
    }
    const int ntc = (k.cwv + 31) >> 5;  // 32-column tiles per head
    const int ntile = CONCAT ? k.nh * ntc : ntc;
    for (int tl = wave; tl < ntile; tl += ATT_THREADS / 64) {
      const int hh0 = CONCAT ? tl / ntc : 0;
      const int tc = CONCAT ? tl - hh0 * ntc : tl;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const int hh_end = CONCAT ? hh0 + 1 : k.nh;
#pragma unroll 1
      for (int hh = hh0; hh < hh_end; ++hh) {
        const float* prow = sP + ((k.h0 + hh) * 32 + l32) * TS + half;
        const float* xcol = sX + half * XS + hh * cw + 32 * tc + l32;
#pragma unroll
        for (int kk = 0; kk < 16; ++kk)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(prow[2 * kk], xcol[2 * kk * XS], acc, 0, 0, 0);
      }
      const int cc = 32 * tc + l32;
      if (cc < k.cwv) {
        const int oc = (CONCAT ? (k.h0 + hh0) * C : 0) + k.c0 + cc;
        const float b = sB[(CONCAT ? hh0 * cw : 0) + cc];
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
    if (ch + ncg < nchunk) {
      __syncthreads();  // chunk consumed before the next one overwrites sX / sB
      store_chunk(cur, x_stride(cur.span));
    }
  }
}

// ---------------------------------------------------------------------------
// backward
// Per graph: dz = act'(dy, y) (· 1/H for the head mean), then per head h
//   G_h   = X_h · dZ_hᵀ          (dPᵀ, [j][i])            wave h mod 4
//   dxs_h = P_dᵀ · dZ_h           (message/gather bwd)    same wave
// and the softmax / leaky_relu backward of G_h gives dl -> d a_src, d a_dst,
// d ae.  Same memory discipline as the forward: every access is a buffer
// load/store (out-of-range offsets read 0 / drop the store, so nothing is
// branched around and vmcnt is counted), the prologue issues all loads of
// the graph's first chunk at once, and the next chunk's loads are in flight
// while the current chunk's MFMAs run.
// LDS: sP[H][32][TS] (signed saved P) | sKB[H][32] keep bits | sRB[32] row
//      bits | sSh[H][32] (self-loop share) | sDad[H][32] (d a_dst) |
//      area: sX[32][XS] + sZ[32][ZS] per chunk (odd strides: conflict-free
//      column reads), after the chunks sDL[H][32][TS] (dl)
// A chunk is heads [h0, h0+hpc) x columns [c0, c0+cw) of each head.
// ---------------------------------------------------------------------------
constexpr int XB = 224;                                   // max xs columns per chunk
constexpr int BV = 32 * XB / 4 / ATT_THREADS;             // 16-B slots per thread per array
constexpr int PV = SV2N_MAX_HEADS * 1024 / 4 / ATT_THREADS;

struct BwdChunking {
  int hpc, cw;
};
static inline BwdChunking bwd_chunking(int H, int C, bool concat) {
  if (H * C <= XB) return {H, C};
  if ((C & 3) == 0 || !concat) {  // every head, balanced column windows
    const int cwmax = (C & 3) == 0 ? ((XB / H) & ~3) : XB / H;
    const int nch = (C + cwmax - 1) / cwmax;
    int cw = (C + nch - 1) / nch;
    if ((C & 3) == 0) cw = (cw + 3) & ~3;
    return {H, cw};
  }
  if (C <= XB) return {XB / C, C};  // whole heads
  return {1, XB};
}

template <int ACT, bool CONCAT>
__global__ __launch_bounds__(ATT_THREADS) void k_attn_bwd(
    const float* __restrict__ dy, const float* __restrict__ y, const float* __restrict__ xs,
    int ldx, const float* __restrict__ psave, const uint8_t* __restrict__ keep, float keep_scale,
    const uint32_t* __restrict__ rowmask, float* __restrict__ dxs, float* __restrict__ dae,
    int ae_edge_order, float* __restrict__ dbias_part, int n, int H, int C, float slope, int hpc,
    int cw) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int g = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int64_t row0 = (int64_t)g * n;
  const int HC = H * C;
  const int OC = CONCAT ? HC : C;
  const float invH = 1.f / (float)H;
  // head groups: with gridDim.y > 1 this workgroup owns heads [hs, hs + hpc)
  // (the chunks of head block blockIdx.y): every quantity of the backward is
  // then complete inside it (G_h sums over that head's own columns only).
  // Shared per graph (head mean: dz and its bias sums) is written by group 0.
  const int hgi = blockIdx.y, nhg = gridDim.y;
  const int hs = nhg > 1 ? hgi * hpc : 0, hn = nhg > 1 ? min(hpc, H - hs) : H;
  const bool lead = hgi == 0;
  float* sP = smem;
  uint32_t* sKB = reinterpret_cast<uint32_t*>(sP + H * 32 * TS);
  uint32_t* sRB = sKB + H * 32;
  float* sSh = reinterpret_cast<float*>(sRB + 32);
  float* sDad = sSh + H * 32;
  float* sArea = sDad + H * 32;
  float* sDL = sArea;

  const rsrc_t rx = make_rsrc(xs + row0 * ldx, (uint32_t)(n * ldx) * 4u);
  const rsrc_t rdy = make_rsrc(dy + row0 * OC, (uint32_t)(n * OC) * 4u);
  const rsrc_t ry = make_rsrc(y + row0 * OC, (uint32_t)(n * OC) * 4u);
  const rsrc_t rps = make_rsrc(psave + (int64_t)g * H * 1024, (uint32_t)H * 4096u);
  const rsrc_t rkp = make_rsrc(keep ? keep + (int64_t)g * H * 1024 : nullptr,
                               keep ? (uint32_t)H * 1024u : 0u);
  const rsrc_t rrm = make_rsrc(rowmask ? rowmask + row0 : nullptr, rowmask ? (uint32_t)n * 4u : 0u);
  const rsrc_t rdx = make_rsrc(dxs + row0 * ldx, (uint32_t)(n * ldx) * 4u);
  const rsrc_t rdb = make_rsrc(dbias_part + (int64_t)g * OC, (uint32_t)OC * 4u);

  // ---- chunk geometry ----
  const int nhb = (H + hpc - 1) / hpc, ncb = (C + cw - 1) / cw;
  const int ch_begin = nhg > 1 ? hgi * ncb : 0;
  const int nchunk = nhg > 1 ? ch_begin + ncb : nhb * ncb;  // end of this group's chunks
  const bool contig = cw == C;
  struct Chunk { int h0, nh, c0, cwv, span, zw; bool vec; };
  auto chunk_of = [&](int ch) {
    Chunk k;
    const int hb = ch / ncb, cb = ch - hb * ncb;
    k.h0 = hb * hpc;
    k.nh = min(hpc, H - k.h0);
    k.c0 = cb * cw;
    k.cwv = min(cw, C - k.c0);
    k.span = k.nh * cw;
    k.zw = CONCAT ? k.span : cw;
    k.vec = ((ldx | OC) & 3) == 0 &&
            (contig ? (((k.h0 * C) | k.span) & 3) == 0 && (CONCAT || (C & 3) == 0) : (C & 3) == 0);
    return k;
  };
  // xs (+ dy, y) chunk -> registers.  vec: 16-B slots over row spans; else
  // one element per slot component.
  f32x4 xr[BV], dyr[BV], yr[BV];
  auto load_chunk = [&](const Chunk& k) {
    int tt = t;
    asm volatile("" : "+v"(tt));  // keep per-slot offsets out of the chunk loop
    if (k.vec) {
      const int nq = k.span >> 2;
      int j = tt / nq, q = tt - j * nq;
      const int dj = ATT_THREADS / nq, dq = ATT_THREADS - dj * nq;
#pragma unroll
      for (int v = 0; v < BV; ++v) {
        const int L = 4 * q;
        int col;
        bool ok = j < n;
        if (contig) {
          col = k.h0 * C + L;
        } else {
          const int seg = L / cw, cc = L - seg * cw;
          ok = ok && cc < k.cwv;
          col = (k.h0 + seg) * C + k.c0 + cc;
        }
        xr[v] = bld4(rx, ok ? (j * ldx + col) * 4 : OOB);
        if (CONCAT) {
          const int off = ok ? (j * OC + col) * 4 : OOB;
          dyr[v] = bld4(rdy, off);
          yr[v] = bld4(ry, off);
        }
        q += dq;
        j += dj;
        if (q >= nq) { q -= nq; ++j; }
      }
      if (!CONCAT) {
        const int nz = cw >> 2;
        int j2 = tt / nz, q2 = tt - j2 * nz;
        const int dj2 = ATT_THREADS / nz, dq2 = ATT_THREADS - dj2 * nz;
#pragma unroll
        for (int v = 0; v < BV; ++v) {
          const int L = 4 * q2;
          const int off = (j2 < n && L < k.cwv) ? (j2 * OC + k.c0 + L) * 4 : OOB;
          dyr[v] = bld4(rdy, off);
          yr[v] = bld4(ry, off);
          q2 += dq2;
          j2 += dj2;
          if (q2 >= nz) { q2 -= nz; ++j2; }
        }
      }
    } else {
#pragma unroll
      for (int v = 0; v < BV; ++v) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int sl = tt + ATT_THREADS * (4 * v + e);
          const int j = sl / k.span, L = sl - j * k.span;
          const int seg = L / cw, cc = L - seg * cw;
          const bool ok = j < n && cc < k.cwv;
          const int col = (k.h0 + seg) * C + k.c0 + cc;
          xr[v][e] = bld(rx, ok ? (j * ldx + col) * 4 : OOB);
          if (CONCAT) {
            const int off = ok ? (j * OC + col) * 4 : OOB;
            dyr[v][e] = bld(rdy, off);
            yr[v][e] = bld(ry, off);
          } else {
            const int j2 = sl / cw, L2 = sl - j2 * cw;
            const int off = (j2 < n && L2 < k.cwv) ? (j2 * OC + k.c0 + L2) * 4 : OOB;
            dyr[v][e] = bld(rdy, off);
            yr[v][e] = bld(ry, off);
          }
        }
      }
    }
  };
  // registers -> sX[j][L], sZ[j][L] = act'(dy, y)
  auto stage_chunk = [&](const Chunk& k, float* sX, int XS, float* sZ, int ZS) {
    int tt = t;
    asm volatile("" : "+v"(tt));
    if (k.vec) {
      const int nq = k.span >> 2;
      int j = tt / nq, q = tt - j * nq;
      const int dj = ATT_THREADS / nq, dq = ATT_THREADS - dj * nq;
#pragma unroll
      for (int v = 0; v < BV; ++v) {
        if (j < 32) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sX[j * XS + 4 * q + e] = xr[v][e];
            if (CONCAT) sZ[j * ZS + 4 * q + e] = act_bwd<ACT>(dyr[v][e], yr[v][e]);
          }
        }
        q += dq;
        j += dj;
        if (q >= nq) { q -= nq; ++j; }
      }
      if (!CONCAT) {
        const int nz = cw >> 2;
        int j2 = tt / nz, q2 = tt - j2 * nz;
        const int dj2 = ATT_THREADS / nz, dq2 = ATT_THREADS - dj2 * nz;
#pragma unroll
        for (int v = 0; v < BV; ++v) {
          if (j2 < 32) {
#pragma unroll
            for (int e = 0; e < 4; ++e) sZ[j2 * ZS + 4 * q2 + e] = act_bwd<ACT>(dyr[v][e], yr[v][e]);
          }
          q2 += dq2;
          j2 += dj2;
          if (q2 >= nz) { q2 -= nz; ++j2; }
        }
      }
    } else {
#pragma unroll
      for (int v = 0; v < BV; ++v) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int sl = tt + ATT_THREADS * (4 * v + e);
          const int j = sl / k.span, L = sl - j * k.span;
          if (j < 32) {
            sX[j * XS + L] = xr[v][e];
            if (CONCAT) sZ[j * ZS + L] = act_bwd<ACT>(dyr[v][e], yr[v][e]);
          }
          if (!CONCAT) {
            const int j2 = sl / cw, L2 = sl - j2 * cw;
            if (j2 < 32) sZ[j2 * ZS + L2] = act_bwd<ACT>(dyr[v][e], yr[v][e]);
          }
        }
      }
    }
  };

  // ---- prologue: saved P, keep bits, row bits, then chunk 0 ----
  f32x4 pr[PV];
#pragma unroll
  for (int v = 0; v < PV; ++v) {
    const int idx4 = t + ATT_THREADS * v;  // 16-B slot of [h][i][32]
    pr[v] = bld4(rps, (idx4 >> 8) < H ? idx4 * 16 : OOB);
  }
  const bool krow = t < H * 32;  // (h, i) = (t >> 5, t & 31)
  const u32x4 kw0 = bld4_u32(rkp, krow ? t * 32 : OOB);
  const u32x4 kw1 = bld4_u32(rkp, krow ? t * 32 + 16 : OOB);
  const uint32_t rmw = bld_u32(rrm, t < n ? t * 4 : OOB);
  Chunk cur = chunk_of(ch_begin);
  load_chunk(cur);

#pragma unroll
  for (int v = 0; v < PV; ++v) {
    const int idx4 = t + ATT_THREADS * v;
    const int h = idx4 >> 8, i = (idx4 >> 3) & 31, j0 = (idx4 & 7) * 4;
    if (h < H) {
#pragma unroll
      for (int e = 0; e < 4; ++e) sP[(h * 32 + i) * TS + j0 + e] = i < n ? pr[v][e] : 0.f;
    }
  }
  if (krow) {
    uint32_t kb = 0u;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      const uint32_t word = w < 4 ? kw0[w] : kw1[w - 4];
#pragma unroll
      for (int b = 0; b < 4; ++b) kb |= ((word >> (8 * b)) & 0xffu) ? (1u << (4 * w + b)) : 0u;
    }
    sKB[t] = kb;
  }
  if (t < 32) {
    const uint32_t all = (n >= 32) ? 0xffffffffu : ((1u << n) - 1u);
    sRB[t] = t < n ? ((rowmask ? rmw : all) & ~(1u << t)) : 0u;
  }

  // ---- chunks ----
  floatx16 G0, G1;  // G_h for heads wave and wave + 4
#pragma unroll
  for (int r = 0; r < 16; ++r) { G0[r] = 0.f; G1[r] = 0.f; }
  for (int ch = ch_begin; ch < nchunk; ++ch) {
    const Chunk k = cur;
    const int XS = k.span | 1, ZS = k.zw | 1;
    float* sX = sArea;
    float* sZ = sArea + 32 * XS;
    __syncthreads();  // previous chunk consumed (first pass: prologue LDS writes ordered)
    stage_chunk(k, sX, XS, sZ, ZS);
    __syncthreads();
    if (ch + 1 < nchunk) {
      cur = chunk_of(ch + 1);
      load_chunk(cur);
    }
    // bias gradient partials: column sums of dz
    for (int L = t; L < k.zw; L += ATT_THREADS) {
      float sb = 0.f;
#pragma unroll 8
      for (int j = 0; j < 32; ++j) sb += sZ[j * ZS + L];
      const int seg = L / cw, cc = L - seg * cw;
      const int oc = (CONCAT ? (k.h0 + seg) * C : 0) + k.c0 + cc;
      bst(rdb, (cc < k.cwv && (CONCAT || lead)) ? oc * 4 : OOB, sb);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int h = wave + 4 * s2;
      const int hh = h - k.h0;
      if (hh < 0 || hh >= k.nh) continue;  // wave-uniform
      floatx16 G = s2 ? G1 : G0;
      const int zoff = CONCAT ? hh * cw : 0;
      const float* xa = sX + l32 * XS + hh * cw + half;
      const float* zb = sZ + l32 * ZS + zoff + half;
      const int nk = (k.cwv + 1) >> 1;
      for (int kk = 0; kk < nk; ++kk) {
        const bool cv = 2 * kk + half < k.cwv;
        const float a = cv ? xa[2 * kk] : 0.f;
        const float b = cv ? (CONCAT ? zb[2 * kk] : zb[2 * kk] * invH) : 0.f;
        G = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, G, 0, 0, 0);
      }
      if (s2) G1 = G; else G0 = G;
      // dxs tiles: D[j][c] = Σ_i P_d[i][j] · dZ[i][c]
      const uint32_t* kbh = sKB + h * 32;
      const float* ph = sP + h * 32 * TS + l32;
      const int ntc = (k.cwv + 31) >> 5;
      for (int tc = 0; tc < ntc; ++tc) {
        floatx16 D;
#pragma unroll
        for (int r = 0; r < 16; ++r) D[r] = 0.f;
        const float* zc = sZ + half * ZS + zoff + 32 * tc + l32;
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
          const int ii = 2 * kk + half;
          float a = fabsf(ph[ii * TS]);
          if (keep) a = ((kbh[ii] >> l32) & 1u) ? a * keep_scale : 0.f;
          const float b = CONCAT ? zc[2 * kk * ZS] : zc[2 * kk * ZS] * invH;
          D = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, D, 0, 0, 0);
        }
        const int cl = 32 * tc + l32;
        const int gcol = h * C + k.c0 + cl;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int jr = crow(r, half);
          bst(rdx, (cl < k.cwv && jr < n) ? (jr * ldx + gcol) * 4 : OOB, D[r]);
        }
      }
    }
  }
  __syncthreads();  // chunk area dead: sDL

  // ---- softmax + leaky_relu backward of G_h: lane column i, rows j = crow(r, half) ----
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int h = wave + 4 * s2;
    if (h >= H || h < hs || h >= hs + hn) continue;  // wave-uniform
    const floatx16 G = s2 ? G1 : G0;
    const int i = l32;
    const bool iv = i < n;
    const uint32_t bits = sRB[i];
    const uint32_t kb = keep ? sKB[h * 32 + i] : 0xffffffffu;
    const float* prw = sP + (h * 32 + i) * TS;
    float ps[16], dp[16];
    float tl = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jr = crow(r, half);
      ps[r] = prw[jr];
      const bool valid = iv && jr < n && (jr == i || ((bits >> jr) & 1u));
      float d = valid ? G[r] : 0.f;
      if (keep) d = ((kb >> jr) & 1u) ? d * keep_scale : 0.f;
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
      const float ds = fabsf(ps[r]) * (dp[r] - tl);
      dl[r] = valid ? (signbit(ps[r]) ? ds * slope : ds) : 0.f;
      dad += dl[r];
    }
    dad += __shfl_xor(dad, 32, 64);
    // dl[i][i] sits in half (i>>2)&1, register (i&3) + 4*(i>>3)
    const int hi = (i >> 2) & 1, ri = (i & 3) + 4 * (i >> 3);
    float mine = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) mine = (r == ri) ? dl[r] : mine;
    const float other = __shfl_xor(mine, 32, 64);
    const float dlii = (half == hi) ? mine : other;
    if (half == 0) {
      const int cnt = __popc(bits);
      sDad[h * 32 + i] = dad;
      sSh[h * 32 + i] = cnt > 0 ? dlii / (float)cnt : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) sDL[(h * 32 + i) * TS + crow(r, half)] = dl[r];
  }
  __syncthreads();

  // ---- d ae, canonical edge order [n(n-1)][H]: complete graph, every (i, j != i) ----
  if (dae && ae_edge_order) {
    const int nae = n * (n - 1) * H;
    const rsrc_t rdae = make_rsrc(dae + (int64_t)g * nae, (uint32_t)nae * 4u);
    if (nhg == 1 && (nae & 3) == 0 && ((((uintptr_t)dae) & 15) == 0)) {
      for (int k4 = 4 * t; k4 < nae; k4 += 4 * ATT_THREADS) {
        int e = k4 / H, h = k4 - e * H;
        CanonIt it;
        it.init(e, n);
        f32x4 v;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int i = it.i();
          v[c] = sDL[(h * 32 + i) * TS + it.j()] + sSh[h * 32 + i];
          if (++h == H) { h = 0; it.next(n); }
        }
        bst4(rdae, k4 * 4, v);
      }
    } else {
      for (int kk = t; kk < nae; kk += ATT_THREADS) {
        const int e = kk / H, h = kk - e * H;
        int i, j;
        canon_decode(e, n, i, j);
        const bool own = h >= hs && h < hs + hn;
        bst(rdae, own ? kk * 4 : OOB, own ? sDL[(h * 32 + i) * TS + j] + sSh[h * 32 + i] : 0.f);
      }
    }
  } else if (dae) {
    // ---- d ae: the graph's [n][n][H] block, four elements per slot ----
    const int nae = n * n * H;
    const rsrc_t rdae = make_rsrc(dae + row0 * n * H, (uint32_t)nae * 4u);
    auto dae_val = [&](int i, int j, int h) {
      const bool e = j != i && ((sRB[i] >> j) & 1u);
      return e ? sDL[(h * 32 + i) * TS + j] + sSh[h * 32 + i] : 0.f;
    };
    if (nhg == 1 && (nae & 3) == 0 && ((((uintptr_t)dae) & 15) == 0)) {
      const int kb = 4 * t;
      int h = kb % H, ij = kb / H;
      int i = ij / n, j = ij - i * n;
      const int step = 4 * ATT_THREADS;
      const int sh = step % H, sij = step / H;
      const int si = sij / n, sj = sij - si * n;
      for (int k4 = kb; k4 < nae; k4 += step) {
        f32x4 v;
        int h2 = h, j2 = j, i2 = i;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = dae_val(i2, j2, h2);
          if (++h2 == H) { h2 = 0; if (++j2 == n) { j2 = 0; ++i2; } }
        }
        bst4(rdae, k4 * 4, v);
        h += sh;
        if (h >= H) { h -= H; ++j; }
        j += sj;
        if (j >= n) { j -= n; ++i; }
        i += si;
      }
    } else {
      for (int kk = t; kk < nae; kk += ATT_THREADS) {
        const int h = kk % H, ij = kk / H;
        const int i = ij / n, j = ij - i * n;
        const bool own = h >= hs && h < hs + hn;
        bst(rdae, own ? kk * 4 : OOB, own ? dae_val(i, j, h) : 0.f);
      }
    }
  }
  // ---- dxs columns [HC, ldx): d a_src (Σ_i dl[i][j]), d a_dst, zero padding ----
  const int ntail = ldx - HC;
  for (int e = t; e < n * ntail; e += ATT_THREADS) {
    const int j = e / ntail, c2 = e - j * ntail;
    float v = 0.f;
    const int hc = c2 < H ? c2 : c2 - H;  // the head of a d a_src / d a_dst column
    const bool own = c2 < 2 * H ? (hc >= hs && hc < hs + hn) : lead;
    if (c2 < H) {
      const float* col = sDL + c2 * 32 * TS + j;
#pragma unroll 8
      for (int ii = 0; ii < 32; ++ii) v += col[ii * TS];
    } else if (c2 < 2 * H) {
      v = sDad[(c2 - H) * 32 + j];
    }
    bst(rdx, own ? (j * ldx + HC + c2) * 4 : OOB, v);
  }
}

}  // namespace sv2n

// ============================ C-ABI ========================================
using namespace sv2n;

namespace sv2n {
// sv2n_attn_canon.hip: complete graphs in canonical edge order
void attn_canon_fwd(int64_t B, hipStream_t st, const float* xs, int ldx, const float* ae,
                    int ae_edge_order, const uint32_t* rowmask, const float* bias,
                    const uint8_t* keep, float keep_scale, float* y, float* psave, int n, int H,
                    int C, int concat, int act, float slope);
void attn_canon_bwd(int64_t B, hipStream_t st, const float* dy, const float* y, const float* xs,
                    int ldx, const float* psave, const uint8_t* keep, float keep_scale,
                    const uint32_t* rowmask, float* dxs, float* dae, int ae_edge_order,
                    float* dbias, int n, int H, int C, int concat, int act, float slope);
}  // namespace sv2n

// The lean kernels (sv2n_attn_canon.hip) take every n <= 32 launch — canonical
// batches (edge logits in edge order) and block layouts (row masks, dense
// [n][n][H] logits) — unless SV2N_ATTN_CANON=0 (A/B switch: the kernels below).
static bool canon_path(int n, int H) {
  static const bool on = [] {
    const char* e = getenv("SV2N_ATTN_CANON");
    return !(e && e[0] == '0');
  }();
  return on && n >= 1 && n <= 32 && H <= 8;
}

static size_t fwd_lds(int H, FwdChunking ck) {
  const size_t xs = (size_t)x_stride(ck.hpc * ck.cw);
  return sizeof(float) * ((size_t)H * 32 * TS + 2 * (size_t)H * 32 + xs +
                          std::max((size_t)ae_floats(H), 32 * xs));
}
static size_t bwd_lds(int H, BwdChunking ck, bool concat) {
  const size_t span = (size_t)ck.hpc * ck.cw;
  const size_t area = 32 * ((span | 1) + ((concat ? span : (size_t)ck.cw) | 1)) + 32;
  return sizeof(float) * ((size_t)H * 32 * TS + 4 * (size_t)H * 32 + 32 +
                          std::max(area, (size_t)H * 32 * TS));
}

template <typename K>
static void raise_lds(K kernel, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
}

// Workgroups per graph for the forward.  A graph whose xs span needs several
// sequential chunks (C3: 6 heads x 500 columns, 8 chunks) is spread over up to
// ncg workgroups (tools/attn_sweep.py, MI355X: C3 69 -> 61 us).  Single-chunk
// graphs (C2) stay one workgroup each: splitting them (head groups, column
// windows) only repeats the per-graph softmax chain (C2 L0 24 -> 32 us,
// L1 18 -> 39 us).
static int64_t att_target_wg() {
  static int64_t v = [] {
    const char* e = getenv("SV2N_ATT_TARGET_WG");  // tuning override (0: no split)
    return e ? (int64_t)atoll(e) : (int64_t)1024;
  }();
  return v;
}
struct FwdSplit { FwdChunking ck; int ncg; };
static inline FwdSplit fwd_split(int64_t B, int H, int C, bool concat) {
  FwdChunking ck = fwd_chunking(H, C, concat);
  const int ncb = (C + ck.cw - 1) / ck.cw;
  int nchunk = concat ? ((H + ck.hpc - 1) / ck.hpc) * ncb : ncb;
  const int64_t target = att_target_wg();
  const int want = target <= 0 ? 1 : (int)std::min<int64_t>(8, (target + B - 1) / B);
  if (want <= 1 || nchunk == 1) return {ck, 1};
  return {ck, std::min(want, nchunk)};
}

template <int ACT, bool CONCAT>
static void launch_fwd(int64_t B, hipStream_t st, const float* xs, int ldx, const float* ae,
                       int ae_edge_order, const uint32_t* rowmask, const float* bias, const uint8_t* keep,
                       float keep_scale, float* y, float* psave, int n, int H, int C, float slope) {
  const FwdSplit sp = fwd_split(B, H, C, CONCAT);
  const size_t lds = fwd_lds(H, sp.ck);
  raise_lds(k_attn_fwd<ACT, CONCAT>, lds);
  hipLaunchKernelGGL((k_attn_fwd<ACT, CONCAT>), dim3((unsigned)B, (unsigned)sp.ncg),
                     dim3(ATT_THREADS), lds, st, xs, ldx, ae, ae_edge_order, rowmask, bias, keep, keep_scale, y,
                     psave, n, H, C, slope, sp.ck.hpc, sp.ck.cw);
}

// Head groups for the backward: a graph whose backward walks many sequential
// chunks (C3: 14 column windows of all 6 heads) is split into head groups, each
// workgroup owning hpc heads and walking only their columns — no cross-
// workgroup reduction (G_h of a head sums over that head's columns alone), at
// the price of re-reading dy / y per group for a head mean.
static int att_bwd_hpc(int H) {
  static int v = [] {
    const char* e = getenv("SV2N_ATT_BWD_HPC");  // tuning override: heads per group
    return e ? atoi(e) : -1;
  }();
  // default: two head groups (tools/attn_sweep.py, C3 shapes on MI355X: bwd
  // 190 us unsplit, 150 / 103 / 95 us at 1 / 2 / 3 heads per group)
  return v >= 0 ? v : (H + 1) / 2;
}
struct BwdSplit { BwdChunking ck; int nhg; };
static inline BwdSplit bwd_split(int64_t B, int H, int C, bool concat) {
  const BwdChunking ck = bwd_chunking(H, C, concat);
  const int nchunk = ((H + ck.hpc - 1) / ck.hpc) * ((C + ck.cw - 1) / ck.cw);
  const int hpc = att_bwd_hpc(H);
  if (nchunk < 4 || hpc <= 0 || hpc >= H || B * ((H + hpc - 1) / hpc) > 4096 ||
      (C & 3) != 0)
    return {ck, 1};
  // head-aligned chunks of hpc heads, balanced column windows within XB
  const int cwmax = (XB / hpc) & ~3;
  const int nch = (C + cwmax - 1) / cwmax;
  const int cw = (((C + nch - 1) / nch) + 3) & ~3;
  return {{hpc, cw}, (H + hpc - 1) / hpc};
}

template <int ACT, bool CONCAT>
static void launch_bwd(int64_t B, hipStream_t st, const float* dy, const float* y,
                       const float* xs, int ldx, const float* psave, const uint8_t* keep,
                       float keep_scale, const uint32_t* rowmask, float* dxs, float* dae,
                       int ae_edge_order, float* dbias, int n, int H, int C, float slope) {
  const BwdSplit sp = bwd_split(B, H, C, CONCAT);
  const size_t lds = bwd_lds(H, sp.ck, CONCAT);
  raise_lds(k_attn_bwd<ACT, CONCAT>, lds);
  hipLaunchKernelGGL((k_attn_bwd<ACT, CONCAT>), dim3((unsigned)B, (unsigned)sp.nhg),
                     dim3(ATT_THREADS), lds, st, dy, y, xs, ldx, psave, keep, keep_scale, rowmask,
                     dxs, dae, ae_edge_order, dbias, n, H, C, slope, sp.ck.hpc, sp.ck.cw);
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

extern "C" int sv2n_gat_attn_fwd(const float* xs, int ldx, const float* ae, int ae_edge_order,
                                 const uint32_t* rowmask, const float* bias, const uint8_t* keep,
                                 float keep_scale, float* y, float* psave, int64_t num_graphs,
                                 int n, int heads, int channels, int concat, int act,
                                 float negative_slope, hipStream_t stream) {
  if (!xs || !y || !psave) return SV2N_ERR_ARG;
  if (int rc = check_attn_args(num_graphs, n, heads, channels, ldx, act)) return rc;
  if (ae_edge_order && (rowmask || n < 2)) return SV2N_ERR_ARG;  // complete graphs only
  if (canon_path(n, heads)) {
    attn_canon_fwd(num_graphs, stream, xs, ldx, ae, ae_edge_order, rowmask, bias, keep,
                   keep_scale, y, psave, n, heads, channels, concat, act, negative_slope);
    return (int)hipGetLastError();
  }
  if (concat) {
    SV2N_DISPATCH_ACT(launch_fwd, true, num_graphs, stream, xs, ldx, ae, ae_edge_order, rowmask,
                      bias, keep, keep_scale, y, psave, n, heads, channels, negative_slope)
  } else {
    SV2N_DISPATCH_ACT(launch_fwd, false, num_graphs, stream, xs, ldx, ae, ae_edge_order, rowmask,
                      bias, keep, keep_scale, y, psave, n, heads, channels, negative_slope)
  }
  return (int)hipGetLastError();
}

extern "C" int sv2n_gat_attn_bwd(const float* dy, const float* y, const float* xs, int ldx,
                                 const float* psave, const uint8_t* keep, float keep_scale,
                                 const uint32_t* rowmask, float* dxs, float* dae,
                                 int ae_edge_order, float* dbias_partial, int64_t num_graphs, int n,
                                 int heads, int channels, int concat, int act,
                                 float negative_slope, hipStream_t stream) {
  if (!dy || !y || !xs || !psave || !dxs || !dbias_partial) return SV2N_ERR_ARG;
  if (int rc = check_attn_args(num_graphs, n, heads, channels, ldx, act)) return rc;
  if (ae_edge_order && (rowmask || n < 2)) return SV2N_ERR_ARG;  // complete graphs only
  if (canon_path(n, heads)) {
    attn_canon_bwd(num_graphs, stream, dy, y, xs, ldx, psave, keep, keep_scale, rowmask, dxs,
                   dae, ae_edge_order, dbias_partial, n, heads, channels, concat, act,
                   negative_slope);
    return (int)hipGetLastError();
  }
  if (concat) {
    SV2N_DISPATCH_ACT(launch_bwd, true, num_graphs, stream, dy, y, xs, ldx, psave, keep,
                      keep_scale, rowmask, dxs, dae, ae_edge_order, dbias_partial, n, heads,
                      channels, negative_slope)
  } else {
    SV2N_DISPATCH_ACT(launch_bwd, false, num_graphs, stream, dy, y, xs, ldx, psave, keep,
                      keep_scale, rowmask, dxs, dae, ae_edge_order, dbias_partial, n, heads,
                      channels, negative_slope)
  }
  return (int)hipGetLastError();
}
