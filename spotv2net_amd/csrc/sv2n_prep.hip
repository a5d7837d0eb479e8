// Weight preparation for the fused GAT stack, and its backward.
//
// Forward (one launch per layer):
//   Waug[ldx][F] = [ W_src ; W_srcᵀatt_src (H rows) ; W_srcᵀatt_dst (H rows) ; 0 ]
//   wfold[d][col0+h] = Σ_c att_edge[h,c] · W_edge[h*C+c][d]
// so the projection GEMM also emits PyG's alpha_src / alpha_dst
// ((x_src*att_src).sum(-1), GATConv.forward) and the edge pass needs one D x H
// matrix per layer instead of lin_edge's [E, H*C] output.
//
// Backward: the projection GEMM produces T = dWaugᵀ [F][ldx]; the fold is
// undone here and the parameter gradients are ACCUMULATED into p.grad:
//   gW[hC+c][f]   += T[f][hC+c] + T[f][HC+h]·att_src[h,c] + T[f][HC+H+h]·att_dst[h,c]
//   g_att_src[h,c] += Σ_f T[f][HC+h] · W[hC+c][f]       (same for dst)
//   gW_e[hC+c][d] += dwfold[d][col0+h] · att_edge[h,c]
//   g_att_edge[h,c] += Σ_d W_e[hC+c][d] · dwfold[d][col0+h]
//   g_bias[o]     += Σ_g dbias_partial[g][o]
#include <algorithm>
#include "sv2n_common.h"
#include "sv2n_gemm3_kernel.h"

namespace sv2n {

// ---------------------------------------------------------------------------
// Forward prep blocks.  A block owns 64 columns (f, or d for the edge fold) of
// one head; its 256 threads are 16 row groups x 16 lanes of 4 columns each.
// Row c of the head belongs to group c % 16; a group walks its rows in
// increasing c, RB rows per round with all their loads in flight, and the
// 16 group partials of a fold are added in a fixed tree (fold_tree16).  The
// same order is used wherever a fold row is recomputed (the T blocks of
// k_prep_fwd_all), so every copy of a fold row is bit-identical.  Depth:
// ceil(C / (16·RB)) rounds (C3: C = 500, 4 rounds; 4 groups of one column per
// lane took 125 dependent rows per thread, 38 us).
// ---------------------------------------------------------------------------
constexpr int PREP_G = 16, PREP_RB = 8;

__device__ __forceinline__ void put3(uint16_t* planes, int64_t plane, int64_t idx, float v,
                                     int np = 3) {
  unsigned short h0, h1, h2;
  split3(v, h0, h1, h2);
  planes[idx] = h0;
  if (np == 3) {
    planes[plane + idx] = h1;
    planes[2 * plane + idx] = h2;
  }
}

__device__ __forceinline__ float fold_tree16(const float* v, int stride) {
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = v[(2 * i) * stride] + v[(2 * i + 1) * stride];
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// rows [cb, ce) of head h copied (waug when given; planes when given: kp columns, zero
// past F); with fold, the att_src / att_dst folds over ALL C rows written to
// waug rows HC+h and HC+H+h (and their planes).  cols: F (node) or D (edge).
struct PrepBlock {
  const float* W; const float* att_s; const float* att_d; int H, C, F, ldx;
  float* waug; uint16_t* planes; int64_t kp, plane; int np;
};

// one row piece (4 columns) of waug (when given) and its bf16 planes; 16-B / 8-B stores when
// the piece lies inside the row
__device__ __forceinline__ void prep_put_piece(const PrepBlock& P, int64_t row, int col,
                                               const float (&w)[4]) {
  const int F = P.F;
  if (P.waug && (F & 3) == 0 && col + 3 < F) {
    *reinterpret_cast<f32x4*>(P.waug + row * F + col) = f32x4{w[0], w[1], w[2], w[3]};
  } else if (P.waug) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (col + j < F) P.waug[row * F + col + j] = w[j];
  }
  if (!P.planes) return;
  if ((P.kp & 3) == 0 && col + 3 < P.kp) {
    unsigned short h[3][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) split3(w[j], h[0][j], h[1][j], h[2][j]);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (q > 0 && P.np != 3) break;
      const uint32_t lo = (uint32_t)h[q][0] | ((uint32_t)h[q][1] << 16);
      const uint32_t hi = (uint32_t)h[q][2] | ((uint32_t)h[q][3] << 16);
      *reinterpret_cast<uint2*>(P.planes + q * P.plane + row * P.kp + col) = make_uint2(lo, hi);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (col + j < P.kp) put3(P.planes, P.plane, row * P.kp + col + j, w[j], P.np);
  }
}

__device__ __forceinline__ void prep_node_block(const PrepBlock& P, int h, int col0, int cb, int ce,
                                                bool fold, float (*s_red)[PREP_G][64], int t) {
  const int g = t >> 4, lq = t & 15, col = col0 + 4 * lq;
  const int C = P.C, F = P.F, HC = P.H * P.C;
  float ss[4] = {0.f, 0.f, 0.f, 0.f}, sd[4] = {0.f, 0.f, 0.f, 0.f};
  const int cs = fold ? 0 : cb, cend = fold ? C : ce;
  const int first = cs + ((g - cs) % PREP_G + PREP_G) % PREP_G;
  const bool vec = (F & 3) == 0 && col + 3 < F;
  // the next round's rows are loaded before this round's stores (software
  // pipelined: one memory round trip per round overlapped with the stores)
  auto load = [&](int c0, float (&w)[PREP_RB][4], float (&as)[PREP_RB], float (&ad)[PREP_RB]) {
#pragma unroll
    for (int u = 0; u < PREP_RB; ++u) {
      const int c = min(c0 + PREP_G * u, C - 1);
      const int64_t row = (int64_t)h * C + c;
      if (vec) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(P.W + row * F + col);
#pragma unroll
        for (int j = 0; j < 4; ++j) w[u][j] = v[j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) w[u][j] = col + j < F ? P.W[row * F + col + j] : 0.f;
      }
      as[u] = P.att_s[row];
      ad[u] = P.att_d[row];
    }
  };
  float w[PREP_RB][4], as[PREP_RB], ad[PREP_RB];
  if (first < cend) load(first, w, as, ad);
  for (int c0 = first; c0 < cend; c0 += PREP_G * PREP_RB) {
    const bool more = c0 + PREP_G * PREP_RB < cend;
    float wn[PREP_RB][4], asn[PREP_RB], adn[PREP_RB];
    if (more) load(c0 + PREP_G * PREP_RB, wn, asn, adn);
#pragma unroll
    for (int u = 0; u < PREP_RB; ++u) {
      const int c = c0 + PREP_G * u;
      if (c < cend) {
        const int64_t row = (int64_t)h * C + c;
        if (c >= cb && c < ce) prep_put_piece(P, row, col, w[u]);
        if (fold) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            ss[j] = fmaf(as[u], w[u][j], ss[j]);
            sd[j] = fmaf(ad[u], w[u][j], sd[j]);
          }
        }
      }
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < PREP_RB; ++u) {
        as[u] = asn[u];
        ad[u] = adn[u];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[u][j] = wn[u][j];
      }
    }
  }
  if (!fold) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s_red[0][g][4 * lq + j] = ss[j];
    s_red[1][g][4 * lq + j] = sd[j];
  }
  __syncthreads();
  if (t < 128) {
    const int q = t >> 6, cl = t & 63, c = col0 + cl;
    const float v = fold_tree16(&s_red[q][0][cl], 64);
    const int64_t row = HC + q * P.H + h;
    if (P.waug && c < F) P.waug[row * F + c] = v;
    if (P.planes && c < P.kp) put3(P.planes, P.plane, row * P.kp + c, v, P.np);
  }
  if (h == 0) {  // zero padding rows
    for (int k = t; k < (P.ldx - HC - 2 * P.H) * 64; k += 256) {
      const int64_t row = HC + 2 * P.H + k / 64;
      const int c = col0 + (k & 63);
      if (P.waug && c < F) P.waug[row * F + c] = 0.f;
      if (P.planes && c < P.kp) put3(P.planes, P.plane, row * P.kp + c, 0.f, P.np);
    }
  }
}

// wfold[d][col0h + h] = Σ_c att_edge[h,c] · W_edge[h*C+c][d], columns [col0, col0+64)
__device__ __forceinline__ void prep_edge_block(const float* We, const float* att_e, int C, int D,
                                                int h, int col0, float* wfold, int hlp, int col0h,
                                                float (*s_red)[PREP_G][64], int t) {
  const int g = t >> 4, lq = t & 15, col = col0 + 4 * lq;
  float se[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = g; c0 < C; c0 += PREP_G * PREP_RB) {
    float w[PREP_RB][4], ae[PREP_RB];
#pragma unroll
    for (int u = 0; u < PREP_RB; ++u) {
      const int64_t row = (int64_t)h * C + min(c0 + PREP_G * u, C - 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) w[u][j] = col + j < D ? We[row * D + col + j] : 0.f;
      ae[u] = att_e[row];
    }
#pragma unroll
    for (int u = 0; u < PREP_RB; ++u)
      if (c0 + PREP_G * u < C)
#pragma unroll
        for (int j = 0; j < 4; ++j) se[j] = fmaf(ae[u], w[u][j], se[j]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) s_red[0][g][4 * lq + j] = se[j];
  __syncthreads();
  if (t < 64 && col0 + t < D)
    wfold[(int64_t)(col0 + t) * hlp + col0h + h] = fold_tree16(&s_red[0][0][t], 64);
}

// grid (ceil(max(F, D)/64), 2H), block 256: one P block per (64 columns, head)
__global__ __launch_bounds__(256) void k_prep_fwd(const float* __restrict__ W,
                                                  const float* __restrict__ att_s,
                                                  const float* __restrict__ att_d, int H, int C,
                                                  int F, float* __restrict__ waug, int ldx,
                                                  const float* __restrict__ We,
                                                  const float* __restrict__ att_e, int D,
                                                  float* __restrict__ wfold, int hlp, int col0) {
  __shared__ float s_red[2][PREP_G][64];
  const int y = blockIdx.y, c0 = blockIdx.x * 64;
  if (y < H) {
    if (c0 >= F) return;
    const PrepBlock P{W, att_s, att_d, H, C, F, ldx, waug, nullptr, 0, 0, 1};
    prep_node_block(P, y, c0, 0, C, true, s_red, threadIdx.x);
  } else {
    if (!We || c0 >= D) return;
    prep_edge_block(We, att_e, C, D, y - H, c0, wfold, hlp, col0, s_red, threadIdx.x);
  }
}

// gW[o][f] += T[f][o] + T[f][HC+h]·att_s[o] + T[f][HC+H+h]·att_d[o], o = h*C+c
// 64(f) x 64(o) tiles transposed through LDS; grid (ceil(F/64), ceil(HC/64)).
__global__ __launch_bounds__(256) void k_prep_bwd_w(const float* __restrict__ T, int ldx,
                                                    const float* __restrict__ att_s,
                                                    const float* __restrict__ att_d, int H, int C,
                                                    int F, float* __restrict__ gW,
                                                    float* __restrict__ g2) {
  __shared__ float tile[64][65];
  __shared__ float sfold[64][2 * SV2N_MAX_HEADS];
  const int HC = H * C;
  const int f0 = blockIdx.x * 64, o0 = blockIdx.y * 64;
  const int t = threadIdx.x;
  for (int idx = t; idx < 64 * 64; idx += 256) {
    const int fr = idx >> 6, oc = idx & 63;
    const int f = f0 + fr, o = o0 + oc;
    tile[fr][oc] = (f < F && o < HC) ? T[(int64_t)f * ldx + o] : 0.f;
  }
  for (int idx = t; idx < 64 * 2 * H; idx += 256) {
    const int fr = idx / (2 * H), k = idx - fr * 2 * H;
    const int f = f0 + fr;
    sfold[fr][k] = (f < F) ? T[(int64_t)f * ldx + HC + k] : 0.f;
  }
  __syncthreads();
  if (blockIdx.y == 0 && g2) {  // compact fold gradients for k_prep_bwd_att: g2[k][f]
    for (int idx = t; idx < 64 * 2 * H; idx += 256) {
      const int k = idx >> 6, fc = idx & 63;
      if (f0 + fc < F) g2[(int64_t)k * F + f0 + fc] = sfold[fc][k];
    }
  }
  if (!gW) return;
  for (int idx = t; idx < 64 * 64; idx += 256) {
    const int orow = idx >> 6, fc = idx & 63;
    const int o = o0 + orow, f = f0 + fc;
    if (o < HC && f < F) {
      const int h = o / C;
      const float v = tile[fc][orow] + sfold[fc][h] * att_s[o] + sfold[fc][H + h] * att_d[o];
      gW[(int64_t)o * F + f] += v;
    }
  }
}

// one wave per row o = h*C+c (grid ceil(HC/4)): g_att_src[o] += Σ_f g2[h][f]·W[o][f],
// g_att_dst[o] += Σ_f g2[H+h][f]·W[o][f]
__global__ __launch_bounds__(256) void k_prep_bwd_att(const float* __restrict__ g2,
                                                      const float* __restrict__ W, int H, int C,
                                                      int F, float* __restrict__ g_att_s,
                                                      float* __restrict__ g_att_d) {
  const int lane = threadIdx.x & 63;
  const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (o >= H * C) return;
  const int h = o / C;
  const float* wr = W + (int64_t)o * F;
  const float* fs = g2 + (int64_t)h * F;
  const float* fd = g2 + (int64_t)(H + h) * F;
  float a = 0.f, b = 0.f;
  for (int f = lane; f < F; f += 64) {
    const float w = wr[f];
    a = fmaf(fs[f], w, a);
    b = fmaf(fd[f], w, b);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    a += __shfl_xor(a, m, 64);
    b += __shfl_xor(b, m, 64);
  }
  if (lane == 0) {
    if (g_att_s) g_att_s[o] += a;
    if (g_att_d) g_att_d[o] += b;
  }
}

// one wave per row o = h*C+c (grid ceil(HC/4)): gW_e[o][d] += dwfold[d][col0+h]·att_e[o],
// g_att_edge[o] += Σ_d W_e[o][d]·dwfold[d][col0+h]
__global__ __launch_bounds__(256) void k_prep_bwd_edge(const float* __restrict__ dwfold, int hlp,
                                                       int col0, const float* __restrict__ We,
                                                       const float* __restrict__ att_e, int H,
                                                       int C, int D, float* __restrict__ gWe,
                                                       float* __restrict__ g_att_e) {
  const int lane = threadIdx.x & 63;
  const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (o >= H * C) return;
  const int h = o / C;
  const float ae = att_e[o];
  float a = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float g = dwfold[(int64_t)d * hlp + col0 + h];
    a = fmaf(We[(int64_t)o * D + d], g, a);
    if (gWe) gWe[(int64_t)o * D + d] += g * ae;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) a += __shfl_xor(a, m, 64);
  if (lane == 0 && g_att_e) g_att_e[o] += a;
}

// every layer in one launch: blockIdx.y = layer (same body, same order)
struct PrepBwdEdgeArgs {
  sv2n_edge_grad_layer l[SV2N_MAX_LAYERS];
};
__global__ __launch_bounds__(256) void k_prep_bwd_edge_all(const float* __restrict__ dwfold,
                                                           int hlp, int D, const PrepBwdEdgeArgs args) {
  const sv2n_edge_grad_layer& P = args.l[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int C = P.channels;
  if (o >= P.heads * C) return;
  const int h = o / C;
  const float ae = P.att_edge[o];
  float a = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float g = dwfold[(int64_t)d * hlp + P.col0 + h];
    a = fmaf(P.W_edge[(int64_t)o * D + d], g, a);
    if (P.gW_edge) P.gW_edge[(int64_t)o * D + d] += g * ae;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) a += __shfl_xor(a, m, 64);
  if (lane == 0 && P.g_att_edge) P.g_att_edge[o] += a;
}

// g[o] += Σ_b part[b][o] (fixed order): block = 16 columns x 16 row groups
__global__ __launch_bounds__(256) void k_colsum_accum(const float* __restrict__ part, int nparts,
                                                      int O, float* __restrict__ g) {
  __shared__ float s_red[16][17];
  const int lo = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int o = blockIdx.x * 16 + lo;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (o < O) {
    int b = grp;
    for (; b + 48 < nparts; b += 64) {
      a0 += part[(int64_t)b * O + o];
      a1 += part[(int64_t)(b + 16) * O + o];
      a2 += part[(int64_t)(b + 32) * O + o];
      a3 += part[(int64_t)(b + 48) * O + o];
    }
    for (; b < nparts; b += 16) a0 += part[(int64_t)b * O + o];
  }
  s_red[grp][lo] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (grp == 0 && o < O) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += s_red[k][lo];
    g[o] += s;
  }
}


// ---------------------------------------------------------------------------
// All layers in one launch (sv2n_gat_prep_fwd_all).  Two kinds of blocks,
// none depending on another:
//   P blocks (layer, 64 columns f, head or edge head): k_prep_fwd's work,
//     plus the bf16 planes of every waug row they write (columns up to kp,
//     zero past F);
//   T blocks (layer, 32 f x 32 o tile): the transposed planes planesT[f][o]
//     = split3(waug[o][f]), the fold rows recomputed from W in k_prep_fwd's
//     summation order (bit-identical to waug), transposed through LDS.
// ---------------------------------------------------------------------------
struct PrepAllArgs {
  sv2n_prep_layer l[SV2N_MAX_LAYERS];
  int64_t kp[SV2N_MAX_LAYERS], kpt[SV2N_MAX_LAYERS];
  int px[SV2N_MAX_LAYERS];       // P blocks along columns
  int rp[SV2N_MAX_LAYERS];       // row parts of the node copy (part 0 also folds)
  int pstart[SV2N_MAX_LAYERS];   // first P block of the layer
  int tf[SV2N_MAX_LAYERS];       // T tiles along f
  int tstart[SV2N_MAX_LAYERS];   // first T block of the layer
  int tcount[SV2N_MAX_LAYERS];
  int pcount[SV2N_MAX_LAYERS];
  int L;
};

__global__ __launch_bounds__(256) void k_prep_fwd_all(const PrepAllArgs a) {
  __shared__ float s_red[2][PREP_G][64];
  __shared__ float tile[32][33];
  const int t = threadIdx.x;
  const int b = blockIdx.x;
  int l = 0, local = -1;
  bool tblock = false;
  for (int k = 0; k < a.L; ++k) {
    if (b >= a.pstart[k] && b < a.pstart[k] + a.pcount[k]) { l = k; local = b - a.pstart[k]; }
    if (b >= a.tstart[k] && b < a.tstart[k] + a.tcount[k]) {
      l = k; local = b - a.tstart[k]; tblock = true;
    }
  }
  if (local < 0) return;
  const sv2n_prep_layer& P = a.l[l];
  const int H = P.heads, C = P.channels, F = P.in_features, ldx = P.ldx, HC = H * C;
  const int np = P.nplanes == 1 ? 1 : 3;
  if (!tblock) {
    const int64_t kp = a.kp[l], plane = (int64_t)ldx * kp;
    const int nxy = a.px[l] * (P.W_edge ? 2 * H : H);
    const int part = local / nxy, lxy = local - part * nxy;
    const int bx = lxy % a.px[l], y = lxy / a.px[l];
    // the block's copy rows [cb, ce) of head h; part 0 also folds all C rows
    const int RPn = a.rp[l], CR = (C + RPn - 1) / RPn;
    const int cb = part * CR, ce = min(C, cb + CR);
    if (y < H) {
      if (bx * 64 >= kp) return;
      const PrepBlock B{P.W, P.att_src, P.att_dst, H, C, F, ldx, P.waug, P.planes, kp, plane, np};
      prep_node_block(B, y, bx * 64, cb, ce, part == 0, s_red, t);
    } else {
      if (!P.W_edge || part != 0 || bx * 64 >= P.edge_dim) return;
      prep_edge_block(P.W_edge, P.att_edge, C, P.edge_dim, y - H, bx * 64, P.wfold, P.hl_pad,
                      P.col0, s_red, t);
    }
    return;
  }
  // ---- T block: planesT[f][o] for a 32 x 32 tile ----
  const int64_t kpt = a.kpt[l], plane = (int64_t)F * kpt;
  const int f0 = (local % a.tf[l]) * 32, o0 = (local / a.tf[l]) * 32;
  {
    const int fl = t & 31, og = t >> 5;
    const int f = f0 + fl;
    for (int oi = og; oi < 32; oi += 8) {
      const int o = o0 + oi;
      float v = 0.f;
      if (f < F && o < HC) {
        v = P.W[(int64_t)o * F + f];
      } else if (f < F && o < HC + 2 * H) {
        const int q = o - HC, h = q % H;
        const float* att = q < H ? P.att_src : P.att_dst;
        float p16[PREP_G];
#pragma unroll
        for (int k = 0; k < PREP_G; ++k) p16[k] = 0.f;
        // the P blocks' 16 row groups (row c in group c % 16, in c order)
        for (int c0 = 0; c0 < C; c0 += 32) {
          float w[32], at[32];
#pragma unroll
          for (int u = 0; u < 32; ++u) {
            const int row = h * C + min(c0 + u, C - 1);
            w[u] = P.W[(int64_t)row * F + f];
            at[u] = att[row];
          }
#pragma unroll
          for (int u = 0; u < 32; ++u)
            if (c0 + u < C) p16[u & 15] = fmaf(at[u], w[u], p16[u & 15]);
        }
        v = fold_tree16(p16, 1);
      }
      tile[oi][fl] = v;
    }
  }
  __syncthreads();
  {
    const int ol = t & 31, fg = t >> 5;
    const int o = o0 + ol;
    for (int fi = fg; fi < 32; fi += 8) {
      const int f = f0 + fi;
      if (f < F && o < kpt) put3(P.planes_t, plane, (int64_t)f * kpt + o, tile[ol][fi], np);
    }
  }
}

}  // namespace sv2n

using namespace sv2n;

extern "C" int sv2n_gat_prep_fwd(const float* W, const float* att_src, const float* att_dst,
                                 int heads, int channels, int in_features, float* waug, int ldx,
                                 const float* W_edge, const float* att_edge, int edge_dim,
                                 float* wfold, int hl_pad, int col0, hipStream_t stream) {
  if (!W || !att_src || !att_dst || !waug || heads < 1 || channels < 1 || in_features < 1)
    return SV2N_ERR_ARG;
  if (heads > SV2N_MAX_HEADS || ldx < heads * channels + 2 * heads) return SV2N_ERR_SHAPE;
  const bool edge = W_edge && att_edge && wfold;
  if (edge && (edge_dim < 1 || col0 + heads > hl_pad)) return SV2N_ERR_SHAPE;
  const int cols = std::max(in_features, edge ? edge_dim : 0);
  dim3 grid((cols + 63) / 64, edge ? 2 * heads : heads);
  hipLaunchKernelGGL(k_prep_fwd, grid, dim3(256), 0, stream, W, att_src, att_dst, heads, channels,
                     in_features, waug, ldx, edge ? W_edge : nullptr, att_edge, edge_dim, wfold,
                     hl_pad, col0);
  return (int)hipGetLastError();
}

extern "C" int64_t sv2n_gat_prep_bwd_workspace(int heads, int in_features) {
  return (int64_t)2 * heads * in_features;
}

extern "C" int sv2n_gat_prep_bwd_node(const float* dwaug_t, int ldx, const float* W,
                                      const float* att_src, const float* att_dst, int heads,
                                      int channels, int in_features, const float* dbias_partial,
                                      int num_parts, int bias_len, float* gW, float* g_att_src,
                                      float* g_att_dst, float* g_bias, float* workspace,
                                      int64_t workspace_floats, hipStream_t stream) {
  const bool weights = gW || g_att_src || g_att_dst;
  if (weights && (!dwaug_t || !W || !att_src || !att_dst)) return SV2N_ERR_ARG;
  if (heads < 1 || channels < 1 || in_features < 1) return SV2N_ERR_ARG;
  if (heads > SV2N_MAX_HEADS || (weights && ldx < heads * channels + 2 * heads))
    return SV2N_ERR_SHAPE;
  const int HC = heads * channels;
  const bool att = g_att_src || g_att_dst;
  if (att && (!workspace || workspace_floats < (int64_t)2 * heads * in_features))
    return SV2N_ERR_WORKSPACE;
  if (gW || att) {
    dim3 grid((in_features + 63) / 64, gW ? (HC + 63) / 64 : 1);
    hipLaunchKernelGGL(k_prep_bwd_w, grid, dim3(256), 0, stream, dwaug_t, ldx, att_src, att_dst,
                       heads, channels, in_features, gW, att ? workspace : nullptr);
  }
  if (att) {
    hipLaunchKernelGGL(k_prep_bwd_att, dim3((HC + 3) / 4), dim3(256), 0, stream, workspace, W,
                       heads, channels, in_features, g_att_src, g_att_dst);
  }
  if (g_bias && dbias_partial && bias_len > 0 && num_parts > 0) {
    hipLaunchKernelGGL(k_colsum_accum, dim3((bias_len + 15) / 16), dim3(256), 0, stream,
                       dbias_partial, num_parts, bias_len, g_bias);
  }
  return (int)hipGetLastError();
}

extern "C" int sv2n_gat_prep_bwd_edge(const float* dwfold, int hl_pad, int col0,
                                      const float* W_edge, const float* att_edge, int heads,
                                      int channels, int edge_dim, float* gW_edge,
                                      float* g_att_edge, hipStream_t stream) {
  if (!dwfold || !W_edge || !att_edge || heads < 1 || channels < 1 || edge_dim < 1)
    return SV2N_ERR_ARG;
  if (col0 + heads > hl_pad) return SV2N_ERR_SHAPE;
  const int HC = heads * channels;
  hipLaunchKernelGGL(k_prep_bwd_edge, dim3((HC + 3) / 4), dim3(256), 0, stream, dwfold, hl_pad,
                     col0, W_edge, att_edge, heads, channels, edge_dim, gW_edge, g_att_edge);
  return (int)hipGetLastError();
}

extern "C" int sv2n_gat_prep_bwd_edge_all(const float* dwfold, int hl_pad, int edge_dim,
                                          const sv2n_edge_grad_layer* layers, int num_layers,
                                          hipStream_t stream) {
  if (!dwfold || !layers || edge_dim < 1 || num_layers < 1 || num_layers > SV2N_MAX_LAYERS)
    return SV2N_ERR_ARG;
  PrepBwdEdgeArgs a{};
  int maxhc = 0;
  for (int l = 0; l < num_layers; ++l) {
    const sv2n_edge_grad_layer& P = layers[l];
    if (!P.W_edge || !P.att_edge || P.heads < 1 || P.channels < 1) return SV2N_ERR_ARG;
    if (P.col0 < 0 || P.col0 + P.heads > hl_pad) return SV2N_ERR_SHAPE;
    a.l[l] = P;
    maxhc = std::max(maxhc, P.heads * P.channels);
  }
  hipLaunchKernelGGL(k_prep_bwd_edge_all, dim3((unsigned)((maxhc + 3) / 4), (unsigned)num_layers),
                     dim3(256), 0, stream, dwfold, hl_pad, edge_dim, a);
  return (int)hipGetLastError();
}

extern "C" int sv2n_gat_prep_fwd_all(const sv2n_prep_layer* layers, int num_layers,
                                     hipStream_t stream) {
  if (!layers || num_layers < 1 || num_layers > SV2N_MAX_LAYERS) return SV2N_ERR_ARG;
  PrepAllArgs a{};
  a.L = num_layers;
  int nb = 0;
  for (int l = 0; l < num_layers; ++l) {
    const sv2n_prep_layer& P = layers[l];
    if (!P.W || !P.att_src || !P.att_dst || !P.planes) return SV2N_ERR_ARG;
    if (P.heads < 1 || P.channels < 1 || P.in_features < 1) return SV2N_ERR_ARG;
    if (P.heads > SV2N_MAX_HEADS || P.ldx < P.heads * P.channels + 2 * P.heads)
      return SV2N_ERR_SHAPE;
    const bool edge = P.W_edge && P.att_edge && P.wfold;
    if (edge && (P.edge_dim < 1 || P.col0 + P.heads > P.hl_pad)) return SV2N_ERR_SHAPE;
    a.l[l] = P;
    if (!edge) a.l[l].W_edge = nullptr;
    a.kp[l] = sv2n_split3_kpad(P.in_features);
    a.kpt[l] = sv2n_split3_kpad(P.ldx);
    const int64_t cols = std::max<int64_t>(a.kp[l], edge ? P.edge_dim : 0);
    a.px[l] = (int)((cols + 63) / 64);
    a.pstart[l] = nb;
    const int nxy = a.px[l] * (edge ? 2 * P.heads : P.heads);
    // split the row copy so the launch has ~512 blocks (C3: 20 x 6 blocks of
    // 500 rows each were a serial 42 us); part 0 keeps the fold
    a.rp[l] = (int)std::max<int64_t>(1, std::min<int64_t>((512 + nxy - 1) / nxy,
                                                          (P.channels + 63) / 64));
    a.pcount[l] = nxy * a.rp[l];
    nb += a.pcount[l];
  }
  for (int l = 0; l < num_layers; ++l) {
    const sv2n_prep_layer& P = layers[l];
    a.tf[l] = (P.in_features + 31) / 32;
    a.tstart[l] = nb;
    a.tcount[l] = P.planes_t ? a.tf[l] * (int)((a.kpt[l] + 31) / 32) : 0;
    nb += a.tcount[l];
  }
  hipLaunchKernelGGL(k_prep_fwd_all, dim3((unsigned)nb), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}
