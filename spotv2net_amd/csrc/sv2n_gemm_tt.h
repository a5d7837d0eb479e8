// Weight-gradient GEMM with BOTH operands k-strided, on bf16 MFMA:
//
//   C[m][n] = Σ_k A[k][m] · B[k][n]      (A = x [K][lda], B = dxs [K][ldb])
//
// i.e. dWaugᵀ = xᵀ·dxs of a GAT layer, K = the batch's
// node count.  The operands are staged as they lie in HBM — row k of the tile
// is BM (BN) contiguous floats — converted to bf16 planes on the way into LDS
// ([k][m] images, no register transpose), and the MFMA fragments are read
// with ds_read_b64_tr_b16 (gfx950's transposing LDS read: a 16-lane group
// gets a 4-row x 16-column block column-major).
//
// Fragment k order.  v_mfma_f32_16x16x32_bf16 wants lane (i, g) (i = l & 15,
// g = l >> 4) to hold 8 k values of row/column i.  Two transposed reads give
// it rows {4g .. 4g+3} and {16+4g .. 16+4g+3} of the 32-row tile: a fixed
// bijection of the 32 k of the step, the same for A and B, so the products
// sum over every k exactly once.  With LDS rows of BM + 16 bf16 (72 dwords
// for BM = 128) the 8 rows one 32-lane half reads fall in 8 distinct 8-bank
// windows: conflict-free.
//
// NP = 1: bf16 operands (bf16 execution mode).  NP = 3: the f32-accurate
// split (x = x0 + x1 + x2 in bf16, six products with plane order p + q <= 2,
// sv2n_gemm3_kernel.h) for the fp32 path.
//
// Workgroup: 4 waves as 2 x 2, wave tile (BM/2) x (BN/2); K steps of 32 with
// the next step's global loads in registers while this step computes (one
// barrier per step, two LDS stages).  gridDim.z K slices write slabs
// C + z*M*ldc (summed in a fixed order by the caller).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "sv2n_common.h"
#include "sv2n_gemm3_kernel.h"

namespace sv2n {

typedef short i16x4 __attribute__((ext_vector_type(4)));

template <int BM, int BN, int NP>
struct GemmTTCfg {
  static constexpr int BK = 32;
  static constexpr int SA = BM + 16, SB = BN + 16;          // bf16 per LDS row
  static constexpr int PLANE_A = BK * SA, PLANE_B = BK * SB;
  static constexpr int STAGE = NP * (PLANE_A + PLANE_B);    // bf16 per stage
  static constexpr size_t LDS = sizeof(unsigned short) * 2 * STAGE;
  static constexpr int AV = BK * BM / 4 / 256, BV = BK * BN / 4 / 256;  // float4 / thread
  static constexpr int MT = BM / 32, NT = BN / 32;           // 16x16 tiles per wave
  static_assert(BK * BM / 4 % 256 == 0 && BK * BN / 4 % 256 == 0, "staging tiles threads");
};

__device__ __forceinline__ bf16x8 tr_frag(const unsigned short* p0, const unsigned short* p1) {
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(p0));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(p1));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

template <int BM, int BN, int NP>
__global__ __launch_bounds__(256) void k_gemm_tt(const float* __restrict__ A, int64_t lda,
                                                 const float* __restrict__ B, int64_t ldb,
                                                 float* __restrict__ C, int64_t ldc, int64_t M,
                                                 int64_t N, int64_t K, int64_t kslice) {
  using Cfg = GemmTTCfg<BM, BN, NP>;
  constexpr int BK = Cfg::BK, SA = Cfg::SA, SB = Cfg::SB, AV = Cfg::AV, BV = Cfg::BV;
  constexpr int MT = Cfg::MT, NT = Cfg::NT, STAGE = Cfg::STAGE;
  constexpr int PA = Cfg::PLANE_A, PB = Cfg::PLANE_B;
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int wm = wave & 1, wn = wave >> 1;
  const int li = lane & 15, lg = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
  const int64_t kbeg = (int64_t)blockIdx.z * kslice, kend = min(K, kbeg + kslice);
  if (gridDim.z > 1) C += (int64_t)blockIdx.z * M * ldc;

  // whole-operand buffer descriptors: rows past K / columns past the array
  // read 0; columns in [M, lda) only feed output rows that are never stored
  const rsrc_t ra = make_rsrc(A, (uint32_t)min<int64_t>(K * lda * 4, 0x7fffffff));
  const rsrc_t rb = make_rsrc(B, (uint32_t)min<int64_t>(K * ldb * 4, 0x7fffffff));

  f32x4 va[AV], vb[BV];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int s = 0; s < AV; ++s) {
      const int idx = t + 256 * s;
      const int r = idx / (BM / 4), c4 = idx - r * (BM / 4);
      const int64_t k = k0 + r, m = m0 + 4 * c4;
      va[s] = bld4(ra, (k < kend && m < lda) ? (int)((k * lda + m) * 4) : OOB);
    }
#pragma unroll
    for (int s = 0; s < BV; ++s) {
      const int idx = t + 256 * s;
      const int r = idx / (BN / 4), c4 = idx - r * (BN / 4);
      const int64_t k = k0 + r, n = n0 + 4 * c4;
      vb[s] = bld4(rb, (k < kend && n < ldb) ? (int)((k * ldb + n) * 4) : OOB);
    }
  };
  auto put = [&](unsigned short* dst, int plane_elems, int stride, int r, int c, const f32x4& v) {
    uint2 w[3];
    if constexpr (NP == 3) {
      split3_pk(v[0], v[1], w[0].x, w[1].x, w[2].x);
      split3_pk(v[2], v[3], w[0].y, w[1].y, w[2].y);
    } else {
      w[0].x = bf16_pk(v[0], v[1]);
      w[0].y = bf16_pk(v[2], v[3]);
    }
#pragma unroll
    for (int p = 0; p < NP; ++p)
      *reinterpret_cast<uint2*>(dst + p * plane_elems + r * stride + c) = w[p];
  };
  auto store = [&](unsigned short* st) {
#pragma unroll
    for (int s = 0; s < AV; ++s) {
      const int idx = t + 256 * s;
      const int r = idx / (BM / 4), c4 = idx - r * (BM / 4);
      put(st, PA, SA, r, 4 * c4, va[s]);
    }
    unsigned short* sb = st + NP * PA;
#pragma unroll
    for (int s = 0; s < BV; ++s) {
      const int idx = t + 256 * s;
      const int r = idx / (BN / 4), c4 = idx - r * (BN / 4);
      put(sb, PB, SB, r, 4 * c4, vb[s]);
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read addresses: lane 4q+p of its 16-lane group -> row q, columns 4p..4p+3
  const int q = li >> 2, p4 = 4 * (li & 3);
  const int rowA0 = (4 * lg + q) * SA, rowA1 = (16 + 4 * lg + q) * SA;
  const int rowB0 = (4 * lg + q) * SB, rowB1 = (16 + 4 * lg + q) * SB;
  auto compute = [&](const unsigned short* st) {
    const unsigned short* sa = st;
    const unsigned short* sb = st + NP * PA;
    bf16x8 af[MT][NP];
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      const int col = wm * (BM / 2) + 16 * a + p4;
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
        af[a][pl] = tr_frag(sa + pl * PA + rowA0 + col, sa + pl * PA + rowA1 + col);
    }
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int col = wn * (BN / 2) + 16 * b + p4;
      bf16x8 bf[NP];
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
        bf[pl] = tr_frag(sb + pl * PB + rowB0 + col, sb + pl * PB + rowB1 + col);
#pragma unroll
      for (int a = 0; a < MT; ++a) acc[a][b] = mfma_planes<NP>(af[a], bf, acc[a][b]);
    }
  };

  const int nsteps = (int)((kend - kbeg + BK - 1) / BK);
  if (nsteps > 0) {
    load(kbeg);
    store(lds);
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
      if (s + 1 < nsteps) load(kbeg + (int64_t)(s + 1) * BK);
      compute(lds + (s & 1) * STAGE);
      if (s + 1 < nsteps) store(lds + ((s + 1) & 1) * STAGE);
      __syncthreads();
    }
  }
  // acc[a][b][r] = C[row 16a + 4lg + r][col 16b + li] of the wave tile
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int64_t gn = n0 + wn * (BN / 2) + 16 * b + li;
      if (gn < N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t gm = m0 + wm * (BM / 2) + 16 * a + 4 * lg + r;
          if (gm < M) C[gm * ldc + gn] = acc[a][b][r];
        }
      }
    }
}

}  // namespace sv2n

namespace sv2n {

// ---------------------------------------------------------------------------
// k_gemm_tt3w: the f32-accurate (bf16x3, six products) weight-gradient GEMM,
//   C[m][n] = Σ_k A[k][m] · B[k][n]      (A = x [K][lda], B = dxs [K][ldb])
// shaped like the f32 kernel it replaces (k_gemm_f32<8, 1, NT, ...>): eight
// waves stacked along M (16 rows each, BM = 128) x all BN = 16·NT columns, so
// two waves share each SIMD — one wave's split VALU and LDS stores issue in
// the other's MFMA shadow (an MFMA 16x16x32 holds the SIMD's issue for 8 of
// its 16 cycles).  K steps of 32; the f32 operands of step s+1 are loaded
// into registers while step s computes, split into three bf16 planes
// (split3_pk) and stored to the other of two LDS stages ([plane][k][row]
// images) after step s's MFMAs are issued; one barrier per step.  Fragments
// come from ds_read_b64_tr_b16 exactly as in k_gemm_tt.  Split-K slices
// write slabs part[z][M][N] with the XCD-grouped slice order of
// k_gemm_f32<..., XR = true> (every tile of a slice on one XCD's L2).
// ---------------------------------------------------------------------------
template <int NT, int MT>
struct GemmTT3WCfg {
  static constexpr int NW = 8, THREADS = 512, BK = 32, BM = 16 * MT * NW, BN = 16 * NT;
  // bf16 per LDS row: the 8 rows a 32-lane half reads by ds_read_b64_tr_b16
  // must start in 8 distinct 8-bank windows: row dwords ≡ 8 (mod 16)
  static constexpr int pad(int w) {
    int p = 16;
    while (((w + p) / 2) % 16 != 8) p += 16;
    return p;
  }
  static constexpr int SA = BM + pad(BM), SB = BN + pad(BN);
  static constexpr int PA = BK * SA, PB = BK * SB;   // bf16 per plane image
  static constexpr int STAGE = 3 * (PA + PB);        // bf16 per stage
  // two stages (one barrier per step) when they fit the 160 KiB LDS, else one
  static constexpr int NSTAGE = sizeof(unsigned short) * 2 * STAGE <= 160 * 1024 ? 2 : 1;
  static constexpr size_t LDS = sizeof(unsigned short) * NSTAGE * STAGE;
  static constexpr int AV = BK * BM / 4 / THREADS;                   // float4 per thread
  static constexpr int BVN = BK * BN / 4, BV = (BVN + THREADS - 1) / THREADS;
  static_assert(BK * BM / 4 % THREADS == 0, "A staging tiles the threads");
};

template <int NT, int MT>
__global__ __launch_bounds__(512) void k_gemm_tt3w(const float* __restrict__ A, int64_t lda,
                                                   const float* __restrict__ B, int64_t ldb,
                                                   float* __restrict__ part, int64_t M, int64_t N,
                                                   int64_t K, int64_t kslice, int nz) {
  using Cfg = GemmTT3WCfg<NT, MT>;
  constexpr int BK = Cfg::BK, BM = Cfg::BM, BN = Cfg::BN, SA = Cfg::SA, SB = Cfg::SB;
  constexpr int PA = Cfg::PA, PB = Cfg::PB, STAGE = Cfg::STAGE, AV = Cfg::AV, BV = Cfg::BV;
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  // XCD-grouped K slices (k_gemm_f32 XR): block b = xcd + 8 * slot
  const int tiles = gridDim.x * gridDim.y;
  const int id = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int xcd = id & 7, slot = id >> 3;
  const int bz = xcd + 8 * (slot / tiles);
  const int tile = slot - (slot / tiles) * tiles;
  const int by = tile / gridDim.x, bx = tile - by * gridDim.x;
  if (bz >= nz) return;

  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, lg = lane >> 4;
  const int64_t m0 = (int64_t)bx * BM, n0 = (int64_t)by * BN;
  const int64_t kbeg = (int64_t)bz * kslice, kend = min(K, kbeg + kslice);
  float* C = part + (int64_t)bz * M * N;
  const rsrc_t ra = make_rsrc(A, (uint32_t)min<int64_t>(K * lda * 4, 0x7fffffff));
  const rsrc_t rb = make_rsrc(B, (uint32_t)min<int64_t>(K * ldb * 4, 0x7fffffff));

  f32x4 va[AV], vb[BV];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int s = 0; s < AV; ++s) {
      const int idx = t + 512 * s;
      const int r = idx / (BM / 4), c4 = idx - r * (BM / 4);
      const int64_t k = k0 + r, m = m0 + 4 * c4;
      va[s] = bld4(ra, (k < kend && m < M) ? (int)((k * lda + m) * 4) : OOB);
    }
#pragma unroll
    for (int s = 0; s < BV; ++s) {
      const int idx = t + 512 * s;
      const int r = idx / (BN / 4), c4 = idx - r * (BN / 4);
      const int64_t k = k0 + r, n = n0 + 4 * c4;
      vb[s] = bld4(rb, (idx < Cfg::BVN && k < kend && n < N) ? (int)((k * ldb + n) * 4) : OOB);
    }
  };
  auto put = [&](unsigned short* dst, int plane, int stride, int r, int c, const f32x4& v) {
    uint2 w[3];
    split3_pk(v[0], v[1], w[0].x, w[1].x, w[2].x);
    split3_pk(v[2], v[3], w[0].y, w[1].y, w[2].y);
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(dst + p * plane + r * stride + c) = w[p];
  };
  auto store = [&](unsigned short* st) {
#pragma unroll
    for (int s = 0; s < AV; ++s) {
      const int idx = t + 512 * s;
      const int r = idx / (BM / 4), c4 = idx - r * (BM / 4);
      put(st, PA, SA, r, 4 * c4, va[s]);
    }
    unsigned short* sb = st + 3 * PA;
#pragma unroll
    for (int s = 0; s < BV; ++s) {
      const int idx = t + 512 * s;
      if (idx < Cfg::BVN) {
        const int r = idx / (BN / 4), c4 = idx - r * (BN / 4);
        put(sb, PB, SB, r, 4 * c4, vb[s]);
      }
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // transposed-read addresses (k_gemm_tt): lane 4q+p of its 16-lane group ->
  // k row q (+4lg, +16), columns 4p..4p+3
  const int q = li >> 2, p4 = 4 * (li & 3);
  const int kA0 = (4 * lg + q) * SA, kA1 = (16 + 4 * lg + q) * SA;
  const int kB0 = (4 * lg + q) * SB, kB1 = (16 + 4 * lg + q) * SB;
  auto compute = [&](const unsigned short* st) {
    const unsigned short* sa = st;
    const unsigned short* sb = st + 3 * PA;
    bf16x8 af[MT][3];
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      const int ca = 16 * (MT * wave + a) + p4;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        af[a][pl] = tr_frag(sa + pl * PA + kA0 + ca, sa + pl * PA + kA1 + ca);
    }
    // B fragments of column tile b+1 read while tile b's MFMAs run (as in
    // k_gemm3<..., PIPE = 1>)
    bf16x8 bq[2][3];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      bq[0][pl] = tr_frag(sb + pl * PB + kB0 + p4, sb + pl * PB + kB1 + p4);
    __builtin_amdgcn_sched_group_barrier(0x100, 6 * (MT + 1), 0);
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      if (b + 1 < NT) {
        const int cb = 16 * (b + 1) + p4;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          bq[(b + 1) & 1][pl] = tr_frag(sb + pl * PB + kB0 + cb, sb + pl * PB + kB1 + cb);
        __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
      }
#pragma unroll
      for (int a = 0; a < MT; ++a) acc[a][b] = mfma_planes<3>(af[a], bq[b & 1], acc[a][b]);
      __builtin_amdgcn_sched_group_barrier(0x008, 6 * MT, 0);
    }
  };

  const int nsteps = (int)((kend - kbeg + BK - 1) / BK);
  if (nsteps > 0) {
    load(kbeg);
    store(lds);
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
      if (s + 1 < nsteps) load(kbeg + (int64_t)(s + 1) * BK);
      if constexpr (Cfg::NSTAGE == 2) {
        compute(lds + (s & 1) * STAGE);
        if (s + 1 < nsteps) store(lds + ((s + 1) & 1) * STAGE);
      } else {
        compute(lds);
        __syncthreads();  // every wave is done reading the stage
        if (s + 1 < nsteps) store(lds);
      }
      __syncthreads();
    }
  }
  // acc[a][b][r] = C[row 16(MT·wave + a) + 4lg + r][col 16b + li] of the block tile
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int64_t gn = n0 + 16 * b + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gm = m0 + 16 * (MT * wave + a) + 4 * lg + r;
        if (gm < M && gn < N) C[gm * N + gn] = acc[a][b][r];
      }
    }
}

// ---------------------------------------------------------------------------
// k_gemm_tt3y: k_gemm_tt3w<NT, MT> with the next step's staging under the
// current step's MFMAs, in the LDS of one A image and two B stages.
//   * A (x, k-strided) is staged per wave: wave w loads, splits and writes the
//     16·MT rows it alone reads.  Its fragments are read into registers at the
//     top of the step, so once those reads land the wave rewrites its rows
//     with step s+1 while its MFMAs run — no second A image, no barrier.
//   * B (dxs) is shared: step s+1 goes to the other of two stages, one
//     staging piece per column tile, published by the step's barrier.
//   * step s+1's operands are loaded at the top of step s and staged, one
//     piece per column tile, in its last tiles (registers: the two-tile
//     tiling is at 240 VGPRs without them); staging is branch-free (slots past the B image repeat the last one; the
//     last steps reload the last K-step and write what nobody reads).
// Same products in the same order as k_gemm_tt3w.  C2 L0 dWᵀ: 98 KiB of
// stage for tt3w's single stage, 144 KiB here.
// ---------------------------------------------------------------------------
template <int NT, int MT>
struct GemmTT3YCfg {
  using W = GemmTT3WCfg<NT, MT>;
  static constexpr int AVW = 16 * MT * W::BK / 4 / 64;  // float4 per lane: the wave's A rows
  static constexpr size_t LDS = sizeof(unsigned short) * (3 * W::PA + 2 * 3 * W::PB);
  static_assert(16 * MT * W::BK / 4 % 64 == 0, "wave A staging tiles the lanes");
};

// BPL = true: B arrives pre-split as three bf16 planes [3][K][ldb] (plane
// stride bplane elements; the producer, the layer's attention backward,
// splits every element once), so only A is split here.
template <int NT, int MT, bool BPL = false>
__global__ __launch_bounds__(512) void k_gemm_tt3y(const float* __restrict__ A, int64_t lda,
                                                   const float* __restrict__ B, int64_t ldb,
                                                   float* __restrict__ part, int64_t M, int64_t N,
                                                   int64_t K, int64_t kslice, int nz,
                                                   int64_t bplane = 0) {
  using Cfg = GemmTT3WCfg<NT, MT>;
  constexpr int BK = Cfg::BK, BN = Cfg::BN, SA = Cfg::SA, SB = Cfg::SB;
  constexpr int PA = Cfg::PA, PB = Cfg::PB, BV = Cfg::BV, BVN = Cfg::BVN;
  constexpr int AVW = GemmTT3YCfg<NT, MT>::AVW;
  constexpr int NPUT = AVW + BV;
  static_assert(AVW + BV <= NT, "one staging piece per column tile");
  constexpr int WR = 16 * MT;  // A rows of one wave
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  unsigned short* const sA = lds;            // [3][BK][SA], rows of wave w at 16·MT·w
  unsigned short* const sB0 = lds + 3 * PA;  // two stages of [3][BK][SB]
  const int tiles = gridDim.x * gridDim.y;
  const int id = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int xcd = id & 7, slot = id >> 3;
  const int bz = xcd + 8 * (slot / tiles);
  const int tile = slot - (slot / tiles) * tiles;
  const int by = tile / gridDim.x, bx = tile - by * gridDim.x;
  if (bz >= nz) return;

  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, lg = lane >> 4;
  const int64_t m0 = (int64_t)bx * Cfg::BM, n0 = (int64_t)by * BN;
  const int64_t kbeg = (int64_t)bz * kslice, kend = min(K, kbeg + kslice);
  float* C = part + (int64_t)bz * M * N;
  const rsrc_t ra = make_rsrc(A, (uint32_t)min<int64_t>(K * lda * 4, 0x7fffffff));
  const rsrc_t rb = make_rsrc(B, (uint32_t)min<int64_t>(BPL ? 3 * bplane * 2 : K * ldb * 4,
                                                       0x7fffffff));
  const int wrow = WR * wave;  // first A row (in the block) of this wave

  f32x4 va[AVW], vb[BPL ? 1 : BV];
  u32x2 vp[BPL ? BV : 1][3];
  auto load_a = [&](int64_t k0) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < AVW; ++s) {
      const int idx = lane + 64 * s;
      const int r = idx / (WR / 4), c4 = idx - r * (WR / 4);
      const int64_t k = k0 + r, m = m0 + wrow + 4 * c4;
      va[s] = bld4(ra, (k < kend && m < M) ? (int)((k * lda + m) * 4) : OOB);
    }
  };
  auto load_b = [&](int64_t k0) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < BV; ++s) {
      const int idx = min(t + 512 * s, BVN - 1);
      const int r = idx / (BN / 4), c4 = idx - r * (BN / 4);
      const int64_t k = k0 + r, n = n0 + 4 * c4;
      if constexpr (BPL) {
        const int off = (k < kend && n < N) ? (int)((k * ldb + n) * 2) : OOB;
#pragma unroll
        for (int p = 0; p < 3; ++p)
          vp[s][p] = bld2_u32(rb, off == OOB ? OOB : off + (int)(p * bplane * 2));
      } else {
        vb[s] = bld4(rb, (k < kend && n < N) ? (int)((k * ldb + n) * 4) : OOB);
      }
    }
  };
  auto put = [&](unsigned short* dst, int plane, int stride, int r, int c, const f32x4& v)
      __attribute__((always_inline)) {
    uint2 w[3];
    split3_pk(v[0], v[1], w[0].x, w[1].x, w[2].x);
    split3_pk(v[2], v[3], w[0].y, w[1].y, w[2].y);
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(dst + p * plane + r * stride + c) = w[p];
  };
  // piece i < AVW: the wave's A rows; else a B slot into stage sb
  auto put_piece = [&](auto i_c, unsigned short* sb) __attribute__((always_inline)) {
    constexpr int i = decltype(i_c)::value;
    if constexpr (i < AVW) {
      const int idx = lane + 64 * i;
      const int r = idx / (WR / 4), c4 = idx - r * (WR / 4);
      put(sA, PA, SA, r, wrow + 4 * c4, va[i]);
    } else {
      const int idx = min(t + 512 * (i - AVW), BVN - 1);
      const int r = idx / (BN / 4), c4 = idx - r * (BN / 4);
      if constexpr (BPL) {
#pragma unroll
        for (int p = 0; p < 3; ++p)
          *reinterpret_cast<u32x2*>(sb + p * PB + r * SB + 4 * c4) = vp[i - AVW][p];
      } else {
        put(sb, PB, SB, r, 4 * c4, vb[i - AVW]);
      }
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int q = li >> 2, p4 = 4 * (li & 3);
  const int kA0 = (4 * lg + q) * SA, kA1 = (16 + 4 * lg + q) * SA;
  const int kB0 = (4 * lg + q) * SB, kB1 = (16 + 4 * lg + q) * SB;

  const int nsteps = (int)((kend - kbeg + BK - 1) / BK);
  auto step = [&](int s, auto cur_c) __attribute__((always_inline)) {
    constexpr int cur = decltype(cur_c)::value, nxt = 1 - cur;
    const unsigned short* sb = sB0 + cur * 3 * PB;
    unsigned short* sw = sB0 + nxt * 3 * PB;
    // step s+1's operands, staged in this step's last column tiles
    load_a(kbeg + (int64_t)min(s + 1, nsteps - 1) * BK);
    load_b(kbeg + (int64_t)min(s + 1, nsteps - 1) * BK);
    bf16x8 af[MT][3];
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      const int ca = 16 * (MT * wave + a) + p4;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        af[a][pl] = tr_frag(sA + pl * PA + kA0 + ca, sA + pl * PA + kA1 + ca);
    }
    bf16x8 bq[2][3];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      bq[0][pl] = tr_frag(sb + pl * PB + kB0 + p4, sb + pl * PB + kB1 + p4);
    __builtin_amdgcn_sched_group_barrier(0x100, 6 * (MT + 1), 0);
    // a wave's LDS operations execute in issue order: its A rows can be
    // rewritten right behind these reads
    static_for<NT>([&](auto bc) __attribute__((always_inline)) {
      constexpr int b = decltype(bc)::value;
      if constexpr (b + 1 < NT) {
        const int cb = 16 * (b + 1) + p4;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          bq[(b + 1) & 1][pl] = tr_frag(sb + pl * PB + kB0 + cb, sb + pl * PB + kB1 + cb);
        __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
      }
      // one staging piece per tile in the last NPUT tiles (loads issued at the
      // top of this step)
      constexpr int i = b - (NT - NPUT);
      if constexpr (i >= 0) {
        put_piece(std::integral_constant<int, i>{}, sw);
        __builtin_amdgcn_sched_group_barrier(0x200, 3, 0);
      }
#pragma unroll
      for (int a = 0; a < MT; ++a) acc[a][b] = mfma_planes<3>(af[a], bq[b & 1], acc[a][b]);
      __builtin_amdgcn_sched_group_barrier(0x008, 6 * MT, 0);
    });
    __syncthreads();
  };
  if (nsteps > 0) {
    load_a(kbeg);
    load_b(kbeg);
    static_for<NPUT>([&](auto ic) __attribute__((always_inline)) { put_piece(ic, sB0); });
    __syncthreads();
    for (int s = 0; s < nsteps; s += 2) {
      step(s, std::integral_constant<int, 0>{});
      if (s + 1 < nsteps) step(s + 1, std::integral_constant<int, 1>{});
    }
  }
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int64_t gn = n0 + 16 * b + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gm = m0 + 16 * (MT * wave + a) + 4 * lg + r;
        if (gm < M && gn < N) C[gm * N + gn] = acc[a][b][r];
      }
    }
}

}  // namespace sv2n
