// f32-accurate GEMM on bf16 MFMA ("bf16x3 split, 6 products"), shared by the
// library and tools/gemm3_tune.hip.
//
//   C[M][N] = Σ_k A[m][k] · B[n][k]      (both operands k-contiguous)
//
// Every fp32 operand is the exact sum of three bf16 terms, x = x0 + x1 + x2
// (x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1): 3 x 8 significant
// bits cover the 24-bit fp32 mantissa).  a·b keeps the six products with
// p + q <= 2; the dropped ones (a1 b2, a2 b1, a2 b2) are <= ~2^-23 |a b|, the
// size of one fp32 rounding.  bf16 x bf16 products are exact in fp32 and the
// MFMA accumulates in fp32, so the result matches an fp32 GEMM to fp32
// rounding while running on v_mfma_f32_16x16x32_bf16 (16x the f32-MFMA rate
// per instruction, 2.67x after the six products).
//
// Operands: A is fp32 and split while it is staged into LDS (each element
// once per workgroup, reused by all of the block's N columns); B comes
// pre-split as three bf16 planes [3][N][K] (the caller splits the small
// weight matrix once per step, k_split3).
//
// LDS images [plane][row][BK bf16] with a 32-B row pad: conflict-free
// ds_read_b128 fragment reads (see Gemm3Cfg::ROW).
// Fragment (16x16x32 bf16): lane l holds row l&15, k = 8(l>>4) .. +7.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include <utility>
#include "sv2n_common.h"

namespace sv2n {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ unsigned short bf16_rn(float x) {
  // round-to-nearest-even f32 -> bf16 (inputs are finite here)
  const unsigned u = __float_as_uint(x);
  return (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_f(unsigned short h) { return __uint_as_float((unsigned)h << 16); }

__device__ __forceinline__ void split3(float x, unsigned short& h0, unsigned short& h1,
                                       unsigned short& h2) {
  h0 = bf16_rn(x);
  const float r1 = x - bf16_f(h0);
  h1 = bf16_rn(r1);
  const float r2 = r1 - bf16_f(h1);
  h2 = bf16_rn(r2);
}

// Two elements at once on v_cvt_pk_bf16_f32 (round-to-nearest-even, as
// bf16_rn): ~5.5 VALU per element instead of ~16 for the integer rounding —
// the split shares the SIMD's issue slots with the MFMAs (an MFMA 16x16x32
// leaves 8 of its 16 cycles), so its cost sets the GEMM's rate.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned bf16_pk(float x, float y) {
  const f32x2_t v = {x, y};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_t));
}
// (x, y) -> packed planes p0, p1, p2 (low half = x), x == x0 + x1 + x2 exactly
__device__ __forceinline__ void split3_pk(float x, float y, unsigned& p0, unsigned& p1,
                                          unsigned& p2) {
  p0 = bf16_pk(x, y);
  const float rx = x - __uint_as_float(p0 << 16), ry = y - __uint_as_float(p0 & 0xffff0000u);
  p1 = bf16_pk(rx, ry);
  const float sx = rx - __uint_as_float(p1 << 16), sy = ry - __uint_as_float(p1 & 0xffff0000u);
  p2 = bf16_pk(sx, sy);
}

// fp32 [rows][K] (k-contiguous, row stride ld) -> 3 bf16 planes [3][rows][Kp]
static __global__ __attribute__((unused)) void k_split3(const float* __restrict__ x, int64_t rows, int64_t K, int64_t ld,
                         unsigned short* __restrict__ out, int64_t Kp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * Kp) return;
  const int64_t r = i / Kp, k = i - r * Kp;
  unsigned short h0 = 0, h1 = 0, h2 = 0;
  if (k < K) split3(x[r * ld + k], h0, h1, h2);
  out[i] = h0;
  out[rows * Kp + i] = h1;
  out[2 * rows * Kp + i] = h2;
}

// NP = number of bf16 planes per operand: 3 = the f32-accurate split (six
// products), 1 = plain bf16 operands (bf16(a)·bf16(b), fp32 accumulation: the
// "bf16 autocast" execution mode, one product; B's plane 0 is bf16_rn(w)).
template <int NW, int MT, int NT, int BK, int NP = 3>
struct Gemm3Cfg {
  static constexpr int THREADS = 64 * NW;
  static constexpr int BM = 16 * MT * NW, BN = 16 * NT;
  // bf16 per LDS row: BK + 16 (96 B at BK 32, 160 B at BK 64) puts the 16
  // (row, slot) pairs of each ds_read_b128 lane group ({0-3,12-15,20-27}, ...:
  // MI355X_MICROARCH.md §LDS) in 16 distinct 16-B bank slots
  static constexpr int ROW = BK + 16;
  static constexpr int AV = BM * (BK / 4) / THREADS;         // float4 per thread
  static constexpr int BV = (NP * BN * (BK / 8) + THREADS - 1) / THREADS;  // uint4 per thread
  static constexpr size_t LDS = sizeof(unsigned short) * NP * (BM + BN) * ROW;
  static_assert(BM * (BK / 4) % THREADS == 0, "A staging must tile the threads");
};

// the MFMA products of one (A, B) fragment pair: NP = 3 keeps the six with
// plane orders p + q <= 2 (small terms first), NP = 1 the single bf16 product
template <int NP>
__device__ __forceinline__ f32x4 mfma_planes(const bf16x8 (&a)[NP], const bf16x8 (&b)[NP],
                                             f32x4 acc) {
  if constexpr (NP == 3) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  }
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
}

// Workgroup = NW waves stacked along M (wave tile MT x NT 16x16 tiles), K
// blocks of BK, PF register sets of staged operands in flight (the loads for
// block kb+PF are issued while block kb is computed from LDS).
// PIPE = 1: the B fragments of column tile b+1 are read while tile b's MFMAs
// run (an explicit register double buffer, with scheduling-group barriers
// holding the compiler to "NP reads, then the tile's MFMAs"); PIPE = 0 lets
// the compiler place the reads (it issued each one a single MFMA ahead of its
// use and waited on lgkmcnt(0) between the MFMAs of one tile).
template <int NW, int MT, int NT, int BK, int PF, int NP = 3, int PIPE = 0>
__global__ __launch_bounds__(64 * NW) void k_gemm3(const float* __restrict__ A, int64_t lda,
                                                   const unsigned short* __restrict__ Bp,
                                                   int64_t ldb, int64_t bplane,
                                                   float* __restrict__ C, int64_t ldc, int64_t M,
                                                   int64_t N, int64_t K) {
  using Cfg = Gemm3Cfg<NW, MT, NT, BK, NP>;
  constexpr int TH = Cfg::THREADS, BM = Cfg::BM, BN = Cfg::BN, ROW = Cfg::ROW;
  constexpr int AV = Cfg::AV, BV = Cfg::BV;
  constexpr int AC = BK / 4, BC = BK / 8;  // float4 / uint4 per row
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  unsigned short* sA = lds;                    // [NP][BM][ROW]
  unsigned short* sB = lds + NP * BM * ROW;    // [NP][BN][ROW]
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, lg = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 ra[PF][AV];
  uint4 rb[PF][BV];
  auto load = [&](int set, int64_t k0) {
#pragma unroll
    for (int s = 0; s < AV; ++s) {
      const int idx = t + TH * s;
      const int r = idx / AC, c4 = idx - r * AC;
      const int64_t gm = min(m0 + r, M - 1);
      const int64_t gk = k0 + 4 * c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gk + 3 < K) {
        v = *reinterpret_cast<const float4*>(A + gm * lda + gk);
      } else {
        float* pv = &v.x;
#pragma unroll
        for (int q = 0; q < 4; ++q) pv[q] = (gk + q < K) ? A[gm * lda + gk + q] : 0.f;
      }
      ra[set][s] = v;
    }
#pragma unroll
    for (int s = 0; s < BV; ++s) {
      const int idx = t + TH * s;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (idx < NP * BN * BC) {
        const int p = idx / (BN * BC), rem = idx - p * BN * BC;
        const int r = rem / BC, c = rem - r * BC;
        const int64_t gn = min(n0 + r, N - 1);
        v = *reinterpret_cast<const uint4*>(Bp + p * bplane + gn * ldb + k0 + 8 * c);
      }
      rb[set][s] = v;
    }
  };
  auto store = [&](int set) {
#pragma unroll
    for (int s = 0; s < AV; ++s) {
      const int idx = t + TH * s;
      const int r = idx / AC, c4 = idx - r * AC;
      const float4 v = ra[set][s];
      uint2 w[3];
      if constexpr (NP == 3) {
        split3_pk(v.x, v.y, w[0].x, w[1].x, w[2].x);
        split3_pk(v.z, v.w, w[0].y, w[1].y, w[2].y);
      } else {
        w[0].x = bf16_pk(v.x, v.y);
        w[0].y = bf16_pk(v.z, v.w);
      }
#pragma unroll
      for (int p = 0; p < NP; ++p)
        *reinterpret_cast<uint2*>(sA + (p * BM + r) * ROW + 4 * c4) = w[p];
    }
#pragma unroll
    for (int s = 0; s < BV; ++s) {
      const int idx = t + TH * s;
      if (idx < NP * BN * BC) {
        const int p = idx / (BN * BC), rem = idx - p * BN * BC;
        const int r = rem / BC, c = rem - r * BC;
        *reinterpret_cast<uint4*>(sB + (p * BN + r) * ROW + 8 * c) = rb[set][s];
      }
    }
  };
  auto compute_pipe = [&]() {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[MT][NP];
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          af[a][p] = *reinterpret_cast<const bf16x8*>(
              sA + (p * BM + wave * 16 * MT + 16 * a + li) * ROW + kk + 8 * lg);
      bf16x8 bq[2][NP];
#pragma unroll
      for (int p = 0; p < NP; ++p)
        bq[0][p] = *reinterpret_cast<const bf16x8*>(sB + (p * BN + li) * ROW + kk + 8 * lg);
      __builtin_amdgcn_sched_group_barrier(0x100, NP * (MT + 1), 0);  // DS reads: A, B tile 0
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        if (b + 1 < NT) {
#pragma unroll
          for (int p = 0; p < NP; ++p)
            bq[(b + 1) & 1][p] = *reinterpret_cast<const bf16x8*>(
                sB + (p * BN + 16 * (b + 1) + li) * ROW + kk + 8 * lg);
          __builtin_amdgcn_sched_group_barrier(0x100, NP, 0);  // DS reads: B tile b+1
        }
#pragma unroll
        for (int a = 0; a < MT; ++a) acc[a][b] = mfma_planes<NP>(af[a], bq[b & 1], acc[a][b]);
        __builtin_amdgcn_sched_group_barrier(0x008, (NP == 3 ? 6 : 1) * MT, 0);  // MFMAs of tile b
      }
    }
  };
  auto compute = [&]() {
    if constexpr (PIPE) {
      compute_pipe();
      return;
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[MT][NP];
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          af[a][p] = *reinterpret_cast<const bf16x8*>(
              sA + (p * BM + wave * 16 * MT + 16 * a + li) * ROW + kk + 8 * lg);
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        bf16x8 bf[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p)
          bf[p] = *reinterpret_cast<const bf16x8*>(sB + (p * BN + 16 * b + li) * ROW + kk + 8 * lg);
#pragma unroll
        for (int a = 0; a < MT; ++a) acc[a][b] = mfma_planes<NP>(af[a], bf, acc[a][b]);
      }
    }
  };

  const int64_t nk = (K + BK - 1) / BK;
#pragma unroll
  for (int s = 0; s < PF; ++s)
    if (s < nk) load(s, (int64_t)s * BK);
  for (int64_t kb = 0; kb < nk; kb += PF) {
#pragma unroll
    for (int s = 0; s < PF; ++s) {
      if (kb + s < nk) {
        __syncthreads();  // previous block's fragments consumed
        store(s);
        __syncthreads();
        if (kb + s + PF < nk) load(s, (kb + s + PF) * BK);
        compute();
      }
    }
  }
  // store: acc[a][b][r] = C[row 16a + 4lg + r][col 16b + li] of the wave tile
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int64_t gn = n0 + 16 * b + li;
      if (gn < N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t gm = m0 + wave * 16 * MT + 16 * a + 4 * lg + r;
          if (gm < M) C[gm * ldc + gn] = acc[a][b][r];
        }
      }
    }
}

// Both operands k-strided (the weight gradients dWᵀ = xᵀ·dxs):
//   C[m][n] = Σ_k A[k][m] · B[k][n]   (A row stride lda, B row stride ldb)
// over the K slice [kz*kslice, min(K, (kz+1)*kslice)) of gridDim.z; with
// more than one slice every slice writes its own slab C + kz*M*N (summed in
// a fixed order by the caller's reduce).  Both operands are split while
// staged: each thread loads 4(k) x 4(row) micro-tiles with 16-B loads along
// the contiguous row index, transposes them in registers and writes 4
// consecutive k per plane (ds_write_b64) into the same [plane][row][k] LDS
// image the k-major kernel reads.
template <int NW, int MT, int NT, int BK, int NP = 3>
struct Gemm3TCfg {
  static constexpr int THREADS = 64 * NW;
  static constexpr int BM = 16 * MT * NW, BN = 16 * NT;
  static constexpr int ROW = BK + 16;
  static constexpr int AU = BM * BK / 16, BU = BN * BK / 16;   // 4x4 micro-tiles
  static constexpr int AV = (AU + THREADS - 1) / THREADS, BV = (BU + THREADS - 1) / THREADS;
  static constexpr size_t LDS = sizeof(unsigned short) * NP * (BM + BN) * ROW;
};

template <int BK, int ROWS, int TH, int V>
__device__ __forceinline__ void t_load(float4 (&r)[V][4], const float* __restrict__ X,
                                       int64_t ld, int64_t row0, int64_t rows, int64_t k0,
                                       int64_t kend, int t) {
  constexpr int UR = ROWS / 4;  // micro-tiles along the row index
#pragma unroll
  for (int s = 0; s < V; ++s) {
    const int idx = t + TH * s;
    const int ug = idx % UR, kg = idx / UR;
    const bool on = idx < UR * (BK / 4);
    int64_t col = row0 + 4 * ug;
    col = col + 3 < rows ? col : (rows >= 4 ? rows - 4 : 0);  // clamped (rows >= M are never stored)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t k = k0 + 4 * kg + q;
      r[s][q] = (on && k < kend) ? *reinterpret_cast<const float4*>(X + k * ld + col)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

template <int BK, int ROWS, int TH, int V, int ROW, int NP = 3>
__device__ __forceinline__ void t_store(const float4 (&r)[V][4], unsigned short* __restrict__ sX,
                                        int t) {
  constexpr int UR = ROWS / 4;
#pragma unroll
  for (int s = 0; s < V; ++s) {
    const int idx = t + TH * s;
    if (idx >= UR * (BK / 4)) continue;
    const int ug = idx % UR, kg = idx / UR;
#pragma unroll
    for (int c = 0; c < 4; ++c) {  // row 4ug + c, k = 4kg .. 4kg+3
      if constexpr (NP == 1) {
        const float* p0 = &r[s][0].x;
        const float* p1 = &r[s][1].x;
        const float* p2 = &r[s][2].x;
        const float* p3 = &r[s][3].x;
        uint2 w;
        w.x = bf16_pk(p0[c], p1[c]);
        w.y = bf16_pk(p2[c], p3[c]);
        *reinterpret_cast<uint2*>(sX + (4 * ug + c) * ROW + 4 * kg) = w;
        continue;
      }
      unsigned short h[3][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float* pv = &r[s][q].x;
        split3(pv[c], h[0][q], h[1][q], h[2][q]);
      }
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        uint2 w;
        w.x = (unsigned)h[p][0] | ((unsigned)h[p][1] << 16);
        w.y = (unsigned)h[p][2] | ((unsigned)h[p][3] << 16);
        *reinterpret_cast<uint2*>(sX + (p * ROWS + 4 * ug + c) * ROW + 4 * kg) = w;
      }
    }
  }
}

template <int NW, int MT, int NT, int BK, int NP = 3>
__global__ __launch_bounds__(64 * NW) void k_gemm3_t(const float* __restrict__ A, int64_t lda,
                                                     const float* __restrict__ B, int64_t ldb,
                                                     float* __restrict__ C, int64_t ldc,
                                                     int64_t M, int64_t N, int64_t K,
                                                     int64_t kslice) {
  using Cfg = Gemm3TCfg<NW, MT, NT, BK, NP>;
  constexpr int TH = Cfg::THREADS, BM = Cfg::BM, BN = Cfg::BN, ROW = Cfg::ROW;
  constexpr int AV = Cfg::AV, BV = Cfg::BV;
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  unsigned short* sA = lds;                    // [NP][BM][ROW]
  unsigned short* sB = lds + NP * BM * ROW;    // [NP][BN][ROW]
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, lg = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
  const int64_t kbeg = (int64_t)blockIdx.z * kslice, kend = min(K, kbeg + kslice);
  if (gridDim.z > 1) C += (int64_t)blockIdx.z * M * ldc;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 ra[AV][4], rb[BV][4];
  t_load<BK, BM, TH, AV>(ra, A, lda, m0, M, kbeg, kend, t);
  t_load<BK, BN, TH, BV>(rb, B, ldb, n0, N, kbeg, kend, t);
  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    t_store<BK, BM, TH, AV, ROW, NP>(ra, sA, t);
    t_store<BK, BN, TH, BV, ROW, NP>(rb, sB, t);
    __syncthreads();
    if (k0 + BK < kend) {
      t_load<BK, BM, TH, AV>(ra, A, lda, m0, M, k0 + BK, kend, t);
      t_load<BK, BN, TH, BV>(rb, B, ldb, n0, N, k0 + BK, kend, t);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[MT][NP];
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          af[a][p] = *reinterpret_cast<const bf16x8*>(
              sA + (p * BM + wave * 16 * MT + 16 * a + li) * ROW + kk + 8 * lg);
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        bf16x8 bf[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p)
          bf[p] = *reinterpret_cast<const bf16x8*>(sB + (p * BN + 16 * b + li) * ROW + kk + 8 * lg);
#pragma unroll
        for (int a = 0; a < MT; ++a) acc[a][b] = mfma_planes<NP>(af[a], bf, acc[a][b]);
      }
    }
  }
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int64_t gn = n0 + 16 * b + li;
      if (gn < N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t gm = m0 + wave * 16 * MT + 16 * a + 4 * lg + r;
          if (gm < M) C[gm * ldc + gn] = acc[a][b][r];
        }
      }
    }
}

// ---------------------------------------------------------------------------
// A-direct variant.  Each wave owns 16*MT rows of A, so A needs no LDS: its
// fragments (lane: row l&15, k = 8(l>>4) .. +7, two 16-B loads) go from
// global straight to registers AP k-steps ahead and are split there.  Only
// the shared B planes are staged through LDS, double-buffered: one barrier
// per K-step, and the next step's B is written while this step's MFMAs run.
// Blocks are ordered so the NN column tiles of one row block are dispatched
// together onto one XCD (id % 8 picks the XCD): they share A through L2.
// Requires K % 4 == 0, lda % 4 == 0, 16-B aligned A (checked by the caller).
// ---------------------------------------------------------------------------
// SWZ (k_gemm3d, BK = 32): B rows unpadded (64 B) with the 16-B chunk c of
// row r stored at c ^ PI[(r >> 2) & 3], PI = {0, 2, 3, 1} (swz_chunk): the 16
// lanes of each ds_read_b128 lane group and the 8 of each ds_write_b128 group
// land in distinct 16-B bank slots, as with the 32-B pad, in 2/3 of the LDS
// (80 KB for NT = 13 double-buffered: two workgroups fit a CU)
template <int NW, int MT, int NT, int BK, bool SWZ = false, int NSTG = 2>
struct Gemm3bCfg {
  static constexpr int THREADS = 64 * NW;
  static constexpr int BM = 16 * MT * NW, BN = 16 * NT;
  static constexpr int ROW = SWZ ? BK : BK + 16;  // conflict-free ds_read_b128 (see Gemm3Cfg)
  static constexpr int BV = (3 * BN * (BK / 8) + THREADS - 1) / THREADS;  // uint4 per thread
  static constexpr int STAGE = 3 * BN * ROW;                              // bf16 per stage
  static constexpr size_t LDS = sizeof(unsigned short) * NSTG * STAGE;
};
__device__ __forceinline__ int swz_chunk(int c, int r) {
  return c ^ ((0x78 >> (2 * ((r >> 2) & 3))) & 3);  // PI = {0, 2, 3, 1}[(r >> 2) & 3]
}

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
// eight elements (two float4) -> the three plane fragments
__device__ __forceinline__ void split3_frag(const f32x4& lo, const f32x4& hi, bf16x8 (&h)[3]) {
  u32x4_t w0, w1, w2;
  unsigned a, b, c;
  split3_pk(lo[0], lo[1], a, b, c); w0[0] = a; w1[0] = b; w2[0] = c;
  split3_pk(lo[2], lo[3], a, b, c); w0[1] = a; w1[1] = b; w2[1] = c;
  split3_pk(hi[0], hi[1], a, b, c); w0[2] = a; w1[2] = b; w2[2] = c;
  split3_pk(hi[2], hi[3], a, b, c); w0[3] = a; w1[3] = b; w2[3] = c;
  h[0] = __builtin_bit_cast(bf16x8, w0);
  h[1] = __builtin_bit_cast(bf16x8, w1);
  h[2] = __builtin_bit_cast(bf16x8, w2);
}

template <int NW, int MT, int NT, int BK, int AP>
__global__ __launch_bounds__(64 * NW) void k_gemm3b(const float* __restrict__ A, int64_t lda,
                                                    const unsigned short* __restrict__ Bp,
                                                    int64_t ldb, int64_t bplane,
                                                    float* __restrict__ C, int64_t ldc, int64_t M,
                                                    int64_t N, int64_t K, int nm, int nn) {
  using Cfg = Gemm3bCfg<NW, MT, NT, BK>;
  constexpr int TH = Cfg::THREADS, BM = Cfg::BM, BN = Cfg::BN, ROW = Cfg::ROW, BV = Cfg::BV;
  constexpr int STAGE = Cfg::STAGE, BC = BK / 8, KS = BK / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, lg = lane >> 4;
  // XCD-grouped block order: id = q*8*nn + n*8 + r  ->  row block q*8 + r, column block n
  const int id = blockIdx.x;
  const int q = id / (8 * nn), rem = id - q * 8 * nn;
  const int nb = rem >> 3, mb = q * 8 + (rem & 7);
  if (mb >= nm) return;
  const int64_t m0 = (int64_t)mb * BM, n0 = (int64_t)nb * BN;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A: rows of this wave through a buffer descriptor (rows >= M read 0)
  const int64_t arow0 = m0 + (int64_t)wave * 16 * MT;
  const int64_t arows = M - arow0;
  const rsrc_t ra_src = make_rsrc(A + (arow0 > M ? 0 : arow0 * lda),
                                  arows > 0 ? (uint32_t)(min(arows, (int64_t)16 * MT) * lda * 4) : 0u);
  f32x4 ra[AP][MT][KS][2];
  auto load_a = [&](int set, int64_t k0) {
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int hv = 0; hv < 2; ++hv) {
          const int64_t k = k0 + 32 * ks + 8 * lg + 4 * hv;
          const int off = k < K ? (int)(((16 * a + li) * lda + k) * 4) : OOB;
          ra[set][a][ks][hv] = bld4(ra_src, off);
        }
  };
  // B planes: [3][N][ldb] bf16, rows >= N clamped (never stored)
  uint4 rb[BV];
  auto load_b = [&](int64_t k0) {
#pragma unroll
    for (int sv = 0; sv < BV; ++sv) {
      const int idx = t + TH * sv;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (idx < 3 * BN * BC) {
        const int p = idx / (BN * BC), r2 = idx - p * BN * BC;
        const int r = r2 / BC, c = r2 - r * BC;
        const int64_t gn = min(n0 + r, N - 1);
        v = *reinterpret_cast<const uint4*>(Bp + p * bplane + gn * ldb + k0 + 8 * c);
      }
      rb[sv] = v;
    }
  };
  auto store_b = [&](unsigned short* sB) {
#pragma unroll
    for (int sv = 0; sv < BV; ++sv) {
      const int idx = t + TH * sv;
      if (idx < 3 * BN * BC) {
        const int p = idx / (BN * BC), r2 = idx - p * BN * BC;
        const int r = r2 / BC, c = r2 - r * BC;
        *reinterpret_cast<uint4*>(sB + (p * BN + r) * ROW + 8 * c) = rb[sv];
      }
    }
  };

  const int nk = (int)((K + BK - 1) / BK);
#pragma unroll
  for (int s = 0; s < AP; ++s)
    if (s < nk) load_a(s, (int64_t)s * BK);
  load_b(0);
  store_b(lds);
  if (nk > 1) load_b(BK);
  __syncthreads();
  for (int s = 0; s < nk; ++s) {
    const unsigned short* sB = lds + (s & 1) * STAGE;
    const int set = s % AP;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 af[MT][3];
#pragma unroll
      for (int a = 0; a < MT; ++a) split3_frag(ra[set][a][ks][0], ra[set][a][ks][1], af[a]);
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        bf16x8 bf[3];
#pragma unroll
        for (int p = 0; p < 3; ++p)
          bf[p] = *reinterpret_cast<const bf16x8*>(sB + (p * BN + 16 * b + li) * ROW + 32 * ks +
                                                   8 * lg);
#pragma unroll
        for (int a = 0; a < MT; ++a) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][2], bf[0], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][1], bf[1], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][0], bf[2], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][1], bf[0], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][0], bf[1], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][0], bf[0], acc[a][b], 0, 0, 0);
        }
      }
    }
    if (s + AP < nk) load_a(set, (int64_t)(s + AP) * BK);
    if (s + 1 < nk) {
      store_b(lds + ((s + 1) & 1) * STAGE);
      if (s + 2 < nk) load_b((int64_t)(s + 2) * BK);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int64_t gn = n0 + 16 * b + li;
      if (gn < N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t gm = arow0 + 16 * a + 4 * lg + r;
          if (gm < M) C[gm * ldc + gn] = acc[a][b][r];
        }
      }
    }
}

// ---------------------------------------------------------------------------
// k_gemm3c: k_gemm3b's operand flow (A straight to registers, split there; B
// planes double-buffered in LDS, one barrier per K-step) with the step
// reordered so no phase of the workgroup runs without MFMAs:
//   top of step s   store the B planes of step s+1 (loaded during step s-1)
//                   into the other stage, issue the loads of step s+2's B;
//   body            the MFMAs of step s, B fragments of column tile b+1 read
//                   while tile b's MFMAs run (scheduling-group barriers);
//   end             A loads of step s+AP, barrier.
// The stage written at the top of step s was last read in step s-1, which
// every wave finished before the barrier that closed it.
// ---------------------------------------------------------------------------
#ifdef SV2N_GEMM_CLOCK
// diagnostic build of tools/gemm3_tune.hip only: per workgroup (shader clock
// ticks, 100 MHz real-time ticks) between the first and the last instruction
// of wave 0, written to a buffer nothing else reads
__device__ unsigned long long g_gemm_clock[2 * 4096];
#endif
// ABL (tools/gemm3_tune.hip timing ablations only; results are wrong when
// set): 1 no A split, 2 no B staging, 3 no barrier in the loop, 4 no A loads
template <int NW, int MT, int NT, int BK, int AP, int ABL = 0, int PD = 1>
__global__ __launch_bounds__(64 * NW) void k_gemm3c(const float* __restrict__ A, int64_t lda,
                                                    const unsigned short* __restrict__ Bp,
                                                    int64_t ldb, int64_t bplane,
                                                    float* __restrict__ C, int64_t ldc, int64_t M,
                                                    int64_t N, int64_t K, int nm, int nn) {
  using Cfg = Gemm3bCfg<NW, MT, NT, BK>;
  constexpr int TH = Cfg::THREADS, BN = Cfg::BN, ROW = Cfg::ROW, BV = Cfg::BV;
  constexpr int STAGE = Cfg::STAGE, BC = BK / 8, KS = BK / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
#ifdef SV2N_GEMM_CLOCK
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, lg = lane >> 4;
  const int id = blockIdx.x;
  const int q = id / (8 * nn), rem = id - q * 8 * nn;
  const int nb = rem >> 3, mb = q * 8 + (rem & 7);
  if (mb >= nm) return;
  const int64_t m0 = (int64_t)mb * Cfg::BM, n0 = (int64_t)nb * BN;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t arow0 = m0 + (int64_t)wave * 16 * MT;
  const int64_t arows = M - arow0;
  const rsrc_t ra_src = make_rsrc(A + (arow0 > M ? 0 : arow0 * lda),
                                  arows > 0 ? (uint32_t)(min(arows, (int64_t)16 * MT) * lda * 4) : 0u);
  f32x4 ra[AP][MT][KS][2];
  auto load_a = [&](int set, int64_t k0) {
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int hv = 0; hv < 2; ++hv) {
          const int64_t k = k0 + 32 * ks + 8 * lg + 4 * hv;
          const int off = k < K ? (int)(((16 * a + li) * lda + k) * 4) : OOB;
          ra[set][a][ks][hv] = ABL == 4 ? f32x4{1.f, 2.f, 3.f, (float)off} : bld4(ra_src, off);
        }
  };
  uint4 rb[BV];
  auto load_b = [&](int64_t k0) {
#pragma unroll
    for (int sv = 0; sv < BV; ++sv) {
      const int idx = t + TH * sv;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (idx < 3 * BN * BC) {
        const int p = idx / (BN * BC), r2 = idx - p * BN * BC;
        const int r = r2 / BC, c = r2 - r * BC;
        const int64_t gn = min(n0 + r, N - 1);
        v = *reinterpret_cast<const uint4*>(Bp + p * bplane + gn * ldb + k0 + 8 * c);
      }
      rb[sv] = v;
    }
  };
  auto store_b = [&](unsigned short* sB) {
#pragma unroll
    for (int sv = 0; sv < BV; ++sv) {
      const int idx = t + TH * sv;
      if (idx < 3 * BN * BC) {
        const int p = idx / (BN * BC), r2 = idx - p * BN * BC;
        const int r = r2 / BC, c = r2 - r * BC;
        *reinterpret_cast<uint4*>(sB + (p * BN + r) * ROW + 8 * c) = rb[sv];
      }
    }
  };

  const int nk = (int)((K + BK - 1) / BK);
#pragma unroll
  for (int s = 0; s < AP; ++s)
    if (s < nk) load_a(s, (int64_t)s * BK);
  load_b(0);
  store_b(lds);
  if (nk > 1) load_b(BK);
  __syncthreads();
  // one step; `set` (the A register set) is a compile-time index
  auto step = [&](int s, auto set_c) {
    constexpr int set = decltype(set_c)::value;
    const unsigned short* sB = lds + (s & 1) * STAGE;
    if (ABL != 2 && s + 1 < nk) {
      store_b(lds + ((s + 1) & 1) * STAGE);
      if (s + 2 < nk) load_b((int64_t)(s + 2) * BK);
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 af[MT][3];
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        if constexpr (ABL == 1) {
          af[a][0] = __builtin_bit_cast(bf16x8, ra[set][a][ks][0]);
          af[a][1] = __builtin_bit_cast(bf16x8, ra[set][a][ks][1]);
          af[a][2] = af[a][0];
        } else {
          split3_frag(ra[set][a][ks][0], ra[set][a][ks][1], af[a]);
        }
      }
      // B fragments PD column tiles ahead, in a ring of PD + 1 register sets
      bf16x8 bq[PD + 1][3];
#pragma unroll
      for (int b = 0; b < PD && b < NT; ++b)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          bq[b][p] = *reinterpret_cast<const bf16x8*>(sB + (p * BN + 16 * b + li) * ROW + 32 * ks +
                                                      8 * lg);
      __builtin_amdgcn_sched_group_barrier(0x100, 3 * (PD < NT ? PD : NT), 0);
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        if (b + PD < NT) {
#pragma unroll
          for (int p = 0; p < 3; ++p)
            bq[(b + PD) % (PD + 1)][p] = *reinterpret_cast<const bf16x8*>(
                sB + (p * BN + 16 * (b + PD) + li) * ROW + 32 * ks + 8 * lg);
          __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        }
#pragma unroll
        for (int a = 0; a < MT; ++a) acc[a][b] = mfma_planes<3>(af[a], bq[b % (PD + 1)], acc[a][b]);
        __builtin_amdgcn_sched_group_barrier(0x008, 6 * MT, 0);
      }
    }
    if (s + AP < nk) load_a(set, (int64_t)(s + AP) * BK);
    if constexpr (ABL != 3) __syncthreads();
  };
  static_assert(AP == 2 || AP == 3, "A register sets");
  for (int s = 0; s < nk; s += AP) {
    step(s, std::integral_constant<int, 0>{});
    if (s + 1 < nk) step(s + 1, std::integral_constant<int, 1>{});
    if constexpr (AP == 3)
      if (s + 2 < nk) step(s + 2, std::integral_constant<int, 2>{});
  }
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int64_t gn = n0 + 16 * b + li;
      if (gn < N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t gm = arow0 + 16 * a + 4 * lg + r;
          if (gm < M) C[gm * ldc + gn] = acc[a][b][r];
        }
      }
    }
#ifdef SV2N_GEMM_CLOCK
  if (t == 0 && blockIdx.x < 4096) {
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    g_gemm_clock[2 * blockIdx.x] = c1 - c0;
    g_gemm_clock[2 * blockIdx.x + 1] = r1 - r0;
  }
#endif
}

// compile-time loop: f(std::integral_constant<int, 0>{}) ... f(<N-1>)
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// ---------------------------------------------------------------------------
// k_gemm3d: k_gemm3c with the work between two barriers spread under the
// step's MFMAs instead of run ahead of them (BK = 32: one K-step per barrier):
//   * the bf16x3 split of step s+1's A fragments runs during step s, a pair
//     of elements per column tile (split3_pk: ~11 VALU) beside its MFMAs
//     (splitting in the last tiles instead: 91.8 vs 88.8 us at C2 L0);
//   * the B planes of step s+1 go to the other LDS stage one ds_write per
//     column tile, and step s+2's loads follow the last write;
// so after the barrier a wave only waits for its first B fragments.
// Scheduling-group barriers hold the compiler to that interleave.
// ---------------------------------------------------------------------------
// BD: B fragments read BD column tiles ahead of their MFMAs (BD + 1 register
// sets; 1 = the next tile's reads under the current tile's MFMAs).
template <int NW, int MT, int NT, int AP, bool MASK = false, int BD = 1, bool SWZ = false,
          bool STG = false>
__global__ __launch_bounds__(64 * NW) void k_gemm3d(const float* __restrict__ A, int64_t lda,
                                                    const unsigned short* __restrict__ Bp,
                                                    int64_t ldb, int64_t bplane,
                                                    float* __restrict__ C, int64_t ldc, int64_t M,
                                                    int64_t N, int64_t K, int nm, int nn,
                                                    const float* __restrict__ Y, int64_t ldy) {
  constexpr int BK = 32;
  static_assert(!STG || SWZ, "three padded stages do not fit the LDS");
  constexpr int NSTG = STG ? 3 : 2;
  using Cfg = Gemm3bCfg<NW, MT, NT, BK, SWZ, NSTG>;
  constexpr int TH = Cfg::THREADS, BN = Cfg::BN, ROW = Cfg::ROW, BV = Cfg::BV;
  constexpr int STAGE = Cfg::STAGE, BC = BK / 8;
  // STG (with SWZ): waves NW/2.. run half a K-step behind the first half —
  // their barrier sits after column tile MIDB, the first half's at the end of
  // the step — so the two waves of a SIMD are never in the same phase (one
  // resumes MFMAs on fragments read before the barrier while the other waits
  // for its first ones).  B stages in a ring of three: during barrier
  // interval k every wave writes stage k+1, the first half reads stage k,
  // the second half stages k-1 and k.
  constexpr int MIDB = (NT + 1) / 2 - 1;
  static_assert(!STG || BV <= MIDB, "the second half stages B before its barrier");
  constexpr int NPAIR = 4 * MT;  // split3_pk pairs per step (8 floats per fragment)
  constexpr int PPT = (NPAIR + NT - 1) / NT;  // pairs split per column tile
  static_assert(BV + 1 < NT, "interleave needs enough column tiles");
  static_assert(AP >= 2 && AP <= 3, "A register sets");
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, lg = lane >> 4;
  const int id = blockIdx.x;
  const int q = id / (8 * nn), rem = id - q * 8 * nn;
  const int nb = rem >> 3, mb = q * 8 + (rem & 7);
  if (mb >= nm) return;
  const int64_t m0 = (int64_t)mb * Cfg::BM, n0 = (int64_t)nb * BN;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t arow0 = m0 + (int64_t)wave * 16 * MT;
  const int64_t arows = M - arow0;
  const rsrc_t ra_src = make_rsrc(A + (arow0 > M ? 0 : arow0 * lda),
                                  arows > 0 ? (uint32_t)(min(arows, (int64_t)16 * MT) * lda * 4) : 0u);
  f32x4 ra[AP][MT][2];
  auto load_a = [&](int set, int64_t k0) __attribute__((always_inline)) {
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int hv = 0; hv < 2; ++hv) {
        const int64_t k = k0 + 8 * lg + 4 * hv;
        const int off = k < K ? (int)(((16 * a + li) * lda + k) * 4) : OOB;
        ra[set][a][hv] = bld4(ra_src, off);
      }
  };
  u32x4_t rb[BV];
  // branch-free staging (branches would split the interleaved block): slots
  // past the image repeat the last one (same value, same address)
  // 16 consecutive slots = 4 rows x 4 chunks, row-minor: each 8-lane group of
  // a ds_write_b128 then covers 8 distinct 4-dword bank windows (96-B rows;
  // row-major slots put lanes 6-7 on lanes 0-1's banks)
  static_assert(BC == 4 && BN % 4 == 0, "slot order assumes 4 chunks per row");
  auto b_slot = [&](int sv, int& p, int& r, int& c) __attribute__((always_inline)) {
    const int idx = min(t + TH * sv, 3 * BN * BC - 1);
    p = idx / (BN * BC);
    const int r2 = idx - p * BN * BC;
    r = ((r2 >> 4) << 2) + (r2 & 3);
    c = (r2 >> 2) & 3;
  };
  auto load_b1 = [&](int sv, int64_t k0) __attribute__((always_inline)) {
    int p, r, c;
    b_slot(sv, p, r, c);
    const int64_t gn = min(n0 + r, N - 1);
    rb[sv] = *reinterpret_cast<const u32x4_t*>(Bp + p * bplane + gn * ldb + k0 + 8 * c);
  };
  auto store_b1 = [&](int sv, unsigned short* sB) __attribute__((always_inline)) {
    int p, r, c;
    b_slot(sv, p, r, c);
    *reinterpret_cast<u32x4_t*>(sB + (p * BN + r) * ROW + 8 * (SWZ ? swz_chunk(c, r) : c)) = rb[sv];
  };
  // fragment chunk of lane group lg in rows 16b + li (the swizzle depends on li only)
  const int bchunk = 8 * (SWZ ? swz_chunk(lg, li) : lg);
  // packed bf16 planes of the current step's A fragments, and the next step's
  u32x4_t afc[MT][3], afn[MT][3];
  auto split_pair = [&](u32x4_t (&dst)[MT][3], const f32x4 (&src)[MT][2], int pr) {
    const int a = pr >> 2, qd = pr & 3;  // fragment a, word qd (elements 2qd, 2qd+1)
    const f32x4& v = src[a][qd >> 1];
    unsigned w0, w1, w2;
    split3_pk(v[2 * (qd & 1)], v[2 * (qd & 1) + 1], w0, w1, w2);
    dst[a][0][qd] = w0;
    dst[a][1][qd] = w1;
    dst[a][2][qd] = w2;
  };

  // MASK: the ReLU backward of the consumer fused into the store, C = (Y > 0)
  // ? A·Bᵀ : 0 (act_bwd<ACT_RELU> exactly; the n <= 32 attention backward then
  // reads dZ instead of dy and y).  Y is loaded before the main loop so its
  // latency hides under the MFMAs (loaded after it, the epilogue waited on
  // it: C2 L1 dX 24 -> 37 us).
  float yv[MASK ? MT : 1][MASK ? NT : 1][4];
  if constexpr (MASK) {
    const rsrc_t ry = make_rsrc(Y + (arow0 > M ? 0 : arow0 * ldy),
                                arows > 0 ? (uint32_t)(min(arows, (int64_t)16 * MT) * ldy * 4) : 0u);
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const int gn = (int)n0 + 16 * b + li;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          yv[a][b][r] = bld(ry, gn < N ? (int)(((16 * a + 4 * lg + r) * ldy + gn) * 4) : OOB);
      }
  }
  const int nk = (int)((K + BK - 1) / BK);
#pragma unroll
  for (int s = 0; s < AP; ++s)
    if (s < nk) load_a(s, (int64_t)s * BK);
#pragma unroll
  for (int sv = 0; sv < BV; ++sv) load_b1(sv, 0);
#pragma unroll
  for (int sv = 0; sv < BV; ++sv) store_b1(sv, lds);
  if (nk > 1)
#pragma unroll
    for (int sv = 0; sv < BV; ++sv) load_b1(sv, BK);
#pragma unroll
  for (int pr = 0; pr < NPAIR; ++pr) split_pair(afc, ra[0], pr);
  __syncthreads();
  if constexpr (MASK) {  // the mask lives in registers from here (no sinking into the epilogue)
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(yv[a][b][r]));
  }

  auto step = [&](int s, auto set_c) __attribute__((always_inline)) {
    constexpr int set = decltype(set_c)::value, nset = (set + 1) % AP;
    const unsigned short* sB = lds + (STG ? s % 3 : s & 1) * STAGE;
    unsigned short* sW = lds + (STG ? (s + 1) % 3 : (s + 1) & 1) * STAGE;
    // the last steps stage a copy nobody reads (the other stage is free after
    // the barrier) and reload the last K-step: no branch in the block
    const int64_t kb2 = (int64_t)min(s + 2, nk - 1) * BK;
    bf16x8 af[MT][3];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int p = 0; p < 3; ++p) af[a][p] = __builtin_bit_cast(bf16x8, afc[a][p]);
    static_assert(BD >= 1 && BD < NT, "B read distance");
    bf16x8 bq[BD + 1][3];
    static_for<BD>([&](auto bc) __attribute__((always_inline)) {
      constexpr int b = decltype(bc)::value;
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bq[b][p] = *reinterpret_cast<const bf16x8*>(sB + (p * BN + 16 * b + li) * ROW + bchunk);
    });
    __builtin_amdgcn_sched_group_barrier(0x100, 3 * BD, 0);
    static_for<NT>([&](auto bc) __attribute__((always_inline)) {
      constexpr int b = decltype(bc)::value;
      if constexpr (b + BD < NT) {
#pragma unroll
        for (int p = 0; p < 3; ++p)
          bq[(b + BD) % (BD + 1)][p] = *reinterpret_cast<const bf16x8*>(
              sB + (p * BN + 16 * (b + BD) + li) * ROW + bchunk);
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
      }
      if constexpr (b < BV) {
        store_b1(b, sW);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      } else if constexpr (b == BV) {
#pragma unroll
        for (int sv = 0; sv < BV; ++sv) load_b1(sv, kb2);
        __builtin_amdgcn_sched_group_barrier(0x020, BV, 0);
      }
      if constexpr (b * PPT < NPAIR) {
        static_for<PPT>([&](auto pc) __attribute__((always_inline)) {
          constexpr int pr = b * PPT + decltype(pc)::value;
          if constexpr (pr < NPAIR) split_pair(afn, ra[nset], pr);
        });
        __builtin_amdgcn_sched_group_barrier(0x002, 11 * PPT, 0);
      }
#pragma unroll
      for (int a = 0; a < MT; ++a) acc[a][b] = mfma_planes<3>(af[a], bq[b % (BD + 1)], acc[a][b]);
      __builtin_amdgcn_sched_group_barrier(0x008, 6 * MT, 0);
      if constexpr (STG && b == MIDB) {
        if (wave >= NW / 2) __syncthreads();  // the second half's barrier: mid-step
      }
    });
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int p = 0; p < 3; ++p) afc[a][p] = afn[a][p];
    if (s + AP < nk) load_a(set, (int64_t)(s + AP) * BK);
    if constexpr (STG) {
      if (wave < NW / 2) __syncthreads();
    } else {
      __syncthreads();
    }
  };
  for (int s = 0; s < nk; s += AP) {
    step(s, std::integral_constant<int, 0>{});
    if (s + 1 < nk) step(s + 1, std::integral_constant<int, 1>{});
    if constexpr (AP == 3)
      if (s + 2 < nk) step(s + 2, std::integral_constant<int, 2>{});
  }
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int64_t gn = n0 + 16 * b + li;
      if (gn < N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t gm = arow0 + 16 * a + 4 * lg + r;
          float v = acc[a][b][r];
          if constexpr (MASK) v = yv[a][b][r] > 0.f ? v : 0.f;
          if (gm < M) C[gm * ldc + gn] = v;
        }
      }
    }
}

}  // namespace sv2n
