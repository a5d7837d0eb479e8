// bf16-operand GEMM with fp32 accumulation for the bf16 execution mode
// (BASELINE config C3: the reference under bf16 autocast): the projection
// C[M][N] = bf16(A)[M][K] · Bᵀ, A fp32 row-major (rounded to bf16 while it is
// staged), B one bf16 plane [N][Kp] (the weight prep's bf16_rn(Waug)).
//
// k_gemm_bf16nt: 256 threads = 4 waves in a 2 x 2 grid, block tile 128 x 128,
// each wave 64 x 64 = 4 x 4 tiles of v_mfma_f32_16x16x32_bf16; K in steps of
// 64 through a double-buffered LDS image of both operands ([row][64 + 16]
// bf16: the 16-B fragment reads of 16 rows land on distinct bank groups).
// Per step: the next step's operands (loaded during the previous step) are
// converted and written to the free stage, the loads of the step after are
// issued, then this step's 32 MFMAs run; one barrier per step.  Every B
// fragment read feeds four MFMAs and every A fragment four (the bf16x3 kernels
// give each wave 16 rows, which made LDS reads, not MFMAs, the bound at one
// product per fragment pair).  Blocks are ordered so the column tiles of one
// row block run on one XCD (they share A through that XCD's L2).
#pragma once
#include "sv2n_gemm3_kernel.h"

namespace sv2n {

constexpr int BF_BM = 128, BF_BN = 128, BF_BK = 64, BF_ROW = BF_BK + 16;
constexpr int BF_STAGE = (BF_BM + BF_BN) * BF_ROW;  // bf16 elements per stage
constexpr size_t BF_LDS = sizeof(unsigned short) * 2 * BF_STAGE;

static __global__ __attribute__((unused)) __launch_bounds__(256, 2) void k_gemm_bf16nt(const float* __restrict__ A, int64_t lda,
                                                         const unsigned short* __restrict__ Bp,
                                                         int64_t ldb, float* __restrict__ C,
                                                         int64_t ldc, int64_t M, int64_t N,
                                                         int64_t K, int nm, int nn) {
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, lg = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-grouped order: id = q*8*nn + nb*8 + r -> row block q*8 + r, column block nb
  const int id = blockIdx.x;
  const int q = id / (8 * nn), rem = id - q * 8 * nn;
  const int nb = rem >> 3, mb = q * 8 + (rem & 7);
  if (mb >= nm) return;
  const int64_t m0 = (int64_t)mb * BF_BM, n0 = (int64_t)nb * BF_BN;

  // staging roles: A — 8 consecutive floats (two 16-B loads) of row ar,
  // k = 8·ac .. +7, four such pieces per thread (rows ar + 32p); B — one 16-B
  // piece (8 bf16) of row br, four per thread (rows br + 32p)
  const int ar = t >> 3, ac = t & 7;
  const rsrc_t ra = make_rsrc(A + m0 * lda, (uint32_t)(min((int64_t)BF_BM, M - m0) * lda * 4));
  const rsrc_t rb = make_rsrc(Bp + n0 * ldb, (uint32_t)(min((int64_t)BF_BN, N - n0) * ldb * 2));
  f32x4 pa[4][2];
  u32x4 pb[4];
  auto load = [&](int64_t k0) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int64_t k = k0 + 8 * ac;
      const int row = ar + 32 * p;
      pa[p][0] = bld4(ra, k < K ? (int)((row * lda + k) * 4) : OOB);
      pa[p][1] = bld4(ra, k + 4 < K ? (int)((row * lda + k + 4) * 4) : OOB);
      pb[p] = bld4_u32(rb, (int)((row * ldb + k0 + 8 * ac) * 2));  // Kp: zero-padded
    }
  };
  auto store = [&](unsigned short* sA) __attribute__((always_inline)) {
    unsigned short* sB = sA + BF_BM * BF_ROW;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = ar + 32 * p;
      u32x4 w;
      w[0] = bf16_pk(pa[p][0][0], pa[p][0][1]);
      w[1] = bf16_pk(pa[p][0][2], pa[p][0][3]);
      w[2] = bf16_pk(pa[p][1][0], pa[p][1][1]);
      w[3] = bf16_pk(pa[p][1][2], pa[p][1][3]);
      *reinterpret_cast<u32x4*>(sA + row * BF_ROW + 8 * ac) = w;
      *reinterpret_cast<u32x4*>(sB + row * BF_ROW + 8 * ac) = pb[p];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((K + BF_BK - 1) / BF_BK);
  load(0);
  store(lds);
  if (nk > 1) load(BF_BK);
  __syncthreads();
  for (int s = 0; s < nk; ++s) {
    const unsigned short* sA = lds + (s & 1) * BF_STAGE;
    const unsigned short* sB = sA + BF_BM * BF_ROW;
    if (s + 1 < nk) {
      store(lds + ((s + 1) & 1) * BF_STAGE);  // that stage was last read in step s - 1
      if (s + 2 < nk) load((int64_t)(s + 2) * BF_BK);
    }
#pragma unroll
    for (int ks = 0; ks < BF_BK / 32; ++ks) {
      bf16x8 af[4], bf[4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
        af[a] = *reinterpret_cast<const bf16x8*>(sA + (wm * 64 + 16 * a + li) * BF_ROW + 32 * ks +
                                                 8 * lg);
#pragma unroll
      for (int b = 0; b < 4; ++b)
        bf[b] = *reinterpret_cast<const bf16x8*>(sB + (wn * 64 + 16 * b + li) * BF_ROW + 32 * ks +
                                                 8 * lg);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
    __syncthreads();
  }
  // C tile: lane (li, lg) holds rows 4lg + r, column li of each 16 x 16 tile
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int64_t gn = n0 + wn * 64 + 16 * b + li;
      if (gn < N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t gm = m0 + wm * 64 + 16 * a + 4 * lg + r;
          if (gm < M) C[gm * ldc + gn] = acc[a][b][r];
        }
      }
    }
}

}  // namespace sv2n
