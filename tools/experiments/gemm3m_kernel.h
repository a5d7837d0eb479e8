// Projection GEMM C[M][N] = A[M][K] · Bᵀ on v_mfma_f32_32x32x16_bf16, A fp32
// (split into NP bf16 planes in registers), B pre-split planes [NP][N][Kp]
// (the weight prep's output, zero past K).  NP = 3: the f32-accurate six
// products with plane orders p + q <= 2; NP = 1: bf16 operands.
//
// Why 32x32x16 (k_gemm3d uses 16x16x32): an MFMA of this shape holds the
// SIMD's vector issue for 8 of its 32 cycles (MI355X_MICROARCH.md, issue
// costs), so the A split (split3_pk), the B staging writes and the address
// work fit in the MFMA gaps at ONE wave per SIMD, and each B fragment read
// from LDS feeds a 32-row tile (half the LDS bytes per product of a 16-row
// wave tile).
//
// Workgroup: 4 waves; wave w owns A rows m0 + 32w .. +31 (loaded straight to
// registers, each lane 16 consecutive k of its row per K-step) and all NT
// 32-column tiles of the block; the 4 waves share the block's B tile, staged
// through a double-buffered LDS image [NP][BN][40] bf16 per K-step of 32
// (80-B rows: the 16 rows each ds_read_b128 lane group reads fall in 16
// distinct 16-B bank slots).  K-step = 2 MFMA substeps of 16; lane (r, h)
// feeds k = k0 + 16h + 8·sub + j to both operands (a fixed bijection of the
// step's 32 k, so every k is summed exactly once).  Per step the next step's
// B planes go to the other LDS stage one slot per column tile, the loads of
// the step after follow, and the next A fragments are split beside the
// MFMAs; one barrier per step.  XCD-grouped block order as k_gemm3d.
#pragma once
#include "../../spotv2net_amd/csrc/sv2n_gemm3_kernel.h"

namespace sv2n {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NT, int NP>
struct Gemm3mCfg {
  static constexpr int NW = 4, THREADS = 256, BK = 32, ROW = BK + 8;  // 80-B rows
  static constexpr int BM = 32 * NW, BN = 32 * NT;
  static constexpr int STAGE = NP * BN * ROW;                         // bf16 per stage
  static constexpr size_t LDS = sizeof(unsigned short) * 2 * STAGE;
  static constexpr int SLOTS = NP * BN * (BK / 8);                    // 16-B pieces per step
  static constexpr int BV = (SLOTS + THREADS - 1) / THREADS;
};

template <int NP>
__device__ __forceinline__ f32x16 mfma32_planes(const bf16x8 (&a)[NP], const bf16x8 (&b)[NP],
                                                f32x16 acc) {
  if constexpr (NP == 3) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  }
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
}

template <int NT, int NP>
__global__ __launch_bounds__(256) void k_gemm3m(const float* __restrict__ A, int64_t lda,
                                                const unsigned short* __restrict__ Bp,
                                                int64_t ldb, int64_t bplane,
                                                float* __restrict__ C, int64_t ldc, int64_t M,
                                                int64_t N, int64_t K, int nm, int nn) {
  using Cfg = Gemm3mCfg<NT, NP>;
  constexpr int BK = Cfg::BK, BN = Cfg::BN, ROW = Cfg::ROW, BV = Cfg::BV, STAGE = Cfg::STAGE;
  constexpr int SLOTS = Cfg::SLOTS;
  constexpr int NG = 2 * NT;                      // MFMA groups per step (substep x tile)
  constexpr int NPAIR = 8;                        // split pairs per step (16 floats)
  static_assert(BV + 1 < NG, "interleave needs enough MFMA groups");
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int id = blockIdx.x;
  const int q8 = id / (8 * nn), rem = id - q8 * 8 * nn;
  const int nb = rem >> 3, mb = q8 * 8 + (rem & 7);
  if (mb >= nm) return;
  const int64_t m0 = (int64_t)mb * Cfg::BM, n0 = (int64_t)nb * BN;

  f32x16 acc[NT];
#pragma unroll
  for (int b = 0; b < NT; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

  // A: this wave's 32 rows; lane (lr, lh) reads k0 + 16lh .. +15 of row lr
  const int64_t arow0 = m0 + (int64_t)wave * 32;
  const int64_t arows = M - arow0;
  const rsrc_t ra_src = make_rsrc(A + (arow0 > M ? 0 : arow0 * lda),
                                  arows > 0 ? (uint32_t)(min(arows, (int64_t)32) * lda * 4) : 0u);
  f32x4 ra[2][4];
  auto load_a = [&](int set, int64_t k0) __attribute__((always_inline)) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t k = k0 + 16 * lh + 4 * v;
      ra[set][v] = bld4(ra_src, k < K ? (int)((lr * lda + k) * 4) : OOB);
    }
  };
  // B staging slots: piece (plane p, row r, 16-B chunk c) of the step's tile;
  // slots past the image repeat the last one (branch-free)
  u32x4_t rb[BV];
  auto b_slot = [&](int sv, int& p, int& r, int& c) __attribute__((always_inline)) {
    const int idx = min(t + 256 * sv, SLOTS - 1);
    p = idx / (BN * 4);
    const int r2 = idx - p * BN * 4;
    r = r2 >> 2;
    c = r2 & 3;
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
    *reinterpret_cast<u32x4_t*>(sB + (p * BN + r) * ROW + 8 * c) = rb[sv];
  };
  // packed bf16 planes of the step's A fragments [substep][plane], current and next
  u32x4_t afc[2][NP], afn[2][NP];
  auto split_pair = [&](u32x4_t (&dst)[2][NP], const f32x4 (&src)[4], int pr) {
    // pair pr: floats 2pr, 2pr+1 of the lane's 16 -> substep pr / 4, word pr % 4
    const f32x4& v = src[pr >> 1];
    const int e = 2 * (pr & 1), sub = pr >> 2, w = pr & 3;
    if constexpr (NP == 3) {
      unsigned w0, w1, w2;
      split3_pk(v[e], v[e + 1], w0, w1, w2);
      dst[sub][0][w] = w0;
      dst[sub][1][w] = w1;
      dst[sub][2][w] = w2;
    } else {
      dst[sub][0][w] = bf16_pk(v[e], v[e + 1]);
    }
  };

  const int nk = (int)((K + BK - 1) / BK);
  load_a(0, 0);
  if (nk > 1) load_a(1, BK);
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

  auto step = [&](int s, auto set_c) __attribute__((always_inline)) {
    constexpr int set = decltype(set_c)::value, nset = set ^ 1;
    const unsigned short* sB = lds + (s & 1) * STAGE;
    unsigned short* sW = lds + ((s + 1) & 1) * STAGE;
    const int64_t kb2 = (int64_t)min(s + 2, nk - 1) * BK;
    bf16x8 af[2][NP];
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int p = 0; p < NP; ++p) af[sb][p] = __builtin_bit_cast(bf16x8, afc[sb][p]);
    // B fragment of group g = (substep g / NT, tile g % NT), plane p
    auto bfrag = [&](int g, int p) __attribute__((always_inline)) {
      const int sb = g / NT, b = g - sb * NT;
      return *reinterpret_cast<const bf16x8*>(sB + (p * BN + 32 * b + lr) * ROW + 16 * lh + 8 * sb);
    };
    bf16x8 bq[2][NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) bq[0][p] = bfrag(0, p);
    __builtin_amdgcn_sched_group_barrier(0x100, NP, 0);
    static_for<NG>([&](auto gc) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value, sb = g / NT, b = g % NT;
      if constexpr (g + 1 < NG) {
#pragma unroll
        for (int p = 0; p < NP; ++p) bq[(g + 1) & 1][p] = bfrag(g + 1, p);
        __builtin_amdgcn_sched_group_barrier(0x100, NP, 0);
      }
      if constexpr (g < BV) {
        store_b1(g, sW);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      } else if constexpr (g == BV) {
#pragma unroll
        for (int sv = 0; sv < BV; ++sv) load_b1(sv, kb2);
        __builtin_amdgcn_sched_group_barrier(0x020, BV, 0);
      }
      if constexpr (g < NPAIR) {
        split_pair(afn, ra[nset], g);
        __builtin_amdgcn_sched_group_barrier(0x002, NP == 3 ? 11 : 2, 0);
      }
      acc[b] = mfma32_planes<NP>(af[sb], bq[g & 1], acc[b]);
      __builtin_amdgcn_sched_group_barrier(0x008, NP == 3 ? 6 : 1, 0);
    });
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int p = 0; p < NP; ++p) afc[sb][p] = afn[sb][p];
    if (s + 2 < nk) load_a(set, (int64_t)(s + 2) * BK);
    __syncthreads();
  };
  for (int s = 0; s < nk; s += 2) {
    step(s, std::integral_constant<int, 0>{});
    if (s + 1 < nk) step(s + 1, std::integral_constant<int, 1>{});
  }
  // acc[b][r] = C[row (r & 3) + 8 (r >> 2) + 4 lh][col lr] of the wave's tile b
#pragma unroll
  for (int b = 0; b < NT; ++b) {
    const int64_t gn = n0 + 32 * b + lr;
    if (gn < N) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gm = arow0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (gm < M) C[gm * ldc + gn] = acc[b][r];
      }
    }
  }
}

}  // namespace sv2n
