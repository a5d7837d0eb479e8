// bf16-operand GEMM with large workgroup tiles for the bf16 execution mode
// (BASELINE config C3: the yaml model under bf16 autocast):
//
//   C[m][n] = Σ_k A(m,k) · B(n,k)      fp32 accumulation, operands bf16
//
//   KO = false ("NT", the projection xs = x·Waugᵀ): A [M][lda], B [N][ldb],
//              both k-contiguous;
//   KO = true  ("TN", the weight gradient dWaug = dxsᵀ·x): A [K][lda],
//              B [K][ldb], both k-outer (row k of the tile is contiguous).
//   AF / BF: the operand is fp32 in HBM (rounded to bf16, RNE, while it is
//   staged) or already bf16.
//
// Why large tiles: at 128 x 128 a step's operands (fp32 A) are ~94 B per
// clock per CU at the MFMA rate, against ~35 B/clk/CU the L2 serves
// (MI355X_MICROARCH.md §Indexed rows: 66-73 GB/s per CU from L2) — the
// round-3 kernels ran at 0.12-0.19 of the bf16 peak, L2-bound.  A 256 x 192
// tile of 8 waves (2 x 4, wave tile 128 x 48 = 8 x 3 MFMA tiles) needs 36-57
// B/clk/CU, and each A fragment read from LDS feeds 3 MFMAs, each B fragment 8.
//
// Pipeline: K steps of 64 through two LDS stages; at step s the operands of
// step s+1 (loaded into registers during step s-1) are rounded and written to
// the free stage, the loads of step s+2 are issued, then step s's 2 x 24
// MFMAs per wave run; one barrier per step.  Fragments: KO = false —
// ds_read_b128 from [row][64 + 16] images (conflict-free); KO = true —
// ds_read_b64_tr_b16 from [k][rows + pad] images (the bijection of
// sv2n_gemm_tt.h, identical for A and B).  Blocks are ordered so the column
// tiles of one row tile run on one XCD; gridDim.z split-K slices write slabs
// C + z·M·ldc (summed by the caller in a fixed order).
#pragma once
#include "sv2n_gemm_tt.h"

namespace sv2n {

// WM x WN waves per workgroup (default 2 x 4); BK_ the K step per barrier
template <int BM, int BN, bool KO, bool AF, bool BF, int WM_ = 2, int WN_ = 4, int BK_ = 64>
struct GemmBWCfg {
  static constexpr int WM = WM_, WN = WN_, NW = WM * WN, THREADS = 64 * NW;
  static constexpr int BK = BK_;
  static constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // MFMA tiles per wave
  static constexpr int padko(int w) {  // k-outer rows: row dwords ≡ 8 (mod 16)
    int p = 8;
    while (((w + p) / 2) % 16 != 8) p += 8;
    return p;
  }
  // bf16 per LDS row
  static constexpr int SA = KO ? BM + padko(BM) : BK + 16;
  static constexpr int SB = KO ? BN + padko(BN) : BK + 16;
  static constexpr int IA = KO ? BK * SA : BM * SA, IB = KO ? BK * SB : BN * SB;  // image sizes
  static constexpr int STAGE = IA + IB;
  static constexpr size_t LDS = sizeof(unsigned short) * 2 * STAGE;
  // 16-B staging pieces: 4 fp32 or 8 bf16 values along the contiguous axis
  static constexpr int PA = AF ? 4 : 8, PB = BF ? 4 : 8;
  static constexpr int NA = BM * BK / PA, NB = BN * BK / PB;  // pieces per tile
  static constexpr int RA = (NA + THREADS - 1) / THREADS, RB = (NB + THREADS - 1) / THREADS;
  static_assert(BM % (16 * WM) == 0 && BN % (16 * WN) == 0, "wave tiling");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// a 16-B piece of an operand -> its bf16 values (4 from fp32, 8 from bf16)
template <bool F32>
struct Piece {
  u32x4 v;
  __device__ __forceinline__ void load(rsrc_t r, int off, int soff) {
    v = __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, 0);
  }
  __device__ __forceinline__ void put(unsigned short* p) const {
    if constexpr (F32) {
      u32x2 w;
      w[0] = bf16_pk(__uint_as_float(v[0]), __uint_as_float(v[1]));
      w[1] = bf16_pk(__uint_as_float(v[2]), __uint_as_float(v[3]));
      *reinterpret_cast<u32x2*>(p) = w;
    } else {
      *reinterpret_cast<u32x4*>(p) = v;
    }
  }
};

template <int BM, int BN, bool KO, bool AF, bool BF, int WM_ = 2, int WN_ = 4, int BK_ = 64>
__global__ __launch_bounds__(64 * WM_ * WN_) void k_gemm_bw(const void* __restrict__ Av, int64_t lda,
                                                 const void* __restrict__ Bv, int64_t ldb,
                                                 float* __restrict__ C, int64_t ldc, int64_t M,
                                                 int64_t N, int64_t K, int64_t kslice, int nm,
                                                 int nn, unsigned short* __restrict__ Aex = nullptr,
                                                 int64_t ldex = 0) {
  using Cfg = GemmBWCfg<BM, BN, KO, AF, BF, WM_, WN_, BK_>;
  constexpr int BK = Cfg::BK, TM = Cfg::TM, TN = Cfg::TN, SA = Cfg::SA, SB = Cfg::SB;
  constexpr int IA = Cfg::IA, STAGE = Cfg::STAGE, TH = Cfg::THREADS;
  constexpr int PA = Cfg::PA, PB = Cfg::PB, RA = Cfg::RA, RB = Cfg::RB;
  constexpr int EA = AF ? 4 : 2, EB = BF ? 4 : 2;  // bytes per element in HBM
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, lg = lane >> 4;
  const int wm = wave / Cfg::WN, wn = wave - wm * Cfg::WN;
  // XCD-grouped order: id = q*8*nn + nb*8 + r -> row tile q*8 + r, column tile nb
  const int id = blockIdx.x;
  const int q = id / (8 * nn), rem = id - q * 8 * nn;
  const int nb = rem >> 3, mb = q * 8 + (rem & 7);
  if (mb >= nm) return;
  const int64_t m0 = (int64_t)mb * BM, n0 = (int64_t)nb * BN;
  const int64_t kbeg = (int64_t)blockIdx.z * kslice, kend = min(K, kbeg + kslice);
  if (gridDim.z > 1) C += (int64_t)blockIdx.z * M * ldc;
  // whole-operand descriptors (offsets past them read 0)
  const int64_t abytes = (KO ? K : M) * lda * EA, bbytes = (KO ? K : N) * ldb * EB;
  const rsrc_t ra = make_rsrc(Av, (uint32_t)min<int64_t>(abytes, 0x7fffffff));
  const rsrc_t rb = make_rsrc(Bv, (uint32_t)min<int64_t>(bbytes, 0x7fffffff));

  // piece i of a tile: KO = false — row i / (BK / P), k-chunk i % (BK / P);
  // KO = true — k-row i / (R / P), column chunk i % (R / P).  Everything but
  // the K-step is fixed per thread: the k-independent byte offset (vo), the
  // row / column bound (ok), the k offset inside a step (kk) and the LDS
  // offset (lo) are computed once; a step adds its k0 through the wave-uniform
  // scalar offset (round 4: the per-step 64-bit index arithmetic made the
  // bf16 weight-gradient GEMM issue ~4,200 VALU per wave against ~890 MFMA).
  Piece<AF> pa[RA];
  Piece<BF> pb[RB];
  int a_vo[RA], a_kk[RA], a_lo[RA], a_r[RA], a_c[RA];
  bool a_ok[RA];
#pragma unroll
  for (int s = 0; s < RA; ++s) {
    const int i = min(t + TH * s, Cfg::NA - 1);
    if constexpr (!KO) {
      const int r = i / (BK / PA), c = (i - r * (BK / PA)) * PA;
      a_vo[s] = (int)(((m0 + r) * lda + c) * EA);
      a_ok[s] = m0 + r < M;
      a_kk[s] = c;
      a_r[s] = r;
      a_c[s] = c;
      a_lo[s] = r * SA + c;
    } else {
      const int r = i / (BM / PA), c = (i - r * (BM / PA)) * PA;
      a_vo[s] = (int)((r * lda + m0 + c) * EA);
      a_ok[s] = m0 + c < lda;
      a_kk[s] = r;
      a_r[s] = r;
      a_c[s] = c;
      a_lo[s] = r * SA + c;
    }
  }
  int b_vo[RB], b_kk[RB], b_lo[RB];
  bool b_ok[RB];
#pragma unroll
  for (int s = 0; s < RB; ++s) {
    const int i = min(t + TH * s, Cfg::NB - 1);
    if constexpr (!KO) {
      const int r = i / (BK / PB), c = (i - r * (BK / PB)) * PB;
      b_vo[s] = (int)(((n0 + r) * ldb + c) * EB);
      b_ok[s] = n0 + r < N;
      b_kk[s] = c;
      b_lo[s] = r * SB + c;
    } else {
      const int r = i / (BN / PB), c = (i - r * (BN / PB)) * PB;
      b_vo[s] = (int)((r * ldb + n0 + c) * EB);
      b_ok[s] = n0 + c < ldb;
      b_kk[s] = r;
      b_lo[s] = r * SB + c;
    }
  }
  auto load = [&](int64_t k0) __attribute__((always_inline)) {
    const int kr = (int)(kend - k0);  // k offsets >= kr are past the slice
    const int sa_off = (int)(KO ? k0 * lda * EA : k0 * EA);
    const int sb_off = (int)(KO ? k0 * ldb * EB : k0 * EB);
#pragma unroll
    for (int s = 0; s < RA; ++s)
      pa[s].load(ra, (a_ok[s] && a_kk[s] < kr) ? a_vo[s] : OOB, sa_off);
#pragma unroll
    for (int s = 0; s < RB; ++s)
      pb[s].load(rb, (b_ok[s] && b_kk[s] < kr) ? b_vo[s] : OOB, sb_off);
  };
  // Aex (NT, fp32 A only): the column-tile-0 workgroups also store the
  // bf16-rounded A tile to Aex [M][ldex] (columns up to the K-step end, zero
  // past K), a bf16 copy of the operand for a later bf16 GEMM
  const bool ex = !KO && AF && Aex != nullptr && nb == 0;
  // (surplus pieces repeat the last one: same value, same address)
  auto store = [&](unsigned short* st, int64_t k0) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < RA; ++s) {
      pa[s].put(st + a_lo[s]);
      if constexpr (!KO && AF) {
        if (ex && a_ok[s] && k0 + a_c[s] < ldex)
          *reinterpret_cast<u32x2*>(Aex + (m0 + a_r[s]) * ldex + k0 + a_c[s]) =
              *reinterpret_cast<const u32x2*>(st + a_lo[s]);
      }
    }
    unsigned short* sb = st + IA;
#pragma unroll
    for (int s = 0; s < RB; ++s) pb[s].put(sb + b_lo[s]);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int qq = li >> 2, p4 = 4 * (li & 3);  // transposed reads (KO)
  auto compute = [&](const unsigned short* st) __attribute__((always_inline)) {
    const unsigned short* sa = st;
    const unsigned short* sb = st + IA;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int row = wm * (BM / Cfg::WM) + 16 * a;
        if constexpr (!KO) {
          af[a] = *reinterpret_cast<const bf16x8*>(sa + (row + li) * SA + 32 * ks + 8 * lg);
        } else {
          const unsigned short* p = sa + (32 * ks + 4 * lg + qq) * SA + row + p4;
          af[a] = tr_frag(p, p + 16 * SA);
        }
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = wn * (BN / Cfg::WN) + 16 * b;
        if constexpr (!KO) {
          bf[b] = *reinterpret_cast<const bf16x8*>(sb + (col + li) * SB + 32 * ks + 8 * lg);
        } else {
          const unsigned short* p = sb + (32 * ks + 4 * lg + qq) * SB + col + p4;
          bf[b] = tr_frag(p, p + 16 * SB);
        }
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
  };

  const int nk = (int)((kend - kbeg + BK - 1) / BK);
  if (nk > 0) {
    load(kbeg);
    store(lds, kbeg);
    if (nk > 1) load(kbeg + BK);
    __syncthreads();
    for (int s = 0; s < nk; ++s) {
      if (s + 1 < nk) {
        // that stage was last read in step s - 1
        store(lds + ((s + 1) & 1) * STAGE, kbeg + (int64_t)(s + 1) * BK);
        if (s + 2 < nk) load(kbeg + (int64_t)(s + 2) * BK);
      }
      compute(lds + (s & 1) * STAGE);
      __syncthreads();
    }
  }
  // acc[a][b][r] = C[row 16a + 4lg + r][col 16b + li] of the wave tile
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int64_t gn = n0 + wn * (BN / Cfg::WN) + 16 * b + li;
      if (gn < N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t gm = m0 + wm * (BM / Cfg::WM) + 16 * a + 4 * lg + r;
          if (gm < M) C[gm * ldc + gn] = acc[a][b][r];
        }
      }
    }
}

}  // namespace sv2n
