// f32-MFMA GEMM kernel template shared by the library (sv2n_gemm.hip) and the
// standalone tuner (tools/gemm_tune.hip).
//
//   C[M][N] = Σ_k A(m,k) · B(n,k)
//   A(m,k) = A[m*lda + k] (AK) or A[k*lda + m];  B(n,k) = B[n*ldb + k] (BK) or B[k*ldb + n]
//
// v_mfma_f32_16x16x4_f32 (exact f32, 157 TF chip peak): lane l supplies
// A[l&15][k = l>>4] and B[k = l>>4][l&15]; C/D: col = l&15, row = 4*(l>>4)+reg.
// Workgroup = NW waves; wave w owns rows [16*MT*w, 16*MT*(w+1)) of the block
// tile and all NT 16-column tiles (BM = 16*MT*NW, BN = 16*NT).  K-steps of KB
// are staged through two LDS buffers in k-major [k][row] images (row stride
// ≡ 16 mod 32 dwords => conflict-free ds_read_b32 fragments); PF register
// sets prefetch the next PF tiles from global memory while the MFMAs of the
// current one run; one barrier per K-step.  gridDim.z = split-K slices, whose
// partial slabs are summed in fixed order by k_splitk_reduce.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sv2n {

typedef float floatx4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int gemm_lds_stride(int rows) {
  return rows + ((16 - rows % 32) + 32) % 32;  // [k][row] image: stride ≡ 16 (mod 32)
}
__host__ __device__ constexpr int gemm_kmajor_stride(int kb) {
  return kb == 16 ? 24 : 40;  // [row][k] image: conflict-free ds_read_b128 fragments
}

// One operand tile (ROWS x KB) of the block.  k-major operands (global [row][k])
// are kept as a [row][k] LDS image (16-B copies, no transpose); the others
// (global [k][row]) as a [k][row] image.  frag() returns, for lane (li, lk),
// X(row rb+li, k = 16*kc + 4*lk + c), c = 0..3 — the k-permuted order in which
// MFMA step c of lane group lk consumes k (A and B agree, so the sum is exact).
template <int ROWS, int KB, bool KMAJOR, int THREADS>
struct GemmTile {
  static constexpr int NV = ROWS * KB / 4;  // float4 slots per tile
  static constexpr int PER = (NV + THREADS - 1) / THREADS;
  static constexpr int STRIDE = KMAJOR ? gemm_kmajor_stride(KB) : gemm_lds_stride(ROWS);
  static constexpr int FLOATS = KMAJOR ? ROWS * STRIDE : KB * STRIDE;
  float4 v[PER];

  // VEC (host-checked: 16-B aligned base, ld % 4 == 0 and the 4-wide extent —
  // k for k-major, rows otherwise — a multiple of 4): branch-free 16-B loads
  // from clamped in-bounds addresses (also for the surplus slots of the last
  // pass, idx >= NV), with the out-of-matrix float4s (wholly outside, the
  // extent being a multiple of 4) zeroed at STORE time so no wait is forced
  // between the load and the MFMAs that run before the store.  Otherwise a
  // guarded scalar path.
  uint32_t okm;

  template <bool VEC>
  __device__ __forceinline__ void load(const float* __restrict__ base, int64_t ld, int64_t r0,
                                       int64_t rmax, int64_t k0, int64_t kmax, int t) {
    okm = 0u;
#pragma unroll
    for (int s = 0; s < PER; ++s) {
      const int idx0 = t + s * THREADS;
      const int idx = (NV % THREADS == 0) ? idx0 : min(idx0, NV - 1);
      int64_t r, k;
      if constexpr (KMAJOR) {
        r = r0 + idx / (KB / 4);
        k = k0 + 4 * (idx % (KB / 4));
      } else {
        k = k0 + idx / (ROWS / 4);
        r = r0 + 4 * (idx % (ROWS / 4));
      }
      if constexpr (VEC) {
        const bool ok = r < rmax && k < kmax;
        const int64_t rc = KMAJOR ? min(r, rmax - 1) : min(r, rmax - 4);
        const int64_t kc = KMAJOR ? min(k, kmax - 4) : min(k, kmax - 1);
        const float* p = KMAJOR ? base + rc * ld + kc : base + kc * ld + rc;
        v[s] = *reinterpret_cast<const float4*>(p);
        okm |= (ok ? 1u : 0u) << s;
      } else {
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (KMAJOR) {
          if (r < rmax) {
            const float* p = base + r * ld + k;
            if (k + 0 < kmax) x.x = p[0];
            if (k + 1 < kmax) x.y = p[1];
            if (k + 2 < kmax) x.z = p[2];
            if (k + 3 < kmax) x.w = p[3];
          }
        } else {
          if (k < kmax) {
            const float* p = base + k * ld + r;
            if (r + 0 < rmax) x.x = p[0];
            if (r + 1 < rmax) x.y = p[1];
            if (r + 2 < rmax) x.z = p[2];
            if (r + 3 < rmax) x.w = p[3];
          }
        }
        v[s] = x;
        okm |= 1u << s;
      }
    }
  }

  __device__ __forceinline__ void store(float* __restrict__ lds, int t) const {
#pragma unroll
    for (int s = 0; s < PER; ++s) {
      const int idx = t + s * THREADS;
      if (NV % THREADS == 0 || idx < NV) {
        const bool ok = (okm >> s) & 1u;
        float4 x;
        x.x = ok ? v[s].x : 0.f;
        x.y = ok ? v[s].y : 0.f;
        x.z = ok ? v[s].z : 0.f;
        x.w = ok ? v[s].w : 0.f;
        if constexpr (KMAJOR) {
          const int r = idx / (KB / 4), k = 4 * (idx % (KB / 4));
          *reinterpret_cast<float4*>(lds + r * STRIDE + k) = x;
        } else {
          const int k = idx / (ROWS / 4), r = 4 * (idx % (ROWS / 4));
          *reinterpret_cast<float4*>(lds + k * STRIDE + r) = x;
        }
      }
    }
  }

  __device__ __forceinline__ static floatx4 frag(const float* __restrict__ lds, int rb, int kc,
                                                 int li, int lk) {
    if constexpr (KMAJOR) {
      return *reinterpret_cast<const floatx4*>(lds + (rb + li) * STRIDE + 16 * kc + 4 * lk);
    } else {
      const float* p = lds + (16 * kc + 4 * lk) * STRIDE + rb + li;
      return floatx4{p[0], p[STRIDE], p[2 * STRIDE], p[3 * STRIDE]};
    }
  }
};

template <int NW, int MT, int NT, int KB, bool AK, bool BK, int PF>
struct GemmCfg {
  static constexpr int THREADS = 64 * NW;
  static constexpr int BM = 16 * MT * NW, BN = 16 * NT;
  using TA = GemmTile<BM, KB, AK, THREADS>;
  using TB = GemmTile<BN, KB, BK, THREADS>;
  static constexpr int AOFF = TA::FLOATS;  // B image follows A's in each buffer
  static constexpr int BUF = TA::FLOATS + TB::FLOATS;
  static constexpr int LDS_BYTES = 2 * BUF * 4;
};

// XR (XCD-grouped K slices, split-K only): workgroups are dealt round-robin
// over the 8 XCDs, so with the plain (x, y, z) order the output tiles of one K
// slice — which all read that slice's A and B panels — land on all eight L2s
// and every panel is fetched up to 8 times.  With XR the linear block id
// b = xcd + 8*slot is mapped to K slice z = xcd + 8*(slot / tiles) and tile
// slot % tiles: every tile of a slice runs on ONE XCD and the panels are read
// into its L2 once.  The grid's z extent is the slice count rounded up to 8;
// blocks with z >= nz exit at once.
template <int NW, int MT, int NT, int KB, bool AK, bool BK, int PF, int ABL = 0, bool AV = true,
          bool BV = true, bool XR = false>
__global__ __launch_bounds__(64 * NW) void k_gemm_f32(
    const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
    float* __restrict__ C, int64_t ldc, int64_t M, int64_t N, int64_t K, int64_t kslice,
    float* __restrict__ part, int nz = 0) {
  using Cfg = GemmCfg<NW, MT, NT, KB, AK, BK, PF>;
  using TA = typename Cfg::TA;
  using TB = typename Cfg::TB;
  constexpr int AOFF = Cfg::AOFF, BUF = Cfg::BUF;
  __shared__ __attribute__((aligned(16))) float lds[2 * BUF];

  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if constexpr (XR) {
    const int tiles = gridDim.x * gridDim.y;
    const int id = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = id & 7, slot = id >> 3;
    bz = xcd + 8 * (slot / tiles);
    const int tile = slot - (slot / tiles) * tiles;
    by = tile / gridDim.x;
    bx = tile - by * gridDim.x;
    if (bz >= nz) return;
  }
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int64_t m0 = (int64_t)bx * Cfg::BM, n0 = (int64_t)by * Cfg::BN;
  const int64_t kb = (int64_t)bz * kslice;
  const int64_t ke = min(K, kb + kslice);
  const int nk = (int)((ke - kb + KB - 1) / KB);

  floatx4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int li = lane & 15, lk = lane >> 4;
  auto compute = [&](const float* sa, const float* sb) {
#pragma unroll
    for (int kc = 0; kc < KB / 16; ++kc) {
      floatx4 af[MT], bf[NT];
#pragma unroll
      for (int a = 0; a < MT; ++a) af[a] = TA::frag(sa, wave * 16 * MT + 16 * a, kc, li, lk);
#pragma unroll
      for (int b = 0; b < NT; ++b) bf[b] = TB::frag(sb, 16 * b, kc, li, lk);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int b = 0; b < NT; ++b)
#pragma unroll
          for (int a = 0; a < MT; ++a)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a][c], bf[b][c], acc[a][b], 0, 0, 0);
    }
  };

  TA ra0, ra1;
  TB rb0, rb1;
  if (nk > 0) {
    ra0.template load<AV>(A, lda, m0, M, kb, ke, t);
    rb0.template load<BV>(B, ldb, n0, N, kb, ke, t);
    ra0.store(lds, t);
    rb0.store(lds + AOFF, t);
    if (PF == 2 && nk > 1) {
      ra1.template load<AV>(A, lda, m0, M, kb + KB, ke, t);
      rb1.template load<BV>(B, ldb, n0, N, kb + KB, ke, t);
    }
  }
  __syncthreads();

  if constexpr (PF == 1) {
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more && !(ABL & 1)) {
        const int64_t k0 = kb + (int64_t)(kt + 1) * KB;
        ra0.template load<AV>(A, lda, m0, M, k0, ke, t);
        rb0.template load<BV>(B, ldb, n0, N, k0, ke, t);
      }
      const float* sa = lds + cur * BUF;
      compute(sa, sa + AOFF);
      if (more && !(ABL & 2)) {
        float* nxt = lds + (cur ^ 1) * BUF;
        ra0.store(nxt, t);
        rb0.store(nxt + AOFF, t);
      }
      if (ABL & 2) {
#pragma unroll
        for (int q = 0; q < TA::PER; ++q) asm volatile("" ::"v"(ra0.v[q].x), "v"(ra0.v[q].w));
#pragma unroll
        for (int q = 0; q < TB::PER; ++q) asm volatile("" ::"v"(rb0.v[q].x), "v"(rb0.v[q].w));
      }
      __syncthreads();
      cur ^= 1;
    }
  } else {
    // two register sets: tile kt+1 is already in (ra1, rb1) when step kt starts
    for (int kt = 0; kt < nk; kt += 2) {
      {  // even step: compute buf 0, refill set 0 with tile kt+2, store set 1 -> buf 1
        if (kt + 2 < nk) {
          const int64_t k0 = kb + (int64_t)(kt + 2) * KB;
          ra0.template load<AV>(A, lda, m0, M, k0, ke, t);
          rb0.template load<BV>(B, ldb, n0, N, k0, ke, t);
        }
        compute(lds, lds + AOFF);
        if (kt + 1 < nk) {
          ra1.store(lds + BUF, t);
          rb1.store(lds + BUF + AOFF, t);
        }
        __syncthreads();
      }
      if (kt + 1 < nk) {  // odd step: compute buf 1, refill set 1 with tile kt+3, store set 0 -> buf 0
        if (kt + 3 < nk) {
          const int64_t k0 = kb + (int64_t)(kt + 3) * KB;
          ra1.template load<AV>(A, lda, m0, M, k0, ke, t);
          rb1.template load<BV>(B, ldb, n0, N, k0, ke, t);
        }
        compute(lds + BUF, lds + BUF + AOFF);
        if (kt + 2 < nk) {
          ra0.store(lds, t);
          rb0.store(lds + AOFF, t);
        }
        __syncthreads();
      }
    }
  }

  float* out = part ? part + (int64_t)bz * M * N : C;
  const int64_t ldo = part ? N : ldc;
#pragma unroll
  for (int a = 0; a < MT; ++a) {
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int64_t col = n0 + 16 * b + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wave * 16 * MT + 16 * a + 4 * lk + r;
        if (row < M && col < N) out[row * ldo + col] = acc[a][b][r];
      }
    }
  }
}

__global__ void k_splitk_reduce(const float* __restrict__ part, int nsplit, int64_t M, int64_t N,
                                float* __restrict__ C, int64_t ldc) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  const int64_t MN = M * N;
  float s0 = 0.f, s1 = 0.f;
  int z = 0;
  for (; z + 1 < nsplit; z += 2) {
    s0 += part[(int64_t)z * MN + idx];
    s1 += part[(int64_t)(z + 1) * MN + idx];
  }
  if (z < nsplit) s0 += part[(int64_t)z * MN + idx];
  const int64_t m = idx / N, n = idx - m * N;
  C[m * ldc + n] = s0 + s1;
}

// as k_splitk_reduce, 4 consecutive outputs per thread (16-B loads, 8 slabs
// in flight), for N % 4 == 0, ldc % 4 == 0 and 16-B aligned part / C; the
// same fixed summation order (two interleaved partial sums, as above)
__global__ __launch_bounds__(256) void k_splitk_reduce4(const float* __restrict__ part, int nsplit,
                                                        int64_t M, int64_t N,
                                                        float* __restrict__ C, int64_t ldc) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t MN = M * N;
  if (4 * q >= MN) return;
  const f32x4* p4 = reinterpret_cast<const f32x4*>(part) + q;
  const int64_t s4 = MN >> 2;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
  int z = 0;
  for (; z + 8 <= nsplit; z += 8) {
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p4 + (int64_t)(z + u) * s4);
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      s0 += v[u];
      s1 += v[u + 1];
    }
  }
  for (; z + 1 < nsplit; z += 2) {
    s0 += p4[(int64_t)z * s4];
    s1 += p4[(int64_t)(z + 1) * s4];
  }
  if (z < nsplit) s0 += p4[(int64_t)z * s4];
  const int64_t e = 4 * q, m = e / N, n = e - m * N;
  *reinterpret_cast<f32x4*>(C + m * ldc + n) = s0 + s1;
}

inline void splitk_reduce(hipStream_t st, const float* part, int nsplit, int64_t M, int64_t N,
                          float* C, int64_t ldc) {
  const int64_t tot = M * N;
  if (N % 4 == 0 && ldc % 4 == 0 && ((uintptr_t)part & 15) == 0 && ((uintptr_t)C & 15) == 0) {
    hipLaunchKernelGGL(k_splitk_reduce4, dim3((unsigned)((tot / 4 + 255) / 256)), dim3(256), 0, st,
                       part, nsplit, M, N, C, ldc);
  } else {
    hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st,
                       part, nsplit, M, N, C, ldc);
  }
}

template <int NW, int MT, int NT, int KB, bool AK, bool BK, int PF, int ABL = 0>
inline void launch_gemm_cfg(int splitk, int64_t kslice, hipStream_t st, const float* A,
                            int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                            int64_t M, int64_t N, int64_t K, bool avec, bool bvec, float* part) {
  using Cfg = GemmCfg<NW, MT, NT, KB, AK, BK, PF>;
  dim3 grid((unsigned)((M + Cfg::BM - 1) / Cfg::BM), (unsigned)((N + Cfg::BN - 1) / Cfg::BN),
            (unsigned)splitk);
  // the vector path needs the 4-wide extent (k for k-major operands, rows
  // otherwise) to be a multiple of 4 as well
  const bool av = avec && ((AK ? K : M) % 4 == 0);
  const bool bv = bvec && ((BK ? K : N) % 4 == 0);
  float* pp = splitk > 1 ? part : nullptr;
  if (av && bv)
    hipLaunchKernelGGL((k_gemm_f32<NW, MT, NT, KB, AK, BK, PF, ABL, true, true>), grid,
                       dim3(Cfg::THREADS), 0, st, A, lda, B, ldb, C, ldc, M, N, K, kslice, pp);
  else
    hipLaunchKernelGGL((k_gemm_f32<NW, MT, NT, KB, AK, BK, PF, ABL, false, false>), grid,
                       dim3(Cfg::THREADS), 0, st, A, lda, B, ldb, C, ldc, M, N, K, kslice, pp);
  if (splitk > 1) splitk_reduce(st, part, splitk, M, N, C, ldc);
}

// As launch_gemm_cfg, but the K slices stay as slabs part[z][M][N] for a
// consumer that reduces them itself (splitk == 1 writes slab 0).
template <int NW, int MT, int NT, int KB, bool AK, bool BK, int PF, int ABL = 0, bool XR = false>
inline void launch_gemm_slabs(int splitk, int64_t kslice, hipStream_t st, const float* A,
                              int64_t lda, const float* B, int64_t ldb, int64_t M, int64_t N,
                              int64_t K, bool avec, bool bvec, float* part) {
  using Cfg = GemmCfg<NW, MT, NT, KB, AK, BK, PF>;
  const bool xr = XR && splitk > 1;
  dim3 grid((unsigned)((M + Cfg::BM - 1) / Cfg::BM), (unsigned)((N + Cfg::BN - 1) / Cfg::BN),
            (unsigned)(xr ? (splitk + 7) / 8 * 8 : splitk));
  const bool av = avec && ((AK ? K : M) % 4 == 0);
  const bool bv = bvec && ((BK ? K : N) % 4 == 0);
  float* pp = splitk > 1 ? part : nullptr;
  if (av && bv) {
    if (xr)
      hipLaunchKernelGGL((k_gemm_f32<NW, MT, NT, KB, AK, BK, PF, ABL, true, true, true>), grid,
                         dim3(Cfg::THREADS), 0, st, A, lda, B, ldb, part, N, M, N, K, kslice, pp,
                         splitk);
    else
      hipLaunchKernelGGL((k_gemm_f32<NW, MT, NT, KB, AK, BK, PF, ABL, true, true>), grid,
                         dim3(Cfg::THREADS), 0, st, A, lda, B, ldb, part, N, M, N, K, kslice, pp,
                         splitk);
  } else {
    hipLaunchKernelGGL((k_gemm_f32<NW, MT, NT, KB, AK, BK, PF, ABL, false, false>), grid,
                       dim3(Cfg::THREADS), 0, st, A, lda, B, ldb, part, N, M, N, K, kslice, pp,
                       splitk);
  }
}

}  // namespace sv2n
