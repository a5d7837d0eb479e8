// f32-input MFMA GEMM for the GATConv projections (PyG lin_src, SURVEY §8a
// row a6) and their backward products.
//
//   C[M][N] = Σ_k A(m,k) · B(n,k)
//   A(m,k) = A[m*lda + k]  (a_kmajor = 1)   or  A[k*lda + m]  (a_kmajor = 0)
//   B(n,k) = B[n*ldb + k]  (b_kmajor = 1)   or  B[k*ldb + n]  (b_kmajor = 0)
//
// gfx950 has exact f32 MFMA (v_mfma_f32_16x16x4_f32: one rounding per product,
// k-ordered fma chain) at the f32 vector peak (157 TF).  Tiling:
//   * workgroup = 4 waves; wave w owns rows [16*MT*w, 16*MT*(w+1)) of the
//     block tile and ALL NT 16-column tiles -> BM = 64*MT, BN = 16*NT.
//     NT = 13 (BN = 208) fits the GAT projection widths H*C+2H (408, 208,
//     3012) with <= 3 % padding; NT = 8 (BN = 128) for the rest.
//   * K-steps of 16 staged through double-buffered LDS in k-major [k][row]
//     images (row stride ≡ 16 mod 32 dwords: conflict-free ds_read_b32 of the
//     A/B fragments), one barrier per K-step, next tile prefetched to
//     registers while the MFMAs of the current one run.
//   * split-K over gridDim.z writes f32 partial slabs, summed in a fixed order
//     by k_splitk_reduce (deterministic; used for the long-K weight gradients).
#include "sv2n_common.h"

namespace sv2n {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int GB_K = 16;
constexpr int G_THREADS = 256;

__host__ __device__ constexpr int lds_stride(int rows) {
  // smallest stride >= rows with stride ≡ 16 (mod 32)
  return rows + ((16 - rows % 32) + 32) % 32;
}

template <int ROWS, bool KMAJOR>
struct TileLoader {
  // float4 slots of a ROWS x GB_K tile spread over 256 threads
  static constexpr int NV = ROWS * GB_K / 4;
  static constexpr int PER = (NV + G_THREADS - 1) / G_THREADS;
  static constexpr int STRIDE = lds_stride(ROWS);
  float4 v[PER];

  __device__ __forceinline__ void load(const float* __restrict__ base, int64_t ld, int64_t r0,
                                       int64_t rmax, int64_t k0, int64_t kmax, bool vec, int t) {
#pragma unroll
    for (int s = 0; s < PER; ++s) {
      const int idx = t + s * G_THREADS;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (idx < NV) {
        int64_t r, k;
        if constexpr (KMAJOR) {
          r = r0 + idx / (GB_K / 4);
          k = k0 + 4 * (idx % (GB_K / 4));
          if (r < rmax) {
            const float* p = base + r * ld + k;
            if (vec && k + 3 < kmax) {
              x = *reinterpret_cast<const float4*>(p);
            } else {
              if (k + 0 < kmax) x.x = p[0];
              if (k + 1 < kmax) x.y = p[1];
              if (k + 2 < kmax) x.z = p[2];
              if (k + 3 < kmax) x.w = p[3];
            }
          }
        } else {
          k = k0 + idx / (ROWS / 4);
          r = r0 + 4 * (idx % (ROWS / 4));
          if (k < kmax) {
            const float* p = base + k * ld + r;
            if (vec && r + 3 < rmax) {
              x = *reinterpret_cast<const float4*>(p);
            } else {
              if (r + 0 < rmax) x.x = p[0];
              if (r + 1 < rmax) x.y = p[1];
              if (r + 2 < rmax) x.z = p[2];
              if (r + 3 < rmax) x.w = p[3];
            }
          }
        }
      }
      v[s] = x;
    }
  }

  __device__ __forceinline__ void store(float* __restrict__ lds, int t) const {
#pragma unroll
    for (int s = 0; s < PER; ++s) {
      const int idx = t + s * G_THREADS;
      if (idx < NV) {
        if constexpr (KMAJOR) {
          const int r = idx / (GB_K / 4), k = 4 * (idx % (GB_K / 4));
          lds[(k + 0) * STRIDE + r] = v[s].x;
          lds[(k + 1) * STRIDE + r] = v[s].y;
          lds[(k + 2) * STRIDE + r] = v[s].z;
          lds[(k + 3) * STRIDE + r] = v[s].w;
        } else {
          const int k = idx / (ROWS / 4), r = 4 * (idx % (ROWS / 4));
          *reinterpret_cast<float4*>(lds + k * STRIDE + r) = v[s];
        }
      }
    }
  }
};

template <int MT, int NT, bool AK, bool BK>
__global__ __launch_bounds__(G_THREADS) void k_gemm_f32(
    const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
    float* __restrict__ C, int64_t ldc, int64_t M, int64_t N, int64_t K, int64_t kslice,
    bool avec, bool bvec, float* __restrict__ part) {
  constexpr int BM = 64 * MT, BN = 16 * NT;
  using LA = TileLoader<BM, AK>;
  using LB = TileLoader<BN, BK>;
  constexpr int SA = LA::STRIDE, SB = LB::STRIDE;
  constexpr int BUF = GB_K * (SA + SB);
  __shared__ __attribute__((aligned(16))) float lds[2 * BUF];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
  const int64_t kb = (int64_t)blockIdx.z * kslice;
  const int64_t ke = min(K, kb + kslice);
  const int nk = (int)((ke - kb + GB_K - 1) / GB_K);

  floatx4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  LA la;
  LB lb;
  if (nk > 0) {
    la.load(A, lda, m0, M, kb, ke, avec, t);
    lb.load(B, ldb, n0, N, kb, ke, bvec, t);
    la.store(lds, t);
    lb.store(lds + GB_K * SA, t);
  }
  __syncthreads();

  const int li = lane & 15, lk = lane >> 4;
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      const int64_t k0 = kb + (int64_t)(kt + 1) * GB_K;
      la.load(A, lda, m0, M, k0, ke, avec, t);
      lb.load(B, ldb, n0, N, k0, ke, bvec, t);
    }
    const float* sa = lds + cur * BUF;
    const float* sb = sa + GB_K * SA;
#pragma unroll
    for (int ks = 0; ks < GB_K / 4; ++ks) {
      const int k = 4 * ks + lk;
      float af[MT];
#pragma unroll
      for (int a = 0; a < MT; ++a) af[a] = sa[k * SA + wave * 16 * MT + 16 * a + li];
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const float bf = sb[k * SB + 16 * b + li];
#pragma unroll
        for (int a = 0; a < MT; ++a)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a], bf, acc[a][b], 0, 0, 0);
      }
    }
    if (more) {
      float* nxt = lds + (cur ^ 1) * BUF;
      la.store(nxt, t);
      lb.store(nxt + GB_K * SA, t);
    }
    __syncthreads();
    cur ^= 1;
  }

  // epilogue: C/D map of 16x16 f32 MFMA: col = lane&15, row = 4*(lane>>4) + reg
  float* out = part ? part + (int64_t)blockIdx.z * M * N : C;
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

struct GemmPlan {
  int mt, nt, splitk;
  int64_t kslice;
};

static GemmPlan plan_gemm(int64_t M, int64_t N, int64_t K) {
  GemmPlan p{};
  const int64_t pad128 = (N + 127) / 128 * 128, pad208 = (N + 207) / 208 * 208;
  p.nt = (pad208 < pad128) ? 13 : 8;
  const int64_t bn = 16 * p.nt;
  const int64_t ntn = (N + bn - 1) / bn;
  p.mt = ((M + 127) / 128) * ntn >= 512 ? 2 : 1;
  const int64_t bm = 64 * p.mt;
  const int64_t tiles = ((M + bm - 1) / bm) * ntn;
  int64_t sk = 1;
  if (tiles < 384 && K >= 512) {
    sk = std::min<int64_t>(32, std::max<int64_t>(1, 768 / tiles));
    sk = std::min<int64_t>(sk, std::max<int64_t>(1, K / 256));
  }
  int64_t ks = (K + sk - 1) / sk;
  ks = (ks + GB_K - 1) / GB_K * GB_K;
  p.splitk = (int)((K + ks - 1) / ks);
  p.kslice = ks;
  return p;
}

}  // namespace sv2n

using namespace sv2n;

extern "C" int64_t sv2n_gemm_f32_workspace(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const GemmPlan p = plan_gemm(M, N, K);
  return p.splitk > 1 ? (int64_t)p.splitk * M * N : 0;
}

template <int MT, int NT, bool AK, bool BK>
static void launch_gemm(dim3 grid, hipStream_t st, const float* A, int64_t lda, const float* B,
                        int64_t ldb, float* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                        int64_t ks, bool avec, bool bvec, float* part) {
  hipLaunchKernelGGL((k_gemm_f32<MT, NT, AK, BK>), grid, dim3(G_THREADS), 0, st, A, lda, B, ldb, C,
                     ldc, M, N, K, ks, avec, bvec, part);
}

#define SV2N_GEMM_LAYOUT(MT, NT)                                                                  \
  if (a_kmajor && b_kmajor)                                                                       \
    launch_gemm<MT, NT, true, true>(grid, stream, A, lda, B, ldb, C, ldc, M, N, K, p.kslice, avec, \
                                    bvec, part);                                                  \
  else if (a_kmajor)                                                                              \
    launch_gemm<MT, NT, true, false>(grid, stream, A, lda, B, ldb, C, ldc, M, N, K, p.kslice,      \
                                     avec, bvec, part);                                           \
  else if (b_kmajor)                                                                              \
    launch_gemm<MT, NT, false, true>(grid, stream, A, lda, B, ldb, C, ldc, M, N, K, p.kslice,      \
                                     avec, bvec, part);                                           \
  else                                                                                            \
    launch_gemm<MT, NT, false, false>(grid, stream, A, lda, B, ldb, C, ldc, M, N, K, p.kslice,     \
                                      avec, bvec, part);

extern "C" int sv2n_gemm_f32(int a_kmajor, int b_kmajor, const float* A, int64_t lda,
                             const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M,
                             int64_t N, int64_t K, float* workspace, int64_t workspace_floats,
                             hipStream_t stream) {
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0) return SV2N_ERR_ARG;
  if (ldc < N || lda < (a_kmajor ? K : M) || ldb < (b_kmajor ? K : N)) return SV2N_ERR_SHAPE;
  const GemmPlan p = plan_gemm(M, N, K);
  float* part = nullptr;
  if (p.splitk > 1) {
    if (!workspace || workspace_floats < (int64_t)p.splitk * M * N) return SV2N_ERR_WORKSPACE;
    part = workspace;
  }
  const bool avec = ((uintptr_t)A % 16 == 0) && (lda % 4 == 0);
  const bool bvec = ((uintptr_t)B % 16 == 0) && (ldb % 4 == 0);
  const int64_t bm = 64 * p.mt, bn = 16 * p.nt;
  dim3 grid((unsigned)((M + bm - 1) / bm), (unsigned)((N + bn - 1) / bn), (unsigned)p.splitk);
  if (p.mt == 2 && p.nt == 13) {
    SV2N_GEMM_LAYOUT(2, 13)
  } else if (p.mt == 2) {
    SV2N_GEMM_LAYOUT(2, 8)
  } else if (p.nt == 13) {
    SV2N_GEMM_LAYOUT(1, 13)
  } else {
    SV2N_GEMM_LAYOUT(1, 8)
  }
  if (part) {
    const int64_t tot = M * N;
    hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream,
                       part, p.splitk, M, N, C, ldc);
  }
  return (int)hipGetLastError();
}
