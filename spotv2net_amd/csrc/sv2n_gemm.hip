// f32-input MFMA GEMM for the GATConv projections (PyG lin_src, SURVEY §8a
// row a6) and their backward products.
//
//   C[M][N] = Σ_k A(m,k) · B(n,k)
//   A(m,k) = A[m*lda + k]  (a_kmajor = 1)   or  A[k*lda + m]  (a_kmajor = 0)
//   B(n,k) = B[n*ldb + k]  (b_kmajor = 1)   or  B[k*ldb + n]  (b_kmajor = 0)
//
// gfx950 has exact f32 MFMA (v_mfma_f32_16x16x4_f32: one rounding per product,
// k-ordered fma chain) at the f32 vector peak (157 TF).  Tiling:
//   kernel template: sv2n_gemm_kernel.h.  Configuration chosen with
//   tools/gemm_tune.hip on MI355X over the five C2 projection shapes
//   (profiles/gemm_tune_r01.txt): 8 waves x 16 rows (BM = 128), BN = 208
//   (NT = 13) for widths > 256 else 128, K-step 16, two register prefetch
//   sets, split-K up to 32 slices aiming at ~480 workgroups for the long-K
//   weight gradients (deterministic slab reduce).  103 TF/s on the layer-0
//   projection (M 15360, N 408, K 1260) vs 76 TF/s for hipBLASLt fp32 on the
//   same box (tools/gemm_ref_blas.py).
#include "sv2n_common.h"
#include "sv2n_gemm_kernel.h"

namespace sv2n {

struct GemmPlan {
  int nt, pf, splitk;
  int64_t kslice;
};

static GemmPlan plan_gemm(int64_t M, int64_t N, int64_t K) {
  constexpr int BM = 128;
  GemmPlan p{};
  const int64_t pad128 = (N + 127) / 128 * 128, pad208 = (N + 207) / 208 * 208;
  p.nt = (N > 256 && pad208 <= pad128) ? 13 : 8;
  const int64_t bn = 16 * p.nt;
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + bn - 1) / bn);
  int64_t sk = 1;
  if (tiles < 240 && K >= 2048) {
    sk = std::min<int64_t>(32, (480 + tiles - 1) / tiles);
    sk = std::min<int64_t>(sk, std::max<int64_t>(1, K / 256));
  }
  int64_t ks = (K + sk - 1) / sk;
  ks = (ks + 15) / 16 * 16;
  p.splitk = (int)((K + ks - 1) / ks);
  p.kslice = ks;
  p.pf = 2;
  return p;
}

}  // namespace sv2n

using namespace sv2n;

extern "C" int64_t sv2n_gemm_f32_workspace(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const GemmPlan p = plan_gemm(M, N, K);
  return p.splitk > 1 ? (int64_t)p.splitk * M * N : 0;
}

template <int NT, int PF>
static void dispatch_layout(int a_kmajor, int b_kmajor, const GemmPlan& p, hipStream_t st,
                            const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                            int64_t ldc, int64_t M, int64_t N, int64_t K, bool avec, bool bvec,
                            float* part) {
  if (a_kmajor && b_kmajor)
    launch_gemm_cfg<8, 1, NT, 16, true, true, PF>(p.splitk, p.kslice, st, A, lda, B, ldb, C, ldc,
                                                  M, N, K, avec, bvec, part);
  else if (a_kmajor)
    launch_gemm_cfg<8, 1, NT, 16, true, false, PF>(p.splitk, p.kslice, st, A, lda, B, ldb, C, ldc,
                                                   M, N, K, avec, bvec, part);
  else if (b_kmajor)
    launch_gemm_cfg<8, 1, NT, 16, false, true, PF>(p.splitk, p.kslice, st, A, lda, B, ldb, C, ldc,
                                                   M, N, K, avec, bvec, part);
  else
    launch_gemm_cfg<8, 1, NT, 16, false, false, PF>(p.splitk, p.kslice, st, A, lda, B, ldb, C,
                                                    ldc, M, N, K, avec, bvec, part);
}

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
  if (p.nt == 13) {
    if (p.pf == 2)
      dispatch_layout<13, 2>(a_kmajor, b_kmajor, p, stream, A, lda, B, ldb, C, ldc, M, N, K, avec,
                             bvec, part);
    else
      dispatch_layout<13, 1>(a_kmajor, b_kmajor, p, stream, A, lda, B, ldb, C, ldc, M, N, K, avec,
                             bvec, part);
  } else {
    if (p.pf == 2)
      dispatch_layout<8, 2>(a_kmajor, b_kmajor, p, stream, A, lda, B, ldb, C, ldc, M, N, K, avec,
                            bvec, part);
    else
      dispatch_layout<8, 1>(a_kmajor, b_kmajor, p, stream, A, lda, B, ldb, C, ldc, M, N, K, avec,
                            bvec, part);
  }
  return (int)hipGetLastError();
}
