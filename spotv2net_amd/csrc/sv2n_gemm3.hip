// f32-accurate projection GEMMs on bf16 MFMA (kernel and numerics:
// sv2n_gemm3_kernel.h).  Used for the GATConv projection xs = x·Waugᵀ
// (PyG lin_src) and its input gradient dx = dxs·Waug,
// where the weight operand is small and is split into its three bf16 planes
// once per call (sv2n_split3).  Configurations from tools/gemm3_tune.hip on
// MI355X (profiles/gemm3_tune_r01.txt).
#include "sv2n_common.h"
#include "sv2n_gemm3_kernel.h"
#include "sv2n_gemm_bf16.h"
#include "sv2n_gemm_bw.h"

#include <algorithm>

namespace sv2n {

constexpr int64_t SPLIT3_KALIGN = 64;  // largest BK

// fp32 [K][rows] (row stride ld) -> 3 bf16 planes [3][rows][Kp] (transposed)
__global__ void k_split3_t(const float* __restrict__ x, int64_t rows, int64_t K, int64_t ld,
                           unsigned short* __restrict__ out, int64_t Kp) {
  // 32 x 32 tile transpose through LDS: coalesced reads along rows of x,
  // coalesced writes along k of the planes
  __shared__ float tile[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  const int64_t k0 = (int64_t)blockIdx.x * 32, n0 = (int64_t)blockIdx.y * 32;
  for (int j = ty; j < 32; j += 8) {
    const int64_t k = k0 + j, n = n0 + tx;
    tile[j][tx] = (k < K && n < rows) ? x[k * ld + n] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int64_t n = n0 + j, k = k0 + tx;
    if (n < rows && k < Kp) {
      unsigned short h0, h1, h2;
      split3(tile[tx][j], h0, h1, h2);
      const int64_t o = n * Kp + k;
      out[o] = h0;
      out[rows * Kp + o] = h1;
      out[2 * rows * Kp + o] = h2;
    }
  }
}

template <int NW, int MT, int NT, int BK, int PIPE>
static int launch_gemm3_p(hipStream_t st, const float* A, int64_t lda, const unsigned short* Bp,
                          int64_t Kp, int64_t N, float* C, int64_t ldc, int64_t M, int64_t K) {
  using Cfg = Gemm3Cfg<NW, MT, NT, BK>;
  constexpr size_t lds = Cfg::LDS;
  static_assert(lds <= 160 * 1024, "LDS budget");
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)k_gemm3<NW, MT, NT, BK, 1, 3, PIPE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const dim3 grid((unsigned)((M + Cfg::BM - 1) / Cfg::BM), (unsigned)((N + Cfg::BN - 1) / Cfg::BN));
  hipLaunchKernelGGL((k_gemm3<NW, MT, NT, BK, 1, 3, PIPE>), grid, dim3(Cfg::THREADS), lds, st, A,
                     lda, Bp, Kp, N * Kp, C, ldc, M, N, K);
  return (int)hipGetLastError();
}

// the LDS-staged kernel: shapes k_gemm3d does not take (K % 4 != 0)
template <int NW, int MT, int NT, int BK>
static int launch_gemm3(hipStream_t st, const float* A, int64_t lda, const unsigned short* Bp,
                        int64_t Kp, int64_t N, float* C, int64_t ldc, int64_t M, int64_t K) {
  return launch_gemm3_p<NW, MT, NT, BK, 1>(st, A, lda, Bp, Kp, N, C, ldc, M, K);
}

// k_gemm3d: A straight to registers, B planes double-buffered, the next
// step's split and B staging spread under the current step's MFMAs,
// XCD-grouped block order (MI355X, tools/gemm3_tune.hip, LDS-staged k_gemm3
// -> k_gemm3d: C2 L0 fwd 15360 x 408 x 1260 104.3 -> 89.8 us, L1 fwd x 208 x
// 400 25.9 -> 22.1, L1 dX x 400 x 208 27.0 -> 22.6, C5 L0 fwd 262144 x 144 x
// 1024 596 -> 567).  Needs K % 4 == 0 (whole 16-B A chunks per row).
template <int NW, int MT, int NT, int AP, bool MASK = false>
static int launch_gemm3d(hipStream_t st, const float* A, int64_t lda, const unsigned short* Bp,
                         int64_t Kp, int64_t N, float* C, int64_t ldc, int64_t M, int64_t K,
                         const float* Y = nullptr, int64_t ldy = 0) {
  using Cfg = Gemm3bCfg<NW, MT, NT, 32>;
  constexpr size_t lds = Cfg::LDS;
  static_assert(lds <= 160 * 1024, "LDS budget");
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_gemm3d<NW, MT, NT, AP, MASK>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    return true;
  }();
  (void)attr;
  const int nm = (int)((M + Cfg::BM - 1) / Cfg::BM), nn = (int)((N + Cfg::BN - 1) / Cfg::BN);
  const unsigned grid = (unsigned)(((nm + 7) / 8) * 8 * nn);
  hipLaunchKernelGGL((k_gemm3d<NW, MT, NT, AP, MASK>), dim3(grid), dim3(Cfg::THREADS), lds, st, A, lda,
                     Bp, Kp, N * Kp, C, ldc, M, N, K, nm, nn, Y, ldy);
  return (int)hipGetLastError();
}

// Round 6: 12-wave workgroups of 192 rows x 144 columns (k_gemm3d<12, 1, 9>:
// three waves per SIMD instead of two, 122 VGPRs) where they fill the chip in
// one round and pad N by at most 10 % (MI355X, tools/gemm3_tune.hip,
// profiles/r06_gemm3_waves.txt: C2 L0 fwd 15360 x 408 x 1260 89.0-90.7 ->
// 85.8-86.3 us, C2 L1 dX x 400 x 208 23.8 -> 23.1-23.3, C5 L0 fwd 262144 x 144
// x 1024 549-559 (8 waves) -> 501-505 us)
static bool twelve_waves(int64_t M, int64_t N) {
  const int64_t nb = (N + 143) / 144;
  return ((M + 191) / 192) * nb >= 240 && nb * 144 * 10 <= 11 * N;
}

// bf16 operands (one plane), fp32 accumulation: the bf16 execution mode
template <int NW, int MT, int NT, int BK>
static int launch_gemm_bf16(hipStream_t st, const float* A, int64_t lda, const unsigned short* Bp,
                            int64_t Kp, int64_t N, float* C, int64_t ldc, int64_t M, int64_t K) {
  using Cfg = Gemm3Cfg<NW, MT, NT, BK, 1>;
  constexpr size_t lds = Cfg::LDS;
  static_assert(lds <= 160 * 1024, "LDS budget");
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)k_gemm3<NW, MT, NT, BK, 1, 1>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const dim3 grid((unsigned)((M + Cfg::BM - 1) / Cfg::BM), (unsigned)((N + Cfg::BN - 1) / Cfg::BN));
  hipLaunchKernelGGL((k_gemm3<NW, MT, NT, BK, 1, 1>), grid, dim3(Cfg::THREADS), lds, st, A, lda,
                     Bp, Kp, N * Kp, C, ldc, M, N, K);
  return (int)hipGetLastError();
}

}  // namespace sv2n

using namespace sv2n;

// a[m][k] -> bf16 (RNE) into ab [M][ld_ab], zero for K <= k < ld_ab
__global__ __launch_bounds__(256) void k_to_bf16(const float* __restrict__ a, int64_t lda,
                                                 int64_t M, int64_t K,
                                                 unsigned short* __restrict__ ab, int64_t ld_ab) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * ld_ab) return;
  const int64_t m = i / ld_ab, k = i - m * ld_ab;
  ab[i] = k < K ? (unsigned short)(bf16_pk(a[m * lda + k], 0.f) & 0xffffu) : (unsigned short)0;
}

static int gemm_bf16(const float* A, int64_t lda, const uint16_t* Bp, float* C, int64_t ldc,
                     int64_t M, int64_t N, int64_t K, uint16_t* a_bf16, int64_t ld_ab,
                     hipStream_t stream);

extern "C" int sv2n_gemm_bf16(const float* A, int64_t lda, const uint16_t* Bp, float* C,
                              int64_t ldc, int64_t M, int64_t N, int64_t K, hipStream_t stream) {
  return gemm_bf16(A, lda, Bp, C, ldc, M, N, K, nullptr, 0, stream);
}

extern "C" int sv2n_gemm_bf16_export(const float* A, int64_t lda, const uint16_t* Bp, float* C,
                                     int64_t ldc, int64_t M, int64_t N, int64_t K,
                                     uint16_t* a_bf16, int64_t ld_ab, hipStream_t stream) {
  if (!a_bf16) return SV2N_ERR_ARG;
  if (ld_ab < (K + 63) / 64 * 64 || (ld_ab & 7)) return SV2N_ERR_SHAPE;
  if ((uintptr_t)a_bf16 & 15) return SV2N_ERR_ALIGN;
  return gemm_bf16(A, lda, Bp, C, ldc, M, N, K, a_bf16, ld_ab, stream);
}

extern "C" int sv2n_gemm_bf16_a16(const uint16_t* A, int64_t lda, const uint16_t* Bp, float* C,
                                  int64_t ldc, int64_t M, int64_t N, int64_t K,
                                  hipStream_t stream) {
  if (!A || !Bp || !C || M <= 0 || N <= 0 || K <= 0 || lda < K || ldc < N) return SV2N_ERR_ARG;
  if (((uintptr_t)A & 15) || (lda & 7) || ((uintptr_t)Bp & 15)) return SV2N_ERR_ALIGN;
  if (M < 1024 || N < 384) return SV2N_ERR_SHAPE;  // the large-tile kernel's shapes
  const int64_t Kp = sv2n_split3_kpad(K);
  using Cfg = GemmBWCfg<256, 192, false, false, false>;
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_gemm_bw<256, 192, false, false, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)Cfg::LDS);
    return true;
  }();
  (void)attr;
  const int nm = (int)((M + 255) / 256), nn = (int)((N + 191) / 192);
  hipLaunchKernelGGL((k_gemm_bw<256, 192, false, false, false>),
                     dim3((unsigned)(((nm + 7) / 8) * 8 * nn)), dim3(Cfg::THREADS), Cfg::LDS,
                     stream, (const void*)A, lda, (const void*)Bp, Kp, C, ldc, M, N, K,
                     (int64_t)K, nm, nn, (unsigned short*)nullptr, (int64_t)0);
  return (int)hipGetLastError();
}

static int gemm_bf16(const float* A, int64_t lda, const uint16_t* Bp, float* C, int64_t ldc,
                     int64_t M, int64_t N, int64_t K, uint16_t* a_bf16, int64_t ld_ab,
                     hipStream_t stream) {
  if (!A || !Bp || !C || M <= 0 || N <= 0 || K <= 0 || lda < K || ldc < N) return SV2N_ERR_ARG;
  if (((uintptr_t)A & 15) || (lda & 3) || ((uintptr_t)Bp & 15)) return SV2N_ERR_ALIGN;
  const int64_t Kp = sv2n_split3_kpad(K);
  const unsigned short* B = reinterpret_cast<const unsigned short*>(Bp);
  unsigned short* Aex = reinterpret_cast<unsigned short*>(a_bf16);
  if (K % 4 == 0 && (lda & 3) == 0 && M >= 1024 && N >= 384) {
    // large-tile kernel (sv2n_gemm_bw.h): 256 x 192 tiles of 8 waves (round 4;
    // the 128 x 128 k_gemm_bf16nt below was L2-bound on the C3 projection)
    using Cfg = GemmBWCfg<256, 192, false, true, false>;
    static bool attr_bw = [] {
      (void)hipFuncSetAttribute((const void*)k_gemm_bw<256, 192, false, true, false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)Cfg::LDS);
      return true;
    }();
    (void)attr_bw;
    const int nm = (int)((M + 255) / 256), nn = (int)((N + 191) / 192);
    hipLaunchKernelGGL((k_gemm_bw<256, 192, false, true, false>),
                       dim3((unsigned)(((nm + 7) / 8) * 8 * nn)), dim3(Cfg::THREADS), Cfg::LDS,
                       stream, (const void*)A, lda, (const void*)B, Kp, C, ldc, M, N, K,
                       (int64_t)K, nm, nn, Aex, ld_ab);
    return (int)hipGetLastError();
  }
  if (Aex) {  // the other kernels: a separate rounding pass
    hipLaunchKernelGGL(k_to_bf16, dim3((unsigned)((M * ld_ab + 255) / 256)), dim3(256), 0, stream,
                       A, lda, M, K, Aex, ld_ab);
  }
  if (K % 4 == 0) {  // k_gemm_bf16nt (sv2n_gemm_bf16.h)
    static bool attr = [] {
      (void)hipFuncSetAttribute((const void*)k_gemm_bf16nt,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)BF_LDS);
      return true;
    }();
    (void)attr;
    const int nm = (int)((M + BF_BM - 1) / BF_BM), nn = (int)((N + BF_BN - 1) / BF_BN);
    hipLaunchKernelGGL(k_gemm_bf16nt, dim3((unsigned)(((nm + 7) / 8) * 8 * nn)), dim3(256), BF_LDS,
                       stream, A, lda, B, Kp, C, ldc, M, N, K, nm, nn);
    return (int)hipGetLastError();
  }
  const int64_t mb = (M + 127) / 128;
  const bool wide = mb * ((N + 207) / 208) >= 240;
  if (wide) return launch_gemm_bf16<8, 1, 13, 64>(stream, A, lda, B, Kp, N, C, ldc, M, K);
  return launch_gemm_bf16<8, 1, 7, 64>(stream, A, lda, B, Kp, N, C, ldc, M, K);
}

extern "C" int64_t sv2n_split3_kpad(int64_t K) {
  return (K + SPLIT3_KALIGN - 1) / SPLIT3_KALIGN * SPLIT3_KALIGN;
}

extern "C" int sv2n_split3(const float* in, int64_t rows, int64_t K, int64_t ld, int transpose,
                           uint16_t* out, hipStream_t stream) {
  if (!in || !out || rows <= 0 || K <= 0) return SV2N_ERR_ARG;
  const int64_t Kp = sv2n_split3_kpad(K);
  if (transpose) {
    if (ld < rows) return SV2N_ERR_ARG;
    const dim3 grid((unsigned)((Kp + 31) / 32), (unsigned)((rows + 31) / 32));
    hipLaunchKernelGGL(k_split3_t, grid, dim3(256), 0, stream, in, rows, K, ld,
                       reinterpret_cast<unsigned short*>(out), Kp);
  } else {
    if (ld < K) return SV2N_ERR_ARG;
    const int64_t n = rows * Kp;
    hipLaunchKernelGGL(k_split3, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, in, rows,
                       K, ld, reinterpret_cast<unsigned short*>(out), Kp);
  }
  return (int)hipGetLastError();
}

extern "C" int sv2n_gemm_f32x3(const float* A, int64_t lda, const uint16_t* Bp, float* C,
                               int64_t ldc, int64_t M, int64_t N, int64_t K, hipStream_t stream) {
  if (!A || !Bp || !C || M <= 0 || N <= 0 || K <= 0 || lda < K || ldc < N) return SV2N_ERR_ARG;
  if (((uintptr_t)A & 15) || (lda & 3) || ((uintptr_t)Bp & 15)) return SV2N_ERR_ALIGN;
  const int64_t Kp = sv2n_split3_kpad(K);
  const unsigned short* B = reinterpret_cast<const unsigned short*>(Bp);
  const int64_t mb = (M + 127) / 128;
  const bool wide = mb * ((N + 207) / 208) >= 240;  // else narrower tiles for more workgroups
  const bool longk = K > 256;
  // 144-column tiles when they pad N less than 208-column ones (C5: N = 144)
  const bool t144 = (N + 143) / 144 * 144 < (N + 207) / 208 * 208 && mb * ((N + 143) / 144) >= 240;
  if (K % 4 == 0) {
    if (twelve_waves(M, N))
      return launch_gemm3d<12, 1, 9, 2>(stream, A, lda, B, Kp, N, C, ldc, M, K);
    if (t144) return launch_gemm3d<8, 1, 9, 2>(stream, A, lda, B, Kp, N, C, ldc, M, K);
    if (wide) return launch_gemm3d<8, 1, 13, 2>(stream, A, lda, B, Kp, N, C, ldc, M, K);
    return launch_gemm3d<8, 1, 7, 2>(stream, A, lda, B, Kp, N, C, ldc, M, K);
  }
  if (t144)
    return longk ? launch_gemm3<8, 1, 9, 64>(stream, A, lda, B, Kp, N, C, ldc, M, K)
                 : launch_gemm3<8, 1, 9, 32>(stream, A, lda, B, Kp, N, C, ldc, M, K);
  if (wide)
    return longk ? launch_gemm3<8, 1, 13, 64>(stream, A, lda, B, Kp, N, C, ldc, M, K)
                 : launch_gemm3<8, 1, 13, 32>(stream, A, lda, B, Kp, N, C, ldc, M, K);
  return longk ? launch_gemm3<8, 1, 7, 64>(stream, A, lda, B, Kp, N, C, ldc, M, K)
               : launch_gemm3<8, 1, 7, 32>(stream, A, lda, B, Kp, N, C, ldc, M, K);
}

// sv2n_gemm_f32x3 with the consumer's ReLU backward in the store: C = (Y > 0)
// ? A·Bᵀ : 0 (Y [M][ldy], the layer's saved activation).  k_gemm3d only (K %
// 4 == 0, else SV2N_ERR_SHAPE: the caller then masks in the attention kernel).
extern "C" int sv2n_gemm_f32x3_relu(const float* A, int64_t lda, const uint16_t* Bp, float* C,
                                    int64_t ldc, int64_t M, int64_t N, int64_t K, const float* Y,
                                    int64_t ldy, hipStream_t stream) {
  if (!A || !Bp || !C || !Y || M <= 0 || N <= 0 || K <= 0 || lda < K || ldc < N || ldy < N)
    return SV2N_ERR_ARG;
  if (((uintptr_t)A & 15) || (lda & 3) || ((uintptr_t)Bp & 15)) return SV2N_ERR_ALIGN;
  if (K % 4 != 0) return SV2N_ERR_SHAPE;
  const int64_t Kp = sv2n_split3_kpad(K);
  const unsigned short* B = reinterpret_cast<const unsigned short*>(Bp);
  const int64_t mb = (M + 127) / 128;
  const bool wide = mb * ((N + 207) / 208) >= 240;
  const bool t144 = (N + 143) / 144 * 144 < (N + 207) / 208 * 208 && mb * ((N + 143) / 144) >= 240;
  if (twelve_waves(M, N))
    return launch_gemm3d<12, 1, 9, 2, true>(stream, A, lda, B, Kp, N, C, ldc, M, K, Y, ldy);
  if (t144)
    return launch_gemm3d<8, 1, 9, 2, true>(stream, A, lda, B, Kp, N, C, ldc, M, K, Y, ldy);
  if (wide)
    return launch_gemm3d<8, 1, 13, 2, true>(stream, A, lda, B, Kp, N, C, ldc, M, K, Y, ldy);
  return launch_gemm3d<8, 1, 7, 2, true>(stream, A, lda, B, Kp, N, C, ldc, M, K, Y, ldy);
}
