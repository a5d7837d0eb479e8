// Speed + correctness harness for the large-tile bf16 GEMM (sv2n_gemm_bw.h)
// against the round-3 kernels on the C3 shapes (bf16 mode, yaml model):
//   projection xs = x·Waugᵀ   M 3840, N 3012, K 1260   (NT)
//   weight gradient dWaug = dxsᵀ·x  M 3012, N 1260, K 3840   (TN)
// Reference: fp64 sums of the bf16-rounded operands.  Build:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gemm_bw_tune.hip -o gemm_bw_tune
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../spotv2net_amd/csrc/sv2n_common.h"
#include "../spotv2net_amd/csrc/sv2n_gemm_bf16.h"
#include "../spotv2net_amd/csrc/sv2n_gemm_bw.h"

using namespace sv2n;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) {                                                                     \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);    \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

__global__ void k_fill(float* p, int64_t n, uint32_t seed, float scale) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x = (uint32_t)i * 2654435761u ^ seed;
  x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
  p[i] = (((x & 0xffffff) / 16777216.0f) * 2.f - 1.f) * scale;
}
__global__ void k_tobf(const float* x, unsigned short* y, int64_t rows, int64_t K, int64_t ld) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * ld) return;
  const int64_t r = i / ld, k = i - r * ld;
  y[i] = k < K ? bf16_rn(x[r * K + k]) : 0;
}
// C[m][n] = Σ_k bf16(A(m,k)) bf16(B(n,k)); ko: A [K][M], B [K][N]
__global__ void k_ref(const float* A, const float* B, double* C, int64_t M, int64_t N, int64_t K,
                      bool ko) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  int64_t m = idx / N, n = idx % N;
  double s = 0;
  for (int64_t k = 0; k < K; ++k) {
    const float a = ko ? A[k * M + m] : A[m * K + k], b = ko ? B[k * N + n] : B[n * K + k];
    s += (double)bf16_f(bf16_rn(a)) * (double)bf16_f(bf16_rn(b));
  }
  C[idx] = s;
}

template <class F>
double timeit(hipStream_t st, F f, int reps = 20) {
  f();
  CK(hipGetLastError());
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / reps;
}

double check(const float* C, const std::vector<double>& ref, int64_t M, int64_t N, int64_t ldc) {
  std::vector<float> out(M * ldc);
  CK(hipMemcpy(out.data(), C, sizeof(float) * out.size(), hipMemcpyDeviceToHost));
  double worst = 0, scale = 0;
  for (int64_t m = 0; m < M; m += 3)
    for (int64_t n = 0; n < N; ++n) {
      worst = fmax(worst, fabs(out[m * ldc + n] - ref[m * N + n]));
      scale = fmax(scale, fabs(ref[m * N + n]));
    }
  return worst / fmax(scale, 1e-30);
}

template <int BM, int BN, bool KO, bool AF, bool BF, int WM = 2, int WN = 4, int BK = 64>
void run_bw(const char* tag, hipStream_t st, const void* A, int64_t lda, const void* B, int64_t ldb,
            float* C, int64_t M, int64_t N, int64_t K, int splitk, const std::vector<double>& ref,
            double flops) {
  using Cfg = GemmBWCfg<BM, BN, KO, AF, BF, WM, WN, BK>;
  auto kern = k_gemm_bw<BM, BN, KO, AF, BF, WM, WN, BK>;
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                         (int)Cfg::LDS));
  const int nm = (int)((M + BM - 1) / BM), nn = (int)((N + BN - 1) / BN);
  int64_t ks = (K + splitk - 1) / splitk;
  ks = (ks + BK - 1) / BK * BK;
  const int nz = (int)((K + ks - 1) / ks);
  const dim3 grid((unsigned)(((nm + 7) / 8) * 8 * nn), 1, (unsigned)nz);
  CK(hipMemset(C, 0, sizeof(float) * M * N * nz));
  auto f = [&]() {
    hipLaunchKernelGGL(kern, grid, dim3(Cfg::THREADS), Cfg::LDS, st, A, lda, B, ldb, C, N, M, N,
                       K, ks, nm, nn, (unsigned short*)nullptr, (int64_t)0);
  };
  const double us = timeit(st, f);
  double err = -1;
  if (nz == 1) err = check(C, ref, M, N, N);
  printf("  %-28s BM%d BN%d W%dx%d BK%d split%d %8.1f us %7.1f TF  err %.2e\n", tag, BM, BN, WM, WN,
         BK, nz, us, flops / us / 1e6, err);
  fflush(stdout);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  // ---- projection (NT): M 3840 nodes, N 3012 Waug rows, K 1260 ----
  {
    const int64_t M = 3840, N = 3012, K = 1260, Kp = 1280;
    float *A, *B, *C;
    unsigned short *Ab, *Bb;
    double* R;
    CK(hipMalloc(&A, 4 * M * K));
    CK(hipMalloc(&B, 4 * N * K));
    CK(hipMalloc(&C, 4 * M * N * 4));
    CK(hipMalloc(&R, 8 * M * N));
    CK(hipMalloc(&Ab, 2 * M * Kp));
    CK(hipMalloc(&Bb, 2 * N * Kp));
    k_fill<<<(M * K + 255) / 256, 256, 0, st>>>(A, M * K, 1, 1.0f);
    k_fill<<<(N * K + 255) / 256, 256, 0, st>>>(B, N * K, 2, 0.05f);
    k_tobf<<<(M * Kp + 255) / 256, 256, 0, st>>>(A, Ab, M, K, Kp);
    k_tobf<<<(N * Kp + 255) / 256, 256, 0, st>>>(B, Bb, N, K, Kp);
    k_ref<<<(M * N + 255) / 256, 256, 0, st>>>(A, B, R, M, N, K, false);
    CK(hipStreamSynchronize(st));
    std::vector<double> ref(M * N);
    CK(hipMemcpy(ref.data(), R, 8 * M * N, hipMemcpyDeviceToHost));
    const double fl = 2.0 * M * N * K;
    printf("== C3 projection NT M=%ld N=%ld K=%ld\n", (long)M, (long)N, (long)K);
    {
      CK(hipFuncSetAttribute((const void*)k_gemm_bf16nt, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)BF_LDS));
      const int nm = (M + BF_BM - 1) / BF_BM, nn = (N + BF_BN - 1) / BF_BN;
      auto f = [&]() {
        hipLaunchKernelGGL(k_gemm_bf16nt, dim3(((nm + 7) / 8) * 8 * nn), dim3(256), BF_LDS, st, A, K,
                           Bb, Kp, C, N, M, N, K, nm, nn);
      };
      const double us = timeit(st, f);
      printf("  %-28s %8.1f us %7.1f TF  err %.2e\n", "round-3 k_gemm_bf16nt", us, fl / us / 1e6,
             check(C, ref, M, N, N));
    }
    run_bw<256, 192, false, true, false>("bw A fp32, B bf16", st, A, K, Bb, Kp, C, M, N, K, 1, ref, fl);
    run_bw<256, 192, false, false, false>("bw A bf16, B bf16", st, Ab, Kp, Bb, Kp, C, M, N, K, 1, ref, fl);
    run_bw<256, 128, false, true, false>("bw A fp32, B bf16", st, A, K, Bb, Kp, C, M, N, K, 1, ref, fl);
    run_bw<256, 128, false, false, false>("bw A bf16, B bf16", st, Ab, Kp, Bb, Kp, C, M, N, K, 1, ref, fl);
    run_bw<128, 256, false, true, false>("bw A fp32, B bf16", st, A, K, Bb, Kp, C, M, N, K, 1, ref, fl);
    run_bw<192, 256, false, true, false>("bw A fp32, B bf16", st, A, K, Bb, Kp, C, M, N, K, 1, ref, fl);
    run_bw<256, 256, false, true, false>("bw A fp32, B bf16", st, A, K, Bb, Kp, C, M, N, K, 1, ref, fl);
    run_bw<256, 256, false, false, false>("bw A bf16, B bf16", st, Ab, Kp, Bb, Kp, C, M, N, K, 1, ref, fl);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(R)); CK(hipFree(Ab)); CK(hipFree(Bb));
  }
  // ---- weight gradient (TN): dWaug[o][f] = Σ_n dxs[n][o] x[n][f]: M 3012, N 1260, K 3840 ----
  {
    const int64_t M = 3012, N = 1260, K = 3840, ldA = 3012, ldB = 1260, ldAb = 3016, ldBb = 1264;
    float *A, *B, *C;
    unsigned short *Ab, *Bb;
    double* R;
    CK(hipMalloc(&A, 4 * K * ldA));
    CK(hipMalloc(&B, 4 * K * ldB));
    CK(hipMalloc(&C, 4 * M * N * 4));
    CK(hipMalloc(&R, 8 * M * N));
    CK(hipMalloc(&Ab, 2 * K * ldAb));
    CK(hipMalloc(&Bb, 2 * K * ldBb));
    k_fill<<<(K * ldA + 255) / 256, 256, 0, st>>>(A, K * ldA, 3, 1e-3f);
    k_fill<<<(K * ldB + 255) / 256, 256, 0, st>>>(B, K * ldB, 4, 1.0f);
    k_tobf<<<(K * ldAb + 255) / 256, 256, 0, st>>>(A, Ab, K, ldA, ldAb);
    k_tobf<<<(K * ldBb + 255) / 256, 256, 0, st>>>(B, Bb, K, ldB, ldBb);
    k_ref<<<(M * N + 255) / 256, 256, 0, st>>>(A, B, R, M, N, K, true);
    CK(hipStreamSynchronize(st));
    std::vector<double> ref(M * N);
    CK(hipMemcpy(ref.data(), R, 8 * M * N, hipMemcpyDeviceToHost));
    const double fl = 2.0 * M * N * K;
    printf("== C3 weight gradient TN M=%ld N=%ld K=%ld\n", (long)M, (long)N, (long)K);
    {
      using Cfg = GemmTTCfg<128, 128, 1>;
      const dim3 grid((M + 127) / 128, (N + 127) / 128, 2);
      const int64_t ks = 1920;
      auto f = [&]() {
        hipLaunchKernelGGL((k_gemm_tt<128, 128, 1>), grid, dim3(256), Cfg::LDS, st, A, ldA, B, ldB,
                           C, N, M, N, K, ks);
      };
      const double us = timeit(st, f);
      printf("  %-28s %8.1f us %7.1f TF  (2 slabs, no check)\n", "round-3 k_gemm_tt<128,128,1>", us,
             fl / us / 1e6);
    }
    run_bw<128, 128, true, false, false>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 1, ref, fl);
    run_bw<128, 128, true, false, false>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 2, ref, fl);
    // round 6: K steps of 128 per barrier (half the barriers, 147 KB of LDS)
    run_bw<128, 128, true, false, false, 2, 4, 128>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 1, ref, fl);
    run_bw<128, 128, true, false, false, 2, 4, 128>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 2, ref, fl);
    run_bw<128, 128, true, false, false, 2, 2, 128>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 2, ref, fl);
    run_bw<128, 128, true, false, false>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 1, ref, fl);
    // round 5: 4-wave workgroups (wave tile 64 x 64: half the LDS reads per MFMA)
    run_bw<128, 128, true, false, false, 2, 2>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 1, ref, fl);
    run_bw<128, 128, true, false, false, 2, 2>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 2, ref, fl);
    run_bw<128, 128, true, false, false, 2, 2>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 3, ref, fl);
    run_bw<128, 256, true, false, false, 2, 4>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 2, ref, fl);
    run_bw<256, 128, true, false, false, 4, 2>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 2, ref, fl);
    run_bw<128, 256, true, false, false, 2, 2>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 2, ref, fl);
    run_bw<64, 128, true, false, false, 1, 2>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 1, ref, fl);
    run_bw<64, 128, true, false, false, 1, 2>("bw A bf16, B bf16", st, Ab, ldAb, Bb, ldBb, C, M, N, K, 2, ref, fl);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(R)); CK(hipFree(Ab)); CK(hipFree(Bb));
  }
  return 0;
}
