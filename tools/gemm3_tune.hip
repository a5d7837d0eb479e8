// Accuracy + speed harness for the bf16x3-split GEMM (spotv2net_amd/csrc/sv2n_gemm3_kernel.h)
// against an fp64 reference and the exact-f32 MFMA GEMM (sv2n_gemm_kernel.h), on the
// C2 forward projection shapes.  Build:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gemm3_tune.hip -o build/gemm3_tune
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>
#include <algorithm>

#include "../spotv2net_amd/csrc/sv2n_common.h"
#include "../spotv2net_amd/csrc/sv2n_gemm3_kernel.h"
#include "../spotv2net_amd/csrc/sv2n_gemm_kernel.h"

using namespace sv2n;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void k_ref(const float* A, const float* B, double* C, double* S, int64_t M, int64_t N,
                      int64_t K) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  int64_t m = idx / N, n = idx % N;
  double s = 0, a = 0;
  for (int64_t k = 0; k < K; ++k) {
    s += (double)A[m * K + k] * B[n * K + k];
    a += fabs((double)A[m * K + k] * B[n * K + k]);
  }
  C[idx] = s;
  S[idx] = a;
}

__global__ void k_fill(float* p, int64_t n, uint32_t seed, float scale) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x = (uint32_t)i * 2654435761u ^ seed;
  x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
  p[i] = (((x & 0xffffff) / 16777216.0f) * 2.f - 1.f) * scale;
}

struct Shape { const char* name; int64_t M, N, K; };

template <int NW, int MT, int NT, int BK, int PF, int PIPE = 1>
void run3(const Shape& sh, hipStream_t st, const float* A, const unsigned short* Bp, int64_t Kp,
          float* C, const std::vector<double>& ref, const std::vector<double>& absr) {
  using Cfg = Gemm3Cfg<NW, MT, NT, BK>;
  const size_t lds = Cfg::LDS;
  if (lds > 160 * 1024) return;
  if (lds > 65536)
    CK(hipFuncSetAttribute((const void*)k_gemm3<NW, MT, NT, BK, PF, 3, PIPE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  dim3 grid((unsigned)((sh.M + Cfg::BM - 1) / Cfg::BM), (unsigned)((sh.N + Cfg::BN - 1) / Cfg::BN));
  auto f = [&]() {
    hipLaunchKernelGGL((k_gemm3<NW, MT, NT, BK, PF, 3, PIPE>), grid, dim3(Cfg::THREADS), lds, st, A, sh.K, Bp, Kp,
                       sh.N * Kp, C, sh.N, sh.M, sh.N, sh.K);
  };
  f();
  CK(hipGetLastError());
  CK(hipStreamSynchronize(st));
  std::vector<float> out(sh.M * sh.N);
  CK(hipMemcpy(out.data(), C, sizeof(float) * out.size(), hipMemcpyDeviceToHost));
  double maxrel = 0, maxabs = 0;
  for (size_t i = 0; i < out.size(); i += 7) {
    const double e = fabs(out[i] - ref[i]);
    maxabs = fmax(maxabs, e);
    maxrel = fmax(maxrel, e / (absr[i] + 1e-30));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  printf("  gemm3 NW%d MT%d NT%-2d BK%d PF%d P%d %8.1f us %7.1f TF(f32-eq)  max|err| %.2e  max err/S|ab| %.2e\n",
         NW, MT, NT, BK, PF, PIPE, us, 2.0 * sh.M * sh.N * sh.K / us / 1e6, maxabs, maxrel);
  fflush(stdout);
}

template <int NW, int MT, int NT, int BK, int AP, bool CV = false, int ABL = 0, int PD = 1, bool DV = false,
          int BD = 1>
void run3b(const Shape& sh, hipStream_t st, const float* A, const unsigned short* Bp, int64_t Kp,
           float* C, const std::vector<double>& ref, const std::vector<double>& absr) {
  using Cfg = Gemm3bCfg<NW, MT, NT, BK>;
  const size_t lds = Cfg::LDS;
  if (lds > 160 * 1024) return;
  static_assert(DV, "k_gemm3d only (the product's projection kernel)");
  auto kern = k_gemm3d<NW, MT, NT, AP, false, BD>;
  if (lds > 65536)
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const int nm = (int)((sh.M + Cfg::BM - 1) / Cfg::BM), nn = (int)((sh.N + Cfg::BN - 1) / Cfg::BN);
  const unsigned grid = (unsigned)(((nm + 7) / 8) * 8 * nn);
  CK(hipMemset(C, 0, sizeof(float) * sh.M * sh.N));
  auto f = [&]() {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(Cfg::THREADS), lds, st, A, sh.K, Bp, Kp, sh.N * Kp,
                       C, sh.N, sh.M, sh.N, sh.K, nm, nn, (const float*)nullptr, (int64_t)0);
  };
  f();
  CK(hipGetLastError());
  CK(hipStreamSynchronize(st));
  std::vector<float> out(sh.M * sh.N);
  CK(hipMemcpy(out.data(), C, sizeof(float) * out.size(), hipMemcpyDeviceToHost));
  double maxrel = 0, maxabs = 0;
  for (size_t i = 0; i < out.size(); i += 7) {
    const double e = fabs(out[i] - ref[i]);
    maxabs = fmax(maxabs, e);
    maxrel = fmax(maxrel, e / (absr[i] + 1e-30));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
#ifdef SV2N_GEMM_CLOCK
  if (CV) {
    std::vector<unsigned long long> ck(2 * 4096);
    CK(hipMemcpyFromSymbol(ck.data(), HIP_SYMBOL(g_gemm_clock), sizeof(unsigned long long) * ck.size()));
    std::vector<double> ghz;
    for (unsigned b = 0; b < std::min<unsigned>(grid, 4096); ++b)
      if (ck[2 * b + 1] > 0) ghz.push_back(ck[2 * b] / (ck[2 * b + 1] * 10.0));
    std::sort(ghz.begin(), ghz.end());
    if (!ghz.empty())
      printf("    in-kernel clock (last launch, median over workgroups): %.3f GHz\n", ghz[ghz.size() / 2]);
  }
#endif
  if (ABL) printf("  [ablation %d]", ABL);
  if (PD != 1) printf("  [PD %d]", PD);
  if (DV) printf("  [3d BD%d]", BD);
  printf("  gemm3%s NW%d MT%d NT%-2d BK%d AP%d %8.1f us %7.1f TF(f32-eq)  max|err| %.2e  max err/S|ab| %.2e\n",
         CV ? "c" : "b", NW, MT, NT, BK, AP, us, 2.0 * sh.M * sh.N * sh.K / us / 1e6, maxabs, maxrel);
  fflush(stdout);
}

int main() {
  std::vector<Shape> shapes = {{"fwd L0", 15360, 408, 1260}, {"fwd L1", 15360, 208, 400},
                               {"dX L1", 15360, 400, 208}, {"C5 fwd L0", 262144, 144, 1024}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (auto& sh : shapes) {
    const int64_t M = sh.M, N = sh.N, K = sh.K;
    const int64_t Kp = (K + 63) / 64 * 64;
    float *A, *B, *C;
    double *R, *S;
    unsigned short* Bp;
    CK(hipMalloc(&A, sizeof(float) * M * K));
    CK(hipMalloc(&B, sizeof(float) * N * K));
    CK(hipMalloc(&C, sizeof(float) * M * N));
    CK(hipMalloc(&R, sizeof(double) * M * N));
    CK(hipMalloc(&S, sizeof(double) * M * N));
    CK(hipMalloc(&Bp, sizeof(unsigned short) * 3 * N * Kp));
    k_fill<<<(M * K + 255) / 256, 256, 0, st>>>(A, M * K, 1, 1.0f);
    k_fill<<<(N * K + 255) / 256, 256, 0, st>>>(B, N * K, 2, 0.05f);
    k_split3<<<(N * Kp + 255) / 256, 256, 0, st>>>(B, N, K, K, Bp, Kp);
    k_ref<<<(M * N + 255) / 256, 256, 0, st>>>(A, B, R, S, M, N, K);
    CK(hipStreamSynchronize(st));
    std::vector<double> ref(M * N), absr(M * N);
    CK(hipMemcpy(ref.data(), R, sizeof(double) * M * N, hipMemcpyDeviceToHost));
    CK(hipMemcpy(absr.data(), S, sizeof(double) * M * N, hipMemcpyDeviceToHost));
    printf("== %s M=%ld N=%ld K=%ld\n", sh.name, (long)M, (long)N, (long)K);
    // exact-f32 MFMA baseline (library config)
    {
      auto f = [&]() {
        launch_gemm_cfg<8, 1, 13, 16, true, true, 2, 0>(1, K, st, A, K, B, K, C, N, M, N, K, true,
                                                       true, nullptr);
      };
      f();
      CK(hipStreamSynchronize(st));
      std::vector<float> out(M * N);
      CK(hipMemcpy(out.data(), C, sizeof(float) * M * N, hipMemcpyDeviceToHost));
      double maxrel = 0, maxabs = 0;
      for (size_t i = 0; i < out.size(); i += 7) {
        const double e = fabs(out[i] - ref[i]);
        maxabs = fmax(maxabs, e);
        maxrel = fmax(maxrel, e / (absr[i] + 1e-30));
      }
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < 20; ++r) f();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / 20;
      printf("  f32 MFMA NT13     %8.1f us %7.1f TF          max|err| %.2e  max err/Σ|ab| %.2e\n", us,
             2.0 * M * N * K / us / 1e6, maxabs, maxrel);
    }
    run3b<8, 1, 13, 32, 2, true, 0, 1, true>(sh, st, A, Bp, Kp, C, ref, absr);
    run3b<8, 1, 7, 32, 2, true, 0, 1, true>(sh, st, A, Bp, Kp, C, ref, absr);
    if (sh.K <= 400) {
      // round 5: the LDS-staged kernel (no interleave constraint) with 2-4 waves
      // per workgroup, so that several short-K workgroups share a CU
      run3<4, 1, 13, 32, 2, 0>(sh, st, A, Bp, Kp, C, ref, absr);
      run3<4, 1, 13, 32, 2, 1>(sh, st, A, Bp, Kp, C, ref, absr);
      run3<4, 1, 7, 32, 2, 1>(sh, st, A, Bp, Kp, C, ref, absr);
      run3<4, 2, 7, 32, 2, 1>(sh, st, A, Bp, Kp, C, ref, absr);
      run3<2, 2, 13, 32, 2, 1>(sh, st, A, Bp, Kp, C, ref, absr);
      run3<4, 1, 13, 64, 1, 1>(sh, st, A, Bp, Kp, C, ref, absr);
      run3<4, 1, 7, 64, 2, 1>(sh, st, A, Bp, Kp, C, ref, absr);
      run3<8, 1, 7, 32, 2, 1>(sh, st, A, Bp, Kp, C, ref, absr);
      run3<4, 2, 13, 32, 1, 1>(sh, st, A, Bp, Kp, C, ref, absr);
    }
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(R)); CK(hipFree(S)); CK(hipFree(Bp));
  }
  return 0;
}
