// Speed + accuracy harness for the weight-gradient GEMM dWaugᵀ = xᵀ · dxs
// (both operands k-strided, split-K into slabs): the transposed-read kernel
// k_gemm_tt (sv2n_gemm_tt.h; NP = 1 bf16, NP = 3 f32-accurate split) against
// the exact-f32 MFMA kernel (launch_gemm_slabs) and k_gemm3_t, on the C2 / C3
// shapes, errors vs an fp64 reference.  Build:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gemm_tt_tune.hip -o build/gemm_tt_tune
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../spotv2net_amd/csrc/sv2n_common.h"
#include "../spotv2net_amd/csrc/sv2n_gemm3_kernel.h"
#include "../spotv2net_amd/csrc/sv2n_gemm_kernel.h"
#include "../spotv2net_amd/csrc/sv2n_gemm_tt.h"

using namespace sv2n;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

// C[m][n] = Σ_k A[k][m] B[k][n]
__global__ void k_ref(const float* A, const float* B, double* C, double* S, int64_t M, int64_t N,
                      int64_t K) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  int64_t m = idx / N, n = idx % N;
  double s = 0, a = 0;
  for (int64_t k = 0; k < K; ++k) {
    const double p = (double)A[k * M + m] * B[k * N + n];
    s += p;
    a += fabs(p);
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

struct Shape { const char* name; int64_t M, N, K; int splitk; };

static void report(const char* tag, const Shape& sh, float* slabs, int splitk, double us,
                   const std::vector<double>& ref, const std::vector<double>& absr) {
  const int64_t MN = sh.M * sh.N;
  std::vector<float> part((size_t)MN * splitk);
  CK(hipMemcpy(part.data(), slabs, sizeof(float) * part.size(), hipMemcpyDeviceToHost));
  double maxrel = 0, maxabs = 0;
  for (int64_t i = 0; i < MN; i += 7) {
    float s = 0.f;
    for (int z = 0; z < splitk; ++z) s += part[(size_t)z * MN + i];
    const double e = fabs(s - ref[i]);
    maxabs = fmax(maxabs, e);
    maxrel = fmax(maxrel, e / (absr[i] + 1e-30));
  }
  printf("  %-34s %8.1f us %7.1f TF(f32-eq)  max|err| %.2e  max err/S|ab| %.2e\n", tag, us,
         2.0 * sh.M * sh.N * sh.K / us / 1e6, maxabs, maxrel);
  fflush(stdout);
}

template <typename F>
static double time_us(F f, hipStream_t st) {
  f();
  CK(hipGetLastError());
  CK(hipStreamSynchronize(st));
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
  return ms * 1e3 / reps;
}

template <int BM, int BN, int NP>
void run_tt(const Shape& sh, int splitk, hipStream_t st, const float* A, const float* B,
            float* slabs, const std::vector<double>& ref, const std::vector<double>& absr) {
  using Cfg = GemmTTCfg<BM, BN, NP>;
  const size_t lds = Cfg::LDS;
  if (lds > 160 * 1024) return;
  if (lds > 65536)
    CK(hipFuncSetAttribute((const void*)k_gemm_tt<BM, BN, NP>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  int64_t ks = (sh.K + splitk - 1) / splitk;
  ks = (ks + 31) / 32 * 32;
  const int sk = (int)((sh.K + ks - 1) / ks);
  dim3 grid((unsigned)((sh.M + BM - 1) / BM), (unsigned)((sh.N + BN - 1) / BN), (unsigned)sk);
  auto f = [&]() {
    hipLaunchKernelGGL((k_gemm_tt<BM, BN, NP>), grid, dim3(256), lds, st, A, sh.M, B, sh.N, slabs,
                       sh.N, sh.M, sh.N, sh.K, ks);
  };
  const double us = time_us(f, st);
  char tag[96];
  snprintf(tag, sizeof tag, "tt NP%d %dx%d split%d (%u wg)", NP, BM, BN, sk, grid.x * grid.y * sk);
  report(tag, sh, slabs, sk, us, ref, absr);
}

int main() {
  std::vector<Shape> shapes = {{"C2 dWT L0", 1260, 408, 15360, 24},
                               {"C2 dWT L1", 400, 208, 15360, 32}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (auto& sh : shapes) {
    const int64_t M = sh.M, N = sh.N, K = sh.K;
    float *A, *B, *slabs;
    double *R, *S;
    CK(hipMalloc(&A, sizeof(float) * M * K));
    CK(hipMalloc(&B, sizeof(float) * N * K));
    CK(hipMalloc(&slabs, sizeof(float) * M * N * 64));
    CK(hipMalloc(&R, sizeof(double) * M * N));
    CK(hipMalloc(&S, sizeof(double) * M * N));
    k_fill<<<(M * K + 255) / 256, 256, 0, st>>>(A, M * K, 1, 1.0f);
    k_fill<<<(N * K + 255) / 256, 256, 0, st>>>(B, N * K, 2, 0.05f);
    k_ref<<<(M * N + 255) / 256, 256, 0, st>>>(A, B, R, S, M, N, K);
    CK(hipStreamSynchronize(st));
    std::vector<double> ref(M * N), absr(M * N);
    CK(hipMemcpy(ref.data(), R, sizeof(double) * M * N, hipMemcpyDeviceToHost));
    CK(hipMemcpy(absr.data(), S, sizeof(double) * M * N, hipMemcpyDeviceToHost));
    printf("== %s M=%ld N=%ld K=%ld\n", sh.name, (long)M, (long)N, (long)K);
    {  // library exact-f32 config
      int64_t ks = (K + sh.splitk - 1) / sh.splitk;
      ks = (ks + 15) / 16 * 16;
      const int sk = (int)((K + ks - 1) / ks);
      auto f = [&]() {
        if (N > 256)
          launch_gemm_slabs<8, 1, 13, 16, false, false, 2>(sk, ks, st, A, M, B, N, M, N, K, true,
                                                           true, slabs);
        else
          launch_gemm_slabs<8, 1, 8, 16, false, false, 2>(sk, ks, st, A, M, B, N, M, N, K, true,
                                                          true, slabs);
      };
      const double us = time_us(f, st);
      char tag[64];
      snprintf(tag, sizeof tag, "f32 MFMA slabs split%d", sk);
      report(tag, sh, slabs, sk, us, ref, absr);
      for (int sk2 : {sk, sk / 2 > 0 ? sk / 2 : 1}) {  // XCD-grouped K slices
        int64_t ks2 = (K + sk2 - 1) / sk2;
        ks2 = (ks2 + 15) / 16 * 16;
        const int s2 = (int)((K + ks2 - 1) / ks2);
        auto fx = [&]() {
          if (N > 256)
            launch_gemm_slabs<8, 1, 13, 16, false, false, 2, 0, true>(s2, ks2, st, A, M, B, N, M,
                                                                      N, K, true, true, slabs);
          else
            launch_gemm_slabs<8, 1, 8, 16, false, false, 2, 0, true>(s2, ks2, st, A, M, B, N, M,
                                                                     N, K, true, true, slabs);
        };
        const double usx = time_us(fx, st);
        snprintf(tag, sizeof tag, "f32 MFMA slabs XCD-grouped split%d", s2);
        report(tag, sh, slabs, s2, usx, ref, absr);
      }
    }
    for (int sk : {sh.splitk}) {
      if (sk < 1) continue;
      run_tt<128, 128, 1>(sh, sk, st, A, B, slabs, ref, absr);
      run_tt<64, 128, 1>(sh, sk, st, A, B, slabs, ref, absr);
      run_tt<128, 64, 1>(sh, sk, st, A, B, slabs, ref, absr);
      run_tt<64, 64, 1>(sh, sk, st, A, B, slabs, ref, absr);
      if (sh.N < 1000) {
        run_tt<128, 128, 3>(sh, sk, st, A, B, slabs, ref, absr);
        run_tt<64, 128, 3>(sh, sk, st, A, B, slabs, ref, absr);
        run_tt<128, 64, 3>(sh, sk, st, A, B, slabs, ref, absr);
        run_tt<64, 64, 3>(sh, sk, st, A, B, slabs, ref, absr);
      }
    }
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(slabs)); CK(hipFree(R)); CK(hipFree(S));
  }
  return 0;
}
