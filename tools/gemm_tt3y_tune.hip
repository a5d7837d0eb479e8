// Speed + accuracy harness for the f32-accurate weight-gradient GEMM
// k_gemm_tt3y (sv2n_gemm_tt.h) on the C2 shapes, with B (dxs) split in the
// kernel or pre-split into bf16 planes by its producer (BPL).  Build:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gemm_tt3y_tune.hip -o tt3y
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../spotv2net_amd/csrc/sv2n_common.h"
#include "../spotv2net_amd/csrc/sv2n_gemm_tt.h"

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
__global__ void k_planes(const float* x, unsigned short* p, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned short a, b, c;
  split3(x[i], a, b, c);
  p[i] = a;
  p[n + i] = b;
  p[2 * n + i] = c;
}
// C[m][n] = Σ_k A[k][m] B[k][n] in fp64, and Σ |.|
__global__ void k_ref(const float* A, const float* B, double* C, double* S, int64_t M, int64_t N,
                      int64_t K) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  int64_t m = idx / N, n = idx % N;
  double s = 0, a = 0;
  for (int64_t k = 0; k < K; ++k) {
    const double v = (double)A[k * M + m] * B[k * N + n];
    s += v;
    a += fabs(v);
  }
  C[idx] = s;
  S[idx] = a;
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

template <int NT, int MT, bool BPL>
void run(const char* tag, hipStream_t st, const float* A, const void* B, float* slabs, int64_t M,
         int64_t N, int64_t K, int splitk, const std::vector<double>& ref,
         const std::vector<double>& absr) {
  using Cfg = GemmTT3WCfg<NT, MT>;
  using CfgY = GemmTT3YCfg<NT, MT>;
  CK(hipFuncSetAttribute((const void*)k_gemm_tt3y<NT, MT, BPL>,
                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)CfgY::LDS));
  int64_t ks = (K + splitk - 1) / splitk;
  ks = (ks + 31) / 32 * 32;
  const int sk = (int)((K + ks - 1) / ks);
  const dim3 g((unsigned)((M + Cfg::BM - 1) / Cfg::BM), (unsigned)((N + Cfg::BN - 1) / Cfg::BN),
               (unsigned)((sk + 7) / 8 * 8));
  auto f = [&]() {
    hipLaunchKernelGGL((k_gemm_tt3y<NT, MT, BPL>), g, dim3(Cfg::THREADS), CfgY::LDS, st, A, M,
                       (const float*)B, N, slabs, M, N, K, ks, sk, K * N);
  };
  const double us = timeit(st, f);
  std::vector<float> part((size_t)M * N * sk);
  CK(hipMemcpy(part.data(), slabs, sizeof(float) * part.size(), hipMemcpyDeviceToHost));
  double worst = 0;
  for (int64_t i = 0; i < M * N; i += 5) {
    float s = 0.f;
    for (int z = 0; z < sk; ++z) s += part[(size_t)z * M * N + i];
    worst = fmax(worst, fabs(s - ref[i]) / (absr[i] + 1e-30));
  }
  printf("  %-26s split%d %8.1f us %7.1f TF(f32-eq)  max err/S|ab| %.2e\n", tag, sk, us,
         2.0 * M * N * K / us / 1e6, worst);
  fflush(stdout);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  struct Sh { const char* name; int64_t M, N, K; int sk; };
  for (const Sh& sh : {Sh{"C2 L0 dW (F 1260, ldx 408)", 1260, 408, 15360, 24},
                       Sh{"C2 L1 dW (F 400, ldx 208)", 400, 208, 15360, 54}}) {
    const int64_t M = sh.M, N = sh.N, K = sh.K;
    float *A, *B, *slabs;
    unsigned short* P;
    double *R, *S;
    CK(hipMalloc(&A, 4 * K * M));
    CK(hipMalloc(&B, 4 * K * N));
    CK(hipMalloc(&P, 2 * 3 * K * N));
    CK(hipMalloc(&slabs, 4 * M * N * 64));
    CK(hipMalloc(&R, 8 * M * N));
    CK(hipMalloc(&S, 8 * M * N));
    k_fill<<<(K * M + 255) / 256, 256, 0, st>>>(A, K * M, 1, 1.0f);
    k_fill<<<(K * N + 255) / 256, 256, 0, st>>>(B, K * N, 2, 1e-3f);
    k_planes<<<(K * N + 255) / 256, 256, 0, st>>>(B, P, K * N);
    k_ref<<<(M * N + 255) / 256, 256, 0, st>>>(A, B, R, S, M, N, K);
    CK(hipStreamSynchronize(st));
    std::vector<double> ref(M * N), absr(M * N);
    CK(hipMemcpy(ref.data(), R, 8 * M * N, hipMemcpyDeviceToHost));
    CK(hipMemcpy(absr.data(), S, 8 * M * N, hipMemcpyDeviceToHost));
    printf("== %s K=%ld\n", sh.name, (long)K);
    if (M > 512) {
      run<13, 2, false>("tt3y<13,2> (product)", st, A, B, slabs, M, N, K, sh.sk, ref, absr);
      run<13, 2, true>("tt3y<13,2> B planes", st, A, P, slabs, M, N, K, sh.sk, ref, absr);
      run<13, 2, true>("tt3y<13,2> B planes", st, A, P, slabs, M, N, K, 16, ref, absr);
    }
    run<13, 1, false>("tt3y<13,1> (product)", st, A, B, slabs, M, N, K, sh.sk, ref, absr);
    run<13, 1, true>("tt3y<13,1> B planes", st, A, P, slabs, M, N, K, sh.sk, ref, absr);
    run<13, 1, true>("tt3y<13,1> B planes", st, A, P, slabs, M, N, K, sh.sk / 2, ref, absr);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(P)); CK(hipFree(slabs)); CK(hipFree(R)); CK(hipFree(S));
  }
  return 0;
}
