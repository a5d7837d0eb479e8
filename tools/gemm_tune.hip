// Standalone tuner for the f32-MFMA GEMM template (spotv2net_amd/csrc/sv2n_gemm_kernel.h)
// on the five projection GEMMs of one C2 training step (B=512 graphs, n=30):
//   fwd L0  M=15360 N=408 K=1260   A=x[M][K] (k-major)   B=Waug[N][K] (k-major)
//   fwd L1  M=15360 N=208 K=400
//   dX  L1  M=15360 N=400 K=208    A=dxs[M][K]           B=Waug[K][N]
//   dWT L0  M=1260  N=408 K=15360  A=x[K][M]             B=dxs[K][N]   (split-K)
//   dWT L1  M=400   N=208 K=15360
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gemm_tune.hip -o build/gemm_tune
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../spotv2net_amd/csrc/sv2n_gemm_kernel.h"

using namespace sv2n;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void k_ref(const float* A, int64_t lda, bool ak, const float* B, int64_t ldb, bool bk,
                      double* C, int64_t M, int64_t N, int64_t K) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  int64_t m = idx / N, n = idx % N;
  double s = 0;
  for (int64_t k = 0; k < K; ++k) {
    double a = ak ? A[m * lda + k] : A[k * lda + m];
    double b = bk ? B[n * ldb + k] : B[k * ldb + n];
    s += a * b;
  }
  C[idx] = s;
}

__global__ void k_fill(float* p, int64_t n, uint32_t seed) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x = (uint32_t)i * 2654435761u ^ seed;
  x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
  p[i] = ((x & 0xffffff) / 16777216.0f) * 2.f - 1.f;
}

struct Shape { const char* name; int64_t M, N, K; bool ak, bk; };

using Launcher = std::function<void(int, int64_t, hipStream_t, const float*, int64_t, const float*,
                                    int64_t, float*, int64_t, int64_t, int64_t, int64_t, float*)>;

template <int NW, int MT, int NT, int KB, int PF, int ABL = 0>
void add_variants(std::vector<std::pair<std::string, Launcher>>& v, bool ak, bool bk) {
  char buf[96];
  snprintf(buf, sizeof buf, "NW%d MT%d NT%d KB%d PF%d%s", NW, MT, NT, KB, PF,
           ABL == 0 ? "" : ABL == 1 ? " -gload" : ABL == 2 ? " -lstore" : " -both");
  Launcher f;
  if (ak && bk)
    f = [](int sk, int64_t ks, hipStream_t s, const float* A, int64_t lda, const float* B,
           int64_t ldb, float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, float* part) {
      launch_gemm_cfg<NW, MT, NT, KB, true, true, PF, ABL>(sk, ks, s, A, lda, B, ldb, C, ldc, M, N, K,
                                                      true, true, part);
    };
  else if (ak)
    f = [](int sk, int64_t ks, hipStream_t s, const float* A, int64_t lda, const float* B,
           int64_t ldb, float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, float* part) {
      launch_gemm_cfg<NW, MT, NT, KB, true, false, PF, ABL>(sk, ks, s, A, lda, B, ldb, C, ldc, M, N, K,
                                                       true, true, part);
    };
  else
    f = [](int sk, int64_t ks, hipStream_t s, const float* A, int64_t lda, const float* B,
           int64_t ldb, float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, float* part) {
      launch_gemm_cfg<NW, MT, NT, KB, false, false, PF, ABL>(sk, ks, s, A, lda, B, ldb, C, ldc, M, N, K,
                                                        true, true, part);
    };
  v.push_back({buf, f});
}

template <int NT>
void add_all(std::vector<std::pair<std::string, Launcher>>& v, bool ak, bool bk) {
  add_variants<8, 1, NT, 16, 1>(v, ak, bk);
  add_variants<8, 1, NT, 16, 2>(v, ak, bk);
  add_variants<8, 1, NT, 32, 1>(v, ak, bk);
  add_variants<8, 1, NT, 32, 2>(v, ak, bk);
  add_variants<8, 1, NT, 16, 2, 3>(v, ak, bk);
  add_variants<4, 1, NT, 16, 1>(v, ak, bk);
  add_variants<4, 1, NT, 16, 2>(v, ak, bk);
  add_variants<4, 1, NT, 32, 2>(v, ak, bk);
  add_variants<4, 2, NT, 16, 2>(v, ak, bk);
  add_variants<4, 2, NT, 32, 2>(v, ak, bk);
  add_variants<8, 2, NT, 16, 2>(v, ak, bk);
}

int main(int argc, char** argv) {
  std::vector<Shape> shapes = {{"fwd L0", 15360, 408, 1260, true, true},
                               {"fwd L1", 15360, 208, 400, true, true},
                               {"dX  L1", 15360, 400, 208, true, false},
                               {"dWT L0", 1260, 408, 15360, false, false},
                               {"dWT L1", 400, 208, 15360, false, false}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  for (auto& sh : shapes) {
    const int64_t M = sh.M, N = sh.N, K = sh.K;
    const int64_t lda = sh.ak ? K : M, ldb = sh.bk ? K : N;
    float *A, *B, *C, *P;
    double* R;
    CK(hipMalloc(&A, sizeof(float) * M * K));
    CK(hipMalloc(&B, sizeof(float) * N * K));
    CK(hipMalloc(&C, sizeof(float) * M * N));
    CK(hipMalloc(&P, sizeof(float) * M * N * 32));
    CK(hipMalloc(&R, sizeof(double) * M * N));
    k_fill<<<(M * K + 255) / 256, 256, 0, st>>>(A, M * K, 1);
    k_fill<<<(N * K + 255) / 256, 256, 0, st>>>(B, N * K, 2);
    k_ref<<<(M * N + 255) / 256, 256, 0, st>>>(A, lda, sh.ak, B, ldb, sh.bk, R, M, N, K);
    CK(hipStreamSynchronize(st));
    std::vector<double> ref(M * N);
    CK(hipMemcpy(ref.data(), R, sizeof(double) * M * N, hipMemcpyDeviceToHost));
    std::vector<std::pair<std::string, Launcher>> vars;
    std::vector<int> nts;
    for (int nt : {8, 13}) {
      const size_t before = vars.size();
      if (nt == 8) add_all<8>(vars, sh.ak, sh.bk); else add_all<13>(vars, sh.ak, sh.bk);
      for (size_t i = before; i < vars.size(); ++i) nts.push_back(nt);
    }
    std::vector<int> splits = {1};
    if (K >= 4096) splits = {8, 16, 24, 32};
    const double flops = 2.0 * M * N * K;
    printf("== %s M=%ld N=%ld K=%ld (%.2f GFLOP)\n", sh.name, (long)M, (long)N, (long)K, flops / 1e9);
    double best = 1e30;
    std::string bestname;
    for (size_t vi = 0; vi < vars.size(); ++vi) {
      for (int sk : splits) {
        int64_t ks = (K + sk - 1) / sk;
        ks = (ks + 31) / 32 * 32;
        const int skr = (int)((K + ks - 1) / ks);
        auto& f = vars[vi].second;
        f(skr, ks, st, A, lda, B, ldb, C, N, M, N, K, P);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(st));
        // check
        std::vector<float> out(M * N);
        CK(hipMemcpy(out.data(), C, sizeof(float) * M * N, hipMemcpyDeviceToHost));
        double maxerr = 0;
        for (int64_t i = 0; i < M * N; i += 97) maxerr = fmax(maxerr, fabs(out[i] - ref[i]));
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; ++r) f(skr, ks, st, A, lda, B, ldb, C, N, M, N, K, P);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        printf("  %-26s split %2d : %8.1f us %7.1f TF  err %.1e%s\n", vars[vi].first.c_str(), skr,
               us, flops / us / 1e6, maxerr,
               (maxerr > 1e-3 && vars[vi].first.find(" -") == std::string::npos) ? "  <-- BAD" : "");
        if (vars[vi].first.find(" -") == std::string::npos && maxerr < 1e-3 && us < best) {
          best = us;
          bestname = vars[vi].first + " split " + std::to_string(skr);
        }
      }
    }
    printf("  BEST %s: %.1f us %.1f TF\n", bestname.c_str(), best, flops / best / 1e6);
    fflush(stdout);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(P)); CK(hipFree(R));
  }
  return 0;
}
