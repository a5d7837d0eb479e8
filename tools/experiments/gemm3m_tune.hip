// Speed + accuracy of the 32x32x16 projection GEMM (k_gemm3m,
// spotv2net_amd/csrc/sv2n_gemm3m.h) against the 16x16x32 kernel k_gemm3d on
// the product's projection shapes, both against an fp64 reference.
// Build:  hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/experiments/gemm3m_tune.hip -o build/gemm3m_tune
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../spotv2net_amd/csrc/sv2n_common.h"
#include "../../spotv2net_amd/csrc/sv2n_gemm3_kernel.h"
#include "gemm3m_kernel.h"

using namespace sv2n;

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e = (x);                                                                      \
    if (e != hipSuccess) {                                                                   \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

__global__ void k_ref(const float* A, const float* B, double* C, double* S, int64_t M, int64_t N,
                      int64_t K, int64_t stride) {
  // every stride-th output row (the reference is slow)
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t rows = (M + stride - 1) / stride;
  if (idx >= rows * N) return;
  int64_t m = (idx / N) * stride, n = idx % N;
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
constexpr int64_t STRIDE = 61;

static void check_time(const char* label, const Shape& sh, hipStream_t st, float* C,
                       const std::vector<double>& ref, const std::vector<double>& absr,
                       void (*launch)(void*), void* ctx, double peak_tf) {
  CK(hipMemset(C, 0, sizeof(float) * sh.M * sh.N));
  launch(ctx);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(st));
  std::vector<float> out(sh.M * sh.N);
  CK(hipMemcpy(out.data(), C, sizeof(float) * out.size(), hipMemcpyDeviceToHost));
  double maxrel = 0, maxabs = 0;
  const int64_t rows = (sh.M + STRIDE - 1) / STRIDE;
  for (int64_t i = 0; i < rows; ++i)
    for (int64_t n = 0; n < sh.N; ++n) {
      const double o = out[(i * STRIDE) * sh.N + n], r = ref[i * sh.N + n];
      const double e = fabs(o - r);
      maxabs = fmax(maxabs, e);
      maxrel = fmax(maxrel, e / (absr[i * sh.N + n] + 1e-30));
    }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) launch(ctx);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double tf = 2.0 * sh.M * sh.N * sh.K / us / 1e6;
  printf("  %-22s %8.1f us %7.1f TF (%.2f of %.0f)  max|err| %.2e  max err/sum|ab| %.2e\n", label,
         us, tf, tf / peak_tf, peak_tf, maxabs, maxrel);
}

struct Ctx {
  hipStream_t st; const float* A; const unsigned short* Bp; int64_t Kp; float* C; Shape sh;
};

template <int NW, int MT, int NT, int AP>
static void launch_d(void* p) {
  Ctx& c = *static_cast<Ctx*>(p);
  using Cfg = Gemm3bCfg<NW, MT, NT, 32>;
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_gemm3d<NW, MT, NT, AP>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)Cfg::LDS);
    return true;
  }();
  (void)attr;
  const int nm = (int)((c.sh.M + Cfg::BM - 1) / Cfg::BM), nn = (int)((c.sh.N + Cfg::BN - 1) / Cfg::BN);
  hipLaunchKernelGGL((k_gemm3d<NW, MT, NT, AP>), dim3((unsigned)(((nm + 7) / 8) * 8 * nn)),
                     dim3(Cfg::THREADS), Cfg::LDS, c.st, c.A, c.sh.K, c.Bp, c.Kp, c.sh.N * c.Kp,
                     c.C, c.sh.N, c.sh.M, c.sh.N, c.sh.K, nm, nn);
}

template <int NT, int NP>
static void launch_m(void* p) {
  Ctx& c = *static_cast<Ctx*>(p);
  using Cfg = Gemm3mCfg<NT, NP>;
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_gemm3m<NT, NP>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)Cfg::LDS);
    return true;
  }();
  (void)attr;
  const int nm = (int)((c.sh.M + Cfg::BM - 1) / Cfg::BM), nn = (int)((c.sh.N + Cfg::BN - 1) / Cfg::BN);
  hipLaunchKernelGGL((k_gemm3m<NT, NP>), dim3((unsigned)(((nm + 7) / 8) * 8 * nn)), dim3(256),
                     Cfg::LDS, c.st, c.A, c.sh.K, c.Bp, c.Kp, c.sh.N * c.Kp, c.C, c.sh.N, c.sh.M,
                     c.sh.N, c.sh.K, nm, nn);
}

int main() {
  std::vector<Shape> shapes = {{"C2 fwd L0", 15360, 408, 1260}, {"C2 fwd L1", 15360, 208, 400},
                               {"C2 dX L1", 15360, 400, 208}, {"C5 fwd L0", 262144, 144, 1024}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const double P3 = 2500.0 / 6;
  for (auto& sh : shapes) {
    const int64_t M = sh.M, N = sh.N, K = sh.K;
    const int64_t Kp = (K + 63) / 64 * 64;
    const int64_t rows = (M + STRIDE - 1) / STRIDE;
    float *A, *B, *C;
    double *R, *S;
    unsigned short* Bp;
    CK(hipMalloc(&A, sizeof(float) * M * K));
    CK(hipMalloc(&B, sizeof(float) * N * K));
    CK(hipMalloc(&C, sizeof(float) * M * N));
    CK(hipMalloc(&R, sizeof(double) * rows * N));
    CK(hipMalloc(&S, sizeof(double) * rows * N));
    CK(hipMalloc(&Bp, sizeof(unsigned short) * 3 * N * Kp));
    k_fill<<<(M * K + 255) / 256, 256, 0, st>>>(A, M * K, 1, 1.0f);
    k_fill<<<(N * K + 255) / 256, 256, 0, st>>>(B, N * K, 2, 0.05f);
    k_split3<<<(N * Kp + 255) / 256, 256, 0, st>>>(B, N, K, K, Bp, Kp);
    k_ref<<<(rows * N + 255) / 256, 256, 0, st>>>(A, B, R, S, M, N, K, STRIDE);
    CK(hipStreamSynchronize(st));
    std::vector<double> ref(rows * N), absr(rows * N);
    CK(hipMemcpy(ref.data(), R, sizeof(double) * rows * N, hipMemcpyDeviceToHost));
    CK(hipMemcpy(absr.data(), S, sizeof(double) * rows * N, hipMemcpyDeviceToHost));
    printf("== %s M=%ld N=%ld K=%ld\n", sh.name, (long)M, (long)N, (long)K);
    Ctx c{st, A, Bp, Kp, C, sh};
    if (N > 300) check_time("k_gemm3d<8,1,13,2>", sh, st, C, ref, absr, launch_d<8, 1, 13, 2>, &c, P3);
    else if (N == 144) check_time("k_gemm3d<8,1,9,2>", sh, st, C, ref, absr, launch_d<8, 1, 9, 2>, &c, P3);
    else check_time("k_gemm3d<8,1,7,2>", sh, st, C, ref, absr, launch_d<8, 1, 7, 2>, &c, P3);
    check_time("k_gemm3m<7,3>", sh, st, C, ref, absr, launch_m<7, 3>, &c, P3);
    check_time("k_gemm3m<5,3>", sh, st, C, ref, absr, launch_m<5, 3>, &c, P3);
    check_time("k_gemm3m<4,3>", sh, st, C, ref, absr, launch_m<4, 3>, &c, P3);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(R)); CK(hipFree(S)); CK(hipFree(Bp));
  }
  return 0;
}
