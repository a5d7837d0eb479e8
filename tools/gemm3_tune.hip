// Accuracy + speed harness for the bf16x3-split GEMM (spotv2net_amd/csrc/sv2n_gemm3_kernel.h)
// against an fp64 reference and the exact-f32 MFMA GEMM (sv2n_gemm_kernel.h), on the
// C2 forward projection shapes.  Build:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gemm3_tune.hip -o build/gemm3_tune
#include <cstring>
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

namespace sv2n {
// ---------------------------------------------------------------------------
// k_gemm3g (round 5, experiment; measured slower than k_gemm3d, kept here in
// the harness only — profiles/r05_gemm3_lds_dma.txt): k_gemm3d's tiling (8 waves x 16 rows, NT
// column tiles of 16, BK = 32, six products) with every operand staged by
// LDS-DMA (buffer_load ... lds) instead of registers, so nothing in the K loop
// is an ordinary VGPR load and the waits are counted by hand:
//   * B: two stages [3 planes][16·NT rows][64 B], lane-linear, the 16-B chunk
//     of row r stored at chunk ^ PI[(r >> 2) & 3] (PI = {0, 2, 3, 1}: the four
//     lanes of each ds_read_b128 bank group then hit distinct slots); each
//     stage is 3·NT·16-row pieces of 1 KiB (one DMA instruction each),
//     padded up to 8·NB pieces so every wave issues NB of them;
//   * A: wave-private ring of 3 slots of [16 rows][128 B] fp32, chunk c of
//     row r at c ^ TAU[(r >> 1) & 7] (TAU = {0,1,4,5,6,7,2,3}), issued two
//     K-steps ahead; the fragments are read back from LDS and split there.
// Step s issues B(s+1) and A(s+2), reads and splits A(s), runs its MFMAs on B
// stage s, then waits until B(s+1) and A(s+1) landed (vmcnt(2): only A(s+2)
// out) and crosses a raw barrier (an LDS-DMA write is ordered before a read by
// the issuer's counted wait followed by a barrier the reader has passed).
// ---------------------------------------------------------------------------
template <int NT>
struct Gemm3gCfg {
  static constexpr int NW = 8, THREADS = 512, BM = 128, BN = 16 * NT, BK = 32;
  static constexpr int BPIECES = 3 * NT;                 // 16-row pieces per B stage
  static constexpr int NB = (BPIECES + NW - 1) / NW;     // B DMA instructions per wave and step
  static constexpr int BSTAGE = NB * NW * 1024;          // bytes per B stage (padded)
  static constexpr int ASLOT = 16 * 128;                 // bytes per wave and A slot
  static constexpr int AOFF = 2 * BSTAGE;                // A ring after the two B stages
  static constexpr size_t LDS = (size_t)AOFF + 3 * NW * ASLOT;
};

__device__ __forceinline__ void lds_dma16(rsrc_t r, unsigned char* lds_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (__attribute__((address_space(3))) void*)lds_base, 16, voff, 0, 0, 0);
}

template <int NT>
__global__ __launch_bounds__(512) void k_gemm3g(const float* __restrict__ A, int64_t lda,
                                                const unsigned short* __restrict__ Bp,
                                                int64_t ldb, int64_t bplane,
                                                float* __restrict__ C, int64_t ldc, int64_t M,
                                                int64_t N, int64_t K, int nm, int nn) {
  using Cfg = Gemm3gCfg<NT>;
  constexpr int BN = Cfg::BN, NB = Cfg::NB, BSTAGE = Cfg::BSTAGE, AOFF = Cfg::AOFF;
  constexpr int ASLOT = Cfg::ASLOT;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds8[];
  const int t = threadIdx.x, lane = t & 63, wave = wave_id();
  const int li = lane & 15, lg = lane >> 4;
  const int id = blockIdx.x;
  const int q = id / (8 * nn), rem = id - q * 8 * nn;
  const int nb = rem >> 3, mb = q * 8 + (rem & 7);
  if (mb >= nm) return;
  const int64_t m0 = (int64_t)mb * Cfg::BM, n0 = (int64_t)nb * BN;
  const int64_t arow0 = m0 + (int64_t)wave * 16;
  const int64_t arows = M - arow0;
  const rsrc_t ra = make_rsrc(A + (arow0 > M ? 0 : arow0 * lda),
                              arows > 0 ? (uint32_t)(min(arows, (int64_t)16) * lda * 4) : 0u);
  const rsrc_t rb = make_rsrc(Bp, (uint32_t)(3 * bplane * 2));
  constexpr int PI[4] = {0, 2, 3, 1};
  constexpr int TAU[8] = {0, 1, 4, 5, 6, 7, 2, 3};

  // this lane's DMA sources (k-independent part): B pieces i = wave + 8j
  int bsrc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int i = min(wave + 8 * j, Cfg::BPIECES - 1);  // padding pieces reload the last
    const int R = 16 * i + (lane >> 2);                // row in [3][BN]
    const int p = R / BN, r = R - p * BN;
    const int c = (lane & 3) ^ PI[(r >> 2) & 3];
    const int64_t gn = min(n0 + r, N - 1);
    bsrc[j] = (int)((p * bplane + gn * ldb + 8 * c) * 2);
  }
  // A: rows 8h + lane / 8, chunk (lane & 7) ^ TAU[...]
  int asrc[2], akk[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int lr = 8 * h + (lane >> 3);
    const int c = (lane & 7) ^ TAU[(lr >> 1) & 7];
    asrc[h] = (int)((lr * lda + 4 * c) * 4);
    akk[h] = 4 * c;
  }
  const int nk = (int)((K + 31) / 32);
  auto issue_b = [&](int s) __attribute__((always_inline)) {
    unsigned char* st = lds8 + (s & 1) * BSTAGE;
#pragma unroll
    for (int j = 0; j < NB; ++j)
      lds_dma16(rb, st + (wave + 8 * j) * 1024, bsrc[j] + s * 64);
  };
  auto issue_a = [&](int s) __attribute__((always_inline)) {
    unsigned char* sl = lds8 + AOFF + ((s % 3) * 8 + wave) * ASLOT;
    const int k0 = 32 * s;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      lds_dma16(ra, sl + h * 1024, k0 + akk[h] < K ? asrc[h] + k0 * 4 : OOB);
  };
  auto read_split_a = [&](int s, bf16x8 (&h3)[3]) __attribute__((always_inline)) {
    const unsigned char* sl = lds8 + AOFF + ((s % 3) * 8 + wave) * ASLOT;
    const int tw = TAU[(li >> 1) & 7];
    const f32x4 lo = *reinterpret_cast<const f32x4*>(sl + li * 128 + ((2 * lg) ^ tw) * 16);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(sl + li * 128 + ((2 * lg + 1) ^ tw) * 16);
    split3_frag(lo, hi, h3);
  };

  f32x4 acc[NT];
#pragma unroll
  for (int b = 0; b < NT; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: B(0), A(0), A(1); B(0) and A(0) landed, then the barrier that
  // orders the DMA writes before any wave's reads
  issue_b(0);
  issue_a(0);
  if (nk > 1) {
    issue_a(1);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  const int bq_off = PI[(li >> 2) & 3];
  for (int s = 0; s < nk; ++s) {
    const bool nxt = s + 1 < nk, nxt2 = s + 2 < nk;
    if (nxt) issue_b(s + 1);   // stage (s+1)&1: last read in step s-1
    if (nxt2) issue_a(s + 2);  // slot (s+2)%3: last read in step s-1
    bf16x8 af[3];
    read_split_a(s, af);
    const unsigned char* sB = lds8 + (s & 1) * BSTAGE;
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      bf16x8 bq[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bq[p] = *reinterpret_cast<const bf16x8*>(sB + (p * BN + 16 * b + li) * 64 +
                                                 ((lg ^ bq_off) * 16));
      acc[b] = mfma_planes<3>(af, bq, acc[b]);
    }
    if (nxt) {
      // B(s+1) and A(s+1) landed (only A(s+2) may be out), every read of this
      // step retired, then the barrier that publishes them
      if (nxt2)
        asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
#pragma unroll
  for (int b = 0; b < NT; ++b) {
    const int64_t gn = n0 + 16 * b + li;
    if (gn < N) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gm = arow0 + 4 * lg + r;
        if (gm < M) C[gm * ldc + gn] = acc[b][r];
      }
    }
  }
}
}  // namespace sv2n

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
          int BD = 1, bool SWZ = false, bool STG = false>
void run3b(const Shape& sh, hipStream_t st, const float* A, const unsigned short* Bp, int64_t Kp,
           float* C, const std::vector<double>& ref, const std::vector<double>& absr) {
  using Cfg = Gemm3bCfg<NW, MT, NT, BK, SWZ, STG ? 3 : 2>;
  const size_t lds = Cfg::LDS;
  if (lds > 160 * 1024) return;
  static_assert(DV, "k_gemm3d only (the product's projection kernel)");
  auto kern = k_gemm3d<NW, MT, NT, AP, false, BD, SWZ, STG>;
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
  if (DV) printf("  [3d BD%d%s%s grid %u, LDS %zu]", BD, SWZ ? " SWZ" : "", STG ? " STG" : "", grid, lds);
  printf("  gemm3%s NW%d MT%d NT%-2d BK%d AP%d %8.1f us %7.1f TF(f32-eq)  max|err| %.2e  max err/S|ab| %.2e\n",
         CV ? "c" : "b", NW, MT, NT, BK, AP, us, 2.0 * sh.M * sh.N * sh.K / us / 1e6, maxabs, maxrel);
  fflush(stdout);
}

template <int NT>
void run3g(const Shape& sh, hipStream_t st, const float* A, const unsigned short* Bp, int64_t Kp,
           float* C, const std::vector<double>& ref, const std::vector<double>& absr) {
  using Cfg = Gemm3gCfg<NT>;
  const size_t lds = Cfg::LDS;
  auto kern = k_gemm3g<NT>;
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int nm = (int)((sh.M + Cfg::BM - 1) / Cfg::BM), nn = (int)((sh.N + Cfg::BN - 1) / Cfg::BN);
  const unsigned grid = (unsigned)(((nm + 7) / 8) * 8 * nn);
  CK(hipMemset(C, 0, sizeof(float) * sh.M * sh.N));
  auto f = [&]() {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, st, A, sh.K, Bp, Kp, sh.N * Kp, C, sh.N,
                       sh.M, sh.N, sh.K, nm, nn);
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
  printf("  [3g LDS-DMA] NT%-2d %8.1f us %7.1f TF(f32-eq)  max|err| %.2e  max err/S|ab| %.2e\n", NT,
         us, 2.0 * sh.M * sh.N * sh.K / us / 1e6, maxabs, maxrel);
  fflush(stdout);
}

int main(int argc, char** argv) {
  std::vector<Shape> shapes = {{"fwd L0", 15360, 408, 1260}, {"fwd L1", 15360, 208, 400},
                               {"dX L1", 15360, 400, 208}, {"C5 fwd L0", 262144, 144, 1024},
                               {"C5 fwd L1", 262144, 144, 128}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (auto& sh : shapes) {
    if (argc > 1 && !strstr(argv[1], sh.name)) continue;  // e.g. "fwd L0|dX L1"
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
    // round 6: XOR-swizzled unpadded B stages (SWZ, 80 KB at NT = 13), 8-wave
    // and 4-wave workgroups (two 4-wave workgroups per CU, barriers apart)
    // (round 6, first pass: SWZ alone is neutral, 4-wave pairs 89.8 -> 138 us);
    // STG: the second half of the waves half a K-step behind, three B stages
    // (second pass: STG 88.1 -> 98.8 us at C2 L0, slower on every shape);
    // third pass: 12- and 16-wave workgroups (3 / 4 waves per SIMD)
    // (third pass: profiles/r06_gemm3_waves.txt — <12, 1, 9> kept where it fills the chip)
    // fourth pass: two row tiles per wave (MT = 2: half the B fragment reads
    // per MFMA)
    for (int rep = 0; rep < 2; ++rep) {
      run3b<12, 1, 9, 32, 2, true, 0, 1, true>(sh, st, A, Bp, Kp, C, ref, absr);
      run3b<8, 1, 7, 32, 2, true, 0, 1, true>(sh, st, A, Bp, Kp, C, ref, absr);
      run3b<8, 2, 7, 32, 2, true, 0, 1, true>(sh, st, A, Bp, Kp, C, ref, absr);
      run3b<12, 2, 5, 32, 2, true, 0, 1, true>(sh, st, A, Bp, Kp, C, ref, absr);
      run3b<8, 2, 5, 32, 2, true, 0, 1, true>(sh, st, A, Bp, Kp, C, ref, absr);
      run3b<4, 2, 13, 32, 2, true, 0, 1, true>(sh, st, A, Bp, Kp, C, ref, absr);
      run3b<8, 2, 4, 32, 2, true, 0, 1, true>(sh, st, A, Bp, Kp, C, ref, absr);
    }
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(R)); CK(hipFree(S)); CK(hipFree(Bp));
  }
  return 0;
}
