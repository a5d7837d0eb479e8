// Ablation harness for the n<=32 attention forward (diagnostic only, not
// shipped): a copy of k_attn_fwd with compile-time switches that drop one
// phase at a time, timed with hipEvents on the C2 layer shapes.
//   AB bit 1: no AE staging          bit 2: no softmax math (P = 1/32)
//   AB bit 4: no aggregation         bit 8: no y stores
//   AB bit 16: no psave stores       bit 32: bias read once before the loop
//   AB bit 64: softmax loops not unrolled
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude
//          -Ispotv2net_amd/csrc tools/attn_ablate.hip -o build/attn_ablate
#include "sv2n_common.h"
#include <cstdio>
#include <vector>
#include <random>

using namespace sv2n;

constexpr int T = 256, TS = 33, SLAB = 128, SXS = SLAB + 4, SLAB_V = 32 * SLAB / 4 / T;
typedef float floatx16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ int crow(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

template <int AB>
__global__ __launch_bounds__(T) void k_fwd(const float* __restrict__ xs, int ldx,
                                           const float* __restrict__ ae,
                                           const float* __restrict__ bias, float* __restrict__ y,
                                           float* __restrict__ psave, int n, int H, int C,
                                           float slope) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sP = smem;
  float* sA = sP + H * 32 * TS;
  float* sD = sA + H * 32;
  float* sE = sD + H * 32;
  float* sX = sE + H * 32 * TS;
  const int g = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int64_t row0 = (int64_t)g * n;
  const int HC = H * C;
  const int nae = n * n * H;
  if (!(AB & 1)) {
    constexpr int AEV = 32 * 32 * SV2N_MAX_HEADS / 4 / T;
    const float* src = ae + row0 * n * H;
    const int nv = nae >> 2;
    float4 av[AEV];
#pragma unroll
    for (int q = 0; q < AEV; ++q) {
      const int k = t + T * q;
      av[q] = k < nv ? reinterpret_cast<const float4*>(src)[k] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < AEV; ++q) {
      const int k = t + T * q;
      if (k < nv) {
        const float* pa = &av[q].x;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int kk = 4 * k + e;
          const int h = kk % H, ij = kk / H;
          const int i = ij / n, jj = ij - i * n;
          sE[(h * 32 + i) * TS + jj] = pa[e];
        }
      }
    }
  }
  for (int idx = t; idx < H * 32; idx += T) {
    const int h = idx >> 5, j = idx & 31;
    float as = 0.f, ad = 0.f;
    if (j < n) {
      const float* r = xs + (row0 + j) * ldx + HC;
      as = r[h];
      ad = r[H + h];
    }
    sA[idx] = as;
    sD[idx] = ad;
  }
  __syncthreads();
  for (int r = t; r < H * 32; r += T) {
    const int h = r >> 5, i = r & 31;
    const bool rv = i < n;
    float* prow = sP + (h * 32 + i) * TS;
    const int64_t pbase = (((int64_t)g * H + h) * 32 + i) * 32;
    if (AB & 2) {
      for (int jj = 0; jj < 32; ++jj) prow[jj] = 1.f / 32;
      continue;
    }
    const uint32_t bits = rv ? row_bits(nullptr, row0 + i, n, i) : 0u;
    const float* er = sE + (h * 32 + i) * TS;
    const float* ar = sA + h * 32;
    const float ad = sD[h * 32 + i];
    float esum = 0.f;
    float lr[32];
    if (AB & 64) {
#pragma unroll 1
      for (int jj = 0; jj < 32; ++jj)
        if ((bits >> jj) & 1u) esum += er[jj];
    } else {
#pragma unroll
      for (int jj = 0; jj < 32; ++jj)
        if ((bits >> jj) & 1u) esum += er[jj];
    }
    const int cnt = __popc(bits);
    const float loopv = cnt > 0 ? esum / (float)cnt : 0.f;
    uint32_t negm = 0u;
    float mx = -INFINITY;
    const uint32_t validm = rv ? (bits | (1u << i)) : 0u;
#pragma unroll
    for (int jj = 0; jj < 32; ++jj) {
      float sv = ar[jj] + ad;
      sv += (jj == i) ? loopv : (((bits >> jj) & 1u) ? er[jj] : 0.f);
      const bool neg = !(sv > 0.f);
      negm |= neg ? (1u << jj) : 0u;
      lr[jj] = neg ? sv * slope : sv;
      if ((validm >> jj) & 1u) mx = fmaxf(mx, lr[jj]);
    }
    float den = 0.f;
#pragma unroll
    for (int jj = 0; jj < 32; ++jj) {
      lr[jj] = ((validm >> jj) & 1u) ? expf(lr[jj] - mx) : 0.f;
      den += lr[jj];
    }
    den += 1e-16f;
#pragma unroll
    for (int jj = 0; jj < 32; jj += 4) {
      float sq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j2 = jj + q;
        const float p = lr[j2] / den;
        const bool valid = (validm >> j2) & 1u;
        sq[q] = valid ? (((negm >> j2) & 1u) ? -p : p) : 0.f;
        prow[j2] = valid ? p : 0.f;
      }
      if (!(AB & 16) && rv)
        *reinterpret_cast<float4*>(psave + pbase + jj) = make_float4(sq[0], sq[1], sq[2], sq[3]);
    }
  }
  if (AB & 4) return;
  const int ncg = (C + SLAB - 1) / SLAB;
  const int nslab = ncg * H;
  float4 reg[SLAB_V];
  auto load_slab = [&](int sl) {
    const int cg = sl / H, h = sl - cg * H;
#pragma unroll
    for (int v = 0; v < SLAB_V; ++v) {
      const int k = t + T * v;
      const int jj = k >> 5, c = cg * SLAB + 4 * (k & 31);
      float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
      if (jj < n && c + 3 < C) w = *reinterpret_cast<const float4*>(xs + (row0 + jj) * ldx + h * C + c);
      reg[v] = w;
    }
  };
  float bv[SV2N_MAX_HEADS];
  if (AB & 32) {
    const int c = 32 * wave + l32;
    for (int h = 0; h < H && h < SV2N_MAX_HEADS; ++h) bv[h] = c < C ? bias[h * C + c] : 0.f;
  }
  load_slab(0);
  floatx16 acc;
  for (int sl = 0; sl < nslab; ++sl) {
    const int cg = sl / H, h = sl - cg * H;
    __syncthreads();
#pragma unroll
    for (int v = 0; v < SLAB_V; ++v) {
      const int k = t + T * v;
      *reinterpret_cast<float4*>(sX + (k >> 5) * SXS + 4 * (k & 31)) = reg[v];
    }
    __syncthreads();
    if (sl + 1 < nslab) load_slab(sl + 1);
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const int cl = 32 * wave + l32;
    const int c = cg * SLAB + cl;
    if (cg * SLAB + 32 * wave < C) {
      const float* prow = sP + (h * 32 + l32) * TS + half;
      const float* xcol = sX + half * SXS + cl;
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(prow[2 * kk], xcol[2 * kk * SXS], acc, 0, 0, 0);
      if (!(AB & 8) && c < C) {
        const int oc = h * C + c;
        float b;
        if (AB & 32) {
          b = 0.f;
#pragma unroll
          for (int q = 0; q < SV2N_MAX_HEADS; ++q) b = q == h ? bv[q] : b;
        } else {
          b = bias[oc];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int i = crow(r, half);
          if (i < n) y[(row0 + i) * HC + oc] = fmaxf(acc[r] + b, 0.f);
        }
      }
    }
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int AB>
static int run(const char* name, int B, int n, int H, int C, int ldx, const float* xs,
               const float* ae, const float* bias, float* y, float* ps) {
  const size_t lds = sizeof(float) * ((size_t)H * 32 * TS * 2 + 2 * H * 32 + 32 * SXS);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w)
    hipLaunchKernelGGL(k_fwd<AB>, dim3(B), dim3(T), lds, 0, xs, ldx, ae, bias, y, ps, n, H, C, 0.2f);
  const int iters = 50;
  CK(hipEventRecord(a, 0));
  for (int w = 0; w < iters; ++w)
    hipLaunchKernelGGL(k_fwd<AB>, dim3(B), dim3(T), lds, 0, xs, ldx, ae, bias, y, ps, n, H, C, 0.2f);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  std::printf("  C=%3d %-34s %8.2f us\n", C, name, 1000.f * ms / iters);
  return 0;
}

int main() {
  const int B = 512, n = 30, H = 4;
  const int Cs[2] = {100, 50};
  for (int li = 0; li < 2; ++li) {
    const int C = Cs[li], ldx = ((H * C + 2 * H) + 3) / 4 * 4;
    std::vector<float> hx((size_t)B * n * ldx), ha((size_t)B * n * n * H), hb(H * C);
    std::mt19937 rng(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    for (auto& v : hx) v = nd(rng);
    for (auto& v : ha) v = nd(rng);
    for (auto& v : hb) v = nd(rng);
    float *xs, *ae, *bias, *y, *ps;
    CK(hipMalloc(&xs, hx.size() * 4));
    CK(hipMalloc(&ae, ha.size() * 4));
    CK(hipMalloc(&bias, hb.size() * 4));
    CK(hipMalloc(&y, (size_t)B * n * H * C * 4));
    CK(hipMalloc(&ps, (size_t)B * H * 32 * 32 * 4));
    CK(hipMemcpy(xs, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(ae, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(bias, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
    if (run<0>("full", B, n, H, C, ldx, xs, ae, bias, y, ps)) return 1;
    if (run<1>("-AE staging", B, n, H, C, ldx, xs, ae, bias, y, ps)) return 1;
    if (run<2>("-softmax math", B, n, H, C, ldx, xs, ae, bias, y, ps)) return 1;
    if (run<4>("-aggregation", B, n, H, C, ldx, xs, ae, bias, y, ps)) return 1;
    if (run<8>("-y stores", B, n, H, C, ldx, xs, ae, bias, y, ps)) return 1;
    if (run<16>("-psave stores", B, n, H, C, ldx, xs, ae, bias, y, ps)) return 1;
    if (run<32>("bias hoisted", B, n, H, C, ldx, xs, ae, bias, y, ps)) return 1;
    if (run<64>("esum loop rolled", B, n, H, C, ldx, xs, ae, bias, y, ps)) return 1;
    if (run<2 | 4>("-softmax -aggregation", B, n, H, C, ldx, xs, ae, bias, y, ps)) return 1;
    if (run<1 | 2 | 4 | 16>("nothing but sA/sD", B, n, H, C, ldx, xs, ae, bias, y, ps)) return 1;
    if (run<1 | 2 | 16>("aggregation only", B, n, H, C, ldx, xs, ae, bias, y, ps)) return 1;
    hipFree(xs); hipFree(ae); hipFree(bias); hipFree(y); hipFree(ps);
  }
  return 0;
}
