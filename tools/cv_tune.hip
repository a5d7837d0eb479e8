// Read-pattern probe for the covariance-layout edge passes (C2: 512 graphs x
// 870 rows x 126 floats; a pass needs the first 42 floats of the 435 upper
// rows of each graph).  Times, with the Infinity Cache flushed before every
// launch (a 1 GiB write in between) and warm (back to back):
//   full   every float of edge_attr, 16 B per lane, grid-stride
//   cov8   the upper rows' 42 covariance floats, flat float2 pieces of 16-row
//          tiles, one 512-thread workgroup per graph, all loads in flight
//   cov16  the same with 16-B pieces where the row start allows (rows alternate
//          8 / 16-B alignment: 8-B pieces on odd rows)
//   covln  the 128-B lines covering each covariance segment (what HBM moves)
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/cv_tune.hip -o cv_tune
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../spotv2net_amd/csrc/sv2n_edge.hip"

using namespace sv2n;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) {                                                                     \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);    \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

constexpr int NN = 30, S = 42, D = 3 * S, E0 = NN * (NN - 1), P = E0 / 2;

__global__ void k_fill(float* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (float)((i * 2654435761ull) & 1023) * 1e-3f;
}

// reads 1 GiB (clean lines: evicting them costs no write-back)
__global__ void k_flush(const float4* p, int64_t n4, float* out) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x)
    s += p[i].x;
  if (s == 12345.f) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_full(const float4* __restrict__ a, int64_t n4,
                                              float* __restrict__ out) {
  float s = 0.f;
  const int64_t st = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * st < n4; i += 4 * st) {
    const float4 x0 = a[i], x1 = a[i + st], x2 = a[i + 2 * st], x3 = a[i + 3 * st];
    s += x0.x + x1.y + x2.z + x3.w;
  }
  for (; i < n4; i += st) s += a[i].x;
  if (s == 12345.f) out[threadIdx.x] = s;
}

// one 512-thread workgroup per graph, waves own 16-row tiles (tile k on wave k % 8)
template <int MODE>  // 0: float2 pieces, 2: whole 128-B lines
__global__ __launch_bounds__(512) void k_cov(const float* __restrict__ ea, float* __restrict__ out) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t g = blockIdx.x;
  const rsrc_t rg = make_rsrc(ea + g * E0 * D, (uint32_t)(E0 * D) * 4u);
  constexpr int TP = (P + 15) / 16;
  float s = 0.f;
  if (MODE == 0) {
    constexpr int NJ = (16 * S + 127) / 128;
    int goff[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int f = 128 * j + 2 * lane, r = f / S, c = f - r * S;
      goff[j] = f < 16 * S ? 4 * (r * D + c) : OOB;
    }
    u32x2 v[4][NJ];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int tile = wave + 8 * k;
      const bool ok = tile < TP;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        v[k][j] = __builtin_amdgcn_raw_buffer_load_b64(rg, ok ? goff[j] : OOB,
                                                        ok ? tile * 16 * D * 4 : 0, 0);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < NJ; ++j) s += __uint_as_float(v[k][j][0]) + __uint_as_float(v[k][j][1]);
  } else {
    // lines covering row r's [r·504, r·504 + 168): lane = (row-in-tile, line)
    // 16 rows x up to 3 lines of 128 B = 48 lines per tile, 8 lanes x 16 B per line
    u32x4 v[4][6];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int tile = wave + 8 * k;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int piece = 64 * j + lane;      // 384 pieces = 48 lines x 8
        const int ln = piece >> 3, q = piece & 7;
        const int r = ln / 3, l3 = ln - 3 * r;
        const int p = tile * 16 + r;
        const int b0 = p * D * 4;              // row start (bytes, graph-relative)
        const int lb = (b0 & ~127) + 128 * l3; // line l3 of the row's cover
        const bool ok = tile < TP && lb < b0 + 4 * S;
        v[k][j] = __builtin_amdgcn_raw_buffer_load_b128(rg, ok ? lb + 16 * q : OOB, 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < 6; ++j) s += __uint_as_float(v[k][j][0]);
  }
  if (s == 12345.f) out[t] = s;
}

int main() {
  const int B = 512;
  const int64_t nf = (int64_t)B * E0 * D;
  float *ea, *out;
  float4* fl;
  const int64_t fl4 = (1ll << 30) / 16;
  CK(hipMalloc(&ea, nf * 4));
  CK(hipMalloc(&out, 4096));
  CK(hipMalloc(&fl, fl4 * 16));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, ea, nf);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch, double bytes) {
    for (int cold = 1; cold >= 0; --cold) {
      float tot = 0.f;
      const int reps = 20;
      for (int r = 0; r < reps + 2; ++r) {
        if (cold) hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, (const float4*)fl, fl4, out);
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) tot += ms;
      }
      const double us = tot * 1e3 / reps;
      printf("%-8s %-5s %8.2f us  %7.2f TB/s of %.1f MB\n", name, cold ? "cold" : "warm", us,
             bytes / us * 1e-6, bytes * 1e-6);
    }
  };
  run("full", [&] { hipLaunchKernelGGL(k_full, dim3(2048), dim3(256), 0, 0, (const float4*)ea, nf / 4, out); },
      nf * 4.0);
  run("cov8", [&] { hipLaunchKernelGGL(k_cov<0>, dim3(B), dim3(512), 0, 0, ea, out); },
      (double)B * P * S * 4);
  run("covln", [&] { hipLaunchKernelGGL(k_cov<2>, dim3(B), dim3(512), 0, 0, ea, out); },
      (double)B * P * S * 4);
  // the library's forward (C2: L 2, H 4; wfold [126][16])
  uint16_t* canon;
  float *wf, *ae0, *ae1;
  CK(hipMalloc(&canon, P * 2));
  std::vector<uint16_t> hc(P);
  for (int u = 0, p = 0; u < NN; ++u)
    for (int v = u + 1; v < NN; ++v) hc[p++] = (uint16_t)((v << 8) | u);
  CK(hipMemcpy(canon, hc.data(), P * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(&wf, D * 16 * 4));
  hipLaunchKernelGGL(k_fill, dim3(16), dim3(256), 0, 0, wf, (int64_t)D * 16);
  CK(hipMalloc(&ae0, (int64_t)B * E0 * 4 * 4));
  CK(hipMalloc(&ae1, (int64_t)B * E0 * 4 * 4));
  LayerPtrs lp{};
  lp.p[0] = ae0;
  lp.p[1] = ae1;
  const double cvb = (double)B * (P * S + NN * S) * 4 + (double)B * E0 * 8 * 4;
  run("fwd", [&] { hipLaunchKernelGGL((k_edge_fwd_cv2<6, 8>), dim3(B), dim3(512), 0, 0, ea, NN, S, canon, wf, 16, lp, 2, 4); }, cvb);
  CK(hipDeviceSynchronize());
  return 0;
}
