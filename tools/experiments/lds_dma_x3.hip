// Probe: where does buffer_load_dwordx3 ... lds put each lane's 12 bytes?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* src, float* out) {
  __shared__ float s[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) s[i] = -1.f;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 4096, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(s + 8), 12,
                                           threadIdx.x * 12, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 64) out[i] = s[i];
}
int main() {
  float h[1024], *d, *o;
  for (int i = 0; i < 1024; ++i) h[i] = (float)i;
  hipMalloc(&d, 4096); hipMalloc(&o, 4096);
  hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  hipMemcpy(h, o, 4096, hipMemcpyDeviceToHost);
  for (int i = 0; i < 8 + 64 * 4 + 8; ++i) printf("%d:%g%c", i, h[i], (i % 16 == 15) ? '\n' : ' ');
  printf("\n");
  return 0;
}
