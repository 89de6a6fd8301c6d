// Prints what ds_read_b64_tr_b16 returns per lane for a [rows][cols] = r*100+c image.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void k(short* out, int stride) {
  __shared__ short img[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) img[i] = (short)((i / stride) * 100 + (i % stride));
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, i = l & 15;
  const int row = 4 * g + (i >> 2), col = 4 * (i & 3);
  typedef __attribute__((address_space(3))) v4s* p_t;
  const uint32_t base = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)img);
  v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((p_t)(uintptr_t)(base + (row * stride + col) * 2));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = r[e];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 48);
  short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 20; ++l) printf("lane %2d: %d %d %d %d\n", l, h[4*l], h[4*l+1], h[4*l+2], h[4*l+3]);
  return 0;
}
