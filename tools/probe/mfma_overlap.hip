// Probe: v_mfma_f32_16x16x32_bf16 whose destination PARTIALLY overlaps its accumulator source (srcC), as hipcc
// emits it in 6 places of the shipped attention objects and 15 of the attn_long select form that gave wrong
// results, e.g.  v_mfma_f32_16x16x32_bf16 v[94:97], v[120:123], v[34:37], v[92:95].
// Each lane seeds v100..v105 = base + 0..5 and runs
//   case 0 (dst above C):   v_mfma v[102:105], A, B, v[100:103]   -> v102..105 = A.B + (base + 0..3)
//   case 1 (dst below C):   v_mfma v[100:103], A, B, v[102:105]   -> v100..103 = A.B + (base + 2..5)
//   case 2 (dst == C):      v_mfma v[100:103], A, B, v[100:103]   -> v100..103 = A.B + (base + 0..3)  (control)
//   case 3 (WAR, VALU):     v_mfma v[102:105], A, B, v[110:113]; v_mov_b32 v110, -1.0; v_mov_b32 v111, -1.0
//                           (srcC overwritten by the next instructions)  -> v102..105 = A.B + (base + 0..3)
//   case 4 (WAR, LDS):      the same with ds_read_b64 v[110:111] of -1.0s issued right after the MFMA
//                           (the select form's `ds_read_b64_tr_b16 v[92:93]` 7 instructions after an MFMA reading v[92:95])
// with A = B = bf16 ones (A.B = 32 in every element) or zeros, and compares every lane with that.
//   hipcc -O3 --offload-arch=gfx950 tools/probe/mfma_overlap.hip -o tools/probe/mfma_overlap && ./tools/probe/mfma_overlap
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define SEED                                   \
  "v_mov_b32 v100, %4\n\t"                     \
  "v_add_f32 v101, 1.0, v100\n\t"              \
  "v_add_f32 v102, 2.0, v100\n\t"              \
  "v_add_f32 v103, 1.0, v102\n\t"              \
  "v_add_f32 v104, 4.0, v100\n\t"              \
  "v_add_f32 v105, 1.0, v104\n\t"              \
  "v_mov_b32 v106, %5\n\t"                     \
  "v_mov_b32 v107, %5\n\t"                     \
  "v_mov_b32 v108, %5\n\t"                     \
  "v_mov_b32 v109, %5\n\t"                     \
  "s_nop 4\n\t"
#define DRAIN "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"
#define CLOB "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113"
#define SEEDC "v_mov_b32 v110, v100\n\tv_mov_b32 v111, v101\n\tv_mov_b32 v112, v102\n\tv_mov_b32 v113, v103\n\ts_nop 4\n\t"

template <int CASE>
__global__ __launch_bounds__(64) void probe(float* out, unsigned ab) {
  const float base = 1000.f * (float)blockIdx.x + 8.f * (float)threadIdx.x;
  float r0, r1, r2, r3;
  if (CASE == 0)
    asm volatile(SEED "v_mfma_f32_16x16x32_bf16 v[102:105], v[106:109], v[106:109], v[100:103]\n\t" DRAIN
                 "v_mov_b32 %0, v102\n\tv_mov_b32 %1, v103\n\tv_mov_b32 %2, v104\n\tv_mov_b32 %3, v105"
                 : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                 : "v"(base), "v"(ab)
                 : CLOB);
  else if (CASE == 1)
    asm volatile(SEED "v_mfma_f32_16x16x32_bf16 v[100:103], v[106:109], v[106:109], v[102:105]\n\t" DRAIN
                 "v_mov_b32 %0, v100\n\tv_mov_b32 %1, v101\n\tv_mov_b32 %2, v102\n\tv_mov_b32 %3, v103"
                 : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                 : "v"(base), "v"(ab)
                 : CLOB);
  else if (CASE == 3)
    asm volatile(SEED SEEDC "v_mfma_f32_16x16x32_bf16 v[102:105], v[106:109], v[106:109], v[110:113]\n\t"
                 "v_mov_b32 v110, -1.0\n\tv_mov_b32 v111, -1.0\n\t" DRAIN
                 "v_mov_b32 %0, v102\n\tv_mov_b32 %1, v103\n\tv_mov_b32 %2, v104\n\tv_mov_b32 %3, v105"
                 : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                 : "v"(base), "v"(ab)
                 : CLOB);
  else if (CASE == 4) {
    __shared__ float junk[128];
    junk[threadIdx.x * 2] = -1.f;
    junk[threadIdx.x * 2 + 1] = -1.f;
    __syncthreads();
    const unsigned addr = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)&junk[threadIdx.x * 2];
    asm volatile(SEED SEEDC "v_mfma_f32_16x16x32_bf16 v[102:105], v[106:109], v[106:109], v[110:113]\n\t"
                 "ds_read_b64 v[110:111], %6\n\ts_waitcnt lgkmcnt(0)\n\t" DRAIN
                 "v_mov_b32 %0, v102\n\tv_mov_b32 %1, v103\n\tv_mov_b32 %2, v104\n\tv_mov_b32 %3, v105"
                 : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                 : "v"(base), "v"(ab), "v"(addr)
                 : CLOB);
  } else
    asm volatile(SEED "v_mfma_f32_16x16x32_bf16 v[100:103], v[106:109], v[106:109], v[100:103]\n\t" DRAIN
                 "v_mov_b32 %0, v100\n\tv_mov_b32 %1, v101\n\tv_mov_b32 %2, v102\n\tv_mov_b32 %3, v103"
                 : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
                 : "v"(base), "v"(ab)
                 : CLOB);
  float* o = out + ((size_t)blockIdx.x * 64 + threadIdx.x) * 4;
  o[0] = r0;
  o[1] = r1;
  o[2] = r2;
  o[3] = r3;
}

int main() {
  const int nb = 1024;
  float* d;
  hipMalloc(&d, sizeof(float) * nb * 64 * 4);
  std::vector<float> h(nb * 64 * 4);
  for (int c = 0; c < 5; ++c)
    for (int one = 0; one < 2; ++one) {
      const unsigned ab = one ? 0x3f803f80u : 0u;   // two bf16 1.0 / two bf16 0.0 per register
      hipMemset(d, 0, sizeof(float) * nb * 64 * 4);
      if (c == 0) hipLaunchKernelGGL(probe<0>, dim3(nb), dim3(64), 0, 0, d, ab);
      else if (c == 1) hipLaunchKernelGGL(probe<1>, dim3(nb), dim3(64), 0, 0, d, ab);
      else if (c == 2) hipLaunchKernelGGL(probe<2>, dim3(nb), dim3(64), 0, 0, d, ab);
      else if (c == 3) hipLaunchKernelGGL(probe<3>, dim3(nb), dim3(64), 0, 0, d, ab);
      else hipLaunchKernelGGL(probe<4>, dim3(nb), dim3(64), 0, 0, d, ab);
      hipMemcpy(h.data(), d, sizeof(float) * h.size(), hipMemcpyDeviceToHost);
      long bad = 0;
      for (int b = 0; b < nb; ++b)
        for (int l = 0; l < 64; ++l)
          for (int k = 0; k < 4; ++k) {
            const float base = 1000.f * b + 8.f * l;
            const float want = (one ? 32.f : 0.f) + base + (float)(k + (c == 1 ? 2 : 0));
            const float got = h[((size_t)b * 64 + l) * 4 + k];
            if (got != want) {
              if (bad < 4) printf("case %d ab %d block %d lane %d reg %d: got %.1f want %.1f\n", c, one, b, l, k, got, want);
              ++bad;
            }
          }
      printf("case %d (%s), A.B = %s: %ld of %d values wrong\n", c,
             c == 0 ? "dst above srcC" : c == 1 ? "dst below srcC" : c == 2 ? "dst == srcC"
             : c == 3 ? "srcC overwritten by VALU right after" : "srcC overwritten by an LDS load right after", one ? "32" : "0", bad, nb * 256);
    }
  hipFree(d);
  return 0;
}
