// Reproducer for round 5's mha_block wrong-result hazard (verdict item 7): an MFMA that reads its accumulator
// input (SrcC) from AGPRs, followed a few instructions later by v_accvgpr_write to those same AGPRs (the
// accumulator shuttle the compiler emitted for the 4-wave layout's branch-guarded third-tile MFMA:
//   v_mfma_f32_16x16x32_bf16 a[8:11], v[12:15], v[58:61], a[4:7]
//   ds_read_b128 ... ; s_and_b64 ... ; s_nop 0
//   v_accvgpr_write_b32 a4, v36          <- 3 wait states after the MFMA that reads a[4:7]
// ).  Each variant runs exactly that pair with N wait states (s_nop) between them, all in one asm block so
// the compiler's hazard recognizer inserts nothing: A = B = 1, SrcC = 1, so the MFMA must produce 32 + 1 = 33
// per element; if the write lands before the MFMA has read SrcC, the element comes out 32 + 1000.
//   hipcc -O3 --offload-arch=gfx950 tools/probe/mfma_war.hip -o /tmp/mfma_war && /tmp/mfma_war
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int N>
__global__ __launch_bounds__(64) void war_kernel(float* out, int iters) {
  bf16x8 one;
#pragma unroll
  for (int i = 0; i < 8; ++i) one[i] = (__bf16)1.0f;
  const float c = 1.0f, big = 1000.0f;
  int bad = 0;
  for (int it = 0; it < iters; ++it) {
    float r0, r1, r2, r3;
    if constexpr (N == 0) {
      asm volatile(
          "v_accvgpr_write_b32 a4, %[c]\n\tv_accvgpr_write_b32 a5, %[c]\n\tv_accvgpr_write_b32 a6, %[c]\n\t"
          "v_accvgpr_write_b32 a7, %[c]\n\ts_nop 7\n\ts_nop 7\n\t"
          "v_mfma_f32_16x16x32_bf16 a[8:11], %[A], %[B], a[4:7]\n\t"
          "v_accvgpr_write_b32 a4, %[big]\n\tv_accvgpr_write_b32 a5, %[big]\n\t"
          "v_accvgpr_write_b32 a6, %[big]\n\tv_accvgpr_write_b32 a7, %[big]\n\t"
          "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"
          "v_accvgpr_read_b32 %[r0], a8\n\tv_accvgpr_read_b32 %[r1], a9\n\t"
          "v_accvgpr_read_b32 %[r2], a10\n\tv_accvgpr_read_b32 %[r3], a11\n\ts_nop 7"
          : [r0] "=v"(r0), [r1] "=v"(r1), [r2] "=v"(r2), [r3] "=v"(r3)
          : [A] "v"(one), [B] "v"(one), [c] "v"(c), [big] "v"(big)
          : "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11");
    } else {
      asm volatile(
          "v_accvgpr_write_b32 a4, %[c]\n\tv_accvgpr_write_b32 a5, %[c]\n\tv_accvgpr_write_b32 a6, %[c]\n\t"
          "v_accvgpr_write_b32 a7, %[c]\n\ts_nop 7\n\ts_nop 7\n\t"
          "v_mfma_f32_16x16x32_bf16 a[8:11], %[A], %[B], a[4:7]\n\t"
          "s_nop %[n]\n\t"
          "v_accvgpr_write_b32 a4, %[big]\n\tv_accvgpr_write_b32 a5, %[big]\n\t"
          "v_accvgpr_write_b32 a6, %[big]\n\tv_accvgpr_write_b32 a7, %[big]\n\t"
          "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"
          "v_accvgpr_read_b32 %[r0], a8\n\tv_accvgpr_read_b32 %[r1], a9\n\t"
          "v_accvgpr_read_b32 %[r2], a10\n\tv_accvgpr_read_b32 %[r3], a11\n\ts_nop 7"
          : [r0] "=v"(r0), [r1] "=v"(r1), [r2] "=v"(r2), [r3] "=v"(r3)
          : [A] "v"(one), [B] "v"(one), [c] "v"(c), [big] "v"(big), [n] "n"(N - 1)
          : "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11");
    }
    bad += (r0 != 33.f) + (r1 != 33.f) + (r2 != 33.f) + (r3 != 33.f);
    if (it == 0) out[threadIdx.x] = r0;
  }
  out[64 + threadIdx.x] = (float)bad;
}


// RAW: the MFMA writes a[8:11] (previously -5), then N wait states, then v_accvgpr_read of a8..a11.  A read that
// is too early returns the stale -5 (or a partial result) instead of 33.  The 4-wave layout's bad schedule had
//   v_mfma_f32_16x16x32_bf16 a[4:7], v[12:15], v[106:109], a[4:7]
//   s_cbranch_vccnz .LBB3_116            <- taken when the wave has only two row tiles
//   ...                                  (fall-through: the third tile's MFMA and its AGPR copies)
// .LBB3_116:
//   v_accvgpr_read_b32 v39, a7           <- 1 wait state after the MFMA on the taken edge
template <int N>
__global__ __launch_bounds__(64) void raw_kernel(float* out, int iters) {
  bf16x8 one;
#pragma unroll
  for (int i = 0; i < 8; ++i) one[i] = (__bf16)1.0f;
  const float c = 1.0f, stale = -5.0f;
  int bad = 0;
  for (int it = 0; it < iters; ++it) {
    float r0, r1, r2, r3;
    if constexpr (N == 0) {
      asm volatile(
          "v_accvgpr_write_b32 a4, %[c]\n\tv_accvgpr_write_b32 a5, %[c]\n\tv_accvgpr_write_b32 a6, %[c]\n\t"
          "v_accvgpr_write_b32 a7, %[c]\n\tv_accvgpr_write_b32 a8, %[s]\n\tv_accvgpr_write_b32 a9, %[s]\n\t"
          "v_accvgpr_write_b32 a10, %[s]\n\tv_accvgpr_write_b32 a11, %[s]\n\ts_nop 7\n\ts_nop 7\n\t"
          "v_mfma_f32_16x16x32_bf16 a[8:11], %[A], %[B], a[4:7]\n\t"
          "v_accvgpr_read_b32 %[r0], a8\n\tv_accvgpr_read_b32 %[r1], a9\n\t"
          "v_accvgpr_read_b32 %[r2], a10\n\tv_accvgpr_read_b32 %[r3], a11\n\ts_nop 7\n\ts_nop 7"
          : [r0] "=v"(r0), [r1] "=v"(r1), [r2] "=v"(r2), [r3] "=v"(r3)
          : [A] "v"(one), [B] "v"(one), [c] "v"(c), [s] "v"(stale)
          : "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11");
    } else {
      asm volatile(
          "v_accvgpr_write_b32 a4, %[c]\n\tv_accvgpr_write_b32 a5, %[c]\n\tv_accvgpr_write_b32 a6, %[c]\n\t"
          "v_accvgpr_write_b32 a7, %[c]\n\tv_accvgpr_write_b32 a8, %[s]\n\tv_accvgpr_write_b32 a9, %[s]\n\t"
          "v_accvgpr_write_b32 a10, %[s]\n\tv_accvgpr_write_b32 a11, %[s]\n\ts_nop 7\n\ts_nop 7\n\t"
          "v_mfma_f32_16x16x32_bf16 a[8:11], %[A], %[B], a[4:7]\n\t"
          "s_nop %[n]\n\t"
          "v_accvgpr_read_b32 %[r0], a8\n\tv_accvgpr_read_b32 %[r1], a9\n\t"
          "v_accvgpr_read_b32 %[r2], a10\n\tv_accvgpr_read_b32 %[r3], a11\n\ts_nop 7\n\ts_nop 7"
          : [r0] "=v"(r0), [r1] "=v"(r1), [r2] "=v"(r2), [r3] "=v"(r3)
          : [A] "v"(one), [B] "v"(one), [c] "v"(c), [s] "v"(stale), [n] "n"(N - 1)
          : "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11");
    }
    bad += (r0 != 33.f) + (r1 != 33.f) + (r2 != 33.f) + (r3 != 33.f);
    if (it == 0) out[threadIdx.x] = r3;
  }
  out[64 + threadIdx.x] = (float)bad;
}

template <int N>
void run_raw(float* d, float* h, int iters) {
  hipLaunchKernelGGL(raw_kernel<N>, dim3(1), dim3(64), 0, 0, d, iters);
  (void)hipMemcpy(h, d, 128 * sizeof(float), hipMemcpyDeviceToHost);
  double bad = 0;
  for (int i = 0; i < 64; ++i) bad += h[64 + i];
  printf("RAW wait states %2d: last element %8.1f (expect 33), wrong elements %6.0f of %d\n", N, h[0], bad, 64 * 4 * iters);
}

// RAW for the 16-pass 32x32x16 bf16 shape (the FCM stem's MFMA): the first destination register read N wait
// states after the MFMA (a stale -5 if too early).  A = B = 1, C = 0: every element 16.
typedef float floatx16 __attribute__((ext_vector_type(16)));
template <int N, int K>
__global__ __launch_bounds__(64) void raw32_kernel(float* out, int iters) {
  bf16x8 one;
#pragma unroll
  for (int i = 0; i < 8; ++i) one[i] = (__bf16)1.0f;
  const float stale = -5.0f;
  int bad = 0;
  for (int it = 0; it < iters; ++it) {
    float r0;
    asm volatile(
        "v_accvgpr_write_b32 a16, %[s]\n\ts_nop 7\n\ts_nop 7\n\t"
        "v_accvgpr_write_b32 a0, 0\n\tv_accvgpr_write_b32 a1, 0\n\tv_accvgpr_write_b32 a2, 0\n\tv_accvgpr_write_b32 a3, 0\n\t"
        "v_accvgpr_write_b32 a4, 0\n\tv_accvgpr_write_b32 a5, 0\n\tv_accvgpr_write_b32 a6, 0\n\tv_accvgpr_write_b32 a7, 0\n\t"
        "v_accvgpr_write_b32 a8, 0\n\tv_accvgpr_write_b32 a9, 0\n\tv_accvgpr_write_b32 a10, 0\n\tv_accvgpr_write_b32 a11, 0\n\t"
        "v_accvgpr_write_b32 a12, 0\n\tv_accvgpr_write_b32 a13, 0\n\tv_accvgpr_write_b32 a14, 0\n\tv_accvgpr_write_b32 a15, 0\n\t"
        "v_accvgpr_write_b32 a17, %[s]\n\tv_accvgpr_write_b32 a18, %[s]\n\tv_accvgpr_write_b32 a19, %[s]\n\t"
        "v_accvgpr_write_b32 a20, %[s]\n\tv_accvgpr_write_b32 a21, %[s]\n\tv_accvgpr_write_b32 a22, %[s]\n\t"
        "v_accvgpr_write_b32 a23, %[s]\n\tv_accvgpr_write_b32 a24, %[s]\n\tv_accvgpr_write_b32 a25, %[s]\n\t"
        "v_accvgpr_write_b32 a26, %[s]\n\tv_accvgpr_write_b32 a27, %[s]\n\tv_accvgpr_write_b32 a28, %[s]\n\t"
        "v_accvgpr_write_b32 a29, %[s]\n\tv_accvgpr_write_b32 a30, %[s]\n\tv_accvgpr_write_b32 a31, %[s]\n\t"
        "s_nop 7\n\ts_nop 7\n\t"
        "v_mfma_f32_32x32x16_bf16 a[16:31], %[A], %[B], a[0:15]\n\t"
        "s_nop %[n]\n\t"
        "v_accvgpr_read_b32 %[r0], a%c[k]\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7"
        : [r0] "=v"(r0)
        : [A] "v"(one), [B] "v"(one), [s] "v"(stale), [n] "n"(N - 1), [k] "n"(16 + K)
        : "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15",
          "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31");
    bad += r0 != 16.f;
    if (it == 0) out[threadIdx.x] = r0;
  }
  out[64 + threadIdx.x] = (float)bad;
}

template <int N, int K>
double raw32_bad(float* d, float* h, int iters) {
  hipLaunchKernelGGL((raw32_kernel<N, K>), dim3(1), dim3(64), 0, 0, d, iters);
  (void)hipMemcpy(h, d, 128 * sizeof(float), hipMemcpyDeviceToHost);
  double bad = 0;
  for (int i = 0; i < 64; ++i) bad += h[64 + i];
  return bad;
}
// per destination register (a16 + K) of the 32x32x16 MFMA: wrong reads at N wait states
template <int N>
void run_raw32(float* d, float* h, int iters) {
  printf("RAW32 wait states %2d, wrong reads per destination register:", N);
  const double b[16] = {raw32_bad<N, 0>(d, h, iters), raw32_bad<N, 1>(d, h, iters), raw32_bad<N, 2>(d, h, iters),
                        raw32_bad<N, 3>(d, h, iters), raw32_bad<N, 4>(d, h, iters), raw32_bad<N, 5>(d, h, iters),
                        raw32_bad<N, 6>(d, h, iters), raw32_bad<N, 7>(d, h, iters), raw32_bad<N, 8>(d, h, iters),
                        raw32_bad<N, 9>(d, h, iters), raw32_bad<N, 10>(d, h, iters), raw32_bad<N, 11>(d, h, iters),
                        raw32_bad<N, 12>(d, h, iters), raw32_bad<N, 13>(d, h, iters), raw32_bad<N, 14>(d, h, iters),
                        raw32_bad<N, 15>(d, h, iters)};
  for (int k = 0; k < 16; ++k) printf(" %.0f", b[k]);
  printf("\n");
}

template <int N>
void run(float* d, float* h, int iters) {
  hipLaunchKernelGGL(war_kernel<N>, dim3(1), dim3(64), 0, 0, d, iters);
  (void)hipMemcpy(h, d, 128 * sizeof(float), hipMemcpyDeviceToHost);
  double bad = 0;
  for (int i = 0; i < 64; ++i) bad += h[64 + i];
  printf("WAR wait states %2d: first element %8.1f (expect 33), wrong elements %6.0f of %d\n", N, h[0], bad, 64 * 4 * iters);
}

int main() {
  float *d = nullptr, h[128];
  if (hipMalloc(&d, 128 * sizeof(float)) != hipSuccess) return 1;
  const int iters = 1000;
  run<0>(d, h, iters);
  run<1>(d, h, iters);
  run<2>(d, h, iters);
  run<3>(d, h, iters);
  run<4>(d, h, iters);
  run<5>(d, h, iters);
  run<6>(d, h, iters);
  run<7>(d, h, iters);
  run<8>(d, h, iters);
  run<10>(d, h, iters);
  run<12>(d, h, iters);
  run<16>(d, h, iters);
  run_raw<0>(d, h, iters);
  run_raw<1>(d, h, iters);
  run_raw<2>(d, h, iters);
  run_raw<3>(d, h, iters);
  run_raw<4>(d, h, iters);
  run_raw<5>(d, h, iters);
  run_raw<6>(d, h, iters);
  run_raw<7>(d, h, iters);
  run_raw<8>(d, h, iters);
  run_raw<9>(d, h, iters);
  run_raw<10>(d, h, iters);
  run_raw<11>(d, h, iters);
  run_raw<12>(d, h, iters);
  run_raw32<4>(d, h, iters);
  run_raw32<6>(d, h, iters);
  run_raw32<8>(d, h, iters);
  run_raw32<9>(d, h, iters);
  run_raw32<10>(d, h, iters);
  run_raw32<11>(d, h, iters);
  run_raw32<12>(d, h, iters);
  run_raw32<13>(d, h, iters);
  run_raw32<14>(d, h, iters);
  run_raw32<15>(d, h, iters);
  run_raw32<16>(d, h, iters);
  (void)hipFree(d);
  return 0;
}
