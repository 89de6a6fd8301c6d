// Weight-stream ceiling probe: every workgroup (one per CU, 8 waves) streams the same P x 24-KiB piece
// sequence through a ring of NS LDS slots with global_load_lds (3 x 1 KiB per wave per piece), waits with
// counted vmcnt + barrier per piece, T times, and does nothing else.  Reports bytes per CU per cycle.
//   hipcc -O3 --offload-arch=gfx950 tools/probe/dma_stream.hip -o /tmp/dma_stream && /tmp/dma_stream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void* lds_ptr_t;
constexpr int kPiece = 12288;   // bf16 elements

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int NS>
__global__ __launch_bounds__(512) void stream(const unsigned short* w, int P, int T, int stride_pieces,
                                              unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(1024))) unsigned short sm[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int total = P * T;
  auto issue = [&](int g) {
    if (g >= total) return;
    const unsigned short* s = w + (size_t)((g % P) * stride_pieces) * kPiece;
    unsigned short* slot = sm + (g % NS) * kPiece;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int f = wv + 8 * j;
      __builtin_amdgcn_global_load_lds((const void*)(s + f * 512 + lane * 8), (lds_ptr_t)(slot + f * 512), 16, 0, 0);
    }
  };
  for (int g = 0; g < NS - 1; ++g) issue(g);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int g = 0; g < total; ++g) {
    const int younger = min(NS - 2, total - 1 - g);
    if (younger <= 0) wait_vm<0>();
    else if (younger == 1) wait_vm<3>();
    else if (younger == 2) wait_vm<6>();
    else if (younger == 3) wait_vm<9>();
    else if (younger == 4) wait_vm<12>();
    else wait_vm<15>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issue(g + NS - 1);
  }
  wait_vm<0>();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int P = 76, T = 20;
  unsigned short* w;
  hipMalloc(&w, (size_t)P * 4 * kPiece * 2);
  hipMemset(w, 0, (size_t)P * 4 * kPiece * 2);
  unsigned long long* cyc;
  hipMalloc(&cyc, cus * 8);
  std::vector<unsigned long long> h(cus);
  auto run = [&](auto kern, int ns, int stride, const char* what) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, ns * kPiece * 2);
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipEventRecord(a);
      hipLaunchKernelGGL(kern, dim3(cus), dim3(512), ns * kPiece * 2, 0, w, P, T, stride, cyc);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      hipMemcpy(h.data(), cyc, cus * 8, hipMemcpyDeviceToHost);
      double avg = 0;
      for (auto c : h) avg += (double)c;
      avg /= cus;
      const double bytes = (double)P * T * kPiece * 2;
      printf("%-28s NS=%d: %.3f ms, %.1f B/clk/CU (s_memtime), %.2f TB/s chip (L2->LDS)\n", what, ns, ms, bytes / avg,
             bytes * cus / (ms * 1e-3) / 1e12);
    }
  };
  run(stream<5>, 5, 1, "1.8 MB shared sequence");
  run(stream<6>, 6, 1, "1.8 MB shared sequence");
  run(stream<5>, 5, 4, "7.3 MB stride-4 sequence");
  return 0;
}
