// Diagnostics for the hipGraph replay investigation (tools/graph_repro.py, tests/test_gpu_graph.py): does a
// kernel node that follows a memset node in a replayed graph read the memset's zeros, or lines its own XCD's L2
// kept from the previous replay?
//   graph = [memsetAsync(X, 0) -> kernel: Y[i] = X[i]; X[i] = replay-independent junk]
// replayed R times; after each replay every Y[i] must be 0.  `fork` puts the kernel behind a fork / join of a
// second captured stream (an event-joined node, as the TS-VAD forward's two window slices are).
#include "common.h"
#include "kernels.h"

namespace sd {
namespace {

__global__ __launch_bounds__(256) void memset_probe_kernel(float* __restrict__ x, float* __restrict__ y, int n) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    y[i] = x[i];
    x[i] = 7.f;   // plain store: the line stays valid (dirty) in this XCD's L2
  }
}

__global__ void count_nonzero_kernel(const float* __restrict__ y, int n, int* __restrict__ bad) {
  int c = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) c += y[i] != 0.f;
  if (c) atomicAdd(bad, c);
}

}  // namespace

void graph_memset_probe(int n, int replays, bool fork, int* bad_per_replay, hipStream_t st) {
  float *x = nullptr, *y = nullptr;
  int* bad = nullptr;
  SD_HIP(hipMalloc(&x, (size_t)n * 4));
  SD_HIP(hipMalloc(&y, (size_t)n * 4));
  SD_HIP(hipMalloc(&bad, sizeof(int) * (replays + 1)));
  SD_HIP(hipMemsetAsync(bad, 0, sizeof(int) * (replays + 1), st));
  SD_HIP(hipMemsetAsync(x, 0x55, (size_t)n * 4, st));
  hipStream_t cap = nullptr, side = nullptr;
  hipEvent_t e1 = nullptr, e2 = nullptr;
  SD_HIP(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  SD_HIP(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
  SD_HIP(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
  SD_HIP(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
  SD_HIP(hipStreamSynchronize(st));
  hipGraph_t g = nullptr;
  hipGraphExec_t ex = nullptr;
  SD_HIP(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
  SD_HIP(hipMemsetAsync(x, 0, (size_t)n * 4, cap));
  if (fork) {
    SD_HIP(hipEventRecord(e1, cap));
    SD_HIP(hipStreamWaitEvent(side, e1, 0));
    hipLaunchKernelGGL(count_nonzero_kernel, dim3(1), dim3(64), 0, side, y, 0, bad + replays);   // empty side work
    SD_HIP(hipEventRecord(e2, side));
    SD_HIP(hipStreamWaitEvent(cap, e2, 0));
  }
  hipLaunchKernelGGL(memset_probe_kernel, dim3(1024), dim3(256), 0, cap, x, y, n);
  SD_HIP(hipStreamEndCapture(cap, &g));
  SD_HIP(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  for (int r = 0; r < replays; ++r) {
    SD_HIP(hipGraphLaunch(ex, st));
    hipLaunchKernelGGL(count_nonzero_kernel, dim3(256), dim3(256), 0, st, y, n, bad + r);
  }
  SD_HIP(hipMemcpyAsync(bad_per_replay, bad, sizeof(int) * replays, hipMemcpyDeviceToHost, st));
  SD_HIP(hipStreamSynchronize(st));
  (void)hipGraphExecDestroy(ex);
  (void)hipGraphDestroy(g);
  (void)hipEventDestroy(e1);
  (void)hipEventDestroy(e2);
  (void)hipStreamDestroy(cap);
  (void)hipStreamDestroy(side);
  (void)hipFree(x);
  (void)hipFree(y);
  (void)hipFree(bad);
}

}  // namespace sd
