// CAM++ pooled head prologue: out_nonlinear BN-ReLU + StatsPool (statistics_pooling,
// egs/alimeeting/ts_vad2/cam_pplus_wespeaker.py:28-39: mean and unbiased std over time).
//
// One workgroup owns 64 channels of one batch row; its 4 waves split the time axis, so
// every wave load is 64 consecutive channels of one frame (128 B bf16 / 256 B fp32).
// Two passes over the (small, L2-resident) rows: sum -> mean, then sum of squared
// deviations, both accumulated in fp64 so the std of near-constant channels keeps its
// digits.  T == 1 gives 0/0 = NaN like torch.std(unbiased=True).
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kGroups = 4;

template <bool BF>
__global__ __launch_bounds__(256) void stats_pool_kernel(const act_t<BF>* __restrict__ x, int T, int C,
                                                         const float* __restrict__ s,
                                                         const float* __restrict__ h, float* __restrict__ stats,
                                                         float* __restrict__ tout) {
  __shared__ double red[kGroups][64];
  const int lane = threadIdx.x & 63;
  const int g = threadIdx.x >> 6;
  const int b = blockIdx.y;
  const int c = blockIdx.x * 64 + lane;
  const act_t<BF>* xb = x + (int64_t)b * T * C + c;
  const float sc = s[c], sh = h[c];
  double sum = 0.0;
  for (int t = g; t < T; t += kGroups) {
    const float v = fmaxf(fmaf(ld_act(xb, (int64_t)t * C), sc, sh), 0.f);
    sum += (double)v;
    if (tout) tout[((int64_t)b * T + t) * C + c] = v;
  }
  if (!stats) return;
  red[g][lane] = sum;
  __syncthreads();
  const double mean = (red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]) / (double)T;
  __syncthreads();
  double ss = 0.0;
  for (int t = g; t < T; t += kGroups) {
    const double d = (double)fmaxf(fmaf(ld_act(xb, (int64_t)t * C), sc, sh), 0.f) - mean;
    ss += d * d;
  }
  red[g][lane] = ss;
  __syncthreads();
  if (g == 0) {
    const double var = (red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]) / (double)(T - 1);
    stats[(int64_t)b * 2 * C + c] = (float)mean;
    stats[(int64_t)b * 2 * C + C + c] = (float)sqrt(var);
  }
}

}  // namespace

void stats_pool(const void* x, bool x_bf16, int B, int T, int C, const float* s, const float* h, float* stats,
                float* tout, hipStream_t st) {
  SD_CHECK(C % 64 == 0 && B >= 1 && T >= 1, kErrInvalid, "stats_pool: C must be a multiple of 64");
  if (!stats && !tout) return;
  const double elems = (double)B * T * C;
  ProfScope prof("stats_pool", 0.0, elems * (x_bf16 ? 2.0 : 4.0) + (tout ? elems * 4.0 : 0.0), st);
  const dim3 grid(C / 64, B);
  if (x_bf16)
    hipLaunchKernelGGL(stats_pool_kernel<true>, grid, dim3(256), 0, st, static_cast<const uint16_t*>(x), T, C, s, h,
                       stats, tout);
  else
    hipLaunchKernelGGL(stats_pool_kernel<false>, grid, dim3(256), 0, st, static_cast<const float*>(x), T, C, s, h,
                       stats, tout);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
